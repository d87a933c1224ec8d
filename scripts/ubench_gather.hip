// Dependent row-gather latency in the configs[1] geometry: the memory floor of the fast kernel.
//
// episode_fast_kernel runs 8192 agents as 256 waves (one per CU, 32 active lanes); every step each
// lane gathers 5 rows (32-B padded f64 Q rows, loaded as dwordx4 + dwordx2) of its own 5.12 MB table
// whose addresses depend on the previous step's rows (act -> T_in bin -> next rows).  This probe
// keeps exactly that and drops everything else: per step each lane issues RPS gathers whose rows are
// derived from the data of the previous step's gathers (a short hash), waits for all of them, and
// folds them in.  So the step time is one dependent round trip of RPS row gathers plus ~15 ALU ops.
// Each agent draws its rows from a pool of POOL pseudo-random distinct rows of its table (the real
// kernel touches ~380 distinct rows per agent per episode, ~100 MB over all 8192 tables); launches
// repeat with the same pools, like the bench's back-to-back episodes, so L2 / MALL warm the same way.
//
// stages=2 is the configs[3] geometry (episode_fast_kernel<4, f64, 2, train, battery>): per step a
// first stage of 2 rows (the round-0 row and the next-state row, both addressed from the previous
// step's data), then a second, DEPENDENT stage of 1 row (the round-1 row, whose p2p bin follows from
// the partners' round-0 actions, i.e. from the first stage's data); the next step's rows follow from
// the second stage.  Two round trips per step, 64 agents per wave (16 scenarios x 4).
//
//   hipcc --offload-arch=gfx950 -O3 -o ubench_gather ubench_gather.hip
//   ./ubench_gather [tables=8192] [pool=381] [rps=5] [steps=96] [lanes=32] [launches=20] [pair=0] [stages=1]
// stages=3: the prefetch study (chase_pf): kernel_us / cycles_per_step without the prefetch, the
// l1_pool1_* fields WITH it (same pool)
// prints one JSON line: kernel us per launch (median of the last half), cycles per step (s_memtime of
// each wave, averaged), the same with an L1-resident pool of 1 row (the ALU + L1 part of the step).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

constexpr uint32_t kStates = 160000;  // 20^4 rows per table
constexpr uint32_t kRowBytes = 32;    // 4 f64 (3 actions + pad)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__global__ void fill_tables(uint32_t* q, size_t n_words, uint32_t seed) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_words; k += (size_t)gridDim.x * blockDim.x)
    q[k] = mix((uint32_t)k ^ mix((uint32_t)(k >> 32) + seed));
}

// pool slot k of agent a -> a row of its table (distinct for k < pool with high probability)
__device__ __forceinline__ uint32_t pool_row(uint32_t a, uint32_t k) {
  return (uint32_t)(((uint64_t)mix(k * 0x9E3779B9u + a * 0x85EBCA6Bu + 1u) * kStates) >> 32);
}

// PAIR: two adjacent lanes per agent, each loading one 16-B half of the row (one dwordx4 per row
// instead of dwordx4 + dwordx2 per lane); `lanes` then counts agents, 2 * lanes <= 64
template <int RPS, bool PAIR>
__global__ __launch_bounds__(64) void chase(const char* __restrict__ q, int lanes, uint32_t pool, int steps,
                                            uint32_t* __restrict__ sink, unsigned long long* __restrict__ cyc) {
  const int lane = (int)threadIdx.x;
  const int ag = PAIR ? lane >> 1 : lane;
  const bool active = ag < lanes;
  const uint32_t a = (uint32_t)(blockIdx.x * lanes + (active ? ag : 0));
  // the kernel's addressing: SGPR base of the wave's first table + a 32-bit lane offset
  const char* const qwave = q + (size_t)blockIdx.x * lanes * kStates * kRowBytes;
  const uint32_t qlane = (active ? (uint32_t)ag * kStates * kRowBytes : 0u) + (PAIR ? 16u * (uint32_t)(lane & 1) : 0u);
  uint32_t h = mix(a + 12345u);
  uint32_t acc = 0;
  unsigned long long t0;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int t = 0; t < steps; ++t) {
    uint4 lo[RPS];
    uint2 hi[RPS];
#pragma unroll
    for (int r = 0; r < RPS; ++r) {
      const uint32_t k = (uint32_t)(((uint64_t)(h + (uint32_t)r * 97u) * pool) >> 32);
      const char* p = qwave + (qlane + pool_row(a, k) * kRowBytes);
      lo[r] = *reinterpret_cast<const uint4*>(p);
      if (!PAIR) hi[r] = *reinterpret_cast<const uint2*>(p + 16);
    }
    uint32_t x = (uint32_t)t;
#pragma unroll
    for (int r = 0; r < RPS; ++r) {
      if (PAIR) {  // both halves in both lanes of the pair (a DPP swap, as an argmax over the row needs)
        const uint32_t o = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo[r].x, 0xB1, 0xF, 0xF, false);
        x ^= ((lane & 1) ? o ^ lo[r].y : lo[r].x ^ o);
      } else {
        x ^= lo[r].x ^ lo[r].w ^ hi[r].y;
      }
    }
    h = mix(x);
    acc += h;
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  sink[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// two dependent gather stages per step: 2 rows, then 1 row addressed from their data (configs[3])
__global__ __launch_bounds__(64) void chase2(const char* __restrict__ q, int lanes, uint32_t pool, int steps,
                                             uint32_t* __restrict__ sink, unsigned long long* __restrict__ cyc) {
  const int lane = (int)threadIdx.x;
  const bool active = lane < lanes;
  const uint32_t a = (uint32_t)(blockIdx.x * lanes + (active ? lane : 0));
  const char* const qwave = q + (size_t)blockIdx.x * lanes * kStates * kRowBytes;
  const uint32_t qlane = active ? (uint32_t)lane * kStates * kRowBytes : 0u;
  uint32_t h = mix(a + 12345u);
  uint32_t acc = 0;
  unsigned long long t0;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int t = 0; t < steps; ++t) {
    uint4 lo[2];
    uint2 hi[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint32_t k = (uint32_t)(((uint64_t)(h + (uint32_t)r * 97u) * pool) >> 32);
      const char* p = qwave + (qlane + pool_row(a, k) * kRowBytes);
      lo[r] = *reinterpret_cast<const uint4*>(p);
      hi[r] = *reinterpret_cast<const uint2*>(p + 16);
    }
    const uint32_t x0 = mix((uint32_t)t ^ lo[0].x ^ lo[0].w ^ hi[0].y);  // round 0 -> the round-1 row
    const uint32_t k1 = (uint32_t)(((uint64_t)x0 * pool) >> 32);
    const char* p1 = qwave + (qlane + pool_row(a, k1) * kRowBytes);
    const uint4 lo1 = *reinterpret_cast<const uint4*>(p1);
    const uint2 hi1 = *reinterpret_cast<const uint2*>(p1 + 16);
    h = mix(x0 ^ lo1.x ^ lo1.w ^ hi1.y ^ lo[1].y ^ hi[1].x);
    acc += h;
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  sink[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// configs[1] with a one-step-ahead prefetch (stages=3 selects it; PF = 0 measures the same access
// pattern without the prefetch): each step's 5 rows are one of 3 candidate sets, picked by a 2-bit
// choice from the previous step's data (the final action: which of 3 next temperature bins).  With
// PF, one dword of every candidate row of step t + 1 (15 loads) is issued together with step t's own
// rows, just before them, so by the time step t + 1's choice is known its rows are in L2 -- if the
// candidates can be known a step ahead, as the next T_in / bins for each action are in
// episode_fast_kernel.  The prefetched dwords are ordinary loads the compiler tracks, folded into the
// result right after the step's rows are waited for (the in-order vmcnt has them complete then: they
// are older).  Round 4's form was an inline-asm global_load_dword into a VGPR the compiler did not
// know was in flight (it could reuse the register under the pending load: the fault of
// profiles/r05_ab/helper_prefetch_ab.txt), and loads whose values are kept across a step make the
// compiler copy (and so wait for) them, or wait for them before the step's rows (global_load_lds):
// neither measured the schedule under study.  This one issues them in the same batch as the rows.
template <bool PF>
__global__ __launch_bounds__(64) void chase_pf(const char* __restrict__ q, int lanes, uint32_t pool, int steps,
                                               uint32_t* __restrict__ sink, unsigned long long* __restrict__ cyc) {
  const int lane = (int)threadIdx.x;
  const bool active = lane < lanes;
  const uint32_t a = (uint32_t)(blockIdx.x * lanes + (active ? lane : 0));
  const char* const qwave = q + (size_t)blockIdx.x * lanes * kStates * kRowBytes;
  const uint32_t qlane = active ? (uint32_t)lane * kStates * kRowBytes : 0u;
  // candidate set c of step t: rows pool_row(a, k) with k = hash(t, c, r) (known ahead; the choice is not)
  auto row_of = [&](int t, uint32_t c, int r) {
    const uint32_t k = (uint32_t)(((uint64_t)mix((uint32_t)t * 0x9E3779B9u + c * 0x632BE5ABu + (uint32_t)r * 97u) * pool) >> 32);
    return qwave + (qlane + pool_row(a, k) * kRowBytes);
  };
  uint32_t choice = mix(a) % 3u;
  uint32_t acc = 0, pfacc = 0;
  uint4 lo[5];
  uint2 hi[5];
  uint32_t pf[15];
  // step t's batch: the prefetch of step t + 1's candidates (PF), then step t's chosen rows
  auto issue = [&](int t) {
    if (PF) {
      const int tn = t + 1 < steps ? t + 1 : 0;
#pragma unroll
      for (uint32_t c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 5; ++r) pf[c * 5 + r] = *reinterpret_cast<const uint32_t*>(row_of(tn, c, r));
    }
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const char* p = row_of(t, choice, r);
      lo[r] = *reinterpret_cast<const uint4*>(p);
      hi[r] = *reinterpret_cast<const uint2*>(p + 16);
    }
  };
  unsigned long long t0;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  issue(0);
  for (int t = 0; t < steps; ++t) {
    uint32_t x = (uint32_t)t;
#pragma unroll
    for (int r = 0; r < 5; ++r) x ^= lo[r].x ^ lo[r].w ^ hi[r].y;
    if (PF) {
#pragma unroll
      for (int k = 0; k < 15; ++k) pfacc ^= pf[k];
    }
    const uint32_t h = mix(x);
    acc += h;
    choice = h % 3u;  // the final action picks the next step's candidate set
    if (t + 1 < steps) issue(t + 1);
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  sink[blockIdx.x * 64 + lane] = acc + (pfacc & 1u);
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// configs[1] as a LEAD-1 pipeline (stages=4): the next step's rows depend on this step's final action
// only through 3 options (the next T_in per heat-pump level), so all 3 candidate sets of step t + 1
// (3 x 5 rows) are loaded at the START of step t, a whole step before they are needed; step t then
// waits only for its own sets (loaded during step t - 1) and picks one by the previous step's choice.
// No dependent round trip remains on the step: the step time is the issue / memory-pipeline cost of
// 30 scattered loads per lane and step.  Registers: 2 x 15 rows.
__global__ __launch_bounds__(64) void chase_lead(const char* __restrict__ q, int lanes, uint32_t pool, int steps,
                                                 uint32_t* __restrict__ sink, unsigned long long* __restrict__ cyc) {
  const int lane = (int)threadIdx.x;
  const bool active = lane < lanes;
  const uint32_t a = (uint32_t)(blockIdx.x * lanes + (active ? lane : 0));
  const char* const qwave = q + (size_t)blockIdx.x * lanes * kStates * kRowBytes;
  const uint32_t qlane = active ? (uint32_t)lane * kStates * kRowBytes : 0u;
  // option x of step t on the known state `base`: pool slot k = (hash(t, base) + 37 x + 7 r) mod pool,
  // row = (rowbase + 311 k) mod 20^4: a few ALU ops per row, like the kernel's strip + bin offsets
  // (one hash per step and option set, not per row)
  const uint32_t rowbase = pool_row(a, 0);
  auto row_of = [&](int t, uint32_t base, uint32_t x, int r) {
    const uint32_t th = mix((uint32_t)t * 0x9E3779B9u + base * 0x27D4EB2Fu);
    const uint32_t k = (th + x * 37u + (uint32_t)r * 7u) & (pool - 1u);  // pool: a power of two <= 512
    const uint32_t row = rowbase + k * 311u;                               // < 2 x 20^4
    return qwave + (qlane + (row >= kStates ? row - kStates : row) * kRowBytes);
  };
  uint32_t c = mix(a) % 3u, base = mix(a + 7u);
  uint32_t acc = 0;
  uint4 loA[3][5], loB[3][5];
  uint2 hiA[3][5], hiB[3][5];
  auto load_sets = [&](uint4 (&lo)[3][5], uint2 (&hi)[3][5], int t, uint32_t b) {
#pragma unroll
    for (uint32_t x = 0; x < 3; ++x)
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        const char* p = row_of(t, b, x, r);
        lo[x][r] = *reinterpret_cast<const uint4*>(p);
        hi[x][r] = *reinterpret_cast<const uint2*>(p + 16);
      }
  };
  auto use_set = [&](uint4 (&lo)[3][5], uint2 (&hi)[3][5], int t) {
    // the chosen set by masks, so every loaded value is consumed (a select would let the compiler
    // sink the three loads into one load of the selected address: a dependent gather again)
    const uint32_t m0 = 0u - (uint32_t)(c == 0), m1 = 0u - (uint32_t)(c == 1), m2 = 0u - (uint32_t)(c == 2);
    uint32_t x = (uint32_t)t;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      x ^= ((lo[0][r].x ^ lo[0][r].w ^ hi[0][r].y) & m0) | ((lo[1][r].x ^ lo[1][r].w ^ hi[1][r].y) & m1) |
           ((lo[2][r].x ^ lo[2][r].w ^ hi[2][r].y) & m2);
    }
    const uint32_t hsh = mix(x);
    acc += hsh;
    base = base * 31u + c;  // the state the next options hang on (known once c is)
    c = hsh % 3u;
  };
  unsigned long long t0;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  load_sets(loA, hiA, 0, base);
  int t = 0;
  for (; t + 2 <= steps; t += 2) {
    load_sets(loB, hiB, t + 1, base * 31u + c);  // step t + 1's options, issued before step t's wait
    use_set(loA, hiA, t);
    if (t + 2 < steps) load_sets(loA, hiA, t + 2, base * 31u + c);
    use_set(loB, hiB, t + 1);
  }
  if (t < steps) use_set(loA, hiA, t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  sink[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int RPS, bool PAIR>
static void run(const char* q, int blocks, int lanes, uint32_t pool, int steps, int launches, uint32_t* sink,
                unsigned long long* cyc, double& us_med, double& cyc_step) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> us;
  std::vector<unsigned long long> hc(blocks);
  double cs = 0.0;
  int nc = 0;
  for (int l = 0; l < launches; ++l) {
    CK(hipEventRecord(e0));
    if constexpr (RPS == 0)
      hipLaunchKernelGGL(chase2, dim3(blocks), dim3(64), 0, 0, q, lanes, pool, steps, sink, cyc);
    else if constexpr (RPS == -1)
      hipLaunchKernelGGL(chase_pf<false>, dim3(blocks), dim3(64), 0, 0, q, lanes, pool, steps, sink, cyc);
    else if constexpr (RPS == -2)
      hipLaunchKernelGGL(chase_pf<true>, dim3(blocks), dim3(64), 0, 0, q, lanes, pool, steps, sink, cyc);
    else if constexpr (RPS == -3)
      hipLaunchKernelGGL(chase_lead, dim3(blocks), dim3(64), 0, 0, q, lanes, pool, steps, sink, cyc);
    else
      hipLaunchKernelGGL((chase<RPS, PAIR>), dim3(blocks), dim3(64), 0, 0, q, lanes, pool, steps, sink, cyc);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (l >= launches / 2) {
      us.push_back(ms * 1e3);
      CK(hipMemcpy(hc.data(), cyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      for (auto c : hc) cs += (double)c / steps;
      nc += blocks;
    }
  }
  std::sort(us.begin(), us.end());
  us_med = us[us.size() / 2];
  cyc_step = cs / nc;
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int tables = argc > 1 ? atoi(argv[1]) : 8192;
  const uint32_t pool = argc > 2 ? (uint32_t)atoi(argv[2]) : 381u;
  const int rps = argc > 3 ? atoi(argv[3]) : 5;
  const int steps = argc > 4 ? atoi(argv[4]) : 96;
  const int lanes = argc > 5 ? atoi(argv[5]) : 32;
  const int launches = argc > 6 ? atoi(argv[6]) : 20;
  const bool pair = argc > 7 && atoi(argv[7]) != 0;
  const int stages = argc > 8 ? atoi(argv[8]) : 1;
  if (tables <= 0 || lanes <= 0 || lanes > (pair ? 32 : 64) || tables % lanes || pool == 0 || steps <= 0 || launches < 2 ||
      (size_t)lanes * kStates * kRowBytes >= (1ull << 32) || !(rps == 1 || rps == 5) || stages < 1 || stages > 4 ||
      (stages >= 2 && pair)) {
    fprintf(stderr, "bad arguments\n");
    return 2;
  }
  const int blocks = tables / lanes;
  const size_t bytes = (size_t)tables * kStates * kRowBytes;
  char* q = nullptr;
  uint32_t* sink = nullptr;
  unsigned long long* cyc = nullptr;
  CK(hipMalloc(&q, bytes));
  CK(hipMalloc(&sink, (size_t)blocks * 64 * sizeof(uint32_t)));
  CK(hipMalloc(&cyc, (size_t)blocks * sizeof(unsigned long long)));
  hipLaunchKernelGGL(fill_tables, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(q), bytes / 4, 7u);
  CK(hipDeviceSynchronize());
  double us = 0, cs = 0, us1 = 0, cs1 = 0;
  if (stages == 2) {
    run<0, false>(q, blocks, lanes, pool, steps, launches, sink, cyc, us, cs);
    run<0, false>(q, blocks, lanes, 1u, steps, launches, sink, cyc, us1, cs1);
  } else if (stages == 3) {  // 3 candidate sets per step, no prefetch (us) / with prefetch (us1)
    run<-1, false>(q, blocks, lanes, pool, steps, launches, sink, cyc, us, cs);
    run<-2, false>(q, blocks, lanes, pool, steps, launches, sink, cyc, us1, cs1);
  } else if (stages == 4) {  // the lead-1 pipeline (us) and the same with an L1-resident pool (us1)
    if ((pool & (pool - 1)) || pool > 512) {
      fprintf(stderr, "stages=4: pool must be a power of two <= 512\n");
      return 2;
    }
    run<-3, false>(q, blocks, lanes, pool, steps, launches, sink, cyc, us, cs);
    run<-3, false>(q, blocks, lanes, 1u, steps, launches, sink, cyc, us1, cs1);
  } else if (rps == 5 && !pair) {
    run<5, false>(q, blocks, lanes, pool, steps, launches, sink, cyc, us, cs);
    run<5, false>(q, blocks, lanes, 1u, steps, launches, sink, cyc, us1, cs1);
  } else if (rps == 5) {
    run<5, true>(q, blocks, lanes, pool, steps, launches, sink, cyc, us, cs);
    run<5, true>(q, blocks, lanes, 1u, steps, launches, sink, cyc, us1, cs1);
  } else if (!pair) {
    run<1, false>(q, blocks, lanes, pool, steps, launches, sink, cyc, us, cs);
    run<1, false>(q, blocks, lanes, 1u, steps, launches, sink, cyc, us1, cs1);
  } else {
    run<1, true>(q, blocks, lanes, pool, steps, launches, sink, cyc, us, cs);
    run<1, true>(q, blocks, lanes, 1u, steps, launches, sink, cyc, us1, cs1);
  }
  printf("{\"probe\": \"ubench_gather\", \"tables\": %d, \"table_bytes\": %zu, \"pool_rows\": %u, \"rows_per_step\": %d, "
         "\"stages\": %d, \"steps\": %d, \"agents_per_wave\": %d, \"pair_lanes\": %d, \"waves\": %d, \"launches\": %d, "
         "\"kernel_us\": %.2f, \"cycles_per_step\": %.1f, \"l1_pool1_kernel_us\": %.2f, \"l1_pool1_cycles_per_step\": %.1f}\n",
         tables, bytes, pool, stages == 2 ? 3 : rps, stages, steps, lanes, pair ? 1 : 0, blocks, launches, us, cs, us1, cs1);
  CK(hipFree(q));
  CK(hipFree(sink));
  CK(hipFree(cyc));
  return 0;
}
