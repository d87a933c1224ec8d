// p2pmg_kernels.hip — gfx950 kernels for the P2PMicrogrid hot path.
//
// Build flags that are part of the numerics contract:
//   -ffp-contract=off   every f32/f64 op rounds separately, as TF eager and NumPy do
//   (default)           correctly-rounded f32 division, f32 denormals kept
//
// Layout (HBM):
//   prof  [T][A] float2 {load_w, pv_w}   time-major: one coalesced 8-B load per lane per step
//   env   [S_env][T][8] f32              time, t_out, buy, inj, p2p (shared when S_env == 1)
//   q     [A][n_states][4] f64|f32       per-agent table, rows padded 3 -> 4 actions so a
//                                        greedy gather is ONE aligned 32-B (f64) / 16-B (f32) sector
//   t_in, t_m, max_in [A] f32            register-resident across the whole episode
// Mapping: one lane per agent; a scenario's N agents occupy a lane group of G = pow2ceil(N)
// lanes inside one wave (64 / G scenarios per wave, one wave per workgroup); the Jacobi
// proposal matrix P never leaves the chip — each lane keeps its row in registers and reads
// its column through a per-wave LDS tile (community.py:75-86).
#include <hip/hip_ext.h>

#include <algorithm>
#include <type_traits>

#include "p2pmg_internal.h"

// The file is compiled once per part (-DP2PMG_PART=k, in parallel by _build.py); each part defines
// a disjoint subset of the launchers below, so each template kernel is instantiated in one part only.
//   0: small kernels + dispatchers   1-4: episode_fast_kernel, N = 1-2 / 3-4 / 5-6 / 7-8
//   5: episode_sq16_kernel           6-8: episode_kernel, N = 1-4 / 5-8 / 16
//   9-10: episode_kernel's LDS-tile form, up to 16 / 32 and 64 agents
// Without -DP2PMG_PART everything is in one translation unit.
#ifndef P2PMG_PART
#define P2PMG_PART -1
#endif
#define P2PMG_IN_PART(k) (P2PMG_PART < 0 || P2PMG_PART == (k))

namespace p2pmg {
namespace {

#include "p2pmg_device.h"

template <typename QT>
struct Row4 {
  QT v[4];
};

// x[a] for a in {0,1,2} as two v_cndmask: written in asm because hipcc turns a select chain
// on a runtime index into a scratch/LDS lookup table (a memory round trip + vmcnt(0) drain)
// 3-way select by a per-lane index a in {0, 1, 2}, as asm so that hipcc never turns it into a
// scratch-indexed array.  The two lane masks are separate (non-volatile) asm: every select on the
// same index shares them (CSE), e.g. the six 32-bit halves of a selected f64 row.
struct Sel3M {
  uint64_t m1, m2;
};
__device__ __forceinline__ Sel3M sel3_masks(int a) {
  uint64_t m1, m2;
  asm("v_cmp_eq_u32_e64 %0, 1, %1" : "=s"(m1) : "v"(a));
  asm("v_cmp_eq_u32_e64 %0, 2, %1" : "=s"(m2) : "v"(a));
  return Sel3M{m1, m2};
}
__device__ __forceinline__ float sel3(const Sel3M& m, float x0, float x1, float x2) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3\n\tv_cndmask_b32_e64 %0, %0, %4, %5"
      : "=&v"(r)
      : "v"(x0), "v"(x1), "s"(m.m1), "v"(x2), "s"(m.m2));
  return r;
}
__device__ __forceinline__ double sel3(const Sel3M& m, double x0, double x1, double x2) {
  const uint64_t b0 = (uint64_t)__double_as_longlong(x0), b1 = (uint64_t)__double_as_longlong(x1),
                 b2 = (uint64_t)__double_as_longlong(x2);
  const uint32_t lo = __float_as_uint(sel3(m, __uint_as_float((uint32_t)b0), __uint_as_float((uint32_t)b1),
                                           __uint_as_float((uint32_t)b2)));
  const uint32_t hi = __float_as_uint(sel3(m, __uint_as_float((uint32_t)(b0 >> 32)),
                                           __uint_as_float((uint32_t)(b1 >> 32)),
                                           __uint_as_float((uint32_t)(b2 >> 32))));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <typename T>
__device__ __forceinline__ T sel3(int a, T x0, T x1, T x2) {
  return sel3(sel3_masks(a), x0, x1, x2);
}
// Timing-only ablation builds (scripts/dev/latency_ablation.py): -DP2PMG_ABLATE=1 replaces the
// episode kernel's Q-row gathers by values derived from the address (no memory access),
// -DP2PMG_ABLATE=2 replaces f32 divisions by reciprocal multiplies; in the fast kernel =8 fakes the
// next step's rows, =9 cuts the TD -> next-step patch dependency, =10 both, =11 drops the final
// round's divide-power and the market (the cost from the net power alone).  Never shipped.
#ifndef P2PMG_ABLATE
#define P2PMG_ABLATE 0
#endif
#if P2PMG_ABLATE == 2
#define FDIV(a, b) ((a) * __frcp_rn(b))
#else
#define FDIV(a, b) ((a) / (b))
#endif
__device__ __forceinline__ Row4<double> load_row(const double* p) {
  const double2 a = *reinterpret_cast<const double2*>(p);
  const double2 b = *reinterpret_cast<const double2*>(p + 2);
  return Row4<double>{{a.x, a.y, b.x, b.y}};
}
__device__ __forceinline__ Row4<float> load_row(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  return Row4<float>{{a.x, a.y, a.z, a.w}};
}
// argmax over 3 actions, first max wins (rl.py:116)
template <typename QT>
__device__ __forceinline__ int argmax3(const Row4<QT>& r) {
  int a = 0;
  QT b = r.v[0];
  if (r.v[1] > b) { b = r.v[1]; a = 1; }
  if (r.v[2] > b) { a = 2; }
  return a;
}
// max over 3 actions (rl.py:127, np.max): two v_max.  Table entries are never NaN and never -0
// (tables start at +0 and a TD step q + alpha * d is +0 when q = +0 and d = -0), so the value is
// the sequential compare's
template <typename QT>
__device__ __forceinline__ QT max3(const Row4<QT>& r) {
  return fmax(fmax(r.v[0], r.v[1]), r.v[2]);
}
// QActor.train rl.py:125-129 under NumPy 2: f64 TD arithmetic on double(reward)
__device__ __forceinline__ double td_update(double qsa, float rw, double qmax, double alpha, double gamma) {
  return qsa + alpha * (((double)rw + gamma * qmax) - qsa);
}
__device__ __forceinline__ float td_update(float qsa, float rw, float qmax, double alpha, double gamma) {
  return qsa + (float)alpha * ((rw + (float)gamma * qmax) - qsa);
}

// ----------------------------------------------------------------- scenario-group exchange
// Lane i of a scenario group owns row i of the proposal matrix P.  exchange() gives every lane
// its column: col[j] = P[j][i].  G <= 8: cross-lane shuffles (no LDS, no barrier — a
// __syncthreads() would also drain every in-flight global load with vmcnt(0)).  G = 16: a
// per-wave LDS tile ordered by wavefront-scope fences (one wave per workgroup, DS ops of a
// wave execute in order).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// xor-shuffle inside a lane group: DPP quad_perm for partners within a quad (a VALU op),
// ds_bpermute beyond
template <int D>
__device__ __forceinline__ float shfl_xor_c(float v) {
  if constexpr (D == 1) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  } else if constexpr (D == 2) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  } else if constexpr (D == 3) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x1B, 0xF, 0xF, false));  // [3,2,1,0]
  } else {
    return __shfl_xor(v, D, 64);
  }
}

template <int N, int D>
__device__ __forceinline__ void exchange_step(const float (&row)[N], float (&col)[N], int i) {
  const int src = i ^ D;  // partner lane in the group; it sends its row[i]
  float v = 0.0f;
#pragma unroll
  for (int k = 0; k < N; ++k) v = (k == src) ? row[k] : v;  // what my partner wants: row[src]
  const float got = shfl_xor_c<D>(v);
#pragma unroll
  for (int k = 0; k < N; ++k) col[k] = (k == src) ? got : col[k];
}

template <int N, int D, int G>
__device__ __forceinline__ void exchange_all(const float (&row)[N], float (&col)[N], int i) {
  if constexpr (D < G) {
    exchange_step<N, D>(row, col, i);
    exchange_all<N, D + 1, G>(row, col, i);
  }
}

template <int N>
__device__ __forceinline__ void exchange(const float (&row)[N], float (&col)[N], int i, int sl, float* sh) {
  constexpr int G = pow2ceil(N);
  if constexpr (G <= 8) {
#pragma unroll
    for (int k = 0; k < N; ++k) col[k] = (k == i) ? row[k] : 0.0f;
    exchange_all<N, 1, G>(row, col, i);
  } else {
    if (i < N) {
#pragma unroll
      for (int j = 0; j < N; ++j) sh[(sl * N + i) * N + j] = row[j];
    }
    wave_lds_fence();
    if (i < N) {
#pragma unroll
      for (int j = 0; j < N; ++j) col[j] = sh[(sl * N + j) * N + i];
    }
    wave_lds_fence();
  }
}

// sum_{j=0..N-1} v_j over the scenario group, sequential from +0.0 (canonical order)
template <int N>
__device__ __forceinline__ float group_sum(float v, int lane, int i, int sl, float* sh) {
  constexpr int G = pow2ceil(N);
  float m = 0.0f;
  if constexpr (G == 1) {
    m = m + v;
  } else if constexpr (G == 2) {
    const float o = shfl_xor_c<1>(v);
    m = m + (i == 0 ? v : o);
    m = m + (i == 0 ? o : v);
  } else if constexpr (G <= 8) {
    const int base = lane - i;
#pragma unroll
    for (int k = 0; k < N; ++k) m = m + __shfl(v, base + k, 64);
  } else {
    if (i < N) sh[sl * N + i] = v;
    wave_lds_fence();
#pragma unroll
    for (int k = 0; k < N; ++k) m = m + sh[sl * N + k];
    wave_lds_fence();
  }
  return m;
}

struct EnvRow {
  float time, t_out, buy, inj, p2p;
};
// {t_out, buy, inj, p2p} of an env row as one 16-B load (the fast kernel's input ring)
typedef float EnvV __attribute__((ext_vector_type(4)));
__device__ __forceinline__ EnvV load_envv(const float* e) {
  EnvV v;
  __builtin_memcpy(&v, e + 1, sizeof(v));
  return v;
}
__device__ __forceinline__ EnvRow load_env(const float* e) {
  const float4 v = *reinterpret_cast<const float4*>(e);
  return EnvRow{v.x, v.y, v.z, v.w, e[4]};
}

// Loop constants pinned in VGPRs.  The kernel-argument struct has ~60 fields: left in SGPRs
// they overflow the scalar file and hipcc reloads them from VGPR lanes (v_readlane) on the
// step's dependency chain.  An opaque v_mov at entry makes each one a VGPR for the whole
// episode (one wave per SIMD leaves ample VGPRs).
__device__ __forceinline__ float vpin(float x) {
  float r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ int vpin(int x) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ double vpin(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  const uint32_t lo = (uint32_t)vpin((int)(uint32_t)b), hi = (uint32_t)vpin((int)(uint32_t)(b >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
struct KC {
  float setpoint, margin, lower, upper;
  float inv_ci, inv_cm, inv_ri, inv_re, inv_rvent, c_in, c_m, solar, cop, spm, slot;
  float mph, kilo, penw;
  double alpha, gamma;
  int nt, nT, nb, np;
};
__device__ __forceinline__ KC pin_constants(const EpisodeParams& p) {
  KC k;
  k.setpoint = vpin(p.setpoint); k.margin = vpin(p.margin); k.lower = vpin(p.lower); k.upper = vpin(p.upper);
  k.inv_ci = vpin(p.inv_ci); k.inv_cm = vpin(p.inv_cm); k.inv_ri = vpin(p.inv_ri); k.inv_re = vpin(p.inv_re);
  k.inv_rvent = vpin(p.inv_rvent); k.c_in = vpin(p.c_in); k.c_m = vpin(p.c_m); k.solar = vpin(p.solar);
  k.cop = vpin(p.cop); k.spm = vpin(p.spm); k.slot = vpin(p.slot); k.mph = vpin(p.mph); k.kilo = vpin(p.kilo);
  k.penw = vpin(p.penw);
  k.alpha = vpin(p.alpha); k.gamma = vpin(p.gamma);
  k.nt = vpin(p.nt); k.nT = vpin(p.nT); k.nb = vpin(p.nb); k.np = vpin(p.np);
  return k;
}

// The same constants left to the compiler (kernel arguments stay in SGPRs): the throughput-bound
// sq16 kernel runs several waves per SIMD, where VGPRs, not the scalar-operand latency, set the pace.
__device__ __forceinline__ KC scalar_constants(const EpisodeParams& p) {
  return KC{p.setpoint, p.margin, p.lower, p.upper, p.inv_ci, p.inv_cm, p.inv_ri, p.inv_re, p.inv_rvent,
            p.c_in,     p.c_m,    p.solar, p.cop,   p.spm,    p.slot,   p.mph,    p.kilo,   p.penw,
            p.alpha,    p.gamma,  p.nt,    p.nT,    p.nb,     p.np};
}

// Everything about step t that is known before its negotiation starts.
struct StepIdx {
  float bal;        // (load - pv) / max_in of this step    agent.py:172-176
  float baln;       // ... of the next step (= next step's bal)
  int it, iT, ib;   // s indices except p2p                 rl.py:89-95
  uint32_t strip;   // row of (it, iT, ib, 0) in the agent's table
  uint32_t nrow;    // next-state row (time_{t+1}, same T_in, bal_{t+1}, p2p = 0)  agent.py:293-296
};
// Q-table dimensions: the reference's 20 x 20 x 20 x 20 (agent.py:258-261) compile to shifts and
// adds; other sizes use the runtime values
template <bool B20>
struct Dims {
  int nt, nT, nb, np;
  __device__ __forceinline__ int t() const { return B20 ? 20 : nt; }
  __device__ __forceinline__ int T() const { return B20 ? 20 : nT; }
  __device__ __forceinline__ int b() const { return B20 ? 20 : nb; }
  __device__ __forceinline__ int p() const { return B20 ? 20 : np; }
};

template <bool B20>
__device__ __forceinline__ StepIdx make_step(const KC& p, const Dims<B20>& D, bool margin_one, float time_t,
                                             float time_n, float bal, float2 f_n, float tin, float mi, int ip_zero) {
  StepIdx st;
  st.bal = bal;
  st.baln = FDIV(f_n.x - f_n.y, mi);
  const float dt = tin - p.setpoint;  // heating.py:118-120 (x / 1.0 == x exactly)
  const float tnorm = margin_one ? dt : dt / p.margin;
  st.it = idx_time(time_t, D.t());
  st.iT = idx_temp(tnorm, D.T());
  st.ib = idx_plain(bal, D.b());
  st.strip = (uint32_t)(((st.it * D.T() + st.iT) * D.b() + st.ib) * D.p());
  const int itn = idx_time(time_n, D.t());
  const int ibn = idx_plain(st.baln, D.b());
  st.nrow = (uint32_t)(((itn * D.T() + st.iT) * D.b() + ibn) * D.p() + ip_zero);
  return st;
}

// Philox exploration codes of every round of step t (p2pmg_device.h::philox_step_codes, layout
// oracle/philox.py::decision_draws): byte r = code of round r, 255 = greedy (QActor.select_action
// rl.py:100-111)
__device__ __forceinline__ uint64_t philox_codes_of(const EpisodeParams& p, int t, uint32_t gid) {
  return philox_step_codes(t, p.R + 1, (uint32_t)p.episode, gid, p.eps_thr, p.eps_all, p.seed_lo, p.seed_hi);
}

// all rounds' codes of step t packed one byte per round (round r in bits 8r..8r+7)
// The code-word buffer always exists (greedy runs read and ignore it), so the loads are
// unconditional and branch-free: a load whose destination is touched under a branch before
// its use is waited for at that branch.  The in-kernel Philox words are built separately.
struct CodeWords {
  uint32_t w0, w1;  // loaded words
  uint64_t gen;     // in-kernel Philox word (p.rng == 1)
};
__device__ __forceinline__ CodeWords step_codes(const EpisodeParams& p, const uint32_t* codes_a, size_t off, int t,
                                                int a, int W, bool gen = true) {
  // code words [T][W][A] (replay upload or Philox pre-pass); off = t * W * A
  CodeWords c;
  c.w0 = codes_a[off];
  c.w1 = codes_a[W > 1 ? off + (size_t)p.A : off];
  c.gen = ~0ull;
  if (gen && p.rng == 1) c.gen = philox_codes_of(p, t, p.agent_offset + (uint32_t)a);
  return c;
}
__device__ __forceinline__ uint64_t code_word(const EpisodeParams& p, const CodeWords& c, bool active) {
  const int R1 = p.R + 1;
  uint64_t w = (uint64_t)c.w0 | ((R1 > 4 ? (uint64_t)c.w1 : 0xFFFFFFFFull) << 32);
  w |= (R1 < 8 ? ~0ull << (8 * R1) : 0ull);
  if (p.rng == 1) w = c.gen;
  return (p.mode != 0 || !active) ? ~0ull : w;
}

// the sq16 kernel's code word: its TRAIN launches are exactly p.mode == 0 (launch_sq16_nw), and a
// masked-off lane's draws reach only its dummy stores, so no per-lane mask stays live in the loop
template <bool TRAIN>
__device__ __forceinline__ uint64_t code_word_t(const EpisodeParams& p, const CodeWords& c) {
  if constexpr (!TRAIN) return ~0ull;
  const int R1 = p.R + 1;
  uint64_t w = (uint64_t)c.w0 | ((R1 > 4 ? (uint64_t)c.w1 : 0xFFFFFFFFull) << 32);
  w |= (R1 < 8 ? ~0ull << (8 * R1) : 0ull);
  if (p.rng == 1) w = c.gen;
  return w;
}

// A TD store can hit a row whose prefetch was issued before it.  The prefetched registers
// are not touched (that would force a wait for the load); the patch is applied at use.
template <typename QT>
struct Patch {
  uint32_t row;  // 0xFFFFFFFF = none
  int act;
  QT val;
};
template <typename QT>
__device__ __forceinline__ Row4<QT> sel_row(int b, const Row4<QT>& x0, const Row4<QT>& x1, const Row4<QT>& x2) {
  Row4<QT> r;
  const Sel3M m = sel3_masks(b);
#pragma unroll
  for (int k = 0; k < 3; ++k) r.v[k] = sel3(m, x0.v[k], x1.v[k], x2.v[k]);
  r.v[3] = (QT)0;
  return r;
}
template <typename QT>
__device__ __forceinline__ Row4<QT> patched(Row4<QT> r, uint32_t addr, const Patch<QT>& pt) {
  if (pt.row == addr) {
#pragma unroll
    for (int k = 0; k < 3; ++k) r.v[k] = (pt.act == k) ? pt.val : r.v[k];
  }
  return r;
}

// heat-pump power of an action without a dynamically indexed kernarg array (that compiles to
// a global load + vmcnt(0) on the critical path)
__device__ __forceinline__ float hp_of(const float4& lv, int act) { return sel3(act, lv.x, lv.y, lv.z); }

// community.py:45-54's bilateral exchange of one pair, sign(pij) * min(|pij|, |pji|) where the
// signs differ and 0 where they agree, as ONE v_med3(pij, -pji, 0): with opposite signs pij and
// -pji share a sign and the median of {0, pij, -pji} is the one nearer 0 (min for positives, max
// for negatives); with equal signs 0 lies between them.  Where the reference's value is 0 the
// median may be -0 instead of +0 (and vice versa): the market sums g and pp start at +0, and
// adding a zero of either sign to a sum that starts at +0 never changes its value, so g, pp and
// everything downstream are the same.  (Operands are never NaN.)
__device__ __forceinline__ float pair_exchange(float pij, float pji) {
  return __builtin_amdgcn_fmed3f(pij, -pji, 0.0f);
}
// _divide_power's numerator out * |f_j| (agent.py:193) as (-|out|) * f_j: the filter keeps f_j <= 0
// for out > 0 and f_j >= 0 for out < 0, so f_j = -sign(out) |f_j| and the two products are the same
// IEEE product up to the sign of a zero (out = 0 or f_j = 0: a zero quotient either way); one
// hoisted -|out| replaces an |.| per column.
__device__ __forceinline__ float nabs_out(float out) { return -fabsf(out); }

// ----------------------------------------------------------------- the episode kernel
// One launch = one episode of T timesteps for every scenario (train_episode / run).
// Latency structure per step (one dependent Q gather per extra round):
//   * env rows, profiles and exploration codes are prefetched ahead;
//   * round 0 always sees P = 0, so its p2p index is the constant ip_zero and its Q row, like
//     the next-state row, is known as soon as the previous step's final action is: both are
//     issued right after that action, before the previous step's market/reward/TD work;
//   * a TD store that hits one of those prefetched rows patches the register copy.
// Shared-table variant: each workgroup sums its agents' int64 TD deltas for the whole episode in
// an LDS hash table (linear probing, ds_cmpst + ds_add_u64) and flushes one global atomic per
// occupied slot at the end.  All agents of a step share the time bin, so the episode's deltas
// hit only a few thousand entries: without the table, millions of same-address global atomics
// per step serialise.  Exact integer sums, so the grouping never changes the result.
constexpr int kSqWaves = 4;          // waves per workgroup
constexpr int kSqSlotBits = 11;      // 2048 slots: 8 KB keys + 16 KB sums
constexpr int kSqSlots = 1 << kSqSlotBits;
constexpr uint32_t kSqEmpty = 0xFFFFFFFFu;
constexpr int kSqProbes = 16;      // linear-probe limit before the global fallback
constexpr int kSqFlushSteps = 8;    // steps between flushes of the LDS table

__device__ __forceinline__ void lds_add_by_key(uint32_t* hk, unsigned long long* hv, uint32_t key, long long v,
                                               unsigned long long* gbase) {
  if (v == 0) return;
  uint32_t h = (key * 2654435761u) >> (32 - kSqSlotBits);
#pragma nounroll
  for (int probe = 0; probe < kSqProbes; ++probe) {
    const uint32_t prev = atomicCAS(hk + h, kSqEmpty, key);
    if (prev == kSqEmpty || prev == key) {
      atomicAdd(hv + h, (unsigned long long)v);
      return;
    }
    h = (h + 1) & (kSqSlots - 1);
  }
  atomicAdd(gbase + key, (unsigned long long)v);  // crowded run of slots: straight to the global replica
}
// Block-uniform: move the table's sums into the XCD's replica and empty it.  Called every
// kSqFlushSteps steps, not once per episode: a 32-scenario workgroup touches ~3.2k distinct
// (state, action) keys per 96-step episode (more than the 2048 slots) but only ~600 in any
// 8-step window, because the time bin moves on; the total number of global atomics grows by
// ~15 % while the table stays below a third full, so a probe run is ~1 slot long.
__device__ __forceinline__ void lds_hash_flush(uint32_t* hk, unsigned long long* hv, unsigned long long* gbase,
                                               int nthreads) {
  __syncthreads();
  for (int k2 = threadIdx.x; k2 < kSqSlots; k2 += nthreads) {
    const uint32_t key = hk[k2];
    if (key != kSqEmpty) {
      const long long x = (long long)hv[k2];
      if (x != 0) atomicAdd(gbase + key, (unsigned long long)x);
      hk[k2] = kSqEmpty;
      hv[k2] = 0;
    }
  }
  __syncthreads();
}

// timing-only ablations of the fast kernel's gathers: 7 = round-R gather fake, 8 = prefetched rows fake
template <typename QT>
__device__ __forceinline__ Row4<QT> fake_row(const QT* p) {
  const uint32_t x = (uint32_t)(reinterpret_cast<uintptr_t>(p) >> 5);
  return Row4<QT>{{(QT)(x & 3), (QT)((x >> 2) & 3), (QT)((x >> 4) & 3), (QT)0}};
}
template <typename QT>
__device__ __forceinline__ Row4<QT> gather_row(const QT* p) {
#if P2PMG_ABLATE == 1 || P2PMG_ABLATE == 4
  const uint32_t x = (uint32_t)(reinterpret_cast<uintptr_t>(p) >> 5);
  return Row4<QT>{{(QT)(x & 3), (QT)((x >> 2) & 3), (QT)((x >> 4) & 3), (QT)0}};
#else
  return load_row(p);
#endif
}
// The proposal matrix P of one scenario as the general kernel holds it (community.py:75-86): lane i
// owns row i; round r reads column i of round r - 1's P (Jacobi: every agent answers the previous
// round's proposals) and writes its new row; the market reads row i and column i of the final P.
//   PRegs<N>  N <= 16 compiled in: row and column in registers, the column by exchange<N>
//   PTile<NC> any community size n <= NC (16, 32, 64) at run time: the scenario's P in two LDS
//             tiles (the round being read, the round being written) with an odd row stride, so the
//             column read (lane i at j * stride + i) and the row read (lane i at i * stride + j) are
//             both conflict-free.  Every agent of a scenario is a lane of the same wave, so a
//             wavefront-scope fence orders the tiles (no workgroup barrier, no vmcnt drain).
template <int N>
struct PRegs {
  float row[N], col[N];
  float* sh;
  int i, sl;
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (int j = 0; j < N; ++j) { row[j] = 0.0f; col[j] = 0.0f; }
  }
  __device__ __forceinline__ void next_round() { exchange<N>(row, col, i, sl, sh); }
  __device__ __forceinline__ float colv(int j) const { return col[j]; }
  __device__ __forceinline__ float rowv(int j) const { return row[j]; }
  __device__ __forceinline__ void put(int j, float v) { row[j] = v; }
};
template <int NC>
struct PTile {
  static constexpr int kStride = NC + 1;
  static constexpr int kTile = NC * kStride;
  float* base;  // this scenario's two tiles
  int i, rd, wr;
  __device__ __forceinline__ void clear() {}  // round 0 reads no column (its powers are all -0)
  __device__ __forceinline__ void next_round() {
    wave_lds_fence();  // every lane's row of the round just written is visible
    rd = wr;
    wr ^= 1;
  }
  __device__ __forceinline__ float colv(int j) const { return base[rd * kTile + j * kStride + i]; }
  __device__ __forceinline__ float rowv(int j) const { return base[rd * kTile + i * kStride + j]; }
  __device__ __forceinline__ void put(int j, float v) { base[wr * kTile + i * kStride + j] = v; }
};
// sum_{k < n} v_k over a scenario group of run-time size n through LDS, sequential from +0.0
template <int NC>
__device__ __forceinline__ float group_sum_n(float v, int i, int sl, int n, float* sh) {
  if (i < n) sh[sl * NC + i] = v;
  wave_lds_fence();
  float m = 0.0f;
  for (int k = 0; k < n; ++k) m = m + sh[sl * NC + k];
  wave_lds_fence();
  return m;
}
// exploration code of round r >= 8 of step t (the 64-bit code word holds rounds 0..7): the replay
// word (r / 4) of the step, or Philox word k = t (R + 1) + r (p2pmg_device.h, oracle/philox.py)
__device__ __forceinline__ int late_code(const EpisodeParams& p, const uint32_t* codes_a, size_t step_off, int t,
                                         int r, int a, bool active) {
  if (p.mode != 0 || !active) return 255;
  if (p.rng == 1)
    return (int)philox_round_code(t, p.R + 1, r, (uint32_t)p.episode, p.agent_offset + (uint32_t)a, p.eps_thr,
                                  p.eps_all, p.seed_lo, p.seed_hi);
  return (int)((codes_a[step_off + (size_t)(r >> 2) * p.A] >> (8 * (r & 3))) & 0xFFu);
}
// workgroup shape of the general kernel: one wave, or (shared table) kSqWaves waves around one LDS
// delta hash; the 64-agent tiles (33 KB per wave) take two
template <int NC, bool WIDE, bool SQ>
constexpr int general_wpb() {
  return SQ ? ((WIDE && NC > 32) ? 2 : kSqWaves) : 1;
}

// episode_kernel<NC, WIDE, QT, B20, SQ>: WIDE = false: N = NC agents per scenario compiled in
// (PRegs); WIDE = true: n = p.N <= NC agents (PTile), the community sizes 9..15 and 17..64.  Both
// sum over j = 0..n-1 in order from +0.0 and divide by n as IEEE quotients, so a scenario gives the
// same bits either way (tests/test_gpu_parity.py runs the tile form at the register form's sizes).
template <int NC, bool WIDE, typename QT, bool B20, bool SQ>
__global__ __launch_bounds__((kWave * general_wpb<NC, WIDE, SQ>())) void episode_kernel(const EpisodeParams p) {
  constexpr int G = pow2ceil(NC);
  constexpr int SPW = kWave / G;
  constexpr int WPB = general_wpb<NC, WIDE, SQ>();  // waves per workgroup
  constexpr int PW = WIDE ? SPW * 2 * PTile<NC>::kTile : (G > 8 ? SPW * NC * NC : 1);
  constexpr int RW = (WIDE || G > 8) ? SPW * NC : 1;
  __shared__ float shPall[WPB * PW];
  __shared__ float shRall[WPB * RW];
  __shared__ uint32_t hkey[SQ ? kSqSlots : 1];
  __shared__ unsigned long long hval[SQ ? kSqSlots : 1];

  const int wv = SQ ? (int)(threadIdx.x / kWave) : 0;
  const int lane = SQ ? (int)(threadIdx.x % kWave) : (int)threadIdx.x;
  float* const shP = shPall + wv * PW;  // this wave's exchange tiles
  float* const shR = shRall + wv * RW;
  const int sl = lane / G;
  const int i = lane % G;
  const int n = WIDE ? p.N : NC;  // agents per scenario
  const float nf = (float)n;
  // x / n (mean over the community, the even split): div_n's power-of-two multiply is the IEEE quotient
  auto divn = [&](float x) -> float {
    if constexpr (WIDE) return x / nf;
    else return div_n<NC>(x);
  };
  const int s = (blockIdx.x * WPB + wv) * SPW + sl;
  const bool in_group = i < n;
  const bool active = in_group && (s < p.S);
  const int a = active ? s * n + i : 0;
  const int s_env = p.n_env == 1 ? 0 : (s < p.S ? s : 0);
  const int T = p.T;
  const int R1 = p.R + 1;
  const int W = (R1 + 3) >> 2;
  const bool train = p.mode == 0;
  const bool margin_one = p.margin == 1.0f;
  const uint32_t rec = (uint32_t)p.record;
  const size_t A = (size_t)p.A;
  const KC k = pin_constants(p);  // loop constants in VGPRs (no SGPR spill reloads on the chain)
  const Dims<B20> D{k.nt, k.nT, k.nb, k.np};
  std::conditional_t<WIDE, PTile<NC>, PRegs<NC>> P;
  if constexpr (WIDE) {
    P.base = shP + sl * 2 * PTile<NC>::kTile;
    P.i = i;
    P.rd = 0;
    P.wr = 0;
  } else {
    P.sh = shP;
    P.i = i;
    P.sl = sl;
  }

  const uint32_t n_states = (uint32_t)(p.nt * p.nT * p.nb * p.np);
  constexpr bool shared = SQ;
  QT* __restrict__ q = reinterpret_cast<QT*>(p.q) + (shared ? (size_t)0 : (size_t)a * n_states * kQPad);
  unsigned long long* const dbase = reinterpret_cast<unsigned long long*>(p.qdelta) +
      (shared ? (size_t)(blockIdx.x % kDeltaCopies) * n_states * kQPad : (size_t)0);
  if constexpr (SQ) {
    for (int k2 = threadIdx.x; k2 < kSqSlots; k2 += WPB * kWave) {
      hkey[k2] = kSqEmpty;
      hval[k2] = 0;
    }
    __syncthreads();
  }
  const float mi = active ? p.max_in[a] : 1.0f;
  const float4 lv = p.hp_lv[a];  // heat-pump power of actions 0..2 for this agent
  const bool bat = p.battery != 0;
  const double bcap = bat ? p.bat_cap[a] : 0.0;
  double soc = bat ? p.soc[a] : 0.0;
  float tin = active ? p.t_in[a] : k.setpoint;
  float tm = active ? p.t_m[a] : k.setpoint;
  // round 0 and the next state both have p2p = mean(-0 ... -0) / max_in = 0 (agent.py:203, community.py:161)
  const int ip_zero = idx_plain(divn(0.0f) / mi, D.p());

  // running offsets (no 64-bit multiplies in the loop)
  const float* envb = p.env + (size_t)s_env * kEnvStride;
  const size_t env_step = (size_t)p.n_env * kEnvStride;
  const size_t env_end = env_step * T;
  const float2* profb = p.prof + a;
  const size_t prof_end = A * T;
  auto prof_at = [&](size_t off) { return profb[off]; };  // inactive lanes read agent 0 (a = 0)
  const uint32_t* codes_a = p.codes + a;
  const size_t code_step = (size_t)W * A;
  float* rec_reward = p.rec_reward + a;
  float* rec_cost = p.rec_cost + a;
  float* rec_grid = p.rec_grid + a;
  float* rec_p2p = p.rec_p2p + a;
  float* rec_tin = p.rec_tin + a;
  uint8_t* rec_action = p.rec_action + a;
  int32_t* rec_index = p.rec_index + a;
  auto adv = [](size_t off, size_t step, size_t end) { off += step; return off >= end ? off - end : off; };
  size_t e1o = adv(0, env_step, env_end), e2o = adv(e1o, env_step, env_end);
  size_t f1o = adv(0, A, prof_end), f2o = adv(f1o, A, prof_end);
  size_t c1o = (T > 1) ? code_step : 0;  // code words of step t + 1 (wrapping to 0 on the last step)

  EnvRow e0 = load_env(envb);
  EnvRow e1 = load_env(envb + e1o);
  const float2 f0 = prof_at(0);
  float2 f1 = prof_at(f1o);
  StepIdx st = make_step(k, D, margin_one, e0.time, e1.time, FDIV(f0.x - f0.y, mi), f1, tin, mi, ip_zero);
  uint64_t cw = code_word(p, step_codes(p, codes_a, 0, 0, a, W), active);
  // Q rows are loaded unconditionally (a load under a divergent branch is waited for at the
  // join, which would serialise the prefetch); a row that is not needed aliases one that is
  // loaded anyway, so it costs no HBM traffic.  Inactive lanes read agent 0's table.
  auto row0_addr = [&](const StepIdx& x, uint64_t c) -> uint32_t {
    const bool need = ((c & 0xFF) == 255) || (train && R1 == 1);  // greedy, or the TD target itself
    return need ? x.strip + (uint32_t)ip_zero : x.nrow;
  };
  uint32_t a0 = row0_addr(st, cw);
  uint32_t aN = train ? st.nrow : a0;
  Row4<QT> row0 = gather_row(q + a0 * kQPad);
  Row4<QT> rowN = gather_row(q + aN * kQPad);
  Patch<QT> pat{0xFFFFFFFFu, 0, (QT)0};
  float ep_sum = 0.0f;
  size_t tA = 0;

  for (int t = 0; t < T; ++t, tA += A) {
    // prefetch ahead: env/profile two steps, exploration codes one step
#if P2PMG_ABLATE >= 3
    const EnvRow e2 = load_env(envb);
    const float2 f2 = prof_at(0);
#else
    const EnvRow e2 = load_env(envb + e2o);
    const float2 f2 = prof_at(f2o);
#endif
    const CodeWords cw1r = step_codes(p, codes_a, c1o, t + 1 == T ? 0 : t + 1, a, W);

    P.clear();
    int act = 0, ip = ip_zero;
    float hp = 0.0f;
    double soc_r = soc;  // tentative SoC of the current round
    row0 = patched(row0, a0, pat);  // the previous step's TD store may have hit a prefetched row
    rowN = patched(rowN, aN, pat);
    Row4<QT> rowR = row0;  // Q row of the final round's state (TD target Q[s, a])

    for (int r = 0; r < R1; ++r) {
      const int code = r < 8 ? (int)((cw >> (8 * r)) & 0xFF) : late_code(p, codes_a, tA * W, t, r, a, active);
      if (r > 0) {
        P.next_round();  // Jacobi: read the previous round's column (community.py:84-86)
        // powers = -P[:, i] with the diagonal zeroed (community.py:76,81); p2p = mean / max_in (agent.py:203)
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < n; ++j) acc = acc + (-((j == i) ? 0.0f : P.colv(j)));
        ip = idx_plain(FDIV(divn(acc), mi), D.p());
        // the final round's row is needed for the TD update even when exploring
        const bool need = code == 255 || (train && r == R1 - 1);
        rowR = gather_row(q + (need ? st.strip + (uint32_t)ip : a0) * kQPad);
      }
      act = code == 255 ? argmax3(rowR) : code;  // QAgent._act / take_decision (agent.py:271-289)
      hp = hp_of(lv, act);

      // RLAgent._divide_power agent.py:186-195 on out = bal * max_in + hp (agent.py:210);
      // with a battery the rule adjusts the net power first (SoC committed by the last round)
      float out = (st.bal * mi) + hp;
      if (bat && bcap > 0.0) {
        soc_r = soc;
        out = (float)battery_rule((double)out, soc_r, bcap, p.bat_min, p.bat_max, p.bat_sqrt_eff);
      }
      const float so = sgn(out);
      // filtered_j: powers_j where its sign differs from out's (agent.py:187-189)
      auto filt = [&](int j) -> float {
        const float pw = -((j == i || r == 0) ? 0.0f : P.colv(j));
        return (so != sgn(pw)) ? pw : 0.0f;
      };
      float tot = 0.0f;
#pragma unroll
      for (int j = 0; j < n; ++j) tot = tot + filt(j);
      tot = fabsf(tot);
      if (tot == 0.0f) {
        const float ev = divn(out * 1.0f);
#pragma unroll
        for (int j = 0; j < n; ++j) P.put(j, ev);
      } else {
        // |f_ii| = 0 (own power is -0): (out * 0) / tot == out * 0 exactly for any non-NaN tot
#pragma unroll
        for (int j = 0; j < n; ++j)
          P.put(j, (j == i) ? (tot == tot ? out * 0.0f : tot) : FDIV(nabs_out(out) * filt(j), tot));
      }
      if (active && (rec & 96u)) {
        const size_t kk = (tA * R1) + (size_t)r * A;
        if (rec & 32u) rec_action[kk] = (uint8_t)act;
        if (rec & 64u) rec_index[kk] = st.it | (st.iT << 8) | (st.ib << 16) | (ip << 24);
      }
    }

    soc = soc_r;  // BatteryStorage state after the final round's decision
    // CommunityMicrogrid._step -> HPHeating.step (community.py:184-188, heating.py:138-143):
    // computed now so the next step's rows can be issued before this step's market work
    float tin1 = tin, tm1 = tm;
    rc_update(k, e0.t_out, hp, tin1, tm1);
    // (after the last step this prefetches a wrapped, unused step: harmless valid addresses)
    const StepIdx st1 = make_step(k, D, margin_one, e1.time, e2.time, st.baln, f2, tin1, mi, ip_zero);
    const uint64_t cw1 = code_word(p, cw1r, active);
    const uint32_t a0n = row0_addr(st1, cw1);
    const uint32_t aNn = train ? st1.nrow : a0n;
    const Row4<QT> row0n = gather_row(q + a0n * kQPad);
    const Row4<QT> rowNn = gather_row(q + aNn * kQPad);
    pat.row = 0xFFFFFFFFu;

    // CommunityMicrogrid._assign_powers community.py:45-54 on the final P (diagonal kept)
    P.next_round();
    float g = 0.0f, pp = 0.0f;
#pragma unroll
    for (int j = 0; j < n; ++j) {
      const float pij = P.rowv(j), pji = P.colv(j);
      const float ex = pair_exchange(pij, pji);
      g = g + (pij - ex);
      pp = pp + ex;
    }
    // CommunityMicrogrid._compute_costs community.py:56-65
    float cost = (g >= 0.0f) ? g * e0.buy : g * e0.inj;
    cost = cost + pp * e0.p2p;
    cost = FDIV(cost * k.slot, k.mph);
    cost = cost * k.kilo;
    // RLAgent.get_reward agent.py:225-232 (pre-update T_in)
    float pen = fmaxf(fmaxf(0.0f, k.lower - tin), fmaxf(0.0f, tin - k.upper));
    pen = pen > 0.0f ? pen + 1.0f : 0.0f;
    const float rw = -(cost + k.penw * pen);

    if (train && active && !shared) {
      // QAgent.train agent.py:293-298 -> QActor.train rl.py:119-129
      const uint32_t srow = st.strip + ip;
      const QT qsa = sel3(act, rowR.v[0], rowR.v[1], rowR.v[2]);
      const QT qnew = td_update(qsa, rw, max3(rowN), k.alpha, k.gamma);
      q[srow * kQPad + act] = qnew;
      pat = Patch<QT>{srow, act, qnew};  // rows issued before this store see the old value
    }
    if (shared && train && active) {
      // frozen shared table: delta = alpha * ((r + gamma * max Q[ns]) - Q[s, a]) in f64, summed in
      // int64 fixed point (order-independent, so every launch and every rank sums identically)
      const QT qsa = sel3(act, rowR.v[0], rowR.v[1], rowR.v[2]);
      const double d = k.alpha * (((double)rw + k.gamma * (double)max3(rowN)) - (double)qsa);
      const long long v = __double2ll_rn(d * kDeltaScale);
#if P2PMG_ABLATE == 5
      if (v == 12345)  // timing-only: drop the accumulation (never true in practice)
#endif
      lds_add_by_key(hkey, hval, (st.strip + (uint32_t)ip) * kQPad + (uint32_t)act, v, dbase);
    }
    if (active && (rec & 31u)) {
      if (rec & 1u) rec_reward[tA] = rw;
      if (rec & 2u) rec_cost[tA] = cost;
      if (rec & 4u) rec_grid[tA] = g;
      if (rec & 8u) rec_p2p[tA] = pp;
      if (rec & 16u) rec_tin[tA] = tin;
    }
    // avg_reward = sum_t mean_i r (community.py:179), canonical sequential order
    float m;
    if constexpr (WIDE) m = group_sum_n<NC>(rw, i, sl, n, shR);
    else m = group_sum<NC>(rw, lane, i, sl, shR);
    ep_sum = ep_sum + divn(m);
    if constexpr (SQ) {
      if (train && (t % kSqFlushSteps == kSqFlushSteps - 1 || t + 1 == T)) lds_hash_flush(hkey, hval, dbase, WPB * kWave);
    }

    tin = tin1;
    tm = tm1;
    e0 = e1;
    e1 = e2;
    f1 = f2;
    e2o = adv(e2o, env_step, env_end);
    f2o = adv(f2o, A, prof_end);
    c1o = (t + 2 >= T) ? (size_t)0 : c1o + code_step;
    st = st1;
    cw = cw1;
    a0 = a0n;
    aN = aNn;
    row0 = row0n;
    rowN = rowNn;
  }
  if (active) {
    p.t_in[a] = tin;
    p.t_m[a] = tm;
    if (bat) p.soc[a] = soc;
    if (i == 0) p.ep_reward[s] = ep_sum;
  }
}

// Q += delta * 2^-40 (f64), delta = 0: the end-of-episode update of the shared table, after the
// optional all-reduce of the int64 deltas over ranks
template <typename QT>
__global__ void apply_delta_kernel(QT* __restrict__ q, long long* __restrict__ d, size_t n) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const long long x = d[k];
  if (x != 0) {
    q[k] = (QT)((double)q[k] + (double)x * (1.0 / kDeltaScale));
    d[k] = 0;
  }
}

// sum the per-XCD delta replicas into copy 0 (and clear the others)
#if P2PMG_IN_PART(0)
__global__ void fold_delta_kernel(long long* __restrict__ d, size_t n) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  long long x = d[k];
#pragma unroll
  for (int c = 1; c < kDeltaCopies; ++c) {
    const long long y = d[(size_t)c * n + k];
    if (y != 0) {
      x += y;
      d[(size_t)c * n + k] = 0;
    }
  }
  d[k] = x;
}
#endif

// battery rule over per-agent sequences (unit parity with storage.py / agent.py:138-153)
#if P2PMG_IN_PART(0)
__global__ void battery_seq_kernel(int agents, int steps, const double* bal, double* out_bal, double* soc_hist,
                                   double* soc, const double* cap, double smin, double smax, double sqrt_eff) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= agents) return;
  double s_ = soc[a];
  for (int t = 0; t < steps; ++t) {
    const size_t k = (size_t)a * steps + t;
    out_bal[k] = battery_rule(bal[k], s_, cap[a], smin, smax, sqrt_eff);
    soc_hist[k] = s_;
  }
  soc[a] = s_;
}
#endif

// Philox pre-pass: every (t, agent) code word of an episode in one parallel launch, so the
// latency-bound episode loop only loads a prefetched word instead of computing R+1 blocks.
#if P2PMG_IN_PART(0)
__global__ void philox_codes_kernel(const EpisodeParams p, uint32_t* __restrict__ words) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // k = t * A + a
  if (k >= (size_t)p.T * p.A) return;
  const int t = (int)(k / p.A), a = (int)(k % p.A);
  const int R1 = p.R + 1, W = (R1 + 3) >> 2;
  const uint32_t gid = p.agent_offset + (uint32_t)a;
  const uint64_t codes = philox_codes_of(p, t, gid);
  for (int w = 0; w < W; ++w)
    words[((size_t)t * W + w) * p.A + a] =
        w < 2 ? (uint32_t)(codes >> (32 * w))
              : philox_code_word(t, R1, w, (uint32_t)p.episode, gid, p.eps_thr, p.eps_all, p.seed_lo, p.seed_hi);
}
#endif

// host replay codes u8 [T][R1][A] -> code words [T][W][A]
#if P2PMG_IN_PART(0)
__global__ void pack_codes_kernel(int T, int R1, int A, const uint8_t* __restrict__ in, uint32_t* __restrict__ words) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (size_t)T * A) return;
  const int t = (int)(k / A), a = (int)(k % A);
  const int W = (R1 + 3) >> 2;
  for (int w = 0; w < W; ++w) {
    uint32_t word = 0xFFFFFFFFu;
    for (int b = 0; b < 4 && 4 * w + b < R1; ++b) {
      const uint32_t c = in[((size_t)t * R1 + 4 * w + b) * A + a];
      word = (word & ~(0xFFu << (8 * b))) | (c << (8 * b));
    }
    words[((size_t)t * W + w) * A + a] = word;
  }
}
#endif

// ----------------------------------------------------------------- the fast per-agent-table path
// IEEE f32 division a / b without its range handling.  hipcc's correctly rounded sequence is
//   v_div_scale(b), v_rcp, y = fma(fma(-b, rcp, 1), rcp, rcp), v_div_scale(a),
//   q = a*y, r = fma(-b, q, a), q = fma(r, y, q), r = fma(-b, q, a), v_div_fmas = fma(r, y, q),
//   v_div_fixup
// The two scale steps are identities (and v_div_fmas a plain fma) while |a| and |b| lie in
// [2^-40, 2^40] (exponent gap below 96, nothing near denormal or overflow), and v_div_fixup only
// rewrites NaN / inf / zero / denormal cases, none of which a quotient of two such numbers is.
// So inside that range these five ops ARE the division, bit for bit; outside it, or for a = 0,
// the caller takes the IEEE operator.  The reciprocal of a loop-invariant divisor (max_in, the
// 60 minutes of an hour, N, the comfort margin) is hoisted out of the episode loop.
struct Recip {
  float b, y;
  bool ok;  // |b| in range
};
__device__ __forceinline__ bool in_div_range(float x) {
  const float m = fabsf(x);
  return m >= 0x1p-40f && m <= 0x1p40f;
}
__device__ __forceinline__ Recip recip(float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  return Recip{b, __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0), in_div_range(b)};
}
// ONE Newton correction of q0 = a y suffices (round 5): with y refined from v_rcp_f32 as in recip(),
// q = fma(fma(-b, q0, a), y, q0) equals the IEEE quotient for every pair of 24-bit significands
// (all 2^46 pairs checked on the GPU, scripts/div_exhaustive.hip, profiles/r05_div_exhaustive.jsonl),
// v_rcp_f32 scales exactly with the divisor's exponent (same run, e in [-40, 40]), and inside the
// range every step scales exactly with the operands' exponents (the residual stays representable),
// so the significand pairs decide every case.  The second correction of rounds 1-4 was a no-op.
__device__ __forceinline__ float fdiv_core(float a, const Recip& d) {
  const float q0 = a * d.y;
  const float r = __builtin_fmaf(-d.b, q0, a);
  const float q = __builtin_fmaf(r, d.y, q0);
  // a = +-0: the steps above give +0; the IEEE quotient carries sign(a) * sign(b) = sign(q0).
  // For every other a the sign of q already equals sign(q0), so the copy is exact either way.
  return __builtin_copysignf(q, q0);
}
__device__ __forceinline__ bool fdiv_ok(float a) {
  const float m = fabsf(a);
  return (m >= 0x1p-40f && m <= 0x1p40f) || m == 0.0f;
}
// the IEEE quotient behind an opaque copy of a: keeps the compiler from speculating this rare path
// (11 instructions) into a select on the common one
__device__ __forceinline__ float fdiv_ieee(float a, float b) {
  asm volatile("" : "+v"(a));
  return a / b;
}
// a / b with a divisor the launcher has checked to lie in range (max_in, 60, N, the margin)
__device__ __forceinline__ float fdiv_b(float a, const Recip& d) {
  float q = fdiv_core(a, d);
  if (!fdiv_ok(a)) q = fdiv_ieee(a, d.b);  // rare: tiny, huge or non-finite numerator
  return q;
}
template <int N>
__device__ __forceinline__ float div_n_r(float x, const Recip& rn) {
  if constexpr ((N & (N - 1)) == 0) return x * (1.0f / (float)N);
  else return fdiv_b(x, rn);
}
// clamp_bin as one v_med3: (int)med3(v, 0, K-1) equals clamp_bin for every non-NaN v (values in
// [0, 1) truncate to 0 like the reference's v < 1 branch)
__device__ __forceinline__ int clamp_bin_f(float v, float km1) { return (int)__builtin_amdgcn_fmed3f(v, 0.0f, km1); }

// T0 ~ N(setpoint, sigma) for (episode, global agent id): Box-Muller on one Philox block
// (HPHeating.reset heating.py:145-152 with a counter-based stream; oracle/philox.py t0_draws)
__device__ __forceinline__ void t0_draw(uint32_t k0, uint32_t k1, int episode, uint32_t gid, float setpoint,
                                        double sigma, float& t_in, float& t_m) {
  uint32_t c0 = 0, c1 = (uint32_t)episode, c2 = gid, c3 = kTagT0;
  philox4x32_10(c0, c1, c2, c3, k0, k1);
  const double u1 = ((double)c0 + 0.5) / 4294967296.0;
  const double u2 = ((double)c1 + 0.5) / 4294967296.0;
  const double rad = sqrt(-2.0 * log(u1));
  const double ang = 6.283185307179586 * u2;
  t_in = (float)((double)setpoint + sigma * (rad * cos(ang)));
  t_m = (float)((double)setpoint + sigma * (rad * sin(ang)));
}
// Step pre-pass: everything of step t that depends only on the inputs (profiles, environment,
// max_in), not on the policy or the temperatures, for every (t, agent) in one parallel launch per
// episode, so the serial episode loop pays for none of these divisions and bins:
//   pre[t][a].x = bits of balw = ((load - pv) / max_in) * max_in      agent.py:172-176, 210
//   pre[t][a].y = (it_t * nT*nb + ib_t) | (it_{t+1} * nT*nb + ib_{t+1}) << 16
//                 (row / np of the state (it, 0, ib, 0) and of the next state, rl.py:89-95;
//                  the next state's balance is that of the next profile row, wrapping at T)
// PHILOX = true also writes the step's exploration code words (philox_codes_kernel's job).
// ep: the episode of a chain (o.n_ep > 1) whose code words to write; the policy-independent words
// are the same for every episode and written with episode 0's.
__device__ __forceinline__ void prepass_one(const EpisodeParams& p, const PrepOut& o, size_t k, int ep = 0) {
  const int t = (int)(k / p.A), a = (int)(k % p.A);
  const int tn = t + 1 == p.T ? 0 : t + 1;
  const int se = p.n_env == 1 ? 0 : a / p.N;
  const float mi = p.max_in[a];
  const float2 f = p.prof[k], fn = p.prof[(size_t)tn * p.A + a];
  const float bal = (f.x - f.y) / mi, baln = (fn.x - fn.y) / mi;
  const float time_t = p.env[((size_t)t * p.n_env + se) * kEnvStride];
  const float time_n = p.env[((size_t)tn * p.n_env + se) * kEnvStride];
  const uint32_t tb = (uint32_t)(p.nT * p.nb);
  const uint32_t lo = (uint32_t)idx_time(time_t, p.nt) * tb + (uint32_t)idx_plain(bal, p.nb);
  const uint32_t hi = (uint32_t)idx_time(time_n, p.nt) * tb + (uint32_t)idx_plain(baln, p.nb);
  if (ep == 0) o.pre[k] = make_uint2(__float_as_uint(bal * mi), lo | (hi << 16));
  if (o.ipc && ep == 0) {
    // N = 2: round 1's p2p feature depends only on the partner's round-0 action b (agent.py:203):
    // its column entry is ev_b = ((balw_p + hp_p[b]) * 1) / 2 (the even split of round 0), summed
    // as in the kernel's acc loop.  Byte b = the bin for b, so the kernel's round-1 rows can be
    // issued a step ahead and picked by the partner's action.
    const int i = a % 2, ap = a ^ 1;
    const float2 fp = p.prof[(size_t)t * p.A + ap];
    const float mip = p.max_in[ap];
    const float balw_p = ((fp.x - fp.y) / mip) * mip;
    const float4 lvp = p.hp_lv[ap];
    const float hpl[3] = {lvp.x, lvp.y, lvp.z};
    uint32_t ipc = 0;
    for (int b = 0; b < 3; ++b) {
      const float ev = div_n<2>((balw_p + hpl[b]) * 1.0f);
      float acc = 0.0f;
      for (int j = 0; j < 2; ++j) acc = acc + (-((j == i) ? 0.0f : ev));
      ipc |= (uint32_t)idx_plain(div_n<2>(acc) / mi, p.np) << (8 * b);
    }
    o.ipc[k] = ipc;
  }
  if (o.words) {
    EpisodeParams q = p;
    const bool chain = o.n_ep > 1;
    q.episode = o.episode + ep;
    q.eps = o.eps;
    q.eps_thr = chain ? o.ep_thr[ep] : o.eps_thr;
    q.eps_all = chain ? (int)((o.ep_all >> ep) & 1u) : o.eps_all;
    const int R1 = p.R + 1, W = (R1 + 3) >> 2;
    const uint32_t gid = p.agent_offset + (uint32_t)a;
    const uint64_t codes = philox_codes_of(q, t, gid);
    uint32_t* words = o.words + (size_t)ep * o.words_stride;
    for (int w = 0; w < W; ++w)
      words[((size_t)t * W + w) * p.A + a] =
          w < 2 ? (uint32_t)(codes >> (32 * w))
                : philox_code_word(t, R1, w, (uint32_t)q.episode, gid, q.eps_thr, q.eps_all, p.seed_lo, p.seed_hi);
  }
}
#if P2PMG_IN_PART(0)
__global__ void step_prepass_kernel(const EpisodeParams p, const PrepOut o) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // k = t * A + a
  if (k >= (size_t)p.T * p.A) return;
  prepass_one(p, o, k, (int)blockIdx.y);  // blockIdx.y: the chain's episode (uniform per workgroup)
}
#endif

// round 1 after an all-even round 0: every lane's row is ev (agent.py:190-191), so the column is
// the group's ev values (one shuffle per partner instead of a row exchange)
template <int N, int D, int G>
__device__ __forceinline__ void gather_even(float ev, float (&col)[N], int i) {
  if constexpr (D < G) {
    const float got = shfl_xor_c<D>(ev);
    const int src = i ^ D;
#pragma unroll
    for (int k = 0; k < N; ++k) col[k] = (k == src) ? got : col[k];
    gather_even<N, D + 1, G>(ev, col, i);
  }
}

// f64 division with a hoisted reciprocal: hipcc's IEEE f64 sequence (v_div_scale, v_rcp_f64, two
// Newton steps, q = n * y, r = fma(-d, q, n), v_div_fmas = fma(r, y, q), v_div_fixup) with the
// scale / fixup steps dropped, which is exact while |n| and |d| lie in [2^-300, 2^300] (the
// exponent gap stays below the 768 where v_div_scale starts scaling); else the IEEE operator.
struct Recip64 {
  double d, y;
  bool ok;
};
__device__ __forceinline__ bool in_div_range64(double x) {
  const double m = fabs(x);
  return m >= 0x1p-300 && m <= 0x1p300;
}
__device__ __forceinline__ Recip64 recip64(double d) {
  const double r0 = __builtin_amdgcn_rcp(d);
  const double r1 = __builtin_fma(r0, __builtin_fma(-d, r0, 1.0), r0);
  return Recip64{d, __builtin_fma(r1, __builtin_fma(-d, r1, 1.0), r1), in_div_range64(d)};
}
// x / 900 s (storage.py) through the correctly rounded reciprocal as a compile-time constant: the
// one Newton correction in qcore64 / qpos64 returns the IEEE quotient from it as from the device's
// refined v_rcp_f64 estimate, and a literal is rematerialised where a kernel-argument-derived value
// would hold two SGPRs across the loop (or spill them to VGPR lanes)
constexpr Recip64 kR900{900.0, 1.0 / 900.0, true};
__device__ __forceinline__ double fdiv64_ieee(double n, double d) {
  asm volatile("" : "+v"(n));
  return n / d;
}
__device__ __forceinline__ double fdiv64(double n, const Recip64& r) {
  const double q = n * r.y;
  double res = __builtin_fma(__builtin_fma(-r.d, q, n), r.y, q);
  res = __builtin_copysign(res, q);  // +-0 / d keeps sign(n) * sign(d), as the IEEE quotient
  if (!(r.ok && (n == 0.0 || in_div_range64(n)))) res = fdiv64_ieee(n, r.d);
  return res;
}
// reciprocals of kernel-uniform divisors, moved to SGPRs (v_readfirstlane): VGPRs set the
// occupancy of the throughput-bound sq16 kernel
__device__ __forceinline__ float sgpr_f(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }
__device__ __forceinline__ double sgpr_d(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ Recip recip_u(float b) {
  const Recip r = recip(b);
  return Recip{b, sgpr_f(r.y), r.ok};
}
__device__ __forceinline__ Recip64 recip64_u(double d) {
  const Recip64 r = recip64(d);
  return Recip64{d, sgpr_d(r.y), r.ok};
}
// battery_rule (agent.py:138-153 + storage.py bookkeeping) with the divisions by the agent's
// capacity, sqrt(efficiency) and 900 s through hoisted reciprocals; same op order, same results.
// Branch-free: the discharge and charge branches divide the same expressions of their own x, so x
// is selected first and x / cap, x / 900, (x / cap) / sqrt(eff) are computed once (4 quotients
// instead of up to 6 on a divergent wave); one range test for all of them, and a lane with an
// operand outside the range-free quotient's domain redoes the rule with IEEE divisions.
struct BatK {
  double smin, smax, se;
  Recip64 rse, r900;
};
// 0, or |n| in [2^-300, 2^300) by its biased exponent (723..1322): the range-free quotient's domain
__device__ __forceinline__ bool q64_ok(double n) {
  const unsigned e = ((unsigned)__double2hiint(n) >> 20) & 0x7FFu;
  return (e - 723u <= 599u) || n == 0.0;
}
// fdiv64 without its range test (the caller tests the operands)
__device__ __forceinline__ double qcore64(double n, const Recip64& r) {
  const double q = n * r.y;
  return __builtin_copysign(__builtin_fma(__builtin_fma(-r.d, q, n), r.y, q), q);
}
// CHECK = false: the launcher has verified the operands' domain (p2pmg_set_battery / set_profiles:
// capacities 0 or in [2^-20, 2^60], SoC bounds in [2^-100, 2^10], sqrt(eff) in [2^-10, 2^10], SoC0 in
// [0, 2^10], |load|, |pv|, heat-pump levels <= 2^100).  Then every numerator is 0 or in
// [2^-252, 2^168] (a positive SoC - bound difference is a multiple of the bound's ulp >= 2^-152; a
// nonzero f32 balance times 900 lies in [2^-140, 2^138]) and the per-lane range tests go.
// The SoC-only terms of the rule (storage.py:52-60: available energy / space, the full test), the
// same for every round of a step: computed once per step (bat_pre) and shared by the rounds.
struct BatPre {
  double avail_energy, avail_space;
  bool full;
};
// x / d for d > 0 and x >= +0: qcore64 without the sign fix, which only matters for x = -0
__device__ __forceinline__ double qpos64(double n, const Recip64& r) {
  const double q = n * r.y;
  return __builtin_fma(__builtin_fma(-r.d, q, n), r.y, q);
}
__device__ __forceinline__ BatPre bat_pre(double soc, double cap, const BatK& b) {
  // space >= +0 (fmax with 0, a positive capacity), so the unsigned quotient is the IEEE one
  return BatPre{(fmax(0.0, soc - b.smin) * cap) * b.se, qpos64(fmax(0.0, b.smax - soc) * cap, b.rse), soc >= b.smax};
}
// battery_rule_r<false> on a step's precomputed SoC terms (the launcher-verified domain): every
// quotient's numerator is positive where it is used (dis: x = min(energy, avail_energy) > 0;
// chg: x = min(-energy, avail_space) > 0 as soc < smax), so the quotients need no sign fix
// (balance * 60) * 15 of a balance that is an f32 value: both products are exact in f64 (24 + 4 + 4
// significant bits), and so is balance * 900 (24 + 8): one multiply, the same double
__device__ __forceinline__ double energy_of(double balance_f32) { return balance_f32 * 900.0; }
// -x if c else x: a sign flip of the high word (x - y == x + (-y) in IEEE arithmetic)
__device__ __forceinline__ double neg_if(double x, bool c) {
  return __hiloint2double(__double2hiint(x) ^ (c ? (int)0x80000000 : 0), __double2loint(x));
}
__device__ __forceinline__ double battery_rule_pre(double balance, double& soc, const Recip64& rcap, const BatK& b,
                                                   const BatPre& pr) {
  const double energy = energy_of(balance);
  const bool dis = balance > 0.0 && pr.avail_energy > 0.0;
  const bool chg = !dis && balance < 0.0 && !pr.full;
  // min(energy, available_energy) / min(-energy, available_space) as v_min_f64 (IEEE minNum): in the
  // launcher-verified domain every operand is finite, and where x is used both are positive (dis:
  // energy > 0, avail_energy > 0; chg: -energy > 0, avail_space >= +0), so minNum returns what the
  // reference's `a <= b ? a : b` does (equal values are the same double); 4 VALU instead of 9
  const double x = dis ? fmin(energy, pr.avail_energy) : fmin(-energy, pr.avail_space);
  const double q1 = qpos64(x, rcap);     // x / capacity
  const double q2 = qpos64(x, b.r900);   // x / 900
  const double q3 = qpos64(q1, b.rse);   // (x / capacity) / sqrt(eff)
  // dis: soc - q3, balance - q2; chg: soc + sqrt(eff) q1, balance + q2 -- one add each
  const double soc_n = soc + (dis ? neg_if(q3, true) : b.se * q1);
  const double bal_n = balance + neg_if(q2, dis);
  soc = (dis || chg) ? soc_n : soc;
  return (dis || chg) ? bal_n : balance;
}
template <bool CHECK = true>
__device__ __forceinline__ double battery_rule_r(double balance, double& soc, double cap, const Recip64& rcap,
                                                 const BatK& b) {
  const double energy = energy_of(balance);  // (balance * 60) * 15, exact for the f32 balances passed in
  const double avail_energy = (fmax(0.0, soc - b.smin) * cap) * b.se;
  const double space_n = fmax(0.0, b.smax - soc) * cap;
  const double avail_space = qcore64(space_n, b.rse);
  const bool dis = balance > 0.0 && avail_energy > 0.0;
  const bool chg = !dis && balance < 0.0 && !(soc >= b.smax);
  const double x = dis ? (energy <= avail_energy ? energy : avail_energy)    // min(energy, available_energy)
                       : (-energy <= avail_space ? -energy : avail_space);  // min(-energy, available_space)
  const double q1 = qcore64(x, rcap);     // x / capacity
  const double q2 = qcore64(x, b.r900);   // x / 900
  const double q3 = qcore64(q1, b.rse);   // (x / capacity) / sqrt(eff)
  if constexpr (CHECK) {
    const bool ok = rcap.ok && b.rse.ok && b.r900.ok && q64_ok(x) && q64_ok(q1) && (!chg || q64_ok(space_n));
    if ((dis || chg) && !ok) return battery_rule(balance, soc, cap, b.smin, b.smax, b.se);  // IEEE divisions
  }
  const double soc_n = dis ? soc - q3 : soc + b.se * q1;
  const double bal_n = dis ? balance - q2 : balance + q2;
  soc = (dis || chg) ? soc_n : soc;
  return (dis || chg) ? bal_n : balance;
}

// episode_fast_kernel: episode_kernel's per-agent-table path (no shared table, G <= 8,
// R + 1 <= 4, or <= 2 with a battery, code words from a pre-pass) with the rounds unrolled at compile time and the
// policy-independent per-step work (balance, time / balance bins, the next state's bins) read
// from step_prepass_kernel's output.  Same op order, same results, bit for bit (tests compare
// both kernels with the oracle).  Latency structure per step:
//   * round 0 always sees P = 0: its row and the next-state row are issued at the end of the
//     previous step (as in episode_kernel), round 0 is an even split, and round 1's column is
//     the group's round-0 even values;
//   * the next step's pre-pass word, env row and code word are issued right after the dependent
//     round-R gather, so waiting for that gather never waits for them (vmcnt counts in order);
//   * every store is unconditional (inactive lanes and disabled records write a per-lane dummy
//     slot), so the number of memory ops behind each load is static and the loop-top wait for
//     the prefetched rows is vmcnt(3), not a vmcnt(0) drain of the step's stores;
//   * records go out as ONE 32-B row per agent-step (FastRec), or as an 8-B {reward, cost} row
//     when only those are requested, and are unpacked on request;
//   * division by max_in / 60 / N uses the hoisted reciprocal (fdiv above);
//   * BAT (configs[3] mixes): every round's net power goes through the battery rule first (f64,
//     SoC committed by the final round, agent.py:138-153), with the capacity / sqrt(eff) / 900 s
//     divisions through hoisted reciprocals (battery_rule_r); agents with capacity 0 skip it.
// spw = scenarios per wave (<= 64 / G): fewer scenarios per wave spread the waves over more CUs.
struct FastRec {         // [T][A], 32 B
  float reward, cost, grid, p2p, tin;
  uint32_t actions;      // byte r: action of round r
  uint32_t bins;         // (it * nT*nb + ib) | iT << 16
  uint32_t ips;          // byte r: p2p bin of round r
};
#ifndef P2PMG_BAT_SPEC  // 1: the final round's battery rule for all 3 actions inside its row's round trip
#define P2PMG_BAT_SPEC 1  // configs[3] 59.6 -> 58.7 ms (profiles/r04_battery_ab.txt)
#endif
// BAT: 0 none, 1 battery with per-lane range tests, 2 battery in the launcher-verified domain
template <int N, typename QT, int R1, bool TRAIN, int BAT, bool NARROW>
__global__ __launch_bounds__(kWave) void episode_fast_kernel(const EpisodeParams p, const uint2* __restrict__ pre,
                                                             FastRec* __restrict__ recs, int spw, int n_cons,
                                                             const PrepOut nxt) {
  // Blocks past the consumer grid are producers: the next episode's step pre-pass (speculating the
  // same epsilon), run beside this episode's latency-bound waves on otherwise idle SIMDs, so the
  // next launch needs neither a pre-pass launch nor a cross-stream wait.
  if ((int)blockIdx.x >= n_cons) {
    const size_t n = (size_t)p.T * p.A, stride = (size_t)(gridDim.x - n_cons) * kWave;
    const int n_ep = nxt.n_ep > 1 ? nxt.n_ep : 1;  // the next launch's chain
    for (int ep = 0; ep < n_ep; ++ep)
      for (size_t k2 = (size_t)(blockIdx.x - n_cons) * kWave + threadIdx.x; k2 < n; k2 += stride)
        prepass_one(p, nxt, k2, ep);
    return;
  }
  constexpr int G = pow2ceil(N);
  static_assert(G <= 8 && R1 >= 1 && R1 <= 4, "fast path: G <= 8, R + 1 <= 4");
  // N = 2: round 1's Q row is one of three (by the partner's round-0 action) whose bins the
  // pre-pass wrote; all three are issued a step ahead, so round 1 waits for no gather
  // (not with a battery: the partner's round-0 power then depends on its state of charge)
  constexpr bool CAND = N == 2 && R1 >= 2 && BAT == 0;
  const int lane = (int)threadIdx.x;
  const int sl = lane / G;
  const int i = lane % G;
  const int s = (int)blockIdx.x * spw + sl;
  const bool active = i < N && sl < spw && s < p.S;
  const int a = active ? s * N + i : 0;
  const int s_env = p.n_env == 1 ? 0 : (active ? s : 0);
  const int T = p.T;
  const size_t A = (size_t)p.A;
  const KC k = pin_constants(p);
  const uint32_t n_states = (uint32_t)(p.nt * p.nT * p.nb * p.np);
  QT* __restrict__ q = reinterpret_cast<QT*>(p.q) + (size_t)a * n_states * kQPad;  // TD stores
  // Row gathers as ONE 32-bit offset from the wave's first table (global_load's SGPR-base + VGPR-offset
  // form: a v_lshl_add_u32 per row instead of a 64-bit address on the act -> gather chain).  The
  // launcher only sends this kernel tables whose 64-lane span fits 4 GiB.  Masked-off lanes read the
  // wave's first table.
  const int a_first = (int)blockIdx.x * spw * N;
  constexpr uint32_t kRowShift = sizeof(QT) == 8 ? 5 : 4;  // padded row: 32 B (f64) / 16 B (f32)
  const char* const qwave = reinterpret_cast<const char*>(p.q) + ((size_t)a_first * n_states << kRowShift);
  const uint32_t qlane = active ? (uint32_t)(a - a_first) * (n_states << kRowShift) : 0u;
  auto gat = [&](uint32_t row) __attribute__((always_inline)) {
    return gather_row(reinterpret_cast<const QT*>(qwave + (qlane + (row << kRowShift))));
  };
  const int np = k.np;
  const int nbv = k.nb;
  const float km1_T = (float)(k.nT - 1), km2_T = (float)(k.nT - 2), km1_p = (float)(np - 1), kp = (float)np;
  const float mi = active ? p.max_in[a] : 1.0f;
  const Recip rmi = recip(mi), rmph = recip(k.mph), rn = recip((float)N);
  const float4 lv = p.hp_lv[a];
  // the heat-pump terms of heating.py:44-45 per action: (c_in hp) cop and (c_m hp) cop, the same ops
  // rc_update applies to the chosen level, hoisted out of the episode
  const float hin[3] = {(k.c_in * lv.x) * k.cop, (k.c_in * lv.y) * k.cop, (k.c_in * lv.z) * k.cop};
  const float hm[3] = {(k.c_m * lv.x) * k.cop, (k.c_m * lv.y) * k.cop, (k.c_m * lv.z) * k.cop};
  float tin = active ? p.t_in[a] : k.setpoint;
  float tm = active ? p.t_m[a] : k.setpoint;
  double bcap = 0.0, soc = 0.0;
  BatK bk{};
  Recip64 rcap{};
  if constexpr (BAT != 0) {
    bcap = active ? p.bat_cap[a] : 0.0;
    soc = active ? p.soc[a] : 0.0;
    bk = BatK{p.bat_min, p.bat_max, p.bat_sqrt_eff, recip64_u(p.bat_sqrt_eff), kR900};
    rcap = recip64(bcap > 0.0 ? bcap : 1.0);
  }
  const int ip_zero = idx_plain(div_n<N>(0.0f) / mi, np);  // round 0 and next state: p2p = 0 (agent.py:203)
  // stores of inactive lanes (and every record when none is requested) go to a per-lane dummy slot
  QT* const q_dummy = reinterpret_cast<QT*>(p.dummy) + lane * kQPad;
  // records: FastRec rows, or only {reward, cost} as float2 when nothing else was requested.
  // A compile-time choice: with a run-time branch between the two store sequences the compiler's
  // vmcnt bookkeeping takes the shortest path through the branch, and the mid-step wait for the
  // round-1 rows then also waits for the previous step's TD store to complete (an HBM write ack).
  constexpr bool narrow = NARROW;
  const size_t rec_bytes = narrow ? sizeof(float2) : sizeof(FastRec);
  char* const rec_dummy = reinterpret_cast<char*>(reinterpret_cast<FastRec*>(p.dummy) + kWave + lane);
  const bool rec_on = p.record != 0 && active;
  const size_t rec_step = rec_on ? A * rec_bytes : 0;

  // idx_temp((T_in - setpoint) / margin) heating.py:118-120, rl.py:93; the launcher sends this
  // kernel the reference's margin of 1 only (x / 1 == x exactly), other margins take episode_kernel
  auto temp_bin = [&](float t_in) {
    const float x = t_in - k.setpoint;
    return clamp_bin_f(((x + 1.0f) / 2.0f) * km2_T + 1.0f, km1_T);
  };
  auto p2p_bin = [&](float x) { return clamp_bin_f(((x + 1.0f) / 2.0f) * kp, km1_p); };

  const float* envb = p.env + (size_t)s_env * kEnvStride;
  const size_t env_step = (size_t)p.n_env * kEnvStride;
  const uint2* preb = pre + a;
  const uint32_t* ipc_a = p.pre_ipc + a;  // read only when CAND
  const int t1 = T > 1 ? 1 : 0, t2 = 2 % T;
  // A chained launch runs p.chain episodes back to back in every wave (no launch boundary between
  // them, and each wave starts its next episode as soon as its own ends): T_in / T_m carry over
  // in registers (with the end-of-episode T0 reset when requested), the Q rows through memory.
  const int n_chain = p.chain > 1 ? p.chain : 1;
  for (int ep = 0; ep < n_chain; ++ep) {
    const uint32_t* codes_a = p.codes + (size_t)ep * p.codes_stride + a;
    char* rec_ptr = rec_on ? reinterpret_cast<char*>(recs) + (size_t)a * rec_bytes : rec_dummy;
    // The per-step inputs (env row, pre-pass word, code word, round-1 bins) are fresh HBM lines every
    // step, loaded three steps ahead into a 3-slot ring: slot t % 3 holds step t's, and step t
    // refills its own slot with step t + 3's once those are dead.  The step loop is unrolled by three,
    // so every slot is a fixed register set (no copies at the back edge, which would wait for the
    // loads), and the refills are issued after the step's row gathers: loads complete in issue order,
    // so a stream load issued ahead of the gathers would hold up the wait for them.
    // Running (uniform, 32-bit) offsets of step t + 3, wrapping at T: T * A < 2^32 on this path.
    const uint32_t TA = (uint32_t)T * (uint32_t)A, env_st = (uint32_t)env_step, env_end = env_st * (uint32_t)T;
    uint32_t o3 = (uint32_t)(3 % T) * (uint32_t)A, eo3 = (uint32_t)(3 % T) * env_st;

    // ring slots as vector values, so each stays one register tuple (a 16-B load's destination)
    EnvV eS[3] = {load_envv(envb), load_envv(envb + (size_t)t1 * env_step), load_envv(envb + (size_t)t2 * env_step)};
    uint2 pS[3] = {preb[0], preb[(size_t)t1 * A], preb[(size_t)t2 * A]};
    uint32_t cS[3] = {codes_a[0], codes_a[(size_t)t1 * A], codes_a[(size_t)t2 * A]};
    // masked-off lanes may explore too: they read agent 0's rows and store only to the dummy slots
    auto code_of = [&](uint32_t w) { return TRAIN ? w : 0xFFFFFFFFu; };
    uint32_t cw = code_of(cS[0]);
    int iT = temp_bin(tin);
    // row arithmetic in 24-bit multiplies (full-rate v_mul_u32_u24; every operand < 2^24)
    auto strip_of = [&](uint32_t base, int it_) { return __umul24(base + __umul24((uint32_t)it_, (uint32_t)nbv), (uint32_t)np); };
    uint32_t strip = strip_of(pS[0].y & 0xFFFFu, iT);
    uint32_t nrow = strip_of(pS[0].y >> 16, iT) + (uint32_t)ip_zero;
    auto row0_addr = [&](uint32_t st, uint32_t nr, uint32_t c) -> uint32_t {
      const bool need = ((c & 0xFF) == 255) || (TRAIN && R1 == 1);  // greedy, or the TD target itself
      return need ? st + (uint32_t)ip_zero : nr;
    };
    uint32_t a0 = row0_addr(strip, nrow, cw);
    uint32_t aN = TRAIN ? nrow : a0;
    Row4<QT> row0 = gat(a0);
    Row4<QT> rowN = gat(aN);
    uint32_t iS[3] = {0u, 0u, 0u};
    Row4<QT> cand[3];
    if constexpr (CAND) {
      iS[0] = ipc_a[0];
      iS[1] = ipc_a[(size_t)t1 * A];
      iS[2] = ipc_a[(size_t)t2 * A];
#pragma unroll
      for (int b = 0; b < 3; ++b) cand[b] = gat((strip + ((iS[0] >> (8 * b)) & 0xFFu)));
    }
    Patch<QT> pat{0xFFFFFFFFu, 0, (QT)0};
    float ep_sum = 0.0f;
    // the end-of-episode T0 reset depends only on (seed, episode + 1, agent): drawn here, while the
    // first rows are in flight, and applied at the end (the f64 transcendentals off the episode tail)
    float t0_in = tin, t0_m = tm;
    if (p.reset_t0 && active)
      t0_draw(p.seed_lo, p.seed_hi, p.episode + ep + 1, p.agent_offset + (uint32_t)a, p.setpoint, p.reset_sigma, t0_in,
              t0_m);
#if P2PMG_TRACE  // timing-only probe: per-step s_memtime splits of one wave, printed at the end
    uint64_t trW = 0, trC = 0, trR = 0, trLast = 0, trA0 = 0, trWC = 0, trA1 = 0, trMid = 0, trCal = 0;
#define P2PMG_STAMP(v) asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(v)::"memory")
#endif
    __builtin_amdgcn_s_waitcnt(0);  // enter the loop with nothing in flight (static waits inside)

    // one step; the loop below runs it three times per iteration (a manual unroll: the DPP exchanges
    // are convergent, so the compiler will not unroll a loop with a runtime trip count): the input
    // ring's slots and the prefetched rows' alternating registers stay put
    auto step = [&](auto par) __attribute__((always_inline)) {
      constexpr int P = decltype(par)::value, P1 = (P + 1) % 3;  // slots of step t and of step t + 1
      const EnvV ev = eS[P];
      const EnvRow e0{0.0f, ev.x, ev.y, ev.z, ev.w};
      const uint2 p0 = pS[P], p1 = pS[P1];
      const uint32_t c1 = cS[P1], ipc0 = iS[P], ipc1 = iS[P1];
      const float balw = __uint_as_float(p0.x);
      float row[N];
      float col[N];
#pragma unroll
      for (int j = 0; j < N; ++j) { row[j] = 0.0f; col[j] = 0.0f; }
      // the next step's T_in, temperature bin and table strips for each of the 3 actions
      // (heating.py:37-56, rl.py:93): they need only this step's state, so they run while the rows
      // are in flight, and the final action then merely selects one set (issue_next)
      float tinA[3];
      uint32_t iTA[3], stA[3], nrA[3];
      {
        const float ain = k.inv_ri * (tm - tin) + k.inv_rvent * (e0.t_out - tin);
#pragma unroll
        for (int x = 0; x < 3; ++x) {
          const float d_in = k.inv_ci * (ain + hin[x]);
          tinA[x] = tin + (d_in * k.spm) * k.slot;
          iTA[x] = (uint32_t)temp_bin(tinA[x]);
          stA[x] = strip_of(p1.y & 0xFFFFu, (int)iTA[x]);
          nrA[x] = strip_of(p1.y >> 16, (int)iTA[x]) + (uint32_t)ip_zero;
        }
      }
      // Between the rows' arrival and the next step's gathers the wave issues on the critical path
      // (the gathers' latency is the rest of the step): only what those addresses need goes there;
      // the TD target row's patch, T_m, the records and the market wait until the gathers are out.
      const Patch<QT> pprev = pat;    // the previous step's TD store
#if P2PMG_TRACE
      uint64_t tr0, tr1;
      P2PMG_STAMP(tr0);
      if (trLast) trR += tr0 - trLast;
      asm volatile("" ::"v"(row0.v[0]), "v"(row0.v[1]), "v"(row0.v[2]));
      P2PMG_STAMP(tr1);
      trW += tr1 - tr0;
      {  // calibration: the cost of one stamp (two back to back)
        uint64_t tcal;
        P2PMG_STAMP(tcal);
        trCal += tcal - tr1;
        tr1 = tcal;
      }
      trMid = tr1;  // no candidate rows (N != 2 or a battery): "round1" runs from the rows' arrival
#endif
      double soc_r = soc;  // tentative SoC of the current round
      BatPre bpre{};
      if constexpr (BAT == 2) bpre = bat_pre(soc, bcap, bk);  // shared by the step's rounds
      auto bat_rule = [&](float o, double& sr) -> float {
        if constexpr (BAT == 2) return (float)battery_rule_pre((double)o, sr, rcap, bk, bpre);
        return (float)battery_rule_r<true>((double)o, sr, bcap, rcap, bk);
      };
      // (round 0's rule for all 3 actions ahead of the rows' wait measured slower: configs[3] 57.1 ->
      // 59.5 ms, profiles/r05_ab/bat_spec0_ab.txt)
      row0 = patched(row0, a0, pat);  // ... may have hit a prefetched row

      // round 0 (P = 0: every filtered power is -0, tot = 0, even split)
      int code = (int)(cw & 0xFF);
      int act = code == 255 ? argmax3(row0) : code;
      float hp = hp_of(lv, act);
      int ip = ip_zero;
      Row4<QT> rowR = row0;
      uint32_t acts = (uint32_t)act, ips = (uint32_t)ip_zero;
      // CommunityMicrogrid._step -> HPHeating.step (community.py:184-188, heating.py:138-143) needs
      // only the final round's heat-pump power: it and the next step's row gathers are issued as soon
      // as that is known, ahead of the final round's divide-power and this step's market work
      float tin1 = tin, tm1 = tm;
      int iT1 = 0;
      uint32_t strip1 = 0, cw1 = 0, a0n = 0, aNn = 0;
      Row4<QT> row0n, rowNn, candn[3];
      Sel3M mnext{};
      auto issue_next = [&](int act_final) {
        const Sel3M m = sel3_masks(act_final);
        mnext = m;
        strip1 = __float_as_uint(sel3(m, __uint_as_float(stA[0]), __uint_as_float(stA[1]), __uint_as_float(stA[2])));
        const uint32_t nrow1 =
            __float_as_uint(sel3(m, __uint_as_float(nrA[0]), __uint_as_float(nrA[1]), __uint_as_float(nrA[2])));
        cw1 = code_of(c1);
        a0n = row0_addr(strip1, nrow1, cw1);
        aNn = TRAIN ? nrow1 : a0n;
#if P2PMG_ABLATE == 8 || P2PMG_ABLATE == 10
        row0n = fake_row(q + a0n * kQPad);
        rowNn = fake_row(q + aNn * kQPad);
#else
        // the rows round 0 and round 1 wait for first, the TD's next-state row last.  Round 0's row
        // only for the lanes that read it (a greedy round 0, or the TD target at R = 0): an exploring
        // lane's gather would be address work in the CU's memory pipeline for nothing (an exec-masked
        // load; configs[1] 79.8 -> 79.0 us, configs[3] 66.2 -> 65.3 ms at the bench's epsilon)
        {
          Row4<QT> r0{};
          if (((cw1 & 0xFF) == 255) || (TRAIN && R1 == 1)) r0 = gat(a0n);
          row0n = r0;
        }
#endif
        if constexpr (CAND) {
#pragma unroll
          for (int b = 0; b < 3; ++b) candn[b] = gat((strip1 + ((ipc1 >> (8 * b)) & 0xFFu)));
        }
#if !(P2PMG_ABLATE == 8 || P2PMG_ABLATE == 10)
        rowNn = gat(aNn);
#endif
      };
      // step t + 3's code word and round-1 bins into this step's slots (dead since step t - 1 / round 1)
      auto refill_words = [&]() {
        cS[P] = codes_a[o3];
        if constexpr (CAND) iS[P] = ipc_a[o3];
      };
      // the rest of HPHeating.step for the chosen level, once the gathers are out
      auto settle_next = [&]() {
        const Sel3M& m = mnext;
        iT1 = (int)__float_as_uint(sel3(m, __uint_as_float(iTA[0]), __uint_as_float(iTA[1]), __uint_as_float(iTA[2])));
        tin1 = sel3(m, tinA[0], tinA[1], tinA[2]);
        const float d_m = k.inv_cm * (((k.inv_ri * (tin - tm) + k.inv_re * (e0.t_out - tm)) + k.solar) +
                                      sel3(m, hm[0], hm[1], hm[2]));  // heating.py:45,48
        tm1 = tm + (d_m * k.spm) * k.slot;
      };
      if constexpr (R1 == 1) {
        issue_next(act);
        refill_words();
        settle_next();
      }
      float out0 = balw + hp;
      if constexpr (BAT != 0) {
        if (bcap > 0.0) out0 = bat_rule(out0, soc_r);
      }
      const float ev0 = div_n_r<N>(out0 * 1.0f, rn);
#pragma unroll
      for (int j = 0; j < N; ++j) row[j] = ev0;
#pragma unroll
      for (int r = 1; r < R1; ++r) {
        if (r == 1) {
          gather_even<N, 1, G>(ev0, col, i);
        } else {
          exchange<N>(row, col, i, sl, nullptr);
        }
        code = (int)((cw >> (8 * r)) & 0xFF);
        if (CAND && r == 1) {
          // the partner's round-0 action picks the prefetched row (its bin is byte b of ipc0)
          const int b = __float_as_int(shfl_xor_c<1>(__int_as_float(act)));
#if P2PMG_TRACE
          {
            uint64_t ta, tb;
            asm volatile("" ::"v"(b));
            P2PMG_STAMP(ta);
            asm volatile("" ::"v"(cand[0].v[0]), "v"(cand[1].v[0]), "v"(cand[2].v[0]), "v"(cand[0].v[2]), "v"(cand[1].v[2]),
                         "v"(cand[2].v[2]));
            P2PMG_STAMP(tb);
            trA0 += ta - tr1;
            trWC += tb - ta;
            trMid = tb;
          }
#endif
          ip = (int)((ipc0 >> (8 * b)) & 0xFFu);
          rowR = patched(sel_row(b, cand[0], cand[1], cand[2]), strip + (uint32_t)ip, pat);
        } else {
          float acc = 0.0f;
#pragma unroll
          for (int j = 0; j < N; ++j) acc = acc + (-((j == i) ? 0.0f : col[j]));
          ip = p2p_bin(fdiv_b(div_n_r<N>(acc, rn), rmi));
          const bool need = code == 255 || (TRAIN && r == R1 - 1);
#if P2PMG_ABLATE == 7
          rowR = fake_row(q + (need ? strip + (uint32_t)ip : a0) * kQPad);
#else
          rowR = gat((need ? strip + (uint32_t)ip : a0));
#endif
        }
#if P2PMG_BAT_SPEC
        // the final round's battery rule for each of the 3 actions while its row is in flight (it
        // needs only balw, the level and this step's SoC): the action then only selects
        float outA[3];
        double socA[3];
        if constexpr (BAT != 0) {
          if (r == R1 - 1) {
#pragma unroll
            for (int x = 0; x < 3; ++x) {
              socA[x] = soc;
              outA[x] = balw + hp_of(lv, x);
              if (bcap > 0.0) outA[x] = bat_rule(outA[x], socA[x]);
            }
          }
        }
#endif
        act = code == 255 ? argmax3(rowR) : code;
        acts |= (uint32_t)act << (8 * r);
        ips |= (uint32_t)ip << (8 * r);
        hp = hp_of(lv, act);
        if (r == R1 - 1) {
#if P2PMG_TRACE
          {
            uint64_t tc;
            asm volatile("" ::"v"(act));
            P2PMG_STAMP(tc);
            trA1 += tc - trMid;
            trMid = tc;
          }
#endif
          issue_next(act);
#if P2PMG_TRACE
          P2PMG_STAMP(trLast);
          trC += trLast - trMid;
#endif
          refill_words();
          settle_next();
        }
        float out = balw + hp;
        if constexpr (BAT != 0) {
#if P2PMG_BAT_SPEC
          if (r == R1 - 1) {
            const Sel3M m = sel3_masks(act);
            out = sel3(m, outA[0], outA[1], outA[2]);
            soc_r = sel3(m, socA[0], socA[1], socA[2]);
          } else
#endif
          {
            soc_r = soc;
            if (bcap > 0.0) out = bat_rule(out, soc_r);
          }
        }
#if P2PMG_ABLATE == 11  // timing-only: no final-round divide-power and no market (cost from out alone)
        if (r == R1 - 1) {
          row[0] = out;
          continue;
        }
#endif
        // _divide_power's filter keeps pw where sign(out) != sign(pw) (agent.py:187-188): for out > 0
        // that is pw <= 0, for out < 0 pw >= 0, for out = 0 any pw.  A kept pw = +-0 and a dropped
        // one (0) are interchangeable: every later use is |f| or a sum that already holds +0.
        // As one clamp: f = med3(pw, out < 0 ? 0 : -inf, out > 0 ? 0 : +inf).
        const float flo = out < 0.0f ? 0.0f : -__builtin_inff(), fhi = out > 0.0f ? 0.0f : __builtin_inff();
        float f[N];
        float tot = 0.0f;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          const float pw = -((j == i) ? 0.0f : col[j]);
          f[j] = __builtin_amdgcn_fmed3f(pw, flo, fhi);
          tot = tot + f[j];
        }
        tot = fabsf(tot);
        const float ev = div_n_r<N>(out * 1.0f, rn);
        // out * |f_j| / tot for every j: the diagonal's f_ii = +-0 gives out * 0 / tot = out * 0, the
        // reference's value for it (agent.py:193-194), for any tot > 0.  One range guard per round.
        const Recip rt = recip(tot == 0.0f ? 1.0f : tot);  // the tot = 0 lanes take ev
        const float nout = nabs_out(out);
        float num[N];
        bool bad = !rt.ok;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          num[j] = nout * f[j];
          row[j] = fdiv_core(num[j], rt);
          bad = bad || !fdiv_ok(num[j]);
        }
        if (bad) {
#pragma unroll
          for (int j = 0; j < N; ++j) row[j] = fdiv_ieee(num[j], rt.b);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) row[j] = (tot == 0.0f) ? ev : row[j];
      }
      soc = soc_r;  // BatteryStorage state after the final round's decision
      pat.row = 0xFFFFFFFFu;  // the next step's rows were issued after the previous TD store

      // CommunityMicrogrid._assign_powers community.py:45-54 on the final P (diagonal kept)
      float g = 0.0f, pp = 0.0f;
#if P2PMG_ABLATE == 11
      g = row[0];
#else
      exchange<N>(row, col, i, sl, nullptr);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        // ex = sign(pij) * min(|pij|, |pji|) where the signs differ (community.py:48-50)
        const float pij = row[j], pji = col[j];
        const float ex = pair_exchange(pij, pji);
        g = g + (pij - ex);
        pp = pp + ex;
      }
#endif
      // CommunityMicrogrid._compute_costs community.py:56-65
      float cost = (g >= 0.0f) ? g * e0.buy : g * e0.inj;
      cost = cost + pp * e0.p2p;
      cost = fdiv_b(cost * k.slot, rmph);
      cost = cost * k.kilo;
      // RLAgent.get_reward agent.py:225-232 (pre-update T_in)
      float pen = fmaxf(fmaxf(0.0f, k.lower - tin), fmaxf(0.0f, tin - k.upper));
      pen = pen > 0.0f ? pen + 1.0f : 0.0f;
      const float rw = -(cost + k.penw * pen);

      if constexpr (TRAIN) {
        // QAgent.train agent.py:293-298 -> QActor.train rl.py:119-129
        const uint32_t srow = strip + (uint32_t)ip;
        const QT qsa = sel3(act, rowR.v[0], rowR.v[1], rowR.v[2]);
        const QT qnew = td_update(qsa, rw, max3(patched(rowN, aN, pprev)), k.alpha, k.gamma);
        *(active ? q + srow * kQPad + act : q_dummy) = qnew;
#if P2PMG_ABLATE == 9 || P2PMG_ABLATE == 10
        pat = Patch<QT>{0xFFFFFFFFu, 0, (QT)0};  // timing-only: the next step does not wait for this TD
#else
        pat = Patch<QT>{srow, act, qnew};  // rows issued before this store see the old value
#endif
      }
      if constexpr (narrow) {
        *reinterpret_cast<float2*>(__builtin_assume_aligned(rec_ptr, 8)) = make_float2(rw, cost);
      } else {
        const uint32_t bins = (p0.y & 0xFFFFu) | ((uint32_t)iT << 16);  // it * nT*nb + ib | iT << 16
        float4* rp = reinterpret_cast<float4*>(__builtin_assume_aligned(rec_ptr, 16));
        rp[0] = make_float4(rw, cost, g, pp);
        rp[1] = make_float4(tin, __uint_as_float(acts), __uint_as_float(bins), __uint_as_float(ips));
      }
      rec_ptr += rec_step;
      // step t's env row and pre-pass word are dead: step t + 3's into their slots (the barrier keeps
      // the scheduler from hoisting the loads above the old values' last use, which would need a
      // second register set and a copy at the loop's back edge)
      asm volatile("" ::: "memory");
      eS[P] = load_envv(envb + eo3);
      pS[P] = preb[o3];
      // avg_reward = sum_t mean_i r (community.py:179), canonical sequential order
      const float m = group_sum<N>(rw, lane, i, sl, nullptr);
      ep_sum = ep_sum + div_n_r<N>(m, rn);

      tin = tin1;
      tm = tm1;
      iT = iT1;
      o3 += (uint32_t)A;
      o3 = o3 == TA ? 0u : o3;
      eo3 += env_st;
      eo3 = eo3 == env_end ? 0u : eo3;
      strip = strip1;
      cw = cw1;
      a0 = a0n;
      aN = aNn;
      row0 = row0n;
      rowN = rowNn;
      if constexpr (CAND) {
#pragma unroll
        for (int b = 0; b < 3; ++b) cand[b] = candn[b];
      }
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using S2 = std::integral_constant<int, 2>;
    int t = 0;
    for (; t + 3 <= T; t += 3) {
      step(S0{});
      step(S1{});
      step(S2{});
    }
    if (t < T) step(S0{});
    if (t + 1 < T) step(S1{});
#if P2PMG_TRACE
    if (threadIdx.x == 0 && (blockIdx.x == 0 || (int)blockIdx.x == n_cons / 2 || (int)blockIdx.x == n_cons - 1))
      printf("TRACE blk %d/%d T %d: per step wait %.1f round0 %.1f waitcand %.1f round1 %.1f issue %.1f rest %.1f "
             "(one stamp %.1f)\n",
             (int)blockIdx.x, n_cons, T, (double)trW / T, (double)trA0 / T, (double)trWC / T, (double)trA1 / T,
             (double)trC / T, (double)trR / (T - 1), (double)trCal / T);
#endif
    if (active) {
      if (p.reset_t0) {  // agent.reset() at the end of train_episode (community.py:181), fused
        tin = t0_in;
        tm = t0_m;
      }
      if (i == 0) {
        if (p.chain_rewards) p.chain_rewards[(size_t)ep * p.S + s] = ep_sum;
        if (ep == n_chain - 1) p.ep_reward[s] = ep_sum;
      }
    }
  }  // chain
  if (active) {
    p.t_in[a] = tin;
    p.t_m[a] = tm;
    if constexpr (BAT != 0) p.soc[a] = soc;
  }
}

// FastRec rows -> the general record buffers (reward, cost, grid, p2p, tin [T][A]; action u8 and
// packed index i32 [T][R+1][A]), for the records the caller asks for
#if P2PMG_IN_PART(0)
__global__ void fast_rec_unpack_kernel(int T, int R1, int A, uint32_t tb, const FastRec* __restrict__ recs, int narrow,
                                       int which, void* __restrict__ out) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // k = t * A + a
  if (k >= (size_t)T * A) return;
  if (narrow) {  // [T][A] float2 {reward, cost}
    const float2 v = reinterpret_cast<const float2*>(recs)[k];
    reinterpret_cast<float*>(out)[k] = which == 0 ? v.x : v.y;
    return;
  }
  const FastRec r = recs[k];
  if (which < 5) {
    const float v[5] = {r.reward, r.cost, r.grid, r.p2p, r.tin};
    reinterpret_cast<float*>(out)[k] = v[which];
    return;
  }
  const size_t t = k / A, a = k % A;
  for (int rr = 0; rr < R1; ++rr) {
    const size_t kk = (t * R1 + rr) * A + a;
    if (which == 5)
      reinterpret_cast<uint8_t*>(out)[kk] = (uint8_t)(r.actions >> (8 * rr));
    else
      reinterpret_cast<int32_t*>(out)[kk] = (int32_t)(((r.bins & 0xFFFFu) / tb) | ((r.bins >> 16) << 8) |
                                                      (((r.bins & 0xFFFFu) % tb) << 16) | (((r.ips >> (8 * rr)) & 0xFFu) << 24));
  }
}
#endif

// hipExtLaunchKernel stamps the start / stop events from the dispatch itself: no marker packets
// between back-to-back episodes
template <int N, typename QT, int R1, int BAT, bool NARROW>
void launch_fast_nw(const EpisodeParams& p, const uint2* pre, FastRec* recs, int blocks, int spw, int prod,
                    const PrepOut& nxt, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  if (p.mode == 0)
    hipExtLaunchKernelGGL((episode_fast_kernel<N, QT, R1, true, BAT, NARROW>), dim3(blocks + prod), dim3(kWave), 0, st,
                          ev0, ev1, 0, p, pre, recs, spw, blocks, nxt);
  else
    hipExtLaunchKernelGGL((episode_fast_kernel<N, QT, R1, false, BAT, NARROW>), dim3(blocks + prod), dim3(kWave), 0, st,
                          ev0, ev1, 0, p, pre, recs, spw, blocks, nxt);
}
template <int N, typename QT, int R1, int BAT>
void launch_fast_b(const EpisodeParams& p, const uint2* pre, FastRec* recs, int blocks, int spw, int prod,
                   const PrepOut& nxt, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  if (p.rec_narrow) return launch_fast_nw<N, QT, R1, BAT, true>(p, pre, recs, blocks, spw, prod, nxt, ev0, ev1, st);
  launch_fast_nw<N, QT, R1, BAT, false>(p, pre, recs, blocks, spw, prod, nxt, ev0, ev1, st);
}
template <int N, typename QT, int R1>
void launch_fast_r(const EpisodeParams& p, const uint2* pre, FastRec* recs, int blocks, int spw, int prod,
                   const PrepOut& nxt, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  if constexpr (R1 <= kFastBatMaxR1) {
    if (p.battery && p.bat_safe) return launch_fast_b<N, QT, R1, 2>(p, pre, recs, blocks, spw, prod, nxt, ev0, ev1, st);
    if (p.battery) return launch_fast_b<N, QT, R1, 1>(p, pre, recs, blocks, spw, prod, nxt, ev0, ev1, st);
  }
  launch_fast_b<N, QT, R1, 0>(p, pre, recs, blocks, spw, prod, nxt, ev0, ev1, st);
}

template <int N, typename QT>
hipError_t launch_fast_n(const EpisodeParams& p, const uint2* pre, void* recs, int spw, const PrepOut* nxt,
                         hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  constexpr int G = pow2ceil(N);
  if (spw <= 0 || spw > kWave / G) spw = kWave / G;
  const int blocks = (p.S + spw - 1) / spw;
  const size_t n = (size_t)p.T * p.A;
  const int prod = nxt ? (int)std::min<size_t>(2048, (n + kWave - 1) / kWave) : 0;
  const PrepOut none{nullptr, nullptr, nullptr, 0, 0.0};
  FastRec* r = reinterpret_cast<FastRec*>(recs);
  switch (p.R + 1) {
    case 1: launch_fast_r<N, QT, 1>(p, pre, r, blocks, spw, prod, nxt ? *nxt : none, ev0, ev1, st); break;
    case 2: launch_fast_r<N, QT, 2>(p, pre, r, blocks, spw, prod, nxt ? *nxt : none, ev0, ev1, st); break;
    case 3: launch_fast_r<N, QT, 3>(p, pre, r, blocks, spw, prod, nxt ? *nxt : none, ev0, ev1, st); break;
    case 4: launch_fast_r<N, QT, 4>(p, pre, r, blocks, spw, prod, nxt ? *nxt : none, ev0, ev1, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// agents per scenario N0 and N0 + 1, f64 or f32 table
template <int N0>
hipError_t launch_fast_pair(const EpisodeParams& p, const uint2* pre, void* recs, int q_dtype, int spw,
                            const PrepOut* nxt, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  if (p.N == N0)
    return q_dtype == 0 ? launch_fast_n<N0, double>(p, pre, recs, spw, nxt, ev0, ev1, st)
                        : launch_fast_n<N0, float>(p, pre, recs, spw, nxt, ev0, ev1, st);
  if (p.N == N0 + 1)
    return q_dtype == 0 ? launch_fast_n<N0 + 1, double>(p, pre, recs, spw, nxt, ev0, ev1, st)
                        : launch_fast_n<N0 + 1, float>(p, pre, recs, spw, nxt, ev0, ev1, st);
  return hipErrorInvalidValue;
}

// __double2ll_rn(x) in two VALU ops while |x| < 2^51: y = x + 1.5 * 2^52 lies in [2^52, 2^53), where
// the f64 spacing is 1, so the add IS the round-to-nearest-even, and the integer sits in y's
// significand: int64 = bits(y) - bits(1.5 * 2^52), whose low word is 0 (only the high word changes,
// no borrow).  Otherwise (a TD delta of 2^11 or more, wave-uniformly tested) the library conversion.
__device__ __forceinline__ long long rne_ll(double x) {
  if (__all(fabs(x) < 0x1p51)) {
    const double y = x + 0x1.8p52;
    const unsigned lo = (unsigned)__double2loint(y);
    const unsigned hi = (unsigned)__double2hiint(y) - 0x43380000u;
    return (long long)(((unsigned long long)hi << 32) | lo);
  }
  return __double2ll_rn(x);
}

// ----------------------------------------------------------------- the fast shared-table path (N = 16)
typedef float pkf2 __attribute__((ext_vector_type(2)));
// v with lane (16 k + J) set to +0 for every k: the diagonal of a 16-agent scenario whose agent i
// sits in lane i of its 16-lane group.  The lane pattern is a constant loaded into VCC right at the
// use: as a C++ compare, the 16 loop-invariant masks get hoisted into 32 SGPRs, spill to VGPR lanes
// and cost two v_readlane per use.
template <int J>
__device__ __forceinline__ float zero_diag16(float v) {
  float r;
  asm volatile("s_mov_b32 vcc_lo, %2\n\ts_mov_b32 vcc_hi, %2\n\tv_cndmask_b32_e64 %0, %1, 0, vcc"
               : "=v"(r) : "v"(v), "i"(0x00010001u << J) : "vcc");
  return r;
}
template <int J = 0>
__device__ __forceinline__ void zero_diag16_all(float (&col)[16]) {
  if constexpr (J < 16) {
    col[J] = zero_diag16<J>(col[J]);
    zero_diag16_all<J + 1>(col);
  }
}
// 0 or |x| in [2^-19, 2^19]: products of two such numbers are 0 or in [2^-38, 2^38]
__device__ __forceinline__ bool in_range19(float x) {
  const float m = fabsf(x);
  return m == 0.0f || (m >= 0x1p-19f && m <= 0x1p19f);
}
// fdiv_core on a packed pair with the residual negated, r' = b q0 - a: the same quotient bit for
// bit (round-to-nearest is sign-symmetric, and an exact-zero residual is +0 either way, which
// leaves q unchanged), and for a = +-0 with a POSITIVE divisor (the only use: tot = |sum| > 0) it
// keeps sign(a) without fdiv_core's copysign: q0 = +-0, r' = +0, q = fma(-0, y, +-0) = +-0.  (With
// a negative divisor q0 = -+0 and the last fma returns +0 for a = +0: not the IEEE -0; the division
// fuzz test checks the positive-divisor domain.)  Both lanes round like the scalar fma.
__device__ __forceinline__ pkf2 fdiv_core_pk(pkf2 a, pkf2 b, pkf2 y) {
  // q0 as two scalar multiplies: v_mul_f32 issues at 2.6 SIMD cycles, v_pk_mul_f32 at 6.6
  // (profiles/r04_ubench_rate.jsonl); the FMAs stay packed (v_pk_fma_f32 6.8 < 2 x 3.8)
  const pkf2 q0 = {a.x * y.x, a.y * y.y};
  const pkf2 r = __builtin_elementwise_fma(b, q0, -a);
  return __builtin_elementwise_fma(-r, y, q0);  // one correction, as fdiv_core
}
// episode_sq16_kernel: episode_kernel's shared-table path for 16-agent scenarios (configs[2]),
// rebuilt for throughput: 1M scenarios keep every SIMD busy, so the cost is instructions per
// agent-step, not latency.  Same op order and results as episode_kernel (tests compare both).
//   * round 0 is an even split: round 1's column is the 16 round-0 values of the group, one LDS
//     write + four 16-B reads instead of a 16 x 16 exchange;
//   * the divisions of _divide_power share one divisor per round (hoisted reciprocal), the
//     battery's f64 divisions share the agent's capacity / sqrt(eff) / 900 s reciprocals;
//   * the final 16 x 16 proposal matrix is transposed through a swizzled LDS tile (4 x 16-B
//     writes, 16 conflict-free 4-B reads);
//   * the table is frozen for the episode: TD deltas go to the workgroup's LDS hash as before.
#ifndef P2PMG_SQ16_OCC
#define P2PMG_SQ16_OCC 4  // min waves per SIMD the register allocation must allow (LDS allows 4)
#endif
constexpr int kSq16Waves = 8;                        // waves per workgroup (one hash per 32 scenarios)
constexpr int kTpStride = 16 * 16 + 16;              // floats per scenario tile (+16: bank offset)
// BAT: 0 none, 1 battery with per-lane range tests, 2 battery in the launcher-verified domain
template <typename QT, int R1, bool TRAIN, int BAT, bool NARROW>
__global__ __launch_bounds__(kWave * kSq16Waves, P2PMG_SQ16_OCC) void episode_sq16_kernel(const EpisodeParams p) {
  constexpr int N = 16, G = 16, SPW = kWave / G;
  __shared__ uint32_t hkey[kSqSlots];
  __shared__ unsigned long long hval[kSqSlots];
  __shared__ double tdk[2];  // {alpha, gamma} of the TD update, read per step (see below)
  __shared__ __attribute__((aligned(16))) float tpall[kSq16Waves * SPW * kTpStride];
  const int wv = (int)(threadIdx.x / kWave);
  const int lane = (int)(threadIdx.x % kWave);
  const int sl = lane / G;
  const int i = lane % G;
  const int s = (blockIdx.x * kSq16Waves + wv) * SPW + sl;
  const bool active = s < p.S;
  const int a = active ? s * N + i : 0;
  const int s_env = p.n_env == 1 ? 0 : (active ? s : 0);
  const int T = p.T;
  const size_t A = (size_t)p.A;
  const KC k = scalar_constants(p);
  const Dims<true> D{k.nt, k.nT, k.nb, k.np};
  // the launcher sends this kernel 20^4 tables only (p2pmg_runtime.cpp, sq16 dispatch): the state
  // count is a literal, not four kernel arguments kept in SGPRs across the loop
  constexpr uint32_t n_states = 20u * 20u * 20u * 20u;
  const QT* __restrict__ q = reinterpret_cast<const QT*>(p.q);
  unsigned long long* const dbase = reinterpret_cast<unsigned long long*>(p.qdelta) +
                                    (size_t)(blockIdx.x % kDeltaCopies) * n_states * kQPad;
  for (int k2 = threadIdx.x; k2 < kSqSlots; k2 += kSq16Waves * kWave) {
    hkey[k2] = kSqEmpty;
    hval[k2] = 0;
  }
  if (threadIdx.x == 0) {
    tdk[0] = p.alpha;
    tdk[1] = p.gamma;
  }
  __syncthreads();
  float* const tp = tpall + (wv * SPW + sl) * kTpStride;  // this scenario's tile
  // column reads of the transpose: element i of row j sits at j*16 + 4*((i>>2) ^ (j&3)) + (i&3)
  int cofs[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) cofs[m] = 4 * ((i >> 2) ^ m) + (i & 3);

  const float mi = active ? p.max_in[a] : 1.0f;
  const Recip rmi = recip(mi), rmph = recip_u(k.mph), rmargin = recip_u(k.margin);
  const float4 lv = p.hp_lv[a];
  // margin == 1 (the reference's) tested per step as a scalar compare of its bits: a loop-invariant
  // bool would be kept as a 64-bit lane mask across the loop (two SGPRs, spilled to VGPR lanes)
  const uint32_t margin_bits = __float_as_uint(p.margin);
  auto margin_one = [&]() __attribute__((always_inline)) {
    uint32_t r;
    asm volatile("s_cmp_eq_u32 %1, 0x3f800000\n\ts_cselect_b32 %0, 1, 0" : "=s"(r) : "s"(margin_bits) : "scc");
    return r != 0;
  };
  double bcap = 0.0, soc = 0.0;
  BatK bk{};
  Recip64 rcap{};
  if constexpr (BAT != 0) {
    bcap = p.bat_cap[a];
    soc = p.soc[a];
    bk = BatK{p.bat_min, p.bat_max, p.bat_sqrt_eff, recip64_u(p.bat_sqrt_eff), kR900};
    rcap = recip64(bcap > 0.0 ? bcap : 1.0);
  }
  float tin = active ? p.t_in[a] : k.setpoint;
  float tm = active ? p.t_m[a] : k.setpoint;
  const int ip_zero = idx_plain(div_n<N>(0.0f) / mi, D.p());
  const int R1r = p.R + 1, W = (R1r + 3) >> 2;

  // running element offsets in 32 bits (the launcher checks T * A * W < 2^32 and the env table
  // size): fewer 64-bit uniform values live across the loop, i.e. fewer SGPR spills
  // (one wrapped step index, t + 2 mod T, and the offsets as scalar products of it: fewer uniform
  // values live across the loop than three running offsets and their wrap points)
  const float* envb = p.env + (size_t)s_env * kEnvStride;
  const uint32_t env_step = (uint32_t)p.n_env * kEnvStride;
  // the policy-independent per-step words {balance, it * 8000 + ib * 20} (sq16_prep_kernel)
  const uint2* sqpb = p.sqp + a;
  const uint32_t A32 = (uint32_t)p.A;
  const uint32_t* codes_a = p.codes + a;
  const uint32_t code_step = (uint32_t)W * A32;
  const uint32_t T32 = (uint32_t)T;
  const uint32_t t1 = T32 > 1 ? 1u : 0u;
  uint32_t t2 = (2u % T32);  // step t + 2 (mod T) of the loop's iteration t
  const uint32_t f1o = t1 * A32;
  // records: FastRec rows, or only {reward, cost} as float2 when nothing else was requested
  // (8 B instead of 32 B of writes per agent-step); masked-off lanes write a dummy row.  Compile
  // time, as in the fast kernel: no store-count branch for the vmcnt bookkeeping to be pessimistic about
  constexpr bool narrow = NARROW;
  const size_t rec_bytes = narrow ? sizeof(float2) : sizeof(FastRec);
  char* const rec_dummy = reinterpret_cast<char*>(reinterpret_cast<FastRec*>(p.dummy) + kWave + lane);
  const bool rec_on = p.record != 0 && active;
  char* rec_ptr = rec_on ? reinterpret_cast<char*>(p.rec_pack) + (size_t)a * rec_bytes : rec_dummy;
  const size_t rec_step = rec_on ? A * rec_bytes : 0;

  const uint2 w0 = sqpb[0];
  uint2 w1 = sqpb[f1o];
  // step t's state: the balance and the time / balance part of the row offset come precomputed
  // (w: step t, wn: step t + 1 for the next-state row); only the temperature bin depends on the
  // policy: rl.py:89-95 as one v_med3 + convert (clamp_bin_f == clamp_bin for every non-NaN value)
  auto step_idx = [&](uint2 w, uint2 wn, float t_in) {
    StepIdx st;
    st.bal = __uint_as_float(w.x);
    const float dt = t_in - k.setpoint;
    const float tnorm = margin_one() ? dt : fdiv_b(dt, rmargin);
    st.iT = clamp_bin_f(((tnorm + 1.0f) / 2.0f) * 18.0f + 1.0f, 19.0f);
    const uint32_t tT = __umul24((uint32_t)st.iT, 400u);
    st.strip = w.y + tT;
    st.nrow = wn.y + tT + (uint32_t)ip_zero;
    st.it = (int)w.y;  // it * 8000 + ib * 20: the records' bins are w.y / 20 (records only)
    return st;
  };
  // the shared table's rows as 32-bit offsets from its (uniform) base: global_load's SGPR-base +
  // VGPR-offset form instead of a 64-bit address per row (the table spans < 4 GiB)
  const char* const qb = reinterpret_cast<const char*>(q);
  constexpr uint32_t kRowShift = sizeof(QT) == 8 ? 5 : 4;
  auto gatq = [&](uint32_t row) __attribute__((always_inline)) {
    return gather_row(reinterpret_cast<const QT*>(qb + (row << kRowShift)));
  };
  StepIdx st = step_idx(w0, w1, tin);
  // R + 1 = 2 in-kernel Philox: one block holds the codes of two steps (p2pmg_device.h), computed
  // at the even step and kept for the odd one in the code word's unused high half
  constexpr bool kPair = R1 == 2 && TRAIN;
  const bool rng1 = p.rng == 1;
  auto block2 = [&](uint32_t blk) -> uint64_t {
    const uint32_t c4 = philox_block_codes(blk, (uint32_t)p.episode, p.agent_offset + (uint32_t)a, p.eps_thr, p.eps_all,
                                           p.seed_lo, p.seed_hi);
    return (uint64_t)(c4 & 0xFFFFu) | ((uint64_t)(c4 >> 16) << 32) | 0xFFFF0000FFFF0000ull;
  };
  uint64_t cw = code_word_t<TRAIN>(p, step_codes(p, codes_a, 0, 0, a, W, !kPair));
  if (kPair && rng1) cw = block2(0);
  auto row0_addr = [&](const StepIdx& x, uint64_t c) -> uint32_t {
    const bool need = ((c & 0xFF) == 255) || (TRAIN && R1 == 1);
    return need ? x.strip + (uint32_t)ip_zero : x.nrow;
  };
  uint32_t a0 = row0_addr(st, cw);
  Row4<QT> row0 = gatq(a0);
  Row4<QT> rowN = gatq(TRAIN ? st.nrow : a0);
  float ep_sum = 0.0f;

  for (int t = 0; t < T; ++t) {
    const uint32_t t1n = t + 1 == T ? 0u : (uint32_t)t + 1u;  // step t + 1 (mod T)
    // step t's env row {t_out, prices} at the top of the step, not carried across the loop: its first
    // use (the RC update) is half a step of this wave's issue away, which the SIMD's other waves fill
    const EnvRow e0 = load_env(envb + (uint32_t)t * env_step);
    const uint2 w2 = sqpb[t2 * A32];
    const CodeWords cw1r = step_codes(p, codes_a, t1n * code_step, (int)t1n, a, W, !kPair);
    const float balw = st.bal * mi;
    float row[N];
    float col[N];

    // round 0 (P = 0: even split); the battery adjusts the tentative net power
    int code = (int)(cw & 0xFF);
    int act = code == 255 ? argmax3(row0) : code;
    float hp = hp_of(lv, act);
    int ip = ip_zero;
    Row4<QT> rowR = row0;
    uint32_t acts = (uint32_t)act, ips = (uint32_t)ip_zero;
    double soc_r = soc;
    float out = balw + hp;
    BatPre bpre{};
    if constexpr (BAT == 2) bpre = bat_pre(soc, bcap, bk);  // shared by the step's two rounds
    auto bat_rule = [&](float o, double& sr) -> float {
      if constexpr (BAT == 2) return (float)battery_rule_pre((double)o, sr, rcap, bk, bpre);
      return (float)battery_rule_r<true>((double)o, sr, bcap, rcap, bk);
    };
    if constexpr (BAT != 0) {
      if (bcap > 0.0) out = bat_rule(out, soc_r);
    }
    const float ev0 = div_n<N>(out * 1.0f);
    const bool ok_ev0 = in_range19(ev0);
#pragma unroll
    for (int j = 0; j < N; ++j) row[j] = ev0;
    if constexpr (R1 == 2) {
      // round 1: the column is the group's 16 round-0 values
      tp[i] = ev0;
      wave_lds_fence();
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float4 v = *reinterpret_cast<const float4*>(tp + 4 * m);
        col[4 * m] = v.x; col[4 * m + 1] = v.y; col[4 * m + 2] = v.z; col[4 * m + 3] = v.w;
      }
      wave_lds_fence();
      zero_diag16_all(col);  // powers = -P[:, i] with P's diagonal zeroed (community.py:76,81)
      float acc = 0.0f;
#pragma unroll
      for (int j = 0; j < N; ++j) acc = acc + (-col[j]);
      ip = clamp_bin_f(((fdiv_b(div_n<N>(acc), rmi) + 1.0f) / 2.0f) * 20.0f, 19.0f);
      code = (int)((cw >> 8) & 0xFF);
      const bool need = code == 255 || TRAIN;
      rowR = gatq(need ? st.strip + (uint32_t)ip : a0);
      act = code == 255 ? argmax3(rowR) : code;
      acts |= (uint32_t)act << 8;
      ips |= (uint32_t)ip << 8;
      hp = hp_of(lv, act);
      out = balw + hp;
      soc_r = soc;
      if constexpr (BAT != 0) {
        if (bcap > 0.0) out = bat_rule(out, soc_r);
      }
      const float flo = out < 0.0f ? 0.0f : -__builtin_inff(), fhi = out > 0.0f ? 0.0f : __builtin_inff();
      float f[N];
      float tot = 0.0f;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        f[j] = __builtin_amdgcn_fmed3f(-col[j], flo, fhi);
        tot = tot + f[j];
      }
      tot = fabsf(tot);
      const float ev = div_n<N>(out * 1.0f);
      const Recip rt = recip(tot == 0.0f ? 1.0f : tot);
      const float nout = nabs_out(out);
      float num[N];
#pragma unroll
      for (int j = 0; j < N; ++j) num[j] = nout * f[j];
      // One wave-uniform range guard instead of one per quotient: the column holds the group's
      // round-0 values, each vouched for by its own lane (ok_ev0), so with out also in range
      // every numerator is 0 or in [2^-38, 2^38] and the packed Newton quotient is exact.
      if (__all(ok_ev0 && in_range19(out) && rt.ok)) {
        const pkf2 y2 = {rt.y, rt.y}, b2 = {rt.b, rt.b};
#pragma unroll
        for (int j = 0; j < N; j += 2) {
          const pkf2 q2 = fdiv_core_pk(pkf2{num[j], num[j + 1]}, b2, y2);
          row[j] = q2.x;
          row[j + 1] = q2.y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) row[j] = fdiv_b(num[j], rt);
        if (!rt.ok) {
#pragma unroll
          for (int j = 0; j < N; ++j) row[j] = fdiv_ieee(num[j], rt.b);
        }
      }
      // tot = 0 (every peer's power on out's side of zero) is rare among 16 peers: one wave-uniform
      // test instead of 16 selects on every step
      if (__any(tot == 0.0f)) {
#pragma unroll
        for (int j = 0; j < N; ++j) row[j] = (tot == 0.0f) ? ev : row[j];
      }
    }
    soc = soc_r;

    // RC update and the next step's rows
    float tin1 = tin, tm1 = tm;
    rc_update(k, e0.t_out, hp, tin1, tm1);
    const StepIdx st1 = step_idx(w1, w2, tin1);
    uint64_t cw1 = code_word_t<TRAIN>(p, cw1r);
    if constexpr (kPair) {
      if (rng1) cw1 = (t1n & 1u) ? ((cw >> 32) | 0xFFFFFFFF00000000ull) : block2(t1n >> 1);
    }
    const uint32_t a0n = row0_addr(st1, cw1);
    const Row4<QT> row0n = gatq(a0n);
    const Row4<QT> rowNn = gatq(TRAIN ? st1.nrow : a0n);

    // the final P's column through the swizzled tile (community.py:45-54 needs P[j][i])
#pragma unroll
    for (int m = 0; m < 4; ++m)
      *reinterpret_cast<float4*>(tp + i * 16 + 4 * (m ^ (i & 3))) =
          make_float4(row[4 * m], row[4 * m + 1], row[4 * m + 2], row[4 * m + 3]);
    wave_lds_fence();
#pragma unroll
    for (int j = 0; j < N; ++j) col[j] = tp[j * 16 + cofs[j & 3]];
    wave_lds_fence();
    // ex = sign(pij) min(|pij|, |pji|) where the signs differ (community.py:48-50), one v_med3
    float g = 0.0f, pp = 0.0f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float pij = row[j], pji = col[j];
      const float ex = pair_exchange(pij, pji);
      g = g + (pij - ex);
      pp = pp + ex;
    }
    float cost = (g >= 0.0f) ? g * e0.buy : g * e0.inj;
    cost = cost + pp * e0.p2p;
    cost = fdiv_b(cost * k.slot, rmph);
    cost = cost * k.kilo;
    float pen = fmaxf(fmaxf(0.0f, k.lower - tin), fmaxf(0.0f, tin - k.upper));
    pen = pen > 0.0f ? pen + 1.0f : 0.0f;
    const float rw = -(cost + k.penw * pen);

    if constexpr (TRAIN) {
      if (active) {
        const QT qsa = sel3(act, rowR.v[0], rowR.v[1], rowR.v[2]);
        // alpha and gamma from LDS through an address the compiler cannot hoist: a broadcast LDS
        // read per step instead of four SGPRs held across the loop (spilled to VGPR lanes and read
        // back with v_readlane on the VALU)
        typedef __attribute__((address_space(3))) const double lds_double;
        uint32_t tdk_addr = (uint32_t)(uintptr_t)(lds_double*)tdk;
        asm volatile("" : "+s"(tdk_addr));
        lds_double* tdp = (lds_double*)(uintptr_t)tdk_addr;
        const double k_alpha = tdp[0], k_gamma = tdp[1];
        const double d = k_alpha * (((double)rw + k_gamma * (double)max3(rowN)) - (double)qsa);
        const long long dv = rne_ll(d * kDeltaScale);
#if P2PMG_SQ_ABL == 1
        if (dv == 0x7123456789LL)  // timing-only ablation: no hash insert (never true in practice)
#endif
        lds_add_by_key(hkey, hval, (st.strip + (uint32_t)ip) * kQPad + (uint32_t)act, dv, dbase);
      }
    }
    if constexpr (narrow) {
      *reinterpret_cast<float2*>(__builtin_assume_aligned(rec_ptr, 8)) = make_float2(rw, cost);
    } else {
      const uint32_t bins = ((uint32_t)st.it / 20u) | ((uint32_t)st.iT << 16);  // it * 400 + ib
      float4* rp = reinterpret_cast<float4*>(__builtin_assume_aligned(rec_ptr, 16));
      rp[0] = make_float4(rw, cost, g, pp);
      rp[1] = make_float4(tin, __uint_as_float(acts), __uint_as_float(bins), __uint_as_float(ips));
    }
    rec_ptr += rec_step;
    // avg_reward = sum_t mean_i r (community.py:179): the group's rewards in agent order
    tp[i] = rw;
    wave_lds_fence();
    float msum = 0.0f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float4 v = *reinterpret_cast<const float4*>(tp + 4 * m);
      msum = msum + v.x; msum = msum + v.y; msum = msum + v.z; msum = msum + v.w;
    }
    wave_lds_fence();
    ep_sum = ep_sum + div_n<N>(msum);
    if constexpr (TRAIN) {
      if (t % kSqFlushSteps == kSqFlushSteps - 1 || t + 1 == T)
        lds_hash_flush(hkey, hval, dbase, kSq16Waves * kWave);
    }

    tin = tin1;
    tm = tm1;
    w1 = w2;
    t2 = t2 + 1u == T32 ? 0u : t2 + 1u;
    st = st1;
    cw = cw1;
    a0 = a0n;
    row0 = row0n;
    rowN = rowNn;
  }
  if (active) {
    if (p.reset_t0)
      t0_draw(p.seed_lo, p.seed_hi, p.episode + 1, p.agent_offset + (uint32_t)a, p.setpoint, p.reset_sigma, tin, tm);
    p.t_in[a] = tin;
    p.t_m[a] = tm;
    if constexpr (BAT != 0) p.soc[a] = soc;
    if (i == 0) p.ep_reward[s] = ep_sum;
  }
}

template <typename QT, int R1, bool NARROW>
void launch_sq16_nw(const EpisodeParams& p, int blocks, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  const dim3 g(blocks), b(kWave * kSq16Waves);
  const int bat = !p.battery ? 0 : (p.bat_safe ? 2 : 1);
  if (p.mode == 0) {
    if (bat == 2) hipExtLaunchKernelGGL((episode_sq16_kernel<QT, R1, true, 2, NARROW>), g, b, 0, st, ev0, ev1, 0, p);
    else if (bat == 1) hipExtLaunchKernelGGL((episode_sq16_kernel<QT, R1, true, 1, NARROW>), g, b, 0, st, ev0, ev1, 0, p);
    else hipExtLaunchKernelGGL((episode_sq16_kernel<QT, R1, true, 0, NARROW>), g, b, 0, st, ev0, ev1, 0, p);
  } else {
    if (bat == 2) hipExtLaunchKernelGGL((episode_sq16_kernel<QT, R1, false, 2, NARROW>), g, b, 0, st, ev0, ev1, 0, p);
    else if (bat == 1) hipExtLaunchKernelGGL((episode_sq16_kernel<QT, R1, false, 1, NARROW>), g, b, 0, st, ev0, ev1, 0, p);
    else hipExtLaunchKernelGGL((episode_sq16_kernel<QT, R1, false, 0, NARROW>), g, b, 0, st, ev0, ev1, 0, p);
  }
}
template <typename QT, int R1>
void launch_sq16_r(const EpisodeParams& p, int blocks, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  if (p.rec_narrow) launch_sq16_nw<QT, R1, true>(p, blocks, ev0, ev1, st);
  else launch_sq16_nw<QT, R1, false>(p, blocks, ev0, ev1, st);
}
template <typename QT>
hipError_t launch_sq16_q(const EpisodeParams& p, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  const int waves = (p.S + kWave / 16 - 1) / (kWave / 16);
  const int blocks = (waves + kSq16Waves - 1) / kSq16Waves;
  if (p.R == 0) launch_sq16_r<QT, 1>(p, blocks, ev0, ev1, st);
  else if (p.R == 1) launch_sq16_r<QT, 2>(p, blocks, ev0, ev1, st);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// ----------------------------------------------------------------- RuleAgent communities
// CommunityMicrogrid.run (community.py:95-123) of get_rule_based_community (community.py:237-238):
// every agent is a RuleAgent (agent.py:106-136), so there is no policy and no exchange round.
// Per step: the hysteresis rule on the pre-update T_in (on at T_in <= setpoint - 1, off at
// T_in >= setpoint + 1, else unchanged; agent.py:130-136), net power (load - pv) + hp
// (agent.py:119-128), the market on the (N, 1) stack (TF broadcasts it against its transpose:
// ex_ij = sign(P_i) min(|P_i|, |P_j|) on differing signs, p_grid_i = sum_j (P_i - ex_ij),
// community.py:45-54), costs (community.py:56-65), then HPHeating.step (heating.py:138-143).
// One lane per agent, G lanes per scenario, the group's P through LDS; hp_on persists.
template <int G>
__global__ __launch_bounds__(kWave) void rule_episode_kernel(const EpisodeParams p, float* __restrict__ hp_on) {
  constexpr int SPW = kWave / G;
  __shared__ float shP[kWave];
  const int lane = (int)threadIdx.x;
  const int sl = lane / G, i = lane % G;
  const int N = p.N;
  const int s = (int)blockIdx.x * SPW + sl;
  const bool active = i < N && s < p.S;
  const int a = active ? s * N + i : 0;
  const int s_env = p.n_env == 1 ? 0 : (s < p.S ? s : 0);
  const size_t A = (size_t)p.A;
  const KC k = scalar_constants(p);
  const Recip rmph = recip(k.mph);
  const float hpmax = p.hp_lv[a].z;  // HeatPump.max_power (hp.power in {0, 1})
  float on = active ? hp_on[a] : 0.0f;
  float tin = active ? p.t_in[a] : k.setpoint;
  float tm = active ? p.t_m[a] : k.setpoint;
  const float* envb = p.env + (size_t)s_env * kEnvStride;
  const size_t env_step = (size_t)p.n_env * kEnvStride;
  const uint32_t rec = (uint32_t)p.record;
  for (int t = 0; t < p.T; ++t) {
    const EnvRow e = load_env(envb + (size_t)t * env_step);
    const float2 f = p.prof[(size_t)t * A + a];
    on = tin <= k.lower ? 1.0f : (tin >= k.upper ? 0.0f : on);
    const float hp = on * hpmax;
    const float P = (f.x - f.y) + hp;
    shP[lane] = P;
    wave_lds_fence();
    float g = 0.0f, pp = 0.0f;
    for (int j = 0; j < N; ++j) {
      const float pj = shP[sl * G + j];
      const float ex = pair_exchange(P, pj);
      g = g + (P - ex);
      pp = pp + ex;
    }
    wave_lds_fence();
    float cost = (g >= 0.0f) ? g * e.buy : g * e.inj;
    cost = cost + pp * e.p2p;
    cost = fdiv_b(cost * k.slot, rmph);
    cost = cost * k.kilo;
    if (active) {
      const size_t tA = (size_t)t * A + a;
      if (rec & 2u) p.rec_cost[tA] = cost;
      if (rec & 4u) p.rec_grid[tA] = g;
      if (rec & 8u) p.rec_p2p[tA] = pp;
      if (rec & 16u) p.rec_tin[tA] = tin;
      if (rec & 32u) p.rec_action[tA] = on != 0.0f ? 2 : 0;  // action 2 = 1.0 x max_power
    }
    rc_update(k, e.t_out, hp, tin, tm);
  }
  if (active) {
    p.t_in[a] = tin;
    p.t_m[a] = tm;
    hp_on[a] = on;
  }
}

template <int G>
void launch_rule_g(const EpisodeParams& p, float* hp_on, hipStream_t st) {
  constexpr int SPW = kWave / G;
  hipLaunchKernelGGL(rule_episode_kernel<G>, dim3((p.S + SPW - 1) / SPW), dim3(kWave), 0, st, p, hp_on);
}

template <int NC, bool WIDE, typename QT, bool SQ>
void launch_nq(const EpisodeParams& p, hipStream_t st) {
  constexpr int SPW = kWave / pow2ceil(NC);
  constexpr int WPB = general_wpb<NC, WIDE, SQ>();
  const int waves = (p.S + SPW - 1) / SPW;
  const int blocks = (waves + WPB - 1) / WPB;
  if (p.nt == 20 && p.nT == 20 && p.nb == 20 && p.np == 20)
    hipLaunchKernelGGL((episode_kernel<NC, WIDE, QT, true, SQ>), dim3(blocks), dim3(kWave * WPB), 0, st, p);
  else
    hipLaunchKernelGGL((episode_kernel<NC, WIDE, QT, false, SQ>), dim3(blocks), dim3(kWave * WPB), 0, st, p);
}

template <int NC, bool WIDE, typename QT>
hipError_t launch_n(const EpisodeParams& p, hipStream_t st) {
  if (p.shared_q)
    launch_nq<NC, WIDE, QT, true>(p, st);
  else
    launch_nq<NC, WIDE, QT, false>(p, st);
  return hipGetLastError();
}

// N compiled in (registers): N in {1..8, 16}
template <int N>
hipError_t launch_nd(const EpisodeParams& p, int q_dtype, hipStream_t st) {
  return q_dtype == 0 ? launch_n<N, false, double>(p, st) : launch_n<N, false, float>(p, st);
}
// any N <= NC at run time (LDS tiles)
template <int NC>
hipError_t launch_wide(const EpisodeParams& p, int q_dtype, hipStream_t st) {
  if (p.N < 1 || p.N > NC) return hipErrorInvalidValue;
  return q_dtype == 0 ? launch_n<NC, true, double>(p, st) : launch_n<NC, true, float>(p, st);
}

// ----------------------------------------------------------------- small kernels
#if P2PMG_IN_PART(0)
__global__ void rc_step_kernel(int n, const float* t_out, const float* t_in, const float* t_m, const float* hp,
                               float* t_in_new, float* t_m_new, RcParams rc) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  float a = t_in[k], b = t_m[k];
  rc_update(rc, t_out[k], hp[k], a, b);
  t_in_new[k] = a;
  t_m_new[k] = b;
}
#endif

#if P2PMG_IN_PART(0)
__global__ void state_indices_kernel(int n, const float* obs, int32_t* idx, int nt, int nT, int nb, int np) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float4 o = reinterpret_cast<const float4*>(obs)[k];
  idx[4 * k + 0] = idx_time(o.x, nt);
  idx[4 * k + 1] = idx_temp(o.y, nT);
  idx[4 * k + 2] = idx_plain(o.z, nb);
  idx[4 * k + 3] = idx_plain(o.w, np);
}
#endif

#if P2PMG_IN_PART(0)
__global__ void t0_philox_kernel(int A, float* t_in, float* t_m, uint32_t k0, uint32_t k1, int episode,
                                 uint32_t agent_offset, float setpoint, double sigma) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= A) return;
  t0_draw(k0, k1, episode, agent_offset + (uint32_t)k, setpoint, sigma, t_in[k], t_m[k]);
}
#endif

// reference layout [count][n_states][n_actions] (host dtype) <-> padded device layout
template <typename D, typename S>
__global__ void q_pack_kernel(size_t rows, int na, const S* src, D* dst) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= rows) return;
#pragma unroll
  for (int c = 0; c < kQPad; ++c) dst[k * kQPad + c] = c < na ? (D)src[k * na + c] : (D)0;
}
template <typename D, typename S>
__global__ void q_unpack_kernel(size_t rows, int na, const S* src, D* dst) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= rows) return;
  for (int c = 0; c < na; ++c) dst[k * na + c] = (D)src[k * kQPad + c];
}

// [A][T] load / pv (the host's per-agent rows) -> [T][A] float2 (time-major, one coalesced 8-B load
// per lane per step): a 32 x 32 tile transposed through LDS, so the reads are 128-B runs of one
// agent's steps and the writes 256-B runs of one step's agents (round 5; the per-element form read
// with stride T, 32x the input in fetched sectors).  Block (32, 8), tile [agent][step] padded to 33.
#if P2PMG_IN_PART(0)
__global__ __launch_bounds__(256) void prof_pack_kernel(int A, int T, const float* __restrict__ load_w,
                                                        const float* __restrict__ pv_w, float2* __restrict__ prof) {
  __shared__ float tl[32][33], tv[32][33];
  const int tx = (int)threadIdx.x, ty = (int)threadIdx.y;
  const int a0 = (int)blockIdx.x * 32, t0 = (int)blockIdx.y * 32;  // grid.x: agents (grid.y <= 65535)
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int a = a0 + ty + k, t = t0 + tx;
    if (a < A && t < T) {
      const size_t src = (size_t)a * T + t;
      tl[ty + k][tx] = load_w[src];
      tv[ty + k][tx] = pv_w[src];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int t = t0 + ty + k, a = a0 + tx;
    if (a < A && t < T) prof[(size_t)t * A + a] = make_float2(tl[tx][ty + k], tv[tx][ty + k]);
  }
}
#endif

// sq16_prep_kernel: the policy-independent part of episode_sq16_kernel's per-step state, once per
// input upload (the runtime reruns it when env, profiles or max_in change): per (t, a) the agent's
// balance (load - pv) / max_in (agent.py:172-176, the IEEE quotient the kernel's guarded fast
// division returns) and the table offset of its time and balance bins, it * 8000 + ib * 20
// (rl.py:89-95 on the 20^4 table the sq16 path serves; the temperature bin is added in the kernel).
// The episode kernel then reads one 8-B word per agent-step instead of {load, pv} and skips the
// division and three of the four bins of every step.
#if P2PMG_IN_PART(5)
__global__ void sq16_prep_kernel(const EpisodeParams p, uint2* __restrict__ out) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // k = t * A + a
  if (k >= (size_t)p.A * p.T) return;
  const int t = (int)(k / (size_t)p.A), a = (int)(k % (size_t)p.A);
  const int s_env = p.n_env == 1 ? 0 : a / p.N;
  const float time = p.env[((size_t)t * p.n_env + s_env) * kEnvStride];
  const float2 f = p.prof[k];
  const float bal = fdiv_ieee(f.x - f.y, p.max_in[a]);
  const int it = clamp_bin_f(time * 20.0f, 19.0f);
  const int ib = clamp_bin_f(((bal + 1.0f) / 2.0f) * 20.0f, 19.0f);
  out[k] = make_uint2(__float_as_uint(bal), (uint32_t)(it * 8000 + ib * 20));
}
#endif

// The fast quotients of the episode kernels next to the IEEE operator, for the division fuzz test
// (tests/test_gpu_division.py): exactly the guarded sequences the kernels run.
//   f32 out[0] fdiv_b (hoisted reciprocal of a divisor checked on the host, IEEE when the numerator
//              is out of range)            - max_in, 60, N, the comfort margin
//       out[1] the divide-power form: recip of a data-dependent divisor, fdiv_core, IEEE when the
//              divisor or the numerator is out of range
//       out[2] the packed sq16 form (fdiv_core_pk) under its range-19 guard, else out[1]'s form
//       out[3] IEEE a / b
//   f64 out[0] fdiv64 (hoisted Recip64 + range test), out[1] qcore64 under q64_ok (battery_rule_r's
//       guard), out[2] IEEE n / d
#if P2PMG_IN_PART(0)
__global__ void fdiv_check_kernel(int n, const float* __restrict__ a, const float* __restrict__ b,
                                  float* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float x = a[k], d = b[k];
  const Recip r = recip(d);
  out[4 * (size_t)k + 0] = r.ok ? fdiv_b(x, r) : fdiv_ieee(x, d);
  float q1 = fdiv_core(x, r);
  if (!r.ok || !fdiv_ok(x)) q1 = fdiv_ieee(x, d);
  out[4 * (size_t)k + 1] = q1;
  float q2 = q1;
  if (r.ok && in_range19(x) && in_range19(d) && d > 0.0f) {  // the kernel's divisor is tot = |sum| > 0
    const pkf2 y2 = {r.y, r.y}, b2 = {d, d};
    q2 = fdiv_core_pk(pkf2{x, x}, b2, y2).x;
  }
  out[4 * (size_t)k + 2] = q2;
  out[4 * (size_t)k + 3] = fdiv_ieee(x, d);
}
__global__ void fdiv64_check_kernel(int n, const double* __restrict__ a, const double* __restrict__ b,
                                    double* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double x = a[k], d = b[k];
  const Recip64 r = recip64(d);
  out[3 * (size_t)k + 0] = fdiv64(x, r);
  double q1 = qcore64(x, r);
  if (!(r.ok && q64_ok(x))) q1 = fdiv64_ieee(x, d);
  out[3 * (size_t)k + 1] = q1;
  out[3 * (size_t)k + 2] = fdiv64_ieee(x, d);
}
#endif

// Episode metrics of the context (community.py:179 avg_reward per scenario): out = {sum_s ep_reward[s],
// S} in f64, one workgroup, a fixed reduction tree (deterministic), ready for the RCCL all-reduce.
#if P2PMG_IN_PART(0)
__global__ __launch_bounds__(256) void metrics_kernel(int S, const float* __restrict__ ep, double* __restrict__ out) {
  __shared__ double sh[256];
  double acc = 0.0;
  for (int s = threadIdx.x; s < S; s += 256) acc += (double)ep[s];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = sh[0];
    out[1] = (double)S;
  }
}
// Order-independent 64-bit fingerprint of a table's bit pattern (sum over words of a splitmix of
// (word, index)): equal on every rank iff the replicas hold the same bits (up to hash collisions)
__global__ void table_hash_kernel(const uint32_t* __restrict__ w, size_t n, unsigned long long* __restrict__ out) {
  unsigned long long acc = 0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
    unsigned long long x = ((unsigned long long)w[k] << 32) ^ (k * 0x9E3779B97F4A7C15ull);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    acc += x ^ (x >> 31);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}
#endif

// Standalone QActor calls, applied in order by a single thread (rl.py:89-129).
template <typename QT>
__global__ void q_calls_kernel(const QCallParams p) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (int k = 0; k < p.n; ++k) {
    QT* q = reinterpret_cast<QT*>(p.q) + (size_t)p.agents[k] * p.n_states * kQPad;
    const float* o = p.s_obs + 4 * k;
    const uint32_t srow = (uint32_t)(((idx_time(o[0], p.nt) * p.nT + idx_temp(o[1], p.nT)) * p.nb +
                                      idx_plain(o[2], p.nb)) * p.np + idx_plain(o[3], p.np));
    const Row4<QT> row = load_row(q + srow * kQPad);
    const int code = p.codes[k];
    const int a = code == 255 ? argmax3(row) : code;
    p.actions[k] = a;
    p.q_out[k] = code == 255 ? (double)row.v[a] : 0.0;
    if (p.train) {
      const float* n = p.ns_obs + 4 * k;
      const uint32_t nrow = (uint32_t)(((idx_time(n[0], p.nt) * p.nT + idx_temp(n[1], p.nT)) * p.nb +
                                        idx_plain(n[2], p.nb)) * p.np + idx_plain(n[3], p.np));
      const QT qmax = max3(load_row(q + nrow * kQPad));
      q[srow * kQPad + a] = td_update(q[srow * kQPad + a], p.rewards[k], qmax, p.alpha, p.gamma);
    }
  }
}

inline unsigned grid_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

#if P2PMG_IN_PART(0)
hipError_t launch_philox_codes(const EpisodeParams& p, uint32_t* words, hipStream_t stream) {
  const size_t n = (size_t)p.T * p.A;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(philox_codes_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, p, words);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_pack_codes(int T, int R1, int A, const uint8_t* in, uint32_t* words, hipStream_t stream) {
  const size_t n = (size_t)T * A;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(pack_codes_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, T, R1, A, in, words);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_fold_delta(long long* qdelta, size_t n, hipStream_t stream) {
  hipLaunchKernelGGL(fold_delta_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, qdelta, n);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_apply_delta(void* q, long long* qdelta, size_t n, int q_dtype, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (q_dtype == 0)
    hipLaunchKernelGGL(apply_delta_kernel<double>, dim3(grid_for(n, 256)), dim3(256), 0, stream, (double*)q, qdelta, n);
  else
    hipLaunchKernelGGL(apply_delta_kernel<float>, dim3(grid_for(n, 256)), dim3(256), 0, stream, (float*)q, qdelta, n);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_battery_seq(int agents, int steps, const double* bal, double* out_bal, double* soc_hist, double* soc,
                              const double* cap, double smin, double smax, double sqrt_eff, hipStream_t stream) {
  if (agents <= 0) return hipSuccess;
  hipLaunchKernelGGL(battery_seq_kernel, dim3(grid_for(agents, 64)), dim3(64), 0, stream, agents, steps, bal, out_bal,
                     soc_hist, soc, cap, smin, smax, sqrt_eff);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_step_prepass(const EpisodeParams& p, const PrepOut& o, hipStream_t stream) {
  const size_t n = (size_t)p.T * p.A;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(step_prepass_kernel, dim3(grid_for(n, 256), o.n_ep > 1 ? o.n_ep : 1), dim3(256), 0, stream, p, o);
  return hipGetLastError();
}
#endif

#define P2PMG_FAST_PART(k, N0)                                                                                   \
  hipError_t launch_fast_part##k(const EpisodeParams& p, const uint2* pre, void* recs, int q_dtype, int spw,       \
                                 const PrepOut* next, hipEvent_t ev0, hipEvent_t ev1, hipStream_t stream) {       \
    return launch_fast_pair<N0>(p, pre, recs, q_dtype, spw, next, ev0, ev1, stream);                              \
  }
#if P2PMG_IN_PART(1)
P2PMG_FAST_PART(1, 1)
#endif
#if P2PMG_IN_PART(2)
P2PMG_FAST_PART(2, 3)
#endif
#if P2PMG_IN_PART(3)
P2PMG_FAST_PART(3, 5)
#endif
#if P2PMG_IN_PART(4)
P2PMG_FAST_PART(4, 7)
#endif
#if P2PMG_IN_PART(0)
hipError_t launch_episode_fast(const EpisodeParams& p, const uint2* pre, void* recs, int q_dtype, int spw,
                               const PrepOut* next, hipEvent_t ev0, hipEvent_t ev1, hipStream_t stream) {
  const int part = p.N <= 2 ? 1 : p.N <= 4 ? 2 : p.N <= 6 ? 3 : 4;
  auto f = part == 1 ? launch_fast_part1 : part == 2 ? launch_fast_part2 : part == 3 ? launch_fast_part3 : launch_fast_part4;
  if (p.N < 1 || p.N > 8) return hipErrorInvalidValue;
  return f(p, pre, recs, q_dtype, spw, next, ev0, ev1, stream);
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_fast_rec_unpack(int T, int R1, int A, uint32_t tb, const void* recs, int narrow, int which, void* out,
                                  hipStream_t stream) {
  const size_t n = (size_t)T * A;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fast_rec_unpack_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, T, R1, A, tb,
                     reinterpret_cast<const FastRec*>(recs), narrow, which, out);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(5)
hipError_t launch_episode_sq16(const EpisodeParams& p, int q_dtype, hipEvent_t ev0, hipEvent_t ev1, hipStream_t stream) {
  return q_dtype == 0 ? launch_sq16_q<double>(p, ev0, ev1, stream) : launch_sq16_q<float>(p, ev0, ev1, stream);
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_rule_episode(const EpisodeParams& p, float* hp_on, hipStream_t stream) {
  const int n = p.N;
  if (n <= 1) launch_rule_g<1>(p, hp_on, stream);
  else if (n <= 2) launch_rule_g<2>(p, hp_on, stream);
  else if (n <= 4) launch_rule_g<4>(p, hp_on, stream);
  else if (n <= 8) launch_rule_g<8>(p, hp_on, stream);
  else if (n <= 16) launch_rule_g<16>(p, hp_on, stream);
  else if (n <= 32) launch_rule_g<32>(p, hp_on, stream);
  else if (n <= 64) launch_rule_g<64>(p, hp_on, stream);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(6)
hipError_t launch_general_part6(const EpisodeParams& p, int q_dtype, hipStream_t stream) {
  switch (p.N) {
    case 1: return launch_nd<1>(p, q_dtype, stream);
    case 2: return launch_nd<2>(p, q_dtype, stream);
    case 3: return launch_nd<3>(p, q_dtype, stream);
    case 4: return launch_nd<4>(p, q_dtype, stream);
    default: return hipErrorInvalidValue;
  }
}
#endif
#if P2PMG_IN_PART(7)
hipError_t launch_general_part7(const EpisodeParams& p, int q_dtype, hipStream_t stream) {
  switch (p.N) {
    case 5: return launch_nd<5>(p, q_dtype, stream);
    case 6: return launch_nd<6>(p, q_dtype, stream);
    case 7: return launch_nd<7>(p, q_dtype, stream);
    case 8: return launch_nd<8>(p, q_dtype, stream);
    default: return hipErrorInvalidValue;
  }
}
#endif
#if P2PMG_IN_PART(8)
hipError_t launch_general_part8(const EpisodeParams& p, int q_dtype, hipStream_t stream) {
  return p.N == 16 ? launch_nd<16>(p, q_dtype, stream) : hipErrorInvalidValue;
}
#endif
#if P2PMG_IN_PART(9)
hipError_t launch_tile_part9(const EpisodeParams& p, int q_dtype, int nc, hipStream_t stream) {
  return nc == 16 ? launch_wide<16>(p, q_dtype, stream) : hipErrorInvalidValue;
}
#endif
#if P2PMG_IN_PART(10)
hipError_t launch_tile_part10(const EpisodeParams& p, int q_dtype, int nc, hipStream_t stream) {
  return nc == 32 ? launch_wide<32>(p, q_dtype, stream) : nc == 64 ? launch_wide<64>(p, q_dtype, stream)
                                                                   : hipErrorInvalidValue;
}
#endif
#if P2PMG_IN_PART(0)
// the general kernel: registers for N in {1..8, 16}, LDS tiles for every other N <= 64 (and for any
// N <= 64 when tile != 0, the cross-check of the two forms)
hipError_t launch_episode(const EpisodeParams& p, int q_dtype, int tile, hipStream_t stream) {
  if (p.N < 1 || p.N > kMaxAgents) return hipErrorInvalidValue;
  if (!tile) {
    if (p.N <= 4) return launch_general_part6(p, q_dtype, stream);
    if (p.N <= 8) return launch_general_part7(p, q_dtype, stream);
    if (p.N == 16) return launch_general_part8(p, q_dtype, stream);
  }
  const int nc = general_tile_cap(p.N);
  return nc == 16 ? launch_tile_part9(p, q_dtype, nc, stream) : launch_tile_part10(p, q_dtype, nc, stream);
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_rc_step(int n, const float* t_out, const float* t_in, const float* t_m, const float* hp,
                          float* t_in_new, float* t_m_new, RcParams rc, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(rc_step_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, t_out, t_in, t_m, hp, t_in_new,
                     t_m_new, rc);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_state_indices(int n, const float* obs, int32_t* idx, int nt, int nT, int nb, int np,
                                hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(state_indices_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, obs, idx, nt, nT, nb, np);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_t0_philox(int A, float* t_in, float* t_m, uint32_t seed_lo, uint32_t seed_hi, int episode,
                            uint32_t agent_offset, float setpoint, double sigma, hipStream_t stream) {
  if (A <= 0) return hipSuccess;
  hipLaunchKernelGGL(t0_philox_kernel, dim3(grid_for(A, 256)), dim3(256), 0, stream, A, t_in, t_m, seed_lo, seed_hi,
                     episode, agent_offset, setpoint, sigma);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_q_pack(int count, size_t n_states, int n_actions, const void* src_ref, void* dst_pad, int q_dtype,
                         int src_dtype, hipStream_t stream) {
  const size_t rows = (size_t)count * n_states;
  if (rows == 0) return hipSuccess;
  const dim3 g(grid_for(rows, 256)), b(256);
  if (q_dtype == 0 && src_dtype == 0)
    hipLaunchKernelGGL((q_pack_kernel<double, double>), g, b, 0, stream, rows, n_actions, (const double*)src_ref, (double*)dst_pad);
  else if (q_dtype == 0)
    hipLaunchKernelGGL((q_pack_kernel<double, float>), g, b, 0, stream, rows, n_actions, (const float*)src_ref, (double*)dst_pad);
  else if (src_dtype == 0)
    hipLaunchKernelGGL((q_pack_kernel<float, double>), g, b, 0, stream, rows, n_actions, (const double*)src_ref, (float*)dst_pad);
  else
    hipLaunchKernelGGL((q_pack_kernel<float, float>), g, b, 0, stream, rows, n_actions, (const float*)src_ref, (float*)dst_pad);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_q_unpack(int count, size_t n_states, int n_actions, const void* src_pad, void* dst_ref, int q_dtype,
                           int dst_dtype, hipStream_t stream) {
  const size_t rows = (size_t)count * n_states;
  if (rows == 0) return hipSuccess;
  const dim3 g(grid_for(rows, 256)), b(256);
  if (q_dtype == 0 && dst_dtype == 0)
    hipLaunchKernelGGL((q_unpack_kernel<double, double>), g, b, 0, stream, rows, n_actions, (const double*)src_pad, (double*)dst_ref);
  else if (q_dtype == 0)
    hipLaunchKernelGGL((q_unpack_kernel<float, double>), g, b, 0, stream, rows, n_actions, (const double*)src_pad, (float*)dst_ref);
  else if (dst_dtype == 0)
    hipLaunchKernelGGL((q_unpack_kernel<double, float>), g, b, 0, stream, rows, n_actions, (const float*)src_pad, (double*)dst_ref);
  else
    hipLaunchKernelGGL((q_unpack_kernel<float, float>), g, b, 0, stream, rows, n_actions, (const float*)src_pad, (float*)dst_ref);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_q_calls(const QCallParams& p, hipStream_t stream) {
  if (p.n <= 0) return hipSuccess;
  if (p.q_dtype == 0)
    hipLaunchKernelGGL(q_calls_kernel<double>, dim3(1), dim3(64), 0, stream, p);
  else
    hipLaunchKernelGGL(q_calls_kernel<float>, dim3(1), dim3(64), 0, stream, p);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_metrics(int S, const float* ep, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(metrics_kernel, dim3(1), dim3(256), 0, stream, S, ep, out);
  return hipGetLastError();
}
hipError_t launch_table_hash(const void* q, size_t bytes, unsigned long long* out, hipStream_t stream) {
  hipError_t e = hipMemsetAsync(out, 0, 8, stream);
  if (e != hipSuccess) return e;
  const size_t n = bytes / 4;
  hipLaunchKernelGGL(table_hash_kernel, dim3((unsigned)std::min<size_t>(2048, grid_for(n, 256))), dim3(256), 0, stream,
                     reinterpret_cast<const uint32_t*>(q), n, out);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_fdiv_check(int n, const float* a, const float* b, float* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fdiv_check_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, a, b, out);
  return hipGetLastError();
}
hipError_t launch_fdiv64_check(int n, const double* a, const double* b, double* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fdiv64_check_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, a, b, out);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(0)
hipError_t launch_prof_pack(int A, int T, const float* load_w, const float* pv_w, float2* prof, hipStream_t stream) {
  if ((size_t)A * T == 0) return hipSuccess;
  if ((T + 31) / 32 > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(prof_pack_kernel, dim3((A + 31) / 32, (T + 31) / 32), dim3(32, 8), 0, stream, A, T, load_w, pv_w,
                     prof);
  return hipGetLastError();
}
#endif

#if P2PMG_IN_PART(5)
hipError_t launch_sq16_prep(const EpisodeParams& p, uint2* out, hipStream_t stream) {
  const size_t n = (size_t)p.A * p.T;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(sq16_prep_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, p, out);
  return hipGetLastError();
}
#endif

}  // namespace p2pmg
