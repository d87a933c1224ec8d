// p2pmg_dqn.hip — gfx950 kernels of the DQN variant (BASELINE.json configs[4]):
//   QNetwork rl.py:135-148, ActorModel rl.py:151-197, ReplayBuffer rl.py:200-248,
//   Trainer._train / _soft_update rl.py:307-359, DQNAgent agent.py:301-350.
//
// One environment step = two launches (plus, for one shared network, one reduce + Adam launch):
//   dqn_act_kernel<N>    one workgroup per scenario, ONE WAVE PER AGENT; lane j is hidden unit j
//                        of the agent's Q-MLP (weights streamed as coalesced 256-B rows), the
//                        R+1 Jacobi rounds exchange the proposal matrix through LDS, then market,
//                        reward, replay-memory append and the RC update (community.py:67-93,
//                        149-182; agent.py:200-213, 225-232; heating.py:37-56).
//   dqn_train_kernel     one 4-wave workgroup per agent (or per run of agents when the network
//                        is shared): samples 32 transitions, target forward over the 96 rows
//                        (ns x 3 action values), online forward + backward over the 32 rows, all
//                        on v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation); wave w
//                        owns hidden units 16w..16w+15 of both 64-wide layers (layer 2 as the
//                        transposed product, so layer 3 reduces in-lane).  Per-agent
//                        networks: clip + Adam + soft update fused in the epilogue; shared: the
//                        workgroup's gradient sum is written as a partial.
// Layouts (HBM): networks [n_nets][4672] f32 (Keras order W1[5][64] b1 W2[64][64] b2 W3[64] b3),
// replay rings [A][cap][10] f32 (s[4], a, r, ns[4]), added [A].
#include "p2pmg_internal.h"

namespace p2pmg {
namespace {
#include "p2pmg_device.h"

constexpr int kH = 64;
constexpr int kB = kDqnBatch;
constexpr int kLdsRow = 68;  // padded activation rows: an MFMA A-operand read (16 rows x 4 k) hits 64 banks
constexpr int kLdsRowT = 48;  // H1oT rows (32 data rows + pad): 16 units x 4 k of one read hit 64 banks

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float relu(float x) { return x > 0.0f ? x : 0.0f; }

// Cross-lane sums as VALU lane moves (DPP and gfx950's v_permlane16/32_swap) instead of
// ds_bpermute round trips through the LDS unit.  x + swap(x) adds the same two operands in both
// lanes of every exchanged pair, so each sum below ends bitwise-identical in all its lanes.
template <int CTRL>
__device__ __forceinline__ float plus_dpp(float v) {  // v + v[lane per the DPP pattern]
  return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float plus_swap16(float v) {  // rows 0 <-> 1, 2 <-> 3 (lane ^ 16)
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float plus_swap32(float v) {  // halves 0 <-> 1 (lane ^ 32)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// over the 16 lanes of a row group: lane ^ 1, lane ^ 2 (quad_perm), the other quad of each 8
// (row_half_mirror), the other 8 of each 16 (row_mirror)
__device__ __forceinline__ float sum16(float v) {
  v = plus_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v = plus_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v = plus_dpp<0x141>(v);  // row_half_mirror
  v = plus_dpp<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ float sum_groups(float v) {  // over the 4 row groups (same lane & 15)
  return plus_swap32(plus_swap16(v));
}
__device__ __forceinline__ float wave_sum(float v) { return sum_groups(sum16(v)); }
// sum over the 4 row groups of four values at once: the first swaps pair row groups (g4, g4 ^ 1)
// of (a, b) and of (c, d), the second (g4, g4 ^ 2) of the two pair sums, so each row group ends
// holding ONE tile's total ((g0 + g1) + (g2 + g3), sum_groups' tree); reduce4_tag() says which
// (the same swaps applied to the tile numbers)
__device__ __forceinline__ float reduce4_groups(float a, float b, float c, float d) {
  const auto r1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  const auto r2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(c), __float_as_uint(d), false, false);
  const float ab = __uint_as_float(r1[0]) + __uint_as_float(r1[1]);
  const float cd = __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
  const auto r3 = __builtin_amdgcn_permlane32_swap(__float_as_uint(ab), __float_as_uint(cd), false, false);
  return __uint_as_float(r3[0]) + __uint_as_float(r3[1]);
}
__device__ __forceinline__ int reduce4_tag() {
  const auto r1 = __builtin_amdgcn_permlane16_swap(0u, 1u, false, false);
  const auto r2 = __builtin_amdgcn_permlane16_swap(2u, 3u, false, false);
  const auto r3 = __builtin_amdgcn_permlane32_swap(r1[0], r2[0], false, false);
  return (int)r3[0];
}

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ReplayBuffer.sample_batch rl.py:226-241 for every agent of the step, ahead of the train kernel:
// one wave per agent draws 32 distinct deque indices (replayed, or Philox + Floyd as in
// oracle/philox.py::sample_draws) and writes their ring slots to d.smp (as int32 [A][32]); the
// train kernel gathers each agent's 32 transitions from the ring one agent ahead (double-buffered),
// so neither kernel waits on the random ring reads behind the serial 32-step selection loop.
// One wave draws agent a's 32 slots; n_added = the agent's transitions including this step's.
__device__ __forceinline__ void sample_slots(const DqnParams& d, int a, int l, int n_added) {
  const EpisodeParams& p = d.e;
  const size_t A = (size_t)p.A;
  const int count = n_added < d.cap ? n_added : d.cap;
  const int first = n_added - count;
  int idx = 0;
  if (d.samples) {
    idx = l < kB ? (int)d.samples[((size_t)d.t * A + a) * kB + l] : 0;
  } else {
    uint32_t c0 = (uint32_t)d.t, c1 = (uint32_t)p.episode, c2 = p.agent_offset + (uint32_t)a,
             c3 = kTagSample + (uint32_t)(l & 31);
    philox4x32_10(c0, c1, c2, c3, p.seed_lo, p.seed_hi);
    const int mj = count - kB + (l & 31);
    const int rj = (int)__umulhi(c0, (uint32_t)(mj + 1));
    idx = rj;
    for (int j = 0; j < kB; ++j) {
      const int r = __builtin_amdgcn_readlane(rj, j);  // lane j's draw (j is uniform: an SGPR read, no LDS trip)
      const bool taken = __ballot(l < j && idx == r) != 0;
      if (l == j) idx = taken ? count - kB + j : r;
    }
  }
  if (l < kB) reinterpret_cast<int*>(d.smp)[(size_t)a * kB + l] = (first + idx) % d.cap;
}
__global__ __launch_bounds__(kWave) void dqn_sample_kernel(const DqnParams d) {
  sample_slots(d, blockIdx.x, threadIdx.x, d.added[blockIdx.x]);
}

// ReplayBuffer.sample_batch (rl.py:226-241) of every env step of a Philox training episode in ONE
// throughput launch ahead of it: thread = (step t, agent a), the 32 draws of
// oracle/philox.py::sample_draws with Floyd's rule walked in order (draw q takes count - 32 + q when
// r_q equals an earlier draw's final index), written as deque indices [T][A][32] u16 -- the layout
// replay mode uploads (p2pmg_dqn_set_samples), which the act kernels read instead of drawing in
// their latency-bound tail.  Every training env step appends one transition per agent before it
// samples (agent.py:338-342), so step t's count follows from the episode-start count.
__global__ __launch_bounds__(256) void dqn_sample_prepass_kernel(const DqnParams d, uint16_t* __restrict__ out) {
  const EpisodeParams& p = d.e;
  const size_t A = (size_t)p.A;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (size_t)p.T * A) return;
  const int t = (int)(k / A), a = (int)(k % A);
  const int n_add = d.added[a] + t + 1;
  const int count = n_add < d.cap ? n_add : d.cap;
  int idx[kB];
#pragma unroll
  for (int q = 0; q < kB; ++q) {
    uint32_t c0 = (uint32_t)t, c1 = (uint32_t)p.episode, c2 = p.agent_offset + (uint32_t)a, c3 = kTagSample + (uint32_t)q;
    philox4x32_10(c0, c1, c2, c3, p.seed_lo, p.seed_hi);
    const int r = (int)__umulhi(c0, (uint32_t)(count - kB + q + 1));
    bool taken = false;
#pragma unroll
    for (int l = 0; l < q; ++l) taken = taken || idx[l] == r;
    idx[q] = taken ? count - kB + q : r;
  }
  uint4* o = reinterpret_cast<uint4*>(out + k * kB);
#pragma unroll
  for (int v = 0; v < kB / 8; ++v) {
    const int* x = idx + 8 * v;
    o[v] = make_uint4((uint32_t)x[0] | ((uint32_t)x[1] << 16), (uint32_t)x[2] | ((uint32_t)x[3] << 16),
                      (uint32_t)x[4] | ((uint32_t)x[5] << 16), (uint32_t)x[6] | ((uint32_t)x[7] << 16));
  }
}

// ----------------------------------------------------------------- act: one env step
// dqn_act_kernel<NC, WIDE>: one workgroup per scenario.  WIDE = false: NC = N agents compiled in
// (N <= 16), one wave per agent.  WIDE = true: any n = p.N <= NC (the community sizes 9..15 and
// 17..64), NW = 16 waves, wave w acting for agents w, w + 16, ... in turn in each round
// (a round is Jacobi: every agent reads the previous round's P, community.py:84-86, so the order of
// the agents within a round does not matter).  Both forms sum over j = 0..n-1 in order and divide
// by n as IEEE quotients: the same bits.
template <int NC, bool WIDE>
constexpr int dqn_act_waves() {
  return WIDE ? 16 : NC;
}
template <int NC, bool WIDE>
__global__ __launch_bounds__((dqn_act_waves<NC, WIDE>() * kWave)) void dqn_act_kernel(const DqnParams d) {
  constexpr int NW = dqn_act_waves<NC, WIDE>();  // waves
  constexpr int APW = (NC + NW - 1) / NW;    // agents per wave
  const EpisodeParams& p = d.e;
  __shared__ float shP[2][NC * NC];
  __shared__ float4 shH[NW][kH];
  __shared__ float shR[NC];
  const int n = WIDE ? p.N : NC;
  const float nf = (float)n;
  auto divn = [&](float x) -> float {
    if constexpr (WIDE) return x / nf;
    else return div_n<NC>(x);
  };
  const int s = blockIdx.x;
  const int w = threadIdx.x / kWave;
  const int lane = threadIdx.x % kWave;
  const int t = d.t, T = p.T, tn = (t + 1 == T) ? 0 : t + 1;
  const int R1 = p.R + 1, W = (R1 + 3) >> 2;
  const size_t A = (size_t)p.A;
  const int s_env = p.n_env == 1 ? 0 : s;
  const float* e0 = p.env + ((size_t)t * p.n_env + s_env) * kEnvStride;
  const float* e1 = p.env + ((size_t)tn * p.n_env + s_env) * kEnvStride;
  const float time_t = e0[0], t_out = e0[1], buy = e0[2], inj = e0[3], p2pp = e0[4];
  const float time_n = e1[0];
  const bool greedy_mode = p.mode == 1;
  // the wave's agents: wave-uniform scalars (registers for one agent per wave, LDS for several) and
  // this lane's hidden unit of the agent's network (rl.py:139-141): first-layer column, biases,
  // output weight (registers for one agent per wave, read where used for several: L2 hits)
  struct Ag {
    int a;
    float mi, tin, tm, bal, baln, tnorm;
    float4 lv;
    int act;
    float hp, p2pf;
  };
  struct Unit {
    float w10, w11, w12, w13, w14, b1, b2, w3, b3;
    const float* w2col;
  };
  auto load_unit = [&](int a) -> Unit {
    const float* th = d.theta + (size_t)(d.n_nets == 1 ? 0 : a) * kNetStride;
    return Unit{th[kOffW1 + 0 * kH + lane], th[kOffW1 + 1 * kH + lane], th[kOffW1 + 2 * kH + lane],
                th[kOffW1 + 3 * kH + lane], th[kOffW1 + 4 * kH + lane], th[kOffB1 + lane],
                th[kOffB2 + lane],          th[kOffW3 + lane],          th[kOffB3],
                th + kOffW2 + lane};
  };
  __shared__ Ag sAg[WIDE ? NC : 1];
  Ag rAg;
  auto agent = [&](int i) -> Ag& {
    if constexpr (WIDE) return sAg[i];
    else return rAg;
  };
  Unit ru{};
  for (int k = 0; k < APW; ++k) {
    const int i = w + k * NW;
    if (i >= n) break;  // wave-uniform
    Ag& g = agent(i);
    g.a = s * n + i;
    const float2 f0 = p.prof[(size_t)t * A + g.a], f1 = p.prof[(size_t)tn * A + g.a];
    g.mi = p.max_in[g.a];
    g.tin = p.t_in[g.a];
    g.tm = p.t_m[g.a];
    g.bal = (f0.x - f0.y) / g.mi;  // RLAgent._get_balance agent.py:172-176
    g.baln = (f1.x - f1.y) / g.mi;
    g.tnorm = (g.tin - p.setpoint) / p.margin;  // HPHeating.normalized_temperature heating.py:118-120
    g.lv = p.hp_lv[g.a];
    g.act = 0;
    g.hp = 0.0f;
    g.p2pf = 0.0f;
    if constexpr (!WIDE) ru = load_unit(g.a);
  }

  for (int k2 = threadIdx.x; k2 < NC * NC; k2 += NW * kWave) shP[0][k2] = 0.0f;  // round 0 reads P = 0
  __syncthreads();
  int cur = 0;
  for (int r = 0; r < R1; ++r) {
    const float* P = shP[cur];
    for (int k = 0; k < APW; ++k) {
      const int i = w + k * NW;
      if (i >= n) break;  // wave-uniform
      Ag& g = agent(i);
      const int a = g.a;
      // powers = -P[:, i], diagonal zeroed (community.py:76,81); p2p = mean / max_in (agent.py:203)
      float acc = 0.0f;
#pragma unroll
      for (int j = 0; j < n; ++j) acc = acc + (-((j == i) ? 0.0f : P[j * n + i]));
      g.p2pf = divn(acc) / g.mi;
      int code = 255;  // ActorModel.select_action rl.py:174-183: explore draw, else greedy
      if (!greedy_mode) {
        if (p.rng == 0) {
          code = (int)((p.codes[((size_t)t * W + (r >> 2)) * A + a] >> (8 * (r & 3))) & 0xFFu);
        } else {
          // word k = t (R + 1) + r of the agent's decision stream (p2pmg_device.h, oracle/philox.py::decision_draws)
          code = (int)philox_round_code(t, R1, r, (uint32_t)p.episode, p.agent_offset + (uint32_t)a, p.eps_thr,
                                        p.eps_all, p.seed_lo, p.seed_hi);
        }
      }
      if (code == 255) {
        // ActorModel.greedy_action rl.py:188-196: Q(obs, a) for a in (0, .5, 1), argmax (first max)
        const Unit u = WIDE ? load_unit(a) : ru;
        float z = g.p2pf * u.w13;
        z = fmaf(g.bal, u.w12, z);
        z = fmaf(g.tnorm, u.w11, z);
        z = fmaf(time_t, u.w10, z);
        const float h0 = relu(z + u.b1), h1 = relu(fmaf(0.5f, u.w14, z) + u.b1), h2 = relu((z + u.w14) + u.b1);
        shH[w][lane] = make_float4(h0, h1, h2, 0.0f);
        wave_lds_fence();
        float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
#pragma unroll 8
        for (int kk = 0; kk < kH; ++kk) {
          const float wk = u.w2col[kk * kH];
          const float4 hk = shH[w][kk];
          a0 = fmaf(hk.x, wk, a0);
          a1 = fmaf(hk.y, wk, a1);
          a2 = fmaf(hk.z, wk, a2);
        }
        wave_lds_fence();
        const float q0 = wave_sum(relu(a0 + u.b2) * u.w3) + u.b3;
        const float q1 = wave_sum(relu(a1 + u.b2) * u.w3) + u.b3;
        const float q2 = wave_sum(relu(a2 + u.b2) * u.w3) + u.b3;
        g.act = 0;
        float best = q0;
        if (q1 > best) { best = q1; g.act = 1; }
        if (q2 > best) g.act = 2;
      } else {
        g.act = code;
      }
      g.hp = g.act == 0 ? g.lv.x : (g.act == 1 ? g.lv.y : g.lv.z);  // heating.set_power(action) -> hp.power * max_power
      // RLAgent._divide_power agent.py:186-195 on out = balance * max_in + hp (agent.py:210)
      const float out = (g.bal * g.mi) + g.hp;
      const float so = sgn(out);
      float tot = 0.0f, fj = 0.0f;
#pragma unroll
      for (int j = 0; j < n; ++j) {
        const float pw = -((j == i || r == 0) ? 0.0f : P[j * n + i]);
        const float f = (so != sgn(pw)) ? pw : 0.0f;
        tot = tot + f;
        if (j == lane) fj = f;
      }
      tot = fabsf(tot);
      if (lane < n) {
        float v;
        if (tot == 0.0f) v = divn(out * 1.0f);
        else v = (lane == i) ? (tot == tot ? out * 0.0f : tot) : (out * fabsf(fj)) / tot;
        shP[cur ^ 1][i * n + lane] = v;
      }
      if (lane == 0 && (p.record & 32)) p.rec_action[((size_t)t * R1 + r) * A + a] = (uint8_t)g.act;
    }
    __syncthreads();
    cur ^= 1;
  }
  const float* P = shP[cur];
  for (int k = 0; k < APW; ++k) {
    const int i = w + k * NW;
    if (i >= n) break;  // wave-uniform
    Ag& g = agent(i);
    const int a = g.a;
    // CommunityMicrogrid._assign_powers community.py:45-54 (final P, diagonal kept)
    float gg = 0.0f, pp = 0.0f;
#pragma unroll
    for (int j = 0; j < n; ++j) {
      const float pij = P[i * n + j], pji = P[j * n + i];
      const float ex = __builtin_amdgcn_fmed3f(pij, -pji, 0.0f);  // pair_exchange (p2pmg_kernels.hip)
      gg = gg + (pij - ex);
      pp = pp + ex;
    }
    // _compute_costs community.py:56-65; RLAgent.get_reward agent.py:225-232 (pre-update T_in)
    float cost = (gg >= 0.0f) ? gg * buy : gg * inj;
    cost = cost + pp * p2pp;
    cost = (cost * p.slot) / p.mph;
    cost = cost * p.kilo;
    float pen = fmaxf(fmaxf(0.0f, p.lower - g.tin), fmaxf(0.0f, g.tin - p.upper));
    pen = pen > 0.0f ? pen + 1.0f : 0.0f;
    const float rw = -(cost + p.penw * pen);

    if (p.mode != 1) {
      // DQNAgent.save_memory agent.py:332-336 -> ReplayBuffer.add rl.py:208-212
      const int32_t n_added = d.added[a];
      float* slot = d.buf + ((size_t)a * d.cap + (size_t)(n_added % d.cap)) * kTrans;
      if (lane < kTrans) {
        const float av = g.act == 0 ? 0.0f : (g.act == 1 ? 0.5f : 1.0f);
        float v;
        switch (lane) {
          case 0: v = time_t; break;
          case 1: v = g.tnorm; break;
          case 2: v = g.bal; break;
          case 3: v = g.p2pf; break;
          case 4: v = av; break;
          case 5: v = rw; break;
          case 6: v = time_n; break;
          case 7: v = g.tnorm; break;  // next state: same (pre-update) temperature (community.py:161)
          case 8: v = g.baln; break;
          default: v = 0.0f / g.mi; break;  // next state p2p = mean(zeros) / max_in
        }
        slot[lane] = v;
      }
      if (lane == 0) d.added[a] = n_added + 1;
      // Trainer.train -> ReplayBuffer.sample_batch (rl.py:299-305, 226-241) right after the append
      // (agent.py:338-342): the same wave draws the agent's 32 slots, no separate launch
      if (p.mode == 0 && d.fused_sample) sample_slots(d, a, lane, n_added + 1);
    }
    if (lane == 0) {
      const size_t kr = (size_t)t * A + a;
      if (p.record & 1) p.rec_reward[kr] = rw;
      if (p.record & 2) p.rec_cost[kr] = cost;
      if (p.record & 4) p.rec_grid[kr] = gg;
      if (p.record & 8) p.rec_p2p[kr] = pp;
      if (p.record & 16) p.rec_tin[kr] = g.tin;
      float tin = g.tin, tm = g.tm;
      rc_update(p, t_out, g.hp, tin, tm);  // HPHeating.step heating.py:138-143
      p.t_in[a] = tin;
      p.t_m[a] = tm;
      shR[i] = rw;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // avg_reward = sum_t mean_i r (community.py:179), canonical order
    float m = 0.0f;
#pragma unroll
    for (int j = 0; j < n; ++j) m = m + shR[j];
    const float ep = (t == 0 ? 0.0f : d.ep_acc[s]) + divn(m);
    d.ep_acc[s] = ep;
    p.ep_reward[s] = ep;
  }
}

// ----------------------------------------------------------------- act, one shared network
// dqn_act_shared_kernel<N, AGW>: the same env step as dqn_act_kernel for ONE network shared by
// every agent (configs[4]), with the greedy forwards of AGW agents on MFMA tiles.  A 256-thread
// workgroup owns AGW / N scenarios.  Per round, thread j < AGW does agent j's scalar work
// (observation, divide-power row); the 3 AGW greedy rows (3 actions x AGW agents) go
// through layer 1 on VALU (thread = hidden unit x AGW / 4 agents), layer 2 as Z2^T = W2^T H1^T on
// v_mfma_f32_16x16x4_f32 (wave w owns hidden units 16w..16w+15; its 16 W2 operands stay in
// registers for the launch; the shared W2 is read once per workgroup instead of once per agent and
// round), layer 3 in-lane.  Bitwise the same Q values as dqn_act_kernel: the f32 MFMA accumulates
// its K products as an fmaf chain in k order (the VALU loop's order), and layer 3's sum over the 64
// units is the same pairwise tree (4 units in-lane, the 16-lane row groups over lane ^ 16 and
// lane ^ 32, then the 4 waves pairwise) as wave_sum over lane = unit.
// AGW agent slots per workgroup (16, or 8 for more, shorter workgroups); row = action * AGW + slot,
// in MT = ceil(3 AGW / 16) row tiles

#ifndef P2PMG_TRACE
#define P2PMG_TRACE 0
#endif
#if P2PMG_TRACE  // timing-only: s_memtime phase splits of wave 0 (scripts/gpu_dqn_trace.sh)
#define ACT_STAMP(k)                                                             \
  do {                                                                           \
    uint64_t t_;                                                                 \
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    atr[k] += t_ - alast;                                                        \
    alast = t_;                                                                  \
  } while (0)
#else
#define ACT_STAMP(k) \
  do {               \
  } while (0)
#endif
// The shared network's post-exchange Adam step of parameter k (NSEG >= d.n_segs): the gathered
// segments summed in global segment order, the mean over every agent of every rank, clip, Keras Adam
// (beta1 .9, beta2 .999) and Trainer._soft_update (rl.py:307-359).  Every segment's value and the Adam
// state are loaded before the first add (one memory round trip).  Returns the new weight; `store`:
// writes the new moments, weight and soft-updated target to the *_out arrays.  One function for the
// standalone launch and the act kernel's fused form, so both give the same bits.
template <int NSEG>
__device__ __forceinline__ float adam_shared_param(const DqnParams& d, int k, bool store) {
  const int n = d.n_segs;
  float sv[NSEG];
#pragma unroll
  for (int g = 0; g < NSEG; ++g) sv[g] = g < n ? d.segs[(size_t)g * kNetStride + k] : 0.0f;
  const float m0 = d.adam_m[k], v0 = d.adam_v[k], w0 = d.theta[k];
  const float tg0 = store ? d.target[k] : 0.0f;
  float t = sv[0];
#pragma unroll
  for (int g = 1; g < NSEG; ++g) t = g < n ? t + sv[g] : t;  // segs 0 + 1 + ... + n-1, in order
  float gk = t * d.inv_agents;
  if (k < kOffB1) gk = fminf(fmaxf(gk, -d.clip), d.clip);
  const float m = m0 + (gk - m0) * d.b1c;
  const float v = v0 + (gk * gk - v0) * d.b2c;
  const float w = w0 - (m * d.lr_t) / (sqrtf(v) + d.adam_eps);
  if (store) {
    d.m_out[k] = m;
    d.v_out[k] = v;
    d.theta_out[k] = w;
    d.target_out[k] = d.tau_c * tg0 + d.tau * w;
  }
  return w;
}

// ADAM: the previous env step's shared Adam step is still pending (the multi-segment / multi-rank
// path): every workgroup computes the new value of each weight it reads from the gathered segments
// (adam_shared_param, the same bits as dqn_adam_shared_kernel), and workgroup 0, whose threads cover
// every parameter once, stores the new state into the other half of the runtime's double buffer, so
// no workgroup of this launch reads a value another one wrote.  This replaces a 4,609-parameter launch
// per env step (one launch plus a memory round trip) with loads issued among the act prologue's own.
template <int N, int AGW, bool ADAM>
__global__ __launch_bounds__(256) void dqn_act_shared_kernel(const DqnParams d) {
  static_assert(AGW == 8 || AGW == 16, "8 or 16 agent slots per workgroup");
  constexpr int SPW = AGW / N;          // scenarios per workgroup
  constexpr int AG = SPW * N;           // agents per workgroup (<= AGW)
  constexpr int MT = (3 * AGW + 15) / 16;  // row tiles of the greedy forward
  constexpr int SPT = AGW / 4;          // layer-1 agent slots per thread (4 waves)
  const EpisodeParams& p = d.e;
#if P2PMG_TRACE
  uint64_t atr[8] = {0, 0, 0, 0, 0, 0, 0, 0}, alast;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(alast)::"memory");
#endif
  __shared__ float shP[2][AG * N];
  __shared__ float4 shX[AGW];   // time, normalised T_in, balance, p2p of agent slot j
  __shared__ float H1[16 * MT][kLdsRow];
  __shared__ float qpart[4][64];  // 4 tiles of reduce4_groups (MT used)
  __shared__ float shR[AG];
  __shared__ int shN[AGW];
  __shared__ float shEp[AGW];
  __shared__ int shFlag[2];
  __shared__ __attribute__((aligned(16))) int shI[AGW][kB];  // Floyd draws of the replay sample
  const int tid = threadIdx.x;
  const int w = tid / kWave, l = tid % kWave;
  const int c16 = l & 15, g4 = l >> 4;
  const int t = d.t, T = p.T, tn = (t + 1 == T) ? 0 : t + 1;
  const int R1 = p.R + 1, W = (R1 + 3) >> 2;
  const size_t A = (size_t)p.A;
  const bool greedy_mode = p.mode == 1;
  const int s0 = blockIdx.x * SPW;
  const float* th = d.theta;

  // agent thread j < AG: agent a = s0 * N + j of scenario s0 + j / N (agent i = j % N)
  const int j = tid;
  const int sl = j / N, i = j % N;
  const int s = s0 + sl;
  const bool agent_thr = j < AG && s < p.S;
  const int a = agent_thr ? s * N + i : 0;
  const int s_env = p.n_env == 1 ? 0 : (agent_thr ? s : 0);
  const float* e0 = p.env + ((size_t)t * p.n_env + s_env) * kEnvStride;
  const float* e1 = p.env + ((size_t)tn * p.n_env + s_env) * kEnvStride;
  float buy = 0.0f, inj = 0.0f, p2pp = 0.0f;
  float time_t = 0.0f, t_out = 0.0f, time_n = 0.0f, mi = 1.0f, tin = 0.0f, tm = 0.0f, bal = 0.0f, baln = 0.0f,
        tnorm = 0.0f;
  float4 lv = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (agent_thr) {
    time_t = e0[0];
    t_out = e0[1];
    buy = e0[2];
    inj = e0[3];
    p2pp = e0[4];
    time_n = e1[0];
    const float2 f0 = p.prof[(size_t)t * A + a], f1 = p.prof[(size_t)tn * A + a];
    mi = p.max_in[a];
    tin = p.t_in[a];
    tm = p.t_m[a];
    bal = (f0.x - f0.y) / mi;  // RLAgent._get_balance agent.py:172-176
    baln = (f1.x - f1.y) / mi;
    tnorm = (tin - p.setpoint) / p.margin;  // HPHeating.normalized_temperature heating.py:118-120
    lv = p.hp_lv[a];
  }
  // loaded with the inputs: a load issued after the step's stores would wait for their completion
  // (vmcnt counts loads and stores in issue order)
  const int32_t n_added = (agent_thr && p.mode != 1) ? d.added[a] : 0;
  const float ep_prev = (tid < SPW && s0 + tid < p.S && t != 0) ? d.ep_acc[s0 + tid] : 0.0f;
  // weight k as this launch uses it; ADAM: after the pending step, stored by workgroup 0's owner
  // thread of k (layer 1: wave 0; W2: every thread; b2 / W3: lanes c16 = 0; b3: thread 0)
  const bool blk0 = ADAM && blockIdx.x == 0;
  auto wt = [&](int k, bool owner) -> float {
    if constexpr (ADAM) return adam_shared_param<kActAdamSegs>(d, k, blk0 && owner);
    else return th[k];
  };
  // layer 1 (thread = hidden unit u of agent slots 4 * (tid / 64) .. + 3): W1 column and b1
  const int u = l;
  const float w10 = wt(kOffW1 + 0 * kH + u, w == 0), w11 = wt(kOffW1 + 1 * kH + u, w == 0),
              w12 = wt(kOffW1 + 2 * kH + u, w == 0), w13 = wt(kOffW1 + 3 * kH + u, w == 0),
              w14 = wt(kOffW1 + 4 * kH + u, w == 0), b1 = wt(kOffB1 + u, w == 0);
  // layer 2 / 3 (wave w, lane: A operand W2[4 kk + g4][16 w + c16]; accumulator units 16 w + 4 g4 + r)
  float w2[16];
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) w2[kk] = wt(kOffW2 + (4 * kk + g4) * kH + 16 * w + c16, true);
  float b2[4], w3[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    b2[r] = wt(kOffB2 + 16 * w + 4 * g4 + r, c16 == 0);
    w3[r] = wt(kOffW3 + 16 * w + 4 * g4 + r, c16 == 0);
  }
  const float b3 = wt(kOffB3, tid == 0);
  // every round's exploration draw (or replayed code) ahead of the rounds: they depend only on
  // (t, episode, agent), so they run under the prologue's load latency, off the rounds' chain
  uint64_t codes_pack = ~0ull;  // byte r: code of round r < 8 (255 = greedy); later rounds are drawn in the loop
  if (agent_thr && !greedy_mode) {
    if (p.rng == 0) {
      for (int w4 = 0; w4 < W && w4 < 2; ++w4)
        codes_pack = (codes_pack & ~(0xFFFFFFFFull << (32 * w4))) |
                     ((uint64_t)p.codes[((size_t)t * W + w4) * A + a] << (32 * w4));
    } else {
      // every round's code of step t (p2pmg_device.h, oracle/philox.py::decision_draws)
      codes_pack = philox_step_codes(t, R1, (uint32_t)p.episode, p.agent_offset + (uint32_t)a, p.eps_thr, p.eps_all,
                                     p.seed_lo, p.seed_hi);
    }
  }
  const int tag4 = reduce4_tag();

  if (tid < AG * N) shP[0][tid] = 0.0f;
  // consumed here, before the rounds' record stores: a later first use would wait for those stores
  if (agent_thr) shN[j] = n_added + 1;
  if (tid < SPW) shEp[tid] = ep_prev;
  __syncthreads();
  ACT_STAMP(0);
  int cur = 0, act = 0, code = 255;
  float hp = 0.0f, p2pf = 0.0f;
  uint64_t act_pack = 0;
  for (int r = 0; r < R1; ++r) {
    const float* P = shP[cur] + sl * N * N;  // this agent's scenario
    bool greedy = false;
    if (agent_thr) {
      // powers = -P[:, i], diagonal zeroed (community.py:76,81); p2p = mean / max_in (agent.py:203)
      float acc = 0.0f;
#pragma unroll
      for (int jj = 0; jj < N; ++jj) acc = acc + (-((jj == i) ? 0.0f : P[jj * N + i]));
      p2pf = div_n<N>(acc) / mi;
      code = 255;  // ActorModel.select_action rl.py:174-183: explore draw, else greedy
      if (!greedy_mode) {
        if (r < 8) code = (int)((codes_pack >> (8 * r)) & 0xFFu);
        else if (p.rng == 0) code = (int)((p.codes[((size_t)t * W + (r >> 2)) * A + a] >> (8 * (r & 3))) & 0xFFu);
        else
          code = (int)philox_round_code(t, R1, r, (uint32_t)p.episode, p.agent_offset + (uint32_t)a, p.eps_thr,
                                        p.eps_all, p.seed_lo, p.seed_hi);
      }
      greedy = code == 255;
      shX[j] = make_float4(time_t, tnorm, bal, p2pf);
    }
    ACT_STAMP(1);
    if (__syncthreads_or(greedy)) {
      // layer 1: the three action rows of agent slots SPT w .. + SPT - 1 at unit u
#pragma unroll
      for (int q = 0; q < SPT; ++q) {
        const int ag = SPT * w + q;
        const float4 x = shX[ag];
        float z = x.w * w13;
        z = fmaf(x.z, w12, z);
        z = fmaf(x.y, w11, z);
        z = fmaf(x.x, w10, z);
        H1[ag][u] = relu(z + b1);
        H1[AGW + ag][u] = relu(fmaf(0.5f, w14, z) + b1);
        H1[2 * AGW + ag][u] = relu((z + w14) + b1);
      }
      __syncthreads();
      f32x4 acc[MT];
#pragma unroll
      for (int rt = 0; rt < MT; ++rt) acc[rt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
#pragma unroll
        for (int rt = 0; rt < MT; ++rt) acc[rt] = mfma4(w2[kk], H1[16 * rt + c16][4 * kk + g4], acc[rt]);
      float sq[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int rt = 0; rt < MT; ++rt) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = relu(acc[rt][q] + b2[q]) * w3[q];
        sq[rt] = (v[0] + v[1]) + (v[2] + v[3]);  // wave_sum's tree: 4 units in-lane, ...
      }
      qpart[w][16 * tag4 + c16] = reduce4_groups(sq[0], sq[1], sq[2], 0.0f);  // ... the 4 row groups
      __syncthreads();
    }
    ACT_STAMP(2);
    if (agent_thr) {
      if (greedy) {
        // ActorModel.greedy_action rl.py:188-196: Q(obs, a) for a in (0, .5, 1), argmax (first max)
        float qv[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int row = AGW * k + j;
          qv[k] = ((qpart[0][row] + qpart[1][row]) + (qpart[2][row] + qpart[3][row])) + b3;
        }
        act = 0;
        float best = qv[0];
        if (qv[1] > best) { best = qv[1]; act = 1; }
        if (qv[2] > best) act = 2;
      } else {
        act = code;
      }
      hp = act == 0 ? lv.x : (act == 1 ? lv.y : lv.z);  // heating.set_power(action) -> hp.power * max_power
      // RLAgent._divide_power agent.py:186-195 on out = balance * max_in + hp (agent.py:210)
      const float out = (bal * mi) + hp;
      const float so = sgn(out);
      float f[N];
      float tot = 0.0f;
#pragma unroll
      for (int jj = 0; jj < N; ++jj) {
        const float pw = -((jj == i || r == 0) ? 0.0f : P[jj * N + i]);
        f[jj] = (so != sgn(pw)) ? pw : 0.0f;
        tot = tot + f[jj];
      }
      tot = fabsf(tot);
      float* Pn = shP[cur ^ 1] + sl * N * N + i * N;
#pragma unroll
      for (int jj = 0; jj < N; ++jj) {
        float v;
        if (tot == 0.0f) v = div_n<N>(out * 1.0f);
        else v = (jj == i) ? (tot == tot ? out * 0.0f : tot) : (out * fabsf(f[jj])) / tot;
        Pn[jj] = v;
      }
      if (p.record & 32) act_pack |= (uint64_t)act << (8 * r);  // stored with the other records at the end
    }
    __syncthreads();
    cur ^= 1;
    ACT_STAMP(3);
  }
  // the step's stores all go out at the end of the kernel, after the replay draws: nothing after them
  // waits on vmcnt (which counts stores and loads alike)
  float g = 0.0f, pp = 0.0f, cost = 0.0f, rw = 0.0f, tin0 = tin;
  if (agent_thr) {
    // CommunityMicrogrid._assign_powers community.py:45-54 (final P, diagonal kept)
    const float* P = shP[cur] + sl * N * N;
#pragma unroll
    for (int jj = 0; jj < N; ++jj) {
      const float pij = P[i * N + jj], pji = P[jj * N + i];
      const float ex = __builtin_amdgcn_fmed3f(pij, -pji, 0.0f);  // pair_exchange (p2pmg_kernels.hip)
      g = g + (pij - ex);
      pp = pp + ex;
    }
    // _compute_costs community.py:56-65; RLAgent.get_reward agent.py:225-232 (pre-update T_in)
    cost = (g >= 0.0f) ? g * buy : g * inj;
    cost = cost + pp * p2pp;
    cost = (cost * p.slot) / p.mph;
    cost = cost * p.kilo;
    float pen = fmaxf(fmaxf(0.0f, p.lower - tin), fmaxf(0.0f, tin - p.upper));
    pen = pen > 0.0f ? pen + 1.0f : 0.0f;
    rw = -(cost + p.penw * pen);
    rc_update(p, t_out, hp, tin, tm);  // HPHeating.step heating.py:138-143
    shR[j] = rw;
  }
  __syncthreads();
  ACT_STAMP(4);
  float ep = 0.0f;
  if (tid < SPW) {  // avg_reward = sum_t mean_i r (community.py:179), canonical order
    float m = 0.0f;
#pragma unroll
    for (int jj = 0; jj < N; ++jj) m = m + shR[tid * N + jj];
    ep = shEp[tid] + div_n<N>(m);
  }
  // Trainer.train -> ReplayBuffer.sample_batch (rl.py:299-305, 226-241) right after the append
  // (agent.py:338-342).  Floyd's draw j keeps r_j unless an earlier draw l < j ended on r_j, when it
  // takes count - 32 + j.  Sixteen threads per agent (draws q and q + 16) solve that recurrence as a
  // fixpoint over the agent's 32 indices in LDS: every pass recomputes each draw from the current
  // indices of the earlier ones, so after pass k the first k draws are final and a pass that changes
  // nothing has reached the sequential result (typically 2 passes instead of 32 serial steps).
  if (p.mode == 0 && d.fused_sample) {
    // AGW = 16: 16 threads per agent, draws q0 and q0 + 16; AGW = 8: 32 threads per agent, one draw
    // each (the second draw duplicates the first: same result, written twice)
    constexpr int TPA = 256 / AGW;
    const int aj = tid / TPA, q0 = tid % TPA, q1 = TPA == 16 ? q0 + 16 : q0;
    const bool va = aj < AG && s0 + aj / N < p.S;
    const int a2 = va ? s0 * N + aj : 0;
    const int n_add = va ? shN[aj] : kB;
    const int count = n_add < d.cap ? n_add : d.cap;
    const int fm = (n_add - count) % d.cap;  // ring slot of the deque's first element
    int i0, i1;
    if (d.samples) {
      i0 = va ? (int)d.samples[((size_t)t * A + a2) * kB + q0] : 0;
      i1 = va ? (int)d.samples[((size_t)t * A + a2) * kB + q1] : 0;
    } else {
      int r[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && TPA != 16) {
          r[1] = r[0];
          break;
        }
        const int q = h ? q1 : q0;
        uint32_t c0 = (uint32_t)t, c1 = (uint32_t)p.episode, c2 = p.agent_offset + (uint32_t)a2, c3 = kTagSample + (uint32_t)q;
        philox4x32_10(c0, c1, c2, c3, p.seed_lo, p.seed_hi);
        r[h] = (int)__umulhi(c0, (uint32_t)(count - kB + q + 1));
      }
      i0 = r[0];
      i1 = r[1];
      shI[aj][q0] = i0;
      shI[aj][q1] = i1;
      if (tid == 0) shFlag[0] = 0;
      __syncthreads();
      // branch-free pass: bit l of hit_h says draw l's current index equals r_h; only l < q counts
      const uint32_t early0 = (1u << q0) - 1u, early1 = (q1 == 31 ? 0x7FFFFFFFu : (1u << q1) - 1u);
      for (int pass = 0;; ++pass) {
        uint32_t hit0 = 0u, hit1 = 0u;
#pragma unroll
        for (int v = 0; v < kB / 4; ++v) {
          const int4 x = *reinterpret_cast<const int4*>(&shI[aj][4 * v]);
          const int xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            hit0 |= xs[e] == r[0] ? 1u << (4 * v + e) : 0u;
            hit1 |= xs[e] == r[1] ? 1u << (4 * v + e) : 0u;
          }
        }
        const int n0 = (hit0 & early0) ? count - kB + q0 : r[0], n1 = (hit1 & early1) ? count - kB + q1 : r[1];
        const bool ch = n0 != i0 || n1 != i1;
        __syncthreads();  // every read of this pass before any write
        i0 = n0;
        i1 = n1;
        shI[aj][q0] = i0;
        shI[aj][q1] = i1;
        if (ch) shFlag[pass & 1] = 1;
        if (tid == 0) shFlag[(pass + 1) & 1] = 0;
        __syncthreads();
        if (shFlag[pass & 1] == 0) break;  // workgroup-uniform: nothing changed in this pass
      }
    }
    if (va) {
      int* out = reinterpret_cast<int*>(d.smp) + (size_t)a2 * kB;
      const int sl0 = fm + i0, sl1 = fm + i1;
      out[q0] = sl0 >= d.cap ? sl0 - d.cap : sl0;
      out[q1] = sl1 >= d.cap ? sl1 - d.cap : sl1;
    }
  }
  if (agent_thr) {
    if (p.mode != 1) {
      // DQNAgent.save_memory agent.py:332-336 -> ReplayBuffer.add rl.py:208-212
      const int n_added = shN[j] - 1;
      float2* slot = reinterpret_cast<float2*>(d.buf + ((size_t)a * d.cap + (size_t)(n_added % d.cap)) * kTrans);
      const float av = act == 0 ? 0.0f : (act == 1 ? 0.5f : 1.0f);
      slot[0] = make_float2(time_t, tnorm);
      slot[1] = make_float2(bal, p2pf);
      slot[2] = make_float2(av, rw);
      slot[3] = make_float2(time_n, tnorm);  // next state: same (pre-update) temperature (community.py:161)
      slot[4] = make_float2(baln, 0.0f / mi);  // next state p2p = mean(zeros) / max_in
      d.added[a] = n_added + 1;
    }
    const size_t k = (size_t)t * A + a;
    if (p.record & 1) p.rec_reward[k] = rw;
    if (p.record & 2) p.rec_cost[k] = cost;
    if (p.record & 4) p.rec_grid[k] = g;
    if (p.record & 8) p.rec_p2p[k] = pp;
    if (p.record & 16) p.rec_tin[k] = tin0;
    if (p.record & 32)
      for (int r = 0; r < R1; ++r) p.rec_action[((size_t)t * R1 + r) * A + a] = (uint8_t)(act_pack >> (8 * r));
    p.t_in[a] = tin;
    p.t_m[a] = tm;
  }
  if (tid < SPW && s0 + tid < p.S) {
    d.ep_acc[s0 + tid] = ep;
    p.ep_reward[s0 + tid] = ep;
  }
#if P2PMG_TRACE
  ACT_STAMP(5);
  if (l == 0 && w == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2) && (d.t == 50 || d.t == 51))
    printf("ACTTRACE blk %d t %d mode %d: prologue %llu agentA %llu forward %llu agentB %llu epilogue %llu sample %llu\n",
           (int)blockIdx.x, d.t, p.mode, (unsigned long long)atr[0], (unsigned long long)atr[1],
           (unsigned long long)atr[2], (unsigned long long)atr[3], (unsigned long long)atr[4],
           (unsigned long long)atr[5]);
#endif
}

// ----------------------------------------------------------------- train: Trainer._train
__device__ __forceinline__ void adam_update(const DqnParams& d, float* th, float* tg, float* mm, float* vv, int idx,
                                            float g, float lr) {
  // Keras Adam (beta1 .9, beta2 .999, eps 1e-7) then Trainer._soft_update (rl.py:335-354)
  float m = mm[idx], v = vv[idx], w = th[idx];
  m = m + (g - m) * d.b1c;
  v = v + (g * g - v) * d.b2c;
  w = w - (m * lr) / (sqrtf(v) + d.adam_eps);
  mm[idx] = m;
  vv[idx] = v;
  th[idx] = w;
  tg[idx] = d.tau_c * tg[idx] + d.tau * w;
}


// one thread's share of agent a's sampled batch (thread t: sample t / 8, floats t % 8 and, for
// t % 8 < 2, t % 8 + 8), gathered from the replay ring through the sample kernel's slot indices
// (a is uniform: the agent's ring and slot row are scalar bases, each lane adds a 32-bit byte offset,
// so no per-lane 64-bit address stays live across the agent loop)
__device__ __forceinline__ int batch_slot(const DqnParams& d, int a, int t) {
  const char* row = reinterpret_cast<const char*>(d.smp) + (size_t)a * kB * sizeof(int);
  return *reinterpret_cast<const int*>(row + (uint32_t)(t >> 3) * (uint32_t)sizeof(int));
}
__device__ __forceinline__ void batch_part_at(const DqnParams& d, int a, int t, int slot, float& v0, float& v1) {
  const int k = t & 7;
  const char* ring = reinterpret_cast<const char*>(d.buf + (size_t)a * d.cap * kTrans);
  const uint32_t off = ((uint32_t)slot * kTrans + (uint32_t)k) * (uint32_t)sizeof(float);  // cap * 40 B < 4 GiB
  v0 = *reinterpret_cast<const float*>(ring + off);
  v1 = k < kTrans - 8 ? *reinterpret_cast<const float*>(ring + off + 8 * sizeof(float)) : 0.0f;
}
__device__ __forceinline__ void batch_part(const DqnParams& d, int a, int t, float& v0, float& v1) {
  batch_part_at(d, a, t, batch_slot(d, a, t), v0, v1);
}
__device__ __forceinline__ void batch_put(float* dst, int t, float v0, float v1) {
  const int b = t >> 3, k = t & 7;
  dst[b * kTrans + k] = v0;
  if (k < kTrans - 8) dst[b * kTrans + k + 8] = v1;
}

// the weights one train workgroup reads, per lane (layer 1 and dH1: column col of wave w;
// layers 2 and 3: the 4 hidden units 16 w + 4 g4 + r of the transposed tiles).  Per-agent networks
// read W2 per MFMA step from L1/L2; a shared network keeps its 48 W2 operands in registers.
struct TrainW {
  float bt0, bo0, bo1, b1t, b1o, b3t, b3o, w14t;  // layer 1: W1[g4][col], W1[4][col] (g4 = 0), biases
  float b2t[4], w3t[4], b2o[4], w3o[4];  // layer 2/3 of the hidden units 16 w + 4 g4 + r
};
__device__ __forceinline__ void load_train_w(TrainW& W, const float* th, const float* tg, int col, int g4, int h0) {
  W.bt0 = tg[kOffW1 + g4 * kH + col];
  W.bo0 = th[kOffW1 + g4 * kH + col];
  W.w14t = tg[kOffW1 + 4 * kH + col];
  W.bo1 = g4 == 0 ? th[kOffW1 + 4 * kH + col] : 0.0f;
  W.b1t = tg[kOffB1 + col];
  W.b1o = th[kOffB1 + col];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    W.b2t[r] = tg[kOffB2 + h0 + r];
    W.w3t[r] = tg[kOffW3 + h0 + r];
    W.b2o[r] = th[kOffB2 + h0 + r];
    W.w3o[r] = th[kOffW3 + h0 + r];
  }
  W.b3t = tg[kOffB3];
  W.b3o = th[kOffB3];
}

// timing-only probe (-DP2PMG_TRACE): per-phase s_memtime splits of the agent loop, printed for env
// step 50 by every wave of two workgroups (scripts/gpu_dqn_trace.sh).  A phase's time includes
// the other workgroup's MFMAs sharing the SIMD, and MFMA results landing after their issue.
#ifndef P2PMG_TRACE
#define P2PMG_TRACE 0
#endif
#if P2PMG_TRACE
#define DQN_STAMP(k)                                                             \
  do {                                                                           \
    uint64_t t_;                                                                 \
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    trp[k] += t_ - tlast;                                                        \
    tlast = t_;                                                                  \
  } while (0)
#else
#define DQN_STAMP(k) \
  do {               \
  } while (0)
#endif
// train workgroups per CU (waves per SIMD): 2 in the default build (about 220 VGPRs)
#ifndef P2PMG_TRAIN_OCC
#define P2PMG_TRAIN_OCC 2
#endif
template <bool SHARED>
__global__ __launch_bounds__(256, P2PMG_TRAIN_OCC) void dqn_train_kernel(const DqnParams d) {
  __shared__ float smpb[2][kB * kTrans];  // this agent's batch and the next one's (prefetched)
  __shared__ float H1t[3 * kB][kLdsRow];
  __shared__ __attribute__((aligned(16))) float H1oT[kH][kLdsRowT];  // online layer-1 activations, unit-major
  __shared__ __attribute__((aligned(16))) float dZ2[kB][kLdsRow];
  __shared__ float qpart[4][4 * kB];  // per-wave partial Q: rows 0..95 target (action x sample), 96..127 online
  const EpisodeParams& p = d.e;
  const int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
  const int c16 = l & 15, g4 = l >> 4;
  const int col = 16 * w + c16;     // this lane's column of layer 1 and of dH1
  const int h0 = 16 * w + 4 * g4;   // this lane's 4 hidden units of layer 2 (transposed tiles)
  const size_t A = (size_t)p.A;

  f32x4 gW2[4], gW1[2];
#pragma unroll
  for (int m = 0; m < 4; ++m) gW2[m] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  gW1[0] = gW1[1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float gx1[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  float gb1 = 0.0f, gb3 = 0.0f;
  float gb2[4] = {0.0f, 0.0f, 0.0f, 0.0f}, gW3[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  // this workgroup's run of agents: block j of gradient segment g covers agents g * seg_agents +
  // j * apb .. (clipped to the segment), so no block straddles two segments (p2pmg_dqn_config)
  const int seg = blockIdx.x / d.bps, sblk = blockIdx.x - seg * d.bps;
  const int a_first = seg * d.seg_agents + sblk * d.apb;
  const int n_ag = d.batch ? 1 : max(0, min(d.apb, (seg + 1) * d.seg_agents - a_first));
  int net = d.batch ? d.net : 0;
  TrainW W;
  // one shared network: the lane's 48 W2 operands (layer 2: W2[4 kk + g4][col] of the target and
  // the online network; dH1: W2[col][4 kk + g4]) stay in registers for the whole launch
  float w2t[SHARED ? 16 : 1], w2o[SHARED ? 16 : 1], w2c[SHARED ? 16 : 1];
  if constexpr (SHARED) {
    const float* th0 = d.theta + (size_t)net * kNetStride;
    const float* tg0 = d.target + (size_t)net * kNetStride;
    load_train_w(W, th0, tg0, col, g4, h0);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      w2t[kk] = tg0[kOffW2 + (4 * kk + g4) * kH + col];
      w2o[kk] = th0[kOffW2 + (4 * kk + g4) * kH + col];
      w2c[kk] = th0[kOffW2 + col * kH + 16 * g4 + kk];  // dH1's K order: unit 16 g4 + kk
    }
  }
  // the first agent's batch (explicit batch, or the sample pre-pass output)
  if (d.batch) {
    for (int k = threadIdx.x; k < kB * kTrans; k += 256) smpb[0][k] = d.batch[k];
  } else {
    float v0 = 0.0f, v1 = 0.0f;
    if (n_ag > 0) batch_part(d, a_first, threadIdx.x, v0, v1);
    batch_put(smpb[0], threadIdx.x, v0, v1);
  }
  // the next agent's slot index, loaded one agent ahead of its transitions: the dependent pair of
  // loads never makes the loop wait for a global round trip
  // (unconditional loads at clamped in-range indices: a branch around them would leave a
  // loop-carried register copy that waits for every load in flight)
  const int a_last = (int)A - 1;
  const int tag4 = reduce4_tag();
  int slot_n = batch_slot(d, min(a_first + 1, a_last), threadIdx.x);
  __syncthreads();

#if P2PMG_TRACE
  uint64_t trp[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(tlast)::"memory");
#endif
  for (int ag = 0; ag < n_ag; ++ag) {
    const int a = d.batch ? 0 : a_first + ag;
    net = d.batch ? d.net : (SHARED ? 0 : a);
    const float* th = d.theta + (size_t)net * kNetStride;
    const float* tg = d.target + (size_t)net * kNetStride;
    if (!SHARED) load_train_w(W, th, tg, col, g4, h0);
    float (*smp)[kTrans] = reinterpret_cast<float (*)[kTrans]>(smpb[ag & 1]);
    // prefetch the next agent's batch into registers; it goes to the other buffer at the end
    const bool has_next = !d.batch && ag + 1 < n_ag;
    float nx0, nx1;
    batch_part_at(d, min(a + 1, a_last), threadIdx.x, (int)min((unsigned)slot_n, (unsigned)(d.cap - 1)), nx0, nx1);
    slot_n = batch_slot(d, min(a + 2, a_last), threadIdx.x);

    // ---- layer 1: Z1 = X W1 + b1, 6 target + 2 online row tiles (K = 4 on MFMA, the action term
    // K = 4 as an fmaf for target tiles, a second MFMA for online tiles)
    const float bt0 = W.bt0, bo0 = W.bo0, bo1 = W.bo1, b1t = W.b1t, b1o = W.b1o;
    unsigned z1mask = 0;  // online rows where z1 > 0 (ReLU derivative), bit 4 rt + r
    __builtin_amdgcn_s_setprio(2);  // MFMA phase (see layer 2)
    // all products first (8 independent accumulators), then the bias / ReLU / LDS stores: no store
    // waits on the MFMA it follows
    f32x4 z1[8];
#pragma unroll
    for (int rt = 0; rt < 6; ++rt) {
      const int b = (16 * rt + c16) % kB;
      z1[rt] = mfma4(smp[b][6 + g4], bt0, f32x4{0.0f, 0.0f, 0.0f, 0.0f});
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) z1[6 + rt] = mfma4(smp[16 * rt + c16][g4], bo0, f32x4{0.0f, 0.0f, 0.0f, 0.0f});
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) z1[6 + rt] = mfma4(g4 == 0 ? smp[16 * rt + c16][4] : 0.0f, bo1, z1[6 + rt]);
    // a target tile holds one action value (rows 16 rt .. + 15: action rt / 2), so its K = 4 term
    // is a per-column fmaf, the same single rounding as an MFMA's second product would give
#pragma unroll
    for (int rt = 0; rt < 6; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        H1t[16 * rt + 4 * g4 + r][col] = relu(fmaf((rt >> 1) == 0 ? 0.0f : ((rt >> 1) == 1 ? 0.5f : 1.0f), W.w14t, z1[rt][r]) + b1t);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = z1[6 + rt][r] + b1o;
        h[r] = relu(z);
        if (z > 0.0f) z1mask |= 1u << (4 * rt + r);
      }
      *reinterpret_cast<float4*>(&H1oT[col][16 * rt + 4 * g4]) = make_float4(h[0], h[1], h[2], h[3]);
    }
    __builtin_amdgcn_s_setprio(0);
    DQN_STAMP(0);
    __syncthreads();
    DQN_STAMP(1);

    // The MFMA phases (layers 1 and 2, the backward products) run at raised wave priority: the
    // SIMD's other wave (another workgroup, in a VALU / LDS phase) then issues into the MFMA shadow
    // instead of competing with the MFMA stream (configs[4] 14.55 -> 13.93 ms per episode)
    __builtin_amdgcn_s_setprio(2);
    // ---- layer 2 as Z2^T = W2^T H1^T (K = 64): the operands of H1 W2 with the MFMA's A and B
    // swapped, so the accumulator of row tile rt holds data row 16 rt + c16 at the hidden units
    // h0 + r.  Layer 3 then sums 4 units in-lane and the 4 row groups with two exchanges, instead
    // of a 16-lane butterfly per (row, unit).
    f32x4 at[6], ao[2];
#pragma unroll
    for (int rt = 0; rt < 6; ++rt) at[rt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    ao[0] = ao[1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const int k = 4 * kk + g4;
      const float bt = SHARED ? w2t[SHARED ? kk : 0] : tg[kOffW2 + k * kH + col];
      const float bo = SHARED ? w2o[SHARED ? kk : 0] : th[kOffW2 + k * kH + col];
#pragma unroll
      for (int rt = 0; rt < 6; ++rt) at[rt] = mfma4(bt, H1t[16 * rt + c16][k], at[rt]);
      ao[0] = mfma4(bo, H1oT[k][c16], ao[0]);
      ao[1] = mfma4(bo, H1oT[k][16 + c16], ao[1]);
    }
    __builtin_amdgcn_s_setprio(0);
    DQN_STAMP(2);
    // ---- layer 3, this wave's 16 units: in-lane over r (a pairwise tree), then over the 4 row
    // groups for four tiles at once (reduce4_groups: 3 lane swaps + 3 adds, row group g4 ends with
    // tile tag4's sum), so every lane stores one value per four tiles, without a masked branch
    float s8[8];
#pragma unroll
    for (int rt = 0; rt < 6; ++rt) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = relu(at[rt][r] + W.b2t[r]) * W.w3t[r];
      s8[rt] = (v[0] + v[1]) + (v[2] + v[3]);
    }
    float h2o[2][4];
    unsigned z2mask = 0;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = ao[rt][r] + W.b2o[r];
        h2o[rt][r] = relu(z);
        if (z > 0.0f) z2mask |= 1u << (4 * rt + r);
        v[r] = h2o[rt][r] * W.w3o[r];
      }
      s8[6 + rt] = (v[0] + v[1]) + (v[2] + v[3]);
    }
    qpart[w][16 * tag4 + c16] = reduce4_groups(s8[0], s8[1], s8[2], s8[3]);
    qpart[w][4 * kB / 2 + 16 * tag4 + c16] = reduce4_groups(s8[4], s8[5], s8[6], s8[7]);
    DQN_STAMP(3);
    __syncthreads();
    DQN_STAMP(1);

    // ---- targets y = r + gamma * max_a' Q_target(ns, a') and dL/dq (rl.py:314-331), for this
    // lane's data rows b = 16 rt + c16
    float dq[2];
    float lsum = 0.0f, dqsum = 0.0f;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int b = 16 * rt + c16;
      float qt[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int row = k * kB + b;
        qt[k] = (((qpart[0][row] + qpart[1][row]) + qpart[2][row]) + qpart[3][row]) + W.b3t;
      }
      const int ro = 3 * kB + b;
      const float q = (((qpart[0][ro] + qpart[1][ro]) + qpart[2][ro]) + qpart[3][ro]) + W.b3o;
      const float y = smp[b][5] + d.gamma * fmaxf(fmaxf(qt[0], qt[1]), qt[2]);
      const float diff = q - y;
      dq[rt] = (2.0f / (float)kB) * diff;
      lsum += diff * diff;
      dqsum += dq[rt];
    }
    // the 16 lanes of a row group hold the 32 rows: dL/db3 = sum dq in wave 0, the loss
    // mean (y - q)^2 (only when it is recorded) in wave 1, so neither holds the others at the barrier
    if (w == 0) {
      const float dqs = sum16(dqsum);
      if (l == 0) gb3 += dqs;
    } else if (w == 1 && (d.batch || d.rec_loss)) {
      const float ls = sum16(lsum);
      if (l == 0) {
        const float loss = ls / (float)kB;
        if (d.batch) d.loss_out[0] = loss;
        else d.rec_loss[(size_t)d.t * A + a] = loss;
      }
    }

    // ---- backward: dZ2 of this lane's (row, units), stored row-major for dW2 and dH1
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float dz2[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool on = (z2mask >> (4 * rt + r)) & 1u;
        dz2[r] = on ? dq[rt] * W.w3o[r] : 0.0f;
        gW3[r] += h2o[rt][r] * dq[rt];
        gb2[r] += dz2[r];
      }
      *reinterpret_cast<float4*>(&dZ2[16 * rt + c16][h0]) = make_float4(dz2[0], dz2[1], dz2[2], dz2[3]);
    }
    DQN_STAMP(4);
    __syncthreads();
    DQN_STAMP(1);
    __builtin_amdgcn_s_setprio(2);
    // Every operand of the backward products is read from LDS up front (16-B reads where the K
    // order allows), so the MFMA chains below never wait on a read between two products.
    // dW2 = H1^T dZ2 over the 32 data rows in the K order b = 8 g4 + q: A = H1oT[16 mt + c16][b]
    // (two 16-B reads per mt), B = dZ2[b][col]; accumulator rows = layer-1 units 16 mt + 4 g4 + r,
    // columns = the wave's layer-2 units col
    float ha[4][8], db[8];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const float4 u0 = *reinterpret_cast<const float4*>(&H1oT[16 * mt + c16][8 * g4]);
      const float4 u1 = *reinterpret_cast<const float4*>(&H1oT[16 * mt + c16][8 * g4 + 4]);
      ha[mt][0] = u0.x; ha[mt][1] = u0.y; ha[mt][2] = u0.z; ha[mt][3] = u0.w;
      ha[mt][4] = u1.x; ha[mt][5] = u1.y; ha[mt][6] = u1.z; ha[mt][7] = u1.w;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) db[q] = dZ2[8 * g4 + q][col];
    // dH1 = dZ2 W2^T (own columns n = col) in the K order unit 16 g4 + kk: A = dZ2[16 rt + c16][16 g4
    // .. + 15] (four 16-B reads per rt), B = W2[col][16 g4 + kk] (registers for a shared network)
#if P2PMG_TRAIN_OCC >= 3  // register budget: dW2's products issue before dH1's operands are read
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) gW2[mt] = mfma4(ha[mt][q], db[q], gW2[mt]);
    __builtin_amdgcn_sched_barrier(0);
#endif
    float za[2][16];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float4 u = *reinterpret_cast<const float4*>(&dZ2[16 * rt + c16][16 * g4 + 4 * v]);
        za[rt][4 * v] = u.x; za[rt][4 * v + 1] = u.y; za[rt][4 * v + 2] = u.z; za[rt][4 * v + 3] = u.w;
      }
    // dW1's A operand: input feature c16 (< 5) of data rows b = 16 rt + 4 g4 + r (lanes c16 >= 5 read
    // feature 4 and select 0: no exec-masked read)
#if P2PMG_TRAIN_OCC < 3
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) gW2[mt] = mfma4(ha[mt][q], db[q], gW2[mt]);
#endif
    f32x4 acc[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
        acc[rt] = mfma4(za[rt][kk], SHARED ? w2c[SHARED ? kk : 0] : th[kOffW2 + col * kH + 16 * g4 + kk], acc[rt]);
    // dZ1 = dH1 * [z1 > 0]; dW1 = X^T dZ1 (two accumulators: independent chains)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const float dz1 = ((z1mask >> (4 * rt + r)) & 1u) ? acc[rt][r] : 0.0f;
        gb1 += dz1;
        // dW1 = X^T dZ1 on VALU: this lane's partial over its 8 data rows, reduced over the row
        // groups once per launch (5 useful output rows of 16 made the MFMA form mostly padding)
        const float* xr = smp[16 * rt + 4 * g4 + r];
#pragma unroll
        for (int k = 0; k < 5; ++k) gx1[k] = fmaf(xr[k], dz1, gx1[k]);
      }
    __builtin_amdgcn_s_setprio(0);
    if (has_next) batch_put(smpb[(ag + 1) & 1], threadIdx.x, nx0, nx1);
    DQN_STAMP(5);
    __syncthreads();  // every wave is done with this agent's LDS and with the online W2
    DQN_STAMP(1);
  }
#if P2PMG_TRACE
  if (l == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2) && !d.batch && d.t == 50)
    printf("DQNTRACE blk %d wave %d agents %d, cycles per agent: layer1 %.0f layer2 %.0f layer3 %.0f "
           "targets+dz2 %.0f backward %.0f barrier waits %.0f\n",
           (int)blockIdx.x, w, n_ag, (double)trp[0] / n_ag, (double)trp[2] / n_ag, (double)trp[3] / n_ag,
           (double)trp[4] / n_ag, (double)trp[5] / n_ag, (double)trp[1] / n_ag);
#endif

  gb1 = sum_groups(gb1);
  float g1t[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) g1t[k] = sum_groups(gx1[k]);
  // lane (g4, r) owns dW1 row 4 g4 + r (< 5): g4 = 0 rows 0..3, g4 = 1 row 4
  auto dw1 = [&](int r) { return g4 == 0 ? g1t[r] : g1t[4]; };
#pragma unroll
  for (int r = 0; r < 4; ++r) {  // over the 16 data-row lanes of each row group
    gb2[r] = sum16(gb2[r]);
    gW3[r] = sum16(gW3[r]);
  }
  const int net_out = net;
  if constexpr (!SHARED) {
    // Trainer._train epilogue: clip the first kernel's gradient, Adam, then update_targets
    float* th = d.theta + (size_t)net_out * kNetStride;
    float* tg = d.target + (size_t)net_out * kNetStride;
    float* mm = d.adam_m + (size_t)net_out * kNetStride;
    float* vv = d.adam_v + (size_t)net_out * kNetStride;
    // each DQNAgent has its own Adam (agent.py:310): its own iteration count, so its own step size
    const float lr = d.lr_net ? d.lr_net[net_out] : d.lr_t;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) adam_update(d, th, tg, mm, vv, kOffW2 + (16 * mt + 4 * g4 + r) * kH + col, gW2[mt][r], lr);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = 4 * g4 + r;
      if (k < 5) adam_update(d, th, tg, mm, vv, kOffW1 + k * kH + col, fminf(fmaxf(dw1(r), -d.clip), d.clip), lr);
    }
    if (g4 == 0) adam_update(d, th, tg, mm, vv, kOffB1 + col, gb1, lr);
    if (c16 == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        adam_update(d, th, tg, mm, vv, kOffB2 + h0 + r, gb2[r], lr);
        adam_update(d, th, tg, mm, vv, kOffW3 + h0 + r, gW3[r], lr);
      }
    }
    if (threadIdx.x == 0) adam_update(d, th, tg, mm, vv, kOffB3, gb3, lr);
  } else {
    float* gp = d.grad + (size_t)blockIdx.x * kNetStride;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) gp[kOffW2 + (16 * mt + 4 * g4 + r) * kH + col] = gW2[mt][r];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g4 + r < 5) gp[kOffW1 + (4 * g4 + r) * kH + col] = dw1(r);
    if (g4 == 0) gp[kOffB1 + col] = gb1;
    if (c16 == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gp[kOffB2 + h0 + r] = gb2[r];
        gp[kOffW3 + h0 + r] = gW3[r];
      }
    }
    if (threadIdx.x == 0) gp[kOffB3] = gb3;
  }
}

// shared network: each gradient segment's sum of its train workgroups' partials (blockIdx.y = the
// local segment).  A 1024-thread workgroup owns 64 parameters; its 16 waves each fold a contiguous
// run of the segment's partials in partial order (8 loads in flight), and wave 0 adds the 16 runs
// in run order: a fixed order that depends only on the segment's block count, so a segment gives the
// same sum on any rank and in any launch.  adam != 0 (one segment over every rank): the Adam step
// on that sum in the same launch; else the sum goes to segs[seg_first + segment] for the gather.
constexpr int kRedParams = 64, kRedSlices = 16, kRedBatch = 48;
__global__ __launch_bounds__(kRedParams * kRedSlices) void dqn_reduce_adam_kernel(const DqnParams d, int adam) {
  __shared__ float part[kRedSlices][kRedParams];
  const int j = threadIdx.x % kRedParams, sl = threadIdx.x / kRedParams;
  const int k = blockIdx.x * kRedParams + j;
  const int n_partials = d.bps;
  const int per = (n_partials + kRedSlices - 1) / kRedSlices;
  const int b0 = sl * per, b1 = min(n_partials, b0 + per);
  // the Adam state of this parameter, loaded ahead of the partials (one memory round trip less)
  float m0 = 0.0f, v0 = 0.0f, w0 = 0.0f, tg0 = 0.0f;
  if (sl == 0 && adam && k < kDqnParams) {
    m0 = d.adam_m[k];
    v0 = d.adam_v[k];
    w0 = d.theta[k];
    tg0 = d.target[k];
  }
  float s = 0.0f;
  if (k < kDqnParams) {
    const float* g = d.grad + (size_t)blockIdx.y * n_partials * kNetStride + k;
    int b = b0;
    if (per <= kRedBatch) {
      // every load of the run in flight at once (one memory round trip instead of per / 8); the
      // zero padding is an exact no-op (s starts at +0 and a float sum of +0 and s is s, never -0)
      float v[kRedBatch];
#pragma unroll
      for (int u = 0; u < kRedBatch; ++u) v[u] = b + u < b1 ? g[(size_t)(b + u) * kNetStride] : 0.0f;
#pragma unroll
      for (int u = 0; u < kRedBatch; ++u) s += v[u];
      b = b1;
    }
    for (; b + 8 <= b1; b += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = g[(size_t)(b + u) * kNetStride];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += g[(size_t)b * kNetStride];
  }
  part[sl][j] = s;
  __syncthreads();
  if (sl != 0 || k >= kDqnParams) return;
  float t = part[0][j];
#pragma unroll
  for (int r = 1; r < kRedSlices; ++r) t += part[r][j];
  if (!adam) {
    d.segs[(size_t)(d.seg_first + blockIdx.y) * kNetStride + k] = t;
    return;
  }
  float gk = t * d.inv_agents;
  if (k < kOffB1) gk = fminf(fmaxf(gk, -d.clip), d.clip);
  // adam_update's arithmetic on the preloaded state
  m0 = m0 + (gk - m0) * d.b1c;
  v0 = v0 + (gk * gk - v0) * d.b2c;
  w0 = w0 - (m0 * d.lr_t) / (sqrtf(v0) + d.adam_eps);
  d.adam_m[k] = m0;
  d.adam_v[k] = v0;
  d.theta[k] = w0;
  d.target[k] = d.tau_c * tg0 + d.tau * w0;
}

// The segment fold alone (the multi-segment / multi-rank path): the same 16 runs, summed in the same
// order as dqn_reduce_adam_kernel, with SPT runs per thread, i.e. 16 / SPT waves per 64 parameters
// instead of 16.  A segment of few partials (8 segments of 64 at configs[4]: 4 per run) gives each
// wave a few loads, and the launch's wave count, not its bytes, set its duration.  The zero padding
// is exact, as in dqn_reduce_adam_kernel.
template <int SPT, int BATCH>
__global__ __launch_bounds__(kRedParams * kRedSlices / SPT) void dqn_fold_kernel(const DqnParams d) {
  __shared__ float part[kRedSlices][kRedParams];
  const int j = threadIdx.x % kRedParams, grp = threadIdx.x / kRedParams;
  const int k = blockIdx.x * kRedParams + j;
  const int n = d.bps, per = (n + kRedSlices - 1) / kRedSlices;
  if (k < kDqnParams) {
    const float* g = d.grad + (size_t)blockIdx.y * n * kNetStride + k;
    float v[SPT][BATCH];  // the first BATCH partials of each of the thread's runs, in flight together
#pragma unroll
    for (int q = 0; q < SPT; ++q) {
      const int b0 = (grp * SPT + q) * per, b1 = min(n, b0 + per);
#pragma unroll
      for (int u = 0; u < BATCH; ++u) v[q][u] = b0 + u < b1 ? g[(size_t)(b0 + u) * kNetStride] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < SPT; ++q) {
      const int sl = grp * SPT + q, b0 = sl * per, b1 = min(n, b0 + per);
      float s = 0.0f;
#pragma unroll
      for (int u = 0; u < BATCH; ++u) s += v[q][u];
      for (int b = b0 + BATCH; b < b1; ++b) s += g[(size_t)b * kNetStride];
      part[sl][j] = s;
    }
  }
  __syncthreads();
  if (grp != 0 || k >= kDqnParams) return;
  float t = part[0][j];
#pragma unroll
  for (int r = 1; r < kRedSlices; ++r) t += part[r][j];
  d.segs[(size_t)(d.seg_first + blockIdx.y) * kNetStride + k] = t;
}

// shared network over several segments / ranks: the segments' sum in global segment order, the mean
// over every agent of every rank, clip, Adam, soft update (every rank computes the same values)
// Latency, not bandwidth (4609 parameters): the Adam state and every segment's value are loaded
// before the first add (one memory round trip instead of one per segment), then summed in order.
// The *_out arrays may be the inputs (in place: each thread reads and writes its own parameter only).
constexpr int kAdamSegBatch = 16;
__global__ __launch_bounds__(256) void dqn_adam_shared_kernel(const DqnParams d) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= kDqnParams) return;
  if (d.n_segs <= kAdamSegBatch) {
    (void)adam_shared_param<kAdamSegBatch>(d, k, true);
    return;
  }
  const float m0 = d.adam_m[k], v0 = d.adam_v[k], w0 = d.theta[k], tg0 = d.target[k];
  float t = d.segs[k];
  for (int g = 1; g < d.n_segs; ++g) t += d.segs[(size_t)g * kNetStride + k];
  float gk = t * d.inv_agents;
  if (k < kOffB1) gk = fminf(fmaxf(gk, -d.clip), d.clip);
  // adam_shared_param's arithmetic
  const float m = m0 + (gk - m0) * d.b1c;
  const float v = v0 + (gk * gk - v0) * d.b2c;
  const float w = w0 - (m * d.lr_t) / (sqrtf(v) + d.adam_eps);
  d.m_out[k] = m;
  d.v_out[k] = v;
  d.theta_out[k] = w;
  d.target_out[k] = d.tau_c * tg0 + d.tau * w;
}

// QNetwork.call on explicit rows (object API, rl.py:147-148): one thread per row
__global__ void dqn_forward_kernel(const float* __restrict__ th, int n, const float* __restrict__ x,
                                   float* __restrict__ q) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  float xi[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) xi[k] = x[(size_t)r * 5 + k];
  float h1[kH];
#pragma unroll
  for (int j = 0; j < kH; ++j) {
    float z = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) z = fmaf(xi[k], th[kOffW1 + k * kH + j], z);
    h1[j] = relu(z + th[kOffB1 + j]);
  }
  float out = 0.0f;
  for (int j = 0; j < kH; ++j) {
    float z = 0.0f;
#pragma unroll 16
    for (int k = 0; k < kH; ++k) z = fmaf(h1[k], th[kOffW2 + k * kH + j], z);
    out = fmaf(relu(z + th[kOffB2 + j]), th[kOffW3 + j], out);
  }
  q[r] = out + th[kOffB3];
}

}  // namespace

static bool act_shared_mfma(const DqnParams& d) {
  // sizes the MFMA act kernel is built for (its action records pack 8 rounds)
  const bool mfma_n = ((d.e.N >= 1 && d.e.N <= 8) || d.e.N == 16) && d.e.R + 1 <= 8;
  return d.n_nets == 1 && !d.act_wave && mfma_n;
}

bool dqn_act_fuses_adam(const DqnParams& d) { return act_shared_mfma(d) && d.n_segs >= 1 && d.n_segs <= kActAdamSegs; }

hipError_t launch_dqn_act(const DqnParams& d, hipStream_t st) {
  if (d.adam_pending && !dqn_act_fuses_adam(d)) return hipErrorInvalidValue;
  if (act_shared_mfma(d)) {  // one shared network: AGW agents per workgroup on MFMA tiles
    // AGW = 16 agent slots per workgroup (default), or 8 (d.act_agw, P2PMG_ACT_AGW=8: more, shorter
    // workgroups; N <= 8 only) -- the same results bit for bit.  A pending Adam step: AGW = 16.
    switch (d.e.N) {
#define P2PMG_DQN_ACT_SHARED(NN)                                                                                     \
  case NN: {                                                                                                         \
    constexpr int spw = 16 / NN;                                                                                     \
    if (d.adam_pending) {                                                                                            \
      hipLaunchKernelGGL((dqn_act_shared_kernel<NN, 16, true>), dim3((d.e.S + spw - 1) / spw), dim3(256), 0, st, d); \
    } else if (NN <= 8 && d.act_agw == 8) {                                                                          \
      constexpr int agw = NN <= 8 ? 8 : 16, spw8 = agw / NN;                                                         \
      hipLaunchKernelGGL((dqn_act_shared_kernel<NN, agw, false>), dim3((d.e.S + spw8 - 1) / spw8), dim3(256), 0, st, \
                         d);                                                                                         \
    } else {                                                                                                         \
      hipLaunchKernelGGL((dqn_act_shared_kernel<NN, 16, false>), dim3((d.e.S + spw - 1) / spw), dim3(256), 0, st, d); \
    }                                                                                                                \
    break;                                                                                                           \
  }
      P2PMG_DQN_ACT_SHARED(1) P2PMG_DQN_ACT_SHARED(2) P2PMG_DQN_ACT_SHARED(3) P2PMG_DQN_ACT_SHARED(4)
      P2PMG_DQN_ACT_SHARED(5) P2PMG_DQN_ACT_SHARED(6) P2PMG_DQN_ACT_SHARED(7) P2PMG_DQN_ACT_SHARED(8)
      P2PMG_DQN_ACT_SHARED(16)
#undef P2PMG_DQN_ACT_SHARED
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  const dim3 grid(d.e.S), wide(16 * kWave), wide64(dqn_act_waves<64, true>() * kWave);
  switch (d.e.N) {
#define P2PMG_DQN_ACT(NN) \
  case NN: hipLaunchKernelGGL((dqn_act_kernel<NN, false>), grid, dim3(NN * kWave), 0, st, d); break;
    P2PMG_DQN_ACT(1) P2PMG_DQN_ACT(2) P2PMG_DQN_ACT(3) P2PMG_DQN_ACT(4) P2PMG_DQN_ACT(5) P2PMG_DQN_ACT(6)
    P2PMG_DQN_ACT(7) P2PMG_DQN_ACT(8) P2PMG_DQN_ACT(16)
#undef P2PMG_DQN_ACT
    default: {  // every other community size: wave w acts for agents w, w + NW, ...
      const int nc = general_tile_cap(d.e.N);
      if (d.e.N < 1 || d.e.N > kMaxAgents) return hipErrorInvalidValue;
      if (nc == 16) hipLaunchKernelGGL((dqn_act_kernel<16, true>), grid, wide, 0, st, d);
      else if (nc == 32) hipLaunchKernelGGL((dqn_act_kernel<32, true>), grid, wide, 0, st, d);
      else hipLaunchKernelGGL((dqn_act_kernel<64, true>), grid, wide64, 0, st, d);
    }
  }
  return hipGetLastError();
}

int dqn_train_blocks_per_cu() { return P2PMG_TRAIN_OCC; }

hipError_t launch_dqn_train(const DqnParams& d, int blocks, bool shared_partials, hipStream_t st) {
  if (shared_partials)
    hipLaunchKernelGGL(dqn_train_kernel<true>, dim3(blocks), dim3(256), 0, st, d);
  else
    hipLaunchKernelGGL(dqn_train_kernel<false>, dim3(blocks), dim3(256), 0, st, d);
  return hipGetLastError();
}

hipError_t launch_dqn_sample_prepass(const DqnParams& d, uint16_t* out, hipStream_t st) {
  const size_t n = (size_t)d.e.T * (size_t)d.e.A;
  if (n == 0 || d.cap < kB || d.cap > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dqn_sample_prepass_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d, out);
  return hipGetLastError();
}

hipError_t launch_dqn_sample(const DqnParams& d, hipStream_t st) {
  hipLaunchKernelGGL(dqn_sample_kernel, dim3(d.e.A), dim3(kWave), 0, st, d);
  return hipGetLastError();
}

hipError_t launch_dqn_reduce_adam(const DqnParams& d, int segments, bool adam, hipStream_t st) {
  if (segments < 1 || d.bps < 1 || (adam && segments != 1)) return hipErrorInvalidValue;
  const dim3 grid((kDqnParams + kRedParams - 1) / kRedParams, segments);
  // the fold: runs of per = ceil(bps / 16) partials, the first 4 or 8 of each run loaded together.
  // fold_spt 0 (auto): 4 runs per thread while a run fits one 8-load batch; longer runs (one segment
  // per rank at world > 1: 512 partials, runs of 32) keep the reduce kernel's form, whose 1024 threads
  // each have a whole run of up to 48 loads in flight
  const int per = (d.bps + kRedSlices - 1) / kRedSlices;
  const bool b4 = per <= 4;
  const int spt = d.fold_spt ? d.fold_spt : (per <= 8 ? 4 : 1);
#define P2PMG_FOLD(SPT)                                                                                           \
  if (b4) hipLaunchKernelGGL((dqn_fold_kernel<SPT, 4>), grid, dim3(kRedParams * kRedSlices / SPT), 0, st, d);   \
  else hipLaunchKernelGGL((dqn_fold_kernel<SPT, 8>), grid, dim3(kRedParams * kRedSlices / SPT), 0, st, d);
  if (adam || spt == 1) {
    hipLaunchKernelGGL(dqn_reduce_adam_kernel, grid, dim3(kRedParams * kRedSlices), 0, st, d, adam ? 1 : 0);
  } else if (spt == 2) {
    P2PMG_FOLD(2)
  } else if (spt == 8) {
    P2PMG_FOLD(8)
  } else if (spt == 16) {
    P2PMG_FOLD(16)
  } else {
    P2PMG_FOLD(4)
  }
#undef P2PMG_FOLD
  return hipGetLastError();
}

hipError_t launch_dqn_adam_shared(const DqnParams& d, hipStream_t st) {
  const int tpb = d.adam_tpb == 64 || d.adam_tpb == 128 ? d.adam_tpb : 256;
  hipLaunchKernelGGL(dqn_adam_shared_kernel, dim3((kDqnParams + tpb - 1) / tpb), dim3(tpb), 0, st, d);
  return hipGetLastError();
}

hipError_t launch_dqn_forward(const float* theta, int n, const float* x, float* q, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(dqn_forward_kernel, dim3((n + 127) / 128), dim3(128), 0, st, theta, n, x, q);
  return hipGetLastError();
}

}  // namespace p2pmg
