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
#include "p2pmg_internal.h"

namespace p2pmg {
namespace {

constexpr int pow2ceil(int n) { return n <= 1 ? 1 : (n <= 2 ? 2 : (n <= 4 ? 4 : (n <= 8 ? 8 : (n <= 16 ? 16 : (n <= 32 ? 32 : 64))))); }

// ----------------------------------------------------------------- reference primitives
// QActor._get_state_indices rl.py:89-95 (NumPy 2: f32 arithmetic, int() truncation, clamp)
__device__ __forceinline__ int clamp_bin(float v, int K) {
  return v >= (float)(K - 1) ? K - 1 : (v < 1.0f ? 0 : (int)v);
}
__device__ __forceinline__ int idx_time(float x, int K) { return clamp_bin(x * (float)K, K); }
__device__ __forceinline__ int idx_temp(float x, int K) {
  return clamp_bin(((x + 1.0f) / 2.0f) * (float)(K - 2) + 1.0f, K);
}
__device__ __forceinline__ int idx_plain(float x, int K) { return clamp_bin(((x + 1.0f) / 2.0f) * (float)K, K); }

// tf.math.sign on f32
__device__ __forceinline__ float sgn(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

// heating.temperature_simulation heating.py:37-56 (f32 casts of the Python constants)
template <typename P>
__device__ __forceinline__ void rc_update(const P& p, float t_out, float hp, float& tin, float& tm) {
  const float d_in = p.inv_ci * ((p.inv_ri * (tm - tin) + p.inv_rvent * (t_out - tin)) + (p.c_in * hp) * p.cop);
  const float d_m = p.inv_cm * (((p.inv_ri * (tin - tm) + p.inv_re * (t_out - tm)) + p.solar) + (p.c_m * hp) * p.cop);
  tin = tin + (d_in * p.spm) * p.slot;
  tm = tm + (d_m * p.spm) * p.slot;
}

// Philox4x32-10 (Random123), see oracle/philox.py for the block layout
__device__ __forceinline__ void philox4x32_10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                              uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
}
constexpr uint32_t kTagDecision = 0x5EED0001u;
constexpr uint32_t kTagT0 = 0x5EED0002u;

template <typename QT>
struct Row4 {
  QT v[4];
};
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
template <typename QT>
__device__ __forceinline__ QT max3(const Row4<QT>& r) {
  QT b = r.v[0];
  if (r.v[1] > b) b = r.v[1];
  if (r.v[2] > b) b = r.v[2];
  return b;
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

template <int N>
__device__ __forceinline__ void exchange(const float (&row)[N], float (&col)[N], int i, int sl, float* sh) {
  constexpr int G = pow2ceil(N);
  if constexpr (G <= 8) {
#pragma unroll
    for (int k = 0; k < N; ++k) col[k] = (k == i) ? row[k] : 0.0f;
#pragma unroll
    for (int d = 1; d < G; ++d) {
      const int src = i ^ d;  // partner lane in the group; it sends its row[i]
      float v = 0.0f;
#pragma unroll
      for (int k = 0; k < N; ++k) v = (k == src) ? row[k] : v;  // what my partner wants: row[partner ^ d] = row[src]
      const float got = __shfl_xor(v, d, 64);
#pragma unroll
      for (int k = 0; k < N; ++k) col[k] = (k == src) ? got : col[k];
    }
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
  if constexpr (G <= 8) {
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
__device__ __forceinline__ EnvRow load_env(const EpisodeParams& p, int t, int s_env) {
  const float* e = p.env + ((size_t)t * p.n_env + s_env) * kEnvStride;
  const float4 a = *reinterpret_cast<const float4*>(e);
  return EnvRow{a.x, a.y, a.z, a.w, e[4]};
}

// Everything about step t that is known before its negotiation starts.
struct StepIdx {
  float bal;        // (load - pv) / max_in           agent.py:172-176
  int it, iT, ib;   // s indices except p2p          rl.py:89-95
  size_t strip;     // row of (it, iT, ib, 0)
  size_t nrow;      // next-state row (time_{t+1}, same T_in, bal_{t+1}, p2p = 0)  agent.py:293-296
};
__device__ __forceinline__ StepIdx make_step(const EpisodeParams& p, float time_t, float time_n, float2 f_t, float2 f_n,
                                             float tin, float mi, int ip_zero) {
  StepIdx st;
  st.bal = (f_t.x - f_t.y) / mi;
  const float baln = (f_n.x - f_n.y) / mi;
  const float tnorm = (tin - p.setpoint) / p.margin;  // heating.py:118-120
  st.it = idx_time(time_t, p.nt);
  st.iT = idx_temp(tnorm, p.nT);
  st.ib = idx_plain(st.bal, p.nb);
  st.strip = (((size_t)st.it * p.nT + st.iT) * p.nb + st.ib) * p.np;
  const int itn = idx_time(time_n, p.nt);
  const int ibn = idx_plain(baln, p.nb);
  st.nrow = (((size_t)itn * p.nT + st.iT) * p.nb + ibn) * p.np + ip_zero;
  return st;
}

// exploration code for (t, r): 255 = greedy (QActor.select_action rl.py:100-111)
__device__ __forceinline__ int decision_code(const EpisodeParams& p, int t, int r, int a, bool active) {
  if (p.mode != 0 || !active) return 255;
  const int R1 = p.R + 1;
  if (p.rng == 0) return p.codes[((size_t)t * R1 + r) * p.A + a];
  uint32_t c0 = (uint32_t)(t * R1 + r), c1 = (uint32_t)p.episode, c2 = p.agent_offset + (uint32_t)a, c3 = kTagDecision;
  philox4x32_10(c0, c1, c2, c3, p.seed_lo, p.seed_hi);
  const double u = ((double)(c0 >> 5) * 67108864.0 + (double)(c1 >> 6)) / 9007199254740992.0;
  return u < p.eps ? (int)(((uint64_t)c2 * 3ull) >> 32) : 255;
}

// ----------------------------------------------------------------- the episode kernel
// One launch = one episode of T timesteps for every scenario (train_episode / run).
// Latency structure per step (one dependent Q gather per extra round):
//   * env rows and profiles are prefetched two steps ahead;
//   * round 0 always sees P = 0, so its p2p index is the constant ip_zero and its Q row, like
//     the next-state row, is known as soon as the previous step's final action is: both are
//     issued right after that action, before the previous step's market/reward/TD work;
//   * a TD store that hits one of those prefetched rows patches the register copy.
template <int N, typename QT>
__global__ __launch_bounds__(kWave) void episode_kernel(const EpisodeParams p) {
  constexpr int G = pow2ceil(N);
  constexpr int SPW = kWave / G;
  __shared__ float shP[G > 8 ? SPW * N * N : 1];
  __shared__ float shR[G > 8 ? SPW * N : 1];

  const int lane = threadIdx.x;
  const int sl = lane / G;
  const int i = lane % G;
  const int s = blockIdx.x * SPW + sl;
  const bool in_group = i < N;
  const bool active = in_group && (s < p.S);
  const int a = active ? s * N + i : 0;
  const int s_env = p.n_env == 1 ? 0 : (s < p.S ? s : 0);
  const int T = p.T;
  const int R1 = p.R + 1;
  const bool train = p.mode == 0;

  const size_t n_states = (size_t)p.nt * p.nT * p.nb * p.np;
  QT* __restrict__ q = reinterpret_cast<QT*>(p.q) + (size_t)a * n_states * kQPad;
  const float mi = active ? p.max_in[a] : 1.0f;
  float tin = active ? p.t_in[a] : p.setpoint;
  float tm = active ? p.t_m[a] : p.setpoint;
  // round 0 and the next state both have p2p = mean(-0 ... -0) / max_in = 0 (agent.py:203, community.py:161)
  const int ip_zero = idx_plain((0.0f / (float)N) / mi, p.np);

  auto wrap = [T](int t) { return t % T; };  // np.roll(-1) pairing (dataset.py:101)
  auto prof = [&](int t) { return active ? p.prof[(size_t)t * p.A + a] : make_float2(0.0f, 0.0f); };

  EnvRow e0 = load_env(p, 0, s_env);
  EnvRow e1 = load_env(p, wrap(1), s_env);
  float2 f0 = prof(0), f1 = prof(wrap(1));
  StepIdx st = make_step(p, e0.time, e1.time, f0, f1, tin, mi, ip_zero);
  int code0 = decision_code(p, 0, 0, a, active);
  const Row4<QT> zrow{{(QT)0, (QT)0, (QT)0, (QT)0}};
  Row4<QT> row0 = (active && code0 == 255) ? load_row(q + (st.strip + ip_zero) * kQPad) : zrow;
  Row4<QT> rowN = (active && train) ? load_row(q + st.nrow * kQPad) : zrow;
  float ep_sum = 0.0f;

  for (int t = 0; t < T; ++t) {
    // prefetch two steps ahead
    const EnvRow e2 = load_env(p, wrap(t + 2), s_env);
    const float2 f2 = prof(wrap(t + 2));

    float row[N];
    float col[N];
#pragma unroll
    for (int j = 0; j < N; ++j) { row[j] = 0.0f; col[j] = 0.0f; }
    int act = 0, ip = ip_zero;
    float hp = 0.0f;
    Row4<QT> rowR = row0;  // Q row of the final round's state (TD target Q[s, a])

    for (int r = 0; r < R1; ++r) {
      int code;
      if (r == 0) {
        code = code0;
      } else {
        exchange<N>(row, col, i, sl, shP);  // Jacobi: read the previous round's column (community.py:84-86)
        // powers = -P[:, i] with the diagonal zeroed (community.py:76,81); p2p = mean / max_in (agent.py:203)
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < N; ++j) acc = acc + (-((j == i) ? 0.0f : col[j]));
        ip = idx_plain((acc / (float)N) / mi, p.np);
        code = decision_code(p, t, r, a, active);
        // the final round's row is needed for the TD update even when exploring
        if (active && (code == 255 || (train && r == R1 - 1))) rowR = load_row(q + (st.strip + ip) * kQPad);
      }
      act = code == 255 ? argmax3(rowR) : code;  // QAgent._act / take_decision (agent.py:271-289)
      hp = p.hp_levels[act];

      // RLAgent._divide_power agent.py:186-195 on out = bal * max_in + hp (agent.py:210)
      const float out = (st.bal * mi) + hp;
      const float so = sgn(out);
      float f[N];
      float tot = 0.0f;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const float pw = -((j == i || r == 0) ? 0.0f : col[j]);
        f[j] = (so != sgn(pw)) ? pw : 0.0f;
        tot = tot + f[j];
      }
      tot = fabsf(tot);
      if (tot == 0.0f) {
        const float ev = (out * 1.0f) / (float)N;
#pragma unroll
        for (int j = 0; j < N; ++j) row[j] = ev;
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) row[j] = (out * fabsf(f[j])) / tot;
      }
      if (active) {
        const size_t k = ((size_t)t * R1 + r) * p.A + a;
        if (p.record & 32) p.rec_action[k] = (uint8_t)act;
        if (p.record & 64) p.rec_index[k] = st.it | (st.iT << 8) | (st.ib << 16) | (ip << 24);
      }
    }
    if (train && active && R1 == 1 && code0 != 255) rowR = load_row(q + (st.strip + ip) * kQPad);

    // CommunityMicrogrid._step -> HPHeating.step (community.py:184-188, heating.py:138-143):
    // computed now so the next step's rows can be issued before this step's market work
    float tin1 = tin, tm1 = tm;
    rc_update(p, e0.t_out, hp, tin1, tm1);
    StepIdx st1 = st;
    int code1 = 255;
    Row4<QT> row0n = zrow, rowNn = zrow;
    if (t + 1 < T) {
      st1 = make_step(p, e1.time, e2.time, f1, f2, tin1, mi, ip_zero);
      code1 = decision_code(p, t + 1, 0, a, active);
      if (active && code1 == 255) row0n = load_row(q + (st1.strip + ip_zero) * kQPad);
      if (active && train) rowNn = load_row(q + st1.nrow * kQPad);
    }

    // CommunityMicrogrid._assign_powers community.py:45-54 on the final P (diagonal kept)
    exchange<N>(row, col, i, sl, shP);
    float g = 0.0f, pp = 0.0f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float pij = row[j], pji = col[j];
      const float si = sgn(pij);
      const float ex = (si != sgn(pji)) ? si * fminf(fabsf(pij), fabsf(pji)) : 0.0f;
      g = g + (pij - ex);
      pp = pp + ex;
    }
    // CommunityMicrogrid._compute_costs community.py:56-65
    float cost = (g >= 0.0f) ? g * e0.buy : g * e0.inj;
    cost = cost + pp * e0.p2p;
    cost = (cost * p.slot) / p.mph;
    cost = cost * p.kilo;
    // RLAgent.get_reward agent.py:225-232 (pre-update T_in)
    float pen = fmaxf(fmaxf(0.0f, p.lower - tin), fmaxf(0.0f, tin - p.upper));
    pen = pen > 0.0f ? pen + 1.0f : 0.0f;
    const float rw = -(cost + p.penw * pen);

    if (train && active) {
      // QAgent.train agent.py:293-298 -> QActor.train rl.py:119-129
      const size_t srow = st.strip + ip;
      const QT qnew = td_update(rowR.v[act], rw, max3(rowN), p.alpha, p.gamma);
      q[srow * kQPad + act] = qnew;
      // rows issued before this store see the old value: patch the register copies
      if (st1.strip + ip_zero == srow) row0n.v[act] = qnew;
      if (st1.nrow == srow) rowNn.v[act] = qnew;
    }
    if (active) {
      const size_t k = (size_t)t * p.A + a;
      if (p.record & 1) p.rec_reward[k] = rw;
      if (p.record & 2) p.rec_cost[k] = cost;
      if (p.record & 4) p.rec_grid[k] = g;
      if (p.record & 8) p.rec_p2p[k] = pp;
      if (p.record & 16) p.rec_tin[k] = tin;
    }
    // avg_reward = sum_t mean_i r (community.py:179), canonical sequential order
    const float m = group_sum<N>(rw, lane, i, sl, shR);
    ep_sum = ep_sum + m / (float)N;

    tin = tin1;
    tm = tm1;
    e0 = e1;
    e1 = e2;
    f0 = f1;
    f1 = f2;
    st = st1;
    code0 = code1;
    row0 = row0n;
    rowN = rowNn;
  }
  if (active) {
    p.t_in[a] = tin;
    p.t_m[a] = tm;
    if (i == 0) p.ep_reward[s] = ep_sum;
  }
}

template <int N, typename QT>
hipError_t launch_n(const EpisodeParams& p, hipStream_t st) {
  constexpr int SPW = kWave / pow2ceil(N);
  const int blocks = (p.S + SPW - 1) / SPW;
  hipLaunchKernelGGL((episode_kernel<N, QT>), dim3(blocks), dim3(kWave), 0, st, p);
  return hipGetLastError();
}

template <typename QT>
hipError_t launch_q(const EpisodeParams& p, hipStream_t st) {
  switch (p.N) {
    case 1: return launch_n<1, QT>(p, st);
    case 2: return launch_n<2, QT>(p, st);
    case 3: return launch_n<3, QT>(p, st);
    case 4: return launch_n<4, QT>(p, st);
    case 5: return launch_n<5, QT>(p, st);
    case 6: return launch_n<6, QT>(p, st);
    case 7: return launch_n<7, QT>(p, st);
    case 8: return launch_n<8, QT>(p, st);
    case 16: return launch_n<16, QT>(p, st);
    default: return hipErrorInvalidValue;
  }
}

// ----------------------------------------------------------------- small kernels
__global__ void rc_step_kernel(int n, const float* t_out, const float* t_in, const float* t_m, const float* hp,
                               float* t_in_new, float* t_m_new, RcParams rc) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  float a = t_in[k], b = t_m[k];
  rc_update(rc, t_out[k], hp[k], a, b);
  t_in_new[k] = a;
  t_m_new[k] = b;
}

__global__ void state_indices_kernel(int n, const float* obs, int32_t* idx, int nt, int nT, int nb, int np) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float4 o = reinterpret_cast<const float4*>(obs)[k];
  idx[4 * k + 0] = idx_time(o.x, nt);
  idx[4 * k + 1] = idx_temp(o.y, nT);
  idx[4 * k + 2] = idx_plain(o.z, nb);
  idx[4 * k + 3] = idx_plain(o.w, np);
}

__global__ void t0_philox_kernel(int A, float* t_in, float* t_m, uint32_t k0, uint32_t k1, int episode,
                                 uint32_t agent_offset, float setpoint, double sigma) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= A) return;
  uint32_t c0 = 0, c1 = (uint32_t)episode, c2 = agent_offset + (uint32_t)k, c3 = kTagT0;
  philox4x32_10(c0, c1, c2, c3, k0, k1);
  const double u1 = ((double)c0 + 0.5) / 4294967296.0;
  const double u2 = ((double)c1 + 0.5) / 4294967296.0;
  const double rad = sqrt(-2.0 * log(u1));
  const double ang = 6.283185307179586 * u2;
  t_in[k] = (float)((double)setpoint + sigma * (rad * cos(ang)));
  t_m[k] = (float)((double)setpoint + sigma * (rad * sin(ang)));
}

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

__global__ void prof_pack_kernel(int A, int T, const float* load_w, const float* pv_w, float2* prof) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // k = t * A + a
  if (k >= (size_t)A * T) return;
  const int t = (int)(k / A), a = (int)(k % A);
  prof[k] = make_float2(load_w[(size_t)a * T + t], pv_w[(size_t)a * T + t]);
}

inline unsigned grid_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

hipError_t launch_episode(const EpisodeParams& p, int q_dtype, hipStream_t stream) {
  return q_dtype == 0 ? launch_q<double>(p, stream) : launch_q<float>(p, stream);
}

hipError_t launch_rc_step(int n, const float* t_out, const float* t_in, const float* t_m, const float* hp,
                          float* t_in_new, float* t_m_new, RcParams rc, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(rc_step_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, t_out, t_in, t_m, hp, t_in_new,
                     t_m_new, rc);
  return hipGetLastError();
}

hipError_t launch_state_indices(int n, const float* obs, int32_t* idx, int nt, int nT, int nb, int np,
                                hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(state_indices_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, obs, idx, nt, nT, nb, np);
  return hipGetLastError();
}

hipError_t launch_t0_philox(int A, float* t_in, float* t_m, uint32_t seed_lo, uint32_t seed_hi, int episode,
                            uint32_t agent_offset, float setpoint, double sigma, hipStream_t stream) {
  if (A <= 0) return hipSuccess;
  hipLaunchKernelGGL(t0_philox_kernel, dim3(grid_for(A, 256)), dim3(256), 0, stream, A, t_in, t_m, seed_lo, seed_hi,
                     episode, agent_offset, setpoint, sigma);
  return hipGetLastError();
}

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

hipError_t launch_prof_pack(int A, int T, const float* load_w, const float* pv_w, float2* prof, hipStream_t stream) {
  const size_t n = (size_t)A * T;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(prof_pack_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, A, T, load_w, pv_w, prof);
  return hipGetLastError();
}

}  // namespace p2pmg
