// Internal declarations shared by p2pmg_kernels.hip (device code + launchers) and
// p2pmg_runtime.cpp (context, C ABI).  Not part of the public ABI (include/p2pmg.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2pmg {

constexpr int kEnvStride = 8;  // floats per env row: time, t_out, buy, inj, p2p, pad x3
constexpr int kQPad = 4;       // Q row padded to 4 actions: 32-B (f64) / 16-B (f32) aligned rows
constexpr int kWave = 64;      // one wave per workgroup
constexpr int kMaxAgents = 64;  // agents per scenario: one 64-lane wave holds a scenario (general kernel)
// R + 1 rounds: no kernel limit (rounds 8 and above read their codes per round); the bound only keeps
// the per-step code and record arrays ([T][ceil((R+1)/4)][A], [T][R+1][A]) in 32-bit row counts
constexpr int kMaxRounds1 = 4096;
// capacity of the general kernel's LDS-tile form for n agents (16, 32 or 64)
inline constexpr int general_tile_cap(int n) { return n <= 16 ? 16 : (n <= 32 ? 32 : 64); }
constexpr double kDeltaScale = 1099511627776.0;  // 2^40: shared-table TD deltas in int64 fixed point
// shared-table delta replicas: workgroup b accumulates into copy (b % 8), i.e. its own XCD\'s copy
// (blocks are dealt round-robin over the 8 XCDs); the copies are folded before use
constexpr int kDeltaCopies = 8;

// Everything the episode kernel needs, passed by value in the kernarg segment.
struct EpisodeParams {
  int S, N, R, T, A;
  int mode, rng, episode, record;  // rng: 0 = code words buffer, 1 = in-kernel Philox
  int n_env;                 // 1 (shared environment) or S (one per scenario)
  const float* env;          // [T][n_env][kEnvStride] time-major
  const float2* prof;        // [T][A] {load_w, pv_w}
  const uint2* sqp;          // sq16 path: [T][A] {bits(balance), it * 8000 + ib * 20} (sq16_prep_kernel)
  const float* max_in;       // [A]
  float* t_in;               // [A] in/out
  float* t_m;                // [A] in/out
  void* q;                   // [A][n_states][kQPad] f64 | f32
  const uint32_t* codes;     // [T][W][A] code words, W = ceil((R+1)/4), one byte per round (255 = greedy)
  double eps;
  // explore test u < eps of a Philox word w (u = w / 2^32, exact) as an integer compare:
  // eps_all || w < eps_thr (eps_threshold below, set with eps)
  uint32_t eps_thr;
  int eps_all;
  uint32_t seed_lo, seed_hi;
  uint32_t agent_offset;     // global id of local agent 0 (Philox counter)
  float* rec_reward;         // [T][A]
  float* rec_cost;
  float* rec_grid;
  float* rec_p2p;
  float* rec_tin;
  uint8_t* rec_action;       // [T][R+1][A]
  int32_t* rec_index;        // [T][R+1][A]
  float* ep_reward;          // [S]
  // shared policy (config 3): every agent reads one frozen table; TD deltas accumulate in
  // int64 fixed point (2^-40) with device atomics, applied at episode end (p2pmg_apply_q_delta)
  int shared_q;
  long long* qdelta;         // [kDeltaCopies][n_states][kQPad] int64 (one replica per XCD)
  // battery (agent.py:138-153 rule, storage.py:36-76 bookkeeping), f64 like the reference
  int battery;
  double* soc;               // [A] in/out
  const double* bat_cap;     // [A] capacity in J (0 = no battery)
  double bat_min, bat_max, bat_sqrt_eff;
  int bat_safe;              // the battery operands lie in battery_rule_r<false>'s verified domain
  const float4* hp_lv;       // [A] per-agent heat-pump power of actions 0..2 (agent.py:268, heating.py:124)
  void* dummy;               // >= 2 * kWave * 32 B scratch: target of the fast kernel's masked-off stores
  uint32_t* pre_ipc;         // fast path, N = 2: [T][A] round-1 p2p bins for the partner's 3 round-0 actions
  void* rec_pack;            // fast paths: packed records [T][A] x 32 B
  int rec_narrow;            // fast / sq16: only reward + cost requested -> records are [T][A] float2
  int reset_t0;              // fast path: draw T0 for episode + 1 at the end (P2PMG_FLAG_RESET_T0)
  double reset_sigma;
  // fast path, chained launch (p2pmg_run_episodes): `chain` consecutive training episodes
  // (episode + k, k < chain) in one launch, each wave running them back to back; episode k reads
  // its code words at codes + k * codes_stride and writes its episode reward to
  // chain_rewards[k * S + s] (when non-null).  0 or 1: one episode.
  int chain;
  size_t codes_stride;
  float* chain_rewards;
  int nt, nT, nb, np;
  double alpha, gamma;
  float hp_levels[4];
  float setpoint, margin, lower, upper;
  float inv_ci, inv_cm, inv_ri, inv_re, inv_rvent, c_in, c_m, solar, cop, spm, slot;
  float mph, kilo, penw;
};

// ---- DQN variant (rl.py:135-359): QNetwork 5 -> 64 -> 64 -> 1 in Keras weight order
constexpr int kNetStride = 4672;  // floats per network slot (4609 used; 64-float aligned)
constexpr int kOffW1 = 0, kOffB1 = 320, kOffW2 = 384, kOffB2 = 4480, kOffW3 = 4544, kOffB3 = 4608;
constexpr int kDqnParams = 4609;
constexpr int kDqnBatch = 32;     // agent.py:308
constexpr int kTrans = 10;        // floats per transition: s[4], a, r, ns[4]
constexpr uint32_t kTagSample = 0x5EED0100u;  // + j: replay-buffer sample draws (oracle/philox.py)

struct DqnParams {
  EpisodeParams e;           // simulation inputs, state, records and constants (q unused)
  int t;                     // timestep of this launch
  int n_nets;                // A (per-agent networks, the reference) or 1 (shared, config 5)
  float* theta;              // [n_nets][kNetStride] online network
  float* target;             // [n_nets][kNetStride] target network
  float* adam_m;
  float* adam_v;
  float* grad;               // shared: [blocks][kNetStride] train-workgroup partial sums
  float* segs;               // shared: [n_segs][kNetStride] gradient segments of every rank (global order)
  int seg_first;             // global index of this context's first segment
  int n_segs;                // segments over every rank
  int seg_agents;            // agents per segment (a segment is whole scenarios)
  int bps;                   // train workgroups per segment: ceil(seg_agents / apb)
  float* buf;                // [A][cap][kTrans] replay rings
  int32_t* added;            // [A] transitions ever added
  int cap;
  const uint16_t* samples;   // replay mode: [T][A][32] deque indices; null = Philox (Floyd)
  float* smp;                // this step's sampled ring slots, int32 [A][32] (dqn_sample_kernel)
  int fused_sample;          // 1: dqn_act_kernel draws them (training env steps); 0: the sample kernel
  int act_wave;              // shared network: 1 = one wave per agent (dqn_act_kernel) instead of the MFMA act kernel
  int act_agw;               // shared network, MFMA act kernel: agent slots per workgroup (16, or 8 for N <= 8)
  float* rec_loss;           // [T][A] or null
  float* ep_acc;             // [S] running sum_t mean_i r
  float gamma, tau, tau_c, lr_t, b1c, b2c, adam_eps, clip;
  const float* lr_net;       // per-agent networks whose Adam step counts differ: [n_nets] step sizes (else null: lr_t)
  float inv_agents;          // shared: 1 / (agents over all ranks)
  int apb;                   // agents per train workgroup
  const float* batch;        // explicit [32][kTrans] batch (p2pmg_dqn_train_batch) or null
  int net;                   // network of the explicit batch
  float* loss_out;           // explicit batch: [1]
  // shared network over segments / ranks: where the post-exchange Adam step stores the new weights,
  // target and moments (the inputs themselves, or the other half of the runtime's double buffer)
  float *theta_out, *target_out, *m_out, *v_out;
  int adam_pending;          // 1: this act launch first applies the previous env step's gathered Adam step
  int adam_tpb;              // post-exchange Adam launch: threads per workgroup (256 default; 64, 128)
  int fold_spt;              // segment fold: runs per thread (0 auto: 4 for runs <= 8, else 1 = the reduce kernel)
};
hipError_t launch_dqn_act(const DqnParams& p, hipStream_t stream);
hipError_t launch_dqn_sample(const DqnParams& p, hipStream_t stream);
// every env step's Philox replay draws of the episode p describes, as deque indices [T][A][32] u16
// (the replay-mode sample layout), from the episode-start counts d.added
hipError_t launch_dqn_sample_prepass(const DqnParams& p, uint16_t* out, hipStream_t stream);
hipError_t launch_dqn_train(const DqnParams& p, int blocks, bool shared_partials, hipStream_t stream);
int dqn_train_blocks_per_cu();  // train workgroups resident per CU (the build's occupancy target)
// each local segment's sum of its train-workgroup partials -> segs[seg_first + j] (segments = local
// segment count); adam (one segment over every rank): the Adam step on it directly
hipError_t launch_dqn_reduce_adam(const DqnParams& p, int segments, bool adam, hipStream_t stream);
// sum of the n_segs segments in global order, then mean, clip, Adam, soft update
hipError_t launch_dqn_adam_shared(const DqnParams& p, hipStream_t stream);
// segments the act kernel's fused Adam step sums (more take the standalone launch)
constexpr int kActAdamSegs = 8;
// true when launch_dqn_act(p) with p.adam_pending = 1 can apply the pending Adam step itself (the shared
// network's MFMA act kernel, at most kActAdamSegs segments)
bool dqn_act_fuses_adam(const DqnParams& p);
hipError_t launch_dqn_forward(const float* theta, int n, const float* x, float* q, hipStream_t stream);

struct RcParams {
  float inv_ci, inv_cm, inv_ri, inv_re, inv_rvent, c_in, c_m, solar, cop, spm, slot;
};

// tile != 0: the LDS-tile form at any N (else registers for N in {1..8, 16}, tiles for the rest)
hipError_t launch_episode(const EpisodeParams& p, int q_dtype, int tile, hipStream_t stream);
// fast per-agent-table path: step pre-pass ([T][A] {balw, bins}; optionally the Philox code
// words) + episode_fast_kernel (N <= 8, R + 1 <= 4, no battery, no shared table)
// Where one step pre-pass writes: its buffers and the episode its Philox draws are for.
constexpr int kMaxChain = 64;  // episodes per chained launch (their thresholds travel in the kernarg)
struct PrepOut {
  uint2* pre;      // [T][A]
  uint32_t* ipc;   // [T][A] or null (N != 2)
  uint32_t* words; // [T][W][A] or null (no Philox draws); a chain: n_ep such buffers, words_stride apart
  int episode;
  double eps;      // the epsilon its Philox draws are for
  uint32_t eps_thr;  // its integer threshold (eps_threshold)
  int eps_all;
  // a chain of n_ep > 1 episodes (episode + k): episode k's threshold ep_thr[k], all-explore bit k of
  // ep_all (eps / eps_thr / eps_all unused)
  int n_ep;
  size_t words_stride;
  uint32_t ep_thr[kMaxChain];
  uint64_t ep_all;
};
// w / 2^32 < eps  <=>  w < ceil(eps * 2^32) for every 32-bit w (w / 2^32 and eps * 2^32 are exact in
// f64): thr = that ceiling, clamped to [0, 2^32]; all = (thr == 2^32), when every w explores
inline void eps_threshold(double eps, uint32_t& thr, int& all) {
  double c = __builtin_ceil(eps * 4294967296.0);
  if (!(c > 0.0)) c = 0.0;  // eps <= 0 or NaN: never
  all = c >= 4294967296.0 ? 1 : 0;
  thr = all ? 0xFFFFFFFFu : (uint32_t)c;
}
hipError_t launch_step_prepass(const EpisodeParams& p, const PrepOut& o, hipStream_t stream);
// next != null: the launch also runs the step pre-pass of the next episode (episode p.episode + 1,
// same epsilon) into *next, in extra workgroups beside the episode's own
// ev0 / ev1: timing events stamped by the dispatch (hipExtLaunchKernel)
hipError_t launch_episode_fast(const EpisodeParams& p, const uint2* pre, void* recs, int q_dtype, int spw,
                               const PrepOut* next, hipEvent_t ev0, hipEvent_t ev1, hipStream_t stream);
// the per-part launchers behind launch_episode_fast / launch_episode (p2pmg_kernels.hip, P2PMG_PART)
#define P2PMG_DECL_FAST_PART(k)                                                                               \
  hipError_t launch_fast_part##k(const EpisodeParams& p, const uint2* pre, void* recs, int q_dtype, int spw, \
                                 const PrepOut* next, hipEvent_t ev0, hipEvent_t ev1, hipStream_t stream);
P2PMG_DECL_FAST_PART(1)
P2PMG_DECL_FAST_PART(2)
P2PMG_DECL_FAST_PART(3)
P2PMG_DECL_FAST_PART(4)
hipError_t launch_general_part6(const EpisodeParams& p, int q_dtype, hipStream_t stream);
hipError_t launch_general_part7(const EpisodeParams& p, int q_dtype, hipStream_t stream);
hipError_t launch_general_part8(const EpisodeParams& p, int q_dtype, hipStream_t stream);
hipError_t launch_tile_part9(const EpisodeParams& p, int q_dtype, int nc, hipStream_t stream);
hipError_t launch_tile_part10(const EpisodeParams& p, int q_dtype, int nc, hipStream_t stream);
// RuleAgent community run (R = 0): rule_episode_kernel; hp_on [A] hysteresis state in/out
hipError_t launch_rule_episode(const EpisodeParams& p, float* hp_on, hipStream_t stream);
// shared table, N = 16, R <= 1 (configs[2]): episode_sq16_kernel; records packed like the fast path
hipError_t launch_episode_sq16(const EpisodeParams& p, int q_dtype, hipEvent_t ev0, hipEvent_t ev1, hipStream_t stream);
// its per-upload pre-pass: out = p.sqp's contents from p.env, p.prof, p.max_in
hipError_t launch_sq16_prep(const EpisodeParams& p, uint2* out, hipStream_t stream);
constexpr size_t kFastRecBytes = 32;  // one packed record row per agent-step (FastRec)
constexpr int kFastBatMaxR1 = 2;      // episode_fast_kernel's battery variants: R + 1 <= 2
// which: 0..4 reward, cost, grid, p2p, tin ([T][A] f32); 5 action (u8), 6 index (i32) [T][R+1][A]
hipError_t launch_fast_rec_unpack(int T, int R1, int A, uint32_t tb, const void* recs, int narrow, int which, void* out,
                                  hipStream_t stream);
hipError_t launch_apply_delta(void* q, long long* qdelta, size_t n, int q_dtype, hipStream_t stream);
hipError_t launch_fold_delta(long long* qdelta, size_t n, hipStream_t stream);
hipError_t launch_battery_seq(int agents, int steps, const double* bal, double* out_bal, double* soc_hist,
                              double* soc, const double* cap, double smin, double smax, double sqrt_eff,
                              hipStream_t stream);
hipError_t launch_philox_codes(const EpisodeParams& p, uint32_t* words, hipStream_t stream);
hipError_t launch_pack_codes(int T, int R1, int A, const uint8_t* in, uint32_t* words, hipStream_t stream);
hipError_t launch_rc_step(int n, const float* t_out, const float* t_in, const float* t_m, const float* hp,
                          float* t_in_new, float* t_m_new, RcParams rc, hipStream_t stream);
hipError_t launch_state_indices(int n, const float* obs, int32_t* idx, int nt, int nT, int nb, int np,
                                hipStream_t stream);
hipError_t launch_t0_philox(int A, float* t_in, float* t_m, uint32_t seed_lo, uint32_t seed_hi, int episode,
                            uint32_t agent_offset, float setpoint, double sigma, hipStream_t stream);
hipError_t launch_q_pack(int count, size_t n_states, int n_actions, const void* src_ref, void* dst_pad,
                         int q_dtype, int src_dtype, hipStream_t stream);
hipError_t launch_q_unpack(int count, size_t n_states, int n_actions, const void* src_pad, void* dst_ref,
                           int q_dtype, int dst_dtype, hipStream_t stream);
struct QCallParams {
  int n, train, q_dtype;
  const int32_t* agents;
  const float* s_obs;
  const uint8_t* codes;
  const float* rewards;
  const float* ns_obs;
  int32_t* actions;
  double* q_out;
  void* q;
  uint32_t n_states;
  int nt, nT, nb, np;
  double alpha, gamma;
};
hipError_t launch_q_calls(const QCallParams& p, hipStream_t stream);
hipError_t launch_metrics(int S, const float* ep, double* out, hipStream_t stream);
hipError_t launch_table_hash(const void* q, size_t bytes, unsigned long long* out, hipStream_t stream);
hipError_t launch_fdiv_check(int n, const float* a, const float* b, float* out, hipStream_t stream);
hipError_t launch_fdiv64_check(int n, const double* a, const double* b, double* out, hipStream_t stream);
hipError_t launch_prof_pack(int A, int T, const float* load_w, const float* pv_w, float2* prof,
                            hipStream_t stream);

}  // namespace p2pmg
