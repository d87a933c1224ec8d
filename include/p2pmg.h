/*
 * p2pmg.h — C ABI of libp2pmg.so, the MI355X (gfx950) batched simulator/trainer for the
 * P2PMicrogrid hot path: per-timestep community rollout + tabular Q-learning update,
 * vectorised over S independent community scenarios x N agents.
 *
 * Reference interfaces replaced (paths relative to /root/reference/microgrid):
 *   p2pmg_run_episode(TRAIN)   CommunityMicrogrid.train_episode          community.py:149-182
 *                              (+ _run :67-93, _assign_powers :45-54, _compute_costs :56-65,
 *                               RLAgent.__call__/_divide_power/get_reward agent.py:172-232,
 *                               QAgent._act/train agent.py:271-298, QActor rl.py:89-129,
 *                               HPHeating.step / temperature_simulation heating.py:37-56,138-143)
 *   p2pmg_run_episode(GREEDY)  CommunityMicrogrid.run                    community.py:95-123
 *                              (QAgent.take_decision agent.py:277-289, QActor.greedy_action rl.py:113-117)
 *   p2pmg_set_env              env.setup(dataset) / GridAgent prices     environment.py:26-45, agent.py:59-67
 *   p2pmg_set_profiles         agent load / Prosumer PV streams          agent.py:78-79,100-103, production.py:23-41
 *   p2pmg_set_agent_params     get_community max_in                      community.py:216-227
 *   p2pmg_set_temperatures     HPHeating.__init__/reset T0               heating.py:101-104,145-152
 *   p2pmg_get_q / p2pmg_set_q  QActor.q_table / set_qtable               rl.py:76-81 (layout (20,20,20,20,3))
 *   p2pmg_rc_step              heating.temperature_simulation (batched)  heating.py:37-56
 *   p2pmg_state_indices        QActor._get_state_indices (batched)       rl.py:89-95
 *   p2pmg_replay_decode        np.random rand()/choice(3) consumption    rl.py:100-111 (legacy MT19937)
 *
 * Conventions: every function returns an int status (P2PMG_OK = 0); no C++ exception crosses
 * the ABI; a per-context error string is available from p2pmg_last_error().  A context owns
 * one device, one HIP stream and every device buffer; host pointers are borrowed for the
 * duration of the call only (copied in/out).  Calls are stream-ordered; p2pmg_sync() (or any
 * p2pmg_get_*) completes outstanding work before host reads.  A context is not thread-safe:
 * use one process per GPU for multi-GPU (scenarios are sharded across ranks).
 */
#ifndef P2PMG_H
#define P2PMG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define P2PMG_ABI_VERSION 8  /* 3: p2pmg_episode_args.next_epsilon; 4: P2PMG_FLAG_NEXT_EPSILON, p2pmg_prepass_stats, per-network Adam steps; 5: p2pmg_collective_ms; 6: DQN gradient segments, p2pmg_dqn_set_exchange, p2pmg_dqn_grad_layout; 7: p2pmg_run_episodes, p2pmg_get_episode_rewards; 8: N up to 64 and any R, P2PMG_FLAG_TILE_KERNEL */

typedef struct p2pmg_ctx p2pmg_ctx;

/* status codes */
#define P2PMG_OK 0
#define P2PMG_E_INVALID 1     /* bad argument / shape */
#define P2PMG_E_HIP 2         /* HIP runtime error (message in p2pmg_last_error) */
#define P2PMG_E_NOMEM 3       /* device allocation failed */
#define P2PMG_E_STATE 4       /* missing prerequisite (e.g. profiles not set) */
#define P2PMG_E_UNSUPPORTED 5 /* configuration not supported (e.g. N > 64) */

/* Q-table element type: f64 = the reference's np.zeros table (rl.py:73), bit-exact;
 * f32 = throughput mode (TD update in f32, held to 1e-5 relative). */
#define P2PMG_Q_F64 0
#define P2PMG_Q_F32 1

#define P2PMG_MODE_TRAIN 0  /* train_episode: epsilon-greedy + TD update */
#define P2PMG_MODE_GREEDY 1 /* run(): greedy actions, no update, no RNG */
#define P2PMG_MODE_FILL 2   /* DQN init_buffers (community.py:125-147): act + store memory, no training */

#define P2PMG_RNG_REPLAY 0 /* exploration codes supplied by the host (reference stream) */
#define P2PMG_RNG_PHILOX 1 /* counter-keyed Philox4x32-10 on (seed, episode, agent, t, round): one 32-bit
                              word per round, explore if w / 2^32 < epsilon, action w % 3 (round-4
                              layout, oracle/philox.py::decision_draws) */

/* per-step records (bit mask for p2pmg_episode_args.record and p2pmg_get_record) */
#define P2PMG_REC_REWARD 1   /* f32 [T][A] reward (agent.py:225-232) */
#define P2PMG_REC_COST 2     /* f32 [T][A] cost   (community.py:56-65) */
#define P2PMG_REC_GRID 4     /* f32 [T][A] p_grid (community.py:51) */
#define P2PMG_REC_P2P 8      /* f32 [T][A] p_p2p  (community.py:52) */
#define P2PMG_REC_TEMP 16    /* f32 [T][A] T_in before the step's RC update (heating.py:139) */
#define P2PMG_REC_ACTION 32  /* u8  [T][R+1][A] action index (decisions, community.py:88-89) */
#define P2PMG_REC_INDEX 64   /* i32 [T][R+1][A] packed state index it | iT<<8 | ib<<16 | ip<<24 */
#define P2PMG_REC_LOSS 128   /* f32 [T][A] DQN loss of the agent's train step (rl.py:331) */

#define P2PMG_GREEDY 255 /* replay code: no exploration in this (t, round, agent) */

typedef struct p2pmg_config {
  int32_t n_scenarios;      /* S */
  int32_t n_agents;         /* N agents per scenario, 1..64 (a scenario is one 64-lane wave) */
  int32_t rounds;           /* R >= 0: negotiation runs R+1 rounds (community.py:75); R + 1 <= 4096 */
  int32_t horizon;          /* T timesteps per episode */
  int32_t q_dtype;          /* P2PMG_Q_F64 | P2PMG_Q_F32 */
  int32_t n_time_states;    /* 20 (agent.py:258-261) */
  int32_t n_temp_states;    /* 20 */
  int32_t n_balance_states; /* 20 */
  int32_t n_p2p_states;     /* 20 */
  int32_t n_actions;        /* 3 (<= 4) */
  double alpha;             /* 1e-5 (rl.py:60) */
  double gamma;             /* 0.9  (rl.py:59) */
  float hp_levels[4];       /* f32(level * max_power) = {0, 1500, 3000} W (agent.py:268, heating.py:124) */
  float setpoint;           /* 21 (community.py:226) */
  float temp_margin;        /* 1  (heating.py:90) */
  float lower_bound;        /* 20 (heating.py:93) */
  float upper_bound;        /* 22 */
  /* RC model, f32 casts of the Python doubles (heating.py:23-56) */
  float inv_ci, inv_cm, inv_ri, inv_re, inv_rvent;
  float one_minus_frad; /* f32(1 - f_rad) */
  float frad;           /* f32(f_rad) */
  float solar_gain;     /* f32(gA * solar_rad) = 0 */
  float hp_cop;         /* f32(3.0) */
  float seconds_per_minute; /* 60 */
  float time_slot;          /* 15 */
  /* costs (community.py:63) and reward (agent.py:230) */
  float minutes_per_hour; /* 60 */
  float kilo;             /* f32(1e-3) */
  float penalty_weight;   /* 10 */
  uint64_t seed;          /* Philox key */
  int64_t scenario_offset; /* global index of this context's scenario 0 (multi-GPU sharding):
                              Philox counters use global agent ids so results do not depend
                              on how scenarios are split over ranks */
  int32_t shared_q;        /* 0: one table per agent (the reference, rl.py:73);
                              1: one shared policy table for every agent of every scenario
                              (config 3, build-defined): frozen during an episode, TD deltas summed
                              in int64 fixed point (2^-40) and applied by p2pmg_apply_q_delta;
                              with learner = DQN: one shared Q-network (config 5, data-parallel) */
  int32_t learner;         /* P2PMG_LEARNER_TABULAR (QAgent) | P2PMG_LEARNER_DQN (DQNAgent) */
} p2pmg_config;

#define P2PMG_LEARNER_TABULAR 0
#define P2PMG_LEARNER_DQN 1

typedef struct p2pmg_episode_args {
  int32_t mode;     /* P2PMG_MODE_TRAIN | P2PMG_MODE_GREEDY */
  int32_t rng;      /* P2PMG_RNG_REPLAY | P2PMG_RNG_PHILOX (TRAIN only) */
  int32_t episode;  /* episode index (Philox counter) */
  int32_t record;   /* P2PMG_REC_* mask */
  double epsilon;   /* exploration rate shared by every agent (QActor._epsilon) */
  int32_t flags;    /* P2PMG_FLAG_* (0 = automatic choice) */
  int32_t scen_per_wave; /* fast kernel: scenarios per 64-lane wave (0 = automatic: 64 / pow2ceil(N)) */
  double reset_sigma;    /* with P2PMG_FLAG_RESET_T0: sigma of the T0 draw */
  double next_epsilon;   /* TRAIN + Philox, fast kernel: epsilon of the NEXT episode, for the
                            speculative pre-pass this launch writes (see P2PMG_FLAG_NEXT_EPSILON;
                            without the flag <= 0 means the same epsilon).  A wrong guess only
                            costs a pre-pass launch next time, never results
                            (p2pmg_prepass_stats counts hits and misses). */
} p2pmg_episode_args;

/* Philox placement: a parallel pre-pass writing per-step code words (latency-bound batches:
 * the episode loop only loads a prefetched word) or inline in the episode kernel (bandwidth-
 * bound batches: no extra HBM traffic).  Automatic: pre-pass below 2^18 agents.  Same stream. */
#define P2PMG_FLAG_PHILOX_PREPASS 1
#define P2PMG_FLAG_PHILOX_INKERNEL 2
/* Kernel choice.  Automatic: the fast per-agent-table kernel (step pre-pass + rounds unrolled at
 * compile time) whenever it applies (N <= 8, R + 1 <= 4, no battery, no shared table, in-range
 * max_in); GENERAL forces the general episode kernel (same results, bit for bit). */
#define P2PMG_FLAG_GENERAL_KERNEL 4
/* End the episode with HPHeating.reset (community.py:181 -> heating.py:145-152): T0 for episode + 1
 * drawn as p2pmg_reset_temperatures_philox(ctx, episode + 1, reset_sigma) would, fused into the
 * episode (no extra launch). */
#define P2PMG_FLAG_RESET_T0 8
/* next_epsilon holds the caller's guess as given, 0.0 included (DQN-style schedules decay to 0).
 * Without this flag only a positive next_epsilon is a guess; anything else means "same epsilon". */
#define P2PMG_FLAG_NEXT_EPSILON 16
/* The general kernel's LDS-tile form (the scenario's P in two LDS tiles, any N <= 64; the form every
 * N outside {1..8, 16} runs) at any N: the cross-check of the register form, same results bit for bit. */
#define P2PMG_FLAG_TILE_KERNEL 32

/* version / defaults */
int p2pmg_abi_version(void);
int p2pmg_device_count(int* count); /* visible HIP devices (0 on a host without GPUs) */
int p2pmg_config_default(p2pmg_config* cfg); /* the reference constants, S = 1, N = 2, R = 1, T = 96 */

/* lifetime */
int p2pmg_create(const p2pmg_config* cfg, int device, p2pmg_ctx** out);
int p2pmg_destroy(p2pmg_ctx* ctx);
const char* p2pmg_last_error(const p2pmg_ctx* ctx);
int p2pmg_sync(p2pmg_ctx* ctx);
int p2pmg_device_info(p2pmg_ctx* ctx, char* name, size_t name_len, size_t* total_mem);
/* which kernel the last episode launch ran, e.g. "episode_fast_kernel<2,f64,R1=2,train>" */
const char* p2pmg_last_kernel(const p2pmg_ctx* ctx);

/* inputs (host arrays, copied to HBM) */
int p2pmg_set_env(p2pmg_ctx* ctx, int n_env, const float* time, const float* t_out,
                  const float* price_buy, const float* price_inj, const float* price_p2p);
                  /* each [n_env][T], n_env in {1, S} */
int p2pmg_set_profiles(p2pmg_ctx* ctx, const float* load_w, const float* pv_w); /* [A][T], A = S*N */
int p2pmg_set_agent_params(p2pmg_ctx* ctx, const float* max_in);              /* [A] */
int p2pmg_set_temperatures(p2pmg_ctx* ctx, const float* t_in, const float* t_m); /* [A] */
int p2pmg_get_temperatures(p2pmg_ctx* ctx, float* t_in, float* t_m);
int p2pmg_reset_temperatures_philox(p2pmg_ctx* ctx, int episode, double sigma); /* T0 ~ N(setpoint, sigma) */
int p2pmg_set_replay_codes(p2pmg_ctx* ctx, const uint8_t* codes);            /* [T][R+1][A] */

/* Q-tables in the reference layout (n_time, n_temp, n_bal, n_p2p, n_actions) per agent */
int p2pmg_zero_q(p2pmg_ctx* ctx);
int p2pmg_set_q(p2pmg_ctx* ctx, int first_agent, int count, const void* host, int host_dtype);
int p2pmg_get_q(p2pmg_ctx* ctx, int first_agent, int count, void* host, int host_dtype);

/* the hot path */
int p2pmg_run_episode(p2pmg_ctx* ctx, const p2pmg_episode_args* args);
/* n consecutive episodes: the loop body of CommunityMicrogrid's training loop (community.py:279-286,
 * train_episode x n), episode args->episode + k at epsilons[k], every other field of args as in
 * p2pmg_run_episode.  Training with Philox draws, where the fast kernel applies, runs as chained
 * launches (up to 64 episodes per launch, every wave running its episodes back to back); anything
 * else as n launches.  Results, tables, T0 resets and the records left behind (the last episode's)
 * are those of the n p2pmg_run_episode calls, bit for bit.  next_n / next_epsilons: the caller's
 * guess of the NEXT call's epsilons for the speculative pre-pass (as next_epsilon; next_n = 0: the
 * same as this call's last).  p2pmg_get_episode_reward returns the last episode's reward. */
int p2pmg_run_episodes(p2pmg_ctx* ctx, const p2pmg_episode_args* args, int n, const double* epsilons, int next_n,
                       const double* next_epsilons);
/* [n][S] episode rewards (community.py:179) of the first n episodes of the last p2pmg_run_episodes call */
int p2pmg_get_episode_rewards(p2pmg_ctx* ctx, int n, float* host);
/* one P2PMG_REC_* bit of the LAST episode launch; P2PMG_E_STATE if that launch did not record it */
int p2pmg_get_record(p2pmg_ctx* ctx, int which, void* host);
/* fast path: episode launches whose step pre-pass the previous launch had already produced (hits)
 * and launches that had to run it themselves (misses), since the context was created */
int p2pmg_prepass_stats(p2pmg_ctx* ctx, int64_t* hits, int64_t* misses);
/* RuleAgent community run (get_rule_based_community community.py:237-238 -> run() community.py:95-123,
 * RuleAgent agent.py:106-136): hysteresis heat pump at the heat pump's max power (level 2 of
 * p2pmg_set_hp_levels), no policy, R = 0.  Records: COST, GRID, P2P, TEMP, ACTION (0 off / 2 on). */
int p2pmg_run_rule_episode(p2pmg_ctx* ctx, int record);
/* HeatPump.power of each RuleAgent (0 or 1; persists across runs like the reference's): [A] */
int p2pmg_set_hp_state(p2pmg_ctx* ctx, const float* on);
int p2pmg_get_hp_state(p2pmg_ctx* ctx, float* on);
int p2pmg_get_episode_reward(p2pmg_ctx* ctx, float* host);     /* [S]: sum_t mean_i r (community.py:179) */
int p2pmg_last_kernel_ms(p2pmg_ctx* ctx, float* ms);           /* HIP-event time of the last episode kernel */
/* HIP-event durations (ms) of the episode kernels launched since the last reset, oldest first
 * (ring of the last 4096 launches, on the context's stream); *count = entries written. */
int p2pmg_kernel_times(p2pmg_ctx* ctx, float* ms, int max, int* count);
int p2pmg_reset_kernel_times(p2pmg_ctx* ctx);
/* Sum of the HIP-event durations (ms) of the data-path collectives (shared-table delta
 * all-reduce, DQN gradient-segment all-gather; not the episode metrics) enqueued since
 * p2pmg_reset_kernel_times; *count = collectives summed (all of them: older ring slots are folded
 * into a running total before reuse).  No reference counterpart (the reference is one process);
 * the multi-GPU bench line reports it. */
int p2pmg_collective_ms(p2pmg_ctx* ctx, double* total_ms, int* count);
/* Stamp the episode kernel's timing events on every period-th episode launch only (default 1 =
 * every launch; the counter restarts here and at p2pmg_reset_kernel_times, so the next launch is
 * timed).  Timing-only: results do not depend on it. */
int p2pmg_set_timing_period(p2pmg_ctx* ctx, int period);

/* batched primitives (device) for unit parity against the reference functions */
int p2pmg_rc_step(p2pmg_ctx* ctx, int n, const float* t_out, const float* t_in, const float* t_m,
                  const float* hp, float* t_in_new, float* t_m_new);
int p2pmg_state_indices(p2pmg_ctx* ctx, int n, const float* obs /* [n][4] */, int32_t* idx /* [n][4] */);
/* The kernels' fast divisions next to the IEEE operator, for the division fuzz test (the quotients
 * the reference takes in agent.py:175,193,203, community.py:63 and storage.py:58,61,64).
 * f32: out [n][4] = {fdiv_b, the divide-power form, the packed sq16 form, IEEE a / b};
 * f64: out [n][3] = {fdiv64, qcore64 under the battery rule's guard, IEEE a / b}. */
int p2pmg_fdiv_check(p2pmg_ctx* ctx, int n, const float* a, const float* b, float* out);
int p2pmg_fdiv64_check(p2pmg_ctx* ctx, int n, const double* a, const double* b, double* out);

/* heterogeneous agents and storage (configs 3-4) */
int p2pmg_set_hp_levels(p2pmg_ctx* ctx, const float* levels /* [A][3] W per action */);
/* Battery per agent (storage.py:36-76, rule agent.py:138-153, f64): capacity [A] in J (0 = none;
 * NULL disables storage), SoC bounds, round-trip efficiency, initial SoC [A] (NULL = 0.5). */
int p2pmg_set_battery(p2pmg_ctx* ctx, const double* capacity, double min_soc, double max_soc,
                      double efficiency, const double* soc0);
int p2pmg_get_soc(p2pmg_ctx* ctx, double* soc);
int p2pmg_battery_seq(p2pmg_ctx* ctx, int agents, int steps, const double* balance /* [agents][steps] */,
                      double* out_balance, double* soc_hist, double* soc /* [agents] in/out */,
                      const double* capacity, double min_soc, double max_soc, double efficiency);

/* shared policy table (config.shared_q = 1) */
int p2pmg_apply_q_delta(p2pmg_ctx* ctx);            /* Q += delta * 2^-40; delta = 0 */
int p2pmg_get_q_delta(p2pmg_ctx* ctx, int64_t* host); /* [n_states][n_actions] fixed point */
int p2pmg_set_q_delta(p2pmg_ctx* ctx, const int64_t* host); /* e.g. after a host-side (gloo) sum */

/* multi-GPU exchange of the shared-table deltas over RCCL (xGMI), loaded at run time */
int p2pmg_comm_unique_id(uint8_t id[128]);
int p2pmg_comm_init(p2pmg_ctx* ctx, const uint8_t id[128], int rank, int nranks);
int p2pmg_allreduce_q_delta(p2pmg_ctx* ctx);        /* int64 sum over ranks, in place, on the stream */
int p2pmg_comm_destroy(p2pmg_ctx* ctx);
/* ranks of the context's communicator (ncclCommCount; 1 without one) */
int p2pmg_comm_nranks(p2pmg_ctx* ctx, int* nranks);
/* episode metrics of the last episode over every rank: out = {sum over scenarios of the episode
 * reward (community.py:179), number of scenarios}; the local sum in f64 on the device, then an
 * RCCL all-reduce (sum) when a communicator exists.  Synchronises. */
int p2pmg_allreduce_metrics(p2pmg_ctx* ctx, double* out /* [2] */);
/* 64-bit fingerprint of the context's Q-table bits, all-gathered over the communicator:
 * out[nranks] in rank order (out[0] alone without one); replicas of a shared table agree. */
int p2pmg_table_hash_allgather(p2pmg_ctx* ctx, uint64_t* out);

/* Standalone QActor calls (rl.py:89-129) on the context's per-agent tables, applied IN ORDER
 * by one device thread: for entry k, s = indices(s_obs[k]); a = codes[k] == P2PMG_GREEDY ?
 * argmax Q[agent[k], s] (first max) : codes[k]; q_out[k] = greedy ? Q[s, a] : 0 (select_action /
 * greedy_action); if train, Q[s, a] += alpha * ((reward[k] + gamma * max Q[ns]) - Q[s, a])
 * (QActor.train).  ns_obs/rewards may be NULL when train == 0. */
int p2pmg_q_calls(p2pmg_ctx* ctx, int n, const int32_t* agents, const float* s_obs /* [n][4] */,
                  const uint8_t* codes, const float* rewards, const float* ns_obs /* [n][4] */,
                  int train, int32_t* actions_out, double* q_out);

/* host-only: decode a block of legacy-MT19937 32-bit words into replay codes, consuming words
 * exactly as rand() (2 words) and choice(3) (masked rejection, 1 word per try) do.
 * eps for decision k is eps[k % n_eps].  Returns P2PMG_E_INVALID if the words run out. */
int p2pmg_replay_decode(const uint32_t* words, size_t n_words, size_t n_decisions,
                        const double* eps, size_t n_eps, uint8_t* codes, size_t* consumed);

/* ---- DQN variant (rl.py:135-359, agent.py:301-350; BASELINE.json configs[4]) -------------
 * create with config.learner = P2PMG_LEARNER_DQN (no Q-table is allocated), then
 * p2pmg_dqn_setup.  Per agent (or ONE network with config.shared_q = 1): online and target
 * QNetwork 5->64->64->1 (Keras weight order, P2PMG_DQN_PARAMS floats), Adam state and a replay
 * ring of `capacity` transitions (s[4], a, r, ns[4]).  p2pmg_run_episode dispatches to the DQN
 * step pipeline: per timestep an act kernel (negotiation rounds with the Q-MLP, market, memory)
 * then, in TRAIN mode, the train kernel (sample 32, target/online forward + backward on f32
 * MFMA, clip, Adam, soft update). */
#define P2PMG_DQN_PARAMS 4609
#define P2PMG_DQN_ONLINE 0
#define P2PMG_DQN_TARGET 1
#define P2PMG_DQN_ADAM_M 2
#define P2PMG_DQN_ADAM_V 3

typedef struct p2pmg_dqn_config {
  double gamma;    /* 0.95 agent.py:309 */
  double tau;      /* 0.005 soft update agent.py:309 */
  double lr;       /* 1e-5 Adam agent.py:310 */
  double beta1, beta2, adam_eps; /* Keras Adam defaults .9, .999, 1e-7 */
  double clip;     /* 1.0: first kernel's gradient clipped to [-clip, clip] (rl.py:329) */
  int32_t batch;   /* 32 (agent.py:308); the only supported value */
  int32_t capacity; /* 5000 (agent.py:308) */
  int32_t agents_per_block; /* shared network: agents whose gradients one workgroup sums (0 = auto:
                               ceil(A / (CUs x workgroups per CU)), i.e. device- and shard-dependent) */
  int32_t grad_segments;    /* shared network: the context's agents split into this many contiguous
                               gradient segments of whole scenarios (0 = 1).  The gradient of an env
                               step is sum over segments (in global segment order) of the segment's
                               sum over its agents_per_block blocks (16 slices, fixed order): with
                               agents_per_block and the TOTAL segment count fixed, 1 rank x G segments
                               == W ranks x G/W segments bit for bit (rl.py:307-333 averaged over
                               agents, build-defined) */
} p2pmg_dqn_config;

int p2pmg_dqn_config_default(p2pmg_dqn_config* cfg);
int p2pmg_dqn_setup(p2pmg_ctx* ctx, const p2pmg_dqn_config* cfg);
/* which = P2PMG_DQN_*; nets [first, first+count) of [count][P2PMG_DQN_PARAMS] f32 */
int p2pmg_dqn_set_weights(p2pmg_ctx* ctx, int which, int first, int count, const float* host);
int p2pmg_dqn_get_weights(p2pmg_ctx* ctx, int which, int first, int count, float* host);
/* Adam iterations done (Keras `iterations`).  Each network has its own count (one optimizer per
 * DQNAgent, agent.py:310): set_step sets every network's, get_step reads network 0's, an episode's
 * env step advances every network's and p2pmg_dqn_train_batch only the network it trains. */
int p2pmg_dqn_set_step(p2pmg_ctx* ctx, int64_t step);
int p2pmg_dqn_get_step(p2pmg_ctx* ctx, int64_t* step);
int p2pmg_dqn_get_net_steps(p2pmg_ctx* ctx, int first, int count, int64_t* steps);
/* replay mode: deque indices (0 = oldest) of random.sample(buffer, 32) (rl.py:238) [T][A][32] */
int p2pmg_dqn_set_samples(p2pmg_ctx* ctx, const uint16_t* samples);
/* replay memory of agents [first, first+count): [count][capacity][10] f32 ring + added[count] */
int p2pmg_dqn_get_buffer(p2pmg_ctx* ctx, int first, int count, float* host, int32_t* added);
int p2pmg_dqn_set_buffer(p2pmg_ctx* ctx, int first, int count, const float* host, const int32_t* added);
/* QNetwork.call (rl.py:147-148) of one network on n rows x = concat(state, action) [n][5] */
int p2pmg_dqn_forward(p2pmg_ctx* ctx, int net, int n, const float* x, float* q);
/* Trainer._train + update_targets (rl.py:307-359) of one network on a given batch [32][10] */
int p2pmg_dqn_train_batch(p2pmg_ctx* ctx, int net, const float* batch, float* loss);

/* Shared network over several ranks (config 5): the gradient segments of every rank are gathered
 * once per env step, then every rank sums all of them in global segment order and takes the same
 * Adam step, so the replicas stay bit-identical.  With an RCCL communicator (p2pmg_comm_init) the
 * gather is an in-place ncclAllGather on the context's stream (xGMI).  Without one, a host exchange
 * function does it: `segments` is [nranks][floats_per_rank] f32 host memory with this rank's part
 * filled in; the function fills every other rank's part (an all-gather over any transport, e.g.
 * gloo) and returns 0 (non-zero aborts the episode with P2PMG_E_STATE).  It is called
 * synchronously from p2pmg_run_episode, on the calling thread, once per training env step.
 * fn = NULL removes it (rank 0 of 1).  No reference counterpart (one process, rl.py:307-333). */
typedef int (*p2pmg_exchange_fn)(void* user, float* segments, int64_t floats_per_rank, int rank, int nranks);
int p2pmg_dqn_set_exchange(p2pmg_ctx* ctx, p2pmg_exchange_fn fn, void* user, int rank, int nranks);
/* the shared-network gradient layout in use: segments of this context, agents per train
 * workgroup, train workgroups per env step */
int p2pmg_dqn_grad_layout(p2pmg_ctx* ctx, int* segments, int* agents_per_block, int* blocks);

#ifdef __cplusplus
}
#endif
#endif /* P2PMG_H */
