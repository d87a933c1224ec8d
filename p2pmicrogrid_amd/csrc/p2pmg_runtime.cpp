// p2pmg_runtime.cpp — context, device buffers and the extern "C" ABI of libp2pmg.so
// (declared in include/p2pmg.h).  No C++ exception crosses the ABI: every entry point
// returns a status and records a message in the context.
#include "p2pmg.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "p2pmg_internal.h"

using p2pmg::EpisodeParams;
using p2pmg::kEnvStride;
using p2pmg::kQPad;

struct p2pmg_ctx {
  p2pmg_config cfg{};
  int device = 0;
  int S = 0, N = 0, R = 0, T = 0, A = 0;
  int n_cu = 256;  // compute units of the device (multiProcessorCount)
  size_t n_states = 0;
  size_t q_elem = 8;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  static constexpr int kRing = 4096;
  std::vector<hipEvent_t> ring;  // 2 * kRing events: start/stop of each episode kernel
  long long n_timed = 0;          // launches recorded since the last reset
  static constexpr int kCRing = 1024;
  std::vector<hipEvent_t> cring;  // 2 * kCRing events: start/stop of each data-path RCCL all-reduce
  long long n_coll = 0;           // collectives recorded since the last reset
  double coll_folded_ms = 0.0;    // durations of ring slots already reused (p2pmg_collective_ms)
  long long n_coll_folded = 0;    // collectives whose durations are in coll_folded_ms
  int timing_period = 1;          // episode launches: stamp timing events on every k-th one
  long long n_launch = 0;         // episode launches since the last reset
  // device buffers
  float* env = nullptr;
  int n_env = 0;
  float2* prof = nullptr;
  uint2* sqp = nullptr;             // sq16 path: per-upload step words (launch_sq16_prep), lazily allocated
  long long sqp_version = -1;       // inputs_version they were computed for
  float* max_in = nullptr;
  float* t_in = nullptr;
  float* t_m = nullptr;
  void* q = nullptr;
  uint32_t* codes = nullptr;  // code words [T][W][A]
  // fast path: step pre-pass outputs, double-buffered.  Episode e's launch also computes, in extra
  // workgroups, slot (e+1)'s pre-pass for episode e + 1 at the same epsilon (it reads only inputs,
  // never Q or T); run_episode(e + 1) uses it when its arguments match (spec_*), else recomputes.
  uint2* pre[2] = {nullptr, nullptr};        // [T][A] {balw, bins}
  uint32_t* pre_ipc[2] = {nullptr, nullptr}; // N = 2: [T][A] round-1 bins per partner action
  uint32_t* pcodes[2] = {nullptr, nullptr};  // Philox code words [T][W][A], one per episode of a chain
  size_t pcodes_cap[2] = {0, 0};             // ... their capacity in words
  int pslot = 0;
  bool spec_valid[2] = {false, false};
  int spec_episode[2] = {0, 0};
  std::vector<double> spec_chain[2];         // the epsilons of the chain a slot holds (one: {eps})
  float* chain_rew = nullptr;                // p2pmg_run_episodes: [n][S] episode rewards of the last call
  // pinned host staging of the small per-episode read-backs (episode rewards, metrics): a pageable
  // destination takes HIP's staged copy path (~26 us for 16 KB with the device idle)
  void* h_small = nullptr;
  size_t h_small_bytes = 0;
  int chain_rew_cap = 0, chain_n = 0;
  long long spec_version[2] = {-1, -1};
  long long inputs_version = 0;  // bumped by every input upload (env, profiles, max_in, hp levels)
  long long spec_hits = 0, spec_misses = 0;  // fast-path launches whose pre-pass was / was not ready
  bool mi_ok = false;         // every max_in inside the fast division range (fdiv in p2pmg_kernels.hip)
  void* dummy = nullptr;      // fast path: target of masked-off stores (2 * 64 * 32 B)
  void* rec_pack = nullptr;   // fast path: packed records [T][A] x 32 B
  int rec_fast_mask = 0;      // records of the last episode that live (packed) in rec_pack
  int rec_narrow = 0;         // ... as [T][A] float2 {reward, cost} (fast / sq16 with only those two requested)
  int code_src = 0;          // what the code buffer holds: 0 none, 1 replay upload, 2 Philox pre-pass
  float* ep_reward = nullptr;
  float* rec_f32[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // reward, cost, grid, p2p, tin
  uint8_t* rec_action = nullptr;
  int32_t* rec_index = nullptr;
  void* rec_stage = nullptr;  // fast / sq16 launches: one staging buffer the packed rows unpack into
  size_t rec_stage_bytes = 0;
  float4* hp_lv = nullptr;     // [A] per-agent heat-pump levels
  float* hp_on = nullptr;      // [A] RuleAgent heat-pump state (lazily allocated, starts off)
  double* soc = nullptr;       // [A]
  double* bat_cap = nullptr;   // [A]
  bool battery = false;
  // operand domains of the battery rule's range-test-free variant (battery_rule_r<false>):
  bool bat_domain = false;   // capacities, SoC bounds, sqrt(eff) and SoC0 in range (set_battery)
  bool prof_bounded = false; // every |load|, |pv| <= 2^100 and finite (set_profiles)
  bool hp_bounded = true;    // every heat-pump level |x| <= 2^100 and finite (defaults: 0 .. 3 kW)
  double bat_min = 0.1, bat_max = 0.9, bat_sqrt_eff = 1.0;
  long long* qdelta = nullptr; // shared table deltas [kDeltaCopies][n_states][4]
  void* comm = nullptr;        // ncclComm_t
  int rank = 0, nranks = 1;    // this context's rank and the world (RCCL communicator or DQN host exchange)
  p2pmg_exchange_fn xfn = nullptr;  // DQN shared network: host gather of the gradient segments
  void* xuser = nullptr;
  double* d_metrics = nullptr;           // [2] episode-metric sum and count (p2pmg_allreduce_metrics)
  unsigned long long* d_hash = nullptr;  // [nranks] table fingerprints (p2pmg_table_hash_allgather)
  bool have_env = false, have_prof = false, have_params = false, have_codes = false;
  // DQN learner (config.learner = P2PMG_LEARNER_DQN)
  bool dqn = false;
  p2pmg_dqn_config dcfg{};
  int n_nets = 0;
  float* d_theta = nullptr;   // [n_nets][kNetStride]
  float* d_target = nullptr;
  float* d_m = nullptr;
  float* d_v = nullptr;
  float* d_grad = nullptr;    // shared network: [d_blocks][kNetStride] partials
  float* d_alt = nullptr;     // shared network: the other half of the Adam double buffer, [4][kNetStride]
                              // (online, target, m, v) for the act kernel's fused post-exchange Adam step
  float* d_segs = nullptr;    // [nranks * d_seg_local][kNetStride] gradient segments, global order
  size_t d_segs_cap = 0;      // floats at d_segs
  float* h_segs = nullptr;    // pinned host copy of d_segs (host exchange)
  size_t h_segs_cap = 0;
  float* d_smp = nullptr;     // [A][32] int32 ring slots sampled for the current step
  int d_blocks = 0, d_apb = 1;
  int d_seg_local = 1, d_seg_agents = 0, d_bps = 0;  // gradient segments of this context (p2pmg_dqn_config)
  float* d_buf = nullptr;     // [A][capacity][10]
  int32_t* d_added = nullptr; // [A]
  uint16_t* d_samples = nullptr;  // [T][A][32]
  uint16_t* d_samples_px = nullptr;  // [T][A][32]: a Philox training episode's draws (dqn_sample_prepass_kernel)
  bool have_samples = false;
  float* d_ep_acc = nullptr;  // [S]
  float* rec_loss = nullptr;  // [T][A]
  std::vector<int64_t> d_steps;  // Adam iterations done, per network (agent.py:310: one optimizer per agent)
  float* d_lr = nullptr;      // [T][n_nets] per-network step sizes of one episode when the counts differ
  size_t d_lr_cap = 0;        // floats allocated at d_lr
  std::vector<float> h_lr;
  int rec_last_mask = 0;      // records the last episode launch wrote (p2pmg_get_record checks it)
  int64_t d_added_min = 0;    // every ring holds at least this many transitions
  std::string err;
  std::string last_kernel;
};

// ---- RCCL, resolved at run time (torch may already have loaded its own librccl; dlopen by
// SONAME then reuses it, and the library stays loadable on hosts without RCCL)
struct Id128 {  // ncclUniqueId, passed by value to ncclCommInitRank
  char b[128];
};
struct Rccl {
  void* h = nullptr;
  int (*getUniqueId)(void*) = nullptr;
  int (*commInitRank)(void**, int, Id128, int) = nullptr;
  int (*allReduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;  // ncclDataType_t, ncclRedOp_t as int
  int (*commDestroy)(void*) = nullptr;
  const char* (*getErrorString)(int) = nullptr;
  int (*allGather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  int (*commCount)(const void*, int*) = nullptr;
};
static Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {
      r.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (r.h) break;
    }
    if (r.h) {
      r.getUniqueId = (int (*)(void*))dlsym(r.h, "ncclGetUniqueId");
      r.commInitRank = (int (*)(void**, int, Id128, int))dlsym(r.h, "ncclCommInitRank");
      r.allReduce = (int (*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(r.h, "ncclAllReduce");
      r.commDestroy = (int (*)(void*))dlsym(r.h, "ncclCommDestroy");
      r.getErrorString = (const char* (*)(int))dlsym(r.h, "ncclGetErrorString");
      r.allGather = (int (*)(const void*, void*, size_t, int, void*, hipStream_t))dlsym(r.h, "ncclAllGather");
      r.commCount = (int (*)(const void*, int*))dlsym(r.h, "ncclCommCount");
    }
  }
  return (r.h && r.getUniqueId && r.commInitRank && r.allReduce && r.commDestroy) ? &r : nullptr;
}

namespace {

int fail(p2pmg_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIP_TRY(ctx, expr)                                                                       \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess)                                                                        \
      return fail((ctx), _e == hipErrorOutOfMemory ? P2PMG_E_NOMEM : P2PMG_E_HIP,                \
                  std::string(#expr) + ": " + hipGetErrorString(_e));                            \
  } while (0)

template <typename T>
hipError_t dmalloc(T** p, size_t n) {
  return hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T) > 0 ? n * sizeof(T) : 16);
}

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree(reinterpret_cast<void*>(p));
  p = nullptr;
}

int rec_slot(int which) {
  switch (which) {
    case P2PMG_REC_REWARD: return 0;
    case P2PMG_REC_COST: return 1;
    case P2PMG_REC_GRID: return 2;
    case P2PMG_REC_P2P: return 3;
    case P2PMG_REC_TEMP: return 4;
    default: return -1;
  }
}

// Ensure every record buffer requested in mask exists (lazily allocated, kept for reuse).
int ensure_records(p2pmg_ctx* c, int mask) {
  const size_t ta = (size_t)c->T * c->A;
  for (int b = 0; b < 5; ++b)
    if ((mask & (1 << b)) && !c->rec_f32[b]) HIP_TRY(c, dmalloc(&c->rec_f32[b], ta));
  const size_t tra = (size_t)c->T * (c->R + 1) * c->A;
  if ((mask & P2PMG_REC_ACTION) && !c->rec_action) HIP_TRY(c, dmalloc(&c->rec_action, tra));
  if ((mask & P2PMG_REC_INDEX) && !c->rec_index) HIP_TRY(c, dmalloc(&c->rec_index, tra));
  if ((mask & P2PMG_REC_LOSS) && !c->rec_loss) HIP_TRY(c, dmalloc(&c->rec_loss, ta));
  return P2PMG_OK;
}

}  // namespace

extern "C" {

int p2pmg_abi_version(void) { return P2PMG_ABI_VERSION; }

int p2pmg_device_count(int* count) {
  if (!count) return P2PMG_E_INVALID;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return P2PMG_OK;
}

int p2pmg_config_default(p2pmg_config* cfg) {
  if (!cfg) return P2PMG_E_INVALID;
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->n_scenarios = 1;
  cfg->n_agents = 2;   // setup.py:33
  cfg->rounds = 1;     // setup.py:34
  cfg->horizon = 96;   // one day of 15-minute slots
  cfg->q_dtype = P2PMG_Q_F64;
  cfg->n_time_states = cfg->n_temp_states = cfg->n_balance_states = cfg->n_p2p_states = 20;
  cfg->n_actions = 3;
  cfg->alpha = 1e-5;
  cfg->gamma = 0.9;
  const double levels[3] = {0.0, 0.5, 1.0};
  for (int k = 0; k < 3; ++k) cfg->hp_levels[k] = (float)(levels[k] * 3e3);
  cfg->setpoint = 21.0f;
  cfg->temp_margin = 1.0f;
  cfg->lower_bound = 20.0f;
  cfg->upper_bound = 22.0f;
  const double Ci = 2.44e6 * 2, Cm = 9.4e7, Ri = 8.64e-4, Re = 1.05e-2, Rvent = 7.98e-3, gA = 11.468, f_rad = 0.3;
  cfg->inv_ci = (float)(1 / Ci);
  cfg->inv_cm = (float)(1 / Cm);
  cfg->inv_ri = (float)(1 / Ri);
  cfg->inv_re = (float)(1 / Re);
  cfg->inv_rvent = (float)(1 / Rvent);
  cfg->one_minus_frad = (float)(1 - f_rad);
  cfg->frad = (float)f_rad;
  cfg->solar_gain = (float)(gA * 0.0);
  cfg->hp_cop = 3.0f;
  cfg->seconds_per_minute = 60.0f;
  cfg->time_slot = 15.0f;
  cfg->minutes_per_hour = 60.0f;
  cfg->kilo = (float)1e-3;
  cfg->penalty_weight = 10.0f;
  cfg->seed = 42;
  cfg->scenario_offset = 0;
  return P2PMG_OK;
}

int p2pmg_create(const p2pmg_config* cfg, int device, p2pmg_ctx** out) {
  if (!cfg || !out) return P2PMG_E_INVALID;
  *out = nullptr;
  if (cfg->n_scenarios <= 0 || cfg->n_agents <= 0 || cfg->rounds < 0 || cfg->horizon <= 0) return P2PMG_E_INVALID;
  if (cfg->rounds + 1 > p2pmg::kMaxRounds1) return P2PMG_E_UNSUPPORTED;
  if (cfg->n_actions != 3) return P2PMG_E_UNSUPPORTED;
  const int N = cfg->n_agents;
  // any community size a scenario's wave holds (get_community takes any n_agents, community.py:198-204)
  if (N > p2pmg::kMaxAgents) return P2PMG_E_UNSUPPORTED;
  if (cfg->q_dtype != P2PMG_Q_F64 && cfg->q_dtype != P2PMG_Q_F32) return P2PMG_E_INVALID;
  p2pmg_ctx* c = new (std::nothrow) p2pmg_ctx();
  if (!c) return P2PMG_E_NOMEM;
  c->cfg = *cfg;
  c->device = device;
  c->S = cfg->n_scenarios;
  c->N = N;
  c->R = cfg->rounds;
  c->T = cfg->horizon;
  c->A = c->S * c->N;
  c->n_states = (size_t)cfg->n_time_states * cfg->n_temp_states * cfg->n_balance_states * cfg->n_p2p_states;
  c->q_elem = cfg->q_dtype == P2PMG_Q_F64 ? 8 : 4;
  auto bail = [&](int code) {
    p2pmg_destroy(c);
    return code;
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return bail(P2PMG_E_HIP);
  hipDeviceProp_t prop{};
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) c->n_cu = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail(P2PMG_E_HIP);
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) return bail(P2PMG_E_HIP);
  const size_t A = (size_t)c->A;
  if (dmalloc(&c->prof, (size_t)c->T * A) != hipSuccess || dmalloc(&c->max_in, A) != hipSuccess ||
      dmalloc(&c->t_in, A) != hipSuccess || dmalloc(&c->t_m, A) != hipSuccess ||
      dmalloc(&c->ep_reward, (size_t)c->S) != hipSuccess)
    return bail(P2PMG_E_NOMEM);
  // the code-word buffer always exists: greedy episodes read (and ignore) it, which keeps the
  // kernel's code loads unconditional
  const size_t ncw = (size_t)c->T * ((c->R + 4) / 4) * A;
  if (dmalloc(&c->codes, ncw) != hipSuccess) return bail(P2PMG_E_NOMEM);
  if (hipMalloc(&c->dummy, 2 * 64 * p2pmg::kFastRecBytes) != hipSuccess) return bail(P2PMG_E_NOMEM);
  if (hipMemsetAsync(c->codes, 0xFF, ncw * 4, c->stream) != hipSuccess) return bail(P2PMG_E_HIP);
  if (cfg->learner != P2PMG_LEARNER_TABULAR && cfg->learner != P2PMG_LEARNER_DQN) return bail(P2PMG_E_INVALID);
  c->dqn = cfg->learner == P2PMG_LEARNER_DQN;
  const size_t n_tables = c->dqn ? 0 : (cfg->shared_q ? 1 : A);
  const size_t qbytes = n_tables * c->n_states * kQPad * c->q_elem;
  if (hipMalloc(&c->q, qbytes ? qbytes : 16) != hipSuccess) return bail(P2PMG_E_NOMEM);
  if (cfg->shared_q && !c->dqn) {
    if (dmalloc(&c->qdelta, p2pmg::kDeltaCopies * c->n_states * kQPad) != hipSuccess) return bail(P2PMG_E_NOMEM);
    if (hipMemsetAsync(c->qdelta, 0, p2pmg::kDeltaCopies * c->n_states * kQPad * 8, c->stream) != hipSuccess)
      return bail(P2PMG_E_HIP);
  }
  if (dmalloc(&c->hp_lv, A) != hipSuccess || dmalloc(&c->soc, A) != hipSuccess) return bail(P2PMG_E_NOMEM);
  {
    std::vector<float4> lv(A, make_float4(cfg->hp_levels[0], cfg->hp_levels[1], cfg->hp_levels[2], 0.0f));
    std::vector<double> s0(A, 0.5);
    if (hipMemcpyAsync(c->hp_lv, lv.data(), A * sizeof(float4), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(c->soc, s0.data(), A * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return bail(P2PMG_E_HIP);
  }
  if (qbytes && hipMemsetAsync(c->q, 0, qbytes, c->stream) != hipSuccess) return bail(P2PMG_E_HIP);
  std::vector<float> t0(A, cfg->setpoint);
  if (hipMemcpyAsync(c->t_in, t0.data(), A * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(c->t_m, t0.data(), A * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return bail(P2PMG_E_HIP);
  *out = c;
  return P2PMG_OK;
}

int p2pmg_destroy(p2pmg_ctx* c) {
  if (!c) return P2PMG_OK;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  dfree(c->env);
  dfree(c->prof);
  dfree(c->sqp);
  dfree(c->max_in);
  dfree(c->t_in);
  dfree(c->t_m);
  if (c->q) (void)hipFree(c->q);
  dfree(c->codes);
  for (int k = 0; k < 2; ++k) {
    dfree(c->pre[k]);
    dfree(c->pre_ipc[k]);
    dfree(c->pcodes[k]);
    c->pcodes_cap[k] = 0;
  }
  if (c->dummy) (void)hipFree(c->dummy);
  if (c->rec_pack) (void)hipFree(c->rec_pack);
  dfree(c->ep_reward);
  dfree(c->chain_rew);
  dfree(c->d_metrics);
  dfree(c->d_hash);
  for (auto& b : c->rec_f32) dfree(b);
  dfree(c->rec_action);
  dfree(c->rec_index);
  if (c->rec_stage) (void)hipFree(c->rec_stage);
  dfree(c->hp_lv);
  dfree(c->hp_on);
  dfree(c->soc);
  dfree(c->bat_cap);
  dfree(c->qdelta);
  dfree(c->d_theta);
  dfree(c->d_target);
  dfree(c->d_m);
  dfree(c->d_v);
  dfree(c->d_alt);
  dfree(c->d_lr);
  dfree(c->d_grad);
  dfree(c->d_segs);
  if (c->h_segs) (void)hipHostFree(c->h_segs);
  if (c->h_small) (void)hipHostFree(c->h_small);
  dfree(c->d_smp);
  dfree(c->d_buf);
  dfree(c->d_added);
  dfree(c->d_samples);
  dfree(c->d_samples_px);
  dfree(c->d_ep_acc);
  dfree(c->rec_loss);
  if (c->comm && rccl()) rccl()->commDestroy(c->comm);
  c->comm = nullptr;
  for (auto& ev : c->ring)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : c->cring)
    if (ev) (void)hipEventDestroy(ev);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return P2PMG_OK;
}

const char* p2pmg_last_error(const p2pmg_ctx* c) { return c ? c->err.c_str() : "null context"; }

int p2pmg_sync(p2pmg_ctx* c) {
  if (!c) return P2PMG_E_INVALID;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_device_info(p2pmg_ctx* c, char* name, size_t name_len, size_t* total_mem) {
  if (!c) return P2PMG_E_INVALID;
  hipDeviceProp_t prop;
  HIP_TRY(c, hipGetDeviceProperties(&prop, c->device));
  if (name && name_len) {
    std::snprintf(name, name_len, "%s (%s)", prop.name, prop.gcnArchName);
  }
  if (total_mem) *total_mem = prop.totalGlobalMem;
  return P2PMG_OK;
}

int p2pmg_set_env(p2pmg_ctx* c, int n_env, const float* time, const float* t_out, const float* buy, const float* inj,
                  const float* p2p) {
  if (c) c->inputs_version++;  // invalidates the speculative pre-pass slots
  if (!c || !time || !t_out || !buy || !inj || !p2p) return P2PMG_E_INVALID;
  if (n_env != 1 && n_env != c->S) return fail(c, P2PMG_E_INVALID, "n_env must be 1 or S");
  const size_t T = c->T;
  std::vector<float> h((size_t)n_env * T * kEnvStride, 0.0f);
  for (int s = 0; s < n_env; ++s)
    for (size_t t = 0; t < T; ++t) {
      float* r = &h[((size_t)t * n_env + s) * kEnvStride];  // time-major [T][n_env][8]
      const size_t k = (size_t)s * T + t;
      r[0] = time[k];
      r[1] = t_out[k];
      r[2] = buy[k];
      r[3] = inj[k];
      r[4] = p2p[k];
    }
  if (c->n_env != n_env) {
    dfree(c->env);
    HIP_TRY(c, dmalloc(&c->env, h.size()));
    c->n_env = n_env;
  }
  HIP_TRY(c, hipMemcpyAsync(c->env, h.data(), h.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->have_env = true;
  return P2PMG_OK;
}

int p2pmg_set_profiles(p2pmg_ctx* c, const float* load_w, const float* pv_w) {
  if (c) c->inputs_version++;  // invalidates the speculative pre-pass slots
  if (!c || !load_w || !pv_w) return P2PMG_E_INVALID;
  const size_t n = (size_t)c->A * c->T;
  float *dl = nullptr, *dp = nullptr;
  HIP_TRY(c, dmalloc(&dl, n));
  hipError_t e = dmalloc(&dp, n);
  if (e != hipSuccess) {
    dfree(dl);
    return fail(c, P2PMG_E_NOMEM, "profile staging");
  }
  {  // the battery rule's range-test-free variant needs bounded, finite balances (p2pmg_kernels.hip)
    bool ok = true;
    for (size_t k = 0; k < n; ++k) ok = ok && std::fabs(load_w[k]) <= 0x1p100f && std::fabs(pv_w[k]) <= 0x1p100f;
    c->prof_bounded = ok;
  }
  e = hipMemcpyAsync(dl, load_w, n * 4, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dp, pv_w, n * 4, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = p2pmg::launch_prof_pack(c->A, c->T, dl, dp, c->prof, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(dl);
  dfree(dp);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("set_profiles: ") + hipGetErrorString(e));
  c->have_prof = true;
  return P2PMG_OK;
}

int p2pmg_set_agent_params(p2pmg_ctx* c, const float* max_in) {
  if (c) c->inputs_version++;  // invalidates the speculative pre-pass slots
  if (!c || !max_in) return P2PMG_E_INVALID;
  HIP_TRY(c, hipMemcpyAsync(c->max_in, max_in, (size_t)c->A * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->mi_ok = true;
  for (int a = 0; a < c->A; ++a) {
    const float m = std::fabs(max_in[a]);
    if (!(m >= 0x1p-40f && m <= 0x1p40f)) c->mi_ok = false;
  }
  c->have_params = true;
  return P2PMG_OK;
}

int p2pmg_set_temperatures(p2pmg_ctx* c, const float* t_in, const float* t_m) {
  if (!c || !t_in || !t_m) return P2PMG_E_INVALID;
  HIP_TRY(c, hipMemcpyAsync(c->t_in, t_in, (size_t)c->A * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->t_m, t_m, (size_t)c->A * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_get_temperatures(p2pmg_ctx* c, float* t_in, float* t_m) {
  if (!c || !t_in || !t_m) return P2PMG_E_INVALID;
  HIP_TRY(c, hipMemcpyAsync(t_in, c->t_in, (size_t)c->A * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(t_m, c->t_m, (size_t)c->A * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_reset_temperatures_philox(p2pmg_ctx* c, int episode, double sigma) {
  if (!c) return P2PMG_E_INVALID;
  const uint32_t off = (uint32_t)(c->cfg.scenario_offset * c->N);
  HIP_TRY(c, p2pmg::launch_t0_philox(c->A, c->t_in, c->t_m, (uint32_t)(c->cfg.seed & 0xFFFFFFFFu),
                                     (uint32_t)(c->cfg.seed >> 32), episode, off, c->cfg.setpoint, sigma, c->stream));
  return P2PMG_OK;
}

static int ensure_codes(p2pmg_ctx* c) {
  if (!c->codes) HIP_TRY(c, dmalloc(&c->codes, (size_t)c->T * ((c->R + 4) / 4) * c->A));
  return P2PMG_OK;
}

int p2pmg_set_replay_codes(p2pmg_ctx* c, const uint8_t* codes) {
  if (!c || !codes) return P2PMG_E_INVALID;
  const size_t n = (size_t)c->T * (c->R + 1) * c->A;
  int rc = ensure_codes(c);
  if (rc != P2PMG_OK) return rc;
  uint8_t* staging = nullptr;
  HIP_TRY(c, dmalloc(&staging, n));
  hipError_t e = hipMemcpyAsync(staging, codes, n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = p2pmg::launch_pack_codes(c->T, c->R + 1, c->A, staging, c->codes, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(staging);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("set_replay_codes: ") + hipGetErrorString(e));
  c->have_codes = true;
  c->code_src = 1;
  return P2PMG_OK;
}

int p2pmg_zero_q(p2pmg_ctx* c) {
  if (!c) return P2PMG_E_INVALID;
  if (c->dqn) return fail(c, P2PMG_E_STATE, "zero_q: DQN context has no Q-table");
  const size_t n_tables = c->cfg.shared_q ? 1 : (size_t)c->A;
  HIP_TRY(c, hipMemsetAsync(c->q, 0, n_tables * c->n_states * kQPad * c->q_elem, c->stream));
  if (c->qdelta) HIP_TRY(c, hipMemsetAsync(c->qdelta, 0, p2pmg::kDeltaCopies * c->n_states * kQPad * 8, c->stream));
  return P2PMG_OK;
}

static int q_range_ok(p2pmg_ctx* c, int first, int count, const void* host, int dtype) {
  if (c && c->dqn) return 0;
  const int n_tables = c && c->cfg.shared_q ? 1 : (c ? c->A : 0);
  if (!c || !host || first < 0 || count < 0 || first + count > n_tables) return 0;
  return dtype == P2PMG_Q_F64 || dtype == P2PMG_Q_F32;
}

int p2pmg_set_q(p2pmg_ctx* c, int first, int count, const void* host, int host_dtype) {
  if (!q_range_ok(c, first, count, host, host_dtype)) return fail(c, P2PMG_E_INVALID, "set_q: bad range/dtype");
  const int na = c->cfg.n_actions;
  const size_t hbytes = (size_t)count * c->n_states * na * (host_dtype == P2PMG_Q_F64 ? 8 : 4);
  void* staging = nullptr;
  HIP_TRY(c, hipMalloc(&staging, hbytes ? hbytes : 16));
  char* dst = static_cast<char*>(c->q) + (size_t)first * c->n_states * kQPad * c->q_elem;
  hipError_t e = hipMemcpyAsync(staging, host, hbytes, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = p2pmg::launch_q_pack(count, c->n_states, na, staging, dst, c->cfg.q_dtype, host_dtype, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(staging);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("set_q: ") + hipGetErrorString(e));
  return P2PMG_OK;
}

int p2pmg_get_q(p2pmg_ctx* c, int first, int count, void* host, int host_dtype) {
  if (!q_range_ok(c, first, count, host, host_dtype)) return fail(c, P2PMG_E_INVALID, "get_q: bad range/dtype");
  const int na = c->cfg.n_actions;
  const size_t hbytes = (size_t)count * c->n_states * na * (host_dtype == P2PMG_Q_F64 ? 8 : 4);
  void* staging = nullptr;
  HIP_TRY(c, hipMalloc(&staging, hbytes ? hbytes : 16));
  const char* src = static_cast<const char*>(c->q) + (size_t)first * c->n_states * kQPad * c->q_elem;
  hipError_t e = p2pmg::launch_q_unpack(count, c->n_states, na, src, staging, c->cfg.q_dtype, host_dtype, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(host, staging, hbytes, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(staging);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("get_q: ") + hipGetErrorString(e));
  return P2PMG_OK;
}

static EpisodeParams episode_params(p2pmg_ctx* c, const p2pmg_episode_args* args) {
  const bool train = args->mode != P2PMG_MODE_GREEDY;
  const p2pmg_config& g = c->cfg;
  EpisodeParams p{};
  p.S = c->S;
  p.N = c->N;
  p.R = c->R;
  p.T = c->T;
  p.A = c->A;
  p.mode = args->mode;
  p.rng = 0;
  p.episode = args->episode;
  p.record = args->record;
  p.n_env = c->n_env;
  p.env = c->env;
  p.prof = c->prof;
  p.max_in = c->max_in;
  p.t_in = c->t_in;
  p.t_m = c->t_m;
  p.q = c->q;
  p.codes = c->codes;
  p.eps = args->epsilon;
  p2pmg::eps_threshold(p.eps, p.eps_thr, p.eps_all);
  if (train && args->rng == P2PMG_RNG_PHILOX) p.rng = 1;  // in-kernel unless the pre-pass below runs
  p.seed_lo = (uint32_t)(g.seed & 0xFFFFFFFFu);
  p.seed_hi = (uint32_t)(g.seed >> 32);
  p.agent_offset = (uint32_t)(g.scenario_offset * c->N);
  p.rec_reward = c->rec_f32[0];
  p.rec_cost = c->rec_f32[1];
  p.rec_grid = c->rec_f32[2];
  p.rec_p2p = c->rec_f32[3];
  p.rec_tin = c->rec_f32[4];
  p.rec_action = c->rec_action;
  p.rec_index = c->rec_index;
  p.ep_reward = c->ep_reward;
  p.shared_q = g.shared_q ? 1 : 0;
  p.qdelta = c->qdelta;
  p.battery = c->battery ? 1 : 0;
  p.bat_safe = (c->battery && c->bat_domain && c->prof_bounded && c->hp_bounded) ? 1 : 0;
  p.soc = c->soc;
  p.bat_cap = c->bat_cap;
  p.bat_min = c->bat_min;
  p.bat_max = c->bat_max;
  p.bat_sqrt_eff = c->bat_sqrt_eff;
  p.hp_lv = c->hp_lv;
  p.dummy = c->dummy;
  p.nt = g.n_time_states;
  p.nT = g.n_temp_states;
  p.nb = g.n_balance_states;
  p.np = g.n_p2p_states;
  p.alpha = g.alpha;
  p.gamma = g.gamma;
  for (int k = 0; k < 4; ++k) p.hp_levels[k] = g.hp_levels[k];
  p.setpoint = g.setpoint;
  p.margin = g.temp_margin;
  p.lower = g.lower_bound;
  p.upper = g.upper_bound;
  p.inv_ci = g.inv_ci;
  p.inv_cm = g.inv_cm;
  p.inv_ri = g.inv_ri;
  p.inv_re = g.inv_re;
  p.inv_rvent = g.inv_rvent;
  p.c_in = g.one_minus_frad;
  p.c_m = g.frad;
  p.solar = g.solar_gain;
  p.cop = g.hp_cop;
  p.spm = g.seconds_per_minute;
  p.slot = g.time_slot;
  p.mph = g.minutes_per_hour;
  p.kilo = g.kilo;
  p.penw = g.penalty_weight;
  return p;
}

static int dqn_run_episode(p2pmg_ctx* c, const p2pmg_episode_args* args);

// divisors the fast kernel divides by with the range-free quotient (fdiv_b in p2pmg_kernels.hip)
static bool host_div_range(float b) {
  const float m = std::fabs(b);
  return m >= 0x1p-40f && m <= 0x1p40f;
}

// fast per-agent-table path (episode_fast_kernel): automatic whenever it applies
static bool fast_applies(const p2pmg_ctx* c, const p2pmg_episode_args* args) {
  static const bool env_general = [] { const char* v = getenv("P2PMG_KERNEL"); return v && !strcmp(v, "general"); }();
  const p2pmg_config& g = c->cfg;
  return !g.shared_q && (!c->battery || c->R + 1 <= p2pmg::kFastBatMaxR1) && c->N <= 8 && c->R + 1 <= 4 && c->mi_ok &&
         (long long)g.n_time_states * g.n_temp_states * g.n_balance_states < 65536 &&
         // a wave's 64 tables span < 4 GiB (the gathers' 32-bit offsets)
         64LL * g.n_time_states * g.n_temp_states * g.n_balance_states * g.n_p2p_states * 4 * (g.q_dtype == 0 ? 8 : 4) <
             (1LL << 32) &&
         (long long)c->T * c->A < (1LL << 32) && host_div_range(g.minutes_per_hour) &&
         g.temp_margin == 1.0f &&  // heating.py:90 (the kernel skips the / margin)
         !(args->flags & (P2PMG_FLAG_GENERAL_KERNEL | P2PMG_FLAG_TILE_KERNEL | P2PMG_FLAG_PHILOX_INKERNEL)) &&
         !env_general;
}

// a chained fast-path launch (p2pmg_run_episodes): n episodes at eps[0..n), the caller's guess of
// the next chain (next_n episodes at next_eps) for the speculative pre-pass, rewards [n][S] on device
struct ChainReq {
  int n;
  const double* eps;
  int next_n;
  const double* next_eps;
  float* rewards;
  int reserve;  // code-word capacity to allocate, in episodes (every chain of the call fits)
};

static int run_episode_impl(p2pmg_ctx* c, const p2pmg_episode_args* args, const ChainReq* ch);

int p2pmg_run_episode(p2pmg_ctx* c, const p2pmg_episode_args* args) {
  if (c) c->chain_n = 0;  // p2pmg_get_episode_rewards covers p2pmg_run_episodes calls only
  return run_episode_impl(c, args, nullptr);
}

static int run_episode_impl(p2pmg_ctx* c, const p2pmg_episode_args* args, const ChainReq* ch) {
  if (!c || !args) return P2PMG_E_INVALID;
  if (c->dqn) return dqn_run_episode(c, args);
  if (!c->have_env || !c->have_prof || !c->have_params)
    return fail(c, P2PMG_E_STATE, "run_episode: env, profiles and agent params must be set first");
  const bool train = args->mode == P2PMG_MODE_TRAIN;
  if (args->mode != P2PMG_MODE_TRAIN && args->mode != P2PMG_MODE_GREEDY) return fail(c, P2PMG_E_INVALID, "mode");
  if (train && args->rng != P2PMG_RNG_REPLAY && args->rng != P2PMG_RNG_PHILOX) return fail(c, P2PMG_E_INVALID, "rng");
  if (train && args->rng == P2PMG_RNG_REPLAY && !c->have_codes)
    return fail(c, P2PMG_E_STATE, "run_episode: replay mode needs p2pmg_set_replay_codes");
  int rc = P2PMG_OK;
  const p2pmg_config& g = c->cfg;
  static const int env_spw = [] { const char* v = getenv("P2PMG_SPW"); return v ? atoi(v) : 0; }();
  static const bool env_general = [] { const char* v = getenv("P2PMG_KERNEL"); return v && !strcmp(v, "general"); }();
  const bool fast = fast_applies(c, args);
  if (ch && !(fast && train && args->rng == P2PMG_RNG_PHILOX))
    return fail(c, P2PMG_E_INVALID, "run_episode: a chained launch needs the fast kernel and Philox training");
  // shared table, 16-agent scenarios (configs[2]): episode_sq16_kernel
  const bool sq16 = g.shared_q && c->N == 16 && c->R <= 1 && c->mi_ok && host_div_range(g.minutes_per_hour) &&
                    (long long)c->T * c->A < (1LL << 32) && (long long)c->T * c->n_env * p2pmg::kEnvStride < (1LL << 32) &&
                    host_div_range(g.temp_margin) && g.n_time_states == 20 && g.n_temp_states == 20 &&
                    g.n_balance_states == 20 && g.n_p2p_states == 20 &&
                    !(args->flags & (P2PMG_FLAG_GENERAL_KERNEL | P2PMG_FLAG_TILE_KERNEL)) && !env_general;
  // the general kernel writes unpacked records; fast / sq16 write packed rows (rec_pack) that
  // p2pmg_get_record unpacks into one staging buffer, so those launches allocate no [T][A] arrays
  // per record (configs[3] at full size: 35 GB less)
  if (!fast && !sq16) {
    rc = ensure_records(c, args->record);
    if (rc != P2PMG_OK) return rc;
  }
  EpisodeParams p = episode_params(c, args);
  const int ps = c->pslot;
  p2pmg::PrepOut next{};
  bool produce = false;
  if (fast) {
    const size_t ta = (size_t)c->T * c->A;
    const size_t wpe = ta * ((c->R + 4) / 4);  // code words per episode
    const bool philox = train && args->rng == P2PMG_RNG_PHILOX;
    const bool want_ipc = c->N == 2 && c->R >= 1 && !c->battery;  // the kernel's CAND path
    // this launch's chain (one episode unless chained) and the caller's guess of the next launch's:
    // P2PMG_FLAG_NEXT_EPSILON: next_epsilon is the guess as given (0 included); without it a
    // positive next_epsilon is the guess and anything else means "the same epsilon"
    std::vector<double> cur(ch ? ch->eps : &args->epsilon, ch ? ch->eps + ch->n : &args->epsilon + 1);
    std::vector<double> nxt_eps;
    if (ch) {
      if (ch->next_n > 0) nxt_eps.assign(ch->next_eps, ch->next_eps + ch->next_n);
      else nxt_eps.assign(cur.size(), cur.back());
    } else {
      const bool have_next = (args->flags & P2PMG_FLAG_NEXT_EPSILON) != 0 || args->next_epsilon > 0.0;
      nxt_eps.assign(1, have_next ? args->next_epsilon : args->epsilon);
    }
    const int n_ep = (int)cur.size(), n_next = (int)nxt_eps.size();
    for (int k = 0; k < 2; ++k) {  // both slots (the launch writes the other one)
      if (!c->pre[k]) HIP_TRY(c, dmalloc(&c->pre[k], ta));
      if (want_ipc && !c->pre_ipc[k]) HIP_TRY(c, dmalloc(&c->pre_ipc[k], ta));
      const size_t need = wpe * (size_t)std::max(n_ep, n_next);
      if (philox && c->pcodes_cap[k] < need) {  // chains: their full capacity at once (no reallocation later)
        const size_t cap = std::max(need, wpe * (size_t)(ch ? ch->reserve : 1));
        dfree(c->pcodes[k]);
        c->pcodes_cap[k] = 0;
        c->spec_valid[k] = false;
        HIP_TRY(c, dmalloc(&c->pcodes[k], cap));
        c->pcodes_cap[k] = cap;
      }
    }
    p.pre_ipc = want_ipc ? c->pre_ipc[ps] : nullptr;
    if (philox) p.codes = c->pcodes[ps];
    p.rng = 0;
    p.chain = n_ep;
    p.codes_stride = wpe;
    p.chain_rewards = ch ? ch->rewards : nullptr;
    if (args->record && !c->rec_pack) HIP_TRY(c, hipMalloc(&c->rec_pack, ta * p2pmg::kFastRecBytes));
    auto prep_out = [&](int slot, int episode, const std::vector<double>& eps) {
      p2pmg::PrepOut o{c->pre[slot], want_ipc ? c->pre_ipc[slot] : nullptr, philox ? c->pcodes[slot] : nullptr,
                       episode, eps[0], 0u, 0};
      p2pmg::eps_threshold(eps[0], o.eps_thr, o.eps_all);
      o.n_ep = (int)eps.size();
      o.words_stride = wpe;
      o.ep_all = 0;
      for (int k = 0; k < o.n_ep; ++k) {
        int all = 0;
        p2pmg::eps_threshold(eps[k], o.ep_thr[k], all);
        o.ep_all |= (uint64_t)all << k;
      }
      return o;
    };
    // this slot's pre-pass: computed by the previous launch if it guessed these arguments
    const bool hit = c->spec_valid[ps] && c->spec_version[ps] == c->inputs_version &&
                     (!philox || (c->spec_episode[ps] == args->episode && c->spec_chain[ps] == cur));
    if (!hit) HIP_TRY(c, p2pmg::launch_step_prepass(p, prep_out(ps, args->episode, cur), c->stream));
    // the next slot, for the episodes after this launch's at the caller's guess (the decay schedule
    // is known, community.py:279-286).  Philox draws only when this one has them.
    // P2PMG_NO_SPEC=1 (profiling only): no producer blocks, so the episode kernel's counters are its own
    static const bool env_no_spec = [] { const char* v = getenv("P2PMG_NO_SPEC"); return v && atoi(v) != 0; }();
    const int ns = ps ^ 1;
    next = prep_out(ns, args->episode + n_ep, nxt_eps);
    produce = !env_no_spec;
    if (hit) c->spec_hits++;
    else c->spec_misses++;
    c->spec_valid[ns] = produce;
    c->spec_version[ns] = c->inputs_version;
    c->spec_episode[ns] = philox ? args->episode + n_ep : -1;
    c->spec_chain[ns] = nxt_eps;
  } else if (train && args->rng == P2PMG_RNG_PHILOX) {
    bool prepass = c->A < (1 << 18) && !sq16;  // sq16: throughput-bound, draws in the kernel
    if (args->flags & P2PMG_FLAG_PHILOX_PREPASS) prepass = true;
    if (args->flags & P2PMG_FLAG_PHILOX_INKERNEL) prepass = false;
    if (prepass) {
      rc = ensure_codes(c);
      if (rc != P2PMG_OK) return rc;
      p.codes = c->codes;
      HIP_TRY(c, p2pmg::launch_philox_codes(p, c->codes, c->stream));
      c->code_src = 2;
      c->have_codes = false;  // a replay upload must be repeated after a pre-pass overwrote it
      p.rng = 0;
    }
  }
  if (c->ring.empty()) {
    c->ring.assign(2 * p2pmg_ctx::kRing, nullptr);
    for (auto& ev : c->ring) HIP_TRY(c, hipEventCreate(&ev));
  }
  // dispatch-stamped events cost ~4 us per launch at configs[1] (~5 % of an episode): with a
  // timing period k only every k-th launch carries them
  const bool stamp = (c->n_launch++ % c->timing_period) == 0;
  const int slot = (int)(c->n_timed % p2pmg_ctx::kRing);
  hipEvent_t r0 = stamp ? c->ring[2 * slot] : nullptr, r1 = stamp ? c->ring[2 * slot + 1] : nullptr;
  if (sq16) {
    if (args->record && !c->rec_pack)
      HIP_TRY(c, hipMalloc(&c->rec_pack, (size_t)c->T * c->A * p2pmg::kFastRecBytes));
    p.rec_pack = c->rec_pack;
    // the step words {balance, time / balance row offset}: recomputed after any input upload
    if (!c->sqp) HIP_TRY(c, dmalloc(&c->sqp, (size_t)c->T * c->A));
    if (c->sqp_version != c->inputs_version) {
      HIP_TRY(c, p2pmg::launch_sq16_prep(p, c->sqp, c->stream));
      c->sqp_version = c->inputs_version;
    }
    p.sqp = c->sqp;
  }
  // fast / sq16: only {reward, cost} requested -> 8-B record rows
  p.rec_narrow = (fast || sq16) && (args->record & ~(P2PMG_REC_REWARD | P2PMG_REC_COST)) == 0 ? 1 : 0;
  const bool ext = fast || sq16;  // launches that stamp their own timing events
  if (!ext && stamp) HIP_TRY(c, hipEventRecord(r0, c->stream));
  int spw = args->scen_per_wave > 0 ? args->scen_per_wave : env_spw;
  if (spw <= 0) {  // automatic: full waves, or spread a small batch over all CUs (one wave per CU)
    const int full = 64 / (c->N <= 1 ? 1 : c->N <= 2 ? 2 : c->N <= 4 ? 4 : 8);
    const int waves = (c->S + full - 1) / full;
    spw = waves >= c->n_cu ? full : std::max(full / 4, (c->S + c->n_cu - 1) / c->n_cu);
    // below epsilon 0.5 most lanes are greedy (a round-0 row gather and two argmaxes on every step):
    // there half-filled waves, two per CU, measured faster (configs[1], chained: 80.7 -> 77.9 us per
    // episode at epsilon 0.1, 76.1 -> 75.0 at 0.39, even at 0.53), above it one wave per CU
    // (71.7 against 73.9 us at 0.729): profiles/r05_chain/spw_epsilon.txt
    if (fast && train && args->epsilon < 0.5 && waves < c->n_cu) spw = std::max(full / 4, (spw + 1) / 2);
    spw = std::min(spw, full);
  }
  const bool reset = (args->flags & P2PMG_FLAG_RESET_T0) != 0;
  // the general kernel's LDS-tile form: every N outside {1..8, 16}, or any N on request
  const bool tile = !fast && !sq16 &&
                    ((args->flags & P2PMG_FLAG_TILE_KERNEL) != 0 || !((c->N >= 1 && c->N <= 8) || c->N == 16));
  p.reset_t0 = (ext && reset) ? 1 : 0;
  p.reset_sigma = args->reset_sigma;
  hipError_t e = fast   ? p2pmg::launch_episode_fast(p, c->pre[ps], c->rec_pack, g.q_dtype, spw,
                                                    produce ? &next : nullptr, r0, r1, c->stream)
                 : sq16 ? p2pmg::launch_episode_sq16(p, g.q_dtype, r0, r1, c->stream)
                        : p2pmg::launch_episode(p, g.q_dtype, tile, c->stream);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("episode launch: ") + hipGetErrorString(e));
  c->rec_fast_mask = ext ? (args->record & 127) : 0;
  c->rec_last_mask = args->record;
  c->rec_narrow = (fast || sq16) ? p.rec_narrow : 0;
  c->last_kernel = std::string(fast ? "episode_fast_kernel<" : sq16 ? "episode_sq16_kernel<" : "episode_kernel<") +
                   std::to_string(c->N) + (tile ? ",tile" + std::to_string(p2pmg::general_tile_cap(c->N)) : "") + "," +
                   (g.q_dtype == 0 ? "f64" : "f32") + ",R1=" + std::to_string(c->R + 1) +
                   (ext ? (train ? ",train" : ",greedy") : "") + (g.shared_q ? ",shared" : "") +
                   (c->battery ? (ext && !p.bat_safe ? ",battery,range-checked>" : ",battery>") : ">");
  if (!ext && stamp) HIP_TRY(c, hipEventRecord(r1, c->stream));
  if (fast) c->pslot ^= 1;
  if (reset && !ext) {  // general kernel: the reset as its own launch
    const uint32_t off = (uint32_t)(g.scenario_offset * c->N);
    HIP_TRY(c, p2pmg::launch_t0_philox(c->A, c->t_in, c->t_m, p.seed_lo, p.seed_hi, args->episode + 1, off,
                                       g.setpoint, args->reset_sigma, c->stream));
  }
  c->timed = true;
  if (stamp) c->n_timed++;
  return P2PMG_OK;
}

int p2pmg_run_episodes(p2pmg_ctx* c, const p2pmg_episode_args* args, int n, const double* epsilons, int next_n,
                       const double* next_epsilons) {
  if (!c || !args || n < 1 || !epsilons || (next_n > 0 && !next_epsilons)) return P2PMG_E_INVALID;
  if (!c->dqn && (!c->have_env || !c->have_prof || !c->have_params))
    return fail(c, P2PMG_E_STATE, "run_episodes: env, profiles and agent params must be set first");
  if (c->chain_rew_cap < n) {  // at least one full chain's worth, so a caller's chains never reallocate
    const int cap = std::max(n, p2pmg::kMaxChain);
    dfree(c->chain_rew);
    c->chain_rew_cap = 0;
    HIP_TRY(c, dmalloc(&c->chain_rew, (size_t)cap * c->S));
    c->chain_rew_cap = cap;
  }
  c->chain_n = 0;
  const bool chain = !c->dqn && args->mode == P2PMG_MODE_TRAIN && args->rng == P2PMG_RNG_PHILOX && fast_applies(c, args);
  p2pmg_episode_args a = *args;
  if (!chain) {  // one launch per episode, the same results
    for (int k = 0; k < n; ++k) {
      a.episode = args->episode + k;
      a.epsilon = epsilons[k];
      a.flags = args->flags | P2PMG_FLAG_NEXT_EPSILON;
      a.next_epsilon = k + 1 < n ? epsilons[k + 1] : next_n > 0 ? next_epsilons[0] : epsilons[k];
      const int rc = run_episode_impl(c, &a, nullptr);
      if (rc != P2PMG_OK) return rc;
      HIP_TRY(c, hipMemcpyAsync(c->chain_rew + (size_t)k * c->S, c->ep_reward,
                                (size_t)c->S * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
    }
    c->chain_n = n;
    return P2PMG_OK;
  }
  // chains of at most kMaxChain episodes whose code words fit 1 GiB per slot
  const size_t wpe_bytes = (size_t)c->T * c->A * ((c->R + 4) / 4) * sizeof(uint32_t);
  const int per = (int)std::max<size_t>(1, std::min<size_t>(p2pmg::kMaxChain, ((size_t)1 << 30) / wpe_bytes));
  for (int k0 = 0; k0 < n; k0 += per) {
    const int m = std::min(per, n - k0);
    const int k1 = k0 + m;
    ChainReq req{m, epsilons + k0, 0, nullptr, c->chain_rew + (size_t)k0 * c->S, per};
    if (k1 < n) {
      req.next_n = std::min(per, n - k1);
      req.next_eps = epsilons + k1;
    } else if (next_n > 0) {
      req.next_n = std::min(per, next_n);
      req.next_eps = next_epsilons;
    }
    a.episode = args->episode + k0;
    a.epsilon = epsilons[k0];
    const int rc = run_episode_impl(c, &a, &req);
    if (rc != P2PMG_OK) return rc;
  }
  c->chain_n = n;
  return P2PMG_OK;
}

int p2pmg_get_episode_rewards(p2pmg_ctx* c, int n, float* host) {
  if (!c || !host || n < 0) return P2PMG_E_INVALID;
  if (n > c->chain_n) return fail(c, P2PMG_E_STATE, "get_episode_rewards: the last run_episodes call ran fewer episodes");
  HIP_TRY(c, hipMemcpyAsync(host, c->chain_rew, (size_t)n * c->S * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_set_timing_period(p2pmg_ctx* c, int period) {
  if (!c || period < 1) return P2PMG_E_INVALID;
  c->timing_period = period;
  c->n_launch = 0;
  return P2PMG_OK;
}

static int ensure_hp_on(p2pmg_ctx* c) {
  if (c->hp_on) return P2PMG_OK;
  HIP_TRY(c, dmalloc(&c->hp_on, (size_t)c->A));
  HIP_TRY(c, hipMemsetAsync(c->hp_on, 0, (size_t)c->A * sizeof(float), c->stream));
  return P2PMG_OK;
}

int p2pmg_set_hp_state(p2pmg_ctx* c, const float* on) {
  if (!c || !on) return P2PMG_E_INVALID;
  int rc = ensure_hp_on(c);
  if (rc != P2PMG_OK) return rc;
  HIP_TRY(c, hipMemcpyAsync(c->hp_on, on, (size_t)c->A * sizeof(float), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_get_hp_state(p2pmg_ctx* c, float* on) {
  if (!c || !on) return P2PMG_E_INVALID;
  int rc = ensure_hp_on(c);
  if (rc != P2PMG_OK) return rc;
  HIP_TRY(c, hipMemcpyAsync(on, c->hp_on, (size_t)c->A * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_run_rule_episode(p2pmg_ctx* c, int record) {
  if (!c) return P2PMG_E_INVALID;
  if (c->dqn) return fail(c, P2PMG_E_STATE, "run_rule_episode: DQN context");
  if (!c->have_env || !c->have_prof || !c->have_params)
    return fail(c, P2PMG_E_STATE, "run_rule_episode: env, profiles and agent params must be set first");
  if (c->R != 0)  // the reference's tensor_diag_part on the (N, 1) stack fails for rounds > 0
    return fail(c, P2PMG_E_INVALID, "run_rule_episode: RuleAgent communities run with rounds = 0");
  if (c->N > 64) return fail(c, P2PMG_E_INVALID, "run_rule_episode: N <= 64");
  const int rec = record & (P2PMG_REC_COST | P2PMG_REC_GRID | P2PMG_REC_P2P | P2PMG_REC_TEMP | P2PMG_REC_ACTION);
  int rc = ensure_records(c, rec);
  if (rc == P2PMG_OK) rc = ensure_hp_on(c);
  if (rc != P2PMG_OK) return rc;
  p2pmg_episode_args args{};
  args.mode = P2PMG_MODE_GREEDY;
  args.record = rec;
  EpisodeParams p = episode_params(c, &args);
  if (c->ring.empty()) {
    c->ring.assign(2 * p2pmg_ctx::kRing, nullptr);
    for (auto& ev : c->ring) HIP_TRY(c, hipEventCreate(&ev));
  }
  const int slot = (int)(c->n_timed % p2pmg_ctx::kRing);
  HIP_TRY(c, hipEventRecord(c->ring[2 * slot], c->stream));
  HIP_TRY(c, p2pmg::launch_rule_episode(p, c->hp_on, c->stream));
  HIP_TRY(c, hipEventRecord(c->ring[2 * slot + 1], c->stream));
  c->rec_fast_mask = 0;
  c->rec_last_mask = rec;
  c->last_kernel = "rule_episode_kernel<" + std::to_string(c->N) + ">";
  c->timed = true;
  c->n_timed++;
  return P2PMG_OK;
}

const char* p2pmg_last_kernel(const p2pmg_ctx* c) { return c ? c->last_kernel.c_str() : ""; }

int p2pmg_last_kernel_ms(p2pmg_ctx* c, float* ms) {
  if (!c || !ms) return P2PMG_E_INVALID;
  if (!c->timed || c->n_timed == 0) return fail(c, P2PMG_E_STATE, "no episode launched yet");
  const int slot = (int)((c->n_timed - 1) % p2pmg_ctx::kRing);  // the ring pair of the last launch
  HIP_TRY(c, hipEventSynchronize(c->ring[2 * slot + 1]));
  HIP_TRY(c, hipEventElapsedTime(ms, c->ring[2 * slot], c->ring[2 * slot + 1]));
  return P2PMG_OK;
}

int p2pmg_kernel_times(p2pmg_ctx* c, float* ms, int max, int* count) {
  if (!c || !ms || max < 0 || !count) return P2PMG_E_INVALID;
  const long long n = c->n_timed < p2pmg_ctx::kRing ? c->n_timed : p2pmg_ctx::kRing;
  const long long first = c->n_timed - n;
  int w = 0;
  for (long long k = first; k < c->n_timed && w < max; ++k, ++w) {
    const int slot = (int)(k % p2pmg_ctx::kRing);
    HIP_TRY(c, hipEventSynchronize(c->ring[2 * slot + 1]));
    HIP_TRY(c, hipEventElapsedTime(&ms[w], c->ring[2 * slot], c->ring[2 * slot + 1]));
  }
  *count = w;
  return P2PMG_OK;
}

int p2pmg_reset_kernel_times(p2pmg_ctx* c) {
  if (!c) return P2PMG_E_INVALID;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->n_timed = 0;
  c->n_launch = 0;
  c->n_coll = 0;
  c->coll_folded_ms = 0.0;
  c->n_coll_folded = 0;
  return P2PMG_OK;
}

int p2pmg_get_record(p2pmg_ctx* c, int which, void* host) {
  if (!c || !host) return P2PMG_E_INVALID;
  const size_t ta = (size_t)c->T * c->A;
  const size_t tra = (size_t)c->T * (c->R + 1) * c->A;
  const void* src = nullptr;
  size_t bytes = 0;
  const int slot = rec_slot(which);
  if (slot >= 0) {
    src = c->rec_f32[slot];
    bytes = ta * 4;
  } else if (which == P2PMG_REC_ACTION) {
    src = c->rec_action;
    bytes = tra;
  } else if (which == P2PMG_REC_INDEX) {
    src = c->rec_index;
    bytes = tra * 4;
  } else if (which == P2PMG_REC_LOSS) {
    src = c->rec_loss;
    bytes = ta * 4;
  } else {
    return fail(c, P2PMG_E_INVALID, "get_record: unknown record");
  }
  if (!(c->rec_last_mask & which))
    return fail(c, P2PMG_E_STATE, "get_record: the last episode launch did not record this");
  if (c->rec_fast_mask & which) {  // the last episode ran the fast / sq16 kernel: unpack its rows
    if (c->rec_stage_bytes < bytes) {
      if (c->rec_stage) (void)hipFree(c->rec_stage);
      c->rec_stage = nullptr;
      c->rec_stage_bytes = 0;
      HIP_TRY(c, hipMalloc(&c->rec_stage, bytes));
      c->rec_stage_bytes = bytes;
    }
    const int w = slot >= 0 ? slot : (which == P2PMG_REC_ACTION ? 5 : 6);
    const uint32_t tb = (uint32_t)(c->cfg.n_temp_states * c->cfg.n_balance_states);
    HIP_TRY(c, p2pmg::launch_fast_rec_unpack(c->T, c->R + 1, c->A, tb, c->rec_pack, c->rec_narrow, w, c->rec_stage,
                                             c->stream));
    src = c->rec_stage;
  }
  if (!src) return fail(c, P2PMG_E_STATE, "get_record: no record buffer");
  HIP_TRY(c, hipMemcpyAsync(host, src, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_prepass_stats(p2pmg_ctx* c, int64_t* hits, int64_t* misses) {
  if (!c) return P2PMG_E_INVALID;
  if (hits) *hits = c->spec_hits;
  if (misses) *misses = c->spec_misses;
  return P2PMG_OK;
}

// device -> caller's host memory through the pinned staging buffer (stream-ordered, then synced)
static int read_small(p2pmg_ctx* c, void* host, const void* dev, size_t bytes) {
  if (c->h_small_bytes < bytes) {
    if (c->h_small) (void)hipHostFree(c->h_small);
    c->h_small = nullptr;
    c->h_small_bytes = 0;
    HIP_TRY(c, hipHostMalloc(&c->h_small, bytes, hipHostMallocDefault));
    c->h_small_bytes = bytes;
  }
  HIP_TRY(c, hipMemcpyAsync(c->h_small, dev, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  std::memcpy(host, c->h_small, bytes);
  return P2PMG_OK;
}

int p2pmg_get_episode_reward(p2pmg_ctx* c, float* host) {
  if (!c || !host) return P2PMG_E_INVALID;
  return read_small(c, host, c->ep_reward, (size_t)c->S * 4);
}

int p2pmg_rc_step(p2pmg_ctx* c, int n, const float* t_out, const float* t_in, const float* t_m, const float* hp,
                  float* t_in_new, float* t_m_new) {
  if (!c || n < 0 || !t_out || !t_in || !t_m || !hp || !t_in_new || !t_m_new) return P2PMG_E_INVALID;
  if (n == 0) return P2PMG_OK;
  float* d = nullptr;
  HIP_TRY(c, dmalloc(&d, (size_t)6 * n));
  const size_t b = (size_t)n * 4;
  hipError_t e = hipMemcpyAsync(d, t_out, b, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d + n, t_in, b, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d + 2 * (size_t)n, t_m, b, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d + 3 * (size_t)n, hp, b, hipMemcpyHostToDevice, c->stream);
  const p2pmg_config& g = c->cfg;
  p2pmg::RcParams rc{g.inv_ci, g.inv_cm, g.inv_ri, g.inv_re, g.inv_rvent, g.one_minus_frad,
                     g.frad, g.solar_gain, g.hp_cop, g.seconds_per_minute, g.time_slot};
  if (e == hipSuccess)
    e = p2pmg::launch_rc_step(n, d, d + n, d + 2 * (size_t)n, d + 3 * (size_t)n, d + 4 * (size_t)n,
                              d + 5 * (size_t)n, rc, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(t_in_new, d + 4 * (size_t)n, b, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(t_m_new, d + 5 * (size_t)n, b, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(d);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("rc_step: ") + hipGetErrorString(e));
  return P2PMG_OK;
}

extern "C++" template <typename T, typename L>
static int div_check(p2pmg_ctx* c, int n, const T* a, const T* b, T* out, int per, L launch, const char* what) {
  if (!c || n < 0 || (n > 0 && (!a || !b || !out))) return P2PMG_E_INVALID;
  if (n == 0) return P2PMG_OK;
  T *da = nullptr, *db = nullptr, *dout = nullptr;
  hipError_t e = dmalloc(&da, (size_t)n);
  if (e == hipSuccess) e = dmalloc(&db, (size_t)n);
  if (e == hipSuccess) e = dmalloc(&dout, (size_t)n * per);
  if (e == hipSuccess) e = hipMemcpyAsync(da, a, (size_t)n * sizeof(T), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(db, b, (size_t)n * sizeof(T), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = launch(n, da, db, dout, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, (size_t)n * per * sizeof(T), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(da);
  dfree(db);
  dfree(dout);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return P2PMG_OK;
}

int p2pmg_fdiv_check(p2pmg_ctx* c, int n, const float* a, const float* b, float* out) {
  return div_check(c, n, a, b, out, 4, p2pmg::launch_fdiv_check, "fdiv_check");
}

int p2pmg_fdiv64_check(p2pmg_ctx* c, int n, const double* a, const double* b, double* out) {
  return div_check(c, n, a, b, out, 3, p2pmg::launch_fdiv64_check, "fdiv64_check");
}

int p2pmg_state_indices(p2pmg_ctx* c, int n, const float* obs, int32_t* idx) {
  if (!c || n < 0 || !obs || !idx) return P2PMG_E_INVALID;
  if (n == 0) return P2PMG_OK;
  float* d = nullptr;
  int32_t* di = nullptr;
  HIP_TRY(c, dmalloc(&d, (size_t)4 * n));
  hipError_t e = dmalloc(&di, (size_t)4 * n);
  if (e == hipSuccess) e = hipMemcpyAsync(d, obs, (size_t)16 * n, hipMemcpyHostToDevice, c->stream);
  const p2pmg_config& g = c->cfg;
  if (e == hipSuccess)
    e = p2pmg::launch_state_indices(n, d, di, g.n_time_states, g.n_temp_states, g.n_balance_states, g.n_p2p_states,
                                    c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(idx, di, (size_t)16 * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(d);
  dfree(di);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("state_indices: ") + hipGetErrorString(e));
  return P2PMG_OK;
}

int p2pmg_set_hp_levels(p2pmg_ctx* c, const float* levels) {
  if (c) c->inputs_version++;  // invalidates the speculative pre-pass slots
  if (!c || !levels) return P2PMG_E_INVALID;
  std::vector<float4> lv((size_t)c->A);
  bool ok = true;
  for (size_t a = 0; a < lv.size(); ++a) {
    lv[a] = make_float4(levels[3 * a], levels[3 * a + 1], levels[3 * a + 2], 0.0f);
    for (int k = 0; k < 3; ++k) ok &= std::fabs(levels[3 * a + k]) <= 0x1p100f;
  }
  c->hp_bounded = ok;
  HIP_TRY(c, hipMemcpyAsync(c->hp_lv, lv.data(), lv.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_set_battery(p2pmg_ctx* c, const double* capacity, double min_soc, double max_soc, double efficiency,
                      const double* soc0) {
  if (!c) return P2PMG_E_INVALID;
  c->inputs_version++;  // the fast path's pre-pass writes the N = 2 round-1 bins only without a battery
  if (!capacity) {
    c->battery = false;
    return P2PMG_OK;
  }
  if (!(efficiency > 0.0) || !(min_soc <= max_soc)) return fail(c, P2PMG_E_INVALID, "set_battery: bad parameters");
  const size_t A = (size_t)c->A;
  if (!c->bat_cap) HIP_TRY(c, dmalloc(&c->bat_cap, A));
  HIP_TRY(c, hipMemcpyAsync(c->bat_cap, capacity, A * 8, hipMemcpyHostToDevice, c->stream));
  std::vector<double> s0(A, 0.5);
  HIP_TRY(c, hipMemcpyAsync(c->soc, soc0 ? soc0 : s0.data(), A * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  {  // battery_rule_r<false>'s domain (see its comment in p2pmg_kernels.hip)
    auto in = [](double x, double lo, double hi) { return x >= lo && x <= hi; };
    const double se = std::sqrt(efficiency);
    bool ok = in(min_soc, 0x1p-100, 0x1p10) && in(max_soc, 0x1p-100, 0x1p10) && in(se, 0x1p-10, 0x1p10);
    for (size_t a = 0; a < A && ok; ++a) {
      ok = capacity[a] == 0.0 || in(capacity[a], 0x1p-20, 0x1p60);
      ok = ok && in(soc0 ? soc0[a] : 0.5, 0.0, 0x1p10);
    }
    c->bat_domain = ok;
  }
  c->battery = true;
  c->bat_min = min_soc;
  c->bat_max = max_soc;
  c->bat_sqrt_eff = std::sqrt(efficiency);  // np.sqrt(self.battery.efficiency), storage.py:86-100
  return P2PMG_OK;
}

int p2pmg_get_soc(p2pmg_ctx* c, double* soc) {
  if (!c || !soc) return P2PMG_E_INVALID;
  HIP_TRY(c, hipMemcpyAsync(soc, c->soc, (size_t)c->A * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_battery_seq(p2pmg_ctx* c, int agents, int steps, const double* bal, double* out_bal, double* soc_hist,
                      double* soc, const double* cap, double smin, double smax, double eff) {
  if (!c || agents < 0 || steps < 0 || !bal || !out_bal || !soc_hist || !soc || !cap) return P2PMG_E_INVALID;
  const size_t n = (size_t)agents * steps;
  double* d = nullptr;
  HIP_TRY(c, dmalloc(&d, 3 * n + 2 * (size_t)agents + 1));
  double *db = d, *dob = d + n, *dsh = d + 2 * n, *ds = d + 3 * n, *dc = d + 3 * n + agents;
  hipError_t e = hipMemcpyAsync(db, bal, n * 8, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(ds, soc, (size_t)agents * 8, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dc, cap, (size_t)agents * 8, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = p2pmg::launch_battery_seq(agents, steps, db, dob, dsh, ds, dc, smin, smax, std::sqrt(eff), c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out_bal, dob, n * 8, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(soc_hist, dsh, n * 8, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(soc, ds, (size_t)agents * 8, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(d);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("battery_seq: ") + hipGetErrorString(e));
  return P2PMG_OK;
}

int p2pmg_apply_q_delta(p2pmg_ctx* c) {
  if (!c) return P2PMG_E_INVALID;
  if (!c->qdelta) return fail(c, P2PMG_E_STATE, "apply_q_delta: context has no shared table");
  HIP_TRY(c, p2pmg::launch_fold_delta(c->qdelta, c->n_states * kQPad, c->stream));
  HIP_TRY(c, p2pmg::launch_apply_delta(c->q, c->qdelta, c->n_states * kQPad, c->cfg.q_dtype, c->stream));
  return P2PMG_OK;
}

int p2pmg_get_q_delta(p2pmg_ctx* c, int64_t* host) {
  if (!c || !host) return P2PMG_E_INVALID;
  if (!c->qdelta) return fail(c, P2PMG_E_STATE, "get_q_delta: context has no shared table");
  const int na = c->cfg.n_actions;
  std::vector<long long> h(c->n_states * kQPad);
  HIP_TRY(c, p2pmg::launch_fold_delta(c->qdelta, c->n_states * kQPad, c->stream));
  HIP_TRY(c, hipMemcpyAsync(h.data(), c->qdelta, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (size_t r = 0; r < c->n_states; ++r)
    for (int k = 0; k < na; ++k) host[r * na + k] = h[r * kQPad + k];
  return P2PMG_OK;
}

int p2pmg_set_q_delta(p2pmg_ctx* c, const int64_t* host) {
  if (!c || !host) return P2PMG_E_INVALID;
  if (!c->qdelta) return fail(c, P2PMG_E_STATE, "set_q_delta: context has no shared table");
  const int na = c->cfg.n_actions;
  std::vector<long long> h(c->n_states * kQPad, 0);
  for (size_t r = 0; r < c->n_states; ++r)
    for (int k = 0; k < na; ++k) h[r * kQPad + k] = host[r * na + k];
  HIP_TRY(c, hipMemsetAsync(c->qdelta, 0, p2pmg::kDeltaCopies * h.size() * 8, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->qdelta, h.data(), h.size() * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_comm_unique_id(uint8_t id[128]) {
  if (!id) return P2PMG_E_INVALID;
  Rccl* r = rccl();
  if (!r) return P2PMG_E_UNSUPPORTED;
  return r->getUniqueId(id) == 0 ? P2PMG_OK : P2PMG_E_HIP;
}

int p2pmg_comm_init(p2pmg_ctx* c, const uint8_t id[128], int rank, int nranks) {
  if (!c || !id || rank < 0 || nranks <= 0 || rank >= nranks) return P2PMG_E_INVALID;
  Rccl* r = rccl();
  if (!r) return fail(c, P2PMG_E_UNSUPPORTED, "RCCL (librccl.so) not found");
  HIP_TRY(c, hipSetDevice(c->device));
  Id128 uid;
  std::memcpy(uid.b, id, 128);
  void* comm = nullptr;
  const int rc = r->commInitRank(&comm, nranks, uid, rank);
  if (rc != 0) return fail(c, P2PMG_E_HIP, std::string("ncclCommInitRank: ") + (r->getErrorString ? r->getErrorString(rc) : "?"));
  c->comm = comm;
  c->rank = rank;
  c->nranks = nranks;
  return P2PMG_OK;
}

// HIP events around each data-path all-reduce (shared-table delta, DQN gradient), on the context's
// stream, so the bench line can report what the exchange step costs at world > 1
static hipError_t coll_mark(p2pmg_ctx* c, int end) {
  if (c->cring.empty()) {
    c->cring.assign(2 * p2pmg_ctx::kCRing, nullptr);
    for (auto& ev : c->cring) {
      const hipError_t e = hipEventCreate(&ev);
      if (e != hipSuccess) return e;
    }
  }
  const int slot = (int)(c->n_coll % p2pmg_ctx::kCRing);
  if (!end && c->n_coll >= p2pmg_ctx::kCRing && c->n_coll_folded == c->n_coll - p2pmg_ctx::kCRing) {
    // the slot's previous pair (kCRing collectives ago) is about to be overwritten: fold its
    // duration into the running total first, so p2pmg_collective_ms counts every collective.
    // Once per collective: a start whose collective then failed (no end mark, n_coll unchanged)
    // is followed by another start on the same slot, which must not fold the slot again
    float ms = 0.0f;
    hipError_t e = hipEventSynchronize(c->cring[2 * slot + 1]);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, c->cring[2 * slot], c->cring[2 * slot + 1]);
    if (e != hipSuccess) return e;
    c->coll_folded_ms += ms;
    c->n_coll_folded++;
  }
  const hipError_t e = hipEventRecord(c->cring[2 * slot + end], c->stream);
  if (end) c->n_coll++;
  return e;
}

int p2pmg_collective_ms(p2pmg_ctx* c, double* total_ms, int* count) {
  if (!c || !total_ms || !count) return P2PMG_E_INVALID;
  const long long n = c->n_coll < p2pmg_ctx::kCRing ? c->n_coll : p2pmg_ctx::kCRing;
  double sum = 0.0;
  for (long long k = c->n_coll - n; k < c->n_coll; ++k) {
    const int slot = (int)(k % p2pmg_ctx::kCRing);
    float ms = 0.0f;
    HIP_TRY(c, hipEventSynchronize(c->cring[2 * slot + 1]));
    HIP_TRY(c, hipEventElapsedTime(&ms, c->cring[2 * slot], c->cring[2 * slot + 1]));
    sum += ms;
  }
  *total_ms = c->coll_folded_ms + sum;
  *count = (int)c->n_coll;
  return P2PMG_OK;
}

int p2pmg_allreduce_q_delta(p2pmg_ctx* c) {
  if (!c) return P2PMG_E_INVALID;
  if (!c->qdelta) return fail(c, P2PMG_E_STATE, "allreduce_q_delta: context has no shared table");
  if (!c->comm) return fail(c, P2PMG_E_STATE, "allreduce_q_delta: p2pmg_comm_init first");
  Rccl* r = rccl();
  // ncclInt64 = 4, ncclSum = 0 (rccl.h)
  HIP_TRY(c, p2pmg::launch_fold_delta(c->qdelta, c->n_states * kQPad, c->stream));
  HIP_TRY(c, coll_mark(c, 0));
  const int rc = r->allReduce(c->qdelta, c->qdelta, c->n_states * kQPad, 4, 0, c->comm, c->stream);
  if (rc != 0) return fail(c, P2PMG_E_HIP, std::string("ncclAllReduce: ") + (r->getErrorString ? r->getErrorString(rc) : "?"));
  HIP_TRY(c, coll_mark(c, 1));
  return P2PMG_OK;
}

int p2pmg_comm_nranks(p2pmg_ctx* c, int* n) {
  if (!c || !n) return P2PMG_E_INVALID;
  if (!c->comm) {
    *n = 1;  // no communicator: a world of one
    return P2PMG_OK;
  }
  Rccl* r = rccl();
  if (!r->commCount) return fail(c, P2PMG_E_UNSUPPORTED, "ncclCommCount not found");
  const int rc = r->commCount(c->comm, n);
  if (rc != 0) return fail(c, P2PMG_E_HIP, std::string("ncclCommCount: ") + (r->getErrorString ? r->getErrorString(rc) : "?"));
  return P2PMG_OK;
}

int p2pmg_allreduce_metrics(p2pmg_ctx* c, double* out) {
  if (!c || !out) return P2PMG_E_INVALID;
  if (!c->ep_reward) return fail(c, P2PMG_E_STATE, "allreduce_metrics: no episode launched");
  if (!c->d_metrics) HIP_TRY(c, dmalloc(&c->d_metrics, 2));
  HIP_TRY(c, p2pmg::launch_metrics(c->S, c->ep_reward, c->d_metrics, c->stream));
  if (c->comm) {  // ncclFloat64 = 8, ncclSum = 0: sum and count over every rank (xGMI)
    Rccl* r = rccl();
    const int rc = r->allReduce(c->d_metrics, c->d_metrics, 2, 8, 0, c->comm, c->stream);
    if (rc != 0) return fail(c, P2PMG_E_HIP, std::string("ncclAllReduce(metrics): ") + (r->getErrorString ? r->getErrorString(rc) : "?"));
  }
  return read_small(c, out, c->d_metrics, 16);
}

int p2pmg_table_hash_allgather(p2pmg_ctx* c, uint64_t* out) {
  if (!c || !out) return P2PMG_E_INVALID;
  if (!c->q) return fail(c, P2PMG_E_STATE, "table_hash: context has no Q-table");
  const int n = c->comm ? c->nranks : 1;
  if (n > 1024) return fail(c, P2PMG_E_UNSUPPORTED, "table_hash: more than 1024 ranks");
  if (!c->d_hash) HIP_TRY(c, dmalloc(&c->d_hash, 1025));
  const size_t bytes = (c->cfg.shared_q ? (size_t)1 : (size_t)c->A) * c->n_states * kQPad * c->q_elem;
  HIP_TRY(c, p2pmg::launch_table_hash(c->q, bytes, c->d_hash + 1024, c->stream));
  if (c->comm) {  // ncclUint64 = 5: every rank's fingerprint, in rank order
    Rccl* r = rccl();
    if (!r->allGather) return fail(c, P2PMG_E_UNSUPPORTED, "ncclAllGather not found");
    const int rc = r->allGather(c->d_hash + 1024, c->d_hash, 1, 5, c->comm, c->stream);
    if (rc != 0) return fail(c, P2PMG_E_HIP, std::string("ncclAllGather: ") + (r->getErrorString ? r->getErrorString(rc) : "?"));
  } else {
    HIP_TRY(c, hipMemcpyAsync(c->d_hash, c->d_hash + 1024, 8, hipMemcpyDeviceToDevice, c->stream));
  }
  HIP_TRY(c, hipMemcpyAsync(out, c->d_hash, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_comm_destroy(p2pmg_ctx* c) {
  if (!c) return P2PMG_E_INVALID;
  if (c->comm && rccl()) rccl()->commDestroy(c->comm);
  c->comm = nullptr;
  if (!c->xfn) c->rank = 0, c->nranks = 1;
  return P2PMG_OK;
}

int p2pmg_q_calls(p2pmg_ctx* c, int n, const int32_t* agents, const float* s_obs, const uint8_t* codes,
                  const float* rewards, const float* ns_obs, int train, int32_t* actions_out, double* q_out) {
  if (!c || n < 0 || !agents || !s_obs || !codes || !actions_out || !q_out) return P2PMG_E_INVALID;
  if (train && (!rewards || !ns_obs)) return fail(c, P2PMG_E_INVALID, "q_calls: train needs rewards and ns_obs");
  if (c->dqn) return fail(c, P2PMG_E_STATE, "q_calls: DQN context has no Q-table");
  for (int k = 0; k < n; ++k)
    if (agents[k] < 0 || agents[k] >= c->A) return fail(c, P2PMG_E_INVALID, "q_calls: agent out of range");
  if (n == 0) return P2PMG_OK;
  // one staging block: agents | s_obs | ns_obs | rewards | codes | actions | q_out
  const size_t nb = (size_t)n;
  const size_t off_s = 0, off_ns = off_s + 16 * nb, off_r = off_ns + 16 * nb, off_a = off_r + 4 * nb,
               off_act = off_a + 4 * nb, off_q = ((off_act + 4 * nb + 7) / 8) * 8, off_c = off_q + 8 * nb,
               total = off_c + nb;
  char* d = nullptr;
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&d), total));
  hipError_t e = hipMemcpyAsync(d + off_s, s_obs, 16 * nb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess && train) e = hipMemcpyAsync(d + off_ns, ns_obs, 16 * nb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess && train) e = hipMemcpyAsync(d + off_r, rewards, 4 * nb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d + off_a, agents, 4 * nb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d + off_c, codes, nb, hipMemcpyHostToDevice, c->stream);
  const p2pmg_config& g = c->cfg;
  p2pmg::QCallParams p{n, train ? 1 : 0, g.q_dtype, reinterpret_cast<const int32_t*>(d + off_a),
                       reinterpret_cast<const float*>(d + off_s), reinterpret_cast<const uint8_t*>(d + off_c),
                       reinterpret_cast<const float*>(d + off_r), reinterpret_cast<const float*>(d + off_ns),
                       reinterpret_cast<int32_t*>(d + off_act), reinterpret_cast<double*>(d + off_q), c->q,
                       (uint32_t)c->n_states, g.n_time_states, g.n_temp_states, g.n_balance_states, g.n_p2p_states,
                       g.alpha, g.gamma};
  if (e == hipSuccess) e = p2pmg::launch_q_calls(p, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(actions_out, d + off_act, 4 * nb, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(q_out, d + off_q, 8 * nb, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("q_calls: ") + hipGetErrorString(e));
  return P2PMG_OK;
}

int p2pmg_replay_decode(const uint32_t* words, size_t n_words, size_t n_decisions, const double* eps, size_t n_eps,
                        uint8_t* codes, size_t* consumed) {
  if (!words || !eps || n_eps == 0 || !codes) return P2PMG_E_INVALID;
  size_t pos = 0;
  for (size_t k = 0; k < n_decisions; ++k) {
    // RandomState.rand(): (a * 2^26 + b) / 2^53 with a = w0 >> 5, b = w1 >> 6 (mt19937 next_double)
    if (pos + 2 > n_words) return P2PMG_E_INVALID;
    const uint32_t a = words[pos] >> 5, b = words[pos + 1] >> 6;
    pos += 2;
    const double u = ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
    if (u < eps[k % n_eps]) {
      // RandomState.choice(3) -> randint(0, 3): masked rejection, mask 3, one word per try
      uint32_t v;
      do {
        if (pos >= n_words) return P2PMG_E_INVALID;
        v = words[pos++] & 3u;
      } while (v > 2u);
      codes[k] = (uint8_t)v;
    } else {
      codes[k] = P2PMG_GREEDY;
    }
  }
  if (consumed) *consumed = pos;
  return P2PMG_OK;
}

// ============================================================================ DQN learner
int p2pmg_dqn_config_default(p2pmg_dqn_config* cfg) {
  if (!cfg) return P2PMG_E_INVALID;
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->gamma = 0.95;  // agent.py:309
  cfg->tau = 0.005;
  cfg->lr = 1e-5;     // agent.py:310
  cfg->beta1 = 0.9;
  cfg->beta2 = 0.999;
  cfg->adam_eps = 1e-7;
  cfg->clip = 1.0;    // rl.py:329
  cfg->batch = 32;    // agent.py:308
  cfg->capacity = 5000;
  cfg->agents_per_block = 0;
  return P2PMG_OK;
}

int p2pmg_dqn_setup(p2pmg_ctx* c, const p2pmg_dqn_config* cfg) {
  if (!c || !cfg) return P2PMG_E_INVALID;
  if (!c->dqn) return fail(c, P2PMG_E_STATE, "dqn_setup: create the context with learner = P2PMG_LEARNER_DQN");
  if (cfg->batch != p2pmg::kDqnBatch) return fail(c, P2PMG_E_UNSUPPORTED, "dqn_setup: batch must be 32");
  if (cfg->capacity < p2pmg::kDqnBatch || cfg->capacity > 65535)
    return fail(c, P2PMG_E_INVALID, "dqn_setup: capacity must be in [32, 65535]");
  if (c->d_theta) return fail(c, P2PMG_E_STATE, "dqn_setup: already set up");
  c->dcfg = *cfg;
  const size_t A = (size_t)c->A, NS = p2pmg::kNetStride;
  c->n_nets = c->cfg.shared_q ? 1 : c->A;
  const size_t nn = (size_t)c->n_nets * NS;
  HIP_TRY(c, dmalloc(&c->d_theta, nn));
  HIP_TRY(c, dmalloc(&c->d_target, nn));
  HIP_TRY(c, dmalloc(&c->d_m, nn));
  HIP_TRY(c, dmalloc(&c->d_v, nn));
  for (float* b : {c->d_theta, c->d_target, c->d_m, c->d_v}) HIP_TRY(c, hipMemsetAsync(b, 0, nn * 4, c->stream));
  if (cfg->agents_per_block < 0 || cfg->grad_segments < 0) return fail(c, P2PMG_E_INVALID, "dqn_setup: negative layout");
  if (c->cfg.shared_q) {
    // gradient segments: contiguous runs of whole scenarios; the train workgroups never straddle two
    const int G = cfg->grad_segments > 0 ? cfg->grad_segments : 1;
    if (c->S % G) return fail(c, P2PMG_E_INVALID, "dqn_setup: grad_segments must divide the scenarios");
    c->d_seg_local = G;
    c->d_seg_agents = c->A / G;
    // default: one wave of train workgroups (2 per CU in the default build: 512 on 256 CUs)
    const size_t slots = (size_t)c->n_cu * (size_t)p2pmg::dqn_train_blocks_per_cu();
    int apb = cfg->agents_per_block > 0 ? cfg->agents_per_block : (int)((A + slots - 1) / slots);
    c->d_apb = apb < 1 ? 1 : apb;
    c->d_bps = (c->d_seg_agents + c->d_apb - 1) / c->d_apb;
    c->d_blocks = G * c->d_bps;
    HIP_TRY(c, dmalloc(&c->d_grad, (size_t)c->d_blocks * NS));
    HIP_TRY(c, dmalloc(&c->d_alt, 4 * NS));
  } else {
    c->d_apb = 1;
    c->d_blocks = c->A;
    c->d_seg_local = 1;
    c->d_seg_agents = c->A;
    c->d_bps = c->A;
  }
  HIP_TRY(c, dmalloc(&c->d_buf, A * (size_t)cfg->capacity * p2pmg::kTrans));
  HIP_TRY(c, dmalloc(&c->d_added, A));
  HIP_TRY(c, dmalloc(&c->d_smp, A * p2pmg::kDqnBatch));
  HIP_TRY(c, hipMemsetAsync(c->d_added, 0, A * 4, c->stream));
  HIP_TRY(c, dmalloc(&c->d_ep_acc, (size_t)c->S));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->d_steps.assign((size_t)c->n_nets, 0);
  c->d_added_min = 0;
  return P2PMG_OK;
}

static float* dqn_array(p2pmg_ctx* c, int which) {
  switch (which) {
    case P2PMG_DQN_ONLINE: return c->d_theta;
    case P2PMG_DQN_TARGET: return c->d_target;
    case P2PMG_DQN_ADAM_M: return c->d_m;
    case P2PMG_DQN_ADAM_V: return c->d_v;
    default: return nullptr;
  }
}

static int dqn_ready(p2pmg_ctx* c, const char* what) {
  if (!c) return P2PMG_E_INVALID;
  if (!c->dqn || !c->d_theta) return fail(c, P2PMG_E_STATE, std::string(what) + ": p2pmg_dqn_setup first");
  return P2PMG_OK;
}

int p2pmg_dqn_set_weights(p2pmg_ctx* c, int which, int first, int count, const float* host) {
  int rc = dqn_ready(c, "dqn_set_weights");
  if (rc != P2PMG_OK) return rc;
  float* dst = dqn_array(c, which);
  if (!dst || !host || first < 0 || count < 0 || first + count > c->n_nets)
    return fail(c, P2PMG_E_INVALID, "dqn_set_weights: bad array/range");
  HIP_TRY(c, hipMemcpy2DAsync(dst + (size_t)first * p2pmg::kNetStride, p2pmg::kNetStride * 4, host,
                              p2pmg::kDqnParams * 4, p2pmg::kDqnParams * 4, count, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_dqn_get_weights(p2pmg_ctx* c, int which, int first, int count, float* host) {
  int rc = dqn_ready(c, "dqn_get_weights");
  if (rc != P2PMG_OK) return rc;
  const float* src = dqn_array(c, which);
  if (!src || !host || first < 0 || count < 0 || first + count > c->n_nets)
    return fail(c, P2PMG_E_INVALID, "dqn_get_weights: bad array/range");
  HIP_TRY(c, hipMemcpy2DAsync(host, p2pmg::kDqnParams * 4, src + (size_t)first * p2pmg::kNetStride,
                              p2pmg::kNetStride * 4, p2pmg::kDqnParams * 4, count, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_dqn_set_step(p2pmg_ctx* c, int64_t step) {
  int rc = dqn_ready(c, "dqn_set_step");
  if (rc != P2PMG_OK) return rc;
  if (step < 0) return P2PMG_E_INVALID;
  std::fill(c->d_steps.begin(), c->d_steps.end(), step);  // every network
  return P2PMG_OK;
}

int p2pmg_dqn_get_step(p2pmg_ctx* c, int64_t* step) {
  int rc = dqn_ready(c, "dqn_get_step");
  if (rc != P2PMG_OK) return rc;
  if (!step) return P2PMG_E_INVALID;
  *step = c->d_steps[0];
  return P2PMG_OK;
}

int p2pmg_dqn_get_net_steps(p2pmg_ctx* c, int first, int count, int64_t* steps) {
  int rc = dqn_ready(c, "dqn_get_net_steps");
  if (rc != P2PMG_OK) return rc;
  if (!steps || first < 0 || count < 0 || first + count > c->n_nets) return fail(c, P2PMG_E_INVALID, "dqn_get_net_steps");
  for (int k = 0; k < count; ++k) steps[k] = c->d_steps[(size_t)first + k];
  return P2PMG_OK;
}

int p2pmg_dqn_set_samples(p2pmg_ctx* c, const uint16_t* samples) {
  int rc = dqn_ready(c, "dqn_set_samples");
  if (rc != P2PMG_OK) return rc;
  if (!samples) return P2PMG_E_INVALID;
  const size_t n = (size_t)c->T * c->A * p2pmg::kDqnBatch;
  if (!c->d_samples) HIP_TRY(c, dmalloc(&c->d_samples, n));
  HIP_TRY(c, hipMemcpyAsync(c->d_samples, samples, n * 2, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->have_samples = true;
  return P2PMG_OK;
}

static int dqn_refresh_added_min(p2pmg_ctx* c) {
  std::vector<int32_t> h(c->A);
  HIP_TRY(c, hipMemcpyAsync(h.data(), c->d_added, (size_t)c->A * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  int64_t m = INT64_MAX;
  for (int32_t v : h) m = v < m ? v : m;
  c->d_added_min = c->A ? m : 0;
  return P2PMG_OK;
}

int p2pmg_dqn_get_buffer(p2pmg_ctx* c, int first, int count, float* host, int32_t* added) {
  int rc = dqn_ready(c, "dqn_get_buffer");
  if (rc != P2PMG_OK) return rc;
  if (first < 0 || count < 0 || first + count > c->A) return fail(c, P2PMG_E_INVALID, "dqn_get_buffer: range");
  const size_t per = (size_t)c->dcfg.capacity * p2pmg::kTrans;
  if (host)
    HIP_TRY(c, hipMemcpyAsync(host, c->d_buf + (size_t)first * per, (size_t)count * per * 4, hipMemcpyDeviceToHost,
                              c->stream));
  if (added)
    HIP_TRY(c, hipMemcpyAsync(added, c->d_added + first, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return P2PMG_OK;
}

int p2pmg_dqn_set_buffer(p2pmg_ctx* c, int first, int count, const float* host, const int32_t* added) {
  int rc = dqn_ready(c, "dqn_set_buffer");
  if (rc != P2PMG_OK) return rc;
  if (first < 0 || count < 0 || first + count > c->A) return fail(c, P2PMG_E_INVALID, "dqn_set_buffer: range");
  const size_t per = (size_t)c->dcfg.capacity * p2pmg::kTrans;
  if (host)
    HIP_TRY(c, hipMemcpyAsync(c->d_buf + (size_t)first * per, host, (size_t)count * per * 4, hipMemcpyHostToDevice,
                              c->stream));
  if (added)
    HIP_TRY(c, hipMemcpyAsync(c->d_added + first, added, (size_t)count * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return dqn_refresh_added_min(c);
}

static p2pmg::DqnParams dqn_params(p2pmg_ctx* c, const EpisodeParams& e) {
  p2pmg::DqnParams d{};
  const p2pmg_dqn_config& q = c->dcfg;
  d.e = e;
  d.n_nets = c->n_nets;
  d.theta = c->d_theta;
  d.target = c->d_target;
  d.adam_m = c->d_m;
  d.adam_v = c->d_v;
  d.grad = c->d_grad;
  d.smp = c->d_smp;
  d.segs = c->d_segs;
  d.seg_first = c->rank * c->d_seg_local;
  d.n_segs = c->nranks * c->d_seg_local;
  d.seg_agents = c->d_seg_agents;
  d.bps = c->d_bps;
  d.buf = c->d_buf;
  d.added = c->d_added;
  d.cap = q.capacity;
  d.samples = nullptr;
  d.rec_loss = (e.record & P2PMG_REC_LOSS) ? c->rec_loss : nullptr;
  d.ep_acc = c->d_ep_acc;
  d.gamma = (float)q.gamma;
  d.tau = (float)q.tau;
  d.tau_c = 1.0f - (float)q.tau;
  d.b1c = 1.0f - (float)q.beta1;
  d.b2c = 1.0f - (float)q.beta2;
  d.adam_eps = (float)q.adam_eps;
  d.clip = (float)q.clip;
  d.inv_agents = 1.0f / (float)((double)c->A * c->nranks);
  d.apb = c->d_apb;
  d.theta_out = d.theta;  // the Adam steps store in place unless the episode loop binds the double buffer
  d.target_out = d.target;
  d.m_out = d.adam_m;
  d.v_out = d.adam_v;
  d.adam_pending = 0;
  d.fold_spt = 0;  // auto (launch_dqn_reduce_adam)
  d.adam_tpb = 256;
  return d;
}

// the network state an Adam step reads (in) and writes (out): online, target, m, v
static void dqn_bind(p2pmg::DqnParams& d, float* const in[4], float* const out[4]) {
  d.theta = in[0];
  d.target = in[1];
  d.adam_m = in[2];
  d.adam_v = in[3];
  d.theta_out = out[0];
  d.target_out = out[1];
  d.m_out = out[2];
  d.v_out = out[3];
}

// Keras Adam step size for iteration `step` (1-based), float64 -> float32 (oracle/dqn.py::adam_lr)
static float adam_lr(const p2pmg_dqn_config& q, int64_t step) {
  const double t = (double)step;
  return (float)(q.lr * std::sqrt(1.0 - std::pow(q.beta2, t)) / (1.0 - std::pow(q.beta1, t)));
}

static bool dqn_steps_same(const p2pmg_ctx* c) {
  for (int64_t st : c->d_steps)
    if (st != c->d_steps[0]) return false;
  return true;
}

// p2pmg_dqn_train_batch advanced some networks on their own, so their Adam step counts differ.
// Every env step advances every network by one, so an episode's per-network step sizes are known
// up front: one [T][n_nets] table, uploaded once per episode (not a copy + sync per env step).
static int dqn_upload_lr_table(p2pmg_ctx* c) {
  const size_t n = c->d_steps.size(), need = (size_t)c->T * n;
  if (c->d_lr_cap < need) {
    dfree(c->d_lr);
    c->d_lr = nullptr;
    c->d_lr_cap = 0;
    HIP_TRY(c, dmalloc(&c->d_lr, need));
    c->d_lr_cap = need;
  }
  c->h_lr.resize(need);
  for (int t = 0; t < c->T; ++t)
    for (size_t k = 0; k < n; ++k) c->h_lr[(size_t)t * n + k] = adam_lr(c->dcfg, c->d_steps[k] + 1 + t);
  HIP_TRY(c, hipMemcpyAsync(c->d_lr, c->h_lr.data(), need * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));  // h_lr is rewritten by the next such episode
  return P2PMG_OK;
}

// The shared network's gradient segments of every rank in d_segs ([nranks * d_seg_local][kNetStride]),
// allocated for the current world (comm_init / set_exchange may come after dqn_setup)
static int dqn_ensure_segs(p2pmg_ctx* c, p2pmg::DqnParams& d) {
  const size_t need = (size_t)c->nranks * c->d_seg_local * p2pmg::kNetStride;
  if (c->d_segs_cap < need) {
    dfree(c->d_segs);
    c->d_segs_cap = 0;
    HIP_TRY(c, dmalloc(&c->d_segs, need));
    c->d_segs_cap = need;
  }
  if (c->xfn && !c->comm && c->h_segs_cap < need) {
    if (c->h_segs) (void)hipHostFree(c->h_segs);
    c->h_segs = nullptr;
    c->h_segs_cap = 0;
    HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_segs), need * 4, hipHostMallocDefault));
    c->h_segs_cap = need;
  }
  d.segs = c->d_segs;
  d.seg_first = c->rank * c->d_seg_local;
  d.n_segs = c->nranks * c->d_seg_local;
  return P2PMG_OK;
}

// every rank's segments into d_segs: RCCL all-gather in place (xGMI), or the host exchange function
static int dqn_gather_segments(p2pmg_ctx* c) {
  const size_t per = (size_t)c->d_seg_local * p2pmg::kNetStride;  // floats per rank
  if (c->comm) {
    Rccl* r = rccl();
    if (!r->allGather) return fail(c, P2PMG_E_UNSUPPORTED, "ncclAllGather not found");
    // ncclFloat32 = 7; in place: this rank's part already sits at d_segs + rank * per
    HIP_TRY(c, coll_mark(c, 0));
    const int rc = r->allGather(c->d_segs + (size_t)c->rank * per, c->d_segs, per, 7, c->comm, c->stream);
    if (rc != 0) return fail(c, P2PMG_E_HIP, std::string("dqn gradient all-gather: ") +
                                                 (r->getErrorString ? r->getErrorString(rc) : "?"));
    HIP_TRY(c, coll_mark(c, 1));
    return P2PMG_OK;
  }
  if (!c->xfn) return fail(c, P2PMG_E_STATE, "dqn: several ranks but neither a communicator nor an exchange");
  float* own = c->h_segs + (size_t)c->rank * per;
  HIP_TRY(c, hipMemcpyAsync(own, c->d_segs + (size_t)c->rank * per, per * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (c->xfn(c->xuser, c->h_segs, (int64_t)per, c->rank, c->nranks) != 0)
    return fail(c, P2PMG_E_STATE, "dqn: the host gradient exchange failed");
  HIP_TRY(c, hipMemcpyAsync(c->d_segs, c->h_segs, (size_t)c->nranks * per * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));  // h_segs is rewritten by the next env step
  return P2PMG_OK;
}

// defer (the shared network's split path, act kernel able to fuse it): the post-exchange Adam step is
// left pending (d.adam_pending) for the next env step's act launch, or the episode loop's settle
static int dqn_train_step(p2pmg_ctx* c, p2pmg::DqnParams& d, bool same, bool defer) {
  // one env step trains every network once (community.py:158-168); the Adam step counters advance
  // only once every launch of the step is enqueued (a failed exchange leaves weights and counters
  // at the previous step: the Adam launch that would change the weights was not issued)
  d.lr_t = adam_lr(c->dcfg, c->d_steps[0] + 1);
  d.lr_net = same ? nullptr : c->d_lr + (size_t)d.t * c->d_steps.size();
  if (!d.fused_sample) HIP_TRY(c, p2pmg::launch_dqn_sample(d, c->stream));
  if (c->n_nets == 1) {
    HIP_TRY(c, p2pmg::launch_dqn_train(d, c->d_blocks, true, c->stream));
    if (c->nranks == 1 && c->d_seg_local == 1) {  // one segment in all: its sum + Adam in one launch
      HIP_TRY(c, p2pmg::launch_dqn_reduce_adam(d, 1, true, c->stream));
    } else {
      HIP_TRY(c, p2pmg::launch_dqn_reduce_adam(d, c->d_seg_local, false, c->stream));
      if (c->nranks > 1 || c->comm) {  // a communicator gathers even at world 1 (the RCCL path, tested)
        const int rc = dqn_gather_segments(c);
        if (rc != P2PMG_OK) return rc;
      }
      if (defer) d.adam_pending = 1;
      else HIP_TRY(c, p2pmg::launch_dqn_adam_shared(d, c->stream));
    }
  } else {
    HIP_TRY(c, p2pmg::launch_dqn_train(d, c->A, false, c->stream));
  }
  for (auto& st : c->d_steps) ++st;
  return P2PMG_OK;
}

static int dqn_run_episode(p2pmg_ctx* c, const p2pmg_episode_args* args) {
  c->rec_fast_mask = 0;
  int rc = dqn_ready(c, "run_episode");
  if (rc != P2PMG_OK) return rc;
  const int mode = args->mode;
  if (mode != P2PMG_MODE_TRAIN && mode != P2PMG_MODE_GREEDY && mode != P2PMG_MODE_FILL)
    return fail(c, P2PMG_E_INVALID, "mode");
  const bool acting = mode != P2PMG_MODE_GREEDY;
  if (acting && args->rng != P2PMG_RNG_REPLAY && args->rng != P2PMG_RNG_PHILOX) return fail(c, P2PMG_E_INVALID, "rng");
  if (acting && args->rng == P2PMG_RNG_REPLAY && !c->have_codes)
    return fail(c, P2PMG_E_STATE, "run_episode: replay mode needs p2pmg_set_replay_codes");
  if (mode == P2PMG_MODE_TRAIN && args->rng == P2PMG_RNG_REPLAY && !c->have_samples)
    return fail(c, P2PMG_E_STATE, "run_episode: DQN replay training needs p2pmg_dqn_set_samples");
  if (mode == P2PMG_MODE_TRAIN && c->d_added_min + 1 < p2pmg::kDqnBatch)
    return fail(c, P2PMG_E_STATE, "run_episode: fill the replay memory first (>= 31 transitions per agent, "
                                  "community.init_buffers)");
  rc = ensure_records(c, args->record);
  if (rc != P2PMG_OK) return rc;
  EpisodeParams e = episode_params(c, args);
  e.rng = (acting && args->rng == P2PMG_RNG_PHILOX) ? 1 : 0;
  p2pmg::DqnParams d = dqn_params(c, e);
  if (mode == P2PMG_MODE_TRAIN && args->rng == P2PMG_RNG_REPLAY) d.samples = c->d_samples;
  if (mode == P2PMG_MODE_TRAIN && c->n_nets == 1 && (c->nranks > 1 || c->d_seg_local > 1)) {
    rc = dqn_ensure_segs(c, d);
    if (rc != P2PMG_OK) return rc;
  }
  if (c->ring.empty()) {
    c->ring.assign(2 * p2pmg_ctx::kRing, nullptr);
    for (auto& ev : c->ring) HIP_TRY(c, hipEventCreate(&ev));
  }
  d.fused_sample = (mode == P2PMG_MODE_TRAIN) ? 1 : 0;  // the act launch of each env step draws the samples
  {  // P2PMG_DQN_ACT=wave: the one-wave-per-agent act kernel for a shared network too (tests, A/B)
    const char* v = getenv("P2PMG_DQN_ACT");
    d.act_wave = (v && !strcmp(v, "wave")) ? 1 : 0;
    const char* g = getenv("P2PMG_ACT_AGW");  // 8: the 8-slot MFMA act workgroups (tests, A/B)
    d.act_agw = (g && atoi(g) == 8) ? 8 : 16;
    const char* f = getenv("P2PMG_FOLD_SPT");  // segment fold runs per thread: 1, 2, 4, 8, 16 (A/B); else auto
    const int fs = f ? atoi(f) : 0;
    d.fold_spt = (fs == 1 || fs == 2 || fs == 4 || fs == 8 || fs == 16) ? fs : 0;
    const char* at = getenv("P2PMG_ADAM_TPB");  // post-exchange Adam workgroup size: 64, 128, 256 (default)
    d.adam_tpb = at ? atoi(at) : 256;
  }
  c->last_kernel = std::string(c->n_nets == 1 && !d.act_wave ? "dqn_act_shared_kernel<" : "dqn_act_kernel<") +
                   std::to_string(c->N) + ">";
  const bool same = mode != P2PMG_MODE_TRAIN || dqn_steps_same(c);
  if (!same) {
    rc = dqn_upload_lr_table(c);
    if (rc != P2PMG_OK) return rc;
  }
  // The shared network's split path (segments / ranks): env step t's post-exchange Adam step runs
  // inside env step t + 1's act launch, which reads the state from one half of a double buffer and
  // stores the stepped state into the other (every act workgroup needs the new weights; workgroup 0
  // stores them); the episode's last step, or any early return, settles into the primary arrays.
  // Opt-in (P2PMG_DQN_ADAM=act): measured on the MI355X the fused form costs the act launch far more
  // than the standalone Adam launch it saves, so the default is that launch.
  const char* adam_env = getenv("P2PMG_DQN_ADAM");
  const bool defer = mode == P2PMG_MODE_TRAIN && c->n_nets == 1 && (c->nranks > 1 || c->d_seg_local > 1) &&
                     c->d_alt && p2pmg::dqn_act_fuses_adam(d) && adam_env && !strcmp(adam_env, "act");
  const size_t NS = p2pmg::kNetStride;
  float* const prim[4] = {c->d_theta, c->d_target, c->d_m, c->d_v};
  float* const alt[4] = {c->d_alt, c->d_alt + NS, c->d_alt + 2 * NS, c->d_alt + 3 * NS};
  bool on_alt = false;  // the current state sits in the alt half
  auto settle = [&]() -> int {
    float* const* cur = on_alt ? alt : prim;
    if (d.adam_pending) {  // the pending step, from the current half into the primary arrays
      dqn_bind(d, cur, prim);
      d.adam_pending = 0;
      HIP_TRY(c, p2pmg::launch_dqn_adam_shared(d, c->stream));
    } else if (on_alt) {
      for (int k = 0; k < 4; ++k)
        HIP_TRY(c, hipMemcpyAsync(prim[k], alt[k], NS * 4, hipMemcpyDeviceToDevice, c->stream));
    }
    on_alt = false;
    dqn_bind(d, prim, prim);
    return P2PMG_OK;
  };
  const int slot = (int)(c->n_timed % p2pmg_ctx::kRing);
  HIP_TRY(c, hipEventRecord(c->ring[2 * slot], c->stream));
  // Philox training: every env step's replay draws in one throughput launch ahead of the episode,
  // read by the act launches like uploaded samples (P2PMG_DQN_SAMPLE_PREPASS=0: drawn in each act
  // launch's tail, as the episode's first form did)
  {
    const char* px_env = getenv("P2PMG_DQN_SAMPLE_PREPASS");
    const bool no_px = px_env && !strcmp(px_env, "0");
    const size_t n = (size_t)c->T * c->A * p2pmg::kDqnBatch;
    if (mode == P2PMG_MODE_TRAIN && args->rng == P2PMG_RNG_PHILOX && !no_px && n <= ((size_t)1 << 30)) {
      if (!c->d_samples_px) HIP_TRY(c, dmalloc(&c->d_samples_px, n));
      HIP_TRY(c, p2pmg::launch_dqn_sample_prepass(d, c->d_samples_px, c->stream));
      d.samples = c->d_samples_px;
    }
  }
  for (int t = 0; t < c->T; ++t) {
    d.t = t;
    d.e.mode = mode;
    if (d.adam_pending) dqn_bind(d, on_alt ? alt : prim, on_alt ? prim : alt);
    const hipError_t e = p2pmg::launch_dqn_act(d, c->stream);
    if (e != hipSuccess) {
      (void)settle();
      return fail(c, P2PMG_E_HIP, std::string("dqn act launch: ") + hipGetErrorString(e));
    }
    if (d.adam_pending) {  // applied: the stepped state is the current one
      on_alt = !on_alt;
      d.adam_pending = 0;
      dqn_bind(d, on_alt ? alt : prim, on_alt ? alt : prim);
    }
    if (mode == P2PMG_MODE_TRAIN) {
      rc = dqn_train_step(c, d, same, defer);
      if (rc != P2PMG_OK) {
        (void)settle();
        return rc;
      }
    }
  }
  rc = settle();
  if (rc != P2PMG_OK) return rc;
  HIP_TRY(c, hipEventRecord(c->ring[2 * slot + 1], c->stream));
  c->timed = true;
  c->n_timed++;
  c->rec_last_mask = args->record;
  if (acting) c->d_added_min += c->T;
  if (acting && args->rng == P2PMG_RNG_REPLAY) c->have_codes = c->code_src == 1;
  return P2PMG_OK;
}

int p2pmg_dqn_forward(p2pmg_ctx* c, int net, int n, const float* x, float* q) {
  int rc = dqn_ready(c, "dqn_forward");
  if (rc != P2PMG_OK) return rc;
  if (net < 0 || net >= c->n_nets || n < 0 || (n > 0 && (!x || !q))) return fail(c, P2PMG_E_INVALID, "dqn_forward");
  if (n == 0) return P2PMG_OK;
  float *dx = nullptr, *dq = nullptr;
  HIP_TRY(c, dmalloc(&dx, (size_t)n * 5));
  hipError_t e = dmalloc(&dq, (size_t)n);
  if (e == hipSuccess) e = hipMemcpyAsync(dx, x, (size_t)n * 20, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = p2pmg::launch_dqn_forward(c->d_theta + (size_t)net * p2pmg::kNetStride, n, dx, dq, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(q, dq, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(dx);
  dfree(dq);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("dqn_forward: ") + hipGetErrorString(e));
  return P2PMG_OK;
}

int p2pmg_dqn_train_batch(p2pmg_ctx* c, int net, const float* batch, float* loss) {
  int rc = dqn_ready(c, "dqn_train_batch");
  if (rc != P2PMG_OK) return rc;
  if (net < 0 || net >= c->n_nets || !batch) return fail(c, P2PMG_E_INVALID, "dqn_train_batch");
  float* db = nullptr;
  HIP_TRY(c, dmalloc(&db, (size_t)p2pmg::kDqnBatch * p2pmg::kTrans + 1));
  p2pmg_episode_args args{P2PMG_MODE_TRAIN, P2PMG_RNG_PHILOX, 0, 0, 0.0, 0, 0};
  p2pmg::DqnParams d = dqn_params(c, episode_params(c, &args));
  d.batch = db;
  d.net = net;
  d.loss_out = db + p2pmg::kDqnBatch * p2pmg::kTrans;
  d.lr_t = adam_lr(c->dcfg, ++c->d_steps[(size_t)net]);  // only this network's Adam iterates
  hipError_t e = hipMemcpyAsync(db, batch, (size_t)p2pmg::kDqnBatch * p2pmg::kTrans * 4, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = p2pmg::launch_dqn_train(d, 1, false, c->stream);
  float l = 0.0f;
  if (e == hipSuccess) e = hipMemcpyAsync(&l, d.loss_out, 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(db);
  if (e != hipSuccess) return fail(c, P2PMG_E_HIP, std::string("dqn_train_batch: ") + hipGetErrorString(e));
  if (loss) *loss = l;
  return P2PMG_OK;
}

int p2pmg_dqn_set_exchange(p2pmg_ctx* c, p2pmg_exchange_fn fn, void* user, int rank, int nranks) {
  if (!c) return P2PMG_E_INVALID;
  if (c->comm) return fail(c, P2PMG_E_STATE, "dqn_set_exchange: the context has an RCCL communicator");
  if (!fn) {
    c->xfn = nullptr;
    c->xuser = nullptr;
    c->rank = 0;
    c->nranks = 1;
    return P2PMG_OK;
  }
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(c, P2PMG_E_INVALID, "dqn_set_exchange: rank / nranks");
  c->xfn = fn;
  c->xuser = user;
  c->rank = rank;
  c->nranks = nranks;
  return P2PMG_OK;
}

int p2pmg_dqn_grad_layout(p2pmg_ctx* c, int* segments, int* agents_per_block, int* blocks) {
  int rc = dqn_ready(c, "dqn_grad_layout");
  if (rc != P2PMG_OK) return rc;
  if (segments) *segments = c->d_seg_local;
  if (agents_per_block) *agents_per_block = c->d_apb;
  if (blocks) *blocks = c->d_blocks;
  return P2PMG_OK;
}

}  // extern "C"