// p2pmg_device.h — device primitives shared by the kernel files (tabular episode kernel and
// the DQN step kernels).  Included INSIDE `namespace p2pmg { namespace {` of each .hip file.
// Part of the numerics contract: built with -ffp-contract=off (each op rounds separately).

// x / N for a compile-time N: a multiply by 1/N is bit-identical when N is a power of two
// (same exact real value, same single rounding), so only other N pay for a division
template <int N>
__device__ __forceinline__ float div_n(float x) {
  if constexpr ((N & (N - 1)) == 0) return x * (1.0f / (float)N);
  else return x / (float)N;
}

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
    // one v_mad_u64_u32 per product instead of v_mul_hi_u32 + v_mul_lo_u32
    const uint64_t m0 = (uint64_t)0xD2511F53u * c0, m1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(m0 >> 32), lo0 = (uint32_t)m0;
    const uint32_t hi1 = (uint32_t)(m1 >> 32), lo1 = (uint32_t)m1;
    // the three-input XORs as one gfx950 v_bitop3_b32 each (truth table 0x96) instead of two
    // v_xor_b32: configs[2] 2.692 -> 2.655 ms per episode (profiles/r05_ab/philox_bitop3_ab.txt)
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96), n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
}
constexpr uint32_t kTagDecision = 0x5EED0004u;  // one 32-bit word per round (oracle/philox.py)
constexpr uint32_t kTagT0 = 0x5EED0002u;
constexpr uint32_t kTagAction = 0x5EED0005u;    // small epsilon: the explore actions' own block
constexpr uint32_t kSmallEpsThr = 1u << 24;     // eps < 2^-8: below it the actions come from kTagAction

// Philox exploration stream (oracle/philox.py::decision_draws; QActor.select_action rl.py:100-111):
// round r of step t of agent gid uses word k % 4 of the block ctr = (k / 4, episode, gid,
// kTagDecision), k = t (R + 1) + r.  The agent explores when w / 2^32 < eps (w < thr, eps_threshold)
// and then takes a uniformly drawn action (rl.py:110-111 draws it separately from the explore test):
//   thr >= 2^24 (eps >= 2^-8, every tabular run: its floor is 0.1): action w % 3 -- given w < thr,
//     w is uniform on [0, thr), so w % 3 is uniform up to 1 / thr <= 2^-24;
//   thr < 2^24 (small eps, e.g. the DQN's unfloored 0.9^e decay): w % 3 of a w below a small thr
//     would be biased (every w < 3: one fixed action), so the action is word k % 4 of the block
//     (k / 4, episode, gid, kTagAction), independent of the explore test, % 3 (bias <= 2^-32).
// The branch is kernel-uniform (thr is a launch argument).  One word per round: a block serves four
// rounds (two steps at R = 1).  255 = greedy.
__device__ __forceinline__ uint32_t decision_code(uint32_t w, uint32_t act_word, uint32_t thr, int all) {
  return (all || w < thr) ? act_word % 3u : 255u;
}
// the four codes of block blk, byte j = word j
__device__ __forceinline__ uint32_t philox_block_codes(uint32_t blk, uint32_t episode, uint32_t gid, uint32_t thr,
                                                       int all, uint32_t k0, uint32_t k1) {
  uint32_t c0 = blk, c1 = episode, c2 = gid, c3 = kTagDecision;
  // the round keys derive from the seed afresh in each call (SALU adds): hoisted out of an episode
  // loop they would be 20 uniform values held across it
  asm volatile("" : "+s"(k0), "+s"(k1));
  philox4x32_10(c0, c1, c2, c3, k0, k1);
  uint32_t a0 = c0, a1 = c1, a2 = c2, a3 = c3;
  if (!all && thr < kSmallEpsThr) {
    a0 = blk, a1 = episode, a2 = gid, a3 = kTagAction;
    philox4x32_10(a0, a1, a2, a3, k0, k1);
  }
  return decision_code(c0, a0, thr, all) | (decision_code(c1, a1, thr, all) << 8) |
         (decision_code(c2, a2, thr, all) << 16) | (decision_code(c3, a3, thr, all) << 24);
}
// the codes of rounds 0 .. min(R1, 8) - 1 of step t, byte r (bytes r >= R1: 255); rounds 8 and up
// (R1 > 8) come from philox_round_code one at a time
__device__ __forceinline__ uint64_t philox_step_codes(int t, int R1, uint32_t episode, uint32_t gid, uint32_t thr,
                                                      int all, uint32_t k0, uint32_t k1) {
  const int R8 = R1 < 8 ? R1 : 8;
  const uint32_t kf = (uint32_t)t * (uint32_t)R1, kl = kf + (uint32_t)R8 - 1u;
  uint64_t out = ~0ull;
  for (uint32_t b = kf >> 2; b <= (kl >> 2); ++b) {
    const uint32_t c4 = philox_block_codes(b, episode, gid, thr, all, k0, k1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (int)(4u * b + (uint32_t)j) - (int)kf;
      if (r >= 0 && r < R8) out = (out & ~(0xFFull << (8 * r))) | ((uint64_t)((c4 >> (8 * j)) & 0xFFu) << (8 * r));
    }
  }
  return out;
}
// the code of round r (any r < R1) of step t: byte k % 4 of block k / 4, k = t R1 + r
__device__ __forceinline__ uint32_t philox_round_code(int t, int R1, int r, uint32_t episode, uint32_t gid,
                                                      uint32_t thr, int all, uint32_t k0, uint32_t k1) {
  const uint32_t k = (uint32_t)t * (uint32_t)R1 + (uint32_t)r;
  return (philox_block_codes(k >> 2, episode, gid, thr, all, k0, k1) >> (8 * (k & 3u))) & 0xFFu;
}
// code word w of step t (rounds 4w .. 4w + 3, byte b = round 4w + b, 255 past R1): the pre-passes'
// words w >= 2 (the 64-bit step codes cover words 0 and 1)
__device__ __forceinline__ uint32_t philox_code_word(int t, int R1, int w, uint32_t episode, uint32_t gid,
                                                     uint32_t thr, int all, uint32_t k0, uint32_t k1) {
  uint32_t word = 0xFFFFFFFFu;
  for (int b = 0; b < 4 && 4 * w + b < R1; ++b)
    word = (word & ~(0xFFu << (8 * b))) | (philox_round_code(t, R1, 4 * w + b, episode, gid, thr, all, k0, k1) << (8 * b));
  return word;
}

// RuleAgent._update_storage (agent.py:138-153) with BatteryStorage bookkeeping (storage.py:79-100),
// f64 like the reference's Python floats.  Returns the adjusted balance (W); soc is updated.
__device__ __forceinline__ double battery_rule(double balance, double& soc, double cap, double smin, double smax,
                                               double sqrt_eff) {
  const double energy = (balance * 60.0) * 15.0;
  const double avail_energy = (fmax(0.0, soc - smin) * cap) * sqrt_eff;
  const double avail_space = (fmax(0.0, smax - soc) * cap) / sqrt_eff;
  if (balance > 0.0 && avail_energy > 0.0) {
    const double x = energy <= avail_energy ? energy : avail_energy;  // min(energy, available_energy)
    soc = soc - (x / cap) / sqrt_eff;
    balance = balance - x / 900.0;
  } else if (balance < 0.0 && !(soc >= smax)) {
    const double x = -energy <= avail_space ? -energy : avail_space;
    soc = soc + sqrt_eff * (x / cap);
    balance = balance + x / 900.0;
  }
  return balance;
}

