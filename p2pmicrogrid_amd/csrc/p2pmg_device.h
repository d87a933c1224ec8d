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
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
}
constexpr uint32_t kTagDecision = 0x5EED0003u;  // one block per two rounds (oracle/philox.py)
constexpr uint32_t kTagT0 = 0x5EED0002u;

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

