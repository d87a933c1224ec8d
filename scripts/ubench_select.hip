// In-situ cost of the lane selects of episode_sq16_kernel (v_cndmask_b32 measured 22.8
// SIMD cycles in scripts/dev/ubench_rate.hip K = 22, against 2.6-2.9 for v_add / v_mul_f32).  Every
// SIMD runs 4 waves; each wave issues 4 independent chains of the pattern, ITERS x 16 pattern
// instances per wave; the kernel time over the instruction count = SIMD cycles one wave64 instruction
// occupies (4 = one per quad-cycle).  Variants:
//   cnd_vcc_e32     v_cndmask_b32_e32 on a loop-invariant VCC written once before the loop
//   cnd_sgpr_e64    v_cndmask_b32_e64 on a loop-invariant SGPR-pair mask
//   cnd_smov_vcc    s_mov_b32 vcc_lo / vcc_hi + v_cndmask_b32_e64 per select (zero_diag16's form)
//   cnd_smov_sgpr   s_mov_b64 of an SGPR pair + v_cndmask_b32_e64 on it per select
//   cnd_consumed    v_cndmask_b32_e64 (SGPR mask) immediately followed by a dependent v_add_f32
//   add_consumed    v_add_f32 immediately followed by a dependent v_add_f32 (the reference chain)
//   bfi_vmask       v_bfi_b32 with a loop-invariant VGPR mask (the bit-select alternative)
//   and_vmask       v_and_b32 with a loop-invariant VGPR mask
//   add_f32         v_add_f32 (baseline)
//   med3_f32        v_med3_f32
//   cnd_*_among_3_adds     one select (VCC e32 / SGPR-pair e64) per three independent v_add_f32
//   cmp_vcc_then_cnd_e32   v_cmp_e32 into VCC then v_cndmask_b32_e32 on it (the compiler's usual pair)
//   cmp_sgpr_then_cnd_e64  v_cmp_e64 into an SGPR pair then v_cndmask_b32_e64 on it
// ubench_rate K = 22 wrote "vcc" as a clobber of every asm block while reading it: the compiler may
// not keep a value in VCC across such blocks, so that number is checked here against the explicit
// forms.  Prints one JSON line per variant.
//   hipcc --offload-arch=gfx950 -O3 -o ubench_select ubench_select.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITERS 4096
#define X4(a) a a a a

template <int K>
__global__ __launch_bounds__(256) void sel(unsigned* out, unsigned a, unsigned b) {
  unsigned x0 = a + threadIdx.x, x1 = x0 * 3u, x2 = x0 ^ 0x55u, x3 = x0 + 7u;
  float f0 = (float)x0, f1 = (float)x1, f2 = (float)x2, f3 = (float)x3, fb = (float)b;
  const unsigned vm = (threadIdx.x & 16) ? 0xFFFFFFFFu : 0u;  // a per-lane mask in a VGPR
  uint64_t sm;  // a per-lane mask in an SGPR pair
  asm volatile("v_cmp_gt_u32_e64 %0, %1, 31" : "=s"(sm) : "v"((unsigned)threadIdx.x));
  if constexpr (K == 0) asm volatile("v_cmp_lt_u32_e32 vcc, 31, %0" ::"v"((unsigned)threadIdx.x) : "vcc");
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (K == 0) {
      // VCC set once before the loop; the asm blocks read it without clobbering it
      X4(asm volatile("v_cndmask_b32_e32 %0, %0, %4, vcc\n v_cndmask_b32_e32 %1, %1, %4, vcc\n"
                      " v_cndmask_b32_e32 %2, %2, %4, vcc\n v_cndmask_b32_e32 %3, %3, %4, vcc"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b));)
    } else if constexpr (K == 1) {
      X4(asm volatile("v_cndmask_b32_e64 %0, %0, %4, %5\n v_cndmask_b32_e64 %1, %1, %4, %5\n"
                      " v_cndmask_b32_e64 %2, %2, %4, %5\n v_cndmask_b32_e64 %3, %3, %4, %5"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b), "s"(sm));)
    } else if constexpr (K == 2) {
      X4(asm volatile("s_mov_b32 vcc_lo, 0x10001\n s_mov_b32 vcc_hi, 0x10001\n v_cndmask_b32_e64 %0, %0, 0, vcc\n"
                      " s_mov_b32 vcc_lo, 0x20002\n s_mov_b32 vcc_hi, 0x20002\n v_cndmask_b32_e64 %1, %1, 0, vcc\n"
                      " s_mov_b32 vcc_lo, 0x40004\n s_mov_b32 vcc_hi, 0x40004\n v_cndmask_b32_e64 %2, %2, 0, vcc\n"
                      " s_mov_b32 vcc_lo, 0x80008\n s_mov_b32 vcc_hi, 0x80008\n v_cndmask_b32_e64 %3, %3, 0, vcc"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)::"vcc");)
    } else if constexpr (K == 3) {
      uint64_t t;
      X4(asm volatile("s_mov_b64 %4, 0x10001\n v_cndmask_b32_e64 %0, %0, 0, %4\n"
                      " s_mov_b64 %4, 0x20002\n v_cndmask_b32_e64 %1, %1, 0, %4\n"
                      " s_mov_b64 %4, 0x40004\n v_cndmask_b32_e64 %2, %2, 0, %4\n"
                      " s_mov_b64 %4, 0x80008\n v_cndmask_b32_e64 %3, %3, 0, %4"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=&s"(t));)
    } else if constexpr (K == 4) {
      X4(asm volatile("v_cndmask_b32_e64 %0, %0, %4, %5\n v_add_f32 %0, %0, %0\n"
                      " v_cndmask_b32_e64 %1, %1, %4, %5\n v_add_f32 %1, %1, %1\n"
                      " v_cndmask_b32_e64 %2, %2, %4, %5\n v_add_f32 %2, %2, %2\n"
                      " v_cndmask_b32_e64 %3, %3, %4, %5\n v_add_f32 %3, %3, %3"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb), "s"(sm));)
    } else if constexpr (K == 5) {
      X4(asm volatile("v_add_f32 %0, %0, %4\n v_add_f32 %0, %0, %0\n v_add_f32 %1, %1, %4\n v_add_f32 %1, %1, %1\n"
                      " v_add_f32 %2, %2, %4\n v_add_f32 %2, %2, %2\n v_add_f32 %3, %3, %4\n v_add_f32 %3, %3, %3"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb));)
    } else if constexpr (K == 6) {
      X4(asm volatile("v_bfi_b32 %0, %4, %5, %0\n v_bfi_b32 %1, %4, %5, %1\n v_bfi_b32 %2, %4, %5, %2\n v_bfi_b32 %3, %4, %5, %3"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(vm), "v"(b));)
    } else if constexpr (K == 7) {
      X4(asm volatile("v_and_b32 %0, %0, %4\n v_and_b32 %1, %1, %4\n v_and_b32 %2, %2, %4\n v_and_b32 %3, %3, %4"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(vm | b));)
    } else if constexpr (K == 8) {
      X4(asm volatile("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb));)
    } else if constexpr (K == 9) {
      X4(asm volatile("v_med3_f32 %0, %0, %4, 0\n v_med3_f32 %1, %1, %4, 0\n v_med3_f32 %2, %2, %4, 0\n v_med3_f32 %3, %3, %4, 0"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb));)
    } else if constexpr (K == 10) {  // one VCC select among three independent adds
      X4(asm volatile("v_cndmask_b32_e32 %0, %0, %8, vcc\n v_add_f32 %4, %4, %9\n v_add_f32 %5, %5, %9\n v_add_f32 %6, %6, %9\n"
                      " v_cndmask_b32_e32 %1, %1, %8, vcc\n v_add_f32 %7, %7, %9\n v_add_f32 %4, %4, %9\n v_add_f32 %5, %5, %9\n"
                      " v_cndmask_b32_e32 %2, %2, %8, vcc\n v_add_f32 %6, %6, %9\n v_add_f32 %7, %7, %9\n v_add_f32 %4, %4, %9\n"
                      " v_cndmask_b32_e32 %3, %3, %8, vcc\n v_add_f32 %5, %5, %9\n v_add_f32 %6, %6, %9\n v_add_f32 %7, %7, %9"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(b), "v"(fb));)
    } else if constexpr (K == 11) {  // one SGPR-pair select among three independent adds
      X4(asm volatile("v_cndmask_b32_e64 %0, %0, %8, %10\n v_add_f32 %4, %4, %9\n v_add_f32 %5, %5, %9\n v_add_f32 %6, %6, %9\n"
                      " v_cndmask_b32_e64 %1, %1, %8, %10\n v_add_f32 %7, %7, %9\n v_add_f32 %4, %4, %9\n v_add_f32 %5, %5, %9\n"
                      " v_cndmask_b32_e64 %2, %2, %8, %10\n v_add_f32 %6, %6, %9\n v_add_f32 %7, %7, %9\n v_add_f32 %4, %4, %9\n"
                      " v_cndmask_b32_e64 %3, %3, %8, %10\n v_add_f32 %5, %5, %9\n v_add_f32 %6, %6, %9\n v_add_f32 %7, %7, %9"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(b), "v"(fb), "s"(sm));)
    } else if constexpr (K == 12) {  // the compiler's pair: v_cmp into VCC, v_cndmask_e32 on it
      X4(asm volatile("v_cmp_gt_f32_e32 vcc, %4, %5\n v_cndmask_b32_e32 %0, %0, %6, vcc\n"
                      " v_cmp_gt_f32_e32 vcc, %5, %4\n v_cndmask_b32_e32 %1, %1, %6, vcc\n"
                      " v_cmp_gt_f32_e32 vcc, %4, %5\n v_cndmask_b32_e32 %2, %2, %6, vcc\n"
                      " v_cmp_gt_f32_e32 vcc, %5, %4\n v_cndmask_b32_e32 %3, %3, %6, vcc"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(f0), "v"(fb), "v"(b) : "vcc");)
    } else if constexpr (K == 13) {  // the same with the compare into an SGPR pair
      uint64_t t0, t1;
      X4(asm volatile("v_cmp_gt_f32_e64 %4, %6, %7\n v_cndmask_b32_e64 %0, %0, %8, %4\n"
                      " v_cmp_gt_f32_e64 %5, %7, %6\n v_cndmask_b32_e64 %1, %1, %8, %5\n"
                      " v_cmp_gt_f32_e64 %4, %6, %7\n v_cndmask_b32_e64 %2, %2, %8, %4\n"
                      " v_cmp_gt_f32_e64 %5, %7, %6\n v_cndmask_b32_e64 %3, %3, %8, %5"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=&s"(t0), "=&s"(t1) : "v"(f0), "v"(fb), "v"(b));)
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + (unsigned)(f0 + f1 + f2 + f3) + (unsigned)sm +
                                                (unsigned)vm;
}

int main() {
  int cus = 0, khz = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0);
  const int blocks = cus * 4;  // 4 x 256 threads per CU = 4 waves per SIMD
  unsigned* out;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(unsigned));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // VALU instructions per pattern instance (the SALU s_movs of K = 2, 3 are listed separately)
  const char* names[] = {"cnd_vcc_e32", "cnd_sgpr_e64", "cnd_smov_vcc", "cnd_smov_sgpr", "cnd_consumed",
                         "add_consumed", "bfi_vmask", "and_vmask", "add_f32", "med3_f32",
                         "cnd_vcc_e32_among_3_adds", "cnd_sgpr_e64_among_3_adds", "cmp_vcc_then_cnd_e32",
                         "cmp_sgpr_then_cnd_e64"};
  const double valu[] = {1, 1, 1, 1, 2, 2, 1, 1, 1, 1, 4, 4, 2, 2};
  const double salu[] = {0, 0, 2, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  auto run = [&](auto k) {
    constexpr int K = decltype(k)::value;
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(sel<K>, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    const double inst = (double)ITERS * 16;  // pattern instances per wave
    const double cyc = best * 1e-3 * khz * 1e3;
    printf("{\"probe\": \"ubench_select\", \"variant\": \"%s\", \"ms\": %.4f, \"simd_cycles_per_instance\": %.2f, "
           "\"valu_per_instance\": %.0f, \"salu_per_instance\": %.0f, \"simd_cycles_per_valu\": %.2f, \"clock_khz\": %d}\n",
           names[K], best, cyc / (inst * 4.0), valu[K], salu[K], cyc / (inst * 4.0 * valu[K]), khz);
  };
  run(std::integral_constant<int, 0>{});
  run(std::integral_constant<int, 1>{});
  run(std::integral_constant<int, 2>{});
  run(std::integral_constant<int, 3>{});
  run(std::integral_constant<int, 4>{});
  run(std::integral_constant<int, 5>{});
  run(std::integral_constant<int, 6>{});
  run(std::integral_constant<int, 7>{});
  run(std::integral_constant<int, 8>{});
  run(std::integral_constant<int, 9>{});
  run(std::integral_constant<int, 10>{});
  run(std::integral_constant<int, 11>{});
  run(std::integral_constant<int, 12>{});
  run(std::integral_constant<int, 13>{});
  hipFree(out);
  return 0;
}
