// Issue-rate microbenchmark for gfx950 under full occupancy: every SIMD runs 4 waves, each wave
// issues 4 independent chains of one instruction kind; the kernel time over the instruction
// count gives the SIMD cycles one wave64 instruction of that kind occupies (4 = a full-rate
// VALU op on a 16-lane SIMD).  Timed with HIP events; results through ordinary stores.
//   hipcc --offload-arch=gfx950 -O3 ubench_rate.hip -o ubench_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096
#define X4(a) a a a a

template <int K>
__global__ __launch_bounds__(256) void rate(unsigned* out, unsigned a, unsigned b) {
  unsigned x0 = a + threadIdx.x, x1 = x0 * 3u, x2 = x0 ^ 0x55u, x3 = x0 + 7u;
  unsigned long long y0 = x0, y1 = x1, y2 = x2, y3 = x3;
  float f0 = (float)x0, f1 = (float)x1, f2 = (float)x2, f3 = (float)x3, fb = (float)b;
  double d0 = f0, d1 = f1, d2 = f2, d3 = f3, db = fb;
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (K == 0) {
      X4(asm volatile("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb));)
    } else if constexpr (K == 1) {
      X4(asm volatile("v_mad_u64_u32 %0, vcc, %4, %5, 0\n v_mad_u64_u32 %1, vcc, %4, %5, 0\n"
                      " v_mad_u64_u32 %2, vcc, %4, %5, 0\n v_mad_u64_u32 %3, vcc, %4, %5, 0"
                      : "=v"(y0), "=v"(y1), "=v"(y2), "=v"(y3) : "v"(x0), "v"(b) : "vcc");
         x0 += (unsigned)y0;)
    } else if constexpr (K == 2) {
      X4(asm volatile("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b));)
    } else if constexpr (K == 3) {
      X4(asm volatile("v_mul_hi_u32 %0, %0, %4\n v_mul_hi_u32 %1, %1, %4\n v_mul_hi_u32 %2, %2, %4\n v_mul_hi_u32 %3, %3, %4"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b));)
    } else if constexpr (K == 4) {
      X4(asm volatile("v_mul_u32_u24 %0, %0, %4\n v_mul_u32_u24 %1, %1, %4\n v_mul_u32_u24 %2, %2, %4\n v_mul_u32_u24 %3, %3, %4"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b));)
    } else if constexpr (K == 5) {
      X4(asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4"
                      : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(db));)
    } else if constexpr (K == 6) {
      X4(asm volatile("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4"
                      : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(db));)
    } else if constexpr (K == 7) {
      X4(asm volatile("v_cvt_f64_u32 %0, %4\n v_cvt_f64_u32 %1, %5\n v_cvt_f64_u32 %2, %6\n v_cvt_f64_u32 %3, %7"
                      : "=v"(d0), "=v"(d1), "=v"(d2), "=v"(d3) : "v"(x0), "v"(x1), "v"(x2), "v"(x3));
         x0 += 1u;)
    } else if constexpr (K == 8) {
      X4(asm volatile("v_med3_f32 %0, %0, %4, 0\n v_med3_f32 %1, %1, %4, 0\n v_med3_f32 %2, %2, %4, 0\n v_med3_f32 %3, %3, %4, 0"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb));)
    } else if constexpr (K == 9) {
      typedef float f2t __attribute__((ext_vector_type(2)));
      f2t p0 = {f0, f1}, p1 = {f2, f3}, p2 = {f1, f0}, p3 = {f3, f2}, pb = {fb, fb};
      X4(asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4"
                      : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));)
      f0 = p0.x + p1.y + p2.x + p3.y;
    } else if constexpr (K == 10) {
      X4(asm volatile("v_cmp_gt_f64 vcc, %4, %5\n v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %0, vcc\n"
                      " v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %2, vcc"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(d0), "v"(db) : "vcc");)
    } else if constexpr (K == 11) {
      X4(asm volatile("v_ldexp_f64 %0, %0, %4\n v_ldexp_f64 %1, %1, %4\n v_ldexp_f64 %2, %2, %4\n v_ldexp_f64 %3, %3, %4"
                      : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(b));)
    } else if constexpr (K == 12) {
      X4(asm volatile("v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4"
                      : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(db));)
    } else if constexpr (K == 13) {
      X4(asm volatile("v_xor_b32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_xor_b32 %2, %2, %4\n v_xor_b32 %3, %3, %4"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b));)
    } else if constexpr (K == 14) {
      X4(asm volatile("v_mul_hi_u32_u24 %0, %0, %4\n v_mul_hi_u32_u24 %1, %1, %4\n v_mul_hi_u32_u24 %2, %2, %4\n v_mul_hi_u32_u24 %3, %3, %4"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b));)    } else if constexpr (K == 15) {
      X4(asm volatile("v_fma_f32 %0, %0, %4, %4\n v_fma_f32 %1, %1, %4, %4\n v_fma_f32 %2, %2, %4, %4\n v_fma_f32 %3, %3, %4, %4"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb));)
    } else if constexpr (K == 16 || K == 17) {
      typedef float f2t __attribute__((ext_vector_type(2)));
      f2t p0 = {f0, f1}, p1 = {f2, f3}, p2 = {f1, f0}, p3 = {f3, f2}, pb = {fb, fb};
      if constexpr (K == 16) {
        X4(asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4"
                        : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));)
      } else {
        X4(asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4"
                        : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));)
      }
      f0 = p0.x + p1.y + p2.x + p3.y;
    } else if constexpr (K == 18) {
      X4(asm volatile("v_mul_f32 %0, %0, %4\n v_mul_f32 %1, %1, %4\n v_mul_f32 %2, %2, %4\n v_mul_f32 %3, %3, %4"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb));)
    } else if constexpr (K == 19) {
      X4(asm volatile("v_cvt_i32_f32 %0, %4\n v_cvt_i32_f32 %1, %5\n v_cvt_i32_f32 %2, %6\n v_cvt_i32_f32 %3, %7"
                      : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3) : "v"(f0), "v"(f1), "v"(f2), "v"(f3));
         f0 += 1.0f;)
    } else if constexpr (K == 20) {
      X4(asm volatile("v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));)
    } else if constexpr (K == 21) {
      X4(asm volatile("v_max_f32 %0, %0, %4\n v_max_f32 %1, %1, %4\n v_max_f32 %2, %2, %4\n v_max_f32 %3, %3, %4"
                      : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(fb));)
    } else if constexpr (K == 22) {
      X4(asm volatile("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b) : "vcc");)
    } else if constexpr (K == 23) {
      X4(asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4"
                      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b));)
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + (unsigned)(y0 + y1 + y2 + y3) +
                                                (unsigned)(f0 + f1 + f2 + f3) + (unsigned)(d0 + d1 + d2 + d3);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int khz = 0;
  hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0);
  const int blocks = cus * 4;  // 4 x 256 threads per CU = 4 waves per SIMD
  unsigned* out;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(unsigned));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v_add_f32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_fma_f64",
                         "v_add_f64", "v_cvt_f64_u32", "v_med3_f32", "v_pk_fma_f32", "v_cmp_f64 + 4 v_cndmask (5 insts)",
                         "v_ldexp_f64", "v_mul_f64", "v_xor_b32", "v_mul_hi_u32_u24", "v_fma_f32", "v_pk_add_f32",
                         "v_pk_mul_f32", "v_mul_f32", "v_cvt_i32_f32", "v_rcp_f32", "v_max_f32", "v_cndmask_b32",
                         "v_add_u32"};
  auto run = [&](auto k, int idx) {
    constexpr int K = decltype(k)::value;
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(rate<K>, dim3(blocks), dim3(256), 0, 0, out, 3u, 5u);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    const double insts = (double)ITERS * 16 * (K == 10 ? 5.0 / 4.0 : 1.0);  // per wave
    const double waves_per_simd = 4.0;
    const double cyc = best * 1e-3 * khz * 1e3;  // at the reported clock
    printf("{\"inst\": \"%s\", \"ms\": %.4f, \"simd_cycles_per_wave_inst\": %.2f, \"clock_khz\": %d}\n", names[idx],
           best, cyc / (insts * waves_per_simd), khz);
  };
  run(std::integral_constant<int, 0>{}, 0); run(std::integral_constant<int, 1>{}, 1);
  run(std::integral_constant<int, 2>{}, 2); run(std::integral_constant<int, 3>{}, 3);
  run(std::integral_constant<int, 4>{}, 4); run(std::integral_constant<int, 5>{}, 5);
  run(std::integral_constant<int, 6>{}, 6); run(std::integral_constant<int, 7>{}, 7);
  run(std::integral_constant<int, 8>{}, 8); run(std::integral_constant<int, 9>{}, 9);
  run(std::integral_constant<int, 10>{}, 10); run(std::integral_constant<int, 11>{}, 11);
  run(std::integral_constant<int, 12>{}, 12); run(std::integral_constant<int, 13>{}, 13);
  run(std::integral_constant<int, 14>{}, 14);
  run(std::integral_constant<int, 15>{}, 15);
  run(std::integral_constant<int, 16>{}, 16);
  run(std::integral_constant<int, 17>{}, 17);
  run(std::integral_constant<int, 18>{}, 18);
  run(std::integral_constant<int, 19>{}, 19);
  run(std::integral_constant<int, 20>{}, 20);
  run(std::integral_constant<int, 21>{}, 21);
  run(std::integral_constant<int, 22>{}, 22);
  run(std::integral_constant<int, 23>{}, 23);
  return 0;
}
