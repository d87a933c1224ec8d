// Issue/latency microbenchmark for gfx950 (one wave alone on its SIMD): cycles per iteration of
// small dependent instruction chains, stamped with s_memtime (a read of the shader clock).
// Results go out through ordinary vector stores.  hipcc --offload-arch=gfx950 -O3 ubench_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2000
#define BODY8(x) x x x x x x x x

template <int K>
__global__ void chain(float* out, long long* cyc, float a, float b) {
  float v1 = a + threadIdx.x, v2 = b, v3 = a * 2.0f;
  double d0 = (double)v1, d1 = (double)b;
  long long t0;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (K == 0) {  // dependent v_add_f32
      BODY8(asm volatile("v_add_f32 %0, %0, %1" : "+v"(v1) : "v"(v2));)
    } else if constexpr (K == 1) {  // v_cmp -> s_and (VALU->SALU) -> v_cndmask
      BODY8(asm volatile("v_cmp_gt_f32 s[20:21], %0, %1\n s_and_b64 s[22:23], s[20:21], exec\n v_cndmask_b32 %0, %0, %2, s[22:23]" : "+v"(v1) : "v"(v2), "v"(v3) : "s20", "s21", "s22", "s23");)
    } else if constexpr (K == 2) {  // v_cmp -> vcc -> v_cndmask
      BODY8(asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %2, vcc" : "+v"(v1) : "v"(v2), "v"(v3) : "vcc");)
    } else if constexpr (K == 3) {  // dependent v_add_f64
      BODY8(asm volatile("v_add_f64 %0, %0, %1" : "+v"(d0) : "v"(d1));)
    } else if constexpr (K == 4) {  // dependent v_rcp_f32
      BODY8(asm volatile("v_rcp_f32 %0, %0" : "+v"(v1));)
    } else if constexpr (K == 5) {  // dpp move chain with its hazard nop
      BODY8(asm volatile("s_nop 1\n v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(v1));)
    } else if constexpr (K == 6) {  // v_cmp_f64 -> vcc -> 2 cndmask (f64 select)
      BODY8(asm volatile("v_cmp_gt_f64 vcc, %2, %3\n v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %0, vcc" : "+v"(v1), "+v"(v3) : "v"(d0), "v"(d1) : "vcc");)
    } else if constexpr (K == 7) {  // divergence guard not taken: v_cmp, s_and_saveexec, branch, restore
      BODY8(asm volatile("v_cmp_gt_f32 vcc, %0, %1\n s_and_saveexec_b64 s[20:21], vcc\n s_cbranch_execz 1f\n v_add_f32 %0, %0, %2\n 1:\n s_or_b64 exec, exec, s[20:21]" : "+v"(v1) : "v"(v2), "v"(v3) : "vcc", "s20", "s21");)
    } else if constexpr (K == 8) {  // independent v_add_f32 (4 chains)
      float x0 = v1, x1 = v2, x2 = v3, x3 = a;
      BODY8(asm volatile("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(b));)
      v1 = x0 + x1 + x2 + x3;
    } else if constexpr (K == 9) {  // s_nop 0 alone
      BODY8(asm volatile("s_nop 0");)
    } else if constexpr (K == 10) {  // v_cmp -> s_and -> s_or (SALU chain on a VALU mask), then cndmask
      BODY8(asm volatile("v_cmp_gt_f32 s[20:21], %0, %1\n v_cmp_lt_f32 s[24:25], %0, %2\n s_or_b64 s[22:23], s[20:21], s[24:25]\n v_cndmask_b32 %0, %0, %2, s[22:23]" : "+v"(v1) : "v"(v2), "v"(v3) : "s20", "s21", "s22", "s23", "s24", "s25");)
    } else if constexpr (K == 11) {  // dependent v_mul_f64
      BODY8(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d0) : "v"(d1));)
    } else if constexpr (K == 12) {  // v_lshl_add_u64 dependent
      unsigned long long p = (unsigned long long)(uintptr_t)out;
      BODY8(asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(p) : "v"(p));)
      v1 += (float)(p & 1);
    } else if constexpr (K == 13) {  // v_pk_fma_f32 dependent
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 x = {v1, v2}, y = {v3, a};
      BODY8(asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(y));)
      v1 = x.x + x.y;
    }
  }
  long long t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  out[threadIdx.x] = v1 + (float)d0;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  float* out; long long* cyc;
  hipMalloc(&out, 64 * sizeof(float));
  hipMalloc(&cyc, sizeof(long long));
  const char* names[] = {"v_add_f32 dep", "v_cmp->s_and->v_cndmask", "v_cmp vcc->v_cndmask", "v_add_f64 dep",
                         "v_rcp_f32 dep", "s_nop1+dpp dep", "v_cmp_f64->2 cndmask", "guard not taken (cmp,saveexec,br,or)",
                         "4 indep v_add_f32", "s_nop 0", "2 v_cmp->s_or->cndmask", "v_mul_f64 dep", "v_lshl_add_u64 dep",
                         "v_pk_fma_f32 dep"};
  auto run = [&](auto k, int idx) {
    constexpr int K = decltype(k)::value;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(chain<K>, dim3(1), dim3(64), 0, 0, out, cyc, 1.0f, 1e-9f);
      hipDeviceSynchronize();
    }
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-40s %.2f cycles per body\n", names[idx], (double)c / (ITERS * 8.0));
  };
  run(std::integral_constant<int, 0>{}, 0); run(std::integral_constant<int, 1>{}, 1);
  run(std::integral_constant<int, 2>{}, 2); run(std::integral_constant<int, 3>{}, 3);
  run(std::integral_constant<int, 4>{}, 4); run(std::integral_constant<int, 5>{}, 5);
  run(std::integral_constant<int, 6>{}, 6); run(std::integral_constant<int, 7>{}, 7);
  run(std::integral_constant<int, 8>{}, 8); run(std::integral_constant<int, 9>{}, 9);
  run(std::integral_constant<int, 10>{}, 10); run(std::integral_constant<int, 11>{}, 11);
  run(std::integral_constant<int, 12>{}, 12); run(std::integral_constant<int, 13>{}, 13);
  return 0;
}
