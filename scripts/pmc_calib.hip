// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of the
// episode kernels (MI355X_MICROARCH.md: only 16-B/lane streaming reads (FETCH_SIZE = 1/2 of the bytes)
// and 16-B/lane streaming stores (exact) are calibrated; every other width must be measured on a
// known byte count).  One launch per pattern, each moving a known number of bytes of a buffer far
// larger than the 256 MiB Infinity Cache, every byte touched once (no reuse a cache could absorb):
//   gather32  one 32-B row per lane (two 16-B loads), rows scattered by a bijective hash   (f64 Q rows)
//   gather16  one 16-B row per lane, scattered                                             (f32 Q rows)
//   stream8   8 B per lane, coalesced (consecutive lanes, consecutive 8 B)        (profile / step words)
//   stream4   4 B per lane, coalesced                                             (exploration code words)
//   wstream8  8-B coalesced stores                                                ({reward, cost} records)
//   wstream32 32-B per lane coalesced stores (two 16-B stores)                   (FastRec record rows)
//   wscat8    8-B stores, one per scattered 32-B row                              (the TD store of a Q entry)
//   wscat32   32-B stores (two 16-B), one per scattered 32-B row
// Run under rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE (separate passes); the kernel trace
// gives one counter value per launch, scripts/summarize_pmc_calib.py divides by the bytes printed here.
//   hipcc --offload-arch=gfx950 -O3 -o pmc_calib pmc_calib.hip && ./pmc_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

constexpr size_t kBuf = 2ull << 30;  // 2 GiB per buffer, 8x the Infinity Cache

// a bijection on [0, 2^bits): odd multiply + xorshift, masked (every row exactly once)
__device__ __forceinline__ uint32_t scatter(uint32_t k, int bits) {
  const uint32_t m = (bits >= 32) ? 0xFFFFFFFFu : ((1u << bits) - 1u);
  k = (k * 0x9E3779B1u) & m;
  k ^= k >> (bits / 2);
  return (k * 0x85EBCA77u) & m;
}

__global__ void fill(uint4* p, size_t n) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x)
    p[k] = make_uint4((uint32_t)k, (uint32_t)(k >> 7), 3u, 5u);
}

template <int ROW>  // 32 or 16 bytes
__global__ void gather(const char* __restrict__ t, uint32_t rows, int bits, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < rows; k += gridDim.x * blockDim.x) {
    const char* p = t + (size_t)scatter(k, bits) * ROW;
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    acc ^= a.x ^ a.w;
    if (ROW == 32) {
      const uint4 b = *reinterpret_cast<const uint4*>(p + 16);
      acc ^= b.y ^ b.z;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads; never true for this fill
}

template <typename V>
__global__ void stream(const V* __restrict__ p, size_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
    const V v = p[k];
    acc ^= reinterpret_cast<const uint32_t*>(&v)[0];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename V>
__global__ void wstream(V* __restrict__ p, size_t n) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
    V v;
    reinterpret_cast<uint32_t*>(&v)[0] = (uint32_t)k;
    for (int j = 1; j < (int)(sizeof(V) / 4); ++j) reinterpret_cast<uint32_t*>(&v)[j] = (uint32_t)j;
    p[k] = v;
  }
}

__global__ void wstream32(uint4* __restrict__ p, size_t n_rows) {  // row k = two 16-B stores
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_rows; k += (size_t)gridDim.x * blockDim.x) {
    p[2 * k] = make_uint4((uint32_t)k, 1u, 2u, 3u);
    p[2 * k + 1] = make_uint4(4u, 5u, 6u, (uint32_t)k);
  }
}

template <int BYTES>  // 8 or 32 bytes stored into each scattered 32-B row
__global__ void wscatter(char* __restrict__ t, uint32_t rows, int bits) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < rows; k += gridDim.x * blockDim.x) {
    char* p = t + (size_t)scatter(k, bits) * 32;
    if (BYTES == 8) {
      *reinterpret_cast<uint2*>(p + 8) = make_uint2(k, 7u);  // entry 1 of a padded f64 row
    } else {
      reinterpret_cast<uint4*>(p)[0] = make_uint4(k, 1u, 2u, 3u);
      reinterpret_cast<uint4*>(p)[1] = make_uint4(4u, 5u, 6u, k);
    }
  }
}

int main() {
  char *a = nullptr, *b = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&a, kBuf));
  CK(hipMalloc(&b, kBuf));
  CK(hipMalloc(&sink, 64));
  const dim3 grid(8192), blk(256);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint4*>(a), kBuf / 16);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint4*>(b), kBuf / 16);
  CK(hipDeviceSynchronize());
  // each pattern: a half-buffer's worth of bytes (1 GiB), every 32-B / 16-B row once
  const int bits32 = 25, bits16 = 26;           // 2^25 rows x 32 B = 1 GiB; 2^26 x 16 B = 1 GiB
  const uint32_t rows32 = 1u << bits32, rows16 = 1u << bits16;
  const size_t n8 = (1ull << 30) / 8, n4 = (1ull << 30) / 4;
  struct Item { const char* name; double bytes; const char* dir; };
  Item items[8];
  int m = 0;
  // reads from a, writes to b, alternating so no launch finds the previous one's lines in a cache
  hipLaunchKernelGGL(gather<32>, grid, blk, 0, 0, a, rows32, bits32, sink);
  items[m++] = {"gather32", (double)rows32 * 32, "read"};
  hipLaunchKernelGGL(gather<16>, grid, blk, 0, 0, b, rows16, bits16, sink);
  items[m++] = {"gather16", (double)rows16 * 16, "read"};
  hipLaunchKernelGGL(stream<uint2>, grid, blk, 0, 0, reinterpret_cast<const uint2*>(a + (1ull << 30)), n8, sink);
  items[m++] = {"stream8", (double)n8 * 8, "read"};
  hipLaunchKernelGGL(stream<uint32_t>, grid, blk, 0, 0, reinterpret_cast<const uint32_t*>(b + (1ull << 30)), n4, sink);
  items[m++] = {"stream4", (double)n4 * 4, "read"};
  hipLaunchKernelGGL(wstream<uint2>, grid, blk, 0, 0, reinterpret_cast<uint2*>(a), n8);
  items[m++] = {"wstream8", (double)n8 * 8, "write"};
  hipLaunchKernelGGL(wstream32, grid, blk, 0, 0, reinterpret_cast<uint4*>(b), (size_t)rows32);
  items[m++] = {"wstream32", (double)rows32 * 32, "write"};
  hipLaunchKernelGGL(wscatter<8>, grid, blk, 0, 0, a + (1ull << 30), rows32, bits32);
  items[m++] = {"wscat8", (double)rows32 * 8, "write"};
  hipLaunchKernelGGL(wscatter<32>, grid, blk, 0, 0, b + (1ull << 30), rows32, bits32);
  items[m++] = {"wscat32", (double)rows32 * 32, "write"};
  CK(hipDeviceSynchronize());
  printf("[");
  for (int k = 0; k < m; ++k)
    printf("%s{\"pattern\": \"%s\", \"launch\": %d, \"bytes\": %.0f, \"dir\": \"%s\"}", k ? ", " : "", items[k].name,
           k + 2, items[k].bytes, items[k].dir);
  printf("]\n");
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
