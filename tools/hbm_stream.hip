// HBM streaming calibration on one MI355X: what read-only, write-only and read+write (copy)
// bandwidth does a plain 16-B-per-lane kernel reach at the log-prob kernels' footprint
// (8192 x 151936 bf16 = 2.49 GB per operand)? Variants: vectors in flight per lane (U),
// non-temporal vs default policy, waves per workgroup, grid = one chunk per WG vs persistent.
// Prints one JSON line per variant. Not part of the product path.
//
//   hipcc -O3 --offload-arch=gfx950 -o gpurun_out/hbm_stream tools/hbm_stream.hip && gpurun_out/hbm_stream

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// MODE 0 copy, 1 read (xor-reduce, one store per thread), 2 write
template <int MODE, int U, bool NT>
__global__ void stream_kernel(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, int64_t n, int64_t iters_stride) {
  const int64_t per_iter = static_cast<int64_t>(gridDim.x) * blockDim.x * U;
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x * U + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * static_cast<int64_t>(blockDim.x) < n; i += per_iter) {
    u32x4 r[U];
    if constexpr (MODE != 2) {
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = ld<NT>(src + i + u * blockDim.x);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = u32x4{(unsigned)i, 1u, 2u, (unsigned)u};
    }
    if constexpr (MODE == 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= r[u];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) st<NT>(dst + i + u * blockDim.x, r[u]);
    }
  }
  (void)iters_stride;
  if constexpr (MODE == 1) {
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) dst[threadIdx.x] = acc;  // keep the loads
  }
}

template <int MODE, int U, bool NT>
int run(const char *name, const u32x4 *src, u32x4 *dst, int64_t n, int block, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((stream_kernel<MODE, U, NT>), dim3(grid), dim3(block), 0, 0, src, dst, n, 0);
  CK(hipDeviceSynchronize());
  const int iters = 20;
  CK(hipEventRecord(a));
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((stream_kernel<MODE, U, NT>), dim3(grid), dim3(block), 0, 0, src, dst, n, 0);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / iters;
  const double bytes = static_cast<double>(n) * 16.0 * (MODE == 0 ? 2.0 : 1.0);
  printf("{\"mode\": \"%s\", \"U\": %d, \"nt\": %d, \"block\": %d, \"grid\": %d, \"us\": %.1f, \"gbps\": %.1f}\n", name, U,
         NT ? 1 : 0, block, grid, us, bytes / us / 1e3);
  fflush(stdout);
  return 0;
}

int main(int argc, char **argv) {
  // one bf16 logits buffer of a micro-batch: rows x 151,936 (argv[1], default 8192 rows)
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 8192;
  const int64_t bytes = rows * 151936 * 2;
  const int64_t n = bytes / 16;
  u32x4 *src, *dst;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMemset(src, 1, bytes));
  CK(hipMemset(dst, 0, bytes));
  const int grids[] = {0, 1024, 2048, 4096};
  for (int g : grids) {
    for (int block : {256, 512}) {
      // g == 0: one U-vector chunk per thread (no grid stride)
      const int grid1 = g ? g : static_cast<int>((n + block * 4 - 1) / (block * 4));
      run<0, 4, true>("copy", src, dst, n, block, grid1);
      run<0, 4, true>("copy_inplace", src, src, n, block, grid1);
      run<0, 4, false>("copy", src, dst, n, block, grid1);
      run<1, 4, true>("read", src, dst, n, block, grid1);
      run<2, 4, true>("write", src, dst, n, block, grid1);
      if (g) {
        run<0, 2, true>("copy", src, dst, n, block, g);
        run<0, 8, true>("copy", src, dst, n, block, g);
        run<1, 8, true>("read", src, dst, n, block, g);
      }
    }
  }
  CK(hipFree(src));
  CK(hipFree(dst));
  return 0;
}
