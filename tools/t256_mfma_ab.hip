// Probe: the f1 transposed 256 x 256 sweep (linear_logprob.hip t256_sweep) with its MFMA shape as the
// variable: v_mfma_f32_16x16x32_bf16 (the product: 8 x 4 blocks per wave, 50 % of the SIMD's issue
// held per MFMA) vs v_mfma_f32_32x32x16_bf16 (4 x 2 blocks per wave, 25 % held: more issue slots for
// the LDS reads, the LDS-DMA and the epilogue). Same LDS images, swizzle, staging and XCD remap.
// Epilogue: EPI = 0 a max over the accumulators (core only), EPI = 1 the f1 online log-softmax
// statistics (max pass, bf16 rounding, exp2, two sums) without the label. Times each on random data.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I verl_amd/csrc -mllvm -amdgpu-mfma-vgpr-form=1 \
//     tools/t256_mfma_ab.hip -o tools/bin/t256_mfma_ab   (the flag: the 4-wave arm spills without it)
//   tools/bin/t256_mfma_ab N K V splits iters
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "va_common.h"
using namespace va;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TB = 256, TK = 64, T_THREADS = 512, T_TILE = TB * TK;
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ int t_img_off(int row, int c) { return row * TK + ((c ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ void t_stage(const uint16_t *__restrict__ src, int64_t row0, int64_t nrows, int64_t ld,
                                        int k0, uint16_t *img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int g = wave * 4 + i;
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    int64_t gr = row0 + row;
    if (gr >= nrows) gr = nrows - 1;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + gr * ld + k0 + lc * 8), img + g * 8 * TK,
                                     16, 0, 0);
  }
}

__device__ __forceinline__ float base_of(float m) { return m == -INFINITY ? 0.f : m * kLog2e; }

// per-token online statistics over NV values of this lane (bf16-rounded logits)
template <int NV>
__device__ __forceinline__ void fold(const float *x, float &m, float &s, float &t) {
  float rm = x[0];
#pragma unroll
  for (int u = 1; u < NV; ++u) rm = fmaxf(rm, x[u]);
  const float lm = round_to_bf16(rm);
  const float nm = fmaxf(m, lm);
  const float nb = base_of(nm);
  const float alpha = __builtin_amdgcn_exp2f(base_of(m) - nb);
  const va_f32x2 l2e = {kLog2e, kLog2e}, nnb = {-nb, -nb};
  va_f32x2 ss = {0.f, 0.f}, tt = {0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NV; u += 2) {
    const uint32_t p = pack2_bf16(x[u], x[u + 1]);
    const va_f32x2 v = {__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
    const va_f32x2 arg = __builtin_elementwise_fma(v, l2e, nnb);
    const va_f32x2 ex = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
    ss = ss + ex;
    tt = __builtin_elementwise_fma(ex, v, tt);
  }
  s = fmaf(s, alpha, ss.x + ss.y);
  t = fmaf(t, alpha, tt.x + tt.y);
  m = nm;
}

template <int MF, int EPI>
__global__ __launch_bounds__(T_THREADS, 1) void sweep_kernel(const uint16_t *__restrict__ hid,
                                                             const uint16_t *__restrict__ w, int64_t N, int K,
                                                             int64_t V, int splits, int per, float *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * T_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  int64_t L = blockIdx.x;
  {
    const int64_t nl = gridDim.x >> 3;
    if ((gridDim.x & 7) == 0) L = (L & 7) * nl + (L >> 3);
  }
  const int64_t rb = L / splits, sp = L % splits, row0 = rb * TB;
  const int64_t n_vt = (V + TB - 1) / TB;
  const int64_t vt_begin = sp * per, vt_end = std::min<int64_t>(vt_begin + per, n_vt);
  const int nk = K / TK;
  const int64_t nsteps = vt_begin < vt_end ? (vt_end - vt_begin) * nk : 0;
  constexpr int NI = MF == 16 ? 8 : 4, NJ = MF == 16 ? 4 : 2;
  typedef typename std::conditional<MF == 16, f32x4, f32x16>::type accT;
  constexpr int NE = MF == 16 ? 4 : 16;
  accT acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[i][j][e] = 0.f;
  float m[NJ], s[NJ], t[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) m[j] = -INFINITY, s[j] = 0.f, t[j] = 0.f;

  if (nsteps > 0) {
    t_stage(w, vt_begin * TB, V, K, 0, lds, wave, lane);
    t_stage(hid, row0, N, K, 0, lds + T_TILE, wave, lane);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int64_t st = 0; st < nsteps; ++st) {
    const int buf = static_cast<int>(st & 1);
    const int kt = static_cast<int>(st % nk);
    const uint16_t *la = lds + buf * 2 * T_TILE;
    const uint16_t *lb = la + T_TILE;
    if (st + 1 < nsteps) {
      uint16_t *na = lds + (buf ^ 1) * 2 * T_TILE;
      const int k1 = static_cast<int>((st + 1) % nk) * TK;
      t_stage(w, (vt_begin + (st + 1) / nk) * TB, V, K, k1, na, wave, lane);
      t_stage(hid, row0, N, K, k1, na + T_TILE, wave, lane);
    }
    if constexpr (MF == 16) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = q * 4 + (lane >> 4);
        bf16x8 fa[8], fb[4];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          fa[i] = *reinterpret_cast<const bf16x8 *>(la + t_img_off(wr * 128 + i * 16 + (lane & 15), c));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          fb[j] = *reinterpret_cast<const bf16x8 *>(lb + t_img_off(wc * 64 + j * 16 + (lane & 15), c));
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = q * 2 + (lane >> 5);
        bf16x8 fa[4], fb[2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[i] = *reinterpret_cast<const bf16x8 *>(la + t_img_off(wr * 128 + i * 32 + (lane & 31), c));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[j] = *reinterpret_cast<const bf16x8 *>(lb + t_img_off(wc * 64 + j * 32 + (lane & 31), c));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt == nk - 1) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float x[NI * NE];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int e = 0; e < NE; ++e) x[i * NE + e] = acc[i][j][e];
        if constexpr (EPI == 0) {
          float rm = x[0];
#pragma unroll
          for (int u = 1; u < NI * NE; ++u) rm = fmaxf(rm, x[u]);
          m[j] = fmaxf(m[j], rm);
        } else {
          fold<NI * NE>(x, m[j], s[j], t[j]);
        }
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int e = 0; e < NE; ++e) acc[i][j][e] = 0.f;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  float r = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) r += m[j] + s[j] + t[j];
  out[static_cast<int64_t>(blockIdx.x) * T_THREADS + tid] = r;
}

// one wave per SIMD: 4 waves of 128 x 128 (2 vocab halves x 2 token halves), 16x16x32, acc[8][8]
// (256 accumulator registers: the compiler must place them in AGPRs)
__device__ __forceinline__ void t_stage4(const uint16_t *__restrict__ src, int64_t row0, int64_t nrows, int64_t ld,
                                         int k0, uint16_t *img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int g = wave * 8 + i;
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    int64_t gr = row0 + row;
    if (gr >= nrows) gr = nrows - 1;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + gr * ld + k0 + lc * 8), img + g * 8 * TK,
                                     16, 0, 0);
  }
}

template <int EPI>
__global__ __launch_bounds__(256, 1) void sweep4_kernel(const uint16_t *__restrict__ hid,
                                                        const uint16_t *__restrict__ w, int64_t N, int K,
                                                        int64_t V, int splits, int per, float *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * T_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  int64_t L = blockIdx.x;
  {
    const int64_t nl = gridDim.x >> 3;
    if ((gridDim.x & 7) == 0) L = (L & 7) * nl + (L >> 3);
  }
  const int64_t rb = L / splits, sp = L % splits, row0 = rb * TB;
  const int64_t n_vt = (V + TB - 1) / TB;
  const int64_t vt_begin = sp * per, vt_end = std::min<int64_t>(vt_begin + per, n_vt);
  const int nk = K / TK;
  const int64_t nsteps = vt_begin < vt_end ? (vt_end - vt_begin) * nk : 0;
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[8], s[8], t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = -INFINITY, s[j] = 0.f, t[j] = 0.f;
  if (nsteps > 0) {
    t_stage4(w, vt_begin * TB, V, K, 0, lds, wave, lane);
    t_stage4(hid, row0, N, K, 0, lds + T_TILE, wave, lane);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int64_t st = 0; st < nsteps; ++st) {
    const int buf = static_cast<int>(st & 1);
    const int kt = static_cast<int>(st % nk);
    const uint16_t *la = lds + buf * 2 * T_TILE;
    const uint16_t *lb = la + T_TILE;
    if (st + 1 < nsteps) {
      uint16_t *na = lds + (buf ^ 1) * 2 * T_TILE;
      const int k1 = static_cast<int>((st + 1) % nk) * TK;
      t_stage4(w, (vt_begin + (st + 1) / nk) * TB, V, K, k1, na, wave, lane);
      t_stage4(hid, row0, N, K, k1, na + T_TILE, wave, lane);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = q * 4 + (lane >> 4);
      bf16x8 fa[8], fb[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        fa[i] = *reinterpret_cast<const bf16x8 *>(la + t_img_off(wr * 128 + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < 8; ++j)
        fb[j] = *reinterpret_cast<const bf16x8 *>(lb + t_img_off(wc * 128 + j * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt == nk - 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x[32];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) x[i * 4 + e] = acc[i][j][e];
        if constexpr (EPI == 0) {
          float rm = x[0];
#pragma unroll
          for (int u = 1; u < 32; ++u) rm = fmaxf(rm, x[u]);
          m[j] = fmaxf(m[j], rm);
        } else {
          fold<32>(x, m[j], s[j], t[j]);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  float r = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) r += m[j] + s[j] + t[j];
  out[static_cast<int64_t>(blockIdx.x) * T_THREADS + tid] = r;
}

__global__ void fill_kernel(uint16_t *p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13, x *= 0x5bd1e995u, x ^= x >> 15;
    const float u = ((x & 0xffffff) / 16777216.f - 0.5f) * 3.4641f * scale;  // unit variance * scale
    p[i] = static_cast<uint16_t>(pack2_bf16(u, 0.f) & 0xffff);
  }
}

template <int MF, int EPI>
static float run(const uint16_t *h, const uint16_t *w, int64_t N, int K, int64_t V, int splits, float *out,
                 int iters) {
  const int64_t n_vt = (V + TB - 1) / TB;
  const int per = (int)((n_vt + splits - 1) / splits);
  const int used = (int)((n_vt + per - 1) / per);
  const int64_t nwg = ((N + TB - 1) / TB) * used;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int it = 0; it < iters + 1; ++it) {
    CK(hipEventRecord(e0));
    if constexpr (MF == 4)
      hipLaunchKernelGGL((sweep4_kernel<EPI>), dim3((unsigned)nwg), dim3(256), 0, 0, h, w, N, K, V, used, per, out);
    else
      hipLaunchKernelGGL((sweep_kernel<MF, EPI>), dim3((unsigned)nwg), dim3(T_THREADS), 0, 0, h, w, N, K, V, used,
                         per, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it > 0) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 131072;
  const int K = argc > 2 ? atoi(argv[2]) : 896;
  const int64_t V = argc > 3 ? atoll(argv[3]) : 151936;
  const int splits = argc > 4 ? atoi(argv[4]) : 8;
  const int iters = argc > 5 ? atoi(argv[5]) : 5;
  if (K % TK) return fprintf(stderr, "K %% 64\n"), 1;
  uint16_t *h, *w;
  float *out;
  CK(hipMalloc(&h, N * K * 2));
  CK(hipMalloc(&w, V * K * 2));
  const int64_t n_vt = (V + TB - 1) / TB;
  CK(hipMalloc(&out, ((N + TB - 1) / TB) * n_vt * T_THREADS * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, h, N * K, 1u, 1.f);
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, w, V * K, 7u, 0.05f);
  CK(hipDeviceSynchronize());
  const double tf = 2.0 * N * K * V / 1e12;
  // interleaved: each arm twice, alternating
  for (int rep = 0; rep < 2; ++rep) {
    const float a0 = run<16, 0>(h, w, N, K, V, splits, out, iters);
    const float b0 = run<32, 0>(h, w, N, K, V, splits, out, iters);
    const float a1 = run<16, 1>(h, w, N, K, V, splits, out, iters);
    const float b1 = run<32, 1>(h, w, N, K, V, splits, out, iters);
    const float c0 = run<4, 0>(h, w, N, K, V, splits, out, iters);
    const float c1 = run<4, 1>(h, w, N, K, V, splits, out, iters);
    printf("{\"N\": %lld, \"K\": %d, \"V\": %lld, \"splits\": %d, \"rep\": %d, \"core_16x16x32_ms\": %.3f, "
           "\"core_32x32x16_ms\": %.3f, \"epi_16x16x32_ms\": %.3f, \"epi_32x32x16_ms\": %.3f, "
           "\"core_4wave_128x128_ms\": %.3f, \"epi_4wave_128x128_ms\": %.3f, "
           "\"core_tflops\": [%.1f, %.1f, %.1f], \"epi_tflops\": [%.1f, %.1f, %.1f]}\n",
           (long long)N, K, (long long)V, splits, rep, a0, b0, a1, b1, c0, c1, tf / a0 * 1e3, tf / b0 * 1e3,
           tf / c0 * 1e3, tf / a1 * 1e3, tf / b1 * 1e3, tf / c1 * 1e3);
    fflush(stdout);
  }
  return 0;
}
