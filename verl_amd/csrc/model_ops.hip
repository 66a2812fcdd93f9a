// Fused elementwise / normalisation kernels for the actor's Qwen2 backbone on MI355X (bf16).
//
// These are not part of the reference's hot path; they replace the ~20 small PyTorch kernels
// per layer that HF Qwen2 issues for RMSNorm, SwiGLU and rotary embedding (plus the layout
// copies around varlen attention), which made the actor step launch-bound (GPU ~80% busy).
// Forward numerics follow the HF modules' bf16 rounding points:
//   RMSNorm  y = bf16(w * bf16(x * rsqrt(mean(x^2) + eps)))           (modeling_qwen2 Qwen2RMSNorm)
//   SwiGLU   y = bf16(bf16(silu(g)) * u)                               (Qwen2MLP)
//   RoPE     q' = bf16(bf16(q * cos) + bf16(rotate_half(q) * sin))    (apply_rotary_pos_emb)
// Backwards compute in fp32 and round once (autograd of the HF graph rounds at every op).
// All kernels are HBM-bound streaming (16-byte vectors where aligned).

#include <math.h>

#include "va_common.h"

namespace va {
namespace {

__device__ __forceinline__ float bf(uint16_t b) { return bf16_to_f32(b); }
__device__ __forceinline__ uint16_t to_bf(float f) { return static_cast<uint16_t>(f32_to_bf16_bits(f)); }
__device__ __forceinline__ float rbf(float f) { return bf(to_bf(f)); }  // round through bf16

// ------------------------------------------------------------------ RMSNorm
// one wave per row; 4 rows per 256-thread workgroup
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const uint16_t *__restrict__ x,
                                                          const uint16_t *__restrict__ w, int64_t T,
                                                          int H, float eps, uint16_t *__restrict__ y,
                                                          float *__restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const uint16_t *xr = x + row * H;
  float ss = 0.f;
  for (int h = lane; h < H; h += kWave) {
    const float v = bf(xr[h]);
    ss = fmaf(v, v, ss);
  }
  ss = wave_sum(ss);
  const float r = 1.0f / sqrtf(ss / static_cast<float>(H) + eps);
  if (lane == 0) rstd[row] = r;
  uint16_t *yr = y + row * H;
  for (int h = lane; h < H; h += kWave) {
    const float xh = rbf(bf(xr[h]) * r);
    yr[h] = to_bf(bf(w[h]) * xh);
  }
}

// dx = r * (g - xh * mean(g * xh)),  g = dy * w,  xh = x * r;  dw partials over row blocks
constexpr int kRowsPerBlock = 64;

__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(
    const uint16_t *__restrict__ dy, const uint16_t *__restrict__ x, const uint16_t *__restrict__ w,
    const float *__restrict__ rstd, int64_t T, int H, uint16_t *__restrict__ dx,
    float *__restrict__ dw_part) {
  extern __shared__ float sdw[];  // [4][H]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int h = threadIdx.x; h < 4 * H; h += 256) sdw[h] = 0.f;
  __syncthreads();
  float *mine = sdw + wave * H;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kRowsPerBlock;
  for (int64_t row = r0 + wave; row < r0 + kRowsPerBlock && row < T; row += 4) {
    const uint16_t *xr = x + row * H;
    const uint16_t *dyr = dy + row * H;
    const float r = rstd[row];
    float dot = 0.f;
    for (int h = lane; h < H; h += kWave) {
      const float xu = bf(xr[h]) * r;
      const float g = bf(dyr[h]) * bf(w[h]);
      dot = fmaf(g, xu, dot);
      mine[h] += bf(dyr[h]) * rbf(xu);  // dw sees the bf16-rounded x_hat; lanes own columns
    }
    dot = wave_sum(dot) / static_cast<float>(H);
    uint16_t *dxr = dx + row * H;
    for (int h = lane; h < H; h += kWave) {
      const float xh = bf(xr[h]) * r;
      const float g = bf(dyr[h]) * bf(w[h]);
      dxr[h] = to_bf(r * (g - xh * dot));
    }
  }
  __syncthreads();
  for (int h = threadIdx.x; h < H; h += 256)
    dw_part[static_cast<int64_t>(blockIdx.x) * H + h] = sdw[h] + sdw[H + h] + sdw[2 * H + h] + sdw[3 * H + h];
}

__global__ __launch_bounds__(256) void colsum_to_bf16_kernel(const float *__restrict__ part, int nblk,
                                                             int H, uint16_t *__restrict__ out) {
  const int h = blockIdx.x * 256 + threadIdx.x;
  if (h >= H) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[static_cast<int64_t>(b) * H + h];
  out[h] = to_bf(s);
}

// ------------------------------------------------------------------ SwiGLU
__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const uint16_t *__restrict__ g,
                                                         const uint16_t *__restrict__ u, int64_t n,
                                                         uint16_t *__restrict__ y) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * 8;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 8; i < n; i += stride) {
    if (i + 8 <= n) {
      const uint4 gv = *reinterpret_cast<const uint4 *>(g + i);
      const uint4 uv = *reinterpret_cast<const uint4 *>(u + i);
      const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w}, uw[4] = {uv.x, uv.y, uv.z, uv.w};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float a0 = rbf(silu(bf16_lo(gw[k]))), a1 = rbf(silu(bf16_hi(gw[k])));
        o[k] = (f32_to_bf16_bits(a0 * bf16_lo(uw[k]))) | (f32_to_bf16_bits(a1 * bf16_hi(uw[k])) << 16);
      }
      *reinterpret_cast<uint4 *>(y + i) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
      for (int64_t j = i; j < n; ++j) y[j] = to_bf(rbf(silu(bf(g[j]))) * bf(u[j]));
    }
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const uint16_t *__restrict__ dy,
                                                         const uint16_t *__restrict__ g,
                                                         const uint16_t *__restrict__ u, int64_t n,
                                                         uint16_t *__restrict__ dg,
                                                         uint16_t *__restrict__ du) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * 8;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 8; i < n; i += stride) {
    const int64_t e = (i + 8 <= n) ? i + 8 : n;
    if (e - i == 8) {
      const uint4 dv = *reinterpret_cast<const uint4 *>(dy + i);
      const uint4 gv = *reinterpret_cast<const uint4 *>(g + i);
      const uint4 uv = *reinterpret_cast<const uint4 *>(u + i);
      const uint32_t dw_[4] = {dv.x, dv.y, dv.z, dv.w}, gw[4] = {gv.x, gv.y, gv.z, gv.w},
                     uw[4] = {uv.x, uv.y, uv.z, uv.w};
      uint32_t og[4], ou[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float r_g[2], r_u[2];
#pragma unroll
        for (int hlf = 0; hlf < 2; ++hlf) {
          const float d = hlf ? bf16_hi(dw_[k]) : bf16_lo(dw_[k]);
          const float gg = hlf ? bf16_hi(gw[k]) : bf16_lo(gw[k]);
          const float uu = hlf ? bf16_hi(uw[k]) : bf16_lo(uw[k]);
          const float s = 1.f / (1.f + __expf(-gg));
          const float a = rbf(gg * s);
          r_u[hlf] = d * a;
          r_g[hlf] = d * uu * (s * (1.f + gg * (1.f - s)));
        }
        og[k] = f32_to_bf16_bits(r_g[0]) | (f32_to_bf16_bits(r_g[1]) << 16);
        ou[k] = f32_to_bf16_bits(r_u[0]) | (f32_to_bf16_bits(r_u[1]) << 16);
      }
      *reinterpret_cast<uint4 *>(dg + i) = make_uint4(og[0], og[1], og[2], og[3]);
      *reinterpret_cast<uint4 *>(du + i) = make_uint4(ou[0], ou[1], ou[2], ou[3]);
    } else {
      for (int64_t j = i; j < e; ++j) {
        const float d = bf(dy[j]), gg = bf(g[j]), uu = bf(u[j]);
        const float s = 1.f / (1.f + __expf(-gg));
        du[j] = to_bf(d * rbf(gg * s));
        dg[j] = to_bf(d * uu * (s * (1.f + gg * (1.f - s))));
      }
    }
  }
}

// ------------------------------------------------------------------ RoPE (rotate_half form)
// q [T, Hq, D], k [T, Hk, D], cos / sin [T, D] -> same layouts; one thread per (t, head, j < D/2)
__global__ __launch_bounds__(256) void rope_kernel(const uint16_t *__restrict__ q,
                                                   const uint16_t *__restrict__ k,
                                                   const uint16_t *__restrict__ cs,
                                                   const uint16_t *__restrict__ sn, int64_t T, int Hq,
                                                   int Hk, int D, int backward,
                                                   uint16_t *__restrict__ qo,
                                                   uint16_t *__restrict__ ko) {
  const int half = D / 2;
  const int64_t per_t = static_cast<int64_t>(Hq + Hk) * half;
  const int64_t total = T * per_t;
  for (int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; idx < total;
       idx += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t t = idx / per_t;
    const int rem = static_cast<int>(idx - t * per_t);
    const int head = rem / half, j = rem - head * half;
    const uint16_t *src;
    uint16_t *dst;
    if (head < Hq) {
      src = q + (t * Hq + head) * D;
      dst = qo + (t * Hq + head) * D;
    } else {
      src = k + (t * Hk + (head - Hq)) * D;
      dst = ko + (t * Hk + (head - Hq)) * D;
    }
    const float x1 = bf(src[j]), x2 = bf(src[j + half]);
    const float c1 = bf(cs[t * D + j]), c2 = bf(cs[t * D + j + half]);
    const float s1 = bf(sn[t * D + j]), s2 = bf(sn[t * D + j + half]);
    if (!backward) {
      // out[j] = x1*c1 + (-x2)*s1 ; out[j+half] = x2*c2 + x1*s2  (bf16 after each op)
      dst[j] = to_bf(rbf(x1 * c1) + rbf(-x2 * s1));
      dst[j + half] = to_bf(rbf(x2 * c2) + rbf(x1 * s2));
    } else {
      // d x1 = g1*c1 + g2*s2 ; d x2 = g2*c2 - g1*s1
      dst[j] = to_bf(x1 * c1 + x2 * s2);
      dst[j + half] = to_bf(x2 * c2 - x1 * s1);
    }
  }
}

int64_t grid_for(int64_t n, int per_thread) {
  int64_t g = (n + 256LL * per_thread - 1) / (256LL * per_thread);
  return g < 1 ? 1 : (g > 65536 ? 65536 : g);
}

}  // namespace
}  // namespace va

using namespace va;

extern "C" int64_t va_rmsnorm_workspace_bytes(int64_t T, int64_t H) {
  return static_cast<int64_t>(sizeof(float)) * ((T + kRowsPerBlock - 1) / kRowsPerBlock) * H;
}

extern "C" int va_rmsnorm_fwd(const void *x, const void *w, int dtype, int64_t T, int64_t H, float eps,
                              void *y, float *rstd, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "rmsnorm: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && H > 0 && H <= 16384, "rmsnorm: bad shape");
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(x && w && y && rstd, "null pointer argument");
  hipLaunchKernelGGL(rmsnorm_fwd_kernel, dim3((T + 3) / 4), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t *>(x), static_cast<const uint16_t *>(w), T, static_cast<int>(H),
                     eps, static_cast<uint16_t *>(y), rstd);
  return check_launch("rmsnorm_fwd");
}

extern "C" int va_rmsnorm_bwd(const void *dy, const void *x, const void *w, const float *rstd, int dtype,
                              int64_t T, int64_t H, void *dx, void *dw, float *workspace, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "rmsnorm: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && H > 0 && H <= 8192, "rmsnorm: bad shape");
  VA_CHECK_ARG(dy && x && w && rstd && dx && dw && workspace, "null pointer argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nblk = (T + kRowsPerBlock - 1) / kRowsPerBlock;
  if (nblk > 0) {
    const size_t shm = static_cast<size_t>(4 * H) * sizeof(float);
    if (shm > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void *>(&rmsnorm_bwd_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(shm)) != hipSuccess) {
      set_error("rmsnorm_bwd: cannot reserve %zu bytes of LDS", shm);
      return VA_E_LAUNCH;
    }
    hipLaunchKernelGGL(rmsnorm_bwd_kernel, dim3(nblk), dim3(256), shm, s, static_cast<const uint16_t *>(dy),
                       static_cast<const uint16_t *>(x), static_cast<const uint16_t *>(w), rstd, T,
                       static_cast<int>(H), static_cast<uint16_t *>(dx), workspace);
  }
  hipLaunchKernelGGL(colsum_to_bf16_kernel, dim3((H + 255) / 256), dim3(256), 0, s, workspace,
                     static_cast<int>(nblk), static_cast<int>(H), static_cast<uint16_t *>(dw));
  return check_launch("rmsnorm_bwd");
}

extern "C" int va_swiglu_fwd(const void *g, const void *u, int dtype, int64_t n, void *y, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "swiglu: only bf16 is implemented");
  if (n == 0) return VA_OK;
  VA_CHECK_ARG(g && u && y && n > 0, "bad arguments");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(g) % 16 == 0 && reinterpret_cast<uintptr_t>(u) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(y) % 16 == 0, "swiglu: 16-byte aligned buffers required");
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(n, 8)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t *>(g), static_cast<const uint16_t *>(u), n,
                     static_cast<uint16_t *>(y));
  return check_launch("swiglu_fwd");
}

extern "C" int va_swiglu_bwd(const void *dy, const void *g, const void *u, int dtype, int64_t n, void *dg,
                             void *du, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "swiglu: only bf16 is implemented");
  if (n == 0) return VA_OK;
  VA_CHECK_ARG(dy && g && u && dg && du && n > 0, "bad arguments");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(dy) % 16 == 0 && reinterpret_cast<uintptr_t>(g) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(u) % 16 == 0 && reinterpret_cast<uintptr_t>(dg) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(du) % 16 == 0, "swiglu: 16-byte aligned buffers required");
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(n, 8)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t *>(dy), static_cast<const uint16_t *>(g),
                     static_cast<const uint16_t *>(u), n, static_cast<uint16_t *>(dg),
                     static_cast<uint16_t *>(du));
  return check_launch("swiglu_bwd");
}

extern "C" int va_rope(const void *q, const void *k, const void *cos, const void *sin, int dtype, int64_t T,
                       int64_t Hq, int64_t Hk, int64_t D, int backward, void *qo, void *ko, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "rope: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && Hq > 0 && Hk >= 0 && D > 0 && D % 2 == 0, "rope: bad shape");
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(q && cos && sin && qo && (Hk == 0 || (k && ko)), "null pointer argument");
  const int64_t total = T * (Hq + Hk) * (D / 2);
  hipLaunchKernelGGL(rope_kernel, dim3(grid_for(total, 4)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t *>(q), static_cast<const uint16_t *>(k),
                     static_cast<const uint16_t *>(cos), static_cast<const uint16_t *>(sin), T,
                     static_cast<int>(Hq), static_cast<int>(Hk), static_cast<int>(D), backward,
                     static_cast<uint16_t *>(qo), static_cast<uint16_t *>(ko));
  return check_launch("rope");
}
