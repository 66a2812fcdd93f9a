// Fused elementwise / normalisation kernels for the actor's Qwen2 backbone on MI355X (bf16).
//
// These are not part of the reference's hot path; they replace the PyTorch op chains HF Qwen2
// issues per decoder layer (RMSNorm ~8 ops, residual add, SwiGLU 2-3 ops, rotary ~10 ops plus
// the layout copies around varlen attention), so that the packed actor step is GEMM/attention
// bound rather than bound by small HBM round trips.
// Forward numerics follow the HF modules' bf16 rounding points:
//   residual  h = bf16(x + r)                                           (Qwen2DecoderLayer)
//   RMSNorm   y = bf16(w * bf16(h * rsqrt(mean(h^2) + eps)))           (Qwen2RMSNorm)
//   SwiGLU    y = bf16(bf16(silu(g)) * u)                               (Qwen2MLP)
//   RoPE      q' = bf16(bf16(q * cos) + bf16(rotate_half(q) * sin))    (apply_rotary_pos_emb)
// Backwards compute in fp32 and round once (autograd of the HF graph rounds at every op).
//
// Layout / mapping (all HBM-bound streaming, 16-byte accesses):
//   * RMSNorm: one wave64 per row, the row held in registers as NV 16-byte vectors per lane
//     (NV = ceil(H / 512)); fwd writes h (when a residual is added), y and rstd.  bwd keeps the
//     per-lane dw partial for its columns in registers across the rows of a workgroup, reduces
//     the 4 waves through LDS into a [n_blocks, H] fp32 partial, then a column-sum kernel
//     produces dw (fixed order: deterministic).
//   * RoPE reads the merged q|k|v projection [T, (Hq+2Hk)*D] once and writes q, k (rotated) and
//     v in flash varlen's [T, H, D] layout; its backward writes the merged gradient directly.

#include <math.h>

#include "va_common.h"

namespace va {
namespace {

__device__ __forceinline__ float bf(uint16_t b) { return bf16_to_f32(b); }
__device__ __forceinline__ uint16_t to_bf(float f) { return static_cast<uint16_t>(pack2_bf16(f, 0.f) & 0xffffu); }
__device__ __forceinline__ float rbf(float f) { return round_to_bf16(f); }  // round through bf16

// 8 bf16 <-> 8 floats
__device__ __forceinline__ void unpack8(const uint4 v, float (&f)[8]) {
  f[0] = bf16_lo(v.x); f[1] = bf16_hi(v.x); f[2] = bf16_lo(v.y); f[3] = bf16_hi(v.y);
  f[4] = bf16_lo(v.z); f[5] = bf16_hi(v.z); f[6] = bf16_lo(v.w); f[7] = bf16_hi(v.w);
}
__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack2_bf16(f[0], f[1]), pack2_bf16(f[2], f[3]), pack2_bf16(f[4], f[5]),
                    pack2_bf16(f[6], f[7]));
}
__device__ __forceinline__ uint4 ld16(const uint16_t *p) { return *reinterpret_cast<const uint4 *>(p); }
__device__ __forceinline__ void st16(uint16_t *p, uint4 v) { *reinterpret_cast<uint4 *>(p) = v; }

// ------------------------------------------------------------------ RMSNorm (+ residual add)
template <int NV>
__global__ __launch_bounds__(256) void add_rmsnorm_fwd_kernel(
    const uint16_t *__restrict__ x, const uint16_t *__restrict__ res, const uint16_t *__restrict__ w,
    int64_t T, int H, float eps, uint16_t *__restrict__ hout, uint16_t *__restrict__ y,
    float *__restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const int nvec = H >> 3;
  const uint16_t *xr = x + row * H;
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = lane + k * kWave;
    if (i < nvec) {
      unpack8(ld16(xr + i * 8), v[k]);
      if (res != nullptr) {
        float r8[8];
        unpack8(ld16(res + row * H + i * 8), r8);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[k][e] = rbf(v[k][e] + r8[e]);
        st16(hout + row * H + i * 8, pack8(v[k]));
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ss = fmaf(v[k][e], v[k][e], ss);
    }
  }
  ss = wave_sum(ss);
  const float r = 1.0f / sqrtf(ss / static_cast<float>(H) + eps);
  if (lane == 0) rstd[row] = r;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = lane + k * kWave;
    if (i < nvec) {
      float w8[8], o[8];
      unpack8(ld16(w + i * 8), w8);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = w8[e] * rbf(v[k][e] * r);
      st16(y + row * H + i * 8, pack8(o));
    }
  }
}

// dh = r * (g - xh * mean(g * xh)) (+ dres),  g = dy * w,  xh = h * r;  dw += dy * bf16(xh)
template <int NV>
__global__ __launch_bounds__(256) void add_rmsnorm_bwd_kernel(
    const uint16_t *__restrict__ dy, const uint16_t *__restrict__ h, const uint16_t *__restrict__ w,
    const float *__restrict__ rstd, const uint16_t *__restrict__ dres, int64_t T, int H,
    int rows_per_block, uint16_t *__restrict__ dx, float *__restrict__ dw_part) {
  extern __shared__ float sdw[];  // [4][H]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nvec = H >> 3;
  float acc[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > T) r1 = T;
  for (int64_t row = r0 + wave; row < r1; row += 4) {
    const float r = rstd[row];
    float hv[NV][8], g[NV][8];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int i = lane + k * kWave;
      if (i < nvec) {
        float d8[8], w8[8];
        unpack8(ld16(h + row * H + i * 8), hv[k]);
        unpack8(ld16(dy + row * H + i * 8), d8);
        unpack8(ld16(w + i * 8), w8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = hv[k][e] * r;
          g[k][e] = d8[e] * w8[e];
          dot = fmaf(g[k][e], xh, dot);
          acc[k][e] = fmaf(d8[e], rbf(xh), acc[k][e]);
        }
      }
    }
    const float mean = wave_sum(dot) / static_cast<float>(H);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int i = lane + k * kWave;
      if (i < nvec) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = r * (g[k][e] - hv[k][e] * r * mean);
        if (dres != nullptr) {
          float a8[8];
          unpack8(ld16(dres + row * H + i * 8), a8);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += a8[e];
        }
        st16(dx + row * H + i * 8, pack8(o));
      }
    }
  }
  // 4 waves -> one [H] partial per workgroup (lanes own disjoint columns: no conflicts)
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = lane + k * kWave;
    if (i < nvec) {
#pragma unroll
      for (int e = 0; e < 8; ++e) sdw[wave * H + i * 8 + e] = acc[k][e];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256)
    dw_part[static_cast<int64_t>(blockIdx.x) * H + c] = (sdw[c] + sdw[H + c]) + (sdw[2 * H + c] + sdw[3 * H + c]);
}

// dw[c] = bf16(sum_b part[b, c]); kColsumCols columns x (1024 / kColsumCols) row groups per workgroup,
// fixed-order merge. 16 columns per workgroup (round 5; 64 before): 56 workgroups instead of 14 at
// H = 896, so the ~1,000 partial rows of a backward are read by 4x as many CUs (19.4 us per launch
// at 14 workgroups, latency-bound)
constexpr int kColsumCols = 16, kColsumGroups = 1024 / kColsumCols;
__global__ __launch_bounds__(1024) void colsum_to_bf16_kernel(const float *__restrict__ part, int nblk,
                                                              int H, uint16_t *__restrict__ out) {
  __shared__ float s[kColsumGroups][kColsumCols + 1];
  const int cl = threadIdx.x % kColsumCols, g = threadIdx.x / kColsumCols;
  const int c = blockIdx.x * kColsumCols + cl;
  float acc = 0.f;
  if (c < H)
    for (int b = g; b < nblk; b += kColsumGroups) acc += part[static_cast<int64_t>(b) * H + c];
  s[g][cl] = acc;
  __syncthreads();
  if (g == 0 && c < H) {
    float t = 0.f;
#pragma unroll 8
    for (int k = 0; k < kColsumGroups; ++k) t += s[k][cl];
    out[c] = to_bf(t);
  }
}

// ------------------------------------------------------------------ column sums (bias gradients)
// part[b][c] = sum over rows [b R, (b + 1) R) of x[r][c] (bf16 [T, C], row stride ld, C % 8 == 0,
// C <= 2048), fp32. Each lane owns one 16-byte column vector; 256 / (C / 8) lanes per column vector
// take every rp-th row, 4 rows in flight per lane, and are merged in fixed order through LDS; then
// colsum_to_bf16_kernel adds the workgroups' partials in fixed order. The q|k|v bias gradient
// db = dY^T 1 over the packed tokens (torch's dy.sum(0) in the linear backward: ~4 TB/s there).
__global__ __launch_bounds__(256) void colsum_rows_kernel(const uint16_t *__restrict__ x, int64_t ld, int64_t T,
                                                          int C, int64_t R, float *__restrict__ part) {
  __shared__ float s[256 * 8];
  const int v8 = C >> 3, rp = 256 / v8;
  const int tid = threadIdx.x, vec = tid % v8, ro = tid / v8;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  const int64_t r1 = r0 + R < T ? r0 + R : T;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (ro < rp) {
    const uint16_t *p = x + vec * 8;
    int64_t r = r0 + ro;
    for (; r + 3 * rp < r1; r += 4 * rp) {  // every load of the group issued before the first use
      const uint4 a = ld16(p + r * ld), b = ld16(p + (r + rp) * ld), c = ld16(p + (r + 2 * rp) * ld),
                  d = ld16(p + (r + 3 * rp) * ld);
      float f[8];
      unpack8(a, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
      unpack8(b, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
      unpack8(c, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
      unpack8(d, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
    }
    for (; r < r1; r += rp) {
      float f[8];
      unpack8(ld16(p + r * ld), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s[ro * C + vec * 8 + e] = acc[e];
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float t = 0.f;
    for (int k = 0; k < rp; ++k) t += s[k * C + c];
    part[static_cast<int64_t>(blockIdx.x) * C + c] = t;
  }
}

// ------------------------------------------------------------------ SwiGLU
// gate / up are rows of a merged [T, ldgu] projection output (u at column offset `uoff`, so the
// plain two-tensor case is ldgu = F, uoff = u - g); y is [T, F].  Backward writes dg / du into the
// same merged layout (the gradient of the merged gate|up GEMM).
__device__ __forceinline__ float silu(float g) { return va_silu(g); }  // va_common.h

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const uint16_t *__restrict__ gu, int64_t ldgu,
                                                         int64_t uoff, int64_t T, int F,
                                                         uint16_t *__restrict__ y) {
  const int vpr = F >> 3;
  const int64_t total = T * vpr;
  for (int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; idx < total;
       idx += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t t = idx / vpr;
    const int c = static_cast<int>(idx - t * vpr) * 8;
    const uint16_t *gr = gu + t * ldgu + c;
    float g8[8], u8[8], o[8];
    unpack8(ld16(gr), g8);
    unpack8(ld16(gr + uoff), u8);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = rbf(silu(g8[e])) * u8[e];
    st16(y + t * F + c, pack8(o));
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const uint16_t *__restrict__ dy,
                                                         const uint16_t *__restrict__ gu, int64_t ldgu,
                                                         int64_t uoff, int64_t T, int F,
                                                         uint16_t *__restrict__ dgu, int64_t lddgu,
                                                         int64_t duoff) {
  const int vpr = F >> 3;
  const int64_t total = T * vpr;
  for (int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; idx < total;
       idx += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t t = idx / vpr;
    const int c = static_cast<int>(idx - t * vpr) * 8;
    const uint16_t *gr = gu + t * ldgu + c;
    float d8[8], g8[8], u8[8], rg[8], ru[8];
    unpack8(ld16(dy + t * F + c), d8);
    unpack8(ld16(gr), g8);
    unpack8(ld16(gr + uoff), u8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float s = va_sigmoid(g8[e]);
      ru[e] = d8[e] * rbf(g8[e] * s);
      rg[e] = d8[e] * u8[e] * (s * (1.f + g8[e] * (1.f - s)));
    }
    uint16_t *dr = dgu + t * lddgu + c;
    st16(dr, pack8(rg));
    st16(dr + duoff, pack8(ru));
  }
}

// Streaming variants (the default): no grid-stride loop; workgroup b owns the 256 x U consecutive
// 16-B vectors [b 256 U, (b + 1) 256 U) of the [T, F/8] vector grid, lane-interleaved per u, and
// issues every load of its U vectors before the first use (U x 2 or 3 16-B loads in flight per
// lane instead of one iteration's 2-3), with non-temporal loads / stores: the operands are
// streamed once and are far larger than the L2s / MALL. Per element the arithmetic is the
// grid-stride kernels' (bitwise identical outputs).
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16nt(const uint16_t *p) {
  return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4v *>(p)));
}
__device__ __forceinline__ void st16nt(uint16_t *p, uint4 v) {
  __builtin_nontemporal_store(__builtin_bit_cast(u32x4v, v), reinterpret_cast<u32x4v *>(p));
}

template <int U>
__global__ __launch_bounds__(256) void swiglu_fwd_stream_kernel(const uint16_t *__restrict__ gu, int64_t ldgu,
                                                                int64_t uoff, uint32_t total, uint32_t vpr,
                                                                int F, uint16_t *__restrict__ y) {
  const uint32_t i0 = blockIdx.x * (256u * U) + threadIdx.x;
  uint4 rg[U], ru[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t idx = min(i0 + u * 256u, total - 1);  // clamped: no branch around the loads
    const uint32_t t = idx / vpr, c = (idx - t * vpr) * 8;
    const uint16_t *gr = gu + static_cast<int64_t>(t) * ldgu + c;
    rg[u] = ld16nt(gr);
    ru[u] = ld16nt(gr + uoff);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t idx = i0 + u * 256u;
    if (idx >= total) continue;
    const uint32_t t = idx / vpr, c = (idx - t * vpr) * 8;
    float g8[8], u8[8], o[8];
    unpack8(rg[u], g8);
    unpack8(ru[u], u8);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = rbf(silu(g8[e])) * u8[e];
    st16nt(y + static_cast<int64_t>(t) * F + c, pack8(o));
  }
}

template <int U>
__global__ __launch_bounds__(256) void swiglu_bwd_stream_kernel(const uint16_t *__restrict__ dy,
                                                                const uint16_t *__restrict__ gu, int64_t ldgu,
                                                                int64_t uoff, uint32_t total, uint32_t vpr, int F,
                                                                uint16_t *__restrict__ dgu, int64_t lddgu,
                                                                int64_t duoff) {
  const uint32_t i0 = blockIdx.x * (256u * U) + threadIdx.x;
  uint4 rd[U], rg[U], ru[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t idx = min(i0 + u * 256u, total - 1);
    const uint32_t t = idx / vpr, c = (idx - t * vpr) * 8;
    const uint16_t *gr = gu + static_cast<int64_t>(t) * ldgu + c;
    rd[u] = ld16nt(dy + static_cast<int64_t>(t) * F + c);
    rg[u] = ld16nt(gr);
    ru[u] = ld16nt(gr + uoff);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t idx = i0 + u * 256u;
    if (idx >= total) continue;
    const uint32_t t = idx / vpr, c = (idx - t * vpr) * 8;
    float d8[8], g8[8], u8[8], og[8], ou[8];
    unpack8(rd[u], d8);
    unpack8(rg[u], g8);
    unpack8(ru[u], u8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float s = va_sigmoid(g8[e]);
      ou[e] = d8[e] * rbf(g8[e] * s);
      og[e] = d8[e] * u8[e] * (s * (1.f + g8[e] * (1.f - s)));
    }
    uint16_t *dr = dgu + static_cast<int64_t>(t) * lddgu + c;
    st16nt(dr, pack8(og));
    st16nt(dr + duoff, pack8(ou));
  }
}

// ------------------------------------------------------------------ RoPE on the merged q|k|v
// thread = (token t, head in [0, Hq + 2 Hk), chunk c of 8 elements in the first half of D)
__global__ __launch_bounds__(256) void rope_qkv_fwd_kernel(
    const uint16_t *__restrict__ qkv, int64_t ld, const uint16_t *__restrict__ cs,
    const uint16_t *__restrict__ sn, int64_t T, int Hq, int Hk, int D, uint16_t *__restrict__ q,
    uint16_t *__restrict__ k, uint16_t *__restrict__ v) {
  const int half = D >> 1, cph = half >> 3, nh = Hq + 2 * Hk;
  const int64_t per_t = static_cast<int64_t>(nh) * cph;
  const int64_t total = T * per_t;
  for (int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; idx < total;
       idx += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t t = idx / per_t;
    const int rem = static_cast<int>(idx - t * per_t);
    const int head = rem / cph, j = (rem - head * cph) * 8;
    const uint16_t *src = qkv + t * ld + static_cast<int64_t>(head) * D;
    const uint4 a = ld16(src + j), b = ld16(src + j + half);
    if (head >= Hq + Hk) {  // v: layout change only
      uint16_t *dst = v + (t * Hk + (head - Hq - Hk)) * D;
      st16(dst + j, a);
      st16(dst + j + half, b);
      continue;
    }
    uint16_t *dst = head < Hq ? q + (t * Hq + head) * D : k + (t * Hk + (head - Hq)) * D;
    float x1[8], x2[8], c1[8], c2[8], s1[8], s2[8], o1[8], o2[8];
    unpack8(a, x1);
    unpack8(b, x2);
    unpack8(ld16(cs + t * D + j), c1);
    unpack8(ld16(cs + t * D + j + half), c2);
    unpack8(ld16(sn + t * D + j), s1);
    unpack8(ld16(sn + t * D + j + half), s2);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // out[j] = x1*c1 + (-x2)*s1 ; out[j+half] = x2*c2 + x1*s2  (bf16 after each op)
      o1[e] = rbf(x1[e] * c1[e]) + rbf(-x2[e] * s1[e]);
      o2[e] = rbf(x2[e] * c2[e]) + rbf(x1[e] * s2[e]);
    }
    st16(dst + j, pack8(o1));
    st16(dst + j + half, pack8(o2));
  }
}

__global__ __launch_bounds__(256) void rope_qkv_bwd_kernel(
    const uint16_t *__restrict__ dq, const uint16_t *__restrict__ dk, const uint16_t *__restrict__ dv,
    const uint16_t *__restrict__ cs, const uint16_t *__restrict__ sn, int64_t T, int Hq, int Hk, int D,
    uint16_t *__restrict__ dqkv, int64_t ld) {
  const int half = D >> 1, cph = half >> 3, nh = Hq + 2 * Hk;
  const int64_t per_t = static_cast<int64_t>(nh) * cph;
  const int64_t total = T * per_t;
  for (int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; idx < total;
       idx += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t t = idx / per_t;
    const int rem = static_cast<int>(idx - t * per_t);
    const int head = rem / cph, j = (rem - head * cph) * 8;
    uint16_t *dst = dqkv + t * ld + static_cast<int64_t>(head) * D;
    if (head >= Hq + Hk) {
      const uint16_t *src = dv + (t * Hk + (head - Hq - Hk)) * D;
      st16(dst + j, ld16(src + j));
      st16(dst + j + half, ld16(src + j + half));
      continue;
    }
    const uint16_t *src = head < Hq ? dq + (t * Hq + head) * D : dk + (t * Hk + (head - Hq)) * D;
    float g1[8], g2[8], c1[8], c2[8], s1[8], s2[8], o1[8], o2[8];
    unpack8(ld16(src + j), g1);
    unpack8(ld16(src + j + half), g2);
    unpack8(ld16(cs + t * D + j), c1);
    unpack8(ld16(cs + t * D + j + half), c2);
    unpack8(ld16(sn + t * D + j), s1);
    unpack8(ld16(sn + t * D + j + half), s2);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // d x1 = g1*c1 + g2*s2 ; d x2 = g2*c2 - g1*s1
      o1[e] = g1[e] * c1[e] + g2[e] * s2[e];
      o2[e] = g2[e] * c2[e] - g1[e] * s1[e];
    }
    st16(dst + j, pack8(o1));
    st16(dst + j + half, pack8(o2));
  }
}

// out[c][r] = in[r][c] for 16-bit elements, 64 x 64 tiles through LDS: each of 256 lanes moves
// two 16-byte row chunks in and two 16-byte column chunks out, so both HBM sides are whole
// 128-byte lines. LDS rows are padded to 66 elements: a column read of 8 rows by a wave touches
// 32 distinct banks (lane pairs share a word). The backward GEMMs use it to give dX = dY W a
// K-contiguous W^T operand (kernels.input_grad).
constexpr int kTT = 64;
__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t *__restrict__ in, int64_t ldi, int64_t R,
                                                          int64_t C, uint16_t *__restrict__ out, int64_t ldo) {
  __shared__ uint32_t tile32[kTT * (kTT + 2) / 2];
  uint16_t *tile = reinterpret_cast<uint16_t *>(tile32);
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kTT, c0 = static_cast<int64_t>(blockIdx.x) * kTT;
  const int t = threadIdx.x;
  uint4 v[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {  // both loads in flight before the LDS writes
    const int64_t gr = r0 + p * 32 + (t >> 3), gc = c0 + (t & 7) * 8;
    v[p] = (gr < R && gc < C) ? *reinterpret_cast<const uint4 *>(in + gr * ldi + gc) : uint4{0, 0, 0, 0};
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    uint32_t *d = reinterpret_cast<uint32_t *>(tile + (p * 32 + (t >> 3)) * (kTT + 2) + (t & 7) * 8);
    d[0] = v[p].x, d[1] = v[p].y, d[2] = v[p].z, d[3] = v[p].w;
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = p * 32 + (t >> 3), rb = (t & 7) * 8;
    const int64_t gc = c0 + c, gr = r0 + rb;
    if (gc < C && gr < R) {
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = static_cast<uint32_t>(tile[(rb + 2 * k) * (kTT + 2) + c]) |
               (static_cast<uint32_t>(tile[(rb + 2 * k + 1) * (kTT + 2) + c]) << 16);
      *reinterpret_cast<uint4 *>(out + gc * ldo + gr) = uint4{w[0], w[1], w[2], w[3]};
    }
  }
}

int64_t grid_for(int64_t n, int per_thread) {
  int64_t g = (n + 256LL * per_thread - 1) / (256LL * per_thread);
  return g < 1 ? 1 : (g > 65536 ? 65536 : g);
}

bool aligned16(const void *p) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % 16 == 0; }

int nv_for(int64_t H) { return static_cast<int>((H / 8 + kWave - 1) / kWave); }

// rows per bwd workgroup: >= 16, and at most ~1024 workgroups (partials stay small)
int64_t bwd_rows_per_block(int64_t T) {
  int64_t r = (T + 1023) / 1024;
  if (r < 16) r = 16;
  return (r + 3) / 4 * 4;
}

}  // namespace
}  // namespace va

using namespace va;

// va_set_tuning(VA_TUNE_SWIGLU_STREAM): -1 auto = streaming kernels (4 / 2 vectors per lane fwd / bwd), 2 / 4 / 8 =
// streaming with that many vectors per lane, 0 = grid-stride kernels
int g_swiglu_variant = -1;

#define VA_NV_DISPATCH(nv, CALL)                   \
  switch (nv) {                                    \
    case 1: { constexpr int NV = 1; CALL; break; } \
    case 2: { constexpr int NV = 2; CALL; break; } \
    case 3:                                        \
    case 4: { constexpr int NV = 4; CALL; break; } \
    default: { constexpr int NV = 8; CALL; break; } \
  }

extern "C" int64_t va_rmsnorm_workspace_bytes(int64_t T, int64_t H) {
  const int64_t nblk = (T + bwd_rows_per_block(T) - 1) / bwd_rows_per_block(T);
  return static_cast<int64_t>(sizeof(float)) * (nblk > 0 ? nblk : 1) * H;
}

extern "C" int va_rmsnorm_fwd(const void *x, const void *residual, const void *w, int dtype, int64_t T,
                              int64_t H, float eps, void *h_out, void *y, float *rstd, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "rmsnorm: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && H > 0 && H % 8 == 0 && H <= 4096, "rmsnorm: need 0 < H <= 4096, H %% 8 == 0 (H=%lld)",
               static_cast<long long>(H));
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(x && w && y && rstd && (residual == nullptr || h_out != nullptr), "null pointer argument");
  if (!(aligned16(x) && aligned16(residual) && aligned16(w) && aligned16(h_out) && aligned16(y))) {
    set_error("rmsnorm: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const auto *xp = static_cast<const uint16_t *>(x);
  const auto *rp = static_cast<const uint16_t *>(residual);
  const auto *wp = static_cast<const uint16_t *>(w);
  VA_NV_DISPATCH(nv_for(H), hipLaunchKernelGGL(add_rmsnorm_fwd_kernel<NV>, dim3((T + 3) / 4), dim3(256), 0, s, xp,
                                               rp, wp, T, static_cast<int>(H), eps,
                                               static_cast<uint16_t *>(h_out), static_cast<uint16_t *>(y), rstd));
  return check_launch("rmsnorm_fwd");
}

extern "C" int va_rmsnorm_bwd(const void *dy, const void *h, const void *w, const float *rstd, const void *dres,
                              int dtype, int64_t T, int64_t H, void *dx, void *dw, float *workspace,
                              void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "rmsnorm: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && H > 0 && H % 8 == 0 && H <= 4096, "rmsnorm: need 0 < H <= 4096, H %% 8 == 0");
  VA_CHECK_ARG(dy && h && w && rstd && dx && dw && workspace, "null pointer argument");
  if (!(aligned16(dy) && aligned16(h) && aligned16(w) && aligned16(dres) && aligned16(dx))) {
    set_error("rmsnorm: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t rpb = bwd_rows_per_block(T);
  const int64_t nblk = (T + rpb - 1) / rpb;
  if (nblk > 0) {
    const size_t shm = static_cast<size_t>(4 * H) * sizeof(float);
    const auto *dyp = static_cast<const uint16_t *>(dy);
    const auto *hp = static_cast<const uint16_t *>(h);
    const auto *wp = static_cast<const uint16_t *>(w);
    const auto *dr = static_cast<const uint16_t *>(dres);
    auto *dxp = static_cast<uint16_t *>(dx);
    VA_NV_DISPATCH(nv_for(H), {
      if (shm > 64 * 1024 &&
          hipFuncSetAttribute(reinterpret_cast<const void *>(&add_rmsnorm_bwd_kernel<NV>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(shm)) != hipSuccess) {
        set_error("rmsnorm_bwd: cannot reserve %zu bytes of LDS", shm);
        return VA_E_LAUNCH;
      }
      hipLaunchKernelGGL(add_rmsnorm_bwd_kernel<NV>, dim3(nblk), dim3(256), shm, s, dyp, hp, wp, rstd, dr, T,
                         static_cast<int>(H), static_cast<int>(rpb), dxp, workspace);
    });
  }
  hipLaunchKernelGGL(colsum_to_bf16_kernel, dim3((H + kColsumCols - 1) / kColsumCols), dim3(1024), 0, s, workspace,
                     static_cast<int>(nblk), static_cast<int>(H), static_cast<uint16_t *>(dw));
  return check_launch("rmsnorm_bwd");
}

// column-sum workgroups: ~1,024 row slabs (>= 64 rows each), ceil-divided
static int64_t colsum_rows_per_wg(int64_t T) {
  int64_t r = (T + 1023) / 1024;
  return r < 64 ? 64 : r;
}

extern "C" int64_t va_column_sum_workspace_bytes(int64_t T, int64_t C) {
  if (T <= 0 || C <= 0) return 0;
  const int64_t R = colsum_rows_per_wg(T);
  return static_cast<int64_t>(sizeof(float)) * ((T + R - 1) / R) * C;
}

extern "C" int va_column_sum(const void *x, int64_t ld, int dtype, int64_t T, int64_t C, float *workspace,
                             int64_t workspace_bytes, void *out, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "column_sum: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && C > 0 && C % 8 == 0 && C <= 2048 && ld >= C && ld % 8 == 0,
               "column_sum: need C %% 8 == 0, C <= 2048 and an 8-element aligned row stride >= C");
  VA_CHECK_ARG(out != nullptr, "null pointer argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (T == 0) {  // no rows: the sums are zero
    if (hipMemsetAsync(out, 0, C * 2, s) != hipSuccess) return check_launch("column_sum");
    return VA_OK;
  }
  VA_CHECK_ARG(x && workspace, "null pointer argument");
  VA_CHECK_ARG(va_column_sum_workspace_bytes(T, C) <= workspace_bytes, "column_sum: workspace too small");
  if (!(aligned16(x) && aligned16(out))) {
    set_error("column_sum: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  const int64_t R = colsum_rows_per_wg(T), nblk = (T + R - 1) / R;
  hipLaunchKernelGGL(colsum_rows_kernel, dim3(static_cast<unsigned>(nblk)), dim3(256), 0, s,
                     static_cast<const uint16_t *>(x), ld, T, static_cast<int>(C), R, workspace);
  hipLaunchKernelGGL(colsum_to_bf16_kernel, dim3(static_cast<unsigned>((C + kColsumCols - 1) / kColsumCols)), dim3(1024), 0, s, workspace,
                     static_cast<int>(nblk), static_cast<int>(C), static_cast<uint16_t *>(out));
  return check_launch("column_sum");
}

extern "C" int va_swiglu_fwd(const void *gu, int64_t ldgu, int64_t uoff, int dtype, int64_t T, int64_t F, void *y,
                             void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "swiglu: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && F > 0 && F % 8 == 0 && ldgu % 8 == 0 && uoff % 8 == 0 && ldgu >= F,
               "swiglu: need F %% 8 == 0 and 8-element aligned strides");
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(gu && y, "null pointer argument");
  if (!(aligned16(gu) && aligned16(y))) {
    set_error("swiglu: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  const int64_t total = T * (F / 8);
  if (g_swiglu_variant != 0 && total < (1LL << 31)) {
    const int u = g_swiglu_variant > 0 ? g_swiglu_variant : 4;
#define VA_SWF(U)                                                                                                  \
  hipLaunchKernelGGL(swiglu_fwd_stream_kernel<U>, dim3(static_cast<unsigned>((total + 256 * U - 1) / (256 * U))), \
                     dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const uint16_t *>(gu), ldgu, uoff, \
                     static_cast<uint32_t>(total), static_cast<uint32_t>(F / 8), static_cast<int>(F),             \
                     static_cast<uint16_t *>(y))
    if (u == 2) VA_SWF(2); else if (u == 8) VA_SWF(8); else VA_SWF(4);
#undef VA_SWF
    return check_launch("swiglu_fwd");
  }
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(total, 1)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t *>(gu), ldgu, uoff, T,
                     static_cast<int>(F), static_cast<uint16_t *>(y));
  return check_launch("swiglu_fwd");
}

extern "C" int va_swiglu_bwd(const void *dy, const void *gu, int64_t ldgu, int64_t uoff, int dtype, int64_t T,
                             int64_t F, void *dgu, int64_t lddgu, int64_t duoff, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "swiglu: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && F > 0 && F % 8 == 0 && ldgu % 8 == 0 && uoff % 8 == 0 && lddgu % 8 == 0 &&
                   duoff % 8 == 0 && ldgu >= F && lddgu >= F,
               "swiglu: need F %% 8 == 0 and 8-element aligned strides");
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(dy && gu && dgu, "null pointer argument");
  if (!(aligned16(dy) && aligned16(gu) && aligned16(dgu))) {
    set_error("swiglu: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  const int64_t total = T * (F / 8);
  if (g_swiglu_variant != 0 && total < (1LL << 31)) {
    const int u = g_swiglu_variant > 0 ? g_swiglu_variant : 2;  // 2: best bwd (tools/elemwise_ab.py at 690aed1)
#define VA_SWB(U)                                                                                                  \
  hipLaunchKernelGGL(swiglu_bwd_stream_kernel<U>, dim3(static_cast<unsigned>((total + 256 * U - 1) / (256 * U))), \
                     dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const uint16_t *>(dy),             \
                     static_cast<const uint16_t *>(gu), ldgu, uoff, static_cast<uint32_t>(total),                   \
                     static_cast<uint32_t>(F / 8), static_cast<int>(F), static_cast<uint16_t *>(dgu), lddgu, duoff)
    if (u == 2) VA_SWB(2); else if (u == 8) VA_SWB(8); else VA_SWB(4);
#undef VA_SWB
    return check_launch("swiglu_bwd");
  }
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(total, 1)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t *>(dy),
                     static_cast<const uint16_t *>(gu), ldgu, uoff, T, static_cast<int>(F),
                     static_cast<uint16_t *>(dgu), lddgu, duoff);
  return check_launch("swiglu_bwd");
}

static int rope_checks(int dtype, int64_t T, int64_t Hq, int64_t Hk, int64_t D, int64_t ld) {
  VA_CHECK_ARG(dtype == VA_BF16, "rope: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && Hq > 0 && Hk > 0 && D > 0 && D % 16 == 0, "rope: need D %% 16 == 0 and Hq, Hk > 0");
  VA_CHECK_ARG(ld >= (Hq + 2 * Hk) * D && ld % 8 == 0, "rope: merged row stride %lld too small or unaligned",
               static_cast<long long>(ld));
  return VA_OK;
}

extern "C" int va_rope_qkv_fwd(const void *qkv, int64_t ld, const void *cos, const void *sin, int dtype,
                               int64_t T, int64_t Hq, int64_t Hk, int64_t D, void *q, void *k, void *v,
                               void *stream) {
  const int rc = rope_checks(dtype, T, Hq, Hk, D, ld);
  if (rc != VA_OK) return rc;
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(qkv && cos && sin && q && k && v, "null pointer argument");
  if (!(aligned16(qkv) && aligned16(cos) && aligned16(sin) && aligned16(q) && aligned16(k) && aligned16(v))) {
    set_error("rope: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  const int64_t total = T * (Hq + 2 * Hk) * (D / 16);
  hipLaunchKernelGGL(rope_qkv_fwd_kernel, dim3(grid_for(total, 1)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t *>(qkv), ld, static_cast<const uint16_t *>(cos),
                     static_cast<const uint16_t *>(sin), T, static_cast<int>(Hq), static_cast<int>(Hk),
                     static_cast<int>(D), static_cast<uint16_t *>(q), static_cast<uint16_t *>(k),
                     static_cast<uint16_t *>(v));
  return check_launch("rope_qkv_fwd");
}

extern "C" int va_rope_qkv_bwd(const void *dq, const void *dk, const void *dv, const void *cos, const void *sin,
                               int dtype, int64_t T, int64_t Hq, int64_t Hk, int64_t D, void *dqkv, int64_t ld,
                               void *stream) {
  const int rc = rope_checks(dtype, T, Hq, Hk, D, ld);
  if (rc != VA_OK) return rc;
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(dq && dk && dv && cos && sin && dqkv, "null pointer argument");
  if (!(aligned16(dq) && aligned16(dk) && aligned16(dv) && aligned16(cos) && aligned16(sin) && aligned16(dqkv))) {
    set_error("rope: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  const int64_t total = T * (Hq + 2 * Hk) * (D / 16);
  hipLaunchKernelGGL(rope_qkv_bwd_kernel, dim3(grid_for(total, 1)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t *>(dq), static_cast<const uint16_t *>(dk),
                     static_cast<const uint16_t *>(dv), static_cast<const uint16_t *>(cos),
                     static_cast<const uint16_t *>(sin), T, static_cast<int>(Hq), static_cast<int>(Hk),
                     static_cast<int>(D), static_cast<uint16_t *>(dqkv), ld);
  return check_launch("rope_qkv_bwd");
}

extern "C" int va_transpose_16(const void *in, int64_t ld_in, int64_t R, int64_t C, void *out, int64_t ld_out,
                               void *stream) {
  VA_CHECK_ARG(R >= 0 && C >= 0 && R % 8 == 0 && C % 8 == 0, "transpose_16: need R, C multiples of 8");
  VA_CHECK_ARG(ld_in >= C && ld_out >= R && ld_in % 8 == 0 && ld_out % 8 == 0,
               "transpose_16: strides must cover the rows and be multiples of 8");
  if (R == 0 || C == 0) return VA_OK;
  VA_CHECK_ARG(in && out, "null pointer argument");
  VA_CHECK_ARG((R + kTT - 1) / kTT <= 65535, "transpose_16: more than 4,194,240 rows");
  if (!(aligned16(in) && aligned16(out))) {
    set_error("transpose_16: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  hipLaunchKernelGGL(transpose16_kernel, dim3((C + kTT - 1) / kTT, (R + kTT - 1) / kTT), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t *>(in), ld_in, R, C,
                     static_cast<uint16_t *>(out), ld_out);
  return check_launch("transpose_16");
}
