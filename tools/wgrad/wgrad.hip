// Weight-gradient GEMM of the actor's linear layers on MI355X: dW[M, N] = dY[T, M]^T X[T, N]
// (M = out_features, N = in_features, K = T tokens; bf16 in, fp32 accumulate, bf16 out).
// EXPERIMENTAL, moved out of the product library (round 3): not built by verl_amd/build.py, not in
// the C-ABI; the actor's weight gradients run in hipBLASLt. Kept as the starting point DESIGN.md §7
// names (a 256-row tile with 128 x 64 wave tiles and LDS-DMA staging). Not a §8 row: written to replace the hipBLASLt calls of torch's linear backward for
// this shape class (huge K, small output), which run at 0.43-0.89 PF/s there
// (profiles/r01/wgrad_layout_T151552.log); at 0.61-0.72 PF/s it does not yet.
//
// Both operands are k-strided in memory (rows of dY / X are tokens), so the workgroup stages each
// 64-token step as [k][m] / [k][n] LDS images (XOR-swizzled 16-B chunks, the attention kernels'
// layout) and reads the MFMA fragments with ds_read_b64_tr_b16 (transposed reads): A = dY^T and
// B = X come out with the same permuted k order, which a dot product over k does not see.
//
// Workgroup = 128 (m) x 128 (n) output tile x one K slice, 4 waves as 2 x 2, wave tile 64 x 64 =
// 2 x 2 v_mfma_f32_32x32x16_bf16 accumulators. One barrier per 64-token step: the next step's
// 2 x 4 16-B loads per lane are in registers during the current step's MFMAs and written to the
// other LDS buffer afterwards. K slices (split-K) write fp32 partial tiles; a second kernel sums
// them in slice order (deterministic) and rounds once to bf16. Workgroup ids are remapped so the
// n-tiles that share one dY tile are dispatched to the same XCD (shared L2).

#include "va_common.h"

namespace va {
namespace {

constexpr int WBM = 128, WBN = 128, WBK = 64;

typedef short bf16x8w __attribute__((ext_vector_type(8)));
typedef short v4sw __attribute__((ext_vector_type(4)));
typedef float f32x16w __attribute__((ext_vector_type(16)));

// [64 rows][64 cols] bf16 image, 16-B chunk c of row r stored at chunk c ^ (r & 7)
__device__ __forceinline__ int wswz(int row, int col) {
  return row * 64 + ((((col >> 3) ^ (row & 7))) << 3) + (col & 7);
}

// MFMA operand fragment (32 rows of the image's columns x 16 k) by transposed reads:
// element j of lane (col = dh * 32 + lane & 31, half h) = image[16 s + 8 (j >> 2) + 4 h + (j & 3)][col]
__device__ __forceinline__ bf16x8w wtr_frag(const uint16_t *img, int s, int dh, int lane) {
  const int h = lane >> 5, g16 = lane >> 4, li = lane & 15;
  const int r0 = 16 * s + 4 * h + (li >> 2);
  const int col = dh * 32 + 16 * (g16 & 1) + 4 * (li & 3);
  const v4sw lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4sw *)(img + wswz(r0, col)));
  const v4sw hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4sw *)(img + wswz(r0 + 8, col)));
  return bf16x8w{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ int wcrow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ uint16_t f2bf(float f) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return static_cast<uint16_t>(__builtin_bit_cast(uint32_t, __builtin_convertvector(f2{f, 0.f}, b2)) & 0xffffu);
}

// OUT_BF16: one K slice, bf16 result; else fp32 partial tile of slice blockIdx-derived s
template <bool OUT_BF16>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(const uint16_t *__restrict__ dy, int64_t ldy,
                                                       const uint16_t *__restrict__ x, int64_t ldx, int64_t T,
                                                       int M, int N, int splits, int64_t kslice,
                                                       float *__restrict__ part, uint16_t *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 4 * 64 * 64];  // [buf][A0 A1 B0 B1][64][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nbn = N / WBN, nbm = M / WBM;
  // XCD-aware bijective remap: ids w, w + 8, ... share an XCD; give them consecutive logical tiles
  const int nwg = nbn * nbm * splits;
  const int w = blockIdx.x, xcd = w & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (w >> 3);
  const int bn = logical % nbn;
  const int rest = logical / nbn;
  const int bm = rest % nbm, s = rest / nbm;
  const int m0 = bm * WBM, n0 = bn * WBN;
  const int64_t k_beg = static_cast<int64_t>(s) * kslice;
  const int64_t k_end = min(T, k_beg + kslice);
  const int nkb = static_cast<int>((k_end - k_beg + WBK - 1) / WBK);

  f32x16w acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // staging: per operand 64 rows x 16 chunks of 16 B = 1024 chunks, 4 per thread
  uint4 ra[4], rb[4];
  auto load_step = [&](int kb) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = tid + u * 256, r = idx >> 4, ch = idx & 15;
      const int64_t k = k_beg + static_cast<int64_t>(kb) * WBK + r;
      const bool ok = k < k_end;
      const int64_t kc = ok ? k : k_end - 1;  // clamped: no branch around the loads
      const uint4 a = *reinterpret_cast<const uint4 *>(dy + kc * ldy + m0 + ch * 8);
      const uint4 b = *reinterpret_cast<const uint4 *>(x + kc * ldx + n0 + ch * 8);
      ra[u] = ok ? a : make_uint4(0, 0, 0, 0);
      rb[u] = ok ? b : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_step = [&](int buf) {
    uint16_t *base = lds + buf * 4 * 64 * 64;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = tid + u * 256, r = idx >> 4, ch = idx & 15;
      const int half = ch >> 3, col = (ch & 7) * 8;
      *reinterpret_cast<uint4 *>(base + half * 64 * 64 + wswz(r, col)) = ra[u];
      *reinterpret_cast<uint4 *>(base + (2 + half) * 64 * 64 + wswz(r, col)) = rb[u];
    }
  };

  if (nkb > 0) {
    load_step(0);
    store_step(0);
  }
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) load_step(kb + 1);
    const uint16_t *base = lds + (kb & 1) * 4 * 64 * 64;
    const uint16_t *ia = base + wm * 64 * 64;
    const uint16_t *ib = base + (2 + wn) * 64 * 64;
#pragma unroll
    for (int ss = 0; ss < 4; ++ss) {
      const bf16x8w a0 = wtr_frag(ia, ss, 0, lane), a1 = wtr_frag(ia, ss, 1, lane);
      const bf16x8w b0 = wtr_frag(ib, ss, 0, lane), b1 = wtr_frag(ib, ss, 1, lane);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kb + 1 < nkb) store_step((kb + 1) & 1);
    __syncthreads();
  }

  // epilogue: lane holds C[m = m0 + wm 64 + i 32 + crow(r, h)][n = n0 + wn 64 + j 32 + (lane & 31)]
  const int h = lane >> 5, nl = lane & 31;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm * 64 + i * 32 + wcrow(r, h);
        const int64_t n = n0 + wn * 64 + j * 32 + nl;
        if constexpr (OUT_BF16) out[m * N + n] = f2bf(acc[i][j][r]);
        else part[(static_cast<int64_t>(s) * M + m) * N + n] = acc[i][j][r];
      }
}

// out[e] = bf16(sum_s part[s][e]) in slice order; 4 elements per thread
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float *__restrict__ part, int splits, int64_t mn,
                                                           uint16_t *__restrict__ out) {
  const int64_t e = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (e >= mn) return;  // mn % 4 == 0 (M, N multiples of 128)
  float4 acc = *reinterpret_cast<const float4 *>(part + e);
  for (int s = 1; s < splits; ++s) {
    const float4 v = *reinterpret_cast<const float4 *>(part + static_cast<int64_t>(s) * mn + e);
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  const uint32_t lo = static_cast<uint32_t>(f2bf(acc.x)) | (static_cast<uint32_t>(f2bf(acc.y)) << 16);
  const uint32_t hi = static_cast<uint32_t>(f2bf(acc.z)) | (static_cast<uint32_t>(f2bf(acc.w)) << 16);
  *reinterpret_cast<uint2 *>(out + e) = make_uint2(lo, hi);
}

}  // namespace
}  // namespace va

using namespace va;

extern "C" int64_t va_wgrad_workspace_bytes(int64_t M, int64_t N, int splits) {
  return splits > 1 ? static_cast<int64_t>(sizeof(float)) * splits * M * N : 0;
}

extern "C" int va_wgrad_bf16(const void *dy, int64_t ldy, const void *x, int64_t ldx, int64_t T, int64_t M,
                             int64_t N, int splits, float *workspace, void *out, void *stream) {
  VA_CHECK_ARG(T >= 0 && M > 0 && N > 0 && M % WBM == 0 && N % WBN == 0,
               "wgrad: need M, N multiples of 128 (M=%lld N=%lld)", static_cast<long long>(M),
               static_cast<long long>(N));
  VA_CHECK_ARG(ldy >= M && ldx >= N && ldy % 8 == 0 && ldx % 8 == 0, "wgrad: bad leading dimensions");
  VA_CHECK_ARG(splits >= 1 && splits <= 256, "wgrad: splits must be in [1, 256]");
  VA_CHECK_ARG(dy && x && out && (splits == 1 || workspace), "null pointer argument");
  if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) % 16) {
    set_error("wgrad: 16-byte aligned buffers required");
    return VA_E_ALIGN;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t mn = M * N;
  if (T == 0) return hipMemsetAsync(out, 0, mn * 2, st) == hipSuccess ? VA_OK : VA_E_LAUNCH;
  const int64_t kslice = ((T + splits - 1) / splits + WBK - 1) / WBK * WBK;
  const int nwg = static_cast<int>((M / WBM) * (N / WBN) * splits);
  if (splits == 1) {
    hipLaunchKernelGGL(wgrad_kernel<true>, dim3(nwg), dim3(256), 0, st, static_cast<const uint16_t *>(dy), ldy,
                       static_cast<const uint16_t *>(x), ldx, T, static_cast<int>(M), static_cast<int>(N), 1, kslice,
                       nullptr, static_cast<uint16_t *>(out));
    return check_launch("wgrad");
  }
  hipLaunchKernelGGL(wgrad_kernel<false>, dim3(nwg), dim3(256), 0, st, static_cast<const uint16_t *>(dy), ldy,
                     static_cast<const uint16_t *>(x), ldx, T, static_cast<int>(M), static_cast<int>(N), splits,
                     kslice, workspace, nullptr);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(static_cast<unsigned>((mn / 4 + 255) / 256)), dim3(256), 0, st,
                     workspace, splits, mn, static_cast<uint16_t *>(out));
  return check_launch("wgrad");
}
