// Weight gradients of the packed backbone's linear layers: dW[M, N] = dY[K, M]^T X[K, N] in bf16
// with fp32 accumulation (K = packed tokens, M = out_features, N = in_features). Not a §8 row: it
// replaces the hipBLASLt GEMMs of torch's linear backward for this shape class (K in the 10^5 range,
// an output of a few hundred 256 x 256 tiles; both operands K-outer), which run at 0.69-0.89 PF/s on
// the bench's shapes (tools/wgrad256_bench.py, profiles/r03/wgrad256_probe.jsonl).
//
// Workgroup = 256 (m) x 256 (n) output tile x one K slice (split-K), 8 waves as 2 (m) x 4 (n), wave
// tile 128 x 64 = 4 x 2 v_mfma_f32_32x32x16_bf16 accumulators (1.5 transposed fragment reads per
// MFMA keep the LDS under half its rate).
// Staging: 32-token steps in a 4-deep LDS ring (4 x 32 KiB); both operands arrive by LDS-DMA
// (global_load_lds, 16 B per lane, 1 KiB per wave-instruction = 2 token rows of a [k][256] image),
// with the image's 16-B chunks XOR-swizzled by (row & 3) << 2 through the per-lane SOURCE address,
// which makes the ds_read_b64_tr_b16 fragment reads conflict-free. At the top of step st a counted
// vmcnt retires this wave's pieces of step st while steps st + 1, st + 2 stay in flight, one raw
// s_barrier publishes every wave's pieces and ends every wave's reads of step st - 1, whose buffer
// the DMA for step st + 3 then refills.
// The transposed reads are inline asm: for the builtin the compiler drains every LDS-DMA in flight
// (vmcnt(0)) before the first read of each step, which would cap the ring at one step of prefetch
// (0.70-0.72 PF/s measured vs 0.93-0.98); the asm results pass through explicit counted lgkmcnt
// waits, so no MFMA is scheduled above the wait that retires its fragments.
// A = dY^T and B = X fragments come out in the same permuted k order (a dot product over k does not
// see it). Split-K slices write fp32 partial tiles, summed in slice order and rounded once to bf16
// by a second kernel (deterministic). Columns past M / N are read clamped and their results dropped.

#include "va_common.h"

namespace va {
namespace {

constexpr int WBM = 256, WBN = 256, WBK = 32, WNT = 512, WNSTAGE = 4;
constexpr int WIMG = WBK * 256;  // bf16 elements of one operand's step image

typedef short wbf16x8 __attribute__((ext_vector_type(8)));
typedef int wv2i __attribute__((ext_vector_type(2)));
typedef float wf32x16 __attribute__((ext_vector_type(16)));

// element offset of (row, col) in a [32][256] image with 16-B chunks XOR-swizzled by (row & 3) << 2
__device__ __forceinline__ int w_off(int row, int col) {
  return row * 256 + (((col >> 3) ^ ((row & 3) << 2)) << 3) + (col & 7);
}

// LDS-DMA of one operand's 32 x 256 step image: wave w issues pieces 2w, 2w + 1, piece g = rows 2g,
// 2g + 1; lane l lands at physical chunk l & 31 of row 2g + (l >> 5) and so fetches the logical
// chunk the swizzle puts there
__device__ __forceinline__ void w_stage(const uint16_t *__restrict__ src, int64_t ld, int64_t k0, int col0, int ncols,
                                        uint16_t *img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = wave * 2 + i;
    const int row = 2 * g + (lane >> 5);
    const int c = (lane & 31) ^ ((row & 3) << 2);
    int col = col0 + c * 8;
    if (col > ncols - 8) col = ncols - 8;  // clamped: results for these columns are dropped
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + (k0 + row) * ld + col), img + g * 512, 16,
                                     0, 0);
  }
}

__device__ __forceinline__ wv2i w_tr_read(const uint16_t *p) {
  wv2i r;
  const uint32_t a =
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint16_t *)p));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

// 32 columns x 16 k fragment (MFMA A or B operand) by two transposed reads; element j of lane
// (column col_base + (lane & 31)) = image[16 ss + 8 (j >> 2) + 4 h + (j & 3)][column]
__device__ __forceinline__ void w_frag(const uint16_t *img, int ss, int col_base, int lane, wv2i &lo, wv2i &hi) {
  const int h = lane >> 5, g16 = lane >> 4, li = lane & 15;
  const int r0 = 16 * ss + 4 * h + (li >> 2);
  const int col = col_base + 16 * (g16 & 1) + 4 * (li & 3);
  lo = w_tr_read(img + w_off(r0, col));
  hi = w_tr_read(img + w_off(r0 + 8, col));
}

__device__ __forceinline__ wbf16x8 w_join(wv2i lo, wv2i hi) {
  return __builtin_bit_cast(wbf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3));
}

__device__ __forceinline__ int w_crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <bool PARTIAL>
__global__ __launch_bounds__(WNT, 1) void wgrad_kernel(const uint16_t *__restrict__ dy, int64_t ldy,
                                                       const uint16_t *__restrict__ x, int64_t ldx, int64_t K, int M,
                                                       int N, int splits, int64_t kslice, float *__restrict__ part,
                                                       uint16_t *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[WNSTAGE * 2 * WIMG];  // [stage][A | B][32][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nbn = (N + WBN - 1) / WBN, nbm = (M + WBM - 1) / WBM;
  // XCD-aware bijective remap: hardware ids w, w + 8, ... share an XCD; give them consecutive
  // logical tiles, n-tile fastest, so the n-tiles of one dY tile and K slice share an L2
  const int nwg = nbn * nbm * splits;
  const int w = blockIdx.x, xcd = w & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (w >> 3);
  const int bn = logical % nbn;
  const int rest = logical / nbn;
  const int bm = rest % nbm, s = rest / nbm;
  const int m0 = bm * WBM, n0 = bn * WBN;
  const int64_t k_beg = static_cast<int64_t>(s) * kslice;
  const int64_t k_end = k_beg + kslice < K ? k_beg + kslice : K;
  const int nsteps = k_end > k_beg ? static_cast<int>((k_end - k_beg) / WBK) : 0;

  wf32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int st) {  // 4 LDS-DMA instructions per wave
    uint16_t *img = lds + (st % WNSTAGE) * 2 * WIMG;
    const int64_t k0 = k_beg + static_cast<int64_t>(st) * WBK;
    w_stage(dy, ldy, k0, m0, M, img, wave, lane);
    w_stage(x, ldx, k0, n0, N, img + WIMG, wave, lane);
  };
  for (int b = 0; b < WNSTAGE - 1; ++b)
    if (b < nsteps) issue(b);
  for (int st = 0; st < nsteps; ++st) {
    const int ahead = nsteps - 1 - st;  // steps issued after st (at most 2 here)
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (st + WNSTAGE - 1 < nsteps) issue(st + WNSTAGE - 1);
    const uint16_t *ia = lds + (st % WNSTAGE) * 2 * WIMG;
    const uint16_t *ib = ia + WIMG;
#pragma unroll
    for (int ss = 0; ss < WBK / 16; ++ss) {
      // issue order A0 B0 B1 A1 A2 A3 (2 reads each); each counted wait releases the fragments it
      // passes through while the later reads stay in flight
      wv2i a0, a1, a2, a3, a4, a5, a6, a7, b0, b1, b2, b3;
      w_frag(ia, ss, wm * 128 + 0, lane, a0, a1);
      w_frag(ib, ss, wn * 64 + 0, lane, b0, b1);
      w_frag(ib, ss, wn * 64 + 32, lane, b2, b3);
      w_frag(ia, ss, wm * 128 + 32, lane, a2, a3);
      w_frag(ia, ss, wm * 128 + 64, lane, a4, a5);
      w_frag(ia, ss, wm * 128 + 96, lane, a6, a7);
      asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1));
      const wbf16x8 fb0 = w_join(b0, b1);
      wbf16x8 fa = w_join(a0, a1);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc[0][0], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(b2), "+v"(b3));
      const wbf16x8 fb1 = w_join(b2, b3);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc[0][1], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(a2), "+v"(a3));
      fa = w_join(a2, a3);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc[1][1], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a4), "+v"(a5));
      fa = w_join(a4, a5);
      acc[2][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc[2][0], 0, 0, 0);
      acc[2][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc[2][1], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a6), "+v"(a7));
      fa = w_join(a6, a7);
      acc[3][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc[3][0], 0, 0, 0);
      acc[3][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc[3][1], 0, 0, 0);
    }
  }

  // lane holds C[m = m0 + wm 128 + i 32 + w_crow(r, h)][n = n0 + wn 64 + j 32 + (lane & 31)]
  const int h = lane >> 5, nl = lane & 31;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + nl;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + i * 32 + w_crow(r, h);
        if (m >= M) continue;
        if constexpr (PARTIAL) part[(static_cast<int64_t>(s) * M + m) * N + n] = acc[i][j][r];
        else out[static_cast<int64_t>(m) * N + n] = static_cast<uint16_t>(pack2_bf16(acc[i][j][r], 0.f) & 0xffffu);
      }
    }
}

// out[e] = bf16(sum_s part[s][e]) in slice order; 4 elements per thread (M N % 4 == 0)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float *__restrict__ part, int splits, int64_t mn,
                                                           uint16_t *__restrict__ out) {
  const int64_t e = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (e >= mn) return;
  float4 acc = *reinterpret_cast<const float4 *>(part + e);
  for (int s = 1; s < splits; ++s) {
    const float4 v = *reinterpret_cast<const float4 *>(part + static_cast<int64_t>(s) * mn + e);
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  *reinterpret_cast<uint2 *>(out + e) = make_uint2(pack2_bf16(acc.x, acc.y), pack2_bf16(acc.z, acc.w));
}

}  // namespace
}  // namespace va

using namespace va;

extern "C" int64_t va_weight_grad_workspace_bytes(int64_t M, int64_t N, int splits) {
  return splits > 1 ? static_cast<int64_t>(sizeof(float)) * splits * M * N : 0;
}

extern "C" int va_weight_grad(const void *dy, int64_t ldy, const void *x, int64_t ldx, int64_t K, int64_t M, int64_t N,
                              int splits, float *workspace, void *out, void *stream) {
  VA_CHECK_ARG(K >= 0 && K % WBK == 0, "weight_grad: K (tokens) must be a multiple of 32 (K=%lld)",
               static_cast<long long>(K));
  VA_CHECK_ARG(M >= 8 && N >= 8 && M % 8 == 0 && N % 8 == 0 && M < (1 << 30) && N < (1 << 30),
               "weight_grad: M, N must be multiples of 8 (M=%lld N=%lld)", static_cast<long long>(M),
               static_cast<long long>(N));
  VA_CHECK_ARG(ldy >= M && ldx >= N && ldy % 8 == 0 && ldx % 8 == 0, "weight_grad: bad leading dimensions");
  VA_CHECK_ARG(splits >= 1 && splits <= 256, "weight_grad: splits must be in [1, 256]");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t mn = M * N;
  VA_CHECK_ARG(out != nullptr, "null pointer argument");
  if (K == 0) {  // no tokens: dW = 0 (the operands may be empty views without storage)
    if (hipMemsetAsync(out, 0, mn * 2, st) != hipSuccess) return check_launch("weight_grad");
    return VA_OK;
  }
  VA_CHECK_ARG(dy && x && (splits == 1 || workspace), "null pointer argument");
  VA_CHECK_ARG(((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) &
                15) == 0,
               "weight_grad: 16-byte aligned buffers required");
  const int64_t steps = K / WBK;
  const int64_t kslice = (steps + splits - 1) / splits * WBK;
  const int64_t nwg = ((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN) * splits;
  VA_CHECK_ARG(nwg < (int64_t{1} << 31), "weight_grad: grid too large");
  const auto *dy16 = static_cast<const uint16_t *>(dy);
  const auto *x16 = static_cast<const uint16_t *>(x);
  if (splits == 1) {
    hipLaunchKernelGGL(wgrad_kernel<false>, dim3(static_cast<unsigned>(nwg)), dim3(WNT), 0, st, dy16, ldy, x16, ldx, K,
                       static_cast<int>(M), static_cast<int>(N), 1, kslice, nullptr, static_cast<uint16_t *>(out));
  } else {
    hipLaunchKernelGGL(wgrad_kernel<true>, dim3(static_cast<unsigned>(nwg)), dim3(WNT), 0, st, dy16, ldy, x16, ldx, K,
                       static_cast<int>(M), static_cast<int>(N), splits, kslice, workspace, nullptr);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(static_cast<unsigned>((mn / 4 + 255) / 256)), dim3(256), 0, st,
                       workspace, splits, mn, static_cast<uint16_t *>(out));
  }
  return check_launch("weight_grad");
}
