// Weight-gradient GEMM probe, 256 x 256 tiles: dW[M, N] = dY[K, M]^T X[K, N] (K = tokens; both
// operands are K-outer: rows of dY / X are tokens). EXPERIMENTAL (tools/, not in the product library).
//
// The round-2 kernel (wgrad.hip: 128 x 128 tiles, 4 waves of 64 x 64, register staging) was LDS-bound
// at 0.61-0.72 PF/s. This one follows DESIGN.md §7's sketch:
//   workgroup = 256 (m) x 256 (n) output tile x one K slice, 8 waves as 2 (m) x 4 (n), wave tile
//   128 x 64 = 4 x 2 v_mfma_f32_32x32x16_bf16 accumulators (1.5 transposed fragment reads per MFMA);
//   per 64-token step both operands arrive by LDS-DMA (global_load_lds, 16 B per lane, 1 KiB per
//   wave-instruction = 2 token rows of the [k][256] image) into a 2-deep ring, one barrier per step;
//   the image's 16-B chunks are XOR-swizzled by (row & 3) << 2 through the per-lane SOURCE address
//   (the DMA writes lane-linearly), which makes the ds_read_b64_tr_b16 fragment reads conflict-free;
//   A = dY^T and B = X fragments come out in the same permuted k order (a dot product over k does
//   not see it).
// Split-K writes fp32 partial tiles; a second kernel sums them in slice order and rounds once.
// Columns past M / N are read clamped and their results dropped; K and every slice are multiples of 64.

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int IMG = BK * 256;  // bf16 elements of one operand's step image

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// element offset of (row, col) in a [64][256] image with 16-B chunks XOR-swizzled by (row & 3) << 2
__device__ __forceinline__ int ioff(int row, int col) {
  return row * 256 + ((((col >> 3) ^ ((row & 3) << 2))) << 3) + (col & 7);
}

// LDS-DMA of one operand's 64 x 256 step image: wave w issues pieces 4w .. 4w+3, piece g = rows
// 2g, 2g + 1; lane l lands at physical chunk l & 31 of row 2g + (l >> 5) and so fetches the logical
// chunk that the swizzle puts there
__device__ __forceinline__ void stage(const uint16_t *__restrict__ src, int64_t ld, int64_t k0, int col0, int ncols,
                                      uint16_t *img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int g = wave * 4 + i;
    const int row = 2 * g + (lane >> 5);
    const int c = (lane & 31) ^ ((row & 3) << 2);
    int col = col0 + c * 8;
    if (col > ncols - 8) col = ncols - 8;  // clamped: results for these columns are dropped
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + (k0 + row) * ld + col), img + g * 512, 16,
                                     0, 0);
  }
}

// 32 columns x 16 k fragment (MFMA A or B operand) by two transposed reads; element j of lane
// (column col_base + (lane & 31)) = image[16 ss + 8 (j >> 2) + 4 h + (j & 3)][column]
__device__ __forceinline__ bf16x8 frag(const uint16_t *img, int ss, int col_base, int lane) {
  const int h = lane >> 5, g16 = lane >> 4, li = lane & 15;
  const int r0 = 16 * ss + 4 * h + (li >> 2);
  const int col = col_base + 16 * (g16 & 1) + 4 * (li & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)(img + ioff(r0, col)));
  const v4s hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)(img + ioff(r0 + 8, col)));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ uint16_t f2bf(float f) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return static_cast<uint16_t>(__builtin_bit_cast(uint32_t, __builtin_convertvector(f2{f, 0.f}, b2)) & 0xffffu);
}

template <bool PARTIAL>
__global__ __launch_bounds__(NT, 1) void wgrad256_kernel(const uint16_t *__restrict__ dy, int64_t ldy,
                                                         const uint16_t *__restrict__ x, int64_t ldx, int64_t K,
                                                         int M, int N, int splits, int64_t kslice,
                                                         float *__restrict__ part, uint16_t *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * IMG];  // [buf][A | B][64][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM;
  // XCD-aware bijective remap: hardware ids w, w + 8, ... share an XCD; give them consecutive
  // logical tiles, n-tile fastest, so the n-tiles of one dY tile and K slice share an L2
  const int nwg = nbn * nbm * splits;
  const int w = blockIdx.x, xcd = w & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (w >> 3);
  const int bn = logical % nbn;
  const int rest = logical / nbn;
  const int bm = rest % nbm, s = rest / nbm;
  const int m0 = bm * BM, n0 = bn * BN;
  const int64_t k_beg = static_cast<int64_t>(s) * kslice;
  const int64_t k_end = k_beg + kslice < K ? k_beg + kslice : K;
  const int nsteps = k_end > k_beg ? static_cast<int>((k_end - k_beg) / BK) : 0;

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nsteps > 0) {
    stage(dy, ldy, k_beg, m0, M, lds, wave, lane);
    stage(x, ldx, k_beg, n0, N, lds + IMG, wave, lane);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    const uint16_t *ia = lds + buf * 2 * IMG;
    const uint16_t *ib = ia + IMG;
    if (st + 1 < nsteps) {
      uint16_t *na = lds + (buf ^ 1) * 2 * IMG;
      const int64_t k1 = k_beg + static_cast<int64_t>(st + 1) * BK;
      stage(dy, ldy, k1, m0, M, na, wave, lane);
      stage(x, ldx, k1, n0, N, na + IMG, wave, lane);
    }
#pragma unroll
    for (int ss = 0; ss < 4; ++ss) {
      bf16x8 fa[4], fb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag(ia, ss, wm * 128 + i * 32, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = frag(ib, ss, wn * 64 + j * 32, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // lane holds C[m = m0 + wm 128 + i 32 + crow(r, h)][n = n0 + wn 64 + j 32 + (lane & 31)]
  const int h = lane >> 5, nl = lane & 31;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + nl;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + i * 32 + crow(r, h);
        if (m >= M) continue;
        if constexpr (PARTIAL) part[(static_cast<int64_t>(s) * M + m) * N + n] = acc[i][j][r];
        else out[static_cast<int64_t>(m) * N + n] = f2bf(acc[i][j][r]);
      }
    }
}

// out[e] = bf16(sum_s part[s][e]) in slice order; 4 elements per thread (M N % 4 == 0)
__global__ __launch_bounds__(256) void reduce_kernel(const float *__restrict__ part, int splits, int64_t mn,
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
  const uint32_t lo = static_cast<uint32_t>(f2bf(acc.x)) | (static_cast<uint32_t>(f2bf(acc.y)) << 16);
  const uint32_t hi = static_cast<uint32_t>(f2bf(acc.z)) | (static_cast<uint32_t>(f2bf(acc.w)) << 16);
  *reinterpret_cast<uint2 *>(out + e) = make_uint2(lo, hi);
}

}  // namespace

extern "C" int64_t wg256_workspace_bytes(int64_t M, int64_t N, int splits) {
  return splits > 1 ? static_cast<int64_t>(sizeof(float)) * splits * M * N : 0;
}

// returns 0, or -1 on bad arguments (checked before any launch)
extern "C" int wg256_bf16(const void *dy, int64_t ldy, const void *x, int64_t ldx, int64_t K, int64_t M, int64_t N,
                          int splits, float *workspace, void *out, void *stream) {
  if (K < 0 || K % BK || M < 8 || N < 8 || M % 8 || N % 8 || ldy % 8 || ldx % 8 || ldy < M || ldx < N) return -1;
  if (splits < 1 || splits > 256 || (splits > 1 && !workspace) || !dy || !x || !out) return -1;
  if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) % 16)
    return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t mn = M * N;
  const int64_t steps = K / BK;
  const int64_t kslice = (steps + splits - 1) / splits * BK;
  const int nwg = static_cast<int>(((M + BM - 1) / BM) * ((N + BN - 1) / BN) * splits);
  if (splits == 1) {
    hipLaunchKernelGGL(wgrad256_kernel<false>, dim3(nwg), dim3(NT), 0, st, static_cast<const uint16_t *>(dy), ldy,
                       static_cast<const uint16_t *>(x), ldx, K, static_cast<int>(M), static_cast<int>(N), 1, kslice,
                       nullptr, static_cast<uint16_t *>(out));
  } else {
    hipLaunchKernelGGL(wgrad256_kernel<true>, dim3(nwg), dim3(NT), 0, st, static_cast<const uint16_t *>(dy), ldy,
                       static_cast<const uint16_t *>(x), ldx, K, static_cast<int>(M), static_cast<int>(N), splits,
                       kslice, workspace, nullptr);
    hipLaunchKernelGGL(reduce_kernel, dim3(static_cast<unsigned>((mn / 4 + 255) / 256)), dim3(256), 0, st, workspace,
                       splits, mn, static_cast<uint16_t *>(out));
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
