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

// LDS-DMA of one operand's ROWS x 256 step image: wave w issues pieces ROWS/16 w .. , piece g = rows
// 2g, 2g + 1; lane l lands at physical chunk l & 31 of row 2g + (l >> 5) and so fetches the logical
// chunk that the swizzle puts there
template <int ROWS = BK>
__device__ __forceinline__ void stage(const uint16_t *__restrict__ src, int64_t ld, int64_t k0, int col0, int ncols,
                                      uint16_t *img, int wave, int lane) {
  constexpr int PW = ROWS / 16;  // pieces per wave (8 waves x PW x 2 rows = ROWS)
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int g = wave * PW + i;
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

// The same transposed read as inline asm: the compiler does not see an LDS access, so it does not
// drain the in-flight LDS-DMA (vmcnt(0)) before it (it does for the builtin, which carries no alias
// information); the results are only valid after an explicit lgkmcnt wait (tr_wait below)
typedef int v2i __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2i tr_read_asm(const uint16_t *p) {
  v2i r;
  const uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint16_t *)p));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
__device__ __forceinline__ void frag_asm(const uint16_t *img, int ss, int col_base, int lane, v2i &lo, v2i &hi) {
  const int h = lane >> 5, g16 = lane >> 4, li = lane & 15;
  const int r0 = 16 * ss + 4 * h + (li >> 2);
  const int col = col_base + 16 * (g16 & 1) + 4 * (li & 3);
  lo = tr_read_asm(img + ioff(r0, col));
  hi = tr_read_asm(img + ioff(r0 + 8, col));
}
__device__ __forceinline__ bf16x8 join(v2i lo, v2i hi) {
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3));
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

// Ring variant: 32-token steps in a 4-deep LDS ring (4 x 32 KiB), 3 steps of DMA in flight across each
// barrier: at the top of step st a counted vmcnt retires this wave's pieces of step st (the pieces of
// st + 1, st + 2 stay in flight), one raw s_barrier publishes every wave's pieces and also ends
// every wave's reads of step st - 1, whose buffer the DMA for step st + 3 then refills.
constexpr int RBK = 32, NSTAGE = 4, RIMG = RBK * 256;

template <bool PARTIAL>
__global__ __launch_bounds__(NT, 1) void wgrad256_ring_kernel(const uint16_t *__restrict__ dy, int64_t ldy,
                                                              const uint16_t *__restrict__ x, int64_t ldx, int64_t K,
                                                              int M, int N, int splits, int64_t kslice,
                                                              float *__restrict__ part, uint16_t *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[NSTAGE * 2 * RIMG];  // [stage][A | B][32][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM;
  const int nwg = nbn * nbm * splits;
  const int w = blockIdx.x, xcd = w & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (w >> 3);
  const int bn = logical % nbn;
  const int rest = logical / nbn;
  const int bm = rest % nbm, s = rest / nbm;
  const int m0 = bm * BM, n0 = bn * BN;
  const int64_t k_beg = static_cast<int64_t>(s) * kslice;
  const int64_t k_end = k_beg + kslice < K ? k_beg + kslice : K;
  const int nsteps = k_end > k_beg ? static_cast<int>((k_end - k_beg) / RBK) : 0;

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // buffer b of the ring is at the compile-time offset b * 2 * RIMG (the step loop is unrolled by the
  // ring depth): with run-time buffer indices the compiler cannot tell the DMA's target buffer from
  // the one being read and drains every DMA (vmcnt(0)) before the first ds_read of each step
  auto issue = [&](int st, uint16_t *img) {  // 4 glds per wave
    const int64_t k0 = k_beg + static_cast<int64_t>(st) * RBK;
    stage<RBK>(dy, ldy, k0, m0, M, img, wave, lane);
    stage<RBK>(x, ldx, k0, n0, N, img + RIMG, wave, lane);
  };
#pragma unroll
  for (int b = 0; b < NSTAGE - 1; ++b)
    if (b < nsteps) issue(b, lds + b * 2 * RIMG);
  for (int st0 = 0; st0 < nsteps; st0 += NSTAGE) {
#pragma unroll
    for (int b = 0; b < NSTAGE; ++b) {
      const int st = st0 + b;
      if (st < nsteps) {
        // retire step st's pieces: the later issued steps (up to 2) may stay in flight
        const int ahead = nsteps - 1 - st;
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (st + NSTAGE - 1 < nsteps) issue(st + NSTAGE - 1, lds + ((b + NSTAGE - 1) % NSTAGE) * 2 * RIMG);
        const uint16_t *ia = lds + b * 2 * RIMG;
        const uint16_t *ib = ia + RIMG;
#pragma unroll
        for (int ss = 0; ss < RBK / 16; ++ss) {
          bf16x8 fa[4], fb[2];
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[i] = frag(ia, ss, wm * 128 + i * 32, lane);
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[j] = frag(ib, ss, wn * 64 + j * 32, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  }

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

// Ring variant 2: the transposed reads as inline asm (tr_read_asm), so the compiler neither drains
// the DMA before them nor needs compile-time buffer offsets: a rolled step loop, fewer registers.
template <bool PARTIAL, int OPT = 0>
__global__ __launch_bounds__(NT, 1) void wgrad256_ring2_kernel(const uint16_t *__restrict__ dy, int64_t ldy,
                                                               const uint16_t *__restrict__ x, int64_t ldx, int64_t K,
                                                               int M, int N, int splits, int64_t kslice,
                                                               float *__restrict__ part, uint16_t *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[NSTAGE * 2 * RIMG];  // [stage][A | B][32][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM;
  const int nwg = nbn * nbm * splits;
  const int w = blockIdx.x, xcd = w & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (w >> 3);
  const int bn = logical % nbn;
  const int rest = logical / nbn;
  const int bm = rest % nbm, s = rest / nbm;
  const int m0 = bm * BM, n0 = bn * BN;
  const int64_t k_beg = static_cast<int64_t>(s) * kslice;
  const int64_t k_end = k_beg + kslice < K ? k_beg + kslice : K;
  const int nsteps = k_end > k_beg ? static_cast<int>((k_end - k_beg) / RBK) : 0;

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int st) {  // 4 glds per wave
    uint16_t *img = lds + (st % NSTAGE) * 2 * RIMG;
    const int64_t k0 = k_beg + static_cast<int64_t>(st) * RBK;
    stage<RBK>(dy, ldy, k0, m0, M, img, wave, lane);
    stage<RBK>(x, ldx, k0, n0, N, img + RIMG, wave, lane);
  };
  for (int b = 0; b < NSTAGE - 1; ++b)
    if (b < nsteps) issue(b);
  for (int st = 0; st < nsteps; ++st) {
    const int ahead = nsteps - 1 - st;
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (st + NSTAGE - 1 < nsteps) issue(st + NSTAGE - 1);
    const uint16_t *ia = lds + (st % NSTAGE) * 2 * RIMG;
    const uint16_t *ib = ia + RIMG;
#pragma unroll
    for (int ss = 0; ss < RBK / 16; ++ss) {
      // issue order A0 B0 B1 A1 A2 A3 (2 reads each); each counted wait releases the fragments it
      // passes through (the MFMAs cannot be scheduled above it) while the later reads stay in flight
      v2i a0, a1, a2, a3, a4, a5, a6, a7, b0, b1, b2, b3;
      frag_asm(ia, ss, wm * 128 + 0, lane, a0, a1);
      frag_asm(ib, ss, wn * 64 + 0, lane, b0, b1);
      frag_asm(ib, ss, wn * 64 + 32, lane, b2, b3);
      frag_asm(ia, ss, wm * 128 + 32, lane, a2, a3);
      frag_asm(ia, ss, wm * 128 + 64, lane, a4, a5);
      frag_asm(ia, ss, wm * 128 + 96, lane, a6, a7);
      asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1));
      if constexpr (OPT == 1) __builtin_amdgcn_s_setprio(1);
      const bf16x8 fb0 = join(b0, b1);
      bf16x8 fa = join(a0, a1);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc[0][0], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(b2), "+v"(b3));
      const bf16x8 fb1 = join(b2, b3);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc[0][1], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(a2), "+v"(a3));
      fa = join(a2, a3);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc[1][1], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a4), "+v"(a5));
      fa = join(a4, a5);
      acc[2][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc[2][0], 0, 0, 0);
      acc[2][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc[2][1], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a6), "+v"(a7));
      fa = join(a6, a7);
      acc[3][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc[3][0], 0, 0, 0);
      acc[3][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc[3][1], 0, 0, 0);
      if constexpr (OPT == 1) __builtin_amdgcn_s_setprio(0);
    }
  }

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
// variant 0: 64-token steps, 2 LDS buffers; 1: 32-token steps in a 4-deep ring; 2: the ring with the
// transposed reads as inline asm (no compiler-inserted DMA drain before them)
extern "C" int wg256_bf16(const void *dy, int64_t ldy, const void *x, int64_t ldx, int64_t K, int64_t M, int64_t N,
                          int splits, float *workspace, void *out, void *stream, int variant) {
  const int bk = variant >= 1 ? RBK : BK;
  if (K < 0 || K % bk || M < 8 || N < 8 || M % 8 || N % 8 || ldy % 8 || ldx % 8 || ldy < M || ldx < N) return -1;
  if (splits < 1 || splits > 256 || (splits > 1 && !workspace) || !dy || !x || !out) return -1;
  if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) % 16)
    return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t mn = M * N;
  const int64_t steps = K / bk;
  const int64_t kslice = (steps + splits - 1) / splits * bk;
  const int nwg = static_cast<int>(((M + BM - 1) / BM) * ((N + BN - 1) / BN) * splits);
  if (variant >= 1) {
    auto kern = splits == 1 ? (variant == 3 ? wgrad256_ring2_kernel<false, 1>
                               : variant == 2 ? wgrad256_ring2_kernel<false, 0> : wgrad256_ring_kernel<false>)
                            : (variant == 3 ? wgrad256_ring2_kernel<true, 1>
                               : variant == 2 ? wgrad256_ring2_kernel<true, 0> : wgrad256_ring_kernel<true>);
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(NT), 0, st, static_cast<const uint16_t *>(dy), ldy,
                       static_cast<const uint16_t *>(x), ldx, K, static_cast<int>(M), static_cast<int>(N), splits,
                       kslice, splits == 1 ? nullptr : workspace,
                       splits == 1 ? static_cast<uint16_t *>(out) : nullptr);
  } else if (splits == 1) {
    hipLaunchKernelGGL(wgrad256_kernel<false>, dim3(nwg), dim3(NT), 0, st, static_cast<const uint16_t *>(dy), ldy,
                       static_cast<const uint16_t *>(x), ldx, K, static_cast<int>(M), static_cast<int>(N), 1, kslice,
                       nullptr, static_cast<uint16_t *>(out));
  } else {
    hipLaunchKernelGGL(wgrad256_kernel<true>, dim3(nwg), dim3(NT), 0, st, static_cast<const uint16_t *>(dy), ldy,
                       static_cast<const uint16_t *>(x), ldx, K, static_cast<int>(M), static_cast<int>(N), splits,
                       kslice, workspace, nullptr);
  }
  if (splits > 1) {
    hipLaunchKernelGGL(reduce_kernel, dim3(static_cast<unsigned>((mn / 4 + 255) / 256)), dim3(256), 0, st, workspace,
                       splits, mn, static_cast<uint16_t *>(out));
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
