// Weight gradients of the packed backbone's linear layers: dW[M, N] = dY[K, M]^T X[K, N] in bf16
// with fp32 accumulation (K = packed tokens, M = out_features, N = in_features). Not a §8 row: it
// replaces the hipBLASLt GEMMs of torch's linear backward for this shape class (K in the 10^5 range,
// an output of a few hundred 256 x 256 tiles; both operands K-outer), which run at 0.69-0.89 PF/s on
// the bench's shapes (tools/wgrad256_bench.py at 690aed1, profiles/r03/wgrad256_probe.jsonl).
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

constexpr int WBK = 32, WNT = 512;

typedef short wbf16x8 __attribute__((ext_vector_type(8)));
typedef int wv2i __attribute__((ext_vector_type(2)));
typedef float wf32x16 __attribute__((ext_vector_type(16)));
typedef float wf32x4 __attribute__((ext_vector_type(4)));

// the wave tile's accumulators: 4 x 2 32x32 blocks (16 fp32 each) for the 128 x 64 wave tile, or
// (WM / 16) x (WN / 16) 16x16 blocks (4 each)
template <bool MF16, int NA = 4, int NB = 2>
struct WAcc {
  wf32x16 v[4][2];
};
template <int NA, int NB>
struct WAcc<true, NA, NB> {
  wf32x4 v[NA][NB];
};

// LDS image width of a tile dimension: 224 / 448 (896 = 4 x 224 = 2 x 448) are staged as 256 / 512
// columns (the XOR swizzle needs whole 256-byte row multiples; the extra 32 / 64 columns are fetched
// and never read)
constexpr int w_img(int t) { return t == 224 ? 256 : (t == 448 ? 512 : t); }

// element offset of (row, col) in a [32][C] image (C = 128, 256 or 512 columns) with 16-B chunks
// XOR-swizzled by (row & 3) << 2 (every row length is a multiple of the 64 banks' 256 bytes' worth of
// words, so the swizzle alone spreads a transposed read's 4 rows over all banks)
// SW16 (the 16x16x32 kernel's images): chunks XOR-swizzled by (row & 7) << 1 instead, since its
// transposed reads cover 2 chunks of 8 consecutive rows per 32 lanes (the 4-row swizzle would put rows
// r and r + 4 on the same banks)
template <int C, bool SW16 = false>
__device__ __forceinline__ int w_swz(int row) {
  return SW16 ? ((row & 7) << 1) : ((row & 3) << 2);
}

template <int C, bool SW16 = false>
__device__ __forceinline__ int w_off(int row, int col) {
  return row * C + (((col >> 3) ^ w_swz<C, SW16>(row)) << 3) + (col & 7);
}

// LDS-DMA of one operand's 32 x C step image: 1 KiB pieces of 512 / C rows, C / 128 per wave; lane l
// of piece g lands at physical chunk l % (C / 8) of row g (512 / C) + l / (C / 8) and so fetches the
// logical chunk the swizzle puts there
template <int C, bool SW16 = false>
__device__ __forceinline__ void w_stage(const uint16_t *__restrict__ src, int64_t ld, int64_t k0, int col0, int ncols,
                                        uint16_t *img, int wave, int lane) {
  constexpr int PW = C / 128, RPP = 512 / C, CPR = C / 8;
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int g = wave * PW + i;
    const int row = g * RPP + lane / CPR;
    const int c = (lane % CPR) ^ w_swz<C, SW16>(row);
    int col = col0 + c * 8;
    if (col > ncols - 8) col = ncols - 8;  // clamped: results for these columns are dropped
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + (k0 + row) * ld + col), img + g * 512, 16,
                                     0, 0);
  }
}

// the same staging through a buffer resource (PIPE kernels): lane offsets (row * ld + clamped column,
// in bytes, 32-bit) are computed once per kernel; per step only the resource's base moves to row k0
template <int C, bool SW16>
__device__ __forceinline__ void w_stage_offsets(int64_t ld, int col0, int ncols, int wave, int lane, int (&off)[C / 128]) {
  constexpr int PW = C / 128, RPP = 512 / C, CPR = C / 8;
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int g = wave * PW + i;
    const int row = g * RPP + lane / CPR;
    const int c = (lane % CPR) ^ w_swz<C, SW16>(row);
    int col = col0 + c * 8;
    if (col > ncols - 8) col = ncols - 8;
    off[i] = static_cast<int>((row * ld + col) * 2);
  }
}

template <int C>
__device__ __forceinline__ void w_stage_buf(const uint16_t *src, int64_t ld, int64_t k0, const int *off,
                                            uint16_t *img, int wave) {
  constexpr int PW = C / 128;
  const __amdgpu_buffer_rsrc_t res =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(src + k0 * ld), 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int i = 0; i < PW; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(res, img + (wave * PW + i) * 512, 16, off[i], 0, 0, 0);
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
template <int C>
__device__ __forceinline__ void w_frag(const uint16_t *img, int ss, int col_base, int lane, wv2i &lo, wv2i &hi) {
  const int h = lane >> 5, g16 = lane >> 4, li = lane & 15;
  const int r0 = 16 * ss + 4 * h + (li >> 2);
  const int col = col_base + 16 * (g16 & 1) + 4 * (li & 3);
  lo = w_tr_read(img + w_off<C>(r0, col));
  hi = w_tr_read(img + w_off<C>(r0 + 8, col));
}

// 16 columns x 32 k fragment (v_mfma_f32_16x16x32_bf16 A or B operand) by two transposed reads: the
// 16-lane group g = lane >> 4 reads rows 4 g .. 4 g + 3 and 16 + 4 g .. 16 + 4 g + 3 of its 16
// columns, so element j of lane (column col_base + (lane & 15)) = image[16 (j >> 2) + 4 g + (j & 3)]
// [column] (A and B in the same k order); each 32-lane half reads 8 distinct rows per instruction
template <int C>
__device__ __forceinline__ void w_frag16(const uint16_t *img, int col_base, int lane, wv2i &lo, wv2i &hi) {
  const int g = lane >> 4, li = lane & 15;
  const int r0 = 4 * g + (li >> 2);
  const int col = col_base + 4 * (li & 3);
  lo = w_tr_read(img + w_off<C, true>(r0, col));
  hi = w_tr_read(img + w_off<C, true>(r0 + 16, col));
}

// retire all but N of this wave's LDS-DMA instructions (N a literal of the counted-wait encoding)
template <int N>
__device__ __forceinline__ void w_vm_wait() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

// retire all but N of this wave's LDS reads, naming the fragment registers those reads produced
template <int N>
__device__ __forceinline__ void w_lgkm_wait(wv2i &lo, wv2i &hi) {
  if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo), "+v"(hi));
  else if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(lo), "+v"(hi));
  else if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(lo), "+v"(hi));
  else if constexpr (N == 6) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(lo), "+v"(hi));
  else if constexpr (N == 8) asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(lo), "+v"(hi));
  else if constexpr (N == 10) asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(lo), "+v"(hi));
  else if constexpr (N == 12) asm volatile("s_waitcnt lgkmcnt(12)" : "+v"(lo), "+v"(hi));
  else if constexpr (N == 14) asm volatile("s_waitcnt lgkmcnt(14)" : "+v"(lo), "+v"(hi));
  else static_assert(N == 0, "unsupported lgkmcnt");
}

// the same with the count as a value that is a constant after unrolling (the switch folds away)
__device__ __forceinline__ void w_lgkm_wait_n(int n, wv2i &lo, wv2i &hi) {
  switch (n) {
    case 0: w_lgkm_wait<0>(lo, hi); break;
    case 2: w_lgkm_wait<2>(lo, hi); break;
    case 4: w_lgkm_wait<4>(lo, hi); break;
    case 6: w_lgkm_wait<6>(lo, hi); break;
    case 8: w_lgkm_wait<8>(lo, hi); break;
    case 10: w_lgkm_wait<10>(lo, hi); break;
    case 12: w_lgkm_wait<12>(lo, hi); break;
    default: w_lgkm_wait<14>(lo, hi); break;
  }
}

__device__ __forceinline__ wbf16x8 w_join(wv2i lo, wv2i hi) {
  return __builtin_bit_cast(wbf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3));
}

__device__ __forceinline__ int w_crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// one 32-token step of the 16x16x32 form: 24 transposed reads issued A0 B0..B3 A1..A7, each counted
// wait releasing the next A fragment while the later reads stay in flight; 32 MFMAs
template <int TM, int TN, int I>
__device__ __forceinline__ void w_step16_row(const uint16_t *ia, int wm, int lane, wv2i (&a)[8][2],
                                             const wbf16x8 (&fb)[4], wf32x4 (&acc)[8][4]) {
  w_lgkm_wait<14 - 2 * I>(a[I][0], a[I][1]);
  const wbf16x8 fa = w_join(a[I][0], a[I][1]);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[I][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[I][j], 0, 0, 0);
}

template <int TM, int TN>
__device__ __forceinline__ void w_step16(const uint16_t *ia, const uint16_t *ib, int wm, int wn, int lane,
                                         wf32x4 (&acc)[8][4]) {
  wv2i a[8][2], b[4][2];
  w_frag16<TM>(ia, wm * 128, lane, a[0][0], a[0][1]);
#pragma unroll
  for (int j = 0; j < 4; ++j) w_frag16<TN>(ib, wn * 64 + j * 16, lane, b[j][0], b[j][1]);
#pragma unroll
  for (int i = 1; i < 8; ++i) w_frag16<TM>(ia, wm * 128 + i * 16, lane, a[i][0], a[i][1]);
  // A0 and B0..B3 are the first 10 reads: 14 may stay outstanding
  asm volatile("s_waitcnt lgkmcnt(14)" : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]), "+v"(b[1][1]), "+v"(b[2][0]),
               "+v"(b[2][1]), "+v"(b[3][0]), "+v"(b[3][1]));
  wbf16x8 fb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[j] = w_join(b[j][0], b[j][1]);
  w_step16_row<TM, TN, 0>(ia, wm, lane, a, fb, acc);
  w_step16_row<TM, TN, 1>(ia, wm, lane, a, fb, acc);
  w_step16_row<TM, TN, 2>(ia, wm, lane, a, fb, acc);
  w_step16_row<TM, TN, 3>(ia, wm, lane, a, fb, acc);
  w_step16_row<TM, TN, 4>(ia, wm, lane, a, fb, acc);
  w_step16_row<TM, TN, 5>(ia, wm, lane, a, fb, acc);
  w_step16_row<TM, TN, 6>(ia, wm, lane, a, fb, acc);
  w_step16_row<TM, TN, 7>(ia, wm, lane, a, fb, acc);
}

// make a wave's uses of lo / hi stay below the counted wait just issued (an empty asm statement is
// ordered with the wait; the MFMA builtins that read the registers follow it)
__device__ __forceinline__ void w_tie(wv2i &lo, wv2i &hi) { asm volatile("" : "+v"(lo), "+v"(hi)); }

// one 32-token step of a general (NA x 16) x (NB x 16) wave tile in the 16x16x32 form (the 896-wide
// tiles' 64 x 112 / 112 x 64 wave tiles): the operand with more fragments is streamed, the other one
// held. Reads are issued H0, S0..S(n-1), H1..H(h-1) for the held operand H (h fragments) and the
// streamed S (n fragments) when h >= n, else S0, H0..H(h-1), S1..S(n-1); one counted wait for the
// first row / column, then one per later fragment (2 transposed reads each, at most 14 outstanding)
template <int IA, int IB, int NA, int NB>
__device__ __forceinline__ void w_step16g(const uint16_t *ia, const uint16_t *ib, int am0, int bn0, int lane,
                                          wf32x4 (&acc)[NA][NB]) {
  static_assert(2 * (NA > NB ? NA : NB) - 2 <= 14, "counted waits reach lgkmcnt(14) at most");
  wv2i a[NA][2], b[NB][2];
  if constexpr (NA >= NB) {
    w_frag16<IA>(ia, am0, lane, a[0][0], a[0][1]);
#pragma unroll
    for (int j = 0; j < NB; ++j) w_frag16<IB>(ib, bn0 + j * 16, lane, b[j][0], b[j][1]);
#pragma unroll
    for (int i = 1; i < NA; ++i) w_frag16<IA>(ia, am0 + i * 16, lane, a[i][0], a[i][1]);
    w_lgkm_wait<2 * (NA - 1)>(a[0][0], a[0][1]);
    wbf16x8 fb[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      w_tie(b[j][0], b[j][1]);
      fb[j] = w_join(b[j][0], b[j][1]);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if (i > 0) w_lgkm_wait_n(2 * (NA - 1 - i), a[i][0], a[i][1]);
      const wbf16x8 fa = w_join(a[i][0], a[i][1]);
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
    }
  } else {
    w_frag16<IB>(ib, bn0, lane, b[0][0], b[0][1]);
#pragma unroll
    for (int i = 0; i < NA; ++i) w_frag16<IA>(ia, am0 + i * 16, lane, a[i][0], a[i][1]);
#pragma unroll
    for (int j = 1; j < NB; ++j) w_frag16<IB>(ib, bn0 + j * 16, lane, b[j][0], b[j][1]);
    w_lgkm_wait<2 * (NB - 1)>(b[0][0], b[0][1]);
    wbf16x8 fa[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      w_tie(a[i][0], a[i][1]);
      fa[i] = w_join(a[i][0], a[i][1]);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (j > 0) w_lgkm_wait_n(2 * (NB - 1 - j), b[j][0], b[j][1]);
      const wbf16x8 fb = w_join(b[j][0], b[j][1]);
#pragma unroll
      for (int i = 0; i < NA; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i][j], 0, 0, 0);
    }
  }
}

// Cross-step software pipeline of the 16x16x32 forms (PIPE): a wave's fragments of step st + 1 are
// read from LDS right after the barrier that publishes them and land while the MFMAs of step st run
// on the fragments read one iteration earlier (two register sets). Without it every wave issues its
// 22-24 transposed reads after the barrier and waits for all of them before its first MFMA, and the
// 8 waves' reads (~90 KB per CU and step, ~350 LDS cycles) are exposed in every step: the partner
// wave on the SIMD is in the same phase, so it cannot cover them.
template <int NA, int NB>
struct WFrags {
  wv2i a[NA][2], b[NB][2];
};

template <int IA, int IB, int NA, int NB>
__device__ __forceinline__ void w_read16g(const uint16_t *ia, const uint16_t *ib, int am0, int bn0, int lane,
                                          WFrags<NA, NB> &f) {
#pragma unroll
  for (int i = 0; i < NA; ++i) w_frag16<IA>(ia, am0 + i * 16, lane, f.a[i][0], f.a[i][1]);
#pragma unroll
  for (int j = 0; j < NB; ++j) w_frag16<IB>(ib, bn0 + j * 16, lane, f.b[j][0], f.b[j][1]);
}

// retire every LDS read of this wave; the fragment registers are named so that no MFMA reading them
// is scheduled above the wait
template <int NA, int NB>
__device__ __forceinline__ void w_frags_ready(WFrags<NA, NB> &f) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f.a[0][0]), "+v"(f.a[0][1]));
#pragma unroll
  for (int i = 1; i < NA; ++i) w_tie(f.a[i][0], f.a[i][1]);
#pragma unroll
  for (int j = 0; j < NB; ++j) w_tie(f.b[j][0], f.b[j][1]);
}

template <int NA, int NB>
__device__ __forceinline__ void w_mma16g(const WFrags<NA, NB> &f, wf32x4 (&acc)[NA][NB]) {
  wbf16x8 fb[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) fb[j] = w_join(f.b[j][0], f.b[j][1]);
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const wbf16x8 fa = w_join(f.a[i][0], f.a[i][1]);
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
  }
}

// retire all but `steps` steps of this wave's LDS-DMA pieces (PER pieces per step; steps a value that
// is a constant per call site after unrolling)
template <int PER>
__device__ __forceinline__ void w_vm_wait_steps(int steps) {
  if (steps >= 3) w_vm_wait<3 * PER>();
  else if (steps == 2) w_vm_wait<2 * PER>();
  else if (steps == 1) w_vm_wait<PER>();
  else w_vm_wait<0>();
}

// TM x TN output tile (256 x 256, or 512 x 128 / 128 x 512 for the 128-wide remainder of a
// dimension that is 128 mod 256): 8 waves of 128 x 64 as (TM / 128) x (TN / 64); NST-deep ring.
// MF16: the wave tile as 8 x 4 v_mfma_f32_16x16x32_bf16 blocks (one MFMA depth per 32-token step,
// 16-column fragments, the 8-row image swizzle) instead of 4 x 2 32x32x16 blocks.
template <bool PARTIAL, int TM, int TN, int NST, bool MF16 = false, int WM = 128, int WN = 64, int PIPE = 0>
__global__ __launch_bounds__(WNT, 1) void wgrad_kernel(const uint16_t *__restrict__ dy, int64_t ldy,
                                                       const uint16_t *__restrict__ x, int64_t ldx, int64_t K, int M,
                                                       int N, int splits, int64_t kslice, float *__restrict__ part,
                                                       uint16_t *__restrict__ out, int64_t ldo) {
  constexpr int WN_W = TN / WN;                      // waves along n
  constexpr int IA = w_img(TM), IB = w_img(TN);      // LDS image widths
  constexpr int AIMG = WBK * IA, BIMG = WBK * IB;    // step images
  constexpr int PER = (IA + IB) / 128;               // LDS-DMA instructions per wave per step
  constexpr int NA = WM / 16, NB = WN / 16;          // 16x16 blocks of the general wave tile
  constexpr bool GEN = !(WM == 128 && WN == 64);     // a 64 x 112 / 112 x 64 wave tile (16x16x32 only)
  static_assert((TM / WM) * WN_W == 8, "8 waves");
  static_assert(!GEN || MF16, "general wave tiles use the 16x16x32 form");
  static_assert(!PIPE || MF16, "the cross-step pipeline is built for the 16x16x32 form");
  __shared__ __attribute__((aligned(16))) uint16_t lds[NST * (AIMG + BIMG)];  // [stage][A | B]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN_W, wn = wave % WN_W;
  const int nbn = (N + TN - 1) / TN, nbm = (M + TM - 1) / TM;
  // XCD-aware bijective remap: hardware ids w, w + 8, ... share an XCD; give them consecutive
  // logical tiles, n-tile fastest, so the n-tiles of one dY tile and K slice share an L2
  const int nwg = nbn * nbm * splits;
  const int w = blockIdx.x, xcd = w & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (w >> 3);
  const int bn = logical % nbn;
  const int rest = logical / nbn;
  const int bm = rest % nbm, s = rest / nbm;
  const int m0 = bm * TM, n0 = bn * TN;
  const int64_t k_beg = static_cast<int64_t>(s) * kslice;
  const int64_t k_end = k_beg + kslice < K ? k_beg + kslice : K;
  const int nsteps = k_end > k_beg ? static_cast<int>((k_end - k_beg) / WBK) : 0;

  WAcc<MF16, (GEN ? NA : 8), (GEN ? NB : 4)> accs;
  auto &acc = accs.v;
  if constexpr (MF16) {
#pragma unroll
    for (int i = 0; i < (GEN ? NA : 8); ++i)
#pragma unroll
      for (int j = 0; j < (GEN ? NB : 4); ++j) acc[i][j] = wf32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  }

  auto issue = [&](int st) {  // PER LDS-DMA instructions per wave
    uint16_t *img = lds + (st % NST) * (AIMG + BIMG);
    const int64_t k0 = k_beg + static_cast<int64_t>(st) * WBK;
    w_stage<IA, MF16>(dy, ldy, k0, m0, M, img, wave, lane);
    w_stage<IB, MF16>(x, ldx, k0, n0, N, img + AIMG, wave, lane);
  };
  // PIPE: a DMA of step `src` into ring buffer `buf` (branch-free: every iteration but the last
  // issues one step's pieces, so the counted waits are constants)
  int offa[IA / 128], offb[IB / 128];
  if constexpr (PIPE) {
    w_stage_offsets<IA, MF16>(ldy, m0, M, wave, lane, offa);
    w_stage_offsets<IB, MF16>(ldx, n0, N, wave, lane, offb);
  }
  auto issue_to = [&](int buf, int src) {
    uint16_t *img = lds + buf * (AIMG + BIMG);
    const int64_t k0 = k_beg + static_cast<int64_t>(src) * WBK;
    w_stage_buf<IA>(dy, ldy, k0, offa, img, wave);
    w_stage_buf<IB>(x, ldx, k0, offb, img + AIMG, wave);
  };
  if constexpr (PIPE) {
    WFrags<NA, NB> f0, f1;
    if (nsteps > 0) {
      // steps 0 .. NST - 1 (past the end: the last step again, into buffers never read)
      for (int b = 0; b < NST; ++b) issue_to(b, b < nsteps ? b : nsteps - 1);
      w_vm_wait<(NST - 1) * PER>();
      asm volatile("s_barrier" ::: "memory");
      w_read16g<IA, IB, NA, NB>(lds, lds + AIMG, wm * WM, wn * WN, lane, f0);
    }
    // iteration st: fragments of step st ready; publish step st + 1 (steps through st + NST - 1 are
    // issued: NST - 2 stay in flight), read its fragments, then the MFMAs of step st with the DMA of
    // step st + NST into step st's buffer (free once every wave passed this barrier) spread between
    // them, PER pieces in gaps of G MFMAs
    constexpr int NM = NA * NB, G = NM / (PER + 1);
    // PIPE 1: the DMA right after the barrier, ahead of the reads (its own scheduling region);
    // PIPE 2: between the MFMAs, PER pieces in gaps of G MFMAs (sched_group_barrier)
    // PIPE 3: the fragment reads of step st + 1 between the MFMAs too (one per MFMA), so no burst of
    // LDS reads sits between the barrier and the first MFMA
    constexpr int NR = 2 * (NA + NB);  // transposed reads per step
    auto body = [&](int st, WFrags<NA, NB> &cur, WFrags<NA, NB> &nxt) {
      w_frags_ready(cur);
      const bool more = st + 1 < nsteps;
      // the last iteration has passed no barrier that ends the other waves' reads of step st's
      // buffer, so its (unneeded) DMA goes to buffer st + 1, which holds no step that is read
      const int buf = (more ? st : st + 1) % NST, src = st + NST < nsteps ? st + NST : nsteps - 1;
      const uint16_t *im = lds + ((st + 1) % NST) * (AIMG + BIMG);
      if constexpr (PIPE == 3) {
        // (the last iteration's reads land in registers nobody uses; no barrier is needed for them)
        if (more) {
          w_vm_wait<(NST - 2) * PER>();
          asm volatile("s_barrier" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        issue_to(buf, src);
        w_read16g<IA, IB, NA, NB>(im, im + AIMG, wm * WM, wn * WN, lane, nxt);
        w_mma16g<NA, NB>(cur, acc);
        int p = 0;
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
          if (i < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one fragment read
          if (i % G == G - 1 && p < PER) {
            __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // one LDS-DMA piece
            ++p;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        return;
      }
      if (more) {
        w_vm_wait<(NST - 2) * PER>();
        asm volatile("s_barrier" ::: "memory");
        if constexpr (PIPE == 1) issue_to(buf, src);
        w_read16g<IA, IB, NA, NB>(im, im + AIMG, wm * WM, wn * WN, lane, nxt);
      } else if constexpr (PIPE == 1) {
        issue_to(buf, src);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (PIPE == 2) issue_to(buf, src);
      w_mma16g<NA, NB>(cur, acc);
      if constexpr (PIPE == 2) {
#pragma unroll
        for (int p = 0; p < PER; ++p) {
          __builtin_amdgcn_sched_group_barrier(0x008, G, 0);  // G MFMAs
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // one LDS-DMA piece
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM - PER * G, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    int st = 0;
    for (; st + 1 < nsteps; st += 2) {
      body(st, f0, f1);
      body(st + 1, f1, f0);
    }
    if (st < nsteps) body(st, f0, f1);
    w_vm_wait<0>();  // no LDS-DMA outlives the workgroup's LDS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else {
  for (int b = 0; b < NST - 1; ++b)
      if (b < nsteps) issue(b);
    for (int st = 0; st < nsteps; ++st) {
      const int ahead = nsteps - 1 - st;  // steps issued after st (at most NST - 2 here)
      if (NST >= 4 && ahead >= 2) w_vm_wait<2 * PER * (NST >= 4)>();
      else if (ahead >= 1) w_vm_wait<PER>();
      else w_vm_wait<0>();
      asm volatile("s_barrier" ::: "memory");
      if (st + NST - 1 < nsteps) issue(st + NST - 1);
      const uint16_t *ia = lds + (st % NST) * (AIMG + BIMG);
      const uint16_t *ib = ia + AIMG;
      if constexpr (GEN) {
        w_step16g<IA, IB, NA, NB>(ia, ib, wm * WM, wn * WN, lane, acc);
      } else if constexpr (MF16) {
        w_step16<IA, IB>(ia, ib, wm, wn, lane, acc);
      } else {
  #pragma unroll
      for (int ss = 0; ss < WBK / 16; ++ss) {
        // issue order A0 B0 B1 A1 A2 A3 (2 reads each); each counted wait releases the fragments it
        // passes through while the later reads stay in flight
        wv2i a0, a1, a2, a3, a4, a5, a6, a7, b0, b1, b2, b3;
        w_frag<IA>(ia, ss, wm * 128 + 0, lane, a0, a1);
        w_frag<IB>(ib, ss, wn * 64 + 0, lane, b0, b1);
        w_frag<IB>(ib, ss, wn * 64 + 32, lane, b2, b3);
        w_frag<IA>(ia, ss, wm * 128 + 32, lane, a2, a3);
        w_frag<IA>(ia, ss, wm * 128 + 64, lane, a4, a5);
        w_frag<IA>(ia, ss, wm * 128 + 96, lane, a6, a7);
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
      }  // MF16
    }
  }

  if constexpr (MF16) {
    // lane holds C[m = m0 + wm WM + i 16 + 4 (lane >> 4) + e][n = n0 + wn WN + j 16 + (lane & 15)]
#pragma unroll
    for (int i = 0; i < (GEN ? NA : 8); ++i)
#pragma unroll
      for (int j = 0; j < (GEN ? NB : 4); ++j) {
        const int n = n0 + wn * WN + j * 16 + (lane & 15);
        if (n >= N) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + wm * WM + i * 16 + 4 * (lane >> 4) + e;
          if (m >= M) continue;
          if constexpr (PARTIAL) part[(static_cast<int64_t>(s) * M + m) * N + n] = acc[i][j][e];
          else out[m * ldo + n] = static_cast<uint16_t>(pack2_bf16(acc[i][j][e], 0.f) & 0xffffu);
        }
      }
  } else {
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
          else out[m * ldo + n] = static_cast<uint16_t>(pack2_bf16(acc[i][j][r], 0.f) & 0xffffu);
        }
      }
  }
}

// out[m][n] (row stride ldo) = bf16(sum_s part[s][m][n]) in slice order; 4 elements per thread (N % 4 == 0)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float *__restrict__ part, int splits, int64_t M,
                                                           int64_t N, uint16_t *__restrict__ out, int64_t ldo) {
  const int64_t e = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  const int64_t mn = M * N;
  if (e >= mn) return;
  float4 acc = *reinterpret_cast<const float4 *>(part + e);
  for (int s = 1; s < splits; ++s) {
    const float4 v = *reinterpret_cast<const float4 *>(part + static_cast<int64_t>(s) * mn + e);
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  const int64_t m = e / N, n = e - m * N;
  *reinterpret_cast<uint2 *>(out + m * ldo + n) = make_uint2(pack2_bf16(acc.x, acc.y), pack2_bf16(acc.z, acc.w));
}

}  // namespace
}  // namespace va

using namespace va;

// va_set_tuning(VA_TUNE_WGRAD_KIND): -1 = the cost model's tile shape, else that kind (A/B runs)
int g_wgrad_kind = -1;

namespace {

// fewest 32-token steps a slice gets: the 4-deep ring keeps 3 in flight, so a shorter slice is mostly
// prologue / epilogue, and every slice costs an fp32 M x N partial that the reduce reads back
constexpr int64_t kMinStepsPerSlice = 8;

// K slices of one launch: one round of workgroups when it fills >= 85 % of the 256 CUs, else about
// three full rounds; at most one slice per kMinStepsPerSlice steps (kernels.own_wgrad_splits mirrors it)
int w_auto_splits(int64_t tiles, int64_t steps) {
  int64_t s = 256 / tiles;
  if (!(s >= 1 && tiles * s * 100 >= 85 * 256)) s = (768 + tiles / 2) / tiles;
  const int64_t cap = steps / kMinStepsPerSlice;
  if (s > cap) s = cap;
  if (s < 1) s = 1;
  return static_cast<int>(s > 256 ? 256 : s);
}

// The launches of one weight gradient. Tile kinds (all 8 waves, 1 workgroup per CU):
//   0: 256 x 256, wave tile 128 x 64 (32x32x16 or, with VA_TUNE_WGRAD_MFMA = 16, 16x16x32 blocks)
//   1: 512 x 128 / 2: 128 x 512 (wave tile 128 x 64): with VA_TUNE_WGRAD_TILES = 0 the 128-wide
//      remainder of a dimension that is 128 mod 256 (VA_TUNE_WGRAD_REMAINDER = 1, a second launch
//      beside kind 0); with the planner (>= 1) whole-launch candidates like the kinds below (896 =
//      7 x 128)
//   3: 256 x 224 / 4: 224 x 256 / 5: 128 x 448 / 6: 448 x 128 (VA_TUNE_WGRAD_TILES = 1): tiles that
//      divide 896 = 4 x 224 = 2 x 448 (Qwen2.5-0.5B's hidden size) exactly, wave tiles 64 x 112 /
//      112 x 64 of 16x16x32 blocks, so none of the MFMA work is spent on padding (256 x 256 tiles
//      compute 1024 columns for 896: 12.5 % of gate|up's and down's MFMAs, 21-23 % of q|k|v's and o's)
struct WPart {
  int kind;
  int64_t m0, n0, M, N;
  int splits;
};

constexpr int w_kind_tm(int k) { return k == 1 ? 512 : k == 2 ? 128 : k == 3 ? 256 : k == 4 ? 224 : k == 5 ? 128 : k == 6 ? 448 : 256; }
constexpr int w_kind_tn(int k) { return k == 1 ? 128 : k == 2 ? 512 : k == 3 ? 224 : k == 4 ? 256 : k == 5 ? 448 : k == 6 ? 128 : 256; }

int w_plan(int64_t K, int64_t M, int64_t N, int splits, WPart (&p)[2]) {
  const int64_t steps = K / WBK;
  int n = 0;
  if (N % 256 == 128 && N > 128) {
    p[n++] = WPart{0, 0, 0, M, N - 128, 0};
    p[n++] = WPart{1, 0, N - 128, M, 128, 0};
  } else if (M % 256 == 128 && M > 128) {
    p[n++] = WPart{0, 0, 0, M - 128, N, 0};
    p[n++] = WPart{2, M - 128, 0, 128, N, 0};
  } else {
    p[n++] = WPart{0, 0, 0, M, N, 0};
  }
  for (int i = 0; i < n; ++i) {
    const int tm = w_kind_tm(p[i].kind), tn = w_kind_tn(p[i].kind);
    const int64_t tiles = ((p[i].M + tm - 1) / tm) * ((p[i].N + tn - 1) / tn);
    p[i].splits = (splits > 0 && n == 1) ? splits : w_auto_splits(tiles, steps);
  }
  return n;
}

// Estimated time of one launch of `kind` with s K slices, in units of one workgroup-step of one
// output element (a 32-token step of a 256 x 256 tile = 65,536 units = ~1 us at ~1.1 PF/s over 256
// CUs): rounds of 256 workgroups x tile area x (steps per slice + 8 steps of ring fill and epilogue)
// x the kind's measured efficiency factor, plus the split-K reduce (8 B per output element and slice
// at ~5 TB/s = 0.11 units, + one launch)
// measured issue efficiency per unit of tile area (profiles/r06/i/wgrad_tiles_ab_2.jsonl, every kind
// forced on the bench's five shapes): the 128 x 64 wave tile (kinds 0-2: 24 fragment reads per 32
// MFMAs) runs ~6-8 % more flops per cycle than 64 x 112 / 112 x 64 (22 per 28), and the 448-wide
// shapes (5, 6) ~4 % more than 256 x 224 / 224 x 256 (3, 4)
constexpr double w_kind_factor(int k) { return k == 0 ? 0.92 : (k <= 2 ? 0.94 : (k <= 4 ? 1.0 : 0.96)); }

double w_cost(int kind, int64_t steps, int64_t M, int64_t N, int64_t s) {
  const int64_t tm = w_kind_tm(kind), tn = w_kind_tn(kind);
  const int64_t tiles = ((M + tm - 1) / tm) * ((N + tn - 1) / tn);
  const int64_t rounds = (tiles * s + 255) / 256;
  const double per_slice = static_cast<double>((steps + s - 1) / s) + 8.0;
  double c = static_cast<double>(rounds) * static_cast<double>(tm * tn) * per_slice * w_kind_factor(kind);
  if (s > 1) c += 0.11 * static_cast<double>(s) * static_cast<double>(M * N) + 2.0e5;
  return c;
}

// VA_TUNE_WGRAD_TILES = 1: one launch of the tile kind and slice count with the least estimated
// time (kind 0 against the 896-dividing kinds; an explicit splits > 0 is taken as given)
int w_plan_tiles(int64_t K, int64_t M, int64_t N, int splits, WPart (&p)[2]) {
  const int64_t steps = K / WBK;
  const int64_t cap = steps / kMinStepsPerSlice < 1 ? 1 : (steps / kMinStepsPerSlice > 256 ? 256 : steps / kMinStepsPerSlice);
  double best = 0.0;
  int bk = -1, bs = 1;
  for (int kind : {0, 1, 2, 3, 4, 5, 6}) {
    if (g_wgrad_kind >= 0 && kind != g_wgrad_kind) continue;
    const int64_t s_lo = splits > 0 ? splits : 1, s_hi = splits > 0 ? splits : (cap < 64 ? cap : 64);
    for (int64_t sv = s_lo; sv <= s_hi; ++sv) {
      const double c = w_cost(kind, steps, M, N, sv);
      if (bk < 0 || c < best * 0.999) {
        best = c;
        bk = kind;
        bs = static_cast<int>(sv);
      }
    }
  }
  p[0] = WPart{bk, 0, 0, M, N, bs};
  return 1;
}

int64_t w_part_bytes(const WPart &p) {
  return p.splits > 1 ? static_cast<int64_t>(sizeof(float)) * p.splits * p.M * p.N : 0;
}

template <int TM, int TN, int NST, bool MF16, int WM = 128, int WN = 64, int PIPE = 0>
int w_launch(const WPart &p, const uint16_t *dy, int64_t ldy, const uint16_t *x, int64_t ldx, int64_t K,
              float *ws, uint16_t *out, int64_t ldo, hipStream_t st) {
  const int64_t steps = K / WBK;
  const int64_t kslice = (steps + p.splits - 1) / p.splits * WBK;
  const int64_t nwg = ((p.M + TM - 1) / TM) * ((p.N + TN - 1) / TN) * p.splits;
  const uint16_t *dyp = dy + p.m0, *xp = x + p.n0;  // column offsets of the operands
  uint16_t *op = out + p.m0 * ldo + p.n0;
  VA_CHECK_ARG(nwg < (int64_t{1} << 31) && (p.M * p.N / 4 + 255) / 256 < (int64_t{1} << 31),
               "weight_grad: grid too large (%lld workgroups)", static_cast<long long>(nwg));
  if (p.splits == 1) {
    hipLaunchKernelGGL((wgrad_kernel<false, TM, TN, NST, MF16, WM, WN, PIPE>), dim3(static_cast<unsigned>(nwg)), dim3(WNT), 0,
                       st, dyp, ldy, xp, ldx, K, static_cast<int>(p.M), static_cast<int>(p.N), 1, kslice, nullptr, op,
                       ldo);
  } else {
    hipLaunchKernelGGL((wgrad_kernel<true, TM, TN, NST, MF16, WM, WN, PIPE>), dim3(static_cast<unsigned>(nwg)), dim3(WNT), 0,
                       st, dyp, ldy, xp, ldx, K, static_cast<int>(p.M), static_cast<int>(p.N), p.splits, kslice, ws,
                       nullptr, ldo);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(static_cast<unsigned>((p.M * p.N / 4 + 255) / 256)), dim3(256), 0,
                       st, ws, p.splits, p.M, p.N, op, ldo);
  }
  return VA_OK;
}

}  // namespace

// va_set_tuning(VA_TUNE_WGRAD_REMAINDER): 0 (default) = every tile 256 x 256; 1 = the 128-wide
// remainder tiles above. Interleaved bench A/B on one MI355X: 182.36 / 182.49K tokens/s with 256 x 256
// tiles vs 182.08 / 181.96K with the remainder tiles (profiles/r04/bench_wgrad_remainder_ab.txt): the
// half-empty 256-wide tiles cost less than a second launch per weight gradient
int g_wgrad_remainder = 0;
// va_set_tuning(VA_TUNE_WGRAD_MFMA): 32 (default) = 4 x 2 v_mfma_f32_32x32x16_bf16 blocks per wave,
// 16 = 8 x 4 v_mfma_f32_16x16x32_bf16 blocks (the MFMA form of f1's sweep)
int g_wgrad_mfma = 32;
// va_set_tuning(VA_TUNE_WGRAD_TILES): 1-4 = the cost-model planner over the 256 x 256 and the
// 896-dividing tile kinds (w_plan_tiles), every kind in the 16x16x32 form; 2 = with the cross-step
// fragment pipeline (buffer-resource LDS-DMA after the barrier), 3 = the pipeline with the LDS-DMA
// spread between the MFMAs, 4 (default) = the fragment reads in the MFMAs' scheduling region too
// (profiles/r06/e/wgrad_tiles_ab_2.jsonl: backbone 395.8 ms per step vs 413.3 for 3 and 463.8 for
// the round-5 kernel (0), lm_head 33.5 ms vs 36.1 for hipBLASLt); 1 = no pipeline; 0 = kind 0 (+ the
// remainder setting) with w_auto_splits
int g_wgrad_tiles = 4;

namespace {
// The launches of one weight gradient under the current tile settings (the size query and the
// launch each plan once; the launch checks its plan against the caller's buffer size)
int w_plan_all(int64_t K, int64_t M, int64_t N, int splits, WPart (&p)[2]) {
  if (g_wgrad_tiles) return w_plan_tiles(K, M, N, splits, p);
  if (g_wgrad_remainder) return w_plan(K, M, N, splits, p);
  p[0] = WPart{0, 0, 0, M, N, splits > 0 ? splits : w_auto_splits(((M + 255) / 256) * ((N + 255) / 256), K / WBK)};
  return 1;
}
}  // namespace

extern "C" int64_t va_weight_grad_workspace_bytes(int64_t K, int64_t M, int64_t N, int splits) {
  WPart p[2];
  const int n = w_plan_all(K, M, N, splits, p);
  int64_t b = 0;
  for (int i = 0; i < n; ++i) b += w_part_bytes(p[i]);
  return b;
}

extern "C" int va_weight_grad(const void *dy, int64_t ldy, const void *x, int64_t ldx, int64_t K, int64_t M, int64_t N,
                              int splits, float *workspace, int64_t workspace_bytes, void *out, void *stream) {
  VA_CHECK_ARG(K >= 0 && K % WBK == 0, "weight_grad: K (tokens) must be a multiple of 32 (K=%lld)",
               static_cast<long long>(K));
  VA_CHECK_ARG(M >= 8 && N >= 8 && M % 8 == 0 && N % 8 == 0 && M < (1 << 30) && N < (1 << 30),
               "weight_grad: M, N must be multiples of 8 (M=%lld N=%lld)", static_cast<long long>(M),
               static_cast<long long>(N));
  VA_CHECK_ARG(ldy >= M && ldx >= N && ldy % 8 == 0 && ldx % 8 == 0, "weight_grad: bad leading dimensions");
  VA_CHECK_ARG(splits >= 0 && splits <= 256, "weight_grad: splits must be in [0, 256] (0 = automatic)");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t mn = M * N;
  VA_CHECK_ARG(out != nullptr, "null pointer argument");
  if (K == 0) {  // no tokens: dW = 0 (the operands may be empty views without storage)
    if (hipMemsetAsync(out, 0, mn * 2, st) != hipSuccess) return check_launch("weight_grad");
    return VA_OK;
  }
  WPart p[2];
  const int n = w_plan_all(K, M, N, splits, p);
  int64_t need = 0;
  for (int i = 0; i < n; ++i) need += w_part_bytes(p[i]);
  VA_CHECK_ARG(dy && x && (need == 0 || workspace), "null pointer argument");
  VA_CHECK_ARG(need <= workspace_bytes, "weight_grad: the plan needs %lld workspace bytes, %lld given",
               static_cast<long long>(need), static_cast<long long>(workspace_bytes));
  VA_CHECK_ARG(((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) &
                15) == 0,
               "weight_grad: 16-byte aligned buffers required");
  const auto *dy16 = static_cast<const uint16_t *>(dy);
  const auto *x16 = static_cast<const uint16_t *>(x);
  auto *o16 = static_cast<uint16_t *>(out);
  float *ws = workspace;
  for (int i = 0; i < n; ++i) {
    int rc;
    const bool mf16 = g_wgrad_mfma == 16;
    const int pipe = g_wgrad_tiles >= 2 ? g_wgrad_tiles - 1 : 0;  // PIPE form of the kernels
    if (p[i].kind == 0 && pipe)
      rc = pipe == 1   ? w_launch<256, 256, 4, true, 128, 64, 1>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 2 ? w_launch<256, 256, 4, true, 128, 64, 2>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                       : w_launch<256, 256, 4, true, 128, 64, 3>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else if (p[i].kind == 0)
      rc = mf16 ? w_launch<256, 256, 4, true>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                : w_launch<256, 256, 4, false>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else if (p[i].kind == 1 && pipe)
      rc = pipe == 3   ? w_launch<512, 128, 4, true, 128, 64, 3>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 2 ? w_launch<512, 128, 4, true, 128, 64, 2>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                       : w_launch<512, 128, 4, true, 128, 64, 1>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else if (p[i].kind == 2 && pipe)
      rc = pipe == 3   ? w_launch<128, 512, 4, true, 128, 64, 3>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 2 ? w_launch<128, 512, 4, true, 128, 64, 2>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                       : w_launch<128, 512, 4, true, 128, 64, 1>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else if (p[i].kind == 1)
      rc = mf16 ? w_launch<512, 128, 3, true>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                : w_launch<512, 128, 3, false>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else if (p[i].kind == 2)
      rc = mf16 ? w_launch<128, 512, 3, true>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                : w_launch<128, 512, 3, false>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else if (p[i].kind == 3)
      rc = pipe == 3   ? w_launch<256, 224, 4, true, 64, 112, 3>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 2 ? w_launch<256, 224, 4, true, 64, 112, 2>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 1 ? w_launch<256, 224, 4, true, 64, 112, 1>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                       : w_launch<256, 224, 4, true, 64, 112>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else if (p[i].kind == 4)
      rc = pipe == 3   ? w_launch<224, 256, 4, true, 112, 64, 3>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 2 ? w_launch<224, 256, 4, true, 112, 64, 2>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 1 ? w_launch<224, 256, 4, true, 112, 64, 1>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                       : w_launch<224, 256, 4, true, 112, 64>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else if (p[i].kind == 5)
      rc = pipe == 3   ? w_launch<128, 448, 4, true, 64, 112, 3>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 2 ? w_launch<128, 448, 4, true, 64, 112, 2>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 1 ? w_launch<128, 448, 4, true, 64, 112, 1>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                       : w_launch<128, 448, 3, true, 64, 112>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    else
      rc = pipe == 3   ? w_launch<448, 128, 4, true, 112, 64, 3>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 2 ? w_launch<448, 128, 4, true, 112, 64, 2>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
           : pipe == 1 ? w_launch<448, 128, 4, true, 112, 64, 1>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st)
                       : w_launch<448, 128, 3, true, 112, 64>(p[i], dy16, ldy, x16, ldx, K, ws, o16, N, st);
    if (rc != VA_OK) return rc;
    ws += w_part_bytes(p[i]) / static_cast<int64_t>(sizeof(float));
  }
  return check_launch("weight_grad");
}
