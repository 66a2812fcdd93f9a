// Experimental bf16 NT GEMM core for f1 (fused lm_head + log-softmax): C[m][n] = sum_k A[m][k] B[n][k]
// with A = hidden [M, K] and B = lm_head weight [N, K], both K-contiguous. Development harness only
// (tools/f1core_bench.py drives it through ctypes); the product kernel lives in
// verl_amd/csrc/linear_logprob.hip once it passes.
//
// v1: 256 x 256 x 64 tile, 8 waves (2 M x 4 N, 128 x 64 per wave = 8 x 4 MFMA 16x16x32 blocks),
// both operands staged by LDS-DMA (global_load_lds 16 B per lane) into 2 buffers (128 KB), the
// 16-byte chunk of row r stored at chunk ^ ((r >> 1) & 7) (source-swizzled: the LDS image stays
// lane-linear) so a 16-lane ds_read_b128 fragment group hits 16 distinct slots.
// Epilogue for the bench: per (row, column tile) fp32 row sums (a checksum that keeps the MFMAs live),
// or the full fp32 C for small correctness runs.

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kThreads = 512;
constexpr int kTileElems = BM * BK;  // one operand's K-step image (bf16 elements)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// element offset of (row, logical 16-byte chunk c) in a [rows][64] bf16 image
__device__ __forceinline__ int img_off(int row, int c) { return row * BK + ((c ^ ((row >> 1) & 7)) << 3); }

// Stage one K-step of one operand: 256 rows x 64 k. Wave w moves row groups g = 4 w .. 4 w + 3 of
// 8 rows (1 KB each). Lane l writes LDS bytes [16 l, 16 l + 16) of the group = row 8 g + l / 8,
// physical chunk l % 8, so it loads logical chunk (l % 8) ^ ((row >> 1) & 7) from global memory.
__device__ __forceinline__ void stage(const uint16_t *__restrict__ src, int64_t row0, int64_t nrows, int ld,
                                      int k0, uint16_t *img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int g = wave * 4 + i;
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    int64_t gr = row0 + row;
    if (gr >= nrows) gr = nrows - 1;  // clamped rows are computed and discarded
    const uint16_t *p = src + gr * ld + k0 + lc * 8;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(p), img + g * 8 * BK, 16, 0, 0);
  }
}

__global__ __launch_bounds__(kThreads, 1) void gemm_nt_v1(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                        int64_t M, int64_t N, int K, float *__restrict__ rowsum,
                                                        float *__restrict__ Cdbg) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * kTileElems];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  // XCD-aware tile order: blocks b and b + 8 share an XCD; give each XCD a contiguous run of tile
  // ids, walked in groups of 8 row tiles (tiles in flight on one XCD share A / B panels)
  const int64_t tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int64_t nt = tiles_m * tiles_n;
  const int64_t b = blockIdx.x;
  const int64_t q = nt / 8, r = nt % 8, x = b % 8;
  const int64_t t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
  constexpr int64_t GM = 8;
  const int64_t group = t / (GM * tiles_n), first_m = group * GM;
  const int64_t gsz = tiles_m - first_m < GM ? tiles_m - first_m : GM;
  const int64_t tm = first_m + (t % (GM * tiles_n)) % gsz, tn = (t % (GM * tiles_n)) / gsz;
  const int64_t m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage(A, m0, M, K, 0, lds, wave, lane);
  stage(B, n0, N, K, 0, lds + kTileElems, wave, lane);
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const uint16_t *la = lds + buf * 2 * kTileElems;
    const uint16_t *lb = la + kTileElems;
    if (kt + 1 < nk) {
      uint16_t *na = lds + (buf ^ 1) * 2 * kTileElems;
      stage(A, m0, M, K, (kt + 1) * BK, na, wave, lane);
      stage(B, n0, N, K, (kt + 1) * BK, na + kTileElems, wave, lane);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = s * 4 + (lane >> 4);
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        fa[i] = *reinterpret_cast<const bf16x8 *>(la + img_off(wr * 128 + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8 *>(lb + img_off(wc * 64 + j * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // epilogue: acc[i][j][e] = C[m0 + wr*128 + i*16 + (lane>>4)*4 + e][n0 + wc*64 + j*16 + (lane&15)]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t row = m0 + wr * 128 + i * 16 + (lane >> 4) * 4 + e;
      float srow = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wc * 64 + j * 16 + (lane & 15);
        const float v = col < N ? acc[i][j][e] : 0.f;
        srow += v;
        if (Cdbg != nullptr && row < M && col < N) Cdbg[row * N + col] = v;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) srow += __shfl_xor(srow, o, 64);
      if ((lane & 15) == 0 && row < M) rowsum[(tn * 4 + wc) * M + row] = srow;
    }
}


// v2: the same tile as 8 phases per 2 K-tiles... organised per K-tile as 4 phases, one C quadrant
// (128 x 128, A half qm x B half qn) per phase in the order (0,0) (0,1) (1,0) (1,1); all 8 waves
// work on the quadrant (wave (wr, wc): rows 64 wr, cols 32 wc of it = 4 x 2 MFMA blocks x 2 k-halves
// = 16 MFMAs). Each half-tile (128 rows x 64 k, 16 KB) has its own LDS slot per buffer; a phase
// issues ONE half-tile of DMA (2 x 16 B per thread) for a K-tile 1-2 ahead, into a half whose last
// ds_read was in an earlier phase:
//   phase 1: A1 of K-tile t+1 (its buffer's A1 was last read in phase 3 of K-tile t-1)
//   phase 2: A0 of K-tile t+2 (buffer of t: A0 last read in phase 1)
//   phase 3: B0 of K-tile t+2 (last read in phase 1)
//   phase 4: B1 of K-tile t+2 (last read in phase 2)
// and phase 4 waits vmcnt(6) (the 3 half-tiles just issued stay in flight) before its first
// barrier, which retires every half of K-tile t+1. Raw s_barrier only (a __syncthreads would drain
// the DMA queue); fragments: phase 1 reads A(qm 0) + B(qn 0), phase 2 B(qn 1), phase 3 A(qm 1).
constexpr int kHalf = 128 * BK;  // bf16 elements of one half-tile image

__device__ __forceinline__ void stage_half(const uint16_t *__restrict__ src, int64_t row0, int64_t nrows, int ld,
                                           int k0, uint16_t *img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = wave * 2 + i;  // 16 groups of 8 rows
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    int64_t gr = row0 + row;
    if (gr >= nrows) gr = nrows - 1;
    const uint16_t *p = src + gr * ld + k0 + lc * 8;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(p), img + g * 8 * BK, 16, 0, 0);
  }
}

// half slot h (0 A0, 1 A1, 2 B0, 3 B1) of buffer b
__device__ __forceinline__ uint16_t *half_img(uint16_t *lds, int b, int h) { return lds + (b * 4 + h) * kHalf; }

__global__ __launch_bounds__(kThreads, 1) void gemm_nt_v2(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                        int64_t M, int64_t N, int K, float *__restrict__ rowsum,
                                                        float *__restrict__ Cdbg) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 4 * kHalf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int64_t tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int64_t nt = tiles_m * tiles_n;
  const int64_t b = blockIdx.x;
  const int64_t q = nt / 8, r = nt % 8, x = b % 8;
  const int64_t t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
  constexpr int64_t GM = 8;
  const int64_t group = t / (GM * tiles_n), first_m = group * GM;
  const int64_t gsz = tiles_m - first_m < GM ? tiles_m - first_m : GM;
  const int64_t tm = first_m + (t % (GM * tiles_n)) % gsz, tn = (t % (GM * tiles_n)) / gsz;
  const int64_t m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  auto issue = [&](int kt, int h) {  // half h of K-tile kt into its buffer
    uint16_t *img = half_img(lds, kt & 1, h);
    if (h < 2) stage_half(A, m0 + h * 128, M, K, kt * BK, img, wave, lane);
    else stage_half(B, n0 + (h - 2) * 128, N, K, kt * BK, img, wave, lane);
  };
  // prologue: all of K-tile 0, and A0 / B0 / B1 of K-tile 1 (its A1 comes in phase 1)
  issue(0, 0), issue(0, 1), issue(0, 2), issue(0, 3);
  if (nk > 1) {
    issue(1, 0), issue(1, 2), issue(1, 3);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  bf16x8 fa[4][2], fb[2][2][2];  // A frags of the current qm; B frags of both qn
  auto read_a = [&](const uint16_t *img) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fa[i][s] = *reinterpret_cast<const bf16x8 *>(img + img_off(wr * 64 + i * 16 + (lane & 15), s * 4 + (lane >> 4)));
  };
  auto read_b = [&](const uint16_t *img, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fb[qn][j][s] =
            *reinterpret_cast<const bf16x8 *>(img + img_off(wc * 32 + j * 16 + (lane & 15), s * 4 + (lane >> 4)));
  };
  auto mfma = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm][qn][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[qn][j][s], acc[qm][qn][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // phase 1: quadrant (0, 0)
    read_a(half_img(lds, cur, 0));
    read_b(half_img(lds, cur, 2), 0);
    if (kt + 1 < nk) issue(kt + 1, 1);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma(0, 0);
    __builtin_amdgcn_s_barrier();
    // phase 2: quadrant (0, 1)
    read_b(half_img(lds, cur, 3), 1);
    if (kt + 2 < nk) issue(kt + 2, 0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma(0, 1);
    __builtin_amdgcn_s_barrier();
    // phase 3: quadrant (1, 0)
    read_a(half_img(lds, cur, 1));
    if (kt + 2 < nk) issue(kt + 2, 2);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma(1, 0);
    __builtin_amdgcn_s_barrier();
    // phase 4: quadrant (1, 1); K-tile kt + 1 must be complete after this phase's first barrier
    if (kt + 2 < nk) {
      issue(kt + 2, 3);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    mfma(1, 1);
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: acc[qm][qn][i][j][e] = C[m0 + qm*128 + wr*64 + i*16 + (lane>>4)*4 + e][n0 + qn*128 + wc*32 + j*16 + (lane&15)]
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = m0 + qm * 128 + wr * 64 + i * 16 + (lane >> 4) * 4 + e;
        float srow = 0.f;
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int64_t col = n0 + qn * 128 + wc * 32 + j * 16 + (lane & 15);
            const float v = col < N ? acc[qm][qn][i][j][e] : 0.f;
            srow += v;
            if (Cdbg != nullptr && row < M && col < N) Cdbg[row * N + col] = v;
          }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) srow += __shfl_xor(srow, o, 64);
        if ((lane & 15) == 0 && row < M) rowsum[(tn * 4 + wc) * M + row] = srow;
      }
}


// v3: v1 made persistent over a run of column tiles (grid = row tiles x splits, as the fused
// kernel runs): the next tile's first K-step is staged during the current tile's last one, so the
// pipeline does not drain between tiles; the row-sum epilogue runs per tile.
__global__ __launch_bounds__(kThreads, 1) void gemm_nt_v3(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                        int64_t M, int64_t N, int K, int tiles_per_split,
                                                        float *__restrict__ rowsum) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * kTileElems];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int64_t tiles_n = (N + BN - 1) / BN;
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * BM;
  const int64_t tn_begin = static_cast<int64_t>(blockIdx.y) * tiles_per_split;
  int64_t tn_end = tn_begin + tiles_per_split;
  if (tn_end > tiles_n) tn_end = tiles_n;
  if (tn_begin >= tn_end) return;
  const int nk = K / BK;
  const int64_t nsteps = (tn_end - tn_begin) * nk;  // (tile, k-step) pairs in order

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(A, m0, M, K, 0, lds, wave, lane);
  stage(B, tn_begin * BN, N, K, 0, lds + kTileElems, wave, lane);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int64_t st = 0; st < nsteps; ++st) {
    const int buf = static_cast<int>(st & 1);
    const int kt = static_cast<int>(st % nk);
    const int64_t tn = tn_begin + st / nk;
    const uint16_t *la = lds + buf * 2 * kTileElems;
    const uint16_t *lb = la + kTileElems;
    if (st + 1 < nsteps) {
      const int nkt = static_cast<int>((st + 1) % nk);
      const int64_t ntn = tn_begin + (st + 1) / nk;
      uint16_t *na = lds + (buf ^ 1) * 2 * kTileElems;
      stage(A, m0, M, K, nkt * BK, na, wave, lane);
      stage(B, ntn * BN, N, K, nkt * BK, na + kTileElems, wave, lane);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = s * 4 + (lane >> 4);
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        fa[i] = *reinterpret_cast<const bf16x8 *>(la + img_off(wr * 128 + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8 *>(lb + img_off(wc * 64 + j * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt == nk - 1) {  // tile done: row sums, then reset the accumulators (the next stage is in flight)
      const int64_t n0 = tn * BN;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t row = m0 + wr * 128 + i * 16 + (lane >> 4) * 4 + e;
          float srow = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t col = n0 + wc * 64 + j * 16 + (lane & 15);
            srow += col < N ? acc[i][j][e] : 0.f;
          }
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) srow += __shfl_xor(srow, o, 64);
          if ((lane & 15) == 0 && row < M) rowsum[(tn * 4 + wc) * M + row] = srow;
        }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
}

// v5: 256 x 128 tile, 3 LDS stages of 48 KB (A 256 x 64 + B 128 x 64), 8 waves as 4 (M) x 2 (N)
// of 64 x 64 (4 x 4 MFMA blocks); stage kt + 2 is issued before stage kt's MFMAs and stays in
// flight across the barrier: vmcnt(6) (the 6 DMA per thread of the newest stage) + raw s_barrier.
constexpr int kBN5 = 128;
__global__ __launch_bounds__(kThreads, 1) void gemm_nt_v5(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                        int64_t M, int64_t N, int K, float *__restrict__ rowsum,
                                                        float *__restrict__ Cdbg) {
  constexpr int kStage = BM * BK + kBN5 * BK;
  __shared__ __attribute__((aligned(16))) uint16_t lds[3 * kStage];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t tiles_m = (M + BM - 1) / BM, tiles_n = (N + kBN5 - 1) / kBN5;
  const int64_t nt = tiles_m * tiles_n;
  const int64_t b = blockIdx.x;
  const int64_t q = nt / 8, r = nt % 8, x = b % 8;
  const int64_t t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
  constexpr int64_t GM = 8;
  const int64_t group = t / (GM * tiles_n), first_m = group * GM;
  const int64_t gsz = tiles_m - first_m < GM ? tiles_m - first_m : GM;
  const int64_t tm = first_m + (t % (GM * tiles_n)) % gsz, tn = (t % (GM * tiles_n)) / gsz;
  const int64_t m0 = tm * BM, n0 = tn * kBN5;
  auto issue = [&](int kt) {
    uint16_t *img = lds + (kt % 3) * kStage;
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // A: 32 groups of 8 rows, 4 per wave
      const int g = wave * 4 + i;
      const int row = g * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ ((row >> 1) & 7);
      int64_t gr = m0 + row;
      if (gr >= M) gr = M - 1;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(A + gr * K + kt * BK + lc * 8), img + g * 8 * BK,
                                       16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // B: 16 groups, 2 per wave
      const int g = wave * 2 + i;
      const int row = g * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ ((row >> 1) & 7);
      int64_t gr = n0 + row;
      if (gr >= N) gr = N - 1;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(B + gr * K + kt * BK + lc * 8),
                                       img + BM * BK + g * 8 * BK, 16, 0, 0);
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / BK;
  issue(0);
  if (nk > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) issue(kt + 2);
    const uint16_t *la = lds + (kt % 3) * kStage;
    const uint16_t *lb = la + BM * BK;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = s * 4 + (lane >> 4);
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = *reinterpret_cast<const bf16x8 *>(la + img_off(wr * 64 + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8 *>(lb + img_off(wc * 64 + j * 16 + (lane & 15), c));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t row = m0 + wr * 64 + i * 16 + (lane >> 4) * 4 + e;
      float srow = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wc * 64 + j * 16 + (lane & 15);
        const float v = col < N ? acc[i][j][e] : 0.f;
        srow += v;
        if (Cdbg != nullptr && row < M && col < N) Cdbg[row * N + col] = v;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) srow += __shfl_xor(srow, o, 64);
      // 2 column halves of 64 per 128-wide tile: slots (tn * 2 + wc) of a [tiles * 4][M] buffer
      if ((lane & 15) == 0 && row < M) rowsum[(tn * 2 + wc) * M + row] = srow;
    }
}


// v6: persistent over a run of column tiles (as v3) with the quadrant phases of v2, but ONE barrier
// per phase and a 2-K-step prefetch distance. Per K-step g (of the (tile, k) sequence), phase s:
//   reads (issued first, retired by lgkmcnt(0) BEFORE the barrier, so after it every wave's reads of
//   this phase are done): s1 A0 + B0 frags, s2 B1, s3 A1, s4 none
//   s4 only: vmcnt(8) before the barrier -> every half of step g+1 has landed (the 4 halves of step
//   g+2 issued in s1..s3 stay in flight)
//   raw s_barrier
//   DMA into the halves this phase just finished reading, for step g+2: s1 A0 + B0, s2 B1, s3 A1
//   16 MFMAs of quadrant s: (0,0) (0,1) (1,0) (1,1)
// A frags of qm live across s1-s2 / s3-s4, B frags of both qn across the step.
__global__ __launch_bounds__(kThreads, 1) void gemm_nt_v6(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                        int64_t M, int64_t N, int K, int tiles_per_split,
                                                        float *__restrict__ rowsum) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 4 * kHalf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int64_t tiles_n = (N + BN - 1) / BN;
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * BM;
  const int64_t tn_begin = static_cast<int64_t>(blockIdx.y) * tiles_per_split;
  int64_t tn_end = tn_begin + tiles_per_split;
  if (tn_end > tiles_n) tn_end = tiles_n;
  if (tn_begin >= tn_end) return;
  const int nk = K / BK;
  const int64_t nsteps = (tn_end - tn_begin) * nk;

  auto issue = [&](int64_t g, int h) {  // half h of step g into buffer g & 1
    uint16_t *img = half_img(lds, static_cast<int>(g & 1), h);
    const int kt = static_cast<int>(g % nk);
    const int64_t tn = tn_begin + g / nk;
    if (h < 2) stage_half(A, m0 + h * 128, M, K, kt * BK, img, wave, lane);
    else stage_half(B, tn * BN + (h - 2) * 128, N, K, kt * BK, img, wave, lane);
  };
  f32x4 acc[2][2][4][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  bf16x8 fa[4][2], fb[2][2][2];
  auto read_a = [&](const uint16_t *img) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fa[i][s] = *reinterpret_cast<const bf16x8 *>(img + img_off(wr * 64 + i * 16 + (lane & 15), s * 4 + (lane >> 4)));
  };
  auto read_b = [&](const uint16_t *img, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fb[qn][j][s] =
            *reinterpret_cast<const bf16x8 *>(img + img_off(wc * 32 + j * 16 + (lane & 15), s * 4 + (lane >> 4)));
  };
  auto mfma = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm][qn][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[qn][j][s], acc[qm][qn][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: steps 0 and 1 in full; wait for step 0
  issue(0, 0), issue(0, 2), issue(0, 3), issue(0, 1);
  if (nsteps > 1) {
    issue(1, 0), issue(1, 2), issue(1, 3), issue(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  for (int64_t g = 0; g < nsteps; ++g) {
    const int cur = static_cast<int>(g & 1);
    const bool pre = g + 2 < nsteps;
    // s1: quadrant (0, 0)
    read_a(half_img(lds, cur, 0));
    read_b(half_img(lds, cur, 2), 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (pre) issue(g + 2, 0), issue(g + 2, 2);
    mfma(0, 0);
    // s2: quadrant (0, 1)
    read_b(half_img(lds, cur, 3), 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (pre) issue(g + 2, 3);
    mfma(0, 1);
    // s3: quadrant (1, 0)
    read_a(half_img(lds, cur, 1));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (pre) issue(g + 2, 1);
    mfma(1, 0);
    // s4: quadrant (1, 1); step g + 1 must have landed before this barrier
    if (pre) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfma(1, 1);
    if (g % nk == nk - 1) {  // tile done
      const int64_t n0 = (tn_begin + g / nk) * BN;
      const int64_t tn = tn_begin + g / nk;
#pragma unroll
      for (int qm = 0; qm < 2; ++qm)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t row = m0 + qm * 128 + wr * 64 + i * 16 + (lane >> 4) * 4 + e;
            float srow = 0.f;
#pragma unroll
            for (int qn = 0; qn < 2; ++qn)
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const int64_t col = n0 + qn * 128 + wc * 32 + j * 16 + (lane & 15);
                srow += col < N ? acc[qm][qn][i][j][e] : 0.f;
              }
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) srow += __shfl_xor(srow, o, 64);
            if ((lane & 15) == 0 && row < M) rowsum[(tn * 4 + wc) * M + row] = srow;
          }
      zero_acc();
    }
  }
}

}  // namespace

extern "C" int f1core_gemm_nt(int variant, const void *A, const void *B, int64_t M, int64_t N, int K, float *rowsum,
                              float *Cdbg, void *stream) {
  if (K % BK != 0) return -1;
  const int64_t nt = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (variant) {
    case 1:
      hipLaunchKernelGGL(gemm_nt_v1, dim3(static_cast<unsigned>(nt)), dim3(kThreads), 0, s,
                         static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), M, N, K, rowsum, Cdbg);
      break;
    case 2:
      hipLaunchKernelGGL(gemm_nt_v2, dim3(static_cast<unsigned>(nt)), dim3(kThreads), 0, s,
                         static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), M, N, K, rowsum, Cdbg);
      break;
    case 3: {
      const int64_t tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
      int splits = static_cast<int>((1024 + tm - 1) / tm);  // ~4 workgroups per CU
      if (splits > tn) splits = static_cast<int>(tn);
      if (splits < 1) splits = 1;
      const int per = static_cast<int>((tn + splits - 1) / splits);
      splits = static_cast<int>((tn + per - 1) / per);
      hipLaunchKernelGGL(gemm_nt_v3, dim3(static_cast<unsigned>(tm), static_cast<unsigned>(splits)), dim3(kThreads), 0,
                         s, static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), M, N, K, per, rowsum);
      break;
    }
    case 6: {
      const int64_t tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
      int splits = static_cast<int>((1024 + tm - 1) / tm);
      if (splits > tn) splits = static_cast<int>(tn);
      if (splits < 1) splits = 1;
      const int per = static_cast<int>((tn + splits - 1) / splits);
      splits = static_cast<int>((tn + per - 1) / per);
      hipLaunchKernelGGL(gemm_nt_v6, dim3(static_cast<unsigned>(tm), static_cast<unsigned>(splits)), dim3(kThreads), 0,
                         s, static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), M, N, K, per, rowsum);
      break;
    }
    case 5: {
      const int64_t nt5 = ((M + BM - 1) / BM) * ((N + kBN5 - 1) / kBN5);
      hipLaunchKernelGGL(gemm_nt_v5, dim3(static_cast<unsigned>(nt5)), dim3(kThreads), 0, s,
                         static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), M, N, K, rowsum, Cdbg);
      break;
    }
    default:
      return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
