// Y [M, N] = X [M, K] . W [N, K]^T (+ b): F.linear's layout ("TN", both operands contiguous along K),
// bf16 in / out, fp32 accumulation, gfx950 MFMA. The backbone's forward projections and, over the
// transposed weight copy (kernels.input_grad), its input gradients — in the reference torch's
// nn.Linear under FSDP (dp_actor.py:331-333 forward, :465-470 backward; no reference kernel).
//
// Why an own kernel: the hidden size 896 (Qwen2.5-0.5B) is 3.5 x 256, so hipBLASLt's 256 x 256 macro
// tiles spend 12.5 % of their MFMA work on padding for every GEMM with 896 output columns (o and down
// forward, the q|k|v / o / gate|up input gradients), and 1,152 (q|k|v) is 4.5 x 256. Here the output
// tile is 256 tokens x WR features with WR = 32 I in {192, 224, 256, 288} chosen to divide N (896 =
// 4 x 224, 1,152 = 4 x 288).
//
// Core: 8 waves = 2 (feature halves of WR / 2 = I blocks of 16) x 4 (token quarters of 64 = 4 blocks),
// v_mfma_f32_16x16x32_bf16 with the weight rows as the MFMA rows, so a lane holds 4 consecutive output
// features of one token per block (one 8-byte store). Both operands stream through two LDS images per
// 64-deep K-step by LDS-DMA (buffer_load ... lds, 16 B per lane) whose 16-byte chunk c of row r sits at
// c ^ ((r >> 1) & 7) (swizzled on the global source address: conflict-free fragment reads), the next
// step's images issued between the current step's two K-halves. Persistent: a workgroup runs `per`
// consecutive tiles of the (token block, feature tile) list, feature tile fastest, staging the next
// tile's first K-step during the current tile's last (no prologue between tiles); workgroups b, b + 8,
// ... share an XCD and get contiguous runs of tiles (the token panels they share stay in its L2).
// Rows past M read 0 through the buffer resource's bound and are not stored.
//
// Bound: MFMA, 2 M N K flops per launch.

#include "va_common.h"

namespace va {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int G_TK = 64;      // K per step
constexpr int G_TM = 256;     // tokens per tile
constexpr int G_THREADS = 512;

__device__ __forceinline__ int g_img_off(int row, int c) { return row * G_TK + ((c ^ ((row >> 1) & 7)) << 3); }

// the kernel body as a device function (the buffer-resource type exists only in the device compilation;
// a __global__ body that names it is not instantiated for the host, whose launch stub then goes missing)
template <int I, bool BIAS, bool REMAP, bool LOCK>
__device__ __forceinline__ void linear_tn_body(const uint16_t *__restrict__ x, int64_t ldx,
                                               const uint16_t *__restrict__ w, int64_t ldw,
                                               const uint16_t *__restrict__ bias, int64_t M, int K, int64_t N,
                                               int per, uint16_t *__restrict__ y, int64_t ldy) {
  constexpr int WR = 32 * I;            // output features per tile
  constexpr int WIMG = WR * G_TK;       // bf16 elements of the weight image of one K-step
  constexpr int XIMG = G_TM * G_TK;     // ... of the token image
  constexpr int BUF = WIMG + XIMG;
  constexpr int WGRP = WR / 8;          // 8-row DMA groups of the weight image
  constexpr int NWS = (WGRP + 7) / 8;   // weight DMA slots per lane (the token image takes 4)
  // two staging buffers, then 1 KB that the weight slots without a group (WR % 64 != 0) write to
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BUF + 512];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int64_t n_nt = N / WR, n_mt = (M + G_TM - 1) / G_TM;
  int64_t L = blockIdx.x;
  if (REMAP) {
    const int64_t nl = gridDim.x >> 3;
    L = (L & 7) * nl + (L >> 3);
  }
  // this workgroup's tiles: LOCK, token blocks [r per, r per + per) of feature tile L % n_nt (the n_nt
  // workgroups of a token range run side by side on one XCD and read each token K-step from its L2 once);
  // else tiles [L per, L per + per) of the list (token block, feature tile), feature tile fastest
  int64_t mt, nt, ntiles;
  if (LOCK) {
    nt = L % n_nt;
    mt = (L / n_nt) * per;
    ntiles = n_mt - mt < per ? n_mt - mt : per;
  } else {
    const int64_t total = n_nt * n_mt, t0 = L * per;
    mt = t0 / n_nt, nt = t0 - mt * n_nt;
    ntiles = total - t0 < per ? total - t0 : per;
  }
  if (ntiles <= 0) return;
  const int nk = K / G_TK;
  const int64_t nsteps = ntiles * nk;

  // per-lane DMA sources (byte offsets within a tile's rows) and wave-uniform LDS destinations
  uint32_t xoff[4], woff[NWS];
  int xdst[4], wdst[NWS];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int g = s * 8 + wave;  // token rows g * 8 .. + 8
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    xoff[s] = static_cast<uint32_t>((row * ldx + lc * 8) * 2);
    xdst[s] = WIMG + g * 8 * G_TK;
  }
#pragma unroll
  for (int s = 0; s < NWS; ++s) {
    const int g = s * 8 + wave;
    const bool ok = g < WGRP;
    const int row = ok ? g * 8 + (lane >> 3) : (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    woff[s] = static_cast<uint32_t>((row * ldw + lc * 8) * 2);
    wdst[s] = ok ? g * 8 * G_TK : -1;
  }
  uint16_t *const idle = lds + 2 * BUF;

  // stage K-step kc of tile t into image pair img (branch-free: it shares a scheduling region with
  // the step's MFMAs)
  auto stage = [&](int64_t mt, int64_t nt, int kc, uint16_t *img) {
    const int64_t m0 = mt * G_TM;
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(x + m0 * ldx), 0, static_cast<int>(rows * ldx * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(w + nt * WR * ldw), 0, static_cast<int>(WR * ldw * 2), 0x00020000);
    const int kb = kc * G_TK * 2;
#pragma unroll
    for (int s = 0; s < NWS; ++s)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wres, wdst[s] >= 0 ? img + wdst[s] : idle, 16, woff[s], kb, 0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) __builtin_amdgcn_raw_ptr_buffer_load_lds(xres, img + xdst[s], 16, xoff[s], kb, 0, 0);
  };

  f32x4 acc[I][4];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // tile counters kept incrementally (a 64-bit division per step costs ~130 scalar instructions)
  int64_t t = 0;
  stage(mt, nt, 0, lds);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  int kt = 0;
  for (int64_t st = 0; st < nsteps; ++st) {
    const int buf = static_cast<int>(st & 1);
    const uint16_t *la = lds + buf * BUF;  // weight image
    const uint16_t *lb = la + WIMG;        // token image
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q == 1) {  // the next step's images; past the last tile, a valid tile re-staged, unread
        const bool adv = kt + 1 == nk && t + 1 < ntiles;
        const bool wrap = LOCK || nt + 1 == n_nt;
        stage(adv && wrap ? mt + 1 : mt, adv && !LOCK ? (wrap ? 0 : nt + 1) : nt, kt + 1 == nk ? 0 : kt + 1,
              lds + (buf ^ 1) * BUF);
      }
      const int c = q * 4 + (lane >> 4);
      bf16x8 fa[I], fb[4];
#pragma unroll
      for (int i = 0; i < I; ++i)
        fa[i] = *reinterpret_cast<const bf16x8 *>(la + g_img_off(wr * (WR / 2) + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8 *>(lb + g_img_off(wc * 64 + j * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt == nk - 1) {
      // epilogue: acc[i][j][e] = Y[token m0 + wc 64 + 16 j + (lane & 15)][feature n0 + wr WR/2 + 16 i + 4 (lane >> 4) + e]
      const int64_t fbase = nt * WR + wr * (WR / 2) + (lane >> 4) * 4;
      uint2 bb[I];
      if constexpr (BIAS) {
#pragma unroll
        for (int i = 0; i < I; ++i) bb[i] = *reinterpret_cast<const uint2 *>(bias + fbase + i * 16);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t tok = mt * G_TM + wc * 64 + j * 16 + (lane & 15);
        if (tok < M) {
          uint16_t *yr = y + tok * ldy + fbase;
#pragma unroll
          for (int i = 0; i < I; ++i) {
            float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
            if constexpr (BIAS) {  // F.linear's bias epilogue: bf16(acc + b)
              v0 += bf16_lo(bb[i].x), v1 += bf16_hi(bb[i].x), v2 += bf16_lo(bb[i].y), v3 += bf16_hi(bb[i].y);
            }
            *reinterpret_cast<uint2 *>(yr + i * 16) = make_uint2(pack2_bf16(v0, v1), pack2_bf16(v2, v3));
          }
        }
      }
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      kt = 0;
      ++t;
      if (LOCK) ++mt;
      else if (++nt == n_nt) nt = 0, ++mt;
    } else {
      ++kt;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// The pipelined form (VA_TUNE_LINEAR_TN = 2): 32-deep K-steps through a 4-stage LDS-DMA ring, the DMA of
// step st + 4 issued while step st computes (2 steps stay in flight across every barrier: counted
// vmcnt, raw s_barrier), and each wave's fragments of step st + 1 read from LDS between the MFMAs of
// step st (two register sets), the DMA pieces spread between them too — the schedule of the weight
// gradients' pipelined tiles (wgrad.hip PIPE 3) on F.linear's K-contiguous operands, whose fragments are
// plain ds_read_b128 of 8 consecutive K of one row. Image rows are 64 B (32 K); 16-byte chunk c of row r
// sits at c ^ ((r >> 2) & 2) (swizzled on the DMA source: conflict-free fragment reads). The tile order
// is LOCK's (one feature tile per workgroup, the workgroups of a token range side by side on one XCD)
// and the ring runs on across the workgroup's tiles; a tile's epilogue stores by buffer stores (rows
// past M dropped by the resource bound), a fixed count per lane that the next NST - 1 waits leave in
// flight behind the DMA pieces issued before them.
constexpr int P_TK = 32;

// chunk c of row r at c ^ ((r >> 2) & 2): conflict-free for ds_read_b128's four 16-lane groups
// ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32) over 16 rows x 4 chunks
__device__ __forceinline__ int p_swz(int row) { return (row >> 2) & 2; }
__device__ __forceinline__ int p_img_off(int row, int c) { return row * P_TK + ((c ^ p_swz(row)) << 3); }

template <int N>
__device__ __forceinline__ void p_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int NA, int NB>
struct PFrags {
  bf16x8 a[NA], b[NB];
};

// WC: token wave-columns — 4 (8 waves, two per SIMD, 64 tokens x I blocks each) or 2 (4 waves, one per
// SIMD, 128 tokens each: twice the MFMAs per fragment read and per barrier, the accumulators in AGPRs)
template <int I, int WC, int NST, bool BIAS>
__device__ __forceinline__ void linear_tn_pipe_body(const uint16_t *__restrict__ x, int64_t ldx,
                                                    const uint16_t *__restrict__ w, int64_t ldw,
                                                    const uint16_t *__restrict__ bias, int64_t M, int K, int64_t N,
                                                    int per, uint16_t *__restrict__ y, int64_t ldy) {
  constexpr int WR = 32 * I;                   // output features per tile
  constexpr int WIMG = WR * P_TK, XIMG = G_TM * P_TK;
  constexpr int BUF = WIMG + XIMG;             // bf16 elements of one ring stage
  constexpr int NW = 2 * WC, NT = 64 * NW;    // waves, threads
  constexpr int NB = 16 / WC;                  // token blocks per wave (256 tokens over WC columns)
  constexpr int WG16 = WR / 16;                // 16-row DMA groups of the weight image
  constexpr int NWS = (WG16 + NW - 1) / NW;    // weight pieces per wave and step
  constexpr int NXS = 16 / NW;                 // token pieces per wave and step
  constexpr int PER = NWS + NXS;               // LDS-DMA pieces per wave and step
  constexpr int S = I * NB;                    // epilogue stores per lane
  constexpr int NM = I * NB, NR = I + NB;      // MFMAs and fragment reads per wave and step
  constexpr int G = NM / (PER + 1);
  // the wait after an epilogue keeps its stores in flight (capped at the 6-bit count: waiting for a
  // few of them too is only slower)
  constexpr int VM_EPI = (NST - 2) * PER + S < 63 ? (NST - 2) * PER + S : 63;
  // the ring, 1 KB for the weight pieces without a group, then the tile's bias (WR bf16)
  __shared__ __attribute__((aligned(16))) uint16_t lds[NST * BUF + 512 + WR];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;

  const int64_t n_nt = N / WR, n_mt = (M + G_TM - 1) / G_TM;
  int64_t L = blockIdx.x;
  {
    const int64_t nl = gridDim.x >> 3;  // the host pads the grid to a multiple of 8 n_nt
    L = (L & 7) * nl + (L >> 3);
  }
  const int64_t nt = L % n_nt, mt0 = (L / n_nt) * per;
  const int64_t ntiles = n_mt - mt0 < per ? n_mt - mt0 : per;
  if (ntiles <= 0) return;
  const int nk = K / P_TK;  // >= NST (K >= 128)
  const int nsteps = static_cast<int>(ntiles) * nk;

  // DMA pieces: lane offsets within a 16-row group (row l >> 2, source chunk (l & 3) ^ swizzle)
  uint32_t xoff[NXS], woff[NWS];
  int xdst[NXS], wdst[NWS];
#pragma unroll
  for (int s2 = 0; s2 < NXS; ++s2) {
    const int g = s2 * NW + wave, row = g * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ p_swz(row);
    xoff[s2] = static_cast<uint32_t>((row * ldx + lc * 8) * 2);
    xdst[s2] = WIMG + g * 16 * P_TK;
  }
#pragma unroll
  for (int s2 = 0; s2 < NWS; ++s2) {
    const int g = s2 * NW + wave;
    const bool ok = g < WG16;
    const int row = (ok ? g * 16 : 0) + (lane >> 2);
    const int lc = (lane & 3) ^ p_swz(row);
    woff[s2] = static_cast<uint32_t>((row * ldw + lc * 8) * 2);
    wdst[s2] = ok ? g * 16 * P_TK : -1;
  }
  uint16_t *const idle = lds + NST * BUF;
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t *>(w + nt * WR * ldw), 0, static_cast<int>(WR * ldw * 2), 0x00020000);
  // step src (of this workgroup's nsteps) into ring buffer buf; branch-free
  auto issue_to = [&](int buf, int tl, int kc) {
    const int64_t m0 = (mt0 + tl) * G_TM;
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(x + m0 * ldx), 0, static_cast<int>(rows * ldx * 2), 0x00020000);
    uint16_t *img = lds + buf * BUF;
    const int kb = kc * P_TK * 2;
#pragma unroll
    for (int s2 = 0; s2 < NWS; ++s2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wres, wdst[s2] >= 0 ? img + wdst[s2] : idle, 16, woff[s2], kb, 0, 0);
#pragma unroll
    for (int s2 = 0; s2 < NXS; ++s2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xres, img + xdst[s2], 16, xoff[s2], kb, 0, 0);
  };
  auto read = [&](const uint16_t *img, PFrags<I, NB> &f) {
    const int c = lane >> 4;
#pragma unroll
    for (int i = 0; i < I; ++i)
      f.a[i] = *reinterpret_cast<const bf16x8 *>(img + p_img_off(wr * (WR / 2) + i * 16 + (lane & 15), c));
#pragma unroll
    for (int j = 0; j < NB; ++j)
      f.b[j] = *reinterpret_cast<const bf16x8 *>(img + WIMG + p_img_off(wc * 16 * NB + j * 16 + (lane & 15), c));
  };
  auto ready = [&](PFrags<I, NB> &f) {  // every LDS read of this wave retired; no MFMA above the wait
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f.a[0]));
#pragma unroll
    for (int i = 1; i < I; ++i) asm volatile("" : "+v"(f.a[i]));
#pragma unroll
    for (int j = 0; j < NB; ++j) asm volatile("" : "+v"(f.b[j]));
  };

  f32x4 acc[I][NB];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int64_t mt = mt0;  // the tile being accumulated
  int kt = 0;
  int st_epi = -NST;  // the last iteration that stored a tile
  int d_tl = NST / nk, d_kc = NST % nk;  // tile and K-step of the DMA source step st + NST
  // the epilogue: acc[i][j][e] = Y[token mt 256 + wc 64 + 16 j + (lane & 15)][feature fb + 16 i + e]
  const int fl = wr * (WR / 2) + (lane >> 4) * 4, fb = static_cast<int>(nt * WR) + fl;
  // the bias through LDS (an ordinary global load in the loop would make hipcc drain the DMA ring)
  const uint16_t *lbias = lds + NST * BUF + 512;
  if constexpr (BIAS) {
    for (int f = tid; f < WR; f += NT) lds[NST * BUF + 512 + f] = bias[nt * WR + f];
    __syncthreads();
  }
  auto epilogue = [&]() {
    const int64_t m0 = mt * G_TM;
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t yres = __builtin_amdgcn_make_buffer_rsrc(
        y + m0 * ldy, 0, static_cast<int>(rows * ldy * 2), 0x00020000);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int tok = wc * 16 * NB + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < I; ++i) {
        float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        if constexpr (BIAS) {  // F.linear's bias epilogue: bf16(acc + b)
          const uint2 bb = *reinterpret_cast<const uint2 *>(lbias + fl + i * 16);
          v0 += bf16_lo(bb.x), v1 += bf16_hi(bb.x), v2 += bf16_lo(bb.y), v3 += bf16_hi(bb.y);
        }
        typedef int v2i __attribute__((ext_vector_type(2)));
        const v2i q = {static_cast<int>(pack2_bf16(v0, v1)), static_cast<int>(pack2_bf16(v2, v3))};
        __builtin_amdgcn_raw_buffer_store_b64(q, yres, (tok * static_cast<int>(ldy) + fb + i * 16) * 2, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // iteration st: fragments of step st ready; publish step st + 1 (steps through st + NST - 1 issued,
  // NST - 2 of them stay in flight, plus a recent epilogue's stores issued after them), read its
  // fragments, MFMAs of step st with the DMA of step st + NST into step st's buffer between them
  auto body = [&](int st, PFrags<I, NB> &cur, PFrags<I, NB> &nxt) {
    ready(cur);
    const bool more = st + 1 < nsteps;
    const int buf = (more ? st : st + 1) % NST;
    // the source step st + NST from the incremental cursor (past the last step: the last step again)
    const bool in_range = st + NST < nsteps;
    const int tl = in_range ? d_tl : static_cast<int>(ntiles) - 1, kc = in_range ? d_kc : nk - 1;
    if (more) {
      if (st - st_epi < NST) p_vm_wait<VM_EPI>();
      else p_vm_wait<(NST - 2) * PER>();
      asm volatile("s_barrier" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    issue_to(buf, tl, kc);
    if (++d_kc == nk) d_kc = 0, ++d_tl;
    read(lds + ((st + 1) % NST) * BUF, nxt);
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.a[i], cur.b[j], acc[i][j], 0, 0, 0);
    int p = 0;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);               // one MFMA
      if (m < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one fragment read
      if (m % G == G - 1 && p < PER) {
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // one LDS-DMA piece
        ++p;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (++kt == nk) {
      epilogue();
      st_epi = st;
      kt = 0;
      ++mt;
    }
  };

  PFrags<I, NB> f0, f1;
  for (int b = 0; b < NST; ++b) {
    const int src = b < nsteps ? b : nsteps - 1;
    issue_to(b, src / nk, src % nk);
  }
  p_vm_wait<(NST - 1) * PER>();
  asm volatile("s_barrier" ::: "memory");
  read(lds, f0);
  int st = 0;
  for (; st + 1 < nsteps; st += 2) {
    body(st, f0, f1);
    body(st + 1, f1, f0);
  }
  if (st < nsteps) body(st, f0, f1);
  p_vm_wait<0>();  // no LDS-DMA outlives the workgroup's LDS
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// The ping-pong form (VA_TUNE_LINEAR_TN = 4): per 32-deep K-step each wave alternates an MFMA phase (the
// step's 28 MFMAs on fragments already in registers) and a load phase (the tile epilogue when one ends,
// the DMA of step st + NST into step st's ring buffer, the fragments of step st + 1 into the same
// registers, the waits that retire them and step st + 2's DMA), a barrier after each; waves 4-7 (the
// partners of waves 0-3 on the four SIMDs) run one barrier behind, so each SIMD's matrix pipe alternates
// between one wave's MFMA phase while its partner loads (cdna_hip_programming.md, the 8-phase template's
// stagger). Ordering, with the stagger: every wave retires DMA(st + 2) at the end of its load phase st,
// before the barrier that its partner group passes into load phase st + 1, which reads it; a ring buffer
// is re-filled in load phase st only after every wave's reads of it (load phase st - 1, retired by the
// lgkmcnt wait before that phase's closing barrier) — both groups' phases pair up so.
template <int I, int NST, bool BIAS, int PROBE = 0>
__device__ __forceinline__ void linear_tn_pp_body(const uint16_t *__restrict__ x, int64_t ldx,
                                                  const uint16_t *__restrict__ w, int64_t ldw,
                                                  const uint16_t *__restrict__ bias, int64_t M, int K, int64_t N,
                                                  int per, uint16_t *__restrict__ y, int64_t ldy) {
  constexpr int WR = 32 * I;
  constexpr int WIMG = WR * P_TK, XIMG = G_TM * P_TK;
  constexpr int BUF = WIMG + XIMG;
  constexpr int WG16 = WR / 16;
  constexpr int NWS = (WG16 + 7) / 8;
  constexpr int PER = NWS + 2;
  constexpr int S = I * 4;
  constexpr int VM = (NST - 2) * PER, VM_EPI = VM + S < 63 ? VM + S : 63;
  __shared__ __attribute__((aligned(16))) uint16_t lds[NST * BUF + 512 + WR];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int64_t n_nt = N / WR, n_mt = (M + G_TM - 1) / G_TM;
  int64_t L = blockIdx.x;
  {
    const int64_t nl = gridDim.x >> 3;
    L = (L & 7) * nl + (L >> 3);
  }
  const int64_t nt = L % n_nt, mt0 = (L / n_nt) * per;
  const int64_t ntiles = n_mt - mt0 < per ? n_mt - mt0 : per;
  if (ntiles <= 0) return;
  const int nk = K / P_TK;
  const int nsteps = static_cast<int>(ntiles) * nk;

  uint32_t xoff[2], woff[NWS];
  int xdst[2], wdst[NWS];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int g = s2 * 8 + wave, row = g * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ p_swz(row);
    xoff[s2] = static_cast<uint32_t>((row * ldx + lc * 8) * 2);
    xdst[s2] = WIMG + g * 16 * P_TK;
  }
#pragma unroll
  for (int s2 = 0; s2 < NWS; ++s2) {
    const int g = s2 * 8 + wave;
    const bool ok = g < WG16;
    const int row = (ok ? g * 16 : 0) + (lane >> 2);
    const int lc = (lane & 3) ^ p_swz(row);
    woff[s2] = static_cast<uint32_t>((row * ldw + lc * 8) * 2);
    wdst[s2] = ok ? g * 16 * P_TK : -1;
  }
  uint16_t *const idle = lds + NST * BUF;
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t *>(w + nt * WR * ldw), 0, static_cast<int>(WR * ldw * 2), 0x00020000);
  auto issue_to = [&](int buf, int tl, int kc) {
    if constexpr (PROBE == 1) return;  // (timing probe: no operand traffic)
    const int64_t m0 = (PROBE == 2 ? 0 : mt0 + tl) * G_TM;  // (probe 2: every workgroup one token block)
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(x + m0 * ldx), 0, static_cast<int>(rows * ldx * 2), 0x00020000);
    uint16_t *img = lds + buf * BUF;
    const int kb = kc * P_TK * 2;
#pragma unroll
    for (int s2 = 0; s2 < NWS; ++s2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wres, wdst[s2] >= 0 ? img + wdst[s2] : idle, 16, woff[s2], kb, 0, 0);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) __builtin_amdgcn_raw_ptr_buffer_load_lds(xres, img + xdst[s2], 16, xoff[s2], kb, 0, 0);
  };
  PFrags<I, 4> f;
  auto read = [&](const uint16_t *img) {
    const int c = lane >> 4;
#pragma unroll
    for (int i = 0; i < I; ++i)
      f.a[i] = *reinterpret_cast<const bf16x8 *>(img + p_img_off(wr * (WR / 2) + i * 16 + (lane & 15), c));
#pragma unroll
    for (int j = 0; j < 4; ++j)
      f.b[j] = *reinterpret_cast<const bf16x8 *>(img + WIMG + p_img_off(wc * 64 + j * 16 + (lane & 15), c));
  };
  auto ready = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f.a[0]));
#pragma unroll
    for (int i = 1; i < I; ++i) asm volatile("" : "+v"(f.a[i]));
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(f.b[j]));
  };

  f32x4 acc[I][4];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int64_t mt = mt0;
  int kt = 0;
  int st_epi = -NST;
  int d_tl = NST / nk, d_kc = NST % nk;
  const int fl = wr * (WR / 2) + (lane >> 4) * 4, fb = static_cast<int>(nt * WR) + fl;
  const uint16_t *lbias = lds + NST * BUF + 512;
  if constexpr (BIAS) {
    for (int q = tid; q < WR; q += G_THREADS) lds[NST * BUF + 512 + q] = bias[nt * WR + q];
    __syncthreads();
  }
  auto epilogue = [&]() {
    const int64_t m0 = mt * G_TM;
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t yres = __builtin_amdgcn_make_buffer_rsrc(
        y + m0 * ldy, 0, static_cast<int>(rows * ldy * 2), 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tok = wc * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < I; ++i) {
        float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        if constexpr (BIAS) {
          const uint2 bb = *reinterpret_cast<const uint2 *>(lbias + fl + i * 16);
          v0 += bf16_lo(bb.x), v1 += bf16_hi(bb.x), v2 += bf16_lo(bb.y), v3 += bf16_hi(bb.y);
        }
        typedef int v2i __attribute__((ext_vector_type(2)));
        const v2i q = {static_cast<int>(pack2_bf16(v0, v1)), static_cast<int>(pack2_bf16(v2, v3))};
        __builtin_amdgcn_raw_buffer_store_b64(q, yres, (tok * static_cast<int>(ldy) + fb + i * 16) * 2, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // prologue: steps 0 .. NST - 1 issued, step 0 (and step 1) retired, step 0's fragments in registers
  for (int b = 0; b < NST; ++b) {
    const int src = b < nsteps ? b : nsteps - 1;
    issue_to(b, src / nk, src % nk);
  }
  p_vm_wait<(NST - 2) * PER>();
  asm volatile("s_barrier" ::: "memory");
  read(lds);
  ready();
  if (wr == 1 && PROBE != 3) asm volatile("s_barrier" ::: "memory");  // the stagger: waves 4-7 one barrier behind
  for (int st = 0; st < nsteps; ++st) {
    // MFMA phase
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i], f.b[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    // load phase
    if (++kt == nk) {
      epilogue();
      st_epi = st;
      kt = 0;
      ++mt;
    }
    const bool in_range = st + NST < nsteps;
    issue_to(st % NST, in_range ? d_tl : static_cast<int>(ntiles) - 1, in_range ? d_kc : nk - 1);
    if (++d_kc == nk) d_kc = 0, ++d_tl;
    if (st + 1 < nsteps) read(lds + ((st + 1) % NST) * BUF);
    // retire DMA(st + 2): NST - 2 younger steps stay in flight (and a recent epilogue's stores, issued
    // between DMA(st + 2) and this step's DMA when st - st_epi <= NST - 3)
    if (st - st_epi <= NST - 3) p_vm_wait<VM_EPI>();
    else p_vm_wait<VM>();
    ready();
    asm volatile("s_barrier" ::: "memory");
  }
  if (wr == 0 && PROBE != 3) asm volatile("s_barrier" ::: "memory");  // the same barrier count for every wave
  p_vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// The ping-pong form over 64-deep K-steps (VA_TUNE_LINEAR_TN = 9): every DMA piece reads 8 rows x 128 B
// (whole cache lines: half the L1 -> L2 requests of the 32-deep steps' 64-B row pieces, whose texture-data
// path was the measured limit), the token operand through a 3-stage ring and the weight operand (read
// by the XCD's 8 workgroups of its feature tile in step, mostly L2 hits) through 2 stages: 152 KB of LDS
// for 224-wide tiles. Load phase st issues W(st + 2), then X(st + 3), then (a tile end) the epilogue's
// stores, reads step st + 1's fragments and retires W(st + 2) (and with it X(st + 2)) leaving X(st + 3)
// and the stores in flight.
constexpr int Q_TK = 64;

__device__ __forceinline__ int q_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int q_img_off(int row, int c) { return row * Q_TK + ((c ^ q_swz(row)) << 3); }

template <int I, bool BIAS>
__device__ __forceinline__ void linear_tn_pp64_body(const uint16_t *__restrict__ x, int64_t ldx,
                                                    const uint16_t *__restrict__ w, int64_t ldw,
                                                    const uint16_t *__restrict__ bias, int64_t M, int K, int64_t N,
                                                    int per, uint16_t *__restrict__ y, int64_t ldy) {
  constexpr int WR = 32 * I;
  constexpr int WIMG = WR * Q_TK, XIMG = G_TM * Q_TK;  // bf16 elements of one stage
  constexpr int NXB = 3, NWB = 2;                      // ring depths
  constexpr int XBASE = 0, WBASE = NXB * XIMG, IDLE = WBASE + NWB * WIMG, BIASO = IDLE + 512;
  constexpr int WG8 = WR / 8;                          // 8-row DMA groups of the weight image
  constexpr int NWS = (WG8 + 7) / 8, NXS = 4;          // pieces per wave and step
  constexpr int S = I * 4;
  constexpr int VM = NXS, VM_EPI = NXS + S < 63 ? NXS + S : 63;
  __shared__ __attribute__((aligned(16))) uint16_t lds[BIASO + WR];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int64_t n_nt = N / WR, n_mt = (M + G_TM - 1) / G_TM;
  int64_t L = blockIdx.x;
  {
    const int64_t nl = gridDim.x >> 3;
    L = (L & 7) * nl + (L >> 3);
  }
  const int64_t nt = L % n_nt, mt0 = (L / n_nt) * per;
  const int64_t ntiles = n_mt - mt0 < per ? n_mt - mt0 : per;
  if (ntiles <= 0) return;
  const int nk = K / Q_TK;
  const int nsteps = static_cast<int>(ntiles) * nk;

  uint32_t xoff[NXS], woff[NWS];
  int xdst[NXS], wdst[NWS];
#pragma unroll
  for (int s2 = 0; s2 < NXS; ++s2) {
    const int g = s2 * 8 + wave, row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ q_swz(row);
    xoff[s2] = static_cast<uint32_t>((row * ldx + lc * 8) * 2);
    xdst[s2] = g * 8 * Q_TK;
  }
#pragma unroll
  for (int s2 = 0; s2 < NWS; ++s2) {
    const int g = s2 * 8 + wave;
    const bool ok = g < WG8;
    const int row = (ok ? g * 8 : 0) + (lane >> 3);
    const int lc = (lane & 7) ^ q_swz(row);
    woff[s2] = static_cast<uint32_t>((row * ldw + lc * 8) * 2);
    wdst[s2] = ok ? g * 8 * Q_TK : -1;
  }
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t *>(w + nt * WR * ldw), 0, static_cast<int>(WR * ldw * 2), 0x00020000);
  auto issue_w = [&](int buf, int kc) {
    uint16_t *img = lds + WBASE + buf * WIMG;
    const int kb = kc * Q_TK * 2;
#pragma unroll
    for (int s2 = 0; s2 < NWS; ++s2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wres, wdst[s2] >= 0 ? img + wdst[s2] : lds + IDLE, 16, woff[s2], kb, 0,
                                               0);
  };
  auto issue_x = [&](int buf, int tl, int kc) {
    const int64_t m0 = (mt0 + tl) * G_TM;
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(x + m0 * ldx), 0, static_cast<int>(rows * ldx * 2), 0x00020000);
    uint16_t *img = lds + XBASE + buf * XIMG;
    const int kb = kc * Q_TK * 2;
#pragma unroll
    for (int s2 = 0; s2 < NXS; ++s2) __builtin_amdgcn_raw_ptr_buffer_load_lds(xres, img + xdst[s2], 16, xoff[s2], kb, 0, 0);
  };
  bf16x8 fa[2][I], fbb[2][4];
  auto read = [&](int step) {
    const uint16_t *iw = lds + WBASE + (step % NWB) * WIMG, *ix = lds + XBASE + (step % NXB) * XIMG;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = q * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < I; ++i)
        fa[q][i] = *reinterpret_cast<const bf16x8 *>(iw + q_img_off(wr * (WR / 2) + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fbb[q][j] = *reinterpret_cast<const bf16x8 *>(ix + q_img_off(wc * 64 + j * 16 + (lane & 15), c));
    }
  };
  auto ready = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[0][0]));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int i = 0; i < I; ++i) asm volatile("" : "+v"(fa[q][i]));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(fbb[q][j]));
    }
  };

  f32x4 acc[I][4];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int64_t mt = mt0;
  int kt = 0;
  int st_epi = -8;
  // DMA cursors: W(st + 2) (K-step only: the weight tile is the workgroup's for every tile) and
  // X(st + 3) (tile, K-step)
  int w_kc = 2 % nk, x_tl = 3 / nk, x_kc = 3 % nk;
  const int fl = wr * (WR / 2) + (lane >> 4) * 4, fb = static_cast<int>(nt * WR) + fl;
  if constexpr (BIAS) {
    for (int q = tid; q < WR; q += G_THREADS) lds[BIASO + q] = bias[nt * WR + q];
    __syncthreads();
  }
  auto epilogue = [&]() {
    const int64_t m0 = mt * G_TM;
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t yres = __builtin_amdgcn_make_buffer_rsrc(
        y + m0 * ldy, 0, static_cast<int>(rows * ldy * 2), 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tok = wc * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < I; ++i) {
        float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        if constexpr (BIAS) {
          const uint2 bb = *reinterpret_cast<const uint2 *>(lds + BIASO + fl + i * 16);
          v0 += bf16_lo(bb.x), v1 += bf16_hi(bb.x), v2 += bf16_lo(bb.y), v3 += bf16_hi(bb.y);
        }
        typedef int v2i __attribute__((ext_vector_type(2)));
        const v2i qv = {static_cast<int>(pack2_bf16(v0, v1)), static_cast<int>(pack2_bf16(v2, v3))};
        __builtin_amdgcn_raw_buffer_store_b64(qv, yres, (tok * static_cast<int>(ldy) + fb + i * 16) * 2, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto clampx = [&](int step, int &tl, int &kc) {  // step -> (tile, K-step); past the end: the last step
    const int st2 = step < nsteps ? step : nsteps - 1;
    tl = st2 / nk, kc = st2 % nk;
  };

  // prologue: W(0) X(0) W(1) X(1) X(2) issued; all but X(2) retired; step 0's fragments in registers
  {
    int tl, kc;
    issue_w(0, 0);
    clampx(0, tl, kc), issue_x(0, tl, kc);
    issue_w(1, 1 % nk);
    clampx(1, tl, kc), issue_x(1, tl, kc);
    clampx(2, tl, kc), issue_x(2, tl, kc);
  }
  p_vm_wait<NXS>();
  asm volatile("s_barrier" ::: "memory");
  read(0);
  ready();
  if (wr == 1) asm volatile("s_barrier" ::: "memory");  // the stagger
  for (int st = 0; st < nsteps; ++st) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[q][i], fbb[q][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    // load phase st
    const bool w_in = st + 2 < nsteps, x_in = st + 3 < nsteps;
    issue_w(st % NWB, w_in ? w_kc : nk - 1);
    if (++w_kc == nk) w_kc = 0;
    issue_x(st % NXB, x_in ? x_tl : static_cast<int>(ntiles) - 1, x_in ? x_kc : nk - 1);
    if (++x_kc == nk) x_kc = 0, ++x_tl;
    if (++kt == nk) {
      epilogue();
      st_epi = st;
      kt = 0;
      ++mt;
    }
    if (st + 1 < nsteps) read(st + 1);
    if (st_epi == st) p_vm_wait<VM_EPI>();
    else p_vm_wait<VM>();
    ready();
    asm volatile("s_barrier" ::: "memory");
  }
  if (wr == 0) asm volatile("s_barrier" ::: "memory");
  p_vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int I, bool BIAS>
__device__ __forceinline__ void linear_tn_pp64s_body(const uint16_t *__restrict__ x, int64_t ldx,
                                                    const uint16_t *__restrict__ w, int64_t ldw,
                                                    const uint16_t *__restrict__ bias, int64_t M, int K, int64_t N,
                                                    int per, uint16_t *__restrict__ y, int64_t ldy) {
  constexpr int WR = 32 * I;
  constexpr int WIMG = WR * Q_TK, XIMG = G_TM * Q_TK;  // bf16 elements of one stage
  constexpr int NXB = 3, NWB = 2;                      // ring depths
  constexpr int XBASE = 0, WBASE = NXB * XIMG, IDLE = WBASE + NWB * WIMG, BIASO = IDLE + 512;
  constexpr int WG8 = WR / 8;                          // 8-row DMA groups of the weight image
  constexpr int NWS = WG8 / 4, NXS = 8;                // pieces per loader wave and step
  static_assert(WG8 % 4 == 0, "whole weight groups per loader wave");
  constexpr int S = I * 4;
  __shared__ __attribute__((aligned(16))) uint16_t lds[BIASO + WR];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int64_t n_nt = N / WR, n_mt = (M + G_TM - 1) / G_TM;
  int64_t L = blockIdx.x;
  {
    const int64_t nl = gridDim.x >> 3;
    L = (L & 7) * nl + (L >> 3);
  }
  const int64_t nt = L % n_nt, mt0 = (L / n_nt) * per;
  const int64_t ntiles = n_mt - mt0 < per ? n_mt - mt0 : per;
  if (ntiles <= 0) return;
  const int nk = K / Q_TK;
  const int nsteps = static_cast<int>(ntiles) * nk;

  uint32_t xoff[NXS], woff[NWS];
  int xdst[NXS], wdst[NWS];
  const int lw = wave & 3;  // the wave's index among its group's four loaders
#pragma unroll
  for (int s2 = 0; s2 < NXS; ++s2) {
    const int g = s2 * 4 + lw, row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ q_swz(row);
    xoff[s2] = static_cast<uint32_t>((row * ldx + lc * 8) * 2);
    xdst[s2] = g * 8 * Q_TK;
  }
#pragma unroll
  for (int s2 = 0; s2 < NWS; ++s2) {
    const int g = s2 * 4 + lw;
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ q_swz(row);
    woff[s2] = static_cast<uint32_t>((row * ldw + lc * 8) * 2);
    wdst[s2] = g * 8 * Q_TK;
  }
  const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t *>(w + nt * WR * ldw), 0, static_cast<int>(WR * ldw * 2), 0x00020000);
  auto issue_w = [&](int buf, int kc) {
    uint16_t *img = lds + WBASE + buf * WIMG;
    const int kb = kc * Q_TK * 2;
#pragma unroll
    for (int s2 = 0; s2 < NWS; ++s2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wres, img + wdst[s2], 16, woff[s2], kb, 0, 0);
  };
  auto issue_x = [&](int buf, int tl, int kc) {
    const int64_t m0 = (mt0 + tl) * G_TM;
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(x + m0 * ldx), 0, static_cast<int>(rows * ldx * 2), 0x00020000);
    uint16_t *img = lds + XBASE + buf * XIMG;
    const int kb = kc * Q_TK * 2;
#pragma unroll
    for (int s2 = 0; s2 < NXS; ++s2) __builtin_amdgcn_raw_ptr_buffer_load_lds(xres, img + xdst[s2], 16, xoff[s2], kb, 0, 0);
  };
  bf16x8 fa[2][I], fbb[2][4];
  auto read = [&](int step) {
    const uint16_t *iw = lds + WBASE + (step % NWB) * WIMG, *ix = lds + XBASE + (step % NXB) * XIMG;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = q * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < I; ++i)
        fa[q][i] = *reinterpret_cast<const bf16x8 *>(iw + q_img_off(wr * (WR / 2) + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fbb[q][j] = *reinterpret_cast<const bf16x8 *>(ix + q_img_off(wc * 64 + j * 16 + (lane & 15), c));
    }
  };
  auto ready = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[0][0]));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int i = 0; i < I; ++i) asm volatile("" : "+v"(fa[q][i]));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(fbb[q][j]));
    }
  };

  f32x4 acc[I][4];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int64_t mt = mt0;
  int kt = 0;
  // DMA cursors: W(st + 2) (K-step only: the weight tile is the workgroup's for every tile) and
  // X(st + 3) (tile, K-step)
  int w_kc = 2 % nk, x_tl = 3 / nk, x_kc = 3 % nk;
  const int fl = wr * (WR / 2) + (lane >> 4) * 4, fb = static_cast<int>(nt * WR) + fl;
  if constexpr (BIAS) {
    for (int q = tid; q < WR; q += G_THREADS) lds[BIASO + q] = bias[nt * WR + q];
    __syncthreads();
  }
  auto epilogue = [&]() {
    const int64_t m0 = mt * G_TM;
    const int64_t rows = M - m0 < G_TM ? M - m0 : G_TM;
    const __amdgpu_buffer_rsrc_t yres = __builtin_amdgcn_make_buffer_rsrc(
        y + m0 * ldy, 0, static_cast<int>(rows * ldy * 2), 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tok = wc * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < I; ++i) {
        float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        if constexpr (BIAS) {
          const uint2 bb = *reinterpret_cast<const uint2 *>(lds + BIASO + fl + i * 16);
          v0 += bf16_lo(bb.x), v1 += bf16_hi(bb.x), v2 += bf16_lo(bb.y), v3 += bf16_hi(bb.y);
        }
        typedef int v2i __attribute__((ext_vector_type(2)));
        const v2i qv = {static_cast<int>(pack2_bf16(v0, v1)), static_cast<int>(pack2_bf16(v2, v3))};
        __builtin_amdgcn_raw_buffer_store_b64(qv, yres, (tok * static_cast<int>(ldy) + fb + i * 16) * 2, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto clampx = [&](int step, int &tl, int &kc) {  // step -> (tile, K-step); past the end: the last step
    const int st2 = step < nsteps ? step : nsteps - 1;
    tl = st2 / nk, kc = st2 % nk;
  };

  // prologue: the weight loaders (waves 4-7) issue W(0), W(1) and retire both; the token loaders (waves
  // 0-3) X(0), X(1), X(2) and retire all but X(2); step 0's fragments in registers
  const bool wload = wr == 1;
  if (wload) {
    issue_w(0, 0);
    issue_w(1, 1 % nk);
    p_vm_wait<0>();
  } else {
    int tl, kc;
    clampx(0, tl, kc), issue_x(0, tl, kc);
    clampx(1, tl, kc), issue_x(1, tl, kc);
    clampx(2, tl, kc), issue_x(2, tl, kc);
    p_vm_wait<NXS>();
  }
  asm volatile("s_barrier" ::: "memory");
  read(0);
  ready();
  if (wload) asm volatile("s_barrier" ::: "memory");  // the stagger
  for (int st = 0; st < nsteps; ++st) {
    __builtin_amdgcn_sched_barrier(0);
    // MFMA phase; a weight loader first issues W(st + 2) into step st's weight buffer, free since every
    // wave's load phase st - 1 (see above)
    if (wload) {
      issue_w(st % NWB, st + 2 < nsteps ? w_kc : nk - 1);
      if (++w_kc == nk) w_kc = 0;
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[q][i], fbb[q][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    // load phase st: a token loader issues X(st + 3); the epilogue at a tile's end; step st + 1's
    // fragments; then the token loaders retire X(st + 2) (X(st + 3) and the stores stay in flight), the
    // weight loaders W(st + 2) (the stores stay in flight)
    if (!wload) {
      const bool x_in = st + 3 < nsteps;
      issue_x(st % NXB, x_in ? x_tl : static_cast<int>(ntiles) - 1, x_in ? x_kc : nk - 1);
      if (++x_kc == nk) x_kc = 0, ++x_tl;
    }
    const bool epi = ++kt == nk;
    if (epi) {
      epilogue();
      kt = 0;
      ++mt;
    }
    if (st + 1 < nsteps) read(st + 1);
    if (wload) {
      if (epi) p_vm_wait<S>();
      else p_vm_wait<0>();
    } else {
      if (epi) p_vm_wait<NXS + S>();
      else p_vm_wait<NXS>();
    }
    ready();
    asm volatile("s_barrier" ::: "memory");
  }
  if (!wload) asm volatile("s_barrier" ::: "memory");
  p_vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int I, bool BIAS>
__global__ __launch_bounds__(G_THREADS, 1) void linear_tn_pp64s_kernel(const uint16_t *__restrict__ x, int64_t ldx,
                                                                       const uint16_t *__restrict__ w, int64_t ldw,
                                                                       const uint16_t *__restrict__ bias, int64_t M,
                                                                       int K, int64_t N, int per,
                                                                       uint16_t *__restrict__ y, int64_t ldy) {
  linear_tn_pp64s_body<I, BIAS>(x, ldx, w, ldw, bias, M, K, N, per, y, ldy);
}

template <int I, bool BIAS>
__global__ __launch_bounds__(G_THREADS, 1) void linear_tn_pp64_kernel(const uint16_t *__restrict__ x, int64_t ldx,
                                                                      const uint16_t *__restrict__ w, int64_t ldw,
                                                                      const uint16_t *__restrict__ bias, int64_t M,
                                                                      int K, int64_t N, int per,
                                                                      uint16_t *__restrict__ y, int64_t ldy) {
  linear_tn_pp64_body<I, BIAS>(x, ldx, w, ldw, bias, M, K, N, per, y, ldy);
}

template <int I, int NST, bool BIAS, int PROBE = 0>
__global__ __launch_bounds__(G_THREADS, 1) void linear_tn_pp_kernel(const uint16_t *__restrict__ x, int64_t ldx,
                                                                    const uint16_t *__restrict__ w, int64_t ldw,
                                                                    const uint16_t *__restrict__ bias, int64_t M, int K,
                                                                    int64_t N, int per, uint16_t *__restrict__ y,
                                                                    int64_t ldy) {
  linear_tn_pp_body<I, NST, BIAS, PROBE>(x, ldx, w, ldw, bias, M, K, N, per, y, ldy);
}

template <int I, int WC, int NST, bool BIAS>
__global__ __launch_bounds__(128 * WC, 1) void linear_tn_pipe_kernel(const uint16_t *__restrict__ x, int64_t ldx,
                                                                      const uint16_t *__restrict__ w, int64_t ldw,
                                                                      const uint16_t *__restrict__ bias, int64_t M,
                                                                      int K, int64_t N, int per,
                                                                      uint16_t *__restrict__ y, int64_t ldy) {
  linear_tn_pipe_body<I, WC, NST, BIAS>(x, ldx, w, ldw, bias, M, K, N, per, y, ldy);
}

template <int I, bool BIAS, bool REMAP, bool LOCK>
__global__ __launch_bounds__(G_THREADS, 1) void linear_tn_kernel(const uint16_t *__restrict__ x, int64_t ldx,
                                                                 const uint16_t *__restrict__ w, int64_t ldw,
                                                                 const uint16_t *__restrict__ bias, int64_t M, int K,
                                                                 int64_t N, int per, uint16_t *__restrict__ y,
                                                                 int64_t ldy) {
  linear_tn_body<I, BIAS, REMAP, LOCK>(x, ldx, w, ldw, bias, M, K, N, per, y, ldy);
}

// output feature tiles (I = tile / 32) in order of preference: the two-buffer form's, and the pipelined
// form's (its two fragment register sets fit the 192 / 224 wave tiles; 256 / 288 then run two-buffer)
constexpr int kTiles[] = {224, 288, 256, 192};
constexpr int kPipeTiles[] = {224, 192, 256, 288};

int pick_tile(int64_t N, bool pipe) {
  for (int t : pipe ? kPipeTiles : kTiles)
    if (N % t == 0) return t;
  return 0;
}

}  // namespace
}  // namespace va

using namespace va;

// va_set_tuning(VA_TUNE_LINEAR_TN): 4 = the ping-pong form; 2 / 3 = the pipelined form with a 4 / 5-stage
// ring; 1 / 0 = the two-buffer form in LOCK / list
// tile order (see linear_tn_body)
int g_linear_tn = 2;

template <int I, int NST>
static void launch_tn_pp(bool has_b, int64_t nwg, hipStream_t s, const uint16_t *x, int64_t ldx, const uint16_t *w,
                         int64_t ldw, const uint16_t *b, int64_t M, int64_t N, int64_t K, int per, uint16_t *y,
                         int64_t ldy) {
  const auto kern = has_b ? linear_tn_pp_kernel<I, NST, true> : linear_tn_pp_kernel<I, NST, false>;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(G_THREADS), 0, s, x, ldx, w, ldw, b, M,
                     static_cast<int>(K), N, per, y, ldy);
}

template <int I, int WC, int NST>
static void launch_tn_pipe(bool has_b, int64_t nwg, hipStream_t s, const uint16_t *x, int64_t ldx, const uint16_t *w,
                           int64_t ldw, const uint16_t *b, int64_t M, int64_t N, int64_t K, int per, uint16_t *y,
                           int64_t ldy) {
  const auto kern = has_b ? linear_tn_pipe_kernel<I, WC, NST, true> : linear_tn_pipe_kernel<I, WC, NST, false>;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(128 * WC), 0, s, x, ldx, w, ldw, b, M,
                     static_cast<int>(K), N, per, y, ldy);
}

template <int I, bool LOCK>
static void launch_tn(bool remap, bool has_b, int64_t nwg, hipStream_t s, const uint16_t *x, int64_t ldx,
                      const uint16_t *w, int64_t ldw, const uint16_t *b, int64_t M, int64_t N, int64_t K, int per,
                      uint16_t *y, int64_t ldy) {
  const auto kern = has_b ? (remap ? linear_tn_kernel<I, true, true, LOCK> : linear_tn_kernel<I, true, false, LOCK>)
                          : (remap ? linear_tn_kernel<I, false, true, LOCK> : linear_tn_kernel<I, false, false, LOCK>);
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(G_THREADS), 0, s, x, ldx, w, ldw, b, M,
                     static_cast<int>(K), N, per, y, ldy);
}

template <int I>
static void launch_tn(bool lock, bool remap, bool has_b, int64_t nwg, hipStream_t s, const uint16_t *x,
                      int64_t ldx, const uint16_t *w, int64_t ldw, const uint16_t *b, int64_t M, int64_t N, int64_t K,
                      int per, uint16_t *y, int64_t ldy) {
  if (lock) launch_tn<I, true>(remap, has_b, nwg, s, x, ldx, w, ldw, b, M, N, K, per, y, ldy);
  else launch_tn<I, false>(remap, has_b, nwg, s, x, ldx, w, ldw, b, M, N, K, per, y, ldy);
}

extern "C" int va_linear_tn_tile(int64_t N) { return pick_tile(N, g_linear_tn >= 2); }

extern "C" int va_linear_tn(const void *x, int64_t ldx, const void *w, int64_t ldw, const void *bias, int dtype,
                            int64_t M, int64_t N, int64_t K, int tile_n, int per, void *y, int64_t ldy,
                            void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "linear_tn: only bf16 is implemented");
  if (tile_n == 0) tile_n = pick_tile(N, g_linear_tn >= 2);
  VA_CHECK_ARG(tile_n == 192 || tile_n == 224 || tile_n == 256 || tile_n == 288,
               "linear_tn: no output tile of {192, 224, 256, 288} divides N=%lld", static_cast<long long>(N));
  VA_CHECK_ARG(M >= 0 && N > 0 && N % tile_n == 0 && K > 0 && K % G_TK == 0 && K <= (1 << 20),
               "linear_tn: need N %% %d == 0 and K %% 64 == 0 (N=%lld, K=%lld)", tile_n, static_cast<long long>(N),
               static_cast<long long>(K));
  VA_CHECK_ARG(ldx >= K && ldw >= K && ldx % 8 == 0 && ldw % 8 == 0 && ldx < (1 << 22) &&
                   static_cast<int64_t>(tile_n) * ldw * 2 < (int64_t{1} << 31) && ldy >= N && ldy % 4 == 0,
               "linear_tn: strides must be >= K (ldy >= N), %% 8 (ldy %% 4), < 2^22 / tile_n ldw 2 < 2^31 "
               "(32-bit buffer offsets)");
  VA_CHECK_ARG(per >= 0, "linear_tn: negative tiles per workgroup");
  if (M == 0) return VA_OK;
  VA_CHECK_ARG(x && w && y, "null pointer argument");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(w) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(y) % 8 == 0 && reinterpret_cast<uintptr_t>(bias) % 8 == 0,
               "linear_tn: 16-byte aligned x / w, 8-byte aligned y / bias required");
  const int64_t n_nt = N / tile_n, n_mt = (M + G_TM - 1) / G_TM;
  const bool lock = g_linear_tn >= 1 && n_nt <= 32;  // (wider outputs: list order, two-buffer form)
  // the pipelined form needs a K of at least its ring (4 / 5 steps of 32); shorter: the two-buffer form
  const bool pipe = g_linear_tn >= 2 && lock && K >= (g_linear_tn == 3 || g_linear_tn == 8 ? 5 : 4) * P_TK &&
                    (g_linear_tn < 9 || K >= 3 * Q_TK);  // (ping-pong: 4)
  // automatic: one round of the 256 CUs (one 512-thread workgroup per CU), tiles spread evenly; in LOCK
  // order whole groups of 8 token ranges (the grid is padded to multiples of 8 n_nt workgroups)
  if (per == 0) {
    per = static_cast<int>((n_nt * n_mt + 255) / 256);
    if (lock) {
      const int64_t groups = 256 / (8 * n_nt) * 8;
      const int64_t p2 = (n_mt + groups - 1) / groups;
      if (p2 > per) per = static_cast<int>(p2);
    }
  }
  int64_t nwg;
  bool remap;
  if (lock) {  // per = token blocks per workgroup; the n_nt workgroups of a range on one XCD
    nwg = (n_mt + per - 1) / per * n_nt;
    const int64_t q = 8 * n_nt;
    nwg = (nwg + q - 1) / q * q;  // padded (idle workgroups) so that no range straddles two XCDs
    remap = true;
  } else {
    nwg = (n_nt * n_mt + per - 1) / per;
    remap = nwg % 8 == 0;
  }
  VA_CHECK_ARG(nwg < (int64_t{1} << 31), "linear_tn: grid too large");
  const bool has_b = bias != nullptr;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const auto *x16 = static_cast<const uint16_t *>(x);
  const auto *w16 = static_cast<const uint16_t *>(w);
  const auto *b16 = static_cast<const uint16_t *>(bias);
  auto *y16 = static_cast<uint16_t *>(y);
  if (pipe && (tile_n == 192 || tile_n == 224)) {  // the two register sets fit these wave tiles only
    if (g_linear_tn == 10) {  // ping-pong, 64-deep steps, split loaders
      const auto kern = tile_n == 192 ? (has_b ? linear_tn_pp64s_kernel<6, true> : linear_tn_pp64s_kernel<6, false>)
                                      : (has_b ? linear_tn_pp64s_kernel<7, true> : linear_tn_pp64s_kernel<7, false>);
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(G_THREADS), 0, s, x16, ldx, w16, ldw, b16, M,
                         static_cast<int>(K), N, per, y16, ldy);
    } else if (g_linear_tn == 9) {  // ping-pong, 64-deep steps
      const auto kern = tile_n == 192 ? (has_b ? linear_tn_pp64_kernel<6, true> : linear_tn_pp64_kernel<6, false>)
                                      : (has_b ? linear_tn_pp64_kernel<7, true> : linear_tn_pp64_kernel<7, false>);
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(G_THREADS), 0, s, x16, ldx, w16, ldw, b16, M,
                         static_cast<int>(K), N, per, y16, ldy);
    } else if (g_linear_tn == 8) {  // ping-pong, 5-stage ring
      if (tile_n == 192) launch_tn_pp<6, 5>(has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy);
      else launch_tn_pp<7, 5>(has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy);
    } else if (g_linear_tn >= 5) {  // timing probes (wrong results): 5 no operand traffic, 6 one token block, 7 no stagger
      const int pr = g_linear_tn - 4;
      const auto kern = pr == 1 ? linear_tn_pp_kernel<7, 4, false, 1>
                                : (pr == 2 ? linear_tn_pp_kernel<7, 4, false, 2> : linear_tn_pp_kernel<7, 4, false, 3>);
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(G_THREADS), 0, s, x16, ldx, w16, ldw, b16, M,
                         static_cast<int>(K), N, per, y16, ldy);
    } else if (g_linear_tn == 4) {  // ping-pong
      if (tile_n == 192) launch_tn_pp<6, 4>(has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy);
      else launch_tn_pp<7, 4>(has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy);
    } else if (g_linear_tn == 3) {  // 5-stage ring
      if (tile_n == 192) launch_tn_pipe<6, 4, 5>(has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy);
      else launch_tn_pipe<7, 4, 5>(has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy);
    } else {
      if (tile_n == 192) launch_tn_pipe<6, 4, 4>(has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy);
      else launch_tn_pipe<7, 4, 4>(has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy);
    }
    return check_launch("linear_tn");
  }
  switch (tile_n) {
    case 192: launch_tn<6>(lock, remap, has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy); break;
    case 224: launch_tn<7>(lock, remap, has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy); break;
    case 256: launch_tn<8>(lock, remap, has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy); break;
    default: launch_tn<9>(lock, remap, has_b, nwg, s, x16, ldx, w16, ldw, b16, M, N, K, per, y16, ldy); break;
  }
  return check_launch("linear_tn");
}
