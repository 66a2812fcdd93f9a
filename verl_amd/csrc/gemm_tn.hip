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
// features of one token per block (one 8-byte store). Operands by LDS-DMA (buffer_load ... lds, 16 B per
// lane, 8 rows x 128 B per piece) into images whose 16-byte chunk c of row r sits at c ^ ((r >> 1) & 7)
// (swizzled on the global source address: conflict-free fragment reads). Persistent: each workgroup keeps
// one feature tile over a range of token blocks, the workgroups of one token range side by side on one
// XCD (each token K-step is read from HBM / the Infinity Cache once per XCD, then from its L2). Two forms:
// the two-buffer form below (the next step's images issued between the current step's two K-halves) and
// the ping-pong form further down (the default where it applies). Rows past M read 0 through the buffer
// resource's bound and are not stored.
//
// Measured against hipBLASLt at the bench's shapes (151,552 tokens, profiles/r06/z): 0.85-1.20 PF/s vs
// 0.96-1.30 — hipBLASLt's 256 x 256 tiles keep its MFMA pipe 78 % busy at a power-limited clock where
// these reach 55 %, more than the 12.5 % of padding the 224-wide tiles save — so the product keeps
// hipBLASLt for these GEMMs; the kernel stays as the measured alternative.
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
// retire all but N of this wave's vector-memory operations (LDS-DMA pieces and buffer stores, in issue order)
template <int N>
__device__ __forceinline__ void p_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// The ping-pong form (VA_TUNE_LINEAR_TN = 2, default for 192 / 224-wide tiles and K >= 192). Per 64-deep
// K-step each wave alternates an MFMA phase (the step's 56 MFMAs on fragments already in registers) and a
// load phase (DMA issue, a finished tile's epilogue, the next step's fragments, the waits that retire
// them), a barrier after each; waves 4-7 — the partners of waves 0-3 on the four SIMDs — run one barrier
// behind, so each SIMD's matrix pipe alternates between one wave's MFMA phase and the other's (the stagger
// of the 8-phase template, cdna_hip_programming.md). Every DMA piece reads 8 rows x 128 B, whole cache
// lines (32-deep steps' 64-B row pieces doubled the L1 -> L2 requests and were texture-data bound:
// profiles/r06/w-x); the token operand goes through a 3-stage ring (1 of the 4 workgroups sharing a token
// step misses L2), the weight operand (8 workgroups per XCD share it) through 2 stages: 152 KB of LDS at
// 224-wide tiles. Load phase st issues W(st + 2) into step st's weight buffer, then X(st + 3) into step
// st's token buffer, then a finished tile's stores (buffer stores: rows past M dropped by the resource
// bound), reads step st + 1's fragments, and retires W(st + 2) — with it X(st + 2) — leaving X(st + 3) and
// the stores in flight. Ordering under the stagger: the barrier that starts a wave's load phase st pairs
// with the one that ends its partner group's load phase st - 1, so (RAW) step st + 1, retired by every
// wave at the end of its load phase st - 1, is complete for both groups' reads in load phase st, and (WAR)
// step st's buffers, read in every wave's load phase st - 1, are free when load phase st refills them.
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
  constexpr int VM = NXS, VM_EPI = VM + S < 63 ? VM + S : 63;  // X(st + 3)'s pieces (+ the stores)
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
  int w_kc = NWB % nk, x_tl = NXB / nk, x_kc = NXB % nk;
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

  // prologue: W(0) X(0) W(1) X(1) X(2) issued, all but X(2) retired, step 0's fragments in registers
  {
    int tl, kc;
    auto xs = [&](int st2) { clampx(st2, tl, kc), issue_x(st2, tl, kc); };
    issue_w(0, 0), xs(0), issue_w(1, 1 % nk), xs(1), xs(2);
  }
  p_vm_wait<VM>();
  asm volatile("s_barrier" ::: "memory");
  read(0);
  ready();
  if (wr == 1) asm volatile("s_barrier" ::: "memory");  // the stagger
  for (int st = 0; st < nsteps; ++st) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[q][i], fbb[q][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    // load phase st: the shallow operand's step st + 2, then the deep one's step st + 3
    const bool w_in = st + NWB < nsteps, x_in = st + NXB < nsteps;
    auto dw = [&]() {
      issue_w(st % NWB, w_in ? w_kc : nk - 1);
      if (++w_kc == nk) w_kc = 0;
    };
    auto dx = [&]() {
      issue_x(st % NXB, x_in ? x_tl : static_cast<int>(ntiles) - 1, x_in ? x_kc : nk - 1);
      if (++x_kc == nk) x_kc = 0, ++x_tl;
    };
    dw(), dx();
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
__global__ __launch_bounds__(G_THREADS, 1) void linear_tn_pp64_kernel(const uint16_t *__restrict__ x, int64_t ldx,
                                                                      const uint16_t *__restrict__ w, int64_t ldw,
                                                                      const uint16_t *__restrict__ bias, int64_t M,
                                                                      int K, int64_t N, int per,
                                                                      uint16_t *__restrict__ y, int64_t ldy) {
  linear_tn_pp64_body<I, BIAS>(x, ldx, w, ldw, bias, M, K, N, per, y, ldy);
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

// va_set_tuning(VA_TUNE_LINEAR_TN): 2 = the ping-pong form; 1 / 0 = the two-buffer form in LOCK / list
// tile order (see linear_tn_body)
int g_linear_tn = 2;

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

extern "C" int va_linear_tn_tile(int64_t N) { return pick_tile(N, g_linear_tn == 2); }

extern "C" int va_linear_tn(const void *x, int64_t ldx, const void *w, int64_t ldw, const void *bias, int dtype,
                            int64_t M, int64_t N, int64_t K, int tile_n, int per, void *y, int64_t ldy,
                            void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "linear_tn: only bf16 is implemented");
  if (tile_n == 0) tile_n = pick_tile(N, g_linear_tn == 2);
  VA_CHECK_ARG(tile_n == 192 || tile_n == 224 || tile_n == 256 || tile_n == 288,
               "linear_tn: no output tile of {192, 224, 256, 288} divides N=%lld", static_cast<long long>(N));
  VA_CHECK_ARG(M >= 0 && N > 0 && N % tile_n == 0 && K > 0 && K % G_TK == 0 && K <= (1 << 20),
               "linear_tn: need N %% %d == 0 and K %% 64 == 0 (N=%lld, K=%lld)", tile_n, static_cast<long long>(N),
               static_cast<long long>(K));
  VA_CHECK_ARG(ldx >= K && ldw >= K && ldx % 8 == 0 && ldw % 8 == 0 && ldx < (1 << 22) &&
                   static_cast<int64_t>(tile_n) * ldw * 2 < (int64_t{1} << 31) && ldy >= N && ldy % 4 == 0 &&
                   ldy < (1 << 22),
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
  // the ping-pong form needs K >= 3 steps of 64 (its prologue fills the token ring); shorter: two-buffer
  const bool pipe = g_linear_tn == 2 && lock && K >= 3 * Q_TK;  // (ping-pong: 4)
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
  // its registers fit the 192-wide wave tiles and the 224-wide ones without a bias (with one: 9 spills)
  if (pipe && (tile_n == 192 || (tile_n == 224 && !has_b))) {
    const auto kern = tile_n == 192 ? (has_b ? linear_tn_pp64_kernel<6, true> : linear_tn_pp64_kernel<6, false>)
                                    : linear_tn_pp64_kernel<7, false>;
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(G_THREADS), 0, s, x16, ldx, w16, ldw, b16, M,
                       static_cast<int>(K), N, per, y16, ldy);
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
