// Causal variable-length flash attention forward for the packed actor backbone (gfx950, bf16,
// head dim 64, GQA). Not a §8 row: it replaces PyTorch-ROCm's AOTriton varlen forward
// (~165 TFLOP/s at D=64) inside the actor's model forward; the backward stays
// aten::_flash_attention_backward, fed with this kernel's O and LSE (same conventions).
//
// Layout: q [T, Hq, 64], k / v [T, Hk, 64] packed tokens (cu_seqlens), o like q, lse [B, Hq, max_len]
// fp32 natural-log sum-exp of the scaled scores (the padded layout aten's varlen flash uses). Work unit = one 128-row query block of one
// sequence x one query head (host-built block table, heaviest blocks first); 4 waves x 32 rows.
//
// Per wave and 64-key block = two 32-key tiles (v_mfma_f32_32x32x16_bf16 throughout):
//   S^T = K Q^T      4 MFMAs; the query sits on the lane, so the softmax row (the tile's keys)
//                    is 16 registers of this lane + the partner lane l^32: no LDS, 1 shuffle
//   online softmax   base-2 over the block's 64 keys, causal / sequence-end mask on the diagonal
//                    blocks only, O rescaled only when the row max moved
//   O^T += V^T P^T   4 MFMAs; P^T is the S^T accumulator converted to bf16 in place (k order
//                    permuted, guide §3), V^T fragments by ds_read_b64_tr_b16 in the same order;
//                    O^T keeps the query on the lane, so the rescale by exp2(m_old - m_new) and
//                    the final 1 / l are lane-local.
// K / V blocks of 64 keys are staged through double-buffered LDS shared by the 4 waves: by LDS-DMA
// (DMA = true, the default: global_load_lds issued at the top of a block for the next one, retired
// by the block's closing barrier) or through registers (the next block's rows are in VGPRs during
// the current block's MFMAs). K rows are XOR-swizzled for the row-fragment reads (through the
// per-lane source address under DMA); V rows are plain for the transposed reads.

#include <math.h>

#include "va_common.h"

namespace va {
namespace {

constexpr int D = 64;
constexpr int QB = 128;  // query rows per workgroup
constexpr int KB = 64;   // keys per staged block
constexpr float kLog2e_ = 1.4426950408889634f;
constexpr float kLn2_ = 0.69314718055994531f;
constexpr float kDeferLog2 = 8.f;  // forward: defer the O rescale until the max grows by 2^8
#ifndef VA_FLASH_FWD_DMA_OCC
#define VA_FLASH_FWD_DMA_OCC 2  // waves per SIMD the LDS-DMA forward is compiled for
#endif
#ifndef VA_FLASH_DKDV_DMA_OCC
#define VA_FLASH_DKDV_DMA_OCC 2  // the same for the LDS-DMA dK / dV backward
#endif
#ifndef VA_FLASH_DQ_DMA_OCC
#define VA_FLASH_DQ_DMA_OCC 2  // the same for the LDS-DMA dQ backward
#endif

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
// v_cvt_pk_bf16_f32 (round to nearest even), the hardware conversion
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v{a, b}, bf16x2v));
}

// row (key / query index inside a 32 x 32 tile) held in register r by lane half h
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// KBF = keys per staged block (64 or 128): 128 halves the barriers (but measures slower: the
// default is 64); each 64-key sub-block runs the same online-softmax step as a 64-key block
template <int KBF, bool DMA>
__global__ __launch_bounds__(256, DMA ? VA_FLASH_FWD_DMA_OCC : 2) void flash_fwd_kernel(
    const uint16_t *__restrict__ q, const uint16_t *__restrict__ k, const uint16_t *__restrict__ v,
    const int32_t *__restrict__ cu, const int32_t *__restrict__ blocks, int64_t lse_ld, int Hq, int Hk,
    float scale, uint16_t *__restrict__ o, float *__restrict__ lse) {
  static_assert(KBF == 64 || KBF == 128, "KBF");
  static_assert(!DMA || KBF == 64, "DMA staging: 64-key blocks");
  constexpr int NCF = KBF * 8 / 256;  // 16-B chunks per thread per operand
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * KBF * D];  // [buf][K | V][KBF keys][64 d]
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, ql = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
  const int seq = blocks[2 * blockIdx.x], qs = blocks[2 * blockIdx.x + 1];
  const int head = blockIdx.y, kvh = head / (Hq / Hk);
  const int s0 = cu[seq], len = cu[seq + 1] - s0;
  const int q_pos = qs + wave * 32 + ql;  // this lane's query (position inside the sequence)
  const bool q_ok = q_pos < len;
  const int64_t ldq = static_cast<int64_t>(Hq) * D, ldk = static_cast<int64_t>(Hk) * D;
  const float c = scale * kLog2e_;

  // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[q][16 s + 8 h + j]
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (q_ok) qf[s] = *reinterpret_cast<const bf16x8 *>(q + (s0 + q_pos) * ldq + head * D + 16 * s + 8 * h);
    else qf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x16 oacc[2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[dh][r] = 0.f;
  float m = -INFINITY, l = 0.f;

  const int kv_end = min(len, qs + QB);  // causal: keys <= the block's last query
  const int nkb = (kv_end + KBF - 1) / KBF;
  const int wave_last_q = qs + wave * 32 + 31;

  // staging: KBF rows x 8 chunks of 16 B per operand, NCF per thread per operand
  uint4 sk[DMA ? 1 : NCF], sv[DMA ? 1 : NCF];
  auto load_block = [&](int kb) {
#pragma unroll
    for (int u = 0; u < NCF; ++u) {
      const int idx = tid + u * 256, r = idx >> 3, ch = idx & 7;
      const int key = kb * KBF + r;
      const bool ok = key < len;
      const int64_t base = (s0 + (ok ? key : len - 1)) * ldk + kvh * D + ch * 8;  // clamped: no branch
      const uint4 a = *reinterpret_cast<const uint4 *>(k + base);
      const uint4 b = *reinterpret_cast<const uint4 *>(v + base);
      sk[u] = ok ? a : make_uint4(0, 0, 0, 0);
      sv[u] = ok ? b : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_block = [&](int buf) {
    uint16_t *lk = lds + buf * 2 * KBF * D;
    uint16_t *lv = lk + KBF * D;
#pragma unroll
    for (int u = 0; u < NCF; ++u) {
      const int idx = tid + u * 256, r = idx >> 3, ch = idx & 7;
      *reinterpret_cast<uint4 *>(lk + r * D + ((ch ^ (r & 7)) << 3)) = sk[u];
      *reinterpret_cast<uint4 *>(lv + r * D + (ch << 3)) = sv[u];
    }
  };

  // DMA: the block's K / V rows go global -> LDS by LDS-DMA (16 B per lane, one 1-KiB piece = 8 rows
  // per wave-instruction, K chunks swizzled through the source address), no staging registers;
  // rows past the sequence end are clamped (their scores are masked, their P is 0)
  auto dma_block = [&](int kb, int buf) {
    uint16_t *lk = lds + buf * 2 * KBF * D;
    uint16_t *lv = lk + KBF * D;
#pragma unroll
    for (int pi = wave; pi < KBF / 8; pi += 4) {
      const int r = pi * 8 + (lane >> 3), p = lane & 7;
      const int key = kb * KBF + r;
      const int64_t base = (s0 + (key < len ? key : len - 1)) * ldk + kvh * D;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(k + base + ((p ^ (r & 7)) << 3)),
                                       lk + pi * 8 * D, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(v + base + (p << 3)), lv + pi * 8 * D, 16, 0,
                                       0);
    }
  };

  if (nkb > 0) {
    if constexpr (DMA) {
      dma_block(0, 0);
    } else {
      load_block(0);
      store_block(0);
    }
  }
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) {
      if constexpr (DMA) dma_block(kb + 1, (kb + 1) & 1);
      else load_block(kb + 1);
    }
#pragma unroll
    for (int sub = 0; sub < KBF / KB; ++sub) {
    const uint16_t *lk = lds + (kb & 1) * 2 * KBF * D + sub * KB * D;
    const uint16_t *lv = lds + (kb & 1) * 2 * KBF * D + KBF * D + sub * KB * D;
    const int key0 = kb * KBF + sub * KB;
    // the whole 64-key sub-block is past this wave's queries (or the wave has none): skip
    if (!(key0 > wave_last_q || qs + wave * 32 >= len || key0 >= kv_end)) {
      const bool t1_live = key0 + 32 <= wave_last_q && key0 + 32 < len;  // second 32-key tile
      // ---- S^T = K Q^T for the block's two 32-key tiles (keys on rows, queries on lanes)
      // both tiles always: a dead second tile (its keys past every query of the wave or past the
      // sequence) costs 4 MFMAs on the few blocks that have one, and need_mask then holds and masks
      // all of its scores to -inf by select below; skipping it instead cost 16 v_mov per block (its
      // registers cleared for the skip path) in this VALU-bound loop (round 6)
      f32x16 sacc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] = 0.f;
        const int krow = t * 32 + ql;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ch = 2 * s + h;
          const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(lk + krow * D + ((ch ^ (krow & 7)) << 3));
          sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[t], 0, 0, 0);
        }
      }
      // ---- online softmax over the block (base 2); masks only on diagonal / sequence-end blocks.
      // The running max m is kept on the RAW scores (c > 0), p = exp2(fma(S, c, -m c)) is one FMA
      // + one exp per score, and O / l are rescaled only when the max grows by more than
      // kDeferLog2 / c (p <= 2^kDeferLog2 meanwhile; l and O see the same factor: exact). Cross-lane
      // work is kept off the steady state (round 5: 547-549 vs 565 us per 151,819-token micro-batch,
      // profiles/r05/attn_fwd_shuffle_skip_ab.jsonl): the row max over both lanes of a query is
      // exchanged only when some lane's own half passes the bound, and each lane sums its half of the
      // row sum, the halves added once at the end.
      const bool need_mask = (key0 + KB - 1 > qs + wave * 32) || (key0 + KB - 1 >= len);
      float x[32];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) x[16 * t + r] = sacc[t][r];
      if (need_mask) {  // wave-uniform: one scalar branch; key offset vs. a per-lane limit
        const int lim = min(q_pos, len - 1) - key0 - 4 * h;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            x[16 * t + r] = (t * 32 + crow(r, 0) > lim) ? -INFINITY : x[16 * t + r];
      }
      float tm0 = x[0], tm1 = x[1];  // two independent max chains
#pragma unroll
      for (int r = 2; r < 32; r += 2) {
        tm0 = fmaxf(tm0, x[r]);
        tm1 = fmaxf(tm1, x[r + 1]);
      }
      float tm = fmaxf(tm0, tm1);
      // the rescale decision needs the max over both halves of the row (this lane and lane ^ 32),
      // but only when some lane's own half passes the bound: the exchange is skipped otherwise
      if (__builtin_amdgcn_ballot_w64(tm > m + kDeferLog2 / c) != 0) {  // wave-uniform
        tm = fmaxf(tm, __shfl_xor(tm, 32, kWave));
        if (tm > m + kDeferLog2 / c) {  // per-lane; O / l rescaled only on these rows
          const float alpha = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m - tm) * c);
          l *= alpha;
#pragma unroll
          for (int dh = 0; dh < 2; ++dh)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[dh][r] *= alpha;
          m = tm;
        }
      }
      const float nmc = m == -INFINITY ? 0.f : -m * c;
      float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
      for (int r = 0; r < 32; r += 2) {
        x[r] = __builtin_amdgcn_exp2f(fmaf(x[r], c, nmc));
        x[r + 1] = __builtin_amdgcn_exp2f(fmaf(x[r + 1], c, nmc));
        rs0 += x[r];
        rs1 += x[r + 1];
      }
      l += rs0 + rs1;  // this lane's half of the row sum (the halves are added once, at the end)
      // ---- O^T += V^T P^T over 4 k-steps of 16 keys; P^T = S^T registers 8s..8s+7 as bf16
      //      (k order permuted, guide §3); V^T fragment element j <-> key 16 s + 8 (j >> 2) + 4 h + (j & 3)
      const int g16 = lane >> 4, li = lane & 15;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (t == 1 && !t1_live) continue;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const float *xs = x + 16 * t + 8 * s;
          const bf16x8 pf = __builtin_bit_cast(
              bf16x8, make_uint4(pk_bf16(xs[0], xs[1]), pk_bf16(xs[2], xs[3]), pk_bf16(xs[4], xs[5]),
                                 pk_bf16(xs[6], xs[7])));
          const int r0 = t * 32 + 16 * s + 4 * h + (li >> 2);
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) {
            const int col = dh * 32 + 16 * (g16 & 1) + 4 * (li & 3);
            const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s *)(lv + r0 * D + col));
            const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s *)(lv + (r0 + 8) * D + col));
            const bf16x8 vf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            oacc[dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, oacc[dh], 0, 0, 0);
          }
        }
      }
    }
    }  // sub
    // the other buffer was last read in iteration kb - 1, which every wave finished before the
    // barrier that ended it: store, then one barrier publishes the block for iteration kb + 1
    if constexpr (!DMA) {
      if (kb + 1 < nkb) store_block((kb + 1) & 1);
    }
    __syncthreads();  // (DMA: its vmcnt(0) retires this wave's pieces of block kb + 1 first)
  }

  // ---- epilogue: O = O^T / l, lane holds O[q][32 dh + crow(r, h)]; lse in natural log
  l += __shfl_xor(l, 32, kWave);  // the two lanes of a query hold the two halves of its row sum
  if (q_ok) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t *orow = o + (s0 + q_pos) * ldq + head * D;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // registers 4g..4g+3 are d = 32 dh + 8 g + 4 h + 0..3
        const uint32_t w0 = pk_bf16(oacc[dh][4 * g + 0] * inv, oacc[dh][4 * g + 1] * inv);
        const uint32_t w1 = pk_bf16(oacc[dh][4 * g + 2] * inv, oacc[dh][4 * g + 3] * inv);
        *reinterpret_cast<uint2 *>(orow + dh * 32 + 8 * g + 4 * h) = make_uint2(w0, w1);
      }
    if (h == 0)
      lse[(static_cast<int64_t>(seq) * Hq + head) * lse_ld + q_pos] = (m * c + __builtin_amdgcn_logf(l)) * kLn2_;
  }
}

// =====================================================================================
// Backward. dS = P * (dP - delta), delta = rowsum(dO * O); P recomputed from Q, K and the
// forward's LSE. Two or three launches, no atomics (dQ, dK, dV are each written once: deterministic):
//   flash_bwd_dq      workgroup = 128 queries x one query head (the forward's block table); wave =
//                     32 queries with Q, dO fragments in registers; computes its queries' delta from
//                     O and dO first (stored in the LSE layout for the next launch), then per 32-key
//                     tile  S^T = K Q^T, dP^T = V dO^T (query on the lane), dQ^T += K^T dS^T
//   flash_bwd_dkdv    workgroup = 128 keys x one KV head (GROUPED: sweeps the query tiles of all the
//                     group's query heads, dK / dV summed in registers, bf16 out) or x one query head
//                     (fp32 partials, when key blocks alone would not fill the chip); wave = 32 keys
//                     whose K, V fragments stay in registers. It sweeps the 32-row query tiles at or
//                     after its keys (Q, dO, LSE, delta staged in double-buffered LDS):
//                       S = Q K^T, dP = dO V^T  with the KEY on the lane (4 MFMAs each), so
//                       P and dS are already the B operands of
//                       dV^T += dO^T P,  dK^T += Q^T dS  (A = transposed reads of the Q / dO images)
//   flash_bwd_group_sum  (per-query-head variant only) dK, dV = fixed-order sum of the fp32
//                     partials over the GQA group
// LDS images are [rows][64] bf16 with 16-B chunk c of row r at c ^ (r & 7): conflict-light row
// reads (ds_read_b128) and per-lane swizzled addresses for the transposed reads.

__device__ __forceinline__ int swz(int row, int d) { return row * D + ((((d >> 3) ^ (row & 7))) << 3) + (d & 7); }

// A operand (32 rows of d x 16 k) from a [k][64] image by transposed reads: element j of lane
// (d = dh*32 + lane&31, half h) = image[16 s + 8 (j >> 2) + 4 h + (j & 3) + rbase][d]
__device__ __forceinline__ bf16x8 tr_frag(const uint16_t *img, int rbase, int s, int dh, int lane) {
  const int h = lane >> 5, g16 = lane >> 4, li = lane & 15;
  const int r0 = rbase + 16 * s + 4 * h + (li >> 2);
  const int col = dh * 32 + 16 * (g16 & 1) + 4 * (li & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)(img + swz(r0, col)));
  const v4s hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)(img + swz(r0 + 8, col)));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ bf16x8 pack_frag(const float *x) {
  return __builtin_bit_cast(bf16x8, make_uint4(pk_bf16(x[0], x[1]), pk_bf16(x[2], x[3]), pk_bf16(x[4], x[5]),
                                               pk_bf16(x[6], x[7])));
}

// GROUPED = false: blockIdx.y = query head, fp32 partial dK / dV per query head (summed by
// flash_bwd_group_sum); GROUPED = true: blockIdx.y = KV head, the workgroup sweeps the query tiles of
// all G query heads of its group in order (head-major) with dK / dV accumulated in registers, and
// writes bf16 dK / dV directly (no partials, no group-sum launch; used when the key blocks alone fill
// the chip).
// QT = query rows per staged tile (32 or 64): the 64-row tile halves the barriers per MFMA; the
// tile's 32-row halves run the same body (a 32-row offset keeps the images' XOR swizzle)
template <bool GROUPED, int QT, bool DMA>
__global__ __launch_bounds__(256, DMA ? VA_FLASH_DKDV_DMA_OCC : 2) void flash_bwd_dkdv_kernel(
    const uint16_t *__restrict__ q, const uint16_t *__restrict__ k, const uint16_t *__restrict__ v,
    const uint16_t *__restrict__ dout, const float *__restrict__ lse, const float *__restrict__ delta,
    const int32_t *__restrict__ cu, const int32_t *__restrict__ kblocks, int64_t ld, int64_t T, int Hq, int Hk,
    float scale, float *__restrict__ pdk, float *__restrict__ pdv, uint16_t *__restrict__ dk_out,
    uint16_t *__restrict__ dv_out) {
  static_assert(QT == 32 || QT == 64 || QT == 128, "QT");
  constexpr int NCH = QT * 8 / 256;  // 16-B chunks per thread per image
  // [buf][Q image QTx64 | dO image QTx64] bf16, then [buf][lse2 QT | delta QT] fp32
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * QT * D + 2 * 2 * QT * 2];
  float *rowc = reinterpret_cast<float *>(lds + 2 * 2 * QT * D);
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, kl = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
  const int seq = kblocks[2 * blockIdx.x], kb0 = kblocks[2 * blockIdx.x + 1];
  const int G = Hq / Hk;
  const int hq0 = GROUPED ? blockIdx.y * G : blockIdx.y;  // (first) query head
  const int g = GROUPED ? blockIdx.y : hq0 / G;
  const int s0 = cu[seq], len = cu[seq + 1] - s0;
  const int64_t ldq = static_cast<int64_t>(Hq) * D, ldk = static_cast<int64_t>(Hk) * D;
  const float c = scale * kLog2e_;
  const int k0 = kb0 + wave * 32;  // this wave's first key
  const int key = k0 + kl;         // this lane's key
  // K^T / V^T fragments (B operands with the key on the lane): lane holds K[key][16 s + 8 h + j]
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (key < len) {
      kf[s] = *reinterpret_cast<const bf16x8 *>(k + (s0 + key) * ldk + g * D + 16 * s + 8 * h);
      vf[s] = *reinterpret_cast<const bf16x8 *>(v + (s0 + key) * ldk + g * D + 16 * s + 8 * h);
    } else {
      kf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      vf[s] = kf[s];
    }
  }
  f32x16 dkt[2], dvt[2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dkt[dh][r] = 0.f;
      dvt[dh][r] = 0.f;
    }
  // iteration space: query tiles from the block's first key to the end of the sequence
  const int qfirst = (kb0 / QT) * QT;
  const int n_qt = len > qfirst ? (len - qfirst + QT - 1) / QT : 0;
  const int n_it = GROUPED ? n_qt * G : n_qt;  // grouped: head-major over the group's query heads
  // staging: one 16-B chunk of the Q tile and one of the dO tile per thread; lse2 / delta by 64 threads
  struct StageQ {
    uint4 q[DMA ? 1 : NCH], d[DMA ? 1 : NCH];
    float rc;
    bool live;
  };
  auto load_it = [&](int it) -> StageQ {
    StageQ st;
    const int hj = GROUPED ? it / n_qt : 0;
    const int hq = hq0 + hj, qt0 = qfirst + (it - hj * n_qt) * QT;
    if constexpr (DMA) {
      // the row constants first, one unconditional (clamped) load per thread: hipcc waits for it
      // only where store_it consumes it, and, issued before the DMA below, that wait leaves the DMA
      // in flight (a conditional load made hipcc drain everything at the top of the iteration)
      const int rr = tid & (QT - 1), qq = qt0 + rr;
      const int64_t idx = (static_cast<int64_t>(seq) * Hq + hq) * ld + (qq < len ? qq : len - 1);
      st.rc = (tid & QT) ? delta[idx] : lse[idx];  // tid < QT: lse, QT <= tid < 2 QT: delta
      st.live = qq < len;
      // Q / dO images by LDS-DMA into buffer it & 1 (the buffer read two iterations ago: every wave
      // passed the barrier that ended that iteration); rows past the sequence end clamped (p = 0)
      uint16_t *img = lds + (it & 1) * 2 * QT * D;
#pragma unroll
      for (int pi = wave; pi < QT / 8; pi += 4) {
        const int r = pi * 8 + (lane >> 3), pch = (lane & 7) ^ (r & 7), qp = qt0 + r;
        const int64_t base = (s0 + (qp < len ? qp : len - 1)) * ldq + hq * D + (pch << 3);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(q + base), img + pi * 8 * D, 16, 0, 0);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(dout + base), img + QT * D + pi * 8 * D, 16,
                                         0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < (DMA ? 0 : NCH); ++u) {
      const int idx = tid + u * 256, r = idx >> 3, ch = idx & 7, qp = qt0 + r;
      const bool ok = qp < len;
      const int64_t base = (s0 + (ok ? qp : len - 1)) * ldq + hq * D + ch * 8;  // clamped: no branch
      const uint4 a = *reinterpret_cast<const uint4 *>(q + base);
      const uint4 b = *reinterpret_cast<const uint4 *>(dout + base);
      st.q[u] = ok ? a : make_uint4(0, 0, 0, 0);
      st.d[u] = ok ? b : make_uint4(0, 0, 0, 0);
    }
    if constexpr (!DMA) {
      st.rc = 0.f;
      if (tid < 2 * QT) {
        const int rr = tid & (QT - 1), qq = qt0 + rr;
        const int64_t idx = (static_cast<int64_t>(seq) * Hq + hq) * ld + qq;
        if (qq < len) st.rc = tid < QT ? lse[idx] * kLog2e_ : delta[idx];
      }
    }
    return st;
  };
  auto store_it = [&](int buf, const StageQ &st) {
    uint16_t *img = lds + buf * 2 * QT * D;
#pragma unroll
    for (int u = 0; u < (DMA ? 0 : NCH); ++u) {
      const int idx = tid + u * 256, r = idx >> 3, ch = idx & 7;
      *reinterpret_cast<uint4 *>(img + swz(r, ch * 8)) = st.q[u];
      *reinterpret_cast<uint4 *>(img + QT * D + swz(r, ch * 8)) = st.d[u];
    }
    if constexpr (DMA) {
      if (tid < 2 * QT) rowc[buf * 2 * QT + tid] = st.live ? (tid < QT ? st.rc * kLog2e_ : st.rc) : 0.f;
    } else {
      if (tid < 2 * QT) rowc[buf * 2 * QT + tid] = st.rc;
    }
  };
  StageQ stq;
  if (n_it > 0) {
    stq = load_it(0);
    store_it(0, stq);
  }
  __syncthreads();
  for (int it = 0; it < n_it; ++it) {
    if (it + 1 < n_it) stq = load_it(it + 1);
    const int buf = it & 1;
#pragma unroll
    for (int sub = 0; sub < QT / 32; ++sub) {
    const uint16_t *qi = lds + buf * 2 * QT * D + sub * 32 * D;
    const uint16_t *di = qi + QT * D;
    const float *lse2 = rowc + buf * 2 * QT + sub * 32;
    const float *dlt = lse2 + QT;
    const int qt0 = qfirst + (GROUPED ? it % n_qt : it) * QT + sub * 32;
    if (qt0 + 31 >= k0 && k0 < len && qt0 < len) {  // some query of the 32-row half sees a wave key
      // S = Q K^T and dP = dO V^T, rows = queries (registers), columns = keys (lanes)
      f32x16 sacc, pacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[r] = 0.f;
        pacc[r] = -dlt[crow(r, h)];  // row constant as the initial accumulator: dP - delta
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8 *>(qi + swz(kl, 16 * s + 8 * h));
        const bf16x8 da = *reinterpret_cast<const bf16x8 *>(di + swz(kl, 16 * s + 8 * h));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[s], pacc, 0, 0, 0);
      }
      const bool need_mask = (qt0 < k0 + 31) || (qt0 + 32 > len) || (k0 + 32 > len);
      float p[16], ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) p[r] = __builtin_amdgcn_exp2f(fmaf(sacc[r], c, -lse2[crow(r, h)]));
      if (need_mask) {  // wave-uniform branch; live rows: key <= q < len, as one unsigned range test
        const int lo = key - qt0 - 4 * h;
        const unsigned span = key < len ? static_cast<unsigned>(len - key) : 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          p[r] = static_cast<unsigned>(crow(r, 0) - lo) >= span ? 0.f : p[r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) ds[r] = p[r] * pacc[r];  // (dP - delta) * p
      // dV^T += dO^T P, dK^T += Q^T dS  (k = queries, permuted order of the accumulator rows)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack_frag(p + 8 * s), db = pack_frag(ds + 8 * s);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          dvt[dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(di, 0, s, dh, lane), pb, dvt[dh], 0, 0, 0);
          dkt[dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(qi, 0, s, dh, lane), db, dkt[dh], 0, 0, 0);
        }
      }
    }
    }  // sub
    if (it + 1 < n_it) store_it((it + 1) & 1, stq);
    __syncthreads();
  }
  // this head's partial dK = scale * (dK^T)^T and dV = (dV^T)^T, fp32 [Hq][T][64]: lane holds
  // column key, rows d = 32 dh + 8 gg + 4 h + i
  if (GROUPED) {
    // dK = scale * (dK^T)^T, dV = (dV^T)^T summed over the group in registers: bf16 [T, Hk, 64]
    if (key < len) {
      uint16_t *dkr = dk_out + (static_cast<int64_t>(s0 + key) * Hk + g) * D;
      uint16_t *dvr = dv_out + (static_cast<int64_t>(s0 + key) * Hk + g) * D;
#pragma unroll
      for (int dh = 0; dh < 2; ++dh)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int d0 = dh * 32 + 8 * gg + 4 * h;
          *reinterpret_cast<uint2 *>(dkr + d0) =
              make_uint2(pk_bf16(dkt[dh][4 * gg] * scale, dkt[dh][4 * gg + 1] * scale),
                         pk_bf16(dkt[dh][4 * gg + 2] * scale, dkt[dh][4 * gg + 3] * scale));
          *reinterpret_cast<uint2 *>(dvr + d0) =
              make_uint2(pk_bf16(dvt[dh][4 * gg], dvt[dh][4 * gg + 1]), pk_bf16(dvt[dh][4 * gg + 2], dvt[dh][4 * gg + 3]));
        }
    }
    return;
  }
  if (key < len) {
    float *dkr = pdk + (static_cast<int64_t>(hq0) * T + s0 + key) * D;
    float *dvr = pdv + (static_cast<int64_t>(hq0) * T + s0 + key) * D;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d0 = dh * 32 + 8 * gg + 4 * h;
        *reinterpret_cast<float4 *>(dkr + d0) = make_float4(dkt[dh][4 * gg] * scale, dkt[dh][4 * gg + 1] * scale,
                                                            dkt[dh][4 * gg + 2] * scale, dkt[dh][4 * gg + 3] * scale);
        *reinterpret_cast<float4 *>(dvr + d0) =
            make_float4(dvt[dh][4 * gg], dvt[dh][4 * gg + 1], dvt[dh][4 * gg + 2], dvt[dh][4 * gg + 3]);
      }
  }
}

// dK / dV [T, Hk, 64] bf16 = sum over the G query heads of a group of the partials, fixed order
__global__ __launch_bounds__(256) void flash_bwd_group_sum_kernel(const float *__restrict__ pdk,
                                                                  const float *__restrict__ pdv, int64_t T, int Hq,
                                                                  int Hk, uint16_t *__restrict__ dk,
                                                                  uint16_t *__restrict__ dv) {
  const int G = Hq / Hk;
  const int64_t total = T * Hk * (D / 4);  // float4 granules
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int c4 = static_cast<int>(i % (D / 4));
    const int64_t tg = i / (D / 4);
    const int gk = static_cast<int>(tg % Hk);
    const int64_t t = tg / Hk;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    for (int j = 0; j < G; ++j) {
      const int64_t off = ((static_cast<int64_t>(gk * G + j)) * T + t) * D + 4 * c4;
      const float4 x = *reinterpret_cast<const float4 *>(pdk + off);
      const float4 y = *reinterpret_cast<const float4 *>(pdv + off);
      a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
      b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
    }
    const int64_t o = (t * Hk + gk) * D + 4 * c4;
    *reinterpret_cast<uint2 *>(dk + o) = make_uint2(pk_bf16(a.x, a.y), pk_bf16(a.z, a.w));
    *reinterpret_cast<uint2 *>(dv + o) = make_uint2(pk_bf16(b.x, b.y), pk_bf16(b.z, b.w));
  }
}

// Also computes delta = rowsum(dO * O) of its queries from the O / dO fragments it loads anyway
// (each query's 64 values are split over lanes l and l ^ 32) and publishes it for the dK / dV
// launch that follows: no separate delta pass over O and dO.
// KBQ = keys per staged block (64 or 128): 128 halves the barriers per MFMA; the block's 32-key
// tiles run the same body
template <int KBQ, bool DMA>
__global__ __launch_bounds__(256, DMA ? VA_FLASH_DQ_DMA_OCC : 2) void flash_bwd_dq_kernel(
    const uint16_t *__restrict__ k, const uint16_t *__restrict__ v, const uint16_t *__restrict__ q,
    const uint16_t *__restrict__ o, const uint16_t *__restrict__ dout, const float *__restrict__ lse,
    float *__restrict__ delta, const int32_t *__restrict__ cu, const int32_t *__restrict__ blocks, int64_t ld,
    int Hq, int Hk, float scale, uint16_t *__restrict__ dq) {
  static_assert(KBQ == 64 || KBQ == 128, "KBQ");
  constexpr int NCK = KBQ * 8 / 256;  // 16-B chunks per thread per operand
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * KBQ * D];  // [buf][K | V][KBQ keys][64 d], swizzled
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, ql = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
  const int seq = blocks[2 * blockIdx.x], qs = blocks[2 * blockIdx.x + 1];
  const int head = blockIdx.y, kvh = head / (Hq / Hk);
  const int s0 = cu[seq], len = cu[seq + 1] - s0;
  const int q_pos = qs + wave * 32 + ql;
  const bool q_ok = q_pos < len;
  const int64_t ldq = static_cast<int64_t>(Hq) * D, ldk = static_cast<int64_t>(Hk) * D;
  const float c = scale * kLog2e_;
  bf16x8 qf[4], df[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (q_ok) {
      qf[s] = *reinterpret_cast<const bf16x8 *>(q + (s0 + q_pos) * ldq + head * D + 16 * s + 8 * h);
      df[s] = *reinterpret_cast<const bf16x8 *>(dout + (s0 + q_pos) * ldq + head * D + 16 * s + 8 * h);
    } else {
      qf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      df[s] = qf[s];
    }
  }
  const int64_t ridx = (static_cast<int64_t>(seq) * Hq + head) * ld + q_pos;
  const float lse2 = q_ok ? lse[ridx] * kLog2e_ : 0.f;
  float dpart = 0.f;
  if (q_ok) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint4 a = *reinterpret_cast<const uint4 *>(o + (s0 + q_pos) * ldq + head * D + 16 * s + 8 * h);
      const uint4 b = __builtin_bit_cast(uint4, df[s]);
      dpart = fmaf(bf16_lo(a.x), bf16_lo(b.x), dpart); dpart = fmaf(bf16_hi(a.x), bf16_hi(b.x), dpart);
      dpart = fmaf(bf16_lo(a.y), bf16_lo(b.y), dpart); dpart = fmaf(bf16_hi(a.y), bf16_hi(b.y), dpart);
      dpart = fmaf(bf16_lo(a.z), bf16_lo(b.z), dpart); dpart = fmaf(bf16_hi(a.z), bf16_hi(b.z), dpart);
      dpart = fmaf(bf16_lo(a.w), bf16_lo(b.w), dpart); dpart = fmaf(bf16_hi(a.w), bf16_hi(b.w), dpart);
    }
  }
  // lane half 0 holds d in {0-7, 16-23, 32-39, 48-55}, half 1 the rest: fixed-order pair sum
  const float dother = __shfl_xor(dpart, 32);
  const float dlt = h == 0 ? dpart + dother : dother + dpart;
  if (q_ok && h == 0) delta[ridx] = dlt;
  f32x16 dqt[2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int r = 0; r < 16; ++r) dqt[dh][r] = 0.f;

  const int kv_end = min(len, qs + QB);
  const int nkb = (kv_end + KBQ - 1) / KBQ;
  const int wave_last_q = qs + wave * 32 + 31;
  uint4 sk[DMA ? 1 : NCK], sv[DMA ? 1 : NCK];
  auto load_block = [&](int kb) {
#pragma unroll
    for (int u = 0; u < NCK; ++u) {
      const int idx = tid + u * 256, r = idx >> 3, ch = idx & 7;
      const int kk = kb * KBQ + r;
      const bool ok = kk < len;
      const int64_t base = (s0 + (ok ? kk : len - 1)) * ldk + kvh * D + ch * 8;  // clamped: no branch
      const uint4 a = *reinterpret_cast<const uint4 *>(k + base);
      const uint4 b = *reinterpret_cast<const uint4 *>(v + base);
      sk[u] = ok ? a : make_uint4(0, 0, 0, 0);
      sv[u] = ok ? b : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_block = [&](int buf) {
    uint16_t *lk = lds + buf * 2 * KBQ * D;
    uint16_t *lv = lk + KBQ * D;
#pragma unroll
    for (int u = 0; u < NCK; ++u) {
      const int idx = tid + u * 256, r = idx >> 3, ch = idx & 7;
      *reinterpret_cast<uint4 *>(lk + swz(r, ch * 8)) = sk[u];
      *reinterpret_cast<uint4 *>(lv + swz(r, ch * 8)) = sv[u];
    }
  };
  // DMA: LDS-DMA staging as in the forward (rows past the sequence end clamped: their dS is 0)
  auto dma_block = [&](int kb, int buf) {
    uint16_t *lk = lds + buf * 2 * KBQ * D;
    uint16_t *lv = lk + KBQ * D;
#pragma unroll
    for (int pi = wave; pi < KBQ / 8; pi += 4) {
      const int r = pi * 8 + (lane >> 3), pch = (lane & 7) ^ (r & 7);
      const int kk = kb * KBQ + r;
      const int64_t base = (s0 + (kk < len ? kk : len - 1)) * ldk + kvh * D + (pch << 3);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(k + base), lk + pi * 8 * D, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(v + base), lv + pi * 8 * D, 16, 0, 0);
    }
  };
  if (nkb > 0) {
    if constexpr (DMA) {
      dma_block(0, 0);
    } else {
      load_block(0);
      store_block(0);
    }
  }
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) {
      if constexpr (DMA) dma_block(kb + 1, (kb + 1) & 1);
      else load_block(kb + 1);
    }
    const uint16_t *lk = lds + (kb & 1) * 2 * KBQ * D;
    const uint16_t *lv = lk + KBQ * D;
#pragma unroll
    for (int t = 0; t < KBQ / 32; ++t) {
      const int key0 = kb * KBQ + t * 32;
      if (key0 > wave_last_q || key0 >= len || qs + wave * 32 >= len) continue;
      f32x16 sacc, pacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[r] = 0.f;
        pacc[r] = -dlt;  // row constant as the initial accumulator: dP - delta
      }
      const int krow = t * 32 + ql;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 ka = *reinterpret_cast<const bf16x8 *>(lk + swz(krow, 16 * s + 8 * h));
        const bf16x8 va = *reinterpret_cast<const bf16x8 *>(lv + swz(krow, 16 * s + 8 * h));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, df[s], pacc, 0, 0, 0);
      }
      const bool need_mask = (key0 + 31 > qs + wave * 32) || (key0 + 31 >= len);
      float ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) ds[r] = __builtin_amdgcn_exp2f(fmaf(sacc[r], c, -lse2));
      if (need_mask) {  // wave-uniform branch; key offset vs. a per-lane limit
        const int lim = min(q_pos, len - 1) - key0 - 4 * h;
#pragma unroll
        for (int r = 0; r < 16; ++r) ds[r] = crow(r, 0) > lim ? 0.f : ds[r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) ds[r] *= pacc[r];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 db = pack_frag(ds + 8 * s);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh)
          dqt[dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(lk, t * 32, s, dh, lane), db, dqt[dh], 0, 0, 0);
      }
    }
    if constexpr (!DMA) {
      if (kb + 1 < nkb) store_block((kb + 1) & 1);
    }
    __syncthreads();
  }
  if (q_ok) {
    uint16_t *qr = dq + (s0 + q_pos) * ldq + head * D;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        *reinterpret_cast<uint2 *>(qr + dh * 32 + 8 * gg + 4 * h) =
            make_uint2(pk_bf16(dqt[dh][4 * gg] * scale, dqt[dh][4 * gg + 1] * scale),
                       pk_bf16(dqt[dh][4 * gg + 2] * scale, dqt[dh][4 * gg + 3] * scale));
  }
}

}  // namespace
}  // namespace va

using namespace va;

// va_set_tuning(VA_TUNE_FLASH_GROUPED_DKDV): -1 auto, 0 per-query-head partials + group sum, 1 grouped
int g_flash_grouped_dkdv = -1;
// va_set_tuning(VA_TUNE_FLASH_DKDV_QT): query rows per staged dK / dV tile, 32, 64 (default) or 128
// (register staging: fwd+bwd 2,485 / 2,421 / 2,383 us at 151,819 tokens, profiles/r01/attn_bwd_staging_ab.log;
// LDS-DMA staging: 64 2,242-2,248 vs 128 2,255-2,268 us, profiles/r04/attn_dma_ab.jsonl)
int g_flash_dkdv_qt = 64;
// va_set_tuning(VA_TUNE_FLASH_DQ_KB): keys per staged dQ block, 64 (default) or 128 (LDS-DMA staging:
// 64 keys = 32 KiB of LDS lets 3 workgroups share a CU; fwd+bwd 2,288-2,301 vs 2,318-2,325 us)
int g_flash_dq_kb = 64;
// va_set_tuning(VA_TUNE_FLASH_FWD_KB): keys per staged forward block, 64 (default) or 128 (slower:
// 654 vs 573 us at 151,819 tokens, profiles/r01/attn_bwd_staging_ab.log)
int g_flash_fwd_kb = 64;
// va_set_tuning(VA_TUNE_FLASH_DMA): bit 1 = forward K / V blocks staged by LDS-DMA (64-key blocks),
// bit 2 = the same for the dQ backward, bit 4 = the dK / dV backward's Q / dO tiles; default 7 (all:
// forward 541-549 vs 591-597 us, fwd+bwd 2,242-2,248 vs 2,368-2,385 us at 151,819 tokens, bitwise
// the same results, profiles/r04/attn_dma_ab.jsonl); 0 = register staging through VGPRs
int g_flash_dma = 7;

extern "C" int va_flash_attn_fwd(const void *q, const void *k, const void *v, const int32_t *cu_seqlens,
                                 const int32_t *block_table, int64_t n_blocks, int64_t T, int64_t Hq, int64_t Hk,
                                 int64_t head_dim, int64_t max_len, float scale, void *o, float *lse, void *stream) {
  VA_CHECK_ARG(head_dim == D, "flash_attn_fwd: head_dim must be 64 (got %lld)", static_cast<long long>(head_dim));
  VA_CHECK_ARG(Hq > 0 && Hk > 0 && Hq % Hk == 0, "flash_attn_fwd: Hq must be a multiple of Hk");
  VA_CHECK_ARG(T >= 0 && n_blocks >= 0 && n_blocks < (1ll << 31) && max_len >= 0, "flash_attn_fwd: bad sizes");
  if (n_blocks == 0 || T == 0) return VA_OK;
  VA_CHECK_ARG(q && k && v && cu_seqlens && block_table && o && lse, "null pointer argument");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(q) % 16 == 0 && reinterpret_cast<uintptr_t>(k) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(v) % 16 == 0 && reinterpret_cast<uintptr_t>(o) % 16 == 0,
               "flash_attn_fwd: 16-byte aligned q / k / v / o required");
#define VA_FWD(KBV, DMAV)                                                                                       \
  hipLaunchKernelGGL((flash_fwd_kernel<KBV, DMAV>), dim3(static_cast<unsigned>(n_blocks), static_cast<unsigned>(Hq)),     \
                     dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const uint16_t *>(q),              \
                     static_cast<const uint16_t *>(k), static_cast<const uint16_t *>(v), cu_seqlens, block_table,  \
                     max_len, static_cast<int>(Hq), static_cast<int>(Hk), scale, static_cast<uint16_t *>(o), lse)
  if (g_flash_dma & 1) VA_FWD(64, true); else if (g_flash_fwd_kb == 64) VA_FWD(64, false); else VA_FWD(128, false);
#undef VA_FWD
  return check_launch("flash_attn_fwd");
}

extern "C" int va_flash_attn_bwd(const void *q, const void *k, const void *v, const void *o, const void *dout,
                                 const float *lse, const int32_t *cu_seqlens, const int32_t *q_blocks,
                                 int64_t n_q_blocks, const int32_t *k_blocks, int64_t n_k_blocks, int64_t T,
                                 int64_t Hq, int64_t Hk, int64_t head_dim, int64_t max_len, float scale, float *delta,
                                 float *partial, void *dq, void *dk, void *dv, void *stream) {
  VA_CHECK_ARG(head_dim == D, "flash_attn_bwd: head_dim must be 64");
  VA_CHECK_ARG(Hq > 0 && Hk > 0 && Hq % Hk == 0, "flash_attn_bwd: Hq must be a multiple of Hk");
  VA_CHECK_ARG(T >= 0 && n_q_blocks >= 0 && n_k_blocks >= 0 && max_len >= 0, "flash_attn_bwd: bad sizes");
  if (n_q_blocks == 0 || T == 0) return VA_OK;
  VA_CHECK_ARG(q && k && v && o && dout && lse && cu_seqlens && q_blocks && k_blocks && delta && partial && dq && dk &&
                   dv,
               "null pointer argument");
  float *pdk = partial, *pdv = partial + Hq * T * D;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // dQ first: it also produces delta for the dK / dV launch
#define VA_DQ(KBV, DMAV)                                                                                         \
  hipLaunchKernelGGL((flash_bwd_dq_kernel<KBV, DMAV>), dim3(static_cast<unsigned>(n_q_blocks), static_cast<unsigned>(Hq)), \
                     dim3(256), 0, s, static_cast<const uint16_t *>(k), static_cast<const uint16_t *>(v),             \
                     static_cast<const uint16_t *>(q), static_cast<const uint16_t *>(o),                              \
                     static_cast<const uint16_t *>(dout), lse, delta, cu_seqlens, q_blocks, max_len,                  \
                     static_cast<int>(Hq), static_cast<int>(Hk), scale, static_cast<uint16_t *>(dq))
  if (g_flash_dma & 2) {
    if (g_flash_dq_kb == 64) VA_DQ(64, true); else VA_DQ(128, true);
  } else {
    if (g_flash_dq_kb == 64) VA_DQ(64, false); else VA_DQ(128, false);
  }
#undef VA_DQ
  // grouped dK / dV (one workgroup per key block x KV head, no partials) once the key blocks alone
  // give >= 2 workgroups per CU; otherwise per query head + the fixed-order group sum
  const bool grouped = g_flash_grouped_dkdv == 1 || (g_flash_grouped_dkdv < 0 && n_k_blocks * Hk >= 512);
  const int qt = g_flash_dkdv_qt;
#define VA_DKDV(GR, QTV)                                                                                         \
  if (g_flash_dma & 4) VA_DKDV_L(GR, QTV, true); else VA_DKDV_L(GR, QTV, false)
#define VA_DKDV_L(GR, QTV, DMAV)                                                                                 \
  hipLaunchKernelGGL((flash_bwd_dkdv_kernel<GR, QTV, DMAV>),                                                           \
                     dim3(static_cast<unsigned>(n_k_blocks), static_cast<unsigned>(GR ? Hk : Hq)), dim3(256), 0, s, \
                     static_cast<const uint16_t *>(q), static_cast<const uint16_t *>(k),                          \
                     static_cast<const uint16_t *>(v), static_cast<const uint16_t *>(dout), lse, delta, cu_seqlens, \
                     k_blocks, max_len, T, static_cast<int>(Hq), static_cast<int>(Hk), scale, pdk, pdv,            \
                     static_cast<uint16_t *>(dk), static_cast<uint16_t *>(dv))
  if (grouped) {
    if (qt == 32) {
      VA_DKDV(true, 32);
    } else if (qt == 128) {
      VA_DKDV(true, 128);
    } else {
      VA_DKDV(true, 64);
    }
  } else {
    if (qt == 32) {
      VA_DKDV(false, 32);
    } else if (qt == 128) {
      VA_DKDV(false, 128);
    } else {
      VA_DKDV(false, 64);
    }
  }
#undef VA_DKDV
#undef VA_DKDV_L
  if (!grouped) {
    const int64_t granules = T * Hk * (D / 4);
    int64_t grid = (granules + 255) / 256;
    if (grid > 16384) grid = 16384;
    hipLaunchKernelGGL(flash_bwd_group_sum_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, s, pdk, pdv, T,
                       static_cast<int>(Hq), static_cast<int>(Hk), static_cast<uint16_t *>(dk),
                       static_cast<uint16_t *>(dv));
  }
  return check_launch("flash_attn_bwd");
}
