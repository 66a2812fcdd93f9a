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
// K / V blocks of 64 keys are staged through double-buffered LDS shared by the 4 waves (the
// block's next K / V rows are in registers during the current block's MFMAs). K rows are
// XOR-swizzled for the row-fragment reads; V rows are plain for the transposed reads.

#include <math.h>

#include "va_common.h"

namespace va {
namespace {

constexpr int D = 64;
constexpr int QB = 128;  // query rows per workgroup
constexpr int KB = 64;   // keys per staged block
constexpr float kLog2e_ = 1.4426950408889634f;
constexpr float kLn2_ = 0.69314718055994531f;

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

__global__ __launch_bounds__(256, 2) void flash_fwd_kernel(
    const uint16_t *__restrict__ q, const uint16_t *__restrict__ k, const uint16_t *__restrict__ v,
    const int32_t *__restrict__ cu, const int32_t *__restrict__ blocks, int64_t lse_ld, int Hq, int Hk,
    float scale, uint16_t *__restrict__ o, float *__restrict__ lse) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * KB * D];  // [buf][K | V][64 keys][64 d]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, ql = lane & 31;
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
  const int nkb = (kv_end + KB - 1) / KB;
  const int wave_last_q = qs + wave * 32 + 31;

  // staging: 64 rows x 8 chunks of 16 B per operand = 512 chunks, 2 per thread per operand
  uint4 sk[2], sv[2];
  auto load_block = [&](int kb) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + u * 256, r = idx >> 3, ch = idx & 7;
      const int key = kb * KB + r;
      if (key < len) {
        const int64_t base = (s0 + key) * ldk + kvh * D + ch * 8;
        sk[u] = *reinterpret_cast<const uint4 *>(k + base);
        sv[u] = *reinterpret_cast<const uint4 *>(v + base);
      } else {
        sk[u] = make_uint4(0, 0, 0, 0);
        sv[u] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_block = [&](int buf) {
    uint16_t *lk = lds + buf * 2 * KB * D;
    uint16_t *lv = lk + KB * D;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + u * 256, r = idx >> 3, ch = idx & 7;
      *reinterpret_cast<uint4 *>(lk + r * D + ((ch ^ (r & 7)) << 3)) = sk[u];
      *reinterpret_cast<uint4 *>(lv + r * D + (ch << 3)) = sv[u];
    }
  };

  if (nkb > 0) {
    load_block(0);
    store_block(0);
  }
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) load_block(kb + 1);
    const uint16_t *lk = lds + (kb & 1) * 2 * KB * D;
    const uint16_t *lv = lk + KB * D;
    const int key0 = kb * KB;
    // the whole 64-key block is past this wave's queries (or the wave has none): skip
    if (!(key0 > wave_last_q || qs + wave * 32 >= len)) {
      const bool t1_live = key0 + 32 <= wave_last_q && key0 + 32 < len;  // second 32-key tile
      // ---- S^T = K Q^T for the block's two 32-key tiles (keys on rows, queries on lanes)
      f32x16 sacc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] = 0.f;
        if (t == 1 && !t1_live) continue;
        const int krow = t * 32 + ql;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ch = 2 * s + h;
          const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(lk + krow * D + ((ch ^ (krow & 7)) << 3));
          sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[t], 0, 0, 0);
        }
      }
      // ---- online softmax over the block (base 2); masks only on diagonal / sequence-end blocks
      const bool need_mask = (key0 + KB - 1 > qs + wave * 32) || (key0 + KB - 1 >= len);
      float x[32];
      float tm = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float xv = sacc[t][r] * c;
          if (need_mask) {
            const int kp = key0 + t * 32 + crow(r, h);
            if (kp > q_pos || kp >= len) xv = -INFINITY;
          }
          x[16 * t + r] = xv;
          tm = fmaxf(tm, xv);
        }
      tm = fmaxf(tm, __shfl_xor(tm, 32, kWave));
      const float mn = fmaxf(m, tm);
      const float msafe = mn == -INFINITY ? 0.f : mn;
      float rs = 0.f;
#pragma unroll
      for (int r = 0; r < 32; ++r) {
        x[r] = __builtin_amdgcn_exp2f(x[r] - msafe);
        rs += x[r];
      }
      rs += __shfl_xor(rs, 32, kWave);
      if (mn != m) {  // rescale only rows whose max moved (all-lane uniform skip is common later on)
        const float alpha = __builtin_amdgcn_exp2f(m - msafe);  // m = -inf -> 0
        l *= alpha;
#pragma unroll
        for (int dh = 0; dh < 2; ++dh)
#pragma unroll
          for (int r = 0; r < 16; ++r) oacc[dh][r] *= alpha;
      }
      l += rs;
      m = mn;
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
    // the other buffer was last read in iteration kb - 1, which every wave finished before the
    // barrier that ended it: store, then one barrier publishes the block for iteration kb + 1
    if (kb + 1 < nkb) store_block((kb + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: O = O^T / l, lane holds O[q][32 dh + crow(r, h)]; lse in natural log
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
      lse[(static_cast<int64_t>(seq) * Hq + head) * lse_ld + q_pos] = (m + __builtin_amdgcn_logf(l)) * kLn2_;
  }
}

}  // namespace
}  // namespace va

using namespace va;

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
  hipLaunchKernelGGL(flash_fwd_kernel, dim3(static_cast<unsigned>(n_blocks), static_cast<unsigned>(Hq)), dim3(256),
                     0, static_cast<hipStream_t>(stream), static_cast<const uint16_t *>(q),
                     static_cast<const uint16_t *>(k), static_cast<const uint16_t *>(v), cu_seqlens, block_table,
                     max_len, static_cast<int>(Hq), static_cast<int>(Hk), scale, static_cast<uint16_t *>(o), lse);
  return check_launch("flash_attn_fwd");
}
