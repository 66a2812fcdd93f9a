// Fused lm_head GEMM + temperature + log-softmax gather + entropy (forward), gfx950 MFMA.
// the [N, V] logits are never written to HBM.
//
// Reference semantics: the unfused path of the actor (dp_actor.py:170-190):
//   logits = hidden @ W^T (bf16 out under autocast), logits.div_(T) (bf16), then
//   logprobs_from_logits / entropy_from_logits (torch_functional.py:64-160) in fp32 math;
// and the reference's own fused option (use_fused_kernels, utils/kernel/kernels.py:120-663:
// linear + log-softmax + entropy in row/vocab tiles with online statistics).
//
// Kernel 1 (linear_logprob_tiles): grid (row blocks of 128, VSPLIT vocab ranges). A 256-thread
// workgroup = 4 waves; each wave owns 32 rows x 128 vocab columns of a 128 x 128 logits tile
// = 2 x 8 blocks of v_mfma_f32_16x16x32_bf16. K (the hidden size, a multiple of 64) streams in
// 64-deep steps through double-buffered, row-padded LDS images with the next step's global loads
// in flight during the MFMAs. Per finished tile the accumulators are
// rounded to bf16 (the logits dtype), divided by T (rounded again, as div_), and folded into
// per-row online (max, sum 2^(xL-B), sum 2^(xL-B) x) statistics: row max by 4 lane shuffles, one
// exp2 per logit, sums by 8 shuffles. The label's logit is written by the one lane that holds it.
// Kernel 2 (linear_logprob_merge): per row, merge the VSPLIT partial states in fixed order ->
// lse, entropy = lse - t/s, logp = x[label] - lse (ignore_index -100 -> 0, out of range -> NaN).
//
// Bound: MFMA (2 N V H flops); HBM traffic is hidden + W per row block (L2 / MALL-served) plus
// 12 B/row of partials per vocab range.

#include <math.h>

#include <type_traits>

#include "va_common.h"

namespace va {
namespace {

constexpr float kLog2eF = 1.4426950408889634f;
constexpr float kLn2F = 0.69314718055994531f;

constexpr int BM = 128, BN = 128, BK = 64;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float base_of(float m) { return m == -INFINITY ? 0.f : m * kLog2eF; }

__device__ __forceinline__ float round_bf16(float x) { return round_to_bf16(x); }

struct RowAcc {
  float m, s, t;
};

__device__ __forceinline__ void merge_state(RowAcc &a, float om, float os, float ot) {
  const float nm = fmaxf(a.m, om);
  const float nb = base_of(nm);
  const float a1 = __builtin_amdgcn_exp2f(base_of(a.m) - nb);
  const float a2 = __builtin_amdgcn_exp2f(base_of(om) - nb);
  a.s = a.s * a1 + os * a2;
  a.t = a.t * a1 + ot * a2;
  a.m = nm;
}

// K streams in 64-deep chunks through two row-padded LDS images (144-B rows: conflict-free
// ds_read_b128 fragments); the next chunk's global loads are in registers while the MFMAs of
// the current one run (2 workgroups per CU hide the rest). A measured alternative with an
// LDS-DMA (global_load_lds) ring of 4 chunks needs 128 KB of LDS -> 1 workgroup / 1 wave per
// SIMD and ran 0.68x as fast (fragment-read latency is no longer hidden).
constexpr int LDS_ROW = BK + 8;  // bf16 elements per padded LDS row
constexpr int TILE_ELEMS = BM * LDS_ROW;

template <bool SCALE, bool ROUND>
__global__ __launch_bounds__(256, 2) void linear_logprob_tiles_kernel(
    const uint16_t *__restrict__ hid, int64_t ldh, const uint16_t *__restrict__ w, int64_t ldw,
    const int64_t *__restrict__ labels, int64_t N, int K, int64_t V, int tiles_per_split, float temperature,
    float *__restrict__ part, float *__restrict__ label_logit) {
  // ONE LDS array: two staging buffers (A, W images), then per-row label, label logit, state
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * TILE_ELEMS + BM * 2 * 5];
  float *s_state = reinterpret_cast<float *>(lds + 2 * 2 * TILE_ELEMS);  // [BM][3] m, s, t
  float *s_lablogit = s_state + BM * 3;                                  // [BM]
  int *s_label = reinterpret_cast<int *>(s_lablogit + BM);               // [BM]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
  const int64_t n_vtiles = (V + BN - 1) / BN;
  const int64_t vt_begin = static_cast<int64_t>(blockIdx.y) * tiles_per_split;
  int64_t vt_end = vt_begin + tiles_per_split;
  if (vt_end > n_vtiles) vt_end = n_vtiles;
  if (tid < BM) {
    const int64_t r = row0 + tid;
    const int64_t lab = r < N ? labels[r] : -1;
    s_label[tid] = (lab >= 0 && lab < V) ? static_cast<int>(lab) : -1;
    s_lablogit[tid] = 0.f;
    s_state[tid * 3 + 0] = -INFINITY;
    s_state[tid * 3 + 1] = 0.f;
    s_state[tid * 3 + 2] = 0.f;
  }
  const int nk = K / BK;
  // staging map: 1024 16-byte vectors per operand chunk, 4 per thread (row v>>3, k (v&7)*8);
  // per-thread source row pointers are fixed for the whole kernel (A) or per tile (W)
  const uint16_t *a_src[4];
  int st_off[4], w_r[4], kc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = tid + u * 256;
    const int r = v >> 3, c = (v & 7) * 8;
    int64_t gr = row0 + r;
    if (gr >= N) gr = N - 1;  // clamped rows / columns are computed and discarded
    a_src[u] = hid + gr * ldh + c;
    st_off[u] = r * LDS_ROW + c;
    w_r[u] = r;
    kc[u] = c;
  }
  struct Stage {
    uint4 a0, a1, a2, a3, b0, b1, b2, b3;
  };
  auto wsrc = [&](int64_t vt, int u) {
    int64_t gc = vt * BN + w_r[u];
    if (gc >= V) gc = V - 1;
    return w + gc * ldw + kc[u];
  };
  auto load_stage = [&](int64_t vt, int kt) -> Stage {
    const int ko = kt * BK;
    Stage g;
    g.a0 = *reinterpret_cast<const uint4 *>(a_src[0] + ko);
    g.a1 = *reinterpret_cast<const uint4 *>(a_src[1] + ko);
    g.a2 = *reinterpret_cast<const uint4 *>(a_src[2] + ko);
    g.a3 = *reinterpret_cast<const uint4 *>(a_src[3] + ko);
    g.b0 = *reinterpret_cast<const uint4 *>(wsrc(vt, 0) + ko);
    g.b1 = *reinterpret_cast<const uint4 *>(wsrc(vt, 1) + ko);
    g.b2 = *reinterpret_cast<const uint4 *>(wsrc(vt, 2) + ko);
    g.b3 = *reinterpret_cast<const uint4 *>(wsrc(vt, 3) + ko);
    return g;
  };
  auto store_stage = [&](int buf, const Stage &g) {
    uint16_t *la_ = lds + buf * 2 * TILE_ELEMS;
    uint16_t *lb_ = la_ + TILE_ELEMS;
    *reinterpret_cast<uint4 *>(la_ + st_off[0]) = g.a0;
    *reinterpret_cast<uint4 *>(la_ + st_off[1]) = g.a1;
    *reinterpret_cast<uint4 *>(la_ + st_off[2]) = g.a2;
    *reinterpret_cast<uint4 *>(la_ + st_off[3]) = g.a3;
    *reinterpret_cast<uint4 *>(lb_ + st_off[0]) = g.b0;
    *reinterpret_cast<uint4 *>(lb_ + st_off[1]) = g.b1;
    *reinterpret_cast<uint4 *>(lb_ + st_off[2]) = g.b2;
    *reinterpret_cast<uint4 *>(lb_ + st_off[3]) = g.b3;
  };

  for (int64_t vt = vt_begin; vt < vt_end; ++vt) {
    f32x4 acc[2][8];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

    Stage g = load_stage(vt, 0);
    __syncthreads();  // the previous tile's last reads of buffer 0 are done
    store_stage(0, g);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) g = load_stage(vt, kt + 1);
      const uint16_t *la = lds + buf * 2 * TILE_ELEMS;
      const uint16_t *lb = la + TILE_ELEMS;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int kof = s * 32 + (lane >> 4) * 8;
        bf16x8 fa[2], fb[8];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
          fa[mb] = *reinterpret_cast<const bf16x8 *>(la + (wave * 32 + mb * 16 + (lane & 15)) * LDS_ROW + kof);
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
          fb[nb] = *reinterpret_cast<const bf16x8 *>(lb + (nb * 16 + (lane & 15)) * LDS_ROW + kof);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
          for (int nb = 0; nb < 8; ++nb)
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mb], fb[nb], acc[mb][nb], 0, 0, 0);
      }
      if (kt + 1 < nk) store_stage(buf ^ 1, g);
      __syncthreads();
    }

    // ---- epilogue: fold the finished 128 x 128 tile into the per-row online statistics
    const int64_t col0 = vt * BN;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int lr = wave * 32 + mb * 16 + (lane >> 4) * 4 + j;  // local row (owned by this wave)
        const int lab = s_label[lr];
        float x[8];
        float cm = -INFINITY;
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) {
          const int64_t col = col0 + nb * 16 + (lane & 15);
          // ROUND: the bf16 logits of the unfused path; else fp32 logits (the reference's fused kernel)
          float v = ROUND ? round_bf16(acc[mb][nb][j]) : acc[mb][nb][j];
          if constexpr (SCALE) v = ROUND ? round_bf16(v / temperature) : v / temperature;
          if (col >= V) v = -INFINITY;
          x[nb] = v;
          cm = fmaxf(cm, v);
          if (col == lab) s_lablogit[lr] = v;
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) cm = fmaxf(cm, __shfl_xor(cm, o, kWave));
        const float om = s_state[lr * 3 + 0], os = s_state[lr * 3 + 1], ot = s_state[lr * 3 + 2];
        const float nm = fmaxf(om, cm);
        const float nbse = base_of(nm);
        float ss = 0.f, tt = 0.f;
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) {
          const float e = __builtin_amdgcn_exp2f(fmaf(x[nb], kLog2eF, -nbse));
          ss += e;
          tt = fmaf(e, x[nb] == -INFINITY ? 0.f : x[nb], tt);
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          ss += __shfl_xor(ss, o, kWave);
          tt += __shfl_xor(tt, o, kWave);
        }
        const float alpha = __builtin_amdgcn_exp2f(base_of(om) - nbse);
        if ((lane & 15) == 0) {
          s_state[lr * 3 + 0] = nm;
          s_state[lr * 3 + 1] = fmaf(os, alpha, ss);
          s_state[lr * 3 + 2] = fmaf(ot, alpha, tt);
        }
      }
  }
  __syncthreads();
  // partial states part[split][row][3]; the label's logit from the split that holds it
  if (tid < BM && row0 + tid < N) {
    const int64_t r = row0 + tid;
    float *p = part + (static_cast<int64_t>(blockIdx.y) * N + r) * 3;
    p[0] = s_state[tid * 3 + 0];
    p[1] = s_state[tid * 3 + 1];
    p[2] = s_state[tid * 3 + 2];
    const int lab = s_label[tid];
    if (lab >= vt_begin * BN && lab < vt_end * BN) label_logit[r] = s_lablogit[tid];
  }
}

// ---------------------------------------------------------------------------------------------
// 256 x 256 TRANSPOSED kernel (VA_TUNE_LINEAR_LOGPROB_TILE = 256, default). The tile is computed as
// S^T = W_tile . H_tile^T: the vocab index is the MFMA row (registers) and the token the MFMA column
// (lane & 15), so every lane owns whole tokens and keeps their online (max, sum 2^(xL-B),
// sum 2^(xL-B) x) state in registers for the whole persistent sweep over its vocab tiles: no
// per-tile cross-lane reduction, LDS round trip or barrier (the round-2 row-on-lane layout spent
// ~20 % of the kernel there). The 4 lane groups and the 2 vocab wave-rows are merged once at the end.
// Core: 8 waves = 2 (vocab halves) x 4 (token quarters), 128 x 64 per wave = 8 x 4
// v_mfma_f32_16x16x32_bf16 blocks; both operands staged by LDS-DMA (global_load_lds, 16 B per lane)
// into two lane-linear buffers whose 16-byte chunk c of row r sits at c ^ ((r >> 1) & 7) (swizzled
// on the global source address: conflict-free fragment reads); the next step's K-chunk is staged
// during the current one, across vocab tiles. Grid: row blocks x vocab splits as ONE dimension,
// remapped so that each XCD gets a contiguous run of (row block, split) ids, split fastest: the few
// row blocks an XCD works on at a time keep their hidden panels in its L2 while the W tiles stream
// (round-3 dev kernel tools/f1core/f1t.hip, git show 690aed1:tools/f1core/f1t.hip; at 131,072 x 896 x 151,936: 30.1 ms core-only vs 32.3 without the remap).
constexpr int TB = 256, TK = 64, T_THREADS = 512;
constexpr int GU_SROW = 72;  // epilogue store scratch row (fused SwiGLU, dlogits): 64 columns + 16 B (bank spread, 16-B reads)

constexpr int T_TILE = TB * TK;  // bf16 elements of one operand's K-step image

__device__ __forceinline__ int t_img_off(int row, int c) { return row * TK + ((c ^ ((row >> 1) & 7)) << 3); }

// image row -> source row of the streamed (weight) operand: the identity for the lm_head; the gate|up
// pairing (GateUpRows below) for the fused SwiGLU projection. kTileStep: source rows one 256-row
// image tile advances, so that map(t * 256 + r) = map(r) + t * kTileStep (the sweep's per-lane
// staging offsets are computed once from map(r)).
struct IdentityRows {
  static constexpr int64_t kTileStep = 256;
  __device__ __forceinline__ int64_t operator()(int64_t r) const { return r; }
  // rows of tile vs's weight window that exist (the last vocab tile may pass V)
  __device__ __forceinline__ int64_t window_rows(int64_t vs, int64_t V) const {
    return V - vs * 256 < 256 ? V - vs * 256 : 256;
  }
};

// the logit as the unfused path holds it: bf16(acc) (ROUND), then bf16(x / T) (SCALE: div_ in bf16)
template <bool SCALE, bool ROUND>
__device__ __forceinline__ float logit_of(float a, float temperature) {
  float v = ROUND ? round_bf16(a) : a;
  if constexpr (SCALE) v = ROUND ? round_bf16(v / temperature) : v / temperature;
  return v;
}

// Fold one finished tile into the lane's per-token state. The logit map (bf16 rounding, division by
// T > 0) is monotonic, so the tile max of the logits is the map of the raw accumulators' max: one
// max pass over acc, then ONE pass of map -> exp2 -> sums. TAIL: the last vocab tile, whose rows
// past V are -inf (weight 0, kept out of the x-weighted sum: 0 * -inf is NaN).
template <bool SCALE, bool ROUND>
__device__ __forceinline__ void t_tile_labels(const f32x4 (&acc)[8][4], int v0, const int (&lab)[4], float (&ll)[4],
                                              float temperature) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = lab[j] - v0;  // the label sits at (i, e) = (d >> 4, d & 3) when d in [0, 128), d & 12 == 0
    if (d >= 0 && d < 128 && (d & 12) == 0) {
      const int uu = (d >> 4) * 4 + (d & 3);
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) v = (i * 4 + e) == uu ? acc[i][j][e] : v;
      ll[j] = logit_of<SCALE, ROUND>(v, temperature);
    }
  }
}

// Fold token column j of a finished tile into the lane's state; branch-free (it shares a scheduling
// region with the next tile's MFMAs). TAIL: vocab rows v0 + 16 i + e >= V are -inf. In three parts
// (the deferred sweep interleaves them with MFMA halves): the max pass (col_begin), the exp / sum
// pass over blocks i in [I0, I1) (col_blocks), and the merge into the running state (col_end).
struct ColState {
  float nm, nb, alpha;
  va_f32x2 ss, tt;
};

template <bool SCALE, bool ROUND, bool TAIL>
__device__ __forceinline__ float col_val(const f32x4 (&acc)[8][4], int i, int j, int e, int v0, int64_t V) {
  return (TAIL && v0 + i * 16 + e >= V) ? -INFINITY : acc[i][j][e];
}

template <bool SCALE, bool ROUND, bool TAIL>
__device__ __forceinline__ ColState col_begin(const f32x4 (&acc)[8][4], int j, int v0, int64_t V, float m,
                                              float temperature) {
  float rm = col_val<SCALE, ROUND, TAIL>(acc, 0, j, 0, v0, V);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) rm = fmaxf(rm, col_val<SCALE, ROUND, TAIL>(acc, i, j, e, v0, V));
  ColState c;
  c.nm = fmaxf(m, logit_of<SCALE, ROUND>(rm, temperature));
  c.nb = base_of(c.nm);
  c.alpha = __builtin_amdgcn_exp2f(base_of(m) - c.nb);
  c.ss = va_f32x2{0.f, 0.f}, c.tt = va_f32x2{0.f, 0.f};
  return c;
}

// pairs of logits in packed fp32 (v_pk_fma_f32 / v_pk_add_f32): ~3 VALU slots + 1 exp per logit
// instead of ~5 + 1, the halves of ss / tt summed once per tile (33.1-33.2 vs 33.6-33.8 ms at
// 131,072 x 896 x 151,936, tools/f1_ab.py; profiles/r03/f1_packed_epilogue_ab.log)
template <bool SCALE, bool ROUND, bool TAIL, int I0, int I1>
__device__ __forceinline__ void col_blocks(const f32x4 (&acc)[8][4], int j, int v0, int64_t V, float temperature,
                                           ColState &c) {
  const va_f32x2 l2e = {kLog2eF, kLog2eF}, nnb = {-c.nb, -c.nb};
#pragma unroll
  for (int i = I0; i < I1; ++i)
#pragma unroll
    for (int e = 0; e < 4; e += 2) {
      const float a0 = col_val<SCALE, ROUND, TAIL>(acc, i, j, e, v0, V);
      const float a1 = col_val<SCALE, ROUND, TAIL>(acc, i, j, e + 1, v0, V);
      va_f32x2 x;
      if constexpr (ROUND && !SCALE) {  // both roundings in one v_cvt_pk_bf16_f32
        const uint32_t p = pack2_bf16(a0, a1);
        x = va_f32x2{__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
      } else {
        x = va_f32x2{logit_of<SCALE, ROUND>(a0, temperature), logit_of<SCALE, ROUND>(a1, temperature)};
      }
      const va_f32x2 arg = __builtin_elementwise_fma(x, l2e, nnb);
      const va_f32x2 ex = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
      c.ss = c.ss + ex;
      if constexpr (TAIL) {
        x.x = x.x == -INFINITY ? 0.f : x.x;
        x.y = x.y == -INFINITY ? 0.f : x.y;
      }
      c.tt = __builtin_elementwise_fma(ex, x, c.tt);
    }
}

__device__ __forceinline__ void col_end(const ColState &c, float &m, float &s, float &t) {
  s = fmaf(s, c.alpha, c.ss.x + c.ss.y);
  t = fmaf(t, c.alpha, c.tt.x + c.tt.y);
  m = c.nm;
}

template <bool SCALE, bool ROUND, bool TAIL>
__device__ __forceinline__ void t_col_epilogue(const f32x4 (&acc)[8][4], int j, int v0, int64_t V, float (&m)[4],
                                               float (&s)[4], float (&t)[4], float temperature) {
  ColState c = col_begin<SCALE, ROUND, TAIL>(acc, j, v0, V, m[j], temperature);
  col_blocks<SCALE, ROUND, TAIL, 0, 8>(acc, j, v0, V, temperature, c);
  col_end(c, m[j], s[j], t[j]);
}

// The forward's tile epilogue as the deferred sweep calls it: labels (rare, branchy) first, then one
// token column at a time, each ahead of that column's first MFMAs of the next tile.
template <bool SCALE, bool ROUND>
struct FwdEpilogue {
  int lab[4];
  float m[4], s[4], t[4], ll[4];  // ll: the label's logit, -inf until this lane meets it
  float temperature;
  int64_t V;
  int vbase;  // wr * 128 + (lane >> 4) * 4: this lane's first vocab row within a tile
  __device__ __forceinline__ int v0(int64_t vt) const { return static_cast<int>(vt * TB) + vbase; }  // V < 2^31
  __device__ __forceinline__ bool tail(int64_t vt) const { return vt * TB + TB > V; }
  __device__ __forceinline__ void pre(const f32x4 (&acc)[8][4], int64_t vt) {
    t_tile_labels<SCALE, ROUND>(acc, v0(vt), lab, ll, temperature);
  }
  template <bool TAIL>
  __device__ __forceinline__ void col(const f32x4 (&acc)[8][4], int64_t vt, int j) {
    t_col_epilogue<SCALE, ROUND, TAIL>(acc, j, v0(vt), V, m, s, t, temperature);
  }
};

// The persistent transposed sweep shared by the forward and the backward kernels: for each vocab tile
// of [vt_begin, vt_end) it accumulates S^T = W_tile . H_tile^T (256 vocab x 256 tokens) over K in acc,
// calls tile(acc, vt) once the tile is complete, and zeroes acc. acc[i][j][e] holds vocab
// vt * 256 + wr * 128 + (lane >> 4) * 4 + i * 16 + e for token row0 + wc * 64 + j * 16 + (lane & 15).
// Staging addresses: each lane's 4 hidden rows (clamped at N) and its 4 weight-image rows' offsets
// within a tile are fixed for the sweep and computed once; per K-step only the scalar tile / chunk
// base moves (in the last vocab tile, rows past V select row V - 1's address instead).
// DEFER (epilogues that store, VA_TUNE_T256_DEFER): tile() runs after the step's wait + barrier
// instead of before, so its global stores are in flight during the next step's MFMAs and drain at
// that step's wait, instead of the wait for the next step's operands also waiting for them.
template <bool DEFER = false, typename Tile, typename WMap = IdentityRows>
__device__ __forceinline__ void t256_sweep(const uint16_t *__restrict__ hid, int64_t ldh,
                                           const uint16_t *__restrict__ w, int64_t ldw, int64_t N, int K, int64_t V,
                                           int64_t row0, int64_t vt_begin, int64_t vt_end, uint16_t *lds, int wave,
                                           int lane, Tile &&tile, const WMap &wmap = WMap{}) {
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = K / TK;
  const int64_t nsteps = vt_begin < vt_end ? (vt_end - vt_begin) * nk : 0;
  // LDS-DMA through buffer resources: per lane a fixed 32-bit byte offset per staged row, the K-chunk
  // as the scalar offset, and the resource's record count as the bound — rows past N (hidden) or past
  // V (weight, last vocab tile) read 0 (computed, then discarded) with no per-lane clamping
  uint32_t hoff[4], woff[4];
  int ldsoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int g = wave * 4 + i;  // 32 groups of 8 rows (1 KB each)
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    hoff[i] = static_cast<uint32_t>((row * ldh + lc * 8) * 2);
    woff[i] = static_cast<uint32_t>((wmap(row) * ldw + lc * 8) * 2);
    ldsoff[i] = g * 8 * TK;
  }
  const int64_t hrows = N - row0 < TB ? N - row0 : TB;
  const __amdgpu_buffer_rsrc_t hres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t *>(hid + row0 * ldh), 0, static_cast<int>(hrows * ldh * 2), 0x00020000);
  // stage K-chunk kc of vocab tile vs (weight) and of the row block (hidden) into image pair img;
  // branch-free, so that it shares one scheduling region with the step's MFMAs
  auto stage = [&](int64_t vs, int kc, uint16_t *img) {
    const int kb = kc * TK * 2;
    const int64_t wbytes = wmap.window_rows(vs, V) * ldw * 2;
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(w + vs * WMap::kTileStep * ldw), 0,
        static_cast<int>(wbytes < 0x7fffffff ? wbytes : 0x7fffffff), 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(wres, img + ldsoff[i], 16, woff[i], kb, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(hres, img + T_TILE + ldsoff[i], 16, hoff[i], kb, 0, 0);
  };
  f32x4 acc[8][4];

  if (nsteps > 0) stage(vt_begin, 0, lds);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  // step counters kept incrementally: a 64-bit division per step is ~130 scalar instructions (two
  // of them per K-step before round 5: 33.08 -> 32.17 ms at the bench shape, f1_counter_ab.jsonl)
  int kt = 0;             // K-chunks of the current tile done so far
  int64_t vt = vt_begin;  // the tile being accumulated
  for (int64_t st = 0; st < nsteps; ++st) {
    const int buf = static_cast<int>(st & 1);
    const uint16_t *la = lds + buf * 2 * T_TILE;
    const uint16_t *lb = la + T_TILE;
    // FIRST (a tile's first K-step): the first K-half's MFMAs start from a zero accumulator operand
    // instead of acc, so a finished tile needs no 128 v_mov to clear acc (round 6)
    auto kstep = [&](auto first) {
      constexpr bool FIRST = decltype(first)::value;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        // the next step's images, issued between the two K-halves: hipcc then spreads the address, M0
        // and DMA issue over the second half's MFMAs instead of running them ahead of the first (30.1
        // vs 31.5 ms issued before the step's MFMAs, f1_stage_at_ab.jsonl); the last step re-stages a
        // valid tile into the free buffer, unread
        if (q == 1) {
          const bool last = kt + 1 == nk;
          int64_t vs = last ? vt + 1 : vt;
          if (vs >= vt_end) vs = vt_end - 1;
          stage(vs, last ? 0 : kt + 1, lds + (buf ^ 1) * 2 * T_TILE);
        }
        const int c = q * 4 + (lane >> 4);
        auto frag_a = [&](int i) {
          return *reinterpret_cast<const bf16x8 *>(la + t_img_off(wr * 128 + i * 16 + (lane & 15), c));
        };
        auto frag_b = [&](int j) {
          return *reinterpret_cast<const bf16x8 *>(lb + t_img_off(wc * 64 + j * 16 + (lane & 15), c));
        };
        bf16x8 fa[8], fb[4];
#pragma unroll
        for (int i = 0; i < 8; ++i) fa[i] = frag_a(i);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = frag_b(j);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fa[i], fb[j], (FIRST && q == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
      }
    };
    if (kt == 0) kstep(std::true_type{});
    else kstep(std::false_type{});
    const bool fin = kt == nk - 1;
    if (!DEFER && fin) tile(acc, vt);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (DEFER && fin) tile(acc, vt);
    if (fin) {
      kt = 0;
      ++vt;
    } else {
      ++kt;
    }
  }
}

// this workgroup's (row block, vocab range): blocks b, b + 8, ... share an XCD, so with REMAP each XCD
// gets a contiguous run of logical ids (split fastest)
template <bool REMAP>
__device__ __forceinline__ void t256_block(int splits, int tiles_per_split, int64_t V, int64_t &row0,
                                           int64_t &sp, int64_t &vt_begin, int64_t &vt_end) {
  int64_t L = blockIdx.x;
  if (REMAP) {
    const int64_t nl = gridDim.x >> 3;
    L = (L & 7) * nl + (L >> 3);
  }
  const int64_t rb = L / splits;
  sp = L % splits;
  row0 = rb * TB;
  const int64_t n_vt = (V + TB - 1) / TB;
  vt_begin = sp * tiles_per_split;
  vt_end = vt_begin + tiles_per_split < n_vt ? vt_begin + tiles_per_split : n_vt;
}

template <bool SCALE, bool ROUND, bool REMAP>
__global__ __launch_bounds__(T_THREADS, 1) void linear_logprob_t256_kernel(
    const uint16_t *__restrict__ hid, int64_t ldh, const uint16_t *__restrict__ w, int64_t ldw,
    const int64_t *__restrict__ labels, int64_t N, int K, int64_t V, int splits, int tiles_per_split,
    float temperature, float *__restrict__ part, float *__restrict__ label_logit) {
  // ONE LDS array (a second __shared__ object can cost a vmcnt(0) per K-step): 2 staging buffers of
  // (weight, hidden) images; reused for the final merge of the two vocab wave-rows
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * T_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar LDS-DMA bases
  const int wr = wave >> 2, wc = wave & 3;
  int64_t row0, sp, vt_begin, vt_end;
  t256_block<REMAP>(splits, tiles_per_split, V, row0, sp, vt_begin, vt_end);

  // this lane's 4 tokens (columns of the transposed tile), their labels and online states
  FwdEpilogue<SCALE, ROUND> epi;
  epi.temperature = temperature, epi.V = V, epi.vbase = wr * 128 + (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t r = row0 + wc * 64 + j * 16 + (lane & 15);
    const int64_t lb = r < N ? labels[r] : -1;
    epi.lab[j] = (lb >= 0 && lb < V) ? static_cast<int>(lb) : -1;
    epi.m[j] = -INFINITY, epi.s[j] = 0.f, epi.t[j] = 0.f, epi.ll[j] = -INFINITY;
  }

  // acc[i][j][e] = logit of vocab v0 + i * 16 + e for token j of this lane; only the last vocab
  // tile has rows past V (TAIL)
  t256_sweep(hid, ldh, w, ldw, N, K, V, row0, vt_begin, vt_end, lds, wave, lane, [&](f32x4(&acc)[8][4], int64_t vt) {
    epi.pre(acc, vt);
    if (epi.tail(vt)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi.template col<true>(acc, vt, j);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi.template col<false>(acc, vt, j);
    }
  });

  float(&m)[4] = epi.m, (&s)[4] = epi.s, (&t)[4] = epi.t, (&ll)[4] = epi.ll;
  // merge the 4 lane groups (lanes l, l ^ 16, l ^ 32, l ^ 48 hold the same tokens), then the two
  // vocab wave-rows through LDS (free now: every DMA was waited for), in fixed order
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    RowAcc a{m[j], s[j], t[j]};
    float l2 = ll[j];
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      const float om = __shfl_xor(a.m, o, kWave), os = __shfl_xor(a.s, o, kWave), ot = __shfl_xor(a.t, o, kWave);
      merge_state(a, om, os, ot);
      l2 = fmaxf(l2, __shfl_xor(l2, o, kWave));  // one lane of the token holds it (or none: -inf)
    }
    m[j] = a.m, s[j] = a.s, t[j] = a.t, ll[j] = l2;
  }
  float *red = reinterpret_cast<float *>(lds);  // [4 wc][64 tokens][4]: m, s, t, label logit
  if (wr == 1 && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float *p = red + (wc * 64 + j * 16 + lane) * 4;
      p[0] = m[j], p[1] = s[j], p[2] = t[j], p[3] = ll[j];
    }
  }
  __syncthreads();
  if (wr == 0 && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float *p = red + (wc * 64 + j * 16 + lane) * 4;
      RowAcc a{m[j], s[j], t[j]};
      merge_state(a, p[0], p[1], p[2]);
      const int64_t r = row0 + wc * 64 + j * 16 + lane;
      if (r < N) {
        float *o = part + (sp * N + r) * 3;
        o[0] = a.m, o[1] = a.s, o[2] = a.t;
        const float lv = fmaxf(ll[j], p[3]);
        if (lv != -INFINITY) label_logit[r] = lv;  // the split holding the label writes it
      }
    }
  }
}

__global__ __launch_bounds__(256) void linear_logprob_merge_kernel(const float *__restrict__ part,
                                                                   const float *__restrict__ label_logit,
                                                                   const int64_t *__restrict__ labels,
                                                                   int64_t N, int64_t V, int splits,
                                                                   float *__restrict__ logp,
                                                                   float *__restrict__ entropy,
                                                                   float *__restrict__ lse_out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (r >= N) return;
  RowAcc a{-INFINITY, 0.f, 0.f};
  for (int sp = 0; sp < splits; ++sp) {
    const float *p = part + (static_cast<int64_t>(sp) * N + r) * 3;
    merge_state(a, p[0], p[1], p[2]);
  }
  float lse;
  if (a.m == -INFINITY) {
    lse = -INFINITY;
  } else {
    const float corr = -fmaf(a.m, kLog2eF, -base_of(a.m));
    lse = a.m + kLn2F * (__builtin_amdgcn_logf(a.s) + corr);
  }
  if (lse_out) lse_out[r] = lse;
  if (entropy) entropy[r] = lse - a.t / a.s;
  const int64_t lab = labels[r];
  float lp;
  if (lab == -100) lp = 0.f;
  else if (lab < 0 || lab >= V) lp = __builtin_nanf("");
  else lp = label_logit[r] - lse;
  logp[r] = lp;
}

// ---------------------------------------------------------------------------------------------
// Fused backward (f1): the same transposed sweep recomputes each 256 x 256 logits tile and turns it
// into dlogits in registers, written once as bf16 [N, V] (row stride ldd) for the lm_head's two
// backward GEMMs; the logits never exist in HBM. Per element the arithmetic is
// logprob_entropy_bwd's (logprob.hip): with z the logit as the forward saw it (bf16 rounding and
// div_(T) unless fp32 logits), p = 2^(z L - lse L), dz = -p (gh z + kk) (+ g_lp at the label),
// kk = gh (H - lse) + g_lp, dx = dz / T, rounded to bf16 (the reference's fused backward,
// kernels.py:1241-1342, forms the same d_logits per vocab split). Each lane owns 4 consecutive vocab
// entries of a token per (i, j): one 8-byte store. Rows >= N and vocab >= V are computed, not stored.
// One launch covers the vocab range [vbase, vbase + V) of a V_full vocabulary (w points at row vbase,
// dlog column 0 is vocab vbase): the reference's _Split_Dlogits_N loop (kernels.py:1491-1548) runs it
// per range so that only [N, range] dlogits exist at a time. A label counts as valid against V_full
// (its g_lp term enters kk for every range); its own +g_lp lands only in the range that holds it.
// WIDE (dlogits 16-byte aligned, ldd % 8 == 0): the stores go through a wave-private LDS scratch as
// whole row segments (8 lanes x 16 B per token row, 64 vocab columns at a time), as the fused SwiGLU's;
// otherwise each lane stores its 4 columns (8 B) directly.
template <bool SCALE, bool ROUND, bool REMAP, bool WIDE, bool DEFER>
__global__ __launch_bounds__(T_THREADS, 1) void linear_logprob_bwd_t256_kernel(
    const uint16_t *__restrict__ hid, int64_t ldh, const uint16_t *__restrict__ w, int64_t ldw,
    const int64_t *__restrict__ labels, const float *__restrict__ lse_in, const float *__restrict__ ent_in,
    const float *__restrict__ g_logp, const float *__restrict__ g_ent, int64_t N, int K, int64_t V, int64_t V_full,
    int64_t vbase, int splits, int tiles_per_split, float temperature, uint16_t *__restrict__ dlog, int64_t ldd) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * T_TILE + (WIDE ? 8 * 16 * GU_SROW : 0)];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar LDS-DMA bases
  const int wr = wave >> 2, wc = wave & 3;
  int64_t row0, sp, vt_begin, vt_end;
  t256_block<REMAP>(splits, tiles_per_split, V, row0, sp, vt_begin, vt_end);

  // this lane's 4 tokens: label, and the row scalars as logprob_entropy_bwd derives them
  int lab[4];
  float glp[4], gh[4], kk[4], nlb[4];
  uint16_t *drow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t r = row0 + wc * 64 + j * 16 + (lane & 15);
    const bool ok = r < N;
    const int64_t lb = ok ? labels[r] : -1;
    const bool has_lab = lb >= 0 && lb < V_full;
    // the label's column in this range (outside [0, V): never matched below)
    lab[j] = (has_lab && lb >= vbase && lb < vbase + V) ? static_cast<int>(lb - vbase) : -1;
    glp[j] = (ok && g_logp != nullptr && has_lab) ? g_logp[r] : 0.f;
    gh[j] = (ok && g_ent != nullptr) ? g_ent[r] : 0.f;
    const float lse = ok ? lse_in[r] : 0.f;
    const float h = (ok && g_ent != nullptr) ? ent_in[r] : 0.f;
    kk[j] = fmaf(gh[j], h - lse, glp[j]);
    nlb[j] = -lse * kLog2eF;
    drow[j] = ok ? dlog + r * ldd : nullptr;
  }

  uint16_t *scr = lds + 2 * 2 * T_TILE + wave * 16 * GU_SROW;  // WIDE only
  // scratch (16 token rows x 64 columns) -> dlogits columns [c0, c0 + 64) of this wave's token rows j:
  // whole 16-B pieces, the range's last piece (V % 8 == 4) as 8 B
  auto flush = [&](int j, int64_t c0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = h * 8 + (lane >> 3);
      const uint4 v = *reinterpret_cast<const uint4 *>(scr + r * GU_SROW + (lane & 7) * 8);
      const int64_t t = row0 + wc * 64 + j * 16 + r;
      const int64_t col = c0 + (lane & 7) * 8;
      if (t < N && col < V) {
        uint16_t *dst = dlog + t * ldd + col;
        if (col + 8 <= V) *reinterpret_cast<uint4 *>(dst) = v;
        else *reinterpret_cast<uint2 *>(dst) = make_uint2(v.x, v.y);
      }
    }
  };
  t256_sweep<DEFER>(hid, ldh, w, ldw, N, K, V, row0, vt_begin, vt_end, lds, wave, lane, [&](f32x4(&acc)[8][4], int64_t vt) {
    const int v0 = static_cast<int>(vt * TB) + wr * 128 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int vb = v0 + i * 16;  // this lane's 4 vocab entries vb .. vb + 3 (V % 4 == 0)
        float d[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float z = logit_of<SCALE, ROUND>(acc[i][j][e], temperature);
          const float p = __builtin_amdgcn_exp2f(fmaf(z, kLog2eF, nlb[j]));
          d[e] = -p * fmaf(gh[j], z, kk[j]);
        }
        const int dl = lab[j] - vb;
        if (dl >= 0 && dl < 4) {  // one lane per token
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (e == dl) d[e] += glp[j];
        }
        if constexpr (SCALE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = d[e] / temperature;
        }
        uint2 q;
        q.x = pack2_bf16(d[0], d[1]);
        q.y = pack2_bf16(d[2], d[3]);
        if constexpr (WIDE) {
          *reinterpret_cast<uint2 *>(scr + (lane & 15) * GU_SROW + (lane >> 4) * 4 + (i & 3) * 16) = q;
          if ((i & 3) == 3) flush(j, static_cast<int64_t>(vt) * TB + wr * 128 + (i >> 2) * 64);
        } else if (drow[j] != nullptr && vb < V) {
          *reinterpret_cast<uint2 *>(drow[j] + vb) = q;
        }
      }
    }
  });
}

// ------------------------------------------------------------------ gate|up projection + SwiGLU
// The merged gate|up GEMM of a SiLU MLP with its SwiGLU applied in the epilogue: y = bf16(bf16(silu(g))
// * u), g / u = bf16 of the [T, 2F] projection x . W^T (W = [gate rows F | up rows F]), so the [T, 2F]
// projection never reaches HBM (the no-grad pass of the actor's old-logp forward, where nothing keeps
// it for a backward). The same transposed sweep as f1 with the feature index as the MFMA row: a
// 256-row weight image of tile t holds, per wave-row wr, gate features t 128 + wr 64 + [0, 64) in its
// blocks i = 0..3 and the SAME features' up rows in blocks 4..7, so acc[i][j][e] and acc[i + 4][j][e]
// are the gate and up of one (feature, token) in one lane: the epilogue is elementwise, each lane
// storing 4 consecutive features of a token (8 bytes) per (i, j). Per element the arithmetic of
// swiglu_fwd (model_ops.hip), so on exact-arithmetic data the output equals GEMM + swiglu bitwise.
// bf16(bf16(silu(bf16 g)) * bf16 u) for two (g, u) pairs: va_silu's operations (v_mul by -log2 e,
// v_exp_f32, + 1, v_rcp_f32, * g) with the multiplies / adds in packed fp32 and each pair rounded to
// bf16 by one v_cvt_pk_bf16_f32 (the same IEEE results as the scalar form swiglu_fwd uses, ~30 % fewer
// VALU issues in an epilogue that runs while the MFMA pipe idles)
__device__ __forceinline__ va_f32x2 unpack2_bf16(uint32_t p) {
  return va_f32x2{__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
}
__device__ __forceinline__ va_f32x2 swiglu_pair(float g0, float g1, float u0, float u1) {
  const va_f32x2 g = unpack2_bf16(pack2_bf16(g0, g1));
  const va_f32x2 u = unpack2_bf16(pack2_bf16(u0, u1));
  const va_f32x2 a = g * va_f32x2{-kLog2eF, -kLog2eF};
  const va_f32x2 d = va_f32x2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)} + va_f32x2{1.f, 1.f};
  const va_f32x2 sg = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const va_f32x2 sl = g * sg;
  return unpack2_bf16(pack2_bf16(sl.x, sl.y)) * u;
}

struct GateUpRows {
  static constexpr int64_t kTileStep = 128;
  int64_t F;
  // tile vs's window reaches its up rows at F + vs * 128 + [0, 128) (F % 128 == 0: every tile whole)
  __device__ __forceinline__ int64_t window_rows(int64_t, int64_t) const { return F + 128; }
  __device__ __forceinline__ int64_t operator()(int64_t r) const {
    const int64_t t = r >> 8;  // 256 image rows per 128 features
    const int q = static_cast<int>(r & 127), blk = q >> 4;
    const int64_t f = t * 128 + ((r >> 7) & 1) * 64 + (blk & 3) * 16 + (q & 15);
    return blk >= 4 ? F + f : f;
  }
};

// SAVE: also store the projection's g / u (bf16, as the merged GEMM writes them) into gu [T, 2F] for
// the training forward, whose SwiGLU backward needs them: the GEMM + swiglu_fwd pair without the
// swiglu_fwd's re-read of the projection.
template <bool REMAP, bool SAVE, bool DEFER>
__global__ __launch_bounds__(T_THREADS, 1) void gate_up_swiglu_t256_kernel(
    const uint16_t *__restrict__ x, int64_t ldx, const uint16_t *__restrict__ w, int64_t ldw, int64_t T, int K,
    int64_t F, int splits, int tiles_per_split, uint16_t *__restrict__ y, int64_t ldy, uint16_t *__restrict__ gu,
    int64_t ldgu) {
  // the staging images, then a wave-private 16 x GU_SROW scratch per wave for the epilogue's stores
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * T_TILE + 8 * 16 * GU_SROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar LDS-DMA bases
  const int wr = wave >> 2, wc = wave & 3;
  int64_t row0, sp, vt_begin, vt_end;
  t256_block<REMAP>(splits, tiles_per_split, 2 * F, row0, sp, vt_begin, vt_end);
  // Stores through LDS: each lane holds 4 consecutive features of one token per (i, j), i.e. 16 rows x
  // 32 B per wave-instruction; the wave writes its 16-token x 64-feature block of one output into its
  // scratch and reads it back as whole 128-B row segments (8 lanes x 16 B per token row), so every
  // global store writes full cache lines. Wave-private: no barrier (a wave's LDS ops stay in order).
  uint16_t *scr = lds + 2 * 2 * T_TILE + wave * 16 * GU_SROW;
  auto put = [&](int i, float a, float b, float c, float d) {
    uint2 q;
    q.x = pack2_bf16(a, b), q.y = pack2_bf16(c, d);
    *reinterpret_cast<uint2 *>(scr + (lane & 15) * GU_SROW + (lane >> 4) * 4 + i * 16) = q;
  };
  auto flush = [&](int j, uint16_t *out, int64_t ld, int64_t col0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = h * 8 + (lane >> 3);
      const uint4 v = *reinterpret_cast<const uint4 *>(scr + r * GU_SROW + (lane & 7) * 8);
      const int64_t t = row0 + wc * 64 + j * 16 + r;
      if (t < T) *reinterpret_cast<uint4 *>(out + t * ld + col0 + (lane & 7) * 8) = v;
    }
  };
  t256_sweep<DEFER>(
      x, ldx, w, ldw, T, K, 2 * F, row0, vt_begin, vt_end, lds, wave, lane,
      [&](f32x4(&acc)[8][4], int64_t vt) {
        const int64_t c0 = vt * 128 + wr * 64;  // this wave's 64 output features
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const va_f32x2 o01 = swiglu_pair(acc[i][j][0], acc[i][j][1], acc[i + 4][j][0], acc[i + 4][j][1]);
            const va_f32x2 o23 = swiglu_pair(acc[i][j][2], acc[i][j][3], acc[i + 4][j][2], acc[i + 4][j][3]);
            put(i, o01.x, o01.y, o23.x, o23.y);
          }
          flush(j, y, ldy, c0);
          if constexpr (SAVE) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              put(i, acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);  // g: bf16 of the GEMM output
            flush(j, gu, ldgu, c0);
#pragma unroll
            for (int i = 0; i < 4; ++i)
              put(i, acc[i + 4][j][0], acc[i + 4][j][1], acc[i + 4][j][2], acc[i + 4][j][3]);  // u
            flush(j, gu, ldgu, F + c0);
          }
        }
      },
      GateUpRows{F});
}

// ------------------------------------------------------------------ q|k|v projection + bias + RoPE
// The attention block's merged q|k|v GEMM with its bias and rotate-half RoPE in the epilogue, writing
// q [T, Hq D], k / v [T, Hk D] directly (head_dim D = 64): the unfused path's [T, (Hq + 2 Hk) D]
// projection and its rope_qkv_fwd pass disappear. A wave-row's 128 features are two whole heads, and
// a lane's features 16 i + 4 (lane >> 4) + e of a head pair d with d + 32 in blocks i and i + 2, so
// RoPE is lane-local; per element the arithmetic of F.linear's bias epilogue (bf16(acc + b)) and of
// rope_qkv_fwd (model_ops.hip: bf16 after each product, then the sum rounded). Stores through the
// wave-private LDS scratch as whole 128-B head rows. cos / sin [T, D] bf16 (row stride D).
template <bool REMAP, bool DEFER>
__global__ __launch_bounds__(T_THREADS, 1) void qkv_rope_t256_kernel(
    const uint16_t *__restrict__ x, int64_t ldx, const uint16_t *__restrict__ w, int64_t ldw,
    const uint16_t *__restrict__ bias, const uint16_t *__restrict__ cs, const uint16_t *__restrict__ sn, int64_t T,
    int K, int Hq, int Hk, int splits, int tiles_per_split, uint16_t *__restrict__ q, uint16_t *__restrict__ k,
    uint16_t *__restrict__ v) {
  constexpr int D = 64;
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * T_TILE + 8 * 16 * GU_SROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3, g4 = (lane >> 4) * 4;
  const int nh = Hq + 2 * Hk;
  const int64_t NF = static_cast<int64_t>(nh) * D;
  int64_t row0, sp, vt_begin, vt_end;
  t256_block<REMAP>(splits, tiles_per_split, NF, row0, sp, vt_begin, vt_end);
  uint16_t *scr = lds + 2 * 2 * T_TILE + wave * 16 * GU_SROW;
  auto put = [&](int i, const float (&o)[4]) {
    uint2 u;
    u.x = pack2_bf16(o[0], o[1]), u.y = pack2_bf16(o[2], o[3]);
    *reinterpret_cast<uint2 *>(scr + (lane & 15) * GU_SROW + g4 + i * 16) = u;
  };
  auto flush = [&](int j, uint16_t *out, int64_t ld, int64_t col0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = h * 8 + (lane >> 3);
      const uint4 val = *reinterpret_cast<const uint4 *>(scr + r * GU_SROW + (lane & 7) * 8);
      const int64_t t = row0 + wc * 64 + j * 16 + r;
      if (t < T) *reinterpret_cast<uint4 *>(out + t * ld + col0 + (lane & 7) * 8) = val;
    }
  };
  // bf16 lanes of a packed pair, as fp32
  auto lo = [](uint32_t u) { return __uint_as_float(u << 16); };
  auto hi = [](uint32_t u) { return __uint_as_float(u & 0xffff0000u); };
  auto el = [&](const uint2 &u, int e) { return e == 0 ? lo(u.x) : e == 1 ? hi(u.x) : e == 2 ? lo(u.y) : hi(u.y); };
  t256_sweep<DEFER>(x, ldx, w, ldw, T, K, NF, row0, vt_begin, vt_end, lds, wave, lane, [&](f32x4(&acc)[8][4], int64_t vt) {
    const int hb = static_cast<int>(vt * 4) + wr * 2;  // this wave-row's two heads
    uint2 bb[8];  // bias of features 16 i + g4 + 0..3 of the two heads (packed bf16)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t f = static_cast<int64_t>(hb) * D + i * 16 + g4;
      bb[i] = (bias != nullptr && f < NF) ? *reinterpret_cast<const uint2 *>(bias + f) : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t t = row0 + wc * 64 + j * 16 + (lane & 15);
      if (t >= T) t = T - 1;  // rows past T: computed, not stored
      uint2 cc[4], ss[4];  // cos / sin at d = 16 i + g4 + 0..3 (i >= 2: the second half), packed bf16
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cc[i] = *reinterpret_cast<const uint2 *>(cs + t * D + i * 16 + g4);
        ss[i] = *reinterpret_cast<const uint2 *>(sn + t * D + i * 16 + g4);
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int head = hb + hh;
        if (head >= nh) continue;  // wave-uniform: the last tile's unused half
        auto xv = [&](int i, int e) { return round_bf16(acc[4 * hh + i][j][e] + el(bb[4 * hh + i], e)); };
        if (head < Hq + Hk) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            float o1[4], o2[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x1 = xv(i, e), x2 = xv(i + 2, e);
              o1[e] = round_bf16(x1 * el(cc[i], e)) + round_bf16(-x2 * el(ss[i], e));
              o2[e] = round_bf16(x2 * el(cc[i + 2], e)) + round_bf16(x1 * el(ss[i + 2], e));
            }
            put(i, o1);
            put(i + 2, o2);
          }
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float o[4] = {xv(i, 0), xv(i, 1), xv(i, 2), xv(i, 3)};
            put(i, o);
          }
        }
        if (head < Hq) flush(j, q, static_cast<int64_t>(Hq) * D, static_cast<int64_t>(head) * D);
        else if (head < Hq + Hk) flush(j, k, static_cast<int64_t>(Hk) * D, static_cast<int64_t>(head - Hq) * D);
        else flush(j, v, static_cast<int64_t>(Hk) * D, static_cast<int64_t>(head - Hq - Hk) * D);
      }
    }
  });
}

}  // namespace
}  // namespace va

using namespace va;

// va_set_tuning(VA_TUNE_LINEAR_LOGPROB_TILE): 128 (the 128 x 128 register-staged kernel) or 256
// (the 256 x 256 LDS-DMA kernel above)
int g_linear_logprob_tile = 256;
// va_set_tuning(VA_TUNE_T256_DEFER): bit 1 = the gate|up + SwiGLU sweeps, bit 2 = the fused backward's
// dlogits sweep, bit 4 = the q|k|v + RoPE sweep run their tile epilogue after the step's wait
// (t256_sweep DEFER), else before it.
// Default 1: gate|up 2.47 vs 2.52 ms (save form 2.80 vs 2.89) at 151,552 tokens, the dlogits sweep
// 38.5 vs 38.0 ms at 131,072 rows (profiles/r06/al/)
int g_t256_defer = 1;

template <bool SC, bool RD>
static void launch_t256(bool remap, dim3 grid, hipStream_t s, const uint16_t *h16, int64_t ldh, const uint16_t *w16,
                        int64_t ldw, const int64_t *labels, int64_t N, int64_t H, int64_t V, int used, int per,
                        float temperature, float *part, float *label_logit) {
  const auto kern = remap ? linear_logprob_t256_kernel<SC, RD, true> : linear_logprob_t256_kernel<SC, RD, false>;
  hipLaunchKernelGGL(kern, grid, dim3(T_THREADS), 0, s, h16, ldh, w16, ldw, labels, N, static_cast<int>(H), V, used,
                     per, temperature, part, label_logit);
}

extern "C" int64_t va_linear_logprob_workspace_bytes(int64_t N, int splits) {
  return static_cast<int64_t>(sizeof(float)) * (static_cast<int64_t>(splits) * N * 3 + N);
}

extern "C" int va_linear_logprob_fwd(const void *hidden, int64_t ldh, const void *weight, int64_t ldw, int dtype,
                                     const int64_t *labels, int64_t N, int64_t H, int64_t V, float temperature,
                                     int splits, float *logp, float *entropy, float *lse, void *workspace,
                                     void *stream) {
  const bool fp32_logits = (dtype & VA_LOGITS_F32) != 0;
  dtype &= ~VA_LOGITS_F32;
  VA_CHECK_ARG(dtype == VA_BF16, "linear_logprob: only bf16 hidden / weight are implemented");
  VA_CHECK_ARG(N >= 0 && H > 0 && V > 0 && H % BK == 0 && H <= (1 << 20),
               "linear_logprob: need H %% 64 == 0 (H=%lld)", static_cast<long long>(H));
  VA_CHECK_ARG(ldh >= H && ldw >= H && ldh % 8 == 0 && ldw % 8 == 0 && ldh < (1 << 22) && ldw < (1 << 22),
               "linear_logprob: strides must be >= H, %% 8, < 2^22 (32-bit buffer offsets of a 256-row tile)");
  VA_CHECK_ARG(splits >= 1 && splits <= 64, "linear_logprob: splits in [1, 64]");
  VA_CHECK_ARG(temperature > 0.f, "linear_logprob: temperature must be > 0");
  if (N == 0) return VA_OK;
  VA_CHECK_ARG(hidden && weight && labels && logp && workspace, "null pointer argument");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(hidden) % 16 == 0 && reinterpret_cast<uintptr_t>(weight) % 16 == 0,
               "linear_logprob: 16-byte aligned hidden / weight required");
  hipStream_t s = static_cast<hipStream_t>(stream);
  float *part = static_cast<float *>(workspace);
  float *label_logit = part + static_cast<int64_t>(splits) * N * 3;
  if (g_linear_logprob_tile == 256) {
    const int64_t n_vt = (V + TB - 1) / TB;
    const int per = static_cast<int>((n_vt + splits - 1) / splits);
    const int used = static_cast<int>((n_vt + per - 1) / per);  // <= splits: ranges the workspace holds
    const int64_t nwg = ((N + TB - 1) / TB) * used;
    VA_CHECK_ARG(nwg < (int64_t{1} << 31), "linear_logprob: grid too large");
    const dim3 grid(static_cast<unsigned>(nwg));
    const bool remap = nwg % 8 == 0;
    const auto *h16 = static_cast<const uint16_t *>(hidden);
    const auto *w16 = static_cast<const uint16_t *>(weight);
    if (temperature == 1.0f) {
      if (fp32_logits) launch_t256<false, false>(remap, grid, s, h16, ldh, w16, ldw, labels, N, H, V, used, per,
                                                 temperature, part, label_logit);
      else launch_t256<false, true>(remap, grid, s, h16, ldh, w16, ldw, labels, N, H, V, used, per, temperature, part,
                                    label_logit);
    } else {
      if (fp32_logits) launch_t256<true, false>(remap, grid, s, h16, ldh, w16, ldw, labels, N, H, V, used, per,
                                                temperature, part, label_logit);
      else launch_t256<true, true>(remap, grid, s, h16, ldh, w16, ldw, labels, N, H, V, used, per, temperature, part,
                                   label_logit);
    }
    hipLaunchKernelGGL(linear_logprob_merge_kernel, dim3(static_cast<unsigned>((N + 255) / 256)), dim3(256), 0, s,
                       part, label_logit, labels, N, V, used, logp, entropy, lse);
    return check_launch("linear_logprob_fwd");
  }
  const int64_t n_vtiles = (V + BN - 1) / BN;
  const int tiles_per_split = static_cast<int>((n_vtiles + splits - 1) / splits);
  const dim3 grid(static_cast<unsigned>((N + BM - 1) / BM), static_cast<unsigned>(splits));
  if (temperature == 1.0f) {
    hipLaunchKernelGGL((fp32_logits ? linear_logprob_tiles_kernel<false, false>
                                     : linear_logprob_tiles_kernel<false, true>), grid, dim3(256), 0, s,
                       static_cast<const uint16_t *>(hidden), ldh, static_cast<const uint16_t *>(weight), ldw,
                       labels, N, static_cast<int>(H), V, tiles_per_split, temperature, part, label_logit);
  } else {
    hipLaunchKernelGGL((fp32_logits ? linear_logprob_tiles_kernel<true, false>
                                     : linear_logprob_tiles_kernel<true, true>), grid, dim3(256), 0, s,
                       static_cast<const uint16_t *>(hidden), ldh, static_cast<const uint16_t *>(weight), ldw,
                       labels, N, static_cast<int>(H), V, tiles_per_split, temperature, part, label_logit);
  }
  hipLaunchKernelGGL(linear_logprob_merge_kernel, dim3(static_cast<unsigned>((N + 255) / 256)), dim3(256), 0, s,
                     part, label_logit, labels, N, V, splits, logp, entropy, lse);
  return check_launch("linear_logprob_fwd");
}

template <bool SC, bool RD>
static void launch_bwd_t256(bool remap, dim3 grid, hipStream_t s, const uint16_t *h16, int64_t ldh,
                            const uint16_t *w16, int64_t ldw, const int64_t *labels, const float *lse,
                            const float *ent, const float *g_logp, const float *g_ent, int64_t N, int64_t H,
                            int64_t V, int64_t V_full, int64_t vbase, int used, int per, float temperature,
                            uint16_t *dlog, int64_t ldd) {
  const bool wide = ldd % 8 == 0 && reinterpret_cast<uintptr_t>(dlog) % 16 == 0;
  const bool defer = (g_t256_defer & 2) != 0;
  const auto kern = remap ? (wide ? (defer ? linear_logprob_bwd_t256_kernel<SC, RD, true, true, true>
                                           : linear_logprob_bwd_t256_kernel<SC, RD, true, true, false>)
                                  : linear_logprob_bwd_t256_kernel<SC, RD, true, false, false>)
                          : (wide ? (defer ? linear_logprob_bwd_t256_kernel<SC, RD, false, true, true>
                                           : linear_logprob_bwd_t256_kernel<SC, RD, false, true, false>)
                                  : linear_logprob_bwd_t256_kernel<SC, RD, false, false, false>);
  hipLaunchKernelGGL(kern, grid, dim3(T_THREADS), 0, s, h16, ldh, w16, ldw, labels, lse, ent, g_logp, g_ent, N,
                     static_cast<int>(H), V, V_full, vbase, used, per, temperature, dlog, ldd);
}

extern "C" int va_linear_logprob_bwd(const void *hidden, int64_t ldh, const void *weight, int64_t ldw, int dtype,
                                     const int64_t *labels, const float *lse, const float *entropy,
                                     const float *g_logp, const float *g_entropy, int64_t N, int64_t H, int64_t V,
                                     int64_t v_begin, int64_t v_end, float temperature, int splits, void *dlogits,
                                     int64_t ldd, void *stream) {
  const bool fp32_logits = (dtype & VA_LOGITS_F32) != 0;
  dtype &= ~VA_LOGITS_F32;
  VA_CHECK_ARG(dtype == VA_BF16, "linear_logprob_bwd: only bf16 hidden / weight are implemented");
  VA_CHECK_ARG(v_begin >= 0 && v_end > v_begin && v_end <= V,
               "linear_logprob_bwd: vocab range [%lld, %lld) must lie in [0, V=%lld)", static_cast<long long>(v_begin),
               static_cast<long long>(v_end), static_cast<long long>(V));
  const int64_t Vr = v_end - v_begin;  // the range's width: dlogits columns
  VA_CHECK_ARG(N >= 0 && H > 0 && H % TK == 0 && H <= (1 << 20) && Vr % 4 == 0 && V < (int64_t{1} << 31),
               "linear_logprob_bwd: need H %% 64 == 0 and V %% 4 == 0 over the range (H=%lld, V=%lld)",
               static_cast<long long>(H), static_cast<long long>(Vr));
  VA_CHECK_ARG(ldh >= H && ldw >= H && ldh % 8 == 0 && ldw % 8 == 0 && ldh < (1 << 22) && ldw < (1 << 22) &&
                   ldd >= Vr && ldd % 4 == 0,
               "linear_logprob_bwd: strides must be >= H (ldd >= the range), %% 8 (ldd %% 4), < 2^22");
  VA_CHECK_ARG(splits >= 1 && splits <= 64, "linear_logprob_bwd: splits in [1, 64]");
  VA_CHECK_ARG(temperature > 0.f, "linear_logprob_bwd: temperature must be > 0");
  if (N == 0) return VA_OK;
  VA_CHECK_ARG(hidden && weight && labels && lse && dlogits && (g_entropy == nullptr || entropy),
               "null pointer argument");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(hidden) % 16 == 0 && reinterpret_cast<uintptr_t>(weight) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(dlogits) % 8 == 0,
               "linear_logprob_bwd: 16-byte aligned hidden / weight and 8-byte aligned dlogits required");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n_vt = (Vr + TB - 1) / TB;
  const int per = static_cast<int>((n_vt + splits - 1) / splits);
  const int used = static_cast<int>((n_vt + per - 1) / per);
  const int64_t nwg = ((N + TB - 1) / TB) * used;
  VA_CHECK_ARG(nwg < (int64_t{1} << 31), "linear_logprob_bwd: grid too large");
  const dim3 grid(static_cast<unsigned>(nwg));
  const bool remap = nwg % 8 == 0;
  const auto *h16 = static_cast<const uint16_t *>(hidden);
  const auto *w16 = static_cast<const uint16_t *>(weight) + v_begin * ldw;  // the range's first weight row
  auto *d16 = static_cast<uint16_t *>(dlogits);
  if (temperature == 1.0f) {
    if (fp32_logits) launch_bwd_t256<false, false>(remap, grid, s, h16, ldh, w16, ldw, labels, lse, entropy, g_logp,
                                                   g_entropy, N, H, Vr, V, v_begin, used, per, temperature, d16, ldd);
    else launch_bwd_t256<false, true>(remap, grid, s, h16, ldh, w16, ldw, labels, lse, entropy, g_logp, g_entropy, N,
                                      H, Vr, V, v_begin, used, per, temperature, d16, ldd);
  } else {
    if (fp32_logits) launch_bwd_t256<true, false>(remap, grid, s, h16, ldh, w16, ldw, labels, lse, entropy, g_logp,
                                                  g_entropy, N, H, Vr, V, v_begin, used, per, temperature, d16, ldd);
    else launch_bwd_t256<true, true>(remap, grid, s, h16, ldh, w16, ldw, labels, lse, entropy, g_logp, g_entropy, N,
                                     H, Vr, V, v_begin, used, per, temperature, d16, ldd);
  }
  return check_launch("linear_logprob_bwd");
}

static int gate_up_swiglu_impl(const void *x, int64_t ldx, const void *w_gate_up, int64_t ldw, int dtype, int64_t T,
                               int64_t H, int64_t F, int splits, void *y, int64_t ldy, void *gu, int64_t ldgu,
                               void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "gate_up_swiglu: only bf16 is implemented");
  VA_CHECK_ARG(T >= 0 && H > 0 && H % TK == 0 && H <= (1 << 20) && F > 0 && F % 128 == 0 && F < (int64_t{1} << 30),
               "gate_up_swiglu: need H %% 64 == 0 and F %% 128 == 0 (H=%lld, F=%lld)", static_cast<long long>(H),
               static_cast<long long>(F));
  VA_CHECK_ARG(ldx >= H && ldw >= H && ldx % 8 == 0 && ldw % 8 == 0 && ldy >= F && ldy % 8 == 0 && ldx < (1 << 22) &&
                   (F + 128) * ldw * 2 < (int64_t{1} << 31),
               "gate_up_swiglu: strides must be >= H (ldy >= F), %% 8; (F + 128) ldw 2 < 2^31 (32-bit buffer "
               "offsets)");
  VA_CHECK_ARG(gu == nullptr || (ldgu >= 2 * F && ldgu % 8 == 0 && reinterpret_cast<uintptr_t>(gu) % 16 == 0),
               "gate_up_swiglu: the saved projection needs ldgu >= 2F, %% 8, 16-byte alignment");
  VA_CHECK_ARG(splits >= 1 && splits <= 64, "gate_up_swiglu: splits in [1, 64]");
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(x && w_gate_up && y, "null pointer argument");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(w_gate_up) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(y) % 16 == 0,
               "gate_up_swiglu: 16-byte aligned x / weight / y required (whole-line 16-B stores)");
  const int64_t n_vt = F / 128;  // 256 image rows (128 gate + 128 up) per tile
  const int per = static_cast<int>((n_vt + splits - 1) / splits);
  const int used = static_cast<int>((n_vt + per - 1) / per);
  const int64_t nwg = ((T + TB - 1) / TB) * used;
  VA_CHECK_ARG(nwg < (int64_t{1} << 31), "gate_up_swiglu: grid too large");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const auto *x16 = static_cast<const uint16_t *>(x);
  const auto *w16 = static_cast<const uint16_t *>(w_gate_up);
  auto *y16 = static_cast<uint16_t *>(y);
  auto *g16 = static_cast<uint16_t *>(gu);
  const bool remap = nwg % 8 == 0;
  const bool defer = (g_t256_defer & 1) != 0;
  const auto kern =
      gu != nullptr
          ? (remap ? (defer ? gate_up_swiglu_t256_kernel<true, true, true> : gate_up_swiglu_t256_kernel<true, true, false>)
                   : (defer ? gate_up_swiglu_t256_kernel<false, true, true> : gate_up_swiglu_t256_kernel<false, true, false>))
          : (remap ? (defer ? gate_up_swiglu_t256_kernel<true, false, true> : gate_up_swiglu_t256_kernel<true, false, false>)
                   : (defer ? gate_up_swiglu_t256_kernel<false, false, true> : gate_up_swiglu_t256_kernel<false, false, false>));
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(T_THREADS), 0, s, x16, ldx, w16, ldw, T,
                     static_cast<int>(H), F, used, per, y16, ldy, g16, ldgu);
  return check_launch("gate_up_swiglu");
}

extern "C" int va_gate_up_swiglu(const void *x, int64_t ldx, const void *w_gate_up, int64_t ldw, int dtype, int64_t T,
                                 int64_t H, int64_t F, int splits, void *y, int64_t ldy, void *stream) {
  return gate_up_swiglu_impl(x, ldx, w_gate_up, ldw, dtype, T, H, F, splits, y, ldy, nullptr, 0, stream);
}

extern "C" int va_gate_up_swiglu_save(const void *x, int64_t ldx, const void *w_gate_up, int64_t ldw, int dtype,
                                      int64_t T, int64_t H, int64_t F, int splits, void *y, int64_t ldy, void *gu,
                                      int64_t ldgu, void *stream) {
  VA_CHECK_ARG(T == 0 || gu != nullptr, "gate_up_swiglu_save: null projection buffer");
  return gate_up_swiglu_impl(x, ldx, w_gate_up, ldw, dtype, T, H, F, splits, y, ldy, gu, ldgu, stream);
}

extern "C" int va_qkv_rope(const void *x, int64_t ldx, const void *w_qkv, int64_t ldw, const void *bias,
                           const void *cos, const void *sin, int dtype, int64_t T, int64_t H, int Hq, int Hk, int D,
                           int splits, void *q, void *k, void *v, void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "qkv_rope: only bf16 is implemented");
  VA_CHECK_ARG(D == 64, "qkv_rope: head_dim 64 only (got %d)", D);
  VA_CHECK_ARG(T >= 0 && H > 0 && H % TK == 0 && H <= (1 << 20) && Hq > 0 && Hk > 0 && Hq % Hk == 0,
               "qkv_rope: need H %% 64 == 0 and Hq a multiple of Hk");
  const int64_t NF = static_cast<int64_t>(Hq + 2 * Hk) * D;
  VA_CHECK_ARG(ldx >= H && ldw >= H && ldx % 8 == 0 && ldw % 8 == 0 && ldx < (1 << 22) && ldw < (1 << 22),
               "qkv_rope: strides must be >= H, %% 8, < 2^22");
  VA_CHECK_ARG(splits >= 1 && splits <= 64, "qkv_rope: splits in [1, 64]");
  if (T == 0) return VA_OK;
  VA_CHECK_ARG(x && w_qkv && cos && sin && q && k && v, "null pointer argument");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(w_qkv) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(q) % 16 == 0 && reinterpret_cast<uintptr_t>(k) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(v) % 16 == 0 && reinterpret_cast<uintptr_t>(cos) % 8 == 0 &&
                   reinterpret_cast<uintptr_t>(sin) % 8 == 0 && reinterpret_cast<uintptr_t>(bias) % 8 == 0,
               "qkv_rope: 16-byte aligned x / w / q / k / v and 8-byte aligned cos / sin / bias required");
  const int64_t n_vt = (NF + TB - 1) / TB;
  const int per = static_cast<int>((n_vt + splits - 1) / splits);
  const int used = static_cast<int>((n_vt + per - 1) / per);
  const int64_t nwg = ((T + TB - 1) / TB) * used;
  VA_CHECK_ARG(nwg < (int64_t{1} << 31), "qkv_rope: grid too large");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool defer = (g_t256_defer & 4) != 0;
  const auto kern = nwg % 8 == 0 ? (defer ? qkv_rope_t256_kernel<true, true> : qkv_rope_t256_kernel<true, false>)
                                 : (defer ? qkv_rope_t256_kernel<false, true> : qkv_rope_t256_kernel<false, false>);
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nwg)), dim3(T_THREADS), 0, s, static_cast<const uint16_t *>(x),
                     ldx, static_cast<const uint16_t *>(w_qkv), ldw, static_cast<const uint16_t *>(bias),
                     static_cast<const uint16_t *>(cos), static_cast<const uint16_t *>(sin), T, static_cast<int>(H), Hq,
                     Hk, used, per, static_cast<uint16_t *>(q), static_cast<uint16_t *>(k), static_cast<uint16_t *>(v));
  return check_launch("qkv_rope");
}
