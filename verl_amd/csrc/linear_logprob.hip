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

template <bool SCALE>
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
          float v = round_bf16(acc[mb][nb][j]);  // the bf16 logits of the unfused path
          if constexpr (SCALE) v = round_bf16(v / temperature);
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

}  // namespace
}  // namespace va

using namespace va;

extern "C" int64_t va_linear_logprob_workspace_bytes(int64_t N, int splits) {
  return static_cast<int64_t>(sizeof(float)) * (static_cast<int64_t>(splits) * N * 3 + N);
}

extern "C" int va_linear_logprob_fwd(const void *hidden, int64_t ldh, const void *weight, int64_t ldw, int dtype,
                                     const int64_t *labels, int64_t N, int64_t H, int64_t V, float temperature,
                                     int splits, float *logp, float *entropy, float *lse, void *workspace,
                                     void *stream) {
  VA_CHECK_ARG(dtype == VA_BF16, "linear_logprob: only bf16 hidden / weight are implemented");
  VA_CHECK_ARG(N >= 0 && H > 0 && V > 0 && H % BK == 0 && H <= (1 << 20),
               "linear_logprob: need H %% 64 == 0 (H=%lld)", static_cast<long long>(H));
  VA_CHECK_ARG(ldh >= H && ldw >= H && ldh % 8 == 0 && ldw % 8 == 0, "linear_logprob: strides must be >= H, %% 8");
  VA_CHECK_ARG(splits >= 1 && splits <= 64, "linear_logprob: splits in [1, 64]");
  VA_CHECK_ARG(temperature > 0.f, "linear_logprob: temperature must be > 0");
  if (N == 0) return VA_OK;
  VA_CHECK_ARG(hidden && weight && labels && logp && workspace, "null pointer argument");
  VA_CHECK_ARG(reinterpret_cast<uintptr_t>(hidden) % 16 == 0 && reinterpret_cast<uintptr_t>(weight) % 16 == 0,
               "linear_logprob: 16-byte aligned hidden / weight required");
  hipStream_t s = static_cast<hipStream_t>(stream);
  float *part = static_cast<float *>(workspace);
  float *label_logit = part + static_cast<int64_t>(splits) * N * 3;
  const int64_t n_vtiles = (V + BN - 1) / BN;
  const int tiles_per_split = static_cast<int>((n_vtiles + splits - 1) / splits);
  const dim3 grid(static_cast<unsigned>((N + BM - 1) / BM), static_cast<unsigned>(splits));
  if (temperature == 1.0f) {
    hipLaunchKernelGGL(linear_logprob_tiles_kernel<false>, grid, dim3(256), 0, s,
                       static_cast<const uint16_t *>(hidden), ldh, static_cast<const uint16_t *>(weight), ldw,
                       labels, N, static_cast<int>(H), V, tiles_per_split, temperature, part, label_logit);
  } else {
    hipLaunchKernelGGL(linear_logprob_tiles_kernel<true>, grid, dim3(256), 0, s,
                       static_cast<const uint16_t *>(hidden), ldh, static_cast<const uint16_t *>(weight), ldw,
                       labels, N, static_cast<int>(H), V, tiles_per_split, temperature, part, label_logit);
  }
  hipLaunchKernelGGL(linear_logprob_merge_kernel, dim3(static_cast<unsigned>((N + 255) / 256)), dim3(256), 0, s,
                     part, label_logit, labels, N, V, splits, logp, entropy, lse);
  return check_launch("linear_logprob_fwd");
}
