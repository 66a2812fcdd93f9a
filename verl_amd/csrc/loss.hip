// Fused PPO clipped policy loss + KL loss + entropy aggregation, and masked aggregation.
//
// Reference semantics (rfahrn/verl):
//   core_algos.py:722-794  compute_policy_loss (dual-clip PPO), the three metrics
//   core_algos.py:686-719  agg_loss (token-mean / seq-mean-token-sum / -token-mean / -sum-norm)
//   core_algos.py:1034-1069 kl_penalty (k1, abs, k2/mse, k3/low_var_kl)
//   torch_functional.py:163-185 masked_sum / masked_mean
//   dp_actor.py:421-470   how the actor combines them (pg - c_H*H_loss + c_kl*kl_loss)
//
// Forward = two launches per micro-batch: a row kernel (one 256-thread workgroup per response
// row) that emits per-row partial sums in fp64, and a one-workgroup finalize that applies the
// aggregation mode and writes the 8-slot output vector. Backward = one elementwise launch
// that reads the row partials and the upstream gradient scalars from device memory (no host
// sync anywhere). Tie / boundary gradients follow torch autograd of the reference expression:
// maximum/minimum give 1/2 to each side on ties, clamp passes gradient inclusive of bounds.
// Bound: launch latency at micro-batch size (8 x 1024), HBM at large B*R.

#include <math.h>

#include "va_common.h"

namespace va {
namespace {

constexpr int kNQ = 8;        // fp64 partial slots per row
constexpr int kTotals = 8;    // fp64 totals slots after the rows

// NaN-propagating maximum / minimum (torch.maximum / torch.minimum semantics).
__device__ __forceinline__ float tmax(float a, float b) {
  return (a != a || b != b) ? __builtin_nanf("") : (a > b ? a : b);
}
__device__ __forceinline__ float tmin(float a, float b) {
  return (a != a || b != b) ? __builtin_nanf("") : (a < b ? a : b);
}
// torch.clamp(x, lo, hi) forward; NaN passes through
__device__ __forceinline__ float tclamp(float x, float lo, float hi) {
  return x != x ? x : (x < lo ? lo : (x > hi ? hi : x));
}
__device__ __forceinline__ float pass_incl(float x, float lo, float hi) {
  return (x >= lo && x <= hi) ? 1.f : 0.f;
}
// gradient share of `a` in maximum(a, b)
__device__ __forceinline__ float gmax_share(float a, float b) {
  return a > b ? 1.f : (a == b ? 0.5f : 0.f);
}

// kl_penalty forward, core_algos.py:1046-1063
template <int KL>
__device__ __forceinline__ float kl_fwd(float lp, float ref) {
  if constexpr (KL == VA_KL_K1) {
    return lp - ref;
  } else if constexpr (KL == VA_KL_ABS) {
    return fabsf(lp - ref);
  } else if constexpr (KL == VA_KL_K2) {
    const float d = lp - ref;
    return 0.5f * (d * d);
  } else if constexpr (KL == VA_KL_K3) {
    const float kc = tclamp(ref - lp, -20.f, 20.f);
    const float ratio = expf(kc);
    const float kld = (ratio - kc) - 1.f;
    return tclamp(kld, -10.f, 10.f);
  } else {
    return 0.f;
  }
}
// d kl / d lp (d kl / d ref is its negative for every estimator)
template <int KL>
__device__ __forceinline__ float kl_dlp(float lp, float ref) {
  if constexpr (KL == VA_KL_K1) {
    return 1.f;
  } else if constexpr (KL == VA_KL_ABS) {
    const float d = lp - ref;
    return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);  // sgn, torch abs backward
  } else if constexpr (KL == VA_KL_K2) {
    return lp - ref;
  } else if constexpr (KL == VA_KL_K3) {
    const float k = ref - lp;
    const float kc = tclamp(k, -20.f, 20.f);
    const float ratio = expf(kc);
    const float kld = (ratio - kc) - 1.f;
    // out = clamp(ratio - kc - 1); d/dkc = ratio - 1; dkc/dk = pass; dk/dlp = -1
    return -(pass_incl(kld, -10.f, 10.f) * (ratio - 1.f) * pass_incl(k, -20.f, 20.f));
  } else {
    return 0.f;
  }
}

struct PolicyElem {
  float pg, clip, negkl, lower;
};

// compute_policy_loss elementwise part, core_algos.py:766-791 (same op order), and the registered
// variants (dispatch dp_actor.py:419-443): gpg core_algos.py:797-815, clip_cov :818-905 (sel = the
// randomly chosen high-covariance tokens whose loss is zeroed, corr = 0), kl_cov :908-972 (sel =
// the top-k covariance tokens that get + coef * |lp - old|). The variants do not clamp lp - old.
__device__ __forceinline__ PolicyElem policy_elem(float old, float lp, float A, float lo,
                                                  float hi, float c, int mode, bool sel,
                                                  float coef) {
  PolicyElem e;
  const float nA = -A;
  if (mode == VA_PL_GPG) {
    e.pg = (-lp) * A;
    e.clip = 0.f;
    e.negkl = 0.f;
    e.lower = 0.f;
    return e;
  }
  if (mode == VA_PL_CLIP_COV || mode == VA_PL_KL_COV) {
    const float d = lp - old;
    const float r = expf(d);
    const float l1 = nA * r;
    if (mode == VA_PL_CLIP_COV) {
      const float l2 = nA * tclamp(r, lo, hi);
      e.pg = tmax(l1, l2) * (sel ? 0.f : 1.f);
      e.clip = sel ? 1.f : 0.f;  // masked_mean((corr == 0).float())
      e.negkl = -d;              // ppo_kl = masked_mean(-negative_approx_kl)
    } else {
      e.pg = sel ? l1 + coef * fabsf(d) : l1;
      e.clip = 0.f;
      e.negkl = fabsf(d);  // the kl_cov metric slot is ppo_kl_abs = masked_mean(|lp - old|)
    }
    e.lower = 0.f;
    return e;
  }
  const float dc = tclamp(lp - old, -20.f, 20.f);
  const float r = expf(dc);
  const float l1 = nA * r;
  const float l2 = nA * tclamp(r, lo, hi);
  const float c1 = tmax(l1, l2);
  const float l3 = nA * c;
  const float c2 = tmin(l3, c1);
  e.pg = (A < 0.f) ? c2 : c1;
  e.clip = (l2 > l1) ? 1.f : 0.f;
  e.negkl = -dc;
  e.lower = ((c1 > l3) ? 1.f : 0.f) * ((A < 0.f) ? 1.f : 0.f);
  return e;
}

// d pg / d lp for a given upstream gradient w on pg (autograd chain order of the reference)
__device__ __forceinline__ float policy_dlp(float w, float old, float lp, float A, float lo,
                                           float hi, float c, int mode, bool sel, float coef) {
  const float nA = -A;
  if (mode == VA_PL_GPG) return -(w * A);  // neg(lp) * A
  if (mode == VA_PL_CLIP_COV) {
    const float d = lp - old;
    const float r = expf(d);
    const float l1 = nA * r;
    const float l2 = nA * tclamp(r, lo, hi);
    const float g_c1 = w * (sel ? 0.f : 1.f);  // maximum(l1, l2) * corr
    const float s1 = gmax_share(l1, l2), s2 = gmax_share(l2, l1);
    const float g_l1 = s1 == 0.5f ? g_c1 / 2.f : g_c1 * s1;
    const float g_l2 = s2 == 0.5f ? g_c1 / 2.f : g_c1 * s2;
    const float g_r = g_l1 * nA + (g_l2 * nA) * pass_incl(r, lo, hi);
    return g_r * r;
  }
  if (mode == VA_PL_KL_COV) {
    const float d = lp - old;
    const float r = expf(d);
    const float g_r = w * nA;
    if (!sel) return g_r * r;
    const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);  // abs backward
    return g_r * r + (w * coef) * sg;
  }
  const float d = lp - old;
  const float dc = tclamp(d, -20.f, 20.f);
  const float r = expf(dc);
  const float l1 = nA * r;
  const float l2 = nA * tclamp(r, lo, hi);
  const float c1 = tmax(l1, l2);
  const float l3 = nA * c;
  float g_c1;
  if (A < 0.f) {
    // c2 = minimum(l3, c1): share of c1
    const float share = c1 < l3 ? 1.f : (c1 == l3 ? 0.5f : 0.f);
    g_c1 = share == 0.5f ? w / 2.f : w * share;
  } else {
    g_c1 = w;
  }
  const float s1 = gmax_share(l1, l2), s2 = gmax_share(l2, l1);
  const float g_l1 = s1 == 0.5f ? g_c1 / 2.f : g_c1 * s1;
  const float g_l2 = s2 == 0.5f ? g_c1 / 2.f : g_c1 * s2;
  const float g_r = g_l1 * nA + (g_l2 * nA) * pass_incl(r, lo, hi);
  return (g_r * r) * pass_incl(d, -20.f, 20.f);
}

// upstream-gradient weight of one element under an aggregation mode (see agg_loss)
__device__ __forceinline__ float agg_weight(int agg, float g, float m, double n_b, double n_tot,
                                            int64_t B, int64_t R) {
  switch (agg) {
    case VA_AGG_TOKEN_MEAN:
      return (g / static_cast<float>(n_tot + 1e-8)) * m;
    case VA_AGG_SEQ_MEAN_TOKEN_SUM:
      return (g / static_cast<float>(B)) * m;
    case VA_AGG_SEQ_MEAN_TOKEN_MEAN:
      return ((g / static_cast<float>(B)) / static_cast<float>(n_b)) * m;
    default:  // VA_AGG_SEQ_MEAN_TOKEN_SUM_NORM
      return (g / static_cast<float>(R)) * m;
  }
}

// ------------------------------------------------------------------ policy loss forward
// Row partial slots q of one row, with the seq-mean-token-mean division applied where it is the
// aggregated quantity (agg_value's per-row term).
__device__ __forceinline__ double agg_term(int agg, double s, double n_b) {
  return agg == VA_AGG_SEQ_MEAN_TOKEN_MEAN ? s / n_b : s;
}
__device__ __forceinline__ double agg_finish(int agg, double acc, double n_tot, int64_t B, int64_t R) {
  switch (agg) {
    case VA_AGG_TOKEN_MEAN: return acc / (n_tot + 1e-8);
    case VA_AGG_SEQ_MEAN_TOKEN_SUM: return acc / static_cast<double>(B);
    case VA_AGG_SEQ_MEAN_TOKEN_MEAN: return acc / static_cast<double>(B);
    default: return acc / static_cast<double>(R);
  }
}

template <int MT, int KL>
__global__ __launch_bounds__(256) void ppo_loss_rows_kernel(
    const float *__restrict__ old_lp, const float *__restrict__ lp, const float *__restrict__ adv,
    const void *__restrict__ mask, const float *__restrict__ ref, const float *__restrict__ ent,
    const uint8_t *__restrict__ sel, int64_t R, float lo, float hi, float c, int agg, int mode,
    float coef, double *__restrict__ part, double *__restrict__ wsum) {
  __shared__ double scratch[4 * 7];
  const int64_t b = blockIdx.x;
  const int64_t base = b * R;
  const bool tok = (agg == VA_AGG_TOKEN_MEAN);
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll 4
  for (int64_t t = threadIdx.x; t < R; t += blockDim.x) {
    const int64_t i = base + t;
    const float m = load_mask<MT>(mask, i);
    const bool mb = (m != 0.f);
    const PolicyElem e =
        policy_elem(old_lp[i], lp[i], adv[i], lo, hi, c, mode, sel != nullptr && sel[i] != 0, coef);
    v[0] += m;
    // masked_sum: where(mask.bool(), x, 0) * mask ; seq modes: x * mask
    v[1] += tok ? (mb ? e.pg : 0.f) * m : e.pg * m;
    v[2] += (mb ? e.clip : 0.f) * m;
    v[3] += (mb ? e.negkl : 0.f) * m;
    v[4] += (mb ? e.lower : 0.f) * m;
    if constexpr (KL != VA_KL_NONE) {
      const float k = kl_fwd<KL>(lp[i], ref[i]);
      v[5] += tok ? (mb ? k : 0.f) * m : k * m;
    }
    if (ent != nullptr) {
      const float h = ent[i];
      v[6] += tok ? (mb ? h : 0.f) * m : h * m;
    }
  }
  block_sum<7>(v, scratch);
  if (threadIdx.x < kNQ) {
    const int q = threadIdx.x;
    const double x = q < 7 ? v[q] : 0.0;
    part[b * kNQ + q] = x;
    wsum[b * kNQ + q] = (q == 1 || q == 5 || q == 6) ? agg_term(agg, x, v[0]) : x;
  }
}

// Streaming forwards, shared tail: the wave-summed slots v[0..NS) of row b go to part[b][0..8)
// (lane q writes slot q, zeros past NS); the slots in term_mask are aggregated per row (agg_term
// with n_b = slot 0) into the lane's running vector `acc`.
template <int NS>
__device__ __forceinline__ void emit_row(const double (&v)[NS], int64_t b, int lane, unsigned term_mask, int agg,
                                         double *__restrict__ part, double &acc) {
  double x = lane < NS ? v[0] : 0.0;
#pragma unroll
  for (int q = 1; q < NS; ++q) x = lane == q ? v[q] : x;
  if (lane < kNQ) part[b * kNQ + lane] = x;
  acc += ((term_mask >> (lane & 31)) & 1u) && lane < kNQ ? agg_term(agg, x, v[0]) : x;
}

// ... then the workgroup's rows in order: the waves' vectors added in wave order into wsum[blockIdx]
__device__ __forceinline__ void wg_sum_vectors(double acc, double *__restrict__ wsum, double *wg /* [16][8] */) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane < kNQ) wg[wave * kNQ + lane] = acc;
  __syncthreads();
  if (threadIdx.x < kNQ) {
    double t = 0.0;
    for (int w = 0; w < nw; ++w) t += wg[w * kNQ + threadIdx.x];
    wsum[static_cast<int64_t>(blockIdx.x) * kNQ + threadIdx.x] = t;
  }
}

// Streaming variant (R % 4 == 0, R <= 256 * JM, 16-byte aligned rows): one wave per row, lane k owns
// the quads t = 256 j + 4 k + {0..3}, so every load is a coalesced 16-byte vector and all of a row's
// loads are issued before the first use (the workgroup-per-row kernel above waits on 4 dependent
// load rounds per row at R = 1024). Same per-element arithmetic; the fp64 row sums are added in a
// different (fixed) order.
// ENT / SEL: the optional entropy rows and token selection exist (compile-time, so that an absent
// input holds no registers: with both absent the k3 / int64-mask kernel drops from 136 VGPRs, 3 waves
// per SIMD, to fewer)
template <int MT, int KL, int JM, bool ENT, bool SEL>
__global__ __launch_bounds__(256) void ppo_loss_rows_vec_kernel(
    const float *__restrict__ old_lp, const float *__restrict__ lp, const float *__restrict__ adv,
    const void *__restrict__ mask, const float *__restrict__ ref, const float *__restrict__ ent,
    const uint8_t *__restrict__ sel, int64_t B, int64_t R, int J, float lo, float hi, float c, int agg,
    int mode, float coef, double *__restrict__ part, double *__restrict__ wsum) {
  __shared__ double wg[4 * kNQ];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const bool tok = (agg == VA_AGG_TOKEN_MEAN);
  double acc = 0.0;  // lane q < 7: slot q of this wave's row, aggregated per row (agg_term)
  // every load is unconditional (compile-time presence): a load under a branch makes the compiler
  // wait for it at the join
  constexpr bool has_ent = ENT, has_sel = SEL;
  {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * nw + wave;
  if (b < B) {
  const int64_t base = b * R;
  float4 o[JM], l[JM], a[JM], rf[JM], h[JM];
  Mask4Raw<MT> mr[JM];
  uint32_t sw[JM];
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int64_t t0 = 256 * j + 4 * lane;
    const bool ok = j < J && t0 < R;
    const int64_t i = base + (ok ? t0 : 0);
    o[j] = ld4(old_lp + i, false);
    l[j] = ld4(lp + i, false);
    a[j] = ld4(adv + i, false);
    if constexpr (KL != VA_KL_NONE) rf[j] = ld4(ref + i, false);
    if constexpr (ENT) h[j] = ld4(ent + i, false);
    mr[j] = load_mask4_raw<MT>(mask, i);
    if constexpr (SEL) sw[j] = *reinterpret_cast<const uint32_t *>(sel + i);
  }
  loads_issued();
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    pin4(o[j]), pin4(l[j]), pin4(a[j]), pin_mask4<MT>(mr[j]);
    if constexpr (ENT) pin4(h[j]);
    if constexpr (SEL) pin1(sw[j]);
    if constexpr (KL != VA_KL_NONE) pin4(rf[j]);
  }
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    if (!(j < J && 256 * j + 4 * lane < R)) continue;
    const float ov[4] = {o[j].x, o[j].y, o[j].z, o[j].w};
    const float lv[4] = {l[j].x, l[j].y, l[j].z, l[j].w};
    const float av[4] = {a[j].x, a[j].y, a[j].z, a[j].w};
    float mv[4];
    cvt_mask4<MT>(mr[j], mv);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float mm = mv[q];
      const bool mb = (mm != 0.f);
      const PolicyElem e =
          policy_elem(ov[q], lv[q], av[q], lo, hi, c, mode, has_sel && ((sw[j] >> (8 * q)) & 0xffu) != 0, coef);
      v[0] += mm;
      v[1] += tok ? (mb ? e.pg : 0.f) * mm : e.pg * mm;
      v[2] += (mb ? e.clip : 0.f) * mm;
      v[3] += (mb ? e.negkl : 0.f) * mm;
      v[4] += (mb ? e.lower : 0.f) * mm;
      if constexpr (KL != VA_KL_NONE) {
        const float rv[4] = {rf[j].x, rf[j].y, rf[j].z, rf[j].w};
        const float k = kl_fwd<KL>(lv[q], rv[q]);
        v[5] += tok ? (mb ? k : 0.f) * mm : k * mm;
      }
      if (has_ent) {
        const float hv[4] = {h[j].x, h[j].y, h[j].z, h[j].w};
        v[6] += tok ? (mb ? hv[q] : 0.f) * mm : hv[q] * mm;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 7; ++q) v[q] = wave_sum(v[q]);
  emit_row<7>(v, b, lane, (1u << 1) | (1u << 5) | (1u << 6), agg, part, acc);
  }
  }
  wg_sum_vectors(acc, wsum, wg);
}

// Totals of the [B, 8] fp64 row partials, read fully coalesced: the flat index f = 8 b + q is
// split over the workgroup's threads so thread t always sees slot q = t % 8 (blockDim % 8 == 0)
// of rows t / 8, t / 8 + blockDim / 8, ...; slots in `term_mask` are aggregated per row with
// agg_term (the row's n_b = slot 0 comes from lane t - q by a shuffle). 16 loads per thread are
// issued before the adds. Every thread gets tot[q] = the sum over rows of slot q (fixed order).
__device__ void sum_row_slots(const double *__restrict__ part, int64_t B, int agg, unsigned term_mask,
                              double (&tot)[kNQ], double *scratch /* [16 waves][8] */) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int q = threadIdx.x & 7;
  const bool term = (term_mask >> q) & 1u;
  const int64_t rows_per_pass = blockDim.x >> 3;
  constexpr int kBatch = 16;
  double acc = 0.0;
  for (int64_t r0 = 0; r0 < B; r0 += kBatch * rows_per_pass) {
    double x[kBatch];
#pragma unroll
    for (int i = 0; i < kBatch; ++i) {
      const int64_t b = r0 + i * rows_per_pass + (threadIdx.x >> 3);
      x[i] = b < B ? part[b * kNQ + q] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < kBatch; ++i) {
      const double nb = __shfl(x[i], lane & ~7, kWave);
      const int64_t b = r0 + i * rows_per_pass + (threadIdx.x >> 3);
      if (b < B) acc += term ? agg_term(agg, x[i], nb) : x[i];
    }
  }
  // lanes holding the same slot: xor 8, 16, 32; then the waves in order
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) acc += __shfl_xor(acc, o, kWave);
  if (lane < 8) scratch[wave * 8 + lane] = acc;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kNQ; ++k) {
    double t = 0.0;
    for (int w = 0; w < nw; ++w) t += scratch[w * 8 + k];
    tot[k] = t;
  }
}

__global__ __launch_bounds__(1024) void ppo_loss_finalize_kernel(const double *__restrict__ wsum,
                                                                int64_t G, int64_t B, int64_t R, int agg,
                                                                int has_kl, int has_ent,
                                                                double *__restrict__ totals,
                                                                float *__restrict__ out) {
  __shared__ double scratch[16 * 8];
  double v[kNQ];
  // slots: 0 n, 1 pg, 2 clip, 3 negkl, 4 lower, 5 kl, 6 ent (1, 5, 6 already aggregated per row)
  sum_row_slots(wsum, G, agg, 0u, v, scratch);
  if (threadIdx.x == 0) {
    const double n = v[0];
    const double den = n + 1e-8;
    out[VA_LOSS_PG] = static_cast<float>(agg_finish(agg, v[1], n, B, R));
    out[VA_LOSS_CLIPFRAC] = static_cast<float>(v[2] / den);
    out[VA_LOSS_PPO_KL] = static_cast<float>(v[3] / den);
    out[VA_LOSS_CLIPFRAC_LOWER] = static_cast<float>(v[4] / den);
    out[VA_LOSS_KL] = has_kl ? static_cast<float>(agg_finish(agg, v[5], n, B, R)) : 0.f;
    out[VA_LOSS_ENTROPY] = has_ent ? static_cast<float>(agg_finish(agg, v[6], n, B, R)) : 0.f;
    out[VA_LOSS_NTOKENS] = static_cast<float>(n);
    out[VA_LOSS_NROWS] = static_cast<float>(B);
  }
  if (threadIdx.x < kTotals) totals[threadIdx.x] = threadIdx.x == 0 ? v[0] : 0.0;
}

// ------------------------------------------------------------------ loss micro-batch segments
// One [B, R] launch can hold several of the reference's loss micro-batches (dp_actor.py:388-470:
// agg_loss per micro-batch of ppo_micro_batch_size_per_gpu rows, each / gradient_accumulation):
// segment s = rows [s * seg_rows, min(B, (s + 1) * seg_rows)) is aggregated on its own, exactly as
// a separate call over those rows would (its own token count n_s, its own row count B_s).
//
// The segments of one launch: `off` (device, n + 1 ascending row offsets, off[0] = 0, off[n] = B,
// every segment non-empty) for variable-size segments (the reference's token-budget micro-batches,
// dp_actor.py:382-384), else uniform runs of `rows` rows (the last one shorter); rows == 0 and off ==
// nullptr: one segment, the whole batch.
struct Segs {
  int64_t rows;
  const int32_t *off;
  int64_t n;
};
__device__ __forceinline__ bool seg_on(const Segs &g) { return g.off != nullptr || g.rows > 0; }
__device__ __forceinline__ void seg_range(const Segs &g, int64_t s, int64_t B, int64_t &b0, int64_t &b1) {
  if (g.off != nullptr) {
    b0 = g.off[s], b1 = g.off[s + 1];
  } else {
    b0 = s * g.rows, b1 = b0 + g.rows < B ? b0 + g.rows : B;
  }
}
// segment of row b (uniform per workgroup: a binary search over the offsets, or a division)
__device__ __forceinline__ int64_t seg_of(const Segs &g, int64_t b) {
  if (g.off == nullptr) return b / g.rows;
  int64_t lo = 0, hi = g.n - 1;  // largest s with off[s] <= b
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (g.off[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Slot q of one segment summed over its rows in a fixed order: lane 8 k + q adds rows b0 + k, b0 + k
// + 8, ... in order, then the 8 k-partials meet by xor 8, 16, 32. Every lane of the wave returns
// the segment sum of its slot q = lane & 7 (term slots aggregated per row with agg_term).
__device__ __forceinline__ double seg_slot_sum(const double *__restrict__ part, int64_t b0, int64_t b1, int agg,
                                               unsigned term_mask) {
  const int lane = threadIdx.x & 63, q = lane & 7, k = lane >> 3;
  const bool term = (term_mask >> q) & 1u;
  constexpr int kU = 4;  // rows per lane whose loads are in flight together (adds stay in row order)
  double acc = 0.0;
  for (int64_t base = b0 + k; base < b1; base += 8 * kU) {
    double x[kU], nb[kU];
#pragma unroll
    for (int i = 0; i < kU; ++i) {
      const int64_t b = base + 8 * i;
      x[i] = b < b1 ? part[b * kNQ + q] : 0.0;
      nb[i] = b < b1 ? part[b * kNQ] : 1.0;
    }
#pragma unroll
    for (int i = 0; i < kU; ++i)
      if (base + 8 * i < b1) acc += term ? agg_term(agg, x[i], nb[i]) : x[i];
  }
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) acc += __shfl_xor(acc, o, kWave);
  return acc;
}

// With segments the 8 batch totals slots after the row partials are zeros (segment workgroup 0
// writes them, so every workspace slot the op returns is written) and segment s's token count n_s
// goes to part[8 B + 8 + s], where the backward reads it (the forward's per-workgroup vectors that
// lived there are consumed by then: the segmented finalize reads the row partials).
__device__ __forceinline__ void seg_write_totals(double *__restrict__ part, int64_t B) {
  if (blockIdx.x == 0 && threadIdx.x < kTotals) part[B * kNQ + threadIdx.x] = 0.0;
}

// One 64-thread workgroup per segment: out[s][VA_LOSS_NOUT] as the one-segment finalize writes it.
__global__ __launch_bounds__(64) void ppo_loss_seg_finalize_kernel(double *__restrict__ part, int64_t B,
                                                                   int64_t R, Segs segs, int agg,
                                                                   int has_kl, int has_ent,
                                                                   float *__restrict__ out) {
  seg_write_totals(part, B);
  const int64_t s = blockIdx.x;
  int64_t b0, b1;
  seg_range(segs, s, B, b0, b1);
  const double x = seg_slot_sum(part, b0, b1, agg, (1u << 1) | (1u << 5) | (1u << 6));
  double v[kNQ];
#pragma unroll
  for (int q = 0; q < kNQ; ++q) v[q] = __shfl(x, q, kWave);
  if (threadIdx.x == 0) {
    const double n = v[0];
    const double den = n + 1e-8;
    const int64_t Bs = b1 - b0;
    part[B * kNQ + kTotals + s] = n;
    float *o = out + s * VA_LOSS_NOUT;
    o[VA_LOSS_PG] = static_cast<float>(agg_finish(agg, v[1], n, Bs, R));
    o[VA_LOSS_CLIPFRAC] = static_cast<float>(v[2] / den);
    o[VA_LOSS_PPO_KL] = static_cast<float>(v[3] / den);
    o[VA_LOSS_CLIPFRAC_LOWER] = static_cast<float>(v[4] / den);
    o[VA_LOSS_KL] = has_kl ? static_cast<float>(agg_finish(agg, v[5], n, Bs, R)) : 0.f;
    o[VA_LOSS_ENTROPY] = has_ent ? static_cast<float>(agg_finish(agg, v[6], n, Bs, R)) : 0.f;
    o[VA_LOSS_NTOKENS] = static_cast<float>(n);
    o[VA_LOSS_NROWS] = static_cast<float>(Bs);
  }
}

// ------------------------------------------------------------------ policy loss backward
// With segments row b belongs to segment s = seg_of(b), whose upstream gradients are g_out[s][*] and
// whose token / row counts replace the batch totals.
template <int MT, int KL>
__global__ __launch_bounds__(256) void ppo_loss_bwd_kernel(
    const float *__restrict__ g_out, const float *__restrict__ old_lp,
    const float *__restrict__ lp, const float *__restrict__ adv, const void *__restrict__ mask,
    const float *__restrict__ ref, const uint8_t *__restrict__ sel, int64_t B, int64_t R, float lo,
    float hi, float c, int agg, int mode, float coef, Segs segs, const double *__restrict__ part,
    float *__restrict__ d_lp, float *__restrict__ d_ent) {
  const int64_t b = blockIdx.y;
  const float *gs = g_out;  // this row's segment's upstream gradients
  double n_tot;
  int64_t Bs = B;
  if (seg_on(segs)) {  // uniform per workgroup: the segment's token count from the forward's finalize
    const int64_t s = seg_of(segs, b);
    int64_t b0, b1;
    seg_range(segs, s, B, b0, b1);
    n_tot = part[B * kNQ + kTotals + s];
    Bs = b1 - b0;
    if (gs) gs += s * VA_LOSS_NOUT;
  } else {
    n_tot = part[B * kNQ + 0];
  }
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= R) return;
  const int64_t i = b * R + t;
  const float g_pg = gs ? gs[VA_LOSS_PG] : 0.f;
  const float g_kl = gs ? gs[VA_LOSS_KL] : 0.f;
  const float g_en = gs ? gs[VA_LOSS_ENTROPY] : 0.f;
  const double n_b = part[b * kNQ + 0];
  const float m = load_mask<MT>(mask, i);
  const bool mb = (m != 0.f);
  const bool tok = (agg == VA_AGG_TOKEN_MEAN);
  // token-mean routes through where(mask.bool(), x, 0): zero where mask == 0
  const float keep = (!tok || mb) ? 1.f : 0.f;
  const float w_pg = agg_weight(agg, g_pg, m, n_b, n_tot, Bs, R) * keep;
  const float x_lp = lp[i];
  float g = policy_dlp(w_pg, old_lp[i], x_lp, adv[i], lo, hi, c, mode, sel != nullptr && sel[i] != 0, coef);
  if constexpr (KL != VA_KL_NONE) {
    const float w_kl = agg_weight(agg, g_kl, m, n_b, n_tot, Bs, R) * keep;
    g += w_kl * kl_dlp<KL>(x_lp, ref[i]);
  }
  d_lp[i] = g;
  if (d_ent != nullptr) d_ent[i] = agg_weight(agg, g_en, m, n_b, n_tot, Bs, R) * keep;
}

// ------------------------------------------------------------------ masked aggregation
// the per-row term of the masked aggregation (masked_sum adds plain row sums)
__device__ __forceinline__ int masked_term_agg(int agg) {
  return agg == VA_REDUCE_MASKED_SUM || agg == VA_REDUCE_ROW_MASKED_MEAN ? VA_AGG_TOKEN_MEAN : agg;
}
// slot 1 carries the sum the mode aggregates: where-form for token-mean / masked_sum / row mean
__device__ __forceinline__ bool masked_where_form(int agg) {
  return agg == VA_AGG_TOKEN_MEAN || agg == VA_REDUCE_MASKED_SUM || agg == VA_REDUCE_ROW_MASKED_MEAN;
}

template <int MT>
__global__ __launch_bounds__(256) void masked_rows_kernel(const float *__restrict__ x,
                                                          const void *__restrict__ mask,
                                                          int64_t R, int agg,
                                                          double *__restrict__ part,
                                                          double *__restrict__ wsum) {
  __shared__ double scratch[4 * 3];
  const int64_t b = blockIdx.x;
  double v[3] = {0, 0, 0};  // n, where-sum, mul-sum
#pragma unroll 4
  for (int64_t t = threadIdx.x; t < R; t += blockDim.x) {
    const int64_t i = b * R + t;
    const float m = load_mask<MT>(mask, i);
    const float xv = x[i];
    v[0] += m;
    v[1] += (m != 0.f ? xv : 0.f) * m;
    v[2] += xv * m;
  }
  block_sum<3>(v, scratch);
  if (threadIdx.x < kNQ) {
    const int q = threadIdx.x;
    const double x = q == 0 ? v[0] : (q == 1 ? (masked_where_form(agg) ? v[1] : v[2]) : 0.0);
    part[b * kNQ + q] = x;
    wsum[b * kNQ + q] = q == 1 ? agg_term(masked_term_agg(agg), x, v[0]) : x;
  }
}

// Streaming form (R % 4 == 0, R <= 256 * JM, 16-byte aligned): one wave per row, 4 rows per
// workgroup summed into one vector for the finalize (as the policy loss).
template <int MT, int JM>
__global__ __launch_bounds__(256) void masked_rows_vec_kernel(const float *__restrict__ x,
                                                              const void *__restrict__ mask, int64_t B,
                                                              int64_t R, int J, int agg,
                                                              double *__restrict__ part,
                                                              double *__restrict__ wsum) {
  __shared__ double wg[4 * kNQ];
  const int lane = threadIdx.x & 63;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  double acc = 0.0;
  if (b < B) {
    const int64_t base = b * R;
    float4 xa[JM];
    Mask4Raw<MT> mr[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      const int64_t t0 = 256 * j + 4 * lane;
      const int64_t i = base + (j < J && t0 < R ? t0 : 0);
      xa[j] = ld4(x + i, false);
      mr[j] = load_mask4_raw<MT>(mask, i);
    }
    double v[3] = {0, 0, 0};  // n, where-sum, mul-sum
#pragma unroll
    for (int j = 0; j < JM; ++j) {  // selects, not a branch: a branch would sink the loads into it
      const bool ok = j < J && 256 * j + 4 * lane < R;
      const float xv[4] = {xa[j].x, xa[j].y, xa[j].z, xa[j].w};
      float mv[4];
      cvt_mask4<MT>(mr[j], mv);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float m = ok ? mv[q] : 0.f, xx = ok ? xv[q] : 0.f;
        v[0] += m;
        v[1] += (m != 0.f ? xx : 0.f) * m;
        v[2] += xx * m;
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) v[q] = wave_sum(v[q]);
    const double rv[2] = {v[0], masked_where_form(agg) ? v[1] : v[2]};
    emit_row<2>(rv, b, lane, 1u << 1, masked_term_agg(agg), part, acc);
  }
  wg_sum_vectors(acc, wsum, wg);
}

__global__ __launch_bounds__(1024) void masked_agg_finalize_kernel(const double *__restrict__ part,
                                                                   const double *__restrict__ wsum, int64_t G,
                                                                   int64_t B, int64_t R, int agg,
                                                                   double *__restrict__ totals,
                                                                   float *__restrict__ out) {
  __shared__ double scratch[16 * 8];
  if (agg == VA_REDUCE_ROW_MASKED_MEAN) {
    for (int64_t b = threadIdx.x; b < B; b += blockDim.x)
      out[b] = static_cast<float>(part[b * kNQ + 1] / (part[b * kNQ + 0] + 1e-8));
    if (threadIdx.x < kTotals) totals[threadIdx.x] = 0.0;
    return;
  }
  double v[kNQ];  // slots: 0 n, 1 sum (already aggregated per row)
  sum_row_slots(wsum, G, agg, 0u, v, scratch);
  if (threadIdx.x == 0) {
    out[0] = static_cast<float>(agg == VA_REDUCE_MASKED_SUM ? v[1] : agg_finish(agg, v[1], v[0], B, R));
  }
  if (threadIdx.x < kTotals) totals[threadIdx.x] = threadIdx.x == 0 ? v[0] : 0.0;
}

template <int MT>
__global__ __launch_bounds__(256) void masked_agg_bwd_kernel(const float *__restrict__ g,
                                                             const void *__restrict__ mask,
                                                             int64_t B, int64_t R, int agg,
                                                             const double *__restrict__ part,
                                                             float *__restrict__ dx) {
  const int64_t b = blockIdx.y;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= R) return;
  const int64_t i = b * R + t;
  const float m = load_mask<MT>(mask, i);
  const bool mb = (m != 0.f);
  float d;
  if (agg == VA_REDUCE_ROW_MASKED_MEAN) {
    d = (g[b] / static_cast<float>(part[b * kNQ + 0] + 1e-8)) * m * (mb ? 1.f : 0.f);
  } else if (agg == VA_REDUCE_MASKED_SUM) {
    d = g[0] * m * (mb ? 1.f : 0.f);
  } else {
    const float keep = (agg != VA_AGG_TOKEN_MEAN || mb) ? 1.f : 0.f;
    d = agg_weight(agg, g[0], m, part[b * kNQ + 0], part[B * kNQ + 0], B, R) * keep;
  }
  dx[i] = d;
}

// ------------------------------------------------------------------ elementwise KL
template <int KL>
__global__ __launch_bounds__(256) void kl_fwd_kernel(const float *__restrict__ lp,
                                                     const float *__restrict__ ref, int64_t n,
                                                     float *__restrict__ out) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    out[i] = kl_fwd<KL>(lp[i], ref[i]);
}
template <int KL>
__global__ __launch_bounds__(256) void kl_bwd_kernel(const float *__restrict__ g,
                                                     const float *__restrict__ lp,
                                                     const float *__restrict__ ref, int64_t n,
                                                     float *__restrict__ d_lp,
                                                     float *__restrict__ d_ref) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const float d = g[i] * kl_dlp<KL>(lp[i], ref[i]);
    if (d_lp) d_lp[i] = d;
    if (d_ref) d_ref[i] = -d;
  }
}

template <int KL, int MT>
__global__ __launch_bounds__(256) void apply_kl_penalty_kernel(
    const float *__restrict__ scores, const float *__restrict__ old_lp,
    const float *__restrict__ ref, const void *__restrict__ mask, int64_t R, float beta,
    float *__restrict__ rewards, float *__restrict__ row_kl) {
  __shared__ double scratch[4 * 2];
  const int64_t b = blockIdx.x;
  double v[2] = {0, 0};
#pragma unroll 4
  for (int64_t t = threadIdx.x; t < R; t += blockDim.x) {
    const int64_t i = b * R + t;
    const float m = load_mask<MT>(mask, i);
    const float kld = kl_fwd<KL>(old_lp[i], ref[i]) * m;  // ray_trainer.py:174-177
    rewards[i] = scores[i] - beta * kld;                  // :180
    v[0] += m;
    v[1] += (m != 0.f ? kld : 0.f) * m;  // masked_mean(kld, mask, axis=-1) :182
  }
  block_sum<2>(v, scratch);
  if (threadIdx.x == 0) row_kl[b] = static_cast<float>(v[1] / (v[0] + 1e-8));
}

// ------------------------------------------------------------------ clipped value loss (critic)
// core_algos.py:992-1031 with verl_F.clip_by_value (torch_functional.py:136-142):
//   vpc = maximum(minimum(vp, v + c), v - c); l1 = (vp - ret)^2; l2 = (vpc - ret)^2
//   vf_loss = 0.5 * agg_loss(maximum(l1, l2)); vf_clipfrac = masked_mean(l2 > l1)
// plus the critic's metric vpred_mean = masked_mean(vp) (dp_critic.py:236-242).
struct ValueElem {
  float loss, clip;
};
__device__ __forceinline__ ValueElem value_elem(float vp, float v, float ret, float c) {
  const float hi = v + c, lo = v - c;
  const float vpc = tmax(tmin(vp, hi), lo);
  const float d1 = vp - ret, d2 = vpc - ret;
  const float l1 = d1 * d1, l2 = d2 * d2;
  ValueElem e;
  e.loss = tmax(l1, l2);
  e.clip = (l2 > l1) ? 1.f : 0.f;
  return e;
}
// d loss / d vp given the upstream weight w on maximum(l1, l2) (torch autograd tie rules)
__device__ __forceinline__ float value_dvp(float w, float vp, float v, float ret, float c) {
  const float hi = v + c, lo = v - c;
  const float m1 = tmin(vp, hi);
  const float vpc = tmax(m1, lo);
  const float d1 = vp - ret, d2 = vpc - ret;
  const float l1 = d1 * d1, l2 = d2 * d2;
  const float s1 = gmax_share(l1, l2), s2 = gmax_share(l2, l1);
  const float g_l1 = s1 == 0.5f ? w / 2.f : w * s1;
  const float g_l2 = s2 == 0.5f ? w / 2.f : w * s2;
  const float g_vpc = g_l2 * (2.f * d2);
  const float sa = gmax_share(m1, lo);  // vpc = maximum(m1, lo)
  const float g_m1 = sa == 0.5f ? g_vpc / 2.f : g_vpc * sa;
  const float sb = vp < hi ? 1.f : (vp == hi ? 0.5f : 0.f);  // m1 = minimum(vp, hi)
  const float g_vp_clip = sb == 0.5f ? g_m1 / 2.f : g_m1 * sb;
  return g_l1 * (2.f * d1) + g_vp_clip;
}

template <int MT>
__global__ __launch_bounds__(256) void value_loss_rows_kernel(
    const float *__restrict__ vp, const float *__restrict__ val, const float *__restrict__ ret,
    const void *__restrict__ mask, int64_t R, float c, int agg, double *__restrict__ part,
    double *__restrict__ wsum) {
  __shared__ double scratch[4 * 4];
  const int64_t b = blockIdx.x;
  const bool tok = (agg == VA_AGG_TOKEN_MEAN);
  double v[4] = {0, 0, 0, 0};  // n, loss, clip, vpred
#pragma unroll 4
  for (int64_t t = threadIdx.x; t < R; t += blockDim.x) {
    const int64_t i = b * R + t;
    const float m = load_mask<MT>(mask, i);
    const bool mb = (m != 0.f);
    const ValueElem e = value_elem(vp[i], val[i], ret[i], c);
    v[0] += m;
    v[1] += tok ? (mb ? e.loss : 0.f) * m : e.loss * m;
    v[2] += (mb ? e.clip : 0.f) * m;
    v[3] += (mb ? vp[i] : 0.f) * m;
  }
  block_sum<4>(v, scratch);
  if (threadIdx.x < kNQ) {
    const int q = threadIdx.x;
    const double x = q < 4 ? v[q] : 0.0;
    part[b * kNQ + q] = x;
    wsum[b * kNQ + q] = q == 1 ? agg_term(agg, x, v[0]) : x;
  }
}

// Streaming form, as the policy loss: one wave per row, 4 rows per workgroup.
template <int MT, int JM>
__global__ __launch_bounds__(256) void value_loss_rows_vec_kernel(
    const float *__restrict__ vp, const float *__restrict__ val, const float *__restrict__ ret,
    const void *__restrict__ mask, int64_t B, int64_t R, int J, float c, int agg, double *__restrict__ part,
    double *__restrict__ wsum) {
  __shared__ double wg[4 * kNQ];
  const int lane = threadIdx.x & 63;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const bool tok = (agg == VA_AGG_TOKEN_MEAN);
  double acc = 0.0;
  if (b < B) {
    const int64_t base = b * R;
    float4 pa[JM], va[JM], ra[JM];
    Mask4Raw<MT> mr[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      const int64_t t0 = 256 * j + 4 * lane;
      const int64_t i = base + (j < J && t0 < R ? t0 : 0);
      pa[j] = ld4(vp + i, false);
      va[j] = ld4(val + i, false);
      ra[j] = ld4(ret + i, false);
      mr[j] = load_mask4_raw<MT>(mask, i);
    }
    loads_issued();
#pragma unroll
    for (int j = 0; j < JM; ++j) pin4(pa[j]), pin4(va[j]), pin4(ra[j]), pin_mask4<MT>(mr[j]);
    double v[4] = {0, 0, 0, 0};  // n, loss, clip, vpred
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      if (!(j < J && 256 * j + 4 * lane < R)) continue;
      const float pv[4] = {pa[j].x, pa[j].y, pa[j].z, pa[j].w};
      const float vv[4] = {va[j].x, va[j].y, va[j].z, va[j].w};
      const float rv[4] = {ra[j].x, ra[j].y, ra[j].z, ra[j].w};
      float mv[4];
      cvt_mask4<MT>(mr[j], mv);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float m = mv[q];
        const bool mb = (m != 0.f);
        const ValueElem e = value_elem(pv[q], vv[q], rv[q], c);
        v[0] += m;
        v[1] += tok ? (mb ? e.loss : 0.f) * m : e.loss * m;
        v[2] += (mb ? e.clip : 0.f) * m;
        v[3] += (mb ? pv[q] : 0.f) * m;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = wave_sum(v[q]);
    emit_row<4>(v, b, lane, 1u << 1, agg, part, acc);
  }
  wg_sum_vectors(acc, wsum, wg);
}

__global__ __launch_bounds__(1024) void value_loss_finalize_kernel(const double *__restrict__ wsum, int64_t G,
                                                                   int64_t B, int64_t R, int agg,
                                                                   double *__restrict__ totals,
                                                                   float *__restrict__ out) {
  __shared__ double scratch[16 * 8];
  double v[kNQ];  // slots: 0 n, 1 loss (already aggregated per row), 2 clip, 3 vpred
  sum_row_slots(wsum, G, agg, 0u, v, scratch);
  if (threadIdx.x == 0) {
    const double n = v[0];
    const double den = n + 1e-8;
    out[VA_VLOSS_LOSS] = 0.5f * static_cast<float>(agg_finish(agg, v[1], n, B, R));
    out[VA_VLOSS_CLIPFRAC] = static_cast<float>(v[2] / den);
    out[VA_VLOSS_VPRED_MEAN] = static_cast<float>(v[3] / den);
    out[VA_VLOSS_NTOKENS] = static_cast<float>(n);
  }
  if (threadIdx.x < kTotals) totals[threadIdx.x] = threadIdx.x == 0 ? v[0] : 0.0;
}

// Loss micro-batch segments as the policy loss (seg_slot_sum): out[s][VA_VLOSS_NOUT] per segment.
__global__ __launch_bounds__(64) void value_loss_seg_finalize_kernel(double *__restrict__ part, int64_t B,
                                                                     int64_t R, Segs segs, int agg,
                                                                     float *__restrict__ out) {
  seg_write_totals(part, B);
  const int64_t s = blockIdx.x;
  int64_t b0, b1;
  seg_range(segs, s, B, b0, b1);
  const double x = seg_slot_sum(part, b0, b1, agg, 1u << 1);
  double v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = __shfl(x, q, kWave);
  if (threadIdx.x == 0) {
    const double n = v[0];
    const double den = n + 1e-8;
    part[B * kNQ + kTotals + s] = n;
    float *o = out + s * VA_VLOSS_NOUT;
    o[VA_VLOSS_LOSS] = 0.5f * static_cast<float>(agg_finish(agg, v[1], n, b1 - b0, R));
    o[VA_VLOSS_CLIPFRAC] = static_cast<float>(v[2] / den);
    o[VA_VLOSS_VPRED_MEAN] = static_cast<float>(v[3] / den);
    o[VA_VLOSS_NTOKENS] = static_cast<float>(n);
  }
}

template <int MT>
__global__ __launch_bounds__(256) void value_loss_bwd_kernel(
    const float *__restrict__ g_out, const float *__restrict__ vp, const float *__restrict__ val,
    const float *__restrict__ ret, const void *__restrict__ mask, int64_t B, int64_t R, float c,
    int agg, Segs segs, const double *__restrict__ part, float *__restrict__ d_vp) {
  const int64_t b = blockIdx.y;
  const float *gs = g_out;  // this row's segment's upstream gradients
  double n_tot;
  int64_t Bs = B;
  if (seg_on(segs)) {  // uniform per workgroup (see ppo_loss_bwd_kernel)
    const int64_t s = seg_of(segs, b);
    int64_t b0, b1;
    seg_range(segs, s, B, b0, b1);
    n_tot = part[B * kNQ + kTotals + s];
    Bs = b1 - b0;
    if (gs) gs += s * VA_VLOSS_NOUT;
  } else {
    n_tot = part[B * kNQ + 0];
  }
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= R) return;
  const int64_t i = b * R + t;
  // vf_loss = 0.5 * agg(.)  ->  d agg = 0.5 * g ;  vpred_mean = masked_mean(vp)
  const float g_loss = gs ? gs[VA_VLOSS_LOSS] * 0.5f : 0.f;
  const float g_mean = gs ? gs[VA_VLOSS_VPRED_MEAN] : 0.f;
  const double n_b = part[b * kNQ + 0];
  const float m = load_mask<MT>(mask, i);
  const bool mb = (m != 0.f);
  const float keep = (agg != VA_AGG_TOKEN_MEAN || mb) ? 1.f : 0.f;
  const float w = agg_weight(agg, g_loss, m, n_b, n_tot, Bs, R) * keep;
  float g = value_dvp(w, vp[i], val[i], ret[i], c);
  g += (g_mean / static_cast<float>(n_tot + 1e-8)) * m * (mb ? 1.f : 0.f);
  d_vp[i] = g;
}

int64_t grid_1d(int64_t n) {
  int64_t g = (n + 255) / 256;
  return g > 8192 ? 8192 : (g < 1 ? 1 : g);
}

}  // namespace
}  // namespace va

using namespace va;

#define VA_DISPATCH_KL(kt, ...)                                                  \
  switch (kt) {                                                                  \
    case VA_KL_NONE: { constexpr int KL = VA_KL_NONE; __VA_ARGS__; break; }       \
    case VA_KL_K1: { constexpr int KL = VA_KL_K1; __VA_ARGS__; break; }           \
    case VA_KL_ABS: { constexpr int KL = VA_KL_ABS; __VA_ARGS__; break; }         \
    case VA_KL_K2: { constexpr int KL = VA_KL_K2; __VA_ARGS__; break; }           \
    case VA_KL_K3: { constexpr int KL = VA_KL_K3; __VA_ARGS__; break; }           \
    default: set_error("unknown kl type %d", (int)(kt)); return VA_E_ARG;         \
  }

// policy / value loss and masked aggregation: [B, 8] row partials | 8 totals | up to B aggregated
// 8-slot vectors (one per forward workgroup) that only the forward's finalize reads
extern "C" int64_t va_ppo_loss_workspace_bytes(int64_t B) {
  return static_cast<int64_t>(sizeof(double)) * (2 * B * kNQ + kTotals);
}
extern "C" int64_t va_agg_workspace_bytes(int64_t B) { return va_ppo_loss_workspace_bytes(B); }

// threads of the one-workgroup finalize: 8 per row slot vector, 16 rows' loads in flight each,
// 256 .. 1,024 (one load pass up to 2,048 rows)
static unsigned finalize_threads(int64_t B) {
  int64_t t = (B * 8 + 15) / 16;
  t = (t + 63) / 64 * 64;
  return static_cast<unsigned>(t < 256 ? 256 : (t > 1024 ? 1024 : t));
}

// va_set_tuning(VA_TUNE_LOSS_VEC): 1 (default) = wave-per-row streaming forward where it applies,
// 0 = the workgroup-per-row kernel (same per-element arithmetic, fp64 row sums in another order)
int g_loss_vec = 1;
// the streaming (wave-per-row, 16-byte quad) forwards apply: VA_TUNE_LOSS_VEC on, R % 4 == 0,
// R <= 2048 and every row base 16-byte aligned
static bool stream_rows(int64_t R, uintptr_t ptr_or) {
  return g_loss_vec != 0 && (R & 3) == 0 && R <= 2048 && (ptr_or & 15) == 0;
}

static bool seg_on_host(const Segs &g) { return g.off != nullptr || g.rows > 0; }

// segments of a policy / value loss launch (see Segs): returns the count S (1 = no segments) or < 0
static int64_t host_segs(int64_t B, int64_t seg_rows, const int32_t *seg_off, int64_t n_seg, Segs &g) {
  g = Segs{0, nullptr, 1};
  if (seg_off != nullptr) {
    if (n_seg < 1 || n_seg > B) return -1;
    g = Segs{0, seg_off, n_seg};
    return n_seg;
  }
  if (seg_rows < 0) return -1;
  if (seg_rows == 0 || seg_rows >= B) return 1;
  g = Segs{seg_rows, nullptr, (B + seg_rows - 1) / seg_rows};
  return g.n;
}

static int check_agg(int agg, bool allow_reduce) {
  const int hi = allow_reduce ? VA_REDUCE_ROW_MASKED_MEAN : VA_AGG_SEQ_MEAN_TOKEN_SUM_NORM;
  VA_CHECK_ARG(agg >= 0 && agg <= hi, "Invalid loss_agg_mode code: %d", agg);
  return VA_OK;
}

static int check_mode(int mode, const uint8_t *sel) {
  VA_CHECK_ARG(mode >= VA_PL_VANILLA && mode <= VA_PL_KL_COV, "unknown policy loss mode %d", mode);
  VA_CHECK_ARG(sel != nullptr || (mode != VA_PL_CLIP_COV && mode != VA_PL_KL_COV),
               "policy loss mode %d needs the token selection", mode);
  return VA_OK;
}

extern "C" int va_ppo_loss_fwd(const float *old_lp, const float *lp, const float *adv,
                               const void *mask, int mask_dtype, const float *ref_lp,
                               const float *entropy, int64_t B, int64_t R, float clip_lo,
                               float clip_hi, float clip_c, int agg_mode, int kl_type,
                               int loss_mode, const uint8_t *sel, float mode_coef,
                               int64_t seg_rows, const int32_t *seg_off, int64_t n_seg, float *out,
                               void *workspace, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty batch (B=%lld, R=%lld)", (long long)B, (long long)R);
  Segs segs;
  const int64_t S = host_segs(B, seg_rows, seg_off, n_seg, segs);
  VA_CHECK_ARG(S >= 1, "bad segments (seg_rows=%lld, n_seg=%lld)", (long long)seg_rows, (long long)n_seg);
  VA_CHECK_ARG(B < (1ll << 31), "B too large");
  VA_CHECK_ARG(old_lp && lp && adv && mask && out && workspace, "null pointer argument");
  VA_CHECK_ARG(kl_type == VA_KL_NONE || ref_lp != nullptr, "ref_lp required for kl_type %d",
               kl_type);
  if (int e = check_agg(agg_mode, false)) return e;
  if (int e = check_mode(loss_mode, sel)) return e;
  hipStream_t s = static_cast<hipStream_t>(stream);
  double *part = static_cast<double *>(workspace);
  const uintptr_t align = reinterpret_cast<uintptr_t>(old_lp) | reinterpret_cast<uintptr_t>(lp) |
                          reinterpret_cast<uintptr_t>(adv) | reinterpret_cast<uintptr_t>(mask) |
                          reinterpret_cast<uintptr_t>(ref_lp) | reinterpret_cast<uintptr_t>(entropy);
  const bool vec = g_loss_vec != 0 && (R & 3) == 0 && R <= 2048 && (align & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(sel) & 3) == 0;
  double *wsum = part + B * kNQ + kTotals;
  int64_t G = B;
  if (vec) {
    const int J = static_cast<int>((R + 255) / 256);
    // 4 rows (waves) per workgroup, whose aggregated vectors are summed in the workgroup, so the
    // finalize's single CU reads B / 4 vectors (a CU reads at ~16-30 GB/s). One row per wave: rows
    // run back to back in a wave (tried: 2 / 4 per wave) hold more registers (3 -> 2 waves per
    // SIMD) and expose their load latency (41 -> 53 us at 8,192 x 1,024)
    constexpr int nw = 4;
    G = (B + nw - 1) / nw;
    const dim3 grid(static_cast<unsigned>(G)), block(64 * nw);
#define VA_PPO_ROWS(JM_, ENT_, SEL_)                                                                            \
  hipLaunchKernelGGL((ppo_loss_rows_vec_kernel<MT, KL, JM_, ENT_, SEL_>), grid, block, 0, s, old_lp, lp, adv, mask, \
                     ref_lp, entropy, sel, B, R, J, clip_lo, clip_hi, clip_c, agg_mode, loss_mode, mode_coef, part,   \
                     wsum)
#define VA_PPO_ROWS_OPT(JM_)                                                                                    \
  if (entropy != nullptr && sel != nullptr) VA_PPO_ROWS(JM_, true, true);                                      \
  else if (entropy != nullptr) VA_PPO_ROWS(JM_, true, false);                                                  \
  else if (sel != nullptr) VA_PPO_ROWS(JM_, false, true);                                                      \
  else VA_PPO_ROWS(JM_, false, false)
    VA_DISPATCH_MASK(mask_dtype, VA_DISPATCH_KL(kl_type, {
      if (J <= 4) {
        VA_PPO_ROWS_OPT(4);
      } else {
        VA_PPO_ROWS_OPT(8);
      }
    }));
#undef VA_PPO_ROWS_OPT
#undef VA_PPO_ROWS
  } else {
    VA_DISPATCH_MASK(mask_dtype, VA_DISPATCH_KL(kl_type, {
      hipLaunchKernelGGL((ppo_loss_rows_kernel<MT, KL>), dim3(B), dim3(256), 0, s, old_lp, lp,
                         adv, mask, ref_lp, entropy, sel, R, clip_lo, clip_hi, clip_c, agg_mode,
                         loss_mode, mode_coef, part, wsum);
    }));
  }
  if (seg_on_host(segs)) {  // several loss micro-batches: one finalize workgroup each
    hipLaunchKernelGGL(ppo_loss_seg_finalize_kernel, dim3(static_cast<unsigned>(S)), dim3(64), 0, s, part, B, R,
                       segs, agg_mode, kl_type != VA_KL_NONE ? 1 : 0, entropy != nullptr ? 1 : 0, out);
    return check_launch("ppo_loss_fwd");
  }
  hipLaunchKernelGGL(ppo_loss_finalize_kernel, dim3(1), dim3(finalize_threads(G)), 0, s, wsum, G, B, R, agg_mode,
                     kl_type != VA_KL_NONE ? 1 : 0, entropy != nullptr ? 1 : 0, part + B * kNQ,
                     out);
  return check_launch("ppo_loss_fwd");
}

extern "C" int va_ppo_loss_bwd(const float *g_out, const float *old_lp, const float *lp,
                               const float *adv, const void *mask, int mask_dtype,
                               const float *ref_lp, int64_t B, int64_t R, float clip_lo,
                               float clip_hi, float clip_c, int agg_mode, int kl_type,
                               int loss_mode, const uint8_t *sel, float mode_coef,
                               int64_t seg_rows, const int32_t *seg_off, int64_t n_seg, const void *workspace,
                               float *d_lp, float *d_entropy, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty batch");
  Segs segs;
  VA_CHECK_ARG(host_segs(B, seg_rows, seg_off, n_seg, segs) >= 1, "bad segments (seg_rows=%lld, n_seg=%lld)",
               (long long)seg_rows, (long long)n_seg);
  VA_CHECK_ARG(B < 65536, "B must be < 65536 for the 2-D backward grid");
  VA_CHECK_ARG(old_lp && lp && adv && mask && workspace && d_lp, "null pointer argument");
  VA_CHECK_ARG(kl_type == VA_KL_NONE || ref_lp != nullptr, "ref_lp required");
  if (int e = check_agg(agg_mode, false)) return e;
  if (int e = check_mode(loss_mode, sel)) return e;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const double *part = static_cast<const double *>(workspace);
  const dim3 grid(static_cast<unsigned>((R + 255) / 256), static_cast<unsigned>(B));
  VA_DISPATCH_MASK(mask_dtype, VA_DISPATCH_KL(kl_type, {
    hipLaunchKernelGGL((ppo_loss_bwd_kernel<MT, KL>), grid, dim3(256), 0, s, g_out, old_lp, lp,
                       adv, mask, ref_lp, sel, B, R, clip_lo, clip_hi, clip_c, agg_mode, loss_mode,
                       mode_coef, segs, part, d_lp, d_entropy);
  }));
  return check_launch("ppo_loss_bwd");
}

extern "C" int va_masked_agg_fwd(const float *x, const void *mask, int mask_dtype, int64_t B,
                                 int64_t R, int mode, float *out, void *workspace,
                                 void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty input");
  VA_CHECK_ARG(x && mask && out && workspace, "null pointer argument");
  if (int e = check_agg(mode, true)) return e;
  hipStream_t s = static_cast<hipStream_t>(stream);
  double *part = static_cast<double *>(workspace);
  double *wsum = part + B * kNQ + kTotals;
  int64_t G = B;
  if (stream_rows(R, reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(mask))) {
    const int J = static_cast<int>((R + 255) / 256);
    G = (B + 3) / 4;
    VA_DISPATCH_MASK(mask_dtype, {
      if (J <= 4)
        hipLaunchKernelGGL((masked_rows_vec_kernel<MT, 4>), dim3(G), dim3(256), 0, s, x, mask, B, R, J, mode, part,
                           wsum);
      else
        hipLaunchKernelGGL((masked_rows_vec_kernel<MT, 8>), dim3(G), dim3(256), 0, s, x, mask, B, R, J, mode, part,
                           wsum);
    });
  } else {
    VA_DISPATCH_MASK(mask_dtype, {
      hipLaunchKernelGGL((masked_rows_kernel<MT>), dim3(B), dim3(256), 0, s, x, mask, R, mode, part, wsum);
    });
  }
  hipLaunchKernelGGL(masked_agg_finalize_kernel, dim3(1), dim3(finalize_threads(mode == VA_REDUCE_ROW_MASKED_MEAN ? B : G)),
                     0, s, part, wsum, G, B, R, mode, part + B * kNQ, out);
  return check_launch("masked_agg_fwd");
}

extern "C" int va_masked_agg_bwd(const float *g, const void *mask, int mask_dtype, int64_t B,
                                 int64_t R, int mode, const void *workspace, float *dx,
                                 void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0 && B < 65536, "bad shape");
  VA_CHECK_ARG(g && mask && workspace && dx, "null pointer argument");
  if (int e = check_agg(mode, true)) return e;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>((R + 255) / 256), static_cast<unsigned>(B));
  VA_DISPATCH_MASK(mask_dtype, {
    hipLaunchKernelGGL((masked_agg_bwd_kernel<MT>), grid, dim3(256), 0, s, g, mask, B, R, mode,
                       static_cast<const double *>(workspace), dx);
  });
  return check_launch("masked_agg_bwd");
}

extern "C" int va_kl_penalty_fwd(const float *lp, const float *ref, int64_t n, int kl_type,
                                 float *kld, void *stream) {
  VA_CHECK_ARG(n >= 0, "n < 0");
  if (n == 0) return VA_OK;
  VA_CHECK_ARG(lp && ref && kld, "null pointer argument");
  VA_CHECK_ARG(kl_type != VA_KL_NONE, "kl_type NONE has no forward");
  hipStream_t s = static_cast<hipStream_t>(stream);
  VA_DISPATCH_KL(kl_type, {
    hipLaunchKernelGGL((kl_fwd_kernel<KL>), dim3(grid_1d(n)), dim3(256), 0, s, lp, ref, n, kld);
  });
  return check_launch("kl_penalty_fwd");
}

extern "C" int va_kl_penalty_bwd(const float *g, const float *lp, const float *ref, int64_t n,
                                 int kl_type, float *d_lp, float *d_ref, void *stream) {
  VA_CHECK_ARG(n >= 0, "n < 0");
  if (n == 0) return VA_OK;
  VA_CHECK_ARG(g && lp && ref, "null pointer argument");
  VA_CHECK_ARG(kl_type != VA_KL_NONE, "kl_type NONE has no backward");
  hipStream_t s = static_cast<hipStream_t>(stream);
  VA_DISPATCH_KL(kl_type, {
    hipLaunchKernelGGL((kl_bwd_kernel<KL>), dim3(grid_1d(n)), dim3(256), 0, s, g, lp, ref, n,
                       d_lp, d_ref);
  });
  return check_launch("kl_penalty_bwd");
}

extern "C" int va_apply_kl_penalty(const float *scores, const float *old_lp, const float *ref_lp,
                                   const void *mask, int mask_dtype, int64_t B, int64_t R,
                                   int kl_type, float beta, float *rewards, float *row_kl,
                                   void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty batch");
  VA_CHECK_ARG(scores && old_lp && ref_lp && mask && rewards && row_kl, "null pointer argument");
  VA_CHECK_ARG(kl_type != VA_KL_NONE, "kl_type NONE");
  hipStream_t s = static_cast<hipStream_t>(stream);
  VA_DISPATCH_MASK(mask_dtype, VA_DISPATCH_KL(kl_type, {
    hipLaunchKernelGGL((apply_kl_penalty_kernel<KL, MT>), dim3(B), dim3(256), 0, s, scores,
                       old_lp, ref_lp, mask, R, beta, rewards, row_kl);
  }));
  return check_launch("apply_kl_penalty");
}

extern "C" int va_value_loss_fwd(const float *vpreds, const float *values, const float *returns,
                                 const void *mask, int mask_dtype, int64_t B, int64_t R,
                                 float cliprange_value, int agg_mode, int64_t seg_rows, const int32_t *seg_off,
                                 int64_t n_seg, float *out, void *workspace, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty batch (B=%lld, R=%lld)", (long long)B, (long long)R);
  Segs segs;
  const int64_t S = host_segs(B, seg_rows, seg_off, n_seg, segs);
  VA_CHECK_ARG(S >= 1, "bad segments (seg_rows=%lld, n_seg=%lld)", (long long)seg_rows, (long long)n_seg);
  VA_CHECK_ARG(B < (1ll << 31), "B too large");
  VA_CHECK_ARG(vpreds && values && returns && mask && out && workspace, "null pointer argument");
  if (int e = check_agg(agg_mode, false)) return e;
  hipStream_t s = static_cast<hipStream_t>(stream);
  double *part = static_cast<double *>(workspace);
  double *wsum = part + B * kNQ + kTotals;
  int64_t G = B;
  if (stream_rows(R, reinterpret_cast<uintptr_t>(vpreds) | reinterpret_cast<uintptr_t>(values) |
                         reinterpret_cast<uintptr_t>(returns) | reinterpret_cast<uintptr_t>(mask))) {
    const int J = static_cast<int>((R + 255) / 256);
    G = (B + 3) / 4;
    VA_DISPATCH_MASK(mask_dtype, {
      if (J <= 4)
        hipLaunchKernelGGL((value_loss_rows_vec_kernel<MT, 4>), dim3(G), dim3(256), 0, s, vpreds, values, returns,
                           mask, B, R, J, cliprange_value, agg_mode, part, wsum);
      else
        hipLaunchKernelGGL((value_loss_rows_vec_kernel<MT, 8>), dim3(G), dim3(256), 0, s, vpreds, values, returns,
                           mask, B, R, J, cliprange_value, agg_mode, part, wsum);
    });
  } else {
    VA_DISPATCH_MASK(mask_dtype, {
      hipLaunchKernelGGL((value_loss_rows_kernel<MT>), dim3(B), dim3(256), 0, s, vpreds, values,
                         returns, mask, R, cliprange_value, agg_mode, part, wsum);
    });
  }
  if (seg_on_host(segs)) {  // several loss micro-batches: one finalize workgroup each
    hipLaunchKernelGGL(value_loss_seg_finalize_kernel, dim3(static_cast<unsigned>(S)), dim3(64), 0, s, part, B, R,
                       segs, agg_mode, out);
    return check_launch("value_loss_fwd");
  }
  hipLaunchKernelGGL(value_loss_finalize_kernel, dim3(1), dim3(finalize_threads(G)), 0, s, wsum, G, B, R, agg_mode,
                     part + B * kNQ, out);
  return check_launch("value_loss_fwd");
}

extern "C" int va_value_loss_bwd(const float *g_out, const float *vpreds, const float *values,
                                 const float *returns, const void *mask, int mask_dtype, int64_t B,
                                 int64_t R, float cliprange_value, int agg_mode, int64_t seg_rows,
                                 const int32_t *seg_off, int64_t n_seg, const void *workspace, float *d_vpreds,
                                 void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0 && B < 65536, "bad shape");
  Segs segs;
  VA_CHECK_ARG(host_segs(B, seg_rows, seg_off, n_seg, segs) >= 1, "bad segments (seg_rows=%lld, n_seg=%lld)",
               (long long)seg_rows, (long long)n_seg);
  VA_CHECK_ARG(vpreds && values && returns && mask && workspace && d_vpreds, "null pointer argument");
  if (int e = check_agg(agg_mode, false)) return e;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>((R + 255) / 256), static_cast<unsigned>(B));
  VA_DISPATCH_MASK(mask_dtype, {
    hipLaunchKernelGGL((value_loss_bwd_kernel<MT>), grid, dim3(256), 0, s, g_out, vpreds, values,
                       returns, mask, B, R, cliprange_value, agg_mode, segs,
                       static_cast<const double *>(workspace), d_vpreds);
  });
  return check_launch("value_loss_bwd");
}
