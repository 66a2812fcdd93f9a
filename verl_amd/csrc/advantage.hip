// Advantage estimation kernels: per-group outcome advantages (GRPO family) and GAE with the
// batch-global masked whitening.
//
// Reference semantics (rfahrn/verl):
//   core_algos.py:246-308  compute_grpo_outcome_advantage (unmasked row-sum score, per-uid
//                          mean / unbiased std, singleton -> (0, 1), broadcast * mask)
//   core_algos.py:428-476  RLOO;  :376-424 RF++-baseline (mean-only half)
//   core_algos.py:193-241  compute_gae_advantage_return (masked reverse recurrence)
//   torch_functional.py:188-223 masked_var (unbiased; ValueError at mask sum 0/1),
//                          masked_whiten: (x - mean) * rsqrt(var + 1e-8)
//
// GRPO family: row scores (one wave per row) -> per-group coefficients (one wave per group, fp64
// statistics in member order) -> a(b) * mask broadcast. The middle phase runs on all-gathered
// scores when the groups of a batch span data-parallel ranks (trainer/ppo/dp_algos.py).
//
// GAE: one wave per response row, a 256-thread workgroup carries 4 rows. The row's rewards,
// values and mask are staged into LDS (coalesced), each lane owns a contiguous chunk of
// L = ceil(R / 64) steps and composes the chunk's affine map on the state (g, nextvalue);
// a wave-level reverse scan of the 64 maps gives each chunk its incoming state; the lane then
// re-runs its chunk in the reference's exact op order, writing g (raw advantage) and returns.
// The same pass emits per-row (count, sum, M2) in fp64 for the whitening, merged afterwards
// in fixed row order (Chan), so results do not depend on scheduling.

#include <math.h>

#include "va_common.h"

namespace va {
namespace {

constexpr int kPartStride = 3;  // (n, sum, M2) per row, fp64

// ---------------------------------------------------------------- outcome advantages
// Three streaming phases (also the data-parallel decomposition: phase 1 runs on each rank's rows,
// the row scores are all-gathered, phase 2 runs on the global scores, phase 3 on local rows):
//   1) row_scores: one wave per row, unmasked row sum of the rewards (core_algos.py:282) and, for
//      OPO, the response length sum(mask) (core_algos.py:505); every 16-B load of the row issued
//      before the first add;
//   2) group_coef: one wave per prompt group; the members' scores are staged in LDS by the lanes,
//      lane 0 forms the statistics in member order in fp64 (torch.mean / torch.std rounded to
//      fp32), the lanes write each member's coefficient a(b);
//   3) broadcast_rows: adv[b, t] = a(b) * mask[b, t] over the [B, R] matrix, 4 columns per lane.
template <int MT, bool LEN>
__global__ __launch_bounds__(256) void row_scores_kernel(const float *__restrict__ rewards,
                                                         const void *__restrict__ mask, int64_t B,
                                                         int64_t R, bool vec, float *__restrict__ scores,
                                                         float *__restrict__ lengths) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= B) return;
  const float *r = rewards + row * R;
  float acc = 0.f;
  if (vec) {
    const float4 *r4 = reinterpret_cast<const float4 *>(r);
    const int64_t nv = R >> 2;
    int64_t j = lane;
    for (; j + 3 * kWave < nv; j += 4 * kWave) {  // 4 independent 16-B loads in flight per lane
      const float4 a = r4[j], b = r4[j + kWave], c = r4[j + 2 * kWave], d = r4[j + 3 * kWave];
      acc += (a.x + a.y) + (a.z + a.w);
      acc += (b.x + b.y) + (b.z + b.w);
      acc += (c.x + c.y) + (c.z + c.w);
      acc += (d.x + d.y) + (d.z + d.w);
    }
    for (; j < nv; j += kWave) {
      const float4 a = r4[j];
      acc += (a.x + a.y) + (a.z + a.w);
    }
  } else {
    for (int64_t j = lane; j < R; j += kWave) acc += r[j];
  }
  acc = wave_sum(acc);
  float len = 0.f;
  if constexpr (LEN) {
    for (int64_t j = lane; j < R; j += kWave) len += load_mask<MT>(mask, row * R + j);
    len = wave_sum(len);
  }
  if (lane == 0) {
    scores[row] = acc;
    if constexpr (LEN) lengths[row] = len;
  }
}

template <int EST>
__global__ __launch_bounds__(64) void group_coef_kernel(const float *__restrict__ scores,
                                                        const float *__restrict__ lengths,
                                                        const int32_t *__restrict__ order,
                                                        const int32_t *__restrict__ offsets, float eps,
                                                        float *__restrict__ coef) {
  extern __shared__ float s_score[];  // [n] scores, [n] lengths (OPO), 4 floats of group stats
  const int g = blockIdx.x;
  const int beg = offsets[g];
  const int n = offsets[g + 1] - beg;
  const int lane = threadIdx.x;
  float *s_len = s_score + n;
  float *s_stat = s_len + n;
  for (int k = lane; k < n; k += kWave) {
    const int row = order[beg + k];
    s_score[k] = scores[row];
    if constexpr (EST == VA_ADV_OPO) s_len[k] = lengths[row];
  }
  __syncthreads();
  if (lane == 0) {
    // group statistics in member order, fp64, rounded to fp32 as torch.mean / torch.std
    float mean32, std32;
    if (n == 1) {
      mean32 = 0.f;  // core_algos.py:293-295
      std32 = 1.f;
    } else {
      double sum = 0.0;
      for (int k = 0; k < n; ++k) sum += s_score[k];
      const double mean = sum / n;
      double m2 = 0.0;
      for (int k = 0; k < n; ++k) {
        const double d = s_score[k] - mean;
        m2 += d * d;
      }
      mean32 = static_cast<float>(mean);
      std32 = static_cast<float>(sqrt(m2 / (n - 1)));
    }
    s_stat[0] = mean32;
    s_stat[1] = std32;
    if constexpr (EST == VA_ADV_OPO) {
      // length-weighted group baseline, singleton -> 0 (core_algos.py:512-520)
      float bsl = 0.f;
      if (n > 1) {
        double num = 0.0, den = 0.0;
        for (int k = 0; k < n; ++k) {
          num += static_cast<double>(static_cast<float>(s_len[k] * s_score[k]));
          den += s_len[k];
        }
        bsl = static_cast<float>(num) / static_cast<float>(den);
      }
      s_stat[0] = bsl;
    }
    if constexpr (EST == VA_ADV_PASSK || EST == VA_ADV_PASSK_NOSTD) {
      // only the best response gets r_max - r_second_max (core_algos.py:350-368); n >= 2
      int imax = 0;
      for (int k = 1; k < n; ++k)
        if (s_score[k] > s_score[imax]) imax = k;
      float second = -INFINITY;
      for (int k = 0; k < n; ++k)
        if (k != imax && s_score[k] > second) second = s_score[k];
      float a = s_score[imax] - second;
      if constexpr (EST == VA_ADV_PASSK) a = a / (std32 + eps);
      s_stat[2] = a;
      s_stat[3] = static_cast<float>(imax);
    }
  }
  __syncthreads();
  const float mean = s_stat[0], stdv = s_stat[1];
  for (int k = lane; k < n; k += kWave) {
    const float s = s_score[k];
    float a;
    if constexpr (EST == VA_ADV_GRPO) {
      a = (s - mean) / (stdv + eps);
    } else if constexpr (EST == VA_ADV_GRPO_NOSTD || EST == VA_ADV_MEAN_ONLY || EST == VA_ADV_OPO) {
      a = s - mean;
    } else if constexpr (EST == VA_ADV_PASSK || EST == VA_ADV_PASSK_NOSTD) {
      a = (k == static_cast<int>(s_stat[3])) ? s_stat[2] : 0.f;
    } else {  // RLOO, core_algos.py:469-473
      if (n > 1) {
        const float nn = static_cast<float>(n), nm1 = static_cast<float>(n - 1);
        a = (s * nn) / nm1 - (mean * nn) / nm1;
      } else {
        a = s;
      }
    }
    coef[order[beg + k]] = a;
  }
}

// adv[b, t] = coef[b] * mask[b, t] (core_algos.py:302-306); 4 consecutive columns per lane when
// R % 4 == 0 (one 16-B store), two such quads in flight per lane per iteration.
template <int MT, bool VEC>
__global__ __launch_bounds__(256) void broadcast_rows_kernel(const float *__restrict__ coef,
                                                             const void *__restrict__ mask,
                                                             int64_t B, int64_t R,
                                                             float *__restrict__ adv) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if constexpr (VEC) {
    const int64_t nq = (B * R) >> 2;
    for (; i < nq; i += stride) {
      const int64_t e = i << 2;
      const float a = coef[e / R];
      float4 o;
      o.x = a * load_mask<MT>(mask, e + 0);
      o.y = a * load_mask<MT>(mask, e + 1);
      o.z = a * load_mask<MT>(mask, e + 2);
      o.w = a * load_mask<MT>(mask, e + 3);
      reinterpret_cast<float4 *>(adv)[i] = o;
    }
  } else {
    for (; i < B * R; i += stride) adv[i] = coef[i / R] * load_mask<MT>(mask, i);
  }
}

// ---------------------------------------------------------------- GAE chunked scan
// Affine map on (g, nv):  g' = a*g + c*nv + b1 ;  nv' = e*nv + b2   (lower-left entry 0)
struct Aff {
  float a, c, e, b1, b2;
};
// compose: apply `second` after `first`
__device__ __forceinline__ Aff compose(const Aff &second, const Aff &first) {
  Aff r;
  r.a = second.a * first.a;
  r.c = second.a * first.c + second.c * first.e;
  r.e = second.e * first.e;
  r.b1 = second.a * first.b1 + second.c * first.b2 + second.b1;
  r.b2 = second.e * first.b2 + second.b2;
  return r;
}

// Register variant for rows of R <= 64 * 16 steps: lane k owns steps [k L, (k + 1) L) as in the
// LDS kernel (same chunking, so the same arithmetic), but loads its chunk straight into registers
// with every load independent and issued before the first use (the LDS kernel's strided staging
// loop waits on each round trip), scans, and stores from registers.
template <int MT, int LM>
__global__ __launch_bounds__(256) void gae_scan_reg_kernel(
    const float *__restrict__ rew, const float *__restrict__ val, const void *__restrict__ mask,
    int64_t B, int64_t R, int L, float gamma, float gl, float *__restrict__ adv_raw,
    float *__restrict__ ret, double *__restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + wave;
  if (row >= B) return;  // waves are independent: no workgroup barrier below
  const int64_t base = row * R;
  const int64_t t0 = static_cast<int64_t>(lane) * L;
  float r[LM], v[LM], m[LM];
#pragma unroll
  for (int i = 0; i < LM; ++i) {
    const bool ok = i < L && t0 + i < R;
    const int64_t t = ok ? t0 + i : 0;  // clamped address: the loads need no branch
    const float rr = rew[base + t], vv = val[base + t], mm = load_mask<MT>(mask, base + t);
    r[i] = ok ? rr : 0.f;
    v[i] = ok ? vv : 0.f;
    m[i] = ok ? mm : 0.f;
  }
  // 1) the chunk's affine map, steps from the chunk's end down to t0
  Aff F{1.f, 0.f, 1.f, 0.f, 0.f};
#pragma unroll
  for (int i = LM - 1; i >= 0; --i) {
    if (i < L && t0 + i < R) {
      Aff st;
      st.a = m[i] * gl + (1.f - m[i]);
      st.c = m[i] * gamma;
      st.e = 1.f - m[i];
      st.b1 = m[i] * (r[i] - v[i]);
      st.b2 = m[i] * v[i];
      F = compose(st, F);
    }
  }
  // 2) reverse inclusive scan over lanes (as gae_scan_kernel)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    Aff nb;
    nb.a = __shfl_down(F.a, o, kWave);
    nb.c = __shfl_down(F.c, o, kWave);
    nb.e = __shfl_down(F.e, o, kWave);
    nb.b1 = __shfl_down(F.b1, o, kWave);
    nb.b2 = __shfl_down(F.b2, o, kWave);
    if (lane + o < 64) F = compose(F, nb);
  }
  float g = __shfl_down(F.b1, 1, kWave);
  float nv = __shfl_down(F.b2, 1, kWave);
  if (lane == 63) {
    g = 0.f;
    nv = 0.f;
  }
  // 3) re-run the chunk in the reference op order (core_algos.py:229-236); r[i] <- g
#pragma unroll
  for (int i = LM - 1; i >= 0; --i) {
    if (i < L && t0 + i < R) {
      const float delta = (r[i] + gamma * nv) - v[i];
      const float gnew = delta + gl * g;
      nv = v[i] * m[i] + (1.f - m[i]) * nv;
      g = gnew * m[i] + (1.f - m[i]) * g;
      r[i] = g;
    }
  }
  // 4) stores + row partials (n, sum, M2) of g over the mask
  double n = 0.0, sum = 0.0;
#pragma unroll
  for (int i = 0; i < LM; ++i) {
    if (i < L && t0 + i < R) {
      adv_raw[base + t0 + i] = r[i];
      ret[base + t0 + i] = r[i] + v[i];
      n += m[i];
      sum += static_cast<double>((m[i] != 0.f ? r[i] : 0.f) * m[i]);
    }
  }
  n = wave_sum(n);
  sum = wave_sum(sum);
  const double mu = n > 0.0 ? sum / n : 0.0;
  double m2 = 0.0;
#pragma unroll
  for (int i = 0; i < LM; ++i) {
    if (i < L && t0 + i < R && m[i] != 0.f) {
      const double d = static_cast<double>(r[i]) - mu;
      m2 += static_cast<double>(m[i]) * d * d;
    }
  }
  m2 = wave_sum(m2);
  if (lane == 0) {
    part[row * kPartStride + 0] = n;
    part[row * kPartStride + 1] = sum;
    part[row * kPartStride + 2] = m2;
  }
}

template <int MT, bool LDS>
__global__ __launch_bounds__(256) void gae_scan_kernel(
    const float *__restrict__ rew, const float *__restrict__ val, const void *__restrict__ mask,
    int64_t B, int64_t R, int L, float gamma, float gl, float *__restrict__ adv_raw,
    float *__restrict__ ret, double *__restrict__ part) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + wave;
  if (row >= B) return;  // waves are independent: no workgroup barrier below
  const int64_t base = row * R;
  // padded LDS image: step t lives at (t / L) * (L + 1) + t % L  (lane-chunk reads conflict-free)
  const int P = 64 * (L + 1);
  float *sr = lds + static_cast<int64_t>(wave) * 3 * P;
  float *sv = sr + P;
  float *sm = sv + P;
  auto pidx = [L](int64_t t) -> int { return static_cast<int>((t / L) * (L + 1) + t % L); };

  if constexpr (LDS) {
    // coalesced staging in batches of 8 row segments: the batch's 24 loads are all issued before
    // the first LDS write waits on them (one memory round trip per batch, not per segment)
    for (int64_t b0 = 0; b0 < R; b0 += 8 * kWave) {
      float rr[8], vv[8], mm[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t t = b0 + j * kWave + lane;
        const int64_t tc = t < R ? t : R - 1;  // clamped: no branch around the loads
        rr[j] = rew[base + tc];
        vv[j] = val[base + tc];
        mm[j] = load_mask<MT>(mask, base + tc);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t t = b0 + j * kWave + lane;
        if (t < R) {
          const int p = pidx(t);
          sr[p] = rr[j];
          sv[p] = vv[j];
          sm[p] = mm[j];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  auto R_ = [&](int64_t t) -> float { return LDS ? sr[pidx(t)] : rew[base + t]; };
  auto V_ = [&](int64_t t) -> float { return LDS ? sv[pidx(t)] : val[base + t]; };
  auto M_ = [&](int64_t t) -> float { return LDS ? sm[pidx(t)] : load_mask<MT>(mask, base + t); };

  const int64_t t0 = static_cast<int64_t>(lane) * L;
  const int64_t t1 = (t0 + L < R) ? t0 + L : R;

  // 1) compose the chunk's map, processing steps from t1-1 down to t0
  Aff F{1.f, 0.f, 1.f, 0.f, 0.f};
  for (int64_t t = t1 - 1; t >= t0; --t) {
    const float m = M_(t), r = R_(t), v = V_(t);
    Aff s;
    s.a = m * gl + (1.f - m);
    s.c = m * gamma;
    s.e = 1.f - m;
    s.b1 = m * (r - v);
    s.b2 = m * v;
    F = compose(s, F);
  }
  // 2) reverse inclusive scan over lanes: lane k holds G_k o G_{k+1} o ... o G_63
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    Aff nb;
    nb.a = __shfl_down(F.a, o, kWave);
    nb.c = __shfl_down(F.c, o, kWave);
    nb.e = __shfl_down(F.e, o, kWave);
    nb.b1 = __shfl_down(F.b1, o, kWave);
    nb.b2 = __shfl_down(F.b2, o, kWave);
    if (lane + o < 64) F = compose(F, nb);
  }
  // incoming state of chunk k = state after chunks 63..k+1 applied to (0, 0)
  float g = __shfl_down(F.b1, 1, kWave);
  float nv = __shfl_down(F.b2, 1, kWave);
  if (lane == 63) {
    g = 0.f;
    nv = 0.f;
  }
  // 3) re-run the chunk in the reference op order (core_algos.py:229-236)
  for (int64_t t = t1 - 1; t >= t0; --t) {
    const float m = M_(t), r = R_(t), v = V_(t);
    const float delta = (r + gamma * nv) - v;
    const float gnew = delta + gl * g;
    nv = v * m + (1.f - m) * nv;
    g = gnew * m + (1.f - m) * g;
    if constexpr (LDS) {
      sr[pidx(t)] = g;  // reuse the rewards slot for g
    } else {
      adv_raw[base + t] = g;
      ret[base + t] = g + v;
    }
  }
  if constexpr (LDS) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // 4) coalesced stores + row partials (n, sum, M2) of g over the mask
  double n = 0.0, s = 0.0;
  for (int64_t t = lane; t < R; t += kWave) {
    float gv, m, v;
    if constexpr (LDS) {
      const int p = pidx(t);
      gv = sr[p];
      v = sv[p];
      m = sm[p];
      adv_raw[base + t] = gv;
      ret[base + t] = gv + v;
    } else {
      gv = adv_raw[base + t];
      m = load_mask<MT>(mask, base + t);
    }
    n += m;
    s += static_cast<double>((m != 0.f ? gv : 0.f) * m);
  }
  n = wave_sum(n);
  s = wave_sum(s);
  const double mu = n > 0.0 ? s / n : 0.0;
  double m2 = 0.0;
  for (int64_t t = lane; t < R; t += kWave) {
    float gv, m;
    if constexpr (LDS) {
      const int p = pidx(t);
      gv = sr[p];
      m = sm[p];
    } else {
      gv = adv_raw[base + t];
      m = load_mask<MT>(mask, base + t);
    }
    if (m != 0.f) {
      const double d = static_cast<double>(gv) - mu;
      m2 += static_cast<double>(m) * d * d;
    }
  }
  m2 = wave_sum(m2);
  if (lane == 0) {
    part[row * kPartStride + 0] = n;
    part[row * kPartStride + 1] = s;
    part[row * kPartStride + 2] = m2;
  }
}

// Per-row (n, sum, M2) of an arbitrary [B, R] matrix (masked_whiten on non-GAE inputs).
template <int MT>
__global__ __launch_bounds__(256) void row_partials_kernel(const float *__restrict__ x,
                                                           const void *__restrict__ mask,
                                                           int64_t B, int64_t R,
                                                           double *__restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= B) return;
  const int64_t base = row * R;
  double n = 0.0, s = 0.0;
  for (int64_t t = lane; t < R; t += kWave) {
    const float m = load_mask<MT>(mask, base + t);
    n += m;
    s += static_cast<double>((m != 0.f ? x[base + t] : 0.f) * m);
  }
  n = wave_sum(n);
  s = wave_sum(s);
  const double mu = n > 0.0 ? s / n : 0.0;
  double m2 = 0.0;
  for (int64_t t = lane; t < R; t += kWave) {
    const float m = load_mask<MT>(mask, base + t);
    if (m != 0.f) {
      const double d = static_cast<double>(x[base + t]) - mu;
      m2 += static_cast<double>(m) * d * d;
    }
  }
  m2 = wave_sum(m2);
  if (lane == 0) {
    part[row * kPartStride + 0] = n;
    part[row * kPartStride + 1] = s;
    part[row * kPartStride + 2] = m2;
  }
}

// Merge K (n, sum, M2) triples; emit the merged triple and the fp32 whitening stats
// {mean, rsqrt(var + 1e-8), n, error_flag} with the reference's formulas. Each thread merges a
// contiguous slice, then a fixed binary tree in LDS: the merge order depends only on K, so the
// result is deterministic run to run.
__global__ __launch_bounds__(256) void whiten_finalize_kernel(const double *__restrict__ part,
                                                              int64_t K, double *__restrict__ merged,
                                                              float *__restrict__ stats) {
  __shared__ double sh[256 * 3];
  Moments acc{0.0, 0.0, 0.0};
  const int64_t per = (K + blockDim.x - 1) / blockDim.x;
  const int64_t lo = threadIdx.x * per, hi = (lo + per < K) ? lo + per : K;
  for (int64_t k = lo; k < hi; ++k) {
    const double n = part[k * kPartStride + 0];
    Moments mk{n, n > 0.0 ? part[k * kPartStride + 1] / n : 0.0, part[k * kPartStride + 2]};
    acc = merge_moments(acc, mk);
  }
  sh[threadIdx.x * 3 + 0] = acc.n;
  sh[threadIdx.x * 3 + 1] = acc.mean;
  sh[threadIdx.x * 3 + 2] = acc.m2;
  __syncthreads();
  for (unsigned s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const unsigned a = threadIdx.x, b = threadIdx.x + s;
      const Moments m = merge_moments(Moments{sh[a * 3], sh[a * 3 + 1], sh[a * 3 + 2]},
                                      Moments{sh[b * 3], sh[b * 3 + 1], sh[b * 3 + 2]});
      sh[a * 3] = m.n;
      sh[a * 3 + 1] = m.mean;
      sh[a * 3 + 2] = m.m2;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const Moments tot{sh[0], sh[1], sh[2]};
    const double n = tot.n;
    merged[0] = n;
    merged[1] = tot.mean * n;
    merged[2] = tot.m2;
    // torch_functional.py:171-185, 188-223
    const double mean = (tot.mean * n) / (n + 1e-8);
    const double dm = tot.mean - mean;
    const double var_b = (tot.m2 + n * dm * dm) / (n + 1e-8);
    float flag = 0.f;
    double var = var_b;
    if (n == 0.0) flag = 1.f;
    else if (n == 1.0) flag = 2.f;
    else var = var_b * (n / (n - 1.0));
    const float var32 = static_cast<float>(var);
    stats[0] = static_cast<float>(mean);
    stats[1] = 1.0f / sqrtf(var32 + 1e-8f);
    stats[2] = static_cast<float>(n);
    stats[3] = flag;
  }
}

template <int MT, bool POSTMASK>
__global__ __launch_bounds__(256) void whiten_apply_kernel(float *__restrict__ x,
                                                           const float *__restrict__ stats,
                                                           const void *__restrict__ mask,
                                                           int64_t n) {
  const float mean = stats[0], rstd = stats[1];
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float v = (x[i] - mean) * rstd;
    if constexpr (POSTMASK) v = v * load_mask<MT>(mask, i);
    x[i] = v;
  }
}

// ---------------------------------------------------------------- discounted returns (RF++ / ReMax)
// One wave per row; lane k owns the contiguous chunk [kL, (k+1)L). The per-step state map is
// affine, s -> A + C s:
//   RF++  (core_algos.py:553-560): out_t = r_t + gamma * s;  s <- out_t * m_t
//   ReMax (core_algos.py:597-599): out_t = s + r_t * m_t   (reverse cumsum of r * m);  s <- out_t
// Chunk maps are composed per lane, a 6-step wave reverse scan gives every chunk its incoming
// state, and each lane re-runs its chunk in the reference's op order.
template <int MT, int MODE>
__global__ __launch_bounds__(256) void discounted_returns_kernel(
    const float *__restrict__ rew, const void *__restrict__ mask, int64_t B, int64_t R, int L,
    float gamma, const float *__restrict__ baselines, float *__restrict__ ret, float *__restrict__ adv) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + wave;
  if (row >= B) return;
  const int64_t base = row * R;
  const int64_t t0 = static_cast<int64_t>(lane) * L;
  const int64_t t1 = (t0 + L < R) ? t0 + L : R;
  float A = 0.f, C = 1.f;  // chunk map, applied to the state entering its last step
  for (int64_t t = t1 - 1; t >= t0; --t) {
    const float r = rew[base + t], m = load_mask<MT>(mask, base + t);
    float a, c;
    if constexpr (MODE == VA_RET_RFPP) {
      a = r * m;
      c = gamma * m;
    } else {
      a = r * m;
      c = 1.f;
    }
    A = a + c * A;  // step o (chunk so far)
    C = c * C;
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float nA = __shfl_down(A, o, kWave), nC = __shfl_down(C, o, kWave);
    if (lane + o < 64) {  // (this chunk) o (chunks after it): s -> A + C (nA + nC s)
      A = A + C * nA;
      C = C * nC;
    }
  }
  float st = __shfl_down(A, 1, kWave);  // state after chunks 63..k+1 from 0
  if (lane == 63) st = 0.f;
  const float b = (MODE == VA_RET_REMAX) ? baselines[row] : 0.f;
  for (int64_t t = t1 - 1; t >= t0; --t) {
    const float r = rew[base + t], m = load_mask<MT>(mask, base + t);
    float out;
    if constexpr (MODE == VA_RET_RFPP) {
      out = r + gamma * st;
      st = out * m;
    } else {
      out = st + r * m;
      st = out;
      adv[base + t] = out - b * m;  // core_algos.py:600
    }
    ret[base + t] = out;
  }
}

int gae_lds_bytes(int L, int waves) { return waves * 3 * 64 * (L + 1) * 4; }

}  // namespace
}  // namespace va

using namespace va;

extern "C" int va_row_scores(const float *rewards, const void *mask, int mask_dtype, int64_t B,
                             int64_t R, float *scores, float *lengths, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "bad shape (B=%lld R=%lld)", (long long)B, (long long)R);
  VA_CHECK_ARG(rewards && scores && (!lengths || mask), "null pointer argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>((B + 3) / 4)), block(256);
  const bool vec = (R & 3) == 0 && (reinterpret_cast<uintptr_t>(rewards) & 15) == 0;
  if (lengths) {
    VA_DISPATCH_MASK(mask_dtype, {
      hipLaunchKernelGGL((row_scores_kernel<MT, true>), grid, block, 0, s, rewards, mask, B, R, vec, scores,
                         lengths);
    });
  } else {
    hipLaunchKernelGGL((row_scores_kernel<VA_MASK_F32, false>), grid, block, 0, s, rewards, nullptr, B, R,
                       vec, scores, nullptr);
  }
  return check_launch("row_scores");
}

extern "C" int va_group_coef(const float *scores, const float *lengths, const int32_t *order,
                             const int32_t *offsets, int64_t n_groups, int64_t max_group_size,
                             float epsilon, int estimator, float *coef, void *stream) {
  VA_CHECK_ARG(n_groups > 0, "no groups");
  VA_CHECK_ARG(max_group_size > 0 && max_group_size <= 16384, "group size %lld out of range",
               (long long)max_group_size);
  VA_CHECK_ARG(scores && order && offsets && coef, "null pointer argument");
  VA_CHECK_ARG(estimator != VA_ADV_OPO || lengths, "OPO needs the response lengths");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t shm = static_cast<size_t>(2 * max_group_size + 4) * sizeof(float);
#define VA_LAUNCH_COEF(E)                                                                      \
  hipLaunchKernelGGL((group_coef_kernel<E>), dim3(n_groups), dim3(64), shm, s, scores, lengths, \
                     order, offsets, epsilon, coef)
  switch (estimator) {
    case VA_ADV_GRPO: VA_LAUNCH_COEF(VA_ADV_GRPO); break;
    case VA_ADV_GRPO_NOSTD: VA_LAUNCH_COEF(VA_ADV_GRPO_NOSTD); break;
    case VA_ADV_RLOO: VA_LAUNCH_COEF(VA_ADV_RLOO); break;
    case VA_ADV_MEAN_ONLY: VA_LAUNCH_COEF(VA_ADV_MEAN_ONLY); break;
    case VA_ADV_OPO: VA_LAUNCH_COEF(VA_ADV_OPO); break;
    case VA_ADV_PASSK: VA_LAUNCH_COEF(VA_ADV_PASSK); break;
    case VA_ADV_PASSK_NOSTD: VA_LAUNCH_COEF(VA_ADV_PASSK_NOSTD); break;
    default: set_error("unknown estimator %d", estimator); return VA_E_ARG;
  }
#undef VA_LAUNCH_COEF
  return check_launch("group_coef");
}

extern "C" int va_broadcast_rows(const float *coef, const void *mask, int mask_dtype, int64_t B,
                                 int64_t R, float *adv, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "bad shape (B=%lld R=%lld)", (long long)B, (long long)R);
  VA_CHECK_ARG(coef && mask && adv, "null pointer argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = (R & 3) == 0 && (reinterpret_cast<uintptr_t>(adv) & 15) == 0;
  const int64_t work = vec ? (B * R) >> 2 : B * R;
  int64_t grid = (work + 255) / 256;
  if (grid > 16384) grid = 16384;
  VA_DISPATCH_MASK(mask_dtype, {
    if (vec)
      hipLaunchKernelGGL((broadcast_rows_kernel<MT, true>), dim3(grid), dim3(256), 0, s, coef, mask, B, R, adv);
    else
      hipLaunchKernelGGL((broadcast_rows_kernel<MT, false>), dim3(grid), dim3(256), 0, s, coef, mask, B, R, adv);
  });
  return check_launch("broadcast_rows");
}

extern "C" int64_t va_outcome_workspace_bytes(int64_t B) {
  return static_cast<int64_t>(sizeof(float)) * 3 * B;
}

extern "C" int va_outcome_advantage(const float *rewards, const void *mask, int mask_dtype,
                                    int64_t B, int64_t R, const int32_t *order,
                                    const int32_t *offsets, int64_t n_groups,
                                    int64_t max_group_size, float epsilon, int estimator,
                                    float *adv, float *scores, void *workspace, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0 && n_groups > 0 && n_groups <= B, "bad shape (B=%lld G=%lld)",
               (long long)B, (long long)n_groups);
  VA_CHECK_ARG(rewards && mask && order && offsets && adv && workspace, "null pointer argument");
  float *ws = static_cast<float *>(workspace);
  float *sc = scores ? scores : ws;
  float *len = ws + B;
  float *coef = ws + 2 * B;
  int e = va_row_scores(rewards, mask, mask_dtype, B, R, sc, estimator == VA_ADV_OPO ? len : nullptr, stream);
  if (e) return e;
  e = va_group_coef(sc, len, order, offsets, n_groups, max_group_size, epsilon, estimator, coef, stream);
  if (e) return e;
  return va_broadcast_rows(coef, mask, mask_dtype, B, R, adv, stream);
}

extern "C" int64_t va_gae_workspace_bytes(int64_t B) {
  return static_cast<int64_t>(sizeof(double)) * (B * kPartStride + 4);
}

// va_set_tuning(VA_TUNE_GAE_VARIANT): 0 auto, 1 register kernel (only where L <= 16), 2 LDS kernel
int g_gae_variant = 0;

extern "C" int va_gae_scan(const float *rewards, const float *values, const void *mask,
                           int mask_dtype, int64_t B, int64_t R, float gamma, float lam,
                           float *adv_raw, float *ret, double *row_partials, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty batch");
  VA_CHECK_ARG(rewards && values && mask && adv_raw && ret && row_partials,
               "null pointer argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int L = static_cast<int>((R + 63) / 64);
  // gamma * lam is a Python-float product in the reference, applied as an fp32 scalar
  const float gl = static_cast<float>(static_cast<double>(gamma) * static_cast<double>(lam));
  // register chunks for short rows of small batches (latency: one round trip, no LDS); many rows
  // stream better through the coalesced LDS staging (lane-chunk loads touch 64 lines per
  // instruction)
  const bool reg = L <= 16 && (g_gae_variant == 1 || (g_gae_variant == 0 && B * R <= (1LL << 20)));
  if (reg) {
    const dim3 block(256), grid(static_cast<unsigned>((B + 3) / 4));
#define VA_GAE_REG(LMV)                                                                              \
  hipLaunchKernelGGL((gae_scan_reg_kernel<MT, LMV>), grid, block, 0, s, rewards, values, mask, B, R, L, \
                     gamma, gl, adv_raw, ret, row_partials)
    VA_DISPATCH_MASK(mask_dtype, {
      if (L <= 4) VA_GAE_REG(4);
      else if (L <= 8) VA_GAE_REG(8);
      else VA_GAE_REG(16);
    });
#undef VA_GAE_REG
    return check_launch("gae_scan");
  }
  int waves = 4;
  while (waves > 1 && gae_lds_bytes(L, waves) > 160 * 1024) waves >>= 1;
  const bool use_lds = gae_lds_bytes(L, waves) <= 160 * 1024;
  const dim3 block(64 * waves);
  const dim3 grid(static_cast<unsigned>((B + waves - 1) / waves));
  if (use_lds) {
    const size_t shm = static_cast<size_t>(gae_lds_bytes(L, waves));
    VA_DISPATCH_MASK(mask_dtype, {
      if (hipFuncSetAttribute(reinterpret_cast<const void *>(&gae_scan_kernel<MT, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(shm)) != hipSuccess) {
        set_error("gae_scan: cannot reserve %zu bytes of LDS", shm);
        return VA_E_LAUNCH;
      }
      hipLaunchKernelGGL((gae_scan_kernel<MT, true>), grid, block, shm, s, rewards, values, mask,
                         B, R, L, gamma, gl, adv_raw, ret, row_partials);
    });
  } else {
    VA_DISPATCH_MASK(mask_dtype, {
      hipLaunchKernelGGL((gae_scan_kernel<MT, false>), grid, block, 0, s, rewards, values, mask,
                         B, R, L, gamma, gl, adv_raw, ret, row_partials);
    });
  }
  return check_launch("gae_scan");
}

extern "C" int va_masked_row_partials(const float *x, const void *mask, int mask_dtype,
                                      int64_t B, int64_t R, double *row_partials, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty input");
  VA_CHECK_ARG(x && mask && row_partials, "null pointer argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  VA_DISPATCH_MASK(mask_dtype, {
    hipLaunchKernelGGL((row_partials_kernel<MT>), dim3((B + 3) / 4), dim3(256), 0, s, x, mask,
                       B, R, row_partials);
  });
  return check_launch("masked_row_partials");
}

extern "C" int va_whiten_finalize(const double *partials, int64_t K, double *merged,
                                  float *stats_out, void *stream) {
  VA_CHECK_ARG(K > 0, "K must be > 0");
  VA_CHECK_ARG(partials && merged && stats_out, "null pointer argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(whiten_finalize_kernel, dim3(1), dim3(256), 0, s, partials, K, merged,
                     stats_out);
  return check_launch("whiten_finalize");
}

extern "C" int va_whiten_apply(float *x, const float *stats, const void *mask, int mask_dtype,
                               int64_t B, int64_t R, int post_multiply_mask, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty input");
  VA_CHECK_ARG(x && stats, "null pointer argument");
  VA_CHECK_ARG(!post_multiply_mask || mask != nullptr, "mask required for post multiply");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = B * R;
  int64_t grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  if (post_multiply_mask) {
    VA_DISPATCH_MASK(mask_dtype, {
      hipLaunchKernelGGL((whiten_apply_kernel<MT, true>), dim3(grid), dim3(256), 0, s, x, stats,
                         mask, n);
    });
  } else {
    hipLaunchKernelGGL((whiten_apply_kernel<VA_MASK_F32, false>), dim3(grid), dim3(256), 0, s, x,
                       stats, nullptr, n);
  }
  return check_launch("whiten_apply");
}

extern "C" int va_gae_advantage_return(const float *rewards, const float *values,
                                       const void *mask, int mask_dtype, int64_t B, int64_t R,
                                       float gamma, float lam, float *adv, float *ret,
                                       float *stats_out, void *workspace, void *stream) {
  VA_CHECK_ARG(workspace && stats_out, "null pointer argument");
  double *part = static_cast<double *>(workspace);
  int e = va_gae_scan(rewards, values, mask, mask_dtype, B, R, gamma, lam, adv, ret, part,
                      stream);
  if (e) return e;
  e = va_whiten_finalize(part, B, part + B * kPartStride, stats_out, stream);
  if (e) return e;
  return va_whiten_apply(adv, stats_out, mask, mask_dtype, B, R, 0, stream);
}

extern "C" int va_discounted_returns(const float *rewards, const void *mask, int mask_dtype, int64_t B,
                                     int64_t R, float gamma, int mode, const float *baselines, float *returns,
                                     float *adv, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty batch");
  VA_CHECK_ARG(rewards && mask && returns, "null pointer argument");
  VA_CHECK_ARG(mode == VA_RET_RFPP || (mode == VA_RET_REMAX && baselines && adv), "bad mode / missing ReMax outputs");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int L = static_cast<int>((R + 63) / 64);
  const dim3 grid(static_cast<unsigned>((B + 3) / 4));
  if (mode == VA_RET_RFPP) {
    VA_DISPATCH_MASK(mask_dtype, {
      hipLaunchKernelGGL((discounted_returns_kernel<MT, VA_RET_RFPP>), grid, dim3(256), 0, s, rewards, mask, B, R,
                         L, gamma, baselines, returns, adv);
    });
  } else {
    VA_DISPATCH_MASK(mask_dtype, {
      hipLaunchKernelGGL((discounted_returns_kernel<MT, VA_RET_REMAX>), grid, dim3(256), 0, s, rewards, mask, B,
                         R, L, gamma, baselines, returns, adv);
    });
  }
  return check_launch("discounted_returns");
}
