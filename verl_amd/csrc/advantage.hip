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

int g_gae_partials = 0;  // va_set_tuning(VA_TUNE_GAE_PARTIALS), see gae_group_rows
// va_set_tuning(VA_TUNE_GAE_NT): cache policy of the GAE streams, bit 0 = non-temporal loads of
// r / v, bit 1 = non-temporal store of the returns, bit 2 = non-temporal stores of the raw
// advantages (re-read by the whitening launch, so cached by default) and of the whitened output
int g_gae_nt = 3;

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

// Streaming variant for R % 4 == 0 and R <= 256 * JM (the headline and its 16x batch: R = 1024,
// J = 4): lane k owns the QUADS of steps t = 256 j + 4 k + {0..3}, j = 0..J-1, so every load and
// store is a fully coalesced 16-byte vector per lane (a wave moves 1 KB per instruction), all
// 4 J + 4 J + (1..2) J loads of the row are issued before the first use, and nothing goes
// through LDS. The scan runs level by level from the last quad row j = J-1 down to 0: each lane
// composes its quad's affine map, a 6-step wave reverse scan gives every quad its incoming
// state from the carry (the state after all levels above), the lane re-runs its 4 steps in the
// reference's op order, and lane 0's inclusive map advances the carry. Row partials (n, sum,
// M2) in fp64 as the other variants.
template <int MT, int JM>
__device__ __forceinline__ Moments gae_row_quads(const float *__restrict__ rew, const float *__restrict__ val,
                                                 const void *__restrict__ mask, int64_t row, int64_t R, int J,
                                                 float gamma, float gl, float *__restrict__ adv_raw,
                                                 float *__restrict__ ret, int nt) {
  const int lane = threadIdx.x & 63;
  const int64_t base = row * R;
  float r[JM][4], v[JM][4], m[JM][4];
  float4 ra[JM], va[JM];
  Mask4Raw<MT> mr[JM];
#pragma unroll
  for (int j = 0; j < JM; ++j) {  // every load of the row first (raw mask: converted after)
    const int64_t t0 = 256 * j + 4 * lane;
    const bool ok = j < J && t0 < R;
    const int64_t tc = ok ? t0 : 0;  // clamped address: no branch around the loads
    ra[j] = ld4(rew + base + tc, nt & 1);
    va[j] = ld4(val + base + tc, nt & 1);
    mr[j] = load_mask4_raw<MT>(mask, base + tc);
  }
  loads_issued();
#pragma unroll
  for (int j = 0; j < JM; ++j) pin4(ra[j]), pin4(va[j]), pin_mask4<MT>(mr[j]);
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const bool ok = j < J && 256 * j + 4 * lane < R;
    const float4 a = ra[j], b = va[j];
    float mm[4];
    cvt_mask4<MT>(mr[j], mm);
    r[j][0] = ok ? a.x : 0.f, r[j][1] = ok ? a.y : 0.f, r[j][2] = ok ? a.z : 0.f, r[j][3] = ok ? a.w : 0.f;
    v[j][0] = ok ? b.x : 0.f, v[j][1] = ok ? b.y : 0.f, v[j][2] = ok ? b.z : 0.f, v[j][3] = ok ? b.w : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) m[j][q] = ok ? mm[q] : 0.f;  // a masked-out step is the identity map
  }
  float cg = 0.f, cnv = 0.f;  // carry: state after every level above the current one
#pragma unroll
  for (int j = JM - 1; j >= 0; --j) {
    if (j >= J) continue;
    Aff F{1.f, 0.f, 1.f, 0.f, 0.f};
#pragma unroll
    for (int q = 3; q >= 0; --q) {
      Aff st;
      st.a = m[j][q] * gl + (1.f - m[j][q]);
      st.c = m[j][q] * gamma;
      st.e = 1.f - m[j][q];
      st.b1 = m[j][q] * (r[j][q] - v[j][q]);
      st.b2 = m[j][q] * v[j][q];
      F = compose(st, F);
    }
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
    // incoming state of quad k: the inclusive map of quad k+1 applied to the carry
    Aff G;
    G.a = __shfl_down(F.a, 1, kWave);
    G.c = __shfl_down(F.c, 1, kWave);
    G.e = __shfl_down(F.e, 1, kWave);
    G.b1 = __shfl_down(F.b1, 1, kWave);
    G.b2 = __shfl_down(F.b2, 1, kWave);
    float g, nv;
    if (lane == 63) {
      g = cg;
      nv = cnv;
    } else {
      g = G.a * cg + G.c * cnv + G.b1;
      nv = G.e * cnv + G.b2;
    }
    // next carry: quad 0's inclusive map (the whole level) applied to the carry
    const float a0 = __shfl(F.a, 0, kWave), c0 = __shfl(F.c, 0, kWave), e0 = __shfl(F.e, 0, kWave);
    const float b10 = __shfl(F.b1, 0, kWave), b20 = __shfl(F.b2, 0, kWave);
    const float ncg = a0 * cg + c0 * cnv + b10;
    cnv = e0 * cnv + b20;
    cg = ncg;
    // re-run the quad in the reference op order (core_algos.py:229-236); r <- g
#pragma unroll
    for (int q = 3; q >= 0; --q) {
      const float delta = (r[j][q] + gamma * nv) - v[j][q];
      const float gnew = delta + gl * g;
      nv = v[j][q] * m[j][q] + (1.f - m[j][q]) * nv;
      g = gnew * m[j][q] + (1.f - m[j][q]) * g;
      r[j][q] = g;
    }
  }
  // stores + row partials (n, sum, M2) of g over the mask
  double n = 0.0, sum = 0.0;
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int64_t t0 = 256 * j + 4 * lane;
    if (j < J && t0 < R) {
      float4 a, b;
      a.x = r[j][0], a.y = r[j][1], a.z = r[j][2], a.w = r[j][3];
      b.x = r[j][0] + v[j][0], b.y = r[j][1] + v[j][1], b.z = r[j][2] + v[j][2], b.w = r[j][3] + v[j][3];
      st4(adv_raw + base + t0, a, nt & 4);
      st4(ret + base + t0, b, nt & 2);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        n += m[j][q];
        sum += static_cast<double>((m[j][q] != 0.f ? r[j][q] : 0.f) * m[j][q]);
      }
    }
  }
  n = wave_sum(n);
  sum = wave_sum(sum);
  const double mu = n > 0.0 ? sum / n : 0.0;
  double m2 = 0.0;
#pragma unroll
  for (int j = 0; j < JM; ++j) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (m[j][q] != 0.f) {
        const double d = static_cast<double>(r[j][q]) - mu;
        m2 += static_cast<double>(m[j][q]) * d * d;
      }
    }
  }
  m2 = wave_sum(m2);
  return Moments{n, mu, m2};
}

// Partial triples of the GAE scan: one per group of w rows (w = 1: one per row, written by the
// row's wave, the default; w = 4 / 8: one per workgroup of w waves, merged in wave order by the
// last wave to finish). P = ceil(B / w). The consumer merges them in a fixed order (first in
// parallel slices of 512 when P > 4096). va_set_tuning(VA_TUNE_GAE_PARTIALS, w) picks w
// (0 = auto).
int gae_group_rows(int64_t B) {
  if (g_gae_partials == 1 || g_gae_partials == 4 || g_gae_partials == 8) return g_gae_partials;
  return 1;  // measured fastest at 512 and 8,192 rows (profiles/r02/gae_partials_ab.txt)
}
int64_t gae_partial_count(int64_t B) {
  const int w = gae_group_rows(B);
  return (B + w - 1) / w;
}

// One partial triple per workgroup without a workgroup barrier at the end: each wave leaves its
// moments in LDS and bumps an LDS counter (workgroup-scope acq_rel: ordering only, no cache
// maintenance); the wave that arrives last merges the entries in wave order (the same order
// whichever wave it is) and writes the triple. Waves retire independently, as with per-row
// partials. `cnt` must be zeroed (and a barrier passed) at kernel start.
__device__ __forceinline__ void store_wg_moments(Moments acc, double *__restrict__ part, double *sh, int *cnt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  int prev = 0;
  if (lane == 0) {
    sh[wave * 3 + 0] = acc.n;
    sh[wave * 3 + 1] = acc.mean;
    sh[wave * 3 + 2] = acc.m2;
    prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  prev = __shfl(prev, 0, kWave);
  if (prev == waves - 1 && lane == 0) {
    Moments t{0.0, 0.0, 0.0};
    for (int w = 0; w < waves; ++w) t = merge_moments(t, Moments{sh[w * 3], sh[w * 3 + 1], sh[w * 3 + 2]});
    part[blockIdx.x * kPartStride + 0] = t.n;
    part[blockIdx.x * kPartStride + 1] = t.mean * t.n;
    part[blockIdx.x * kPartStride + 2] = t.m2;
  }
}

template <int MT, int JM, bool WG_MERGE>
__global__ __launch_bounds__(512) void gae_scan_vec_kernel(
    const float *__restrict__ rew, const float *__restrict__ val, const void *__restrict__ mask,
    int64_t B, int64_t R, int J, float gamma, float gl, float *__restrict__ adv_raw,
    float *__restrict__ ret, double *__restrict__ part, int nt) {
  const int wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * waves + wave;
  if constexpr (!WG_MERGE) {
    if (row >= B) return;  // waves are independent: no workgroup barrier
    const Moments m = gae_row_quads<MT, JM>(rew, val, mask, row, R, J, gamma, gl, adv_raw, ret, nt);
    if ((threadIdx.x & 63) == 0) {
      part[row * kPartStride + 0] = m.n;
      part[row * kPartStride + 1] = m.mean * m.n;
      part[row * kPartStride + 2] = m.m2;
    }
  } else {
    __shared__ double sh[8 * 3];
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();  // at kernel start, before any load: costs no overlap
    Moments acc{0.0, 0.0, 0.0};
    if (row < B) acc = gae_row_quads<MT, JM>(rew, val, mask, row, R, J, gamma, gl, adv_raw, ret, nt);
    store_wg_moments(acc, part, sh, &cnt);
  }
}

// Group the per-row triples of the fallback scan variants (rows[3 B]) into the same P partials
// the streaming kernel writes: workgroup g merges rows g w .. g w + w - 1 in order.
__global__ __launch_bounds__(64) void gae_group_partials_kernel(const double *__restrict__ rows, int64_t B,
                                                                int w, double *__restrict__ part) {
  __shared__ double sh[16 * 3];
  if (threadIdx.x < w) {
    Moments acc{0.0, 0.0, 0.0};
    const int64_t row = static_cast<int64_t>(blockIdx.x) * w + threadIdx.x;
    if (row < B) {
      const double n = rows[row * kPartStride + 0];
      acc = Moments{n, n > 0.0 ? rows[row * kPartStride + 1] / n : 0.0, rows[row * kPartStride + 2]};
    }
    sh[threadIdx.x * 3 + 0] = acc.n;
    sh[threadIdx.x * 3 + 1] = acc.mean;
    sh[threadIdx.x * 3 + 2] = acc.m2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Moments t{0.0, 0.0, 0.0};
    for (int k = 0; k < w; ++k) t = merge_moments(t, Moments{sh[k * 3], sh[k * 3 + 1], sh[k * 3 + 2]});
    part[blockIdx.x * kPartStride + 0] = t.n;
    part[blockIdx.x * kPartStride + 1] = t.mean * t.n;
    part[blockIdx.x * kPartStride + 2] = t.m2;
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

// Merge the (n, sum, M2) triples k = beg, beg + step, ... < end (triple k at part[3 k]) with one
// 256-thread workgroup: thread t accumulates its entries t, t + 256, ... in order (the loads of a
// batch of 8 issued before the first add), then a fixed wave / workgroup sum. The order depends
// only on (beg, end, step): deterministic.
constexpr int kMergeThreads = 256;
constexpr int64_t kMergeSlice = 512;  // triples per first-level workgroup when K is large

__device__ Moments block_merge(const double *__restrict__ part, int64_t beg, int64_t end, int64_t step,
                               double *sh) {
  // Shifted sums instead of a Chan tree: with c = the first partial's mean, every partial becomes
  // (n, S1 = n (mean - c), S2 = M2 + n (mean - c)^2), which merge by plain additions (wave
  // shuffles, no fp64 divisions, no LDS tree); mean = c + S1 / N, M2 = S2 - S1^2 / N at the end.
  // c is a data value, so the final subtraction cancels at most a digit or two of fp64.
  const double n0 = end > beg ? part[beg * kPartStride + 0] : 0.0;
  const double c = n0 > 0.0 ? part[beg * kPartStride + 1] / n0 : 0.0;
  double acc[3] = {0.0, 0.0, 0.0};
  constexpr int kBatch = 8;
  const int64_t count = end > beg ? (end - beg + step - 1) / step : 0;
  for (int64_t i0 = 0; i0 < count; i0 += static_cast<int64_t>(kBatch) * kMergeThreads) {
    double pn[kBatch], ps[kBatch], pm[kBatch];
#pragma unroll
    for (int i = 0; i < kBatch; ++i) {
      const int64_t idx = i0 + static_cast<int64_t>(i) * kMergeThreads + threadIdx.x;
      const bool ok = idx < count;
      const int64_t k = beg + (ok ? idx : 0) * step;
      pn[i] = ok ? part[k * kPartStride + 0] : 0.0;
      ps[i] = ok ? part[k * kPartStride + 1] : 0.0;
      pm[i] = ok ? part[k * kPartStride + 2] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < kBatch; ++i) {
      if (pn[i] > 0.0) {
        const double d = ps[i] / pn[i] - c;
        acc[0] += pn[i];
        acc[1] += pn[i] * d;
        acc[2] += pm[i] + pn[i] * d * d;
      }
    }
  }
  block_sum<3>(acc, sh);
  const double N = acc[0];
  if (N <= 0.0) return Moments{0.0, 0.0, 0.0};
  return Moments{N, c + acc[1] / N, acc[2] - acc[1] * acc[1] / N};
}

__device__ __forceinline__ void whiten_stats_of(Moments tot, double *merged, float *stats, float &mean_out,
                                                float &rstd_out) {
  const double n = tot.n;
  const double mean = (tot.mean * n) / (n + 1e-8);  // torch_functional.py:171-185, 188-223
  const double dm = tot.mean - mean;
  const double var_b = (tot.m2 + n * dm * dm) / (n + 1e-8);
  float flag = 0.f;
  double var = var_b;
  if (n == 0.0) flag = 1.f;
  else if (n == 1.0) flag = 2.f;
  else var = var_b * (n / (n - 1.0));
  const float var32 = static_cast<float>(var);
  mean_out = static_cast<float>(mean);
  rstd_out = 1.0f / sqrtf(var32 + 1e-8f);
  if (merged != nullptr) {
    merged[0] = n;
    merged[1] = tot.mean * n;
    merged[2] = tot.m2;
    stats[0] = mean_out;
    stats[1] = rstd_out;
    stats[2] = static_cast<float>(n);
    stats[3] = flag;
  }
}

// First level for large K: workgroup g merges the slice [g S, (g + 1) S) and writes the result
// over the slice's first triple (no other workgroup reads that slot).
__global__ __launch_bounds__(kMergeThreads) void whiten_merge_slices_kernel(double *__restrict__ part, int64_t K) {
  __shared__ double sh[kMergeThreads * 3];
  const int64_t beg = static_cast<int64_t>(blockIdx.x) * kMergeSlice;
  const int64_t end = beg + kMergeSlice < K ? beg + kMergeSlice : K;
  const Moments m = block_merge(part, beg, end, 1, sh);
  if (threadIdx.x == 0) {
    part[beg * kPartStride + 0] = m.n;
    part[beg * kPartStride + 1] = m.mean * m.n;
    part[beg * kPartStride + 2] = m.m2;
  }
}

// Merge the triples 0, step, 2 step, ... < K; emit the merged triple and the fp32 whitening stats
// {mean, rsqrt(var + 1e-8), n, error_flag} with the reference's formulas.
__global__ __launch_bounds__(kMergeThreads) void whiten_finalize_kernel(const double *__restrict__ part,
                                                                        int64_t K, int64_t step,
                                                                        double *__restrict__ merged,
                                                                        float *__restrict__ stats) {
  __shared__ double sh[kMergeThreads * 3];
  const Moments tot = block_merge(part, 0, K, step, sh);
  if (threadIdx.x == 0) {
    float mean, rstd;
    whiten_stats_of(tot, merged, stats, mean, rstd);
  }
}

// whiten_finalize + whiten_apply in one launch: every workgroup merges the K (<= a few hundred)
// partial triples itself, in the same fixed order, so all of them apply identical statistics
// (workgroup 0 also writes the merged triple and the stats for the caller's error check), then
// streams its share of x = (x - mean) * rstd with 16-byte vectors.
__global__ __launch_bounds__(kMergeThreads) void whiten_stats_apply_kernel(float *__restrict__ x,
                                                                           const double *__restrict__ part,
                                                                           int64_t K, int64_t step,
                                                                           double *__restrict__ merged,
                                                                           float *__restrict__ stats, int64_t nq,
                                                                           int nt) {
  __shared__ double sh[kMergeThreads * 3];
  // chunks of U quads per thread; the first chunk's loads are issued BEFORE the merge of the
  // partials (they do not depend on the statistics), so the merge's dependent loads and barriers
  // run under their latency instead of in front of the stream
  constexpr int U = 8;
  const int64_t chunk = static_cast<int64_t>(blockDim.x) * U;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * chunk;
  int64_t c0 = static_cast<int64_t>(blockIdx.x) * chunk;
  float4 a[U];
  auto load_chunk = [&](int64_t c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {  // clamped, unconditional loads: all U in flight at once
      const int64_t i = c + static_cast<int64_t>(u) * blockDim.x + threadIdx.x;
      a[u] = ld4(x + 4 * (i < nq ? i : nq - 1), false);
    }
  };
  if (c0 < nq) load_chunk(c0);
  const Moments tot = block_merge(part, 0, K, step, sh);
  float mean, rstd;
  const bool writer = blockIdx.x == 0 && threadIdx.x == 0;
  whiten_stats_of(tot, writer ? merged : nullptr, stats, mean, rstd);
  for (; c0 < nq; c0 += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = c0 + static_cast<int64_t>(u) * blockDim.x + threadIdx.x;
      if (i < nq) {
        float4 v = a[u];
        v.x = (v.x - mean) * rstd, v.y = (v.y - mean) * rstd, v.z = (v.z - mean) * rstd, v.w = (v.w - mean) * rstd;
        st4(x + 4 * i, v, nt & 4);
      }
    }
    if (c0 + stride < nq) load_chunk(c0 + stride);
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

// The same with 16-byte vectors (n % 4 == 0, x 16-byte aligned): two quads per lane in flight.
template <int MT, bool POSTMASK>
__global__ __launch_bounds__(256) void whiten_apply_vec_kernel(float *__restrict__ x,
                                                               const float *__restrict__ stats,
                                                               const void *__restrict__ mask,
                                                               int64_t nq) {
  const float mean = stats[0], rstd = stats[1];
  float4 *x4 = reinterpret_cast<float4 *>(x);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + stride < nq; i += 2 * stride) {
    float4 a = x4[i], b = x4[i + stride];
    a.x = (a.x - mean) * rstd, a.y = (a.y - mean) * rstd, a.z = (a.z - mean) * rstd, a.w = (a.w - mean) * rstd;
    b.x = (b.x - mean) * rstd, b.y = (b.y - mean) * rstd, b.z = (b.z - mean) * rstd, b.w = (b.w - mean) * rstd;
    if constexpr (POSTMASK) {
      float ma[4], mb[4];
      load_mask4<MT>(mask, 4 * i, ma);
      load_mask4<MT>(mask, 4 * (i + stride), mb);
      a.x *= ma[0], a.y *= ma[1], a.z *= ma[2], a.w *= ma[3];
      b.x *= mb[0], b.y *= mb[1], b.z *= mb[2], b.w *= mb[3];
    }
    x4[i] = a;
    x4[i + stride] = b;
  }
  for (; i < nq; i += stride) {
    float4 a = x4[i];
    a.x = (a.x - mean) * rstd, a.y = (a.y - mean) * rstd, a.z = (a.z - mean) * rstd, a.w = (a.w - mean) * rstd;
    if constexpr (POSTMASK) {
      float ma[4];
      load_mask4<MT>(mask, 4 * i, ma);
      a.x *= ma[0], a.y *= ma[1], a.z *= ma[2], a.w *= ma[3];
    }
    x4[i] = a;
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

// workspace layout (doubles): [P <= B partial triples | B per-row triples (fallback variants) | merged 3 | pad]
extern "C" int64_t va_gae_workspace_bytes(int64_t B) {
  return static_cast<int64_t>(sizeof(double)) * (2 * B * kPartStride + 8);
}
extern "C" int64_t va_gae_partial_count(int64_t B) { return B > 0 ? gae_partial_count(B) : 0; }

// va_set_tuning(VA_TUNE_GAE_VARIANT): 0 auto (quad-streaming kernel where it applies), 1 register
// kernel (only where L <= 16), 2 LDS kernel, 3 quad-streaming kernel
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
  // streaming quad variant: 16-byte coalesced loads / stores straight to registers (default
  // wherever it applies: R % 4 == 0, R <= 2048, 16-byte aligned rows)
  const bool aligned = ((reinterpret_cast<uintptr_t>(rewards) | reinterpret_cast<uintptr_t>(values) |
                         reinterpret_cast<uintptr_t>(adv_raw) | reinterpret_cast<uintptr_t>(ret)) & 15) == 0 &&
                       (reinterpret_cast<uintptr_t>(mask) & 15) == 0;
  if ((g_gae_variant == 0 || g_gae_variant == 3) && (R & 3) == 0 && R <= 2048 && aligned) {
    const int J = static_cast<int>((R + 255) / 256);
    const int w = gae_group_rows(B);
    const dim3 block(w == 8 ? 512 : 256), grid(static_cast<unsigned>(w == 1 ? (B + 3) / 4 : gae_partial_count(B)));
#define VA_GAE_VEC(JMV)                                                                                     \
  do {                                                                                                      \
    if (w == 1)                                                                                             \
      hipLaunchKernelGGL((gae_scan_vec_kernel<MT, JMV, false>), grid, block, 0, s, rewards, values, mask, B, \
                         R, J, gamma, gl, adv_raw, ret, row_partials, g_gae_nt);                            \
    else                                                                                                    \
      hipLaunchKernelGGL((gae_scan_vec_kernel<MT, JMV, true>), grid, block, 0, s, rewards, values, mask, B,  \
                         R, J, gamma, gl, adv_raw, ret, row_partials, g_gae_nt);                            \
  } while (0)
    VA_DISPATCH_MASK(mask_dtype, {
      if (J <= 1) VA_GAE_VEC(1);
      else if (J <= 2) VA_GAE_VEC(2);
      else if (J <= 4) VA_GAE_VEC(4);
      else VA_GAE_VEC(8);
    });
#undef VA_GAE_VEC
    return check_launch("gae_scan");
  }
  // fallback variants: per-row triples (directly the partials when w == 1, else in the scratch half
  // of the workspace, then grouped)
  const int64_t P = gae_partial_count(B);
  const int wg = gae_group_rows(B);
  double *rows = wg == 1 ? row_partials : row_partials + B * kPartStride;
  auto group_rows = [&]() -> int {
    if (int e = check_launch("gae_scan")) return e;
    if (wg == 1) return VA_OK;
    hipLaunchKernelGGL(gae_group_partials_kernel, dim3(static_cast<unsigned>(P)), dim3(64), 0, s, rows, B, wg,
                       row_partials);
    return check_launch("gae_group_partials");
  };
  const bool reg = L <= 16 && (g_gae_variant == 1 || (g_gae_variant == 0 && B * R <= (1LL << 20)));
  if (reg) {
    const dim3 block(256), grid(static_cast<unsigned>((B + 3) / 4));
#define VA_GAE_REG(LMV)                                                                              \
  hipLaunchKernelGGL((gae_scan_reg_kernel<MT, LMV>), grid, block, 0, s, rewards, values, mask, B, R, L, \
                     gamma, gl, adv_raw, ret, rows)
    VA_DISPATCH_MASK(mask_dtype, {
      if (L <= 4) VA_GAE_REG(4);
      else if (L <= 8) VA_GAE_REG(8);
      else VA_GAE_REG(16);
    });
#undef VA_GAE_REG
    return group_rows();
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
                         B, R, L, gamma, gl, adv_raw, ret, rows);
    });
  } else {
    VA_DISPATCH_MASK(mask_dtype, {
      hipLaunchKernelGGL((gae_scan_kernel<MT, false>), grid, block, 0, s, rewards, values, mask,
                         B, R, L, gamma, gl, adv_raw, ret, rows);
    });
  }
  return group_rows();
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

extern "C" int va_whiten_finalize(double *partials, int64_t K, double *merged,
                                  float *stats_out, void *stream) {
  VA_CHECK_ARG(K > 0, "K must be > 0");
  VA_CHECK_ARG(partials && merged && stats_out, "null pointer argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (K > 2 * kMergeSlice) {
    // two levels: slices of kMergeSlice triples merged in parallel (in place), then their results
    const int64_t G = (K + kMergeSlice - 1) / kMergeSlice;
    hipLaunchKernelGGL(whiten_merge_slices_kernel, dim3(static_cast<unsigned>(G)), dim3(kMergeThreads), 0, s,
                       partials, K);
    hipLaunchKernelGGL(whiten_finalize_kernel, dim3(1), dim3(kMergeThreads), 0, s, partials, K, kMergeSlice,
                       merged, stats_out);
  } else {
    hipLaunchKernelGGL(whiten_finalize_kernel, dim3(1), dim3(kMergeThreads), 0, s, partials, K, int64_t(1),
                       merged, stats_out);
  }
  return check_launch("whiten_finalize");
}

extern "C" int va_whiten_apply(float *x, const float *stats, const void *mask, int mask_dtype,
                               int64_t B, int64_t R, int post_multiply_mask, void *stream) {
  VA_CHECK_ARG(B > 0 && R > 0, "empty input");
  VA_CHECK_ARG(x && stats, "null pointer argument");
  VA_CHECK_ARG(!post_multiply_mask || mask != nullptr, "mask required for post multiply");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = B * R;
  const bool vec = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                   (!post_multiply_mask || (reinterpret_cast<uintptr_t>(mask) & 15) == 0);
  if (vec) {
    const int64_t nq = n >> 2;
    int64_t grid = (nq + 511) / 512;  // two quads per lane
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    if (post_multiply_mask) {
      VA_DISPATCH_MASK(mask_dtype, {
        hipLaunchKernelGGL((whiten_apply_vec_kernel<MT, true>), dim3(grid), dim3(256), 0, s, x, stats, mask, nq);
      });
    } else {
      hipLaunchKernelGGL((whiten_apply_vec_kernel<VA_MASK_F32, false>), dim3(grid), dim3(256), 0, s, x, stats,
                         nullptr, nq);
    }
    return check_launch("whiten_apply");
  }
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

// va_set_tuning(VA_TUNE_WHITEN_SLICE_MIN / VA_TUNE_WHITEN_GRID): partial count above which the
// partials are first merged in parallel slices (default 4,096), and the statistics + whitening
// launch's grid cap (default 2,048)
int g_whiten_slice_min = 8 * 512;
int g_whiten_grid = 2048;

extern "C" int va_gae_advantage_return(const float *rewards, const float *values,
                                       const void *mask, int mask_dtype, int64_t B, int64_t R,
                                       float gamma, float lam, float *adv, float *ret,
                                       float *stats_out, void *workspace, void *stream) {
  VA_CHECK_ARG(workspace && stats_out, "null pointer argument");
  double *part = static_cast<double *>(workspace);
  int e = va_gae_scan(rewards, values, mask, mask_dtype, B, R, gamma, lam, adv, ret, part,
                      stream);
  if (e) return e;
  int64_t P = gae_partial_count(B);
  double *merged = part + 2 * B * kPartStride;
  const int64_t n = B * R;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(adv) & 15) == 0) {
    // statistics + whitening in one launch (every workgroup merges the partials itself); many
    // partials are first merged in parallel slices of kMergeSlice (in place)
    int64_t step = 1;
    if (P > g_whiten_slice_min) {
      const int64_t G = (P + kMergeSlice - 1) / kMergeSlice;
      hipLaunchKernelGGL(whiten_merge_slices_kernel, dim3(static_cast<unsigned>(G)), dim3(kMergeThreads), 0, s,
                         part, P);
      step = kMergeSlice;
    }
    const int64_t nq = n >> 2;
    int64_t grid = (nq + 8 * kMergeThreads - 1) / (8 * kMergeThreads);  // 8 quads per lane
    if (grid > g_whiten_grid) grid = g_whiten_grid;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(whiten_stats_apply_kernel, dim3(static_cast<unsigned>(grid)), dim3(kMergeThreads), 0, s, adv,
                       part, P, step, merged, stats_out, nq, g_gae_nt);
    return check_launch("whiten_stats_apply");
  }
  e = va_whiten_finalize(part, P, merged, stats_out, stream);
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
