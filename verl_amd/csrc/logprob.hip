// Fused per-token log-prob + entropy over the vocab (forward and backward), gfx950.
//
// Reference semantics (rfahrn/verl):
//   dp_actor.py:182            logits.div_(temperature)       (in the logits dtype)
//   torch_functional.py:64-100 logprobs_from_logits -> flash-attn cross_entropy_loss:
//                              logp = x[label] - logsumexp(x), fp32 math, ignore_index -100
//   torch_functional.py:145-149 entropy = logsumexp(x) - sum(softmax(x) * x)
//   experimental/torch_functional.py:55-67 backward:
//                              dx = g_lp*(onehot - p) - g_H*p*(log p + H), then / T
//
// Design: one wave64 streams one row (all V logits) exactly once with 16-byte loads, four
// vectors in flight per lane, and keeps an online (max, sum 2^(xL - m), sum 2^(...)*x)
// accumulator in the base-2 domain (L = log2 e), so a row costs one v_exp_f32 per element
// and one rescale per 32 elements. Rows are independent: no LDS, no barriers; a 256-thread
// workgroup carries 4 rows. The backward streams the row once more, reading the saved lse
// and entropy, and writes dlogits in the logits dtype (optionally in place).
// Bound: HBM. Algorithmic bytes per row: fwd  s*V + 8 + 12;  bwd  2*s*V + 28.

#include <math.h>

#include "va_common.h"

namespace va {
namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.69314718055994531f;
constexpr int kUnroll = 4;  // 16-byte vectors in flight per lane

typedef float float2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

// ---- element traits ------------------------------------------------------------------
template <typename T>
struct Elem;

template <>
struct Elem<float> {
  static constexpr int kVec = 4;
  __device__ static float load1(const float *p) { return *p; }
  __device__ static void unpack(const uint4 &r, float *x) {
    x[0] = __uint_as_float(r.x); x[1] = __uint_as_float(r.y);
    x[2] = __uint_as_float(r.z); x[3] = __uint_as_float(r.w);
  }
  // reference: logits.div_(T) on an fp32 tensor
  __device__ static float scale(float x, float T) { return x / T; }
  __device__ static uint4 pack(const float *x) {
    return make_uint4(__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]),
                      __float_as_uint(x[3]));
  }
  __device__ static void store1(float *p, float v) { *p = v; }
};

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  float2v f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2v));
}
__device__ __forceinline__ uint32_t pack_f16x2(float a, float b) {
  float2v f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, f16x2v));
}

struct bf16_t { uint16_t bits; };
struct f16_t { uint16_t bits; };

template <>
struct Elem<bf16_t> {
  static constexpr int kVec = 8;
  __device__ static float load1(const bf16_t *p) { return bf16_to_f32(p->bits); }
  __device__ static void unpack(const uint4 &r, float *x) {
    x[0] = bf16_lo(r.x); x[1] = bf16_hi(r.x); x[2] = bf16_lo(r.y); x[3] = bf16_hi(r.y);
    x[4] = bf16_lo(r.z); x[5] = bf16_hi(r.z); x[6] = bf16_lo(r.w); x[7] = bf16_hi(r.w);
  }
  // reference: bf16 tensor .div_(T) computes in fp32 and rounds back to bf16
  __device__ static float scale(float x, float T) {
    return bf16_lo(pack_bf16x2(x / T, 0.f));
  }
  __device__ static uint4 pack(const float *x) {
    return make_uint4(pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                      pack_bf16x2(x[6], x[7]));
  }
  __device__ static void store1(bf16_t *p, float v) {
    p->bits = static_cast<uint16_t>(pack_bf16x2(v, 0.f) & 0xffffu);
  }
};

template <>
struct Elem<f16_t> {
  static constexpr int kVec = 8;
  __device__ static float load1(const f16_t *p) { return f16_to_f32(p->bits); }
  __device__ static void unpack(const uint4 &r, float *x) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[2 * k] = f16_to_f32(static_cast<uint16_t>(w[k] & 0xffffu));
      x[2 * k + 1] = f16_to_f32(static_cast<uint16_t>(w[k] >> 16));
    }
  }
  __device__ static float scale(float x, float T) {
    return f16_to_f32(static_cast<uint16_t>(pack_f16x2(x / T, 0.f) & 0xffffu));
  }
  __device__ static uint4 pack(const float *x) {
    return make_uint4(pack_f16x2(x[0], x[1]), pack_f16x2(x[2], x[3]), pack_f16x2(x[4], x[5]),
                      pack_f16x2(x[6], x[7]));
  }
  __device__ static void store1(f16_t *p, float v) {
    p->bits = static_cast<uint16_t>(pack_f16x2(v, 0.f) & 0xffffu);
  }
};

// ---- online softmax accumulator (base-2) ----------------------------------------------
// m: running max of the (scaled) logits; s = sum 2^(x*L - B(m)), t = sum 2^(x*L - B(m)) * x,
// with B(m) = fl(m * L) (0 while m = -inf so that all-(-inf) prefixes stay finite).
struct Acc {
  float m, s, t;
};

__device__ __forceinline__ float base_of(float m) { return m == -INFINITY ? 0.f : m * kLog2e; }

template <int N>
__device__ __forceinline__ void acc_chunk(Acc &a, const float *x) {
  float cm = x[0];
#pragma unroll
  for (int k = 1; k < N; ++k) cm = fmaxf(cm, x[k]);
  const float nm = fmaxf(a.m, cm);
  const float nb = base_of(nm);
  const float alpha = __builtin_amdgcn_exp2f(base_of(a.m) - nb);
  // two partial sums per quantity to shorten the dependent add chains
  float s0 = 0.f, s1 = 0.f, t0 = 0.f, t1 = 0.f;
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    const float e0 = __builtin_amdgcn_exp2f(fmaf(x[k], kLog2e, -nb));
    s0 += e0;
    t0 = fmaf(e0, x[k], t0);
    if (k + 1 < N) {
      const float e1 = __builtin_amdgcn_exp2f(fmaf(x[k + 1], kLog2e, -nb));
      s1 += e1;
      t1 = fmaf(e1, x[k + 1], t1);
    }
  }
  a.s = fmaf(a.s, alpha, s0 + s1);
  a.t = fmaf(a.t, alpha, t0 + t1);
  a.m = nm;
}

__device__ __forceinline__ void acc_merge(Acc &a, float om, float os, float ot) {
  const float nm = fmaxf(a.m, om);
  const float nb = base_of(nm);
  const float a1 = __builtin_amdgcn_exp2f(base_of(a.m) - nb);
  const float a2 = __builtin_amdgcn_exp2f(base_of(om) - nb);
  a.s = a.s * a1 + os * a2;
  a.t = a.t * a1 + ot * a2;
  a.m = nm;
}

// ---- forward ---------------------------------------------------------------------------
template <typename T, bool SCALE, bool VECTOR>
__global__ __launch_bounds__(256) void logprob_entropy_fwd_kernel(
    const T *__restrict__ logits, int64_t n_rows, int64_t V, int64_t stride,
    const int64_t *__restrict__ labels, float temperature, float *__restrict__ logp,
    float *__restrict__ entropy, float *__restrict__ lse_out) {
  using E = Elem<T>;
  constexpr int VEC = E::kVec;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= n_rows) return;  // wave-uniform
  const T *xr = logits + row * stride;

  Acc a{-INFINITY, 0.f, 0.f};
  int64_t tail_begin = 0;
  if constexpr (VECTOR) {
    const uint4 *xv = reinterpret_cast<const uint4 *>(xr);
    const int64_t nvec = V / VEC;
    int64_t i = lane;
    for (; i + (kUnroll - 1) * kWave < nvec; i += kUnroll * kWave) {
      uint4 raw[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) raw[u] = xv[i + u * kWave];
      float x[kUnroll * VEC];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) E::unpack(raw[u], x + u * VEC);
      if constexpr (SCALE) {
#pragma unroll
        for (int k = 0; k < kUnroll * VEC; ++k) x[k] = E::scale(x[k], temperature);
      }
      acc_chunk<kUnroll * VEC>(a, x);
    }
    for (; i < nvec; i += kWave) {
      float x[VEC];
      E::unpack(xv[i], x);
      if constexpr (SCALE) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[k] = E::scale(x[k], temperature);
      }
      acc_chunk<VEC>(a, x);
    }
    tail_begin = nvec * VEC;
  }
  for (int64_t j = tail_begin + lane; j < V; j += kWave) {
    float x = E::load1(xr + j);
    if constexpr (SCALE) x = E::scale(x, temperature);
    acc_chunk<1>(a, &x);
  }

#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(a.m, o, kWave);
    const float os = __shfl_xor(a.s, o, kWave);
    const float ot = __shfl_xor(a.t, o, kWave);
    acc_merge(a, om, os, ot);
  }

  if (lane == 0) {
    // lse = m + ln(s) + ln 2 * (B(m) - m L): keeps the max exact and corrects fl(m L)
    float lse;
    if (a.m == -INFINITY) {
      lse = -INFINITY;
    } else {
      const float corr = -fmaf(a.m, kLog2e, -base_of(a.m));  // B(m) - m*L, |corr| <= ulp/2
      lse = a.m + kLn2 * (__builtin_amdgcn_logf(a.s) + corr);
    }
    lse_out[row] = lse;
    if (entropy != nullptr) entropy[row] = lse - a.t / a.s;
    const int64_t lab = labels[row];
    float lp;
    if (lab == -100) {
      lp = 0.f;  // flash-attn ignore_index: loss 0
    } else if (lab < 0 || lab >= V) {
      lp = __builtin_nanf("");
    } else {
      float xl = E::load1(xr + lab);
      if constexpr (SCALE) xl = E::scale(xl, temperature);
      lp = xl - lse;
    }
    logp[row] = lp;
  }
}

// ---- backward --------------------------------------------------------------------------
template <typename T, bool SCALE, bool VECTOR>
__global__ __launch_bounds__(256) void logprob_entropy_bwd_kernel(
    const float *__restrict__ g_logp, const float *__restrict__ g_ent, const T *logits,
    int64_t n_rows, int64_t V, int64_t stride, const int64_t *__restrict__ labels,
    const float *__restrict__ lse_in, const float *__restrict__ ent_in, float temperature,
    T *dlogits, int64_t dstride) {
  using E = Elem<T>;
  constexpr int VEC = E::kVec;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const T *xr = logits + row * stride;
  T *dr = dlogits + row * dstride;

  const int64_t lab = labels[row];
  const bool has_lab = (lab >= 0 && lab < V);
  const float glp = (g_logp != nullptr && has_lab) ? g_logp[row] : 0.f;
  const float gh = (g_ent != nullptr) ? g_ent[row] : 0.f;
  const float lse = lse_in[row];
  const float h = (g_ent != nullptr) ? ent_in[row] : 0.f;
  const float inv_out = SCALE ? 1.f / temperature : 1.f;

  // dz_j = -p_j * (glp + gh * (log p_j + H)) + glp * [j == label]
  auto grad = [&](float z, int64_t j) -> float {
    const float lp = z - lse;
    const float p = __builtin_amdgcn_exp2f(lp * kLog2e);
    float d = -p * fmaf(gh, lp + h, glp);
    if (j == lab) d += glp;
    if constexpr (SCALE) d = d / temperature;
    return d;
  };
  (void)inv_out;

  int64_t tail_begin = 0;
  if constexpr (VECTOR) {
    const uint4 *xv = reinterpret_cast<const uint4 *>(xr);
    uint4 *dv = reinterpret_cast<uint4 *>(dr);
    const int64_t nvec = V / VEC;
    int64_t i = lane;
    for (; i + (kUnroll - 1) * kWave < nvec; i += kUnroll * kWave) {
      uint4 raw[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) raw[u] = xv[i + u * kWave];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        float x[VEC];
        E::unpack(raw[u], x);
        const int64_t j0 = (i + u * kWave) * VEC;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          float z = x[k];
          if constexpr (SCALE) z = E::scale(z, temperature);
          x[k] = grad(z, j0 + k);
        }
        dv[i + u * kWave] = E::pack(x);
      }
    }
    for (; i < nvec; i += kWave) {
      float x[VEC];
      E::unpack(xv[i], x);
      const int64_t j0 = i * VEC;
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        float z = x[k];
        if constexpr (SCALE) z = E::scale(z, temperature);
        x[k] = grad(z, j0 + k);
      }
      dv[i] = E::pack(x);
    }
    tail_begin = nvec * VEC;
  }
  for (int64_t j = tail_begin + lane; j < V; j += kWave) {
    float z = E::load1(xr + j);
    if constexpr (SCALE) z = E::scale(z, temperature);
    E::store1(dr + j, grad(z, j));
  }
}

template <typename T>
int launch_fwd(const void *logits, int64_t n_rows, int64_t V, int64_t stride,
               const int64_t *labels, float temperature, float *logp, float *entropy,
               float *lse, hipStream_t stream) {
  const T *x = static_cast<const T *>(logits);
  const bool vec = (reinterpret_cast<uintptr_t>(logits) % 16 == 0) &&
                   ((stride * static_cast<int64_t>(sizeof(T))) % 16 == 0);
  const bool scale = (temperature != 1.0f);
  const dim3 block(256);
  const dim3 grid(static_cast<unsigned>((n_rows + 3) / 4));
#define VA_LAUNCH_FWD(S, VV)                                                                 \
  hipLaunchKernelGGL((logprob_entropy_fwd_kernel<T, S, VV>), grid, block, 0, stream, x, n_rows, \
                     V, stride, labels, temperature, logp, entropy, lse)
  if (scale) {
    if (vec) VA_LAUNCH_FWD(true, true); else VA_LAUNCH_FWD(true, false);
  } else {
    if (vec) VA_LAUNCH_FWD(false, true); else VA_LAUNCH_FWD(false, false);
  }
#undef VA_LAUNCH_FWD
  return check_launch("logprob_entropy_fwd");
}

template <typename T>
int launch_bwd(const float *g_logp, const float *g_ent, const void *logits, int64_t n_rows,
               int64_t V, int64_t stride, const int64_t *labels, const float *lse,
               const float *ent, float temperature, void *dlogits, int64_t dstride,
               hipStream_t stream) {
  const T *x = static_cast<const T *>(logits);
  T *d = static_cast<T *>(dlogits);
  const bool vec = (reinterpret_cast<uintptr_t>(logits) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(dlogits) % 16 == 0) &&
                   ((stride * static_cast<int64_t>(sizeof(T))) % 16 == 0) &&
                   ((dstride * static_cast<int64_t>(sizeof(T))) % 16 == 0);
  const bool scale = (temperature != 1.0f);
  const dim3 block(256);
  const dim3 grid(static_cast<unsigned>((n_rows + 3) / 4));
#define VA_LAUNCH_BWD(S, VV)                                                                  \
  hipLaunchKernelGGL((logprob_entropy_bwd_kernel<T, S, VV>), grid, block, 0, stream, g_logp,    \
                     g_ent, x, n_rows, V, stride, labels, lse, ent, temperature, d, dstride)
  if (scale) {
    if (vec) VA_LAUNCH_BWD(true, true); else VA_LAUNCH_BWD(true, false);
  } else {
    if (vec) VA_LAUNCH_BWD(false, true); else VA_LAUNCH_BWD(false, false);
  }
#undef VA_LAUNCH_BWD
  return check_launch("logprob_entropy_bwd");
}

}  // namespace
}  // namespace va

extern "C" int va_logprob_entropy_fwd(const void *logits, int dtype, int64_t n_rows,
                                      int64_t vocab, int64_t row_stride, const int64_t *labels,
                                      float temperature, float *logp, float *entropy,
                                      float *lse, void *stream) {
  VA_CHECK_ARG(n_rows >= 0, "n_rows must be >= 0 (got %lld)", (long long)n_rows);
  if (n_rows == 0) return VA_OK;
  VA_CHECK_ARG(vocab > 0 && row_stride >= vocab, "bad vocab/row_stride (%lld/%lld)",
               (long long)vocab, (long long)row_stride);
  VA_CHECK_ARG(logits && labels && logp && lse, "null pointer argument");
  VA_CHECK_ARG(temperature > 0.f, "temperature must be > 0");
  VA_CHECK_ARG((n_rows + 3) / 4 < (1ll << 31), "too many rows");
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (dtype) {
    case VA_F32:
      return va::launch_fwd<float>(logits, n_rows, vocab, row_stride, labels, temperature, logp,
                                   entropy, lse, s);
    case VA_BF16:
      return va::launch_fwd<va::bf16_t>(logits, n_rows, vocab, row_stride, labels, temperature,
                                        logp, entropy, lse, s);
    case VA_F16:
      return va::launch_fwd<va::f16_t>(logits, n_rows, vocab, row_stride, labels, temperature,
                                       logp, entropy, lse, s);
    default:
      va::set_error("unsupported logits dtype %d", dtype);
      return VA_E_ARG;
  }
}

extern "C" int va_logprob_entropy_bwd(const float *g_logp, const float *g_entropy,
                                      const void *logits, int dtype, int64_t n_rows,
                                      int64_t vocab, int64_t row_stride, const int64_t *labels,
                                      const float *lse, const float *entropy, float temperature,
                                      void *dlogits, int64_t dlogits_row_stride, void *stream) {
  VA_CHECK_ARG(n_rows >= 0, "n_rows must be >= 0");
  if (n_rows == 0) return VA_OK;
  VA_CHECK_ARG(vocab > 0 && row_stride >= vocab && dlogits_row_stride >= vocab,
               "bad vocab/row strides");
  VA_CHECK_ARG(logits && labels && lse && dlogits, "null pointer argument");
  VA_CHECK_ARG(g_entropy == nullptr || entropy != nullptr,
               "entropy is required when g_entropy is given");
  VA_CHECK_ARG(temperature > 0.f, "temperature must be > 0");
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (dtype) {
    case VA_F32:
      return va::launch_bwd<float>(g_logp, g_entropy, logits, n_rows, vocab, row_stride, labels,
                                   lse, entropy, temperature, dlogits, dlogits_row_stride, s);
    case VA_BF16:
      return va::launch_bwd<va::bf16_t>(g_logp, g_entropy, logits, n_rows, vocab, row_stride,
                                        labels, lse, entropy, temperature, dlogits,
                                        dlogits_row_stride, s);
    case VA_F16:
      return va::launch_bwd<va::f16_t>(g_logp, g_entropy, logits, n_rows, vocab, row_stride,
                                       labels, lse, entropy, temperature, dlogits,
                                       dlogits_row_stride, s);
    default:
      va::set_error("unsupported logits dtype %d", dtype);
      return VA_E_ARG;
  }
}
