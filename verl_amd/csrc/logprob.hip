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

#include <type_traits>

#include "va_common.h"

namespace va {
namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.69314718055994531f;

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

// ---- 16-byte vector access ------------------------------------------------------------
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 vload(const u32x4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void vstore(u32x4 *p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// element k of a 16-byte vector, as fp32
template <typename T>
__device__ __forceinline__ float elem(const u32x4 &r, int k);
template <>
__device__ __forceinline__ float elem<float>(const u32x4 &r, int k) { return __uint_as_float(r[k]); }
template <>
__device__ __forceinline__ float elem<bf16_t>(const u32x4 &r, int k) {
  return (k & 1) ? bf16_hi(r[k >> 1]) : bf16_lo(r[k >> 1]);
}
template <>
__device__ __forceinline__ float elem<f16_t>(const u32x4 &r, int k) {
  const uint32_t w = r[k >> 1];
  return f16_to_f32(static_cast<uint16_t>((k & 1) ? (w >> 16) : (w & 0xffffu)));
}
template <typename T>
__device__ __forceinline__ u32x4 pack_vec(const float *x) {
  const uint4 q = Elem<T>::pack(x);
  u32x4 r = {q.x, q.y, q.z, q.w};
  return r;
}

// Online-softmax update with U raw vectors. Without temperature the fp32 values are re-derived
// from the raw registers in each pass (one VALU op each) instead of being kept live, which keeps
// the kernel at <= 64 VGPRs (8 waves per SIMD).
template <typename T, int U, bool SCALE>
__device__ __forceinline__ void acc_raw(Acc &a, const u32x4 *raw, float temperature) {
  constexpr int VEC = Elem<T>::kVec;
  if constexpr (SCALE) {
    float x[U * VEC];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < VEC; ++k) x[u * VEC + k] = Elem<T>::scale(elem<T>(raw[u], k), temperature);
    acc_chunk<U * VEC>(a, x);
  } else {
    float cm = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < VEC; ++k) cm = fmaxf(cm, elem<T>(raw[u], k));
    const float nm = fmaxf(a.m, cm);
    const float nb = base_of(nm);
    const float alpha = __builtin_amdgcn_exp2f(base_of(a.m) - nb);
    float s0 = 0.f, s1 = 0.f, t0 = 0.f, t1 = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < VEC; k += 2) {
        const float x0 = elem<T>(raw[u], k), x1 = elem<T>(raw[u], k + 1);
        const float e0 = __builtin_amdgcn_exp2f(fmaf(x0, kLog2e, -nb));
        const float e1 = __builtin_amdgcn_exp2f(fmaf(x1, kLog2e, -nb));
        s0 += e0;
        s1 += e1;
        t0 = fmaf(e0, x0, t0);
        t1 = fmaf(e1, x1, t1);
      }
    a.s = fmaf(a.s, alpha, s0 + s1);
    a.t = fmaf(a.t, alpha, t0 + t1);
    a.m = nm;
  }
}

// ---- forward ---------------------------------------------------------------------------
// A 256-thread workgroup = 4 waves = 4/WPR rows; the WPR waves of a row interleave 1 KiB
// segments of it and merge their accumulators through LDS.
template <typename T, bool SCALE, bool VECTOR, int WPR, bool NT, int U, bool PIPE>
__global__ __launch_bounds__(256, 8) void logprob_entropy_fwd_kernel(
    const T *__restrict__ logits, int64_t n_rows, int64_t V, int64_t stride,
    const int64_t *__restrict__ labels, float temperature, float *__restrict__ logp,
    float *__restrict__ entropy, float *__restrict__ lse_out) {
  using E = Elem<T>;
  constexpr int VEC = E::kVec;
  constexpr int RPB = 4 / WPR;
  constexpr int STEP = kWave * WPR;
  __shared__ float sh[4][3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int part = wave % WPR;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * RPB + wave / WPR;
  const bool active = row < n_rows;
  Acc a{-INFINITY, 0.f, 0.f};
  if (active) {
    const T *xr = logits + row * stride;
    int64_t tail_begin = 0;
    if constexpr (VECTOR) {
      const u32x4 *xv = reinterpret_cast<const u32x4 *>(xr);
      const int64_t nvec = V / VEC;
      int64_t i = static_cast<int64_t>(part) * kWave + lane;
      if constexpr (PIPE) {
        // software pipeline: the next U vectors are in flight while the current U are reduced
        if (i + (U - 1) * STEP < nvec) {
          u32x4 cur[U];
#pragma unroll
          for (int u = 0; u < U; ++u) cur[u] = vload<NT>(xv + i + u * STEP);
          while (true) {
            const int64_t nx = i + U * STEP;
            const bool more = nx + (U - 1) * STEP < nvec;
            u32x4 nxt[U];
            if (more) {
#pragma unroll
              for (int u = 0; u < U; ++u) nxt[u] = vload<NT>(xv + nx + u * STEP);
            }
            acc_raw<T, U, SCALE>(a, cur, temperature);
            i = nx;
            if (!more) break;
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
          }
        }
      } else {
        for (; i + (U - 1) * STEP < nvec; i += U * STEP) {
          u32x4 raw[U];
#pragma unroll
          for (int u = 0; u < U; ++u) raw[u] = vload<NT>(xv + i + u * STEP);
          acc_raw<T, U, SCALE>(a, raw, temperature);
        }
      }
      for (; i < nvec; i += STEP) {
        const u32x4 r = vload<NT>(xv + i);
        acc_raw<T, 1, SCALE>(a, &r, temperature);
      }
      tail_begin = nvec * VEC;
    }
    for (int64_t j = tail_begin + static_cast<int64_t>(part) * kWave + lane; j < V; j += STEP) {
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
  }
  if constexpr (WPR > 1) {
    if (lane == 0) {
      sh[wave][0] = a.m;
      sh[wave][1] = a.s;
      sh[wave][2] = a.t;
    }
    __syncthreads();
    if (part == 0 && lane == 0 && active) {
#pragma unroll
      for (int w = 1; w < WPR; ++w) acc_merge(a, sh[wave + w][0], sh[wave + w][1], sh[wave + w][2]);
    }
  }
  if (part == 0 && lane == 0 && active) {
    const T *xr = logits + row * stride;
    // lse = m + ln(s) + ln 2 * (B(m) - m L): keeps the max exact and corrects fl(m L)
    float lse;
    if (a.m == -INFINITY) {
      lse = -INFINITY;
    } else {
      const float corr = -fmaf(a.m, kLog2e, -base_of(a.m));
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
// The gradient is elementwise once the row's (lse, H, g_lp, g_H, label) are known, so the
// backward is a flat stream: workgroup b = chunk b % chunks_per_row of row b / chunks_per_row,
// 256 lanes x U x 16 B contiguous, loaded at once, written once. Workgroups in flight therefore
// sweep a contiguous address range (as a copy does) instead of thousands of rows at once: on
// MI355X this moves read+write from 5.2 to ~5.8 TB/s (tools/hbm_stream.hip calibration).
template <typename T, bool SCALE, bool VECTOR, bool NT, int U>
__global__ __launch_bounds__(256) void logprob_entropy_bwd_kernel(
    const float *__restrict__ g_logp, const float *__restrict__ g_ent, const T *logits,
    int64_t V, int64_t stride, const int64_t *__restrict__ labels, const float *__restrict__ lse_in,
    const float *__restrict__ ent_in, float temperature, T *dlogits, int64_t dstride,
    int chunks_per_row) {
  using E = Elem<T>;
  constexpr int VEC = E::kVec;
  constexpr int CH = 256 * U * VEC;  // elements per workgroup
  const int64_t row = blockIdx.x / chunks_per_row;
  const int64_t e0 = static_cast<int64_t>(blockIdx.x - row * chunks_per_row) * CH;
  const T *xr = logits + row * stride;
  T *dr = dlogits + row * dstride;

  const int64_t lab = labels[row];
  const bool has_lab = (lab >= 0 && lab < V);
  const float glp = (g_logp != nullptr && has_lab) ? g_logp[row] : 0.f;
  const float gh = (g_ent != nullptr) ? g_ent[row] : 0.f;
  const float lse = lse_in[row];
  const float h = (g_ent != nullptr) ? ent_in[row] : 0.f;

  // dz_j = -p_j * (glp + gh * (log p_j + H)) + glp * [j == label];  dx = dz / T.
  // With log p_j = z_j - lse:  p_j = 2^(z_j L - lse L),  glp + gh (log p_j + H) = gh z_j + kk,
  // kk = gh (H - lse) + glp: 2 FMAs + 1 exp + 1 mul per element; the label term is added by the
  // one lane whose vector holds it.
  const float nlb = -lse * kLog2e;
  const float kk = fmaf(gh, h - lse, glp);
  auto grad = [&](float z) -> float {
    const float p = __builtin_amdgcn_exp2f(fmaf(z, kLog2e, nlb));
    return -p * fmaf(gh, z, kk);
  };
  auto finish = [&](float d, bool is_lab) -> float {
    if (is_lab) d += glp;
    if constexpr (SCALE) d = d / temperature;
    return d;
  };

  if constexpr (VECTOR) {
    const u32x4 *xv = reinterpret_cast<const u32x4 *>(xr);
    u32x4 *dv = reinterpret_cast<u32x4 *>(dr);
    const int64_t nvec = V / VEC;
    const int64_t i0 = e0 / VEC + threadIdx.x;
    const int64_t lab_vec = has_lab ? lab / VEC : -1;
    // all U loads issued before any use; the row's partial last chunk clamps its addresses
    // (duplicate in-row reads, no stores) so no load sits behind a branch
    auto body = [&](auto partial) {
      u32x4 raw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (decltype(partial)::value) raw[u] = vload<NT>(xv + min(i0 + u * 256, nvec - 1));
        else raw[u] = vload<NT>(xv + i0 + u * 256);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * 256;
        if (decltype(partial)::value && i >= nvec) continue;
        float x[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          float z = elem<T>(raw[u], k);
          if constexpr (SCALE) z = E::scale(z, temperature);
          x[k] = grad(z);
        }
        if (i == lab_vec) {  // one lane of one workgroup per row
          const int lk = static_cast<int>(lab - i * VEC);
#pragma unroll
          for (int k = 0; k < VEC; ++k)
            if (k == lk) x[k] += glp;
        }
        if constexpr (SCALE) {
#pragma unroll
          for (int k = 0; k < VEC; ++k) x[k] = x[k] / temperature;
        }
        vstore<NT>(dv + i, pack_vec<T>(x));
      }
    };
    if (e0 + CH <= nvec * VEC) body(std::false_type{});
    else body(std::true_type{});
    // V % VEC trailing elements: the row's last workgroup
    if (e0 + CH >= V) {
      for (int64_t j = nvec * VEC + threadIdx.x; j < V; j += 256) {
        float z = E::load1(xr + j);
        if constexpr (SCALE) z = E::scale(z, temperature);
        E::store1(dr + j, finish(grad(z), j == lab));
      }
    }
  } else {
    const int64_t end = min(V, e0 + CH);
    for (int64_t j = e0 + threadIdx.x; j < end; j += 256) {
      float z = E::load1(xr + j);
      if constexpr (SCALE) z = E::scale(z, temperature);
      E::store1(dr + j, finish(grad(z), j == lab));
    }
  }
}

// Flat variant for dense [n_rows, V] logits and dlogits (stride = dstride = V, V a multiple of the
// 16-B vector, V >= one workgroup chunk): the whole tensor is one stream of 16-B vectors cut into
// equal 256 x U-vector chunks, so no workgroup carries a row's partial last chunk (the per-row
// variant launches 19 chunks per 151,936-wide bf16 row, the last one 55 % full). A chunk spans at
// most two rows: their scalars are two uniform loads each, the lane picks by its vector index.
// Per element the arithmetic is the per-row kernel's (bitwise identical results).
template <typename T, bool SCALE, bool NT, int U>
__global__ __launch_bounds__(256) void logprob_entropy_bwd_flat_kernel(
    const float *__restrict__ g_logp, const float *__restrict__ g_ent, const T *logits, int64_t n_rows,
    int64_t V, const int64_t *__restrict__ labels, const float *__restrict__ lse_in,
    const float *__restrict__ ent_in, float temperature, T *dlogits) {
  using E = Elem<T>;
  constexpr int VEC = E::kVec;
  const int64_t nvec_row = V / VEC, nvec = n_rows * nvec_row;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * (256 * U);  // first vector of the chunk
  const int64_t r0 = c0 / nvec_row;                                    // wave-uniform
  const int64_t split = (r0 + 1) * nvec_row;                           // first vector of row r0 + 1
  const bool two = split < nvec && split < c0 + 256 * U;
  const u32x4 *xv = reinterpret_cast<const u32x4 *>(logits);
  u32x4 *dv = reinterpret_cast<u32x4 *>(dlogits);

  u32x4 raw[U];
#pragma unroll
  for (int u = 0; u < U; ++u) raw[u] = vload<NT>(xv + min(c0 + u * 256 + threadIdx.x, nvec - 1));

  // the (up to) two rows' scalars (as the per-row kernel derives them)
  float glp_r[2], gh_r[2], kk_r[2], nlb_r[2];
  int64_t lab_r[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t row = (j == 1 && two) ? r0 + 1 : r0;
    const int64_t lab = labels[row];
    const bool has_lab = (lab >= 0 && lab < V);
    const float glp = (g_logp != nullptr && has_lab) ? g_logp[row] : 0.f;
    const float gh = (g_ent != nullptr) ? g_ent[row] : 0.f;
    const float lse = lse_in[row];
    const float h = (g_ent != nullptr) ? ent_in[row] : 0.f;
    glp_r[j] = glp;
    gh_r[j] = gh;
    kk_r[j] = fmaf(gh, h - lse, glp);
    nlb_r[j] = -lse * kLog2e;
    lab_r[j] = has_lab ? row * nvec_row * VEC + lab : -1;  // flat element index of the label
  }

#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = c0 + u * 256 + threadIdx.x;
    if (i >= nvec) continue;
    const int j = (two && i >= split) ? 1 : 0;
    const float gh = j ? gh_r[1] : gh_r[0], kk = j ? kk_r[1] : kk_r[0], nlb = j ? nlb_r[1] : nlb_r[0];
    float x[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      float z = elem<T>(raw[u], k);
      if constexpr (SCALE) z = E::scale(z, temperature);
      const float p = __builtin_amdgcn_exp2f(fmaf(z, kLog2e, nlb));
      x[k] = -p * fmaf(gh, z, kk);
    }
    const int64_t lab = j ? lab_r[1] : lab_r[0];
    if (lab >= i * VEC && lab < (i + 1) * VEC) {  // one lane per row
      const int lk = static_cast<int>(lab - i * VEC);
      const float glp = j ? glp_r[1] : glp_r[0];
#pragma unroll
      for (int k = 0; k < VEC; ++k)
        if (k == lk) x[k] += glp;
    }
    if constexpr (SCALE) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) x[k] = x[k] / temperature;
    }
    vstore<NT>(dv + i, pack_vec<T>(x));
  }
}

// ---- tuning (va_set_tuning) ---------------------------------------------------------------
int g_fwd_wpr = 0;  // 0 = auto
int g_bwd_wpr = 0;
int g_nt = -1;
int g_bwd_flat = -1;  // -1 auto (flat stream where the layout allows), 0 per-row chunks
int g_pipe = 0;  // 0: 4 vectors per lane, no pipeline; 1: 2+2 pipelined; 2: 4+4 pipelined  // -1 = auto (non-temporal on: +10-12% fwd, +1-2% bwd measured)

int auto_wpr(int64_t n_rows, int64_t V, int override_wpr) {
  if (override_wpr == 1 || override_wpr == 2 || override_wpr == 4) return override_wpr;
  // split long rows over several waves so that a launch is many waves deep per CU slot
  // (avoids the partial last round of 1-wave-per-row at a few thousand rows)
  if (V >= 16384) return 4;
  if (V >= 4096) return 2;
  (void)n_rows;
  return 1;
}

template <typename T, bool S, bool VV, int W>
void launch_fwd_w(const T *x, int64_t n_rows, int64_t V, int64_t stride, const int64_t *labels,
                  float temperature, float *logp, float *entropy, float *lse, hipStream_t stream,
                  bool nt) {
  const dim3 block(256);
  const dim3 grid(static_cast<unsigned>((n_rows + (4 / W) - 1) / (4 / W)));
#define VA_K(NTV, UU, PP)                                                                         \
  hipLaunchKernelGGL((logprob_entropy_fwd_kernel<T, S, VV, W, NTV, UU, PP>), grid, block, 0, stream, x, \
                     n_rows, V, stride, labels, temperature, logp, entropy, lse)
  const int pipe = VV ? g_pipe : 0;
  if (nt) {
    if (pipe == 1) VA_K(true, 2, true); else if (pipe == 2) VA_K(true, 4, true); else VA_K(true, 4, false);
  } else {
    if (pipe == 1) VA_K(false, 2, true); else if (pipe == 2) VA_K(false, 4, true); else VA_K(false, 4, false);
  }
#undef VA_K
}

template <typename T>
int launch_fwd(const void *logits, int64_t n_rows, int64_t V, int64_t stride,
               const int64_t *labels, float temperature, float *logp, float *entropy,
               float *lse, hipStream_t stream) {
  const T *x = static_cast<const T *>(logits);
  const bool vec = (reinterpret_cast<uintptr_t>(logits) % 16 == 0) &&
                   ((stride * static_cast<int64_t>(sizeof(T))) % 16 == 0);
  const bool scale = (temperature != 1.0f);
  const int w = auto_wpr(n_rows, V, g_fwd_wpr);
  const bool nt = g_nt != 0;  // auto (-1) and 1 both select non-temporal
#define VA_FWD(S, VV)                                                                        \
  do {                                                                                       \
    if (w == 4) launch_fwd_w<T, S, VV, 4>(x, n_rows, V, stride, labels, temperature, logp, entropy, lse, stream, nt); \
    else if (w == 2) launch_fwd_w<T, S, VV, 2>(x, n_rows, V, stride, labels, temperature, logp, entropy, lse, stream, nt); \
    else launch_fwd_w<T, S, VV, 1>(x, n_rows, V, stride, labels, temperature, logp, entropy, lse, stream, nt); \
  } while (0)
  if (scale) {
    if (vec) VA_FWD(true, true); else VA_FWD(true, false);
  } else {
    if (vec) VA_FWD(false, true); else VA_FWD(false, false);
  }
#undef VA_FWD
  return check_launch("logprob_entropy_fwd");
}

template <typename T, bool S, bool VV>
void launch_bwd_u(const float *g_logp, const float *g_ent, const T *x, int64_t n_rows, int64_t V,
                  int64_t stride, const int64_t *labels, const float *lse, const float *ent,
                  float temperature, T *d, int64_t dstride, hipStream_t stream, bool nt) {
  // vectors per lane: 4 (default), 2 (VA_TUNE_PIPELINE = 1) or 8 (= 2)
  const int u = g_pipe == 1 ? 2 : (g_pipe == 2 ? 8 : 4);
  const int64_t ch = 256LL * u * Elem<T>::kVec;
  const int cpr = static_cast<int>((V + ch - 1) / ch);
  const dim3 block(256), grid(static_cast<unsigned>(n_rows * cpr));
#define VA_K(NTV, UU)                                                                          \
  hipLaunchKernelGGL((logprob_entropy_bwd_kernel<T, S, VV, NTV, UU>), grid, block, 0, stream, g_logp, g_ent, x, V, \
                     stride, labels, lse, ent, temperature, d, dstride, cpr)
  if (nt) {
    if (u == 2) VA_K(true, 2); else if (u == 8) VA_K(true, 8); else VA_K(true, 4);
  } else {
    if (u == 2) VA_K(false, 2); else if (u == 8) VA_K(false, 8); else VA_K(false, 4);
  }
#undef VA_K
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
  const bool nt = g_nt != 0;  // auto (-1) and 1 both select non-temporal
  const int fu = g_pipe == 1 ? 2 : (g_pipe == 2 ? 8 : 4);  // vectors per lane, as the per-row path
  const int64_t nvec_row = V / Elem<T>::kVec;
  if (g_bwd_flat != 0 && vec && stride == V && dstride == V && V % Elem<T>::kVec == 0 &&
      nvec_row >= 256 * fu) {
    const int64_t chunks = (n_rows * nvec_row + 256 * fu - 1) / (256 * fu);
    const dim3 block(256), grid(static_cast<unsigned>(chunks));
#define VA_KF(S, NTV, UU)                                                                         \
  hipLaunchKernelGGL((logprob_entropy_bwd_flat_kernel<T, S, NTV, UU>), grid, block, 0, stream, g_logp, \
                     g_ent, x, n_rows, V, labels, lse, ent, temperature, d)
#define VA_KFU(S, NTV) \
  do { if (fu == 2) VA_KF(S, NTV, 2); else if (fu == 8) VA_KF(S, NTV, 8); else VA_KF(S, NTV, 4); } while (0)
    if (scale) {
      if (nt) VA_KFU(true, true); else VA_KFU(true, false);
    } else {
      if (nt) VA_KFU(false, true); else VA_KFU(false, false);
    }
#undef VA_KFU
#undef VA_KF
    return check_launch("logprob_entropy_bwd");
  }
#define VA_BWD(S, VV) \
  launch_bwd_u<T, S, VV>(g_logp, g_ent, x, n_rows, V, stride, labels, lse, ent, temperature, d, dstride, stream, nt)
  if (scale) {
    if (vec) VA_BWD(true, true); else VA_BWD(true, false);
  } else {
    if (vec) VA_BWD(false, true); else VA_BWD(false, false);
  }
#undef VA_BWD
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
  VA_CHECK_ARG(n_rows * ((vocab + 2047) / 2048) < (1LL << 31), "too many rows x vocab chunks for one launch");
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

extern int g_flash_grouped_dkdv;  // attention.hip
extern int g_gae_variant;         // advantage.hip
extern int g_gae_partials;        // advantage.hip
extern int g_gae_nt;              // advantage.hip
extern int g_loss_vec;            // loss.hip
extern int g_whiten_slice_min;    // advantage.hip
extern int g_linear_logprob_tile;  // linear_logprob.hip
extern int g_wgrad_remainder;      // wgrad.hip
extern int g_wgrad_mfma;           // wgrad.hip
extern int g_wgrad_tiles;          // wgrad.hip
extern int g_adamw_math;           // optim.hip
extern int g_wgrad_kind;           // wgrad.hip
extern int g_linear_tn;            // gemm_tn.hip
extern int g_t256_defer;           // linear_logprob.hip
extern int g_whiten_grid;         // advantage.hip
extern int g_swiglu_variant;      // model_ops.hip
extern int g_flash_dkdv_qt;       // attention.hip
extern int g_flash_dq_kb;         // attention.hip
extern int g_flash_fwd_kb;        // attention.hip
extern int g_flash_dma;           // attention.hip

extern "C" int va_set_tuning(int key, int value) {
  switch (key) {
    case VA_TUNE_FWD_WAVES_PER_ROW: va::g_fwd_wpr = value; return VA_OK;
    case VA_TUNE_BWD_WAVES_PER_ROW: va::g_bwd_wpr = value; return VA_OK;
    case VA_TUNE_NONTEMPORAL: va::g_nt = value; return VA_OK;
    case VA_TUNE_PIPELINE: va::g_pipe = value; return VA_OK;
    case VA_TUNE_FLASH_GROUPED_DKDV: g_flash_grouped_dkdv = value; return VA_OK;
    case VA_TUNE_GAE_VARIANT: g_gae_variant = value; return VA_OK;
    case VA_TUNE_GAE_PARTIALS:
      if (value != 0 && value != 1 && value != 4 && value != 8) {
        va::set_error("VA_TUNE_GAE_PARTIALS must be 0, 1, 4 or 8 (got %d)", value);
        return VA_E_ARG;
      }
      g_gae_partials = value;
      return VA_OK;
    case VA_TUNE_GAE_NT: g_gae_nt = value & 7; return VA_OK;
    case VA_TUNE_LOSS_VEC: g_loss_vec = value; return VA_OK;
    case VA_TUNE_WGRAD_REMAINDER: g_wgrad_remainder = value; return VA_OK;
    case VA_TUNE_WGRAD_MFMA:
      if (value != 16 && value != 32) {
        va::set_error("va_set_tuning: VA_TUNE_WGRAD_MFMA must be 16 or 32");
        return VA_E_ARG;
      }
      g_wgrad_mfma = value;
      return VA_OK;
    case VA_TUNE_WGRAD_KIND:
      if (value < -1 || value > 6) {
        va::set_error("va_set_tuning: VA_TUNE_WGRAD_KIND must be -1 .. 6");
        return VA_E_ARG;
      }
      g_wgrad_kind = value;
      return VA_OK;
    case VA_TUNE_T256_DEFER:
      if (value < 0 || value > 7) {
        va::set_error("va_set_tuning: VA_TUNE_T256_DEFER must be 0 .. 7");
        return VA_E_ARG;
      }
      g_t256_defer = value;
      return VA_OK;
    case VA_TUNE_LINEAR_TN:
      if (value < 0 || value > 2) {
        va::set_error("va_set_tuning: VA_TUNE_LINEAR_TN must be 0 .. 2");
        return VA_E_ARG;
      }
      g_linear_tn = value;
      return VA_OK;
    case VA_TUNE_ADAMW_MATH:
      if (value < 0 || value > 7) {
        va::set_error("va_set_tuning: VA_TUNE_ADAMW_MATH must be 0 .. 7");
        return VA_E_ARG;
      }
      g_adamw_math = value;
      return VA_OK;
    case VA_TUNE_WGRAD_TILES:
      if (value < 0 || value > 4) {
        va::set_error("va_set_tuning: VA_TUNE_WGRAD_TILES must be 0 .. 4");
        return VA_E_ARG;
      }
      g_wgrad_tiles = value;
      return VA_OK;
    case VA_TUNE_LINEAR_LOGPROB_TILE:
      if (value != 128 && value != 256) {
        va::set_error("VA_TUNE_LINEAR_LOGPROB_TILE must be 128 or 256 (got %d)", value);
        return VA_E_ARG;
      }
      g_linear_logprob_tile = value;
      return VA_OK;
    case VA_TUNE_WHITEN_SLICE_MIN: g_whiten_slice_min = value < 0 ? 0 : value; return VA_OK;
    case VA_TUNE_WHITEN_GRID:
      if (value < 1 || value > 65536) {
        va::set_error("VA_TUNE_WHITEN_GRID must be 1..65536 (got %d)", value);
        return VA_E_ARG;
      }
      g_whiten_grid = value;
      return VA_OK;
    case VA_TUNE_BWD_FLAT: va::g_bwd_flat = value; return VA_OK;
    case VA_TUNE_SWIGLU_STREAM: g_swiglu_variant = value; return VA_OK;
    case VA_TUNE_FLASH_DKDV_QT:
      if (value != 32 && value != 64 && value != 128) {
        va::set_error("VA_TUNE_FLASH_DKDV_QT must be 32, 64 or 128 (got %d)", value);
        return VA_E_ARG;
      }
      g_flash_dkdv_qt = value;
      return VA_OK;
    case VA_TUNE_FLASH_DQ_KB:
      if (value != 64 && value != 128) {
        va::set_error("VA_TUNE_FLASH_DQ_KB must be 64 or 128 (got %d)", value);
        return VA_E_ARG;
      }
      g_flash_dq_kb = value;
      return VA_OK;
    case VA_TUNE_FLASH_FWD_KB:
      if (value != 64 && value != 128) {
        va::set_error("VA_TUNE_FLASH_FWD_KB must be 64 or 128 (got %d)", value);
        return VA_E_ARG;
      }
      g_flash_fwd_kb = value;
      return VA_OK;
    case VA_TUNE_FLASH_DMA: g_flash_dma = value & 7; return VA_OK;
    default: va::set_error("unknown tuning key %d", key); return VA_E_ARG;
  }
}
