// Shared device helpers for the gfx950 kernels of libverl_amd.
// Wave = 64 lanes (CDNA4); every reduction below is written for that width.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/verl_amd.h"

namespace va {

constexpr int kWave = 64;

// ---------------------------------------------------------------- error reporting (host)
void set_error(const char *fmt, ...);
int check_launch(const char *what);

// ---------------------------------------------------------------- dtype helpers (device)
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
// Round-to-nearest-even f32 -> bf16 bits; NaN stays NaN (quiet).
__device__ __forceinline__ uint32_t f32_to_bf16_bits(float f) {
  uint32_t u = __float_as_uint(f);
  uint32_t r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  return ((u & 0x7fffffffu) > 0x7f800000u) ? ((u >> 16) | 0x40u) : r;
}
// the same RNE conversion in one v_cvt_pk_bf16_f32 (2 values per instruction)
typedef float va_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 va_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(va_f32x2{a, b}, va_bf16x2));
}
__device__ __forceinline__ float round_to_bf16(float x) { return __uint_as_float(pack2_bf16(x, 0.f) << 16); }
// logistic sigmoid and SiLU as every SwiGLU kernel computes them (forward, backward, the fused gate|up
// epilogue: one definition, so they agree bitwise): v_exp_f32 (__expf) and the hardware reciprocal
// v_rcp_f32 (1 ulp) instead of an IEEE division, whose div_scale / div_fmas / div_fixup expansion costs
// ~6 VALU slots more per element (hidden in the streaming kernels, not in an MFMA epilogue)
__device__ __forceinline__ float va_sigmoid(float g) { return __builtin_amdgcn_rcpf(1.f + __expf(-g)); }
__device__ __forceinline__ float va_silu(float g) { return g * va_sigmoid(g); }
__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  return static_cast<float>(__builtin_bit_cast(_Float16, h));
}
__device__ __forceinline__ uint32_t f32_to_f16_bits(float f) {
  return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<_Float16>(f)));
}

// Mask element -> float weight (response_mask is int64 in the reference, float/bool in tests).
template <int MT>
__device__ __forceinline__ float load_mask(const void *p, int64_t i) {
  if constexpr (MT == VA_MASK_F32) return static_cast<const float *>(p)[i];
  else if constexpr (MT == VA_MASK_I64) return static_cast<float>(static_cast<const int64_t *>(p)[i]);
  else if constexpr (MT == VA_MASK_I32) return static_cast<float>(static_cast<const int32_t *>(p)[i]);
  else return static_cast<float>(static_cast<const uint8_t *>(p)[i]);
}

// 16-byte fp32 vector access with an optional non-temporal (streaming) hint.
typedef float va_f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld4(const float *p, bool nt) {
  const va_f32x4 v = nt ? __builtin_nontemporal_load(reinterpret_cast<const va_f32x4 *>(p))
                        : *reinterpret_cast<const va_f32x4 *>(p);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st4(float *p, float4 v, bool nt) {
  const va_f32x4 w{v.x, v.y, v.z, v.w};
  if (nt) __builtin_nontemporal_store(w, reinterpret_cast<va_f32x4 *>(p));
  else *reinterpret_cast<va_f32x4 *>(p) = w;
}

// Four consecutive mask elements starting at i (i % 4 == 0, base 16-byte aligned): one 16-byte
// load for f32 / i32, two for i64, one 4-byte load for u8.
template <int MT>
__device__ __forceinline__ void load_mask4(const void *p, int64_t i, float (&o)[4]) {
  if constexpr (MT == VA_MASK_F32) {
    const float4 q = *reinterpret_cast<const float4 *>(static_cast<const float *>(p) + i);
    o[0] = q.x, o[1] = q.y, o[2] = q.z, o[3] = q.w;
  } else if constexpr (MT == VA_MASK_I64) {
    const longlong2 *q = reinterpret_cast<const longlong2 *>(static_cast<const int64_t *>(p) + i);
    const longlong2 a = q[0], b = q[1];
    o[0] = static_cast<float>(a.x), o[1] = static_cast<float>(a.y);
    o[2] = static_cast<float>(b.x), o[3] = static_cast<float>(b.y);
  } else if constexpr (MT == VA_MASK_I32) {
    const int4 q = *reinterpret_cast<const int4 *>(static_cast<const int32_t *>(p) + i);
    o[0] = static_cast<float>(q.x), o[1] = static_cast<float>(q.y);
    o[2] = static_cast<float>(q.z), o[3] = static_cast<float>(q.w);
  } else {
    const uint32_t w = *reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(p) + i);
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = static_cast<float>((w >> (8 * q)) & 0xffu);
  }
}

// Pin a loaded value in registers: the empty asm makes the value an asm output, so the compiler
// cannot drop it under register pressure and re-issue the (read-only) load later, which would put
// a second memory round trip on the wave's critical path.
__device__ __forceinline__ void pin4(float4 &x) {
  asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w));
}
__device__ __forceinline__ void pin1(uint32_t &x) { asm volatile("" : "+v"(x)); }
// Keep the loads issued so far above the pins that follow (a pin consumes its register, so a load
// the compiler sank below an earlier pin would wait for that pin's load first).
__device__ __forceinline__ void loads_issued() { asm volatile("" ::: "memory"); }

// The same split in two: the raw 16-byte loads (issued with the other streams' loads) and the
// conversion (done where the values are used), so no load waits on an earlier conversion.
template <int MT> struct Mask4Raw { float4 f; };
template <> struct Mask4Raw<VA_MASK_I64> { longlong2 a, b; };
template <> struct Mask4Raw<VA_MASK_I32> { int4 q; };
template <> struct Mask4Raw<VA_MASK_U8> { uint32_t w; };

template <int MT>
__device__ __forceinline__ Mask4Raw<MT> load_mask4_raw(const void *p, int64_t i) {
  Mask4Raw<MT> r;
  if constexpr (MT == VA_MASK_F32) {
    r.f = *reinterpret_cast<const float4 *>(static_cast<const float *>(p) + i);
  } else if constexpr (MT == VA_MASK_I64) {
    const longlong2 *q = reinterpret_cast<const longlong2 *>(static_cast<const int64_t *>(p) + i);
    r.a = q[0], r.b = q[1];
  } else if constexpr (MT == VA_MASK_I32) {
    r.q = *reinterpret_cast<const int4 *>(static_cast<const int32_t *>(p) + i);
  } else {
    r.w = *reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(p) + i);
  }
  return r;
}

template <int MT>
__device__ __forceinline__ void pin_mask4(Mask4Raw<MT> &r) {
  if constexpr (MT == VA_MASK_F32) {
    pin4(r.f);
  } else if constexpr (MT == VA_MASK_I64) {
    asm volatile("" : "+v"(r.a.x), "+v"(r.a.y), "+v"(r.b.x), "+v"(r.b.y));
  } else if constexpr (MT == VA_MASK_I32) {
    asm volatile("" : "+v"(r.q.x), "+v"(r.q.y), "+v"(r.q.z), "+v"(r.q.w));
  } else {
    pin1(r.w);
  }
}

template <int MT>
__device__ __forceinline__ void cvt_mask4(const Mask4Raw<MT> &r, float (&o)[4]) {
  if constexpr (MT == VA_MASK_F32) {
    o[0] = r.f.x, o[1] = r.f.y, o[2] = r.f.z, o[3] = r.f.w;
  } else if constexpr (MT == VA_MASK_I64) {
    o[0] = static_cast<float>(r.a.x), o[1] = static_cast<float>(r.a.y);
    o[2] = static_cast<float>(r.b.x), o[3] = static_cast<float>(r.b.y);
  } else if constexpr (MT == VA_MASK_I32) {
    o[0] = static_cast<float>(r.q.x), o[1] = static_cast<float>(r.q.y);
    o[2] = static_cast<float>(r.q.z), o[3] = static_cast<float>(r.q.w);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = static_cast<float>((r.w >> (8 * q)) & 0xffu);
  }
}

// ---------------------------------------------------------------- wave / block reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum of NV doubles; every thread gets the totals. `scratch` holds NV * nwaves
// doubles. Deterministic: fixed xor-tree inside waves, waves summed in index order.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double *scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) scratch[w * NV + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = 0.0;
    for (int j = 0; j < nw; ++j) s += scratch[j * NV + k];
    v[k] = s;
  }
  __syncthreads();
}

// Chan et al. merge of (count, mean, M2) statistics; exact in exact arithmetic.
struct Moments {
  double n, mean, m2;
};
__device__ __forceinline__ Moments merge_moments(Moments a, Moments b) {
  if (b.n == 0.0) return a;
  if (a.n == 0.0) return b;
  const double n = a.n + b.n;
  const double d = b.mean - a.mean;
  Moments r;
  r.n = n;
  r.mean = a.mean + d * (b.n / n);
  r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / n);
  return r;
}

}  // namespace va

#define VA_CHECK_ARG(cond, ...)        \
  do {                                 \
    if (!(cond)) {                     \
      ::va::set_error(__VA_ARGS__);    \
      return VA_E_ARG;                 \
    }                                  \
  } while (0)

#define VA_DISPATCH_MASK(mt, KERNEL_CALL)                                    \
  switch (mt) {                                                              \
    case VA_MASK_F32: { constexpr int MT = VA_MASK_F32; KERNEL_CALL; break; } \
    case VA_MASK_I64: { constexpr int MT = VA_MASK_I64; KERNEL_CALL; break; } \
    case VA_MASK_I32: { constexpr int MT = VA_MASK_I32; KERNEL_CALL; break; } \
    case VA_MASK_U8: { constexpr int MT = VA_MASK_U8; KERNEL_CALL; break; }   \
    default: ::va::set_error("unknown mask dtype %d", (int)(mt)); return VA_E_ARG; \
  }
