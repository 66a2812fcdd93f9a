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
