// Multi-tensor accumulation of bf16 / fp16 / fp32 parameter gradients into fp32 master-gradient
// buckets — the mixed-precision half of the DP gradient path (the reference's FSDP keeps fp32
// gradients for reduction, fsdp_workers.py:337-347).
//
// One launch per gradient bucket instead of one mixed-dtype elementwise launch per parameter.
// The tensor list travels in the kernel arguments (up to kMaxTensors per launch); workgroups are
// dealt to tensors by a prefix table of chunk counts. 16-byte loads/stores where aligned.
// Bound: HBM, 2 (src) + 4 + 4 (dst read + write) = 10 bytes per bf16 element.

#include "va_common.h"

namespace va {
namespace {

constexpr int kMaxTensors = 40;
constexpr int kChunk = 256 * 8 * 2;  // elements per workgroup

struct TensorList {
  const void *src[kMaxTensors];
  float *dst[kMaxTensors];
  int64_t numel[kMaxTensors];
  int32_t chunk_begin[kMaxTensors + 1];
  int32_t n;
};

template <int DT>
__device__ __forceinline__ float ld(const void *p, int64_t i) {
  if constexpr (DT == VA_F32) return static_cast<const float *>(p)[i];
  else if constexpr (DT == VA_BF16) return bf16_to_f32(static_cast<const uint16_t *>(p)[i]);
  else return f16_to_f32(static_cast<const uint16_t *>(p)[i]);
}

template <int DT>
__global__ __launch_bounds__(256) void accumulate_kernel(TensorList tl, float scale) {
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < tl.n && tl.chunk_begin[t + 1] <= b) ++t;
  const int64_t n = tl.numel[t];
  const int64_t beg = static_cast<int64_t>(b - tl.chunk_begin[t]) * kChunk;
  const int64_t end = (beg + kChunk < n) ? beg + kChunk : n;
  const void *src = tl.src[t];
  float *dst = tl.dst[t];
  const bool vec = DT == VA_BF16 && (reinterpret_cast<uintptr_t>(src) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(dst) % 16 == 0);
  if (vec) {
    // 8 bf16 (16 B) -> 2 x float4 per lane per step
    for (int64_t i = beg + threadIdx.x * 8; i + 8 <= end; i += 256 * 8) {
      const uint4 s = *reinterpret_cast<const uint4 *>(static_cast<const uint16_t *>(src) + i);
      float4 *d = reinterpret_cast<float4 *>(dst + i);
      float4 d0 = d[0], d1 = d[1];
      d0.x += scale * bf16_lo(s.x); d0.y += scale * bf16_hi(s.x);
      d0.z += scale * bf16_lo(s.y); d0.w += scale * bf16_hi(s.y);
      d1.x += scale * bf16_lo(s.z); d1.y += scale * bf16_hi(s.z);
      d1.z += scale * bf16_lo(s.w); d1.w += scale * bf16_hi(s.w);
      d[0] = d0;
      d[1] = d1;
    }
    // ragged tail of the last chunk
    const int64_t full = beg + ((end - beg) / 8) * 8;
    for (int64_t i = full + threadIdx.x; i < end; i += 256) dst[i] += scale * ld<DT>(src, i);
  } else {
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) dst[i] += scale * ld<DT>(src, i);
  }
}

}  // namespace
}  // namespace va

extern "C" int va_accumulate_grads(int n_tensors, const void *const *src, const int64_t *numel,
                                   int src_dtype, float *const *dst, float scale, void *stream) {
  VA_CHECK_ARG(n_tensors >= 0, "n_tensors < 0");
  VA_CHECK_ARG(n_tensors == 0 || (src && numel && dst), "null pointer argument");
  VA_CHECK_ARG(src_dtype == VA_F32 || src_dtype == VA_BF16 || src_dtype == VA_F16, "bad dtype %d",
               src_dtype);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int i = 0;
  while (i < n_tensors) {
    va::TensorList tl;
    tl.n = 0;
    int32_t chunks = 0;
    while (i < n_tensors && tl.n < va::kMaxTensors) {
      VA_CHECK_ARG(numel[i] >= 0 && (src[i] || numel[i] == 0), "bad tensor %d", i);
      if (numel[i] > 0) {
        const int64_t c = (numel[i] + va::kChunk - 1) / va::kChunk;
        VA_CHECK_ARG(chunks + c < (1ll << 31), "too many chunks");
        tl.src[tl.n] = src[i];
        tl.dst[tl.n] = dst[i];
        tl.numel[tl.n] = numel[i];
        tl.chunk_begin[tl.n] = chunks;
        chunks += static_cast<int32_t>(c);
        ++tl.n;
      }
      ++i;
    }
    if (tl.n == 0) continue;
    tl.chunk_begin[tl.n] = chunks;
    switch (src_dtype) {
      case VA_F32:
        hipLaunchKernelGGL((va::accumulate_kernel<VA_F32>), dim3(chunks), dim3(256), 0, s, tl, scale);
        break;
      case VA_BF16:
        hipLaunchKernelGGL((va::accumulate_kernel<VA_BF16>), dim3(chunks), dim3(256), 0, s, tl, scale);
        break;
      default:
        hipLaunchKernelGGL((va::accumulate_kernel<VA_F16>), dim3(chunks), dim3(256), 0, s, tl, scale);
        break;
    }
    if (int e = va::check_launch("accumulate_grads")) return e;
  }
  return VA_OK;
}
