// AdamW over flat fp32 buffers — the optimizer half of the actor's _optimizer_step (dp_actor.py:272-288:
// clip_grad_norm_, then actor_optimizer.step() = torch.optim.AdamW, fsdp_workers.py:418-423), for the
// parameter manager's flat master / gradient buckets (workers/grad_sync.MixedPrecisionParams).
//
// torch's fused AdamW runs over the ~290 per-parameter views of those buckets in ~100 multi-tensor
// launches at ~2.4 TB/s (profiles/r06/d: 5.7 ms per step); here one streaming launch per bucket, with
// the gradient clip's scale (the clip's in-place multiply, folded) and the gradient zeroing of the next
// zero_grad (folded) in the same pass. Arithmetic: torch's fused ADAMW step (ATen
// native/cuda/fused_adam_utils.cuh adam_math, ADAMW mode, no amsgrad / maximize), including its
// double-precision intermediates: decoupled weight decay, the two moment updates in double rounded to
// fp32 (the multiply-adds contracted to FMAs, as torch's build compiles them), step_size = lr /
// bias_correction1 and denom = sqrt(v) / sqrt(bias_correction2) + eps, correctly rounded.
// A non-finite gradient norm (found_inf != 0) leaves parameters and moments untouched (the GradScaler
// skip of torch's fused kernel); the gradients are still zeroed when asked (the reference drops them).
// Bound: HBM, 28 B per element (p, g, m, v read; p, m, v written) + 4 B with the zeroing.

#include "va_common.h"

namespace va {
namespace {

struct AdamWArgs {
  double lr, beta1, beta2, eps, weight_decay;
};

// MATH (va_set_tuning VA_TUNE_ADAMW_MATH, for matching torch's build): bit 1 = v_sqrt_f32 (1 ulp)
// instead of the correctly rounded square root, bit 2 = divisions by the hardware reciprocal, bit 4 =
// the double-precision multiply-adds contracted to FMAs
template <int MATH>
__device__ __forceinline__ float w_sqrt(float x) {
  if constexpr (MATH & 1) return __builtin_amdgcn_sqrtf(x);
  else return sqrtf(x);
}
template <int MATH>
__device__ __forceinline__ float w_div(float a, float b) {
  if constexpr (MATH & 2) return a * __builtin_amdgcn_rcpf(b);
  else return a / b;
}

template <int MATH>
__device__ __forceinline__ void adamw_elem(float &p, float g, float &m, float &v, const AdamWArgs &a, float step_size,
                                           float bc2_sqrt) {
  const double pd = p, gd = g;
  if constexpr (MATH & 4) {
    if (a.weight_decay != 0.0) p = static_cast<float>(fma(-(a.lr * a.weight_decay), pd, pd));
    m = static_cast<float>(fma(a.beta1, static_cast<double>(m), (1.0 - a.beta1) * gd));
    v = static_cast<float>(fma(a.beta2, static_cast<double>(v), (1.0 - a.beta2) * gd * gd));
  } else {
    if (a.weight_decay != 0.0) p = static_cast<float>(pd - a.lr * a.weight_decay * pd);
    m = static_cast<float>(a.beta1 * static_cast<double>(m) + (1.0 - a.beta1) * gd);
    v = static_cast<float>(a.beta2 * static_cast<double>(v) + (1.0 - a.beta2) * gd * gd);
  }
  const float denom = static_cast<float>(static_cast<double>(w_div<MATH>(w_sqrt<MATH>(v), bc2_sqrt)) + a.eps);
  p -= w_div<MATH>(step_size * m, denom);
}

template <int MATH>
__global__ __launch_bounds__(256) void adamw_flat_kernel(float *__restrict__ param, float *__restrict__ grad,
                                                         float *__restrict__ exp_avg, float *__restrict__ exp_avg_sq,
                                                         int64_t n, AdamWArgs a, const float *__restrict__ step,
                                                         const float *__restrict__ grad_scale,
                                                         const float *__restrict__ found_inf, int zero_grad) {
  const bool skip = found_inf != nullptr && *found_inf != 0.f;
  const int64_t n4 = n / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  if (skip) {
    if (zero_grad) {
      for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride)
        reinterpret_cast<float4 *>(grad)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int64_t i = n4 * 4 + static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        grad[i] = 0.f;
    }
    return;
  }
  // the fused kernel's per-step constants (double, then the fp32 its adam_math takes)
  const double st = static_cast<double>(*step);
  const float bc1 = static_cast<float>(1.0 - pow(a.beta1, st));
  const float bc2_sqrt = static_cast<float>(sqrt(1.0 - pow(a.beta2, st)));
  const float step_size = static_cast<float>(a.lr / static_cast<double>(bc1));
  const float scale = grad_scale != nullptr ? *grad_scale : 1.f;
  const bool scaled = grad_scale != nullptr;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = reinterpret_cast<const float4 *>(param)[i];
    float4 g = reinterpret_cast<const float4 *>(grad)[i];
    float4 m = reinterpret_cast<const float4 *>(exp_avg)[i];
    float4 v = reinterpret_cast<const float4 *>(exp_avg_sq)[i];
    if (scaled) {  // the clip's in-place grads *= coef (fp32), folded
      g.x *= scale; g.y *= scale; g.z *= scale; g.w *= scale;
    }
    adamw_elem<MATH>(p.x, g.x, m.x, v.x, a, step_size, bc2_sqrt);
    adamw_elem<MATH>(p.y, g.y, m.y, v.y, a, step_size, bc2_sqrt);
    adamw_elem<MATH>(p.z, g.z, m.z, v.z, a, step_size, bc2_sqrt);
    adamw_elem<MATH>(p.w, g.w, m.w, v.w, a, step_size, bc2_sqrt);
    reinterpret_cast<float4 *>(param)[i] = p;
    reinterpret_cast<float4 *>(exp_avg)[i] = m;
    reinterpret_cast<float4 *>(exp_avg_sq)[i] = v;
    if (zero_grad) reinterpret_cast<float4 *>(grad)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int64_t i = n4 * 4 + static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    float p = param[i], g = grad[i], m = exp_avg[i], v = exp_avg_sq[i];
    if (scaled) g *= scale;
    adamw_elem<MATH>(p, g, m, v, a, step_size, bc2_sqrt);
    param[i] = p;
    exp_avg[i] = m;
    exp_avg_sq[i] = v;
    if (zero_grad) grad[i] = 0.f;
  }
}

}  // namespace
}  // namespace va

using namespace va;

// va_set_tuning(VA_TUNE_ADAMW_MATH), see adamw_elem; default 4 (correctly rounded sqrt / divisions,
// the double multiply-adds as FMAs): bitwise equal to torch 2.10.0+rocm7.0's fused AdamW on 1M
// elements x 5 steps, where the other flavours differ in 424-87,508 parameters
// (profiles/r06/g/adamw_math_probe_1.jsonl)
int g_adamw_math = 4;

extern "C" int va_adamw_flat(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, double lr,
                             double beta1, double beta2, double eps, double weight_decay, const float *step,
                             const float *grad_scale, const float *found_inf, int zero_grad, void *stream) {
  VA_CHECK_ARG(n >= 0, "adamw_flat: negative length");
  if (n == 0) return VA_OK;
  VA_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && step, "null pointer argument");
  VA_CHECK_ARG(((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                 reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq)) & 15) == 0,
               "adamw_flat: 16-byte aligned buffers required");
  VA_CHECK_ARG(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0 && lr >= 0.0,
               "adamw_flat: invalid hyper-parameters");
  const int64_t vecs = (n + 3) / 4;
  int64_t grid = (vecs + 255) / 256;
  if (grid > 4096) grid = 4096;  // 16 resident workgroups per CU, grid-stride over the rest
  const AdamWArgs a{lr, beta1, beta2, eps, weight_decay};
  const dim3 gr(static_cast<unsigned>(grid)), bl(256);
  hipStream_t st = static_cast<hipStream_t>(stream);
#define VA_ADAMW_LAUNCH(M)                                                                                           \
  hipLaunchKernelGGL(adamw_flat_kernel<M>, gr, bl, 0, st, param, grad, exp_avg, exp_avg_sq, n, a, step, grad_scale, \
                     found_inf, zero_grad)
  switch (g_adamw_math & 7) {
    case 0: VA_ADAMW_LAUNCH(0); break;
    case 1: VA_ADAMW_LAUNCH(1); break;
    case 2: VA_ADAMW_LAUNCH(2); break;
    case 3: VA_ADAMW_LAUNCH(3); break;
    case 4: VA_ADAMW_LAUNCH(4); break;
    case 5: VA_ADAMW_LAUNCH(5); break;
    case 6: VA_ADAMW_LAUNCH(6); break;
    default: VA_ADAMW_LAUNCH(7); break;
  }
#undef VA_ADAMW_LAUNCH
  return check_launch("adamw_flat");
}
