// Development harness for f1 v3 (fused lm_head + log-softmax + entropy, forward): the logits tile
// is computed TRANSPOSED, S^T = W_tile . H_tile^T, so the vocab index is the MFMA row (registers)
// and the token is the MFMA column (lane & 15). Every lane then owns whole tokens: the online
// (max, sum 2^(xL-B), sum 2^(xL-B) x) state of its 4 tokens lives in registers for the whole
// persistent sweep over the vocab tiles, with NO per-tile cross-lane reduction, LDS round trip or
// barrier; the 4 lane groups (lane >> 4) and the 2 vocab wave-rows are merged once at the end.
// Driven by tools/f1t_bench.py through ctypes; the product kernel is verl_amd/csrc/linear_logprob.hip.
//
// Geometry (as the round-2 256 x 256 core): tile 256 vocab x 256 tokens x 64 k, 8 waves = 2 (vocab
// halves, wr) x 4 (token quarters, wc), 128 x 64 per wave = 8 x 4 v_mfma_f32_16x16x32_bf16 blocks,
// both operands staged by LDS-DMA into 2 source-swizzled buffers; persistent over the workgroup's
// vocab tiles, the next tile's first K-step staged during the current one's last.
// Grid: row blocks x vocab splits, XCD-remapped (REMAP=1) so that an XCD's resident workgroups
// cover a few row blocks x all splits (hidden panels stay in its L2; W tiles shared by row blocks).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace {

constexpr float kLog2eF = 1.4426950408889634f;
constexpr float kLn2F = 0.69314718055994531f;
constexpr int TB = 256, TK = 64, NT = 512;
constexpr int T_TILE = TB * TK;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ float base_of(float m) { return m == -INFINITY ? 0.f : m * kLog2eF; }

__device__ __forceinline__ int img_off(int row, int c) { return row * TK + ((c ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ void stage(const uint16_t *__restrict__ src, int64_t row0, int64_t nrows, int64_t ld,
                                      int k0, uint16_t *img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int g = wave * 4 + i;
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    int64_t gr = row0 + row;
    if (gr >= nrows) gr = nrows - 1;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + gr * ld + k0 + lc * 8), img + g * 8 * TK,
                                     16, 0, 0);
  }
}

struct St {
  float m, s, t;
};
__device__ __forceinline__ void merge_st(St &a, float om, float os, float ot) {
  const float nm = fmaxf(a.m, om);
  const float nb = base_of(nm);
  const float a1 = __builtin_amdgcn_exp2f(base_of(a.m) - nb);
  const float a2 = __builtin_amdgcn_exp2f(base_of(om) - nb);
  a.s = a.s * a1 + os * a2;
  a.t = a.t * a1 + ot * a2;
  a.m = nm;
}

// Fold one finished 256 x 256 tile into the lane's per-token online state. Rounding to bf16 is
// monotonic, so the tile max of the rounded logits is the rounded max of the raw accumulators: one
// max pass over acc (v_max3), then ONE pass of round -> exp2 -> sums. TAIL: the last vocab tile,
// whose rows past V are -inf (weight 0; kept out of the x-weighted sum, 0 * -inf being NaN).
template <bool TAIL>
__device__ __forceinline__ void tile_epilogue(const f32x4 (&acc)[8][4], int v0, const int (&lab)[4], float (&m)[4],
                                              float (&s)[4], float (&t)[4], float (&ll)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float rm = acc[0][j][0];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) rm = fmaxf(rm, acc[i][j][e]);
    const float lm = __uint_as_float(pack2_bf16(rm, 0.f) << 16);
    const int d = lab[j] - v0;  // label at (i, e) = (d >> 4, d & 3) when d in [0, 128), d & 12 == 0
    if (d >= 0 && d < 128 && (d & 12) == 0) {
      const int uu = (d >> 4) * 4 + (d & 3);
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) v = (i * 4 + e) == uu ? acc[i][j][e] : v;
      ll[j] = __uint_as_float(pack2_bf16(v, 0.f) << 16);
    }
    const float nm = fmaxf(m[j], lm);
    const float nb = base_of(nm);
    const float alpha = __builtin_amdgcn_exp2f(base_of(m[j]) - nb);
    float ss = 0.f, tt = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const uint32_t p = pack2_bf16(acc[i][j][e], acc[i][j][e + 1]);
        float x0 = __uint_as_float(p << 16), x1 = __uint_as_float(p & 0xffff0000u);
        const float e0 = __builtin_amdgcn_exp2f(fmaf(x0, kLog2eF, -nb));
        const float e1 = __builtin_amdgcn_exp2f(fmaf(x1, kLog2eF, -nb));
        ss += e0 + e1;
        if (TAIL) {
          x0 = x0 == -INFINITY ? 0.f : x0;
          x1 = x1 == -INFINITY ? 0.f : x1;
        }
        tt = fmaf(e0, x0, fmaf(e1, x1, tt));
      }
    s[j] = fmaf(s[j], alpha, ss);
    t[j] = fmaf(t[j], alpha, tt);
    m[j] = nm;
  }
}

// EPI 0: core only (a cheap checksum keeps the MFMAs live); 1: full online-softmax epilogue
template <int EPI, bool REMAP>
__global__ __launch_bounds__(NT, 1) void lp_t_kernel(const uint16_t *__restrict__ hid, int64_t ldh,
                                                     const uint16_t *__restrict__ w, int64_t ldw,
                                                     const int64_t *__restrict__ labels, int64_t N, int K, int64_t V,
                                                     int splits, int tiles_per_split, float *__restrict__ part,
                                                     float *__restrict__ label_logit) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * T_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  int64_t L = blockIdx.x;
  if (REMAP) {  // contiguous logical ids per XCD (blocks b, b + 8, ... share one); gridDim.x % 8 == 0
    const int64_t nl = gridDim.x >> 3;
    L = (L & 7) * nl + (L >> 3);
  }
  const int64_t rb = L / splits, sp = L % splits;
  const int64_t row0 = rb * TB;
  const int64_t n_vt = (V + TB - 1) / TB;
  const int64_t vt_begin = sp * tiles_per_split;
  const int64_t vt_end = vt_begin + tiles_per_split < n_vt ? vt_begin + tiles_per_split : n_vt;
  const int nk = K / TK;
  const int64_t nsteps = vt_begin < vt_end ? (vt_end - vt_begin) * nk : 0;

  // this lane's 4 tokens (columns of the transposed tile) and their labels
  int lab[4];
  float m[4], s[4], t[4], ll[4];  // ll: the label's logit, -inf until this lane meets it
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t r = row0 + wc * 64 + j * 16 + (lane & 15);
    const int64_t lb = r < N ? labels[r] : -1;
    lab[j] = (lb >= 0 && lb < V) ? static_cast<int>(lb) : -1;
    m[j] = -INFINITY, s[j] = 0.f, t[j] = 0.f, ll[j] = -INFINITY;
  }
  float chk = 0.f;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nsteps > 0) {
    stage(w, vt_begin * TB, V, ldw, 0, lds, wave, lane);
    stage(hid, row0, N, ldh, 0, lds + T_TILE, wave, lane);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int64_t st = 0; st < nsteps; ++st) {
    const int buf = static_cast<int>(st & 1);
    const int kt = static_cast<int>(st % nk);
    const int64_t vt = vt_begin + st / nk;
    const uint16_t *la = lds + buf * 2 * T_TILE;
    const uint16_t *lb = la + T_TILE;
    if (st + 1 < nsteps) {
      uint16_t *na = lds + (buf ^ 1) * 2 * T_TILE;
      const int k1 = static_cast<int>((st + 1) % nk) * TK;
      stage(w, (vt_begin + (st + 1) / nk) * TB, V, ldw, k1, na, wave, lane);
      stage(hid, row0, N, ldh, k1, na + T_TILE, wave, lane);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = q * 4 + (lane >> 4);
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        fa[i] = *reinterpret_cast<const bf16x8 *>(la + img_off(wr * 128 + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8 *>(lb + img_off(wc * 64 + j * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt == nk - 1) {
      if constexpr (EPI == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) chk += acc[i][j][0] + acc[i][j][3];
      } else {
        // acc[i][j][e] = logit of vocab v0 + i*16 + e (v0 below) for token j of this lane.
        const int v0 = static_cast<int>(vt * TB) + wr * 128 + (lane >> 4) * 4;
        if (vt * TB + TB > V) {  // uniform: only the last vocab tile has rows past V
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (v0 + i * 16 + e >= V)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j][e] = -INFINITY;
          tile_epilogue<true>(acc, v0, lab, m, s, t, ll);
        } else {
          tile_epilogue<false>(acc, v0, lab, m, s, t, ll);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // ---- merge the 4 lane groups (lanes l, l ^ 16, l ^ 32, l ^ 48 hold the same tokens), then the
  //      two vocab wave-rows through LDS (the staging buffers are free now)
  float *red = reinterpret_cast<float *>(lds);  // [4 wc][64 tokens][4]: m, s, t, label logit
  if constexpr (EPI == 0) {
    if (lane == 0 && chk == 12345.f) part[0] = chk;  // keep the checksum live
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    St a{m[j], s[j], t[j]};
    float l2 = ll[j];
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      const float om = __shfl_xor(a.m, o, 64), os = __shfl_xor(a.s, o, 64), ot = __shfl_xor(a.t, o, 64);
      merge_st(a, om, os, ot);
      l2 = fmaxf(l2, __shfl_xor(l2, o, 64));  // one lane of the token holds it (or none: -inf)
    }
    m[j] = a.m, s[j] = a.s, t[j] = a.t, ll[j] = l2;
  }
  if (wr == 1 && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float *p = red + ((wc * 64) + j * 16 + lane) * 4;
      p[0] = m[j], p[1] = s[j], p[2] = t[j], p[3] = ll[j];
    }
  }
  __syncthreads();
  if (wr == 0 && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float *p = red + ((wc * 64) + j * 16 + lane) * 4;
      St a{m[j], s[j], t[j]};
      merge_st(a, p[0], p[1], p[2]);
      const int64_t r = row0 + wc * 64 + j * 16 + lane;
      if (r < N) {
        float *o = part + (sp * N + r) * 3;
        o[0] = a.m, o[1] = a.s, o[2] = a.t;
        const float lv = fmaxf(ll[j], p[3]);
        if (lv != -INFINITY) label_logit[r] = lv;
      }
    }
  }
}

__global__ __launch_bounds__(256) void merge_kernel(const float *__restrict__ part, const float *__restrict__ label_logit,
                                                    const int64_t *__restrict__ labels, int64_t N, int64_t V, int splits,
                                                    float *__restrict__ logp, float *__restrict__ entropy,
                                                    float *__restrict__ lse_out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (r >= N) return;
  St a{-INFINITY, 0.f, 0.f};
  for (int sp = 0; sp < splits; ++sp) {
    const float *p = part + (static_cast<int64_t>(sp) * N + r) * 3;
    merge_st(a, p[0], p[1], p[2]);
  }
  float lse;
  if (a.m == -INFINITY) {
    lse = -INFINITY;
  } else {
    const float corr = -fmaf(a.m, kLog2eF, -base_of(a.m));
    lse = a.m + kLn2F * (__builtin_amdgcn_logf(a.s) + corr);
  }
  lse_out[r] = lse;
  entropy[r] = lse - a.t / a.s;
  const int64_t lab = labels[r];
  logp[r] = (lab < 0 || lab >= V) ? __builtin_nanf("") : label_logit[r] - lse;
}

}  // namespace

// variant: 0 core only + remap, 1 full + remap, 2 full without remap, 3 core only without remap
extern "C" int f1t_fwd(int variant, const void *hidden, const void *weight, const int64_t *labels, int64_t N, int64_t H,
                       int64_t V, int splits, float *logp, float *entropy, float *lse, float *workspace, void *stream) {
  if (H % TK || N <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t n_vt = (V + TB - 1) / TB;
  const int per = static_cast<int>((n_vt + splits - 1) / splits);
  const int used = static_cast<int>((n_vt + per - 1) / per);
  int64_t rbs = (N + TB - 1) / TB;
  int64_t nwg = rbs * used;
  const bool remap = (variant == 0 || variant == 1) && nwg % 8 == 0;
  float *part = workspace;
  float *label_logit = workspace + static_cast<int64_t>(used) * N * 3;
  const auto *h = static_cast<const uint16_t *>(hidden);
  const auto *w = static_cast<const uint16_t *>(weight);
  const dim3 grid(static_cast<unsigned>(nwg));
  if (variant == 0 || variant == 3) {
    if (remap) hipLaunchKernelGGL((lp_t_kernel<0, true>), grid, dim3(NT), 0, st, h, H, w, H, labels, N, (int)H, V, used, per, part, label_logit);
    else hipLaunchKernelGGL((lp_t_kernel<0, false>), grid, dim3(NT), 0, st, h, H, w, H, labels, N, (int)H, V, used, per, part, label_logit);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  if (remap) hipLaunchKernelGGL((lp_t_kernel<1, true>), grid, dim3(NT), 0, st, h, H, w, H, labels, N, (int)H, V, used, per, part, label_logit);
  else hipLaunchKernelGGL((lp_t_kernel<1, false>), grid, dim3(NT), 0, st, h, H, w, H, labels, N, (int)H, V, used, per, part, label_logit);
  hipLaunchKernelGGL(merge_kernel, dim3(static_cast<unsigned>((N + 255) / 256)), dim3(256), 0, st, part, label_logit,
                     labels, N, V, used, logp, entropy, lse);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int64_t f1t_workspace_floats(int64_t N, int splits) { return static_cast<int64_t>(splits) * N * 3 + N; }
