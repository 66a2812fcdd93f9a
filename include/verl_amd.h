/*
 * verl_amd.h — C-ABI of the MI355X-native PPO/GRPO actor-update hot path.
 *
 * One shared library (verl_amd/lib/libverl_amd.so, built for gfx950 by hipcc) exports the
 * functions below. Signatures use plain pointers, sizes and a hipStream_t passed as void*;
 * no torch types cross this boundary. Every entry point:
 *   - borrows caller-owned device buffers (row-major, contiguous along the last dim unless a
 *     stride argument says otherwise);
 *   - launches asynchronously on `stream` and never synchronises the host;
 *   - performs no allocation (scratch space is a caller-provided `workspace`; its byte size is
 *     given by the matching *_workspace_bytes() query), so it is safe under hipGraph capture;
 *   - returns 0 on success, or a negative VA_E* code with a message readable through
 *     va_last_error() (thread-local).
 *
 * Which reference interface each entry point replaces is cited as file:line of rfahrn/verl
 * (verl 0.4.1.dev). The Python mirror of that interface lives in verl_amd/ (same module
 * names, function names, argument meaning and error texts) and binds this header via ctypes
 * (verl_amd/_lib.py); INTEGRATION.md shows the binding a maintainer of the reference adds.
 */
#ifndef VERL_AMD_H
#define VERL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VA_ABI_VERSION 11

/* error codes */
#define VA_OK 0
#define VA_E_ARG -1    /* invalid size / pointer / enum */
#define VA_E_ALIGN -2  /* a pointer does not meet the stated alignment */
#define VA_E_LAUNCH -3 /* hipLaunch / hip runtime error */

/* element dtype codes (logits) */
#define VA_F32 0
#define VA_BF16 1
#define VA_F16 2
/* flag OR-ed into va_linear_logprob_fwd's dtype: fp32 logits (no bf16 rounding), the numerics of
 * the reference's fused kernel (utils/kernel/kernels.py:120-663) instead of the unfused bf16 path */
#define VA_LOGITS_F32 256

/* mask dtype codes (response_mask / attention_mask slices) */
#define VA_MASK_F32 0
#define VA_MASK_I64 1
#define VA_MASK_I32 2
#define VA_MASK_U8 3 /* torch.bool */

/* loss_agg_mode (core_algos.py:686-719) */
#define VA_AGG_TOKEN_MEAN 0
#define VA_AGG_SEQ_MEAN_TOKEN_SUM 1
#define VA_AGG_SEQ_MEAN_TOKEN_MEAN 2
#define VA_AGG_SEQ_MEAN_TOKEN_SUM_NORM 3

/* kl_penalty type (core_algos.py:1034-1069); "full" has no code: NotImplementedError on host */
#define VA_KL_NONE (-1)
#define VA_KL_K1 0  /* "kl", "k1" */
#define VA_KL_ABS 1 /* "abs" */
#define VA_KL_K2 2  /* "mse", "k2" */
#define VA_KL_K3 3  /* "low_var_kl", "k3" */

/* outcome-advantage estimators sharing the per-group kernel (core_algos.py:245-476) */
#define VA_ADV_GRPO 0      /* (s - mean) / (std + eps)              core_algos.py:246-308 */
#define VA_ADV_GRPO_NOSTD 1 /* s - mean (Dr.GRPO)                   core_algos.py:304-305 */
#define VA_ADV_RLOO 2      /* s*n/(n-1) - mean*n/(n-1)              core_algos.py:428-476 */
#define VA_ADV_MEAN_ONLY 3 /* s - mean, first half of RF++-baseline core_algos.py:376-424 */
#define VA_ADV_OPO 4       /* s - sum(len*s)/sum(len), singleton 0  core_algos.py:479-530 */
#define VA_ADV_PASSK 5     /* best row: (r_max - r_2nd)/(std + eps)  core_algos.py:311-370 */
#define VA_ADV_PASSK_NOSTD 6 /* best row: r_max - r_2nd             core_algos.py:363-366 */

/* discounted-return modes of va_discounted_returns */
#define VA_RET_RFPP 0      /* REINFORCE++ return with reset after EOS core_algos.py:553-560 */
#define VA_RET_REMAX 1     /* reverse cumsum of r*m, adv = ret - b*m  core_algos.py:597-600 */

/* policy-loss modes of va_ppo_loss_fwd/bwd (register_policy_loss, dispatch dp_actor.py:419-443) */
#define VA_PL_VANILLA 0  /* dual-clip PPO                          core_algos.py:722-794 */
#define VA_PL_GPG 1      /* -lp * A                                core_algos.py:797-815 */
#define VA_PL_CLIP_COV 2 /* max(l1, l2) * (1 - sel), unclamped     core_algos.py:818-905 */
#define VA_PL_KL_COV 3   /* l1 + sel * coef * |lp - old|, unclamped core_algos.py:908-972 */

/* scalar slots of the fused policy-loss output vector out[VA_LOSS_NOUT] */
#define VA_LOSS_PG 0            /* pg_loss                 core_algos.py:791-792 */
#define VA_LOSS_CLIPFRAC 1      /* pg_clipfrac             core_algos.py:783 */
#define VA_LOSS_PPO_KL 2        /* ppo_kl                  core_algos.py:770 */
#define VA_LOSS_CLIPFRAC_LOWER 3 /* pg_clipfrac_lower      core_algos.py:787-789 */
#define VA_LOSS_KL 4            /* agg_loss(kl_penalty)    dp_actor.py:456-459 */
#define VA_LOSS_ENTROPY 5       /* agg_loss(entropy)       dp_actor.py:446 */
#define VA_LOSS_NTOKENS 6       /* sum(response_mask)      (diagnostic) */
#define VA_LOSS_NROWS 7         /* batch rows              (diagnostic) */
#define VA_LOSS_NOUT 8

int va_abi_version(void);
const char *va_last_error(void);
/* number of compute units / name of the device the library is bound to (diagnostics). */
int va_device_info(int *num_cu, int *arch_major, int *arch_minor);

/* ---------------------------------------------------------------------------------------
 * Per-token log-prob + entropy over the vocab, fused in one HBM pass.
 * Replaces: verl/utils/torch_functional.py:64-100 (logprobs_from_logits, flash-attn
 * cross_entropy_loss path), :116-133 (logprobs_from_logits_v2), :145-149
 * (entropy_from_logits), and the temperature division dp_actor.py:182 (logits.div_(T)),
 * applied on load with the reference's rounding (bf16 -> bf16(x / T)).
 *   logits  [n_rows, row_stride] of `dtype`, first `vocab` columns used
 *   labels  [n_rows] int64; label == -100 gives logp = 0 (flash-attn ignore_index);
 *           any other label outside [0, vocab) gives NaN
 *   logp, lse [n_rows] fp32 (required); entropy [n_rows] fp32 (may be NULL)
 * ------------------------------------------------------------------------------------ */
int va_logprob_entropy_fwd(const void *logits, int dtype, int64_t n_rows, int64_t vocab,
                           int64_t row_stride, const int64_t *labels, float temperature,
                           float *logp, float *entropy, float *lse, void *stream);

/* Backward of the above w.r.t. the raw (pre-temperature) logits:
 *   dz = g_logp*(onehot - p) - g_entropy*p*(log p + H);   dlogits = dz / T
 * (experimental/torch_functional.py:55-67; flash-attn in-place CE backward).
 * g_logp / g_entropy may be NULL (zero). dlogits may alias logits (in-place backward,
 * torch_functional.py:64 inplace_backward=True); it has `dtype` and its own row stride. */
int va_logprob_entropy_bwd(const float *g_logp, const float *g_entropy, const void *logits,
                           int dtype, int64_t n_rows, int64_t vocab, int64_t row_stride,
                           const int64_t *labels, const float *lse, const float *entropy,
                           float temperature, void *dlogits, int64_t dlogits_row_stride,
                           void *stream);

/* Launch-shape knobs of the log-prob kernels (results are identical for every setting):
 *   VA_TUNE_FWD_WAVES_PER_ROW: 0 = auto, 1 / 2 / 4 waves stream one row together;
 *   VA_TUNE_BWD_WAVES_PER_ROW: accepted, no effect (the backward is a flat chunk stream);
 *   VA_TUNE_NONTEMPORAL: 1 = non-temporal (streaming) loads/stores of the logits (default),
 *   0 = default cache policy;
 *   VA_TUNE_PIPELINE: fwd 0: 4 vectors/lane, 1: 2+2 software-pipelined, 2: 4+4 pipelined;
 *   bwd 16-B vectors per lane per workgroup chunk 0: 4, 1: 2, 2: 8;
 *   VA_TUNE_FLASH_GROUPED_DKDV (va_flash_attn_bwd): -1 = auto, 0 = per-query-head fp32 partials +
 *   fixed-order group sum, 1 = one workgroup per key block x KV head summing its group in registers
 *   (results differ only in fp32 summation order);
 *   VA_TUNE_GAE_VARIANT (va_gae_scan): 0 = auto (quad-streaming kernel where R % 4 == 0, R <= 2048
 *   and the rows are 16-byte aligned), 1 = register chunks (rows of R <= 1024 only; longer rows keep
 *   the LDS kernel), 2 = LDS-staged kernel (1 and 2: advantages/returns bitwise identical, the fp64
 *   row partials differ only in summation order), 3 = quad-streaming kernel (4-step lane quads
 *   instead of 16-step lane chunks: the scan reassociates differently, within the same budget);
 *   VA_TUNE_BWD_FLAT (va_logprob_entropy_bwd): -1 = auto (one flat stream of equal 16-KB chunks over
 *   the whole tensor when logits and dlogits are dense, row stride = vocab), 0 = per-row chunks
 *   (bitwise identical results);
 *   VA_TUNE_SWIGLU_STREAM (va_swiglu_fwd/bwd): -1 = auto (streaming kernels: 4 / 2 vectors per lane
 *   fwd / bwd, all loads issued first, non-temporal), 2 / 4 / 8 = streaming with that many vectors
 *   per lane, 0 = grid-stride kernels (bitwise identical results);
 *   VA_TUNE_FLASH_DKDV_QT (va_flash_attn_bwd): query rows per staged dK / dV tile, 64 (default), 128
 *   or 32 (bitwise identical results: the same per-32-row products in the same order);
 *   VA_TUNE_FLASH_DQ_KB (va_flash_attn_bwd): keys per staged dQ block, 64 (default) or 128 (bitwise
 *   identical results);
 *   VA_TUNE_FLASH_FWD_KB (va_flash_attn_fwd): keys per staged forward block, 64 (default) or 128
 *   (bitwise identical results: the same 64-key online-softmax steps);
 *   VA_TUNE_GAE_PARTIALS (va_gae_scan): rows per whitening partial triple, 0 = auto, 1 (per row),
 *   4 or 8 (per workgroup); results differ only in the fp64 merge order;
 *   VA_TUNE_GAE_NT (va_gae_scan / va_gae_advantage_return): streaming-cache bits, 1 = non-temporal
 *   r / v loads, 2 = non-temporal returns store, 4 = non-temporal raw / whitened advantage stores
 *   (default 3; identical results);
 *   VA_TUNE_LOSS_VEC (va_ppo_loss_fwd): 1 = one wave per row with 16-byte lane quads (default where
 *   R % 4 == 0, R <= 2048 and the rows are 16-byte aligned), 0 = one workgroup per row (fp64 row
 *   sums in another order);
 *   VA_TUNE_WHITEN_SLICE_MIN / VA_TUNE_WHITEN_GRID (va_gae_advantage_return): partial count above
 *   which partials are merged in parallel slices first (default 4,096) and the statistics +
 *   whitening launch's grid cap (default 2,048); only the fp64 merge order changes;
 *   VA_TUNE_WGRAD_REMAINDER (va_weight_grad): 0 (default) = 256 x 256 tiles throughout; 1 = a
 *     dimension that is 128 mod 256 gets its last 128 rows / columns as 128 x 512 / 512 x 128 tiles.
 *   VA_TUNE_WGRAD_MFMA (va_weight_grad): 32 (default) = 32x32x16 MFMA blocks; 16 = 16x16x32 blocks
 *     (same tiles and staging; results differ only in the MFMA's internal summation order).
 *   VA_TUNE_WGRAD_TILES (va_weight_grad): 4 (default), 3, 2, 1 = one launch whose tile shape (256 x 256,
 *     or 256 x 224 / 224 x 256 / 128 x 448 / 448 x 128, which divide 896 exactly) and K-slice count
 *     are chosen by a cost model (rounds of 256 workgroups x tile area x steps + the split-K reduce),
 *     16x16x32 MFMA blocks; 2 / 3 read each step's fragments one step ahead (two register sets),
 *     3 also spreads the LDS-DMA between the MFMAs, 4 the fragment reads too; 0 = 256 x 256 tiles (+ VA_TUNE_WGRAD_REMAINDER)
 *     with the round-4 slice rule. Results differ only in the fp32 summation order of the slices
 *     and the MFMA blocks.
 *   VA_TUNE_WGRAD_KIND (va_weight_grad, VA_TUNE_WGRAD_TILES >= 1): -1 (default) = the cost model's tile
 *     shape, 0 / 3 / 4 / 5 / 6 = that shape (256 x 256, 256 x 224, 224 x 256, 128 x 448, 448 x 128)
 *     with the model's slice count for it (A/B runs; the same results up to fp32 summation order).
 *   VA_TUNE_ADAMW_MATH (va_adamw_flat): rounding flavour of the step's square root / divisions / double
 *     multiply-adds (bit 1 hardware sqrt, bit 2 reciprocal-based division, bit 4 FMA contraction),
 *     to match a given torch build's fused AdamW bit for bit.
 *   VA_TUNE_LINEAR_TN (va_linear_tn): 2 (default) = the ping-pong form for 192 / 224-wide tiles at K >= 192
 *     (else 1); 1 = the two-buffer form, each workgroup keeping one feature tile over a range of token blocks,
 *     the workgroups of one token range side by side on one XCD; 0 = the two-buffer form over consecutive
 *     tiles of the (token block, feature tile) list (all bitwise identical).
 *   VA_TUNE_T256_DEFER (bit flags, default 1): the 256 x 256 sweep runs a finished tile's storing
 *     epilogue after the step's operand wait, its stores draining during the next step, for
 *     va_gate_up_swiglu / _save (bit 1), va_linear_logprob_bwd (bit 2) and va_qkv_rope (bit 4); else
 *     before that wait (bitwise identical either way).
 *   VA_TUNE_LINEAR_LOGPROB_TILE (va_linear_logprob_fwd): 256 (default) = 256 x 256 LDS-DMA tiles,
*   8 waves; 128 = the 128 x 128 register-staged kernel (same results up to fp32 merge order);
 *   VA_TUNE_FLASH_DMA (va_flash_attn_fwd / _bwd): bit 1 = forward K / V blocks staged by LDS-DMA
 *   (64-key blocks), bit 2 = the same for the dQ backward, bit 4 = the dK / dV backward's Q / dO
 *   tiles; 7 (default) = all three, 0 = register-staged (bitwise identical results). */
#define VA_TUNE_FWD_WAVES_PER_ROW 1
#define VA_TUNE_BWD_WAVES_PER_ROW 2
#define VA_TUNE_NONTEMPORAL 3
#define VA_TUNE_PIPELINE 4
#define VA_TUNE_FLASH_GROUPED_DKDV 5
#define VA_TUNE_GAE_VARIANT 6
#define VA_TUNE_BWD_FLAT 7
#define VA_TUNE_SWIGLU_STREAM 8
#define VA_TUNE_FLASH_DKDV_QT 9
#define VA_TUNE_FLASH_DQ_KB 10
#define VA_TUNE_FLASH_FWD_KB 11
#define VA_TUNE_GAE_PARTIALS 12
#define VA_TUNE_GAE_NT 13
#define VA_TUNE_LOSS_VEC 14
#define VA_TUNE_WHITEN_SLICE_MIN 15
#define VA_TUNE_WHITEN_GRID 16
#define VA_TUNE_LINEAR_LOGPROB_TILE 17
#define VA_TUNE_WGRAD_REMAINDER 18
#define VA_TUNE_FLASH_DMA 19
#define VA_TUNE_WGRAD_MFMA 20
#define VA_TUNE_WGRAD_TILES 21
#define VA_TUNE_ADAMW_MATH 22
#define VA_TUNE_WGRAD_KIND 23
#define VA_TUNE_LINEAR_TN 24
#define VA_TUNE_T256_DEFER 25
int va_set_tuning(int key, int value);

/* ---------------------------------------------------------------------------------------
 * Fused PPO policy loss (vanilla dual-clip or a registered variant) + optional KL-loss +
 * optional entropy term, with loss aggregation and the three metrics, over one [B, R]
 * micro-batch.
 * Replaces: core_algos.py:722-794 (compute_policy_loss), :797-972 (gpg / clip_cov / kl_cov),
 * :686-719 (agg_loss), :1034-1069 (kl_penalty) as called at dp_actor.py:419-461.
 *   old_lp, lp, adv [B,R] fp32; mask [B,R] of `mask_dtype`;
 *   ref_lp [B,R] fp32 or NULL (kl_type must then be VA_KL_NONE);
 *   entropy [B,R] fp32 or NULL.
 *   clip_lo = 1 - clip_ratio_low, clip_hi = 1 + clip_ratio_high (rounded to fp32 on host, as
 *   torch.clamp casts its scalar bounds), clip_c = clip_ratio_c (> 1, asserted on host).
 *   loss_mode = VA_PL_*; sel [B,R] uint8 = the variant's token selection (clip_cov: tokens whose
 *   loss is zeroed; kl_cov: tokens that get + mode_coef * |lp - old|), chosen on the host side
 *   with the reference's top-k / random draw; NULL for vanilla and gpg. Metric slots per mode:
 *   vanilla as the reference; gpg: 0, 0, 0; clip_cov: masked_mean(sel), masked_mean(old - lp), 0;
 *   kl_cov: 0, masked_mean(|lp - old|) (ppo_kl_abs), 0.
 *   seg_rows: 0 (or >= B) aggregates the whole [B, R] batch into out[VA_LOSS_NOUT]; 0 < seg_rows < B
 *   splits it into S = ceil(B / seg_rows) loss micro-batches of seg_rows consecutive rows (the last
 *   may be shorter), each aggregated on its own as a separate call over its rows would be (its own
 *   token and row counts: the reference's agg_loss per micro-batch, dp_actor.py:419-470), into
 *   out[S][VA_LOSS_NOUT]. seg_off (device, n_seg + 1 ascending int32 row offsets, seg_off[0] = 0,
 *   seg_off[n_seg] = B, every segment non-empty, 1 <= n_seg <= B) instead gives n_seg segments of
 *   any sizes (the reference's token-budget micro-batches, dp_actor.py:382-384); seg_rows is then
 *   ignored. The offsets are device data: the host checks only n_seg.
 *   out fp32 (device). workspace: va_ppo_loss_workspace_bytes(B) = 8 (16 B + 8):
 *   [B, 8] fp64 row partials, 8 fp64 totals (n first; zeros with segments), then up to B per-workgroup aggregated
 *   vectors that only the forward reads, whose first S slots the segmented forward overwrites with
 *   the segments' token counts. The first 8 B + 8 doubles (+ S with segments) are what the backward
 *   reads: keep them alive between the forward and the backward of the same micro-batch. */
int64_t va_ppo_loss_workspace_bytes(int64_t B);
int va_ppo_loss_fwd(const float *old_lp, const float *lp, const float *adv, const void *mask,
                    int mask_dtype, const float *ref_lp, const float *entropy, int64_t B,
                    int64_t R, float clip_lo, float clip_hi, float clip_c, int agg_mode,
                    int kl_type, int loss_mode, const uint8_t *sel, float mode_coef,
                    int64_t seg_rows, const int32_t *seg_off, int64_t n_seg, float *out,
                    void *workspace, void *stream);

/* Backward: g_out[S][VA_LOSS_NOUT] is d(loss)/d(out) as a device array (only slots PG, KL,
 * ENTROPY are read; may be NULL = zeros), seg_rows as in the forward (S = 1 when 0). Writes
 * d_lp [B,R] and, if non-NULL, d_entropy.
 * Tie and boundary gradients follow torch autograd of the reference expression:
 * maximum/minimum split ties 1/2-1/2, clamp passes inclusive of its bounds, abs' gradient at 0 is 0. */
int va_ppo_loss_bwd(const float *g_out, const float *old_lp, const float *lp, const float *adv,
                    const void *mask, int mask_dtype, const float *ref_lp, int64_t B, int64_t R,
                    float clip_lo, float clip_hi, float clip_c, int agg_mode, int kl_type,
                    int loss_mode, const uint8_t *sel, float mode_coef, int64_t seg_rows,
                    const int32_t *seg_off, int64_t n_seg, const void *workspace, float *d_lp,
                    float *d_entropy, void *stream);

/* ---------------------------------------------------------------------------------------
 * Elementwise KL estimators (core_algos.py:1034-1069), n elements.
 *   fwd: kld = f(lp, ref).  bwd: d_lp = g * df/dlp, d_ref = g * df/dref (either may be NULL).
 * ------------------------------------------------------------------------------------ */
int va_kl_penalty_fwd(const float *lp, const float *ref, int64_t n, int kl_type, float *kld,
                      void *stream);
int va_kl_penalty_bwd(const float *g, const float *lp, const float *ref, int64_t n, int kl_type,
                      float *d_lp, float *d_ref, void *stream);

/* ---------------------------------------------------------------------------------------
 * Masked aggregation of a [B, R] fp32 matrix (agg_loss core_algos.py:686-719; masked_mean /
 * masked_sum torch_functional.py:163-185).
 *   mode = VA_AGG_*, or VA_REDUCE_MASKED_SUM (4): sum(where(m, x, 0) * m),
 *   or VA_REDUCE_ROW_MASKED_MEAN (5): out[b] = masked_mean over row b (axis=-1).
 *   out: 1 float (modes 0-4) or B floats (mode 5).  workspace: va_agg_workspace_bytes(B).
 * Backward: dx[b,t] = g * weight(b,t), read from the same workspace. */
#define VA_REDUCE_MASKED_SUM 4
#define VA_REDUCE_ROW_MASKED_MEAN 5
int64_t va_agg_workspace_bytes(int64_t B);
int va_masked_agg_fwd(const float *x, const void *mask, int mask_dtype, int64_t B, int64_t R,
                      int mode, float *out, void *workspace, void *stream);
int va_masked_agg_bwd(const float *g, const void *mask, int mask_dtype, int64_t B, int64_t R,
                      int mode, const void *workspace, float *dx, void *stream);

/* ---------------------------------------------------------------------------------------
 * Outcome advantages over prompt groups (GRPO and relatives).
 * Replaces: core_algos.py:246-308 (compute_grpo_outcome_advantage), :311-370 (pass@k),
 * :428-476 (RLOO), :479-530 (OPO) and the group-mean part of :376-424 (RF++-baseline). Groups
 * are given in CSR form built on host from the uid array (np.unique(return_inverse) + stable
 * argsort; the host-side grouping of core_algos.py:290-291): rows of group g are
 * order[offsets[g] .. offsets[g+1]), in batch order (the reference's member order).
 *   score[b] = sum_t rewards[b,t] (unmasked, core_algos.py:282)
 *   adv[b,t] = a(b) * mask[b,t]; also writes scores[B] fp32 if non-NULL.
 * Singleton group: mean 0, std 1 (core_algos.py:293-295).
 * workspace: va_outcome_workspace_bytes(B). Three launches: va_row_scores, va_group_coef,
 * va_broadcast_rows, which are also exported for the data-parallel form, where a batch's groups
 * span ranks (the reference computes over the whole batch on the driver after _balance_batch,
 * ray_trainer.py:1204-1205, 262-273): each rank scores its own rows, the (score, length) pairs
 * are all-gathered, va_group_coef runs on the gathered batch and va_broadcast_rows on the
 * rank's own rows (coef pointer offset by the rank's first global row).
 *   va_row_scores:    scores[B] (+ lengths[B] = sum_t mask[b,t] if non-NULL, OPO)
 *   va_group_coef:    coef[N] = a(b) for every row of the N-row (gathered) batch
 *   va_broadcast_rows: adv[b,t] = coef[b] * mask[b,t]
 * ------------------------------------------------------------------------------------ */
int64_t va_outcome_workspace_bytes(int64_t B);
int va_outcome_advantage(const float *rewards, const void *mask, int mask_dtype, int64_t B,
                         int64_t R, const int32_t *order, const int32_t *offsets,
                         int64_t n_groups, int64_t max_group_size, float epsilon, int estimator,
                         float *adv, float *scores, void *workspace, void *stream);
int va_row_scores(const float *rewards, const void *mask, int mask_dtype, int64_t B, int64_t R,
                  float *scores, float *lengths, void *stream);
int va_group_coef(const float *scores, const float *lengths, const int32_t *order,
                  const int32_t *offsets, int64_t n_groups, int64_t max_group_size, float epsilon,
                  int estimator, float *coef, void *stream);
int va_broadcast_rows(const float *coef, const void *mask, int mask_dtype, int64_t B, int64_t R,
                      float *adv, void *stream);

/* ---------------------------------------------------------------------------------------
 * GAE (core_algos.py:193-241): masked reverse recurrence per row as a chunked affine scan, then
 * the batch-global masked whitening (torch_functional.py:188-223).
 *   rewards, values [B,R] fp32, mask [B,R] -> adv [B,R] (whitened), ret [B,R] (= raw + values)
 *   row_stats: workspace (va_gae_workspace_bytes(B)).
 *   stats_out[4] fp32 (device): {mean, rsqrt(var + 1e-8), mask_sum, error_flag}
 *   error_flag = 1 when mask_sum == 0, 2 when mask_sum == 1 (the ValueErrors of
 *   torch_functional.py:195-200, raised by the host wrapper).
 * Two or three launches: the scan (one wave per row, 16-byte quads per lane) writes P =
 * va_gae_partial_count(B) partial (n, sum, M2) triples (one per row, or per workgroup of 4 / 8
 * rows, see VA_TUNE_GAE_PARTIALS) into the workspace; when P > 4096 they are first merged in
 * parallel slices; the last launch merges them in every workgroup (fixed order) and whitens adv
 * in place.
 * For data-parallel whitening the phases are exported separately:
 *   va_gae_scan        -> adv_raw, ret, and the P partial triples at the start of row_partials
 *                         (a workspace of va_gae_workspace_bytes(B) bytes)
 *   va_whiten_finalize -> merges K partial triples in a fixed order (Chan), emits the merged
 *                         fp64 triple and the fp32 stats (call it again on all-gathered triples);
 *                         for K > 1024 it merges slices of 512 in parallel first, writing each
 *                         slice's result over the slice's first triple (the partials are scratch)
 *   va_whiten_apply    -> x = (x - mean) * rstd [* mask] in place.
 * ------------------------------------------------------------------------------------ */
int64_t va_gae_workspace_bytes(int64_t B);
int64_t va_gae_partial_count(int64_t B);
int va_gae_scan(const float *rewards, const float *values, const void *mask, int mask_dtype,
                int64_t B, int64_t R, float gamma, float lam, float *adv_raw, float *ret,
                double *row_partials, void *stream);
int va_masked_row_partials(const float *x, const void *mask, int mask_dtype, int64_t B,
                           int64_t R, double *row_partials, void *stream);
int va_whiten_finalize(double *partials, int64_t K, double *merged, float *stats_out,
                       void *stream);
int va_whiten_apply(float *x, const float *stats, const void *mask, int mask_dtype, int64_t B,
                    int64_t R, int post_multiply_mask, void *stream);
int va_gae_advantage_return(const float *rewards, const float *values, const void *mask,
                            int mask_dtype, int64_t B, int64_t R, float gamma, float lam,
                            float *adv, float *ret, float *stats_out, void *workspace,
                            void *stream);

/* ---------------------------------------------------------------------------------------
 * In-reward KL penalty (ray_trainer.py:153-193 apply_kl_penalty):
 *   kld = kl_penalty(old, ref) * mask; rewards = scores - beta * kld;
 *   row_kl[b] = masked_mean(kld[b], mask[b]) (the per-sequence current_kl before the batch mean)
 * ------------------------------------------------------------------------------------ */
int va_apply_kl_penalty(const float *scores, const float *old_lp, const float *ref_lp,
                        const void *mask, int mask_dtype, int64_t B, int64_t R, int kl_type,
                        float beta, float *rewards, float *row_kl, void *stream);

/* ---------------------------------------------------------------------------------------
 * Mixed-precision gradient accumulation (the fp32 gradient side of the reference's FSDP
 * MixedPrecision, fsdp_workers.py:337-347): dst[i][:] += scale * src[i][:] for n_tensors
 * tensors in one or a few launches. src: device pointers of `src_dtype` (VA_BF16 / VA_F16 /
 * VA_F32), dst: device fp32 pointers; the pointer / size arrays themselves live on the host.
 * ------------------------------------------------------------------------------------ */
int va_accumulate_grads(int n_tensors, const void *const *src, const int64_t *numel,
                        int src_dtype, float *const *dst, float scale, void *stream);

/* adamw_flat (ABI 10): one AdamW step over n fp32 elements of flat buffers (a parameter manager's
 * master-weight / gradient bucket and its moments), torch's fused AdamW arithmetic (ADAMW mode, no
 * amsgrad / maximize, its double-precision intermediates). Replaces: actor_optimizer.step() of the
 * reference's _optimizer_step (dp_actor.py:272-288; torch.optim.AdamW, fsdp_workers.py:418-423) over
 * the masters' per-parameter views. step: device fp32 step count, already advanced (bias corrections
 * 1 - beta^step); grad_scale: device fp32 scalar the gradients are multiplied by first (the
 * clip_grad_norm_ coefficient, folded; NULL = 1); found_inf: device fp32 flag (NULL = never), != 0
 * leaves parameters and moments untouched; zero_grad != 0 also writes 0 to the gradients (then also
 * when skipped). 16-byte aligned buffers. */
int va_adamw_flat(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, double lr,
                  double beta1, double beta2, double eps, double weight_decay, const float *step,
                  const float *grad_scale, const float *found_inf, int zero_grad, void *stream);

/* ---------------------------------------------------------------------------------------
 * Fused bf16 model ops for the actor backbone. Not the reference's hot path: they replace the
 * HF Qwen2 residual-add / RMSNorm / SwiGLU / rotary PyTorch op chains on the packed actor path
 * (verl_amd/workers/actor/qwen2_fused.py). All buffers 16-byte aligned, H % 8 == 0, H <= 4096.
 *   rmsnorm_fwd: h = x + residual (skipped when residual is NULL: h is x), y = RMSNorm(h) * w,
 *                rstd [T] fp32. x, residual, h_out, y [T, H]; w [H].
 *   rmsnorm_bwd: dx = d/dh of y given dy, plus dres (the gradient reaching h through the residual
 *                stream; NULL = none); dw [H] bf16; workspace of va_rmsnorm_workspace_bytes(T, H).
 *   swiglu:      y [T, F] = silu(g) * u where g / u are rows of gu [T, ldgu] (u at column offset uoff;
 *                the merged gate|up projection has ldgu = 2F, uoff = F); bwd writes dg / du into dgu
 *                [T, lddgu] at column offsets 0 / duoff. F, strides and offsets multiples of 8.
 *   rope_qkv:    qkv [T, ld] holds q | k | v ([Hq | Hk | Hk] x D per row); fwd writes rotated
 *                q [T, Hq, D], k [T, Hk, D] and v [T, Hk, D] (rotate_half convention, cos / sin
 *                [T, D]); bwd applies the transposed rotation and writes dqkv [T, ld]. D % 16 == 0.
 * ------------------------------------------------------------------------------------ */
int64_t va_rmsnorm_workspace_bytes(int64_t T, int64_t H);
int va_rmsnorm_fwd(const void *x, const void *residual, const void *w, int dtype, int64_t T, int64_t H, float eps,
                   void *h_out, void *y, float *rstd, void *stream);
int va_rmsnorm_bwd(const void *dy, const void *h, const void *w, const float *rstd, const void *dres, int dtype,
                   int64_t T, int64_t H, void *dx, void *dw, float *workspace, void *stream);
int va_swiglu_fwd(const void *gu, int64_t ldgu, int64_t uoff, int dtype, int64_t T, int64_t F, void *y,
                  void *stream);
int va_swiglu_bwd(const void *dy, const void *gu, int64_t ldgu, int64_t uoff, int dtype, int64_t T, int64_t F,
                  void *dgu, int64_t lddgu, int64_t duoff, void *stream);
/* gate_up_swiglu (ABI 7): y [T, F] (row stride ldy >= F, % 8, 16-byte aligned) = swiglu of the merged
 * gate|up projection x [T, H] . w_gate_up [2F, H]^T (gate rows 0..F-1, up rows F..2F-1; row strides ldx /
 * ldw, 16-byte aligned) without writing the [T, 2F] projection: g / u rounded to bf16 as the GEMM's
 * output, then swiglu_fwd's arithmetic. H % 64 == 0, F % 128 == 0; `splits` feature ranges per 256-token
 * block (1..64). For the no-grad forward (nothing keeps the projection for a backward); no reference
 * counterpart: HF Qwen2MLP's act_fn(gate_proj(x)) * up_proj(x) under the actor's no-grad old-logp pass,
 * dp_actor.py:331-333 (compute_log_prob's torch.no_grad forward). Not a §8 row. */
int va_gate_up_swiglu(const void *x, int64_t ldx, const void *w_gate_up, int64_t ldw, int dtype, int64_t T,
                      int64_t H, int64_t F, int splits, void *y, int64_t ldy, void *stream);
/* gate_up_swiglu_save (ABI 8): as va_gate_up_swiglu, and also the projection's g | u (bf16, exactly
 * the merged GEMM's output) into gu [T, 2F] (row stride ldgu >= 2F, % 8, 16-byte aligned): the
 * training forward's gate|up GEMM + swiglu_fwd in one kernel, gu kept for va_swiglu_bwd (HF
 * Qwen2MLP under autograd, dp_actor.py:331-333 in update_policy's forward). Not a §8 row. */
int va_gate_up_swiglu_save(const void *x, int64_t ldx, const void *w_gate_up, int64_t ldw, int dtype, int64_t T,
                           int64_t H, int64_t F, int splits, void *y, int64_t ldy, void *gu, int64_t ldgu,
                           void *stream);
/* qkv_rope (ABI 9): q [T, Hq D], k / v [T, Hk D] (contiguous, 16-byte aligned) from x [T, H] and the merged
 * q|k|v weight w_qkv [(Hq + 2 Hk) D, H] (row strides ldx / ldw, 16-byte aligned) plus its bias [(Hq + 2 Hk) D]
 * (nullable): bf16(x w^T + b), then rope_qkv_fwd's rotate-half RoPE on q and k with cos / sin [T, D] (row
 * stride D) — the GEMM + rope_qkv_fwd pair without the [T, (Hq + 2 Hk) D] projection in HBM. D == 64,
 * H % 64 == 0; `splits` feature ranges per 256-token block (1..64). Qwen2Attention's q/k/v_proj +
 * apply_rotary_pos_emb under the actor's forwards (dp_actor.py:331-333). Not a §8 row. */
int va_qkv_rope(const void *x, int64_t ldx, const void *w_qkv, int64_t ldw, const void *bias, const void *cos,
                const void *sin, int dtype, int64_t T, int64_t H, int Hq, int Hk, int D, int splits, void *q, void *k,
                void *v, void *stream);
int va_rope_qkv_fwd(const void *qkv, int64_t ld, const void *cos, const void *sin, int dtype, int64_t T,
                    int64_t Hq, int64_t Hk, int64_t D, void *q, void *k, void *v, void *stream);
int va_rope_qkv_bwd(const void *dq, const void *dk, const void *dv, const void *cos, const void *sin, int dtype,
                    int64_t T, int64_t Hq, int64_t Hk, int64_t D, void *dqkv, int64_t ld, void *stream);

/* linear_tn (ABI 11): y [M, N] (row stride ldy >= N, % 4, 8-byte aligned) = bf16(x [M, K] . w [N, K]^T (+ bias
 * [N])), fp32 accumulation — F.linear's layout, both operands contiguous along K (row strides ldx / ldw, % 8,
 * 16-byte aligned), the bias added to the fp32 sum before the one rounding (nullable, 8-byte aligned). Output
 * tiles of 256 rows x tile_n columns, tile_n in {192, 224, 256, 288} dividing N (0 = the first of 224, 288,
 * 256, 192 that does: va_linear_tn_tile(N), 0 when none does); K % 64 == 0; `per` tiles per persistent
 * workgroup (0 = automatic: one round of 256 workgroups). The backbone's projections (forward, and the input
 * gradients over a transposed weight copy) whose widths 896 / 1,152 are not multiples of 256: torch's
 * nn.Linear under FSDP in the reference (dp_actor.py:331-333, :465-470). Not a §8 row. */
int va_linear_tn_tile(int64_t N);
int va_linear_tn(const void *x, int64_t ldx, const void *w, int64_t ldw, const void *bias, int dtype, int64_t M,
                 int64_t N, int64_t K, int tile_n, int per, void *y, int64_t ldy, void *stream);

/* transpose_16: out [C, R] (row stride ld_out) = in [R, C] (row stride ld_in)^T for any 16-bit
 * element type; R, C, strides multiples of 8, 16-byte aligned buffers. The layout step of the
 * backward input-gradient GEMMs (dX = dY W over a K-contiguous W^T; no reference counterpart:
 * the reference leaves this GEMM's layout to FSDP / autograd, dp_actor.py:465-470). */
int va_transpose_16(const void *in, int64_t ld_in, int64_t R, int64_t C, void *out, int64_t ld_out, void *stream);

/* weight_grad: dW [M, N] bf16 (row-major, contiguous) = dY [K, M]^T X [K, N] (row strides ldy / ldx,
 * bf16, fp32 accumulation), the backward weight gradient of the backbone's linear layers (K = packed
 * tokens; no reference counterpart: torch's linear backward under FSDP, dp_actor.py:465-470). K a
 * multiple of 32; M, N, strides multiples of 8; 16-byte aligned buffers. splits: K slices (0 =
 * automatic; fp32 partials in workspace = va_weight_grad_workspace_bytes(K, M, N, splits), summed in
 * slice order, rounded once). workspace_bytes: the size of the buffer passed (ABI 6): the launch
 * plans its tiles and slices once and fails with VA_E_ARG when that plan needs more than this (the
 * plan depends on VA_TUNE_WGRAD_TILES / _REMAINDER, which may change between the size query and the launch).
 * Not a §8 row. */
int64_t va_weight_grad_workspace_bytes(int64_t K, int64_t M, int64_t N, int splits);
/* column_sum: out [C] bf16 = sum over the T rows of x [T, C] bf16 (row stride ld), fp32 accumulation in
 * a fixed order (row slabs, then their partials): the bias gradient of the merged q|k|v projection
 * (no reference counterpart: torch's dy.sum(0) in the linear backward under FSDP, dp_actor.py:465-470).
 * C % 8 == 0, C <= 2048, 16-byte aligned x / out; workspace of va_column_sum_workspace_bytes(T, C)
 * bytes, its size passed as workspace_bytes. Not a §8 row. */
int64_t va_column_sum_workspace_bytes(int64_t T, int64_t C);
int va_column_sum(const void *x, int64_t ld, int dtype, int64_t T, int64_t C, float *workspace,
                  int64_t workspace_bytes, void *out, void *stream);
int va_weight_grad(const void *dy, int64_t ldy, const void *x, int64_t ldx, int64_t K, int64_t M, int64_t N,
                   int splits, float *workspace, int64_t workspace_bytes, void *out, void *stream);

/* ---------------------------------------------------------------------------------------
 * Fused lm_head + log-prob + entropy forward (the reference's use_fused_kernels
 * path, utils/kernel/kernels.py:120-663 + linear_cross_entropy.py:40-117): for hidden [N, H]
 * (row stride ldh) and weight [V, H] (row stride ldw), both bf16 and 16-byte aligned,
 *   logits = bf16(hidden @ weight^T), x = bf16(logits / temperature) (skipped at T == 1) — or,
 *   with dtype = VA_BF16 | VA_LOGITS_F32, the same in fp32 without the two roundings,
 *   logp[i] = x[i, labels[i]] - lse_i, entropy[i] = lse_i - sum softmax(x_i) x_i, lse[i],
 * without writing the logits. `splits` vocab ranges run in parallel and merge in fixed order.
 * workspace: va_linear_logprob_workspace_bytes(N, splits). entropy / lse may be NULL.
 * ------------------------------------------------------------------------------------ */
int64_t va_linear_logprob_workspace_bytes(int64_t N, int splits);
int va_linear_logprob_fwd(const void *hidden, int64_t ldh, const void *weight, int64_t ldw, int dtype,
                          const int64_t *labels, int64_t N, int64_t H, int64_t V, float temperature, int splits,
                          float *logp, float *entropy, float *lse, void *workspace, void *stream);

/* Fused lm_head + log-prob + entropy backward, first half (f1; the reference's
 * efficient_entropy_backward_kernel_general_d_logits_split_N, utils/kernel/kernels.py:1241-1342,
 * dispatched at :1491-1548): recomputes the logits tile by tile from hidden / weight exactly as
 * va_linear_logprob_fwd does (same dtype flags) and writes
 *   dlogits[i, v] = bf16( ( -p (g_entropy[i] (x - lse_i + H_i) + g_logp[i]) + g_logp[i] [v == labels[i]] ) / T ),
 *   p = exp(x - lse_i), x the logit as the forward saw it,
 * i.e. va_logprob_entropy_bwd's arithmetic, without the logits in HBM. lse / entropy: the forward's
 * outputs; g_logp / g_entropy may be NULL (zero). Only the vocab range [v_begin, v_end) of the V
 * entries is computed (ABI 6; [0, V) for all of it): dlogits [N, v_end - v_begin] bf16, column 0 =
 * vocab v_begin, row stride ldd >= v_end - v_begin (8-byte aligned, ldd % 4 == 0), (v_end - v_begin)
 * % 4 == 0 — the reference's vocab_per_split loop (kernels.py:1491-1548), so that only one range of
 * dlogits exists at a time; labels are valid against the whole V. The caller runs the lm_head's two
 * backward GEMMs on it (dhidden += dlogits W[v_begin:v_end], dW[v_begin:v_end] = dlogits^T hidden).
 * `splits` vocab sub-ranges per row block as in the forward. Only rows [v_begin, v_end) of weight are
 * read, so a vocabulary shard of a tensor-parallel lm_head (the reference's dist_process_group path,
 * kernels.py:1345-1553 with its rank offset) passes the address its full matrix's row 0 would have
 * (shard - v_begin * ldw), V = the whole vocabulary and the shard's range, with global label ids. */
int va_linear_logprob_bwd(const void *hidden, int64_t ldh, const void *weight, int64_t ldw, int dtype,
                          const int64_t *labels, const float *lse, const float *entropy, const float *g_logp,
                          const float *g_entropy, int64_t N, int64_t H, int64_t V, int64_t v_begin, int64_t v_end,
                          float temperature, int splits, void *dlogits, int64_t ldd, void *stream);

/* ---------------------------------------------------------------------------------------
 * Discounted returns for REINFORCE++ (mode VA_RET_RFPP, gamma) and ReMax (VA_RET_REMAX:
 * baselines [B] required, adv [B, R] written). rewards / returns / adv [B, R] fp32.
 * ------------------------------------------------------------------------------------ */
int va_discounted_returns(const float *rewards, const void *mask, int mask_dtype, int64_t B, int64_t R, float gamma,
                          int mode, const float *baselines, float *returns, float *adv, void *stream);

/* ---------------------------------------------------------------------------------------
 * Critic: fused clipped value loss (core_algos.py:992-1031, clip_by_value torch_functional.py:
 * 136-142) + the critic's vpred_mean metric (dp_critic.py:236-242).
 *   vpreds, values, returns [B, R] fp32; mask [B, R] of mask_dtype; agg_mode = VA_AGG_*.
 *   seg_rows / seg_off / n_seg as va_ppo_loss_fwd: 0 / NULL aggregates the whole batch into out[VA_VLOSS_NOUT]; 0 < seg_rows
 *   < B gives out[S][VA_VLOSS_NOUT] for the S loss micro-batches of seg_rows rows (dp_critic.py:
 *   218-242 per micro-batch). workspace: va_ppo_loss_workspace_bytes(B).
 * Backward: g_out[S][VA_VLOSS_NOUT] = d(loss)/d(out) (slots LOSS and VPRED_MEAN are read) ->
 *   d_vpreds [B, R]. Ties follow torch.maximum / minimum autograd (gradient halves).
 * ------------------------------------------------------------------------------------ */
#define VA_VLOSS_LOSS 0       /* vf_loss            core_algos.py:1029 */
#define VA_VLOSS_CLIPFRAC 1   /* vf_clipfrac        core_algos.py:1030 */
#define VA_VLOSS_VPRED_MEAN 2 /* critic/vpred_mean  dp_critic.py:241 */
#define VA_VLOSS_NTOKENS 3    /* sum(response_mask) (diagnostic) */
#define VA_VLOSS_NOUT 4
int va_value_loss_fwd(const float *vpreds, const float *values, const float *returns, const void *mask,
                      int mask_dtype, int64_t B, int64_t R, float cliprange_value, int agg_mode,
                      int64_t seg_rows, const int32_t *seg_off, int64_t n_seg, float *out, void *workspace,
                      void *stream);
int va_value_loss_bwd(const float *g_out, const float *vpreds, const float *values, const float *returns,
                      const void *mask, int mask_dtype, int64_t B, int64_t R, float cliprange_value,
                      int agg_mode, int64_t seg_rows, const int32_t *seg_off, int64_t n_seg,
                      const void *workspace, float *d_vpreds, void *stream);

/* ---------------------------------------------------------------------------------------
 * Causal varlen flash-attention forward for the actor backbone (not a §8 row). q [T, Hq, 64],
 * k / v [T, Hk, 64] bf16 packed by cu_seqlens [B+1] int32; block_table [n_blocks][2] int32 =
 * (sequence, first query row) of every 128-row query block (every query row of a sequence must
 * be < max_len); o [T, Hq, 64] bf16, lse [B, Hq, max_len] fp32 = ln sum exp(scale * q.k) (the
 * padded layout aten::_flash_attention_backward reads; rows >= a sequence's length untouched).
 * ------------------------------------------------------------------------------------ */
int va_flash_attn_fwd(const void *q, const void *k, const void *v, const int32_t *cu_seqlens,
                      const int32_t *block_table, int64_t n_blocks, int64_t T, int64_t Hq, int64_t Hk,
                      int64_t head_dim, int64_t max_len, float scale, void *o, float *lse, void *stream);
/* Backward of the above (no atomics, deterministic): dq / dk / dv bf16 like q / k / v. q_blocks
 * = the forward's block table; k_blocks = (sequence, first key) of every 128-key block; delta =
 * fp32 workspace [B, Hq, max_len] (rowsum(dO * O), written here); partial = fp32 workspace of
 * 2 * Hq * T * 64 (per-query-head dK / dV before the GQA group sum). */
int va_flash_attn_bwd(const void *q, const void *k, const void *v, const void *o, const void *dout, const float *lse,
                      const int32_t *cu_seqlens, const int32_t *q_blocks, int64_t n_q_blocks, const int32_t *k_blocks,
                      int64_t n_k_blocks, int64_t T, int64_t Hq, int64_t Hk, int64_t head_dim, int64_t max_len,
                      float scale, float *delta, float *partial, void *dq, void *dk, void *dv, void *stream);

/* ---------------------------------------------------------------------------------------
 * Host-side (no GPU) sequence-length balancing. Replaces verl/utils/seqlen_balancing.py:26-127
 * `karmarkar_karp(seqlen_list, k_partitions, equal_size)` with identical partitions.
 *   seqlens [n]; order [n] receives the item indices of partition 0, then 1, ... in the
 *   reference's item order; offsets [k + 1] the partition boundaries. equal_size requires n % k == 0.
 * ------------------------------------------------------------------------------------ */
int va_karmarkar_karp(const int64_t *seqlens, int64_t n, int64_t k, int equal_size, int64_t *order,
                      int64_t *offsets);

#ifdef __cplusplus
}
#endif
#endif /* VERL_AMD_H */
