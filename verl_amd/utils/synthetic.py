"""Synthetic GRPO batches with the shapes of SURVEY.md §8(d) (no datasets offline).

Layout follows the reference's fit loop (ray_trainer.py:1160-1219): prompts left-padded to P,
responses right-padded to R, each prompt repeated n times with interleave (protocol.py:772-814)
and then permuted (as _balance_batch does, ray_trainer.py:1064-1079), uid per prompt,
response_mask = attention_mask[:, -R:], and a 0/1 outcome score at the last valid response
token (reward_manager/naive.py:98).
"""

from __future__ import annotations

import numpy as np
import torch

from ..protocol import DataProto


def make_grpo_batch(
    n_prompts: int = 64,
    n: int = 8,
    prompt_len: int = 256,
    response_len: int = 1024,
    vocab: int = 151936,
    min_prompt: int = 64,
    dense_responses: bool = True,
    min_response: int = 128,
    seed: int = 1234,
    device="cpu",
    permute: bool = True,
    step_noise: bool = False,
) -> DataProto:
    """``step_noise``: also attach ``old_noise`` / ``ref_noise`` [B, R] ~ N(0, 1) drawn per row
    before the permutation, so the bench's perturbations of the recomputed log-probs (SURVEY §8d:
    old = new + 0.05 N, ref = new + 0.1 N) travel with their rows and do not depend on how the
    batch is split over ranks."""
    g = torch.Generator().manual_seed(seed)
    rs = np.random.RandomState(seed)
    B, P, R = n_prompts * n, prompt_len, response_len
    p_len = torch.randint(min_prompt, P + 1, (n_prompts,), generator=g).repeat_interleave(n)
    if dense_responses:
        r_len = torch.full((B,), R, dtype=torch.long)
    else:
        r_len = torch.randint(min_prompt if min_response is None else min_response, R + 1, (B,), generator=g)
    prompt_ids = torch.randint(0, vocab, (n_prompts, P), generator=g).repeat_interleave(n, dim=0)
    responses = torch.randint(0, vocab, (B, R), generator=g)
    cols_p = torch.arange(P)[None, :]
    cols_r = torch.arange(R)[None, :]
    p_mask = (cols_p >= (P - p_len)[:, None]).long()
    r_mask = (cols_r < r_len[:, None]).long()
    prompt_ids = prompt_ids * p_mask
    responses = responses * r_mask
    input_ids = torch.cat([prompt_ids, responses], dim=1)
    attention_mask = torch.cat([p_mask, r_mask], dim=1)
    position_ids = torch.clamp(torch.cumsum(attention_mask, dim=1) - 1, min=0)
    scores = torch.bernoulli(torch.full((B,), 0.5), generator=g)
    token_level_scores = torch.zeros(B, R)
    token_level_scores[torch.arange(B), r_len - 1] = scores
    uid = np.array([f"prompt-{i // n}" for i in range(B)], dtype=object)
    data = DataProto.from_dict(
        tensors=dict(
            input_ids=input_ids, attention_mask=attention_mask, position_ids=position_ids, responses=responses,
            response_mask=attention_mask[:, -R:].clone(), token_level_scores=token_level_scores,
            token_level_rewards=token_level_scores.clone(),
        ),
        non_tensors=dict(uid=uid),
        meta_info=dict(temperature=1.0),
    )
    if step_noise:
        gn = torch.Generator().manual_seed(seed + 7)
        data.batch["old_noise"] = torch.randn(B, R, generator=gn)
        data.batch["ref_noise"] = torch.randn(B, R, generator=gn)
    if permute:
        data.reorder(torch.from_numpy(rs.permutation(B)))
    data.meta_info["global_token_num"] = data.batch["attention_mask"].sum(-1).tolist()
    return data.to(device)


def make_vl_grpo_batch(
    model,
    n_prompts: int = 4,
    n: int = 4,
    prompt_len: int = 96,
    response_len: int = 128,
    image_grid=(1, 4, 8),
    min_text: int = 8,
    dense_responses: bool = False,
    min_response: int = 16,
    seed: int = 1234,
    device="cpu",
    permute: bool = True,
) -> DataProto:
    """A Qwen2-VL GRPO batch (BASELINE config 4): each prompt is left padding, <vision_start>, the
    image's placeholder tokens (t*h*w / merge^2 of them), <vision_end>, text; one image per prompt
    with random pixel patches. position_ids [B, 3, P+R]: the model's get_rope_index over the
    prompt (rl_dataset's mrope ids), then last prompt position + 1..R on all three rows
    (vllm_rollout_spmd.py:353-363). multi_modal_inputs: one dict per row (pixel_values,
    image_grid_thw), as the reference's dataset emits them."""
    cfg = model.config
    vcfg = cfg.vision_config
    vocab = cfg.text_config.vocab_size
    g = torch.Generator().manual_seed(seed)
    rs = np.random.RandomState(seed)
    B, P, R = n_prompts * n, prompt_len, response_len
    t, h, w = image_grid
    merge = vcfg.spatial_merge_size
    n_img = t * h * w // (merge * merge)
    fixed = n_img + 2
    assert P >= fixed + min_text
    text_hi = min(vocab, cfg.image_token_id, cfg.video_token_id, cfg.vision_start_token_id) - 1
    p_len = torch.randint(fixed + min_text, P + 1, (n_prompts,), generator=g)
    prompts = torch.zeros(n_prompts, P, dtype=torch.long)
    types = torch.zeros(n_prompts, P, dtype=torch.int32)
    p_mask = torch.zeros(n_prompts, P, dtype=torch.long)
    for i in range(n_prompts):
        s = P - int(p_len[i])
        body = torch.randint(0, text_hi, (int(p_len[i]),), generator=g)
        body[0] = cfg.vision_start_token_id
        body[1 : 1 + n_img] = cfg.image_token_id
        body[1 + n_img] = cfg.vision_end_token_id
        prompts[i, s:] = body
        types[i, s + 1 : s + 1 + n_img] = 1
        p_mask[i, s:] = 1
    grid = torch.tensor([list(image_grid)] * n_prompts)
    with torch.no_grad():
        pos, _ = model.model.get_rope_index(prompts.to(model.device), types.to(model.device), image_grid_thw=grid,
                                            attention_mask=p_mask.to(model.device))
    pos = pos.cpu().transpose(0, 1)  # [n_prompts, 3, P]
    feat = vcfg.in_channels * vcfg.temporal_patch_size * vcfg.patch_size ** 2
    pixels = [torch.randn(t * h * w, feat, generator=g) for _ in range(n_prompts)]

    prompts, p_mask, pos = (x.repeat_interleave(n, dim=0) for x in (prompts, p_mask, pos))
    if dense_responses:
        r_len = torch.full((B,), R, dtype=torch.long)
    else:
        r_len = torch.randint(min_response, R + 1, (B,), generator=g)
    r_mask = (torch.arange(R)[None, :] < r_len[:, None]).long()
    responses = torch.randint(0, text_hi, (B, R), generator=g) * r_mask
    delta = torch.arange(1, R + 1).view(1, 1, R).expand(B, 3, R)
    position_ids = torch.cat([pos, pos[..., -1:] + delta], dim=-1)
    input_ids = torch.cat([prompts, responses], dim=1)
    attention_mask = torch.cat([p_mask, r_mask], dim=1)
    scores = torch.bernoulli(torch.full((B,), 0.5), generator=g)
    token_level_scores = torch.zeros(B, R)
    token_level_scores[torch.arange(B), r_len - 1] = scores
    uid = np.array([f"prompt-{i // n}" for i in range(B)], dtype=object)
    mm = np.empty(B, dtype=object)
    for i in range(B):
        mm[i] = {"pixel_values": pixels[i // n], "image_grid_thw": grid[i // n : i // n + 1]}
    data = DataProto.from_dict(
        tensors=dict(
            input_ids=input_ids, attention_mask=attention_mask, position_ids=position_ids, responses=responses,
            response_mask=attention_mask[:, -R:].clone(), token_level_scores=token_level_scores,
            token_level_rewards=token_level_scores.clone(),
        ),
        non_tensors=dict(uid=uid, multi_modal_inputs=mm),
        meta_info=dict(temperature=1.0),
    )
    if permute:
        data.reorder(torch.from_numpy(rs.permutation(B)))
    data.meta_info["global_token_num"] = data.batch["attention_mask"].sum(-1).tolist()
    return data.to(device)
