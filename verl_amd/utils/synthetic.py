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
) -> DataProto:
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
    if permute:
        data.reorder(torch.from_numpy(rs.permutation(B)))
    data.meta_info["global_token_num"] = data.batch["attention_mask"].sum(-1).tolist()
    return data.to(device)
