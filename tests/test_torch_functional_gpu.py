"""The log-prob family of verl/utils/torch_functional.py on the gfx950 kernels against the CPU oracle
(logprobs_from_logits_naive, _flash_attn, log_probs_from_logits_response, the two remove-padding
variants with the reference's rolled packed labels, post_process_logits)."""

import pytest
import torch

from oracle import reference_ops as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(B=3, S=12, V=1000, R=5, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (B, S), generator=g)
    am = torch.ones(B, S, dtype=torch.int64)
    am[0, :4] = 0  # left padding
    am[1, :2] = 0
    logits = torch.randn(B, S, V, generator=g)
    return ids, am, logits, R


def test_logprob_variants_match_the_oracle():
    from verl_amd.utils import torch_functional as vF

    ids, am, logits, R = _case()
    x = logits.reshape(-1, logits.shape[-1])
    want = ref.logprobs_from_logits(x, ids.reshape(-1)).view(ids.shape)
    for fn in (vF.logprobs_from_logits_naive, vF.logprobs_from_logits_flash_attn):
        got = fn(x.to(DEV).clone(), ids.reshape(-1).to(DEV)).view(ids.shape).cpu()
        torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-5)
    got = vF.log_probs_from_logits_response(ids.to(DEV), logits.to(DEV).clone(), R).cpu()
    want = ref.logprobs_from_logits(logits[:, -R - 1:-1].reshape(-1, logits.shape[-1]), ids[:, -R:].reshape(-1))
    torch.testing.assert_close(got, want.view(-1, R), atol=1e-5, rtol=1e-5)


def test_rmpad_logprob_variants_follow_the_rolled_packed_stream():
    """torch_functional.py:438-490: logits of the packed valid tokens, labels = packed ids rolled by
    one over the WHOLE stream (a row's last token is labelled by the next row's first), scattered back
    to [B, S] with zeros at the padding, cut to [:, -R-1:-1]."""
    from verl_amd.utils import torch_functional as vF

    ids, am, logits, R = _case(seed=1)
    B, S, V = logits.shape
    idx = torch.nonzero(am.flatten()).flatten()
    ids_rmpad = ids.flatten()[idx]
    logits_rmpad = logits.reshape(B * S, V)[idx]
    rolled = torch.roll(ids_rmpad, -1)
    full = torch.zeros(B * S)
    full[idx] = ref.logprobs_from_logits(logits_rmpad, rolled)
    want = full.view(B, S)[:, -R - 1:-1]
    got = vF.log_probs_from_logits_response_rmpad(ids.to(DEV), am.to(DEV), logits_rmpad.to(DEV).clone(), R).cpu()
    torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-5)
    got = vF.log_probs_from_logits_all_rmpad(ids_rmpad.unsqueeze(0).to(DEV), logits_rmpad.to(DEV).clone(),
                                             idx.to(DEV), B, S, R).cpu()
    torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-5)


def test_post_process_logits_divides_in_place():
    from verl_amd.utils import torch_functional as vF

    x = torch.randn(4, 10, device=DEV)
    y = x.clone()
    out = vF.post_process_logits(None, y, 2.0, None, None)
    assert out.data_ptr() == y.data_ptr() and torch.equal(out, x / 2.0)
    assert vF.post_process_logits(None, x, 1.0, 5, 0.9) is x
