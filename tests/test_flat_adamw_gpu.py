"""grad_sync.FlatAdamW (va_adamw_flat, csrc/optim.hip): AdamW over the mixed-precision manager's flat
fp32 buckets with the gradient clip and the next zero_grad folded in, against the reference's
optimizer step (dp_actor.py:272-288: clip_grad_norm_ then torch.optim.AdamW, fsdp_workers.py:418-423)
run as torch.optim.AdamW(fused=True) over the same masters with the manager's in-place clip."""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(96, 200), torch.nn.GELU(), torch.nn.Linear(200, 67, bias=False),
                               torch.nn.Linear(67, 5)).to(DEV)


def _pair(bucket_bytes=40_000):
    from verl_amd.workers.grad_sync import FlatAdamW, MixedPrecisionParams

    base = _model(0)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    ma = MixedPrecisionParams(a, bucket_bytes=bucket_bytes, sync_params=False)
    mb = MixedPrecisionParams(b, bucket_bytes=bucket_bytes, sync_params=False)
    assert len(ma.buckets) > 1  # several flat buckets, parameters straddling none
    oa = FlatAdamW(ma, lr=1e-3, betas=(0.9, 0.999), weight_decay=0.01)
    ob = torch.optim.AdamW(mb.optimizer_params(), lr=1e-3, betas=(0.9, 0.999), weight_decay=0.01, fused=True)
    return (a, ma, oa), (b, mb, ob)


def _backward(model, manager, x):
    manager.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = model(x).float().square().mean()
    loss.backward()
    manager.after_backward()


@pytest.mark.parametrize("max_norm", [1e-3, 1e3])  # the clip active / inactive
def test_flat_adamw_equals_torch_fused_adamw(max_norm):
    """Masters, moments and step counts after several steps (an LR change between them, a clip that
    scales the gradients or not) equal torch.optim.AdamW(fused=True) + the in-place clip bit for bit;
    the folded zero_grad leaves every gradient bucket zero."""
    (a, ma, oa), (b, mb, ob) = _pair()
    g = torch.Generator(device=DEV).manual_seed(1)
    for it in range(4):
        x = torch.randn(33, 96, device=DEV, generator=g)
        _backward(a, ma, x)
        _backward(b, mb, x)
        for ba, bb in zip(ma.buckets, mb.buckets, strict=True):  # identical gradients on both sides
            bb.buf.copy_(ba.buf)
        na = ma.clip_grad_norm_(max_norm)
        nb = mb.clip_grad_norm_(max_norm)
        assert torch.equal(na, nb)
        if it == 2:
            for opt in (oa, ob):
                opt.param_groups[0]["lr"] = 3e-4
        oa.step()
        ob.step()
        ma.after_step()
        mb.after_step()
        for (fa, ga), (fb, _) in zip(ma.flat_buckets(), mb.flat_buckets(), strict=True):
            assert torch.equal(fa, fb), (it, (fa - fb).abs().max().item())
            assert torch.count_nonzero(ga) == 0
        for pa, pb in zip(ma.optimizer_params(), mb.optimizer_params(), strict=True):
            sa, sb = oa.state[pa], ob.state[pb]
            assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"])
            assert float(sa["step"]) == float(sb["step"]) == it + 1
    for pa, pb in zip(a.parameters(), b.parameters(), strict=True):
        assert torch.equal(pa, pb)  # the bf16 compute weights derived from the masters


def test_flat_adamw_skips_on_found_inf_and_drops_the_gradients():
    """found_inf = 1 (the non-finite grad-norm skip, set by dp_actor.step_unless_nonfinite): masters,
    moments and the step count unchanged, gradients zeroed; found_inf = 0 then steps as usual."""
    (a, ma, oa), _ = _pair()
    x = torch.randn(8, 96, device=DEV)
    _backward(a, ma, x)
    ma.clip_grad_norm_(1.0)
    oa.step()
    before = [f.clone() for f, _ in ma.flat_buckets()]
    m_before = [m.clone() for m in oa._m]
    _backward(a, ma, x)
    ma.clip_grad_norm_(1.0)
    oa.found_inf = torch.ones((), device=DEV)
    oa.step()
    oa.found_inf = None
    for (f, gbuf), f0, m, m0 in zip(ma.flat_buckets(), before, oa._m, m_before, strict=True):
        assert torch.equal(f, f0) and torch.equal(m, m0) and torch.count_nonzero(gbuf) == 0
    assert float(oa._step) == 1.0
    _backward(a, ma, x)
    ma.clip_grad_norm_(1.0)
    oa.found_inf = torch.zeros((), device=DEV)
    oa.step()
    oa.found_inf = None
    assert float(oa._step) == 2.0
    assert any(not torch.equal(f, f0) for (f, _), f0 in zip(ma.flat_buckets(), before, strict=True))


def test_zero_grad_after_a_folded_step_and_accumulation():
    """The manager's zero_grad skips the buckets the step already zeroed, and zeroes them again once
    a backward accumulated into them without a step (e.g. a dropped mini-batch)."""
    (a, ma, oa), _ = _pair()
    x = torch.randn(8, 96, device=DEV)
    _backward(a, ma, x)
    assert any(torch.count_nonzero(b.buf) for b in ma.buckets)
    ma.zero_grad()
    assert all(torch.count_nonzero(b.buf) == 0 for b in ma.buckets)
    _backward(a, ma, x)
    ma.clip_grad_norm_(1.0)
    oa.step()
    ma.zero_grad()
    assert all(torch.count_nonzero(b.buf) == 0 for b in ma.buckets)


def test_adamw_flat_rejects_bad_arguments():
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    t = torch.zeros(16, device=DEV)
    s = torch.ones((), device=DEV)
    with pytest.raises(RuntimeError, match="hyper-parameters"):
        L.call("va_adamw_flat", K._p(t), K._p(t), K._p(t), K._p(t), 16, 1e-3, 1.5, 0.999, 1e-8, 0.0, K._p(s), None,
               None, 0, K._stream(t))
    with pytest.raises(RuntimeError, match="aligned"):
        L.call("va_adamw_flat", K._p(t[1:]), K._p(t), K._p(t), K._p(t), 8, 1e-3, 0.9, 0.999, 1e-8, 0.0, K._p(s), None,
               None, 0, K._stream(t))


def test_state_dict_round_trip_resumes_bitwise():
    """A checkpoint of FlatAdamW (torch's Optimizer.state_dict) loaded into a fresh one resumes the
    same trajectory bit for bit: the loaded moments and step land in the flat buffers the kernel updates."""
    import copy as _copy

    from verl_amd.workers.grad_sync import FlatAdamW

    (a, ma, oa), (b, mb, _) = _pair()
    ob = FlatAdamW(mb, lr=1e-3, betas=(0.9, 0.999), weight_decay=0.01)
    g = torch.Generator(device=DEV).manual_seed(3)
    xs = [torch.randn(16, 96, device=DEV, generator=g) for _ in range(4)]
    for x in xs[:2]:
        _backward(a, ma, x)
        ma.clip_grad_norm_(1.0)
        oa.step()
        ma.after_step()
    sd = _copy.deepcopy(oa.state_dict())
    for (fb, _), (fa, _) in zip(mb.flat_buckets(), ma.flat_buckets(), strict=True):
        fb.copy_(fa)  # the model checkpoint: masters (and the bf16 weights derived from them)
    mb.after_step()
    ob.load_state_dict(sd)
    assert float(ob._step) == 2.0
    for x in xs[2:]:
        for model, man, opt in ((a, ma, oa), (b, mb, ob)):
            _backward(model, man, x)
            man.clip_grad_norm_(1.0)
            opt.step()
            man.after_step()
    for (fa, _), (fb, _) in zip(ma.flat_buckets(), mb.flat_buckets(), strict=True):
        assert torch.equal(fa, fb)
    for ma_, mb_ in zip(oa._m + oa._v, ob._m + ob._v, strict=True):
        assert torch.equal(ma_, mb_)
