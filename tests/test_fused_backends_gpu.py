"""The reference's two fused lm_head backends as drop-ins: verl.utils.kernel.linear_cross_entropy
(Triton; reduction none / sum / mean, vocab tensor parallelism over dist_process_group) and
verl.utils.experimental.torch_functional.FusedLinearForPPO (chunked torch), both on the gfx950 fused
kernels. Checked against the reference tests' own torch formulations (tests/utils/
test_linear_cross_entropy.py run_torch_entropy, test_linear_cross_entropy_tp.py TorchEntropyTP) at
their tolerances, and TP against the single-shard result: emulated in one process at 2 and 4 shards
and as 2 real ranks (gloo, both on cuda:0)."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _torch_entropy(hidden, weight, labels, temperature, reduction="none"):
    """tests/utils/test_linear_cross_entropy.py:57-80: fp32 logits, -cross_entropy, lse - sum p x."""
    logits = torch.matmul(hidden.float(), weight.float().t()) / temperature
    pd = torch.softmax(logits, dim=-1)
    entropy = torch.logsumexp(logits, dim=-1) - torch.sum(pd * logits, dim=-1)
    logprobs = -torch.nn.functional.cross_entropy(logits, labels, reduction=reduction)
    return logprobs, entropy


def _inputs(N=1000, H=896, V=4096, seed=0, dtype=torch.bfloat16):
    g = torch.Generator(device=DEV).manual_seed(seed)
    # the reference test's distributions (test_linear_cross_entropy.py:140-152)
    hidden = torch.empty(N, H, device=DEV).uniform_(-0.5, 0.5, generator=g).to(dtype)
    weight = torch.empty(V, H, device=DEV).uniform_(-0.5, 0.5, generator=g).to(dtype)
    labels = torch.randint(0, V, (N,), device=DEV, generator=g)
    return hidden, weight, labels


@pytest.mark.parametrize("reduction", ["none", "sum", "mean"])
@pytest.mark.parametrize("V", [4096, 4098, 151936])
def test_linear_cross_entropy_matches_reference_torch(reduction, V):
    from verl_amd.utils.kernel.linear_cross_entropy import linear_cross_entropy

    N = 1000 if V < 100000 else 256
    hidden, weight, labels = _inputs(N=N, V=V, seed=V)
    T = 1.5
    h1, w1 = hidden.clone().requires_grad_(True), weight.clone().requires_grad_(True)
    lp, ent = linear_cross_entropy(h1, w1, labels, T, reduction)
    h2, w2 = hidden.clone().requires_grad_(True), weight.clone().requires_grad_(True)
    lp_ref, ent_ref = _torch_entropy(h2, w2, labels, T, reduction)  # -(sum / mean of the cross entropies)
    assert lp.shape == lp_ref.shape and ent.shape == (N,)
    # the reference test's kernel tolerances (:210-216)
    torch.testing.assert_close(lp, lp_ref, atol=1e-3 * (N if reduction == "sum" else 1), rtol=2e-4)
    torch.testing.assert_close(ent, ent_ref, atol=5e-3, rtol=5e-4)
    g = torch.Generator(device=DEV).manual_seed(1)
    g_lp = torch.randn(lp.shape, device=DEV, generator=g)
    g_ent = torch.randn(N, device=DEV, generator=g)
    torch.autograd.backward([lp, ent], [g_lp, g_ent])
    torch.autograd.backward([lp_ref, ent_ref], [g_lp, g_ent])
    torch.testing.assert_close(h1.grad.float(), h2.grad.float(), atol=2e-2, rtol=4e-2)
    torch.testing.assert_close(w1.grad.float(), w2.grad.float(), atol=2e-2, rtol=4e-2)


@pytest.mark.parametrize("method", ["_Total_Separate", "_Total_Fuse_MN"])
def test_backward_methods_give_the_split_dlogits_gradients(method):
    """kernels.set_backward_method (the reference's kernels.py:112-117): _Total_Separate runs one
    vocabulary range ([N, V] dlogits), _Total_Fuse_MN the vocabulary-range path; both give the default
    _Split_Dlogits_N gradients up to fp32 summation order (16 ranges vs 1 for d_hidden, the weight-gradient
    tiling of a 9,504-row range vs the whole vocabulary)."""
    from verl_amd.utils.kernel import kernels as KK
    from verl_amd.utils.kernel.linear_cross_entropy import linear_cross_entropy

    hidden, weight, labels = _inputs(N=512, V=151936, seed=5)
    g = torch.Generator(device=DEV).manual_seed(2)
    g_lp, g_ent = torch.randn(512, device=DEV, generator=g), torch.randn(512, device=DEV, generator=g)
    grads = {}
    try:
        for m in ("_Split_Dlogits_N", method):
            KK.set_backward_method(getattr(KK.BackwardEnum, m))
            h, w = hidden.clone().requires_grad_(True), weight.clone().requires_grad_(True)
            lp, ent = linear_cross_entropy(h, w, labels, 1.0, "none")
            torch.autograd.backward([lp, ent], [g_lp, g_ent])
            grads[m] = (h.grad.float(), w.grad.float())
        KK.set_backward_method(KK.BackwardEnum._Split_Dlogits_M)
        h = hidden.clone().requires_grad_(True)
        lp, ent = linear_cross_entropy(h, weight, labels, 1.0, "none")
        with pytest.raises(NotImplementedError):
            lp.sum().backward()
    finally:
        KK.set_backward_method(KK.BackwardEnum._Split_Dlogits_N)
    a, b = grads["_Split_Dlogits_N"], grads[method]
    for x, y in zip(a, b):  # bf16 gradients: fp32 sums in another order, one rounding each
        assert ((x - y).norm() / x.norm()).item() < 5e-3


def test_linear_cross_entropy_shapes_and_contract():
    from verl_amd.utils.kernel.linear_cross_entropy import linear_cross_entropy

    hidden, weight, labels = _inputs(N=2 * 300, V=4096)
    lp, ent = linear_cross_entropy(hidden.view(2, 300, -1), weight, labels.view(2, 300), 1.0, "none")
    assert lp.shape == (600,) and ent.shape == (600,)  # flat, as the reference's kernel returns them
    with pytest.raises(ValueError, match="Invalid reduction"):
        linear_cross_entropy(hidden, weight, labels, 1.0, "max")
    with pytest.raises(AssertionError, match="temperature must be a float"):
        linear_cross_entropy(hidden, weight, labels, 1, "none")


def _shard_run(hidden, weight, labels, T, tp, g_lp, g_ent):
    """tp shards in one process: each shard's forward (labels shifted), the merge with the all-reduces
    done by hand, then each shard's backward through LinearCrossEntropy.backward's own code path."""
    import types

    from verl_amd import kernels as K
    from verl_amd.utils.kernel.linear_cross_entropy import tp_merge

    V = weight.shape[0]
    vs = V // tp
    parts = [K._linear_logprob_fwd_raw(hidden, weight[r * vs:(r + 1) * vs], labels - r * vs, T, fp32_logits=True,
                                       with_label_logit=True) for r in range(tp)]
    m = torch.stack([p[2] for p in parts]).max(0).values
    packed = None
    outs = []
    for r, (lp_l, ent_l, lse_l, xl) in enumerate(parts):
        cap = {}

        def amax(t):
            t.copy_(m)

        def asum(t, cap=cap):
            cap["t"] = t

        tp_merge(labels, r * vs, vs, V, lp_l, ent_l, lse_l, amax, asum, label_logit_l=xl)
        packed = cap["t"].clone() if packed is None else packed + cap["t"]
    for r, (lp_l, ent_l, lse_l, xl) in enumerate(parts):
        def amax(t):
            t.copy_(m)

        def asum(t):
            t.copy_(packed)

        outs.append(tp_merge(labels, r * vs, vs, V, lp_l, ent_l, lse_l, amax, asum, label_logit_l=xl))
    logp, ent, lse = outs[0]
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(o, outs[0]))  # every rank sees the same result
    dh, dws = torch.zeros(hidden.shape, dtype=torch.float32, device=DEV), []
    for r in range(tp):
        ctx = types.SimpleNamespace(needs_input_grad=(True, True), temperature=T, fp32_logits=True,
                                    vocab_offset=r * vs, vocab_total=V)
        d_h, d_w = K._LinearLogprob._vocab_split_backward(ctx, hidden, weight[r * vs:(r + 1) * vs].contiguous(),
                                                          labels, lse, ent, g_lp, g_ent)
        dh += d_h.float()
        dws.append(d_w)
    return logp, ent, dh, torch.cat(dws)


@pytest.mark.parametrize("tp", [2, 4])
def test_vocab_parallel_emulated_matches_single_shard(tp):
    from verl_amd.utils.kernel.linear_cross_entropy import linear_cross_entropy

    hidden, weight, labels = _inputs(N=777, V=4096 * 2, seed=tp)
    labels[5] = -100  # ignore_index: 0, as the single-shard kernel
    T = 1.5
    h1, w1 = hidden.clone().requires_grad_(True), weight.clone().requires_grad_(True)
    lp, ent = linear_cross_entropy(h1, w1, labels, T, "none")
    g = torch.Generator(device=DEV).manual_seed(2)
    g_lp, g_ent = torch.randn(777, device=DEV, generator=g), torch.randn(777, device=DEV, generator=g)
    g_lp[5] = 0.0
    torch.autograd.backward([lp, ent], [g_lp, g_ent])
    lp_t, ent_t, dh_t, dw_t = _shard_run(hidden, weight, labels, T, tp, g_lp, g_ent)
    assert lp_t[5].item() == 0.0 and lp[5].item() == 0.0
    torch.testing.assert_close(lp_t, lp, atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(ent_t, ent, atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(dh_t, h1.grad.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(dw_t.float(), w1.grad.float(), atol=2e-2, rtol=2e-2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from verl_amd.utils.kernel.linear_cross_entropy import linear_cross_entropy

        hidden, weight, labels = _inputs(N=512, V=4096 * world, seed=11)
        T = 1.0
        vs = weight.shape[0] // world
        h = hidden.clone().requires_grad_(True)
        w = weight[rank * vs:(rank + 1) * vs].clone().requires_grad_(True)
        lp, ent = linear_cross_entropy(h, w, labels, T, "none", dist.group.WORLD)
        g = torch.Generator(device=DEV).manual_seed(3)
        g_lp, g_ent = torch.randn(512, device=DEV, generator=g), torch.randn(512, device=DEV, generator=g)
        torch.autograd.backward([lp, ent], [g_lp, g_ent])
        dh = h.grad.float()
        dist.all_reduce(dh, op=dist.ReduceOp.SUM)  # the caller's all-reduce, as in the reference test
        # single-shard result on the whole vocabulary, and the reference test's torch formulation
        h1, w1 = hidden.clone().requires_grad_(True), weight.clone().requires_grad_(True)
        lp1, ent1 = linear_cross_entropy(h1, w1, labels, T, "none")
        torch.autograd.backward([lp1, ent1], [g_lp, g_ent])
        torch.testing.assert_close(lp, lp1, atol=2e-5, rtol=1e-5)
        torch.testing.assert_close(ent, ent1, atol=2e-5, rtol=1e-5)
        torch.testing.assert_close(dh, h1.grad.float(), atol=2e-2, rtol=2e-2)
        torch.testing.assert_close(w.grad.float(), w1.grad[rank * vs:(rank + 1) * vs].float(), atol=2e-2, rtol=2e-2)
        lp_ref, ent_ref = _torch_entropy(hidden, weight, labels, T)
        torch.testing.assert_close(lp, lp_ref, atol=1e-1, rtol=1e-2)  # test_linear_cross_entropy_tp.py:397-398
        torch.testing.assert_close(ent, ent_ref, atol=1e-1, rtol=1e-2)
        open(os.path.join(out_dir, f"ok{rank}"), "w").close()
    finally:
        dist.destroy_process_group()


def test_vocab_parallel_two_ranks_gloo(tmp_path):
    world = 2
    mp.spawn(_tp_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert all(os.path.exists(tmp_path / f"ok{r}") for r in range(world))


@pytest.mark.parametrize("T", [1.0, 0.7])
@pytest.mark.parametrize("ndim", [2, 3])
def test_fused_linear_for_ppo_matches_reference_torch_backend(T, ndim):
    """FusedLinearForPPO (utils/experimental/torch_functional.py) against the reference's own chunked
    torch formulation of the same function (:20-75, restated here): outputs in the inputs' dtype
    (bf16), shaped like input_ids; gradients within bf16 resolution."""
    from verl_amd.utils.experimental.torch_functional import FusedLinearForPPO

    hidden, weight, labels = _inputs(N=600, V=4096, seed=7)
    if ndim == 3:
        hidden, labels = hidden.view(2, 300, -1), labels.view(2, 300)

    def ref_fwd(h, w, ids):
        logits = (h @ w.t()) / T  # bf16 GEMM, bf16 division
        lg = logits.float()
        probs = lg.softmax(-1)
        lps = lg.log_softmax(-1).gather(-1, ids.unsqueeze(-1)).squeeze(-1)
        ent = torch.logsumexp(lg, -1) - (probs * lg).sum(-1)
        return lps.to(h.dtype), ent.to(h.dtype)

    h1, w1 = hidden.clone().requires_grad_(True), weight.clone().requires_grad_(True)
    lp, ent = FusedLinearForPPO(chunk_size=256)(h1, w1, labels, T)
    h2, w2 = hidden.clone().requires_grad_(True), weight.clone().requires_grad_(True)
    lp_r, ent_r = ref_fwd(h2, w2, labels)
    assert lp.dtype == torch.bfloat16 and lp.shape == labels.shape and ent.shape == labels.shape
    torch.testing.assert_close(lp.float(), lp_r.float(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(ent.float(), ent_r.float(), atol=2e-2, rtol=1e-2)
    g = torch.Generator(device=DEV).manual_seed(4)
    g_lp = torch.randn(labels.shape, device=DEV, generator=g).to(torch.bfloat16)
    g_ent = torch.randn(labels.shape, device=DEV, generator=g).to(torch.bfloat16)
    torch.autograd.backward([lp, ent], [g_lp, g_ent])
    torch.autograd.backward([lp_r, ent_r], [g_lp, g_ent])
    for a, b, what in ((h1.grad, h2.grad, "d hidden"), (w1.grad, w2.grad, "d weight")):
        err = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert err < 2e-2, f"{what}: relative L2 {err:.3e}"
