"""Microbenchmark of the verl_amd HIP kernels at the headline shapes, with HIP-event timing.

Reports, per kernel: average launch time, algorithmic bytes per launch (SURVEY §8d figures)
and achieved GB/s against the 8 TB/s HBM spec and a measured device-copy bandwidth.

  python tools/kernel_bench.py [--rows 8192] [--vocab 151936] [--iters 20] [--only logprob]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from verl_amd import _lib as L  # noqa: E402
from verl_amd import kernels as K  # noqa: E402

PEAK = 8000.0


def timeit(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    evs = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    ts = [a.elapsed_time(b) for a, b in evs]
    return float(np.median(ts)), float(np.min(ts))


def report(name, nbytes, med_ms, min_ms, copy_gbps, extra=None):
    gbps = nbytes / (med_ms * 1e-3) / 1e9
    d = dict(kernel=name, avg_us=round(med_ms * 1e3, 2), min_us=round(min_ms * 1e3, 2), algo_bytes=int(nbytes),
             gbps=round(gbps, 1), frac_spec=round(gbps / PEAK, 4),
             frac_copy=round(gbps / copy_gbps, 4) if copy_gbps else None)
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)
    return d


def bwd_ab(args, src, rounds=6):
    """Interleaved A/B of the log-prob backward: flat stream vs per-row chunks, out of place vs
    in place, 4 vs 8 vectors per lane (guide rule 24: interleave, report medians)."""
    dev = src.device
    x = src.view(args.rows, args.vocab)
    labels = torch.randint(0, args.vocab, (args.rows,), device=dev)
    lp, ent, lse = (torch.empty(args.rows, device=dev) for _ in range(3))
    g1 = torch.randn(args.rows, device=dev)
    dx = torch.empty_like(x)
    lib = L.load()
    st = K._stream(x)
    L.call("va_logprob_entropy_fwd", K._p(x), L.VA_BF16, args.rows, args.vocab, args.vocab, K._p(labels), 1.0,
           K._p(lp), K._p(ent), K._p(lse), st)

    def bwd(out):
        L.call("va_logprob_entropy_bwd", K._p(g1), None, K._p(x), L.VA_BF16, args.rows, args.vocab, args.vocab,
               K._p(labels), K._p(lse), K._p(ent), 1.0, K._p(out), args.vocab, st)

    variants = [(flat, ip, pipe) for flat in (-1, 0) for ip in (0, 1) for pipe in (0, 2)]
    times = {v: [] for v in variants}
    for _ in range(rounds):
        for flat, ip, pipe in variants:
            lib.va_set_tuning(L.VA_TUNE_BWD_FLAT, flat)
            lib.va_set_tuning(L.VA_TUNE_PIPELINE, pipe)
            times[(flat, ip, pipe)].append(timeit(lambda: bwd(x if ip else dx), 4, warmup=1)[0])
    lib.va_set_tuning(L.VA_TUNE_BWD_FLAT, -1)
    lib.va_set_tuning(L.VA_TUNE_PIPELINE, 0)
    bb = args.rows * (4 * args.vocab + 28)
    for (flat, ip, pipe), ts in times.items():
        med = float(np.median(ts))
        print(json.dumps(dict(kernel=f"bwd_{'flat' if flat else 'rows'}_{'inplace' if ip else 'outplace'}_u{8 if pipe else 4}",
                              rows=args.rows, median_us=round(med * 1e3, 1), min_us=round(min(ts) * 1e3, 1),
                              gbps=round(bb / (med * 1e-3) / 1e9, 1))), flush=True)


def sweep(args, src, copy_gbps):
    """Interleaved A/B of waves-per-row x non-temporal for fwd and bwd (guide rule 24)."""
    dev = src.device
    x = src.view(args.rows, args.vocab)
    labels = torch.randint(0, args.vocab, (args.rows,), device=dev)
    lp, ent, lse = (torch.empty(args.rows, device=dev) for _ in range(3))
    g1 = torch.randn(args.rows, device=dev)
    dx = torch.empty_like(x)
    lib = L.load()
    st = K._stream(x)

    def fwd():
        L.call("va_logprob_entropy_fwd", K._p(x), L.VA_BF16, args.rows, args.vocab, args.vocab, K._p(labels), 1.0,
               K._p(lp), K._p(ent), K._p(lse), st)

    def bwd():
        L.call("va_logprob_entropy_bwd", K._p(g1), None, K._p(x), L.VA_BF16, args.rows, args.vocab, args.vocab,
               K._p(labels), K._p(lse), K._p(ent), 1.0, K._p(dx), args.vocab, st)

    fwd()
    variants = [(4, 1, 0), (4, 1, 1), (4, 1, 2), (2, 1, 1), (1, 1, 1), (4, 0, 1), (2, 1, 0)]
    times = {("fwd",) + v: [] for v in variants}
    times.update({("bwd",) + v: [] for v in variants})
    for _ in range(5):
        for w, nt, pipe in variants:
            lib.va_set_tuning(L.VA_TUNE_FWD_WAVES_PER_ROW, w)
            lib.va_set_tuning(L.VA_TUNE_BWD_WAVES_PER_ROW, w)
            lib.va_set_tuning(L.VA_TUNE_NONTEMPORAL, nt)
            lib.va_set_tuning(L.VA_TUNE_PIPELINE, pipe)
            times[("fwd", w, nt, pipe)].append(timeit(fwd, 5, warmup=1)[0])
            times[("bwd", w, nt, pipe)].append(timeit(bwd, 5, warmup=1)[0])
    fb = args.rows * (2 * args.vocab + 20)
    bb = args.rows * (4 * args.vocab + 28)
    for k, ts in times.items():
        nb = fb if k[0] == "fwd" else bb
        med = float(np.median(ts))
        print(json.dumps(dict(kernel=f"{k[0]}_wpr{k[1]}_nt{k[2]}_pipe{k[3]}", median_us=round(med * 1e3, 1),
                              min_us=round(min(ts) * 1e3, 1), gbps=round(nb / (med * 1e-3) / 1e9, 1))), flush=True)
    for key, default in ((L.VA_TUNE_FWD_WAVES_PER_ROW, 0), (L.VA_TUNE_BWD_WAVES_PER_ROW, 0),
                         (L.VA_TUNE_NONTEMPORAL, -1), (L.VA_TUNE_PIPELINE, 0)):
        lib.va_set_tuning(key, default)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--vocab", type=int, default=151936)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="all")
    ap.add_argument("--sweep", action="store_true", help="A/B the log-prob launch shapes (interleaved rounds)")
    ap.add_argument("--bwd-ab", action="store_true", help="A/B the log-prob backward layouts (interleaved rounds)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    res = []

    # measured device copy bandwidth (read + write), same footprint as the logits
    n_el = args.rows * args.vocab
    src = torch.empty(n_el, dtype=torch.bfloat16, device=dev).normal_()
    dst = torch.empty_like(src)
    med, mn = timeit(lambda: dst.copy_(src), args.iters)
    copy_gbps = 2 * n_el * 2 / (med * 1e-3) / 1e9
    print(json.dumps(dict(kernel="device_copy_bf16", avg_us=round(med * 1e3, 1), gbps=round(copy_gbps, 1))), flush=True)
    del dst

    if args.sweep:
        sweep(args, src, copy_gbps)
        return
    if args.bwd_ab:
        bwd_ab(args, src)
        return

    if args.only in ("all", "logprob"):
        logits = (src.view(args.rows, args.vocab) * 2.0)
        del src
        labels = torch.randint(0, args.vocab, (args.rows,), device=dev)
        s = 2
        fwd_bytes = args.rows * (s * args.vocab + 8 + 12)
        x = logits

        def fwd():
            K.logprob_entropy(x, labels, 1.0)

        med, mn = timeit(fwd, args.iters)
        res.append(report("logprob_entropy_fwd", fwd_bytes, med, mn, copy_gbps, dict(rows=args.rows, vocab=args.vocab)))
        lp = torch.empty(args.rows, device=dev)
        ent = torch.empty(args.rows, device=dev)
        lse = torch.empty(args.rows, device=dev)
        L.call("va_logprob_entropy_fwd", K._p(x), L.VA_BF16, args.rows, args.vocab, args.vocab, K._p(labels), 1.0,
               K._p(lp), K._p(ent), K._p(lse), K._stream(x))
        g1 = torch.randn(args.rows, device=dev)
        dx = torch.empty_like(x)
        bwd_bytes = args.rows * (2 * s * args.vocab + 28)

        def bwd():
            L.call("va_logprob_entropy_bwd", K._p(g1), None, K._p(x), L.VA_BF16, args.rows, args.vocab, args.vocab,
                   K._p(labels), K._p(lse), K._p(ent), 1.0, K._p(dx), args.vocab, K._stream(x))

        med, mn = timeit(bwd, args.iters)
        res.append(report("logprob_entropy_bwd", bwd_bytes, med, mn, copy_gbps, dict(rows=args.rows, vocab=args.vocab)))
        L.call("va_set_tuning", L.VA_TUNE_BWD_FLAT, 0)  # A/B: per-row chunks
        med, mn = timeit(bwd, args.iters)
        res.append(report("logprob_entropy_bwd_rowchunks", bwd_bytes, med, mn, copy_gbps))
        L.call("va_set_tuning", L.VA_TUNE_BWD_FLAT, -1)
        med, mn = timeit(bwd, args.iters)
        res.append(report("logprob_entropy_bwd_flat_again", bwd_bytes, med, mn, copy_gbps))

        def bwd_inplace():
            L.call("va_logprob_entropy_bwd", K._p(g1), None, K._p(x), L.VA_BF16, args.rows, args.vocab, args.vocab,
                   K._p(labels), K._p(lse), K._p(ent), 1.0, K._p(x), args.vocab, K._stream(x))

        med, mn = timeit(bwd_inplace, 5, warmup=1)
        res.append(report("logprob_entropy_bwd_inplace", bwd_bytes, med, mn, copy_gbps))
        del logits, x, dx

    if args.only in ("all", "small"):
        for B, R, tag in [(512, 1024, "headline"), (8192, 1024, "16x")]:
            rewards = torch.zeros(B, R, device=dev)
            rewards[:, -1] = (torch.rand(B, device=dev) > 0.5).float()
            values = torch.randn(B, R, device=dev)
            mask = torch.ones(B, R, dtype=torch.int64, device=dev)
            mask_u8 = torch.ones(B, R, dtype=torch.bool, device=dev)
            index = np.array([f"p{i // 8}" for i in range(B)], dtype=object)
            order, offsets, G, gmax = K.group_csr(index, dev)
            adv = torch.empty_like(rewards)

            def grpo(m=mask, code=L.VA_MASK_I64):
                L.call("va_outcome_advantage", K._p(rewards), K._p(m), code, B, R, K._p(order), K._p(offsets), G, gmax,
                       1e-6, L.VA_ADV_GRPO, K._p(adv), None, K._stream(rewards))

            med, mn = timeit(grpo, args.iters)
            res.append(report(f"grpo_adv_{tag}_i64mask", B * (4 * R + 8 * R + 4 * R + 4), med, mn, copy_gbps))
            med, mn = timeit(lambda: grpo(mask_u8, L.VA_MASK_U8), args.iters)
            res.append(report(f"grpo_adv_{tag}_u8mask", B * (4 * R + 1 * R + 4 * R + 4), med, mn, copy_gbps))
            ret = torch.empty_like(rewards)
            stats = torch.empty(4, device=dev)
            ws = torch.empty(L.load().va_gae_workspace_bytes(B) // 8 + 1, dtype=torch.float64, device=dev)

            def gae(m=mask, code=L.VA_MASK_I64):
                L.call("va_gae_advantage_return", K._p(rewards), K._p(values), K._p(m), code, B, R, 0.99, 0.95,
                       K._p(adv), K._p(ret), K._p(stats), K._p(ws), K._stream(rewards))

            med, mn = timeit(gae, args.iters)
            res.append(report(f"gae_whiten_{tag}_i64mask", B * R * (4 + 4 + 8 + 4 + 4 + 4 + 4), med, mn, copy_gbps))
            med, mn = timeit(lambda: gae(mask_u8, L.VA_MASK_U8), args.iters)
            res.append(report(f"gae_whiten_{tag}_u8mask", B * R * (4 + 4 + 1 + 4 + 4 + 4 + 4), med, mn, copy_gbps))
            for variant, vname in ((1, "reg"), (2, "lds")):  # A/B of the scan kernels (VA_TUNE_GAE_VARIANT)
                L.call("va_set_tuning", L.VA_TUNE_GAE_VARIANT, variant)
                med, mn = timeit(gae, args.iters)
                res.append(report(f"gae_whiten_{tag}_i64mask_{vname}", B * R * (4 + 4 + 8 + 4 + 4 + 4 + 4), med, mn,
                                  copy_gbps))
            L.call("va_set_tuning", L.VA_TUNE_GAE_VARIANT, 0)
            old = -torch.rand(B, R, device=dev)
            new = old + 0.05 * torch.randn(B, R, device=dev)
            refl = old + 0.1 * torch.randn(B, R, device=dev)
            newr = new.clone().requires_grad_(True)

            def loss_fb():
                out = K.fused_policy_loss(old, newr, rewards, mask, 0.2, 0.2, 3.0, "token-mean", ref_log_prob=refl,
                                          kl_loss_type="low_var_kl")
                (out[0] + 0.001 * out[4]).backward()

            med, mn = timeit(loss_fb, args.iters)
            res.append(report(f"ppo_loss_fwd_bwd_{tag}", B * R * (4 * 4 + 8 + 4) + B * R * (4 * 4 + 8 + 4), med, mn,
                              copy_gbps))
        for B, R in [(8, 1024)]:
            old = -torch.rand(B, R, device=dev)
            new = (old + 0.05 * torch.randn(B, R, device=dev)).requires_grad_(True)
            advs = torch.randn(B, R, device=dev)
            m = torch.ones(B, R, dtype=torch.int64, device=dev)

            def mb():
                out = K.fused_policy_loss(old, new, advs, m, 0.2, 0.2, 3.0, "token-mean", ref_log_prob=old,
                                          kl_loss_type="low_var_kl")
                out[0].backward()

            med, mn = timeit(mb, args.iters)
            res.append(report("ppo_loss_fwd_bwd_microbatch_8x1024", B * R * 48, med, mn, copy_gbps))


if __name__ == "__main__":
    main()
