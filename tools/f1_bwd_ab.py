"""Fused lm_head backward (va_linear_logprob_bwd) vs the composition it replaces, at the bench's
131,072-row update pass (Qwen2.5-0.5B head: H = 896, V = 151,936). Prints one JSON line:

  * kernel level: the fused dlogits kernel (recompute + dlogits, bf16 [N, V] out) vs hipBLASLt's
    logits recompute + the streaming va_logprob_entropy_bwd in place;
  * pass level: the whole fused path (f1 forward + fused backward incl. the two lm_head GEMMs, per
    vocab range of --vocab-splits columns: the reference's _Split_Dlogits_N loop) vs the unfused
    update pass (hipBLASLt logits + logprob_entropy fwd + bwd + the two GEMMs), with the peak HBM
    of each.

  python tools/f1_bwd_ab.py [--rows 131072] [--iters 3] [--vocab-splits 9504,37984,151936]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2], ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--vocab-splits", default="9504", help="comma-separated vocab range widths of the fused pass")
    ap.add_argument("--skip-kernel", action="store_true", help="pass level only")
    ap.add_argument("--breakdown", action="store_true",
                    help="also time each component of both passes (HIP events between the launches)")
    ap.add_argument("--tune", action="append", default=[], help="KEY=VALUE for va_set_tuning (A/B runs)")
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    for kv in args.tune:
        key, val = (int(x) for x in kv.split("="))
        L.call("va_set_tuning", key, val)

    dev = torch.device("cuda", 0)
    H, V, N = 896, 151936, args.rows
    g = torch.Generator(device=dev).manual_seed(1)
    w = (torch.randn(V, H, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    h = torch.randn(N, H, device=dev, generator=g).to(torch.bfloat16)
    lab = torch.randint(0, V, (N,), device=dev, generator=g)
    g1 = torch.randn(N, device=dev, generator=g)
    out = {"rows": N, "H": H, "V": V, "tune": args.tune}
    with torch.no_grad():
        _, ent, lse = torch.ops.verl_amd.logprob_entropy_fwd(h @ w.t(), lab, 1.0, 0)
    flops = 2.0 * N * V * H

    # ---- kernel level
    if args.skip_kernel:
        return pass_level(args, K, h, w, lab, g1, out)
    dlog = torch.empty(N, V, dtype=torch.bfloat16, device=dev)
    ms, ts = timed(lambda: K._linear_logprob_bwd_raw(h, w, lab, lse, ent, g1, None, 1.0, False, dlog), args.iters)
    out["fused_dlogits_ms"] = round(ms, 3)
    out["fused_dlogits_tflops"] = round(flops / ms / 1e9, 1)
    logits = dlog  # reuse the buffer for the composition

    def compose():
        torch.matmul(h, w.t(), out=logits)
        torch.ops.verl_amd.logprob_entropy_bwd_(g1, None, logits, lab, lse, ent, 1.0)

    ms_c, _ = timed(compose, args.iters)
    out["compose_gemm_plus_stream_bwd_ms"] = round(ms_c, 3)
    del dlog, logits
    torch.cuda.empty_cache()
    pass_level(args, K, h, w, lab, g1, out)


def pass_level(args, K, h, w, lab, g1, out):
    """forward + backward of the lm_head + log-prob, with GEMMs"""

    def fused_pass():
        ha, wa = h.detach().requires_grad_(True), w.detach().requires_grad_(True)
        lp, _ = K.linear_logprob_entropy(ha, wa, lab, 1.0)
        (lp * g1).sum().backward()

    def unfused_pass():
        ha, wa = h.detach().requires_grad_(True), w.detach().requires_grad_(True)
        lp, _ = K.logprob_entropy(K.linear(ha, wa), lab, 1.0, inplace_backward="auto")
        (lp * g1).sum().backward()

    if args.breakdown:
        out.update(breakdown(K, h, w, lab, g1))
    runs = [(f"fused_pass_split{int(s)}", fused_pass, int(s)) for s in args.vocab_splits.split(",")]
    for name, fn, split in runs + [("unfused_pass", unfused_pass, None)]:
        if split is not None:
            K._LinearLogprob.VOCAB_PER_SPLIT = split
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        ms_p, _ = timed(fn, args.iters)
        out[f"{name}_ms"] = round(ms_p, 3)
        out[f"{name}_peak_extra_gb"] = round((torch.cuda.max_memory_allocated() - base) / 1e9, 2)
    print(json.dumps(out), flush=True)


def breakdown(K, h, w, lab, g1, reps: int = 3):
    """Per-component device time (ms, median of ``reps``) of one lm_head forward + backward: the fused
    path's forward, per vocab range backward kernel, fp32 d_hidden addmm and weight gradient (summed
    over the 16 ranges of 9,504 columns), and the unfused path's logits GEMM, streaming log-prob
    forward / backward, d_hidden GEMM and weight gradient — what VERDICT r5 #5 asks to split."""
    N, H = h.shape
    V = w.shape[0]
    width = K._LinearLogprob.VOCAB_PER_SPLIT

    def run_fused(ev):
        with torch.no_grad():
            ev("fwd")
            lp, ent, lse = K._linear_logprob_fwd_raw(h, w, lab, 1.0, False, None)
            ev("fwd")
            buf = torch.empty(N, width, dtype=h.dtype, device=h.device)
            wt = K.transpose16(w)
            dh32 = torch.zeros(N, H, dtype=torch.float32, device=h.device)
            dw = torch.empty_like(w)
            for v0 in range(0, V, width):
                v1 = min(V, v0 + width)
                dl = buf[:, : v1 - v0]
                ev("bwd_kernel")
                K._linear_logprob_bwd_raw(h, w, lab, lse, ent, g1, None, 1.0, False, dl, v0, v1)
                ev("bwd_kernel")
                ev("dh_addmm")
                torch.addmm(dh32, dl, wt[:, v0:v1].t(), out_dtype=torch.float32, out=dh32)
                ev("dh_addmm")
                ev("dw")
                dw[v0:v1].copy_(K.weight_grad(dl, h))
                ev("dw")

    def run_unfused(ev):
        with torch.no_grad():
            ev("logits_gemm")
            logits = K.linear(h, w)
            ev("logits_gemm")
            ev("logprob_fwd")
            lp, ent, lse = torch.ops.verl_amd.logprob_entropy_fwd(logits, lab, 1.0, 0)
            ev("logprob_fwd")
            ev("logprob_bwd")
            dl = torch.ops.verl_amd.logprob_entropy_bwd(g1, None, logits, lab, lse, ent, 1.0)
            ev("logprob_bwd")
            del logits
            ev("dh_gemm")
            K.input_grad(dl, w)
            ev("dh_gemm")
            ev("dw")
            K.weight_grad(dl, h)
            ev("dw")

    res = {}
    for name, fn in (("fused", run_fused), ("unfused", run_unfused)):
        per = {}
        for _ in range(reps + 1):
            marks = []

            def ev(tag):
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                marks.append((tag, e))

            fn(ev)
            torch.cuda.synchronize()
            acc = {}
            for (tag, e0), (_, e1) in zip(marks[0::2], marks[1::2], strict=True):
                acc[tag] = acc.get(tag, 0.0) + e0.elapsed_time(e1)
            for tag, v in acc.items():
                per.setdefault(tag, []).append(v)
        torch.cuda.empty_cache()  # between the paths only: inside, the first rep warms the allocator
        res[f"breakdown_{name}_ms"] = {t: round(sorted(v[1:])[len(v[1:]) // 2], 3) for t, v in per.items()}
        res[f"breakdown_{name}_total_ms"] = round(sum(res[f"breakdown_{name}_ms"].values()), 3)
    return res


if __name__ == "__main__":
    main()
