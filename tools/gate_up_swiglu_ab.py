"""The no-grad MLP activation at the bench's packed micro-batch (151,552 tokens, Qwen2.5-0.5B: H = 896,
F = 4,864): va_gate_up_swiglu (one kernel, no [T, 2F] projection) at several feature-range splits vs
the product's unfused path (merged gate|up GEMM through the TunableOp table + the streaming SwiGLU).
Interleaved reps, HIP-event medians; one JSON line.

  python tools/gate_up_swiglu_ab.py [--tokens 151552] [--splits auto,2,7,19,38] [--reps 3] [--defer]

--defer: the default split of the no-grad kernel and of the training kernel that also writes the
projection (va_gate_up_swiglu_save), each with VA_TUNE_T256_DEFER 0 and 1, against the unfused paths.
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=151552)
    ap.add_argument("--splits", default="auto,2,7,19,38")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--defer", action="store_true")
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K
    from verl_amd.utils.gemm_tuning import use_tuned_gemms

    tuned = use_tuned_gemms("default")
    T, H, F = args.tokens, 896, 4864
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(T, H, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(2 * F, H, device="cuda", generator=g) * 0.03).to(torch.bfloat16)
    arms = {"unfused_gemm_plus_swiglu": lambda: K.swiglu_merged(x @ w.t()),
            "unfused_gemm_only": lambda: x @ w.t()}
    if args.defer:
        def with_defer(d, fn):
            def run():
                L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, d)
                try:
                    return fn()
                finally:
                    L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, 1)  # the default
            return run
        split = K._gate_up_swiglu_splits(T, F // 128)
        arms["unfused_gemm_plus_swiglu_keep_proj"] = lambda: (lambda gu: (K.swiglu_merged(gu), gu))(x @ w.t())
        for d in (0, 1):
            arms[f"fused_defer{d}"] = with_defer(d, lambda: K._gate_up_swiglu_raw(x, w, split, False))
            arms[f"fused_save_defer{d}"] = with_defer(d, lambda: K._gate_up_swiglu_raw(x, w, split, True))
    else:
        for s in args.splits.split(","):
            arms[f"fused_splits_{s}"] = (lambda s=s: K.gate_up_swiglu(x, w, splits=None if s == "auto" else int(s)))
    res = {k: [] for k in arms}
    with torch.no_grad():
        for _ in range(args.reps):
            for k, fn in arms.items():
                res[k].append(round(timed(fn), 4))
        ref = K.swiglu_merged(x @ w.t()).float()
        got = K.gate_up_swiglu(x, w).float()
        if args.defer:  # the two epilogue placements: the same bits
            L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, 0)
            y0, g0 = K._gate_up_swiglu_raw(x, w, K._gate_up_swiglu_splits(T, F // 128), True)
            L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, 1)
            y1, g1 = K._gate_up_swiglu_raw(x, w, K._gate_up_swiglu_splits(T, F // 128), True)
            assert torch.equal(y0, y1) and torch.equal(g0, g1)
    err = ((got - ref).norm() / ref.norm()).item()
    tf = 2.0 * T * H * 2 * F / 1e12
    out = {"tokens": T, "H": H, "F": F, "tuned_table": tuned, "auto_splits": K._gate_up_swiglu_splits(T, F // 128),
           "ms": res, "median_ms": {k: sorted(v)[len(v) // 2] for k, v in res.items()},
           "fused_vs_unfused_rel_l2": err, "gemm_tflop": tf}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
