"""va_linear_tn (csrc/gemm_tn.hip: 256-token x {192, 224, 256, 288}-feature tiles, persistent) against the
product's hipBLASLt path (F.linear with the TunableOp table) on the backbone's linears whose output width
is not a multiple of 256 at the bench's packed token count: the o / down / q|k|v forward projections and
the o / q|k|v / gate|up input gradients (dY against the transposed weight: same TN layout). Interleaved
rounds, HIP-event medians of `--iters` launches; relative L2 error of both against an fp32 product; one
JSON line per shape, then the per-step totals (x 24 layers x the passes each GEMM runs in: forwards in
the no-grad and the update passes, input gradients in the update pass; `--passes` update passes).

  python tools/linear_tn_ab.py [--tokens 151552] [--reps 3] [--iters 10] [--arms 0/0,224/0,288/0]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = [  # name, K, N, bias, runs per layer and update pass (forwards: no-grad + update)
    ("o_fwd", 896, 896, False, 2), ("qkv_fwd", 896, 1152, True, 2), ("down_fwd", 4864, 896, False, 2),
    ("o_dgrad", 896, 896, False, 1), ("qkv_dgrad", 1152, 896, False, 1), ("gateup_dgrad", 9728, 896, False, 1)]
# opt-in (--cases): the lm_head's input gradient dH = dlogits W over the transposed weight, 131,072 rows,
# once per update pass (runs counted per layer: 1 / 24)
EXTRA = {"lmhead_dgrad": (151936, 896, False, 1 / 24, 131072)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=151552)
    ap.add_argument("--passes", type=int, default=4, help="update passes per step")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--arms", default="0/0", help="own-kernel arms tile_n/per[/VA_TUNE_LINEAR_TN] (0 = automatic; "
                                                  "the setting default 1)")
    ap.add_argument("--cases", default="", help="subset of the case names, comma-separated")
    ap.add_argument("--no-ref", action="store_true", help="skip the fp32 reference (profiling runs)")
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K
    from verl_amd.utils import gemm_tuning

    gemm_tuning.use_tuned_gemms("default")
    dev = torch.device("cuda", 0)
    T = args.tokens
    g = torch.Generator(device=dev).manual_seed(4)
    own_arms = [tuple(int(v) for v in a.split("/")) for a in args.arms.split(",")]
    totals = {"hipblaslt": 0.0, "own_best": 0.0, "mixed_best": 0.0}
    cases = [c + (args.tokens,) for c in CASES] + [(nm, *v) for nm, v in EXTRA.items()]
    for name, k, n, has_bias, runs, T in cases:
        if (args.cases and name not in args.cases.split(",")) or (not args.cases and name in EXTRA):
            continue
        x = torch.randn(T, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * 0.03).to(torch.bfloat16)
        b = (torch.randn(n, device=dev, generator=g) * 0.1).to(torch.bfloat16) if has_bias else None
        ref = None if args.no_ref else torch.nn.functional.linear(x.float(), w.float(),
                                                                  b.float() if b is not None else None)
        outs = {}

        def blas():
            return torch.nn.functional.linear(x, w, b)

        def own_fn(tile, per, mode):
            def f():
                L.call("va_set_tuning", L.VA_TUNE_LINEAR_TN, mode)
                out = torch.empty(T, n, dtype=torch.bfloat16, device=dev)
                L.call("va_linear_tn", K._p(x), x.stride(0), K._p(w), w.stride(0), K._p(b) if b is not None else None,
                       L.VA_BF16, T, n, k, tile, per, K._p(out), out.stride(0), K._stream(x))
                return out
            return f

        arms = [("hipblaslt", blas)]
        for arm in own_arms:
            tile, per, mode = (*arm, 1) if len(arm) == 2 else arm
            t_eff = tile or L.load().va_linear_tn_tile(n)
            if t_eff and n % t_eff == 0:
                arms.append((f"own_{t_eff}_{per}_{mode}", own_fn(tile, per, mode)))
        res = {a: [] for a, _ in arms}
        for _ in range(args.reps):
            for arm, fn in arms:
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    outs[arm] = fn()
                e1.record()
                torch.cuda.synchronize()
                res[arm].append(round(e0.elapsed_time(e1) / args.iters * 1e3, 1))
        L.call("va_set_tuning", L.VA_TUNE_LINEAR_TN, 1)
        med = {a: sorted(v)[len(v) // 2] for a, v in res.items()}
        fl = 2.0 * T * k * n
        rel = {} if ref is None else {a: float((o.float() - ref).norm() / ref.norm()) for a, o in outs.items()}
        same = {a: bool(torch.equal(o, outs["hipblaslt"])) for a, o in outs.items() if a != "hipblaslt"}
        per_step = round(24 * args.passes * runs)
        totals["hipblaslt"] += med["hipblaslt"] * per_step / 1e3
        own_med = [v for a, v in med.items() if a != "hipblaslt"]
        if own_med:
            totals["own_best"] += min(own_med) * per_step / 1e3
            totals["mixed_best"] += min(min(own_med), med["hipblaslt"]) * per_step / 1e3
        print(json.dumps({"gemm": name, "M": T, "N": n, "K": k, "bias": has_bias, "us": res, "median_us": med,
                          "pflops": {a: round(fl / v / 1e9, 3) for a, v in med.items()}, "rel_l2_vs_fp32": rel,
                          "bitwise_equal_to_hipblaslt": same}), flush=True)
        del x, w, b, ref, outs
        torch.cuda.empty_cache()
    print(json.dumps({"per_step_ms": {a: round(v, 1) for a, v in totals.items()}, "tokens": T,
                      "update_passes": args.passes}), flush=True)


if __name__ == "__main__":
    main()
