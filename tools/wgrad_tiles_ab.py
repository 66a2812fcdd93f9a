"""va_weight_grad's tile planners, interleaved on one GPU (VA_TUNE_WGRAD_TILES = 0: 256 x 256 tiles
in the 32x32x16 form with the round-4 slice rule; 1: the cost-model planner's 896-dividing tiles,
16x16x32; 2: the same with the cross-step fragment pipeline; 3: the pipeline with its LDS-DMA spread
between the MFMAs; 4: the fragment reads in the MFMAs' scheduling region too) at the bench's backbone shapes (dW =
dY^T X, K = 151,552 packed tokens) and the lm_head's (V = 151,936 x H = 896, K = 131,072 rows; also
hipBLASLt's swapped product + transpose, the previous default). HIP-event medians of `--reps`
interleaved rounds of `--iters` launches; one JSON line per shape, then the per-step totals (x 96
backbone launches of each shape = 4 update micro-batches x 24 layers; x 4 lm_head launches).

  python tools/wgrad_tiles_ab.py [--tokens 151552] [--rows 131072] [--reps 3] [--iters 10] [--modes 0,1,2]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=151552)
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--modes", default="0,3,4")
    ap.add_argument("--no-lm-head", action="store_true")
    ap.add_argument("--shapes", default="",
                    help="instead of the bench's shapes: name=MxNxK,... (e.g. gate_up7b=37888x3584x16384); adds "
                         "hipBLASLt's dY^T @ X as an arm")
    ap.add_argument("--kind-sweep", action="store_true",
                    help="per shape: every tile kind forced (VA_TUNE_WGRAD_KIND, the model's slices for it) vs auto")
    ap.add_argument("--lm-head-plans", default="",
                    help="also time the lm_head at these kind/splits plans, e.g. 3/1,3/2,3/3,5/2 (VA_TUNE_WGRAD_KIND)")
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    modes = [int(m) for m in args.modes.split(",")]
    shapes = {"qkv": (1152, 896, args.tokens), "o": (896, 896, args.tokens), "gate_up": (9728, 896, args.tokens),
              "down": (896, 4864, args.tokens)}
    if not args.no_lm_head:
        shapes["lm_head"] = (151936, 896, args.rows)
    custom = bool(args.shapes)
    if custom:
        shapes = {}
        for item in args.shapes.split(","):
            name, dims = item.split("=")
            shapes[name] = tuple(int(v) for v in dims.split("x"))
    g = torch.Generator(device="cuda").manual_seed(0)
    totals = {}

    def own(dy, x):
        M, N, T = dy.shape[1], x.shape[1], dy.shape[0]
        o = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        nb = L.load().va_weight_grad_workspace_bytes(T, M, N, 0)
        ws = torch.empty(max(nb // 4, 1), dtype=torch.float32, device="cuda")
        L.call("va_weight_grad", K._p(dy), dy.stride(0), K._p(x), x.stride(0), T, M, N, 0, K._p(ws), nb, K._p(o),
               K._stream(dy))
        return o

    def hipblaslt(dy, x):
        if dy.shape[1] >= K.WGRAD_SWAP_MIN_OUT:
            return K.transpose16(x.t() @ dy)
        return dy.t() @ x

    for name, (M, N, T) in shapes.items():
        scale = 1e-3 if name == "lm_head" else 0.1
        dy = (torch.randn(T, M, device="cuda", generator=g) * scale).to(torch.bfloat16)
        x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
        arms = [(f"tiles{m}", m) for m in modes] + ([("hipblaslt", None)] if name == "lm_head" or custom else [])
        res = {a: [] for a, _ in arms}
        outs = {}
        iters = max(2, args.iters // 4) if name == "lm_head" else args.iters
        for _ in range(args.reps):
            for arm, mode in arms:
                if mode is not None:
                    L.call("va_set_tuning", L.VA_TUNE_WGRAD_TILES, mode)
                fn = hipblaslt if mode is None else own
                fn(dy, x)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    outs[arm] = fn(dy, x)
                e1.record()
                torch.cuda.synchronize()
                res[arm].append(round(e0.elapsed_time(e1) / iters * 1e3, 1))
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_TILES, 4)
        med = {a: sorted(v)[len(v) // 2] for a, v in res.items()}
        per_step = 4 if name == "lm_head" else 96
        for a, v in med.items():
            totals.setdefault(("lm_head " if name == "lm_head" else "backbone ") + a, 0.0)
            totals[("lm_head " if name == "lm_head" else "backbone ") + a] += v * per_step / 1e3
        base = outs[arms[0][0]].float()
        rel = {a: ((o.float() - base).norm() / base.norm()).item() for a, o in outs.items()}
        tf = 2.0 * T * M * N / 1e12
        print(json.dumps({"shape": name, "M": M, "N": N, "K": T, "plan": K.own_wgrad_plan(M, N, T), "us": res,
                          "median_us": med, "pflops": {a: round(tf / v * 1e3, 3) for a, v in med.items()},
                          "rel_l2_vs_first": rel}), flush=True)
    print(json.dumps({"per_step_ms": {k: round(v, 1) for k, v in totals.items()}}), flush=True)
    if args.kind_sweep:
        for name, (M, N, T) in shapes.items():
            dy = (torch.randn(T, M, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
            x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
            kinds = [-1, 0, 1, 2, 3, 4, 5, 6]
            res = {k: [] for k in kinds}
            iters = 2 if name == "lm_head" else args.iters
            for _ in range(args.reps):
                for kind in kinds:
                    L.call("va_set_tuning", L.VA_TUNE_WGRAD_KIND, kind)
                    own(dy, x)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(iters):
                        own(dy, x)
                    e1.record()
                    torch.cuda.synchronize()
                    res[kind].append(round(e0.elapsed_time(e1) / iters * 1e3, 1))
            L.call("va_set_tuning", L.VA_TUNE_WGRAD_KIND, -1)
            print(json.dumps({"kind_sweep": name, "M": M, "N": N, "K": T, "auto_plan": K.own_wgrad_plan(M, N, T),
                              "us": {str(k): v for k, v in res.items()},
                              "median_us": {str(k): sorted(v)[len(v) // 2] for k, v in res.items()}}), flush=True)
            del dy, x
    if args.lm_head_plans:
        M, N, T = 151936, 896, args.rows
        dy = (torch.randn(T, M, device="cuda", generator=g) * 1e-3).to(torch.bfloat16)
        x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)

        def own_at(splits):
            o = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            nb = L.load().va_weight_grad_workspace_bytes(T, M, N, splits)
            ws = torch.empty(max(nb // 4, 1), dtype=torch.float32, device="cuda")
            L.call("va_weight_grad", K._p(dy), dy.stride(0), K._p(x), x.stride(0), T, M, N, splits, K._p(ws), nb,
                   K._p(o), K._stream(dy))
            return o

        plans = [tuple(int(v) for v in pl.split("/")) for pl in args.lm_head_plans.split(",")]
        res = {f"{k}/{sp}": [] for k, sp in plans}
        for _ in range(args.reps):
            for kind, sp in plans:
                L.call("va_set_tuning", L.VA_TUNE_WGRAD_KIND, kind)
                own_at(sp)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    own_at(sp)
                e1.record()
                torch.cuda.synchronize()
                res[f"{kind}/{sp}"].append(round(e0.elapsed_time(e1) / 3, 3))
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_KIND, -1)
        print(json.dumps({"lm_head_plans_ms": res, "auto_plan": K.own_wgrad_plan(M, N, T)}), flush=True)


if __name__ == "__main__":
    main()
