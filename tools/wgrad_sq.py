"""The backbone weight gradients (dW = dY^T X, K = tokens) at the bench's update micro-batch: the own
va_weight_grad kernel vs hipBLASLt's dY^T @ X on the same operands. One JSON line per shape (median
of 5 blocks of --iters launches each). Run under rocprofv3 --pmc (SQ / GRBM counters) with
--shape to get one shape's MFMA busy share and clock per kernel (tools/gpu_r04_l.sh).

  python tools/wgrad_sq.py [--tokens 153600] [--shape gateup] [--iters 5]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (1152, 896), "o": (896, 896), "gateup": (9728, 896), "down": (896, 4864)}


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=153600)
    ap.add_argument("--shape", default="")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tiles", type=int, default=None, help="VA_TUNE_WGRAD_TILES for the own kernel (0 / 1 / 2)")
    ap.add_argument("--lm-head", action="store_true", help="also the lm_head shape (151,936 x 896, K = 131,072)")
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    if args.tiles is not None:
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_TILES, args.tiles)
    if args.lm_head:
        SHAPES["lm_head"] = (151936, 896)

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    for name, (n_out, n_in) in SHAPES.items():
        if args.shape and name != args.shape:
            continue
        T = 131072 if name == "lm_head" else args.tokens
        x = torch.randn(T, n_in, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(T, n_out, device=dev, generator=g).to(torch.bfloat16)
        fl = 2.0 * T * n_out * n_in
        own = K.weight_grad(dy, x)
        rel = None
        if name != "lm_head":  # the lm_head's fp32 reference would take ~160 GB
            ref = (dy.t().float() @ x.float())
            rel = float((own.float() - ref).norm() / ref.norm())
            del ref
        ms_own = timed(lambda: K.weight_grad(dy, x), args.iters)
        ms_blas = timed(lambda: dy.t() @ x, args.iters)
        print(json.dumps({"shape": name, "tokens": T, "n_out": n_out, "n_in": n_in, "tiles": args.tiles,
                          "plan": K.own_wgrad_plan(n_out, n_in, T),
                          "own_ms": round(ms_own, 4), "own_pflops": round(fl / ms_own / 1e12, 3),
                          "hipblaslt_ms": round(ms_blas, 4), "hipblaslt_pflops": round(fl / ms_blas / 1e12, 3),
                          "own_rel_err_vs_fp32": rel}), flush=True)
        del x, dy, own
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
