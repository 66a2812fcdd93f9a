"""The lm_head weight gradient (dW = dlogits^T h: V = 151,936 outputs x H = 896, K = 131,072 update-pass
rows) on the own K-outer kernel (va_weight_grad, 256 x 256 tiles, with and without the 128-wide
remainder tiles for 896 = 3.5 x 256) against the product's hipBLASLt path (kernels.weight_grad:
swapped product + transpose). HIP-event medians; one JSON line.

  python tools/lm_head_wgrad_own.py [--rows 131072] [--iters 3]
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
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    dev = torch.device("cuda", 0)
    T, V, H = args.rows, 151936, 896
    g = torch.Generator(device=dev).manual_seed(5)
    dy = (torch.randn(T, V, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    x = torch.randn(T, H, device=dev, generator=g).to(torch.bfloat16)
    fl = 2.0 * T * V * H
    out = {"rows": T, "V": V, "H": H}
    ref = K.weight_grad(dy, x)
    out["hipblaslt_ms"] = round(timed(lambda: K.weight_grad(dy, x), args.iters), 3)

    def own():
        o = torch.empty(V, H, dtype=torch.bfloat16, device=dev)
        nb = L.load().va_weight_grad_workspace_bytes(T, V, H, 0)
        ws = torch.empty(max(nb // 4, 1), dtype=torch.float32, device=dev) if nb else None
        L.call("va_weight_grad", K._p(dy), dy.stride(0), K._p(x), x.stride(0), T, V, H, 0, K._p(ws), nb, K._p(o),
               K._stream(dy))
        return o

    for rem in (0, 1):
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_REMAINDER, rem)
        o = own()
        out[f"own_rem{rem}_ms"] = round(timed(own, args.iters), 3)
        out[f"own_rem{rem}_pflops"] = round(fl / out[f"own_rem{rem}_ms"] / 1e12, 3)
        out[f"own_rem{rem}_rel_vs_hipblaslt"] = float((o.float() - ref.float()).norm() / ref.float().norm())
        out[f"own_rem{rem}_workspace_mb"] = L.load().va_weight_grad_workspace_bytes(T, V, H, 0) >> 20
    L.call("va_set_tuning", L.VA_TUNE_WGRAD_REMAINDER, 0)
    out["hipblaslt_pflops"] = round(fl / out["hipblaslt_ms"] / 1e12, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
