"""Why the update pass's lm_head forward GEMM runs slower in the bench step than standalone
(36.4 ms in the step vs 29.95 ms in tools/f1_ab.py).

The bench routes every GEMM through TunableOp with the committed solution table
(utils/gemm_tuning.py); the table holds the lm_head forward for 65,536 rows but not for the
131,072-row pass, and f1_ab.py never loads the table. This times the same product
(h [N, 896] @ W[151936, 896]^T, bf16) four ways, each after its own warm-up:
  plain      torch's default BLAS path (no TunableOp)           — what f1_ab.py measured
  tunable    TunableOp on, table loaded, lookup only            — what the bench step does
  linear     K.linear (the actor's call: F.linear in _MergedLinear) with the table
  linear_plain K.linear without TunableOp
Run under rocprofv3 --kernel-trace --stats to see which kernel each mode dispatches.
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=5):
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
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--modes", default="plain,linear_plain,tunable,linear")
    args = ap.parse_args()
    from verl_amd import kernels as K
    from verl_amd.utils import gemm_tuning

    dev = torch.device("cuda", 0)
    H, V, N = 896, 151936, args.rows
    g = torch.Generator(device=dev).manual_seed(1)
    w = (torch.randn(V, H, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    h = torch.randn(N, H, device=dev, generator=g).to(torch.bfloat16)
    out = {"rows": N}
    with torch.no_grad():
        for mode in args.modes.split(","):
            if mode in ("tunable", "linear"):
                gemm_tuning.use_tuned_gemms("default")
            else:
                torch.cuda.tunable.enable(False)
            if mode.startswith("linear"):
                fn = lambda: K.linear(h, w)  # noqa: E731
            else:
                fn = lambda: h @ w.t()  # noqa: E731
            out[f"{mode}_ms"] = round(timed(fn), 3)
            torch.cuda.tunable.enable(False)
            gemm_tuning._loaded = None
    out["table_has_shape"] = gemm_tuning.has_tuned("tn", V, N, H)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
