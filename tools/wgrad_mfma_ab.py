"""va_weight_grad's two MFMA forms (VA_TUNE_WGRAD_MFMA = 32: 4 x 2 32x32x16 blocks per wave, 16: 8 x 4
16x16x32 blocks) at the bench's backbone shapes (dW = dY^T X, K = 151,552 packed tokens), interleaved
reps, HIP-event means over 10 launches; one JSON line per shape plus the per-step total (x 96 = 4
micro-batches x 24 layers).

  python tools/wgrad_mfma_ab.py [--tokens 151552] [--reps 3]
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
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    T = args.tokens
    shapes = {"qkv": (1152, 896), "o": (896, 896), "gate_up": (9728, 896), "down": (896, 4864)}
    g = torch.Generator(device="cuda").manual_seed(0)
    total = {16: 0.0, 32: 0.0}
    for name, (M, N) in shapes.items():
        dy = torch.randn(T, M, device="cuda", generator=g).to(torch.bfloat16)
        x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
        res = {16: [], 32: []}
        outs = {}
        for _ in range(args.reps):
            for mf in (32, 16):
                L.call("va_set_tuning", L.VA_TUNE_WGRAD_MFMA, mf)
                K.weight_grad(dy, x)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    outs[mf] = K.weight_grad(dy, x)
                e1.record()
                torch.cuda.synchronize()
                res[mf].append(round(e0.elapsed_time(e1) / 10 * 1e3, 1))
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_MFMA, 32)
        med = {mf: sorted(v)[len(v) // 2] for mf, v in res.items()}
        for mf in med:
            total[mf] += med[mf]
        rel = ((outs[16].float() - outs[32].float()).norm() / outs[32].float().norm()).item()
        tf = 2.0 * T * M * N / 1e12
        print(json.dumps({"shape": name, "M": M, "N": N, "K": T, "us_32x32x16": res[32], "us_16x16x32": res[16],
                          "median_us": med, "pflops": {mf: round(tf / med[mf] * 1e3, 3) for mf in med},
                          "rel_l2_16_vs_32": rel}), flush=True)
    print(json.dumps({"per_layer_us": {mf: round(v, 1) for mf, v in total.items()},
                      "per_step_ms_x96": {mf: round(v * 96 / 1e3, 1) for mf, v in total.items()}}), flush=True)


if __name__ == "__main__":
    main()
