"""The backbone GEMMs whose output is H = 896 wide (3.5 tiles of 256) at the bench's packed token
count, through the product's path (K.linear / K.input_grad with the TunableOp table), against the
896-in / wide-out GEMMs of the same layer for reference. HIP-event medians; one JSON line per GEMM.

  python tools/gemm_n896_bench.py [--tokens 153600]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=10):
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
    args = ap.parse_args()
    from verl_amd import kernels as K
    from verl_amd.utils import gemm_tuning

    gemm_tuning.use_tuned_gemms("default")
    dev = torch.device("cuda", 0)
    T = args.tokens
    g = torch.Generator(device=dev).manual_seed(2)
    cases = {  # name: (activation width K, weight [N_out, K]) for Y = X W^T
        "o_fwd": (896, 896), "down_fwd": (4864, 896), "qkv_fwd": (896, 1152), "gateup_fwd": (896, 9728),
    }
    for name, (k, n) in cases.items():
        x = torch.randn(T, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ms = timed(lambda: K.linear(x, w))
        print(json.dumps({"gemm": name, "T": T, "K": k, "N": n, "ms": round(ms, 4),
                          "pflops": round(2.0 * T * k * n / ms / 1e12, 3)}), flush=True)
        del x, w
    # input gradients dX = dY W (output width = the layer's input width)
    for name, (n_out, n_in) in {"o_dgrad": (896, 896), "qkv_dgrad": (1152, 896), "gateup_dgrad": (9728, 896),
                                "down_dgrad": (896, 4864)}.items():
        dy = torch.randn(T, n_out, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n_out, n_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ms = timed(lambda: K.input_grad(dy, w))
        print(json.dumps({"gemm": name, "T": T, "K": n_out, "N": n_in, "ms": round(ms, 4),
                          "pflops": round(2.0 * T * n_in * n_out / ms / 1e12, 3)}), flush=True)
        del dy, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
