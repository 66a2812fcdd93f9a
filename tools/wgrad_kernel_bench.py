"""Own weight-gradient kernel (wgrad.hip) vs hipBLASLt split-K at the bench's token count, per
actor linear shape and split count. One JSON line per (shape, variant).

  python tools/wgrad_kernel_bench.py [T]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from verl_amd import kernels as K  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 151552
    dev = "cuda"
    for name, (m, n) in {"gateup": (9728, 896), "down": (896, 4864), "qkv": (1152, 896), "o": (896, 896)}.items():
        dy = torch.randn(T, m, device=dev).to(torch.bfloat16)
        x = torch.randn(T, n, device=dev).to(torch.bfloat16)
        fl = 2.0 * T * m * n
        r = {"case": name, "T": T, "hipblaslt_current_us": round(timeit(lambda: K.weight_grad(dy, x)), 1)}
        for s in (1, 2, 4, 8, 16):
            r[f"own_s{s}_us"] = round(timeit(lambda: K.wgrad_gemm(dy, x, s)), 1)
        best = min((v, k) for k, v in r.items() if k.startswith("own"))
        r["own_best"] = best[1]
        r["own_best_tf"] = round(fl / best[0] / 1e6, 1)
        r["hipblaslt_tf"] = round(fl / r["hipblaslt_current_us"] / 1e6, 1)
        print(json.dumps(r), flush=True)
        del dy, x


if __name__ == "__main__":
    main()
