"""add+RMSNorm backward (va_rmsnorm_bwd with a residual gradient) at the bench's packed token count:
HIP-event median and algorithmic GB/s (reads dy, h, dres, writes dx: 4 x T x H bf16).

  python tools/rmsnorm_bwd_bench.py [T] [H]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from verl_amd import _lib as L  # noqa: E402
from verl_amd import kernels as K  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 151552
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 896
    dev = "cuda"
    dy, h, dres = (torch.randn(T, H, device=dev).to(torch.bfloat16) for _ in range(3))
    w = (1 + 0.1 * torch.randn(H, device=dev)).to(torch.bfloat16)
    rstd = torch.rand(T, device=dev) + 0.5
    dx = torch.empty_like(dy)
    dw = torch.empty(H, device=dev, dtype=torch.bfloat16)
    ws = torch.empty(L.load().va_rmsnorm_workspace_bytes(T, H) // 4, device=dev)

    def run():
        L.call("va_rmsnorm_bwd", K._p(dy), K._p(h), K._p(w), K._p(rstd), K._p(dres), L.VA_BF16, T, H, K._p(dx),
               K._p(dw), K._p(ws), K._stream(dy))

    ts = []
    for _ in range(5):
        run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            run()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 20 * 1e3)
    med = float(np.median(ts))
    print(json.dumps({"kernel": "rmsnorm_bwd_with_residual", "T": T, "H": H, "median_us": round(med, 1),
                      "gbps": round(4 * T * H * 2 / (med * 1e-6) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
