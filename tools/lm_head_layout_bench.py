"""lm_head backward GEMMs by dlogits layout at the bench's micro-batch: dlogits [N, V] (as the
log-prob backward writes it today) vs dlogits^T [V, N] (a transposed write), for the dgrad
dh = dlogits W and the wgrad dW = dlogits^T h (with h or a transposed copy h^T). JSON lines.

  python tools/lm_head_layout_bench.py [ROWS]
"""
import json
import sys

import torch


def timeit(fn, iters=5, warm=2):
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
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    V, H = 151936, 896
    dev = "cuda"
    fl = 2.0 * N * V * H
    dl = torch.randn(N, V, device=dev, dtype=torch.bfloat16)
    h = torch.randn(N, H, device=dev, dtype=torch.bfloat16)
    w = torch.randn(V, H, device=dev, dtype=torch.bfloat16)
    res = {}
    res["dgrad_rowmajor"] = timeit(lambda: dl @ w)
    res["wgrad_rowmajor"] = timeit(lambda: dl.t() @ h)
    dt = dl.t().contiguous()
    del dl
    ht = h.t().contiguous()
    res["dgrad_transposed"] = timeit(lambda: dt.t() @ w)
    res["wgrad_transposed_h"] = timeit(lambda: dt @ h)
    res["wgrad_transposed_hT"] = timeit(lambda: dt @ ht.t())
    res["transpose_h"] = timeit(lambda: h.t().contiguous())
    for k, us in res.items():
        print(json.dumps({"case": k, "rows": N, "us": round(us, 1),
                          "tflops": round(fl / us / 1e6, 1) if not k.startswith("transpose") else None}), flush=True)


if __name__ == "__main__":
    main()
