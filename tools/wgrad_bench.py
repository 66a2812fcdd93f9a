"""Weight-gradient GEMM variants for the actor's linear shapes (dW = dY^T X, K = tokens):
plain bf16 mm, fp32-output mm / addmm (accumulate straight into an fp32 gradient), and split-K
over S token slices as one batched GEMM with fp32 output summed in fp32. One JSON line each.

  python tools/wgrad_bench.py [T]
"""
import json
import sys

import torch


def timeit(fn, iters=20, warm=3):
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


dev = "cuda"
T = int(sys.argv[1]) if len(sys.argv) > 1 else 77824
for name, (n_out, n_in) in {"qkv": (1152, 896), "o": (896, 896), "gateup": (9728, 896), "down": (896, 4864)}.items():
    x = torch.randn(T, n_in, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(T, n_out, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * T * n_out * n_in
    r = {"case": name, "T": T, "bf16_mm_us": round(timeit(lambda: dy.t() @ x), 1)}
    acc = torch.zeros(n_out, n_in, device=dev, dtype=torch.float32)
    try:
        r["fp32out_mm_us"] = round(timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)), 1)
        r["fp32out_addmm_us"] = round(timeit(lambda: torch.addmm(acc, dy.t(), x, out_dtype=torch.float32)), 1)
    except Exception as ex:  # noqa: BLE001
        r["fp32out_error"] = str(ex)[:160]
    for S in (2, 4, 8, 16):
        if T % S:
            continue
        dys = dy.view(S, T // S, n_out).transpose(1, 2)
        xs = x.view(S, T // S, n_in)
        r[f"splitk{S}_bmm_us"] = round(timeit(lambda: torch.bmm(dys, xs, out_dtype=torch.float32).sum(0)), 1)
        r[f"splitk{S}_gemm_only_us"] = round(timeit(lambda: torch.bmm(dys, xs, out_dtype=torch.float32)), 1)
    best = min((v, k) for k, v in r.items() if k.endswith("_us") and "gemm_only" not in k)
    r["best"] = best[1]
    r["best_tflops"] = round(fl / best[0] / 1e6, 1)
    print(json.dumps(r), flush=True)
