"""Probe: the gate|up weight gradient dW [9728, 896] = dGU^T X at the bench's token count
(151,552) — the product path (kernels.weight_grad: the tuned plain GEMM) against split-K as one
batched fp32-output GEMM + sum for S = 2..8, with the committed tuned table loaded. One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ms(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / iters)
    return round(sorted(ts)[2], 3)


def main():
    from verl_amd import kernels as K
    from verl_amd.utils.gemm_tuning import use_tuned_gemms

    dev = "cuda"
    T, M, N = 151552, 9728, 896
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.randn(T, M, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(T, N, device=dev, generator=g).to(torch.bfloat16)
    rec = {"T": T, "M": M, "N": N, "tflop": round(2.0 * T * M * N / 1e12, 3)}
    rec["untuned_plain_ms"] = ms(lambda: dy.t() @ x)
    rec["tuned_table"] = use_tuned_gemms("default")
    rec["product_weight_grad_ms"] = ms(lambda: K.weight_grad(dy, x))
    rec["tuned_plain_ms"] = ms(lambda: dy.t() @ x)
    ref = (dy.t() @ x).float()
    for S in (2, 3, 4, 6, 8):
        h = T // S

        def split():
            part = torch.bmm(dy[: S * h].view(S, h, M).transpose(1, 2), x[: S * h].reshape(S, h, N),
                             out_dtype=torch.float32)
            return part.sum(0).to(torch.bfloat16)
        rec[f"split{S}_ms"] = ms(split)
        rec[f"split{S}_maxdiff"] = float((split().float() - ref).abs().max())
    for k in list(rec):
        if k.endswith("_ms"):
            rec[k.replace("_ms", "_tflops")] = round(rec["tflop"] / rec[k] * 1e3, 1)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
