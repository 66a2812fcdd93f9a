"""Fused lm_head + log-prob (linear_logprob.hip) vs the unfused path (hipBLASLt GEMM -> bf16
logits -> streaming log-prob kernel) at the actor's shapes. One JSON line per case."""
import json

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from verl_amd import kernels as K


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


from verl_amd import _lib as L  # noqa: E402

torch.manual_seed(0)
H, V = 896, 151936
w = (torch.randn(V, H, device="cuda") * 0.05).to(torch.bfloat16)
TILES = [int(t) for t in sys.argv[1:]] or [256, 128]
for N, tile in [(n, t) for n in (8192, 16384, 65536) for t in TILES]:
    L.call("va_set_tuning", L.VA_TUNE_LINEAR_LOGPROB_TILE, tile)
    h = torch.randn(N, H, device="cuda").to(torch.bfloat16)
    lab = torch.randint(0, V, (N,), device="cuda")
    fl = 2.0 * N * V * H
    with torch.no_grad():
        t_f = timeit(lambda: K.linear_logprob_entropy(h, w, lab, 1.0))
        t_g = timeit(lambda: h @ w.t())
        t_u = timeit(lambda: K.logprob_entropy(h @ w.t(), lab, 1.0))
    print(json.dumps({"N": N, "tile": tile, "fused_us": round(t_f, 1), "fused_tflops": round(fl / t_f / 1e6, 1),
                      "gemm_only_us": round(t_g, 1), "gemm_tflops": round(fl / t_g / 1e6, 1),
                      "unfused_us": round(t_u, 1), "speedup_vs_unfused": round(t_u / t_f, 3)}), flush=True)
