"""Interleaved A/B of the SwiGLU kernels (streaming vs grid-stride, VA_TUNE_SWIGLU_STREAM) at the
bench's packed token count, HIP-event timed, with algorithmic bytes and GB/s per variant.

  python tools/elemwise_ab.py [T] [F]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from verl_amd import _lib as L  # noqa: E402
from verl_amd import kernels as K  # noqa: E402


def timeit(fn, iters=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    evs = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 151552
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 4864
    dev = "cuda"
    gu = (torch.randn(T, 2 * F, device=dev) * 2).to(torch.bfloat16)
    dy = torch.randn(T, F, device=dev).to(torch.bfloat16)
    y = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
    dgu = torch.empty_like(gu)
    st = K._stream(gu)

    def fwd():
        L.call("va_swiglu_fwd", K._p(gu), 2 * F, F, L.VA_BF16, T, F, K._p(y), st)

    def bwd():
        L.call("va_swiglu_bwd", K._p(dy), K._p(gu), 2 * F, F, L.VA_BF16, T, F, K._p(dgu), 2 * F, F, st)

    nbytes = {"fwd": T * F * 2 * 3, "bwd": T * F * 2 * 5}  # fwd: read g, u, write y; bwd: + dy, dg, du
    times = {(k, v): [] for k in ("fwd", "bwd") for v in (2, 4, 8, 0)}
    for _ in range(5):
        for v in (2, 4, 8, 0):
            L.call("va_set_tuning", L.VA_TUNE_SWIGLU_STREAM, v)
            times[("fwd", v)].append(timeit(fwd))
            times[("bwd", v)].append(timeit(bwd))
    L.call("va_set_tuning", L.VA_TUNE_SWIGLU_STREAM, -1)
    for (k, v), ts in times.items():
        med = float(np.median(ts))
        print(json.dumps(dict(kernel=f"swiglu_{k}_{f'stream_u{v}' if v else 'gridstride'}", T=T, F=F,
                              median_us=round(med * 1e3, 1), algo_bytes=nbytes[k],
                              gbps=round(nbytes[k] / (med * 1e-3) / 1e9, 1))), flush=True)


if __name__ == "__main__":
    main()
