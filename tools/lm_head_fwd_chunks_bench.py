"""lm_head forward at the bench's 131,072-row micro-batch: one GEMM vs the same logits produced as
2 / 4 / 8 row chunks into one [N, V] buffer (bitwise equality reported). One JSON line; the committed GEMM
table is loaded as the actor does.

  python tools/lm_head_fwd_chunks_bench.py [ROWS]
"""
import json
import sys

import os
import sys as _sys

import torch

_sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    from verl_amd.utils.gemm_tuning import use_tuned_gemms

    use_tuned_gemms("default")
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    V, H = 151936, 896
    g = torch.Generator(device="cuda").manual_seed(0)
    h = torch.randn(N, H, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(V, H, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    out = torch.empty(N, V, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * N * V * H
    ref = torch.nn.functional.linear(h, w)
    res = {"rows": N}
    res["one_us"] = timeit(lambda: torch.nn.functional.linear(h, w))
    for k in (2, 4, 8):
        r = N // k

        def rows():
            for i in range(k):
                torch.mm(h[i * r:(i + 1) * r], w.t(), out=out[i * r:(i + 1) * r])
        res[f"rows{k}_us"] = timeit(rows)
        res[f"rows{k}_bitwise"] = bool(torch.equal(out, ref))
        res[f"rows{k}_maxdiff_first1024rows"] = float((out[:1024].float() - ref[:1024].float()).abs().max())
    for k, v in list(res.items()):
        if isinstance(v, float) and k.endswith("_us"):
            res[k.replace("_us", "_tf")] = round(fl / (v * 1e-6) / 1e12, 1)
            res[k] = round(v, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
