"""lm_head weight-gradient variants at the bench's micro-batch (dW = dlogits^T h, M = vocab,
N = hidden, K = response rows): autograd's plain bf16 mm, the transposed product, fp32 output,
vocab-chunked GEMMs and split-K. One JSON line each (HIP-event timing, random bf16 data).

  python tools/lm_head_wgrad_bench.py [ROWS] [VOCAB] [HIDDEN]
"""
import json
import sys

import torch


def timeit(fn, iters=6, warm=2):
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
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    V = int(sys.argv[2]) if len(sys.argv) > 2 else 151936
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 896
    dev = "cuda"
    dy = torch.randn(T, V, device=dev, dtype=torch.bfloat16)
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * T * V * H
    want = (dy.t() @ x).float()

    def rep(name, fn, check=True):
        us = timeit(fn)
        r = {"case": name, "T": T, "V": V, "H": H, "us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}
        if check:
            got = fn().float()
            r["max_rel_err"] = float(((got - want).abs().max() / want.abs().max()).item())
        print(json.dumps(r), flush=True)

    rep("plain_bf16_dyT_x", lambda: dy.t() @ x)
    rep("transposed_xT_dy", lambda: (x.t() @ dy).t(), check=True)
    rep("transposed_xT_dy_contig", lambda: (x.t() @ dy).t().contiguous())
    rep("fp32out_dyT_x", lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    rep("fp32out_xT_dy", lambda: torch.mm(x.t(), dy, out_dtype=torch.float32).t())
    for c in (16384, 38016, 75968):
        def chunked(c=c):
            out = torch.empty(V, H, device=dev, dtype=torch.bfloat16)
            for v0 in range(0, V, c):
                torch.mm(dy[:, v0:v0 + c].t(), x, out=out[v0:v0 + c])
            return out
        rep(f"vocab_chunks_{c}", chunked)
    for S in (2, 4):
        h = T // S

        def splitk(S=S, h=h):
            return torch.bmm(dy.view(S, h, V).transpose(1, 2), x.view(S, h, H), out_dtype=torch.float32).sum(0)
        rep(f"splitk{S}_fp32", splitk)


if __name__ == "__main__":
    main()
