"""Weight-gradient GEMM dW = dY^T X at the bench's token count, by operand layout: the natural one
(dY [T, n_out], X [T, n_in] row-major: K = T strided for both operands) against K-contiguous
transposed copies (dY^T [n_out, T], X^T [n_in, T]), plain and split-K, plus the cost of producing
a transposed copy. Decides whether writing transposed side outputs would pay.

  python tools/wgrad_layout_bench.py [T]
"""
import json
import sys

import torch


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
    for name, (n_out, n_in) in {"gateup": (9728, 896), "down": (896, 4864), "qkv": (1152, 896), "o": (896, 896)}.items():
        dy = torch.randn(T, n_out, device=dev, dtype=torch.bfloat16)
        x = torch.randn(T, n_in, device=dev, dtype=torch.bfloat16)
        dyt = dy.t().contiguous()
        xt = x.t().contiguous()
        fl = 2.0 * T * n_out * n_in
        r = {"case": name, "T": T}

        def rec(k, us):
            r[k + "_us"] = round(us, 1)
            r[k + "_tf"] = round(fl / us / 1e6, 1)

        rec("natural", timeit(lambda: dy.t() @ x))
        rec("kcontig", timeit(lambda: dyt @ xt.t()))
        rec("kcontig_fp32", timeit(lambda: torch.mm(dyt, xt.t(), out_dtype=torch.float32)))
        for S in (2, 4, 8):
            h = T // S
            a = dyt.view(n_out, S, h).permute(1, 0, 2)  # [S, n_out, h], K contiguous
            b = xt.view(n_in, S, h).permute(1, 2, 0)    # [S, h, n_in] as a transposed view
            rec(f"kcontig_splitk{S}", timeit(lambda: torch.bmm(a, b, out_dtype=torch.float32).sum(0)))
            an = dy.view(S, h, n_out).transpose(1, 2)
            bn = x.view(S, h, n_in)
            rec(f"natural_splitk{S}", timeit(lambda: torch.bmm(an, bn, out_dtype=torch.float32).sum(0)))
        r["transpose_dy_us"] = round(timeit(lambda: dy.t().contiguous()), 1)
        r["transpose_x_us"] = round(timeit(lambda: x.t().contiguous()), 1)
        print(json.dumps(r), flush=True)
        del dy, x, dyt, xt


if __name__ == "__main__":
    main()
