"""va_linear_tn (the f1 sweep as a plain TN GEMM) against the product's hipBLASLt path with the
TunableOp table, on the backbone's short-K linears at the bench's packed token count: the q|k|v and o
projections (forward, with / without bias) and their input gradients (dY against the transposed
weight). Relative error of both against an fp32 product; HIP-event medians; one JSON line each.

  python tools/linear_tn_ab.py [--tokens 153600] [--per 0]

The probe kernel (va_linear_tn: t256_sweep with a bf16 store epilogue, ABI 6) was measured with this
script (profiles/r04/linear_tn_ab.jsonl) and not kept, so at HEAD the script stops at its first call;
it records the method.
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=153600)
    ap.add_argument("--per", type=int, action="append", default=None, help="tiles per workgroup (0 = auto)")
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K
    from verl_amd.utils import gemm_tuning

    gemm_tuning.use_tuned_gemms("default")
    dev = torch.device("cuda", 0)
    T = args.tokens
    g = torch.Generator(device=dev).manual_seed(4)
    cases = [("o_fwd", 896, 896, False), ("qkv_fwd", 896, 1152, True), ("o_dgrad", 896, 896, False),
             ("qkv_dgrad", 1152, 896, False), ("down_fwd", 4864, 896, False), ("gateup_dgrad", 9728, 896, False)]
    for name, k, n, has_bias in cases:
        x = torch.randn(T, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * 0.03).to(torch.bfloat16)
        b = (torch.randn(n, device=dev, generator=g) * 0.1).to(torch.bfloat16) if has_bias else None
        ref = torch.nn.functional.linear(x.float(), w.float(), b.float() if b is not None else None)
        blas = lambda: torch.nn.functional.linear(x, w, b)  # noqa: E731
        yb = blas()
        rec = {"gemm": name, "T": T, "K": k, "N": n, "bias": has_bias,
               "hipblaslt_ms": round(timed(blas), 4),
               "hipblaslt_rel": float((yb.float() - ref).norm() / ref.norm())}
        out = torch.empty(T, n, dtype=torch.bfloat16, device=dev)
        for per in (args.per or [0, 1, 2, 4]):
            def own():
                L.call("va_linear_tn", K._p(x), x.stride(0), K._p(w), w.stride(0), K._p(b) if b is not None else None,
                       L.VA_BF16, T, k, n, per, K._p(out), out.stride(0), K._stream(x))
            own()
            torch.cuda.synchronize()
            rec[f"own_per{per}_ms"] = round(timed(own), 4)
            rec[f"own_per{per}_rel"] = float((out.float() - ref).norm() / ref.norm())
            rec[f"own_per{per}_max_ulp_vs_hipblaslt"] = float(((out.float() - yb.float()).abs() /
                                                             yb.float().abs().clamp_min(1e-30)).max())
        fl = 2.0 * T * k * n
        rec["hipblaslt_pflops"] = round(fl / rec["hipblaslt_ms"] / 1e12, 3)
        best = min((v, kk) for kk, v in rec.items() if kk.startswith("own_per") and kk.endswith("_ms"))
        rec["own_best"] = best[1]
        rec["own_best_pflops"] = round(fl / best[0] / 1e12, 3)
        print(json.dumps(rec), flush=True)
        del x, w, b, ref, yb, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
