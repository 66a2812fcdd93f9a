"""A/B of the product fused lm_head + log-prob kernel (va_linear_logprob_fwd) between two builds of
libverl_amd.so: run once per build with VERL_AMD_LIB pointing at it; prints one JSON line (median
of 5 timed blocks of --iters launches, and the largest deviation from the unfused path).

  VERL_AMD_LIB=scratch/ab/libverl_amd_old.so python tools/f1_ab.py --tag old

--pre-gemm-ms X runs X ms of back-to-back hipBLASLt GEMMs (the backbone's gate|up forward shape)
right before each timed block, with no host sync in between: the f1 launches then start in the
power / clock state the bench step leaves them in (the in-step penalty question).
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tune", action="append", default=[], help="KEY=VALUE va_set_tuning before timing")
    ap.add_argument("--unfused", action="store_true",
                    help="also time the unfused path (hipBLASLt lm_head GEMM + logprob_entropy_fwd), e.g. under rocprofv3")
    ap.add_argument("--pre-gemm-ms", type=float, default=0.0,
                    help="back-to-back GEMM load (ms) right before each timed block")
    args = ap.parse_args()
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    for kv in args.tune:
        key, val = (int(x) for x in kv.split("="))
        L.call("va_set_tuning", key, val)
    dev = torch.device("cuda", 0)
    H, V, N = 896, 151936, args.rows
    g = torch.Generator(device=dev).manual_seed(1)
    w = (torch.randn(V, H, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    h = torch.randn(N, H, device=dev, generator=g).to(torch.bfloat16)
    lab = torch.randint(0, V, (N,), device=dev, generator=g)
    with torch.no_grad():
        lp, ent = K.linear_logprob_entropy(h, w, lab, 1.0)[:2]
        ref_lp, ref_ent = K.logprob_entropy(h @ w.t(), lab, 1.0)[:2]
        dlp = float((lp - ref_lp).abs().max())
        dent = float((ent - ref_ent).abs().max())
        for _ in range(3):
            K.linear_logprob_entropy(h, w, lab, 1.0)
        torch.cuda.synchronize()
        pre = None
        if args.pre_gemm_ms > 0:  # ~2.0 ms per gate|up forward GEMM at 163,840 tokens
            xa = torch.randn(163840, 896, device=dev).to(torch.bfloat16)
            wa = torch.randn(9728, 896, device=dev).to(torch.bfloat16)
            ya = torch.empty(163840, 9728, dtype=torch.bfloat16, device=dev)
            pre = (xa, wa, ya, max(1, int(args.pre_gemm_ms / 2.0)))
        times = []
        for _ in range(5):
            if pre is not None:
                for _ in range(pre[3]):
                    torch.matmul(pre[0], pre[1].t(), out=pre[2])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                K.linear_logprob_entropy(h, w, lab, 1.0)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / args.iters)
    times.sort()
    ms = times[len(times) // 2]
    unfused_ms = None
    if args.unfused:
        logits = torch.empty(N, V, dtype=torch.bfloat16, device=dev)
        with torch.no_grad():
            for _ in range(3):
                K.logprob_entropy(torch.matmul(h, w.t(), out=logits), lab, 1.0)
            torch.cuda.synchronize()
            ut = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    K.logprob_entropy(torch.matmul(h, w.t(), out=logits), lab, 1.0)
                e1.record()
                torch.cuda.synchronize()
                ut.append(e0.elapsed_time(e1) / args.iters)
        unfused_ms = round(sorted(ut)[2], 3)
        del logits
    print(json.dumps({"tag": args.tag, "lib": str(L.LIB_PATH), "rows": N, "pre_gemm_ms": args.pre_gemm_ms,
                      "iters": args.iters, "ms_median": round(ms, 3),
                      "ms_all": [round(t, 3) for t in times], "tflops": round(2.0 * N * V * H / ms / 1e9, 1),
                      "max_dlp_vs_unfused": dlp, "max_dent_vs_unfused": dent, "unfused_ms": unfused_ms}), flush=True)


if __name__ == "__main__":
    main()
