"""The backbone GEMMs with a 896- (or 1,152-) wide output, whose last 256-wide hipBLASLt tile is half
empty, as ONE GEMM (the product's F.linear, TunableOp table) against TWO GEMMs over column slices of
the same output (768 + 128 or 1,024 + 128 columns, ldc = the full width; each slice's solution
searched by TunableOp on first use). HIP-event medians, the two forms interleaved; one JSON line per
GEMM with the largest difference between the two results.

  python tools/gemm_split_ab.py [--tokens 151552] [--tune-out gpurun_out/split.csv] [--cases o_fwd,...]
"""

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=10, reps=5):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return sorted(ts)[len(ts) // 2]


def split_linear(x, w, b, n0):
    y = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
    if b is None:
        torch.mm(x, w[:n0].t(), out=y[:, :n0])
        torch.mm(x, w[n0:].t(), out=y[:, n0:])
    else:
        torch.addmm(b[:n0], x, w[:n0].t(), out=y[:, :n0])
        torch.addmm(b[n0:], x, w[n0:].t(), out=y[:, n0:])
    return y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=151552)
    ap.add_argument("--tune-out", default="gpurun_out/gemm_split_tuned.csv")
    ap.add_argument("--cases", default="")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    from verl_amd.utils import gemm_tuning

    assert gemm_tuning.use_tuned_gemms("default")
    tun = torch.cuda.tunable
    os.makedirs(os.path.dirname(os.path.abspath(args.tune_out)), exist_ok=True)
    tun.set_filename(os.path.abspath(args.tune_out), False)
    tun.tuning_enable(True)
    tun.set_max_tuning_iterations(10)
    tun.set_max_tuning_duration(30)
    dev = torch.device("cuda", 0)
    T = args.tokens
    g = torch.Generator(device=dev).manual_seed(5)
    # name: (K, N_out, bias, first slice width); dgrads as the product runs them: dY [T, out] x W^T copy
    cases = {"o_fwd": (896, 896, False, 768), "down_fwd": (4864, 896, False, 768), "qkv_fwd": (896, 1152, True, 1024),
             "o_dgrad": (896, 896, False, 768), "qkv_dgrad": (1152, 896, False, 768),
             "gateup_dgrad": (9728, 896, False, 768)}
    if args.cases:
        cases = {k: v for k, v in cases.items() if k in args.cases.split(",")}
    t0 = time.time()
    for name, (k, n, bias, n0) in cases.items():
        x = torch.randn(T, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * 0.03).to(torch.bfloat16)
        b = (torch.randn(n, device=dev, generator=g) * 0.1).to(torch.bfloat16) if bias else None
        full = lambda: torch.nn.functional.linear(x, w, b)  # noqa: E731
        split = lambda: split_linear(x, w, b, n0)  # noqa: E731
        print(f"[split +{time.time() - t0:6.1f}s] {name}: tuning the slices", flush=True)
        ya, yb = full(), split()
        torch.cuda.synchronize()
        diff = (ya.float() - yb.float()).abs().max().item()
        print(f"[split +{time.time() - t0:6.1f}s] {name}: timing", flush=True)
        tf, ts = [], []
        for _ in range(args.rounds):
            tf.append(timed(full))
            ts.append(timed(split))
        mf, ms = min(tf), min(ts)
        fl = 2.0 * T * k * n
        print(json.dumps({"gemm": name, "T": T, "K": k, "N": n, "slice": n0, "full_ms": round(mf, 4),
                          "split_ms": round(ms, 4), "full_pflops": round(fl / mf / 1e12, 3),
                          "split_pflops": round(fl / ms / 1e12, 3), "speedup": round(mf / ms, 4),
                          "max_abs_diff": diff, "full_all": [round(t, 4) for t in tf],
                          "split_all": [round(t, 4) for t in ts]}), flush=True)
        del x, w, b, ya, yb
    # TunableOp writes the searched entries to --tune-out at exit


if __name__ == "__main__":
    main()
