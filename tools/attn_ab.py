"""Flash-attention timing on a bench-shaped packed micro-batch (128 sequences of prompt U[64, 256]
+ 1024 tokens, 14 query / 2 KV heads, D = 64) with the library VERL_AMD_LIB points at: forward
(no grad) and forward + backward, HIP-event medians over rounds. One JSON line; run once per build.

  VERL_AMD_LIB=scratch/ab/lib_x.so python tools/attn_ab.py --tag x
  python tools/attn_ab.py --tag dma --tune 19=1
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from verl_amd import _lib as L  # noqa: E402
from verl_amd.workers.actor import attention as A  # noqa: E402


def _median_us(fn, reps, rounds=6):
    ts = []
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return round(float(np.median(ts)), 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--seqs", type=int, default=128)
    ap.add_argument("--tune", action="append", default=[], help="KEY=VALUE va_set_tuning before timing")
    args = ap.parse_args()
    for kv in args.tune:
        key, val = (int(x) for x in kv.split("="))
        L.call("va_set_tuning", key, val)
    rng = np.random.default_rng(0)
    lens = (rng.integers(64, 257, args.seqs) + 1024).tolist()
    cu = np.zeros(args.seqs + 1, dtype=np.int64)
    np.cumsum(lens, out=cu[1:])
    T, dev = int(cu[-1]), "cuda"
    g0 = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(T, 14, 64, device=dev, generator=g0).to(torch.bfloat16).requires_grad_(True)
    k = torch.randn(T, 2, 64, device=dev, generator=g0).to(torch.bfloat16).requires_grad_(True)
    v = torch.randn(T, 2, 64, device=dev, generator=g0).to(torch.bfloat16).requires_grad_(True)
    g = torch.randn(T, 14, 64, device=dev, generator=g0).to(torch.bfloat16)
    cu_d = torch.tensor(cu, dtype=torch.int32, device=dev)
    blocks = torch.tensor(A.flash_block_table(cu), device=dev)
    kblocks = torch.tensor(A.flash_key_block_table(cu), device=dev)
    mx = int(max(lens))
    A.FLASH_BWD = "gfx950"
    with torch.no_grad():
        o = A.flash_attention(q, k, v, cu_d, mx, blocks)
        fwd = _median_us(lambda: A.flash_attention(q, k, v, cu_d, mx, blocks), 10)
    out = A.flash_attention(q, k, v, cu_d, mx, blocks, kblocks=kblocks)
    out.backward(g)
    dq = q.grad.float().clone()
    both = _median_us(lambda: A.flash_attention(q, k, v, cu_d, mx, blocks, kblocks=kblocks).backward(g), 5)
    print(json.dumps({"tag": args.tag, "lib": str(L.LIB_PATH), "T": T, "fwd_us": fwd, "fwd_bwd_us": both,
                      "o_checksum": float(o.float().abs().sum()), "dq_checksum": float(dq.abs().sum())}), flush=True)


if __name__ == "__main__":
    main()
