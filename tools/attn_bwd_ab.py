"""Interleaved A/B of the flash-attention backward's staging sizes (dK / dV query-tile height
VA_TUNE_FLASH_DKDV_QT, dQ key-block width VA_TUNE_FLASH_DQ_KB) on a bench-shaped packed micro-batch (128 sequences of prompt U[64, 256] + 1024 tokens,
14 query / 2 KV heads, D = 64). HIP-event timed fwd + bwd, median over rounds.

  python tools/attn_bwd_ab.py [N_SEQ]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from verl_amd import _lib as L  # noqa: E402
from verl_amd.workers.actor import attention as A  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    rng = np.random.default_rng(0)
    lens = (rng.integers(64, 257, n) + 1024).tolist()
    cu = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=cu[1:])
    T, dev = int(cu[-1]), "cuda"
    q = torch.randn(T, 14, 64, device=dev).to(torch.bfloat16).requires_grad_(True)
    k = torch.randn(T, 2, 64, device=dev).to(torch.bfloat16).requires_grad_(True)
    v = torch.randn(T, 2, 64, device=dev).to(torch.bfloat16).requires_grad_(True)
    g = torch.randn(T, 14, 64, device=dev).to(torch.bfloat16)
    cu_d = torch.tensor(cu, dtype=torch.int32, device=dev)
    blocks = torch.tensor(A.flash_block_table(cu), device=dev)
    kblocks = torch.tensor(A.flash_key_block_table(cu), device=dev)
    mx = int(max(lens))
    A.FLASH_BWD = "gfx950"
    L.call("va_set_tuning", L.VA_TUNE_FLASH_FWD_KB, 64)

    def step():
        A.flash_attention(q, k, v, cu_d, mx, blocks, kblocks=kblocks).backward(g)

    variants = [(32, 64), (64, 128), (128, 128)]
    times = {v: [] for v in variants}
    for _ in range(6):
        for qt, kb in variants:
            L.call("va_set_tuning", L.VA_TUNE_FLASH_DKDV_QT, qt)
            L.call("va_set_tuning", L.VA_TUNE_FLASH_DQ_KB, kb)
            step()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                step()
            b.record()
            torch.cuda.synchronize()
            times[(qt, kb)].append(a.elapsed_time(b) / 5 * 1e3)
    for key, val in L.FLASH_TUNING_DEFAULTS.items():
        L.call("va_set_tuning", key, val)
    fwd_times = {64: [], 128: []}
    with torch.no_grad():
        for _ in range(6):
            for kbf in (64, 128):
                L.call("va_set_tuning", L.VA_TUNE_FLASH_FWD_KB, kbf)
                A.flash_attention(q, k, v, cu_d, mx, blocks)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    A.flash_attention(q, k, v, cu_d, mx, blocks)
                b.record()
                torch.cuda.synchronize()
                fwd_times[kbf].append(a.elapsed_time(b) / 10 * 1e3)
    L.call("va_set_tuning", L.VA_TUNE_FLASH_FWD_KB, 64)
    for kbf, ts in fwd_times.items():
        print(json.dumps({"case": f"flash_fwd_kb{kbf}", "T": T, "median_us": round(float(np.median(ts)), 1)}),
              flush=True)
    for (qt, kb), ts in times.items():
        print(json.dumps({"case": f"flash_fwd_bwd_dkdv_qt{qt}_dq_kb{kb}", "T": T,
                          "median_us": round(float(np.median(ts)), 1)}), flush=True)


if __name__ == "__main__":
    main()
