"""Device-time microbenchmark of the §8 core-algos kernels at the headline (512 x 1024) and 16x
(8,192 x 1,024) batch, called straight through the C-ABI with preallocated buffers (no autograd,
no allocation in the loop), for rocprofv3 --kernel-trace --stats: the per-kernel average
durations of that profile are the device-only times DESIGN §3 divides the algorithmic bytes by.

Also prints HIP-event wall times per group of launches (what a caller sees, launch gaps included).

Algorithmic bytes per token (int64 mask, m = 8):
  gae_scan (quad/reg/LDS): read r, v, m + write adv_raw, ret      = 4 + 4 + 8 + 4 + 4 = 24
  whiten_apply:            read + write adv                       = 8
  row_scores:              read rewards                           = 4
  broadcast_rows:          read mask + write adv                  = 8 + 4 = 12
  ppo_loss_rows (+k3 KL):  read old, lp, adv, ref, mask           = 16 + 8 = 24
  ppo_loss_bwd  (+k3 KL):  read old, lp, adv, ref, mask + write d = 24 + 4 = 28
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from verl_amd import _lib as L  # noqa: E402
from verl_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rows", type=int, nargs="*", default=[128, 512, 8192])
    ap.add_argument("--loss-vec", type=int, default=1)
    ap.add_argument("--whiten-slice-min", type=int, default=4096)
    ap.add_argument("--whiten-grid", type=int, default=2048)
    ap.add_argument("--R", type=int, default=1024)
    ap.add_argument("--gae-variant", type=int, default=0)
    ap.add_argument("--gae-partials", type=int, default=0)
    ap.add_argument("--gae-nt", type=int, default=3)
    ap.add_argument("--seg-rows", type=int, default=0, help="policy / value loss micro-batch segments (seg_rows)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L.call("va_set_tuning", L.VA_TUNE_GAE_VARIANT, args.gae_variant)
    L.call("va_set_tuning", L.VA_TUNE_GAE_PARTIALS, args.gae_partials)
    L.call("va_set_tuning", L.VA_TUNE_GAE_NT, args.gae_nt)
    L.call("va_set_tuning", L.VA_TUNE_LOSS_VEC, args.loss_vec)
    L.call("va_set_tuning", L.VA_TUNE_WHITEN_SLICE_MIN, args.whiten_slice_min)
    L.call("va_set_tuning", L.VA_TUNE_WHITEN_GRID, args.whiten_grid)
    s = K._vp(torch.cuda.current_stream(dev).cuda_stream)
    out = []
    for B in args.rows:
        R = args.R
        g = torch.Generator(device=dev).manual_seed(B)
        rew = torch.zeros(B, R, device=dev)
        lens = torch.randint(R // 8, R + 1, (B,), device=dev, generator=g)
        rew[torch.arange(B, device=dev), lens - 1] = torch.randn(B, device=dev, generator=g)
        mask = (torch.arange(R, device=dev)[None, :] < lens[:, None]).long()
        val = torch.randn(B, R, device=dev, generator=g)
        adv = torch.empty(B, R, device=dev)
        ret = torch.empty(B, R, device=dev)
        stats = torch.empty(4, device=dev)
        ws = torch.zeros(L.load().va_gae_workspace_bytes(B) // 8, dtype=torch.float64, device=dev)
        index = np.array([f"p{i}" for i in np.random.RandomState(0).permutation(B) // 8], dtype=object)
        order, offsets, G, gmax = K.group_csr(index, dev)
        ows = torch.empty(3 * B, device=dev)
        old = -torch.rand(B, R, device=dev, generator=g)
        lp = old + 0.05 * torch.randn(B, R, device=dev, generator=g)
        ref = old + 0.1 * torch.randn(B, R, device=dev, generator=g)
        nseg = -(-B // args.seg_rows) if 0 < args.seg_rows < B else 1  # output rows (loss micro-batches)
        lout = torch.empty(nseg * 8, device=dev)
        lws = torch.zeros(L.load().va_ppo_loss_workspace_bytes(B) // 8, dtype=torch.float64, device=dev)
        vout = torch.empty(nseg * 8, device=dev)
        aout = torch.empty(1, device=dev)
        vgrad = torch.empty(B, R, device=dev)
        gout = torch.zeros(nseg, 8, device=dev)
        gout[:, 0] = 1.0
        gout[:, 4] = 0.001
        dlp = torch.empty(B, R, device=dev)

        def gae():
            L.call("va_gae_advantage_return", K._p(rew), K._p(val), K._p(mask), L.VA_MASK_I64, B, R, 0.99, 0.95,
                   K._p(adv), K._p(ret), K._p(stats), K._p(ws), s)

        def grpo():
            L.call("va_outcome_advantage", K._p(rew), K._p(mask), L.VA_MASK_I64, B, R, K._p(order), K._p(offsets), G,
                   gmax, 1e-6, L.VA_ADV_GRPO, K._p(adv), None, K._p(ows), s)

        def loss():
            L.call("va_ppo_loss_fwd", K._p(old), K._p(lp), K._p(adv), K._p(mask), L.VA_MASK_I64, K._p(ref), None, B, R,
                   0.8, 1.2, 3.0, 0, L.VA_KL_K3, 0, None, 0.0, args.seg_rows, None, 0, K._p(lout), K._p(lws), s)
            L.call("va_ppo_loss_bwd", K._p(gout), K._p(old), K._p(lp), K._p(adv), K._p(mask), L.VA_MASK_I64, K._p(ref),
                   B, R, 0.8, 1.2, 3.0, 0, L.VA_KL_K3, 0, None, 0.0, args.seg_rows, None, 0, K._p(lws), K._p(dlp), None, s)

        def vloss():  # critic: vpreds = values + noise, returns = ret of the GAE call
            L.call("va_value_loss_fwd", K._p(lp), K._p(old), K._p(ref), K._p(mask), L.VA_MASK_I64, B, R, 0.5, 0, args.seg_rows, None, 0,
                   K._p(vout), K._p(lws), s)
            L.call("va_value_loss_bwd", K._p(gout), K._p(lp), K._p(old), K._p(ref), K._p(mask), L.VA_MASK_I64, B, R,
                   0.5, 0, args.seg_rows, None, 0, K._p(lws), K._p(vgrad), s)

        def agg():  # agg_loss(entropy, mask, token-mean): the actor/entropy metric
            L.call("va_masked_agg_fwd", K._p(lp), K._p(mask), L.VA_MASK_I64, B, R, 0, K._p(aout), K._p(lws), s)

        for name, fn in (("gae_whiten", gae), ("grpo_adv", grpo), ("ppo_loss_fwd_bwd", loss),
                         ("value_loss_fwd_bwd", vloss), ("masked_agg_fwd", agg)):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = 1e3 * e0.elapsed_time(e1) / args.iters
            rec = {"op": name, "B": B, "R": R, "wall_us_per_call": round(us, 2), "gae_variant": args.gae_variant,
                   "gae_partials": args.gae_partials, "gae_nt": args.gae_nt, "loss_vec": args.loss_vec,
                   "seg_rows": args.seg_rows}
            print(json.dumps(rec), flush=True)
            out.append(rec)
    L.call("va_set_tuning", L.VA_TUNE_GAE_VARIANT, 0)


if __name__ == "__main__":
    main()
