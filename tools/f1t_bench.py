"""Development bench for tools/f1core/f1t.hip (f1 v3: transposed tile, lane-local online softmax):
exact-arithmetic correctness against the unfused semantics (bf16 logits -> fp32 log-softmax /
entropy), then time at the lm_head shape next to hipBLASLt + the streaming log-prob kernel and the
product fused kernel.

  python tools/f1t_bench.py [--rows 32768 131072] [--splits 1 8] [--variants 0 1 2 3]
Build first (CPU): hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/f1core/f1t.hip -o tools/f1core/libf1t.so
"""

import argparse
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def want(h, w, labels):
    x = (h.float() @ w.float().t()).to(torch.bfloat16).float()
    lse = torch.logsumexp(x, -1)
    lp = x.gather(-1, labels[:, None]).squeeze(-1) - lse
    p = torch.softmax(x, -1)
    ent = lse - (p * x).sum(-1)
    return lp, ent


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="*", default=[32768, 131072])
    ap.add_argument("--splits", type=int, nargs="*", default=[1, 8])
    ap.add_argument("--variants", type=int, nargs="*", default=[0, 1, 2, 3])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--no-product", action="store_true")
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "f1core", "libf1t.so"))
    lib.f1t_fwd.restype = ctypes.c_int
    lib.f1t_fwd.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_int] + \
        [ctypes.c_void_p] * 5
    lib.f1t_workspace_floats.restype = ctypes.c_int64
    lib.f1t_workspace_floats.argtypes = [ctypes.c_int64, ctypes.c_int]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run(v, h, w, lab, splits):
        N, H = h.shape
        V = w.shape[0]
        lp = torch.empty(N, device=dev)
        ent = torch.empty(N, device=dev)
        lse = torch.empty(N, device=dev)
        ws = torch.empty(lib.f1t_workspace_floats(N, splits), device=dev)
        rc = lib.f1t_fwd(v, h.data_ptr(), w.data_ptr(), lab.data_ptr(), N, H, V, splits, lp.data_ptr(), ent.data_ptr(),
                         lse.data_ptr(), ws.data_ptr(), stream)
        assert rc == 0, rc
        return lp, ent

    g = torch.Generator().manual_seed(0)
    for (N, H, V) in [(300, 64, 1000), (512, 896, 151936), (77, 128, 37), (2048, 896, 4100)]:
        h = (torch.randint(-4, 5, (N, H), generator=g).float() / 8).to(torch.bfloat16).to(dev)
        w = (torch.randint(-4, 5, (V, H), generator=g).float() / 16).to(torch.bfloat16).to(dev)
        lab = torch.randint(0, V, (N,), generator=g).to(dev)
        wl, we = want(h, w, lab)
        for v in (1, 2, 5, 10):
            for sp in (1, 3, 8):
                if v in (5, 6, 8, 10) and ((N + 255) // 256) * min(sp, (V + 255) // 256) % 8:
                    continue  # remap-only variants need a grid that is a multiple of 8
                lp, ent = run(v, h, w, lab, sp)
                torch.cuda.synchronize()
                e1 = float((lp - wl).abs().max())
                e2 = float((ent - we).abs().max())
                ok = e1 <= 1e-5 * (1 + float(wl.abs().max())) and e2 <= 1e-5 * (1 + float(we.abs().max()))
                print(json.dumps({"check": [N, H, V], "variant": v, "splits": sp, "lp_err": e1, "ent_err": e2,
                                  "ok": ok}), flush=True)
                assert ok

    from verl_amd import kernels as K

    def timeit(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.iters

    H, V = 896, 151936
    gd = torch.Generator(device=dev).manual_seed(1)
    w = (torch.randn(V, H, device=dev, generator=gd) * 0.05).to(torch.bfloat16)
    for N in args.rows:
        h = torch.randn(N, H, device=dev, generator=gd).to(torch.bfloat16)
        lab = torch.randint(0, V, (N,), device=dev, generator=gd)
        flop = 2.0 * N * V * H
        rec = {"N": N}
        with torch.no_grad():
            rec["gemm_ms"] = timeit(lambda: h @ w.t())
            rec["unfused_ms"] = timeit(lambda: K.logprob_entropy(h @ w.t(), lab, 1.0))
            if not args.no_product:
                rec["product_fused_ms"] = timeit(lambda: K.linear_logprob_entropy(h, w, lab, 1.0))
            for v in args.variants:
                for sp in args.splits:
                    rec[f"v{v}_s{sp}_ms"] = timeit(lambda: run(v, h, w, lab, sp))
            ref_lp, ref_ent = K.logprob_entropy(h @ w.t(), lab, 1.0)
            lp, ent = run(1, h, w, lab, args.splits[-1])
            rec["max_dlp_vs_unfused"] = float((lp - ref_lp).abs().max())
            rec["max_dent_vs_unfused"] = float((ent - ref_ent).abs().max())
        out = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in rec.items()}
        out.update({k.replace("_ms", "_tflops"): round(flop / v / 1e9, 1) for k, v in rec.items() if k.endswith("_ms")})
        print(json.dumps(out), flush=True)
        del h


if __name__ == "__main__":
    main()
