"""Microbenchmarks of the actor backbone's non-verl_amd work on one MI355X: packed varlen
attention (AOTriton vs CK backends) and the Qwen2.5-0.5B GEMM shapes of one micro-batch.
Prints one JSON line per case. Not part of the product path."""

import json
import sys

import torch
import torch.nn.functional as F


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def attn_case(backend, n_seq=8, seqlen=1184, hq=14, hk=2, d=64):
    from torch.nn.attention.varlen import varlen_attn

    torch.backends.cuda.preferred_rocm_fa_library(backend)
    dev = "cuda"
    T = n_seq * seqlen
    cu = torch.arange(0, T + 1, seqlen, dtype=torch.int32, device=dev)
    q = torch.randn(T, hq, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(T, hk, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(T, hk, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    gqa = True
    try:
        out = varlen_attn(q, k, v, cu, cu, seqlen, seqlen, is_causal=True)
    except Exception as ex:  # noqa: BLE001
        gqa = False
        print(json.dumps({"case": f"attn_{backend}", "gqa_native_error": str(ex)[:200]}))
        k = k.detach().repeat_interleave(hq // hk, dim=1).requires_grad_(True)
        v = v.detach().repeat_interleave(hq // hk, dim=1).requires_grad_(True)
        out = varlen_attn(q, k, v, cu, cu, seqlen, seqlen, is_causal=True)
    g = torch.randn_like(out)

    def fwd():
        varlen_attn(q, k, v, cu, cu, seqlen, seqlen, is_causal=True)

    def fwdbwd():
        o = varlen_attn(q, k, v, cu, cu, seqlen, seqlen, is_causal=True)
        torch.autograd.grad(o, (q, k, v), g)

    flops_fwd = 2.0 * n_seq * seqlen * seqlen * d * hq  # causal: half of 4*S^2*D
    tf = timeit(fwd)
    tfb = timeit(fwdbwd)
    print(json.dumps({"case": f"attn_{backend}", "gqa_native": gqa, "fwd_us": round(tf, 1),
                      "fwd_tflops": round(flops_fwd / tf / 1e6, 1), "fwdbwd_us": round(tfb, 1),
                      "fwdbwd_tflops": round(3.5 * flops_fwd / tfb / 1e6, 1)}))


def gemm_cases(T=9472, H=896, FF=4864, QKV=1152):
    dev = "cuda"
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    for name, (n_out, n_in) in {"qkv": (QKV, H), "o": (H, H), "gate": (FF, H), "gateup": (2 * FF, H),
                                "down": (H, FF)}.items():
        w = torch.randn(n_out, n_in, device=dev, dtype=torch.bfloat16) * 0.02
        a = torch.randn(T, n_in, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, n_out, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * n_out * n_in
        r = {"case": f"gemm_{name}", "T": T}
        r["fwd_us"] = round(timeit(lambda: F.linear(a, w)), 1)
        r["dgrad_us"] = round(timeit(lambda: dy @ w), 1)
        r["wgrad_us"] = round(timeit(lambda: dy.t() @ a), 1)
        for k in ("fwd", "dgrad", "wgrad"):
            r[f"{k}_tflops"] = round(fl / r[f"{k}_us"] / 1e6, 1)
        print(json.dumps(r))
    del x


def attn_gfx950(n_seq=8, seqlen=1184, hq=14, hk=2, d=64, grouped=-1):
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import numpy as np

    from verl_amd import _lib as L
    from verl_amd.workers.actor import attention as A

    L.call("va_set_tuning", L.VA_TUNE_FLASH_GROUPED_DKDV, grouped)

    dev = "cuda"
    T = n_seq * seqlen
    cu_h = np.arange(0, T + 1, seqlen)
    cu = torch.tensor(cu_h, dtype=torch.int32, device=dev)
    blocks = torch.tensor(A.flash_block_table(cu_h), device=dev)
    kblocks = torch.tensor(A.flash_key_block_table(cu_h), device=dev)
    q = torch.randn(T, hq, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(T, hk, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(T, hk, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn_like(q)

    def fwd():
        A.flash_attention(q, k, v, cu, seqlen, blocks)

    def fwdbwd():
        o = A.flash_attention(q, k, v, cu, seqlen, blocks, kblocks=kblocks)
        torch.autograd.grad(o, (q, k, v), g)

    flops_fwd = 2.0 * n_seq * seqlen * seqlen * d * hq
    tf = timeit(fwd)
    tfb = timeit(fwdbwd)
    L.call("va_set_tuning", L.VA_TUNE_FLASH_GROUPED_DKDV, -1)
    print(json.dumps({"case": f"attn_gfx950_fwd_n{n_seq}", "grouped_dkdv": grouped, "fwd_us": round(tf, 1),
                      "fwd_tflops": round(flops_fwd / tf / 1e6, 1), "fwdbwd_us": round(tfb, 1),
                      "fwdbwd_tflops": round(3.5 * flops_fwd / tfb / 1e6, 1)}))


if __name__ == "__main__":
    what = sys.argv[1:] or ["attn", "gemm"]
    if "gfx950" in what:
        attn_case("aotriton")
        attn_gfx950()
        attn_gfx950(n_seq=16)
    if "gfx950_n64" in what:
        for gr in (0, 1):
            attn_gfx950(n_seq=64, grouped=gr)
    if "attn" in what:
        for b in ("aotriton", "ck"):
            try:
                attn_case(b)
            except Exception as ex:  # noqa: BLE001
                print(json.dumps({"case": f"attn_{b}", "error": str(ex)[:300]}))
    if "gemm" in what:
        gemm_cases()
        gemm_cases(T=18944)
