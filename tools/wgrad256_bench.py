"""Probe of tools/wgrad/wgrad256.hip (256 x 256 weight-gradient tiles, LDS-DMA + transposed fragment
reads) against the product's weight gradient (verl_amd.kernels.weight_grad: hipBLASLt with the
committed GEMM table) on the actor's dW = dY^T X shapes at the bench's token counts.

Correctness: max |ours - fp32 reference| relative to max |reference| (bf16 output: ~2^-8).
Timing: HIP events over --iters calls after warm-up, median of --reps.

  hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/wgrad/libwg256.so tools/wgrad/wgrad256.hip
  python tools/wgrad256_bench.py [--cases gateup down qkv o lm_head]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = {  # (K tokens, M = n_out, N = n_in, splits to try)
    "gateup": (151552, 9728, 896, [1, 2, 3, 4, 5, 6, 8]),
    "down": (151552, 896, 4864, [2, 3, 4, 6, 7, 10, 13]),
    "qkv": (151552, 1152, 896, [8, 12, 16, 24, 32]),
    "o": (151552, 896, 896, [8, 16, 24, 32]),
    "lm_head": (131072, 151936, 896, [1, 2]),
    # BASELINE configs 3 / 5 (Llama-3-8B, Qwen2.5-7B) at 32,768 tokens per pass: the product's split choice
    "l8_gateup": (32768, 28672, 4096, [1]),
    "l8_down": (32768, 4096, 14336, [1]),
    "l8_qkv": (32768, 6144, 4096, [1, 2]),
    "l8_o": (32768, 4096, 4096, [1, 3]),
    "q7_gateup": (32768, 37888, 3584, [1]),
    "q7_qkv": (32768, 4608, 3584, [1, 2]),
}


def timed(fn, iters, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(1e3 * e0.elapsed_time(e1) / iters)
    out.sort()
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", nargs="*", default=list(CASES))
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", type=int, nargs="*", default=[0, 1], help="0: 64-token steps, 2 buffers; 1: ring")
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "wgrad", "libwg256.so"))
    lib.wg256_bf16.restype = ctypes.c_int
    lib.wg256_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                               ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_int]
    lib.wg256_workspace_bytes.restype = ctypes.c_int64
    lib.wg256_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    from verl_amd import kernels as K
    from verl_amd.utils.gemm_tuning import use_tuned_gemms

    use_tuned_gemms("default")
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name in args.cases:
        Kt, M, N, splits_list = CASES[name]
        dy = (torch.randn(Kt, M, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        x = torch.randn(Kt, N, device=dev, generator=g).to(torch.bfloat16)
        flops = 2.0 * Kt * M * N
        ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
        scale = ref.abs().max().item()
        prod = K.weight_grad(dy, x)
        prod_err = (prod.float() - ref).abs().max().item() / scale
        prod_us = timed(lambda: K.weight_grad(dy, x), args.iters, args.reps)
        rec = {"case": name, "K": Kt, "M": M, "N": N, "product_us": round(prod_us, 1),
               "product_tflops": round(flops / prod_us / 1e6, 1), "product_rel_err": prod_err}
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        s_ = torch.cuda.current_stream(dev).cuda_stream
        for var in args.variants:
            for sp in splits_list:
                ws_b = lib.wg256_workspace_bytes(M, N, sp)
                ws = torch.empty(max(ws_b // 4, 1), dtype=torch.float32, device=dev)

                def run(sp=sp, ws=ws, var=var):
                    rc = lib.wg256_bf16(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), Kt, M, N, sp,
                                        ws.data_ptr(), out.data_ptr(), s_, var)
                    assert rc == 0, rc

                out.zero_()
                run()
                torch.cuda.synchronize()
                err = (out.float() - ref).abs().max().item() / scale
                us = timed(run, args.iters, args.reps)
                rec[f"v{var}s{sp}_us"] = round(us, 1)
                rec[f"v{var}s{sp}_tflops"] = round(flops / us / 1e6, 1)
                rec[f"v{var}s{sp}_rel_err"] = err
        print(json.dumps(rec), flush=True)
        del dy, x, ref, prod, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
