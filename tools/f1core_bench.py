"""Development bench for the f1 GEMM core (tools/f1core/f1core.hip): correctness against torch at
small shapes (full fp32 C), then TF/s at the lm_head shape next to hipBLASLt (torch.matmul, bf16 out).

  python tools/f1core_bench.py [--variants 1 2] [--M 32768] [--iters 10]
The .so is built beforehand on the CPU: hipcc -O3 --offload-arch=gfx950 -shared -fPIC
tools/f1core/f1core.hip -o tools/f1core/libf1core.so"""

import argparse
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", type=int, nargs="*", default=[1])
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--N", type=int, default=151936)
    ap.add_argument("--K", type=int, default=896)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "f1core", "libf1core.so"))
    lib.f1core_gemm_nt.restype = ctypes.c_int
    lib.f1core_gemm_nt.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run(v, A, B, rs, C=None):
        rc = lib.f1core_gemm_nt(v, A.data_ptr(), B.data_ptr(), A.shape[0], B.shape[0], A.shape[1], rs.data_ptr(),
                                C.data_ptr() if C is not None else None, stream)
        assert rc == 0, rc

    g = torch.Generator(device=dev).manual_seed(0)
    for v in args.variants:
        for (M, N, K) in [(256, 256, 64), (512, 1000, 128), (768, 2304, 896), (300, 777, 896)]:
            A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            B = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
            C = torch.zeros(M, N, device=dev)
            rs = torch.zeros(((N + 255) // 256) * 4 * M, device=dev)
            run(v, A, B, rs, C)
            ref = A.float() @ B.float().T
            rsum = rs.view(-1, M).sum(0)
            rerr = (rsum - ref.sum(1)).abs().max().item()
            if v in (3, 6):  # no full-C output: the row sums carry the check
                err, tol = rerr, 1e-3 * ref.sum(1).abs().max().item() + 1e-2
            else:
                err, tol = (C - ref).abs().max().item(), 1e-3 * ref.abs().max().item()
            print(json.dumps({"variant": v, "shape": [M, N, K], "max_abs_err": err, "tol": tol, "ok": err <= tol,
                              "rowsum_err": rerr}), flush=True)
            assert err <= tol
    M, N, K = args.M, args.N, args.K
    A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
    rs = torch.zeros(((N + 255) // 256) * 4 * M, device=dev)
    flop = 2.0 * M * N * K

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

    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ms = timeit(lambda: torch.matmul(A, B.T, out=out))
    print(json.dumps({"kernel": "hipBLASLt (torch.matmul, bf16 out)", "shape": [M, N, K], "ms": round(ms, 3),
                      "tflops": round(flop / ms / 1e9, 1)}), flush=True)
    del out
    for v in args.variants:
        ms = timeit(lambda: run(v, A, B, rs))
        print(json.dumps({"kernel": f"f1core v{v} (row-sum epilogue)", "shape": [M, N, K], "ms": round(ms, 3),
                          "tflops": round(flop / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
