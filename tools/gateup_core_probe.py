"""Probe: the f1 transposed NT core (tools/f1core/f1t.hip variant 0, core only, no output) on the
gate|up forward shape (151,552 tokens x 896 -> 9,728) next to hipBLASLt with the committed tuned
table (the product's GEMM) and the SwiGLU stream kernel it would absorb. One JSON line."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def ms(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / iters)
    return sorted(ts)[2]


def main():
    from verl_amd import kernels as K
    from verl_amd.utils.gemm_tuning import use_tuned_gemms

    lib = ctypes.CDLL(os.path.join(HERE, "f1core", "libf1t.so"))
    lib.f1t_fwd.restype = ctypes.c_int
    lib.f1t_fwd.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_int] + \
        [ctypes.c_void_p] * 5
    lib.f1t_workspace_floats.restype = ctypes.c_int64
    lib.f1t_workspace_floats.argtypes = [ctypes.c_int64, ctypes.c_int]
    dev = torch.device("cuda", 0)
    T, H, F2 = 151552, 896, 9728
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(T, H, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(F2, H, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    lab = torch.zeros(T, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rec = {"T": T, "H": H, "N": F2, "tflop": 2.0 * T * F2 * H / 1e12}
    out = torch.empty(T, F2, dtype=torch.bfloat16, device=dev)
    rec["hipblaslt_default_ms"] = ms(lambda: torch.nn.functional.linear(x, w))
    rec["tuned_table"] = use_tuned_gemms("default")
    rec["hipblaslt_tuned_ms"] = ms(lambda: torch.nn.functional.linear(x, w))
    gu = torch.nn.functional.linear(x, w)
    rec["swiglu_ms"] = ms(lambda: K.swiglu_merged(gu))
    for splits in (1, 2, 4):
        lp = torch.empty(T, device=dev)
        ent = torch.empty(T, device=dev)
        lse = torch.empty(T, device=dev)
        ws = torch.empty(lib.f1t_workspace_floats(T, splits), device=dev)

        def core():
            rc = lib.f1t_fwd(0, x.data_ptr(), w.data_ptr(), lab.data_ptr(), T, H, F2, splits, lp.data_ptr(),
                             ent.data_ptr(), lse.data_ptr(), ws.data_ptr(), stream)
            assert rc == 0, rc
        rec[f"f1_core_s{splits}_ms"] = ms(core)
    rec = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in rec.items()}
    for k in list(rec):
        if k.endswith("_ms") and k != "swiglu_ms":
            rec[k.replace("_ms", "_tflops")] = round(rec["tflop"] / rec[k] * 1e3, 1)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
