"""Probe: how much would PyTorch TunableOp (exhaustive hipBLASLt / rocBLAS solution search) gain
over hipBLASLt's default heuristic on the actor backbone's GEMM shapes? One packed micro-batch
(T tokens), Qwen2.5-0.5B shapes, fwd / dgrad / wgrad. Prints one JSON line per shape.
Not part of the product path."""

import json
import os
import sys

import torch
import torch.nn.functional as F


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 9472
    dev = "cuda"
    H, FF, V = 896, 4864, 151936
    shapes = {"qkv": (1152, H), "o": (H, H), "gateup": (2 * FF, H), "down": (H, FF), "lm_head": (V, H)}
    tun = torch.cuda.tunable
    tun.set_filename(os.path.join("gpurun_out", "tunableop_probe.csv"))
    tun.set_max_tuning_duration(40)
    tun.set_max_tuning_iterations(20)
    tot_def, tot_tun = 0.0, 0.0
    for name, (n_out, n_in) in shapes.items():
        Tn = T if name != "lm_head" else 8192
        w = torch.randn(n_out, n_in, device=dev, dtype=torch.bfloat16) * 0.02
        a = torch.randn(Tn, n_in, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(Tn, n_out, device=dev, dtype=torch.bfloat16)
        ops = {"fwd": lambda: F.linear(a, w), "dgrad": lambda: dy @ w, "wgrad": lambda: dy.t() @ a}
        for k, fn in ops.items():
            tun.enable(False)
            t0 = timeit(fn)
            tun.enable(True)
            tun.tuning_enable(True)
            fn()  # tunes this shape
            torch.cuda.synchronize()
            tun.tuning_enable(False)
            t1 = timeit(fn)
            tun.enable(False)
            fl = 2.0 * Tn * n_out * n_in
            tot_def += t0
            tot_tun += t1
            print(json.dumps({"shape": f"{name}_{k}", "T": Tn, "default_us": round(t0, 1), "tuned_us": round(t1, 1),
                              "default_tflops": round(fl / t0 / 1e6, 1), "tuned_tflops": round(fl / t1 / 1e6, 1),
                              "gain": round(t0 / t1, 3)}), flush=True)
    print(json.dumps({"total_default_us": round(tot_def, 1), "total_tuned_us": round(tot_tun, 1),
                      "gain": round(tot_def / tot_tun, 3)}))


if __name__ == "__main__":
    main()
