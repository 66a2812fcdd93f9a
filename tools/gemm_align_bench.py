"""How hipBLASLt GEMM time depends on the packed token count T (alignment) for the
Qwen2.5-0.5B actor shapes. Prints one JSON line per (shape, T)."""
import json

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


dev = "cuda"
H, FF = 896, 4864
shapes = {"qkv": (1152, H), "o": (H, H), "gateup": (2 * FF, H), "down": (H, FF)}
for T in (9472, 9473, 9500, 9599, 9600, 9728, 18944, 18999, 19200):
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for name, (n_out, n_in) in shapes.items():
        w = torch.randn(n_out, n_in, device=dev, dtype=torch.bfloat16) * 0.02
        a = torch.randn(T, n_in, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, n_out, device=dev, dtype=torch.bfloat16)
        tot["fwd"] += timeit(lambda: F.linear(a, w))
        tot["dgrad"] += timeit(lambda: dy @ w)
        tot["wgrad"] += timeit(lambda: dy.t() @ a)
    fl = 2.0 * T * sum(o * i for o, i in shapes.values())
    print(json.dumps({"T": T, **{k: round(v, 1) for k, v in tot.items()},
                      **{k + "_tflops": round(fl / v / 1e6, 1) for k, v in tot.items()}}), flush=True)
