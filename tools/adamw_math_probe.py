"""Which rounding flavour of va_adamw_flat (VA_TUNE_ADAMW_MATH bits: 1 hardware sqrt, 2 reciprocal
division, 4 double FMA contraction) reproduces this torch build's torch.optim.AdamW(fused=True) bit for
bit: 5 steps over 1M random fp32 elements (weight decay, the folded clip scale) per mode; one JSON line
with the differing masters / moments per mode.

  python tools/adamw_math_probe.py
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    dev = "cuda"
    n = 1 << 20
    g = torch.Generator(device=dev).manual_seed(0)
    p0 = torch.randn(n, device=dev, generator=g) * 0.05
    grads = [torch.randn(n, device=dev, generator=g) * 10 ** torch.empty(n, device=dev).uniform_(-6, 0, generator=g)
             for _ in range(5)]
    coef = torch.tensor(0.37, device=dev)
    # torch reference
    pt = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([pt], lr=1e-3, betas=(0.9, 0.999), weight_decay=0.01, fused=True)
    for gr in grads:
        pt.grad = gr * coef
        opt.step()
    st = opt.state[pt]
    out = {}
    for mode in range(8):
        L.call("va_set_tuning", L.VA_TUNE_ADAMW_MATH, mode)
        p, m, v = p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        step = torch.zeros((), device=dev)
        for gr in grads:
            gg = gr.clone()
            step.add_(1.0)
            L.call("va_adamw_flat", K._p(p), K._p(gg), K._p(m), K._p(v), n, 1e-3, 0.9, 0.999, 1e-8, 0.01, K._p(step),
                   K._p(coef), None, 0, K._stream(p))
        torch.cuda.synchronize()
        out[mode] = {"param_diff": int((p != pt.detach()).sum()), "exp_avg_diff": int((m != st["exp_avg"]).sum()),
                     "exp_avg_sq_diff": int((v != st["exp_avg_sq"]).sum()),
                     "max_abs_param": float((p - pt.detach()).abs().max())}
    L.call("va_set_tuning", L.VA_TUNE_ADAMW_MATH, 0)
    print(json.dumps({"n": n, "steps": 5, "torch": torch.__version__, "modes": out}), flush=True)


if __name__ == "__main__":
    main()
