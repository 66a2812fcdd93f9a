"""Input-gradient (dgrad) GEMM of the backbone linears: dX = dY @ W as hipBLASLt / rocBLAS "NN"
(W [out, in] row-major: the reduction dim `out` is W's row index, not contiguous) against the same
product over a transposed weight copy W^T [in, out] ("TN": both operands contiguous along the
reduction dim, the layout the forward GEMMs run in at 1.4-1.9 PF/s). The copy costs one transpose
of the weight per optimizer step.

  --mode tune --table T   search TunableOp solutions for the TN shapes, appended to table T
                          (start from a copy of the committed table)
  --mode time --table T   time NN vs TN (lookup only in table T), print one JSON line per shape
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [("gate_up", 9728, 896), ("down", 896, 4864), ("qkv", 1152, 896), ("o", 896, 896)]
LM_HEAD = ("lm_head", 151936, 896)  # rows = response tokens of a 128-response micro-batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["tune", "time"], required=True)
    ap.add_argument("--table", required=True)
    ap.add_argument("--tokens", default="151552,153600")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lm-head-tokens", type=int, default=131072)
    args = ap.parse_args()

    import torch
    import torch.nn.functional as F

    from verl_amd import kernels as K
    from verl_amd.utils import gemm_tuning

    dev = torch.device("cuda", 0)
    if args.mode == "tune":
        gemm_tuning.start_tuning(os.path.abspath(args.table), 20, 50)
    else:
        assert gemm_tuning.use_tuned_gemms(os.path.abspath(args.table))
    g = torch.Generator(device=dev).manual_seed(0)
    cases = [(int(t), s) for t in args.tokens.split(",") for s in SHAPES]
    if args.lm_head_tokens:
        cases.append((args.lm_head_tokens, LM_HEAD))
    for T, (name, n_out, n_in) in cases:
        w = (torch.randn(n_out, n_in, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        dy = torch.randn(T, n_out, device=dev, generator=g).to(torch.bfloat16)
        wt = w.t().contiguous()
        if args.mode == "tune":
            F.linear(dy, wt)
            torch.cuda.synchronize()
            print(f"tuned {name} T={T}", flush=True)
            continue

        def timed(fn):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            return sorted(ts)[len(ts) // 2]

        nn = timed(lambda: dy @ w)
        tn = timed(lambda: F.linear(dy, wt))
        tr = timed(lambda: w.t().contiguous())
        tr16 = timed(lambda: K.transpose16(w))
        rows = slice(0, 8192)  # fp32 reference on a row sample
        ref = dy[rows].float() @ w.float()
        e_nn = float(((dy @ w)[rows].float() - ref).abs().max())
        e_tn = float((F.linear(dy, wt)[rows].float() - ref).abs().max())
        fl = 2.0 * T * n_out * n_in
        print(json.dumps({"shape": name, "T": T, "out": n_out, "in": n_in, "nn_us": round(nn, 1),
                          "tn_us": round(tn, 1), "transpose_w_us": round(tr, 1),
                          "transpose16_us": round(tr16, 1),
                          "nn_tf": round(fl / nn / 1e6, 1), "tn_tf": round(fl / tn / 1e6, 1),
                          "max_abs_err_nn": e_nn, "max_abs_err_tn": e_tn}), flush=True)
        del w, dy, wt
    if args.mode == "tune":
        gemm_tuning.finish_tuning()  # TunableOp writes the table at exit


if __name__ == "__main__":
    main()
