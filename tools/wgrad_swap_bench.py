"""Weight-gradient GEMM layouts of the backbone linears at the bench's packed token counts.

dW [out, in] = dY^T X (K = tokens; both operands have the reduction dim as their row index) as
  * current:  kernels.weight_grad (tuned plain GEMM or split-K batched GEMM, fp32 slice sum)
  * swapped:  dW^T [in, out] = X^T dY, then va_transpose_16 of the small result
  * swapped_sS: the swapped product as S token slices (fp32 batched GEMM, summed, rounded once)

  --mode tune --table T   search TunableOp solutions for the swapped shapes (appended to T)
  --mode time --table T   time all variants (lookup only), one JSON line per shape
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [("gate_up", 9728, 896), ("down", 896, 4864), ("qkv", 1152, 896), ("o", 896, 896),
          ("lm_head", 151936, 896)]  # lm_head rows: --tokens 131072 (response tokens of 128 responses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["tune", "time"], required=True)
    ap.add_argument("--table", required=True)
    ap.add_argument("--tokens", default="151552")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--shapes", default="gate_up,down,qkv,o")
    args = ap.parse_args()

    import torch

    from verl_amd import kernels as K
    from verl_amd.utils import gemm_tuning

    dev = torch.device("cuda", 0)
    if args.mode == "tune":
        gemm_tuning.start_tuning(os.path.abspath(args.table), 20, 50)
    else:
        assert gemm_tuning.use_tuned_gemms(os.path.abspath(args.table))
    g = torch.Generator(device=dev).manual_seed(0)
    want = set(args.shapes.split(","))

    def swapped(dy, x, s=1):
        T = x.shape[0]
        if s == 1:
            return K.transpose16(x.t() @ dy)
        h = T // s
        part = torch.bmm(x[: s * h].view(s, h, -1).transpose(1, 2), dy[: s * h].view(s, h, -1),
                         out_dtype=torch.float32)
        acc = part.sum(0)
        if s * h < T:
            acc += torch.mm(x[s * h:].t(), dy[s * h:], out_dtype=torch.float32)
        return K.transpose16(acc.to(dy.dtype))

    for T in (int(t) for t in args.tokens.split(",")):
        for name, n_out, n_in in SHAPES:
            if name not in want:
                continue
            dy = torch.randn(T, n_out, device=dev, generator=g).to(torch.bfloat16)
            x = torch.randn(T, n_in, device=dev, generator=g).to(torch.bfloat16)
            if args.mode == "tune":
                for s in (1, 2, 4, 8):
                    swapped(dy, x, s)
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
                return round(sorted(ts)[len(ts) // 2], 1)

            ref = K.weight_grad(dy, x).float()
            rec = {"shape": name, "T": T, "out": n_out, "in": n_in, "current_us": timed(lambda: K.weight_grad(dy, x)),
                   "current_splits": K.wgrad_splits(T, n_out, n_in)}
            for s in ((1, 2) if n_out > 65536 else (1, 2, 4, 8)):
                rec[f"swapped_s{s}_us"] = timed(lambda s=s: swapped(dy, x, s))
                err = float((swapped(dy, x, s).float() - ref).abs().max() / ref.abs().max())
                rec[f"swapped_s{s}_relerr"] = round(err, 5)
            print(json.dumps(rec), flush=True)
            del dy, x
    if args.mode == "tune":
        gemm_tuning.finish_tuning()  # TunableOp writes the table at exit


if __name__ == "__main__":
    main()
