"""Offline TunableOp search for weight-gradient GEMMs dW = dY^T X (the exact torch.mm call of
verl_amd.kernels.weight_grad / autograd's linear backward) at given (n_out, n_in, T), appended to a
table that utils/gemm_tuning.py can load. Prints progress every 30 s (one search takes minutes).

  python tools/tune_wgrad.py --out gpurun_out/wgrad_table.csv 9728,896,151552 9728,896,153600
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--duration-ms", type=int, default=20)
    ap.add_argument("shapes", nargs="+", help="n_out,n_in,T")
    args = ap.parse_args()

    import torch

    from verl_amd.utils import gemm_tuning

    t0 = time.time()
    state = {"what": "setup"}

    def log(msg):
        print(f"[tune-wgrad +{time.time() - t0:7.1f}s] {msg}", flush=True)

    def watchdog():
        while True:
            time.sleep(30)
            log(f"still tuning: {state['what']}")

    threading.Thread(target=watchdog, daemon=True).start()
    dev = torch.device("cuda", 0)
    gemm_tuning.start_tuning(os.path.abspath(args.out), args.iters, args.duration_ms)
    for spec in args.shapes:
        n_out, n_in, T = (int(v) for v in spec.split(","))
        state["what"] = spec
        dy = torch.randn(T, n_out, device=dev).to(torch.bfloat16)
        x = torch.randn(T, n_in, device=dev).to(torch.bfloat16)
        torch.mm(dy.t(), x)
        torch.cuda.synchronize()
        log(f"{spec} tuned")
        del dy, x
    gemm_tuning.finish_tuning()
    for line in open(args.out):
        if line.startswith("Gemm"):
            log(line.strip())


if __name__ == "__main__":
    main()
