"""Offline TunableOp search for the lm_head GEMMs of the actor (fwd, dgrad, wgrad at rows =
micro-batch x response length), appended to a verl_amd/tuned/*.csv table. Companion of
tools/tune_gemms.py (which tunes the backbone with a small vocabulary). A watchdog thread prints
the elapsed tuning time every 30 s (one shape's search takes minutes).

  python tools/tune_lm_head.py --out gpurun_out/lm_head_table.csv --rows 65536
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
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=151936)
    ap.add_argument("--hidden", type=int, default=896)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--duration-ms", type=int, default=60)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    args = ap.parse_args()

    import torch

    from verl_amd.utils import gemm_tuning

    t0 = time.time()
    state = {"what": "setup"}

    def log(msg):
        print(f"[tune-lm +{time.time() - t0:7.1f}s] {msg}", flush=True)

    def watchdog():
        while True:
            time.sleep(30)
            log(f"still tuning: {state['what']}")

    threading.Thread(target=watchdog, daemon=True).start()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    h = (torch.randn(args.rows, args.hidden, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(args.vocab, args.hidden, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    dy = (torch.randn(args.rows, args.vocab, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    gemm_tuning.start_tuning(os.path.abspath(args.out), args.iters, args.duration_ms)
    only = set(args.only.split(","))
    # the exact calls autograd issues for y = F.linear(h, w): fwd, dgrad dy @ w, wgrad dy^T @ h
    if "fwd" in only:
        state["what"] = "fwd"
        torch.nn.functional.linear(h, w)
        torch.cuda.synchronize()
        log("fwd tuned")
    if "dgrad" in only:
        state["what"] = "dgrad"
        torch.mm(dy, w)
        torch.cuda.synchronize()
        log("dgrad tuned")
    if "wgrad" in only:
        state["what"] = "wgrad"
        torch.mm(dy.t(), h)
        torch.cuda.synchronize()
        log("wgrad tuned")
    gemm_tuning.finish_tuning()
    for line in open(args.out):
        if line.startswith("Gemm"):
            log(line.strip())


if __name__ == "__main__":
    main()
