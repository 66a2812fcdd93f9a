"""GPU idle time from a rocprofv3 --kernel-trace CSV: busy-interval union over the last
``--window`` seconds of the trace (the timed steps), total idle, and the largest gaps with the
kernels on either side. Not part of the product path.

  python tools/trace_gaps.py gpurun_out/prof/..._kernel_trace.csv [--window 3.5] [--top 15]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=0.0, help="seconds at the end of the trace (0 = all)")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--timeline", type=float, default=0.0,
                    help="also list, in time order, every gap >= this many us and each step end (AdamW)")
    a = ap.parse_args()
    ev = []
    for r in csv.DictReader(open(a.trace)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    ev.sort()
    t_end = max(e[1] for e in ev)
    t0 = t_end - int(a.window * 1e9) if a.window > 0 else ev[0][0]
    ev = [e for e in ev if e[0] >= t0]
    busy, gaps, tl = 0, [], []
    cur_s, cur_e, prev_name = ev[0][0], ev[0][1], ev[0][2]
    last_opt = None
    for s, e, n in ev[1:]:
        if a.timeline and "multi_tensor_apply" in n:
            if last_opt is None or s - last_opt > 20e6:
                tl.append((s, "---- optimizer step", ""))
            last_opt = s
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, n))
            if a.timeline and s - cur_e >= a.timeline * 1e3:
                tl.append((cur_e, f"gap {(s - cur_e) / 1e3:9.1f} us after {prev_name[:45]}", f"before {n[:45]}"))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n if e >= cur_e else prev_name
    busy += cur_e - cur_s
    span = ev[-1][1] - ev[0][0]
    idle = span - busy
    print(f"span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, idle {idle / 1e6:.1f} ms ({100 * idle / span:.1f}%), "
          f"{len(gaps)} gaps, {len(ev)} kernels")
    big = sorted(gaps, reverse=True)[: a.top]
    for g, p, n in big:
        print(f"  gap {g / 1e3:9.1f} us  after {p:60s} before {n}")
    hist = {}
    for g, _, _ in gaps:
        k = "<5us" if g < 5e3 else "<50us" if g < 5e4 else "<1ms" if g < 1e6 else ">=1ms"
        hist.setdefault(k, [0, 0])
        hist[k][0] += 1
        hist[k][1] += g
    for k, (c, t) in hist.items():
        print(f"  {k:6s} {c:6d} gaps {t / 1e6:8.1f} ms")
    for t, what, nxt in tl:
        print(f"  {(t - ev[0][0]) / 1e6:9.2f} ms  {what} {nxt}")


if __name__ == "__main__":
    main()
