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
    ap.add_argument("--steps", type=int, default=0,
                    help="per-step idle over the last N steps (a step = from the end of one optimizer step's "
                         "AdamW launches to the end of the next), and the gaps of those steps summed by the "
                         "kernel pair around them")
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
    if a.steps:
        per_step(ev, a.steps, a.top)


def per_step(ev, n_steps, top):
    """Idle time of each of the last ``n_steps`` steps, bounded by the optimizer (AdamW
    multi_tensor_apply) launch groups, and their gaps summed by (kernel before, kernel after)."""
    groups, last = [], None
    for s, e, n in ev:
        if "multi_tensor_apply" in n:
            if last is None or s - last > 20e6:
                groups.append([s, e])
            else:
                groups[-1][1] = max(groups[-1][1], e)
            last = s
    if len(groups) < n_steps + 1:
        print(f"per-step: only {len(groups)} optimizer steps in the trace")
        return
    pairs, tot_idle, tot_span = {}, 0, 0
    for i in range(len(groups) - n_steps, len(groups)):
        lo, hi = groups[i - 1][1], groups[i][1]
        sev = [x for x in ev if x[0] >= lo and x[1] <= hi]
        cur_e, prev = lo, "(previous optimizer step)"
        idle, big, cnt = 0, (0, "", ""), 0
        for s, e, n in sev:
            if s > cur_e:
                g = s - cur_e
                idle += g
                cnt += 1
                big = max(big, (g, prev, n))
                k = (prev[:40], n[:40])
                pairs.setdefault(k, [0, 0])
                pairs[k][0] += 1
                pairs[k][1] += g
            if e >= cur_e:
                cur_e, prev = e, n
        span = hi - lo
        tot_idle += idle
        tot_span += span
        print(f"step {i}: span {span / 1e6:8.2f} ms, idle {idle / 1e6:7.2f} ms ({100 * idle / span:.2f}%) in {cnt} "
              f"gaps; largest {big[0] / 1e3:.1f} us after {big[1][:40]} before {big[2][:40]}")
    print(f"last {n_steps} steps: idle {tot_idle / 1e6:.2f} of {tot_span / 1e6:.2f} ms ({100 * tot_idle / tot_span:.2f}%)")
    for (p, n), (c, g) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {g / 1e6 / n_steps:7.3f} ms/step {c / n_steps:6.1f} gaps/step  after {p:40s} before {n}")


if __name__ == "__main__":
    main()
