"""Per-kernel statistics from a rocprofv3 rocpd database (run_results.db), optionally split by grid
size (one line per kernel name x grid): count, average / min / max duration in microseconds.

  python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--match ppo_loss] [--by-grid]
"""

from __future__ import annotations

import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--by-grid", action="store_true")
    args = ap.parse_args()
    cur = sqlite3.connect(args.db).cursor()
    key = "name, grid_x, grid_y" if args.by_grid else "name"
    rows = cur.execute(
        f"select {key}, count(*), avg(duration), min(duration), max(duration) from kernels "
        f"where name like ? group by {key} order by sum(duration) desc", (f"%{args.match}%",)).fetchall()
    for r in rows:
        name = r[0][:90]
        grid = f" grid=({r[1]},{r[2]})" if args.by_grid else ""
        n, avg, mn, mx = r[-4:]
        print(f"{name:90s}{grid} n={n:5d} avg={avg / 1e3:9.2f} us min={mn / 1e3:9.2f} max={mx / 1e3:9.2f}")


if __name__ == "__main__":
    main()
