"""Per-dispatch timeline of a rocprofv3 --kernel-trace run (rocpd SQLite): kernels in issue order with their
durations and the gap before each, optionally restricted to the dispatches between two occurrences of a marker
kernel (one training step). Usage:
  python tools/dispatch_timeline.py <run_results.db> [--after NAME_SUBSTR --nth N --count K] [--top T]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after", default=None, help="start at the nth dispatch whose name contains this")
    ap.add_argument("--nth", type=int, default=0)
    ap.add_argument("--count", type=int, default=400, help="dispatches to list from there")
    ap.add_argument("--grid-min", type=int, default=0)
    ap.add_argument("--summary", action="store_true", help="sum by kernel name over the window instead")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    names = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
    rows = list(c.execute("select kernel_id, start, end, grid_size_x, grid_size_y, workgroup_size_x "
                          "from rocpd_kernel_dispatch order by start"))
    i0 = 0
    if a.after:
        hits = [i for i, r in enumerate(rows) if a.after in names[r[0]]]
        i0 = hits[a.nth]
    win = rows[i0:i0 + a.count]
    if a.summary:
        agg = defaultdict(lambda: [0, 0.0])
        for r in win:
            agg[names[r[0]]][0] += 1
            agg[names[r[0]]][1] += (r[2] - r[1]) / 1e3
        span = (win[-1][2] - win[0][1]) / 1e3
        busy = sum(v[1] for v in agg.values())
        print(f"window: {len(win)} dispatches, span {span:.1f} us, kernel busy {busy:.1f} us")
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{v[1]:10.1f} us {v[0]:5d}x  {k[:110]}")
        return
    prev_end = None
    for r in win:
        gap = (r[1] - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = r[2]
        print(f"{(r[2] - r[1]) / 1e3:9.1f} us  gap {gap:7.1f}  grid {r[3] // max(r[5], 1):6d}x{r[4]:<3d} "
              f"{names[r[0]][:100]}")


if __name__ == "__main__":
    main()
