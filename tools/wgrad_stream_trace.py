"""Split a rocprofv3 trace of tools/wgrad_stream_legs.py at its marker kernels (hold_cu_kernel) and summarise each
leg's timed steps: span, GPU busy (union of kernel intervals) vs idle, sum of kernel durations per stream, the largest
idle gaps, the kernels whose per-call time changed most, and (with --hip-trace / --runtime-trace data in the database)
the HIP API calls inside the window by name, count and total time.

  python tools/wgrad_stream_trace.py <profile dir> [top]
"""
import glob
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name)[:70]


def query(c, sqls):
    for q in sqls:
        try:
            return list(c.execute(q))
        except sqlite3.OperationalError:
            continue
    return []


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    print("tables/views:", ", ".join(t for t in tables if not t.startswith("sqlite")))
    ks = query(c, ["select name, start, end, stream_id from kernels order by start",
                   "select kernel_name, start, end, stream_id from kernels order by start"])
    marks = [i for i, r in enumerate(ks) if "hold_cu_kernel" in r[0]]
    print(f"{len(ks)} kernels, {len(marks)} markers")
    api = query(c, ["select name, start, end from regions order by start",
                    "select name, start, end from region order by start",
                    "select function, start, end from hip_api order by start"])
    bounds = [ks[m][2] for m in marks] + [ks[-1][2] + 1]
    for li in range(len(marks)):
        lo, hi = bounds[li], bounds[li + 1]
        rows = [r for r in ks if lo <= r[1] < hi]
        if not rows:
            continue
        t0, t1 = rows[0][1], max(r[2] for r in rows)
        busy, cs, ce = 0, rows[0][1], rows[0][2]
        gaps = []
        last = rows[0]
        for r in rows[1:]:
            if r[1] > ce:
                busy += ce - cs
                gaps.append((r[1] - ce, short(last[0]), short(r[0])))
                cs, ce, last = r[1], r[2], r
            elif r[2] > ce:
                ce, last = r[2], r
        busy += ce - cs
        per_stream = defaultdict(float)
        per_kernel = defaultdict(lambda: [0, 0.0])
        for r in rows:
            per_stream[r[3]] += (r[2] - r[1]) / 1e6
            per_kernel[short(r[0])][0] += 1
            per_kernel[short(r[0])][1] += (r[2] - r[1]) / 1e6
        print(f"\n== leg {li}: {len(rows)} kernels, span {(t1 - t0) / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, "
              f"idle {(t1 - t0 - busy) / 1e6:.1f} ms; kernel time per stream (ms): "
              + ", ".join(f"{s}: {v:.1f}" for s, v in sorted(per_stream.items())))
        gaps.sort(reverse=True)
        print(f"  largest idle gaps (of {len(gaps)}, sum {sum(g[0] for g in gaps) / 1e6:.1f} ms):")
        for g in gaps[:top]:
            print(f"    {g[0] / 1e3:9.1f} us  after {g[1]}  before {g[2]}")
        print("  kernels by total time (ms, calls, avg us):")
        for k, (n, t) in sorted(per_kernel.items(), key=lambda x: -x[1][1])[:top]:
            print(f"    {t:8.2f} {n:5d} {t / n * 1e3:9.1f}  {k}")
        if api:
            calls = defaultdict(lambda: [0, 0.0])
            for n, s, e in api:
                if lo <= s < hi:
                    calls[n][0] += 1
                    calls[n][1] += (e - s) / 1e6
            print("  HIP API calls in the window (ms total, calls):")
            for n, (k, t) in sorted(calls.items(), key=lambda x: -x[1][1])[:top]:
                print(f"    {t:9.2f} {k:6d}  {n[:70]}")


if __name__ == "__main__":
    main()
