"""Summarise a rocprofv3 kernel trace (rocpd .db or *_kernel_stats.csv) as per-kernel totals.
usage: python tools/kstats.py <profile dir> [steps] [top]"""
import csv
import glob
import os
import re
import sqlite3
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:90]


def rows_from(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if dbs:
        c = sqlite3.connect(dbs[0])
        q = "select name, count(*), sum(duration) from kernels group by name"
        try:
            return [(n, k, t / 1e3) for n, k, t in c.execute(q)]
        except sqlite3.OperationalError:
            q = "select kernel_name, count(*), sum(end - start) from kernels group by kernel_name"
            return [(n, k, t / 1e3) for n, k, t in c.execute(q)]
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    out = []
    for r in csv.DictReader(open(f)):
        out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3))
    return out


def main():
    d = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    agg = {}
    for n, k, us in rows_from(d):
        s = short(n)
        a = agg.setdefault(s, [0, 0.0])
        a[0] += k
        a[1] += us
    tot = sum(v[1] for v in agg.values())
    print(f"total {tot / 1e3:.1f} ms  ({tot / 1e3 / steps:.1f} ms per step over {steps:g} steps)")
    print(f"{'ms/step':>8} {'%':>5} {'calls':>7} {'avg us':>8}  kernel")
    for s, (k, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{us / 1e3 / steps:8.2f} {100 * us / tot:5.1f} {k:7d} {us / k:8.1f}  {s}")


if __name__ == "__main__":
    main()
