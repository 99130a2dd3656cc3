"""Per-kernel PMC totals from rocprofv3 rocpd databases: python tools/pmc.py <dir> [<dir> ...] [--match substr]"""
import glob
import re
import sqlite3
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    return re.sub(r"^void ", "", n)[:60]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    for a in sys.argv[1:]:
        if a.startswith("--match="):
            match = a.split("=", 1)[1]
    agg = {}
    for d in args:
        for db in glob.glob(d + "/**/*.db", recursive=True):
            c = sqlite3.connect(db)
            q = ("select kernel_name, counter_name, sum(value), count(distinct dispatch_id), sum(distinct duration) "
                 "from counters_collection group by kernel_name, counter_name")
            for kn, cn, v, nd, dur in c.execute(q):
                k = short(kn)
                if match and match not in k:
                    continue
                e = agg.setdefault(k, {})
                e[cn] = e.get(cn, 0) + v
                e["_dispatches"] = max(e.get("_dispatches", 0), nd)
    for k, e in agg.items():
        if "tw_" not in k and "tblock" not in k and not match:
            continue
        print(k)
        nd = e.pop("_dispatches")
        for cn in sorted(e):
            print(f"   {cn:28s} {e[cn] / nd:16.4g} per dispatch")


if __name__ == "__main__":
    main()
