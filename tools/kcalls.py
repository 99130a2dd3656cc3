"""Per-call durations, in launch order, of the kernels whose name contains a pattern (rocpd .db of a rocprofv3
kernel trace): python tools/kcalls.py <profile dir> <pattern> [last N calls]"""
import glob
import os
import re
import sqlite3
import sys


def main():
    d, pat = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    try:
        rows = list(c.execute("select name, start, end from kernels order by start"))
    except sqlite3.OperationalError:
        rows = list(c.execute("select kernel_name, start, end from kernels order by start"))
    sel = [(re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "")).replace("void ", "")[:90], (e - s) / 1e3)
           for n, s, e in rows if pat in n]
    for n, us in sel[-last:]:
        print(f"{us:10.1f} us  {n}")


if __name__ == "__main__":
    main()
