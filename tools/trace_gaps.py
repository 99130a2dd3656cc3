"""Busy vs idle time of a rocprofv3 kernel trace (rocpd .db): the union of kernel intervals over the traced span,
the largest idle gaps (with the kernels on either side) and per-kernel totals, so a slow step can be split into
"kernels got slower" and "the GPU sat idle".  usage: python tools/trace_gaps.py <profile dir> [top]"""
import glob
import os
import re
import sqlite3
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name)[:80]


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    try:
        rows = list(c.execute("select name, start, end, stream_id from kernels order by start"))
    except sqlite3.OperationalError:
        try:
            rows = list(c.execute("select kernel_name, start, end, stream_id from kernels order by start"))
        except sqlite3.OperationalError:
            rows = [(n, s, e, 0) for n, s, e in c.execute("select kernel_name, start, end from kernels order by start")]
    if not rows:
        print("no kernels")
        return
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    busy, cur_s, cur_e = 0, rows[0][1], rows[0][2]
    gaps = []
    prev = rows[0]
    last_end_kernel = rows[0]
    for r in rows[1:]:
        if r[1] > cur_e:
            busy += cur_e - cur_s
            gaps.append((r[1] - cur_e, short(last_end_kernel[0]), short(r[0])))
            cur_s, cur_e = r[1], r[2]
            last_end_kernel = r
        elif r[2] > cur_e:
            cur_e = r[2]
            last_end_kernel = r
        prev = r
    busy += cur_e - cur_s
    span = t1 - t0
    print(f"{len(rows)} kernels, span {span / 1e6:.1f} ms, busy (union) {busy / 1e6:.1f} ms, "
          f"idle {(span - busy) / 1e6:.1f} ms, sum of durations {sum(r[2] - r[1] for r in rows) / 1e6:.1f} ms")
    streams = {}
    for r in rows:
        streams.setdefault(r[3], [0, 0])
        streams[r[3]][0] += 1
        streams[r[3]][1] += r[2] - r[1]
    for s, (n, t) in sorted(streams.items()):
        print(f"  stream {s}: {n} kernels, {t / 1e6:.1f} ms")
    gaps.sort(reverse=True)
    print(f"largest idle gaps (of {len(gaps)}; sum {sum(g[0] for g in gaps) / 1e6:.1f} ms):")
    for g in gaps[:top]:
        print(f"  {g[0] / 1e3:9.1f} us  after {g[1]}  before {g[2]}")
    tot = {}
    for r in rows:
        k = short(r[0])
        tot.setdefault(k, [0, 0])
        tot[k][0] += 1
        tot[k][1] += r[2] - r[1]
    print("per kernel (ms total, calls, avg us):")
    for k, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {t / 1e6:9.2f} {n:6d} {t / n / 1e3:9.1f}  {k}")


if __name__ == "__main__":
    main()
