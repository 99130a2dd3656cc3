"""Compare tools/conv_ab.sh output: per-shape ms of each library (mean over repetitions), sorted by default ms.
usage: python tools/conv_ab_cmp.py gpurun_out/<tag>_conv.txt [min_ms]"""
import collections
import re
import sys

path = sys.argv[1]
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
cur = None
data = collections.defaultdict(lambda: collections.defaultdict(list))
tot = collections.defaultdict(list)
for line in open(path):
    m = re.match(r"== (\S+)", line)
    if m:
        cur = m.group(1)
        continue
    m = re.match(r"conv total ([\d.]+) ms", line)
    if m and cur:
        tot[cur].append(float(m.group(1)))
        continue
    m = re.match(r"\s*([\d.]+) ms\s+(\d+)x\s+[\d.]+ TF/s\s+(\S+)\s+(.*)$", line)
    if m and cur:
        data[(m.group(3), m.group(4).strip())][cur].append(float(m.group(1)))
libs = list(tot)
print("total", {k: round(sum(v) / len(v), 2) for k, v in tot.items()})
rows = []
for key, d in data.items():
    means = {k: sum(v) / len(v) for k, v in d.items()}
    if means.get(libs[0], 0) >= mn:
        rows.append((means.get(libs[0], 0), key, means))
for ms, key, means in sorted(rows, reverse=True):
    print(f"{key[0]:5s} {key[1]:45s} " + "  ".join(f"{lib} {means.get(lib, float('nan')):.3f}" for lib in libs))
