"""Instruction histogram of one kernel in a device .s: python tools/isa_hist.py file.s substr [top]"""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
key = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
names = [l.split(":")[0] for l in s.split("\n") if key in l and not l.startswith((".", "\t")) and ":" in l]
name = names[0]
i = s.index("\n" + name + ":")
j = s.index(".Lfunc_end", i)
c = Counter()
n = 0
for l in s[i:j].split("\n"):
    l = l.strip()
    if not l or l.startswith((".", ";", "_")) or l.endswith(":"):
        continue
    c[l.split()[0]] += 1
    n += 1
print(name, n, "instructions (static)")
for k, v in c.most_common(top):
    print(f"{v:5d} {k}")
