"""Per-kernel MFMA / LDS-wait statistics from hipcc --save-temps assembly: how many MFMAs issue right after an
`s_waitcnt lgkmcnt(0..1)` (the MFMA waits on an LDS read issued just before it: exposed LDS latency).
usage: python tools/isa_waits.py file.s [...]"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\w+):", text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        yield name, text[m.end():end]


def main():
    rows = []
    for path in sys.argv[1:]:
        for name, body in kernels(open(path).read()):
            ins = [l.strip() for l in body.split("\n")]
            ins = [l for l in ins if l and not l.startswith((";", "."))]
            n_mfma = exposed = 0
            recent_wait = 99
            for l in ins:
                if l.startswith("s_waitcnt") and re.search(r"lgkmcnt\([01]\)", l):
                    recent_wait = 0
                elif l.startswith("v_mfma"):
                    n_mfma += 1
                    if recent_wait <= 2:
                        exposed += 1
                    recent_wait = 99
                else:
                    recent_wait += 1
            if n_mfma:
                rows.append((exposed / n_mfma, n_mfma, exposed, name[:90]))
    for r in sorted(rows, reverse=True):
        print(f"{r[0]:5.2f} {r[1]:6d} {r[2]:6d}  {r[3]}")


if __name__ == "__main__":
    main()
