"""Straight-line scan of MFMA result -> dependent-read distances in a kernel's device assembly.

For every instruction that reads a VGPR / AGPR written by an earlier MFMA (other than a following MFMA taking it as
its exact SrcC accumulator), the number of wait states between the MFMA and the read (1 per instruction issued,
N + 1 per s_nop N) is recorded.  The per-opcode minimum of a build whose output is repeatable gives the distances the
compiler's hazard recognizer keeps; a build that shows shorter distances for some reader is the suspect.  Branches are
ignored (text order), so loop back edges are not followed.

  python tools/mfma_hazard_scan.py kernel.s twh_bwd_kernelILi3 [max_ws]
"""
import re
import sys
from collections import defaultdict

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(tok):
    out = []
    for m in REG.finditer(tok):
        k = m.group(1)
        if m.group(4) is not None:
            out.append((k, int(m.group(4))))
        else:
            out += [(k, i) for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    return out


def body_of(path, pat):
    cur = None
    out = []
    for line in open(path):
        m = re.match(r"^(\S+):\s+; @", line)
        if m:
            cur = m.group(1) if pat in m.group(1) else None
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            break
        out.append(line.split(";")[0].strip())
    return out


NOSTORE = ("global_store", "buffer_store", "ds_write", "ds_store", "flat_store", "scratch_store", "s_")


def scan(lines, max_ws):
    t = 0
    last = {}  # reg -> (time of MFMA issue, mfma text)
    mins = defaultdict(lambda: (10 ** 9, ""))
    for ln in lines:
        if not ln or ln.endswith(":") or ln.startswith("."):
            continue
        op, _, rest = ln.partition(" ")
        ops = [o.strip() for o in rest.split(",")] if rest else []
        if op == "s_nop":
            t += int(ops[0], 0) + 1
            continue
        t += 1
        is_mfma = op.startswith("v_mfma")
        if op.startswith(NOSTORE):
            defs, uses = [], ops
        else:
            defs, uses = ops[:1], ops[1:]
        if is_mfma:
            src_c = set(regs(uses[2])) if len(uses) > 2 else set()
            d = set(regs(defs[0]))
            for i, o in enumerate(uses[:2]):
                for r in regs(o):
                    if r in last:
                        dist = t - last[r][0]
                        key = "mfma-srcAB"
                        if dist < mins[key][0]:
                            mins[key] = (dist, f"{last[r][1]}  ->  {ln}")
            for r in src_c:
                if r in last and not (src_c == d):
                    dist = t - last[r][0]
                    if dist < mins["mfma-srcC(non-acc)"][0]:
                        mins["mfma-srcC(non-acc)"] = (dist, f"{last[r][1]}  ->  {ln}")
            for r in d:
                last[r] = (t, ln)
            continue
        for o in uses:
            for r in regs(o):
                if r in last:
                    dist = t - last[r][0]
                    if dist <= max_ws and dist < mins[op][0]:
                        mins[op] = (dist, f"{last[r][1]}  ->  {ln}")
        for o in defs:
            for r in regs(o):
                last.pop(r, None)
    return mins


if __name__ == "__main__":
    path, pat = sys.argv[1], sys.argv[2]
    max_ws = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    mins = scan(body_of(path, pat), max_ws)
    for op, (d, ex) in sorted(mins.items(), key=lambda kv: kv[1][0]):
        print(f"{d:4d}  {op:28s} {ex[:200]}")
