"""Per-kernel HBM bytes per launch of the bench step from two rocprofv3 PMC passes over tools/step_pmc.py
(FETCH_SIZE, WRITE_SIZE), written as the JSON bench.py reads (profiles/step_traffic.json).

Calibration (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a wide coalesced
streaming read on gfx950 and the counter unit is not bytes; the workload ends with one device copy of a
known byte count N (read N, write N, past the Infinity Cache) whose counters give the counter->byte
factors applied to every kernel.  The first (warm-up) step's dispatches are excluded.
usage: python tools/step_traffic.py <pmc_fetch_dir> <pmc_write_dir> <batch> <frames> <config> <steps>"""
import glob
import json
import re
import sqlite3
import sys

COPY_BYTES = 1 << 30


def demangle(name):
    """minimal Itanium demangler for this library's kernels (binutils' c++filt rejects the DF16b bf16 type):
    [_ZN12_GLOBAL__N_1]<len><name>[I<template args>E]... -> name<args>; args: Li<n>E, Lb0E / Lb1E, DF16b, f"""
    m = re.match(r"_ZN?(?:12_GLOBAL__N_1)?(\d+)", name)
    if not m:
        return name
    n = int(m.group(1))
    base = name[m.end():m.end() + n]
    rest = name[m.end() + n:]
    if not rest.startswith("I"):
        return base
    args, i = [], 1
    while i < len(rest) and rest[i] != "E":
        t = re.match(r"L([ib])(\d+)E|DF16b|f|i|b", rest[i:])
        if not t:
            break
        tok = t.group(0)
        if tok.startswith("L"):
            args.append(("true" if t.group(2) == "1" else "false") if t.group(1) == "b" else t.group(2))
        else:
            args.append({"DF16b": "__bf16", "f": "float", "i": "int", "b": "bool"}[tok])
        i += len(tok)
    return f"{base}<{','.join(args)}>"


def norm(name):
    """demangled kernel name without namespace / parameters / spaces: tw_bwd_kernel<64,3>"""
    if name.startswith("_Z"):
        name = demangle(name)
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:  # cut the parameter list (first '(' outside template brackets)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out).replace(" ", "")


def per_dispatch(d, counter):
    rows = []
    for db in glob.glob(d + "/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        q = ("select kernel_name, dispatch_id, sum(value) from counters_collection "
             "where counter_name = ? group by dispatch_id order by dispatch_id")
        rows += [(k, v) for k, _, v in c.execute(q, (counter,))]
    return rows


def main():
    fd, wd, B, F, cfg, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], int(sys.argv[6])
    res, cache = {}, {}
    for d, cn in ((fd, "FETCH_SIZE"), (wd, "WRITE_SIZE")):
        rows = per_dispatch(d, cn)
        copy = [i for i, (k, _) in enumerate(rows) if "elementwise" in k.lower() or "copy" in k.lower()]
        if not copy:
            raise SystemExit(f"{cn}: no calibration copy dispatch")
        factor = COPY_BYTES / rows[copy[-1]][1]
        work = rows[:copy[-1]]
        # drop the warm-up step: the optimizer's adamw_kernel closes every step
        ends = [i for i, (k, _) in enumerate(work) if "adamw_kernel" in k]
        if len(ends) >= steps + 1:
            work = work[ends[-steps - 1] + 1:ends[-1] + 1]
        for k, v in work:
            n = cache.setdefault(k, norm(k))
            e = res.setdefault(n, {"dispatches": 0, "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0})
            if cn == "FETCH_SIZE":
                e["dispatches"] += 1
            e[cn] += v * factor
        res.setdefault("_calibration", {})[cn] = {"copy_counter": rows[copy[-1]][1], "bytes_per_unit": factor}
    cal = res.pop("_calibration")
    kernels = {}
    for n, e in res.items():
        if e["dispatches"]:
            fb, wb = e["FETCH_SIZE"] / e["dispatches"], e["WRITE_SIZE"] / e["dispatches"]
            kernels[n] = {"bytes_per_launch": fb + wb, "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                          "launches_per_step": e["dispatches"] / steps}
    print(json.dumps({"batch": B, "frames": F, "config": cfg, "steps": steps, "calibration": cal,
                      "kernels": dict(sorted(kernels.items(), key=lambda kv: -kv[1]["bytes_per_launch"]
                                             * kv[1]["launches_per_step"]))}, indent=1))


if __name__ == "__main__":
    main()
