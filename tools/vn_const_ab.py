"""bench.py with module constants of cesm_emulator_amd.video_net overridden (whole-step A/B of host-side dispatch
choices, run in a fresh process per arm): python tools/vn_const_ab.py NAME=VALUE[,NAME=VALUE] [bench args...]
Prints 'NAME=VALUE,... value ms_per_step'."""
import ast
import json
import os
import runpy
import sys
import io
import contextlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cesm_emulator_amd.video_net as V  # noqa: E402

if __name__ == "__main__":
    spec = sys.argv[1]
    for kv in filter(None, spec.split(",")):
        if kv == "-":  # the default arm
            continue
        k, v = kv.split("=", 1)
        assert hasattr(V, k), k
        setattr(V, k, ast.literal_eval(v))
    sys.argv = ["bench.py"] + sys.argv[2:]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"),
                       run_name="__main__")
    d = json.loads(buf.getvalue().strip().splitlines()[-1])
    print(spec, d["value"], d["ms_per_step"], flush=True)
