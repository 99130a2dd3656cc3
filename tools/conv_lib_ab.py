"""3x3 conv A/B between two libraries: every bench-step shape (tools/ws_check.py's list) under the default dispatch,
run once per library (CESM_HIP_LIB), outputs compared bit for bit and launches timed.

  python tools/conv_lib_ab.py cesm_emulator_amd/libcesm_hip.so cesm_emulator_amd/libcesm_hip_<variant>.so
"""
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    libs = sys.argv[1:3]
    outs = []
    for i, lib in enumerate(libs):
        path = f"/tmp/conv_lib_ab_{i}.pt"
        env = dict(os.environ, CESM_HIP_LIB=lib)
        r = subprocess.run([sys.executable, os.path.join(HERE, "ws_check.py"), "--run", path], env=env, timeout=600)
        if r.returncode != 0:
            sys.exit(f"run {lib} failed: {r.returncode}")
        outs.append(torch.load(path, weights_only=False))  # written by ws_check.run above
    ok = True
    for k in outs[0]:
        a, b = outs[0][k], outs[1][k]
        eq = bool((a["y"] == b["y"]).all()) and bool((a["yr"] == b["yr"]).all())
        if a["gn"] is not None:
            eq = eq and bool((a["gn"][0] == b["gn"][0]).all()) and bool((a["gn"][1] == b["gn"][1]).all())
        ok = ok and eq and a["var"] == b["var"]
        print(f"{k}: {a['var']} {a['us']:.1f} us -> {b['us']:.1f} us ({a['us'] / b['us']:.3f}x); "
              f"outputs {'bit-equal' if eq else 'DIFFER'}")
    print("CONV LIB AB", "PASS" if ok else "FAIL")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
