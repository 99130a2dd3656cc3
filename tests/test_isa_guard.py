"""Build-time ISA guard for the RoPE sources (DESIGN §6b "The RoPE-epilogue repeatability").

With the SLP vectorizer on, the RoPE epilogues of tblock.hip / tflash.hip / attn.hip are lowered to packed fp32
(v_pk_{fma,mul,add}_f32) and gave run-to-run different q / k on gfx950; build.py compiles those three sources with
-fno-slp-vectorize.  This test reads the device code of the BUILT library (the gfx950 code objects inside its
offload bundles) and fails if packed-fp32 VALU shows up in their kernels again -- i.e. if the flag is dropped, or a
new kernel in these files is written with explicit packed math.  Measured (hipcc -S of each source): tblock 4658 /
tflash 2906 / attn 2485 packed-fp32 instructions with SLP, 183 / 0 / 0 without (tblock's 183 are explicit vector
code in tw_fwd / tw_bwd, not the RoPE epilogues).  Round 4 adds explicit packed math to the softmax-gradient step of
twh_bwd and tflash_bwd_kv, away from the RoPE code; those kernels get their own allowance and the repeatability tests
(test_gpu_determinism, the full-grid F = 120 two-step test) cover them.  CPU only: no GPU
needed, skipped if the library is not built.
"""
import os
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = Path(os.environ.get("CESM_ISA_GUARD_LIB", ROOT / "cesm_emulator_amd" / "libcesm_hip.so"))  # override: a lib to audit
OBJDUMP = Path("/opt/rocm/llvm/bin/llvm-objdump")
PK = re.compile(r"\bv_pk_(?:fma|mul|add)_f32\b")
FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")
# kernel-name markers of the three NO_SLP sources -> max packed-fp32 instructions over that source's kernels
LIMITS = {"tblock": (re.compile(r"tw_fwd_kernel|tw_bwd_kernel|tblock_\w+_kernel"), 400),
          "twh": (re.compile(r"twh_bwd_kernel"), 3 * 40),  # packed softmax gradient: 3 instantiations (NV 1-3) x <= 40
          "tflash": (re.compile(r"tflash_(?!bwd_kv_)\w+_kernel"), 0),
          "tflash_kv": (re.compile(r"tflash_bwd_kv_kernel"), 80),  # packed softmax gradient: 1 instantiation x <= 80
          "attn": (re.compile(r"tattn_\w+_kernel|rope_table_kernel"), 0)}


def _device_disassembly(tmp_path):
    lib = tmp_path / LIB.name
    shutil.copy(LIB, lib)
    subprocess.run([str(OBJDUMP), "--offloading", lib.name], cwd=tmp_path, check=True, capture_output=True)
    cos = sorted(tmp_path.glob(lib.name + ".*.hipv4-amdgcn-amd-amdhsa--gfx950"))
    assert cos, "no gfx950 code objects in the library"
    for co in cos:
        yield subprocess.run([str(OBJDUMP), "-d", "--no-show-raw-insn", str(co)], check=True, capture_output=True,
                             text=True).stdout


@pytest.mark.skipif(not LIB.exists() or not OBJDUMP.exists(), reason="library not built / no llvm-objdump")
def test_rope_sources_have_no_packed_fp32(tmp_path):
    counts = {k: 0 for k in LIMITS}
    seen = {k: 0 for k in LIMITS}
    for text in _device_disassembly(tmp_path):
        cur = None
        for line in text.splitlines():
            m = FUNC.match(line)
            if m:
                cur = None
                for k, (pat, _) in LIMITS.items():
                    if pat.search(m.group(1)):
                        cur = k
                        seen[k] += 1
                continue
            if cur is not None and PK.search(line):
                counts[cur] += 1
    for k, (_, lim) in LIMITS.items():
        assert seen[k] > 0, f"no {k} kernels found in the library"
        assert counts[k] <= lim, f"{k}: {counts[k]} packed-fp32 instructions (limit {lim}): built without -fno-slp-vectorize?"
