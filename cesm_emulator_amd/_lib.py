"""Loader for libcesm_hip.so.

The ctypes signatures are parsed from include/cesm_hip.h so the header stays the single
source of truth for the C ABI.  There is no fallback: if the library is missing or a symbol
is absent, importing the product path raises.
"""
from __future__ import annotations

import ctypes
import re
from pathlib import Path

PKG = Path(__file__).resolve().parent
HEADER = PKG.parent / "include" / "cesm_hip.h"
import os

# CESM_HIP_LIB selects a diagnostic build (tools/build_diag.sh); default: the in-tree product library
LIBPATH = Path(os.environ["CESM_HIP_LIB"]) if os.environ.get("CESM_HIP_LIB") else PKG / "libcesm_hip.so"

def header_abi_version(path: Path = HEADER) -> int:
    m = re.search(r"#define\s+CESM_ABI_VERSION\s+(\d+)", path.read_text())
    if not m:
        raise RuntimeError(f"{path}: no CESM_ABI_VERSION")
    return int(m.group(1))


_CTYPE = {"int": ctypes.c_int, "int64_t": ctypes.c_int64, "float": ctypes.c_float, "double": ctypes.c_double}


def parse_header(path: Path = HEADER):
    """Return {name: (restype, [argtypes])} for every `int cesm_*(...)` / `int64_t cesm_*(...)` /
    `const char* cesm_*(...)` declaration (the last two: host-only queries)."""
    text = path.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(int|int64_t|const\s+char\s*\*)\s*(cesm_\w+)\s*\(([^)]*)\)\s*;", text, flags=re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        types = []
        for a in args.split(","):
            a = " ".join(a.replace("const", " ").split())
            if not a or a == "void":
                continue
            if "*" in a or a.startswith("hipStream_t"):
                types.append(ctypes.c_void_p)
            else:
                base = a.rsplit(" ", 1)[0]
                types.append(_CTYPE[base])
        decls[name] = ({"int": ctypes.c_int, "int64_t": ctypes.c_int64}.get(ret, ctypes.c_char_p), types)
    return decls


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIBPATH.exists():
            raise RuntimeError(f"{LIBPATH} not built: run `python -m cesm_emulator_amd.build` "
                               "(the HIP path has no CPU/PyTorch fallback)")
        handle = ctypes.CDLL(str(LIBPATH))
        for name, (res, args) in parse_header().items():
            fn = getattr(handle, name)  # AttributeError -> missing export, fail loudly
            fn.restype = res
            fn.argtypes = args
        have, want = handle.cesm_abi_version(), header_abi_version()
        if have != want:
            raise RuntimeError(f"{LIBPATH} has C ABI version {have}, include/cesm_hip.h declares {want}: rebuild "
                               "the library (python -m cesm_emulator_amd.build)")
        _lib = handle
    return _lib


class KernelError(RuntimeError):
    pass


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise KernelError(f"{name} failed with code {rc}")
    return rc
