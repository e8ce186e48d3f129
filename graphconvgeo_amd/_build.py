"""In-tree build of the native library (hipcc, gfx950) -- no JIT cache, no pip install.

The built `libgcg_spmm.so` lives next to this file so it travels with the repo
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
SRC = os.path.join(PKG_DIR, "csrc", "gcg_spmm.hip")
HEADER = os.path.join(REPO_DIR, "include", "gcg_spmm.h")
LIB = os.path.join(PKG_DIR, "libgcg_spmm.so")
ARCH = os.environ.get("GCG_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: every product and sum is rounded separately, as scipy's csr_matvecs does.
HIPCC_FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
               f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-command-line-argument"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the graphconvgeo_amd native library cannot be built")


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in (SRC, HEADER, __file__))


def build_native(force: bool = False, verbose: bool = False) -> str:
    """Compile csrc/gcg_spmm.hip into libgcg_spmm.so for gfx950. Returns the path."""
    if not force and not needs_build():
        return LIB
    tmp = LIB + ".tmp"
    cmd = [_hipcc(), *HIPCC_FLAGS, "-o", tmp, SRC]
    if verbose:
        print(" ".join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
