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
CSRC = os.path.join(PKG_DIR, "csrc")
# Translation units of libgcg_spmm.so: SpMM kernels + planner, CSR utilities, graph build,
# SpGEMM, MFMA dense projection + softmax/xent, error/version helpers. Compiled in parallel, linked into one shared library.
SOURCES = [os.path.join(CSRC, f) for f in
           ("spmm.hip", "csr_ops.hip", "graph_build.hip", "spgemm.hip", "dense.hip", "errors.cpp")]
INTERNAL_HEADERS = [os.path.join(CSRC, h) for h in ("common.h", "index_kernels.h", "gemm_epilogue.inc")]
HEADER = os.path.join(REPO_DIR, "include", "gcg_spmm.h")
LIB = os.path.join(PKG_DIR, "libgcg_spmm.so")
ARCH = os.environ.get("GCG_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: every product and sum is rounded separately, as scipy's csr_matvecs does.
HIPCC_FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", f"--offload-arch={ARCH}",
               "-Wall", "-Wno-unused-command-line-argument"]
# Per-file extra flags. dense.hip: no SLP vectorizer (round 6) -- it packed the NT GEMM's
# epilogue (bias add, rectify) and fallback arithmetic into v_pk_add_f32 / v_pk_mul_f32, and a
# packed f32 op beside another workgroup's MFMAs on the same SIMD costs far more than its issue
# slot (MI355X_MICROARCH.md, "price of one filler beside MFMAs"): the bf16x6 projection 167 ->
# 183-185 TF, dP 167 -> 175 on one box, bitwise the same results (profiles/r06/dense_ab.jsonl).
FILE_FLAGS = {"dense.hip": ["-fno-slp-vectorize"]}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the graphconvgeo_amd native library cannot be built")


def source_hash() -> str:
    """Content hash of every file the library is built from (sources, headers, flags). Baked
    into the library (gcg_source_hash) so a stale binary is detected by content, not mtime
    (a snapshot copied to another machine does not keep mtimes reliably)."""
    import hashlib

    h = hashlib.sha256()
    for p in (*SOURCES, *INTERNAL_HEADERS, HEADER):
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read() + b"\0")
    h.update(" ".join(HIPCC_FLAGS).encode())
    for name in sorted(FILE_FLAGS):
        h.update((name + ":" + " ".join(FILE_FLAGS[name])).encode())
    return h.hexdigest()[:16]


HASH_FILE = LIB + ".hash"


def needs_build() -> bool:
    """True when the library is missing or was built from different sources. Decided by the
    content hash written next to the library after a successful link (the same hash the
    library bakes in and `_native._check_fresh` compares), never by mtime."""
    if not os.path.exists(LIB) or not os.path.exists(HASH_FILE):
        return True
    with open(HASH_FILE) as f:
        return f.read().strip() != source_hash()


def build_native(force: bool = False, verbose: bool = False) -> str:
    """Compile csrc/* for gfx950 and link libgcg_spmm.so (in-tree). Returns the path."""
    if not force and not needs_build():
        return LIB
    import concurrent.futures as cf
    import tempfile

    hipcc = _hipcc()
    digest = source_hash()
    with tempfile.TemporaryDirectory(prefix="gcg_build_") as tmpd:
        objs = [os.path.join(tmpd, os.path.basename(src) + ".o") for src in SOURCES]

        def compile_one(src_obj):
            src, obj = src_obj
            cmd = [hipcc, *HIPCC_FLAGS, *FILE_FLAGS.get(os.path.basename(src), []),
                   f'-DGCG_SOURCE_HASH="{digest}"', "-c", "-o", obj, src]
            if src.endswith(".cpp"):
                cmd = [hipcc, "-x", "hip", *cmd[1:]]
            if verbose:
                print(" ".join(cmd))
            return subprocess.run(cmd, capture_output=True, text=True), src

        workers = min(len(SOURCES), max(1, (os.cpu_count() or 2)), 8)
        with cf.ThreadPoolExecutor(max_workers=workers) as ex:
            for res, src in ex.map(compile_one, zip(SOURCES, objs)):
                if res.returncode != 0:
                    raise RuntimeError(f"hipcc failed on {src} ({res.returncode}):\n{res.stdout}\n{res.stderr}")
        tmp = LIB + ".tmp"
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp, *objs]
        if verbose:
            print(" ".join(cmd))
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, LIB)
        with open(HASH_FILE + ".tmp", "w") as f:
            f.write(digest + "\n")
        os.replace(HASH_FILE + ".tmp", HASH_FILE)
    return LIB


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
