#!/usr/bin/env python
"""Build a variant of libgcg_spmm.so for a library A/B on the GPU box (loaded through GCG_LIB):
the csrc tree copied to a temp dir, optional text patches applied (a JSON list of
[file, old, new]), extra -D flags, output wherever asked (tools/varlibs/ travels with gpurun).

  python tools/build_variant.py tools/varlibs/libgcg_x.so [-D FOO] [--patch patches.json]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import _build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--patch", default=None)
    ap.add_argument("--flag", action="append", default=[], help="extra hipcc flag (every TU)")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory(prefix="gcg_var_") as tmpd:
        csrc = os.path.join(tmpd, "pkg", "csrc")  # common.h includes ../../include/gcg_spmm.h
        shutil.copytree(_build.CSRC, csrc)
        os.makedirs(os.path.join(tmpd, "include"))
        shutil.copy(_build.HEADER, os.path.join(tmpd, "include", "gcg_spmm.h"))
        if a.patch:
            for fn, old, new in json.load(open(a.patch)):
                p = os.path.join(csrc, fn)
                s = open(p).read()
                if old not in s:
                    raise SystemExit(f"patch text not found in {fn}: {old[:80]!r}")
                open(p, "w").write(s.replace(old, new))
        objs = []
        flags = [*_build.HIPCC_FLAGS, f'-DGCG_SOURCE_HASH="variant"', *[f"-D{d}" for d in a.D], *a.flag]
        procs = []
        for src in _build.SOURCES:
            name = os.path.basename(src)
            obj = os.path.join(tmpd, name + ".o")
            cmd = [_build._hipcc(), *flags, *_build.FILE_FLAGS.get(name, []), "-c", "-o", obj,
                   os.path.join(csrc, name)]
            if name.endswith(".cpp"):
                cmd = [cmd[0], "-x", "hip", *cmd[1:]]
            procs.append(subprocess.Popen(cmd))
            objs.append(obj)
        if any(p.wait() != 0 for p in procs):
            raise SystemExit("compile failed")
        subprocess.run([_build._hipcc(), "-shared", "-fPIC", f"--offload-arch={_build.ARCH}", "-o",
                        a.out, *objs], check=True)
    print(a.out)


if __name__ == "__main__":
    main()
