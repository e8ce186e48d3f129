"""A plain C caller of the C-ABI on the GPU (tests/c/abi_gpu_consumer.c): hipMalloc'd CSR and
dense operand, gcg_spmm_csr_f32 / plan + _planned / the gate form on a stream, bitwise against
the csr_matvecs loop in C -- the binding a C, cgo or JNI consumer of include/gcg_spmm.h uses
(INTEGRATION.md), with no Python or torch between it and the kernels."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_caller_on_gpu(native_lib, tmp_path):
    from graphconvgeo_amd import _native
    lib = _native.lib_path()
    exe = tmp_path / "abi_gpu_consumer"
    src = os.path.join(ROOT, "tests", "c", "abi_gpu_consumer.c")
    subprocess.run(["gcc", "-std=c99", "-O2", "-ffp-contract=off", "-Wall", "-Werror",
                    "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I", os.path.join(ROOT, "include"), src, lib, "-L/opt/rocm/lib",
                    "-lamdhip64", "-lm", "-Wl,-rpath,/opt/rocm/lib",
                    f"-Wl,-rpath,{os.path.dirname(lib)}", "-o", str(exe)], check=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, (res.returncode, res.stdout, res.stderr)
    assert "gpu abi ok" in res.stdout
