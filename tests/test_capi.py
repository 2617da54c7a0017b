"""C-ABI library: loads, exports every symbol declared in include/shiftgcn.h, rejects bad
arguments without touching the GPU (CPU-only checks)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "shiftgcn.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sgcn_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "sgcn_tshift_fwd" in syms and "sgcn_tshift_bwd" in syms
    assert len(syms) >= 4


def test_library_exports_every_declared_symbol():
    from shiftgcn import _lib
    lib = _lib.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert set(declared_symbols()) <= set(_lib.SIGNATURES), "ctypes signatures out of date"
    assert lib.sgcn_abi_version() == _lib.ABI_VERSION


def test_invalid_arguments_rejected_before_launch():
    from shiftgcn import _lib
    lib = _lib.load()
    # NULL pointers / bad stride / mismatched affine: EINVAL, nothing enqueued
    assert lib.sgcn_tshift_fwd(None, None, None, None, None, None, None, 2, 3, 4, 5, 1, 1,
                               None) == _lib.EINVAL
    assert lib.sgcn_tshift_fwd(None, None, None, None, None, None, None, 2, 3, 4, 5, 0, 1,
                               None) == _lib.EINVAL
    assert lib.sgcn_tshift_bwd(None, None, None, None, None, None, 0, None, None, None, None,
                               None, None, None, 0, 2, 3, 4, 5, 3, 1, None) == _lib.EINVAL
    assert lib.sgcn_tshift_bwd_ws_bytes(4, 8) == 4 * 8 * 8


def test_cpu_tensor_raises_like_reference():
    import torch
    from shiftgcn import ShiftFunction
    x = torch.zeros(1, 2, 4, 3)
    p = torch.zeros(2)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        ShiftFunction.apply(x, p, p, 1)


DIAG_MACROS = ["-DSGCN_PW_DIAG=1", "-DSGCN_PW_STAMPS", "-DSGCN_DIAG_X1B_BOUND=128",
               "-DSGCN_DIAG_F2_BOUND", "-DSGCN_DIAG_F1B_BOUND", "-DSGCN_DIAG_F1B_REAL",
               "-DSGCN_DIAG_DW64_SKIP"]


@pytest.mark.parametrize("flag", DIAG_MACROS)
def test_product_build_refuses_diagnostic_macros(flag):
    """`make` cannot produce libshiftgcn_hip.so with a wrong-result diagnostic macro, whether
    it comes in through HIPCC (as tools/ab_variant.sh passes flags) or EXTRA."""
    import subprocess
    csrc = os.path.join(REPO, "shift-gcn_amd", "csrc")
    for var in (f"HIPCC=/opt/rocm/bin/hipcc {flag}", f"EXTRA={flag}"):
        r = subprocess.run(["make", "-n", "-C", csrc, var], capture_output=True, text=True)
        assert r.returncode != 0 and "make diag" in r.stderr, (var, r.stderr)


def test_loader_refuses_a_diagnostic_library(tmp_path):
    """A library built with a diagnostic macro reports SGCN_ABI_DIAG_FLAG in
    sgcn_abi_version(), and the loader refuses it (checked before any other symbol)."""
    import shutil
    import subprocess
    from shiftgcn import _lib
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not installed")
    src = os.path.join(REPO, "shift-gcn_amd", "csrc", "version.hip")
    out = tmp_path / "libshiftgcn_hip.so"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O1", "-std=c++17", "-fPIC", "-shared",
                    "-DSGCN_PW_DIAG=1", src, "-o", str(out)], check=True)
    lib = ctypes.CDLL(str(out))
    assert lib.sgcn_abi_version() == _lib.ABI_VERSION | _lib.ABI_DIAG_FLAG
    with pytest.raises(_lib.NativeLibraryError, match="DIAGNOSTIC"):
        _lib._open(str(out))
    # a renamed copy is refused too unless a tool opts in explicitly
    other = tmp_path / "libshiftgcn_hip_probe.so"
    shutil.copy(out, other)
    with pytest.raises(_lib.NativeLibraryError, match="DIAGNOSTIC"):
        _lib._open(str(other))
