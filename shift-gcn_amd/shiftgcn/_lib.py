"""Loader for the in-tree gfx950 HIP library (``libshiftgcn_hip.so``) behind
``include/shiftgcn.h``.

The product path has NO CPU or eager fallback: if the library is missing, or a tensor
is not on a ROCm device, calls raise. ``torch`` is imported first so that the HIP
runtime it already loaded (soname ``libamdhip64.so.7``) is the one the library binds to.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen: one HIP runtime per process)

LIB_NAME = "libshiftgcn_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# same-box A/B of two builds (tuning only, e.g. tools/ab_lib.sh): another in-tree build of
# the same ABI
LIB_PATH = os.environ.get("SGCN_LIB_PATH", LIB_PATH)
ABI_VERSION = 23
BATCH_MAX = 32            # include/shiftgcn.h SGCN_BATCH_MAX
ABI_DIAG_FLAG = 0x10000   # include/shiftgcn.h SGCN_ABI_DIAG_FLAG: a diagnostic build
EINVAL = -22

_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_Z = ctypes.c_size_t
_L = ctypes.c_longlong

# name -> (restype, argtypes); mirrors include/shiftgcn.h
SIGNATURES = {
    "sgcn_abi_version": (_I, []),
    "sgcn_sgd_chunk_elems": (_I, []),
    "sgcn_sgd_step": (_I, [_P, _P, _P, _I, _F, _I, _P]),
    "sgcn_tshift_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "sgcn_tshift_fwd_pre": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I,
                                 _I, _I, _P]),
    "sgcn_tshift_fwd_tail": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I,
                                  _I, _I, _P]),
    "sgcn_tshift_bwd_ws_bytes": (_Z, [_I, _I]),
    "sgcn_tshift_pos_finalize": (_I, [_P, _I, _I, _P, _P, _P]),
    "sgcn_tshift_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _Z, _I,
                             _I, _I, _I, _I, _I, _P]),
    "sgcn_tshift_fwd_f64": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "sgcn_tshift_bwd_f64_ws_bytes": (_Z, [_I, _I]),
    "sgcn_tshift_bwd_f64": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _I,
                                 _P]),
    "sgcn_pw_fwd": (_I, [_P, _I, _P, _P, _L, _L, _I, _I, _P, _P, _L, _L, _I, _I, _I, _I, _I,
                         _I, _I, _I, _I, _P]),
    "sgcn_pw_tshift_ws_bytes": (_Z, [_I]),
    "sgcn_pw_fwd_tshift": (_I, [_P, _P, _P, _L, _L, _P, _P, _P, _P, _P, _P, _Z, _P, _L, _L, _I,
                                _I, _I, _I, _I, _I, _I, _P]),
    "sgcn_pw_dw_ws_bytes": (_Z, [_I, _I, _I, _I, _I]),
    "sgcn_pw_dw": (_I, [_P, _L, _L, _I, _I, _P, _L, _L, _I, _I, _P, _P, _I, _I, _P, _I, _P, _Z,
                        _I, _I, _I, _I, _I, _P]),
    "sgcn_moments_ws_bytes": (_Z, [_I, _I, _I, _I]),
    "sgcn_moments": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "sgcn_bn_finalize": (_I, [_P, _I, _I, _I, _I, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P,
                              _P]),
    "sgcn_bn_eval_coef": (_I, [_I, _I, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P]),
    "sgcn_bn_apply": (_I, [_P, _P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I,
                           _P]),
    "sgcn_bn_bwd_reduce": (_I, [_P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I,
                                _I, _P]),
    "sgcn_bn_bwd_finalize": (_I, [_P, _I, _I, _L, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P]),
    "sgcn_bn_bwd_apply": (_I, [_P, _P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I,
                               _P]),
    "sgcn_mask_prep": (_I, [_P, _P, _I, _P]),
    "sgcn_gcn_gather": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "sgcn_gcn_dx_finish": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I,
                                _P]),
    "sgcn_tshift_bwd_bnin": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I,
                                  _I, _I, _P]),
    "sgcn_mask_grad_finalize": (_I, [_P, _P, _I, _I, _I, _P, _I, _P]),
    "sgcn_modalities": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "sgcn_tshift_bwd_gbn": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                 _P, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _P]),
    "sgcn_bn_bwd_finalize_gbn": (_I, [_P, _I, _I, _I, _L, _P, _P, _P, _P, _P, _P, _P, _I, _I,
                                      _P, _P]),
    "sgcn_head_ws_bytes": (_Z, [_I, _I, _I, _I]),
    "sgcn_head_moments": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "sgcn_head_apply": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "sgcn_head_bwd_reduce": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "sgcn_head_bwd_apply": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "sgcn_pool": (_I, [_P, _P, _I, _I, _I, _L, _P]),
    "sgcn_pool_bwd": (_I, [_P, _P, _I, _I, _I, _L, _P]),
    "sgcn_tshift_pos_finalize_many": (_I, [_P, _P, _P, _P, _P, _I, _P]),
    "sgcn_mask_prep_many": (_I, [_P, _P, _P, _I, _P]),
    "sgcn_mask_grad_finalize_many": (_I, [_P, _P, _P, _P, _P, _P, _I, _P]),
}


class NativeLibraryError(RuntimeError):
    pass


def _open(path):
    """dlopen ``path``, check its ABI (refusing a diagnostic build), bind the signatures."""
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    lib.sgcn_abi_version.restype = _I
    lib.sgcn_abi_version.argtypes = []
    abi = lib.sgcn_abi_version()
    if abi & ABI_DIAG_FLAG:
        # timing probes that drop loads or stores (results are wrong): tools/ only
        if os.environ.get("SGCN_ALLOW_DIAG_LIB") != "1" or os.path.basename(path) == LIB_NAME:
            raise NativeLibraryError(
                f"{path} is a DIAGNOSTIC build (SGCN_PW_DIAG / SGCN_PW_STAMPS / SGCN_DIAG_*: "
                "its results are wrong); rebuild with `make -C shift-gcn_amd/csrc`")
        abi &= ~ABI_DIAG_FLAG
    if abi != ABI_VERSION:
        raise NativeLibraryError(f"{path}: ABI version {abi} != {ABI_VERSION}; rebuild it")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def load():
    """Return the loaded ctypes library; raise NativeLibraryError when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (or `make -C shift-gcn_amd/csrc`). There is no CPU fallback.")
    _lib = _open(LIB_PATH)
    return _lib


def check(rc: int, name: str) -> None:
    if rc == 0:
        return
    if rc == EINVAL:
        raise ValueError(f"{name}: invalid argument (shape/pointer/stride)")
    raise RuntimeError(f"{name}: HIP error {rc}")
