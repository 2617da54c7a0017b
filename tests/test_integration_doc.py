"""INTEGRATION.md §3 is executable: the ctypes binding a maintainer would add on the
reference's Python side (replacing ``shift_cuda``, ``shift_cuda.cpp:19-47``).

CPU: the snippet's argtypes/restypes equal the library table in ``shiftgcn/_lib.py``
(itself checked against the exported symbols by ``tests/test_capi.py``).
GPU: the snippet's ``forward``/``backward`` run against the library and match
``shiftgcn.shift_cuda`` bit for bit (stride 1 and 2).
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO

DOC = os.path.join(REPO, "INTEGRATION.md")
LIB = os.path.join(REPO, "shift-gcn_amd", "shiftgcn", "libshiftgcn_hip.so")


def _snippet():
    text = open(DOC).read()
    sec = text[text.index("## 3."):text.index("## 4.")]
    blocks = re.findall(r"```python\n(.*?)```", sec, re.S)
    assert len(blocks) == 1, "INTEGRATION.md §3 must hold exactly one python block"
    return blocks[0]


def _exec_snippet():
    code = _snippet().replace('"shift-gcn_amd/shiftgcn/libshiftgcn_hip.so"', repr(LIB))
    ns = {}
    exec(compile(code, "INTEGRATION.md#3", "exec"), ns)   # noqa: S102 (our own doc)
    return ns


def test_doc_binding_signatures_match_library_table():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    from shiftgcn import _lib
    ns = _exec_snippet()
    lib = ns["lib"]
    for name in ("sgcn_tshift_fwd", "sgcn_tshift_bwd", "sgcn_tshift_bwd_ws_bytes"):
        res, args = _lib.SIGNATURES[name]
        fn = getattr(lib, name)
        assert list(fn.argtypes) == list(args), (name, len(fn.argtypes), len(args))
        assert fn.restype == res, name
    assert len(lib.sgcn_tshift_bwd.argtypes) == 22
    assert callable(ns["forward"]) and callable(ns["backward"])


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_doc_binding_runs_and_matches_shift_cuda(stride):
    from shiftgcn import shift_cuda
    ns = _exec_snippet()
    dev = "cuda"
    g = torch.Generator().manual_seed(3 + stride)
    B, C, H, W = 3, 16, 24, 25
    x = torch.randn(B, C, H, W, generator=g).to(dev)
    xpos = (torch.rand(C, generator=g) * 2e-8 - 1e-8).to(dev)
    ypos = (torch.rand(C, generator=g) * 4 - 2).to(dev)
    yeff = ypos if stride == 1 else ypos + 0.5       # what the reference glue passes
    gout = torch.randn(B, C, H // stride, W, generator=g).to(dev)
    y_doc = ns["forward"](x, xpos, yeff, stride)
    y_pkg = shift_cuda.forward(x, xpos, yeff, stride)
    gin_d, gx_d, gy_d = ns["backward"](gout, x, y_doc, xpos, yeff, stride)
    gin_p, gx_p, gy_p = shift_cuda.backward(gout, x, y_pkg, xpos, yeff, stride)
    torch.cuda.synchronize()
    for a, b in ((y_doc, y_pkg), (gin_d, gin_p), (gx_d, gx_p), (gy_d, gy_p)):
        assert np.array_equal(a.cpu().numpy(), b.cpu().numpy())
