"""The C-ABI library loads and exports every entry point include/visionseg.h declares.
CPU only: no kernel is launched (argument validation runs before any HIP call)."""
import ctypes
import os
import re
import subprocess

import pytest

from visionseg import _lib as L


def declared_symbols():
    txt = open(L.HEADER_PATH).read()
    return sorted(set(re.findall(r"VS_API\s+[\w ]+?\*?\s*\b(vs_\w+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "vs_msda_forward" in syms and "vs_window_partition" in syms
    assert set(syms) == set(L.SIGNATURES), "ctypes table out of sync with include/visionseg.h"


def test_library_exports_every_declared_symbol():
    assert os.path.exists(L.LIB_PATH), "library not built (run __graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (vs_\w+)", out))
    missing = set(declared_symbols()) - exported
    assert not missing, missing


def test_load_version_and_error_path():
    lib = L.lib()
    assert lib.vs_abi_version() == 1
    # channels != 32 is rejected before touching the device
    sh = (ctypes.c_int64 * 2)(4, 4)
    st = (ctypes.c_int64 * 1)(0)
    rc = lib.vs_msda_forward(0, ctypes.c_void_p(16), sh, st, ctypes.c_void_p(16), ctypes.c_void_p(16),
                             ctypes.c_void_p(16), 1, 16, 1, 16, 1, 1, 1, None)
    assert rc == -1
    assert b"channels per head must be 32" in lib.vs_last_error()
    with pytest.raises(RuntimeError, match="channels per head"):
        L.check(rc, "msda_forward")
    rc = lib.vs_window_partition(ctypes.c_void_p(16), ctypes.c_void_p(16), 2, 1, 4, 4, 8, 4, 4, None)
    assert rc == -1 and b"shift" in lib.vs_last_error()


def test_ops_refuse_cpu_tensors():
    import torch
    from visionseg import ops
    with pytest.raises(RuntimeError, match="HIP device"):
        ops.window_partition(torch.zeros(1, 4, 4, 8), 4, 0)


# the operator surface of SURVEY §8(b): TORCH_LIBRARY(visionseg) in csrc/torch_ops.cpp
TORCH_OPS = ["msda_fwd", "msda_bwd", "swin_window_fwd", "swin_window_bwd", "win_attn_fwd", "win_attn_bwd",
             "win_attn_fwd_img", "win_attn_bwd_img",
             "mask_head_fwd", "mask_head_bwd", "attn_bitmask", "masked_xattn_fwd", "masked_xattn_bwd"]


def test_torch_library_registers_every_op():
    import torch
    assert os.path.exists(L.TORCH_LIB_PATH), "torch ops library not built (run __graft_entry__.build())"
    ns = L.tops()
    for name in TORCH_OPS:
        op = getattr(ns, name).default
        assert op._schema.name == f"visionseg::{name}"
    sch = str(ns.msda_fwd.default._schema)
    assert "Tensor spatial_shapes" in sch and "int im2col_step" in sch
    # grad_pixel of mask_head_bwd is declared as written in place
    assert "Tensor(a!) grad_pixel" in str(ns.mask_head_bwd.default._schema)
    del torch


def test_torch_ops_refuse_cpu_tensors():
    """No CPU kernel is registered: a CPU tensor never reaches a fallback."""
    import torch
    ns = L.tops()
    with pytest.raises((RuntimeError, NotImplementedError)):
        ns.swin_window_fwd(torch.zeros(1, 4, 4, 8), 4, 0)
    sh, st = L.level_tensors([(2, 2)])
    with pytest.raises((RuntimeError, NotImplementedError)):
        ns.msda_fwd(torch.zeros(1, 4, 1, 32), sh, st, torch.zeros(1, 1, 1, 1, 1, 2), torch.zeros(1, 1, 1, 1, 1), 64)
    assert sh.tolist() == [[2, 2]] and st.tolist() == [0]
