"""CPU-side checks of the C ABI: the library loads, exports every declared symbol, and
rejects bad arguments before touching the device (no GPU needed)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(REPO, "include", "skp.h")).read()
    return sorted(set(re.findall(r"\b(skp_[a-z0-9_]+)\s*\(", hdr)))


def test_header_matches_binding_table():
    from stablekeypoints_amd import _lib
    assert sorted(_lib.exported_symbols()) == declared_symbols()


def test_library_exports_every_symbol():
    from stablekeypoints_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libskp.so not built (run __graft_entry__.build())")
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert _lib.lib().skp_version() == 1


def test_library_reads_no_environment():
    """r06: every A/B switch left the shipped library: no libc
    getenv import and no SKP_* variable name in its strings; variants are build options
    (tools/build_variant.sh), not runtime paths."""
    from stablekeypoints_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libskp.so not built")
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"getenv" not in blob
    assert re.search(rb"SKP_[A-Z0-9_]{3,}", blob) is None


def test_bad_arguments_rejected_without_gpu():
    from stablekeypoints_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libskp.so not built")
    L = _lib.lib()
    rc = L.skp_capture_fwd(None, 8, 16, 500, 128, None, None, None)
    assert rc == -1 and b"null" in L.skp_last_error()
    rc = L.skp_capture_fwd(ctypes.c_void_p(16), 8, 16, 5000, 128, ctypes.c_void_p(16), None, None)
    assert rc == -1 and b"1024" in L.skp_last_error()
    rc = L.skp_fps(ctypes.c_void_p(16), 10, 8, 8, ctypes.c_void_p(16), 1, 4, ctypes.c_void_p(16), None,
                   ctypes.c_void_p(16), None)
    assert rc == -1 and b"two candidates" in L.skp_last_error()
    a = ctypes.c_void_p(256)   # aligned non-null dummies: every check below fails before any HIP call
    rc = L.skp_layernorm_fwd(a, a, a, 4, 6, 1e-5, a, a, None)
    assert rc == -1 and b"multiple of 4" in L.skp_last_error()
    rc = L.skp_attn_bwd_flash(a, a, a, a, a, a, a, a, a, 2, 100, 64, 40, 0.1, None)
    assert rc == -1 and b"multiple of 64" in L.skp_last_error()
    rc = L.skp_attn_fwd(a, a, a, a, None, 2, 128, 77, 48, 0.1, None)
    assert rc == -1 and b"head dim" in L.skp_last_error()
    rc = L.skp_conv3x3_wino(a, a, None, None, a, 2, 64, 48, 8, 8, 1, None, None)
    assert rc == -1 and b"multiple of 32" in L.skp_last_error()


def test_ops_refuse_cpu_tensors():
    import torch
    from stablekeypoints_amd import ops
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.find_max_pixel(torch.zeros(2, 4, 4))


def test_vae_downsample_edge_pad_equals_f_pad():
    """Downsample2D(padding=0) pads with a copy + edge zeroing instead of F.pad's full fill:
    same output and input gradient as F.pad(x, (0, 1, 0, 1)) + the stride-2 conv (host logic)."""
    import torch
    import torch.nn.functional as F
    from stablekeypoints_amd.sd.unet import Downsample2D
    torch.manual_seed(0)
    m = Downsample2D(6, padding=0)
    x = torch.randn(2, 6, 10, 12, requires_grad=True)
    y = m(x)
    y.sum().backward()
    g = x.grad.clone()
    x.grad = None
    ref = m.conv(F.pad(x, (0, 1, 0, 1)))
    ref.sum().backward()
    assert torch.equal(y, ref) and torch.equal(g, x.grad)


def test_sparse_capture_backward_workspace_and_arguments():
    """skp_capture_maps_bwd_sel: the workspace query sizes both paths and refuses bad shapes;
    the entry point rejects bad arguments before any launch (no GPU needed)."""
    from stablekeypoints_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libskp.so not built")
    L = _lib.lib()
    sizes = (ctypes.c_int * 4)(16, 16, 16, 32)
    fast = L.skp_capture_maps_bwd_sel_workspace(sizes, 4, 8, 8, 500, 128, 10)
    # zsel + E (one layer) + pix (all layers) + es (all layers), floats
    BH, RR = 64, 128 * 128
    assert fast >= BH * 32 * 32 * 10 + BH * 10 * RR + 4 * BH * RR * 2 + 4 * BH * 10 * 32 * 32
    odd = (ctypes.c_int * 2)(5, 3)
    slow = L.skp_capture_maps_bwd_sel_workspace(odd, 2, 2, 3, 36, 40, 4)   # no compiled kernel: dense fallback
    assert slow >= 2 * 36 * 40 * 40 * 2
    assert L.skp_capture_maps_bwd_sel_workspace(sizes, 0, 8, 8, 500, 128, 10) == -1
    assert L.skp_capture_maps_bwd_sel_workspace(sizes, 4, 8, 8, 500, 128, 0) == -1
    p = ctypes.c_void_p(256)
    arr = (ctypes.c_void_p * 4)(256, 256, 256, 256)
    parr = ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p))
    rc = L.skp_capture_maps_bwd_sel(parr, sizes, 4, 8, 8, 500, 128, p, 33, p, 1.0, parr, parr, p, None)
    assert rc == -1 and b"K must be" in L.skp_last_error()
    rc = L.skp_capture_maps_bwd_sel(parr, sizes, 4, 8, 8, 502, 128, p, 10, p, 1.0, parr, parr, p, None)
    assert rc == -1 and b"multiple of 4" in L.skp_last_error()
    rc = L.skp_capture_maps_bwd_sel(parr, sizes, 4, 8, 8, 500, 128, p, 10, p, 1.0, None, parr, p, None)
    assert rc == -1 and b"null" in L.skp_last_error()
