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
