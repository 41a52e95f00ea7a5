"""ctypes binding of libskp.so (the C ABI declared in include/skp.h).

The library is built in-tree by ``__graft_entry__.build()`` /
``make -C stablekeypoints_amd/csrc``.  There is no fallback: if the library is
missing or cannot be loaded, every op raises ``SkpLibraryError``.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SKP_LIB", os.path.join(_HERE, "libskp.so"))

_c_int, _c_float, _c_ll, _p = ctypes.c_int, ctypes.c_float, ctypes.c_longlong, ctypes.c_void_p

# name -> argtypes (restype int unless noted)
_SIGS = {
    "skp_capture_fwd": [_p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p],
    "skp_capture_bwd": [_p, _c_int, _c_int, _c_int, _c_int, _p, _c_int, _c_ll, _c_ll, _c_ll, _c_float, _p, _p, _p,
                        _p],
    "skp_capture_maps_fwd": [ctypes.POINTER(_p), ctypes.POINTER(_c_int), _c_int, _c_int, _c_int, _c_int, _c_int, _p,
                             ctypes.POINTER(_p), _p],
    "skp_capture_maps_bwd": [ctypes.POINTER(_p), ctypes.POINTER(_c_int), _c_int, _c_int, _c_int, _c_int, _c_int, _p,
                             _c_float, ctypes.POINTER(_p), ctypes.POINTER(_p), _p, _p],
    "skp_capture_maps_bwd_sel": [ctypes.POINTER(_p), ctypes.POINTER(_c_int), _c_int, _c_int, _c_int, _c_int, _c_int,
                                 _p, _c_int, _p, _c_float, ctypes.POINTER(_p), ctypes.POINTER(_p), _p, _p],
    "skp_sel_bwd_timing": [_c_int],
    "skp_sel_bwd_timing_read": [_p, _p],
    "skp_capture_maps_bwd_sel_workspace": [ctypes.POINTER(_c_int), _c_int, _c_int, _c_int, _c_int, _c_int, _c_int],
    "skp_aggregate": [ctypes.POINTER(_p), _c_int, _c_int, _c_int, _c_int, _p, _c_int, _p, _p],
    "skp_resize_bilinear": [_p, _c_int, _c_int, _c_int, _p, _p],
    "skp_resize_bilinear_bwd": [_p, _c_int, _c_int, _c_int, _p, _p],
    "skp_argmax2d": [_p, _c_int, _c_int, _c_int, _p, _c_int, _p, _p, _p],
    "skp_k_max_pixels": [_p, _c_int, _c_int, _c_int, _c_int, _c_float, _p, _p, _p],
    "skp_mask_radius": [_p, _c_int, _c_int, _c_int, _p, _c_float, _p, _p],
    "skp_weighted_avg": [_p, _c_int, _c_int, _c_int, _c_float, _c_int, _p, _p],
    "skp_gaussian_target": [_p, _c_int, _c_int, _c_int, _c_float, _p, _p],
    "skp_topk_gaussian": [_p, _c_int, _c_int, _c_int, _c_int, _c_float, _c_float, _c_int, _p, _p, _p, _p],
    "skp_topk_gaussian_batch": [_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _c_float, _c_int, _p, _p, _p,
                                _p],
    "skp_topk_keys": [_p, _c_int, _c_int, _c_int, _p, _p],
    "skp_entropy_sort": [_p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p, _p],
    "skp_fps": [_p, _c_int, _c_int, _c_int, _p, _c_int, _c_int, _p, _p, _p, _p],
    "skp_fps_batch": [_p, _c_int, _c_int, _c_int, _c_int, _p, _c_int, _c_int, _p, _p, _p, _p],
    "skp_fps_keys_batch": [_p, _p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _p, _p, _p, _p, _p],
    "skp_sharpen_fwd": [_p, _c_int, _c_int, _c_int, _c_float, _c_int, _p, _p, _p, _p],
    "skp_sharpen_bwd": [_p, _c_int, _c_int, _c_int, _c_float, _c_int, _p, _p, _p, _p],
    "skp_wino_in_transform": [_p, _c_int, _c_int, _c_int, _c_int, _p, _p],
    "skp_wino_out_transform": [_p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p, _p],
    "skp_wino_out_transform_kt": [_p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p, _p, _p],
    "skp_sharpen_fwd_batch": [_p, _c_int, _c_int, _c_int, _c_int, _c_float, _c_int, _p, _p, _p, _p],
    "skp_sharpen_bwd_batch": [_p, _c_int, _c_int, _c_int, _c_int, _c_float, _c_int, _p, _p, _p, _p],
    "skp_affine_warp": [_p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p],
    "skp_affine_warp_bwd": [_p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p],
    "skp_equiv_fwd": [_p, _p, _c_int, _c_int, _c_int, _p, _p, _p, _p],
    "skp_equiv_bwd": [_p, _p, _c_int, _c_int, _c_int, _p, _p, _p, _p, _p],
    "skp_equiv_fwd_batch": [_p, _p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p, _p],
    "skp_equiv_bwd_batch": [_p, _p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p, _p, _p],
    "skp_bgemm_f32": [_p, _c_ll, _c_ll, _c_ll, _p, _c_ll, _c_ll, _c_ll, _p, _c_ll, _c_ll, _c_ll, _c_int, _c_int,
                      _c_int, _c_int, _c_float, _c_int, _p],
    "skp_bgemm_f32_2b": [_p, _c_ll, _c_ll, _c_ll, _c_ll, _p, _c_ll, _c_ll, _c_ll, _c_ll, _p, _c_ll, _c_ll, _c_ll,
                         _c_ll, _c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _c_int, _p],
    "skp_groupnorm_workspace": [_c_int, _c_int, _c_ll, _c_int],
    "skp_groupnorm_fwd": [_p, _p, _p, _p, _c_int, _c_int, _c_ll, _c_int, _c_float, _c_int, _p, _p, _p, _p],
    "skp_groupnorm_bwd": [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_ll, _c_int, _c_int, _p, _p, _p],
    "skp_groupnorm_bwd_add": [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_ll, _c_int, _c_int, _p, _p, _p, _p],
    "skp_residual_bias_add": [_p, _p, _p, _c_int, _c_int, _c_ll, _p, _p],
    "skp_softmax_bwd": [_p, _p, _c_ll, _c_int, _c_float, _p],
    "skp_softmax_fwd": [_p, _c_ll, _c_int, _p],
    "skp_attn_dscore": [_p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_float, _p],
    "skp_attn_bwd_kv": [_p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_float, _p],
    "skp_attn_fwd": [_p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_float, _p],
    "skp_attn_bwd_flash": [_p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_float, _p],
    "skp_attn_fwd_bshd": [_p, _c_ll, _c_int, _p, _c_ll, _c_int, _p, _c_ll, _c_int, _p, _c_ll, _c_int, _p, _c_int, _c_int,
                          _c_int, _c_int, _c_int, _c_float, _p],
    "skp_attn_bwd_flash_bshd": [_p, _c_ll, _c_int, _p, _c_ll, _c_int, _p, _c_ll, _c_int, _p, _c_ll, _c_int, _p, _p, _p,
                                _p, _c_ll, _c_int, _p, _c_ll, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_float,
                                _p],
    "skp_layernorm_fwd": [_p, _p, _p, _c_ll, _c_int, _c_float, _p, _p, _p],
    "skp_layernorm_bwd": [_p, _p, _p, _p, _c_ll, _c_int, _p, _p],
    "skp_layernorm_bwd_add": [_p, _p, _p, _p, _c_ll, _c_int, _p, _p, _p],
    "skp_geglu_fwd": [_p, _c_ll, _c_int, _p, _p],
    "skp_geglu_bwd": [_p, _p, _c_ll, _c_int, _p, _p],
    "skp_wino_weights": [_p, _c_int, _c_int, _c_int, _p, _p],
    "skp_conv3x3_wino": [_p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _p, _p],
    "skp_wino2_weights": [_p, _c_int, _c_int, _c_int, _p, _p],
    "skp_conv3x3_wino2": [_p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _p, _p],
    "skp_conv3x3_wino2_gn": [_p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _p, _p, _p],
    "skp_groupnorm_fwd_part": [_p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_ll, _c_int, _c_float, _c_int, _p, _p, _p,
                               _p],
    "skp_conv3x3s2_wino2": [_p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _p, _p],
    "skp_version": [],
}


_RESTYPE = {"skp_capture_maps_bwd_sel_workspace": _c_ll}
# measurement hooks (not on the reference's interface) that A/B runs against older builds may lack
_MEASUREMENT_ONLY = {"skp_sel_bwd_timing", "skp_sel_bwd_timing_read"}


class SkpLibraryError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libskp.so once; raise loudly if it is absent (no CPU/torch fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SkpLibraryError(f"libskp.so not found at {LIB_PATH}: build it with "
                                  "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C stablekeypoints_amd/csrc`")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise SkpLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, args in _SIGS.items():
            if name in _MEASUREMENT_ONLY and not hasattr(L, name):
                continue   # an older library in an A/B run (SKP_LIB): the bench skips what it lacks
            f = getattr(L, name)
            f.argtypes = args
            f.restype = _RESTYPE.get(name, _c_int)
        L.skp_last_error.argtypes = []
        L.skp_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS) + ["skp_last_error"]


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().skp_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (rc={rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise ValueError("stablekeypoints_amd ops run on the HIP device only; got a CPU tensor "
                             "(there is no CPU fallback: the CPU oracle lives under oracle/ and is test-only)")
