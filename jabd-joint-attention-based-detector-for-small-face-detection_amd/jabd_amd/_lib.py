"""ctypes binding of libjabd.so (the C-ABI declared in include/jabd.h).

This is the Python side of the drop-in boundary: every function of the
header is declared here with its exact C signature, and `call()` turns a
non-zero status into a RuntimeError carrying `jabd_last_error()`.

There is no fallback: if libjabd.so is missing or the HIP runtime is not
usable, `lib()` raises.  The library is loaded *after* torch so that its
libamdhip64.so.7 dependency binds to the HIP runtime torch already loaded
(one runtime per process, so torch streams are valid handles here).
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (load torch's HIP runtime first; see docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libjabd.so")

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_size = ctypes.c_size_t
c_vp = ctypes.c_void_p
c_sizep = ctypes.POINTER(ctypes.c_size_t)

# name -> argtypes (every function returns int status unless listed in _RESTYPE)
SIGNATURES = {
    "jabd_version": [],
    "jabd_last_error": [ctypes.c_char_p, c_size],
    "jabd_decode_f32": [c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_vp, c_vp],
    "jabd_decode_landm_f32": [c_vp, c_vp, c_i64, c_i64, c_f32, c_vp, c_vp],
    "jabd_nms_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_batched_nms_f32": [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                             c_f64, c_f32, c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_detect_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_detect_f32": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_f32, c_f64,
                        c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_match_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_match_encode_f32": [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_f32, c_f32, c_f32,
                              c_vp, c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_multibox_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_multibox_loss_fwd_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_int,
                                   c_vp, c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_multibox_loss_bwd_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_multibox_loss_finalize_f32": [c_vp, c_vp, c_vp, c_vp],
}
_RESTYPE = {"jabd_version": ctypes.c_char_p}

_lock = threading.Lock()
_lib = None


def lib():
    """Load libjabd.so once (thread-safe) and declare every signature."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"libjabd.so not built at {LIB_PATH}; run __graft_entry__.build() "
                    "(the HIP path has no CPU fallback)")
            h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
            for name, args in SIGNATURES.items():
                fn = getattr(h, name)
                fn.argtypes = args
                fn.restype = _RESTYPE.get(name, ctypes.c_int)
            _lib = h
    return _lib


def last_error() -> str:
    buf = ctypes.create_string_buffer(512)
    lib().jabd_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def call(name, *args):
    st = getattr(lib(), name)(*args)
    if st != 0:
        raise RuntimeError(f"{name} failed (status {st}): {last_error()}")


def exported_symbols():
    """Names declared in include/jabd.h that the loaded library must export."""
    return list(SIGNATURES)
