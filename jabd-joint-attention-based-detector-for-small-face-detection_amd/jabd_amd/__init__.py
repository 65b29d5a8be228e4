"""jabd_amd — MI355X-native runtime for the JABD detection hot path.

`ops` wraps the libjabd.so C-ABI (include/jabd.h) at tensor level; the
reference-compatible modules live beside this package in `nets/` and
`utils/` (put the package directory on sys.path to use them as drop-ins).
"""
__all__ = ["ops", "synth"]
