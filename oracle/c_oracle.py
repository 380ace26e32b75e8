"""ctypes loader for the C oracle (oracle/rs_oracle.c).

TEST INFRASTRUCTURE ONLY: used by tests/ (checker) and bench.py's cpu_baseline leg."""
import ctypes
import os
import subprocess
from ctypes import POINTER, c_char, c_double, c_int, c_size_t, c_uint8, c_uint64, c_void_p

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # repo root
LIB = os.path.join(ROOT, "oracle", "build", "liboracle.so")

_lib = None


def load_c_oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           stdout=subprocess.DEVNULL)
        lib = ctypes.CDLL(LIB)
        lib.orc_matrix.argtypes = [c_int, c_int, POINTER(c_uint8)]
        lib.orc_encode.argtypes = [c_int, c_int, POINTER(c_void_p), POINTER(c_void_p), c_size_t]
        lib.orc_reconstruct.argtypes = [c_int, c_int, POINTER(c_void_p), POINTER(c_uint8),
                                        c_size_t, c_int]
        lib.orc_sha256_hex.argtypes = [c_void_p, c_size_t, POINTER(c_char)]
        lib.orc_sha256_hex.restype = None
        lib.orc_fill_synthetic.argtypes = [c_void_p, c_size_t, c_size_t, c_uint64, c_uint64]
        lib.orc_fill_synthetic.restype = None
        lib.orc_encode_batch.argtypes = [c_int, c_int, c_void_p, c_void_p, c_size_t, c_size_t,
                                         c_int, c_int]
        lib.orc_encode_batch.restype = c_double
        lib.orc_set_simd.argtypes = [c_int]
        lib.orc_segment_ops.argtypes = [c_int, c_int, POINTER(c_void_p), c_size_t, c_int, c_int]
        lib.orc_segment_ops.restype = c_double
        _lib = lib
    return _lib


def ptrs(arrs):
    return (c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def c_encode(lib, k, m, data):
    import numpy as np
    par = [np.zeros(len(data[0]), np.uint8) for _ in range(m)]
    assert lib.orc_encode(k, m, ptrs(data), ptrs(par), len(data[0])) == 0
    return par


def c_sha256_hex(lib, buf):
    import numpy as np
    a = np.ascontiguousarray(np.frombuffer(bytes(buf), np.uint8)) if not isinstance(
        buf, np.ndarray) else buf
    out = ctypes.create_string_buffer(64)
    lib.orc_sha256_hex(a.ctypes.data if len(a) else None, len(a), out)
    return out.raw
