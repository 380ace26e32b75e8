"""ctypes binding of libcessec (include/cess_ec.h). No fallback: a missing or unloadable library
raises, so nothing silently runs on the CPU."""
from __future__ import annotations

import ctypes
import os
from ctypes import (CFUNCTYPE, POINTER, Structure, c_char_p, c_double, c_int, c_longlong,
                    c_int32, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CESS_EC_LIB", os.path.join(_HERE, "libcessec.so"))
# tuning build of the same library: every kernel variant of the sweeps (CEC_OPT_CT_VARIANT);
# used only by bench.py --sweep and the variant tests, never by the product path
TUNE_LIB_PATH = os.path.join(_HERE, "libcessec_tune.so")

# cec_pipeline_* callback and struct types (include/cess_ec.h)
READ_FN = CFUNCTYPE(c_longlong, c_void_p, c_void_p, c_size_t)
FRAGMENTS_FN = CFUNCTYPE(c_int, c_void_p, c_uint64, POINTER(c_void_p), c_size_t)
RECORD_FN = CFUNCTYPE(c_int, c_void_p, c_uint64, c_void_p, c_void_p)
# cec_pipeline_run_files callbacks: (user, file, ...)
FILE_FRAGMENTS_FN = CFUNCTYPE(c_int, c_void_p, c_size_t, c_uint64, POINTER(c_void_p), c_size_t)
FILE_RECORD_FN = CFUNCTYPE(c_int, c_void_p, c_size_t, c_uint64, c_void_p, c_void_p)
# cec_dist_degraded_read locate callback
LOCATE_FN = CFUNCTYPE(c_void_p, c_void_p, c_uint64, c_int)


class PipelineOpts(Structure):
    _fields_ = [("shard_len", c_size_t), ("batch_segments", c_size_t), ("depth", c_int),
                ("hash", c_int), ("window", c_int), ("max_segments", c_uint64),
                ("host_threads", c_int), ("tail_batches", c_int)]


class Source(Structure):
    _fields_ = [("read", READ_FN), ("user", c_void_p), ("size", c_uint64)]


class DistMove(Structure):
    _fields_ = [("seg", c_uint64), ("frag", c_int32), ("src", c_int32), ("dst", c_int32),
                ("kind", c_int32)]


class PipelineStats(Structure):
    _fields_ = [("segments", c_uint64), ("bytes_in", c_uint64), ("seconds", c_double),
                ("read_seconds", c_double), ("wait_seconds", c_double)]


FILE_DONE_FN = CFUNCTYPE(c_int, c_void_p, c_size_t, POINTER(PipelineStats))


# exported symbols and their (restype, argtypes); tests check this against include/cess_ec.h
SIGNATURES = {
    "cec_version": (c_char_p, []),
    "cec_strerror": (c_char_p, [c_int]),
    "cec_last_error": (c_char_p, []),
    "cec_device_count": (c_int, []),
    "cec_create": (c_int, [c_int, c_int, c_int, POINTER(c_void_p)]),
    "cec_destroy": (None, [c_void_p]),
    "cec_codec_info": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "cec_matrix": (c_int, [c_void_p, POINTER(c_uint8)]),
    "cec_encode": (c_int, [c_void_p, POINTER(c_void_p), c_size_t]),
    "cec_reconstruct": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_uint8), c_size_t, c_int]),
    "cec_verify": (c_int, [c_void_p, POINTER(c_void_p), c_size_t, POINTER(c_int)]),
    "cec_encode_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t, c_void_p]),
    "cec_reconstruct_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t,
                                      POINTER(c_uint8), c_int, c_int, c_void_p]),
    "cec_reconstruct_partial_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t,
                                              POINTER(c_uint8), POINTER(c_uint8), c_int,
                                              c_void_p]),
    "cec_verify_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t, c_void_p,
                                 c_void_p]),
    "cec_xor_batch": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_size_t, c_void_p]),
    "cec_sha256_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t, c_void_p,
                                 c_void_p]),
    "cec_sha256_hex": (c_int, [POINTER(c_void_p), c_size_t, c_size_t, POINTER(c_uint8),
                               c_void_p]),
    "cec_sha256_host": (c_int, [POINTER(c_void_p), c_size_t, c_size_t, c_void_p, c_size_t,
                                c_void_p, c_int]),
    "cec_sha256_host_state": (c_int, [POINTER(c_void_p), c_size_t, c_size_t, c_void_p,
                                      c_void_p, c_int]),
    "cec_host_sha_set_form": (c_int, [c_int]),
    "cec_host_sha_form": (c_int, []),
    "cec_host_sha_pool_threads": (c_int, []),
    "cec_host_sha_probe": (c_double, [c_int, c_size_t, c_int]),
    "cec_split_segment": (c_int, [c_void_p, c_size_t, c_int, POINTER(c_void_p), c_size_t]),
    "cec_fill_synthetic": (c_int, [c_void_p, c_size_t, c_size_t, c_uint64, c_uint64, c_void_p]),
    "cec_set_option": (c_int, [c_void_p, c_int, c_int]),
    "cec_get_stat": (c_int, [c_void_p, c_int, POINTER(c_uint64)]),
    "cec_hashq_create": (c_int, [c_int, c_size_t, c_void_p, POINTER(c_void_p)]),
    "cec_hashq_destroy": (None, [c_void_p]),
    "cec_hashq_add": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_size_t, c_size_t,
                              c_size_t, c_void_p, c_size_t, POINTER(c_uint64)]),
    "cec_hashq_add_prefix": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_size_t, c_size_t,
                                     c_size_t, c_void_p, c_size_t, c_size_t, c_void_p, c_size_t,
                                     POINTER(c_uint64)]),
    "cec_hashq_add_resume": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_size_t, c_size_t,
                                     c_size_t, c_size_t, c_void_p, c_void_p, c_size_t,
                                     POINTER(c_uint64)]),
    "cec_hashq_tick": (c_int, [c_void_p, c_uint32]),
    "cec_hashq_finish": (c_int, [c_void_p]),
    "cec_hashq_status": (c_int, [c_void_p, c_uint64, POINTER(c_int), POINTER(c_size_t),
                                 POINTER(c_uint64)]),
    "cec_hashq_set_option": (c_int, [c_void_p, c_int, c_int]),
    "cec_pipeline_create": (c_int, [c_void_p, POINTER(PipelineOpts), POINTER(c_void_p)]),
    "cec_pipeline_destroy": (None, [c_void_p]),
    "cec_pipeline_run": (c_int, [c_void_p, READ_FN, FRAGMENTS_FN, RECORD_FN, c_void_p,
                                 POINTER(PipelineStats)]),
    "cec_pipeline_info": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "cec_pipeline_run_files": (c_int, [c_void_p, POINTER(Source), c_size_t, FILE_FRAGMENTS_FN,
                                       FILE_RECORD_FN, FILE_DONE_FN, c_void_p,
                                       POINTER(PipelineStats)]),
    "cec_challenge_indices": (c_int, [POINTER(c_uint64), c_size_t, c_uint32, c_uint32,
                                      POINTER(c_uint32), POINTER(c_size_t)]),
    "cec_audit_chunks": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t, c_uint32,
                                 POINTER(c_uint32), c_uint32, c_void_p, c_void_p, c_void_p]),
    "cec_scale_compact": (c_int, [c_uint32, c_void_p, c_size_t, POINTER(c_size_t)]),
    "cec_scale_deal_info": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_void_p, c_size_t,
                                    POINTER(c_size_t)]),
    "cec_scale_upload_declaration": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t,
                                             c_void_p, c_void_p, c_size_t, c_void_p, c_size_t,
                                             c_void_p, c_size_t, POINTER(c_size_t)]),
    "cec_shard_id": (c_int, [c_void_p, c_uint32, c_void_p]),
    "cec_dist_unique_id": (c_int, [c_void_p]),
    "cec_dist_create": (c_int, [c_void_p, c_void_p, c_int, c_int, POINTER(c_void_p)]),
    "cec_dist_destroy": (None, [c_void_p]),
    "cec_dist_plan": (c_int, [c_int, c_int, c_int, POINTER(c_uint64), POINTER(c_uint8), c_size_t,
                              POINTER(DistMove), c_size_t, POINTER(c_size_t), POINTER(c_int32)]),
    "cec_dist_plan_ex": (c_int, [c_int, c_int, c_int, c_int, POINTER(c_uint64), POINTER(c_uint8),
                                 c_size_t, POINTER(DistMove), c_size_t, POINTER(c_size_t),
                                 POINTER(c_int32)]),
    "cec_dist_set_option": (c_int, [c_void_p, c_int, c_int]),
    "cec_dist_groups": (c_int, [c_void_p, POINTER(c_uint64)]),
    "cec_dist_plan_groups": (c_int, [c_int, c_int, c_int, c_int, c_int, POINTER(c_uint64),
                                     POINTER(c_uint8), c_size_t, POINTER(c_uint64), c_size_t,
                                     POINTER(c_size_t)]),
    "cec_dist_degraded_read": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint8), c_size_t,
                                       c_size_t, LOCATE_FN, c_void_p, POINTER(c_void_p), c_void_p,
                                       POINTER(c_size_t)]),
    "cec_hash_from_shard_id": (c_int, [c_void_p, c_void_p]),
    "cec_scale_upload_filler": (c_int, [c_void_p, POINTER(c_uint32), c_void_p, c_void_p, c_size_t,
                                        c_void_p, c_size_t, POINTER(c_size_t)]),
    "cec_scale_generate_restoral_order": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t,
                                                  POINTER(c_size_t)]),
    "cec_scale_claim_restoral_order": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(c_size_t)]),
    "cec_scale_claim_restoral_exist_order": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p,
                                                     c_size_t, POINTER(c_size_t)]),
    "cec_scale_restoral_order_complete": (c_int, [c_void_p, c_void_p, c_size_t,
                                                  POINTER(c_size_t)]),
    "cec_audit_random_subject": (c_int, [c_void_p, c_uint32, c_void_p]),
    "cec_audit_random_u64": (c_int, [c_void_p, c_size_t, POINTER(c_uint64)]),
    "cec_survivors": (c_int, [c_int, c_int, c_void_p, c_void_p]),
    "cec_challenge_random_list": (c_int, [c_void_p, c_size_t, c_uint32, c_void_p,
                                          POINTER(c_size_t)]),
}

CEC_OK = 0
CEC_EINVAL = -1
CEC_ETOOFEW = -2
CEC_ESHARDLEN = -3
CEC_EHIP = -4
CEC_ENOMEM = -5
CEC_ENCCL = -6
CEC_ESHORTDATA = -7
CEC_ENODEV = -8
CEC_ESEGCOUNT = -9
CEC_ECALLBACK = -10
CEC_CHUNK_COUNT = 1024
CEC_SEGMENT_COUNT = 1000
CEC_FRAGMENT_COUNT = 3
CEC_UPLOAD_FILLER_LIMIT = 10
CEC_FILLER_SIZE = 8 << 20
CEC_AUDIT_PALLET_ID = b"rewardpt"
CEC_RANDOMNESS_BYTES = 32
CEC_CHALLENGE_RANDOM_BYTES = 20

CEC_OPT_FORCE_GENERIC = 1
CEC_OPT_CT_VARIANT = 2
CEC_OPT_SHA_MODE = 3
CEC_OPT_RT_MODE = 4
CEC_OPT_DECODE_CACHE = 6
CEC_OPT_FFTDEC_MIN = 7
CEC_OPT_FFTDEC_MODE = 8
CEC_STAT_DECODE_CACHED = 1
CEC_STAT_RETIRED_PENDING = 2
CEC_STAT_POOL_BYTES = 3
CEC_STAT_FFTDEC_SEGMENTS = 4
CEC_STAT_FFTDEC_D_SEGMENTS = 5
CEC_HQOPT_TICK = 1
CEC_PIPE_HASH_NONE = 0
CEC_PIPE_HASH_GPU = 1
CEC_PIPE_HASH_HOST = 2
CEC_PIPE_HASH_HYBRID = 3
CEC_HSHA_SCALAR = 0
CEC_HSHA_NI1 = 1
CEC_HSHA_NI2 = 2
CEC_HSHA_NI4 = 3
CEC_HSHA_X16 = 4
CEC_DIST_ID_BYTES = 128
CEC_DIST_SURVIVOR = 0
CEC_DIST_PARTIAL = 1
CEC_DIST_OPT_EXCHANGE = 1
CEC_DIST_OPT_TEST_ABORT = 2
CEC_DIST_OPT_GROUP_OPS = 3

_libs = {}


def load(tuning: bool = False) -> ctypes.CDLL:
    """Load libcessec (or its tuning build) once; raises OSError with a build hint when it is
    missing."""
    path = TUNE_LIB_PATH if tuning else LIB_PATH
    lib = _libs.get(path)
    if lib is None:
        if not os.path.exists(path):
            raise OSError(f"libcessec not found at {path}: build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` "
                          "or `make -C cess_amd/csrc`")
        # One HIP runtime per process: torch's wheel carries its own libamdhip64 (SONAME
        # libamdhip64.so.7, but its libraries NEED it as "libamdhip64.so"). Loaded after torch,
        # libcessec binds to torch's copy by SONAME; loaded first, it maps /opt/rocm's, torch
        # later maps a second runtime beside it and its device init fails ("No HIP GPUs are
        # available"). So torch, when present, goes first.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _libs[path] = lib
    return lib
