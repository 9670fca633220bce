"""ctypes binding of include/fac.h (libfac.so, built in-tree by csrc/Makefile).

The library is mandatory: there is no Python or CPU fallback for the search path. Importing this
module raises if libfac.so is missing; search calls return FAC_E_NO_DEVICE (raised as
`DeviceError`) when no gfx950 GPU is visible.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FAC_LIB", os.path.join(_HERE, "_lib", "libfac.so"))

FAC_OK = 0
FAC_E_HAYSTACK_TOO_LARGE = 1
FAC_E_INVALID = 100
FAC_E_UNSUPPORTED = 101
FAC_E_HIP = 102
FAC_E_NO_DEVICE = 103
FAC_E_OOM = 104
FAC_E_CAPACITY = 105
FAC_E_OUTPUT_CAPACITY = 106
FAC_E_INTERNAL = 107
LIMIT_NONE = -1


class fac_limits(ctypes.Structure):
    _fields_ = [("insertions", ctypes.c_int32), ("deletions", ctypes.c_int32),
                ("substitutions", ctypes.c_int32), ("swaps", ctypes.c_int32),
                ("edits", ctypes.c_int32)]


class fac_pattern(ctypes.Structure):
    _fields_ = [("utf8", ctypes.c_char_p), ("len", ctypes.c_uint64), ("weight", ctypes.c_float),
                ("has_limits", ctypes.c_int32), ("limits", fac_limits)]


class fac_mapping(ctypes.Structure):
    _fields_ = [("a", ctypes.c_char_p), ("a_len", ctypes.c_uint64), ("b", ctypes.c_char_p),
                ("b_len", ctypes.c_uint64), ("score", ctypes.c_float)]


class fac_config(ctypes.Structure):
    _fields_ = [("case_insensitive", ctypes.c_int32), ("has_limits", ctypes.c_int32),
                ("limits", fac_limits), ("penalty_insertion", ctypes.c_float),
                ("penalty_deletion", ctypes.c_float), ("penalty_substitution", ctypes.c_float),
                ("penalty_swap", ctypes.c_float), ("beam_width", ctypes.c_uint64),
                ("has_auto_beam", ctypes.c_int32), ("auto_beam_budget", ctypes.c_uint64),
                ("auto_beam_width", ctypes.c_uint64), ("min_symbol_similarity", ctypes.c_float),
                ("similarity_ascii", ctypes.POINTER(ctypes.c_float)),
                ("n_similarity_pairs", ctypes.c_uint64),
                ("similarity_pairs", ctypes.POINTER(ctypes.c_uint32)),
                ("similarity_pair_values", ctypes.POINTER(ctypes.c_float)),
                ("n_mappings", ctypes.c_uint64), ("mappings", ctypes.POINTER(fac_mapping)),
                ("device", ctypes.c_int32)]


def _match_dtype():
    import numpy as np
    return np.dtype([("start", "<u8"), ("end", "<u8"), ("pattern_index", "<u4"), ("similarity", "<f4"),
                     ("insertions", "u1"), ("deletions", "u1"), ("substitutions", "u1"), ("swaps", "u1"),
                     ("edits", "u1"), ("pad", "V3")])


MATCH_DTYPE = _match_dtype()  # the 32-byte fac_match / OwnedMatch record
REC_BYTES = 32


class fac_match(ctypes.Structure):
    _fields_ = [("start", ctypes.c_uint64), ("end", ctypes.c_uint64),
                ("pattern_index", ctypes.c_uint32), ("similarity", ctypes.c_float),
                ("insertions", ctypes.c_uint8), ("deletions", ctypes.c_uint8),
                ("substitutions", ctypes.c_uint8), ("swaps", ctypes.c_uint8),
                ("edits", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 3)]


class fac_stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("prefilter_ms", ctypes.c_double),
                ("kernel_launches", ctypes.c_uint64), ("windows", ctypes.c_uint64),
                ("states_popped", ctypes.c_uint64), ("graphemes", ctypes.c_uint64),
                ("bytes", ctypes.c_uint64), ("retries", ctypes.c_uint64), ("cache_ms", ctypes.c_double),
                ("states_cached", ctypes.c_uint64), ("lane_ms", ctypes.c_double),
                ("lane_windows", ctypes.c_uint64)]


class fac_search_args(ctypes.Structure):
    _fields_ = [("window_begin", ctypes.c_uint64), ("window_end", ctypes.c_uint64), ("threshold", ctypes.c_float),
                ("stream", ctypes.c_void_p), ("auto_beam_prefix", ctypes.c_uint64), ("device_out", ctypes.c_void_p),
                ("device_cap", ctypes.c_uint64)]


assert ctypes.sizeof(fac_match) == 32

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libfac.so not found at {LIB_PATH}; build it with `make -C fuzzy-aho-corasick-rs_amd/csrc` "
        "(or __graft_entry__.build()). There is no fallback implementation.")

# torch (used beside the library for device buffers, streams and torch.distributed) brings up its
# own HIP runtime first: on some hosts torch's bundled runtime fails to initialise ("No HIP GPUs are
# available") once another HIP runtime in the process -- this library's -- has made device calls.
try:
    import torch as _torch
    _torch.cuda.is_available()
except ImportError:
    pass
lib = ctypes.CDLL(LIB_PATH)

_P = ctypes.POINTER
_u64p = _P(ctypes.c_uint64)
_engine_p = ctypes.c_void_p
_hay_p = ctypes.c_void_p

SIGNATURES = {
    "fac_last_error": (ctypes.c_char_p, []),
    "fac_build": (ctypes.c_int, [_P(fac_pattern), ctypes.c_uint64, _P(fac_config), _P(_engine_p)]),
    "fac_engine_free": (None, [_engine_p]),
    "fac_trim_scratch": (None, []),
    "fac_search_raw": (ctypes.c_int, [_engine_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_float,
                                      _P(_P(fac_match)), _u64p, _u64p]),
    "fac_matches_free": (None, [_P(fac_match)]),
    "fac_prefilter_active": (ctypes.c_int, [_engine_p]),
    "fac_search_prefiltered": (ctypes.c_int, [_engine_p, ctypes.c_char_p, ctypes.c_uint64,
                                              ctypes.c_float, _P(_P(fac_match)), _u64p, _u64p]),
    "fac_max_match_graphemes": (ctypes.c_uint64, [_engine_p]),
    "fac_haystack_stage": (ctypes.c_int, [_engine_p, ctypes.c_char_p, ctypes.c_uint64,
                                          _P(_hay_p), _u64p]),
    "fac_haystack_graphemes": (ctypes.c_uint64, [_hay_p]),
    "fac_haystack_free": (None, [_hay_p]),
    "fac_haystack_grapheme_starts": (ctypes.c_uint64, [_hay_p, _u64p, ctypes.c_uint64]),
    "fac_search_staged": (ctypes.c_int, [_engine_p, _hay_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_float, ctypes.c_void_p, _P(_P(fac_match)), _u64p,
                                         _P(fac_stats)]),
    "fac_search_staged_ex": (ctypes.c_int, [_engine_p, _hay_p, _P(fac_search_args), _P(_P(fac_match)), _u64p,
                                            _P(fac_stats)]),
    "fac_auto_beam_total": (ctypes.c_int, [_engine_p, _hay_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_float,
                                           ctypes.c_void_p, _u64p]),
    "fac_shard_plan": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint64,
                                      ctypes.c_uint64, _P(ctypes.c_uint64)]),
    "fac_haystack_stage_shard": (ctypes.c_int, [_engine_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, _P(_hay_p), _u64p]),
    "fac_haystack_stage_shard_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_void_p,
                                                       ctypes.POINTER(ctypes.c_void_p), _u64p]),
    "fac_haystack_owned_windows": (ctypes.c_uint64, [_hay_p]),
    "fac_haystack_set_key_partition": (ctypes.c_int, [_engine_p, _hay_p, ctypes.c_uint32, ctypes.c_uint32]),
    "fac_stream_window_staged": (ctypes.c_int, [_engine_p, _hay_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_uint64, ctypes.c_float, ctypes.c_int32, ctypes.c_void_p,
                                                _P(_P(fac_match)), _u64p, _P(fac_stats)]),
    "fac_stream_window_staged_device": (ctypes.c_int, [_engine_p, _hay_p, ctypes.c_uint64, ctypes.c_uint64,
                                                       ctypes.c_uint64, ctypes.c_uint64, ctypes.c_float, ctypes.c_int32,
                                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, _u64p,
                                                       _P(fac_stats)]),
    "fac_stream_windows_staged_device": (ctypes.c_int, [_engine_p, _hay_p, _u64p, ctypes.c_uint64, ctypes.c_float,
                                                        ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                        _u64p, _P(fac_stats)]),
    "fac_search_staged_prefiltered": (ctypes.c_int, [_engine_p, _hay_p, ctypes.c_float, ctypes.c_void_p,
                                                     _P(_P(fac_match)), _u64p, _P(fac_stats)]),
    "fac_matches_apply": (ctypes.c_int, [_engine_p, _P(fac_match), ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                                         _u64p, _u64p]),
    "fac_stream_open": (ctypes.c_int, [_engine_p, ctypes.c_float, ctypes.c_uint64, _P(ctypes.c_void_p)]),
    "fac_stream_feed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int32,
                                       _P(_P(fac_match)), _u64p, _P(_P(ctypes.c_uint8)), _u64p]),
    "fac_stream_total": (ctypes.c_uint64, [ctypes.c_void_p]),
    "fac_stream_committed": (ctypes.c_uint64, [ctypes.c_void_p]),
    "fac_stream_close": (None, [ctypes.c_void_p]),
    "fac_buffer_free": (None, [ctypes.c_void_p]),
    "fac_prefilter_windows": (ctypes.c_int64, [_engine_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_float,
                                               _u64p, ctypes.c_uint64]),
    "fac_engine_num_nodes": (ctypes.c_uint64, [_engine_p]),
    "fac_engine_max_edits_fast": (ctypes.c_uint32, [_engine_p]),
    "fac_segment_graphemes": (ctypes.c_uint64, [ctypes.c_char_p, ctypes.c_uint64, _u64p,
                                                ctypes.c_uint64]),
    "fac_fold_first_char": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int32]),
    "fac_haystack_stage_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                 ctypes.POINTER(ctypes.c_void_p), _u64p]),
    "fac_edge_order": (None, [ctypes.POINTER(ctypes.c_uint32), _u64p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)]),
    "fac_diag_beam_select": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
}

for _name, (_res, _args) in SIGNATURES.items():
    if "FAC_LIB" in os.environ and not hasattr(lib, _name):
        continue  # an older diagnostics build (FAC_LIB) may lack newer entry points
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args


def last_error() -> str:
    return lib.fac_last_error().decode("utf-8", "replace")


def shard_plan(max_match_graphemes: int, data: bytes, n_shards: int, shard: int, is_ascii: int = -1):
    """fac_shard_plan (host only): (a, b, e, global_ascii, open_end) — the shard owns the start
    windows of bytes [a, b) and stages bytes [a, e)."""
    plan = (ctypes.c_uint64 * 4)()
    rc = lib.fac_shard_plan(max_match_graphemes, data, len(data), is_ascii, n_shards, shard, plan)
    if rc:
        raise ValueError(last_error())
    return int(plan[0]), int(plan[1]), int(plan[2]), bool(plan[3] & 1), bool(plan[3] & 2)


def grapheme_starts(data: bytes):
    """UAX #29 grapheme start byte offsets (host helper, no GPU needed)."""
    n = len(data)
    if n == 0:
        return []
    buf = (ctypes.c_uint64 * (n + 1))()
    cnt = lib.fac_segment_graphemes(data, n, buf, n + 1)
    return list(buf[:cnt])


def take_records(ptr, n):
    """Hand a library-allocated fac_match array to NumPy without a copy: a structured array of 32 B
    records (no per-record Python objects) viewing the library buffer, which is freed with
    fac_matches_free when the last view of it goes away."""
    import numpy as np
    import weakref
    if n == 0:
        lib.fac_matches_free(ptr)
        return np.zeros(0, dtype=MATCH_DTYPE)
    addr = ctypes.cast(ptr, ctypes.c_void_p).value
    buf = (ctypes.c_uint8 * (n * 32)).from_address(addr)
    weakref.finalize(buf, lib.fac_matches_free, ctypes.cast(addr, ctypes.POINTER(fac_match)))
    return np.frombuffer(buf, dtype=MATCH_DTYPE)


def take_matches(ptr, n):
    """Copy a library-allocated fac_match array into Python tuples and free it."""
    out = []
    try:
        for i in range(n):
            m = ptr[i]
            out.append((m.start, m.end, m.pattern_index, m.similarity, m.insertions, m.deletions,
                        m.substitutions, m.swaps, m.edits))
    finally:
        lib.fac_matches_free(ptr)
    return out
