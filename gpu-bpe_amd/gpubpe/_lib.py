"""ctypes declarations for libgpubpe.so (include/gpubpe.h).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, every entry point raises.  Build it with ``make -C gpu-bpe_amd`` (or
``python -c "import __graft_entry__ as g; g.build()"``).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GBPE_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libgpubpe.so"))

GBPE_OK = 0
GBPE_E_INVALID = -1
GBPE_E_OOM = -2
GBPE_E_DEVICE = -3
GBPE_E_CAPACITY = -4
GBPE_E_CANCELLED = -5
GBPE_E_EMPTY = -6
GBPE_E_INTERNAL = -7

GBPE_TRAIN_EXACT_COMPACTION = 1 << 0
GBPE_TRAIN_DENSE_ONLY = 1 << 3
GBPE_TRAIN_SPARSE_EARLY = 1 << 4
GBPE_TRAIN_TIMING = 1 << 1
GBPE_TRAIN_GPT4_BOUNDARIES = 1 << 2

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)


class TrainOpts(C.Structure):
    _fields_ = [("target_vocab_size", C.c_uint32), ("vocab_size", C.c_uint32), ("next_token_id", C.c_uint32),
                ("batch_size", C.c_uint32), ("flags", C.c_uint32), ("table_log2", C.c_uint32)]


class Progress(C.Structure):
    _fields_ = [("merge_index", C.c_uint32), ("total_merges", C.c_uint32), ("best_count", C.c_uint32),
                ("symbol_count", C.c_uint32), ("batch_merges", C.c_uint32), ("early_stop", C.c_uint32),
                ("elapsed_s", C.c_double)]


class TrainerStats(C.Structure):
    _fields_ = [("symbol_count", C.c_uint64), ("merges_done", C.c_uint64), ("stream_bytes_moved", C.c_uint64),
                ("tail_dropped", C.c_uint64), ("live_pairs", C.c_uint64), ("table_slots", C.c_uint64),
                ("table_used", C.c_uint64), ("max_live_pairs", C.c_uint64), ("bytes_per_symbol", C.c_uint32),
                ("early_stop", C.c_uint32), ("ms_merge", C.c_double), ("ms_select", C.c_double),
                ("ms_other", C.c_double), ("timed_merges", C.c_uint64),
                ("ms_delta", C.c_double), ("ms_compact", C.c_double),
                ("sparse_merges", C.c_uint64), ("sparse_enters", C.c_uint32), ("sparse_exits", C.c_uint32),
                ("sparse_sectors", C.c_uint64), ("sparse_zone", C.c_uint64), ("body_bytes", C.c_uint64),
                ("zone_bytes", C.c_uint64), ("dense_bytes", C.c_uint64), ("ms_dense", C.c_double),
                ("ms_sparse", C.c_double), ("ms_body", C.c_double),
                ("lexicon_builds", C.c_uint32), ("lexicon_fallbacks", C.c_uint32), ("lexicon_words", C.c_uint64),
                ("lexicon_entries", C.c_uint64), ("lexicon_symbols", C.c_uint64),
                ("ms_create", C.c_double), ("paired_merges", C.c_uint64)]


class LexShardInfo(C.Structure):
    _fields_ = [("symbols", C.c_uint64), ("body", C.c_uint64), ("zone", C.c_uint64), ("store_symbols", C.c_uint64),
                ("entries", C.c_uint64), ("words", C.c_uint64), ("top_count", C.c_uint32),
                ("bytes_per_symbol", C.c_uint32)]


GBPE_LEXSHARD_STORE, GBPE_LEXSHARD_MUL, GBPE_LEXSHARD_OCC, GBPE_LEXSHARD_ZONE = 0, 1, 2, 3

PROGRESS_CB = C.CFUNCTYPE(C.c_int, C.POINTER(Progress), u32p, C.c_void_p)

# (name, restype, argtypes)
_SIGS = [
    ("gbpe_ctx_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("gbpe_ctx_destroy", None, [C.c_void_p]),
    ("gbpe_ctx_trim", C.c_int, [C.c_void_p]),
    ("gbpe_ctx_limits", C.c_int, [C.c_void_p, u64p]),
    ("gbpe_last_error", C.c_char_p, [C.c_void_p]),
    ("gbpe_version", C.c_char_p, []),
    ("gbpe_abi_version", C.c_int, []),
    ("gbpe_trainer_stats_size", C.c_uint64, []),
    ("gbpe_kernel_count", C.c_int, []),
    ("gbpe_kernel_name", C.c_char_p, [C.c_int]),
    ("gbpe_word_boundary", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    ("gbpe_train", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.POINTER(TrainOpts), PROGRESS_CB,
                             C.c_void_p, u32p, C.c_uint32, u32p, u32p]),
    ("gbpe_trainer_create", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int,
                                      C.POINTER(TrainOpts), C.POINTER(C.c_void_p)]),
    ("gbpe_trainer_step", C.c_int, [C.c_void_p, C.c_uint32, u32p, u32p, u32p]),
    ("gbpe_trainer_stats_get", C.c_int, [C.c_void_p, C.POINTER(TrainerStats)]),
    ("gbpe_trainer_symbols", C.c_int, [C.c_void_p, u32p, C.c_uint64, u64p]),
    ("gbpe_trainer_pair_counts", C.c_int, [C.c_void_p, u32p, u32p, C.c_uint64, u64p]),
    ("gbpe_trainer_destroy", None, [C.c_void_p]),
    ("gbpe_trie_upload", C.c_int, [C.c_void_p, u32p, C.c_uint32, u32p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("gbpe_trie_free", None, [C.c_void_p]),
    ("gbpe_trie_compile", C.c_int, [C.c_void_p, u64p, C.c_uint32, C.c_void_p, C.c_uint64, u64p]),
    ("gbpe_dxft_pack", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                 u64p]),
    ("gbpe_trie_info", C.c_int, [C.c_void_p, u32p, u32p, u32p]),
    ("gbpe_encode", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, u32p, C.c_uint64, u64p]),
    ("gbpe_encode_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                     C.c_uint64, u64p]),
    ("gbpe_bpe_upload", C.c_int, [C.c_void_p, u32p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("gbpe_bpe_encode", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, u32p, C.c_uint64, u64p]),
    ("gbpe_bpe_free", None, [C.c_void_p]),
    ("gbpe_encode_last_timing", C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                          C.POINTER(C.c_double)]),
    ("gbpe_device_alloc", C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    ("gbpe_device_free", C.c_int, [C.c_void_p, C.c_void_p]),
    ("gbpe_memcpy_h2d", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    ("gbpe_memcpy_d2h", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    ("gbpe_synchronize", C.c_int, [C.c_void_p]),
    ("gbpe_pretokenize_gpt4", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    ("gbpe_pretokenize_gpt4_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    ("gbpe_ctx_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("gbpe_ctx_get_stream", C.c_void_p, [C.c_void_p]),
    ("gbpe_trainer_export_state", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, u64p, C.c_void_p, C.c_uint64, u64p,
                                            C.c_int]),
    ("gbpe_trainer_create_from_state", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int,
                                                 C.POINTER(TrainOpts), C.POINTER(C.c_void_p)]),
    ("gbpe_lexshard_create", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int, C.POINTER(TrainOpts),
                                       C.POINTER(C.c_void_p)]),
    ("gbpe_lexshard_build", C.c_int, [C.c_void_p, C.c_uint64]),
    ("gbpe_lexshard_info_get", C.c_int, [C.c_void_p, C.POINTER(LexShardInfo)]),
    ("gbpe_lexshard_copy", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64, C.c_int]),
    ("gbpe_lexshard_release", C.c_int, [C.c_void_p]),
    ("gbpe_lexshard_remap", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int]),
    ("gbpe_lexshard_destroy", None, [C.c_void_p]),
    ("gbpe_trainer_create_from_lexicon", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                                   C.c_uint64, C.c_uint64, C.c_int, C.POINTER(TrainOpts), C.c_void_p,
                                                   C.c_uint64, u64p, C.c_int, C.POINTER(C.c_void_p)]),
    ("gbpe_trainer_expand", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p, C.c_uint64, u64p,
                                      C.c_int]),
]

EXPORTED = [s[0] for s in _SIGS]

_lib = None


def load(path: str | None = None):
    """Load libgpubpe.so (raises OSError / RuntimeError when absent — no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"gpubpe native library not found at {p}: build it with `make -C gpu-bpe_amd` "
                           "(the HIP path is the only implementation; there is no CPU fallback)")
    lib = C.CDLL(p)
    for name, res, args in _SIGS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


class GpuBpeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def check(rc: int, ctx=None, what: str = ""):
    if rc == GBPE_OK:
        return
    msg = ""
    if ctx is not None:
        raw = load().gbpe_last_error(ctx)
        msg = raw.decode("utf-8", "replace") if raw else ""
    raise GpuBpeError(rc, f"{what}: {msg or 'gpubpe error'} (status {rc})")
