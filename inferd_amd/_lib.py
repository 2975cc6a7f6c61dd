"""ctypes binding of include/inferd_span.h (libinferd_span.so, built in-tree for gfx950).

There is no fallback: if the library is missing or cannot be loaded, every product
call raises.  Build it with `python -c "import __graft_entry__ as g; g.build()"` or
`make -C inferd_amd/csrc`.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# INFERD_LIB: another build of the same library (A/B timing runs of tools/ builds only)
LIB_PATH = os.environ.get("INFERD_LIB") or os.path.join(_HERE, "libinferd_span.so")

ABI_VERSION = 5   # inferd_abi_version() of the header this table binds
INFERD_OK = 0
INFERD_ERR_ARG, INFERD_ERR_NOMEM = 1, 4
EPI_NONE, EPI_RESID, EPI_SILU = 0, 1, 2
KV_PAGE = 64
PROF_CLASSES = ("rmsnorm", "qkv_gemm", "qk_norm_rope_kv", "attention", "o_gemm", "gateup_gemm", "down_gemm",
                "lm_head_argmax")

# symbol -> (restype, argtypes); the header is the source of truth
c_i32, c_i64, c_u64, c_u32, c_f, c_p = C.c_int32, C.c_int64, C.c_uint64, C.c_uint32, C.c_float, C.c_void_p


class SpanConfig(C.Structure):
    _fields_ = [(n, c_i32) for n in ("hidden", "intermediate", "heads", "kv_heads", "head_dim", "vocab",
                                     "first_layer", "n_layers", "has_embed", "has_lm_head")] + \
               [("rms_eps", c_f), ("rope_theta", c_f)] + \
               [(n, c_i32) for n in ("max_positions", "kv_pages", "max_tokens", "max_seqs", "skip_first_attn",
                                     "skip_last_mlp", "gateup_split_first", "gateup_split_last", "o_split_first",
                                     "o_split_last", "qkv_split_first", "qkv_split_last", "head_first", "head_rows",
                                     "final_norm_out")]


class Batch(C.Structure):
    _fields_ = [(n, c_i32) for n in ("n_seqs", "n_tokens", "max_q_len", "max_ctx_len", "max_pages", "decode")] + \
               [(n, c_p) for n in ("seq_start", "positions", "slots", "ctx_lens", "block_table")]


SIGNATURES = {
    "inferd_last_error": (C.c_char_p, []),
    "inferd_abi_version": (C.c_int, []),
    "inferd_span_create": (C.c_int, [C.POINTER(SpanConfig), C.POINTER(c_p)]),
    "inferd_span_destroy": (None, [c_p]),
    "inferd_span_get_config": (C.c_int, [c_p, C.POINTER(SpanConfig)]),
    "inferd_span_init_synthetic": (C.c_int, [c_p, c_u64, c_p]),
    "inferd_span_set_weight": (C.c_int, [c_p, c_i32, C.c_char_p, c_p, c_i64, c_i64, c_p]),
    "inferd_span_forward": (C.c_int, [c_p, C.POINTER(Batch), c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "inferd_span_profile_start": (C.c_int, [c_p, c_i32]),
    "inferd_span_profile_stop": (C.c_int, [c_p, C.POINTER(C.c_double), C.POINTER(c_i32), c_i32]),
    "inferd_span_lm_head": (C.c_int, [c_p, c_p, c_i32, c_p, c_p]),
    "inferd_span_io_elems": (C.c_int64, [c_p, c_i32, c_i32, c_i32, c_i32]),
    "inferd_span_head_shard": (C.c_int, [c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "inferd_argmax_combine": (C.c_int, [c_p, c_i32, c_i32, c_p, c_p]),
    "inferd_span_graph_capture": (C.c_int, [c_p, C.POINTER(Batch), c_i32, c_p, c_p, c_p, c_p, c_p, c_p,
                                            C.POINTER(c_p)]),
    "inferd_graph_launch": (C.c_int, [c_p, c_p]),
    "inferd_span_step": (C.c_int, [c_p, C.POINTER(Batch), c_i32, c_p, c_p, c_p, c_p, c_p, c_p]),
    "inferd_graph_destroy": (None, [c_p]),
    "inferd_span_error_flags": (C.c_int, [c_p, C.POINTER(c_i32)]),
    "inferd_span_kv_layer": (C.c_int, [c_p, c_i32, C.POINTER(c_p)]),
    "inferd_span_kv_clear": (C.c_int, [c_p, c_p]),
    "inferd_weightgen": (C.c_int, [c_p, c_i64, c_u64, c_u32, c_f, c_f, c_p]),
    "inferd_pack_weight": (C.c_int, [c_p, c_i64, c_i64, c_p, c_p]),
    "inferd_unpack_weight": (C.c_int, [c_p, c_i64, c_i64, c_p, c_p]),
    "inferd_rmsnorm": (C.c_int, [c_p, c_p, c_p, c_i32, c_i32, c_f, c_p]),
    "inferd_gemm": (C.c_int, [c_p, c_p, c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_p]),
    "inferd_rope_table": (C.c_int, [c_f, c_i32, c_i32, c_p, c_p, c_p]),
    "inferd_qk_norm_rope_kv": (C.c_int, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i32, c_i32, c_i32, c_f, c_p]),
    "inferd_attention": (C.c_int, [c_p, c_p, C.POINTER(Batch), c_i32, c_i32, c_p, c_p, c_i64, c_p]),
    "inferd_attention_workspace_bytes": (c_i64, [c_i32, c_i32, c_i32]),
    "inferd_kv_create": (C.c_int, [c_i32, C.POINTER(c_p)]),
    "inferd_kv_destroy": (None, [c_p]),
    "inferd_kv_reserve": (C.c_int, [c_p, c_u64, c_i32]),
    "inferd_kv_advance": (C.c_int, [c_p, c_u64, c_i32]),
    "inferd_kv_advance_many": (C.c_int, [c_p, C.POINTER(c_u64), c_i32, c_i32]),
    "inferd_kv_release": (C.c_int, [c_p, c_u64]),
    "inferd_kv_query": (C.c_int, [c_p, c_u64, C.POINTER(c_i32), C.POINTER(c_i32)]),
    "inferd_kv_pages": (C.c_int, [c_p, c_u64, C.POINTER(c_i32), c_i32]),
    "inferd_kv_free_pages": (C.c_int, [c_p, C.POINTER(c_i32)]),
    "inferd_kv_batch_words": (c_i64, [c_p, C.POINTER(c_u64), C.POINTER(c_i32), c_i32]),
    "inferd_kv_build_batch": (C.c_int, [c_p, C.POINTER(c_u64), C.POINTER(c_i32), c_i32, C.POINTER(c_i32), c_i64, c_p,
                                        C.POINTER(Batch)]),
    "inferd_kv_decode_batch_words": (c_i64, [c_p, C.POINTER(c_u64), c_i32, c_i32]),
    "inferd_kv_build_decode_batch": (C.c_int, [c_p, C.POINTER(c_u64), c_i32, c_i32, C.POINTER(c_i32), c_i64, c_p,
                                               C.POINTER(Batch)]),
    "inferd_probe_hbm_read": (C.c_int, [c_p, c_i64, c_p, c_i32, c_p]),
    "inferd_probe_mfma": (C.c_int, [c_i32, c_i32, c_p, c_p, C.POINTER(C.c_double)]),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load the C-ABI library (raises OSError/RuntimeError when unavailable)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libinferd_span.so not built ({path}); run __graft_entry__.build()")
    lib = C.CDLL(path)
    lib.inferd_abi_version.restype = C.c_int
    if lib.inferd_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{path}: ABI version {lib.inferd_abi_version()}, this binding needs {ABI_VERSION}; rebuild")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int):
    if rc != INFERD_OK:
        msg = load().inferd_last_error()
        msg = msg.decode() if msg else ''
        if rc == INFERD_ERR_NOMEM:
            raise RuntimeError(msg)
        raise RuntimeError(f"inferd error {rc}: {msg}")


def ptr(t) -> int | None:
    """device pointer of a torch tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def batch_struct(words, shape) -> Batch:
    """The InferdBatch of a descriptor (int32 words tensor + shape [n_seqs, n_tokens, max_q_len,
    max_ctx_len, max_pages, decode], e.g. runtime.KvTable.build_batch's), for the single-op
    entry points called through this binding.  The words must outlive every use."""
    n, m, mq, mc, mp, dec = (int(v) for v in shape)
    assert words.numel() >= n + 1 + 2 * m + n + n * mp
    base = words.data_ptr()
    o = [0, n + 1, n + 1 + m, n + 1 + 2 * m, n + 1 + 2 * m + n]
    return Batch(n_seqs=n, n_tokens=m, max_q_len=mq, max_ctx_len=mc, max_pages=mp, decode=dec,
                 seq_start=base + 4 * o[0], positions=base + 4 * o[1], slots=base + 4 * o[2],
                 ctx_lens=base + 4 * o[3], block_table=base + 4 * o[4])


def stream_ptr(stream=None) -> int | None:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
