"""Host-side span runtime: one InferdSpan handle (C-ABI) per pipeline stage, a paged KV
pool allocator and the per-session cache table.

Semantics mirrored from the reference:
  * a span is `layers[start_layer .. end_layer]` plus embed (first) / final norm +
    lm_head (last)                                   -- split_model.py:92-102
  * per-session KV cache keyed by session id, prefill then single-token steps whose
    positions continue from the cached length        -- qwen3_server_module.py:220,253;
                                                        client.py:244-266
  * a session-less call is a stateless full recompute (positions 0..T-1) whose cache
    pages are released afterwards                    -- partitioned_models.py:139-151
The page table and the batch descriptors are native (inferd_kv_*, kvtable.hip); device
memory for activations is torch (plumbing); all compute runs in libinferd_span.so, driven
through its PyTorch-ROCm extension (torch.ops.inferd / torch.classes.inferd, csrc/torch_ops.cpp).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass

import torch

from .ops import KV_PAGE, PROF_CLASSES, ops as T  # noqa: F401  (KV_PAGE re-exported: pipeline, tests)


@dataclass(frozen=True)
class ModelDims:
    """Qwen3 model constants (0.6B row == models/qwen3/qwen3_config.py:10-24)."""
    name: str
    hidden: int
    intermediate: int
    heads: int
    kv_heads: int
    layers: int
    vocab: int
    head_dim: int = 128
    eps: float = 1e-6
    rope_theta: float = 1_000_000.0
    max_positions: int = 40960

    def params_per_layer(self) -> int:
        h, I, H, KV, d = self.hidden, self.intermediate, self.heads, self.kv_heads, self.head_dim
        return h * (H + 2 * KV) * d + H * d * h + 3 * h * I + 2 * h + 2 * d


MODELS = {
    "tiny": ModelDims("tiny", 256, 512, 4, 2, 4, 1024),
    "qwen3-0.6b": ModelDims("qwen3-0.6b", 1024, 3072, 16, 8, 28, 151936),
    "qwen3-8b": ModelDims("qwen3-8b", 4096, 12288, 32, 8, 36, 151936),
    "qwen3-32b": ModelDims("qwen3-32b", 5120, 25600, 64, 8, 64, 151936),
}

# Counter-based synthetic weights (the engine's inferd_weightgen; oracle/weightgen.py
# defines the same values): tensor ids and (scale, center) per kind.
LAYER_TENSOR_IDS = {"q_proj": 0, "k_proj": 1, "v_proj": 2, "o_proj": 3, "q_norm": 4, "k_norm": 5,
                    "input_layernorm": 6, "post_attention_layernorm": 7, "gate_proj": 8, "up_proj": 9,
                    "down_proj": 10}
GLOBAL_TENSOR_IDS = {"embed_tokens": 0xFFFF0000, "norm": 0xFFFF0001, "lm_head": 0xFFFF0002}
LINEAR_SCALE, NORM_SCALE = 0.034641016151377546, 0.1
# "peaked" profile (oracle/weightgen.py documents it): embed * EMBED_BOOST and lm_head row
# p(t) = (PERM_MUL * t + PERM_ADD) mod V gets LM_MIX * embed[t] added -- large top-1 logit
# margins for greedy-parity runs; every layer weight is unchanged.
EMBED_BOOST, LM_MIX = 64.0, 1.0
PERM_MUL, PERM_ADD = 7919, 17
# embedding factor per profile ("peaked_deep": x512 for Qwen3-8B-deep spans, whose random
# layers otherwise drown the x64 embedding; oracle/weightgen.py PROFILE_BOOST)
PROFILE_BOOST = {"peaked": EMBED_BOOST, "peaked_deep": 512.0}


def gen_tensor(seed: int, tid: int, shape, norm: bool, device) -> torch.Tensor:
    """One synthetic weight tensor (bf16, row-major) generated on the device."""
    n = 1
    for s in shape:
        n *= s
    device = torch.device(device)
    t = torch.empty(n, dtype=torch.bfloat16, device=device)
    with torch.cuda.device(device):
        T.weightgen(t, seed, tid, NORM_SCALE if norm else LINEAR_SCALE, 1.0 if norm else 0.0)
    return t.reshape(tuple(shape))


class Batch:
    """A batch descriptor: the device (or host) int32 words [seq_start | positions | slots |
    ctx_lens | block_table] the native table wrote and their shape [n_seqs, n_tokens, max_q_len,
    max_ctx_len, max_pages, decode] (InferdBatch, include/inferd_span.h).  Holding it keeps the
    words alive for the launches that read them."""
    __slots__ = ("words", "shape")

    def __init__(self, words: torch.Tensor, shape):
        self.words, self.shape = words, [int(v) for v in shape]

    n_seqs = property(lambda self: self.shape[0])
    n_tokens = property(lambda self: self.shape[1])
    max_q_len = property(lambda self: self.shape[2])
    max_ctx_len = property(lambda self: self.shape[3])
    max_pages = property(lambda self: self.shape[4])
    decode = property(lambda self: self.shape[5])


class KvTable:
    """The span's KV page table: the native one behind the C-ABI (inferd_kv_*, kvtable.hip).
    Sequences are 64-bit keys; pages come lowest id first."""

    def __init__(self, n_pages: int):
        self.n_pages = n_pages
        self.handle = T.kv_create(n_pages)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            T.kv_destroy(h)
            self.handle = None

    def reserve(self, seq: int, n_new: int):
        T.kv_reserve(self.handle, seq, n_new)

    def advance(self, seq: int, n: int):
        T.kv_advance(self.handle, [seq], n)

    def advance_many(self, seqs, n: int):
        """every sequence of `seqs` by n tokens; all or nothing"""
        T.kv_advance(self.handle, list(seqs), n)

    def release(self, seq: int):
        T.kv_release(self.handle, seq)

    def query(self, seq: int):
        """(cached length or -1 if absent, reserved pages)"""
        return tuple(T.kv_query(self.handle, seq))

    def pages(self, seq: int) -> list:
        return list(T.kv_pages(self.handle, seq))

    @property
    def n_free(self) -> int:
        return T.kv_free_pages(self.handle)

    def build_batch(self, seqs, device) -> Batch:
        """seqs: [(key, n_new)], pages already reserved.  The words are built natively, then
        copied to `device`."""
        words, shape = T.kv_build_batch(self.handle, [k for k, _ in seqs], [m for _, m in seqs],
                                        torch.device(device))
        return Batch(words, shape)


class SeqView:
    """One sequence of a span's KvTable under a caller's session key: `length` (cached
    tokens; assigning a larger value advances it) and `pages`, read from the native table."""
    __slots__ = ("kv", "seq")

    def __init__(self, kv: KvTable, seq: int):
        self.kv, self.seq = kv, seq

    @property
    def length(self) -> int:
        return max(self.kv.query(self.seq)[0], 0)

    @length.setter
    def length(self, v: int):
        self.kv.advance(self.seq, v - self.length)

    @property
    def pages(self) -> list:
        return self.kv.pages(self.seq)


class DecodeGraph:
    """One decode step of a fixed set of sessions captured as a HIP graph
    (torch.classes.inferd.DecodeGraph: inferd_span_graph_capture with advance=1 over the
    native decode descriptor of inferd_kv_build_decode_batch): every launch decodes one more
    token of each session, reading `ids` (first span) or `x`, writing `hidden_out` and/or
    `next_ids` -- fixed device buffers chosen at capture, kept alive by the graph object.
    `ids` and `next_ids` may alias (greedy feedback on a single-span model).  Pages for
    `n_steps` tokens are reserved up front; launching more than n_steps times raises.
    `logits` (last span, optional): bf16 [sessions, vocab] receives every replay's last-row
    logits."""

    def __init__(self, span: "SpanRuntime", sessions, n_steps: int, ids=None, x=None, hidden_out=None,
                 next_ids=None, logits=None):
        self.span, self.n_steps = span, n_steps
        # reserve(sid, 0) enters a never-prefilled session into the native table (empty), so a
        # graph may also start a session from position 0
        self.states = [span.reserve(sid, 0) for sid in sessions]
        with torch.cuda.device(span.device):
            self.graph = torch.classes.inferd.DecodeGraph(span.handle, span.kv.handle, [st.seq for st in self.states],
                                                          n_steps, ids, x, hidden_out, next_ids, logits, span.device)

    @property
    def launched(self) -> int:
        return self.n_steps - self.graph.steps_left()

    def launch(self, stream=None):
        if stream is None:
            self.graph.launch()
        else:
            with torch.cuda.stream(stream):
                self.graph.launch()

    def launch_eager(self):
        """The same step launched kernel by kernel on the current stream (inferd_span_step): no
        graph launch on the GPU, host launch time instead."""
        self.graph.launch_eager()


class SpanRuntime:
    """One layer span on one GPU (FirstStage / StageInner / LastStage compute)."""

    def __init__(self, dims: ModelDims, first_layer: int, n_layers: int, *, has_embed: bool,
                 has_lm_head: bool, kv_pages: int = 256, max_tokens: int = 4096, max_seqs: int = 64,
                 max_positions: int | None = None, device: str | torch.device = "cuda",
                 skip_first_attn: bool = False, skip_last_mlp: bool = False, gateup_split_first: int = 0,
                 gateup_split_last: int = 0, o_split_first: bool = False, o_split_last: bool = False,
                 qkv_split_first: bool = False, qkv_split_last: bool = False, head_first: int = 0,
                 head_rows: int = 0, final_norm_out: bool = False):
        """skip_first_attn / skip_last_mlp: sub-layer stage boundaries (InferdSpanConfig): the
        span starts at its first layer's MLP half (x = that layer's post-attention residual)
        and/or ends after its last layer's attention half (hidden out = that residual).
        gateup_split_first / _last: the boundary sits inside that layer's gate/up projection at
        this column; decode calls then hand over a record (h1, then the packed SwiGLU product,
        record_elems()) instead of h1 alone.  o_split_first / _last: the boundary sits between a
        layer's attention and its o projection; every call hands over a record (the layer's input
        residual, then the attention output: o_record_elems()).  qkv_split_first / _last: the
        boundary sits between a layer's q/k/v projection and its attention; a pure decode call
        hands over a record (x, then the raw q/k/v rows: q_record_elems()), other calls x alone
        (the receiver runs the whole layer).
        head_first / head_rows: this span's shard of a vocab-parallel lm_head (head_shard());
        final_norm_out: the model's last span of such a head -- it owns the final norm, and its
        forward / decode steps write the final-normed last rows, fragment-packed (normed_elems()),
        to the hidden output instead of the last layer's rows (InferdSpanConfig, ABI 5)."""
        self.dims = dims
        self.first_layer, self.n_layers = first_layer, n_layers
        self.has_embed, self.has_lm_head = has_embed, has_lm_head
        self.skip_first_attn, self.skip_last_mlp = bool(skip_first_attn), bool(skip_last_mlp)
        self.gateup_split_first, self.gateup_split_last = int(gateup_split_first), int(gateup_split_last)
        self.o_split_first, self.o_split_last = bool(o_split_first), bool(o_split_last)
        self.qkv_split_first, self.qkv_split_last = bool(qkv_split_first), bool(qkv_split_last)
        self.head_first, self.head_rows, self.final_norm_out = int(head_first), int(head_rows), bool(final_norm_out)
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.max_tokens, self.max_seqs = max_tokens, max_seqs
        self.max_positions = max_positions or dims.max_positions
        cfg = [dims.hidden, dims.intermediate, dims.heads, dims.kv_heads, dims.head_dim, dims.vocab, first_layer,
               n_layers, int(has_embed), int(has_lm_head), self.max_positions, kv_pages, max_tokens, max_seqs,
               int(skip_first_attn), int(skip_last_mlp), int(gateup_split_first), int(gateup_split_last),
               int(o_split_first), int(o_split_last), int(qkv_split_first), int(qkv_split_last), int(head_first),
               int(head_rows), int(final_norm_out)]
        self.handle = None
        self.handle = T.span_create(cfg, dims.eps, dims.rope_theta, self.device)
        self.kv = KvTable(kv_pages)
        self.sessions: dict = {}   # session key -> SeqView
        self._seq_ids = itertools.count(1)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            T.span_destroy(h)
            self.handle = None

    def record_elems(self, rows: int) -> int:
        """bf16 elements of a decode hand-off record at a gate/up boundary: h1 [rows][hidden]
        then the packed SwiGLU product [rows rounded to 16][intermediate]
        (include/inferd_span.h, InferdSpanConfig gateup_split_*)."""
        return rows * self.dims.hidden + (rows + 15) // 16 * 16 * self.dims.intermediate

    def o_record_elems(self, rows: int, decode: bool) -> int:
        """bf16 elements of an attention|o-boundary record: the layer's input residual
        [rows][hidden], then the attention output [rows, or rows rounded to 16 in a pure decode
        call (fragment-packed)][heads * 128]."""
        d = self.dims
        return rows * d.hidden + ((rows + 15) // 16 * 16 if decode else rows) * d.heads * d.head_dim

    def q_record_elems(self, rows: int, decode: bool) -> int:
        """bf16 elements of a q/k/v|attention-boundary hand-off: x [rows][hidden], then (a pure
        decode call) the raw q/k/v rows [rows][(heads + 2 kv_heads) * head_dim]."""
        d = self.dims
        return rows * d.hidden + (rows * (d.heads + 2 * d.kv_heads) * d.head_dim if decode else 0)

    def normed_elems(self, rows: int) -> int:
        """bf16 elements of a final_norm_out span's hand-off: the final-normed last rows,
        fragment-packed over 16-row tiles (the A operand of every stage's head_shard)."""
        return (rows + 15) // 16 * 16 * self.dims.hidden

    @property
    def head_range(self):
        """(first, rows) of the lm_head rows this span owns: all of them with the whole head,
        its shard of a vocab-parallel head, or (0, 0)."""
        return (0, self.dims.vocab) if self.has_lm_head else (self.head_first, self.head_rows)

    # ----------------------------------------------------------------- weights
    def _stream(self):
        return torch.cuda.current_stream(self.device)

    def init_synthetic(self, seed: int, profile: str = "random"):
        """Counter-based weights (the offline stand-in for a checkpoint).  profile="peaked" /
        "peaked_deep" re-compose embed / lm_head as oracle/weightgen.py's peaked profiles (large
        greedy margins for token-exact parity runs)."""
        if profile != "random" and profile not in PROFILE_BOOST:
            raise ValueError(f"unknown synthetic profile {profile!r}")
        with torch.cuda.device(self.device):
            T.span_init_synthetic(self.handle, seed, self.device)
            h0, hn = self.head_range
            if profile in PROFILE_BOOST and (self.has_embed or hn):
                d = self.dims
                emb = gen_tensor(seed, GLOBAL_TENSOR_IDS["embed_tokens"], (d.vocab, d.hidden), False,
                                 self.device).float()
                if self.has_embed:
                    self.set_weight(-1, "embed_tokens", (emb * PROFILE_BOOST[profile]).to(torch.bfloat16))
                if hn:     # the whole head or this span's rows of it
                    lm = gen_tensor(seed, GLOBAL_TENSOR_IDS["lm_head"], (d.vocab, d.hidden), False,
                                    self.device).float()
                    perm = (torch.arange(d.vocab, device=self.device, dtype=torch.int64) * PERM_MUL + PERM_ADD) \
                        % d.vocab
                    lm[perm] = lm[perm] + LM_MIX * emb
                    self.set_weight(-1, "lm_head", lm[h0:h0 + hn].to(torch.bfloat16).contiguous())
                    del lm
                del emb
            self._stream().synchronize()

    def set_weight(self, layer: int, name: str, w: torch.Tensor):
        """layer: span-local index or -1 for embed_tokens / norm / lm_head.  Packs on this
        span's device and stream, then waits so the source tensor may be freed."""
        with torch.cuda.device(self.device):
            w = w.to(device=self.device, dtype=torch.bfloat16).contiguous()
            T.span_set_weight(self.handle, layer, name, w)
            self._stream().synchronize()

    def load_layer_state_dict(self, layer: int, sd: dict):
        """Keys as in Qwen3DecoderLayer (qwen3_server_module.py:165-176): self_attn.q_proj.weight ...
        (any order: the span's RMSNorms read their weights as set)."""
        items = [(k.split(".")[-2] if k.endswith(".weight") else k, v) for k, v in sd.items()]
        for leaf, v in items:
            self.set_weight(layer, leaf, v)

    def check_errors(self):
        """Read (and clear) the span's sticky device error flags; raise on any.  Bit 0: a
        token id outside [0, vocab) reached the embedding gather (the reference's
        nn.Embedding raises IndexError); bit 1: a decode graph ran past its reserved pages."""
        f = T.span_error_flags(self.handle, self.device)
        if f & 1:
            raise IndexError("index out of range in self (token id outside the vocabulary)")
        if f:
            raise RuntimeError(f"span device error flags 0x{f:x} (decode slot overflow)")

    # ----------------------------------------------------------------- sessions
    def release(self, session_id):
        st = self.sessions.pop(session_id, None)
        if st is not None:
            self.kv.release(st.seq)

    def release_all(self):
        for sid in list(self.sessions):
            self.release(sid)

    def _seq(self, session_id) -> SeqView:
        st = self.sessions.get(session_id)
        if st is None:
            st = self.sessions[session_id] = SeqView(self.kv, next(self._seq_ids))
        return st

    def build_batch(self, seqs) -> Batch:
        """seqs: [(SeqView, n_new)] with pages reserved -> the Batch (it holds its words)."""
        return self.kv.build_batch([(st.seq, n) for st, n in seqs], self.device)

    # ----------------------------------------------------------------- fast path
    def run(self, batch, ids=None, x=None, hidden=None, next_ids=None, logits=None, layers=None, stream=None):
        """Launch one span forward on a prebuilt Batch with caller-owned device tensors
        (no host sync, no allocation).  Used by the pipeline runtime and the bench."""
        if stream is None:
            T.span_forward(self.handle, batch.words, batch.shape, ids, x, hidden, next_ids, logits, layers)
        else:
            with torch.cuda.stream(stream):
                T.span_forward(self.handle, batch.words, batch.shape, ids, x, hidden, next_ids, logits, layers)

    def profile_start(self, max_pairs: int = 1 << 16):
        T.span_profile_start(self.handle, max_pairs)

    def profile_stop(self) -> dict:
        """{class: (total_ms, launches)} from the HIP events recorded since profile_start."""
        ms, cnt = T.span_profile_stop(self.handle, len(PROF_CLASSES))
        return {name: (ms[i], cnt[i]) for i, name in enumerate(PROF_CLASSES)}

    def reserve(self, session_id, n_tokens: int) -> SeqView:
        """Make sure `session_id` has pages for n_tokens more tokens (no forward)."""
        st = self._seq(session_id)
        self.kv.reserve(st.seq, n_tokens)
        return st

    def head_shard(self, normed: torch.Tensor, rows: int, keys_in: torch.Tensor | None = None,
                   keys_out: torch.Tensor | None = None, ids: torch.Tensor | None = None,
                   logits: torch.Tensor | None = None):
        """This span's lm_head rows (head_range) over `rows` final-normed rows (fragment-packed,
        normed_elems): keys_out int64 [rows] = max(keys_in, each row's (logit, lowest global index)
        key over the shard), ids int32 [rows] = the greedy token of that key, logits bf16 [rows,
        head rows] -- every output optional (torch.ops.inferd.span_head_shard; stream ordered, no
        sync).  Chained over all shards, the ids are argmax over the whole vocabulary."""
        T.span_head_shard(self.handle, normed, rows, keys_in, keys_out, ids, logits)

    @torch.no_grad()
    def lm_head(self, hidden: torch.Tensor) -> torch.Tensor:
        """Final norm + lm_head over every row of `hidden` (bf16 [rows, vocab]), in chunks of
        max_tokens rows -- LastStage's all-position logits (partitioned_models.py:95-96)."""
        d = self.dims
        with torch.cuda.device(self.device):
            x = hidden.to(device=self.device, dtype=torch.bfloat16).reshape(-1, d.hidden).contiguous()
            out = torch.empty((x.shape[0], d.vocab), dtype=torch.bfloat16, device=self.device)
            for r0 in range(0, x.shape[0], self.max_tokens):
                n = min(self.max_tokens, x.shape[0] - r0)
                T.span_lm_head(self.handle, x[r0:r0 + n], out[r0:r0 + n])
        return out

    # ----------------------------------------------------------------- forward
    def _plan(self, requests):
        """Cut the requests into engine calls of <= max_tokens rows and <= max_seqs
        sequences, in order: [[(request index, first row within it, rows)]].  A request
        longer than what is left of a call continues in the next call (chunked prefill:
        the chunk attends to the pages its earlier chunks wrote), so two pieces of one
        sequence never share a call."""
        calls, cur, cur_tok = [], [], 0
        for i, (_, n) in enumerate(requests):
            done = 0
            while done < n:
                if len(cur) == self.max_seqs or cur_tok == self.max_tokens:
                    calls.append(cur)
                    cur, cur_tok = [], 0
                take = min(n - done, self.max_tokens - cur_tok)
                cur.append((i, done, take))
                cur_tok += take
                done += take
        if cur:
            calls.append(cur)
        return calls

    @torch.no_grad()
    def forward(self, requests, ids: torch.Tensor | None = None, x: torch.Tensor | None = None, *,
                want_hidden: bool = True, want_next_ids: bool = False, want_logits: bool = False,
                want_layers: bool = False) -> dict:
        """requests: list of (session_id or None, n_new_tokens), tokens concatenated in order.
        ids: int tensor [M] (first span); x: bf16 [M, hidden] (other spans).  A session-less
        request is a stateless recompute from position 0 whose pages are released afterwards.
        Calls larger than the span's workspace (max_tokens rows / max_seqs sequences) run as
        several engine calls, long sequences chunk by chunk through their own pages."""
        d = self.dims
        dev = self.device
        if not requests or any(n <= 0 for _, n in requests):
            raise ValueError("forward needs at least one request with n_new_tokens >= 1")
        sids = [sid for sid, _ in requests if sid is not None]
        if len(set(sids)) != len(sids):
            raise ValueError("a session may appear only once per forward call")
        total = sum(n for _, n in requests)
        # hand-off records (InferdSpanConfig): decode calls at a gate/up boundary, every call at an
        # attention|o boundary (the attention output fragment-packed in a pure decode call)
        pure = all(n == 1 for _, n in requests)
        packed = total <= 64 and pure
        in_rec = (self.record_elems(total) if self.gateup_split_first and total <= 64 else
                  self.o_record_elems(total, packed) if self.o_split_first else
                  self.q_record_elems(total, True) if self.qkv_split_first and pure else 0)
        out_rec = (self.record_elems(total) if self.gateup_split_last and total <= 64 else
                   self.o_record_elems(total, packed) if self.o_split_last else
                   self.q_record_elems(total, True) if self.qkv_split_last and pure else 0)
        with torch.cuda.device(dev):
            ids_d = x_d = None
            if self.has_embed:
                if ids is None:
                    raise ValueError("first span needs token ids")
                ids_d = ids.to(device=dev, dtype=torch.int32).reshape(-1).contiguous()
                if ids_d.numel() != total:
                    raise ValueError(f"{ids_d.numel()} ids for {total} request tokens")
                lo, hi = torch.aminmax(ids_d)
                if int(lo) < 0 or int(hi) >= d.vocab:     # nn.Embedding's IndexError (reference :48)
                    raise IndexError("index out of range in self (token id outside the vocabulary)")
            else:
                if x is None:
                    raise ValueError("span needs hidden states x")
                if in_rec:   # a hand-off record (h1 | act, or x | attention output)
                    x_d = x.to(device=dev, dtype=torch.bfloat16).reshape(-1).contiguous()
                    if x_d.numel() < in_rec:
                        raise ValueError(f"x: a {in_rec}-element hand-off record expected for {total} rows, "
                                         f"got {x_d.numel()}")
                else:
                    x_d = x.to(device=dev, dtype=torch.bfloat16).reshape(total, d.hidden).contiguous()
            rec_in = x_d is not None and x_d.dim() == 1
            rec_out = bool(out_rec) and want_hidden
            if (self.o_split_last or self.qkv_split_last) and not want_hidden:
                raise ValueError("a span ending before an o projection or an attention always hands over its record")
            temp = []
            states = []
            for sid, _ in requests:
                if sid is None:   # stateless: a table sequence of its own, released below
                    st = SeqView(self.kv, next(self._seq_ids))
                    temp.append(st)
                else:
                    st = self._seq(sid)
                states.append(st)
            ok, advanced = False, False
            try:
                for st, (_, n) in zip(states, requests):
                    self.kv.reserve(st.seq, n)
                B = len(requests)
                lm = self.has_lm_head
                hid = torch.empty((total, d.hidden), dtype=torch.bfloat16, device=dev) if want_hidden else None
                rec = None
                if rec_out:      # h1 then the packed act columns (or x then the attention output)
                    rec = torch.empty(out_rec, dtype=torch.bfloat16, device=dev)
                    hid = rec[:total * d.hidden].view(total, d.hidden)
                if self.final_norm_out and want_hidden:     # the final-normed last rows (packed)
                    if len(self._plan(requests)) > 1:
                        raise ValueError("a final_norm_out span hands over one engine call's normed rows")
                    hid = torch.zeros(self.normed_elems(B), dtype=torch.bfloat16, device=dev)
                nid = torch.empty((B,), dtype=torch.int32, device=dev) if (want_next_ids and lm) else None
                lg = torch.empty((B, d.vocab), dtype=torch.bfloat16, device=dev) if (want_logits and lm) else None
                lay = torch.empty((self.n_layers, total, d.hidden), dtype=torch.bfloat16, device=dev) \
                    if want_layers else None
                row0 = [0]
                for _, n in requests:
                    row0.append(row0[-1] + n)
                calls = self._plan(requests)
                if (rec_in or rec_out) and len(calls) > 1:
                    raise ValueError("a call handing over a record is one engine call "
                                     f"(at most {self.max_tokens} tokens / {self.max_seqs} sequences)")
                if (self.gateup_split_first or self.gateup_split_last) and \
                        total > 64 and any(sum(t for _, _, t in c) <= 64 for c in calls):
                    raise ValueError("across a gate/up boundary a call is either one decode-sized engine call "
                                     "(<= 64 rows, record hand-off) or only prefill-sized ones (> 64 rows)")
                if (self.qkv_split_first or self.qkv_split_last) and not pure and \
                        any(all(t == 1 for _, _, t in c) for c in calls):
                    raise ValueError("across a q/k/v|attention boundary an engine call of one-token pieces is a "
                                     "decode call (record hand-off): split such a request differently")
                if (self.o_split_first or self.o_split_last) and len(calls) > 1:
                    raise ValueError("across an attention|o boundary a forward call is one engine call "
                                     f"(at most {self.max_tokens} tokens / {self.max_seqs} sequences)")
                keep = []
                for call in calls:
                    r0 = row0[call[0][0]] + call[0][1]
                    m = sum(t for _, _, t in call)
                    single = len(calls) == 1
                    batch = self.build_batch([(states[i], t) for i, _, t in call])
                    keep.append(batch)
                    finals = [j for j, (i, s0, t) in enumerate(call) if s0 + t == requests[i][1]]
                    c_nid = nid if single else (torch.empty((len(call),), dtype=torch.int32, device=dev)
                                                if nid is not None and finals else None)
                    c_lg = lg if single else (torch.empty((len(call), d.vocab), dtype=torch.bfloat16, device=dev)
                                              if lg is not None and finals else None)
                    c_lay = lay if single else (torch.empty((self.n_layers, m, d.hidden), dtype=torch.bfloat16,
                                                            device=dev) if lay is not None else None)
                    self.run(batch, ids=None if ids_d is None else ids_d[r0:r0 + m],
                             x=None if x_d is None else (x_d if rec_in else x_d[r0:r0 + m]),
                             hidden=None if hid is None else (rec if rec is not None else
                                                              hid if self.final_norm_out else hid[r0:r0 + m]),
                             next_ids=c_nid, logits=c_lg, layers=c_lay)
                    for i, _, t in call:
                        self.kv.advance(states[i].seq, t)
                    advanced = True
                    if not single:
                        if finals:
                            dst = torch.tensor([call[j][0] for j in finals], device=dev)
                            src = torch.tensor(finals, device=dev)
                            if c_nid is not None:
                                nid[dst] = c_nid[src]
                            if c_lg is not None:
                                lg[dst] = c_lg[src]
                        if c_lay is not None:
                            lay[:, r0:r0 + m] = c_lay
                        keep.append((c_nid, c_lg, c_lay))
                ok = True
            finally:
                for st in temp:
                    self.kv.release(st.seq)
                if not ok and advanced:   # a chunked call that failed part-way leaves no
                    for sid in sids:      # half-advanced session behind: drop its sessions
                        self.release(sid)
        out = {}
        if hid is not None:
            out["hidden"] = hid
        if rec_out:
            out["record"] = rec
        if nid is not None:
            out["next_ids"] = nid
        if lg is not None:
            out["logits"] = lg
        if lay is not None:
            out["layers"] = lay
        # batch descriptors and inputs stay referenced until the caller is done with the
        # outputs (the launches are stream-ordered, nothing here synchronises)
        out["_keep"] = (keep, ids_d, x_d)
        return out
