"""FuzzyAhoCorasickBuilder / FuzzyAhoCorasick: the crate's public surface (builder.rs, query.rs,
prefilter.rs, replacer.rs) over the C ABI of include/fac.h. Every search goes to the GPU."""
from __future__ import annotations

import ctypes
import os
import sys
import time
from typing import Iterable, List, Optional, Tuple

from . import _native

_TIMING = bool(os.environ.get("FAC_TIMING"))  # diagnostics: host-side phase times
from .matches import FuzzyMatch, FuzzyMatches
from .structs import (DeviceError, FuzzyLimits, FuzzyPenalties, HaystackTooLarge, Order, Overlap,
                      Pattern, SearchOptions, Similarity, UnsupportedConfiguration, f32)


def _default_device() -> int:
    for var in ("FAC_DEVICE", "LOCAL_RANK"):
        if var in os.environ:
            return int(os.environ[var])
    return 0


def _raise(rc: int, err_graphemes: int = 0):
    if rc == _native.FAC_E_HAYSTACK_TOO_LARGE:
        raise HaystackTooLarge(err_graphemes)
    if rc == _native.FAC_E_UNSUPPORTED:
        raise UnsupportedConfiguration(_native.last_error())
    raise DeviceError(rc, _native.last_error())


class FuzzyAhoCorasickBuilder:
    """builder.rs:22-168. Chainable; `build` uploads the automaton to the GPU."""

    def __init__(self):
        self._similarity: Optional[Similarity] = None
        self._limits: Optional[FuzzyLimits] = None
        self._penalties = FuzzyPenalties()
        self._case_insensitive = False
        self._beam_width: Optional[int] = None
        self._auto_beam: Optional[Tuple[int, int]] = None
        self._mappings: List[Tuple[str, str, float]] = []
        self._min_symbol_similarity = 0.0
        self._device = _default_device()

    @classmethod
    def new(cls) -> "FuzzyAhoCorasickBuilder":
        return cls()

    def similarity(self, sim: Similarity) -> "FuzzyAhoCorasickBuilder":
        self._similarity = sim
        return self

    def fuzzy(self, limits: FuzzyLimits) -> "FuzzyAhoCorasickBuilder":
        self._limits = limits.finalize()
        return self

    def penalties(self, p: FuzzyPenalties) -> "FuzzyAhoCorasickBuilder":
        self._penalties = p
        return self

    def case_insensitive(self, value: bool) -> "FuzzyAhoCorasickBuilder":
        self._case_insensitive = bool(value)
        return self

    def beam_width(self, width: int) -> "FuzzyAhoCorasickBuilder":
        self._beam_width = int(width)
        return self

    def auto_beam(self, budget: int, width: int) -> "FuzzyAhoCorasickBuilder":
        self._auto_beam = (int(budget), int(width))
        return self

    def mapping(self, a: str, b: str) -> "FuzzyAhoCorasickBuilder":
        return self.mapping_scored(a, b, 1.0)

    def mapping_scored(self, a: str, b: str, score: float) -> "FuzzyAhoCorasickBuilder":
        self._mappings.append((a, b, f32(score)))
        return self

    def min_symbol_similarity(self, m: float) -> "FuzzyAhoCorasickBuilder":
        self._min_symbol_similarity = f32(m)
        return self

    def device(self, ordinal: int) -> "FuzzyAhoCorasickBuilder":
        """Extension: HIP device that holds this engine's tables."""
        self._device = int(ordinal)
        return self

    def build(self, inputs: Iterable) -> "FuzzyAhoCorasick":
        patterns = [Pattern.from_(x) for x in inputs]
        return FuzzyAhoCorasick(self, patterns)

    def build_replacer(self, pairs: Iterable) -> "FuzzyReplacer":
        pats, repl = [], []
        for p, r in pairs:
            pats.append(Pattern.from_(p))
            repl.append(str(r))
        return FuzzyReplacer(self.build(pats), repl)


class FuzzyAhoCorasick:
    """structs.rs:528-567 + search/query entry points (query.rs:30-202)."""

    def __init__(self, builder: FuzzyAhoCorasickBuilder, patterns: List[Pattern]):
        self.patterns_ = patterns
        self.builder = builder
        self._keep = []  # keep ctypes buffers alive during the call
        cfg = _native.fac_config()
        cfg.case_insensitive = int(builder._case_insensitive)
        cfg.has_limits = int(builder._limits is not None)
        cfg.limits = (builder._limits or FuzzyLimits()).to_c()
        pen = builder._penalties
        cfg.penalty_insertion = pen.insertion
        cfg.penalty_deletion = pen.deletion
        cfg.penalty_substitution = pen.substitution
        cfg.penalty_swap = pen.swap
        cfg.beam_width = builder._beam_width or 0
        if builder._beam_width == 0:
            raise ValueError("beam_width must be >= 1")
        cfg.has_auto_beam = int(builder._auto_beam is not None)
        if builder._auto_beam:
            cfg.auto_beam_budget, cfg.auto_beam_width = builder._auto_beam
        cfg.min_symbol_similarity = builder._min_symbol_similarity
        if builder._similarity is not None:
            tab = (ctypes.c_float * (128 * 128))(*builder._similarity.ascii_table())
            extra = builder._similarity.extra_pairs()
            ab = (ctypes.c_uint32 * (2 * max(1, len(extra))))()
            vals = (ctypes.c_float * max(1, len(extra)))()
            for i, (a, b, s) in enumerate(extra):
                ab[2 * i], ab[2 * i + 1], vals[i] = a, b, s
            cfg.similarity_ascii = tab
            cfg.n_similarity_pairs = len(extra)
            cfg.similarity_pairs = ab
            cfg.similarity_pair_values = vals
            self._keep += [tab, ab, vals]
        cfg.n_mappings = len(builder._mappings)
        if builder._mappings:  # builder.rs:116-132
            maps = (_native.fac_mapping * len(builder._mappings))()
            for i, (a, b, score) in enumerate(builder._mappings):
                ea, eb = a.encode("utf-8"), b.encode("utf-8")
                self._keep += [ea, eb]
                maps[i].a, maps[i].a_len, maps[i].b, maps[i].b_len, maps[i].score = ea, len(ea), eb, len(eb), score
            cfg.mappings = maps
            self._keep.append(maps)
        cfg.device = builder._device
        arr = (_native.fac_pattern * max(1, len(patterns)))()
        enc = []
        for i, p in enumerate(patterns):
            b = p.pattern.encode("utf-8")
            enc.append(b)
            arr[i].utf8 = b
            arr[i].len = len(b)
            arr[i].weight = p.weight
            arr[i].has_limits = int(p.limits is not None)
            arr[i].limits = (p.limits or FuzzyLimits()).to_c()
        handle = ctypes.c_void_p()
        rc = _native.lib.fac_build(arr, len(patterns), ctypes.byref(cfg), ctypes.byref(handle))
        if rc:
            _raise(rc)
        self._h = handle
        self.device = builder._device

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _native.lib is not None:  # the module may already be torn down at exit
            _native.lib.fac_engine_free(h)
            self._h = None

    # -- introspection
    def patterns(self) -> List[Pattern]:
        return self.patterns_

    def num_nodes(self) -> int:
        return int(_native.lib.fac_engine_num_nodes(self._h))

    def max_edits_fast(self) -> int:
        return int(_native.lib.fac_engine_max_edits_fast(self._h))

    def max_match_graphemes(self) -> int:
        """stream.rs:213-253"""
        return int(_native.lib.fac_max_match_graphemes(self._h))

    # -- raw search (search.rs:187-395)
    def _to_matches(self, haystack: str, data: bytes, rows) -> FuzzyMatches:
        inner = []
        for (s, e, p, sim, ins, dele, sub, swp, ed) in rows:
            inner.append(FuzzyMatch(ins, dele, sub, swp, ed, p, self.patterns_[p], s, e, sim,
                                    data[s:e].decode("utf-8")))
        return FuzzyMatches(haystack, inner, data)

    def search_raw(self, haystack: str, threshold: float, prefilter: bool = False) -> FuzzyMatches:
        data = haystack.encode("utf-8")
        out = ctypes.POINTER(_native.fac_match)()
        n = ctypes.c_uint64()
        eg = ctypes.c_uint64()
        fn = _native.lib.fac_search_prefiltered if prefilter else _native.lib.fac_search_raw
        rc = fn(self._h, data, len(data), f32(threshold), ctypes.byref(out), ctypes.byref(n), ctypes.byref(eg))
        if rc:
            _raise(rc, eg.value)
        return self._to_matches(haystack, data, _native.take_matches(out, n.value))

    def _unique_ids(self):
        """Uniqueness key per pattern for NonOverlappingUnique (matches.rs:118-122): custom ids and
        automatic (index) ids never compare equal."""
        if getattr(self, "_uid", None) is None:
            keys = [(1 << 63) | p.custom_unique_id_ if p.custom_unique_id_ is not None else i
                    for i, p in enumerate(self.patterns_)]
            self._uid = (ctypes.c_uint64 * max(1, len(keys)))(*keys)
        return self._uid

    def _search_ranked(self, haystack: str, threshold: float, order: Order, overlap: Overlap,
                       prefilter: bool = False) -> FuzzyMatches:
        """search_raw + FuzzyMatches::apply, the ranking / overlap resolution on the device
        (fac_matches_apply, matches.rs:7-149) before any Python object is built."""
        data = haystack.encode("utf-8")
        out = ctypes.POINTER(_native.fac_match)()
        n = ctypes.c_uint64()
        eg = ctypes.c_uint64()
        fn = _native.lib.fac_search_prefiltered if prefilter else _native.lib.fac_search_raw
        rc = fn(self._h, data, len(data), f32(threshold), ctypes.byref(out), ctypes.byref(n), ctypes.byref(eg))
        if rc:
            _raise(rc, eg.value)
        count = n.value
        if count and (order != Order.Unsorted or overlap != Overlap.Keep):
            kept = ctypes.c_uint64()
            rc = _native.lib.fac_matches_apply(self._h, out, count, order.value, overlap.value, self._unique_ids(),
                                               ctypes.byref(kept))
            if rc:
                _native.lib.fac_matches_free(out)
                _raise(rc)
            count = kept.value
        return self._to_matches(haystack, data, _native.take_matches(out, count))

    # -- stream.rs
    def search_stream(self, reader, threshold: float, on_match, window: int = 0) -> int:
        """stream.rs:299-328: search a byte stream (anything with .read(n)) in overlapping windows,
        calling `on_match(StreamMatch)` with absolute offsets; returns the bytes read."""
        st = _Stream(self, threshold, window)
        while True:
            chunk = reader.read(READ_CHUNK)
            for m in st.feed(chunk or b"", eof=not chunk):
                on_match(m)
            if not chunk:
                return st.total()

    def stream_matches(self, reader, threshold: float, window: int = 0):
        """stream.rs:330-352: the same, lazily, as an iterator of StreamMatch."""
        st = _Stream(self, threshold, window)
        while True:
            chunk = reader.read(READ_CHUNK)
            yield from st.feed(chunk or b"", eof=not chunk)
            if not chunk:
                return

    def search_stream_parallel(self, reader, threshold: float, threads: int, on_match) -> int:
        """stream.rs:378-429. The device path already searches two windows at a time (one HIP
        stream each, fac_stream); `threads` is accepted for API parity."""
        return self.search_stream(reader, threshold, on_match)

    def replace_stream(self, reader, writer, threshold: float, callback, window: int = 0) -> int:
        """stream.rs:462-503 + ReplaceCursor::emit_window (:645-705): streaming find-and-replace.
        Every owned match (per window: sorted().non_overlapping(), start < commit, ordered by
        (start, end)) is replaced by `callback(m)` (a str; None keeps the matched text) unless it
        starts inside text already written; everything else is copied through. Text before the
        stream's commit point is written as soon as it is committed. Returns the bytes written."""
        st = _Stream(self, threshold, window)
        pending = bytearray()  # stream bytes [emitted, read) not yet written
        emitted = written = 0

        def out(b: bytes):
            nonlocal written
            if b:
                writer.write(b)
                written += len(b)

        def emit(ms, upto):
            nonlocal emitted, pending
            for m in sorted(ms, key=lambda m: (m.start, m.end)):
                if m.start < emitted:  # overlaps text an earlier window's match already wrote
                    continue
                out(bytes(pending[: m.start - emitted]))
                repl = callback(m)
                out(m.text.encode("utf-8") if repl is None else str(repl).encode("utf-8"))
                del pending[: m.end - emitted]
                emitted = m.end
            if emitted < upto:  # verbatim up to the commit point
                out(bytes(pending[: upto - emitted]))
                del pending[: upto - emitted]
                emitted = upto

        while True:
            chunk = reader.read(READ_CHUNK)
            pending += chunk or b""
            ms = st.feed(chunk or b"", eof=not chunk)
            if not chunk:
                emit(ms, st.total())
                return written
            emit(ms, max(emitted, st.committed()))

    def replace_stream_parallel(self, reader, writer, threads: int, threshold: float, callback) -> int:
        """stream.rs:533-638: same output as replace_stream (windows are pipelined on the device)."""
        return self.replace_stream(reader, writer, threshold, callback)

    def apply_on_device(self, matches: FuzzyMatches, order: Order, overlap: Overlap) -> FuzzyMatches:
        """FuzzyMatches::apply of an existing match list through fac_matches_apply (same input
        order in, so Unsorted + NonOverlapping walks the same sequence as the host)."""
        n = len(matches.inner)
        arr = (_native.fac_match * max(1, n))()
        for i, m in enumerate(matches.inner):
            arr[i] = _native.fac_match(m.start, m.end, m.pattern_index, m.similarity, m.insertions, m.deletions,
                                       m.substitutions, m.swaps, m.edits)
        kept = ctypes.c_uint64()
        rc = _native.lib.fac_matches_apply(self._h, arr, n, order.value, overlap.value, self._unique_ids(),
                                           ctypes.byref(kept))
        if rc:
            _raise(rc)
        rows = [(a.start, a.end, a.pattern_index, a.similarity, a.insertions, a.deletions, a.substitutions, a.swaps,
                 a.edits) for a in arr[:kept.value]]
        return self._to_matches(matches.haystack, matches.haystack.encode("utf-8"), rows)

    # -- query.rs
    def search(self, haystack: str, opts: SearchOptions = None) -> FuzzyMatches:
        opts = opts or SearchOptions()
        return self._search_ranked(haystack, opts.threshold_, opts.order_, opts.overlap_)

    def _segmented(self, haystack: str, opts: SearchOptions) -> FuzzyMatches:
        order = Order.Default if opts.order_ == Order.Unsorted else opts.order_
        overlap = Overlap.NonOverlapping if opts.overlap_ == Overlap.Keep else opts.overlap_
        return self._search_ranked(haystack, opts.threshold_, order, overlap)

    def replace(self, text: str, opts: SearchOptions, callback) -> str:
        return self._segmented(text, opts).replace(callback)

    def strip_prefix(self, haystack: str, opts: SearchOptions) -> str:
        return self._segmented(haystack, opts).strip_prefix()

    def strip_suffix(self, haystack: str, opts: SearchOptions) -> str:
        return self._segmented(haystack, opts).strip_suffix()

    def split(self, haystack: str, opts: SearchOptions):
        return self._segmented(haystack, opts).split()

    def segment_iter(self, haystack: str, opts: SearchOptions):
        return self._segmented(haystack, opts).segment_iter()

    def segment_text(self, haystack: str, opts: SearchOptions) -> str:
        return self._segmented(haystack, opts).segment_text()

    # -- prefilter.rs:113-155
    def with_prefilter(self) -> "Prefiltered":
        return Prefiltered(self)

    # -- device-resident haystacks (bench / sharding)
    def stage(self, haystack: bytes) -> "StagedHaystack":
        return StagedHaystack(self, haystack)


class Prefiltered:
    """prefilter.rs:57-156"""

    def __init__(self, engine: FuzzyAhoCorasick):
        self.engine = engine

    def is_active(self) -> bool:
        return bool(_native.lib.fac_prefilter_active(self.engine._h))

    def search(self, haystack: str, opts: SearchOptions = None) -> FuzzyMatches:
        opts = opts or SearchOptions()
        return self.engine._search_ranked(haystack, opts.threshold_, opts.order_, opts.overlap_, prefilter=True)


def prefilter_windows(engine: "FuzzyAhoCorasick", haystack: str, threshold: float):
    """Diagnostics: merged bitap candidate windows (grapheme ranges), or None on fallback."""
    data = haystack.encode("utf-8")
    cap = 2 * len(data) + 16
    buf = (ctypes.c_uint64 * (2 * cap))()
    n = _native.lib.fac_prefilter_windows(engine._h, data, len(data), f32(threshold), buf, cap)
    if n < 0:
        return None
    return [(buf[2 * i], buf[2 * i + 1]) for i in range(n)]


# read() size of the streaming methods. The library cuts windows as the crate's WindowReader does with
# its 64 KiB reads (stream.rs:94, 102-158) whatever the feed size, so a larger read only means fewer
# calls across the C ABI (and lets a feed fill whole batches of windows).
READ_CHUNK = 4 << 20


class StreamMatch:
    """stream.rs:33-59: a match with absolute (stream-wide) byte offsets and its owned text."""
    __slots__ = ("start", "end", "pattern_index", "similarity", "insertions", "deletions", "substitutions",
                 "swaps", "edits", "text")

    def __init__(self, row, text: str):
        (self.start, self.end, self.pattern_index, self.similarity, self.insertions, self.deletions,
         self.substitutions, self.swaps, self.edits) = row
        self.text = text

    def __repr__(self):
        return f"StreamMatch({self.start}..{self.end} p{self.pattern_index} {self.similarity:.4f} {self.text!r})"


class _Stream:
    """fac_stream: WindowReader + per-window search on the GPU (stream.rs:77-297)."""

    def __init__(self, engine: "FuzzyAhoCorasick", threshold: float, window: int = 0):
        h = ctypes.c_void_p()
        rc = _native.lib.fac_stream_open(engine._h, f32(threshold), window, ctypes.byref(h))
        if rc:
            _raise(rc)
        self._h = h
        self.engine = engine

    def feed(self, data: bytes, eof: bool = False) -> List[StreamMatch]:
        out = ctypes.POINTER(_native.fac_match)()
        n = ctypes.c_uint64()
        text = ctypes.POINTER(ctypes.c_uint8)()
        tlen = ctypes.c_uint64()
        rc = _native.lib.fac_stream_feed(self._h, data, len(data), int(eof), ctypes.byref(out), ctypes.byref(n),
                                         ctypes.byref(text), ctypes.byref(tlen))
        if rc:
            _raise(rc)
        raw = ctypes.string_at(text, tlen.value) if tlen.value else b""
        _native.lib.fac_buffer_free(text)
        res, pos = [], 0
        for row in _native.take_matches(out, n.value):
            k = row[1] - row[0]
            res.append(StreamMatch(row, raw[pos:pos + k].decode("utf-8")))
            pos += k
        return res

    def total(self) -> int:
        return int(_native.lib.fac_stream_total(self._h))

    def committed(self) -> int:
        return int(_native.lib.fac_stream_committed(self._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _native.lib is not None:
            _native.lib.fac_stream_close(h)
            self._h = None


class StagedHaystack:
    """A haystack staged into HBM once (fac_haystack_stage) and searched many times.

    `StagedHaystack.shard(engine, data, n, r)` stages only shard r of n of `data` (its owned bytes
    plus the halo, fac_shard_plan): searching it yields search_raw's records for the shard's start
    windows at global byte offsets."""

    def __init__(self, engine: FuzzyAhoCorasick, data: bytes, _shard=None):
        self.engine = engine
        self.data = data
        h = ctypes.c_void_p()
        eg = ctypes.c_uint64()
        if _shard is None:
            rc = _native.lib.fac_haystack_stage(engine._h, data, len(data), ctypes.byref(h), ctypes.byref(eg))
            self.base, self.owned_bytes, self.open_end, self.plan = 0, len(data), False, None
        else:
            a, b, e, asc, open_end = _shard
            piece = data[a:e]
            rc = _native.lib.fac_haystack_stage_shard(engine._h, piece, len(piece), b - a, int(asc), int(open_end), a,
                                                      ctypes.byref(h), ctypes.byref(eg))
            self.base, self.owned_bytes, self.open_end, self.plan = a, b - a, open_end, _shard
        if rc:
            _raise(rc, eg.value)
        self._h = h
        self.graphemes = int(_native.lib.fac_haystack_graphemes(h))
        self.owned_windows = int(_native.lib.fac_haystack_owned_windows(h))
        self._dev_out = None  # growable device record buffer (search_device)

    @classmethod
    def from_device(cls, engine: FuzzyAhoCorasick, d_utf8: int, length: int, stream=None,
                    reuse: "StagedHaystack" = None) -> "StagedHaystack":
        """fac_haystack_stage_device: search_raw's staging (UTF-8 check, is_ascii, UAX #29 segmentation
        and folding, search.rs:196-203/296-302) of `length` bytes already in HBM at device address
        `d_utf8` (borrowed: keep the buffer alive). `reuse`: a haystack staged this way before, whose
        device buffers are reused (it is restaged in place and returned)."""
        h = ctypes.c_void_p(reuse._h.value if reuse is not None else None)
        eg = ctypes.c_uint64()
        rc = _native.lib.fac_haystack_stage_device(engine._h, ctypes.c_void_p(d_utf8), length, ctypes.c_void_p(stream or 0),
                                                   ctypes.byref(h), ctypes.byref(eg))
        if rc:
            if reuse is not None:  # a failed restage leaves the haystack empty (and searchable)
                reuse.owned_bytes, reuse.graphemes, reuse.owned_windows = 0, 0, 0
            _raise(rc, eg.value)
        obj = reuse
        if obj is None:
            obj = cls.__new__(cls)
            obj.engine, obj.data, obj._h, obj._dev_out = engine, None, h, None
            obj.base, obj.open_end, obj.plan = 0, False, None
        obj.owned_bytes = length
        obj.graphemes = int(_native.lib.fac_haystack_graphemes(obj._h))
        obj.owned_windows = int(_native.lib.fac_haystack_owned_windows(obj._h))
        return obj

    @classmethod
    def shard(cls, engine: FuzzyAhoCorasick, data: bytes, n_shards: int, shard: int, is_ascii: int = -1):
        plan = _native.shard_plan(engine.max_match_graphemes(), data, n_shards, shard, is_ascii)
        return cls(engine, data, _shard=plan)

    @classmethod
    def shard_from_device(cls, engine: FuzzyAhoCorasick, d_utf8: int, plan, stream=None,
                          reuse: "StagedHaystack" = None) -> "StagedHaystack":
        """fac_haystack_stage_shard_device: shard `plan` (a, b, e, global_ascii, open_end from
        _native.shard_plan) whose bytes [a, e) are already in HBM at `d_utf8` (borrowed), staged on the
        device like from_device (the per-step staging of a sharded search_raw). `reuse`: a shard
        staged this way before, restaged in place."""
        a, b, e, asc, open_end = plan
        h = ctypes.c_void_p(reuse._h.value if reuse is not None else None)
        eg = ctypes.c_uint64()
        rc = _native.lib.fac_haystack_stage_shard_device(engine._h, ctypes.c_void_p(d_utf8), e - a, b - a, int(asc),
                                                         int(open_end), a, ctypes.c_void_p(stream or 0),
                                                         ctypes.byref(h), ctypes.byref(eg))
        if rc:
            if reuse is not None:
                reuse.owned_bytes, reuse.graphemes, reuse.owned_windows = 0, 0, 0
            _raise(rc, eg.value)
        obj = reuse
        if obj is None:
            obj = cls.__new__(cls)
            obj.engine, obj.data, obj._h, obj._dev_out = engine, None, h, None
        obj.base, obj.open_end, obj.plan, obj.owned_bytes = a, open_end, plan, b - a
        obj.graphemes = int(_native.lib.fac_haystack_graphemes(obj._h))
        obj.owned_windows = int(_native.lib.fac_haystack_owned_windows(obj._h))
        return obj

    def set_key_partition(self, parts: int, part: int) -> "StagedHaystack":
        """fac_haystack_set_key_partition: later searches cover only the start windows whose first two
        characters hash to `part` of `parts` (a strong-scaling split that keeps whole prefix-cache keys
        on one GPU). parts = 1 restores the whole haystack."""
        rc = _native.lib.fac_haystack_set_key_partition(self.engine._h, self._h, parts, part)
        if rc:
            _raise(rc)
        self.key_partition = (parts, part)
        return self

    def search_device(self, threshold: float, window_begin: int = 0, window_end: int = None, stream=None,
                      auto_beam_prefix: int = 0, torch_device=None):
        """fac_search_staged_ex with the records left in HBM: (uint8 tensor of n * 32 bytes on the
        engine's device, n, fac_stats). The buffer is reused across calls and grown on demand."""
        import torch
        dev = torch_device or torch.device("cuda", self.engine.device)
        if window_end is None:
            window_end = self.graphemes
        while True:
            if self._dev_out is None:
                self._dev_out = torch.empty(max(4096, self.owned_windows // 64) * 32, dtype=torch.uint8, device=dev)
            a = _native.fac_search_args(window_begin, window_end, f32(threshold), ctypes.c_void_p(stream or 0),
                                        auto_beam_prefix, ctypes.c_void_p(self._dev_out.data_ptr()),
                                        self._dev_out.numel() // 32)
            n = ctypes.c_uint64()
            st = _native.fac_stats()
            rc = _native.lib.fac_search_staged_ex(self.engine._h, self._h, ctypes.byref(a), None, ctypes.byref(n),
                                                  ctypes.byref(st))
            if rc == _native.FAC_E_OUTPUT_CAPACITY:
                self._dev_out = torch.empty(int(n.value * 1.25 + 1024) * 32, dtype=torch.uint8, device=dev)
                continue
            if rc:
                _raise(rc)
            return self._dev_out[: n.value * 32], int(n.value), st

    def auto_beam_total(self, threshold: float, window_begin: int = 0, window_end: int = None, stream=None) -> int:
        """fac_auto_beam_total: sum of queue.len() over the windows searched unbeamed."""
        if window_end is None:
            window_end = self.graphemes
        t = ctypes.c_uint64()
        rc = _native.lib.fac_auto_beam_total(self.engine._h, self._h, window_begin, window_end, f32(threshold),
                                             ctypes.c_void_p(stream or 0), ctypes.byref(t))
        if rc:
            _raise(rc)
        return int(t.value)

    def stream_window(self, g_begin: int, g_end: int, commit_bytes: int, base: int, threshold: float,
                      prefilter: bool, stream=None):
        """fac_stream_window_staged (stream.rs:262-297 window_matches on a device-resident window):
        NumPy records (MATCH_DTYPE) of the window's owned matches at absolute offsets + fac_stats."""
        out = ctypes.POINTER(_native.fac_match)()
        n = ctypes.c_uint64()
        st = _native.fac_stats()
        rc = _native.lib.fac_stream_window_staged(self.engine._h, self._h, g_begin, g_end, commit_bytes, base,
                                                  f32(threshold), int(prefilter), ctypes.c_void_p(stream or 0),
                                                  ctypes.byref(out), ctypes.byref(n), ctypes.byref(st))
        if rc:
            _raise(rc)
        return _native.take_records(out, n.value), st

    def stream_window_device(self, g_begin: int, g_end: int, commit_bytes: int, base: int, threshold: float,
                             prefilter: bool, out, offset: int = 0, stream=None):
        """fac_stream_window_staged_device: the window's owned records (stream.rs:262-297) written in HBM
        to `out` (a uint8 CUDA tensor of 32-byte records) from record `offset` on, never visiting the
        host; `out` is grown (a new tensor, the records before `offset` copied) when it is too small.
        Returns (out, owned count, fac_stats)."""
        import torch
        n = ctypes.c_uint64()
        st = _native.fac_stats()
        while True:
            cap = out.numel() // _native.REC_BYTES - offset
            ptr = out.data_ptr() + offset * _native.REC_BYTES
            rc = _native.lib.fac_stream_window_staged_device(
                self.engine._h, self._h, g_begin, g_end, commit_bytes, base, f32(threshold), int(prefilter),
                ctypes.c_void_p(stream or 0), ctypes.c_void_p(ptr), max(0, cap), ctypes.byref(n), ctypes.byref(st))
            if rc == _native.FAC_E_OUTPUT_CAPACITY:
                grown = torch.empty(max(2 * out.numel(), (offset + n.value) * _native.REC_BYTES * 2),
                                    dtype=torch.uint8, device=out.device)
                grown[: offset * _native.REC_BYTES].copy_(out[: offset * _native.REC_BYTES])
                out = grown
                continue
            if rc:
                _raise(rc)
            return out, n.value, st

    def stream_windows_device(self, windows, threshold: float, prefilter: bool, out, offset: int = 0, stream=None):
        """fac_stream_windows_staged_device: a batch of stream windows, `windows` = [(g_begin, g_end,
        commit_bytes, base), ...] in stream order, searched together (one pre-filter pass and one search
        launch on an ASCII haystack); their owned records, in window order, written in HBM to `out`
        from record `offset` on (grown like stream_window_device). Returns (out, owned count, fac_stats)."""
        import numpy as np
        import torch
        arr = np.ascontiguousarray(np.asarray(windows, dtype=np.uint64).reshape(-1, 4))
        wp = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        n = ctypes.c_uint64()
        st = _native.fac_stats()
        while True:
            cap = out.numel() // _native.REC_BYTES - offset
            ptr = out.data_ptr() + offset * _native.REC_BYTES
            rc = _native.lib.fac_stream_windows_staged_device(
                self.engine._h, self._h, wp, len(arr), f32(threshold), int(prefilter), ctypes.c_void_p(stream or 0),
                ctypes.c_void_p(ptr), max(0, cap), ctypes.byref(n), ctypes.byref(st))
            if rc == _native.FAC_E_OUTPUT_CAPACITY:
                grown = torch.empty(max(2 * out.numel(), (offset + n.value) * _native.REC_BYTES * 2),
                                    dtype=torch.uint8, device=out.device)
                grown[: offset * _native.REC_BYTES].copy_(out[: offset * _native.REC_BYTES])
                out = grown
                continue
            if rc:
                _raise(rc)
            return out, n.value, st

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _native.lib is not None:
            _native.lib.fac_haystack_free(h)
            self._h = None

    def search_windows(self, threshold: float, window_begin: int = 0, window_end: int = None, stream=None):
        """Raw rows (start, end, pattern, sim, ins, del, sub, swp, edits) + fac_stats."""
        if window_end is None:
            window_end = self.graphemes
        out = ctypes.POINTER(_native.fac_match)()
        n = ctypes.c_uint64()
        st = _native.fac_stats()
        rc = _native.lib.fac_search_staged(self.engine._h, self._h, window_begin, window_end, f32(threshold),
                                           ctypes.c_void_p(stream or 0), ctypes.byref(out), ctypes.byref(n),
                                           ctypes.byref(st))
        if rc:
            _raise(rc)
        return _native.take_matches(out, n.value), st

    def search_windows_records(self, threshold: float, window_begin: int = 0, window_end: int = None,
                               stream=None):
        """search_windows returning a NumPy array of 32-byte match records (MATCH_DTYPE)."""
        if window_end is None:
            window_end = self.graphemes
        out = ctypes.POINTER(_native.fac_match)()
        n = ctypes.c_uint64()
        st = _native.fac_stats()
        t0 = time.perf_counter()
        rc = _native.lib.fac_search_staged(self.engine._h, self._h, window_begin, window_end, f32(threshold),
                                           ctypes.c_void_p(stream or 0), ctypes.byref(out), ctypes.byref(n),
                                           ctypes.byref(st))
        if rc:
            _raise(rc)
        t1 = time.perf_counter()
        rows = _native.take_records(out, n.value)
        if _TIMING:
            print(f"FAC_TIMING native call {1e3 * (t1 - t0):.2f} ms, records to NumPy {1e3 * (time.perf_counter() - t1):.2f} ms",
                  file=sys.stderr)
        return rows, st

    def search_prefiltered_records(self, threshold: float, stream=None):
        out = ctypes.POINTER(_native.fac_match)()
        n = ctypes.c_uint64()
        st = _native.fac_stats()
        rc = _native.lib.fac_search_staged_prefiltered(self.engine._h, self._h, f32(threshold),
                                                       ctypes.c_void_p(stream or 0), ctypes.byref(out),
                                                       ctypes.byref(n), ctypes.byref(st))
        if rc:
            _raise(rc)
        return _native.take_records(out, n.value), st

    def search_prefiltered(self, threshold: float, stream=None):
        """Prefiltered::raw on the device-resident text (prefilter.rs:146-155, 304-374): raw rows
        (best per (start, end, pattern), sorted) + fac_stats (prefilter_ms = bitap + merge)."""
        out = ctypes.POINTER(_native.fac_match)()
        n = ctypes.c_uint64()
        st = _native.fac_stats()
        rc = _native.lib.fac_search_staged_prefiltered(self.engine._h, self._h, f32(threshold),
                                                       ctypes.c_void_p(stream or 0), ctypes.byref(out),
                                                       ctypes.byref(n), ctypes.byref(st))
        if rc:
            _raise(rc)
        return _native.take_matches(out, n.value), st


class FuzzyReplacer:
    """replacer.rs:9-52"""

    def __init__(self, engine: FuzzyAhoCorasick, replacements: List[str]):
        self.engine = engine
        self.replacements = replacements

    def replace(self, text: str, opts: SearchOptions) -> str:
        return self.engine.replace(text, opts, lambda m: self.replacements[m.pattern_index])

    def replace_stream(self, reader, writer, threshold: float) -> int:
        """replacer.rs:35-44"""
        return self.engine.replace_stream(reader, writer, threshold, lambda m: self.replacements[m.pattern_index])
