"""Test-side wrapper of oracle/liboracle.so (the CPU restatement; TEST INFRASTRUCTURE ONLY).

Staging is done here with the `regex` module (`\\X` = UAX #29 extended grapheme clusters) and
`str.lower`, independently of the product's generated C++ tables, so a parity test compares two
independently staged pipelines. `OracleEngine` exposes the same search surface as
`fuzzy_aho_corasick.FuzzyAhoCorasick` so the translated reference tests can run on either.
"""
import ctypes
import os
import subprocess
import sys

import regex

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "fuzzy-aho-corasick-rs_amd")
if PKG_DIR not in sys.path:
    sys.path.insert(0, PKG_DIR)

# FuzzyMatch / FuzzyMatches are used only as result containers (and for the out-of-scope replace /
# split helpers); ranking and overlap resolution come from the oracle's own orc_apply
from fuzzy_aho_corasick.matches import FuzzyMatch, FuzzyMatches  # noqa: E402
from fuzzy_aho_corasick.structs import (FuzzyLimits, FuzzyPenalties, Pattern, SearchOptions, f32)  # noqa: E402

ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")


def ensure_oracle():
    if not os.path.exists(ORACLE_LIB) or (os.path.getmtime(ORACLE_LIB) <
                                          os.path.getmtime(os.path.join(ORACLE_DIR, "oracle.cpp"))):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    return ctypes.CDLL(ORACLE_LIB)


class orc_config(ctypes.Structure):
    _fields_ = [("case_insensitive", ctypes.c_int32), ("has_limits", ctypes.c_int32),
                ("lim", ctypes.c_int32 * 5), ("p_ins", ctypes.c_float), ("p_del", ctypes.c_float),
                ("p_sub", ctypes.c_float), ("p_swp", ctypes.c_float), ("beam_width", ctypes.c_uint64),
                ("has_auto_beam", ctypes.c_int32), ("ab_budget", ctypes.c_uint64),
                ("ab_width", ctypes.c_uint64), ("min_symbol_similarity", ctypes.c_float),
                ("custom_similarity", ctypes.c_int32), ("sim_ascii", ctypes.POINTER(ctypes.c_float)),
                ("n_sim_pairs", ctypes.c_uint64), ("sim_pair_ab", ctypes.POINTER(ctypes.c_uint32)),
                ("sim_pair_val", ctypes.POINTER(ctypes.c_float)), ("n_map", ctypes.c_uint64),
                ("map_side_off", ctypes.POINTER(ctypes.c_uint32)), ("map_g_off", ctypes.POINTER(ctypes.c_uint32)),
                ("map_cps", ctypes.POINTER(ctypes.c_uint32)), ("map_score", ctypes.POINTER(ctypes.c_float))]


class orc_match(ctypes.Structure):
    _fields_ = [("start", ctypes.c_uint64), ("end", ctypes.c_uint64), ("pattern", ctypes.c_uint32),
                ("similarity", ctypes.c_float), ("ins", ctypes.c_uint8), ("dele", ctypes.c_uint8),
                ("sub", ctypes.c_uint8), ("swp", ctypes.c_uint8), ("edits", ctypes.c_uint8),
                ("pad", ctypes.c_uint8 * 3)]


_lib = ensure_oracle()
_U32P = ctypes.POINTER(ctypes.c_uint32)
_lib.orc_build.restype = ctypes.c_void_p
_lib.orc_build.argtypes = [ctypes.POINTER(orc_config), ctypes.c_uint64, _U32P, ctypes.POINTER(ctypes.c_float),
                           ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), _U32P, _U32P, _U32P]
_lib.orc_free.argtypes = [ctypes.c_void_p]
_lib.orc_num_nodes.restype = ctypes.c_uint64
_lib.orc_num_nodes.argtypes = [ctypes.c_void_p]
_lib.orc_max_edits_fast.restype = ctypes.c_uint32
_lib.orc_max_edits_fast.argtypes = [ctypes.c_void_p]
_lib.orc_prefilter_active.restype = ctypes.c_int32
_lib.orc_prefilter_active.argtypes = [ctypes.c_void_p]
_lib.orc_search.restype = ctypes.c_int32
_lib.orc_search.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, _U32P, _U32P,
                            ctypes.POINTER(ctypes.c_uint64), ctypes.c_float, ctypes.c_int32,
                            ctypes.POINTER(ctypes.POINTER(orc_match)), ctypes.POINTER(ctypes.c_uint64),
                            ctypes.POINTER(ctypes.c_uint64)]
_lib.orc_matches_free.argtypes = [ctypes.POINTER(orc_match)]
_lib.orc_search_windows.restype = ctypes.c_int32
_lib.orc_search_windows.argtypes = _lib.orc_search.argtypes + [ctypes.c_uint32, ctypes.c_uint32]
_lib.orc_prefilter_windows.restype = ctypes.c_int64
_lib.orc_prefilter_windows.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, _U32P, _U32P,
                                       ctypes.c_float, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
_lib.orc_apply.restype = ctypes.c_uint64
_lib.orc_apply.argtypes = [ctypes.POINTER(orc_match), ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                           ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
_lib.orc_set_modes.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
_lib.orc_bitap_ends.restype = ctypes.c_uint64
_lib.orc_bitap_ends.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]

_GRAPHEME = regex.compile(r"\X")


def set_modes(edge_order: int = -1, beam_rule: int = -1, sel_limit: int = -1):
    """Oracle restatement modes for engines built afterwards (oracle.cpp g_edge_order / g_beam_rule):
    edge order 0 = insertion, 1 = the reference's FxHashMap iteration order (default); beam rule
    0 = canonical ties, 1 = ties towards the latest queue position, 2 = select_nth_unstable_by
    (default); sel_limit = select.rs's 16 partition rounds before median_of_medians (tests lower it).
    Diagnostics only: the defaults are what the GPU path implements."""
    _lib.orc_set_modes(edge_order, beam_rule, sel_limit)


def graphemes(s: str):
    return _GRAPHEME.findall(s)


def fold(g: str, ci: bool) -> str:
    # search.rs:406-412 / builder.rs:197-205: per-grapheme to_lowercase when case-insensitive
    return g.lower() if ci else g


def _lim_arr(lim):
    n = lambda v: -1 if v is None else v  # noqa: E731
    return [n(v) for v in lim.as_tuple()]


class OracleEngine:
    """Same construction inputs and search surface as fuzzy_aho_corasick.FuzzyAhoCorasick."""

    def __init__(self, builder, inputs):
        self.patterns_ = [Pattern.from_(x) for x in inputs]
        b = builder
        self.ci = b._case_insensitive
        cfg = orc_config()
        cfg.case_insensitive = int(self.ci)
        cfg.has_limits = int(b._limits is not None)
        if b._limits is not None:
            cfg.lim[:] = _lim_arr(b._limits)
        pen = b._penalties
        cfg.p_ins, cfg.p_del, cfg.p_sub, cfg.p_swp = pen.insertion, pen.deletion, pen.substitution, pen.swap
        cfg.beam_width = b._beam_width or 0
        cfg.has_auto_beam = int(b._auto_beam is not None)
        if b._auto_beam:
            cfg.ab_budget, cfg.ab_width = b._auto_beam
        cfg.min_symbol_similarity = b._min_symbol_similarity
        self._keep = []
        if b._similarity is not None:
            tab = (ctypes.c_float * (128 * 128))(*b._similarity.ascii_table())
            extra = b._similarity.extra_pairs()
            ab = (ctypes.c_uint32 * (2 * max(1, len(extra))))()
            vals = (ctypes.c_float * max(1, len(extra)))()
            for i, (x, y, s) in enumerate(extra):
                ab[2 * i], ab[2 * i + 1], vals[i] = x, y, s
            cfg.custom_similarity = 1
            cfg.sim_ascii, cfg.n_sim_pairs, cfg.sim_pair_ab, cfg.sim_pair_val = tab, len(extra), ab, vals
            self._keep += [tab, ab, vals]
        if b._mappings:  # builder.rs:392-402: both sides grapheme-split and folded like patterns
            side_off, m_goff, m_cps, scores = [0], [0], [], []
            for a, c, score in b._mappings:
                for side in (a, c):
                    for g in graphemes(side):
                        m_cps += [ord(ch) for ch in fold(g, self.ci)]
                        m_goff.append(len(m_cps))
                    side_off.append(len(m_goff) - 1)
                scores.append(score)
            arrs = [(ctypes.c_uint32 * len(side_off))(*side_off), (ctypes.c_uint32 * len(m_goff))(*m_goff),
                    (ctypes.c_uint32 * max(1, len(m_cps)))(*m_cps), (ctypes.c_float * len(scores))(*scores)]
            cfg.n_map = len(b._mappings)
            cfg.map_side_off, cfg.map_g_off, cfg.map_cps, cfg.map_score = arrs
            self._keep += arrs
        n = len(self.patterns_)
        glen, weight, flag, lim, pg_off, g_off, cps = [], [], [], [], [0], [0], []
        for p in self.patterns_:
            gs = graphemes(p.pattern)
            glen.append(len(gs))  # structs.rs:664 graphemes(true).count() on the original text
            weight.append(p.weight)
            flag.append(int(p.limits is not None))
            lim += _lim_arr(p.limits) if p.limits is not None else [-1] * 5
            for g in gs:
                cps += [ord(c) for c in fold(g, self.ci)]
                g_off.append(len(cps))
            pg_off.append(len(g_off) - 1)
        A = lambda t, v: (t * max(1, len(v)))(*v)  # noqa: E731
        self._h = _lib.orc_build(ctypes.byref(cfg), n, A(ctypes.c_uint32, glen), A(ctypes.c_float, weight),
                                 A(ctypes.c_int32, flag), A(ctypes.c_int32, lim), A(ctypes.c_uint32, pg_off),
                                 A(ctypes.c_uint32, g_off), A(ctypes.c_uint32, cps))
        self.states_popped = 0

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.orc_free(self._h)
            self._h = None

    def num_nodes(self):
        return int(_lib.orc_num_nodes(self._h))

    def max_edits_fast(self):
        return int(_lib.orc_max_edits_fast(self._h))

    def raw_rows(self, haystack, threshold, prefilter=False, windows=None):
        data = haystack.encode("utf-8") if isinstance(haystack, str) else haystack
        text = data.decode("utf-8")
        goff, cps, boff = [0], [], []
        if not data.isascii():
            pos = 0
            for g in graphemes(text):
                boff.append(pos)
                pos += len(g.encode("utf-8"))
                cps += [ord(c) for c in fold(g, self.ci)]
                goff.append(len(cps))
        ng = len(boff)
        out = ctypes.POINTER(orc_match)()
        cnt = ctypes.c_uint64()
        popped = ctypes.c_uint64()
        w0, w1 = windows if windows is not None else (0, 0xFFFFFFFF)
        rc = _lib.orc_search_windows(self._h, data, len(data), ng, (ctypes.c_uint32 * max(1, len(goff)))(*goff),
                                     (ctypes.c_uint32 * max(1, len(cps)))(*cps),
                                     (ctypes.c_uint64 * max(1, ng))(*boff), f32(threshold), int(prefilter),
                                     ctypes.byref(out), ctypes.byref(cnt), ctypes.byref(popped), w0, w1)
        if rc:
            raise RuntimeError(f"oracle error {rc}")
        rows = []
        for i in range(cnt.value):
            m = out[i]
            rows.append((m.start, m.end, m.pattern, m.similarity, m.ins, m.dele, m.sub, m.swp, m.edits))
        _lib.orc_matches_free(out)
        self.states_popped = popped.value
        return rows

    def prepare(self, data: bytes) -> "PreparedText":
        return PreparedText(self, data)

    def prefilter_windows(self, haystack, threshold):
        data = haystack.encode("utf-8")
        goff, cps = [0], []
        if not data.isascii():
            for g in graphemes(haystack):
                cps += [ord(c) for c in fold(g, self.ci)]
                goff.append(len(cps))
        cap = 2 * len(data) + 16
        buf = (ctypes.c_uint64 * (2 * cap))()
        n = _lib.orc_prefilter_windows(self._h, data, len(data), len(goff) - 1,
                                       (ctypes.c_uint32 * max(1, len(goff)))(*goff),
                                       (ctypes.c_uint32 * max(1, len(cps)))(*cps), f32(threshold), buf, cap)
        if n < 0:
            return None
        return [(buf[2 * i], buf[2 * i + 1]) for i in range(n)]

    # same surface as FuzzyAhoCorasick
    def search_raw(self, haystack, threshold, prefilter=False):
        data = haystack.encode("utf-8")
        inner = [FuzzyMatch(ins, dele, sub, swp, ed, p, self.patterns_[p], s, e, sim, data[s:e].decode("utf-8"))
                 for (s, e, p, sim, ins, dele, sub, swp, ed) in self.raw_rows(haystack, threshold, prefilter)]
        return FuzzyMatches(haystack, inner, data)

    def apply_rows(self, rows, order, overlap):
        """FuzzyMatches::apply (matches.rs:7-149) on raw rows, by the oracle's own C++ restatement
        (orc_apply), independent of the product's ranking code. Returns rows in the result order."""
        n = len(rows)
        arr = (orc_match * max(1, n))()
        for i, (s, e, p, sim, ins, dele, sub, swp, ed) in enumerate(rows):
            arr[i].start, arr[i].end, arr[i].pattern, arr[i].similarity = s, e, p, sim
            arr[i].ins, arr[i].dele, arr[i].sub, arr[i].swp, arr[i].edits = ins, dele, sub, swp, ed
        plen = (ctypes.c_uint64 * max(1, len(self.patterns_)))(*[len(p.pattern.encode("utf-8")) for p in self.patterns_])
        # uniqueness keys: custom ids and automatic (index) ids never compare equal (matches.rs:118-122)
        uid = (ctypes.c_uint64 * max(1, len(self.patterns_)))(
            *[(1 << 63) | p.custom_unique_id_ if p.custom_unique_id_ is not None else i
              for i, p in enumerate(self.patterns_)])
        k = _lib.orc_apply(arr, n, int(order.value), int(overlap.value), plen, uid)
        return [(a.start, a.end, a.pattern, a.similarity, a.ins, a.dele, a.sub, a.swp, a.edits) for a in arr[:k]]

    def _applied(self, haystack, threshold, order, overlap, prefilter=False):
        data = haystack.encode("utf-8")
        rows = self.apply_rows(self.raw_rows(haystack, threshold, prefilter), order, overlap)
        inner = [FuzzyMatch(ins, dele, sub, swp, ed, p, self.patterns_[p], s, e, sim, data[s:e].decode("utf-8"))
                 for (s, e, p, sim, ins, dele, sub, swp, ed) in rows]
        return FuzzyMatches(haystack, inner, data)

    def search(self, haystack, opts=None):
        opts = opts or SearchOptions()
        return self._applied(haystack, opts.threshold_, opts.order_, opts.overlap_)

    def _segmented(self, haystack, opts):
        from fuzzy_aho_corasick.structs import Order, Overlap
        order = Order.Default if opts.order_ == Order.Unsorted else opts.order_
        overlap = Overlap.NonOverlapping if opts.overlap_ == Overlap.Keep else opts.overlap_
        return self._applied(haystack, opts.threshold_, order, overlap)

    def replace(self, text, opts, callback):
        return self._segmented(text, opts).replace(callback)

    def strip_prefix(self, haystack, opts):
        return self._segmented(haystack, opts).strip_prefix()

    def strip_suffix(self, haystack, opts):
        return self._segmented(haystack, opts).strip_suffix()

    def split(self, haystack, opts):
        return self._segmented(haystack, opts).split()

    def segment_text(self, haystack, opts):
        return self._segmented(haystack, opts).segment_text()

    def with_prefilter(self):
        return OraclePrefiltered(self)


class OraclePrefiltered:
    def __init__(self, engine):
        self.engine = engine

    def is_active(self):
        return bool(_lib.orc_prefilter_active(self.engine._h))

    def search(self, haystack, opts=None):
        opts = opts or SearchOptions()
        return self.engine._applied(haystack, opts.threshold_, opts.order_, opts.overlap_, prefilter=True)


class OracleReplacer:
    def __init__(self, engine, replacements):
        self.engine = engine
        self.replacements = replacements

    def replace(self, text, opts):
        return self.engine.replace(text, opts, lambda m: self.replacements[m.pattern_index])


class PreparedText:
    """A haystack staged once for the oracle (regex \\X segmentation + str.lower folding, as in
    raw_rows, but into NumPy arrays so large prefixes stage in seconds) and searched with one or
    several threads. ctypes releases the GIL around the oracle call, so `threads` > 1 runs the
    oracle on that many cores at once: the start windows are split into contiguous ranges (the
    union is search_raw's result, like search_stream_parallel, stream.rs:378-429); with the
    pre-filter every thread searches its own slice of the text (stream windows with
    max_match_graphemes() + 1 of overlap, each keeping the matches that start in its slice)."""

    def __init__(self, engine: "OracleEngine", data: bytes):
        import numpy as np
        self.engine, self.data = engine, data
        text = data.decode("utf-8")
        self.ascii = data.isascii()
        if self.ascii:
            self.n = len(data)
            goff = np.zeros(1, np.uint32)
            cps = np.zeros(1, np.uint32)
            boff = np.zeros(1, np.uint64)
        else:
            gs = graphemes(text)
            self.n = len(gs)
            cp = np.frombuffer(text.encode("utf-32-le"), dtype=np.uint32)
            simple = len(cp) == len(gs)
            if simple and engine.ci:
                uniq = np.unique(cp)
                low = [chr(int(c)).lower() for c in uniq]
                simple = all(len(x) == 1 for x in low)
                if simple:
                    cp = np.array([ord(x) for x in low], np.uint32)[np.searchsorted(uniq, cp)]
            if simple:  # one code point per grapheme, folding keeps it one code point
                cps = cp.astype(np.uint32)
                goff = np.arange(self.n + 1, dtype=np.uint32)
                raw = np.frombuffer(text.encode("utf-32-le"), dtype=np.uint32)
                ln = 1 + (raw >= 0x80) + (raw >= 0x800) + (raw >= 0x10000)
                boff = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
            else:
                c, go, bo, pos = [], [0], [], 0
                for g in gs:
                    bo.append(pos)
                    pos += len(g.encode("utf-8"))
                    c += [ord(ch) for ch in fold(g, engine.ci)]
                    go.append(len(c))
                cps, goff, boff = (np.array(c or [0], np.uint32), np.array(go, np.uint32),
                                   np.array(bo or [0], np.uint64))
        self._arrs = (goff, cps, boff)

    def _run(self, threshold, prefilter, w0, w1, data=None, arrs=None, n=None, full=False):
        data = self.data if data is None else data
        goff, cps, boff = self._arrs if arrs is None else arrs
        n = (0 if self.ascii else self.n) if n is None else n
        P = ctypes.POINTER
        out = P(orc_match)()
        cnt = ctypes.c_uint64()
        popped = ctypes.c_uint64()
        rc = _lib.orc_search_windows(self.engine._h, data, len(data), n,
                                     goff.ctypes.data_as(_U32P), cps.ctypes.data_as(_U32P),
                                     boff.ctypes.data_as(P(ctypes.c_uint64)), f32(threshold), int(prefilter),
                                     ctypes.byref(out), ctypes.byref(cnt), ctypes.byref(popped), w0, w1)
        if rc:
            raise RuntimeError(f"oracle error {rc}")
        if full:
            rows = [(out[i].start, out[i].end, out[i].pattern, out[i].similarity, out[i].ins, out[i].dele,
                     out[i].sub, out[i].swp, out[i].edits) for i in range(cnt.value)]
        else:
            rows = [(out[i].start, out[i].end, out[i].pattern) for i in range(cnt.value)]
        _lib.orc_matches_free(out)
        return rows

    def search(self, threshold, prefilter=False, threads=1, full=False):
        """Raw (start, end, pattern) triples of search_raw / Prefiltered::raw (full=True: every field,
        without the pre-filter)."""
        if threads <= 1:
            return self._run(threshold, prefilter, 0, 0xFFFFFFFF, full=full)
        import threading
        res = [None] * threads
        if not prefilter:
            def work(t):
                a, b = self.n * t // threads, self.n * (t + 1) // threads
                res[t] = self._run(threshold, False, a, b, full=full)
        else:
            # stream windows: byte slices cut at spaces (ASCII) with max_match + 1 of overlap
            over = 64 + 4 * max(len(p.pattern) for p in self.engine.patterns_)
            cuts = [0]
            for t in range(1, threads):
                c = len(self.data) * t // threads
                while c < len(self.data) and self.data[c - 1] != 0x20:
                    c += 1
                cuts.append(c)
            cuts.append(len(self.data))

            def work(t):
                a, b = cuts[t], cuts[t + 1]
                piece = self.data[a:min(len(self.data), b + over)]
                sub = PreparedText(self.engine, piece)
                res[t] = [(s + a, e + a, p) for (s, e, p) in sub._run(threshold, True, 0, 0xFFFFFFFF)
                          if s < b - a]
        ts = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
        for th in ts:
            th.start()
        for th in ts:
            th.join()
        return [r for part in res for r in part]


def bitap_ends(pattern: bytes, text: bytes, k: int):
    buf = (ctypes.c_uint64 * (len(text) + 1))()
    n = _lib.orc_bitap_ends(pattern, len(pattern), text, len(text), k, buf)
    return list(buf[:n])
