"""CPU-only checks (no GPU): the C-ABI library loads and exports every symbol of include/fac.h, host
staging (UAX #29 segmentation, case folding) agrees with the `regex` module, and the CPU oracle is
pinned by the reference's own fuzz/known-answer checks."""
import ctypes
import os
import random
import re
import struct

import numpy as np
import pytest
import regex

from oracle_harness import OracleEngine, bitap_ends, graphemes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def f32bits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


# ------------------------------------------------------------------ C ABI
def test_library_exports_every_header_symbol():
    from fuzzy_aho_corasick import _native
    header = open(os.path.join(REPO, "include", "fac.h")).read()
    names = set(re.findall(r"^\s*(?:[a-z_0-9]+\s*\*?\s+\**)(fac_[a-z_0-9]+)\s*\(", header, re.M))
    assert len(names) >= 15, names
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_native.SIGNATURES) >= names


def test_match_record_is_32_bytes():
    from fuzzy_aho_corasick import _native
    assert ctypes.sizeof(_native.fac_match) == 32


def test_build_without_gpu_fails_loudly_or_builds_on_gpu():
    """No CPU fallback: on a box without gfx950 the build reports FAC_E_NO_DEVICE."""
    from fuzzy_aho_corasick import DeviceError, FuzzyAhoCorasickBuilder
    try:
        eng = FuzzyAhoCorasickBuilder().build(["abc"])
    except DeviceError as e:
        assert e.code == 103, e
    else:  # running on the GPU box
        assert eng.num_nodes() == 4


# ------------------------------------------------------------------ staging
ALPHA = (["a", "b", "é", "é", "\r", "\n", "\r\n", " ", "Σ", "ς", "İ", "ß", "Ω", "ﬁ", "ǅ", "‍", "́",
          "̈", "👍", "🏽", "👨", "👩", "\U0001F1FA", "\U0001F1F8", "ᄀ", "ᅡ", "ᆨ", "가",
          "क", "्", "ष", "ि", "؀", "ä", "\t", "\x00", "﻿", "ক", "্", "‌"])


def test_grapheme_segmentation_matches_regex_X():
    from fuzzy_aho_corasick import _native
    rng = random.Random(0xC0FFEE)
    for _ in range(3000):
        s = "".join(rng.choice(ALPHA) for _ in range(rng.randint(0, 14)))
        data = s.encode("utf-8")
        want, pos = [], 0
        for g in graphemes(s):
            want.append(pos)
            pos += len(g.encode("utf-8"))
        assert _native.grapheme_starts(data) == want, repr(s)


def test_first_char_folding_matches_python_lower():
    from fuzzy_aho_corasick import _native
    for cp in list(range(0x20, 0x250)) + list(range(0x370, 0x530)) + [0x130, 0x1E9E, 0x2126, 0x212A, 0x10400]:
        ch = chr(cp)
        b = ch.encode("utf-8")
        assert _native.lib.fac_fold_first_char(b, len(b), 1) == ord(ch.lower()[0]), hex(cp)
        assert _native.lib.fac_fold_first_char(b, len(b), 0) == cp


def test_pattern_grapheme_len():
    from fuzzy_aho_corasick import Pattern
    assert Pattern("école").grapheme_len == 5
    assert Pattern("école").grapheme_len == 5
    assert Pattern("👨‍👩").grapheme_len == 1
    assert Pattern("").grapheme_len == 0
    assert Pattern("a\r\nb").grapheme_len == 3


# ------------------------------------------------------------------ f32 constants
def test_default_penalty_bits():
    from fuzzy_aho_corasick import FuzzyPenalties
    p = FuzzyPenalties()
    assert f32bits(p.substitution) == 0x3FB70A3D
    assert f32bits(p.insertion) == 0x3F051EB8 and f32bits(p.swap) == 0x3F051EB8
    assert f32bits(p.deletion) == 0x3F68F5C2


# ------------------------------------------------------------------ oracle pins
def brute_force_ends(pattern, text, k):  # examples/bitap_prototype.rs:59-79
    m = len(pattern)
    prev = list(range(m + 1))
    ends = []
    for i in range(1, len(text) + 1):
        cur = [0] * (m + 1)
        for j in range(1, m + 1):
            cur[j] = min(prev[j - 1] + (pattern[j - 1] != text[i - 1]), prev[j] + 1, cur[j - 1] + 1)
        if cur[m] <= k:
            ends.append(i)
        prev = cur
    return ends


class XS:
    def __init__(self, s):
        self.s = s

    def next(self):
        x = self.s
        x ^= (x << 13) & 0xFFFFFFFFFFFFFFFF
        x ^= x >> 7
        x ^= (x << 17) & 0xFFFFFFFFFFFFFFFF
        self.s = x
        return x


def test_bitap_recurrence_matches_brute_force_dp():
    """examples/bitap_prototype.rs:97-120: 20 000 random cases, seed 0x9E37_79B9_7F4A_7C15."""
    rng = XS(0x9E37_79B9_7F4A_7C15)
    for _ in range(20_000):
        alphabet = 2 + rng.next() % 4
        m = 1 + rng.next() % 12
        n = rng.next() % 40
        k = rng.next() % 4
        pat = bytes(ord("a") + rng.next() % alphabet for _ in range(m))
        text = bytes(ord("a") + rng.next() % alphabet for _ in range(n))
        assert bitap_ends(pat, text, k) == brute_force_ends(pat, text, k), (pat, text, k)


def _differential(seed, vocab, filler, trials):
    """prefilter.rs:467-529 on the oracle: Prefiltered::search == search, key incl. sim bits/edits."""
    from fuzzy_aho_corasick import FuzzyAhoCorasickBuilder, FuzzyLimits, FuzzyPenalties, SearchOptions
    rng = XS(seed)
    for trial in range(trials):
        npat = 1 + rng.next() % 3
        patterns = [vocab[rng.next() % len(vocab)] for _ in range(npat)]
        edits = rng.next() % 3
        ci = rng.next() & 1 == 0
        b = FuzzyAhoCorasickBuilder().case_insensitive(ci)
        if edits > 0:
            b = b.fuzzy(FuzzyLimits().edits(edits))
        if trial % 5 == 0:
            b = b.penalties(FuzzyPenalties.default().with_swap(0.6).with_insertion(0.5).with_deletion(0.8))
        eng = OracleEngine(b, patterns)
        pf = eng.with_prefilter()
        hay = ""
        for _ in range(rng.next() % 60):
            if rng.next() % 7 == 0:
                hay += patterns[rng.next() % len(patterns)] + " "
            else:
                hay += filler[rng.next() % len(filler)]
        thr = 0.6 + (rng.next() % 4) * 0.1
        key = lambda m: (m.start, m.end, m.pattern_index, m.sim_bits(), m.edits)  # noqa: E731
        exp = sorted(key(m) for m in eng.search(hay, SearchOptions().threshold(thr)))
        got = sorted(key(m) for m in pf.search(hay, SearchOptions().threshold(thr)))
        assert exp == got, (trial, patterns, edits, ci, thr, hay)


def test_oracle_prefilter_matches_full_search_ascii():  # prefilter.rs:531-537
    _differential(0x1234_5678_9abc_def1, ["hello", "world", "vestibulum", "abc", "lorem", "cell"],
                  ["a", "b", "c", "d", "e", " ", "1", "o", "0", "l"], 4000)


def test_oracle_prefilter_matches_full_search_unicode():  # prefilter.rs:539-546
    _differential(0xdead_beef_0bad_f00d, ["café", "naïve", "Ωμέγα", "Москва", "señor", "école"],
                  ["a", "é", "ñ", "ω", "м", " ", "o", "0", "é"], 4000)


def test_oracle_known_answer_similarity():
    """README.md:55-62: hello/helllo and world/wolrd score 0.896 (one insertion / one swap)."""
    from fuzzy_aho_corasick import FuzzyAhoCorasickBuilder, FuzzyLimits, SearchOptions
    e = OracleEngine(FuzzyAhoCorasickBuilder().fuzzy(FuzzyLimits().edits(1)).case_insensitive(True),
                     ["hello", "world"])
    ms = e.search("helllo wolrd", SearchOptions().threshold(0.8).sorted().non_overlapping())
    assert [round(m.similarity, 7) for m in ms] == [0.896, 0.896]
    assert {f32bits(m.similarity) for m in ms} == {f32bits(np.float32(0.8960000277))}
    assert [(m.insertions, m.swaps) for m in ms] == [(1, 0), (0, 1)]


def test_oracle_output_merge_quirk_span():
    """STOCK reported with the JOINT STOCK span (builder.rs:264-268, search.rs:659-678)."""
    from fuzzy_aho_corasick import FuzzyAhoCorasickBuilder, SearchOptions
    e = OracleEngine(FuzzyAhoCorasickBuilder(), ["JOINT STOCK COMPANY", "STOCK", "JOINT STOCK"])
    rows = {(m.start, m.end, m.pattern.as_str()) for m in e.search("JOINT STOCK", SearchOptions().threshold(0.8))}
    assert (0, 11, "STOCK") in rows and (6, 11, "STOCK") in rows and (0, 11, "JOINT STOCK") in rows
