"""Seeded synthetic workloads of BASELINE.json `configs` (generator spec: SURVEY.md §8(d)).

xorshift64 (x ^= x << 13; x ^= x >> 7; x ^= x << 17, as in prefilter.rs:441-452) drives a
numpy-vectorised generator: N distinct pattern words, a haystack of random words separated by
' ', and every `plant_every` bytes a random pattern planted with exactly E' ~ U{0..E} random
edits (insertion / deletion / substitution / swap).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import numpy as np

ASCII_LOWER = [chr(c) for c in range(ord("a"), ord("z") + 1)]
# C3 alphabet: upper/lower Latin, Latin-1 precomposed, Greek, Cyrillic; single-code-point
# graphemes whose lowercase is a single code point in every Unicode version involved.
LATIN1 = [chr(c) for c in range(0xC0, 0x100) if c not in (0xD7, 0xF7, 0xDF, 0xFF)]
GREEK = [chr(c) for c in range(0x391, 0x3AA) if c != 0x3A2] + [chr(c) for c in range(0x3B1, 0x3CA)]
CYRILLIC = [chr(c) for c in range(0x410, 0x450)]
SCRIPTS_C3 = [
    [chr(c) for c in range(ord("a"), ord("z") + 1)] + [chr(c) for c in range(ord("A"), ord("Z") + 1)],
    LATIN1, GREEK, CYRILLIC,
]


class XorShift:
    def __init__(self, seed: int):
        self.s = (seed or 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF

    def next(self) -> int:
        x = self.s
        x ^= (x << 13) & 0xFFFFFFFFFFFFFFFF
        x ^= x >> 7
        x ^= (x << 17) & 0xFFFFFFFFFFFFFFFF
        self.s = x
        return x

    def numpy(self) -> np.random.Generator:
        """A numpy generator seeded from the xorshift stream (for the bulk vectorised parts)."""
        return np.random.Generator(np.random.PCG64(self.next()))


@dataclass
class Workload:
    name: str
    patterns: List[str]
    haystack: bytes
    edits: int
    beam: int
    case_insensitive: bool
    threshold: float
    prefilter: bool = False


def _words(rng: np.random.Generator, alphabets, n: int, lo: int, hi: int, distinct: bool) -> List[str]:
    out, seen = [], set()
    while len(out) < n:
        m = max(n - len(out), 64) * 2
        lens = rng.integers(lo, hi + 1, size=m)
        scr = rng.integers(0, len(alphabets), size=m)
        for L, s in zip(lens, scr):
            al = alphabets[s]
            w = "".join(al[i] for i in rng.integers(0, len(al), size=L))
            if distinct:
                key = w.lower()
                if key in seen:
                    continue
                seen.add(key)
            out.append(w)
            if len(out) == n:
                break
    return out


def _mutate(rng: np.random.Generator, w: str, edits: int, alphabet) -> str:
    s = list(w)
    for _ in range(edits):
        op = int(rng.integers(0, 4))
        if op == 0 or len(s) < 2:  # insertion
            s.insert(int(rng.integers(0, len(s) + 1)), alphabet[int(rng.integers(0, len(alphabet)))])
        elif op == 1:  # deletion
            del s[int(rng.integers(0, len(s)))]
        elif op == 2:  # substitution
            s[int(rng.integers(0, len(s)))] = alphabet[int(rng.integers(0, len(alphabet)))]
        else:  # swap
            i = int(rng.integers(0, len(s) - 1))
            s[i], s[i + 1] = s[i + 1], s[i]
    return "".join(s)


def _fresh_filler(rng: np.random.Generator, alphabets, nbytes: int, word_lo: int, word_hi: int) -> bytes:
    """Fresh random words: every word draws its own length in [word_lo, word_hi], its
    script and each of its characters, independently; words end with ' '. Vectorised over all words."""
    cps = [np.array([ord(c) for c in al], np.uint32) for al in alphabets]
    width = max(len(a) for a in cps)
    table = np.zeros((len(cps), width), np.uint32)
    for i, a in enumerate(cps):
        table[i, : len(a)] = a
    alen = np.array([len(a) for a in cps], np.int64)
    ascii_only = int(table.max()) < 0x80
    bpc = 1.0 if ascii_only else float(np.mean([np.mean(1 + (a >= 0x80) + (a >= 0x800)) for a in cps]))
    mean = (word_lo + word_hi) / 2.0 * bpc + 1.0
    out, total = [], 0
    while total < nbytes:
        n = int((nbytes - total) / mean * 1.02) + 64
        lens = rng.integers(word_lo, word_hi + 1, size=n)
        scr = rng.integers(0, len(cps), size=n)
        wid = np.repeat(np.arange(n), lens + 1)             # the word of every character (+ its space)
        pos = np.arange(len(wid)) - np.repeat(np.cumsum(lens + 1) - (lens + 1), lens + 1)
        idx = (rng.random(len(wid)) * alen[scr[wid]]).astype(np.int64)
        ch = table[scr[wid], idx]
        ch[pos == lens[wid]] = 0x20
        b = ch.astype(np.uint8).tobytes() if ascii_only else ch.tobytes().decode("utf-32-le").encode("utf-8")
        out.append(b)
        total += len(b)
    return b"".join(out)


def _haystack(rng: np.random.Generator, alphabets, patterns: List[str], nbytes: int, edits: int,
              plant_every: int, word_lo=2, word_hi=12, vocab=50_000) -> bytes:
    """Random words separated by ' ' with a planted (mutated) pattern every `plant_every` bytes.
    vocab: the filler words are drawn with replacement from a fixed vocabulary of this many random
    words (rounds 1-2 default); None: every filler word is fresh (SURVEY.md §8(d) taken literally)."""
    flat_alpha = [c for al in alphabets for c in al]
    if vocab is None:
        filler = _fresh_filler(rng, alphabets, nbytes, word_lo, word_hi)
        sp = np.flatnonzero(np.frombuffer(filler, np.uint8) == 0x20)
        cuts = sp[np.searchsorted(sp, np.arange(plant_every, len(filler), plant_every))[:-1]] + 1
        pieces, prev = [], 0
        for c in cuts.tolist() + [len(filler)]:
            pieces.append(filler[prev:c])
            p = patterns[int(rng.integers(0, len(patterns)))]
            e = int(rng.integers(0, edits + 1))
            pieces.append(_mutate(rng, p, e, flat_alpha).encode("utf-8") + b" ")
            prev = c
        data = b"".join(pieces)
    else:
        # vocabulary of filler words, sampled with replacement (vectorised join)
        vocab_w = _words(rng, alphabets, vocab, word_lo, word_hi, distinct=False)
        vocab_b = [w.encode("utf-8") for w in vocab_w]
        mean = sum(len(b) for b in vocab_b) / len(vocab_b) + 1
        chunks = []
        total = 0
        while total < nbytes:
            nw = max(1, int(plant_every / mean))
            idx = rng.integers(0, len(vocab_b), size=nw)
            part = b" ".join(vocab_b[i] for i in idx)
            p = patterns[int(rng.integers(0, len(patterns)))]
            e = int(rng.integers(0, edits + 1))
            planted = _mutate(rng, p, e, flat_alpha).encode("utf-8")
            piece = part + b" " + planted + b" "
            chunks.append(piece)
            total += len(piece)
        data = b"".join(chunks)
    # cut at a character boundary, then drop a trailing partial word
    cut = min(nbytes, len(data))
    while cut > 0 and (data[cut - 1] & 0xC0) == 0x80:
        cut -= 1
    if cut > 0 and data[cut - 1] >= 0xC0:
        cut -= 1
    return data[:cut]


def config(name: str, nbytes: int = None, seed: int = None, hay_seed: int = None, vocab=50_000) -> Workload:
    """BASELINE.json configs: c1 (exact, 16 ASCII patterns, 1 MiB), c2 (edits 1, 1K ASCII, 1 GiB),
    c3 (edits 2, beam 64, 10K patterns, case-insensitive Unicode), c4 (c2 engine, 128 MiB per
    haystack), c5 (sparse, 1K patterns of 10-16, edits 1, threshold 0.85, prefilter).
    vocab: filler words from a fixed vocabulary of that many random words, or None for fresh words."""
    hs = lambda default: XorShift(hay_seed if hay_seed is not None else default).numpy()  # noqa: E731
    if name == "c1":
        rng = XorShift(seed or 1).numpy()
        pats = _words(rng, [ASCII_LOWER], 16, 4, 16, True)
        hay = _haystack(hs((seed or 1) + 1000), [ASCII_LOWER], pats, nbytes or (1 << 20), 0, 4096, vocab=vocab)
        return Workload("c1", pats, hay, 0, 0, False, 0.8)
    if name in ("c2", "c4"):
        base = seed or 2  # C4 runs the C2 engine on haystacks of seeds 40..47
        rng = XorShift(base).numpy()
        pats = _words(rng, [ASCII_LOWER], 1000, 4, 16, True)
        default = (1 << 30) if name == "c2" else (128 << 20)
        hay = _haystack(hs(base + 1000 if name == "c2" else 40), [ASCII_LOWER], pats, nbytes or default, 1, 4096, vocab=vocab)
        return Workload(name, pats, hay, 1, 0, False, 0.8)
    if name == "c3":
        rng = XorShift(seed or 3).numpy()
        pats = _words(rng, SCRIPTS_C3, 10_000, 4, 16, True)
        hay = _haystack(hs((seed or 3) + 1000), SCRIPTS_C3, pats, nbytes or (256 << 20), 2, 4096, vocab=vocab)
        return Workload("c3", pats, hay, 2, 64, True, 0.8)
    if name == "c5":
        rng = XorShift(seed or 5).numpy()
        pats = _words(rng, [ASCII_LOWER], 1000, 10, 16, True)
        hay = _haystack(hs((seed or 5) + 1000), [ASCII_LOWER], pats, nbytes or (1 << 30), 1,
                        1 << 20, vocab=vocab)
        return Workload("c5", pats, hay, 1, 0, False, 0.85, prefilter=True)
    raise ValueError(name)


def builder_for(w: Workload):
    from .engine import FuzzyAhoCorasickBuilder
    from .structs import FuzzyLimits
    b = FuzzyAhoCorasickBuilder().case_insensitive(w.case_insensitive)
    if w.edits:
        b = b.fuzzy(FuzzyLimits().edits(w.edits))
    if w.beam:
        b = b.beam_width(w.beam)
    return b
