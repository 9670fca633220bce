"""FuzzyMatch / FuzzyMatches host-side post-processing (src/matches.rs, src/structs.rs:756-889).

Ranking and overlap resolution (FuzzyMatches::apply, matches.rs:7-149) run on the device
(rank_kernels.hip via the C ABI's fac_matches_apply) before any Python object is
built; the host-side code here wraps the ranked records as FuzzyMatch objects and keeps a pure-Python
apply only for record lists built by hand.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Callable, Iterator, List, Optional

import numpy as np

from .structs import Order, Overlap, Pattern, f32_total_key


@dataclass
class FuzzyMatch:
    """structs.rs:757-781. `start`/`end` are BYTE offsets into the UTF-8 haystack."""
    insertions: int
    deletions: int
    substitutions: int
    swaps: int
    edits: int
    pattern_index: int
    pattern: Pattern
    start: int
    end: int
    similarity: float
    text: str

    def key(self):
        return (self.start, self.end, self.pattern_index)

    def sim_bits(self) -> int:
        return struct.unpack("<I", struct.pack("<f", self.similarity))[0]


@dataclass
class UnmatchedSegment:
    start: int
    end: int
    text: str


class Segment:
    """Segment::Matched / Segment::Unmatched (structs.rs:786-846)."""

    def __init__(self, matched: Optional[FuzzyMatch] = None, unmatched: Optional[UnmatchedSegment] = None):
        self._m = matched
        self._u = unmatched

    def matched(self):
        return self._m

    def unmatched(self):
        return self._u

    def as_str(self) -> str:
        return self._m.text if self._m is not None else self._u.text

    def __len__(self):
        return len(self.as_str().encode("utf-8"))

    def __repr__(self):
        return f"Matched({self._m!r})" if self._m is not None else f"Unmatched({self._u!r})"


_SPACE = ("\x20", "\t")
_NO_LEADING_SPACE_PUNCTUATION = (",", ".", "?", "!", ";", ":", "—", "-", "…")


class FuzzyMatches:
    """structs.rs:853-889 + matches.rs. Behaves like a list of FuzzyMatch."""

    def __init__(self, haystack: str, inner: List[FuzzyMatch], haystack_bytes: bytes = None):
        self.haystack = haystack
        self.hay_bytes = haystack_bytes if haystack_bytes is not None else haystack.encode("utf-8")
        self.inner = inner

    # -- container protocol
    def __len__(self):
        return len(self.inner)

    def __iter__(self) -> Iterator[FuzzyMatch]:
        return iter(self.inner)

    def __getitem__(self, i):
        return self.inner[i]

    def __repr__(self):
        return f"FuzzyMatches({self.inner!r})"

    def iter(self):
        return iter(self.inner)

    def len(self):
        return len(self.inner)

    def is_empty(self):
        return not self.inner

    def _slice(self, a: int, b: int) -> str:
        return self.hay_bytes[a:b].decode("utf-8")

    # -- ranking (matches.rs:7-81); comparators are total orders over distinct keys
    def apply(self, order: Order, overlap: Overlap) -> "FuzzyMatches":
        if order == Order.Default:
            self.default_sort()
        elif order == Order.Greedy:
            self.greedy_sort()
        elif order == Order.CoverageWeighted:
            self.coverage_weighted_sort()
        if overlap == Overlap.NonOverlapping:
            self.non_overlapping()
        elif overlap == Overlap.NonOverlappingUnique:
            self.non_overlapping_unique()
        return self

    def default_sort(self):
        self.inner.sort(key=lambda m: (-f32_total_key(m.similarity), -m.pattern.len(),
                                       -len(m.text.encode("utf-8")), m.start, m.end, m.pattern_index))

    def greedy_sort(self):
        self.inner.sort(key=lambda m: (-m.pattern.len(), -f32_total_key(m.similarity), m.start, m.end,
                                       m.pattern_index))

    def coverage_weighted_sort(self):
        def score(m):  # similarity * similarity * len as f32 (matches.rs:69-70)
            s = np.float32(m.similarity)
            return float(np.float32(np.float32(s * s) * np.float32(m.pattern.len())))
        self.inner.sort(key=lambda m: (-f32_total_key(score(m)), -f32_total_key(m.similarity), m.start,
                                       m.end, m.pattern_index))

    # -- overlap resolution (matches.rs:86-149)
    def non_overlapping(self):
        occupied: List[tuple] = []
        starts: List[int] = []  # occupied's starts, kept beside it (one bisect per match)
        kept = []
        import bisect
        for m in self.inner:
            # binary_search Ok(idx)/Err(idx): equal starts occur only for empty spans, where every
            # choice of idx gives the same accept/reject decisions
            pos = bisect.bisect_left(starts, m.start)
            prev_ok = pos == 0 or occupied[pos - 1][1] <= m.start
            next_ok = pos == len(occupied) or occupied[pos][0] >= m.end
            if prev_ok and next_ok:
                occupied.insert(pos, (m.start, m.end))
                starts.insert(pos, m.start)
                kept.append(m)
        kept.sort(key=lambda m: m.start)
        self.inner = kept

    def non_overlapping_unique(self):
        import bisect
        used = set()
        occupied: List[tuple] = []
        starts: List[int] = []
        kept = []
        for m in self.inner:
            uid = ("custom", m.pattern.custom_unique_id_) if m.pattern.custom_unique_id_ is not None \
                else ("auto", m.pattern_index)
            if uid in used:
                continue
            pos = bisect.bisect_left(starts, m.start)
            prev_ok = pos == 0 or occupied[pos - 1][1] <= m.start
            next_ok = pos == len(occupied) or occupied[pos][0] >= m.end
            if prev_ok and next_ok:
                used.add(uid)
                occupied.insert(pos, (m.start, m.end))
                starts.insert(pos, m.start)
                kept.append(m)
        kept.sort(key=lambda m: m.start)
        self.inner = kept

    # -- segmentation helpers (matches.rs:165-594)
    def replace(self, callback: Callable[[FuzzyMatch], Optional[str]]) -> str:
        out = []
        last = 0
        for m in self.inner:
            if m.start >= last:
                out.append(self._slice(last, m.start))
                last = m.end
                r = callback(m)
                out.append(m.text if r is None else str(r))
        out.append(self._slice(last, len(self.hay_bytes)))
        return "".join(out)

    def segment_iter(self) -> Iterator[Segment]:
        segs = []
        last = 0
        for m in self.inner:
            if m.start >= last:
                if m.start > last:
                    segs.append(Segment(unmatched=UnmatchedSegment(last, m.start, self._slice(last, m.start))))
                last = m.end
                segs.append(Segment(matched=m))
        n = len(self.hay_bytes)
        if last < n:
            segs.append(Segment(unmatched=UnmatchedSegment(last, n, self._slice(last, n))))
        return iter(segs)

    def strip_prefix(self) -> str:
        out = []
        skipping = True
        for seg in self.segment_iter():
            if seg.matched() is not None:
                if skipping:
                    continue
                out.append(seg.matched().text)
            else:
                u = seg.unmatched()
                if skipping:
                    if u.text.strip() == "":
                        continue
                    skipping = False
                    out.append(u.text.lstrip())
                else:
                    out.append(u.text)
        return "".join(out)

    def strip_suffix(self) -> str:
        buf = []
        keep = 0
        for seg in self.segment_iter():
            buf.append(seg)
            if seg.unmatched() is not None and seg.unmatched().text.strip() != "":
                keep = len(buf)
        out = []
        for i, seg in enumerate(buf[:keep]):
            last = i + 1 == keep
            if seg.matched() is not None:
                out.append(seg.matched().text)
            else:
                out.append(seg.unmatched().text.rstrip() if last else seg.unmatched().text)
        return "".join(out)

    def split(self) -> Iterator[str]:
        return (s.unmatched().text for s in self.segment_iter() if s.unmatched() is not None)

    def segment_text(self) -> str:
        out = ""
        prev_matched = False
        for seg in self.segment_iter():
            if seg.matched() is not None:
                if prev_matched or (out and not out.endswith(_SPACE)):
                    out += " "
                prev_matched = True
                out += seg.matched().text
            else:
                u = seg.unmatched()
                if prev_matched and not u.text.startswith(_NO_LEADING_SPACE_PUNCTUATION):
                    out += " "
                prev_matched = False
                out += u.text
        return out

    def retain(self, pred) -> "FuzzyMatches":
        self.inner = [m for m in self.inner if pred(m)]
        return self

    def filter(self, pred) -> "FuzzyMatches":
        return FuzzyMatches(self.haystack, [m for m in self.inner if pred(m)], self.hay_bytes)

    def matched_spans(self):
        return [(m.start, m.end) for m in self.inner]

    def matched_strings(self):
        return [m.text for m in self.inner]
