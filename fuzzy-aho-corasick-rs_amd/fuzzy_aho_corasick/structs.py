"""Data model mirroring src/structs.rs and src/options.rs of the reference crate."""
from __future__ import annotations

import enum
import struct
from dataclasses import dataclass, field
from typing import Dict, Iterable, Optional, Tuple

from . import _native

f32 = lambda x: struct.unpack("<f", struct.pack("<f", float(x)))[0]  # noqa: E731  (round to f32)


def f32_total_key(x: float) -> int:
    """f32::total_cmp as an integer sort key."""
    (u,) = struct.unpack("<I", struct.pack("<f", x))
    return (~u & 0xFFFFFFFF) if (u & 0x80000000) else (u | 0x80000000)


class FuzzyLimits:
    """FuzzyLimits (structs.rs:293-363): chainable builder; unset per-type caps default to 0 unless
    a total `edits` budget is set (finalize, structs.rs:319-335)."""

    def __init__(self):
        self.insertions_: Optional[int] = None
        self.deletions_: Optional[int] = None
        self.substitutions_: Optional[int] = None
        self.swaps_: Optional[int] = None
        self.edits_: Optional[int] = None

    @classmethod
    def new(cls) -> "FuzzyLimits":
        return cls()

    def _set(self, name, num):
        if not (0 <= int(num) <= 255):
            raise ValueError("edit counts are u8 (0..=255)")
        setattr(self, name, int(num))
        return self

    def insertions(self, num: int) -> "FuzzyLimits":
        return self._set("insertions_", num)

    def deletions(self, num: int) -> "FuzzyLimits":
        return self._set("deletions_", num)

    def substitutions(self, num: int) -> "FuzzyLimits":
        return self._set("substitutions_", num)

    def swaps(self, num: int) -> "FuzzyLimits":
        return self._set("swaps_", num)

    def edits(self, num: int) -> "FuzzyLimits":
        return self._set("edits_", num)

    def clone(self) -> "FuzzyLimits":
        c = FuzzyLimits()
        c.__dict__.update(self.__dict__)
        return c

    def finalize(self) -> "FuzzyLimits":
        c = self.clone()
        if c.edits_ is None:
            for name in ("insertions_", "deletions_", "substitutions_", "swaps_"):
                if getattr(c, name) is None:
                    setattr(c, name, 0)
        return c

    def as_tuple(self):
        return (self.insertions_, self.deletions_, self.substitutions_, self.swaps_, self.edits_)

    def to_c(self) -> _native.fac_limits:
        n = lambda v: _native.LIMIT_NONE if v is None else v  # noqa: E731
        return _native.fac_limits(n(self.insertions_), n(self.deletions_), n(self.substitutions_),
                                  n(self.swaps_), n(self.edits_))

    def __eq__(self, other):
        return isinstance(other, FuzzyLimits) and self.as_tuple() == other.as_tuple()

    def __repr__(self):
        i, d, s, w, e = self.as_tuple()
        return f"FuzzyLimits(insertions={i}, deletions={d}, substitutions={s}, swaps={w}, edits={e})"


class FuzzyPenalties:
    """FuzzyPenalties (structs.rs:370-420); default m = 1.3 scaling (structs.rs:381-393), f32."""

    def __init__(self, insertion=None, deletion=None, substitution=None, swap=None):
        m = f32(1.3)
        self.substitution = f32(f32(1.1) * m) if substitution is None else f32(substitution)
        self.insertion = f32(f32(0.4) * m) if insertion is None else f32(insertion)
        self.deletion = f32(f32(0.7) * m) if deletion is None else f32(deletion)
        self.swap = f32(f32(0.4) * m) if swap is None else f32(swap)

    @classmethod
    def default(cls) -> "FuzzyPenalties":
        return cls()

    def _with(self, **kw):
        p = FuzzyPenalties(self.insertion, self.deletion, self.substitution, self.swap)
        for k, v in kw.items():
            setattr(p, k, f32(v))
        return p

    # The Rust setters share the field names (structs.rs:395-420); Python needs distinct names.
    def with_insertion(self, v) -> "FuzzyPenalties":
        return self._with(insertion=v)

    def with_deletion(self, v) -> "FuzzyPenalties":
        return self._with(deletion=v)

    def with_substitution(self, v) -> "FuzzyPenalties":
        return self._with(substitution=v)

    def with_swap(self, v) -> "FuzzyPenalties":
        return self._with(swap=v)

    def __repr__(self):
        return (f"FuzzyPenalties(insertion={self.insertion}, deletion={self.deletion}, "
                f"substitution={self.substitution}, swap={self.swap})")


class Similarity:
    """Similarity (structs.rs:9-93): ordered (char, char) -> score pairs; unlisted pairs score 0,
    identical chars 1. ASCII pairs go to a 128x128 f32 table."""

    def __init__(self, pairs: Dict[Tuple[str, str], float]):
        self.pairs = {(a, b): f32(s) for (a, b), s in dict(pairs).items()}

    @classmethod
    def from_map(cls, pairs) -> "Similarity":
        return cls(dict(pairs))

    def ascii_table(self):
        t = [0.0] * (128 * 128)
        for i in range(128):
            t[i * 128 + i] = 1.0
        for (a, b), s in self.pairs.items():
            if ord(a) < 128 and ord(b) < 128:
                t[ord(a) * 128 + ord(b)] = s
        return t

    def extra_pairs(self):
        return [(ord(a), ord(b), s) for (a, b), s in self.pairs.items()
                if not (ord(a) < 128 and ord(b) < 128)]


def _grapheme_len(s: str) -> int:
    return len(_native.grapheme_starts(s.encode("utf-8")))


@dataclass
class Pattern:
    """Pattern (structs.rs:598-754). `grapheme_len` counts extended grapheme clusters."""
    pattern: str
    weight: float = 1.0
    limits: Optional[FuzzyLimits] = None
    custom_unique_id_: Optional[int] = None
    grapheme_len: int = field(default=-1)

    def __post_init__(self):
        self.weight = f32(self.weight)
        if self.grapheme_len < 0:
            self.grapheme_len = _grapheme_len(self.pattern)

    @classmethod
    def from_(cls, x) -> "Pattern":
        """The `From` conversions: str, (str, weight), (str, weight, max_edits), Pattern."""
        if isinstance(x, Pattern):
            return x
        if isinstance(x, str):
            return cls(x)
        if isinstance(x, tuple):
            if len(x) == 2:
                return cls(x[0], x[1])
            if len(x) == 3:
                return cls(x[0], x[1], FuzzyLimits().edits(x[2]).finalize())
        raise TypeError(f"cannot convert {x!r} into a Pattern")

    def as_str(self) -> str:
        return self.pattern

    def len(self) -> int:
        """Length in BYTES (structs.rs:628-630)."""
        return len(self.pattern.encode("utf-8"))

    def is_empty(self) -> bool:
        return self.len() == 0

    def fuzzy(self, limits: FuzzyLimits) -> "Pattern":
        self.limits = limits.finalize()
        return self

    def custom_unique_id(self, id_: int) -> "Pattern":
        self.custom_unique_id_ = id_
        return self

    def with_weight(self, w: float) -> "Pattern":
        self.weight = f32(w)
        return self

    def __str__(self):
        return self.pattern


class Order(enum.Enum):
    """options.rs:10-22"""
    Unsorted = 0
    Default = 1
    Greedy = 2
    CoverageWeighted = 3


class Overlap(enum.Enum):
    """options.rs:25-35"""
    Keep = 0
    NonOverlapping = 1
    NonOverlappingUnique = 2


DEFAULT_THRESHOLD = 0.0  # options.rs:7


class SearchOptions:
    """SearchOptions (options.rs:44-132)."""

    def __init__(self, threshold: float = DEFAULT_THRESHOLD, order: Order = Order.Unsorted,
                 overlap: Overlap = Overlap.Keep):
        self.threshold_ = f32(threshold)
        self.order_ = order
        self.overlap_ = overlap

    @classmethod
    def new(cls) -> "SearchOptions":
        return cls()

    def _copy(self, **kw):
        o = SearchOptions(self.threshold_, self.order_, self.overlap_)
        for k, v in kw.items():
            setattr(o, k, v)
        return o

    def threshold(self, t: float) -> "SearchOptions":
        return self._copy(threshold_=f32(t))

    def order(self, o: Order) -> "SearchOptions":
        return self._copy(order_=o)

    def overlap(self, o: Overlap) -> "SearchOptions":
        return self._copy(overlap_=o)

    def sorted(self) -> "SearchOptions":
        return self.order(Order.Default)

    def greedy(self) -> "SearchOptions":
        return self.order(Order.Greedy)

    def coverage_weighted(self) -> "SearchOptions":
        return self.order(Order.CoverageWeighted)

    def non_overlapping(self) -> "SearchOptions":
        return self.overlap(Overlap.NonOverlapping)

    def non_overlapping_unique(self) -> "SearchOptions":
        return self.overlap(Overlap.NonOverlappingUnique)


class SearchError(Exception):
    """SearchError (error.rs:7-17). Only HaystackTooLarge is a reference variant; the others are
    the new #[non_exhaustive] cases of the GPU engine."""


class HaystackTooLarge(SearchError):
    def __init__(self, graphemes: int):
        super().__init__(f"haystack has {graphemes} grapheme clusters, exceeding the u32 position "
                         "space this engine indexes with; use the streaming API for inputs larger "
                         "than ~4 GiB")
        self.graphemes = graphemes


class DeviceError(SearchError):
    """HIP / device / capacity failures of the GPU engine (codes >= 100 in include/fac.h)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"[fac error {code}] {message}")
        self.code = code


class UnsupportedConfiguration(SearchError):
    """A configuration the GPU path does not implement (never silently diverges)."""
