"""MI355X-native drop-in for the hot path of kakserpom/fuzzy-aho-corasick-rs.

Mirrors the crate's public API (lib.rs:96-105): FuzzyAhoCorasickBuilder, FuzzyAhoCorasick,
FuzzyLimits, FuzzyPenalties, Pattern, SearchOptions, Order, Overlap, FuzzyMatch, FuzzyMatches,
Segment, Similarity, SearchError. The search itself runs in HIP kernels (libfac.so).
"""
from .engine import (FuzzyAhoCorasick, FuzzyAhoCorasickBuilder, FuzzyReplacer, Prefiltered,
                     StagedHaystack, StreamMatch)
from .matches import FuzzyMatch, FuzzyMatches, Segment, UnmatchedSegment
from .structs import (DEFAULT_THRESHOLD, DeviceError, FuzzyLimits, FuzzyPenalties, HaystackTooLarge,
                      Order, Overlap, Pattern, SearchError, SearchOptions, Similarity,
                      UnsupportedConfiguration)

__all__ = [
    "FuzzyAhoCorasick", "FuzzyAhoCorasickBuilder", "FuzzyReplacer", "Prefiltered", "StagedHaystack", "StreamMatch",
    "FuzzyMatch", "FuzzyMatches", "Segment", "UnmatchedSegment", "DEFAULT_THRESHOLD", "DeviceError",
    "FuzzyLimits", "FuzzyPenalties", "HaystackTooLarge", "Order", "Overlap", "Pattern", "SearchError",
    "SearchOptions", "Similarity", "UnsupportedConfiguration",
]
