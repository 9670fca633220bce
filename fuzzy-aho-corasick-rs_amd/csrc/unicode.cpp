// unicode.cpp — host-side UTF-8 staging: UAX #29 extended grapheme clusters and case folding.
//
// Replaces the reference's third-party boundary: `unicode-segmentation` ^1.13
// `graphemes(true)` / `grapheme_indices(true)` (builder.rs:197-205, search.rs:398-416,
// prefilter.rs:264, structs.rs:664) and Rust `str::to_lowercase` (builder.rs:198-200,
// search.rs:406-412). Property tables are generated offline (tools/gen_unicode_tables.py).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fac_internal.h"

namespace fac {
namespace {

struct GcbRange { uint32_t lo, hi; uint8_t prop; };
struct CpRange { uint32_t lo, hi; };
struct LowerMap { uint32_t cp; uint32_t out[3]; uint8_t n; };

#define FAC_UNICODE_QUAL
#include "unicode_data.inc"
#undef FAC_UNICODE_QUAL

enum Gcb : uint8_t {
  GCB_Other = 0, GCB_CR, GCB_LF, GCB_Control, GCB_Extend, GCB_ZWJ, GCB_RI, GCB_Prepend,
  GCB_SpacingMark, GCB_L, GCB_V, GCB_T, GCB_LV, GCB_LVT
};
enum Incb : uint8_t { INCB_None = 0, INCB_Linker, INCB_Consonant, INCB_Extend };

template <typename R>
const R* find_range(const R* tab, size_t n, uint32_t cp) {
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (tab[mid].hi < cp) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && tab[lo].lo <= cp && cp <= tab[lo].hi) return &tab[lo];
  return nullptr;
}

inline uint8_t gcb(uint32_t cp) {
  if (cp < 0x80) {  // ASCII fast path
    if (cp == '\r') return GCB_CR;
    if (cp == '\n') return GCB_LF;
    if (cp < 0x20 || cp == 0x7F) return GCB_Control;
    return GCB_Other;
  }
  const GcbRange* r = find_range(kGcbRanges, sizeof(kGcbRanges) / sizeof(kGcbRanges[0]), cp);
  return r ? r->prop : GCB_Other;
}
inline bool ext_pict(uint32_t cp) {
  if (cp < 0xA9) return false;
  return find_range(kExtPictRanges, sizeof(kExtPictRanges) / sizeof(kExtPictRanges[0]), cp) != nullptr;
}
inline uint8_t incb(uint32_t cp) {
  if (cp < 0x300) return INCB_None;
  const GcbRange* r = find_range(kIncbRanges, sizeof(kIncbRanges) / sizeof(kIncbRanges[0]), cp);
  return r ? r->prop : INCB_None;
}

struct Props {
  uint8_t g, ib;
  bool pict;
};
inline Props props(uint32_t cp) { return {gcb(cp), incb(cp), ext_pict(cp)}; }

inline bool is_ctl(uint8_t g) { return g == GCB_Control || g == GCB_CR || g == GCB_LF; }

}  // namespace

uint32_t utf8_decode(const uint8_t* s, uint64_t n, uint64_t& i) {
  uint8_t b0 = s[i];
  if (b0 < 0x80) { i += 1; return b0; }
  if ((b0 & 0xE0) == 0xC0 && i + 1 < n) {
    uint32_t cp = ((b0 & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu);
    i += 2;
    return cp;
  }
  if ((b0 & 0xF0) == 0xE0 && i + 2 < n) {
    uint32_t cp = ((b0 & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu);
    i += 3;
    return cp;
  }
  if ((b0 & 0xF8) == 0xF0 && i + 3 < n) {
    uint32_t cp = ((b0 & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) |
                  (s[i + 3] & 0x3Fu);
    i += 4;
    return cp;
  }
  i += 1;  // invalid; callers validate first
  return 0xFFFD;
}

// Length of the longest valid UTF-8 prefix (Rust's Utf8Error::valid_up_to).
uint64_t utf8_valid_prefix(const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    uint8_t b = s[i];
    if (b < 0x80) { ++i; continue; }
    int len;
    uint32_t min;
    if ((b & 0xE0) == 0xC0) { len = 2; min = 0x80; }
    else if ((b & 0xF0) == 0xE0) { len = 3; min = 0x800; }
    else if ((b & 0xF8) == 0xF0) { len = 4; min = 0x10000; }
    else return i;
    if (i + len > n) return i;
    for (int k = 1; k < len; ++k)
      if ((s[i + k] & 0xC0) != 0x80) return i;
    uint64_t j = i;
    uint32_t cp = utf8_decode(s, n, j);
    if (cp < min || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return i;
    i += len;
  }
  return n;
}

namespace {
// Rust's str::from_utf8 acceptance (no overlongs, surrogates or code points past U+10FFFF); ASCII
// runs are skipped eight bytes at a time
bool utf8_valid_serial(const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    if (i + 8 <= n) {
      uint64_t w;
      std::memcpy(&w, s + i, 8);
      if (!(w & 0x8080808080808080ull)) {
        i += 8;
        continue;
      }
    }
    uint8_t b = s[i];
    if (b < 0x80) { ++i; continue; }
    int len;
    uint32_t min;
    if ((b & 0xE0) == 0xC0) { len = 2; min = 0x80; }
    else if ((b & 0xF0) == 0xE0) { len = 3; min = 0x800; }
    else if ((b & 0xF8) == 0xF0) { len = 4; min = 0x10000; }
    else return false;
    if (i + len > n) return false;
    for (int k = 1; k < len; ++k)
      if ((s[i + k] & 0xC0) != 0x80) return false;
    uint64_t j = i;
    uint32_t cp = utf8_decode(s, n, j);
    if (cp < min || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
    i += len;
  }
  return true;
}
}  // namespace

// Large inputs are validated in up to 16 pieces on host threads, cut in front of a byte that is
// not a continuation byte: every sequence then lies inside one piece (a sequence truncated by a
// cut is invalid anyway, and so is a run of four continuation bytes that leaves no cut point).
bool utf8_valid(const uint8_t* s, uint64_t n, bool* ascii) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const uint64_t T = std::min<uint64_t>(std::min<uint64_t>(16, hw), n >> 22);  // >= 4 MiB a piece
  if (T <= 1) {
    const bool v = utf8_valid_serial(s, n);
    if (ascii) *ascii = v && ascii_only(s, n);
    return v;
  }
  std::vector<uint64_t> cut(T + 1);
  cut[0] = 0;
  cut[T] = n;
  for (uint64_t t = 1; t < T; ++t) {
    uint64_t p = n * t / T;
    for (int k = 0; k < 4 && p < n && (s[p] & 0xC0) == 0x80; ++k) ++p;
    cut[t] = std::max(cut[t - 1], p);
  }
  std::vector<char> ok(T, 1), asc(T, 1);
  std::vector<std::thread> th;
  for (uint64_t t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      ok[t] = utf8_valid_serial(s + cut[t], cut[t + 1] - cut[t]) ? 1 : 0;
      // the ASCII check of search.rs:196 on the same piece (early exit at the first non-ASCII 4 KiB)
      if (ascii && ok[t]) asc[t] = ascii_only(s + cut[t], cut[t + 1] - cut[t]) ? 1 : 0;
    });
  for (auto& x : th) x.join();
  const bool v = std::all_of(ok.begin(), ok.end(), [](char c) { return c != 0; });
  if (ascii) *ascii = v && std::all_of(asc.begin(), asc.end(), [](char c) { return c != 0; });
  return v;
}

// UAX #29 extended grapheme cluster boundaries (rules GB3-GB13, GB999, with GB9c InCB).
// Appends the byte offset of each grapheme start (the first is always 0 when n > 0).
void segment_graphemes(const uint8_t* s, uint64_t n, std::vector<uint64_t>& starts) {
  starts.clear();
  if (n == 0) return;
  uint64_t i = 0;
  uint32_t cp = utf8_decode(s, n, i);
  Props L = props(cp);
  starts.push_back(0);
  // state describing the text ending at the left character
  uint32_t ri_run = L.g == GCB_RI ? 1 : 0;  // consecutive RIs ending at left
  bool pict = L.pict;                         // left is in "ExtPict Extend*"
  bool gb11 = false;                          // left is ZWJ preceded by ExtPict Extend*
  int incb_state = L.ib == INCB_Consonant ? 1 : 0;  // 1: Consonant [Ext|Lnk]*, 2: ... with Linker
  while (i < n) {
    uint64_t pos = i;
    uint32_t c = utf8_decode(s, n, i);
    Props R = props(c);
    bool brk;
    if (L.g == GCB_CR && R.g == GCB_LF) brk = false;                        // GB3
    else if (is_ctl(L.g)) brk = true;                                      // GB4
    else if (is_ctl(R.g)) brk = true;                                      // GB5
    else if (L.g == GCB_L && (R.g == GCB_L || R.g == GCB_V || R.g == GCB_LV || R.g == GCB_LVT)) brk = false;  // GB6
    else if ((L.g == GCB_LV || L.g == GCB_V) && (R.g == GCB_V || R.g == GCB_T)) brk = false;  // GB7
    else if ((L.g == GCB_LVT || L.g == GCB_T) && R.g == GCB_T) brk = false;                   // GB8
    else if (R.g == GCB_Extend || R.g == GCB_ZWJ) brk = false;             // GB9
    else if (R.g == GCB_SpacingMark) brk = false;                          // GB9a
    else if (L.g == GCB_Prepend) brk = false;                              // GB9b
    else if (incb_state == 2 && R.ib == INCB_Consonant) brk = false;       // GB9c
    else if (gb11 && R.pict) brk = false;                                  // GB11
    else if (L.g == GCB_RI && R.g == GCB_RI && (ri_run & 1)) brk = false;   // GB12/13
    else brk = true;                                                       // GB999
    if (brk) starts.push_back(pos);
    // advance state: R becomes the left character
    ri_run = R.g == GCB_RI ? ri_run + 1 : 0;
    gb11 = R.g == GCB_ZWJ && pict;
    pict = R.pict ? true : (R.g == GCB_Extend ? pict : false);
    if (R.ib == INCB_Consonant) incb_state = 1;
    else if (R.ib == INCB_Linker && incb_state >= 1) incb_state = 2;
    else if (R.ib == INCB_Extend && incb_state >= 1) { /* unchanged */ }
    else incb_state = 0;
    L = R;
  }
}

// A shard cut at byte p (safe_cut): the previous character is ASCII and not CR, so no rule of
// segment_graphemes above keeps p inside a cluster unless the character at p is Extend, ZWJ or
// SpacingMark (GB9, GB9a); and after an ASCII character every piece of state (ri_run, pict, gb11,
// incb_state) depends on the character at p alone, so segmenting from p reproduces exactly the
// boundaries the whole text has from p on. Text without ASCII cuts before a character that starts
// a cluster in every context (see safe_cut).
bool nth_grapheme_from_end(const uint8_t* s, uint64_t len, uint64_t n, uint64_t& off) {
  if (n == 0) return false;
  std::vector<uint64_t> st;
  for (uint64_t span = 8 * n + 64;; span *= 2) {
    // segment a tail that starts at a context-free cut: its boundaries are the whole text's
    uint64_t p = span >= len ? 0 : len - span;
    while (p > 0 && !safe_cut(s, len, p)) --p;
    segment_graphemes(s + p, len - p, st);
    if (st.size() >= n) {
      off = p + st[st.size() - n];
      return true;
    }
    if (p == 0) return false;
  }
}

bool ascii_only(const uint8_t* s, uint64_t n) {
  uint64_t i = 0, acc = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, s + i, 8);
    acc |= w;
    if ((i & 4095) == 0 && (acc & 0x8080808080808080ull)) return false;
  }
  for (; i < n; ++i) acc |= s[i];
  return (acc & 0x8080808080808080ull) == 0;
}

bool safe_cut(const uint8_t* s, uint64_t n, uint64_t p) {
  if (p == 0 || p >= n) return true;
  if ((s[p] & 0xC0) == 0x80) return false;  // not a code point start
  uint64_t i = p;
  const uint32_t r = utf8_decode(s, n, i);
  const uint8_t g = gcb(r);
  const uint8_t prev = s[p - 1];
  if (prev < 0x80) {
    if (prev == '\r') return false;
    return g != GCB_Extend && g != GCB_ZWJ && g != GCB_SpacingMark;
  }
  // After a non-ASCII character (text with no ASCII, e.g. CJK without spaces): a character that
  // starts a cluster on its own -- GCB Other or a Hangul LV / LVT syllable (no GB7-GB9a, GB12/13),
  // not Extended_Pictographic (GB11), no InCB class (GB9c) -- is preceded by a boundary in every
  // context unless the previous character is Prepend (GB9b) or a leading jamo L (GB6), and it resets
  // every piece of segmenter state.
  if ((g != GCB_Other && g != GCB_LV && g != GCB_LVT) || ext_pict(r) || incb(r) != INCB_None) return false;
  uint64_t q = p - 1;
  while (q > 0 && (s[q] & 0xC0) == 0x80 && p - q < 4) --q;
  uint64_t t = q;
  const uint8_t lg = gcb(utf8_decode(s, n, t));
  return lg != GCB_Prepend && lg != GCB_L;
}

int lower_full(uint32_t cp, uint32_t out[3]) {
  if (cp < 0x80) {
    out[0] = (cp >= 'A' && cp <= 'Z') ? cp + 32 : cp;
    return 1;
  }
  size_t lo = 0, hi = sizeof(kLowerMap) / sizeof(kLowerMap[0]);
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (kLowerMap[mid].cp < cp) lo = mid + 1;
    else hi = mid;
  }
  if (lo < sizeof(kLowerMap) / sizeof(kLowerMap[0]) && kLowerMap[lo].cp == cp) {
    for (int k = 0; k < kLowerMap[lo].n; ++k) out[k] = kLowerMap[lo].out[k];
    return kLowerMap[lo].n;
  }
  out[0] = cp;
  return 1;
}

// One grapheme's folded code points: `to_lowercase()` when case-insensitive (search.rs:406-412;
// builder.rs:198-200). Per-char full mapping; a lone capital sigma at grapheme start is never
// word-final, so char-wise mapping equals Rust's context-sensitive `str::to_lowercase` here.
void fold_grapheme(const uint8_t* s, uint64_t b, uint64_t e, bool ci, std::u32string& out) {
  out.clear();
  uint64_t i = b;
  while (i < e) {
    uint32_t cp = utf8_decode(s, e, i);
    if (ci) {
      uint32_t lo[3];
      int k = lower_full(cp, lo);
      for (int t = 0; t < k; ++t) out.push_back(lo[t]);
    } else {
      out.push_back(cp);
    }
  }
}

uint32_t fold_first_char(const uint8_t* s, uint64_t b, uint64_t e, bool ci) {
  if (b >= e) return 0;
  uint64_t i = b;
  uint32_t cp = utf8_decode(s, e, i);
  if (!ci) return cp;
  uint32_t lo[3];
  lower_full(cp, lo);
  return lo[0];
}

}  // namespace fac
