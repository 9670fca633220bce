// stage_kernels.hip — search_raw's Unicode staging on the MI355X (search.rs:296-302, 398-416):
// UAX #29 extended grapheme clusters (the reference's `unicode-segmentation`
// `grapheme_indices(true)`) and the folded first code point per grapheme (`to_lowercase`).
//
// The segmenter is the host state machine of unicode.cpp (same generated tables), run per
// 256-byte chunk: the state a boundary decision needs (left properties, regional-indicator parity,
// "ExtPict Extend*" / "... ZWJ" for GB11, the InCB conjunct state for GB9c) is fully reset after any
// code point that is not RI, ZWJ, Extend, Extended_Pictographic or InCB-classified, so each
// thread starts at the last such "resync" code point before its chunk (any letter, digit, space or
// punctuation of ordinary text) and decides every boundary inside its chunk exactly. Text with no
// resync point within 1 KiB before a chunk (long emoji / RI / combining runs) is segmented by one
// sequential device thread instead. Grapheme starts are compacted per 16 KiB unit: one wave counts
// each unit, one workgroup scans the counts, one wave writes each unit's starts in order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>

#include "fac_internal.h"

namespace fac {
namespace {

struct GcbRange { uint32_t lo, hi; uint8_t prop; };
struct CpRange { uint32_t lo, hi; };
struct LowerMap { uint32_t cp; uint32_t out[3]; uint8_t n; };

#define FAC_UNICODE_QUAL __device__
#include "unicode_data.inc"
#undef FAC_UNICODE_QUAL

enum Gcb : uint8_t {
  GCB_Other = 0, GCB_CR, GCB_LF, GCB_Control, GCB_Extend, GCB_ZWJ, GCB_RI, GCB_Prepend,
  GCB_SpacingMark, GCB_L, GCB_V, GCB_T, GCB_LV, GCB_LVT
};
enum Incb : uint8_t { INCB_None = 0, INCB_Linker, INCB_Consonant, INCB_Extend };

constexpr uint32_t kLookback = 1024;   // bytes searched backwards for a resync code point

template <typename R>
__device__ const R* find_range(const R* tab, uint32_t n, uint32_t cp) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (tab[mid].hi < cp) lo = mid + 1;
    else hi = mid;
  }
  return (lo < n && tab[lo].lo <= cp && cp <= tab[lo].hi) ? &tab[lo] : nullptr;
}

struct Props {
  uint8_t g, ib;
  bool pict;
};

__device__ Props props(uint32_t cp) {  // unicode.cpp gcb / ext_pict / incb
  Props p{GCB_Other, INCB_None, false};
  if (cp < 0x80) {
    p.g = cp == '\r' ? GCB_CR : cp == '\n' ? GCB_LF : (cp < 0x20 || cp == 0x7F) ? GCB_Control : GCB_Other;
    return p;
  }
  const GcbRange* r = find_range(kGcbRanges, sizeof(kGcbRanges) / sizeof(kGcbRanges[0]), cp);
  p.g = r ? r->prop : GCB_Other;
  if (cp >= 0xA9) p.pict = find_range(kExtPictRanges, sizeof(kExtPictRanges) / sizeof(kExtPictRanges[0]), cp) != nullptr;
  if (cp >= 0x300) {
    const GcbRange* q = find_range(kIncbRanges, sizeof(kIncbRanges) / sizeof(kIncbRanges[0]), cp);
    p.ib = q ? q->prop : INCB_None;
  }
  return p;
}

__device__ uint32_t decode(const uint8_t* s, uint64_t n, uint64_t& i) {  // unicode.cpp utf8_decode
  const uint8_t b0 = s[i];
  if (b0 < 0x80) {
    i += 1;
    return b0;
  }
  if ((b0 & 0xE0) == 0xC0 && i + 1 < n) {
    const uint32_t cp = ((b0 & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu);
    i += 2;
    return cp;
  }
  if ((b0 & 0xF0) == 0xE0 && i + 2 < n) {
    const uint32_t cp = ((b0 & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu);
    i += 3;
    return cp;
  }
  if ((b0 & 0xF8) == 0xF0 && i + 3 < n) {
    const uint32_t cp = ((b0 & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu);
    i += 4;
    return cp;
  }
  i += 1;
  return 0xFFFD;
}

__device__ inline bool is_ctl(uint8_t g) { return g == GCB_Control || g == GCB_CR || g == GCB_LF; }

// a code point after which the segmenter state is the initial state of its own properties
__device__ inline bool resync(const Props& p) {
  return p.g != GCB_RI && p.g != GCB_ZWJ && p.g != GCB_Extend && !p.pict && p.ib == INCB_None;
}

struct SegState {  // unicode.cpp segment_graphemes, the text ending at the left code point
  Props L;
  uint32_t ri_run;
  bool pict, gb11;
  int incb_state;
};

__device__ SegState seg_init(const Props& L) {
  return SegState{L, L.g == GCB_RI ? 1u : 0u, L.pict, false, L.ib == INCB_Consonant ? 1 : 0};
}

// boundary before code point R (GB3-GB999), then R becomes the left code point
__device__ bool seg_step(SegState& st, const Props& R) {
  const Props& L = st.L;
  // two plain code points (GCB Other, not Extended_Pictographic, no InCB: letters, digits, spaces,
  // most punctuation) -- no rule but GB999 applies, and the state resets; most of the text
  if (L.g == GCB_Other && R.g == GCB_Other && !L.pict && !R.pict && L.ib == INCB_None && R.ib == INCB_None) {
    st = SegState{R, 0u, false, false, 0};
    return true;
  }
  bool brk;
  if (L.g == GCB_CR && R.g == GCB_LF) brk = false;                                              // GB3
  else if (is_ctl(L.g)) brk = true;                                                             // GB4
  else if (is_ctl(R.g)) brk = true;                                                             // GB5
  else if (L.g == GCB_L && (R.g == GCB_L || R.g == GCB_V || R.g == GCB_LV || R.g == GCB_LVT)) brk = false;  // GB6
  else if ((L.g == GCB_LV || L.g == GCB_V) && (R.g == GCB_V || R.g == GCB_T)) brk = false;   // GB7
  else if ((L.g == GCB_LVT || L.g == GCB_T) && R.g == GCB_T) brk = false;                    // GB8
  else if (R.g == GCB_Extend || R.g == GCB_ZWJ) brk = false;                                   // GB9
  else if (R.g == GCB_SpacingMark) brk = false;                                                // GB9a
  else if (L.g == GCB_Prepend) brk = false;                                                    // GB9b
  else if (st.incb_state == 2 && R.ib == INCB_Consonant) brk = false;                          // GB9c
  else if (st.gb11 && R.pict) brk = false;                                                     // GB11
  else if (L.g == GCB_RI && R.g == GCB_RI && (st.ri_run & 1)) brk = false;                     // GB12/13
  else brk = true;                                                                             // GB999
  st.ri_run = R.g == GCB_RI ? st.ri_run + 1 : 0;
  st.gb11 = R.g == GCB_ZWJ && st.pict;
  st.pict = R.pict ? true : (R.g == GCB_Extend ? st.pict : false);
  if (R.ib == INCB_Consonant) st.incb_state = 1;
  else if (R.ib == INCB_Linker && st.incb_state >= 1) st.incb_state = 2;
  else if (R.ib == INCB_Extend && st.incb_state >= 1) { /* unchanged */ }
  else st.incb_state = 0;
  st.L = R;
  return brk;
}

__device__ uint32_t lower_first(uint32_t cp) {  // unicode.cpp lower_full, first code point
  if (cp < 0x80) return (cp >= 'A' && cp <= 'Z') ? cp + 32 : cp;
  uint32_t lo = 0, hi = sizeof(kLowerMap) / sizeof(kLowerMap[0]);
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (kLowerMap[mid].cp < cp) lo = mid + 1;
    else hi = mid;
  }
  return (lo < sizeof(kLowerMap) / sizeof(kLowerMap[0]) && kLowerMap[lo].cp == cp) ? kLowerMap[lo].out[0] : cp;
}

// ---- BMP property / lowercase tables (built once per device from the range tables above): one
// byte per code point (GCB | Extended_Pictographic << 4 | InCB << 5) and the first code point of its
// full lowercase (0 when it lies outside the BMP: the range search decides then)
__global__ void bmp_tables_kernel(uint8_t* ptab, uint16_t* ltab) {
  const uint32_t cp = blockIdx.x * blockDim.x + threadIdx.x;
  if (cp >= 0x10000u) return;
  const Props p = props(cp);
  ptab[cp] = (uint8_t)(p.g | (p.pict ? 16u : 0u) | ((uint32_t)p.ib << 5));
  const uint32_t l = lower_first(cp);
  ltab[cp] = l < 0x10000u ? (uint16_t)l : (uint16_t)0;
}

__device__ __forceinline__ Props props_fast(const uint8_t* __restrict__ ptab, uint32_t cp) {
  if (cp < 0x80u)
    return Props{(uint8_t)(cp == '\r' ? GCB_CR : cp == '\n' ? GCB_LF : (cp < 0x20u || cp == 0x7Fu) ? GCB_Control : GCB_Other),
                 INCB_None, false};
  if (cp < 0x10000u) {
    const uint32_t v = ptab[cp];
    return Props{(uint8_t)(v & 15u), (uint8_t)(v >> 5), (v & 16u) != 0};
  }
  return props(cp);
}

__device__ __forceinline__ uint32_t fold_fast(const uint16_t* __restrict__ ltab, uint32_t cp) {
  if (cp < 0x80u) return (cp - 'A' < 26u) ? cp + 32u : cp;
  if (cp < 0x10000u) {
    const uint32_t v = ltab[cp];
    if (v) return v;
  }
  return lower_first(cp);
}

constexpr uint32_t kPropLds = 0x800;  // code points whose property / lowercase bytes the staging kernels keep in LDS
__device__ __forceinline__ Props props_of(uint32_t v) { return Props{(uint8_t)(v & 15u), (uint8_t)(v >> 5), (v & 16u) != 0}; }

// Per 16 KiB tile (one workgroup, 64 bytes per thread, the tile staged in LDS): the C ABI's UTF-8
// check (unicode.cpp utf8_valid_serial = Rust's str::from_utf8) over the code points starting in the
// thread's bytes -- a segment runs from the first byte that is not a continuation byte to the next
// thread's, so every sequence lies in one segment and stray continuation bytes are caught -- fused
// with the UAX #29 boundary decisions of those code points (seg_step from the last resync code point
// before them, usually the previous one). Boundaries go out as one 64-bit mask per thread, the
// tile's grapheme count to ucnt. A thread without a resync point within kLookback marks its bytes
// hard (seg_hard_kernel). scal: [0] flags (bit 0 invalid, bit 1 a byte >= 0x80), [1] any hard.
constexpr uint32_t kTile = 16384;
__global__ __launch_bounds__(256) void seg_tile_kernel(const uint8_t* __restrict__ s, uint64_t n, int aligned,
                                                       const uint8_t* __restrict__ ptab, unsigned long long* __restrict__ bits,
                                                       uint32_t* __restrict__ ucnt, uint8_t* __restrict__ hard,
                                                       unsigned long long* __restrict__ scal, int skip_if_ascii) {
  if (skip_if_ascii && !(scal[0] & 2ull)) return;  // ascii_or_kernel found no byte >= 0x80
  // the tile, transposed: word w of thread t's 64 bytes at word w * 256 + t, so the threads' reads
  // of their own bytes (byte j of each, together) fall in 64 different banks; the row-major tile made
  // every such read a 32-way conflict (lanes 64 bytes apart)
  __shared__ __attribute__((aligned(16))) uint32_t tileT[kTile / 4];
  __shared__ uint8_t s_pt[kPropLds];  // ptab[0, kPropLds): Latin, Greek, Cyrillic, ... in LDS
  __shared__ uint32_t red[8];
  uint8_t* const tileB = reinterpret_cast<uint8_t*>(tileT);
  auto tix = [](uint32_t q) { return ((((q >> 2) & 15u) << 8 | (q >> 6)) << 2) | (q & 3u); };  // tile byte q -> LDS byte
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile, t1 = min(n, t0 + (uint64_t)kTile);
  for (uint32_t i = threadIdx.x; i < kPropLds; i += 256u) s_pt[i] = ptab[i];
  if (aligned && t1 - t0 == kTile) {
    for (uint32_t i = threadIdx.x * 16u; i < kTile; i += 256u * 16u) {
      const uint4 v = *reinterpret_cast<const uint4*>(s + t0 + i);
      const uint32_t tp = i >> 6, w0 = (i >> 2) & 15u;
      tileT[(w0 << 8) | tp] = v.x;
      tileT[((w0 + 1) << 8) | tp] = v.y;
      tileT[((w0 + 2) << 8) | tp] = v.z;
      tileT[((w0 + 3) << 8) | tp] = v.w;
    }
  } else {
    for (uint32_t i = threadIdx.x; i < kTile; i += 256u) tileB[tix(i)] = t0 + i < n ? s[t0 + i] : 0;
  }
  __syncthreads();
  auto at = [&](uint64_t p) -> uint32_t { return (p >= t0 && p < t1) ? tileB[tix((uint32_t)(p - t0))] : s[p]; };
  auto props_fast = [&](const uint8_t* tab, uint32_t cp) { return cp >= 0x80u && cp < kPropLds ? props_of(s_pt[cp]) : fac::props_fast(tab, cp); };
  auto cont = [&](uint64_t p) { return (at(p) & 0xC0u) == 0x80u; };
  auto dec = [&](uint64_t& i) -> uint32_t {  // unicode.cpp utf8_decode, bounded by n
    const uint32_t b0 = at(i);
    if (b0 < 0x80u) { i += 1; return b0; }
    if ((b0 & 0xE0u) == 0xC0u && i + 1 < n) { const uint32_t c = ((b0 & 0x1Fu) << 6) | (at(i + 1) & 0x3Fu); i += 2; return c; }
    if ((b0 & 0xF0u) == 0xE0u && i + 2 < n) {
      const uint32_t c = ((b0 & 0x0Fu) << 12) | ((at(i + 1) & 0x3Fu) << 6) | (at(i + 2) & 0x3Fu);
      i += 3;
      return c;
    }
    if ((b0 & 0xF8u) == 0xF0u && i + 3 < n) {
      const uint32_t c = ((b0 & 0x07u) << 18) | ((at(i + 1) & 0x3Fu) << 12) | ((at(i + 2) & 0x3Fu) << 6) | (at(i + 3) & 0x3Fu);
      i += 4;
      return c;
    }
    i += 1;
    return 0xFFFD;
  };
  auto seg_start = [&](uint64_t p, bool& bad) {  // first non-continuation byte at or after p
    uint32_t k = 0;
    while (p < n && cont(p) && k < 4) ++p, ++k;
    bad = p < n && cont(p);
    return p;
  };
  const uint64_t a = t0 + threadIdx.x * 64ull;
  unsigned long long mask = 0;
  bool bad = false, is_hard = false;
  uint32_t hi = 0;
  if (a < n) {
    const uint64_t b = min(a + 64, n);
#pragma unroll
    for (uint32_t w = 0; w < 16; ++w) hi |= tileT[(w << 8) | threadIdx.x];  // own bytes (0 past n)
    uint64_t i = seg_start(a, bad);
    if (a == 0 && i != 0) bad = true;
    bool bad2 = false;
    const uint64_t e = b < n ? seg_start(b, bad2) : n;
    SegState st{};
    if (!bad && i < e && i > 0) {  // the segmenter's state before the code point at i
      uint64_t q = i;
      bool found = false;
      while (q > 0 && i - q < kLookback) {
        do --q;
        while (q > 0 && cont(q));
        uint64_t t = q;
        if (resync(props_fast(ptab, dec(t)))) {
          found = true;
          break;
        }
      }
      if (!found && q > 0) {
        is_hard = true;
      } else {  // from the resync point (or the text's first code point) up to i
        uint64_t k = q;
        st = seg_init(props_fast(ptab, dec(k)));
        while (k < i) seg_step(st, props_fast(ptab, dec(k)));
      }
    }
    // the UTF-8 check covers every thread's code points, hard ones included (their boundaries are
    // decided by seg_hard_kernel, which decodes leniently and never flags a bad sequence)
    for (uint64_t k = i; !bad && k < e;) {
      const uint64_t pos = k;
      const uint32_t b0 = at(k);
      uint32_t cp;
      if (b0 < 0x80u) {
        cp = b0;
        k += 1;
      } else {
        uint32_t len, mn;
        if ((b0 & 0xE0u) == 0xC0u) len = 2, mn = 0x80;
        else if ((b0 & 0xF0u) == 0xE0u) len = 3, mn = 0x800;
        else if ((b0 & 0xF8u) == 0xF0u) len = 4, mn = 0x10000;
        else {
          bad = true;
          break;
        }
        if (k + len > e) {
          bad = true;
          break;
        }
        for (uint32_t c = 1; c < len; ++c) bad = bad || !cont(k + c);
        if (bad) break;
        cp = dec(k);
        if (cp < mn || cp > 0x10FFFFu || (cp >= 0xD800u && cp <= 0xDFFFu)) {
          bad = true;
          break;
        }
      }
      if (is_hard) continue;
      const Props R = props_fast(ptab, cp);
      bool br;
      if (pos == 0) {
        st = seg_init(R);
        br = true;
      } else {
        br = seg_step(st, R);
      }
      if (br) mask |= 1ull << (pos - a);
    }
    bits[a >> 6] = is_hard ? 0ull : mask;
    hard[a >> 6] = is_hard ? 1 : 0;
  }
  uint32_t c = (uint32_t)__popcll(mask);
  uint32_t f = (bad ? 1u : 0u) | ((hi & 0x80808080u) ? 2u : 0u) | (is_hard ? 4u : 0u);
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_down(c, o, 64);
    f |= (uint32_t)__shfl_down((int)f, o, 64);
  }
  if ((threadIdx.x & 63u) == 0) {
    red[threadIdx.x >> 6] = c;
    red[4 + (threadIdx.x >> 6)] = f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ucnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
    const uint32_t ff = red[4] | red[5] | red[6] | red[7];
    if (ff & 3u) atomicOr(scal, (unsigned long long)(ff & 3u));
    if (ff & 4u) atomicOr(scal + 1, 1ull);
  }
}

// search.rs:196's is_ascii on the device: bit 1 of scal[0] when some byte is >= 0x80
__global__ __launch_bounds__(256) void ascii_or_kernel(const uint8_t* __restrict__ s, uint64_t n, int aligned,
                                                       unsigned long long* scal) {
  uint32_t hi = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t nv = aligned ? n / 16 : 0;
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const uint4 w = reinterpret_cast<const uint4*>(s)[v];
    hi |= w.x | w.y | w.z | w.w;
  }
  for (uint64_t p = nv * 16 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += stride) hi |= s[p];
  if (__ballot((hi & 0x80808080u) != 0) && (threadIdx.x & 63u) == 0) atomicOr(scal, 2ull);
}

// Threads without a resync code point within kLookback (long emoji / RI / combining runs): one
// thread walks each maximal run of such 64-byte ranges once, from the run's own (unbounded) resync
// point -- linear in the text overall. Then every tile is recounted.
__global__ void seg_hard_kernel(const uint8_t* s, uint64_t n, const uint8_t* ptab, const uint8_t* hard, uint64_t ranges,
                                unsigned long long* bits, const unsigned long long* scal) {
  if (blockIdx.x != 0 || threadIdx.x != 0 || !scal[1]) return;
  for (uint64_t c = 0; c < ranges; ++c) {
    if (!hard[c]) continue;
    uint64_t r = c;
    while (r + 1 < ranges && hard[r + 1]) ++r;
    const uint64_t a = c * 64, b = min((r + 1) * 64, n);
    uint64_t q = a;
    while (q > 0) {
      do --q;
      while (q > 0 && (s[q] & 0xC0) == 0x80);
      uint64_t t = q;
      if (resync(props_fast(ptab, decode(s, n, t)))) break;
    }
    uint64_t i = q;
    SegState st = seg_init(props_fast(ptab, decode(s, n, i)));
    for (uint64_t w = c; w <= r; ++w) bits[w] = 0;
    while (i < b) {
      const uint64_t pos = i;
      const bool br = seg_step(st, props_fast(ptab, decode(s, n, i)));
      if (pos >= a && br) bits[pos >> 6] |= 1ull << (pos & 63);
    }
    c = r;
  }
}
__global__ __launch_bounds__(256) void recount_kernel(const unsigned long long* bits, uint64_t ranges, uint32_t* ucnt,
                                                      uint64_t n_units, const unsigned long long* scal) {
  if (!scal[1]) return;
  const uint64_t u = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const uint32_t lane = threadIdx.x & 63u;
  if (u >= n_units) return;
  uint32_t c = 0;
  for (uint64_t w = u * (kTile / 64) + lane; w < min(ranges, (u + 1) * (kTile / 64)); w += 64) c += __popcll(bits[w]);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if (lane == 0) ucnt[u] = c;
}

__global__ __launch_bounds__(1024) void unit_scan_kernel(const uint32_t* ucnt, uint64_t* ubase, uint64_t n_units,
                                                         unsigned long long* total) {
  __shared__ unsigned long long wsum[16];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t per = (n_units + 1023) / 1024;
  const uint64_t a = min(n_units, (uint64_t)t * per), b = min(n_units, a + per);
  unsigned long long sum = 0;
  for (uint64_t i = a; i < b; ++i) sum += ucnt[i];
  unsigned long long x = sum;  // inclusive scan over the wave
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (t == 0) {
    unsigned long long run = 0;
    for (int i = 0; i < 16; ++i) {
      const unsigned long long v = wsum[i];
      wsum[i] = run;
      run += v;
    }
    *total = run;
  }
  __syncthreads();
  unsigned long long run = wsum[w] + x - sum;
  for (uint64_t i = a; i < b; ++i) {
    ubase[i] = run;
    run += ucnt[i];
  }
}

// Grapheme starts (h.d_off) and text_chars (h.d_text32: the folded first code point per grapheme,
// search.rs:406-412, grapheme.rs:112-119), one wave per tile in byte order: four boundary bits per
// lane per step, a wave scan gives each start its slot, so consecutive lanes write consecutive slots.
// A lane reads its 4 bytes and the next 4 as two words with its boundary word (one round trip per
// step: every code point starting in its 4 bytes decodes from those 8), and folds through an LDS copy
// of ltab below kPropLds (was: a dependent byte load per continuation byte and a global ltab load).
__global__ __launch_bounds__(256) void write_tile_kernel(const uint8_t* __restrict__ s, uint64_t n, int aligned,
                                                         const unsigned long long* __restrict__ bits,
                                                         const uint64_t* __restrict__ ubase, uint64_t n_units,
                                                         const uint16_t* __restrict__ ltab, int ci, uint64_t* __restrict__ off,
                                                         uint32_t* __restrict__ text32) {
  __shared__ uint16_t s_lt[kPropLds];
  __shared__ uint64_t s_off[4][256];  // a step's grapheme starts and chars, written out coalesced
  __shared__ uint32_t s_tx[4][256];
  if (ci)
    for (uint32_t i = threadIdx.x; i < kPropLds; i += blockDim.x) s_lt[i] = ltab[i];
  __syncthreads();
  uint64_t* const w_off = s_off[threadIdx.x / 64];
  uint32_t* const w_tx = s_tx[threadIdx.x / 64];
  const uint64_t u = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const uint32_t lane = threadIdx.x & 63u;
  if (u >= n_units) return;  // whole waves
  uint64_t base = ubase[u];
  const uint64_t b = u * kTile, e = min(n, b + (uint64_t)kTile);
  for (uint64_t p0 = b; p0 < e; p0 += 256) {
    const uint64_t p = p0 + 4ull * lane;
    uint32_t f = 0, wa = 0, wb = 0;
    if (p < e) {
      f = (uint32_t)(bits[p >> 6] >> (p & 63)) & 0xFu;
      if (p + 4 > e) f &= (1u << (uint32_t)(e - p)) - 1u;
      if (aligned && p + 8 <= n) {
        wa = *reinterpret_cast<const uint32_t*>(s + p);
        wb = *reinterpret_cast<const uint32_t*>(s + p + 4);
      } else {
        for (uint32_t q = 0; q < 8; ++q)
          if (p + q < n) (q < 4 ? wa : wb) |= (uint32_t)s[p + q] << (8 * (q & 3u));
      }
    }
    const uint32_t c = __popc(f);
    uint32_t x = c;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    uint32_t o = x - c;  // the grapheme's slot in this step
    const uint64_t w8 = (uint64_t)wa | ((uint64_t)wb << 32);
    for (uint32_t k = 0; k < 4; ++k)
      if ((f >> k) & 1u) {
        const uint64_t i = p + k;
        auto at = [&](uint32_t d) { return (uint32_t)(w8 >> (8 * (k + d))) & 0xFFu; };  // byte i + d (d <= 3)
        const uint32_t b0 = at(0);
        uint32_t cp;  // decode(s, n, i) on the registers
        if (b0 < 0x80u) cp = b0;
        else if ((b0 & 0xE0u) == 0xC0u && i + 1 < n) cp = ((b0 & 0x1Fu) << 6) | (at(1) & 0x3Fu);
        else if ((b0 & 0xF0u) == 0xE0u && i + 2 < n) cp = ((b0 & 0x0Fu) << 12) | ((at(1) & 0x3Fu) << 6) | (at(2) & 0x3Fu);
        else if ((b0 & 0xF8u) == 0xF0u && i + 3 < n)
          cp = ((b0 & 0x07u) << 18) | ((at(1) & 0x3Fu) << 12) | ((at(2) & 0x3Fu) << 6) | (at(3) & 0x3Fu);
        else cp = 0xFFFD;
        uint32_t fc = cp;
        if (ci) fc = cp >= 0x80u && cp < kPropLds && s_lt[cp] ? (uint32_t)s_lt[cp] : fold_fast(ltab, cp);
        w_off[o] = i;
        w_tx[o] = fc;
        ++o;
      }
    const uint32_t tot = __shfl(x, 63, 64);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t q = lane; q < tot; q += 64) {
      off[base + q] = w_off[q];
      text32[base + q] = w_tx[q];
    }
    __builtin_amdgcn_wave_barrier();
    base += tot;
  }
}

}  // namespace

#define ST_TRY(x)                                         \
  do {                                                    \
    hipError_t _e = (x);                                  \
    if (_e != hipSuccess) {                               \
      err = std::string(#x ": ") + hipGetErrorString(_e); \
      return FAC_E_HIP;                                   \
    }                                                     \
  } while (0)

namespace {
struct BmpTabs {
  uint8_t* p = nullptr;
  uint16_t* l = nullptr;
};
// the BMP tables of `device`, built on first use (kept for the process)
int bmp_tables(int device, hipStream_t st, BmpTabs& out, std::string& err) {
  static std::mutex mu;
  static BmpTabs tabs[64];
  if (device < 0 || device >= 64) {
    err = "device ordinal out of range";
    return FAC_E_INVALID;
  }
  std::lock_guard<std::mutex> lk(mu);
  BmpTabs& t = tabs[device];
  if (!t.p) {
    ST_TRY(hipMalloc((void**)&t.p, 0x10000));
    ST_TRY(hipMalloc((void**)&t.l, 0x10000 * sizeof(uint16_t)));
    hipLaunchKernelGGL(bmp_tables_kernel, dim3(256), dim3(256), 0, st, t.p, t.l);
    ST_TRY(hipGetLastError());
    ST_TRY(hipStreamSynchronize(st));
  }
  out = t;
  return FAC_OK;
}
}  // namespace

// Device staging of a haystack whose bytes are resident at h.d_utf8 (search.rs:196-203, 296-302):
// mode -2 checks the UTF-8 and decides is_ascii on the device, 0 stages Unicode graphemes (the caller
// checked the bytes / decided is_ascii for the whole text), 1 is an ASCII haystack (nothing to do).
// Unicode: h.n, h.d_off (grapheme byte starts + off[n] = len) and h.d_text32 (folded first code
// points); the scratch and the grapheme arrays are kept in h and reused when it is staged again.
int stage_device(const Engine& e, Haystack& h, hipStream_t st, std::string& err, int mode) {
  const uint64_t len = h.len;
  if (mode == 1 || len == 0) {
    h.ascii = mode != 0;
    h.n = h.ascii ? len : 0;
    if (!h.ascii) {
      if (h.off_cap < 1) {
        if (h.d_off) ST_TRY(hipFree(h.d_off));
        h.d_off = nullptr;
        ST_TRY(hipMalloc((void**)&h.d_off, 16));
        if (h.d_text32) ST_TRY(hipFree(h.d_text32));
        h.d_text32 = nullptr;
        ST_TRY(hipMalloc((void**)&h.d_text32, 16));
        h.off_cap = 1;
      }
      ST_TRY(hipMemcpyAsync(h.d_off, &h.len, 8, hipMemcpyHostToDevice, st));
    }
    return FAC_OK;
  }
  BmpTabs tabs;
  if (int trc = bmp_tables(h.device, st, tabs, err)) return trc;
  const uint64_t ranges = (len + 63) / 64, n_units = (len + kTile - 1) / kTile;
  // scratch: scal[4] | bits[ranges] | ubase[n_units] | ucnt[n_units] | hard[ranges]
  const size_t need = 32 + ranges * 8 + n_units * 8 + n_units * 4 + ranges + 16;
  if (h.stage_cap < need) {
    if (h.d_stage) ST_TRY(hipFree(h.d_stage));
    h.d_stage = nullptr;
    h.stage_cap = 0;
    ST_TRY(hipMalloc(&h.d_stage, need));
    h.stage_cap = need;
  }
  unsigned long long* scal = static_cast<unsigned long long*>(h.d_stage);
  unsigned long long* bits = scal + 4;
  uint64_t* ubase = reinterpret_cast<uint64_t*>(bits + ranges);
  uint32_t* ucnt = reinterpret_cast<uint32_t*>(ubase + n_units);
  uint8_t* hard = reinterpret_cast<uint8_t*>(ucnt + n_units);
  const int aligned = (reinterpret_cast<uintptr_t>(h.d_utf8) & 15u) == 0 ? 1 : 0;
  ST_TRY(hipMemsetAsync(scal, 0, 32, st));
  if (mode == -2) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h.device);
    const uint64_t want = (len / 16 + 255) / 256;
    hipLaunchKernelGGL(ascii_or_kernel, dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cus * 8))),
                       dim3(256), 0, st, h.d_utf8, len, aligned, scal);
    ST_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(seg_tile_kernel, dim3((uint32_t)n_units), dim3(256), 0, st, h.d_utf8, len, aligned, tabs.p, bits,
                     ucnt, hard, scal, mode == -2 ? 1 : 0);
  hipLaunchKernelGGL(seg_hard_kernel, dim3(1), dim3(64), 0, st, h.d_utf8, len, tabs.p, hard, ranges, bits, scal);
  hipLaunchKernelGGL(recount_kernel, dim3((uint32_t)((n_units + 3) / 4)), dim3(256), 0, st, bits, ranges, ucnt, n_units,
                     scal);
  hipLaunchKernelGGL(unit_scan_kernel, dim3(1), dim3(1024), 0, st, ucnt, ubase, n_units, scal + 2);
  ST_TRY(hipGetLastError());
  unsigned long long sc[4] = {0, 0, 0, 0};
  ST_TRY(hipMemcpyAsync(sc, scal, sizeof(sc), hipMemcpyDeviceToHost, st));
  ST_TRY(hipStreamSynchronize(st));
  if (sc[0] & 1ull) {  // seg_tile_kernel checks every code point (modes -2 and 0)
    err = "haystack is not valid UTF-8";
    return FAC_E_INVALID;
  }
  if (mode == -2) {
    h.ascii = !(sc[0] & 2ull);
    if (h.ascii) {
      h.n = len;
      return FAC_OK;
    }
  }
  h.ascii = false;
  h.n = sc[2];
  if (h.n > grapheme_limit()) return FAC_E_HAYSTACK_TOO_LARGE;
  if (h.off_cap < h.n + 1) {  // grapheme starts + off[n] = len (a shard's halo end), folded first chars
    if (h.d_off) ST_TRY(hipFree(h.d_off));
    if (h.d_text32) ST_TRY(hipFree(h.d_text32));
    h.d_off = nullptr;
    h.d_text32 = nullptr;
    h.off_cap = 0;
    ST_TRY(hipMalloc((void**)&h.d_off, (h.n + 1) * 8));
    ST_TRY(hipMalloc((void**)&h.d_text32, std::max<uint64_t>(h.n * 4, 16)));
    h.off_cap = h.n + 1;
  }
  ST_TRY(hipMemcpyAsync(h.d_off + h.n, &h.len, 8, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(write_tile_kernel, dim3((uint32_t)((n_units + 3) / 4)), dim3(256), 0, st, h.d_utf8, len, aligned, bits, ubase,
                     n_units, tabs.l, e.case_insensitive ? 1 : 0, h.d_off, h.d_text32);
  ST_TRY(hipGetLastError());
  return FAC_OK;
}

// graphemes starting before byte `b` (a grapheme boundary) of a staged Unicode haystack: lower_bound
// over the device grapheme starts, one thread
__global__ void starts_before_kernel(const uint64_t* off, uint64_t n, uint64_t b, unsigned long long* out) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (off[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  *out = lo;
}

int graphemes_before(const Haystack& h, uint64_t b, hipStream_t st, uint64_t& out, std::string& err) {
  // an empty (e.g. the last, empty shard of a short text) or unstaged haystack: stage_device returned
  // before allocating d_stage, and no grapheme starts before any byte
  if (h.ascii || h.n == 0 || !h.d_stage) {
    out = std::min(b, h.n);
    return FAC_OK;
  }
  unsigned long long* d = static_cast<unsigned long long*>(h.d_stage);  // scal[3]: free after staging
  hipLaunchKernelGGL(starts_before_kernel, dim3(1), dim3(1), 0, st, h.d_off, h.n, b, d + 3);
  ST_TRY(hipGetLastError());
  unsigned long long v = 0;
  ST_TRY(hipMemcpyAsync(&v, d + 3, 8, hipMemcpyDeviceToHost, st));
  ST_TRY(hipStreamSynchronize(st));
  out = v;
  return FAC_OK;
}

}  // namespace fac
