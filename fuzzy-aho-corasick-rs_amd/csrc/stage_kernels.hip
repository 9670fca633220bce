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

constexpr uint32_t kChunk = 256;       // bytes decided per thread
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

// decide the boundaries at code point starts in [a, b), starting from code point q (q <= a)
__device__ void seg_range(const uint8_t* s, uint64_t n, uint64_t q, uint64_t a, uint64_t b, uint8_t* brk) {
  uint64_t i = q;
  SegState st = seg_init(props(decode(s, n, i)));
  if (q == 0 && a == 0) brk[0] = 1;
  while (i < b) {
    const uint64_t pos = i;
    const Props R = props(decode(s, n, i));
    const bool br = seg_step(st, R);
    if (pos >= a) brk[pos] = br ? 1 : 0;
  }
}

__global__ void seg_chunk_kernel(const uint8_t* s, uint64_t n, uint8_t* brk, uint8_t* hard, unsigned int* any_hard) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t a = c * kChunk;
  if (a >= n) return;
  const uint64_t b = min(a + kChunk, n);
  if (a == 0) {
    seg_range(s, n, 0, 0, b, brk);
    return;
  }
  // latest resync code point strictly before a (code point starts only)
  uint64_t q = a;
  bool found = false;
  while (q > 0 && a - q < kLookback) {
    do --q;
    while (q > 0 && (s[q] & 0xC0) == 0x80);
    uint64_t t = q;
    if (resync(props(decode(s, n, t)))) {
      found = true;
      break;
    }
  }
  if (!found && q > 0) {
    hard[c] = 1;
    atomicOr(any_hard, 1u);
    return;
  }
  seg_range(s, n, q, a, b, brk);  // q == 0: the text's own initial state
}

// Chunks with no resync code point within kLookback: one thread walks each maximal run of such
// chunks once, from the run's own (unbounded) resync point — linear in the text overall.
__global__ void seg_hard_kernel(const uint8_t* s, uint64_t n, const uint8_t* hard, uint64_t chunks, uint8_t* brk) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (uint64_t c = 0; c < chunks; ++c) {
    if (!hard[c]) continue;
    uint64_t e = c;
    while (e + 1 < chunks && hard[e + 1]) ++e;
    const uint64_t a = c * kChunk, b = min((e + 1) * kChunk, n);
    uint64_t q = a;
    while (q > 0) {
      do --q;
      while (q > 0 && (s[q] & 0xC0) == 0x80);
      uint64_t t = q;
      if (resync(props(decode(s, n, t)))) break;
    }
    seg_range(s, n, q, a, b, brk);
    c = e;
  }
}

// The C ABI's UTF-8 check (search_raw takes a &str, always valid) and search.rs:196's is_ascii, on
// the device: unicode.cpp's utf8_valid_serial (Rust's str::from_utf8 acceptance: no overlongs,
// surrogates or code points past U+10FFFF) per 16-byte chunk, over the segment from the chunk's first
// byte that is not a continuation byte to the next chunk's -- every sequence then lies in one segment;
// four continuation bytes in a row leave no start, and text must not begin with one. flags: bit 0
// invalid, bit 1 some byte >= 0x80. 16-byte chunks keep a wave's reads inside 1 KiB (256-byte ones
// spread each byte load over 128 lines: 48 GB fetched for 256 MiB).
constexpr uint32_t kValChunk = 16;
__global__ __launch_bounds__(256) void validate_kernel(const uint8_t* s, uint64_t n, unsigned int* flags) {
  const uint64_t c0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kValChunk;
  if (c0 >= n) return;
  auto cont = [&](uint64_t p) { return (s[p] & 0xC0) == 0x80; };
  auto seg_start = [&](uint64_t p, bool& bad) {  // first non-continuation byte at or after p
    uint32_t k = 0;
    while (p < n && cont(p) && k < 4) ++p, ++k;
    bad = p < n && cont(p);
    return p;
  };
  bool bad = false, bad2 = false;
  uint64_t i = seg_start(c0, bad);
  if (c0 == 0 && i != 0) bad = true;
  const uint64_t e = c0 + kValChunk < n ? seg_start(c0 + kValChunk, bad2) : n;
  uint32_t hi = 0;
  for (uint64_t p = c0; p < min(n, c0 + kValChunk); ++p) hi |= s[p];
  while (!bad && i < e) {
    const uint8_t b = s[i];
    if (b < 0x80) {
      ++i;
      continue;
    }
    uint32_t len, mn;
    if ((b & 0xE0) == 0xC0) len = 2, mn = 0x80;
    else if ((b & 0xF0) == 0xE0) len = 3, mn = 0x800;
    else if ((b & 0xF8) == 0xF0) len = 4, mn = 0x10000;
    else {
      bad = true;
      break;
    }
    if (i + len > e) {
      bad = true;
      break;
    }
    for (uint32_t k = 1; k < len; ++k)
      if (!cont(i + k)) bad = true;
    if (bad) break;
    uint64_t j = i;
    const uint32_t cp = decode(s, n, j);
    if (cp < mn || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) bad = true;
    i += len;
  }
  const unsigned f = (bad ? 1u : 0u) | ((hi & 0x80u) ? 2u : 0u);
  if (f) atomicOr(flags, f);
}

// Grapheme-start compaction (brk bytes are 0/1): unit u = bytes [u * kUnit, (u + 1) * kUnit), one
// wave each. unit_count_kernel counts, unit_scan_kernel (one workgroup) turns the counts into each
// unit's first output slot and the total, unit_write_kernel writes the positions in order.
constexpr uint32_t kUnit = 16384;
__global__ __launch_bounds__(256) void unit_count_kernel(const uint8_t* brk, uint64_t n, uint32_t* ucnt, uint64_t n_units) {
  const uint64_t u = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const uint32_t lane = threadIdx.x & 63;
  if (u >= n_units) return;  // whole waves
  const uint64_t b = u * kUnit, e = min(n, b + (uint64_t)kUnit);
  uint32_t c = 0;
  if (e - b == kUnit) {  // 16-byte aligned (b is a multiple of kUnit, hipMalloc'd base)
    const uint4* p = reinterpret_cast<const uint4*>(brk + b);
    for (uint32_t i = lane; i < kUnit / 16; i += 64) {
      const uint4 v = p[i];
      c += __popc(v.x & 0x01010101u) + __popc(v.y & 0x01010101u) + __popc(v.z & 0x01010101u) + __popc(v.w & 0x01010101u);
    }
  } else {
    for (uint64_t i = b + lane; i < e; i += 64) c += brk[i];
  }
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
__global__ __launch_bounds__(256) void unit_write_kernel(const uint8_t* brk, uint64_t n, const uint64_t* ubase, uint64_t n_units,
                                                         uint64_t* off) {
  const uint64_t u = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const uint32_t lane = threadIdx.x & 63;
  if (u >= n_units) return;  // whole waves
  uint64_t base = ubase[u];
  const uint64_t b = u * kUnit, e = min(n, b + (uint64_t)kUnit);
  for (uint64_t p0 = b; p0 < e; p0 += 256) {  // four flags per lane, in byte order across the wave
    const uint64_t p = p0 + 4ull * lane;
    uint32_t f = 0;
    if (p + 4 <= e) {
      f = *reinterpret_cast<const uint32_t*>(brk + p) & 0x01010101u;
    } else {
      for (uint32_t k = 0; k < 4; ++k)
        if (p + k < e && brk[p + k]) f |= 1u << (8 * k);
    }
    const uint32_t c = __popc(f);
    uint32_t x = c;  // inclusive scan of the lanes' counts
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    uint64_t o = base + x - c;
    for (uint32_t k = 0; k < 4; ++k)
      if ((f >> (8 * k)) & 1u) off[o++] = p + k;
    base += __shfl(x, 63, 64);
  }
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

// text_chars[g]: the folded first code point of grapheme g (search.rs:406-412, grapheme.rs:112-119)
__global__ void fold_kernel(const uint8_t* s, uint64_t len, const uint64_t* off, uint64_t ng, int ci, uint32_t* text32) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  uint64_t i = off[g];
  const uint64_t e = g + 1 < ng ? off[g + 1] : len;
  const uint32_t cp = decode(s, e, i);
  text32[g] = ci ? lower_first(cp) : cp;
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

// flags of validate_kernel over the device copy of a haystack (synchronous): bit 0 invalid UTF-8,
// bit 1 not ASCII
int validate_device(const uint8_t* d_utf8, uint64_t len, hipStream_t st, unsigned int& flags_out, std::string& err) {
  flags_out = 0;
  if (!len) return FAC_OK;
  unsigned int* flags = nullptr;
  ST_TRY(hipMalloc((void**)&flags, 4));
  struct Free {
    void* p;
    ~Free() {
      if (p) (void)hipFree(p);
    }
  } f_flags{flags};
  ST_TRY(hipMemsetAsync(flags, 0, 4, st));
  const uint64_t chunks = (len + kValChunk - 1) / kValChunk;
  hipLaunchKernelGGL(validate_kernel, dim3((uint32_t)((chunks + 255) / 256)), dim3(256), 0, st, d_utf8, len, flags);
  ST_TRY(hipGetLastError());
  ST_TRY(hipMemcpyAsync(&flags_out, flags, 4, hipMemcpyDeviceToHost, st));
  ST_TRY(hipStreamSynchronize(st));
  return FAC_OK;
}

// Device staging of a valid, non-ASCII UTF-8 haystack already resident at h.d_utf8: fills
// h.n, h.d_off (grapheme byte starts), h.d_text32 (folded first code points) and the host copy of
// the starts (fetched to the host only on demand: ensure_host).
int stage_unicode_device(const Engine& e, Haystack& h, hipStream_t st, std::string& err) {
  const uint64_t len = h.len;
  uint8_t* brk = nullptr;
  ST_TRY(hipMalloc((void**)&brk, std::max<uint64_t>(len, 16)));
  struct Free {
    void* p;
    ~Free() {
      if (p) (void)hipFree(p);
    }
  } f_brk{brk};
  const uint64_t chunks = (len + kChunk - 1) / kChunk;
  uint8_t* hard = nullptr;
  ST_TRY(hipMalloc((void**)&hard, std::max<uint64_t>(chunks, 16)));
  Free f_hard{hard};
  unsigned long long* scal = nullptr;  // [0] any hard chunk, [1] grapheme count
  ST_TRY(hipMalloc((void**)&scal, 16));
  Free f_scal{scal};
  ST_TRY(hipMemsetAsync(brk, 0, len, st));
  ST_TRY(hipMemsetAsync(hard, 0, chunks, st));
  ST_TRY(hipMemsetAsync(scal, 0, 16, st));
  hipLaunchKernelGGL(seg_chunk_kernel, dim3((uint32_t)((chunks + 255) / 256)), dim3(256), 0, st, h.d_utf8, len, brk,
                     hard, reinterpret_cast<unsigned int*>(scal));
  ST_TRY(hipGetLastError());
  unsigned long long scal_h[2] = {0, 0};
  ST_TRY(hipMemcpyAsync(scal_h, scal, 8, hipMemcpyDeviceToHost, st));
  ST_TRY(hipStreamSynchronize(st));
  if (scal_h[0]) {
    hipLaunchKernelGGL(seg_hard_kernel, dim3(1), dim3(64), 0, st, h.d_utf8, len, hard, chunks, brk);
    ST_TRY(hipGetLastError());
  }
  const uint64_t n_units = (len + kUnit - 1) / kUnit;
  uint32_t* ucnt = nullptr;
  uint64_t* ubase = nullptr;
  ST_TRY(hipMalloc((void**)&ucnt, std::max<uint64_t>(n_units, 1) * 4));
  Free f_ucnt{ucnt};
  ST_TRY(hipMalloc((void**)&ubase, std::max<uint64_t>(n_units, 1) * 8));
  Free f_ubase{ubase};
  const uint32_t ugrid = (uint32_t)((n_units + 3) / 4);
  if (n_units) {
    hipLaunchKernelGGL(unit_count_kernel, dim3(ugrid), dim3(256), 0, st, brk, len, ucnt, n_units);
    hipLaunchKernelGGL(unit_scan_kernel, dim3(1), dim3(1024), 0, st, ucnt, ubase, n_units, scal + 1);
    ST_TRY(hipGetLastError());
  }
  ST_TRY(hipMemcpyAsync(scal_h + 1, scal + 1, 8, hipMemcpyDeviceToHost, st));
  ST_TRY(hipStreamSynchronize(st));
  h.n = scal_h[1];
  if (h.n > grapheme_limit()) return FAC_E_HAYSTACK_TOO_LARGE;
  // grapheme starts = positions with brk set, plus off[n] = len (a shard's halo end: an emission
  // at j == n of an open-ended shard reads it before the halo check flags the window)
  ST_TRY(hipMalloc((void**)&h.d_off, (h.n + 1) * 8));
  ST_TRY(hipMemcpyAsync(h.d_off + h.n, &h.len, 8, hipMemcpyHostToDevice, st));
  if (n_units) {
    hipLaunchKernelGGL(unit_write_kernel, dim3(ugrid), dim3(256), 0, st, brk, len, ubase, n_units, h.d_off);
    ST_TRY(hipGetLastError());
  }
  ST_TRY(hipMalloc((void**)&h.d_text32, std::max<uint64_t>(h.n * 4, 16)));
  if (h.n) {
    hipLaunchKernelGGL(fold_kernel, dim3((uint32_t)((h.n + 255) / 256)), dim3(256), 0, st, h.d_utf8, len, h.d_off, h.n,
                       e.case_insensitive ? 1 : 0, h.d_text32);
    ST_TRY(hipGetLastError());
  }
  ST_TRY(hipStreamSynchronize(st));
  return FAC_OK;
}

}  // namespace fac
