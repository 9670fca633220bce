// api.cpp — the extern "C" boundary declared in include/fac.h.
//
// fac_search_raw is the drop-in for FuzzyAhoCorasick::search_raw (src/search.rs:187-395):
// host staging (is_ascii + grapheme segmentation/folding, :196-203 / :296-302), then the GPU
// window kernel over every start position. fac_search_prefiltered is the drop-in for
// Prefiltered::raw (src/prefilter.rs:146-155, 304-374): k_for on the host, the bitap scan and the
// window merge on the GPU, then the window kernel over the merged slices. There is no CPU search
// path: without a usable gfx950 device every search entry point returns FAC_E_NO_DEVICE.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <tuple>

#include "fac_internal.h"

struct fac_engine {
  fac::Engine e;
};
struct fac_haystack {
  fac::Haystack h;
};
struct fac_stream {
  fac::StreamCore* s = nullptr;
};

namespace fac {

const char* diag_env(const char* name) {
  static const bool on = [] {
    const char* d = std::getenv("FAC_DIAGNOSTICS");
    return d && *d && std::strcmp(d, "0") != 0;
  }();
  return on ? std::getenv(name) : nullptr;
}

uint64_t grapheme_limit() {
  const char* v = diag_env("FAC_GRAPHEME_LIMIT");
  return v ? std::strtoull(v, nullptr, 10) : 0xFFFFFFFFull;
}

namespace {
// Result buffers handed across the C ABI. A search's records are copied D2H straight into the
// buffer the caller receives; buffers of >= 1 MiB are pinned and go back to this pool on
// fac_matches_free, so repeated searches land their records in already-mapped, already-pinned
// pages (a fresh malloc'd buffer faults every page on first touch: C2's 72 MB of records per call
// cost 20-40 ms of page faults, varying by box).
struct PoolBlock {
  void* p;
  uint64_t bytes;
  bool used;
};
std::mutex g_pool_mu;
std::vector<PoolBlock> g_pool;
constexpr uint64_t kPinnedMin = 1ull << 20;
constexpr uint64_t kPoolKeep = 4ull << 30;  // pinned bytes kept while unused
}  // namespace

fac_match* result_alloc(uint64_t n_records) {
  const uint64_t bytes = std::max<uint64_t>(n_records, 1) * sizeof(fac_match);
  if (bytes < kPinnedMin) return static_cast<fac_match*>(std::malloc(bytes));
  std::lock_guard<std::mutex> g(g_pool_mu);
  PoolBlock* best = nullptr;
  for (PoolBlock& b : g_pool)
    if (!b.used && b.bytes >= bytes && b.bytes <= 4 * bytes && (!best || b.bytes < best->bytes)) best = &b;
  if (best) {
    best->used = true;
    return static_cast<fac_match*>(best->p);
  }
  const uint64_t want = bytes + bytes / 4;  // headroom: the next call's count differs a little
  void* p = nullptr;
  if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess || !p)
    return static_cast<fac_match*>(std::malloc(bytes));  // unpinned: result_free recognises it
  g_pool.push_back({p, want, true});
  return static_cast<fac_match*>(p);
}

void result_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    for (size_t i = 0; i < g_pool.size(); ++i)
      if (g_pool[i].p == p) {
        g_pool[i].used = false;
        uint64_t idle = 0;
        for (const PoolBlock& b : g_pool)
          if (!b.used) idle += b.bytes;
        // trim the largest idle blocks beyond the keep budget
        while (idle > kPoolKeep) {
          size_t big = g_pool.size();
          for (size_t k = 0; k < g_pool.size(); ++k)
            if (!g_pool[k].used && (big == g_pool.size() || g_pool[k].bytes > g_pool[big].bytes)) big = k;
          if (big == g_pool.size()) break;
          (void)hipHostFree(g_pool[big].p);
          idle -= g_pool[big].bytes;
          g_pool.erase(g_pool.begin() + (std::ptrdiff_t)big);
        }
        return;
      }
  }
  std::free(p);
}

namespace {
int grow_pinned(MatchSink& s, uint64_t need, std::string& err) {
  if (need <= s.pinned_cap) return FAC_OK;
  const uint64_t cap = std::max<uint64_t>(need, 2 * s.pinned_cap);
  fac_match* p = result_alloc(cap);
  if (!p) {
    err = "out of host memory";
    return FAC_E_OOM;
  }
  if (s.n) std::memcpy(p, s.pinned, s.n * sizeof(fac_match));
  result_free(s.pinned);
  s.pinned = p;
  s.pinned_cap = cap;
  return FAC_OK;
}
}  // namespace

int sink_append_device(MatchSink& s, const fac_match* d_src, uint64_t cnt, hipStream_t stream, std::string& err) {
  if (!cnt) return FAC_OK;
  hipError_t he = hipSuccess;
  if (s.dev) {
    const uint64_t fit = s.n >= s.dev_cap ? 0 : std::min(cnt, s.dev_cap - s.n);
    if (fit) he = hipMemcpyAsync(s.dev + s.n, d_src, fit * sizeof(fac_match), hipMemcpyDeviceToDevice, stream);
  } else if (s.vec) {
    s.vec->resize(s.n + cnt);
    he = hipMemcpyAsync(s.vec->data() + s.n, d_src, cnt * sizeof(fac_match), hipMemcpyDeviceToHost, stream);
    if (he == hipSuccess) he = hipStreamSynchronize(stream);  // pageable destination
  } else {
    if (int rc = grow_pinned(s, s.n + cnt, err)) return rc;
    he = hipMemcpyAsync(s.pinned + s.n, d_src, cnt * sizeof(fac_match), hipMemcpyDeviceToHost, stream);
  }
  if (he != hipSuccess) {
    err = std::string("record copy: ") + hipGetErrorString(he);
    return FAC_E_HIP;
  }
  s.n += cnt;
  return FAC_OK;
}

int sink_append_host(MatchSink& s, const fac_match* src, uint64_t cnt, hipStream_t stream, std::string& err) {
  if (!cnt) return FAC_OK;
  if (s.dev) {
    const uint64_t fit = s.n >= s.dev_cap ? 0 : std::min(cnt, s.dev_cap - s.n);
    if (fit) {
      hipError_t he = hipMemcpyAsync(s.dev + s.n, src, fit * sizeof(fac_match), hipMemcpyHostToDevice, stream);
      if (he == hipSuccess) he = hipStreamSynchronize(stream);  // pageable source
      if (he != hipSuccess) {
        err = std::string("record copy: ") + hipGetErrorString(he);
        return FAC_E_HIP;
      }
    }
  } else if (s.vec) {
    s.vec->resize(s.n + cnt);
    std::memcpy(s.vec->data() + s.n, src, cnt * sizeof(fac_match));
  } else {
    if (int rc = grow_pinned(s, s.n + cnt, err)) return rc;
    std::memcpy(s.pinned + s.n, src, cnt * sizeof(fac_match));
  }
  s.n += cnt;
  return FAC_OK;
}

}  // namespace fac

namespace {

thread_local std::string g_err;

int fail(int rc, const std::string& msg) {
  g_err = msg;
  return rc;
}

// hands a pinned sink's buffer to the C ABI caller (freed by fac_matches_free)
int hand_out(fac::MatchSink& s, fac_match** out, uint64_t* n_out) {
  if (!s.pinned) {
    s.pinned = fac::result_alloc(1);
    if (!s.pinned) return fail(FAC_E_OOM, "out of host memory");
  }
  *out = s.pinned;
  *n_out = s.n;
  s.pinned = nullptr;
  return FAC_OK;
}

int check_device(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
    return fail(FAC_E_NO_DEVICE, "no HIP device available (the engine has no CPU fallback)");
  if (device < 0 || device >= count) return fail(FAC_E_NO_DEVICE, "device ordinal out of range");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fail(FAC_E_HIP, "hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(FAC_E_NO_DEVICE, std::string("kernels are built for gfx950, device is ") + prop.gcnArchName);
  return FAC_OK;
}

int copy_out(const std::vector<fac_match>& v, fac_match** out, uint64_t* n_out) {
  *n_out = v.size();
  *out = static_cast<fac_match*>(std::malloc(std::max<size_t>(v.size(), 1) * sizeof(fac_match)));
  if (!*out) return fail(FAC_E_OOM, "out of host memory");
  if (!v.empty()) std::memcpy(*out, v.data(), v.size() * sizeof(fac_match));
  return FAC_OK;
}

// The staged haystack as search_raw's text: a shard whose text continues past its resident halo
// (open_end) has no end inside the resident bytes (the kernels flag any window that would read
// past them), and only its owned start windows are searched.
constexpr uint64_t kOpenEnd = 1ull << 62;
fac::SegDesc whole(const fac::Haystack& h) {
  fac::SegDesc s{};
  s.text_base = 0;
  s.n = h.open_end ? kOpenEnd : h.n;
  s.avail = h.n;
  s.hay_len = h.open_end ? kOpenEnd : h.len;
  s.byte_base = 0;
  s.w_begin = 0;
  s.w_end = std::min(h.n, h.owned);
  s.ascii = h.ascii ? 1u : 0u;
  return s;
}

// k_for (prefilter.rs:285-302). Returns false if some pattern needs k > 24 (full-search fallback).
bool prefilter_ks(const fac::Engine& e, float threshold, std::vector<uint32_t>& ks) {
  ks.clear();
  for (size_t i = 0; i < e.bp_m.size(); ++i) {
    const float nf = (float)e.bp_m[i];
    volatile float ratio = threshold / e.bp_weight[i];
    volatile float p_max = nf * (1.0f - ratio);
    uint64_t k_pen;
    if (p_max <= 0.0f) {
      k_pen = 0;
    } else {
      volatile float prod = p_max * e.edit_cost_mult;
      const float kf = std::floor((float)prod);
      if (std::isnan(kf)) k_pen = 0;  // Rust `as usize` saturates; NaN -> 0
      else if (kf >= 1.8446744e19f) k_pen = UINT64_MAX;
      else k_pen = (uint64_t)kf;
    }
    uint64_t k = e.bp_k_limit[i] >= 0 ? std::min<uint64_t>(k_pen, (uint64_t)e.bp_k_limit[i]) : k_pen;
    if (k > 24) return false;
    ks.push_back((uint32_t)k);
  }
  return true;
}

int search_staged_all(const fac::Engine& e, const fac::Haystack& h, float thr, hipStream_t stream,
                      fac::MatchSink& res, fac_stats* stats) {
  std::string err;
  std::vector<fac::SegDesc> segs{whole(h)};
  int rc = fac::launch_search_sink(e, h, segs, thr, stream, 0, res, stats, err);
  if (rc) return fail(rc, err);
  return FAC_OK;
}

}  // namespace

extern "C" {

const char* fac_last_error(void) { return g_err.c_str(); }

int fac_build(const fac_pattern* patterns, uint64_t n_patterns, const fac_config* cfg, fac_engine** out) {
  if (!out || !cfg || (n_patterns && !patterns)) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  if (cfg->beam_width == 0 && cfg->has_auto_beam && cfg->auto_beam_width == 0)
    return fail(FAC_E_INVALID, "auto_beam width must be >= 1");
  int rc = check_device(cfg->device);
  if (rc) return rc;
  fac_engine* fe = new (std::nothrow) fac_engine();
  if (!fe) return fail(FAC_E_OOM, "out of host memory");
  std::string err;
  rc = fac::build_engine(patterns, n_patterns, cfg, fe->e, err);
  if (!rc) rc = fac::upload_engine(fe->e, err);
  if (rc) {
    fac::free_engine_device(fe->e);
    delete fe;
    return fail(rc, err);
  }
  *out = fe;
  return FAC_OK;
}

void fac_engine_free(fac_engine* engine) {
  if (!engine) return;
  fac::free_engine_device(engine->e);
  delete engine;
  fac::call_scratch_trim();  // the kept call scratch is invisible to callers' allocators
}

void fac_trim_scratch(void) { fac::call_scratch_trim(); }

uint64_t fac_engine_num_nodes(const fac_engine* engine) { return engine ? engine->e.nodes.size() : 0; }
uint32_t fac_engine_max_edits_fast(const fac_engine* engine) { return engine ? engine->e.max_edits_fast : 0; }
uint64_t fac_max_match_graphemes(const fac_engine* engine) { return engine ? engine->e.max_match_graphemes : 0; }
int fac_prefilter_active(const fac_engine* engine) { return engine && engine->e.bitap_ok ? 1 : 0; }

void fac_matches_free(fac_match* matches) { fac::result_free(matches); }

static int stage_common(const fac_engine* engine, const uint8_t* utf8, uint64_t len, int force_ascii, fac_haystack** out,
                 uint64_t* err_graphemes, fac_haystack*& fh) {
  fh = new (std::nothrow) fac_haystack();
  if (!fh) return fail(FAC_E_OOM, "out of host memory");
  std::string err;
  int rc = fac::stage_haystack(engine->e, utf8, len, fh->h, err, force_ascii);
  if (rc == FAC_E_HAYSTACK_TOO_LARGE) {
    if (err_graphemes) *err_graphemes = fh->h.n;
    fac::free_haystack(fh->h);
    delete fh;
    fh = nullptr;
    return fail(rc, "haystack has more than u32::MAX grapheme clusters");
  }
  if (rc) {
    fac::free_haystack(fh->h);
    delete fh;
    fh = nullptr;
    return fail(rc, err);
  }
  *out = fh;
  return FAC_OK;
}

int fac_haystack_stage(const fac_engine* engine, const uint8_t* utf8, uint64_t len, fac_haystack** out,
                       uint64_t* err_graphemes) {
  if (!engine || !out || (len && !utf8)) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  // the UTF-8 check and search.rs:196's is_ascii run on the device after the upload (validate_kernel:
  // 256 MiB in well under a millisecond against ~19 ms on 16 host threads)
  const auto t0 = std::chrono::steady_clock::now();
  fac_haystack* fh = nullptr;
  const int rc = stage_common(engine, utf8, len, -2, out, err_graphemes, fh);
  if (fac::diag_env("FAC_TIMING"))
    std::fprintf(stderr, "FAC_TIMING stage: upload + device check + staging %.2f ms (host wall clock)\n",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return rc;
}

int fac_haystack_stage_device(const fac_engine* engine, const uint8_t* d_utf8, uint64_t len, void* stream,
                              fac_haystack** hay, uint64_t* err_graphemes) {
  if (!engine || !hay || (len && !d_utf8)) return fail(FAC_E_INVALID, "NULL argument");
  fac_haystack* fh = *hay;
  const bool fresh = fh == nullptr;
  if (fresh) {
    fh = new (std::nothrow) fac_haystack();
    if (!fh) return fail(FAC_E_OOM, "out of host memory");
  } else if (fh->h.own_utf8 && fh->h.d_utf8) {
    return fail(FAC_E_INVALID, "haystack was not staged from device memory");
  }
  std::string err;
  const int rc = fac::stage_haystack_device(engine->e, d_utf8, len, fh->h, err, static_cast<hipStream_t>(stream));
  if (rc) {
    if (rc == FAC_E_HAYSTACK_TOO_LARGE && err_graphemes) *err_graphemes = fh->h.failed_n;
    if (fresh) {
      fac::free_haystack(fh->h);
      delete fh;
    }
    return fail(rc, rc == FAC_E_HAYSTACK_TOO_LARGE ? std::string("haystack has more than u32::MAX grapheme clusters") : err);
  }
  *hay = fh;
  return FAC_OK;
}

int fac_haystack_stage_shard_device(const fac_engine* engine, const uint8_t* d_utf8, uint64_t len, uint64_t owned_bytes,
                                    int32_t global_ascii, int32_t open_end, uint64_t base, void* stream, fac_haystack** hay,
                                    uint64_t* err_graphemes) {
  if (!engine || !hay || (len && !d_utf8) || owned_bytes > len) return fail(FAC_E_INVALID, "bad argument");
  fac_haystack* fh = *hay;
  const bool fresh = fh == nullptr;
  if (fresh) {
    fh = new (std::nothrow) fac_haystack();
    if (!fh) return fail(FAC_E_OOM, "out of host memory");
  } else if (fh->h.own_utf8 && fh->h.d_utf8) {
    return fail(FAC_E_INVALID, "haystack was not staged from device memory");
  }
  std::string err;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : engine->e.stream;
  // the whole haystack's is_ascii decides the grapheme mode (search.rs:196); a Unicode shard's bytes
  // are UTF-8 checked by the segmentation
  int rc = fac::stage_haystack_device(engine->e, d_utf8, len, fh->h, err, st, global_ascii ? 1 : 0);
  uint64_t owned = 0;
  if (!rc) rc = fac::graphemes_before(fh->h, owned_bytes, st, owned, err);
  if (rc) {
    if (rc == FAC_E_HAYSTACK_TOO_LARGE && err_graphemes) *err_graphemes = fh->h.failed_n;
    if (fresh) {
      fac::free_haystack(fh->h);
      delete fh;
    } else {  // a failed restage leaves the haystack empty (searchable)
      fh->h.n = 0;
      fh->h.len = 0;
    }
    return fail(rc, rc == FAC_E_HAYSTACK_TOO_LARGE ? std::string("haystack has more than u32::MAX grapheme clusters") : err);
  }
  fh->h.base = base;
  fh->h.open_end = open_end != 0;
  fh->h.owned = owned;
  *hay = fh;
  return FAC_OK;
}

int fac_shard_plan(uint64_t max_match_graphemes, const uint8_t* utf8, uint64_t len, int32_t is_ascii, uint64_t n_shards,
                   uint64_t shard, uint64_t plan[4]) {
  if (!plan || (len && !utf8) || n_shards == 0 || shard >= n_shards) return fail(FAC_E_INVALID, "bad argument");
  const bool ascii = is_ascii < 0 ? fac::ascii_only(utf8, len) : is_ascii != 0;
  // cut r: the first safe cut at or after r * len / n (ASCII text: graphemes are bytes, any byte)
  auto cut = [&](uint64_t r) -> uint64_t {
    if (r == 0) return 0;
    if (r >= n_shards) return len;
    uint64_t p = (uint64_t)((unsigned __int128)len * r / n_shards);
    if (ascii) return p;
    while (p < len && !fac::safe_cut(utf8, len, p)) ++p;
    return p;
  };
  const uint64_t a = cut(shard), b = std::max(a, cut(shard + 1));
  // halo: max_match_graphemes() + 2 graphemes past b (the +1 of stream_overlap, stream.rs:256-258,
  // and the text[j + 1] lookahead of the last owned window's deepest state)
  const uint64_t halo = max_match_graphemes + 2;
  uint64_t e = b;
  if (ascii) {
    e = std::min<uint64_t>(len, b + halo);
  } else if (b < len) {
    // segment forward from b (a safe cut, or the text end) until `halo` graphemes are complete:
    // boundaries before the last character of the segmented piece are exact (UAX #29 rules look
    // at most one character ahead)
    std::vector<uint64_t> st;
    for (uint64_t span = 16 * halo + 64;; span *= 2) {
      const uint64_t end = std::min(len, b + span);
      uint64_t endc = end;
      while (endc < len && (utf8[endc] & 0xC0) == 0x80) ++endc;  // whole code points
      fac::segment_graphemes(utf8 + b, endc - b, st);
      if (st.size() > halo + 1) {
        e = b + st[halo];
        break;
      }
      if (endc >= len) {
        e = len;
        break;
      }
    }
  }
  plan[0] = a;
  plan[1] = b;
  plan[2] = e;
  plan[3] = (ascii ? 1u : 0u) | (e < len ? 2u : 0u);
  return FAC_OK;
}

int fac_haystack_stage_shard(const fac_engine* engine, const uint8_t* utf8, uint64_t len, uint64_t owned_bytes,
                             int32_t global_ascii, int32_t open_end, uint64_t base, fac_haystack** out,
                             uint64_t* err_graphemes) {
  if (!engine || !out || (len && !utf8) || owned_bytes > len) return fail(FAC_E_INVALID, "bad argument");
  *out = nullptr;
  if (!fac::utf8_valid(utf8, len)) return fail(FAC_E_INVALID, "shard is not valid UTF-8 (cut inside a code point)");
  fac_haystack* fh = nullptr;
  int rc = stage_common(engine, utf8, len, global_ascii ? 1 : 0, out, err_graphemes, fh);
  if (rc) return rc;
  fac::Haystack& h = fh->h;
  h.base = base;
  h.open_end = open_end != 0;
  if (h.ascii) {
    h.owned = owned_bytes;
  } else {
    std::string err;
    if (int hrc = fac::ensure_host(h, err)) {
      fac_haystack_free(fh);
      *out = nullptr;
      return fail(hrc, err);
    }
    h.owned = (uint64_t)(std::lower_bound(h.starts.begin(), h.starts.end(), owned_bytes) - h.starts.begin());
  }
  return FAC_OK;
}

uint64_t fac_haystack_owned_windows(const fac_haystack* hay) { return hay ? std::min(hay->h.n, hay->h.owned) : 0; }

int fac_haystack_set_key_partition(const fac_engine* engine, fac_haystack* hay, uint32_t parts, uint32_t part) {
  if (!engine || !hay || parts == 0 || part >= parts) return fail(FAC_E_INVALID, "bad argument");
  // auto-beam switches the beam on after a running count over the windows in order
  // (search.rs:1096-1103): a key partition has no such order
  if (parts > 1 && engine->e.has_auto_beam) return fail(FAC_E_UNSUPPORTED, "key partitions do not support auto_beam");
  hay->h.kparts = parts;
  hay->h.kpart = part;
  return FAC_OK;
}

uint64_t fac_haystack_graphemes(const fac_haystack* hay) { return hay ? hay->h.n : 0; }

uint64_t fac_haystack_grapheme_starts(const fac_haystack* hay, uint64_t* out, uint64_t cap) {
  if (!hay) return 0;
  const fac::Haystack& h = hay->h;
  std::string err;
  if (!h.ascii && fac::ensure_host(h, err)) return 0;
  for (uint64_t g = 0; g < h.n && g < cap; ++g) out[g] = h.ascii ? g : h.starts[g];
  return h.n;
}

void fac_haystack_free(fac_haystack* hay) {
  if (!hay) return;
  fac::free_haystack(hay->h);
  delete hay;
}

int fac_search_staged(const fac_engine* engine, const fac_haystack* hay, uint64_t window_begin,
                      uint64_t window_end, float threshold, void* stream, fac_match** out, uint64_t* n_out,
                      fac_stats* stats) {
  if (!engine || !hay || !out || !n_out) return fail(FAC_E_INVALID, "NULL argument");
  fac_search_args a{};
  a.window_begin = window_begin;
  a.window_end = window_end;
  a.threshold = threshold;
  a.stream = stream;
  return fac_search_staged_ex(engine, hay, &a, out, n_out, stats);
}

int fac_search_staged_ex(const fac_engine* engine, const fac_haystack* hay, const fac_search_args* args,
                         fac_match** out, uint64_t* n_out, fac_stats* stats) {
  if (!engine || !hay || !args || !n_out || (!out && !args->device_out)) return fail(FAC_E_INVALID, "NULL argument");
  if (out) *out = nullptr;
  *n_out = 0;
  const fac::Haystack& h = hay->h;
  fac::SegDesc s = whole(h);
  s.w_begin = std::min(args->window_begin, s.w_end);
  s.w_end = std::min(args->window_end, s.w_end);
  fac::MatchSink sink;
  sink.dev = static_cast<fac_match*>(args->device_out);
  sink.dev_cap = args->device_cap;
  std::string err;
  int rc = fac::launch_search_sink(engine->e, h, {s}, args->threshold, static_cast<hipStream_t>(args->stream),
                                   args->auto_beam_prefix, sink, stats, err);
  if (rc) {
    fac::result_free(sink.pinned);
    return fail(rc, err);
  }
  if (sink.dev) {
    *n_out = sink.n;
    if (sink.n > sink.dev_cap) return fail(FAC_E_OUTPUT_CAPACITY, "device output buffer too small (*n_out = records needed)");
    return FAC_OK;
  }
  return hand_out(sink, out, n_out);
}

int fac_auto_beam_total(const fac_engine* engine, const fac_haystack* hay, uint64_t window_begin, uint64_t window_end,
                        float threshold, void* stream, uint64_t* total) {
  if (!engine || !hay || !total) return fail(FAC_E_INVALID, "NULL argument");
  *total = 0;
  const fac::Haystack& h = hay->h;
  fac::SegDesc s = whole(h);
  s.w_begin = std::min(window_begin, s.w_end);
  s.w_end = std::min(window_end, s.w_end);
  std::string err;
  const int rc = fac::auto_beam_total(engine->e, h, {s}, threshold, static_cast<hipStream_t>(stream), *total, err);
  if (rc) return fail(rc, err);
  return FAC_OK;
}

int fac_search_raw(const fac_engine* engine, const uint8_t* utf8, uint64_t len, float threshold, fac_match** out,
                   uint64_t* n_out, uint64_t* err_graphemes) {
  if (!engine || !out || !n_out) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  *n_out = 0;
  fac_haystack* hay = nullptr;
  int rc = fac_haystack_stage(engine, utf8, len, &hay, err_graphemes);
  if (rc) return rc;
  fac::MatchSink sink;
  rc = search_staged_all(engine->e, hay->h, threshold, nullptr, sink, nullptr);
  fac_haystack_free(hay);
  if (rc) {
    fac::result_free(sink.pinned);
    return rc;
  }
  return hand_out(sink, out, n_out);
}

}  // extern "C"

namespace {

// scratch device memory of one call on stream s (reused by the thread's later calls on s)
struct DevMem {
  void* p = nullptr;
  hipStream_t s = nullptr;
  explicit DevMem(hipStream_t st) : s(st) {}
  ~DevMem() {
    if (p) fac::call_scratch_give(p, s);
  }
  int alloc(size_t bytes, std::string& err) {
    hipError_t he = hipSuccess;
    p = fac::call_scratch_take(std::max<size_t>(bytes, 16), s, &he);
    if (he != hipSuccess) {
      p = nullptr;
      err = std::string("hipMalloc: ") + hipGetErrorString(he);
      return FAC_E_OOM;
    }
    return FAC_OK;
  }
};

// The staged bytes [bs, be) = graphemes [g0, g1) searched as a text of their own (search_raw on a
// slice: is_ascii is re-decided on the slice, search.rs:196, prefilter.rs:349-350). A Unicode
// haystack's host copies must be fetched first (ensure_host).
fac::SegDesc slice_view(const fac::Haystack& h, uint64_t g0, uint64_t g1) {
  const uint64_t bs = h.ascii ? g0 : (g0 < h.n ? h.starts[g0] : h.len);
  const uint64_t be = h.ascii ? g1 : (g1 < h.n ? h.starts[g1] : h.len);
  const bool asc = h.ascii || fac::ascii_only(h.utf8.data() + bs, be - bs);
  fac::SegDesc s{};
  s.ascii = asc ? 1u : 0u;
  s.text_base = asc ? bs : g0;
  s.n = asc ? be - bs : g1 - g0;
  s.avail = s.n;
  s.hay_len = be - bs;
  s.byte_base = bs;
  s.w_begin = 0;
  s.w_end = s.n;
  return s;
}

// Prefiltered::raw on a text view of a staged haystack (prefilter.rs:304-374): bitap windows on the
// device, each merged window re-searched as its own sub-haystack, best per (start, end, pattern) by
// strictly greater similarity, sorted. Falls back to the full search of the view where the
// reference does (:311-317).
int prefiltered_view(const fac::Engine& e, const fac::Haystack& h, const fac::SegDesc& view, float threshold,
                     hipStream_t stream, std::vector<fac_match>& merged, fac_stats* stats, std::string& err) {
  merged.clear();
  std::vector<uint32_t> ks;
  if (!e.bitap_ok || !prefilter_ks(e, threshold, ks))  // prefilter.rs:151-155, 311-317
    return fac::launch_search(e, h, {view}, threshold, stream, merged, stats, err);
  std::vector<std::pair<uint64_t, uint64_t>> windows;
  int rc = fac::prefilter_windows(e, h, view, ks, stream, windows, stats, err);
  if (rc) return rc;
  if (!view.ascii && (rc = fac::ensure_host(h, err))) return rc;  // slice_view reads the host copies
  // Re-search each merged window as its own haystack (prefilter.rs:344-350): the slice re-decides
  // is_ascii, so an all-ASCII slice of a Unicode haystack is searched byte-wise.
  std::vector<fac::SegDesc> segs;
  segs.reserve(windows.size());
  for (auto& w : windows) {
    const uint64_t gs = w.first, ge = std::min<uint64_t>(w.second, view.n);
    if (view.ascii) {  // byte-wise view: windows are bytes of h.d_utf8 from view.text_base
      fac::SegDesc s{};
      s.ascii = 1u;
      s.text_base = view.text_base + gs;
      s.n = ge - gs;
      s.avail = s.n;
      s.hay_len = s.n;
      s.byte_base = view.text_base + gs;
      s.w_begin = 0;
      s.w_end = s.n;
      segs.push_back(s);
    } else {
      segs.push_back(slice_view(h, view.text_base + gs, view.text_base + ge));
    }
  }
  if (segs.empty()) return FAC_OK;
  std::vector<fac_match> res;
  rc = fac::launch_search(e, h, segs, threshold, stream, res, stats, err);
  if (rc) return rc;
  std::map<std::tuple<uint64_t, uint64_t, uint32_t>, fac_match> best;
  for (const fac_match& m : res) {
    auto key = std::make_tuple(m.start, m.end, m.pattern_index);
    auto it = best.find(key);
    if (it == best.end()) best.emplace(key, m);
    else if (m.similarity > it->second.similarity) it->second = m;
  }
  merged.reserve(best.size());
  for (auto& kv : best) merged.push_back(kv.second);
  return FAC_OK;
}

int prefiltered_staged(const fac::Engine& e, const fac::Haystack& h, float threshold, hipStream_t stream,
                       std::vector<fac_match>& merged, fac_stats* stats, std::string& err) {
  if (h.open_end) {
    err = "the pre-filtered search needs a whole haystack, not an open-ended shard";
    return FAC_E_INVALID;
  }
  return prefiltered_view(e, h, whole(h), threshold, stream, merged, stats, err);
}


}  // namespace

namespace fac {

// A batch of stream windows of one staged ASCII haystack searched together (stream.rs
// window_matches for each, :262-297): wins holds (g_begin, g_end, commit_bytes, base) per window,
// sorted by g_begin, each overlapping only its neighbours. With the pre-filter, one q-gram pass over
// the windows' union gives every window its own merged bitap windows (the automaton starts at the
// window's first byte, its coverage stays inside it); without it each window is one segment. All
// segments, tagged with their window, go to one launch; then every window's records are ranked
// sorted().non_overlapping() and cut at its commit point on the host. FAC_E_UNSUPPORTED (nothing
// done) when the batch does not qualify: a Unicode haystack (a window's grapheme segmentation
// depends on where its text starts and ends), windows out of order or overlapping beyond their
// neighbours, or pre-filter tables that need the packed full scan.
int stream_windows_batch(const Engine& e, const Haystack& h, const uint64_t* wins, uint64_t n_windows, float threshold,
                         bool prefilter, hipStream_t st, std::vector<fac_match>& owned, fac_stats* stats, std::string& err) {
  owned.clear();
  if (!h.ascii || h.open_end || h.base || n_windows == 0 || n_windows >= (1u << 24) || h.len >= (1ull << kWinTagShift))
    return FAC_E_UNSUPPORTED;
  std::vector<std::pair<uint64_t, uint64_t>> span(n_windows);
  std::vector<WinOwn> own(n_windows);
  uint64_t u0 = UINT64_MAX, u1 = 0;
  for (uint64_t w = 0; w < n_windows; ++w) {
    const uint64_t ge = std::min<uint64_t>(wins[4 * w + 1], h.n), gb = std::min<uint64_t>(wins[4 * w], ge);
    span[w] = {gb, ge};
    own[w] = WinOwn{gb, wins[4 * w + 2], wins[4 * w + 3]};  // ASCII: grapheme = byte
    u0 = std::min(u0, gb);
    u1 = std::max(u1, ge);
    if (w && gb < span[w - 1].first) return FAC_E_UNSUPPORTED;
    if (w >= 2 && span[w - 2].second >= gb) return FAC_E_UNSUPPORTED;  // same parity must not touch
  }
  if (u1 <= u0) return FAC_OK;
  const SegDesc view = slice_view(h, u0, u1);
  std::vector<SegDesc> segs;
  std::vector<uint32_t> ks;
  if (prefilter && e.bitap_ok && prefilter_ks(e, threshold, ks)) {
    std::vector<std::pair<uint64_t, uint64_t>> rel(n_windows), runs;
    for (uint64_t w = 0; w < n_windows; ++w) rel[w] = {span[w].first - u0, span[w].second - u0};
    std::vector<uint32_t> run_win;
    // (one window is the whole view: the plain pass, no window bounds or second bitmap)
    if (int rc = prefilter_windows_ex(e, h, view, ks, st, n_windows > 1 ? &rel : nullptr, runs, &run_win, stats, err))
      return rc;
    if (n_windows == 1) run_win.assign(runs.size(), 0u);
    segs.reserve(runs.size());
    for (size_t r = 0; r < runs.size(); ++r) {
      SegDesc s{};
      s.ascii = 1u;
      s.text_base = view.text_base + runs[r].first;
      s.n = runs[r].second - runs[r].first;
      s.avail = s.n;
      s.hay_len = s.n;
      s.byte_base = s.text_base | ((uint64_t)run_win[r] << kWinTagShift);  // the window tag (WinOwn)
      s.w_begin = 0;
      s.w_end = s.n;
      segs.push_back(s);
    }
  } else {  // no pre-filter (or the reference's fallback to a full search, prefilter.rs:311-317)
    for (uint64_t w = 0; w < n_windows; ++w) {
      if (span[w].second <= span[w].first) continue;
      SegDesc s = slice_view(h, span[w].first, span[w].second);
      s.byte_base |= (uint64_t)w << kWinTagShift;  // the window tag (WinOwn)
      segs.push_back(s);
    }
  }
  if (segs.empty()) return FAC_OK;
  uint64_t cap = 1u << 16;
  for (;;) {  // raw records into a device buffer, grown and searched again if it was too small
    DevMem raw(st);
    if (int rc = raw.alloc(cap * sizeof(fac_match), err)) return rc;
    MatchSink sink;
    sink.dev = static_cast<fac_match*>(raw.p);
    sink.dev_cap = cap;
    if (int rc = launch_search_sink(e, h, segs, threshold, st, 0, sink, stats, err)) return rc;
    if (sink.n > cap) {
      cap = sink.n;
      continue;
    }
    std::vector<fac_match> recs(sink.n);
    if (sink.n) {
      if (hipMemcpyAsync(recs.data(), sink.dev, sink.n * sizeof(fac_match), hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess) {
        err = "hipMemcpyAsync of a stream batch's records failed";
        return FAC_E_HIP;
      }
    }
    windows_owned_host(e, recs, own, owned);
    return FAC_OK;
  }
}

}  // namespace fac

namespace {
}  // namespace

extern "C" {

int fac_search_prefiltered(const fac_engine* engine, const uint8_t* utf8, uint64_t len, float threshold,
                           fac_match** out, uint64_t* n_out, uint64_t* err_graphemes) {
  if (!engine || !out || !n_out) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  *n_out = 0;
  fac_haystack* hay = nullptr;
  int rc = fac_haystack_stage(engine, utf8, len, &hay, err_graphemes);
  if (rc) return rc;
  std::vector<fac_match> merged;
  std::string err;
  rc = prefiltered_staged(engine->e, hay->h, threshold, nullptr, merged, nullptr, err);
  fac_haystack_free(hay);
  if (rc) return fail(rc, err);
  return copy_out(merged, out, n_out);
}

int fac_search_staged_prefiltered(const fac_engine* engine, const fac_haystack* hay, float threshold, void* stream,
                                  fac_match** out, uint64_t* n_out, fac_stats* stats) {
  if (!engine || !hay || !out || !n_out) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  *n_out = 0;
  std::vector<fac_match> merged;
  std::string err;
  const int rc =
      prefiltered_staged(engine->e, hay->h, threshold, static_cast<hipStream_t>(stream), merged, stats, err);
  if (rc) return fail(rc, err);
  return copy_out(merged, out, n_out);
}

int fac_stream_window_staged(const fac_engine* engine, const fac_haystack* hay, uint64_t g_begin, uint64_t g_end,
                             uint64_t commit_bytes, uint64_t base, float threshold, int32_t prefilter, void* stream,
                             fac_match** out, uint64_t* n_out, fac_stats* stats) {
  if (!engine || !hay || !out || !n_out) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  *n_out = 0;
  const fac::Haystack& h = hay->h;
  if (h.open_end || h.base) return fail(FAC_E_INVALID, "stream windows are cut from a whole staged haystack");
  g_end = std::min(g_end, h.n);
  g_begin = std::min(g_begin, g_end);
  std::string herr;
  if (!h.ascii)
    if (int hrc = fac::ensure_host(h, herr)) return fail(hrc, herr);
  const fac::SegDesc view = slice_view(h, g_begin, g_end);
  const fac::Engine& e = engine->e;
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<fac_match> v;
  std::string err;
  int rc = prefilter ? prefiltered_view(e, h, view, threshold, st, v, stats, err)
                     : fac::launch_search(e, h, {view}, threshold, st, v, stats, err);
  if (rc) return fail(rc, err);
  // window_matches (stream.rs:262-297): sorted().non_overlapping() within the window, then the
  // matches the window owns (start < commit), at absolute offsets
  if (!v.empty() && (rc = fac::apply_matches(e, v, 1, 1, nullptr, err))) return fail(rc, err);
  std::vector<fac_match> owned;
  owned.reserve(v.size());
  for (fac_match m : v) {
    m.start -= view.byte_base;
    m.end -= view.byte_base;
    if (m.start < commit_bytes) {
      m.start += base;
      m.end += base;
      owned.push_back(m);
    }
  }
  return copy_out(owned, out, n_out);
}

int fac_stream_window_staged_device(const fac_engine* engine, const fac_haystack* hay, uint64_t g_begin, uint64_t g_end,
                                    uint64_t commit_bytes, uint64_t base, float threshold, int32_t prefilter, void* stream,
                                    void* device_out, uint64_t device_cap, uint64_t* n_out, fac_stats* stats) {
  if (!engine || !hay || !n_out || (!device_out && device_cap)) return fail(FAC_E_INVALID, "NULL argument");
  *n_out = 0;
  const fac::Haystack& h = hay->h;
  if (h.open_end || h.base) return fail(FAC_E_INVALID, "stream windows are cut from a whole staged haystack");
  g_end = std::min(g_end, h.n);
  g_begin = std::min(g_begin, g_end);
  std::string err;
  if (!h.ascii)
    if (int hrc = fac::ensure_host(h, err)) return fail(hrc, err);
  const fac::SegDesc view = slice_view(h, g_begin, g_end);
  const fac::Engine& e = engine->e;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hipSetDevice(e.device) != hipSuccess) return fail(FAC_E_HIP, "hipSetDevice failed");
  // the window's searched segments: Prefiltered::raw's merged bitap windows (disjoint and not
  // adjacent, so their records never share a (start, end, pattern) key and the reference's
  // best-per-key merge is a no-op before the ranking), or the whole view where it falls back
  std::vector<fac::SegDesc> segs;
  std::vector<uint32_t> ks;
  const bool timing = fac::diag_env("FAC_TIMING") != nullptr;  // diagnostics: host wall-clock phases
  const auto t0 = std::chrono::steady_clock::now();
  auto ms_since = [&](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  };
  double t_pf = 0, t_segs = 0, t_search = 0;
  if (prefilter && e.bitap_ok && prefilter_ks(e, threshold, ks)) {
    std::vector<std::pair<uint64_t, uint64_t>> windows;
    if (int rc = fac::prefilter_windows(e, h, view, ks, st, windows, stats, err)) return fail(rc, err);
    t_pf = ms_since(t0);
    for (auto& w : windows) {
      const uint64_t gs = w.first, ge = std::min<uint64_t>(w.second, view.n);
      if (view.ascii) {
        fac::SegDesc s{};
        s.ascii = 1u;
        s.text_base = view.text_base + gs;
        s.n = ge - gs;
        s.avail = s.n;
        s.hay_len = s.n;
        s.byte_base = view.text_base + gs;
        s.w_begin = 0;
        s.w_end = s.n;
        segs.push_back(s);
      } else {
        segs.push_back(slice_view(h, view.text_base + gs, view.text_base + ge));
      }
    }
  } else {
    segs.push_back(view);
  }
  t_segs = ms_since(t0);
  if (segs.empty()) return FAC_OK;
  // raw records into a device buffer (grown and searched again if a window ever needs more)
  uint64_t cap = 1u << 16;
  for (;;) {
    DevMem raw(st);
    if (int rc = raw.alloc(2 * cap * sizeof(fac_match), err)) return fail(rc, err);
    fac::MatchSink sink;
    sink.dev = static_cast<fac_match*>(raw.p);
    sink.dev_cap = cap;
    if (int rc = fac::launch_search_sink(e, h, segs, threshold, st, 0, sink, stats, err)) return fail(rc, err);
    if (sink.n > cap) {
      cap = sink.n;
      continue;
    }
    t_search = ms_since(t0);
    const int rc = fac::window_owned_device(e, sink.dev, sink.dev + cap, sink.n, view.byte_base, commit_bytes, base, st,
                                            static_cast<fac_match*>(device_out), device_cap, n_out, err);
    if (timing)
      std::fprintf(stderr, "FAC_TIMING window: prefilter %.3f, segs %.3f (%zu), search %.3f, owned %.3f ms\n", t_pf,
                   t_segs - t_pf, segs.size(), t_search - t_segs, ms_since(t0) - t_search);
    if (rc == FAC_E_OUTPUT_CAPACITY) return fail(rc, "device output buffer too small (*n_out = records needed)");
    if (rc) return fail(rc, err);
    return FAC_OK;
  }
}

int fac_stream_windows_staged_device(const fac_engine* engine, const fac_haystack* hay, const uint64_t* windows,
                                     uint64_t n_windows, float threshold, int32_t prefilter, void* stream, void* device_out,
                                     uint64_t device_cap, uint64_t* n_out, fac_stats* stats) {
  if (!engine || !hay || !n_out || (!windows && n_windows) || (!device_out && device_cap))
    return fail(FAC_E_INVALID, "NULL argument");
  *n_out = 0;
  const fac::Haystack& h = hay->h;
  if (h.open_end || h.base) return fail(FAC_E_INVALID, "stream windows are cut from a whole staged haystack");
  const fac::Engine& e = engine->e;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hipSetDevice(e.device) != hipSuccess) return fail(FAC_E_HIP, "hipSetDevice failed");
  std::vector<fac_match> owned;
  std::string err;
  int rc = fac::stream_windows_batch(e, h, windows, n_windows, threshold, prefilter != 0, st, owned, stats, err);
  if (rc == FAC_E_UNSUPPORTED) {  // window by window (fac_stream_window_staged)
    owned.clear();
    for (uint64_t w = 0; w < n_windows; ++w) {
      fac_match* part = nullptr;
      uint64_t np = 0;
      rc = fac_stream_window_staged(engine, hay, windows[4 * w], windows[4 * w + 1], windows[4 * w + 2], windows[4 * w + 3],
                                    threshold, prefilter, stream, &part, &np, stats);
      if (rc) return rc;
      owned.insert(owned.end(), part, part + np);
      fac_matches_free(part);
    }
  } else if (rc) {
    return fail(rc, err);
  }
  *n_out = owned.size();
  if (owned.size() > device_cap) return fail(FAC_E_OUTPUT_CAPACITY, "device output buffer too small (*n_out = records needed)");
  if (!owned.empty() &&
      (hipMemcpyAsync(device_out, owned.data(), owned.size() * sizeof(fac_match), hipMemcpyHostToDevice, st) != hipSuccess ||
       hipStreamSynchronize(st) != hipSuccess))
    return fail(FAC_E_HIP, "hipMemcpyAsync of the owned records failed");
  return FAC_OK;
}

int fac_matches_apply(const fac_engine* engine, fac_match* matches, uint64_t n, int32_t order, int32_t overlap,
                      const uint64_t* unique_ids, uint64_t* n_out) {
  if (!engine || (!matches && n) || !n_out) return fail(FAC_E_INVALID, "NULL argument");
  if (order < 0 || order > 3 || overlap < 0 || overlap > 2) return fail(FAC_E_INVALID, "bad order/overlap");
  std::vector<fac_match> v(matches, matches + n);
  std::string err;
  const int rc = fac::apply_matches(engine->e, v, order, overlap, unique_ids, err);
  if (rc) return fail(rc, err);
  if (!v.empty()) std::memcpy(matches, v.data(), v.size() * sizeof(fac_match));
  *n_out = v.size();
  return FAC_OK;
}

int fac_stream_open(const fac_engine* engine, float threshold, uint64_t window_bytes, fac_stream** out) {
  if (!engine || !out) return fail(FAC_E_INVALID, "NULL argument");
  fac_stream* fs = new (std::nothrow) fac_stream();
  if (!fs) return fail(FAC_E_OOM, "out of host memory");
  fs->s = fac::stream_open(engine->e, threshold, window_bytes);
  *out = fs;
  return FAC_OK;
}

int fac_stream_feed(fac_stream* stream, const uint8_t* data, uint64_t len, int32_t eof, fac_match** out,
                    uint64_t* n_out, uint8_t** text, uint64_t* text_len) {
  if (!stream || !out || !n_out || !text || !text_len || (len && !data)) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  *n_out = 0;
  *text = nullptr;
  *text_len = 0;
  std::string err;
  fac::StreamCore& s = *stream->s;
  const int rc = fac::stream_feed(s, data, len, eof != 0, err);
  if (rc) return fail(rc, err);
  int r = copy_out(s.ready, out, n_out);
  if (r) return r;
  *text_len = s.ready_text.size();
  *text = static_cast<uint8_t*>(std::malloc(std::max<size_t>(s.ready_text.size(), 1)));
  if (!*text) return fail(FAC_E_OOM, "out of host memory");
  if (!s.ready_text.empty()) std::memcpy(*text, s.ready_text.data(), s.ready_text.size());
  s.ready.clear();
  s.ready_text.clear();
  return FAC_OK;
}

uint64_t fac_stream_total(const fac_stream* stream) { return stream ? stream->s->total : 0; }
uint64_t fac_stream_committed(const fac_stream* stream) { return stream ? fac::stream_committed(*stream->s) : 0; }

void fac_stream_close(fac_stream* stream) {
  if (!stream) return;
  fac::stream_close(stream->s);
  delete stream;
}

void fac_buffer_free(void* p) { std::free(p); }

int64_t fac_prefilter_windows(const fac_engine* engine, const uint8_t* utf8, uint64_t len, float threshold,
                              uint64_t* out, uint64_t cap) {
  if (!engine) return fail(FAC_E_INVALID, "NULL argument"), -1;
  const fac::Engine& e = engine->e;
  std::vector<uint32_t> ks;
  if (!e.bitap_ok || !prefilter_ks(e, threshold, ks)) return -1;
  fac_haystack* hay = nullptr;
  if (fac_haystack_stage(engine, utf8, len, &hay, nullptr)) return -1;
  std::string err;
  std::vector<std::pair<uint64_t, uint64_t>> windows;
  int rc = fac::prefilter_windows(e, hay->h, whole(hay->h), ks, nullptr, windows, nullptr, err);
  fac_haystack_free(hay);
  if (rc) return fail(rc, err), -1;
  for (size_t i = 0; i < windows.size() && i < cap; ++i) {
    out[2 * i] = windows[i].first;
    out[2 * i + 1] = windows[i].second;
  }
  return (int64_t)windows.size();
}

uint64_t fac_segment_graphemes(const uint8_t* utf8, uint64_t len, uint64_t* starts, uint64_t cap) {
  std::vector<uint64_t> s;
  fac::segment_graphemes(utf8, len, s);
  for (uint64_t i = 0; i < s.size() && i < cap; ++i) starts[i] = s[i];
  return s.size();
}

uint32_t fac_fold_first_char(const uint8_t* utf8, uint64_t len, int32_t case_insensitive) {
  return fac::fold_first_char(utf8, 0, len, case_insensitive != 0);
}

void fac_edge_order(const uint32_t* cps, const uint64_t* off, uint64_t n, uint32_t* order) {
  std::vector<std::u32string> g(n);
  for (uint64_t i = 0; i < n; ++i) g[i].assign(cps + off[i], cps + off[i + 1]);
  const std::vector<uint32_t> o = fac::transitions_order(g);
  for (uint64_t i = 0; i < n; ++i) order[i] = o[i];
}

int fac_diag_beam_select(const float* keys, const uint64_t* offs, uint64_t count, uint32_t bw, int32_t lds,
                         int32_t sel_limit, uint32_t* perm) {
  if (!keys || !offs || !perm) return fail(FAC_E_INVALID, "null argument");
  if (int rc = check_device(0)) return rc;
  std::string err;
  int rc = fac::diag_beam_select(keys, offs, count, bw, lds, sel_limit, perm, err);
  return rc ? fail(rc, err) : FAC_OK;
}

}  // extern "C"
