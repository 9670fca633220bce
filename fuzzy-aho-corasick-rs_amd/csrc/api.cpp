// api.cpp — the extern "C" boundary declared in include/fac.h.
//
// fac_search_raw is the drop-in for FuzzyAhoCorasick::search_raw (src/search.rs:187-395):
// host staging (is_ascii + grapheme segmentation/folding, :196-203 / :296-302), then the GPU
// window kernel over every start position. fac_search_prefiltered is the drop-in for
// Prefiltered::raw (src/prefilter.rs:146-155, 304-374): k_for on the host, the bitap scan and the
// window merge on the GPU, then the window kernel over the merged slices. There is no CPU search
// path: without a usable gfx950 device every search entry point returns FAC_E_NO_DEVICE.
#include <algorithm>
#include <cmath>
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

namespace {

thread_local std::string g_err;

int fail(int rc, const std::string& msg) {
  g_err = msg;
  return rc;
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

fac::SegDesc whole(const fac::Haystack& h) {
  fac::SegDesc s{};
  s.text_base = 0;
  s.n = h.n;
  s.avail = h.n;
  s.hay_len = h.len;
  s.byte_base = 0;
  s.w_begin = 0;
  s.w_end = h.n;
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
                      std::vector<fac_match>& res, fac_stats* stats) {
  std::string err;
  std::vector<fac::SegDesc> segs{whole(h)};
  int rc = fac::launch_search(e, h, segs, thr, stream, res, stats, err);
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
}

uint64_t fac_engine_num_nodes(const fac_engine* engine) { return engine ? engine->e.nodes.size() : 0; }
uint32_t fac_engine_max_edits_fast(const fac_engine* engine) { return engine ? engine->e.max_edits_fast : 0; }
uint64_t fac_max_match_graphemes(const fac_engine* engine) { return engine ? engine->e.max_match_graphemes : 0; }
int fac_prefilter_active(const fac_engine* engine) { return engine && engine->e.bitap_ok ? 1 : 0; }

void fac_matches_free(fac_match* matches) { std::free(matches); }

int fac_haystack_stage(const fac_engine* engine, const uint8_t* utf8, uint64_t len, fac_haystack** out,
                       uint64_t* err_graphemes) {
  if (!engine || !out || (len && !utf8)) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  if (!fac::utf8_valid(utf8, len)) return fail(FAC_E_INVALID, "haystack is not valid UTF-8");
  fac_haystack* fh = new (std::nothrow) fac_haystack();
  if (!fh) return fail(FAC_E_OOM, "out of host memory");
  std::string err;
  int rc = fac::stage_haystack(engine->e, utf8, len, fh->h, err);
  if (rc == FAC_E_HAYSTACK_TOO_LARGE) {
    if (err_graphemes) *err_graphemes = fh->h.n;
    fac::free_haystack(fh->h);
    delete fh;
    return fail(rc, "haystack has more than u32::MAX grapheme clusters");
  }
  if (rc) {
    fac::free_haystack(fh->h);
    delete fh;
    return fail(rc, err);
  }
  *out = fh;
  return FAC_OK;
}

uint64_t fac_haystack_graphemes(const fac_haystack* hay) { return hay ? hay->h.n : 0; }

uint64_t fac_haystack_grapheme_starts(const fac_haystack* hay, uint64_t* out, uint64_t cap) {
  if (!hay) return 0;
  const fac::Haystack& h = hay->h;
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
  const fac::Haystack& h = hay->h;
  fac::SegDesc s = whole(h);
  s.w_begin = std::min(window_begin, h.n);
  s.w_end = std::min(window_end, h.n);
  std::vector<fac_match> res;
  std::string err;
  int rc = fac::launch_search(engine->e, h, {s}, threshold, static_cast<hipStream_t>(stream), res, stats, err);
  if (rc) return fail(rc, err);
  return copy_out(res, out, n_out);
}

int fac_search_raw(const fac_engine* engine, const uint8_t* utf8, uint64_t len, float threshold, fac_match** out,
                   uint64_t* n_out, uint64_t* err_graphemes) {
  if (!engine || !out || !n_out) return fail(FAC_E_INVALID, "NULL argument");
  *out = nullptr;
  *n_out = 0;
  fac_haystack* hay = nullptr;
  int rc = fac_haystack_stage(engine, utf8, len, &hay, err_graphemes);
  if (rc) return rc;
  std::vector<fac_match> res;
  rc = search_staged_all(engine->e, hay->h, threshold, nullptr, res, nullptr);
  fac_haystack_free(hay);
  if (rc) return rc;
  return copy_out(res, out, n_out);
}

}  // extern "C"

namespace {

// Prefiltered::raw on a staged haystack (prefilter.rs:304-374): bitap windows on the device, each
// merged window re-searched as its own sub-haystack, best per (start, end, pattern) by strictly
// greater similarity, sorted. Falls back to the full search where the reference does (:311-317).
int prefiltered_staged(const fac::Engine& e, const fac::Haystack& h, float threshold, hipStream_t stream,
                       std::vector<fac_match>& merged, fac_stats* stats, std::string& err) {
  merged.clear();
  std::vector<uint32_t> ks;
  if (!e.bitap_ok || !prefilter_ks(e, threshold, ks))  // prefilter.rs:151-155, 311-317
    return fac::launch_search(e, h, {whole(h)}, threshold, stream, merged, stats, err);
  std::vector<std::pair<uint64_t, uint64_t>> windows;
  int rc = fac::prefilter_windows(e, h, ks, stream, windows, stats, err);
  if (rc) return rc;
  // Re-search each merged window as its own haystack (prefilter.rs:344-350): the slice re-decides
  // is_ascii, so an all-ASCII slice of a Unicode haystack is searched byte-wise.
  std::vector<fac::SegDesc> segs;
  segs.reserve(windows.size());
  for (auto& w : windows) {
    const uint64_t gs = w.first, ge = std::min<uint64_t>(w.second, h.n);
    const uint64_t bs = h.ascii ? gs : h.starts[gs];
    const uint64_t be = h.ascii ? ge : (ge < h.n ? h.starts[ge] : h.len);
    fac::SegDesc s{};
    bool sub_ascii = h.ascii;
    if (!sub_ascii) {
      sub_ascii = true;
      for (uint64_t i = bs; i < be; ++i)
        if (h.utf8[i] & 0x80) {
          sub_ascii = false;
          break;
        }
    }
    s.ascii = sub_ascii ? 1u : 0u;
    s.text_base = sub_ascii ? bs : gs;
    s.n = sub_ascii ? be - bs : ge - gs;
    s.avail = s.n;
    s.hay_len = be - bs;
    s.byte_base = bs;
    s.w_begin = 0;
    s.w_end = s.n;
    segs.push_back(s);
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
  int rc = fac::prefilter_windows(e, hay->h, ks, nullptr, windows, nullptr, err);
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

}  // extern "C"
