// stream.cpp — the crate's streaming search (src/stream.rs) over the GPU search path.
//
// WindowReader (stream.rs:77-159): bytes are fed in the reader's read() pieces; once the buffer
// holds >= `window` bytes (or the input ended) a window is cut: its text is the buffer's valid
// UTF-8 prefix, and unless it is the last window it owns only the matches that start before the
// commit point — the byte start of the `overlap`-th grapheme from the end (overlap =
// max_match_graphemes + 1, stream.rs:256-258); with too few graphemes the window grows and more
// input is awaited. Each window is staged and searched on the device as its own haystack, ranked
// with `sorted().non_overlapping()` (stream.rs:262-297) and filtered to the owned matches, whose
// offsets become absolute. The buffer then drops the committed prefix.
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fac_internal.h"

namespace fac {


namespace {

// Search one window and append the matches it owns (stream.rs:262-297).
int window_matches(StreamCore& s, const uint8_t* text, uint64_t len, uint64_t commit, const Haystack& h,
                   std::string& err) {
  SegDesc seg{};
  seg.text_base = 0;
  seg.n = h.n;
  seg.avail = h.n;
  seg.hay_len = h.len;
  seg.byte_base = 0;
  seg.w_begin = 0;
  seg.w_end = h.n;
  seg.ascii = h.ascii ? 1u : 0u;
  std::vector<fac_match> res;
  int rc = launch_search(*s.e, h, {seg}, s.threshold, nullptr, res, nullptr, err);
  if (rc) return rc;
  rc = apply_matches(*s.e, res, /*Default*/ 1, /*NonOverlapping*/ 1, nullptr, err);
  if (rc) return rc;
  for (const fac_match& m : res) {
    if (m.start >= commit) continue;
    fac_match a = m;
    a.start += s.base;
    a.end += s.base;
    s.ready.push_back(a);
    s.ready_text.insert(s.ready_text.end(), text + m.start, text + m.end);
  }
  (void)len;
  return FAC_OK;
}

// Cut and search windows while the buffer allows (next_window, stream.rs:102-158).
int pump(StreamCore& s, bool eof, std::string& err) {
  while (!s.done && (eof || s.buf.size() >= s.window)) {
    const uint64_t valid = utf8_valid_prefix(s.buf.data(), s.buf.size());
    const bool last = s.buf.size() < s.window;  // reached only at end of input
    Haystack h;
    int rc = stage_haystack(*s.e, s.buf.data(), valid, h, err);
    if (rc) {
      free_haystack(h);
      return rc;
    }
    uint64_t commit = valid;
    if (!last) {
      // byte start of the overlap-th grapheme from the end; none or 0: grow and read more
      uint64_t off = 0;
      const bool have = h.n >= s.overlap;
      if (have) off = h.ascii ? h.n - s.overlap : h.starts[h.n - s.overlap];
      if (!have || off == 0) {
        free_haystack(h);
        s.window += std::max<uint64_t>(s.window, 64 * 1024);
        if (eof) continue;  // input ended: the next round is the last window
        return FAC_OK;
      }
      commit = off;
    }
    rc = window_matches(s, s.buf.data(), valid, commit, h, err);
    free_haystack(h);
    if (rc) return rc;
    if (last) {
      s.done = true;
      break;
    }
    s.buf.erase(s.buf.begin(), s.buf.begin() + (ptrdiff_t)commit);
    s.base += commit;
  }
  return FAC_OK;
}

}  // namespace

int stream_feed(StreamCore& s, const uint8_t* data, uint64_t len, bool eof, std::string& err) {
  if (s.done) return FAC_OK;
  if (len) {
    s.buf.insert(s.buf.end(), data, data + len);
    s.total += len;
  }
  return pump(s, eof, err);
}

StreamCore* stream_open(const Engine& e, float threshold, uint64_t window) {
  StreamCore* s = new StreamCore();
  s->e = &e;
  s->threshold = threshold;
  if (window) s->window = window;
  s->overlap = e.max_match_graphemes + 1;  // stream_overlap (stream.rs:256-258)
  return s;
}

void stream_close(StreamCore* s) { delete s; }

}  // namespace fac
