// stream.cpp — the crate's streaming search (src/stream.rs) over the GPU search path.
//
// WindowReader (stream.rs:77-159): bytes are fed in the reader's read() pieces; once the buffer
// holds >= `window` bytes (or the input ended) a window is cut: its text is the buffer's valid
// UTF-8 prefix, and unless it is the last window it owns only the matches that start before the
// commit point — the byte start of the `overlap`-th grapheme from the end (overlap =
// max_match_graphemes + 1, stream.rs:256-258), found on the host from a short tail of the text;
// with too few graphemes the window grows and more input is awaited. The buffer then drops the
// committed prefix.
//
// Consecutive windows are collected into batches of about 32 MiB of text, and each batch is handed
// to one of `depth` (2) worker threads, batch k to worker k % depth. A worker owns a HIP stream and
// a device scratch set. An all-ASCII batch is staged once (H2D) and its windows searched in one
// launch, each as its own text (stream_windows_batch); a batch with other text stages and searches
// its windows one by one (H2D + device segmentation + folding each). Every window is ranked
// sorted().non_overlapping() and keeps the matches it owns (stream.rs:262-297). Batch k + 1's
// copies and kernels overlap batch k's (double buffering) while the host cuts the windows of batch
// k + 2. Finished batches are handed out strictly in window order.
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <new>
#include <stdexcept>
#include <thread>
#include <vector>

#include "fac_internal.h"

namespace fac {

// A batch of consecutive windows: text holds stream bytes [base, base + text.size()), window w is
// text[off, off + len) and owns the matches starting before off + commit.
struct StreamWin {
  uint64_t off, len, commit;
};
struct StreamTask {
  std::vector<uint8_t> text;
  uint64_t base = 0;
  std::vector<StreamWin> wins;
  std::vector<fac_match> res;  // owned matches of every window, in window order, absolute offsets
  std::vector<uint8_t> res_text;
  int rc = FAC_OK;
  std::string err;
  bool done = false;
};

struct StreamWorker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<StreamTask*> q;
  bool stop = false;
  hipStream_t stream = nullptr;
  ScratchSet scratch;
};

namespace {

std::mutex g_done_mu;  // guards StreamTask::done across workers and the feeding thread
std::condition_variable g_done_cv;

// Search one window (text[off, off + len) of the task) and keep the matches it owns (stream.rs:262-297).
int search_one_window(const StreamCore& s, StreamWorker& w, const StreamTask& t, const StreamWin& win,
                      std::vector<fac_match>& owned, std::string& err) {
  Haystack h;
  int rc = stage_haystack(*s.e, t.text.data() + win.off, win.len, h, err, -1, w.stream);
  if (!rc) {
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
    rc = launch_search(*s.e, h, {seg}, s.threshold, w.stream, res, nullptr, err);
    if (!rc) rc = apply_matches(*s.e, res, /*Default*/ 1, /*NonOverlapping*/ 1, nullptr, err);
    if (!rc)
      for (const fac_match& m : res) {
        if (m.start >= win.commit) continue;
        fac_match a = m;
        a.start += t.base + win.off;
        a.end += t.base + win.off;
        owned.push_back(a);
      }
  }
  free_haystack(h);
  return rc;
}

// Search a batch of windows. An all-ASCII batch is staged once and searched as one launch over its
// windows (stream_windows_batch: each window its own text, ranked and cut per window); otherwise each
// window is staged and searched alone (its grapheme segmentation depends on where its text starts
// and ends).
void run_window_task(const StreamCore& s, StreamWorker& w, StreamTask& t) {
  std::vector<fac_match> owned;
  bool batched = false;
  if (t.wins.size() > 1 && ascii_only(t.text.data(), t.text.size())) {
    Haystack h;
    t.rc = stage_haystack(*s.e, t.text.data(), t.text.size(), h, t.err, 1, w.stream);
    if (!t.rc) {
      std::vector<uint64_t> wins(4 * t.wins.size());
      for (size_t i = 0; i < t.wins.size(); ++i) {
        wins[4 * i] = t.wins[i].off;
        wins[4 * i + 1] = t.wins[i].off + t.wins[i].len;
        wins[4 * i + 2] = t.wins[i].commit;
        wins[4 * i + 3] = t.base + t.wins[i].off;
      }
      const int rc = stream_windows_batch(*s.e, h, wins.data(), t.wins.size(), s.threshold, false, w.stream, owned,
                                          nullptr, t.err);
      if (rc != FAC_E_UNSUPPORTED) {
        t.rc = rc;
        batched = true;
      }
    }
    free_haystack(h);
    if (t.rc) batched = true;  // a staging failure is the task's error
  }
  if (!batched) {
    owned.clear();
    for (const StreamWin& win : t.wins)
      if ((t.rc = search_one_window(s, w, t, win, owned, t.err))) break;
  }
  if (!t.rc)
    for (const fac_match& m : owned) {
      t.res.push_back(m);
      t.res_text.insert(t.res_text.end(), t.text.begin() + (ptrdiff_t)(m.start - t.base),
                        t.text.begin() + (ptrdiff_t)(m.end - t.base));
    }
  std::vector<uint8_t>().swap(t.text);
}

void worker_loop(const StreamCore* s, StreamWorker* w) {
  (void)hipSetDevice(s->e->device);
  scratch_bind(&w->scratch);
  for (;;) {
    StreamTask* t = nullptr;
    {
      std::unique_lock<std::mutex> lk(w->mu);
      w->cv.wait(lk, [&] { return w->stop || !w->q.empty(); });
      if (w->q.empty()) break;  // stop requested and nothing queued
      t = w->q.front();
      w->q.pop_front();
    }
    try {  // an allocation failure becomes the window's error code, not std::terminate
      run_window_task(*s, *w, *t);
    } catch (const std::bad_alloc&) {
      t->rc = FAC_E_OOM;
      t->err = "out of host memory while searching a stream window";
    } catch (const std::exception& ex) {
      t->rc = FAC_E_INTERNAL;
      t->err = std::string("stream window: ") + ex.what();
    }
    {
      std::lock_guard<std::mutex> lk(g_done_mu);
      t->done = true;
    }
    g_done_cv.notify_all();
  }
  scratch_bind(nullptr);
}

// Hand out finished windows in order; `all`: wait for every window in flight.
int collect(StreamCore& s, bool all, std::string& err) {
  while (!s.inflight.empty()) {
    StreamTask* t = s.inflight.front();
    {
      std::unique_lock<std::mutex> lk(g_done_mu);
      if (!t->done && !all) return FAC_OK;
      g_done_cv.wait(lk, [&] { return t->done; });
    }
    s.inflight.erase(s.inflight.begin());
    if (!t->wins.empty()) s.handed = t->base + t->wins.back().off + t->wins.back().commit;
    if (t->rc && !s.failed) {
      s.failed = t->rc;
      s.fail_msg = t->err;
    }
    s.ready.insert(s.ready.end(), t->res.begin(), t->res.end());
    s.ready_text.insert(s.ready_text.end(), t->res_text.begin(), t->res_text.end());
    delete t;
  }
  if (s.failed) {
    err = s.fail_msg;
    return s.failed;
  }
  return FAC_OK;
}

int dispatch(StreamCore& s, StreamTask* t, std::string& err) {
  // the worker of this window finished its previous window (at most `depth` in flight)
  while (s.inflight.size() >= StreamCore::depth) {
    StreamTask* f = s.inflight.front();
    {
      std::unique_lock<std::mutex> lk(g_done_mu);
      g_done_cv.wait(lk, [&] { return f->done; });
    }
    if (int rc = collect(s, false, err)) {
      delete t;
      return rc;
    }
  }
  StreamWorker* w = s.workers[s.seq++ % StreamCore::depth];
  s.inflight.push_back(t);
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->q.push_back(t);
  }
  w->cv.notify_one();
  return FAC_OK;
}

// Cut windows while the buffer allows (next_window, stream.rs:102-158). The crate's reader reads
// 64 KiB pieces until it holds >= window bytes, so a window's text is the carry left by the previous
// window plus whole 64 KiB reads (the last one partial at the end of the input); fed in larger pieces,
// the buffer is cut the same way. Consecutive windows join the pending batch, dispatched once it holds
// kBatchBytes of text or the input ends.
constexpr uint64_t kRead = 64 * 1024, kBatchBytes = 32ull << 20;

int flush_batch(StreamCore& s, std::string& err) {
  if (!s.pending) return FAC_OK;
  StreamTask* t = s.pending;
  s.pending = nullptr;
  return dispatch(s, t, err);
}

int pump(StreamCore& s, bool eof, std::string& err) {
  // the buffer's unconsumed bytes start at `at` (the committed prefix is dropped once per call: an
  // erase per window moved the rest of a large feed again for every window)
  uint64_t at = 0;
  while (!s.done) {
    const uint8_t* b = s.buf.data() + at;
    const uint64_t avail = s.buf.size() - at;
    const uint64_t want = s.carry >= s.window ? s.carry : s.carry + (s.window - s.carry + kRead - 1) / kRead * kRead;
    if (!eof && avail < want) break;  // the reader would block for more input
    const uint64_t len = std::min(avail, want);
    // the valid UTF-8 prefix of the window's bytes; bytes a previous window already validated (up to
    // valid_end, a character boundary) are not scanned again
    const uint64_t vfrom = std::min<uint64_t>(len, s.valid_end > s.base ? s.valid_end - s.base : 0);
    const uint64_t valid = vfrom + utf8_valid_prefix(b + vfrom, len - vfrom);
    s.valid_end = s.base + valid;
    const bool last = len < s.window;  // reached only at end of input
    uint64_t commit = valid;
    if (!last) {
      // byte start of the overlap-th grapheme from the end; none or 0: grow and read more
      uint64_t off = 0;
      if (!nth_grapheme_from_end(b, valid, s.overlap, off) || off == 0) {
        s.window += std::max<uint64_t>(s.window, 64 * 1024);
        continue;  // (at end of input the next round is the last window)
      }
      commit = off;
    }
    if (!s.pending) {
      s.pending = new StreamTask();
      s.pending->base = s.base;
    }
    StreamTask* t = s.pending;
    const uint64_t off = s.base - t->base;  // the window's first byte in the batch text
    if (off + valid > t->text.size()) t->text.insert(t->text.end(), b + (t->text.size() - off), b + valid);
    t->wins.push_back(StreamWin{off, valid, commit});
    if (last) {
      s.done = true;
      break;
    }
    at += commit;
    s.base += commit;
    s.carry = len - commit;
    if (t->text.size() >= kBatchBytes)
      if (int rc = flush_batch(s, err)) {
        s.buf.erase(s.buf.begin(), s.buf.begin() + (ptrdiff_t)at);
        return rc;
      }
  }
  s.buf.erase(s.buf.begin(), s.buf.begin() + (ptrdiff_t)at);
  if (eof || s.done)
    if (int rc = flush_batch(s, err)) return rc;
  return collect(s, eof, err);
}

}  // namespace

int stream_feed(StreamCore& s, const uint8_t* data, uint64_t len, bool eof, std::string& err) {
  if (s.done) return collect(s, true, err);
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
  (void)hipSetDevice(e.device);
  for (uint32_t i = 0; i < StreamCore::depth; ++i) {
    StreamWorker* w = new StreamWorker();
    (void)hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking);
    w->th = std::thread(worker_loop, s, w);
    s->workers[i] = w;
  }
  return s;
}

void stream_close(StreamCore* s) {
  std::string err;
  delete s->pending;  // windows cut but never dispatched (an abandoned stream)
  s->pending = nullptr;
  (void)collect(*s, true, err);  // windows still in flight
  for (StreamWorker* w : s->workers) {
    if (!w) continue;
    {
      std::lock_guard<std::mutex> lk(w->mu);
      w->stop = true;
    }
    w->cv.notify_one();
    w->th.join();
    (void)hipSetDevice(s->e->device);
    scratch_free(w->scratch);
    if (w->stream) {
      call_scratch_release_stream(w->stream);
      (void)hipStreamDestroy(w->stream);
    }
    delete w;
  }
  delete s;
}

uint64_t stream_committed(const StreamCore& s) { return s.handed; }

}  // namespace fac
