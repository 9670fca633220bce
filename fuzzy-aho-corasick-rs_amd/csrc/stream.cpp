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
// Each cut window is handed to one of `depth` (2) worker threads, window k to worker k % depth. A
// worker owns a HIP stream and a device scratch set: it stages the window (H2D + device
// segmentation + folding), searches it as its own haystack, ranks it sorted().non_overlapping()
// and keeps the matches it owns (stream.rs:262-297), so window k + 1's copies and kernels overlap
// window k's (double buffering) while the host cuts window k + 2. Finished windows are handed out
// strictly in window order.
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

struct StreamTask {
  std::vector<uint8_t> text;  // the window's text (valid UTF-8 prefix of the buffer)
  uint64_t base = 0, commit = 0;
  std::vector<fac_match> res;  // owned matches, absolute offsets
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

// Search one window and keep the matches it owns (stream.rs:262-297).
void run_window_task(const StreamCore& s, StreamWorker& w, StreamTask& t) {
  Haystack h;
  t.rc = stage_haystack(*s.e, t.text.data(), t.text.size(), h, t.err, -1, w.stream);
  if (!t.rc) {
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
    t.rc = launch_search(*s.e, h, {seg}, s.threshold, w.stream, res, nullptr, t.err);
    if (!t.rc) t.rc = apply_matches(*s.e, res, /*Default*/ 1, /*NonOverlapping*/ 1, nullptr, t.err);
    if (!t.rc)
      for (const fac_match& m : res) {
        if (m.start >= t.commit) continue;
        fac_match a = m;
        a.start += t.base;
        a.end += t.base;
        t.res.push_back(a);
        t.res_text.insert(t.res_text.end(), t.text.begin() + (ptrdiff_t)m.start, t.text.begin() + (ptrdiff_t)m.end);
      }
  }
  free_haystack(h);
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
    s.handed = t->base + t->commit;
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

// Cut windows while the buffer allows (next_window, stream.rs:102-158).
int pump(StreamCore& s, bool eof, std::string& err) {
  while (!s.done && (eof || s.buf.size() >= s.window)) {
    const uint64_t valid = utf8_valid_prefix(s.buf.data(), s.buf.size());
    const bool last = s.buf.size() < s.window;  // reached only at end of input
    uint64_t commit = valid;
    if (!last) {
      // byte start of the overlap-th grapheme from the end; none or 0: grow and read more
      uint64_t off = 0;
      if (!nth_grapheme_from_end(s.buf.data(), valid, s.overlap, off) || off == 0) {
        s.window += std::max<uint64_t>(s.window, 64 * 1024);
        if (eof) continue;  // input ended: the next round is the last window
        return FAC_OK;
      }
      commit = off;
    }
    StreamTask* t = new StreamTask();
    t->text.assign(s.buf.begin(), s.buf.begin() + (ptrdiff_t)valid);
    t->base = s.base;
    t->commit = commit;
    if (int rc = dispatch(s, t, err)) return rc;
    if (last) {
      s.done = true;
      break;
    }
    s.buf.erase(s.buf.begin(), s.buf.begin() + (ptrdiff_t)commit);
    s.base += commit;
  }
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
  (void)collect(*s, true, err);  // windows still in flight (an abandoned stream)
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
