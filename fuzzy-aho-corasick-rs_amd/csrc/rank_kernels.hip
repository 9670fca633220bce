// rank_kernels.hip — ranking and overlap resolution of raw matches on the MI355X
// (FuzzyMatches::apply, src/matches.rs:7-149), the step right after the search path.
//
// * Orders (matches.rs:23-81) are total orders over (start, end, pattern_index)-unique records, so
//   a device merge sort (rocPRIM) with the same comparator reproduces the reference's
//   sort_unstable_by exactly.
// * non_overlapping (matches.rs:83-112) walks the ranked list and accepts a match iff it does not
//   intersect an accepted one (binary search on accepted starts). Two matches can only influence
//   each other's test if their spans touch, so the matches split — in start order, at every point
//   where a start lies strictly beyond all earlier ends — into clusters that are resolved
//   independently, one thread per cluster, each walking its members in rank order with the
//   reference's own test. Kept matches are re-sorted by start (ties: rank order).
// * non_overlapping_unique (matches.rs:114-149) adds a global "pattern used once" constraint, so it
//   runs on the host over the device-ranked list (O(n log n)).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include <rocprim/device/device_merge_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <mutex>
#include <set>
#include <unordered_set>
#include <vector>

#include "fac_internal.h"

namespace fac {
namespace {

// f32 total_cmp as an unsigned key (ascending key order == total order)
__device__ inline uint32_t total_key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

struct RankCmp {  // "a before b" for Order::{Default, Greedy, CoverageWeighted}
  const uint32_t* plen;  // pattern byte length (structs.rs:628-630: Pattern::len is bytes)
  int order;             // 1 default, 2 greedy, 3 coverage-weighted
  __device__ bool operator()(const fac_match& a, const fac_match& b) const {
    const uint32_t sa = total_key(a.similarity), sb = total_key(b.similarity);
    const uint32_t la = plen[a.pattern_index], lb = plen[b.pattern_index];
    if (order == 1) {  // matches.rs:24-38
      if (sa != sb) return sa > sb;
      if (la != lb) return la > lb;
      const uint64_t ta = a.end - a.start, tb = b.end - b.start;
      if (ta != tb) return ta > tb;
    } else if (order == 2) {  // matches.rs:43-57
      if (la != lb) return la > lb;
      if (sa != sb) return sa > sb;
    } else {  // matches.rs:63-81: similarity * similarity * len as f32, left to right
      const float ca = __fmul_rn(__fmul_rn(a.similarity, a.similarity), (float)la);
      const float cb = __fmul_rn(__fmul_rn(b.similarity, b.similarity), (float)lb);
      const uint32_t ka = total_key(ca), kb = total_key(cb);
      if (ka != kb) return ka > kb;
      if (sa != sb) return sa > sb;
    }
    if (a.start != b.start) return a.start < b.start;
    if (a.end != b.end) return a.end < b.end;
    return a.pattern_index < b.pattern_index;
  }
};

// The same order on the host (window_owned_device's small-window path): host f32 products are
// rounded once each like __fmul_rn (-ffp-contract=off), and the order is total, so std::sort
// gives the device sort's result
inline uint32_t total_key_host(float f) {
  uint32_t b;
  std::memcpy(&b, &f, 4);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
struct RankCmpHost {
  const uint32_t* plen;
  int order;
  bool operator()(const fac_match& a, const fac_match& b) const {
    const uint32_t sa = total_key_host(a.similarity), sb = total_key_host(b.similarity);
    const uint32_t la = plen[a.pattern_index], lb = plen[b.pattern_index];
    if (order == 1) {
      if (sa != sb) return sa > sb;
      if (la != lb) return la > lb;
      const uint64_t ta = a.end - a.start, tb = b.end - b.start;
      if (ta != tb) return ta > tb;
    } else if (order == 2) {
      if (la != lb) return la > lb;
      if (sa != sb) return sa > sb;
    } else {
      const volatile float a2 = a.similarity * a.similarity, b2 = b.similarity * b.similarity;
      const volatile float ca = a2 * (float)la, cb = b2 * (float)lb;
      const uint32_t ka = total_key_host(ca), kb = total_key_host(cb);
      if (ka != kb) return ka > kb;
      if (sa != sb) return sa > sb;
    }
    if (a.start != b.start) return a.start < b.start;
    if (a.end != b.end) return a.end < b.end;
    return a.pattern_index < b.pattern_index;
  }
};

struct Span {
  uint64_t start, end;
  uint32_t rank;     // position in the ranked list
  uint32_t cluster;  // filled after the start-order pass
};

struct SpanByStart {
  __host__ __device__ bool operator()(const Span& a, const Span& b) const {
    if (a.start != b.start) return a.start < b.start;
    if (a.end != b.end) return a.end < b.end;
    return a.rank < b.rank;
  }
};

struct SpanByClusterRank {
  __host__ __device__ bool operator()(const Span& a, const Span& b) const {
    if (a.cluster != b.cluster) return a.cluster < b.cluster;
    return a.rank < b.rank;
  }
};

struct KeptByStart {  // final sort_unstable_by_key(start); ties kept in acceptance (rank) order
  __host__ __device__ bool operator()(const Span& a, const Span& b) const {
    if (a.start != b.start) return a.start < b.start;
    return a.rank < b.rank;
  }
};

__global__ void spans_kernel(const fac_match* m, uint64_t n, Span* s) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) s[i] = Span{m[i].start, m[i].end, (uint32_t)i, 0u};
}

// cluster id = number of strict gaps before the element, in start order (max end by a scan)
__global__ void cluster_flags_kernel(const Span* s, const uint64_t* max_end_incl, uint64_t n, uint32_t* flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flag[i] = (i > 0 && s[i].start > max_end_incl[i - 1]) ? 1u : 0u;
}

__global__ void ends_kernel(const Span* s, uint64_t n, uint64_t* e) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) e[i] = s[i].end;
}

__global__ void assign_cluster_kernel(Span* s, const uint32_t* cid, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) s[i].cluster = cid[i];
}

// first member index of every cluster (members ordered by (cluster, rank))
__global__ void cluster_heads_kernel(const Span* s, uint64_t n, uint64_t* head) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (i == 0 || s[i].cluster != s[i - 1].cluster)) head[s[i].cluster] = i;
}

// One thread per cluster: the reference's walk (matches.rs:87-110) over the cluster's members in
// rank order; `occ` holds the cluster's accepted (start, end) sorted by start in the same index
// range as its members.
__global__ void resolve_kernel(const Span* s, const uint64_t* head, uint64_t n_clusters, uint64_t n, uint2* occ_lo,
                               uint2* occ_hi, uint8_t* keep) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_clusters) return;
  const uint64_t b = head[c], e = (c + 1 < n_clusters) ? head[c + 1] : n;
  uint64_t k = 0;  // accepted so far
  for (uint64_t i = b; i < e; ++i) {
    const uint64_t ms = s[i].start, me = s[i].end;
    uint64_t lo = 0, hi = k;  // bisect_left on accepted starts
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      const uint64_t st = ((uint64_t)occ_hi[b + mid].x << 32) | occ_lo[b + mid].x;
      if (st < ms) lo = mid + 1;
      else hi = mid;
    }
    const uint64_t pos = lo;
    const bool prev_ok = pos == 0 || ((((uint64_t)occ_hi[b + pos - 1].y << 32) | occ_lo[b + pos - 1].y) <= ms);
    const bool next_ok = pos == k || ((((uint64_t)occ_hi[b + pos].x << 32) | occ_lo[b + pos].x) >= me);
    if (prev_ok && next_ok) {
      for (uint64_t t = k; t > pos; --t) {
        occ_lo[b + t] = occ_lo[b + t - 1];
        occ_hi[b + t] = occ_hi[b + t - 1];
      }
      occ_lo[b + pos] = make_uint2((uint32_t)ms, (uint32_t)me);
      occ_hi[b + pos] = make_uint2((uint32_t)(ms >> 32), (uint32_t)(me >> 32));
      ++k;
      keep[s[i].rank] = 1;
    }
  }
}

__global__ void kept_spans_kernel(const fac_match* m, const uint8_t* keep, const uint32_t* pos, uint64_t n, Span* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && keep[i]) out[pos[i] - 1] = Span{m[i].start, m[i].end, (uint32_t)i, 0u};
}

__global__ void gather_kernel(const fac_match* m, const Span* order, uint64_t n, fac_match* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = m[order[i].rank];
}

#define RK_TRY(x)                                                   \
  do {                                                              \
    hipError_t _e = (x);                                            \
    if (_e != hipSuccess) {                                         \
      err = std::string(#x ": ") + hipGetErrorString(_e);           \
      return FAC_E_HIP;                                             \
    }                                                               \
  } while (0)

// stream-ordered call scratch (call_scratch_take): every use below is on the stream it was taken for
thread_local hipStream_t t_buf_stream = nullptr;
struct Buf {
  void* p = nullptr;
  hipStream_t s = t_buf_stream;
  ~Buf() {
    if (p) call_scratch_give(p, s);
  }
  hipError_t alloc(size_t bytes) {
    hipError_t e = hipSuccess;
    p = call_scratch_take(bytes, s, &e);
    return e;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

template <class T, class Cmp>
hipError_t dev_sort(T* in, T* out, uint64_t n, Cmp cmp, hipStream_t s) {
  size_t bytes = 0;
  hipError_t e = rocprim::merge_sort(nullptr, bytes, in, out, n, cmp, s);
  if (e != hipSuccess) return e;
  Buf tmp;
  if ((e = tmp.alloc(bytes)) != hipSuccess) return e;
  return rocprim::merge_sort(tmp.p, bytes, in, out, n, cmp, s);
}

constexpr uint64_t kMaxCluster = 1u << 14;  // larger clusters: the host walk (O(n log n))
constexpr uint64_t kHostRank = 1u << 14;    // window_owned_device: fewer records are ranked on the host

// The reference's non_overlapping(_unique) walk (matches.rs:83-149) on the host.
void walk_host(std::vector<fac_match>& v, const uint64_t* unique_ids, bool unique) {
  std::multiset<std::pair<uint64_t, uint64_t>> occ;  // (start, end) by start
  std::unordered_set<uint64_t> used;
  std::vector<std::pair<uint64_t, uint32_t>> kept;  // (start, rank)
  for (uint32_t r = 0; r < v.size(); ++r) {
    const fac_match& m = v[r];
    const uint64_t uid = unique_ids ? unique_ids[m.pattern_index] : m.pattern_index;
    if (unique && used.count(uid)) continue;
    auto it = occ.lower_bound({m.start, 0});  // bisect_left on starts
    const bool next_ok = it == occ.end() || it->first >= m.end;
    const bool prev_ok = it == occ.begin() || std::prev(it)->second <= m.start;
    if (prev_ok && next_ok) {
      occ.insert(it, {m.start, m.end});
      if (unique) used.insert(uid);
      kept.push_back({m.start, r});
    }
  }
  std::stable_sort(kept.begin(), kept.end(), [](auto& a, auto& b) { return a.first < b.first; });
  std::vector<fac_match> out;
  out.reserve(kept.size());
  for (auto& k : kept) out.push_back(v[k.second]);
  v.swap(out);
}

}  // namespace

// Device-resident core: the n records at d_a (device) are ranked / resolved; d_b is scratch of n
// records. *res points at the result (d_a or d_b), *n_res its count. The host walks (unique overlap,
// clusters above kMaxCluster) bring the ranked list to the host and put their result back into d_a.
int apply_matches_device(const Engine& e, fac_match* d_a, fac_match* d_b, uint64_t n, int order, int overlap,
                         const uint64_t* unique_ids, hipStream_t s, fac_match** res, uint64_t* n_res, std::string& err) {
  *res = d_a;
  *n_res = n;
  if (n == 0 || (order == 0 && overlap == 0)) return FAC_OK;
  t_buf_stream = s;
  const uint32_t T = 256;
  const uint32_t G = (uint32_t)((n + T - 1) / T);
  fac_match* ranked = d_a;
  if (order != 0) {
    RK_TRY(dev_sort(d_a, d_b, n, RankCmp{e.d_pat_bytes, order}, s));
    ranked = d_b;
  }
  auto host_walk = [&](bool unique) -> int {
    std::vector<fac_match> v(n);
    RK_TRY(hipMemcpyAsync(v.data(), ranked, n * sizeof(fac_match), hipMemcpyDeviceToHost, s));
    RK_TRY(hipStreamSynchronize(s));
    walk_host(v, unique_ids, unique);
    if (!v.empty()) RK_TRY(hipMemcpyAsync(d_a, v.data(), v.size() * sizeof(fac_match), hipMemcpyHostToDevice, s));
    RK_TRY(hipStreamSynchronize(s));
    *res = d_a;
    *n_res = v.size();
    return FAC_OK;
  };
  if (overlap == 0) {
    *res = ranked;
    return FAC_OK;
  }
  if (overlap == 2) return host_walk(true);  // the unique walk on the host
  // ---- non_overlapping: clusters in start order, resolved one thread per cluster
  Buf d_sp, d_sp2, d_ends, d_maxe, d_flag, d_cid, d_head, d_lo, d_hi, d_keep, d_pos, d_kept;
  RK_TRY(d_sp.alloc(n * sizeof(Span)));
  RK_TRY(d_sp2.alloc(n * sizeof(Span)));
  hipLaunchKernelGGL(spans_kernel, dim3(G), dim3(T), 0, s, ranked, n, d_sp.as<Span>());
  RK_TRY(dev_sort(d_sp.as<Span>(), d_sp2.as<Span>(), n, SpanByStart{}, s));
  RK_TRY(d_ends.alloc(n * 8));
  RK_TRY(d_maxe.alloc(n * 8));
  hipLaunchKernelGGL(ends_kernel, dim3(G), dim3(T), 0, s, d_sp2.as<Span>(), n, d_ends.as<uint64_t>());
  {
    size_t bytes = 0;
    RK_TRY(rocprim::inclusive_scan(nullptr, bytes, d_ends.as<uint64_t>(), d_maxe.as<uint64_t>(), n,
                                   rocprim::maximum<uint64_t>(), s));
    Buf tmp;
    RK_TRY(tmp.alloc(bytes));
    RK_TRY(rocprim::inclusive_scan(tmp.p, bytes, d_ends.as<uint64_t>(), d_maxe.as<uint64_t>(), n,
                                   rocprim::maximum<uint64_t>(), s));
  }
  RK_TRY(d_flag.alloc(n * 4));
  RK_TRY(d_cid.alloc(n * 4));
  hipLaunchKernelGGL(cluster_flags_kernel, dim3(G), dim3(T), 0, s, d_sp2.as<Span>(), d_maxe.as<uint64_t>(), n,
                     d_flag.as<uint32_t>());
  {
    size_t bytes = 0;
    RK_TRY(rocprim::inclusive_scan(nullptr, bytes, d_flag.as<uint32_t>(), d_cid.as<uint32_t>(), n,
                                   rocprim::plus<uint32_t>(), s));
    Buf tmp;
    RK_TRY(tmp.alloc(bytes));
    RK_TRY(rocprim::inclusive_scan(tmp.p, bytes, d_flag.as<uint32_t>(), d_cid.as<uint32_t>(), n,
                                   rocprim::plus<uint32_t>(), s));
  }
  hipLaunchKernelGGL(assign_cluster_kernel, dim3(G), dim3(T), 0, s, d_sp2.as<Span>(), d_cid.as<uint32_t>(), n);
  RK_TRY(dev_sort(d_sp2.as<Span>(), d_sp.as<Span>(), n, SpanByClusterRank{}, s));
  uint32_t last_cid = 0;
  RK_TRY(hipMemcpyAsync(&last_cid, d_cid.as<uint32_t>() + (n - 1), 4, hipMemcpyDeviceToHost, s));
  RK_TRY(hipStreamSynchronize(s));
  const uint64_t n_clusters = (uint64_t)last_cid + 1;
  RK_TRY(d_head.alloc(n_clusters * 8));
  hipLaunchKernelGGL(cluster_heads_kernel, dim3(G), dim3(T), 0, s, d_sp.as<Span>(), n, d_head.as<uint64_t>());
  {  // largest cluster: a thread's walk is quadratic in its cluster, keep it bounded
    std::vector<uint64_t> heads(n_clusters);
    RK_TRY(hipMemcpyAsync(heads.data(), d_head.p, n_clusters * 8, hipMemcpyDeviceToHost, s));
    RK_TRY(hipStreamSynchronize(s));
    uint64_t biggest = 0;
    for (uint64_t c = 0; c < n_clusters; ++c) biggest = std::max(biggest, (c + 1 < n_clusters ? heads[c + 1] : n) - heads[c]);
    if (biggest > kMaxCluster) return host_walk(false);
  }
  RK_TRY(d_lo.alloc(n * sizeof(uint2)));
  RK_TRY(d_hi.alloc(n * sizeof(uint2)));
  RK_TRY(d_keep.alloc(n));
  RK_TRY(hipMemsetAsync(d_keep.p, 0, n, s));
  hipLaunchKernelGGL(resolve_kernel, dim3((uint32_t)((n_clusters + T - 1) / T)), dim3(T), 0, s, d_sp.as<Span>(),
                     d_head.as<uint64_t>(), n_clusters, n, d_lo.as<uint2>(), d_hi.as<uint2>(), d_keep.as<uint8_t>());
  // compact the kept matches (rank order), then order them by start
  RK_TRY(d_pos.alloc(n * 4));
  {
    size_t bytes = 0;
    RK_TRY(rocprim::inclusive_scan(nullptr, bytes, d_keep.as<uint8_t>(), d_pos.as<uint32_t>(), n,
                                   rocprim::plus<uint32_t>(), s));
    Buf tmp;
    RK_TRY(tmp.alloc(bytes));
    RK_TRY(rocprim::inclusive_scan(tmp.p, bytes, d_keep.as<uint8_t>(), d_pos.as<uint32_t>(), n,
                                   rocprim::plus<uint32_t>(), s));
  }
  uint32_t kept = 0;
  RK_TRY(hipMemcpyAsync(&kept, d_pos.as<uint32_t>() + (n - 1), 4, hipMemcpyDeviceToHost, s));
  RK_TRY(hipStreamSynchronize(s));
  *n_res = kept;
  if (kept == 0) return FAC_OK;
  RK_TRY(d_kept.alloc((uint64_t)kept * sizeof(Span)));
  hipLaunchKernelGGL(kept_spans_kernel, dim3(G), dim3(T), 0, s, ranked, d_keep.as<uint8_t>(), d_pos.as<uint32_t>(), n,
                     d_kept.as<Span>());
  RK_TRY(dev_sort(d_kept.as<Span>(), d_sp2.as<Span>(), kept, KeptByStart{}, s));
  fac_match* out = (ranked == d_a) ? d_b : d_a;
  hipLaunchKernelGGL(gather_kernel, dim3((kept + T - 1) / T), dim3(T), 0, s, ranked, d_sp2.as<Span>(), (uint64_t)kept,
                     out);
  RK_TRY(hipGetLastError());
  *res = out;
  return FAC_OK;
}

int apply_matches(const Engine& e, std::vector<fac_match>& v, int order, int overlap, const uint64_t* unique_ids,
                  std::string& err) {
  const uint64_t n = v.size();
  if (n == 0 || (order == 0 && overlap == 0)) return FAC_OK;
  RK_TRY(hipSetDevice(e.device));
  hipStream_t s = e.stream;
  t_buf_stream = s;
  Buf d_a, d_b;
  RK_TRY(d_a.alloc(n * sizeof(fac_match)));
  RK_TRY(d_b.alloc(n * sizeof(fac_match)));
  RK_TRY(hipMemcpyAsync(d_a.p, v.data(), n * sizeof(fac_match), hipMemcpyHostToDevice, s));
  fac_match* res = nullptr;
  uint64_t nres = 0;
  if (int rc = apply_matches_device(e, d_a.as<fac_match>(), d_b.as<fac_match>(), n, order, overlap, unique_ids, s, &res,
                                    &nres, err))
    return rc;
  v.resize(nres);
  if (nres) RK_TRY(hipMemcpyAsync(v.data(), res, nres * sizeof(fac_match), hipMemcpyDeviceToHost, s));
  RK_TRY(hipStreamSynchronize(s));
  return FAC_OK;
}

// stream.rs window_matches' ownership on the device: of a window's records ranked sorted().
// non_overlapping() (start order), the ones starting before the commit point (a prefix), rebased
// from the window's bytes to the stream offset `base`, go to out[0 .. owned).
__global__ void owned_kernel(const fac_match* in, uint64_t n, uint64_t byte_base, uint64_t commit, uint64_t base,
                             fac_match* out, unsigned long long* owned) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fac_match m = in[i];
  const uint64_t st = m.start - byte_base;
  const bool own = st < commit;
  if (own) {
    m.start = st + base;
    m.end = m.end - byte_base + base;
    out[i] = m;
  }
  const uint64_t b = __ballot(own);
  if (b && (threadIdx.x & 63u) == (uint32_t)(__ffsll((unsigned long long)b) - 1)) atomicAdd(owned, (unsigned long long)__popcll(b));
}

int window_owned_device(const Engine& e, fac_match* d_a, fac_match* d_b, uint64_t n, uint64_t byte_base, uint64_t commit,
                        uint64_t base, hipStream_t s, fac_match* d_out, uint64_t cap, uint64_t* n_owned, std::string& err) {
  *n_owned = 0;
  if (n == 0) return FAC_OK;
  if (n <= kHostRank) {  // few records (C5: ~1 000 per 1 GiB window): ranked on the host, not by ~20 launches
    std::vector<fac_match> v(n);
    RK_TRY(hipMemcpyAsync(v.data(), d_a, n * sizeof(fac_match), hipMemcpyDeviceToHost, s));
    RK_TRY(hipStreamSynchronize(s));
    std::sort(v.begin(), v.end(), RankCmpHost{e.pat_bytes.data(), 1});
    walk_host(v, nullptr, false);  // non_overlapping, start order
    uint64_t owned = 0;
    for (const fac_match& m0 : v) {
      const uint64_t st = m0.start - byte_base;
      if (st >= commit) continue;
      fac_match m = m0;
      m.start = st + base;
      m.end = m.end - byte_base + base;
      v[owned++] = m;
    }
    *n_owned = owned;
    if (owned > cap) return FAC_E_OUTPUT_CAPACITY;
    if (owned) RK_TRY(hipMemcpyAsync(d_out, v.data(), owned * sizeof(fac_match), hipMemcpyHostToDevice, s));
    RK_TRY(hipStreamSynchronize(s));
    return FAC_OK;
  }
  fac_match* res = nullptr;
  uint64_t nres = 0;
  if (int rc = apply_matches_device(e, d_a, d_b, n, 1, 1, nullptr, s, &res, &nres, err)) return rc;
  if (nres == 0) return FAC_OK;
  t_buf_stream = s;
  // the owned count first (a prefix of the start-ordered list), then the copy if it fits
  Buf d_cnt, d_tmp;
  RK_TRY(d_cnt.alloc(8));
  RK_TRY(d_tmp.alloc(nres * sizeof(fac_match)));
  RK_TRY(hipMemsetAsync(d_cnt.p, 0, 8, s));
  const uint32_t T = 256;
  hipLaunchKernelGGL(owned_kernel, dim3((uint32_t)((nres + T - 1) / T)), dim3(T), 0, s, res, nres, byte_base, commit, base,
                     d_tmp.as<fac_match>(), d_cnt.as<unsigned long long>());
  RK_TRY(hipGetLastError());
  unsigned long long owned = 0;
  RK_TRY(hipMemcpyAsync(&owned, d_cnt.p, 8, hipMemcpyDeviceToHost, s));
  RK_TRY(hipStreamSynchronize(s));
  *n_owned = owned;
  if (owned > cap) return FAC_E_OUTPUT_CAPACITY;
  if (owned) RK_TRY(hipMemcpyAsync(d_out, d_tmp.p, owned * sizeof(fac_match), hipMemcpyDeviceToDevice, s));
  RK_TRY(hipStreamSynchronize(s));
  return FAC_OK;
}

// A batch of stream windows' raw records (start and end tagged with the window, kWinTagShift): per window,
// sorted().non_overlapping() and the matches starting before its commit point, rebased to stream
// offsets (stream.rs:262-297), appended to `out` in window order with the tag cleared.
void windows_owned_host(const Engine& e, std::vector<fac_match>& recs, const std::vector<WinOwn>& wins,
                        std::vector<fac_match>& out) {
  const size_t nw = wins.size();
  std::vector<uint64_t> first(nw + 1, 0);
  auto tag = [](const fac_match& m) { return (uint32_t)(m.start >> kWinTagShift); };
  constexpr uint64_t low = (1ull << kWinTagShift) - 1;
  for (const fac_match& m : recs) ++first[tag(m) + 1];
  for (size_t w = 0; w < nw; ++w) first[w + 1] += first[w];
  std::vector<fac_match> by(recs.size());
  {
    std::vector<uint64_t> at(first.begin(), first.end() - 1);
    for (const fac_match& m : recs) {
      fac_match u = m;
      u.start &= low;
      u.end &= low;
      by[at[tag(m)]++] = u;
    }
  }
  std::vector<fac_match> v;
  for (size_t w = 0; w < nw; ++w) {
    if (first[w] == first[w + 1]) continue;
    v.assign(by.begin() + (ptrdiff_t)first[w], by.begin() + (ptrdiff_t)first[w + 1]);
    std::sort(v.begin(), v.end(), RankCmpHost{e.pat_bytes.data(), 1});
    walk_host(v, nullptr, false);  // non_overlapping, start order
    for (fac_match m : v) {
      const uint64_t st = m.start - wins[w].byte_base;
      if (st >= wins[w].commit) continue;
      m.start = st + wins[w].base;
      m.end = m.end - wins[w].byte_base + wins[w].base;
      out.push_back(m);
    }
  }
}

namespace {
// One pool per process (not per thread: a stream's blocks must be found again by whoever destroys
// the stream), keyed by (device, stream, size class). Size classes are powers of two up to 64 MiB
// and 16 MiB multiples above, so a 0.5 GB block is not rounded to 1 GiB. Given-back blocks are kept
// up to kPoolCap bytes in all (the oldest go first); call_scratch_release_stream frees a stream's
// blocks before the library destroys that stream (a new stream may get the same handle), and
// fac_trim_scratch frees every kept block.
struct CallBlock {
  void* p;
  size_t bytes;
  hipStream_t s;
  int device;
};
constexpr size_t kPoolCap = size_t(2) << 30;
struct CallPool {
  std::mutex mu;
  std::vector<CallBlock> free_blocks;  // oldest first
  std::vector<CallBlock> live;         // handed out: their sizes for the give-back
  size_t free_bytes = 0;
  void drop_front_locked() {
    (void)hipFree(free_blocks.front().p);  // hipFree orders after the block's stream work
    free_bytes -= free_blocks.front().bytes;
    free_blocks.erase(free_blocks.begin());
  }
};
CallPool& call_pool() {
  static CallPool* p = new CallPool();  // never destroyed: blocks outlive static destructors' order
  return *p;
}
size_t size_class(size_t bytes) {
  if (bytes > (size_t(64) << 20)) return (bytes + (size_t(16) << 20) - 1) & ~((size_t(16) << 20) - 1);
  size_t cls = 256;
  while (cls < bytes) cls <<= 1;
  return cls;
}
}  // namespace

void* call_scratch_take(size_t bytes, hipStream_t s, hipError_t* e) {
  const size_t cls = size_class(bytes);
  int dev = 0;
  (void)hipGetDevice(&dev);
  CallPool& pool = call_pool();
  {
    std::lock_guard<std::mutex> lk(pool.mu);
    auto& fb = pool.free_blocks;
    for (size_t i = fb.size(); i-- > 0;)  // newest first: likeliest to be warm
      if (fb[i].s == s && fb[i].bytes == cls && fb[i].device == dev) {
        const CallBlock b = fb[i];
        fb.erase(fb.begin() + (ptrdiff_t)i);
        pool.free_bytes -= b.bytes;
        pool.live.push_back(b);
        *e = hipSuccess;
        return b.p;
      }
  }
  void* p = nullptr;
  *e = hipMalloc(&p, cls);
  if (*e != hipSuccess) {  // kept blocks may be what fills the device: free them and retry once
    call_scratch_trim();
    *e = hipMalloc(&p, cls);
    if (*e != hipSuccess) return nullptr;
  }
  std::lock_guard<std::mutex> lk(pool.mu);
  pool.live.push_back(CallBlock{p, cls, s, dev});
  return p;
}

void call_scratch_give(void* p, hipStream_t s) {
  CallPool& pool = call_pool();
  std::lock_guard<std::mutex> lk(pool.mu);
  for (size_t i = 0; i < pool.live.size(); ++i)
    if (pool.live[i].p == p) {
      CallBlock b = pool.live[i];
      pool.live[i] = pool.live.back();
      pool.live.pop_back();
      b.s = s;
      pool.free_blocks.push_back(b);
      pool.free_bytes += b.bytes;
      while (pool.free_blocks.size() > 64 || (pool.free_bytes > kPoolCap && pool.free_blocks.size() > 1))
        pool.drop_front_locked();
      return;
    }
  (void)hipFree(p);  // not from the pool
}

void call_scratch_trim() {
  CallPool& pool = call_pool();
  std::lock_guard<std::mutex> lk(pool.mu);
  while (!pool.free_blocks.empty()) pool.drop_front_locked();
}

void call_scratch_release_stream(hipStream_t s) {
  CallPool& pool = call_pool();
  std::lock_guard<std::mutex> lk(pool.mu);
  auto& fb = pool.free_blocks;
  for (size_t i = 0; i < fb.size();)
    if (fb[i].s == s) {
      (void)hipFree(fb[i].p);
      pool.free_bytes -= fb[i].bytes;
      fb.erase(fb.begin() + (ptrdiff_t)i);
    } else {
      ++i;
    }
}

}  // namespace fac
