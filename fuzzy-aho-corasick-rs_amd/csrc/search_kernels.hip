// search_kernels.hip — CDNA4 (gfx950) kernels for the per-start-window fuzzy automaton search
// and the bit-parallel pre-filter.
//
// Reference hot path: FuzzyAhoCorasick::search_unsorted_impl (src/search.rs:418-1119). For every
// grapheme position `start` the reference restarts a FIFO breadth-first exploration of
// (node, j, matched_end, penalties, edit counts) states from the trie root, deduplicates states
// per window (search.rs:608-628), prunes against per-node ceilings (:638-642), emits
// best-per-(start,end,pattern) matches (:659-737) and fans out exact / substitution / swap /
// insertion / deletion successors (:742-1089), optionally beaming the frontier (:577-589).
//
// MI355X mapping:
//   * windows are independent (the best-map key holds the start byte), so they are the unit of
//     parallelism; `bfs_window_kernel` gives each start window to ONE wavefront;
//   * the wave pops states in exact FIFO order (so beam cuts and dedup see the reference's
//     sequence), while its 64 lanes evaluate the popped state's edges in parallel; pushes are
//     compacted in edge order with ballot + mbcnt, so the queue order equals the reference's
//     push order;
//   * the frontier ring and the dedup table live in LDS (per-wave slices), probed 64 slots at a
//     time; per-node data is read with wave-uniform loads from L2-resident tables;
//   * every f32 expression keeps the reference's operation order with no contraction
//     (-ffp-contract=off plus explicit __fmul_rn/__fsub_rn/__fadd_rn/__fdiv_rn).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <type_traits>
#include <tuple>
#include <vector>

#include "fac_internal.h"

namespace fac {
namespace {

constexpr uint32_t EMPTY = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t prefix_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
// Reads from a wave-uniform lane: v_readlane (scalar path), not ds_bpermute through the LDS unit.
__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ float shfl_f32(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int l) {
  const uint32_t lo = shfl_u32((uint32_t)v, l), hi = shfl_u32((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int first_lane(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }

// err flags are set identically by every lane inside a window; a ballot is enough to test them.
__device__ __forceinline__ bool any_err(unsigned err) { return __ballot(err != 0) != 0; }

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

// Wave-wide minimum with DPP row shifts + row broadcasts (no LDS round trip); result is uniform.
__device__ __forceinline__ uint64_t shfl_var_u64(uint64_t v, int src) {  // per-lane source (ds_bpermute)
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}

// f32 -> u32 preserving the order of every non-NaN value: penalties compared as u32
__device__ __forceinline__ uint32_t pen_order(float f) {
  uint32_t b = __float_as_uint(f);
  b = b == 0x80000000u ? 0u : b;  // -0 == +0, as the reference's <= compares them
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  const int I = -1;  // identity for unsigned min (0xFFFFFFFF)
  int x = (int)v;
  x = (int)min((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(I, x, 0x111, 0xF, 0xF, false));  // row_shr:1
  x = (int)min((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(I, x, 0x112, 0xF, 0xF, false));  // row_shr:2
  x = (int)min((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(I, x, 0x114, 0xF, 0xF, false));  // row_shr:4
  x = (int)min((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(I, x, 0x118, 0xF, 0xF, false));  // row_shr:8
  x = (int)min((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(I, x, 0x142, 0xA, 0xF, false));  // row_bcast:15
  x = (int)min((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(I, x, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane(x, 63);
}

__device__ __forceinline__ uint32_t edits_of(uint32_t packed) {
  return (packed & 0xFFu) + ((packed >> 8) & 0xFFu) + ((packed >> 16) & 0xFFu) + (packed >> 24);
}

__device__ __forceinline__ uint32_t total_order_key(float f) {  // f32::total_cmp as a u32 order
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ bool lim_lt(int32_t m, uint32_t v) { return m == LIM_NONE || (int32_t)v < m; }
__device__ __forceinline__ bool lim_le(int32_t m, uint32_t v) { return m == LIM_NONE || (int32_t)v <= m; }

struct Lim {  // Option<&FuzzyLimits> by value
  bool has;
  DevLimits l;
};

// limits.or(self.limits.as_ref()) (search.rs:93, 109, 125, 140, 160); `pi` = pattern whose limits
// apply (-1 = None)
__device__ __forceinline__ Lim pick_limits(const SearchParams& P, int32_t pi) {
  if (pi >= 0) return Lim{true, P.pats[pi].lim};
  return Lim{P.has_glim != 0, P.glim};
}

// get_node_limits (search.rs:67-71): the node's pattern, if that pattern has its own limits
__device__ __forceinline__ int32_t node_limits(const SearchParams& P, uint32_t node) {
  const int32_t pi = P.node_pidx[node];
  if (pi < 0) return -1;
  return P.pats[pi].has_limits ? pi : -1;
}

// get_similarity (search.rs:76-82) -> Similarity::get (structs.rs:82-92)
__device__ __forceinline__ float similarity(const SearchParams& P, uint32_t a, uint32_t b) {
  if (a == b) return 1.0f;
  if (a < 128u && b < 128u) return P.sim_ascii[a * 128u + b];
  if (P.n_sim == 0) return 0.0f;
  const uint64_t key = ((uint64_t)a << 32) | b;
  uint32_t lo = 0, hi = P.n_sim;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P.sim_keys[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return (lo < P.n_sim && P.sim_keys[lo] == key) ? P.sim_vals[lo] : 0.0f;
}

// text_chars[j] of the (sub)haystack (search.rs:203/302 + grapheme.rs:66-68, 112-119)
__device__ __forceinline__ uint32_t text_char(const SearchParams& P, const SegDesc& S, uint64_t j, unsigned& err) {
  if (j >= S.avail) {  // beyond this shard's resident halo: host bug, flag it
    err |= ERR_HALO;
    return 0;
  }
  if (S.ascii) {
    uint32_t b = P.utf8[S.text_base + j];
    if (P.case_insensitive && b - 'A' < 26u) b += 32u;
    return b;
  }
  return P.text32[S.text_base + j];
}

// id of the whole folded grapheme at j (gs_text, grapheme.rs:61-63, 100-109), engines with
// mappings only: 0 = not in the engine's grapheme dictionary (equal to no edge or mapping side)
__device__ __forceinline__ uint32_t text_gid(const SearchParams& P, const SegDesc& S, uint64_t j, unsigned& err) {
  if (j >= S.avail) {
    err |= ERR_HALO;
    return 0;
  }
  if (S.ascii) return P.ascii_gid[P.utf8[S.text_base + j] & 0x7Fu];
  return P.gid32[S.text_base + j];
}

// Node::find_transition for a whole grapheme (structs.rs:452-464) by id: the edge whose grapheme
// is the text grapheme (a one-byte grapheme can only equal a single-byte edge), -1 if none
__device__ __forceinline__ int64_t find_gid(const SearchParams& P, uint32_t node, uint32_t gid) {
  if (gid == 0) return -1;
  const DevNode nd = P.nodes[node];
  for (uint32_t e = nd.edge_begin; e < nd.edge_begin + (nd.degf & NODE_DEG_MASK); ++e)
    if (P.edge_gid[e] == gid) return (int64_t)(P.edges[e].next & EDGE_NEXT_MASK);
  return -1;
}

// Multi-character mappings applicable at (node, j) (search.rs:883-922): bit t = the node's t-th
// transition consumes text[j .. j + hlen) and stays within max_penalties
__device__ uint64_t map_mask(const SearchParams& P, const SegDesc& S, uint32_t node, uint64_t j, float pen,
                             unsigned& err) {
  const uint2 r = P.map_range[node];
  uint64_t m = 0;
  for (uint32_t t = r.x; t < r.y; ++t) {
    const uint4 mt = P.map_ent[t];
    if (j + mt.y > S.n) continue;
    bool ok = true;
    for (uint32_t k = 0; k < mt.y && ok; ++k) ok = text_gid(P, S, j + k, err) == P.map_hay[mt.x + k];
    if (!ok || __fadd_rn(pen, __uint_as_float(mt.w)) > P.max_penalties) continue;
    m |= 1ull << (t - r.x);
  }
  return m;
}

// gs_byte_offset, relative to the (sub)haystack (grapheme.rs:59-61, 95-97)
__device__ __forceinline__ uint64_t local_byte(const SearchParams& P, const SegDesc& S, uint64_t g) {
  if (S.ascii) return g;
  return P.off[S.text_base + g] - S.byte_base;
}

// has_matching_edge_char (structs.rs:471-475) via the node's single-byte edge bitmap
__device__ __forceinline__ bool sb_has(const SearchParams& P, uint32_t node, uint32_t ch) {
  if (ch >= 128u) return false;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&P.nodes[node].sb);
  return (w[ch >> 5] >> (ch & 31u)) & 1u;
}

__device__ __forceinline__ uint32_t node_deg(const DevNode& n) { return n.degf & NODE_DEG_MASK; }
__device__ __forceinline__ uint32_t node_end(const DevNode& n) { return n.edge_begin + (n.degf & NODE_DEG_MASK); }
__device__ __forceinline__ bool node_has_out(const DevNode& n) { return (n.degf & NODE_HAS_OUT) != 0; }

// goto-table lookup (fac_internal.h): both cuckoo slots read at once, branch-free
__device__ __forceinline__ bool gt_get_h(const SearchParams& P, uint64_t kv, uint32_t h, bool live, uint64_t& val) {
  uint32_t s1, s2;
  gt_slots_h(h, P.gt_mask, s1, s2);
  const uint4 a = P.gt[live ? s1 : 0u];
  const uint4 b = P.gt[live ? s2 : 0u];
  const uint32_t lo = (uint32_t)kv, hi = (uint32_t)(kv >> 32);
  const bool ma = a.x == lo && a.y == hi, mb = b.x == lo && b.y == hi;
  val = ma ? (((uint64_t)a.w << 32) | a.z) : mb ? (((uint64_t)b.w << 32) | b.z) : 0ull;
  return live && (ma || mb);
}
__device__ __forceinline__ bool gt_get(const SearchParams& P, uint64_t kv, bool live, uint64_t& val) {
  const uint32_t node = (uint32_t)((kv >> 21) & CHILD26_MASK), ch = (uint32_t)(kv & 0x1FFFFFu);
  return gt_get_h(P, kv, gt_kind_hash(gt_base(node, ch, P.gt_seed1), (kv & GT_SB) != 0), live, val);
}

// find_transition_char_no_mappings (structs.rs:512-519): first edge whose first char is `ch`
__device__ __forceinline__ int64_t goto_char(const SearchParams& P, uint32_t eb, uint32_t ee, uint32_t ch) {
  const uint32_t lane = lane_id();
  for (uint32_t base = eb; base < ee; base += 64) {
    const uint32_t i = base + lane;
    const bool valid = i < ee;
    const DevEdge ed = valid ? P.edges[i] : DevEdge{0, 0};
    const uint64_t m = __ballot(valid && ed.ch == ch);
    if (m) return (int64_t)(shfl_u32(ed.next, first_lane(m)) & EDGE_NEXT_MASK);
  }
  return -1;
}

// Per-wave best map for one window (search.rs:444, 705-735), in global scratch: the start byte is
// fixed per window so the key is (matched_end, pattern). Entries: x = me_rel, y = pattern,
// z = similarity bits, w = packed counts. First-found wins ties; strictly greater replaces.
struct EmitList {
  uint4* buf;
  uint32_t cap;
  uint32_t n;
};

__device__ __forceinline__ void wave_mem_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); }

__device__ void emit_update(EmitList& L, uint32_t me_rel, uint32_t p, float sim, uint32_t packed, unsigned& err) {
  const uint32_t lane = lane_id();
  wave_mem_fence();
  for (uint32_t base = 0; base < L.n; base += 64) {
    const uint32_t i = base + lane;
    uint4 ent = make_uint4(EMPTY, EMPTY, 0, 0);
    if (i < L.n) ent = L.buf[i];
    const uint64_t m = __ballot(i < L.n && ent.x == me_rel && ent.y == p);
    if (m) {
      const int l = first_lane(m);
      const float old = __uint_as_float(shfl_u32(ent.z, l));
      if (sim > old && lane == (uint32_t)l) L.buf[i] = make_uint4(me_rel, p, __float_as_uint(sim), packed);
      wave_mem_fence();
      return;
    }
  }
  if (L.n >= L.cap) {
    err |= ERR_EMIT;
    return;
  }
  if (lane == 0) L.buf[L.n] = make_uint4(me_rel, p, __float_as_uint(sim), packed);
  L.n += 1;
  wave_mem_fence();
}

// ---- Beam (search.rs:577-589): queue[q_idx..].select_nth_unstable_by(bw - 1, total_cmp) +
// truncate(q_idx + bw), restated from core (Rust >= 1.81: core/src/slice/select.rs, the ipnsort
// partition of core/src/slice/sort/unstable/quicksort.rs and the pivot of sort/shared/pivot.rs) so
// the survivors AND their order are the reference's. The wave runs the introselect loop on a copy of
// the pending slice in its global scratch slice (A), partitions through a second slice (T), and
// writes the first bw states back to the ring. oracle/oracle.cpp (rsel) is the CPU restatement.
//
// Scratch per wave (uint4 units): A[QCAP], T[QCAP], W[48] (per 64 partition positions: the "is less"
// mask as two words, then the exclusive prefix counts).
__host__ __device__ constexpr uint32_t bsel_stride(uint32_t qcap) { return 2u * qcap + 48u; }

__device__ __forceinline__ uint32_t sel_key(const uint4& s) { return total_order_key(__uint_as_float(s.z)); }

// median3 (sort/shared/pivot.rs) on (position, key) pairs
__device__ __forceinline__ void sel_median3(uint32_t pa, uint32_t ka, uint32_t pb, uint32_t kb, uint32_t pc, uint32_t kc,
                                            uint32_t& p, uint32_t& k) {
  const bool x = ka < kb, y = ka < kc;
  if (x == y) {
    const bool z = kb < kc;
    if (z ^ x) { p = pc; k = kc; } else { p = pb; k = kb; }
  } else {
    p = pa;
    k = ka;
  }
}

// choose_pivot (len >= 17 here): median3 of v[0], v[4 len/8], v[7 len/8] below 64 elements, else the
// recursive pseudo-median median3_rec. The recursion tree is evaluated bottom-up: one lane per leaf
// triple (3^D of them, D <= 3 for len <= 4096), then groups of three lanes per level.
__device__ uint32_t sel_pivot(const uint4* v, uint32_t len) {
  const uint32_t lane = lane_id();
  uint32_t s[4] = {len / 8, 0u, 0u, 0u};
  uint32_t D = 0;
  if (len >= 64)
    while (D < 3 && s[D] >= 8) {  // median3_rec recurses while n * 8 >= 64
      s[D + 1] = s[D] / 8;
      ++D;
    }
  uint32_t nleaf = 1;
  for (uint32_t d = 0; d < D; ++d) nleaf *= 3;
  uint32_t p = 0, k = 0;
  if (lane < nleaf) {
    uint32_t base = 0, rem = lane, div = nleaf;
    for (uint32_t d = 0; d < D; ++d) {  // digit d (most significant first) picks a, b or c at level d
      div /= 3;
      const uint32_t dig = rem / div;
      rem -= dig * div;
      base += (dig == 0 ? 0u : dig == 1 ? 4u : 7u) * s[d];
    }
    const uint32_t pa = base, pb = base + 4u * s[D], pc = base + 7u * s[D];
    sel_median3(pa, sel_key(v[pa]), pb, sel_key(v[pb]), pc, sel_key(v[pc]), p, k);
  }
  for (uint32_t n = nleaf; n > 1; n /= 3) {  // one level up: lane g takes lanes 3g, 3g + 1, 3g + 2
    const int b = (int)(3u * lane) & 63;
    const uint32_t pa = (uint32_t)__shfl((int)p, b), ka = (uint32_t)__shfl((int)k, b);
    const uint32_t pb = (uint32_t)__shfl((int)p, (b + 1) & 63), kb = (uint32_t)__shfl((int)k, (b + 1) & 63);
    const uint32_t pc = (uint32_t)__shfl((int)p, (b + 2) & 63), kc = (uint32_t)__shfl((int)k, (b + 2) & 63);
    if (lane < n / 3) sel_median3(pa, ka, pb, kb, pc, kc, p, k);
  }
  return shfl_u32(p, 0);
}

// partition (quicksort.rs) of v[0..len) around v[pp] with is_less (le: a <= pivot), through T;
// returns num_lt. swap(v[0], v[pp]), then partition_lomuto_branchless_cyclic over w = v[1..len): it
// takes w[1], ..., w[m-1], then w[0] (r = 1..m: e_r) and writes each to w[num_lt], moving the previous
// occupant into the gap the previous element left. Closed form, lane-parallel (oracle.cpp
// rsel::lomuto_cyclic is the sequential restatement; tests/test_rust_select.py checks both):
//   * the lt elements end at w[0..F) in processing order (w position = their exclusive lt count L_r);
//   * w[p] for p >= F: e_m if p == F and e_m is not lt; else follow r = p + 1: while e_{r-1} is lt,
//     r = L_r + 1; then e_{r-1};
// then swap(v[0], v[F]): w[F-1] goes to v[0], the pivot to v[F], every other w[p] to v[p + 1].
__device__ uint32_t sel_partition(uint4* v, uint4* T, uint32_t* W, uint32_t len, uint32_t pp, bool le) {
  const uint32_t lane = lane_id();
  const uint32_t m = len - 1;
  const uint4 piv = v[pp];
  const uint32_t pkey = sel_key(piv);
  auto src = [&](uint32_t r) -> uint32_t {  // e_r's position in v before the pivot swap
    const uint32_t x = r < m ? r + 1u : 1u;
    return x == pp ? 0u : x;
  };
  uint32_t F = 0;
  for (uint32_t c = 0; c * 64u < m; ++c) {  // bit b = r - 1
    const uint32_t b = c * 64u + lane;
    const bool valid = b < m;
    uint4 e = make_uint4(0, 0, 0, 0);
    bool lt = false;
    if (valid) {
      e = v[src(b + 1u)];
      const uint32_t k = sel_key(e);
      lt = le ? k <= pkey : k < pkey;
    }
    const uint64_t mk = __ballot(lt);
    if (lane == 0) {
      W[2u * c] = (uint32_t)mk;
      W[2u * c + 1u] = (uint32_t)(mk >> 32);
      W[128u + c] = F;
    }
    if (lt) T[F + prefix_below(mk) + 1u] = e;  // w position L_r, v position + 1 (fixed below for F - 1)
    F += (uint32_t)__popcll(mk);
  }
  wave_mem_fence();
  if (lane == 0) {
    if (F) T[0] = T[F];
    T[F] = piv;
  }
  auto bit = [&](uint32_t b) -> bool { return (W[2u * (b >> 6) + ((b >> 5) & 1u)] >> (b & 31u)) & 1u; };
  auto lcount = [&](uint32_t r) -> uint32_t {  // L_r: lt elements among e_1 .. e_{r-1}
    const uint32_t b = r - 1u, c = b >> 6, o = b & 63u;
    const uint64_t mk = ((uint64_t)W[2u * c + 1u] << 32) | W[2u * c];
    return W[128u + c] + (uint32_t)__popcll(mk & ((1ull << o) - 1ull));
  };
  const bool lt_m = m ? bit(m - 1u) : false;
  for (uint32_t p = F + lane; p < m; p += 64u) {
    uint32_t sidx;
    if (p == F && !lt_m) {
      sidx = m;
    } else {
      uint32_t r = p + 1u;
      while (bit(r - 2u)) r = lcount(r) + 1u;
      sidx = r - 1u;
    }
    T[p + 1u] = v[src(sidx)];
  }
  wave_mem_fence();
  for (uint32_t i = lane; i < len; i += 64u) v[i] = T[i];
  wave_mem_fence();
  return F;
}

// insertion_sort_shift_left(v, 1) for len <= 16: stable by key (rank = smaller keys + equal keys
// before), in place through the lanes' registers
__device__ void sel_small_sort(uint4* v, uint32_t len) {
  const uint32_t lane = lane_id();
  uint4 e = make_uint4(0, 0, 0, 0);
  uint32_t k = 0xFFFFFFFFu;
  if (lane < len) {
    e = v[lane];
    k = sel_key(e);
  }
  uint32_t rank = 0;
  for (uint32_t j = 0; j < len; ++j) {
    const uint32_t kj = shfl_u32(k, (int)j);
    rank += (kj < k || (kj == k && j < lane)) ? 1u : 0u;
  }
  wave_mem_fence();
  if (lane < len) v[rank] = e;
  wave_mem_fence();
}

// ---- median_of_medians fallback (select.rs), taken after 16 partition rounds: one lane, sequential,
// over an element accessor (SelG: states in the global scratch, SelL: (key, position) pairs in LDS)
struct SelG {
  uint4* v;
  using E = uint4;
  __device__ uint32_t key(uint32_t i) const { return sel_key(v[i]); }
  __device__ E get(uint32_t i) const { return v[i]; }
  __device__ void set(uint32_t i, const E& e) const { v[i] = e; }
  __device__ SelG sub(uint32_t o) const { return SelG{v + o}; }
};
struct SelL {
  uint32_t* K;
  uint16_t* I;
  using E = uint2;
  __device__ uint32_t key(uint32_t i) const { return K[i]; }
  __device__ E get(uint32_t i) const { return make_uint2(K[i], I[i]); }
  __device__ void set(uint32_t i, const E& e) const {
    K[i] = e.x;
    I[i] = (uint16_t)e.y;
  }
  __device__ SelL sub(uint32_t o) const { return SelL{K + o, I + o}; }
};
template <typename A>
__device__ void sel_s_swap(const A& v, uint32_t a, uint32_t b) {
  const typename A::E t = v.get(a);
  v.set(a, v.get(b));
  v.set(b, t);
}
template <typename A>
__device__ void sel_s_insertion(const A& v, uint32_t len) {  // insertion_sort_shift_left(v, 1)
  for (uint32_t i = 1; i < len; ++i) {
    const typename A::E tmp = v.get(i);
    const uint32_t kt = v.key(i);
    if (!(kt < v.key(i - 1))) continue;
    uint32_t j = i;
    for (;;) {
      v.set(j, v.get(j - 1));
      --j;
      if (j == 0 || !(kt < v.key(j - 1))) break;
    }
    v.set(j, tmp);
  }
}
template <typename A>
__device__ uint32_t sel_s_partition(const A& v, uint32_t len, uint32_t pivot) {  // quicksort.rs partition
  if (len == 0) return 0;
  sel_s_swap(v, 0, pivot);
  const uint32_t pk = v.key(0);
  const A w = v.sub(1);
  const uint32_t m = len - 1;
  uint32_t num_lt = 0;
  if (m) {  // partition_lomuto_branchless_cyclic
    const typename A::E gv = w.get(0);
    const bool glt = w.key(0) < pk;
    uint32_t gap = 0;
    for (uint32_t r = 1; r < m; ++r) {
      const typename A::E x = w.get(r);
      const bool lt = w.key(r) < pk;
      w.set(gap, w.get(num_lt));
      w.set(num_lt, x);
      gap = r;
      num_lt += lt ? 1u : 0u;
    }
    w.set(gap, w.get(num_lt));
    w.set(num_lt, gv);
    num_lt += glt ? 1u : 0u;
  }
  sel_s_swap(v, 0, num_lt);
  return num_lt;
}
template <typename A>
__device__ uint32_t sel_s_median_idx(const A& v, uint32_t a, uint32_t b, uint32_t c) {
  if (v.key(c) < v.key(a)) {
    const uint32_t t = a;
    a = c;
    c = t;
  }
  if (v.key(c) < v.key(b)) return c;
  if (v.key(b) < v.key(a)) return a;
  return b;
}
// ninther (select.rs): the median of the medians of (a, b, c), (d, e, f), (g, h, i), swapped into e
template <typename A>
__device__ void sel_s_ninther(const A& v, uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e, uint32_t f,
                              uint32_t g, uint32_t h, uint32_t i) {
  auto lt = [&](uint32_t x, uint32_t y) { return v.key(x) < v.key(y); };
  b = sel_s_median_idx(v, a, b, c);
  h = sel_s_median_idx(v, g, h, i);
  if (lt(h, b)) { const uint32_t t = b; b = h; h = t; }
  if (lt(f, d)) { const uint32_t t = d; d = f; f = t; }
  if (lt(e, d)) {
    // the middle triple's median is d
  } else if (lt(f, e)) {
    d = f;
  } else {
    if (lt(e, b)) sel_s_swap(v, e, b);
    else if (lt(h, e)) sel_s_swap(v, e, h);
    return;
  }
  if (lt(d, b)) d = b;
  else if (lt(h, d)) d = h;
  sel_s_swap(v, d, e);
}
template <int D, typename A>
__device__ void sel_s_mom(const A& v, uint32_t len, uint32_t k);
template <int D, typename A>
__device__ uint32_t sel_s_ninthers(const A& v, uint32_t len) {  // median_of_ninthers
  const uint32_t frac = len <= 1024u ? len / 12u : (len <= 128u * 1024u ? len / 64u : len / 1024u);
  const uint32_t pivot = frac / 2u, lo = len / 2u - pivot, hi = frac + lo, gap = (len - 9u * frac) / 4u;
  uint32_t a = lo - 4u * frac - gap, b = hi + gap;
  for (uint32_t i = lo; i < hi; ++i) {
    sel_s_ninther(v, a, i - frac, b, a + 1u, i, b + 1u, a + 2u, i + frac, b + 2u);
    a += 3u;
    b += 3u;
  }
  sel_s_mom<D - 1>(v.sub(lo), frac, pivot);
  return sel_s_partition(v, len, lo + pivot);
}
template <int D, typename A>
__device__ void sel_s_mom(const A& v0, uint32_t len, uint32_t k) {  // median_of_medians
  A v = v0;
  for (;;) {
    if (len <= 16u) {
      if (len >= 2u) sel_s_insertion(v, len);
      return;
    }
    if (k == len - 1u || k == 0u) {  // max_index keeps the first maximum, min_index the first minimum
      uint32_t acc = 0;
      for (uint32_t i = 1; i < len; ++i)
        if (k ? v.key(acc) < v.key(i) : v.key(i) < v.key(acc)) acc = i;
      sel_s_swap(v, acc, k);
      return;
    }
    uint32_t p;
    if constexpr (D > 0) {
      p = sel_s_ninthers<D>(v, len);
    } else {  // unreachable for len <= 4096 (three levels of ninthers reach <= 16 elements)
      sel_s_insertion(v, len);
      return;
    }
    if (p == k) return;
    if (p > k) {
      len = p;
    } else {
      v = v.sub(p + 1u);
      len -= p + 1u;
      k -= p + 1u;
    }
  }
}

// The selects are real calls (not inlined into run_window): inlined, their registers raised the
// window loop's pressure past the dedup variants' budget and the loop spilled to scratch on every
// batch (rc_build_kernel<256>: 45 VGPRs spilled, 1168 B/lane scratch). Measured C3: 212.5 -> 162.0 ms
// per step (prefix cache 79.1 -> 44.8 ms, wave kernels 109.3 -> 93.6 ms; profiles/r03o).
#ifndef FAC_SEL_ATTR
#define FAC_SEL_ATTR __attribute__((noinline))
#endif
template <uint32_t QCAP>
__device__ FAC_SEL_ATTR void beam_select(KState* q, uint32_t head, uint32_t tail, uint32_t bw, uint4* scratch, uint32_t limit0) {
  const uint32_t lane = lane_id();
  const uint32_t P = tail - head;
  uint4* qq = reinterpret_cast<uint4*>(q);
  if (bw == 1) {  // partition_at_index, index == 0: min_index (first minimum), swapped to the front
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t i = lane; i < P; i += 64u) best = min(best, sel_key(qq[(head + i) & (QCAP - 1)]));
    best = wave_min_u32(best);
    uint32_t first = 0xFFFFFFFFu;
    for (uint32_t i = lane; i < P; i += 64u)
      if (sel_key(qq[(head + i) & (QCAP - 1)]) == best) first = min(first, i);
    first = wave_min_u32(first);
    const uint4 e = qq[(head + first) & (QCAP - 1)];
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) qq[head & (QCAP - 1)] = e;
    __builtin_amdgcn_wave_barrier();
    tail = head + 1u;
    return;
  }
  uint4* A = scratch;
  uint4* T = scratch + QCAP;
  uint32_t* W = reinterpret_cast<uint32_t*>(scratch + 2u * QCAP);
  for (uint32_t i = lane; i < P; i += 64u) A[i] = qq[(head + i) & (QCAP - 1)];
  wave_mem_fence();
  // partition_at_index_loop (bw - 1 is never len - 1 here: P > 2 bw)
  uint32_t a = 0, len = P, index = bw - 1u, limit = limit0;
  bool has_anc = false;
  uint32_t anc = 0;
  for (;;) {
    if (len <= 16u) {
      if (len >= 2u) sel_small_sort(A + a, len);
      break;
    }
    if (limit == 0) {
      if (lane == 0) sel_s_mom<4>(SelG{A + a}, len, index);
      wave_mem_fence();
      break;
    }
    --limit;
    const uint32_t pp = sel_pivot(A + a, len);
    const uint32_t pk = sel_key(A[a + pp]);
    if (has_anc && !(anc < pk)) {  // pivot equal to the ancestor pivot: split off the equal run
      const uint32_t mid = sel_partition(A + a, T + a, W, len, pp, true) + 1u;
      if (index < mid) break;  // core: `if mid > index { return; }`
      a += mid;
      len -= mid;
      index -= mid;
      has_anc = false;
      continue;
    }
    const uint32_t mid = sel_partition(A + a, T + a, W, len, pp, false);
    if (mid < index) {
      has_anc = true;
      anc = pk;
      a += mid + 1u;
      len -= mid + 1u;
      index -= mid + 1u;
    } else if (mid > index) {
      len = mid;
    } else {
      break;
    }
  }
  for (uint32_t i = lane; i < bw; i += 64u) qq[(head + i) & (QCAP - 1)] = A[i];
  __builtin_amdgcn_wave_barrier();
  tail = head + bw;
}

// The same select for rings of <= 256 states, on (key, ring position) pairs in the wave's LDS
// dedup-claim words (free between batches; zeroed again on exit): K[256] keys, I[256] positions
// (u16), W[8] "is less" masks + W[8..12) their exclusive counts. Each partition reads every moved
// element into registers (<= 4 per lane) before any is written; the survivors' states are gathered
// from the ring at the end. Same algorithm and result as beam_select (global scratch, larger rings).
constexpr uint32_t SEL_LDS_WORDS = 256 + 128 + 8 + 4;
static_assert(SEL_LDS_WORDS <= 512, "the LDS select must fit the smallest claim region");

__device__ uint32_t sel_pivot_lds(const uint32_t* K, uint32_t a, uint32_t len) {
  const uint32_t lane = lane_id();
  uint32_t s[4] = {len / 8, 0u, 0u, 0u};
  uint32_t D = 0;
  if (len >= 64)
    while (D < 3 && s[D] >= 8) {
      s[D + 1] = s[D] / 8;
      ++D;
    }
  uint32_t nleaf = 1;
  for (uint32_t d = 0; d < D; ++d) nleaf *= 3;
  uint32_t p = 0, k = 0;
  if (lane < nleaf) {
    uint32_t base = 0, rem = lane, div = nleaf;
    for (uint32_t d = 0; d < D; ++d) {
      div /= 3;
      const uint32_t dig = rem / div;
      rem -= dig * div;
      base += (dig == 0 ? 0u : dig == 1 ? 4u : 7u) * s[d];
    }
    const uint32_t pa = base, pb = base + 4u * s[D], pc = base + 7u * s[D];
    sel_median3(pa, K[a + pa], pb, K[a + pb], pc, K[a + pc], p, k);
  }
  for (uint32_t n = nleaf; n > 1; n /= 3) {
    const int b = (int)(3u * lane) & 63;
    const uint32_t pa = (uint32_t)__shfl((int)p, b), ka = (uint32_t)__shfl((int)k, b);
    const uint32_t pb = (uint32_t)__shfl((int)p, (b + 1) & 63), kb = (uint32_t)__shfl((int)k, (b + 1) & 63);
    const uint32_t pc = (uint32_t)__shfl((int)p, (b + 2) & 63), kc = (uint32_t)__shfl((int)k, (b + 2) & 63);
    if (lane < n / 3) sel_median3(pa, ka, pb, kb, pc, kc, p, k);
  }
  return shfl_u32(p, 0);
}

// partition (see sel_partition) of the elements at [a, a + len), len <= 256
__device__ uint32_t sel_partition_lds(uint32_t* K, uint16_t* I, uint32_t* W, uint32_t a, uint32_t len, uint32_t pp,
                                      bool le) {
  const uint32_t lane = lane_id();
  const uint32_t m = len - 1;
  const uint32_t pkey = K[a + pp];
  const uint16_t pidx = I[a + pp];
  auto src = [&](uint32_t r) -> uint32_t {
    const uint32_t x = r < m ? r + 1u : 1u;
    return a + (x == pp ? 0u : x);
  };
  // phase 1: the lt masks; every lane keeps its processing positions' elements and lt destinations
  uint32_t F = 0, ek[4], ei[4], ed[4];
#pragma unroll
  for (uint32_t c = 0; c < 4; ++c) {
    const uint32_t b = c * 64u + lane;
    const bool valid = b < m;
    ek[c] = 0;
    ei[c] = 0;
    bool lt = false;
    if (valid) {
      const uint32_t sp = src(b + 1u);
      ek[c] = K[sp];
      ei[c] = I[sp];
      lt = le ? ek[c] <= pkey : ek[c] < pkey;
    }
    const uint64_t mk = __ballot(lt);
    ed[c] = lt ? F + prefix_below(mk) : 0xFFFFFFFFu;  // w position L_r
    if (lane == 0 && c * 64u < m) {
      W[2u * c] = (uint32_t)mk;
      W[2u * c + 1u] = (uint32_t)(mk >> 32);
      W[8u + c] = F;
    }
    F += (uint32_t)__popcll(mk);
  }
  wave_mem_fence();
  auto bit = [&](uint32_t b) -> bool { return (W[2u * (b >> 6) + ((b >> 5) & 1u)] >> (b & 31u)) & 1u; };
  auto lcount = [&](uint32_t r) -> uint32_t {
    const uint32_t b = r - 1u, c = b >> 6, o = b & 63u;
    const uint64_t mk = ((uint64_t)W[2u * c + 1u] << 32) | W[2u * c];
    return W[8u + c] + (uint32_t)__popcll(mk & ((1ull << o) - 1ull));
  };
  const bool lt_m = bit(m - 1u);
  // phase 2: the other positions pull their element (w positions p >= F)
  uint32_t gk[4], gi[4];
#pragma unroll
  for (uint32_t c = 0; c < 4; ++c) {
    const uint32_t p = F + c * 64u + lane;
    gk[c] = 0;
    gi[c] = 0;
    if (p < m) {
      uint32_t sidx;
      if (p == F && !lt_m) {
        sidx = m;
      } else {
        uint32_t r = p + 1u;
        while (bit(r - 2u)) r = lcount(r) + 1u;
        sidx = r - 1u;
      }
      const uint32_t sp = src(sidx);
      gk[c] = K[sp];
      gi[c] = I[sp];
    }
  }
  wave_mem_fence();
  // phase 3: write back; w position q goes to a + q + 1, except w[F - 1] -> a and the pivot -> a + F
#pragma unroll
  for (uint32_t c = 0; c < 4; ++c) {
    if (ed[c] != 0xFFFFFFFFu) {
      const uint32_t d = a + (ed[c] == F - 1u ? 0u : ed[c] + 1u);
      K[d] = ek[c];
      I[d] = (uint16_t)ei[c];
    }
    const uint32_t p = F + c * 64u + lane;
    if (p < m) {
      K[a + p + 1u] = gk[c];
      I[a + p + 1u] = (uint16_t)gi[c];
    }
  }
  if (lane == 0) {
    K[a + F] = pkey;
    I[a + F] = pidx;
  }
  wave_mem_fence();
  return F;
}

template <uint32_t QCAP>
__device__ FAC_SEL_ATTR void beam_select_lds(KState* q, uint32_t head, uint32_t tail, uint32_t bw, uint32_t* scratch, uint32_t limit0) {
  static_assert(QCAP <= 256, "LDS select: rings of up to 256 states");
  const uint32_t lane = lane_id();
  const uint32_t P = tail - head;
  uint4* qq = reinterpret_cast<uint4*>(q);
  if (bw == 1) {  // partition_at_index, index == 0: min_index (first minimum), swapped to the front
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t i = lane; i < P; i += 64u) best = min(best, sel_key(qq[(head + i) & (QCAP - 1)]));
    best = wave_min_u32(best);
    uint32_t first = 0xFFFFFFFFu;
    for (uint32_t i = lane; i < P; i += 64u)
      if (sel_key(qq[(head + i) & (QCAP - 1)]) == best) first = min(first, i);
    first = wave_min_u32(first);
    const uint4 e = qq[(head + first) & (QCAP - 1)];
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) qq[head & (QCAP - 1)] = e;
    __builtin_amdgcn_wave_barrier();
    tail = head + 1u;
    return;
  }
  uint32_t* K = scratch;
  uint16_t* I = reinterpret_cast<uint16_t*>(scratch + 256);
  uint32_t* W = scratch + 384;
  for (uint32_t i = lane; i < P; i += 64u) {
    K[i] = sel_key(qq[(head + i) & (QCAP - 1)]);
    I[i] = (uint16_t)i;
  }
  wave_mem_fence();
  uint32_t a = 0, len = P, index = bw - 1u, limit = limit0;
  bool has_anc = false;
  uint32_t anc = 0;
  for (;;) {
    if (len <= 16u) {
      if (len >= 2u) {  // insertion_sort_shift_left: stable by key
        uint32_t k = 0xFFFFFFFFu, ix = 0;
        if (lane < len) {
          k = K[a + lane];
          ix = I[a + lane];
        }
        uint32_t rank = 0;
        for (uint32_t j = 0; j < len; ++j) {
          const uint32_t kj = shfl_u32(k, (int)j);
          rank += (kj < k || (kj == k && j < lane)) ? 1u : 0u;
        }
        wave_mem_fence();
        if (lane < len) {
          K[a + rank] = k;
          I[a + rank] = (uint16_t)ix;
        }
        wave_mem_fence();
      }
      break;
    }
    if (limit == 0) {  // median_of_medians: one lane, sequential
      if (lane == 0) sel_s_mom<4>(SelL{K + a, I + a}, len, index);
      wave_mem_fence();
      break;
    }
    --limit;
    const uint32_t pp = sel_pivot_lds(K, a, len);
    const uint32_t pk = K[a + pp];
    if (has_anc && !(anc < pk)) {  // pivot equal to the ancestor pivot: split off the equal run
      const uint32_t mid = sel_partition_lds(K, I, W, a, len, pp, true) + 1u;
      if (index < mid) break;  // core: `if mid > index { return; }`
      a += mid;
      len -= mid;
      index -= mid;
      has_anc = false;
      continue;
    }
    const uint32_t mid = sel_partition_lds(K, I, W, a, len, pp, false);
    if (mid < index) {
      has_anc = true;
      anc = pk;
      a += mid + 1u;
      len -= mid + 1u;
      index -= mid + 1u;
    } else if (mid > index) {
      len = mid;
    } else {
      break;
    }
  }
  // the survivors' states, gathered from the ring (every read before any write; bw < 128 here)
  uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
  if (lane < bw) v0 = qq[(head + I[lane]) & (QCAP - 1)];
  if (lane + 64u < bw) v1 = qq[(head + I[lane + 64u]) & (QCAP - 1)];
  wave_mem_fence();
  if (lane < bw) qq[(head + lane) & (QCAP - 1)] = v0;
  if (lane + 64u < bw) qq[(head + lane + 64u) & (QCAP - 1)] = v1;
  for (uint32_t i = lane; i < SEL_LDS_WORDS; i += 64u) scratch[i] = 0u;  // claim words stay <= 64
  wave_mem_fence();
  tail = head + bw;
}

// Diagnostics only (FAC_BEAM_CANONICAL, rounds 1-2's rule): keep the bw smallest by (penalty,
// queue position) in queue order -- not the reference's order; for A/B measurements of the tie rule.
template <uint32_t QCAP>
__device__ FAC_SEL_ATTR void beam_select_canonical(KState* q, uint32_t head, uint32_t tail, uint32_t bw) {
  constexpr int PER = QCAP / 64;
  const uint32_t lane = lane_id();
  const uint32_t P = tail - head;
  uint32_t key[PER];
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const uint32_t i = (uint32_t)t * 64 + lane;
    key[t] = i < P ? total_order_key(q[(head + i) & (QCAP - 1)].pen) : 0xFFFFFFFFu;
  }
  uint32_t left = bw, T = 0xFFFFFFFFu, need_eq = 0;
  bool have_last = false;
  uint32_t last = 0;
  for (;;) {
    uint32_t m = 0xFFFFFFFFu;
#pragma unroll
    for (int t = 0; t < PER; ++t)
      if (!have_last || key[t] > last) m = min(m, key[t]);
    m = wave_min_u32(m);
    uint32_t c = 0;
#pragma unroll
    for (int t = 0; t < PER; ++t) c += __popcll(__ballot(key[t] == m && (uint32_t)t * 64 + lane < P));
    if (c >= left || m == 0xFFFFFFFFu) {
      T = m;
      need_eq = left;
      break;
    }
    left -= c;
    last = m;
    have_last = true;
  }
  uint32_t w = head, eq_seen = 0;
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const uint32_t i = (uint32_t)t * 64 + lane;
    const bool valid = i < P;
    const uint32_t k = key[t];
    const bool eq = valid && k == T;
    const uint64_t meq = __ballot(eq);
    const bool keep = valid && (k < T || (eq && eq_seen + prefix_below(meq) < need_eq));
    const uint64_t mk = __ballot(keep);
    const uint4 v = keep ? reinterpret_cast<const uint4*>(q)[(head + i) & (QCAP - 1)] : make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    if (keep) reinterpret_cast<uint4*>(q)[(w + prefix_below(mk)) & (QCAP - 1)] = v;
    __builtin_amdgcn_wave_barrier();
    w += __popcll(mk);
    eq_seen += __popcll(meq);
  }
  tail = head + bw;
}

// Append the lanes whose `pred` holds, in lane order (= the reference's push order).
template <uint32_t QCAP>
__device__ __forceinline__ void push_lanes(KState* q, uint32_t head, uint32_t& tail, bool pred, const KState& s,
                                           unsigned& err) {
  const uint64_t m = __ballot(pred);
  if (!m) return;
  const uint32_t cnt = __popcll(m);
  if (tail + cnt - head > QCAP) {
    err |= ERR_QUEUE;
    return;
  }
  if (pred) q[(tail + prefix_below(m)) & (QCAP - 1)] = s;
  tail += cnt;
}

__device__ __forceinline__ uint32_t vis_hash(const KState& s) {
  uint32_t h = s.node * 0x9E3779B1u;
  h ^= s.jm * 0x85EBCA77u + (h >> 13);
  h ^= s.packed * 0xC2B2AE3Du + (h >> 16);
  h ^= h >> 15;
  return h;
}

// State dedup (search.rs:608-628). Returns true when the state must be skipped.
template <uint32_t VCAP>
__device__ __forceinline__ bool visited_check(KState* vis, uint32_t& vcount, const KState& s, bool exact_needed,
                                              unsigned& err) {
  const uint32_t lane = lane_id();
  const uint32_t h = vis_hash(s);
  for (uint32_t probe = 0; probe < VCAP; probe += 64) {
    const uint32_t slot = (h + probe + lane) & (VCAP - 1);
    const KState e = vis[slot];
    const bool is_empty = e.node == EMPTY;
    const bool is_match = !is_empty && e.node == s.node && e.jm == s.jm && e.packed == s.packed;
    const uint64_t me = __ballot(is_empty), mm = __ballot(is_match);
    const int fe = me ? first_lane(me) : 64;
    const int fm = mm ? first_lane(mm) : 64;
    if (fm < fe) {
      const float stored = shfl_f32(e.pen, fm);
      if (stored <= s.pen) return true;
      if (lane == (uint32_t)fm) vis[slot].pen = s.pen;
      return false;
    }
    if (fe < 64) {
      if (vcount + 1 >= VCAP - VCAP / 8) {  // table "full": keep probe chains short
        if (exact_needed) err |= ERR_VISITED;
        return false;  // without a beam, expanding a duplicate cannot change results
      }
      if (lane == (uint32_t)fe) vis[slot] = s;
      vcount = __builtin_amdgcn_readfirstlane(vcount + 1);  // wave-uniform: kept in an SGPR
      return false;
    }
  }
  if (exact_needed) err |= ERR_VISITED;
  return false;
}

// Emission (search.rs:659-737) for one accepted state; lanes spread over the node's output list.
// Called in FIFO pop order, so the per-window best list keeps the reference's first-found ties.
__device__ void emit_state(const SearchParams& P, EmitList& EL, uint32_t me_rel, float pen, uint32_t packed,
                           uint32_t node, unsigned& err) {
  const uint2 orr = P.out_range[node];
  const uint32_t out_begin = orr.x, out_end = orr.y;
  const uint32_t lane = lane_id();
  const bool fast = P.mef != 255u;
  const uint32_t edits = edits_of(packed);
  const uint32_t ins = packed & 0xFFu, del = (packed >> 8) & 0xFFu, sub = (packed >> 16) & 0xFFu, swp = packed >> 24;
  for (uint32_t base = out_begin; base < out_end; base += 64) {
    const uint32_t i = base + lane;
    bool ok = i < out_end;
    uint32_t p = 0;
    float sim = 0.f;
    if (ok) {
      p = P.out_pat[i];
      const DevPattern pt = P.pats[p];
      if (fast) {
        ok = edits <= P.mef;
      } else {  // within_limits (:151-169)
        const Lim m = pick_limits(P, pt.has_limits ? (int32_t)p : -1);
        ok = m.has ? (lim_le(m.l.edits, edits) && lim_le(m.l.ins, ins) && lim_le(m.l.del, del) &&
                      lim_le(m.l.sub, sub) && lim_le(m.l.swp, swp))
                   : (edits == 0);
      }
      if (ok) {
        const float total = pt.glen;
        sim = __fmul_rn(__fdiv_rn(__fsub_rn(total, pen), total), pt.weight);  // :696-699
        ok = !(sim < P.thr);                                                   // :701
      }
    }
    uint64_t m = __ballot(ok);
    while (m) {
      const int l = first_lane(m);
      m &= m - 1;
      emit_update(EL, me_rel, shfl_u32(p, l), shfl_f32(sim, l), packed, err);
    }
  }
}

// Edge-parallel expansion of ONE accepted state (dedup and ceiling passed, emission done): the
// exact / substitution / swap / insertion / deletion pushes with the 64 lanes spread over the
// node's edges (search.rs:742-1089). Used for nodes with more than 64 edges.
// find_gid, edge-parallel over the wave (every lane calls it with the same arguments)
__device__ __forceinline__ int64_t wave_find_gid(const SearchParams& P, uint32_t node, uint32_t gid) {
  if (gid == 0) return -1;
  const DevNode nd = P.nodes[node];
  const uint32_t end = node_end(nd);
  for (uint32_t base = nd.edge_begin; base < end; base += 64) {
    const uint32_t i = base + lane_id();
    const uint64_t m = __ballot(i < end && P.edge_gid[i] == gid);
    if (m) return (int64_t)(P.edges[base + first_lane(m)].next & EDGE_NEXT_MASK);
  }
  return -1;
}

template <uint32_t QCAP, bool MAP>
__device__ void expand_wide(const SearchParams& P, const SegDesc& S, KState* q, uint32_t head, uint32_t& tail,
                            const KState& st, const DevNode& nd, uint64_t start, unsigned& err) {
  const uint32_t lane = lane_id();
  const bool fast = P.mef != 255u;
  const uint64_t n = S.n;
  const float pen = st.pen;
  const float remaining = __fsub_rn(P.max_penalties, pen);  // :648
  const uint32_t packed = st.packed;
  const uint32_t edits = edits_of(packed);
  const uint32_t j_rel = st.jm & 0xFFFFu, me_rel = st.jm >> 16;
  const uint64_t j = start + j_rel;
  const int32_t nlim = P.has_pattern_limits ? node_limits(P, st.node) : -1;  // :653-657
    const bool is_last_edit = fast && edits + 1u >= P.mef;  // :742
    const uint32_t cur_ch = j < n ? text_char(P, S, j, err) : 0u;
    // Nodes with <= 64 edges (all but the top trie levels) are handled from one register-resident
    // chunk: lane l holds edge l and, at the last edit level, its child's single-byte edge map.
    const uint32_t deg = node_deg(nd);
    const bool small = deg <= 64u;
    uint32_t e_ch = 0, e_next = 0;
    uint4 e_sb = make_uint4(0, 0, 0, 0);
    const bool e_valid = small && lane < deg;
    if (e_valid) {
      const DevEdge ed = P.edges[nd.edge_begin + lane];
      e_ch = ed.ch;
      e_next = ed.next;
      if (is_last_edit) e_sb = P.sb_edge[nd.edge_begin + lane];
    }
    auto sb_bit = [](uint4 m, uint32_t ch) -> bool {  // branch-free word select (no stack indexing)
      const uint32_t lo = (ch & 32u) ? m.y : m.x;
      const uint32_t hi = (ch & 32u) ? m.w : m.z;
      const uint32_t w = (ch & 64u) ? hi : lo;
      return ch < 128u && ((w >> (ch & 31u)) & 1u);
    };
    auto small_goto = [&](uint32_t ch) -> int64_t {
      const uint64_t m = __ballot(e_valid && e_ch == ch);
      return m ? (int64_t)(shfl_u32(e_next, first_lane(m)) & EDGE_NEXT_MASK) : -1;
    };
    if (j < n) {
      bool have_next = false;
      uint32_t next_ch = 0;
      if (is_last_edit && (!fast || edits < P.mef) && j + 1 < n) {  // :758-765
        have_next = true;
        next_ch = text_char(P, S, j + 1, err);
      }
      // exact transition (:766-798); matched_start stays `start` for every state
      const uint64_t nk = GT_VALID | GT_GOTO | ((uint64_t)st.node << 21);
      uint64_t gx;
      const int64_t exact_next =
          MAP ? wave_find_gid(P, st.node, text_gid(P, S, j, err))  // :776-780 with MAPPINGS
          : small   ? small_goto(cur_ch)
                    : (gt_get(P, nk | cur_ch, true, gx) ? (int64_t)(gx & CHILD26_MASK) : -1);
      const uint32_t jm1 = (j_rel + 1u) | ((j_rel + 1u) << 16);
      push_lanes<QCAP>(q, head, tail, lane == 0 && exact_next >= 0,
                       KState{(uint32_t)exact_next, jm1, pen, packed}, err);

      // substitutions (:803-874)
      bool subst_ok;
      if (fast) {
        subst_ok = edits < P.mef;
      } else {  // within_limits_subst (:134-146)
        const Lim m = pick_limits(P, nlim);
        subst_ok = m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.sub, (packed >> 16) & 0xFFu))
                         : (edits == 0 && ((packed >> 16) & 0xFFu) == 0);
      }
      if (subst_ok) {
        for (uint32_t base = nd.edge_begin; base < node_end(nd); base += 64) {
          const uint32_t i = base + lane;
          bool keep;
          uint32_t ch, nx;
          if (small) {
            keep = e_valid;
            ch = e_ch;
            nx = e_next;
          } else {
            keep = i < node_end(nd);
            const DevEdge ed = keep ? P.edges[i] : DevEdge{0, 0};
            ch = ed.ch;
            nx = ed.next;
          }
          KState st2{};
          if (keep) {
            const uint32_t child = nx & EDGE_NEXT_MASK;
            keep = !(exact_next >= 0 && child == (uint32_t)exact_next);
            const float sim = similarity(P, ch, cur_ch);
            keep = keep && !(sim < P.min_sym);
            const float penalty = __fmul_rn(P.p_sub, __fsub_rn(1.0f, sim));
            keep = keep && !(penalty > remaining);
            if (keep && is_last_edit)  // dead-end filter (:839-847)
              keep = (nx & EDGE_CHILD_OUTPUT) ||
                     (have_next && (small ? sb_bit(e_sb, next_ch) : sb_has(P, child, next_ch)));
            st2 = KState{child, jm1, __fadd_rn(pen, penalty), packed + 0x10000u};
          }
          push_lanes<QCAP>(q, head, tail, keep, st2, err);
        }
        if constexpr (MAP) {  // 1b) multi-character mappings (:883-922), one transition per lane
          const uint2 r = P.map_range[st.node];
          const uint64_t mm = map_mask(P, S, st.node, j, pen, err);  // wave-uniform
          const bool keep = lane < r.y - r.x && ((mm >> lane) & 1ull);
          KState st2{};
          if (keep) {
            const uint4 mt = P.map_ent[r.x + lane];
            const uint32_t jh = j_rel + mt.y;
            st2 = KState{mt.z, jh | (jh << 16), __fadd_rn(pen, __uint_as_float(mt.w)), packed + 0x10000u};
          }
          push_lanes<QCAP>(q, head, tail, keep, st2, err);
        }
      }

      // swap (:935-989)
      if (j + 1 < n && P.p_swp <= remaining && (!fast || edits < P.mef)) {
        const uint32_t nch = have_next ? next_ch : text_char(P, S, j + 1, err);
        const int64_t x = MAP ? wave_find_gid(P, st.node, text_gid(P, S, j + 1, err))  // :945-961
                          : small   ? small_goto(nch)
                                    : (gt_get(P, nk | nch, true, gx) ? (int64_t)(gx & CHILD26_MASK) : -1);
        if (x >= 0) {
          const int64_t node2 = MAP ? wave_find_gid(P, (uint32_t)x, text_gid(P, S, j, err))
                                : gt_get(P, GT_VALID | GT_GOTO | ((uint64_t)x << 21) | cur_ch, true, gx)
                                    ? (int64_t)(gx & CHILD26_MASK) : -1;
          bool ok = node2 >= 0;
          if (ok && !fast) {  // within_limits_swap_ahead with node2's limits (:962-967)
            const Lim m = pick_limits(P, node_limits(P, (uint32_t)node2));
            ok = m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.swp, packed >> 24)) : false;
          }
          const uint32_t jm2 = (j_rel + 2u) | ((j_rel + 2u) << 16);
          push_lanes<QCAP>(q, head, tail, lane == 0 && ok,
                           KState{(uint32_t)node2, jm2, __fadd_rn(pen, P.p_swp), packed + 0x1000000u}, err);
        }
      }

      // insertion (:994-1029): never before the first consumed grapheme
      if ((me_rel != 0u || j_rel != 0u) && P.p_ins <= remaining) {
        bool ok;
        if (fast) {
          ok = edits < P.mef;
        } else {
          const Lim m = pick_limits(P, nlim);
          ok = m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.ins, packed & 0xFFu)) : false;
        }
        if (ok && is_last_edit && !node_has_out(nd) && !(have_next && sb_has(P, st.node, next_ch)))
          ok = false;
        const uint32_t jmi = (j_rel + 1u) | (me_rel << 16);
        push_lanes<QCAP>(q, head, tail, lane == 0 && ok, KState{st.node, jmi, __fadd_rn(pen, P.p_ins), packed + 1u},
                         err);
      }
    }

    // deletion (:1035-1089), allowed even at j == n
    if (P.p_del <= remaining) {
      bool ok;
      if (fast) {
        ok = edits < P.mef;
      } else {
        const Lim m = pick_limits(P, nlim);
        ok = m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.del, (packed >> 8) & 0xFFu)) : false;
      }
      if (ok) {
        const bool have_cur = is_last_edit && j < n;
        const float npen = __fadd_rn(pen, P.p_del);
        for (uint32_t base = nd.edge_begin; base < node_end(nd); base += 64) {
          const uint32_t i = base + lane;
          bool keep;
          uint32_t nx;
          if (small) {
            keep = e_valid;
            nx = e_next;
          } else {
            keep = i < node_end(nd);
            nx = keep ? P.edges[i].next : 0u;
          }
          const uint32_t child = nx & EDGE_NEXT_MASK;
          if (keep && is_last_edit)  // dead-end filter (:1057-1063)
            keep = (nx & EDGE_CHILD_OUTPUT) ||
                   (have_cur && (small ? sb_bit(e_sb, cur_ch) : sb_has(P, child, cur_ch)));
          push_lanes<QCAP>(q, head, tail, keep, KState{child, st.jm, npen, packed + 0x100u}, err);
        }
      }
    }
}

// One state per lane: the expansion decisions of a <=64-edge node, computed lane-serially into
// register bitmasks (bit e of msub/mdel = edge e pushes a substitution/deletion successor).
struct LaneExp {
  int64_t exact;     // exact successor node or -1
  int64_t swap;      // swap successor node or -1
  bool ins;          // insertion successor
  uint64_t msub, mdel;
  uint32_t count;    // pushes of this state
  uint64_t mmap;     // MAP: applicable mapping transitions of the node (bit t = its t-th)
};

__device__ __forceinline__ bool sb_word_bit(uint4 m, uint32_t ch) {  // branch-free (no stack indexing)
  const uint32_t lo = (ch & 32u) ? m.y : m.x;
  const uint32_t hi = (ch & 32u) ? m.w : m.z;
  const uint32_t w = (ch & 64u) ? hi : lo;
  return ch < 128u && ((w >> (ch & 31u)) & 1u);
}

// Wave-wide inclusive prefix sum (DPP row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return (uint32_t)x;
}

// Per-state expansion decisions that do not depend on the edge (search.rs:742-765, 787-800,
// 935-937, 994-1045): one lane per state.
struct Prep {
  uint32_t cur_ch, next_ch, nch;
  uint32_t flags;  // PF_* bits
  float remaining;
  uint32_t gcur, gnx;  // MAP: grapheme ids at j and j + 1 (0 otherwise)
};
constexpr uint32_t PF_SUB = 1u, PF_DEL = 2u, PF_LAST = 4u, PF_CSB = 8u, PF_NEXT = 16u, PF_CUR = 32u, PF_SWAP = 64u,
                   PF_EX = 128u, PF_INS = 256u;

__device__ Prep lane_prep(const SearchParams& P, const SegDesc& S, const KState& st, const DevNode& nd, uint64_t start,
                          uint32_t c0, uint32_t c1, uint4 own_sb) {  // c0/c1: text at j / j + 1 (0 past the end)
  Prep r{0u, 0u, 0u, 0u, 0.0f};
  const bool fast = P.mef != 255u;
  const uint64_t n = S.n;
  r.remaining = __fsub_rn(P.max_penalties, st.pen);  // :648
  const uint32_t packed = st.packed;
  const uint32_t edits = edits_of(packed);
  const uint32_t j_rel = st.jm & 0xFFFFu, me_rel = st.jm >> 16;
  const uint64_t j = start + j_rel;
  const int32_t nlim = P.has_pattern_limits ? node_limits(P, st.node) : -1;
  const bool is_last_edit = fast && edits + 1u >= P.mef;  // :742
  const bool in_text = j < n;
  r.cur_ch = in_text ? c0 : 0u;
  bool have_next = false;
  if (in_text && is_last_edit && (!fast || edits < P.mef) && j + 1 < n) {  // :758-765
    have_next = true;
    r.next_ch = c1;
  }
  bool subst_ok = false, swap_ok = false, ins_ok = false, del_ok = false;
  if (in_text) {
    if (fast) {
      subst_ok = edits < P.mef;
    } else {  // within_limits_subst (:134-146)
      const Lim m = pick_limits(P, nlim);
      subst_ok = m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.sub, (packed >> 16) & 0xFFu))
                       : (edits == 0 && ((packed >> 16) & 0xFFu) == 0);
    }
    swap_ok = j + 1 < n && P.p_swp <= r.remaining && (!fast || edits < P.mef);  // :935-937
    if (swap_ok) r.nch = c1;
    if ((me_rel != 0u || j_rel != 0u) && P.p_ins <= r.remaining) {  // :994-1007
      if (fast) {
        ins_ok = edits < P.mef;
      } else {
        const Lim m = pick_limits(P, nlim);
        ins_ok = m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.ins, packed & 0xFFu)) : false;
      }
      if (ins_ok && is_last_edit && !node_has_out(nd)) ins_ok = have_next && sb_word_bit(own_sb, r.next_ch);
    }
  }
  if (P.p_del <= r.remaining) {  // :1035-1045
    if (fast) {
      del_ok = edits < P.mef;
    } else {
      const Lim m = pick_limits(P, nlim);
      del_ok = m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.del, (packed >> 8) & 0xFFu)) : false;
    }
  }
  r.flags = (in_text && subst_ok ? PF_SUB : 0u) | (del_ok ? PF_DEL : 0u) | (is_last_edit ? PF_LAST : 0u) |
            // the child's map is only read when the tested char is ASCII (a bit test on >= 128 is false)
            (is_last_edit && ((in_text && subst_ok && have_next && r.next_ch < 128u) ||
                              (del_ok && in_text && r.cur_ch < 128u))
                 ? PF_CSB
                 : 0u) |
            (have_next ? PF_NEXT : 0u) |
            (is_last_edit && in_text ? PF_CUR : 0u) | (swap_ok ? PF_SWAP : 0u) | (in_text ? PF_EX : 0u) |
            (ins_ok ? PF_INS : 0u);
  return r;
}

// Wave-wide inclusive max-scan (DPP), unsigned.
// adds the wave's sum of v to a global counter with one atomic (every lane of the wave calls it): a
// per-lane atomic on one address serialises at one L2 channel (1M of them at the end of a lookup)
__device__ __forceinline__ void wave_add_counter(unsigned long long* c, unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if (lane_id() == 0 && v) atomicAdd(c, v);
}
__device__ __forceinline__ uint32_t wave_inclusive_max(uint32_t v) {
  int x = (int)v;
  x = (int)max((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false));
  x = (int)max((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false));
  x = (int)max((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false));
  x = (int)max((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false));
  x = (int)max((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false));
  x = (int)max((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false));
  return (uint32_t)x;
}

// LDS scratch of one batch's edge expansion. It aliases the dedup claim words: zeroed before use
// (claims of the previous batch) and after (the claim protocol reads values < 128 as stale).
struct ExpScratch {
  unsigned long long msub[64];
  unsigned long long mdel[64];
  uint32_t exx[128];  // [2s]: (63 - first exact edge) << 26 | its child (0: none); [2s+1]: same, swap edge
  uint32_t mark[64];  // unit -> owner state lane + 1 (per round)
};
static_assert(sizeof(ExpScratch) <= 4u * 512u, "scratch must fit the smallest claim region");

// Owner state lane of unit R + lane: states' unit ranges are consecutive in lane order, so the
// owner is the last state whose first unit is at or before it (LDS marks + max-scan).
__device__ __forceinline__ int unit_owner(ExpScratch* X, uint32_t R, uint32_t nunit, uint32_t ubase, bool valid,
                                          uint32_t& carry) {
  const uint32_t lane = lane_id();
  X->mark[lane] = 0u;
  __builtin_amdgcn_wave_barrier();
  if (nunit && ubase >= R && ubase < R + 64u) X->mark[ubase - R] = lane + 1u;
  __builtin_amdgcn_wave_barrier();
  uint32_t v = X->mark[lane];
  if (lane == 0) v = max(v, carry);
  v = wave_inclusive_max(v);
  carry = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  return (int)(valid ? v - 1u : lane);
}

// Edge work of a batch, balanced over lanes: each state's edges are cut into units of UK edges and
// the units of all states are dealt to lanes in rounds of 64 (a lane-per-state loop would run
// for the batch's largest degree). Per edge: the exact/swap first-char match (structs.rs:512-519),
// substitution (:814-874) and deletion (:1055-1088) keep tests incl. the last-edit dead-end filter.
template <uint32_t UK, bool MAP>
__device__ void expand_units(const SearchParams& P, ExpScratch* X, const DevNode& nd, const Prep& pr, bool act,
                             uint64_t& msub, uint64_t& mdel, uint32_t& ex, uint32_t& xe) {
  const uint32_t lane = lane_id();
  const uint32_t deg = act ? node_deg(nd) : 0u;
  const uint32_t nunit = (deg + UK - 1) / UK;
  const uint32_t uincl = wave_inclusive_sum(nunit);
  const uint32_t ubase = uincl - nunit;
  const uint32_t U = (uint32_t)__builtin_amdgcn_readlane((int)uincl, 63);
  const uint32_t pk = pr.flags | (deg << 9) | (ubase << 16);  // flags 9 bits, deg <= 64, ubase < 4096
  // the words may hold dedup claims of the previous batch
  X->msub[lane] = 0ull;
  X->mdel[lane] = 0ull;
  reinterpret_cast<uint2*>(X->exx)[lane] = make_uint2(0u, 0u);
  uint32_t carry = 0;
  for (uint32_t R = 0; R < U; R += 64) {
    const bool valid = R + lane < U;
    const int o = unit_owner(X, R, nunit, ubase, valid, carry);
    const uint32_t o_pk = __shfl(pk, o), o_eb = __shfl(nd.edge_begin, o);
    const uint32_t cur = __shfl(pr.cur_ch, o), nxt = __shfl(pr.next_ch, o), nc = __shfl(pr.nch, o);
    const float rem = __shfl(pr.remaining, o);
    uint32_t gc = 0, gn = 0;
    if constexpr (MAP) {
      gc = __shfl(pr.gcur, o);
      gn = __shfl(pr.gnx, o);
    }
    const uint32_t o_deg = (o_pk >> 9) & 0x7Fu, e0 = (R + lane - (o_pk >> 16)) * UK;
    const bool sub_on = o_pk & PF_SUB, del_ok = o_pk & PF_DEL, is_last = o_pk & PF_LAST, need_csb = o_pk & PF_CSB;
    const bool have_next = o_pk & PF_NEXT, have_cur = o_pk & PF_CUR, swap_ok = o_pk & PF_SWAP, ex_on = o_pk & PF_EX;
    uint32_t sb = 0, db = 0, fe = 0u, fx = 0u;  // fe/fx: exx encodings of the unit's first matches
#pragma unroll
    for (uint32_t i = 0; i < UK; ++i) {
      const uint32_t e = e0 + i;
      const bool ok = valid && e < o_deg;
      const DevEdge ed = P.edges[ok ? o_eb + e : 0u];
      const bool child_out = (ed.next & EDGE_CHILD_OUTPUT) != 0;
      const uint4 csb = P.sb_edge[(ok && need_csb) ? o_eb + e : 0u];  // parallel with the edge load
      const uint32_t enc = ((63u - e) << 26) | (ed.next & CHILD26_MASK);  // child ids < 2^26 (builder)
      bool mex, msw;
      if constexpr (MAP) {  // whole-grapheme transitions (structs.rs:452-464)
        const uint32_t eg = P.edge_gid[ok ? o_eb + e : 0u];
        mex = eg == gc;
        msw = eg == gn;
      } else {  // first-char transitions (structs.rs:512-519)
        mex = ed.ch == cur;
        msw = ed.ch == nc;
      }
      fe = (ok && ex_on && fe == 0u && mex) ? enc : fe;
      fx = (ok && swap_ok && fx == 0u && msw) ? enc : fx;
      const float sim = similarity(P, ed.ch, cur);
      const float penalty = __fmul_rn(P.p_sub, __fsub_rn(1.0f, sim));
      const bool sb_next = child_out || (have_next && sb_word_bit(csb, nxt));
      const bool sb_cur = child_out || (have_cur && sb_word_bit(csb, cur));
      // the exact edge's bit is cleared by the owner once the first match is known
      const bool keep_sub = ok && sub_on && !(sim < P.min_sym) && !(penalty > rem) && (!is_last || sb_next);
      const bool keep_del = ok && del_ok && (!is_last || sb_cur);
      sb |= (keep_sub ? 1u : 0u) << i;
      db |= (keep_del ? 1u : 0u) << i;
    }
    if (sb) atomicOr(&X->msub[o], (unsigned long long)sb << e0);
    if (db) atomicOr(&X->mdel[o], (unsigned long long)db << e0);
    if (fe) atomicMax(&X->exx[2 * o], fe);  // max = smallest edge index
    if (fx) atomicMax(&X->exx[2 * o + 1], fx);
  }
  __builtin_amdgcn_wave_barrier();
  msub = X->msub[lane];
  mdel = X->mdel[lane];
  const uint2 exw = reinterpret_cast<const uint2*>(X->exx)[lane];
  ex = exw.x;
  xe = exw.y;
  __builtin_amdgcn_wave_barrier();
  X->msub[lane] = 0ull;
  X->mdel[lane] = 0ull;
  reinterpret_cast<uint2*>(X->exx)[lane] = make_uint2(0u, 0u);
  __builtin_amdgcn_wave_barrier();
}

// O(1) expansion of one state (deg <= 64) when similarity cannot drop a substitution
// (gt_fast && p_sub <= remaining, see builder.cpp): every edge is a substitution and deletion
// candidate, filtered at the last edit by "child has output" (aux.xy) and "child has a single-byte
// edge for the tested char" (GT_SB maps), exactly the per-edge tests of expand_units; the exact and
// swap edges are the goto entries of text[j] and text[j+1]. A lookup whose char filter bit is clear
// (aux.z: the node's edge chars, aux.w: its children's single-byte chars) is known to miss and is
// not issued; a swap edge whose child's folded filter rules out text[j] has no swap target.
__device__ __forceinline__ bool filt_has(uint32_t f, uint32_t c) { return (f >> ch_filt_bit(c)) & 1u; }

// A state with P_sub > remaining pushes a substitution only if p_sub * (1 - sim) <= remaining
// (:864-866), i.e. for a large enough similarity. With no non-ASCII similarity pairs an edge whose
// first char differs from text[j] has similarity 0 unless both chars are ASCII (structs.rs:82-92),
// and then at most the table's largest similarity towards text[j] (sim_ascii[16384 + c]); an edge
// with text[j]'s first char is the exact edge unless two edges share a first char. When none of
// these can pass, the state has no substitution at all and the O(1) expansion applies (C3: most
// states past the first edit read a non-ASCII char or a space).
__device__ __forceinline__ bool no_subs(const SearchParams& P, const DevNode& nd, uint32_t cur, float remaining) {
  if (P.n_sim != 0 || (nd.degf & NODE_DUP_CH)) return false;
  if (cur >= 128u || !(nd.degf & NODE_ASCII_EDGE)) return true;
  return __fmul_rn(P.p_sub, __fsub_rn(1.0f, P.sim_ascii[128u * 128u + cur])) > remaining;
}

__device__ void expand_fast(const SearchParams& P, const KState& st, const DevNode& nd, const Prep& pr, uint4 aux,
                            uint64_t& msub, uint64_t& mdel, uint32_t& ex, uint32_t& xe) {
  const uint32_t deg = node_deg(nd);
  const uint64_t dm = deg >= 64u ? ~0ull : ((1ull << deg) - 1ull);
  const bool is_last = pr.flags & PF_LAST, in_text = pr.flags & PF_EX, sub_on = pr.flags & PF_SUB;
  const bool del_ok = pr.flags & PF_DEL, swap_ok = pr.flags & PF_SWAP;
  const uint64_t nk = GT_VALID | ((uint64_t)st.node << 21);
  const uint64_t cout = ((uint64_t)aux.y << 32) | aux.x;
  const bool l0 = in_text && filt_has(aux.z, pr.cur_ch);
  const bool l1 = swap_ok && filt_has(aux.z, pr.nch);
  const bool ns0 = is_last && del_ok && (pr.flags & PF_CUR) && pr.cur_ch < 128u && filt_has(aux.w, pr.cur_ch);
  const bool ns1 = is_last && sub_on && (pr.flags & PF_NEXT) && pr.next_ch < 128u && filt_has(aux.w, pr.next_ch);
  // one base hash per (node, char); c1 serves both the swap edge and the next-char dead-end map
  const uint32_t b0 = gt_base(st.node, pr.cur_ch, P.gt_seed1);
  const uint32_t c1 = (pr.flags & PF_SWAP) ? pr.nch : pr.next_ch;
  const uint32_t b1 = gt_base(st.node, c1, P.gt_seed1);
  uint64_t g0 = 0, g1 = 0, s0 = 0, s1 = 0;  // lookups in flight together
  bool h0 = false, h1 = false;
  if (__ballot(l0 || l1)) {
    h0 = gt_get_h(P, nk | GT_GOTO | pr.cur_ch, b0, l0, g0);
    h1 = gt_get_h(P, nk | GT_GOTO | pr.nch, b1, l1, g1);
  }
  if (__ballot(ns0 || ns1)) {  // child single-byte maps: last edit on an ASCII char only
    gt_get_h(P, nk | GT_SB | pr.cur_ch, gt_kind_hash(b0, true), ns0, s0);
    gt_get_h(P, nk | GT_SB | pr.next_ch, gt_kind_hash(b1, true), ns1, s1);
  }
  uint64_t exbit = 0;
  if (h0) {
    const uint32_t k = (uint32_t)(g0 >> 32) & 0xFFu;
    ex = ((63u - k) << 26) | (uint32_t)(g0 & CHILD26_MASK);
    exbit = 1ull << k;
  }
  if (h1 && ((uint32_t)(g1 >> 48) >> (ch_filt_bit(pr.cur_ch) & 15u) & 1u))
    xe = ((63u - ((uint32_t)(g1 >> 32) & 0xFFu)) << 26) | (uint32_t)(g1 & CHILD26_MASK);
  msub = (sub_on && P.p_sub <= pr.remaining) ? (dm & ~exbit & (is_last ? (cout | s1) : ~0ull)) : 0ull;  // else no_subs
  mdel = del_ok ? (dm & (is_last ? (cout | s0) : ~0ull)) : 0ull;
}

// Per-state completion: exact successor, the exact edge leaves the substitution set, swap target
// goto(goto(node, text[j+1]), text[j]) (:945-967), push count.
template <bool MAP>
__device__ LaneExp lane_finish(const SearchParams& P, const SegDesc& S, uint64_t start, const KState& st,
                               const DevNode& nd, const Prep& pr, uint64_t msub, uint64_t mdel, uint32_t ex,
                               uint32_t xe, unsigned& err) {
  LaneExp x{-1, -1, false, msub, mdel, 0u, 0ull};
  if (ex) {  // exx encodings (expand_units)
    x.exact = (int64_t)(ex & CHILD26_MASK);
    x.msub &= ~(1ull << (63u - (ex >> 26)));
  }
  if (xe) {  // node2 = goto(xnode, text[j]) through the goto table
    if constexpr (MAP) {
      x.swap = find_gid(P, xe & CHILD26_MASK, pr.gcur);
    } else {
      uint64_t g;
      if (gt_get(P, GT_VALID | GT_GOTO | ((uint64_t)(xe & CHILD26_MASK) << 21) | pr.cur_ch, true, g))
        x.swap = (int64_t)(g & CHILD26_MASK);
    }
    if (x.swap >= 0 && P.mef == 255u) {  // within_limits_swap_ahead with node2's limits (:962-967)
      const uint32_t packed = st.packed, edits = edits_of(packed);
      const Lim m = pick_limits(P, node_limits(P, (uint32_t)x.swap));
      if (!(m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.swp, packed >> 24)) : false)) x.swap = -1;
    }
  }
  x.ins = (pr.flags & PF_INS) != 0;
  if constexpr (MAP)  // inside the substitution block (:883), i.e. j < n and subst_ok
    if (pr.flags & PF_SUB) x.mmap = map_mask(P, S, st.node, start + (st.jm & 0xFFFFu), st.pen, err);
  x.count = (x.exact >= 0 ? 1u : 0u) + (uint32_t)__popcll(x.msub) + (x.swap >= 0 ? 1u : 0u) + (x.ins ? 1u : 0u) +
            (uint32_t)__popcll(x.mdel) + (uint32_t)__popcll(x.mmap);
  return x;
}

// position of the r-th (0-based) set bit of m; r < popcount(m)
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t m, uint32_t r) {
  uint32_t w = (uint32_t)m, base = 0;
  const uint32_t c32 = (uint32_t)__popc(w);
  if (r >= c32) {
    r -= c32;
    w = (uint32_t)(m >> 32);
    base = 32;
  }
#pragma unroll
  for (uint32_t half = 16; half >= 1; half >>= 1) {
    const uint32_t c = (uint32_t)__popc(w & ((1u << half) - 1u));
    const bool up = r >= c;
    r = up ? r - c : r;
    w = up ? w >> half : w;
    base = up ? base + half : base;
  }
  return base;
}

// Pushes of the committed states in the reference's order (search.rs:787-1088): per state exact,
// substitutions (edge order), swap, insertion, deletions (edge order), written at the state's
// exclusive-prefix offset. The owner lane writes exact/swap/insertion; substitutions and deletions
// are written by the units that cover their edges (balanced like expand_units).
template <uint32_t QCAP, uint32_t UK, bool MAP>
__device__ void push_units(const SearchParams& P, ExpScratch* X, KState* q, uint32_t base, const KState& st,
                           const DevNode& nd, const LaneExp& x, uint32_t cur_ch, bool act) {
  const uint32_t lane = lane_id();
  const float pen = st.pen;
  const uint32_t j_rel = st.jm & 0xFFFFu;
  const uint32_t jm1 = (j_rel + 1u) | ((j_rel + 1u) << 16);
  const uint32_t nex = x.exact >= 0 ? 1u : 0u, nsw = x.swap >= 0 ? 1u : 0u, nins = x.ins ? 1u : 0u;
  const uint32_t sub_base = base + nex;
  const uint32_t map_pos = sub_base + (uint32_t)__popcll(x.msub);
  const uint32_t sw_pos = map_pos + (uint32_t)__popcll(x.mmap);
  const uint32_t del_base = sw_pos + nsw + nins;
  if (act) {
    if (nex) q[base & (QCAP - 1)] = KState{(uint32_t)x.exact, jm1, pen, st.packed};
    if (nsw) {
      const uint32_t jm2 = (j_rel + 2u) | ((j_rel + 2u) << 16);
      q[sw_pos & (QCAP - 1)] = KState{(uint32_t)x.swap, jm2, __fadd_rn(pen, P.p_swp), st.packed + 0x1000000u};
    }
    if (nins) {
      const uint32_t jmi = (j_rel + 1u) | ((st.jm >> 16) << 16);
      q[(sw_pos + nsw) & (QCAP - 1)] = KState{st.node, jmi, __fadd_rn(pen, P.p_ins), st.packed + 1u};
    }
    if constexpr (MAP)
      if (x.mmap) {  // mapping pushes, after the substitutions (:883-922)
        const uint32_t mb = P.map_range[st.node].x;
        uint64_t mm = x.mmap;
        uint32_t pos = map_pos;
        while (mm) {
          const uint32_t t = (uint32_t)__ffsll((unsigned long long)mm) - 1u;
          mm &= mm - 1;
          const uint4 mt = P.map_ent[mb + t];
          const uint32_t jh = j_rel + mt.y;
          q[(pos++) & (QCAP - 1)] = KState{mt.z, jh | (jh << 16), __fadd_rn(pen, __uint_as_float(mt.w)), st.packed + 0x10000u};
        }
      }
  }
  // substitutions and deletions, one push per lane: push k of a state is the k-th set bit of its
  // msub, then of its mdel
  const uint32_t nsub = act ? (uint32_t)__popcll(x.msub) : 0u;
  const uint32_t npush = act ? nsub + (uint32_t)__popcll(x.mdel) : 0u;
  const uint32_t fincl = wave_inclusive_sum(npush);
  const uint32_t fbase = fincl - npush;
  const uint32_t F = (uint32_t)__builtin_amdgcn_readlane((int)fincl, 63);
  uint32_t carry = 0;
  for (uint32_t R = 0; R < F; R += 64) {
    const bool valid = R + lane < F;
    const int o = unit_owner(X, R, npush, fbase, valid, carry);
    const uint32_t o_fb = __shfl(fbase, o), o_ns = __shfl(nsub, o), o_eb = __shfl(nd.edge_begin, o);
    const uint64_t o_ms = shfl_var_u64(x.msub, o), o_md = shfl_var_u64(x.mdel, o);
    const uint32_t o_sb = __shfl(sub_base, o), o_db = __shfl(del_base, o), o_cur = __shfl(cur_ch, o);
    const float o_pen = __shfl(pen, o);
    const uint32_t o_jm = __shfl(st.jm, o), o_packed = __shfl(st.packed, o);
    if (valid) {
      const uint32_t k = R + lane - o_fb;
      const bool is_sub = k < o_ns;
      const uint32_t r = is_sub ? k : k - o_ns;
      const uint32_t e = nth_set_bit(is_sub ? o_ms : o_md, r);
      const DevEdge ed = P.edges[o_eb + e];
      const uint32_t child = ed.next & EDGE_NEXT_MASK;
      if (is_sub) {
        const float sim = similarity(P, ed.ch, o_cur);
        const float penalty = __fmul_rn(P.p_sub, __fsub_rn(1.0f, sim));
        const uint32_t o_j1 = (o_jm & 0xFFFFu) + 1u;
        q[(o_sb + r) & (QCAP - 1)] = KState{child, o_j1 | (o_j1 << 16), __fadd_rn(o_pen, penalty), o_packed + 0x10000u};
      } else {
        q[(o_db + r) & (QCAP - 1)] = KState{child, o_jm, __fadd_rn(o_pen, P.p_del), o_packed + 0x100u};
      }
    }
  }
}


// Read-only dedup lookup (per lane, linear probing). found/stored describe the table entry.
template <uint32_t VCAP>
__device__ __forceinline__ void vis_lookup(const KState* vis, const KState& s, bool& found, uint32_t& stored_bits,
                                           uint32_t& slot) {
  uint32_t h = vis_hash(s) & (VCAP - 1);
  found = false;
  stored_bits = 0;
  slot = EMPTY;
  for (uint32_t it = 0; it < VCAP; ++it) {
    const uint4 e = reinterpret_cast<const uint4*>(vis)[h];
    if (e.x == EMPTY) {
      slot = h;
      return;
    }
    if (e.x == s.node && e.y == s.jm && e.w == s.packed) {
      found = true;
      stored_bits = e.z;
      slot = h;
      return;
    }
    h = (h + 1) & (VCAP - 1);
  }
}

#ifndef FAC_UK
#define FAC_UK 2  // edges per expansion unit (measured: 2 > 4 > 8 on C2/C3)
#endif

#ifdef FAC_DUP  // analysis builds: a region executed twice, the copy fed opaque inputs
__device__ __forceinline__ uint32_t opq(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ float opqf(float v) { return __uint_as_float(opq(__float_as_uint(v))); }
__device__ __forceinline__ uint64_t opq64(uint64_t v) {
  return ((uint64_t)opq((uint32_t)(v >> 32)) << 32) | opq((uint32_t)v);
}
__device__ __forceinline__ void sink(uint32_t v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void sink64(uint64_t v) {
  sink((uint32_t)v);
  sink((uint32_t)(v >> 32));
}
#endif

constexpr uint32_t RC_POOL_CHUNK = 4096;  // largest pool chunk (words, 64 KiB) a building wave takes
// snapshot header words: {head, tail, nv, pops}, {ne, jcheck | ncheck << 16, jbeam, jp1} (the key's
// chars are read from the representative's text by rc_publish_kernel); jp1 = 1 + the largest j popped in the chain, jbeam = jp1 at the chain's last beam event (0:
// none), jcheck = min(jbeam, 1 + the largest j of the dedup entries): the entries a resumed dedup-free
// run must still honour have j < jcheck (the others were popped after every beam: their subtrees are
// intact); they are the first ncheck dedup entries (0: none)
constexpr uint32_t RC_HDR = 2;  // {head, tail, nv, pops}, {ne, jcheck | ncheck << 16, jbeam, jp1}
struct RcHit {  // prefix-cache snapshot of a window (rc_lookup): pool offset and header
  uint32_t off, head, tail, nv_nel, pops;
  uint32_t lvl = 0;  // rc_tab index of the hit (diagnostics)
};

// one best-map entry {me_rel, pattern, similarity bits, packed counts} of the window at `start`
// as the crate's OwnedMatch record (search.rs:1111-1118); sb = the window's start byte
__device__ __forceinline__ fac_match match_record(const SearchParams& P, const SegDesc& S, uint64_t start, uint64_t sb,
                                                  const uint4& ent) {
  const uint64_t me = start + ent.x;
  fac_match m;
  m.start = P.out_shift + sb;
  m.end = P.out_shift + S.byte_base + (me < S.n ? local_byte(P, S, me) : S.hay_len);
  m.pattern_index = ent.y;
  m.similarity = __uint_as_float(ent.z);
  m.insertions = ent.w & 0xFFu;
  m.deletions = (ent.w >> 8) & 0xFFu;
  m.substitutions = (ent.w >> 16) & 0xFFu;
  m.swaps = ent.w >> 24;
  m.edits = (uint8_t)edits_of(ent.w);
  m.pad[0] = m.pad[1] = m.pad[2] = 0;
  return m;
}

constexpr uint32_t claim_slots(uint32_t vcap) { return vcap / 2 < 512 ? 512 : vcap / 2; }  // >= ExpScratch

__device__ unsigned long long g_live_dbg[12];  // diagnostics (FAC_RC_DEBUG): live-dedup checks / hits, spills
__device__ unsigned long long g_bad[8];       // diagnostics (FAC_RC_DEBUG): uncached keys by reason
__device__ unsigned long long g_lk_dbg[16];   // diagnostics (FAC_RC_DEBUG): main lookups by level x final, misses, skips
#ifdef FAC_WIN_HIST  // diagnostics build (make hist): windows, pops and cycles by pops per window
__device__ unsigned long long g_hist[24];
__device__ __forceinline__ uint32_t hist_bucket(uint64_t pops) {  // 0, 1-15, 16-63, 64-255, 256-1023, 1024+
  return pops == 0 ? 0u : pops < 16 ? 1u : pops < 64 ? 2u : pops < 256 ? 3u : pops < 1024 ? 4u : 5u;
}
#endif
#ifdef FAC_PHASE_PROF  // diagnostics build (make prof): cycles per phase of run_window
constexpr int kProf = 48;  // accumulator slots per pass kind
__device__ unsigned long long g_prof[2 * kProf];  // [0, kProf): main passes, [kProf, 2 kProf): cache builds
#define PROF_T(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#define PROF_ACC(i, t0) prof_acc[i] += __builtin_amdgcn_s_memtime() - (t0)
#else
#define PROF_T(t)
#define PROF_ACC(i, t0)
#endif

// Wave slots (SearchParams::slot_ring): lane 0 takes the next position of the free ring and waits
// for the slot returned into it (positions are filled in return order); the ring starts as 0..n-1.
// A release waits until its cell is EMPTY (the previous lap's acquirer took its value), so a slow
// acquirer never has its value overwritten by a later lap's release (grids larger than n slots).
__device__ uint32_t slot_acquire(const SearchParams& P) {
  uint32_t s = 0;
  if (lane_id() == 0) {
    const unsigned int h = atomicAdd(P.slot_ctr, 1u);
    unsigned int* cell = P.slot_ring + (h % P.n_slots);
    while ((s = atomicExch(cell, EMPTY)) == EMPTY) __builtin_amdgcn_s_sleep(2);
  }
  return shfl_u32(s, 0);
}
__device__ void slot_release(const SearchParams& P, uint32_t s) {
  if (lane_id() == 0) {
    const unsigned int t = atomicAdd(P.slot_ctr + 1, 1u);
    unsigned int* cell = P.slot_ring + (t % P.n_slots);
    while (atomicCAS(cell, EMPTY, s) != EMPTY) __builtin_amdgcn_s_sleep(2);
  }
}
__global__ void slot_init_kernel(unsigned int* ring, unsigned int* ctr, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) ring[i] = i;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctr[0] = 0u;
    ctr[1] = n;
  }
}

// One start window, explored by one wavefront. States are popped in the reference's FIFO order in
// batches of up to 64 (one state per lane); a batch is cut exactly where the reference's sequential
// semantics would diverge: before the first in-batch dedup conflict, before the first pop at which
// the beam would trigger, and before the first >64-edge node (expanded alone, edge-parallel).
// LIVE (dedup-free variants of beamed engines, VCAP == 0): the resumed snapshot's live dedup entries
// go into a read-only table (live, LIVE_CAP slots) and a popped state equal to one of them with a
// stored penalty <= its own is skipped as the reference's visited map would (search.rs:618-622): the
// window itself runs dedup-free, which cannot change results while no beam triggers -- except against
// states popped before the snapshot, whose subtrees a beam may have pruned (live_dup).
constexpr uint32_t LIVE_CAP = 256;
template <uint32_t VCAP, uint32_t QCAP, bool MAP, bool LIVE = false>
__device__ __forceinline__ uint32_t run_window(const SearchParams& P, const SegDesc& S, KState* vis, KState* q, uint32_t* claim,
                           uint32_t& cseq, EmitList& EL, uint64_t start, const RcHit& rc, uint64_t& popped,
                           uint64_t& cached, unsigned& err, uint32_t& head_out, uint32_t& vcount_out,
                           KState* live = nullptr, uint32_t* jbeam_out = nullptr, uint4* bsel = nullptr
#ifdef FAC_PHASE_PROF
                           , uint64_t* prof_acc = nullptr  // the wave's accumulators (bfs_window_body), added up at its end
#endif
                           ) {
  const uint32_t lane = lane_id();
  const uint64_t popped_w0 = popped;  // diagnostics: this window's pops
  if constexpr (LIVE)  // a window resuming with a long queue would most likely beam: the exact variant takes it
    if (P.live_nqmax && rc.off != EMPTY && rc.tail - rc.head > P.live_nqmax) {
      err |= ERR_QUEUE;
      head_out = rc.head;
      vcount_out = 0;
      return rc.tail;
    }
  // FAC_PHASE_PROF slots: 12: per-edge states, 13: fast states, 14: committed, 15: loaded, 16-19: Bc
  // buckets, 20: prologue (table clear, snapshot load), 21: flush
  PROF_T(t_win);
  if constexpr (VCAP > 0)
    for (uint32_t i = lane; i < VCAP; i += 64) vis[i].node = EMPTY;
  PROF_ACC(37, t_win);
  PROF_T(t_load);
  uint32_t vcount = 0;
  EL.n = 0;
  uint32_t head = 0, tail = 1;
  // LIVE: the snapshot's entries a popped state may still meet have j < jlive (0: none); the table is
  // filled on the first batch that holds such a state (live_loaded), most windows never need it
  uint32_t jlive = 0;
  bool live_loaded = false;
  if constexpr (LIVE) {
    const uint32_t nv = rc.off != EMPTY ? (rc.nv_nel & 0xFFFFu) : 0u;
    if (nv) jlive = P.rc_pool[rc.off + 1].y;  // jcheck | ncheck << 16
    if (P.lane_debug && lane == 0) atomicAdd(&g_live_dbg[jlive ? 4 : 5], 1ull);
  }
  // cache builds of beamed engines: jbeam = 1 + the largest j popped before the last beam event of the
  // snapshot chain (0: none). Only dedup entries popped before a beam can have beam-pruned subtrees,
  // i.e. only they matter to a resumed dedup-free run (run_window LIVE, lane_window_kernel).
  // jp1: 1 + the largest j popped in the chain so far (0: none), kept per lane (the lanes' committed
  // states) and reduced over the wave only at beam events and at the end
  uint32_t jp1 = 0, jbeam = 0;
  const bool track_beam = P.rc_mode == 2 && P.beam;
  if (track_beam && rc.off != EMPTY) {
    const uint4 h1 = P.rc_pool[rc.off + 1];
    jbeam = h1.z;
    jp1 = h1.w;
  }
  if (rc.off != EMPTY) {  // prefix cache hit: resume from the snapshot of the key's representative
    const uint4* src = P.rc_pool + rc.off + RC_HDR;  // queue, dedup entries, best list (header in rc)
    head = rc.head;
    tail = rc.tail;
    const uint32_t nq = tail - head, nv = rc.nv_nel & 0xFFFFu, ne = rc.nv_nel >> 16, nw = nq + nv + ne;
    if constexpr (VCAP > 0) __builtin_amdgcn_wave_barrier();  // the table clear above
    for (uint32_t b = 0; b < nw; b += 256) {  // four loads in flight per lane, then their stores
      uint4 w[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t i = b + u * 64 + lane;
        // (a dedup-free variant has no table for the snapshot's dedup entries: not loaded)
        if (i < nw && (VCAP > 0 || i < nq || i >= nq + nv)) w[u] = src[i];
      }
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t i = b + u * 64 + lane;
        if (i >= nw) continue;
        if (i < nq) {
          q[(head + i) & (QCAP - 1)] = KState{w[u].x, w[u].y, __uint_as_float(w[u].z), w[u].w};
        } else if (i < nq + nv) {
          if constexpr (VCAP > 0) {  // a live popped key with its stored penalty (slot re-hashed)
            uint32_t slot = vis_hash(KState{w[u].x, w[u].y, 0.f, w[u].w}) & (VCAP - 1);
            while (atomicCAS(&vis[slot].node, EMPTY, w[u].x) != EMPTY) slot = (slot + 1) & (VCAP - 1);
            vis[slot].jm = w[u].y;
            vis[slot].pen = __uint_as_float(w[u].z);
            vis[slot].packed = w[u].w;
          }
        } else {
          EL.buf[i - nq - nv] = w[u];
        }
      }
    }
    if constexpr (VCAP > 0) vcount = __builtin_amdgcn_readfirstlane(nv);
    EL.n = ne;
    cached += rc.pops;  // the snapshot's pops (not counted as popped: that is executed work)
  } else if (lane == 0) {
    q[0] = KState{0u, 0u, 0.0f, 0u};
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t beam2 = 2u * P.beam;
  PROF_ACC(38, t_load);
  PROF_ACC(20, t_win);

  while (head < tail) {
    PROF_T(t0);
    if constexpr (VCAP > 0) {
      if (P.beam && tail - head > beam2) {
        // (tail by value: a reference into these noinline calls kept it in scratch memory for the whole
        // window loop, reloaded with a full vmcnt wait wherever it was read)
        if (P.beam_canonical) beam_select_canonical<QCAP>(q, head, tail, P.beam);  // diagnostics
        else if constexpr (QCAP <= 256) beam_select_lds<QCAP>(q, head, tail, P.beam, claim, P.sel_limit);  // :577-589
        else beam_select<QCAP>(q, head, tail, P.beam, bsel, P.sel_limit);
        tail = head + P.beam;  // truncate(bw) (:587)
        if (track_beam) jbeam = max(jbeam, shfl_u32(wave_inclusive_max(jp1), 63));
      }
    } else if (P.beam && tail - head > beam2) {
      // a beamed window in a dedup-free variant: until its pending count first passes 2·bw the
      // beam never triggers and dedup cannot change results (a dedup-free queue is
      // never shorter than the dedup queue at the same pop). Here it would: the window is spilled
      // and re-run from its start (snapshot) on a dedup variant.
      err |= ERR_QUEUE;
      if (P.lane_debug && lane == 0) {  // spilled windows: their live pops, snapshot queue, pops / queue at the spill
        atomicAdd(&g_live_dbg[6], 1ull);
        atomicAdd(&g_live_dbg[7], (unsigned long long)(popped - popped_w0));
        atomicAdd(&g_live_dbg[8], (unsigned long long)(rc.off != EMPTY ? rc.tail - rc.head : 1u));
        atomicAdd(&g_live_dbg[9], (unsigned long long)(tail - (rc.off != EMPTY ? rc.head : 0u)));
        if (tail - (rc.off != EMPTY ? rc.head : 0u) <= QCAP) atomicAdd(&g_live_dbg[10], 1ull);
      }
      break;
    }
    // cache build: stop before the first state that reads text past the key
    if (P.rc_mode == 2 && (q[head & (QCAP - 1)].jm & 0xFFFFu) + 1u >= P.rc_k) break;
    PROF_ACC(0, t0);
    PROF_T(t1);
    const uint32_t B = min(tail - head, 64u);
    const bool in_b = lane < B;
    KState st{EMPTY, 0u, 0.0f, 0u};
    if (in_b) st = q[(head + lane) & (QCAP - 1)];
    // ---- phase A: the state's global reads go out first (node record, own single-byte map,
    // text at j and j + 1) and overlap the dedup probe; then dedup, node ceiling, width
    DevNode nd{};
    uint32_t c0 = 0, c1 = 0;
    uint4 aux = make_uint4(0, 0, 0, 0);
    if (in_b) {
      nd = P.nodes[st.node];
      aux = P.aux[st.node];
      const uint64_t j = start + (st.jm & 0xFFFFu);
      if (j < S.n) c0 = text_char(P, S, j, err);
      if (j + 1 < S.n) c1 = text_char(P, S, j + 1, err);
    }
    uint32_t g0 = 0, g1 = 0;
    if constexpr (MAP)
      if (in_b) {
        const uint64_t j = start + (st.jm & 0xFFFFu);
        if (j < S.n) g0 = text_gid(P, S, j, err);
        if (j + 1 < S.n) g1 = text_gid(P, S, j + 1, err);
      }

    bool found = false;
    uint32_t stored_bits = 0, vslot = EMPTY;
    if constexpr (VCAP > 0)  // VCAP == 0: no dedup (unbeamed only)
      if (in_b) vis_lookup<VCAP>(vis, st, found, stored_bits, vslot);
#if defined(FAC_DUP) && FAC_DUP == 3
    if constexpr (VCAP > 0)
      if (in_b) {
        KState s2{opq(st.node), opq(st.jm), opqf(st.pen), opq(st.packed)};
        bool f2;
        uint32_t b2, v2;
        vis_lookup<VCAP>(vis, s2, f2, b2, v2);
        sink(b2 + v2 + (f2 ? 1u : 0u));
      }
#endif
    if constexpr (LIVE) {  // read-only: the snapshot's popped states (run_window LIVE)
      const bool chk = jlive && in_b && (st.jm & 0xFFFFu) + 1u <= (jlive & 0xFFFFu);
      if (__ballot(chk) && !live_loaded) {  // first need: the snapshot's check entries into the table
        const uint32_t nv = jlive >> 16, nq = rc.tail - rc.head;
        if (nv > LIVE_CAP - LIVE_CAP / 4) {  // too many for the table: the dedup variant takes the window
          err |= ERR_QUEUE;
          break;
        }
        for (uint32_t i = lane; i < LIVE_CAP; i += 64) live[i].node = EMPTY;
        __builtin_amdgcn_wave_barrier();
        const uint4* src = P.rc_pool + rc.off + RC_HDR + nq;
        for (uint32_t i = lane; i < nv; i += 64) {
          const uint4 w = src[i];
          uint32_t slot = vis_hash(KState{w.x, w.y, 0.f, w.w}) & (LIVE_CAP - 1);
          while (atomicCAS(&live[slot].node, EMPTY, w.x) != EMPTY) slot = (slot + 1) & (LIVE_CAP - 1);
          live[slot].jm = w.y;
          live[slot].pen = __uint_as_float(w.z);
          live[slot].packed = w.w;
        }
        __builtin_amdgcn_wave_barrier();
        live_loaded = true;
      }
      if (chk) vis_lookup<LIVE_CAP>(live, st, found, stored_bits, vslot);
      if (P.lane_debug && lane == 0) {
        atomicAdd(&g_live_dbg[2], (unsigned long long)__popcll(__ballot(chk)));
        atomicAdd(&g_live_dbg[3], (unsigned long long)__popcll(__ballot(found && __uint_as_float(stored_bits) <= st.pen)));
      }
    }
    const bool skip = in_b && found && __uint_as_float(stored_bits) <= st.pen;  // :620
    const bool alive =
        in_b && !skip && !(st.pen > __fsub_rn(nd.prune_len, __fmul_rn(nd.prune_lw, P.thr)));  // :638-642
    if (!alive) nd = DevNode{};
    const bool wide = alive && node_deg(nd) > 64u;
    const uint64_t mwide = __ballot(wide);
    PROF_ACC(1, t1);
    if (mwide & 1ull) {  // first state alone, edge-parallel
      PROF_T(t2);
      const KState s0 = q[head & (QCAP - 1)];
      head += 1;
      popped += 1;
      if (track_beam) jp1 = max(jp1, (s0.jm & 0xFFFFu) + 1u);
      if constexpr (VCAP > 0)
        if (visited_check<VCAP>(vis, vcount, s0, P.exact_dedup != 0, err)) continue;
      const DevNode n0 = P.nodes[s0.node];
      if (node_has_out(n0)) emit_state(P, EL, s0.jm >> 16, s0.pen, s0.packed, s0.node, err);
      expand_wide<QCAP, MAP>(P, S, q, head, tail, s0, n0, start, err);
      PROF_ACC(2, t2);
      if (any_err(err)) break;
      continue;
    }
    PROF_T(t3);
    uint32_t Bc = mwide ? (uint32_t)first_lane(mwide) : B;
    // ---- phase B: per-lane expansion decisions and push counts
    LaneExp x{-1, -1, false, 0ull, 0ull, 0u, 0ull};
    const bool act = alive && lane < Bc;
    Prep pr{0u, 0u, 0u, 0u, 0.0f};
    PROF_T(tb0);
    if (act) pr = lane_prep(P, S, st, nd, start, c0, c1, nd.sb);
    if constexpr (MAP) {
      pr.gcur = g0;
      pr.gnx = g1;
    }
    PROF_ACC(9, tb0);
    PROF_T(tb1);
    uint64_t msub = 0, mdel = 0;
    uint32_t ex = 0u, xe = 0u;
    const bool fast =
        act && P.gt_fast && (!(pr.flags & PF_SUB) || P.p_sub <= pr.remaining || no_subs(P, nd, pr.cur_ch, pr.remaining));
#ifdef FAC_PHASE_PROF
    prof_acc[12] += (uint64_t)__popcll(__ballot(act && !fast));
    prof_acc[13] += (uint64_t)__popcll(__ballot(fast));
#endif
    if (__ballot(act && !fast))  // per-edge path for the states similarity can prune
      expand_units<FAC_UK, MAP>(P, reinterpret_cast<ExpScratch*>(claim), nd, pr, act && !fast, msub, mdel, ex, xe);
    if (fast) expand_fast(P, st, nd, pr, aux, msub, mdel, ex, xe);
#if defined(FAC_DUP) && FAC_DUP == 1
    if (fast) {
      KState s2{opq(st.node), opq(st.jm), opqf(st.pen), opq(st.packed)};
      DevNode n2{opqf(nd.prune_len), opqf(nd.prune_lw), opq(nd.edge_begin), opq(nd.degf),
                 make_uint4(opq(nd.sb.x), opq(nd.sb.y), opq(nd.sb.z), opq(nd.sb.w))};
      Prep p2{opq(pr.cur_ch), opq(pr.next_ch), opq(pr.nch), opq(pr.flags), opqf(pr.remaining)};
      uint64_t a = 0, b = 0;
      uint32_t c = 0, d = 0;
      expand_fast(P, s2, n2, p2, make_uint4(opq(aux.x), opq(aux.y), opq(aux.z), opq(aux.w)), a, b, c, d);
      sink64(a);
      sink64(b);
      sink(c);
      sink(d);
    }
#endif
    PROF_ACC(10, tb1);
    PROF_T(tb2);
    if (act) x = lane_finish<MAP>(P, S, start, st, nd, pr, msub, mdel, ex, xe, err);
#if defined(FAC_DUP) && FAC_DUP == 2
    if (act) {
      KState s2{opq(st.node), opq(st.jm), opqf(st.pen), opq(st.packed)};
      DevNode n2{opqf(nd.prune_len), opqf(nd.prune_lw), opq(nd.edge_begin), opq(nd.degf),
                 make_uint4(opq(nd.sb.x), opq(nd.sb.y), opq(nd.sb.z), opq(nd.sb.w))};
      const Prep p2 = lane_prep(P, S, s2, n2, start, opq(c0), opq(c1), n2.sb);
      const LaneExp x2 = lane_finish<MAP>(P, S, start, s2, n2, p2, opq64(msub), opq64(mdel), opq(ex), opq(xe), err);
      sink(p2.flags);
      sink(p2.cur_ch);
      sink(x2.count);
      sink64(x2.msub);
      sink64((uint64_t)x2.exact);
      sink64((uint64_t)x2.swap);
    }
#endif
    PROF_ACC(11, tb2);
    const uint32_t cnt = (lane < Bc) ? x.count : 0u;
    const uint32_t incl = wave_inclusive_sum(cnt);
    const uint32_t excl = incl - cnt;
    // cut: before pop k (k >= 1) the reference checks pending = P0 - k + S_k (:579-580); the queue
    // ring must also hold everything pushed by the committed states.
    const uint32_t P0 = tail - head;
    const bool trig = lane >= 1 && lane < Bc && P.beam && (P0 - lane + excl > beam2);
    const bool ovf = lane < Bc && (P0 - lane - 1 + incl > QCAP);
    const bool past = P.rc_mode == 2 && lane < Bc && (st.jm & 0xFFFFu) + 1u >= P.rc_k;  // cache build
    const uint64_t mcut = __ballot(trig) | __ballot(ovf) | __ballot(past);
#ifdef FAC_PHASE_PROF
    {  // cut reasons (the first cut lane's): 25 beam trigger, 26 ring, 27 key end (builds), 29 wide node
      const uint64_t mt = __ballot(trig), mo = __ballot(ovf), mp = __ballot(past);
      const uint32_t f = mcut ? (uint32_t)first_lane(mcut) : 64u;
      if (f < Bc) {
        prof_acc[25] += ((mt >> f) & 1ull) ? 1 : 0;
        prof_acc[26] += ((mo >> f) & 1ull) ? 1 : 0;
        prof_acc[27] += ((mp >> f) & 1ull) ? 1 : 0;
      } else if (Bc < B) {
        prof_acc[29] += 1;
      }
      prof_acc[31] += B == 64u ? 1 : 0;
    }
#endif
    if (mcut) Bc = min(Bc, (uint32_t)first_lane(mcut));
    if (Bc == 0) {
      err |= ERR_QUEUE;
      break;
    }
    PROF_ACC(3, t3);
    PROF_T(t4);
    // ---- phase C: dedup commit (search.rs:617-627 in FIFO order). Lanes with the same key found
    // the same slot in phase A, so each writer claims its slot (lowest lane wins). A writer whose key
    // equals an earlier writer's sees, in sequential order, the table entry that earlier pop left:
    // it is skipped iff the smallest penalty among the same-key writers before it (the stored
    // penalty is above all of them) is <= its own (search.rs:618-622), else it lowers the entry. Those
    // in-batch duplicates are resolved here (a segmented prefix minimum over the batch) instead of
    // cutting the batch before them; their pushes drop out of the prefix sums below, and the beam /
    // ring cuts taken above with their pushes counted stay conservative (a cut only ends the batch
    // early; the next batch re-checks the beam at its first pop). Winners write in parallel; losers
    // (distinct keys that met at one claim word or empty slot) insert serially in lane order.
    uint64_t nskip = 0;  // wave-uniform: in-batch duplicates the sequential order skips
    if constexpr (VCAP > 0) {
      const bool wr = lane < Bc && !skip;
      cseq += 1;
      if (cseq >= (1u << 26)) {  // sequence wrap: forget all claims
        for (uint32_t i = lane; i < claim_slots(VCAP); i += 64) claim[i] = 0u;
        __builtin_amdgcn_wave_barrier();
        cseq = 2;
      }
      // claims are hashed to VCAP/2 words: lanes of different slots may share one (then they are
      // "losers" with distinct keys and take the serial insert, which also handles found keys)
      const uint32_t cs = vslot & (claim_slots(VCAP) - 1);
      if (wr && vslot != EMPTY) atomicMax(&claim[cs], (cseq << 6) | (63u - lane));
      __builtin_amdgcn_wave_barrier();
      const uint32_t w = (wr && vslot != EMPTY) ? 63u - (claim[cs] & 63u) : lane;
      const uint32_t wn = __shfl(st.node, (int)w), wj = __shfl(st.jm, (int)w), wp = __shfl(st.packed, (int)w);
      const bool same = wr && w != lane && wn == st.node && wj == st.jm && wp == st.packed;
      const bool loser = wr && w != lane && !same;
      uint64_t dup = __ballot(same);
      const uint64_t lmask = __ballot(loser);
      if (lmask && P.dup_cut) {
        bool d2 = false;
        uint64_t mm = lmask;
        while (mm) {
          const int l = first_lane(mm);
          mm &= mm - 1;
          const uint32_t kn = shfl_u32(st.node, l), kj = shfl_u32(st.jm, l), kp = shfl_u32(st.packed, l);
          d2 = d2 || (loser && lane > (uint32_t)l && kn == st.node && kj == st.jm && kp == st.packed);
        }
        dup |= __ballot(d2);
      }
#ifdef FAC_PHASE_PROF
      prof_acc[28] += (dup && (uint32_t)first_lane(dup) < Bc) ? 1 : 0;  // batches holding an in-batch duplicate
      prof_acc[30] += (uint64_t)__popcll(dup & ((Bc >= 64u) ? ~0ull : ((1ull << Bc) - 1ull)));  // duplicate lanes
#endif
      if (P.dup_cut) {  // diagnostics (FAC_DUP_CUT): the round-5 rule, cut before the first duplicate
        if (dup) Bc = min(Bc, (uint32_t)first_lane(dup));  // lane 0 is never a duplicate
        dup = 0;
      }
      // same-key duplicates of a winner: prefix minimum over the writers of their key before them
      const uint64_t bmask = Bc >= 64u ? ~0ull : ((1ull << Bc) - 1ull);
      uint64_t ds = dup & bmask;
      while (ds) {
        const int l = first_lane(ds);
        ds &= ds - 1;
        const uint32_t kn = shfl_u32(st.node, l), kj = shfl_u32(st.jm, l), kp = shfl_u32(st.packed, l);
        const bool eq = wr && lane < (uint32_t)l && kn == st.node && kj == st.jm && kp == st.packed;
        const uint32_t mn = wave_min_u32(eq ? pen_order(st.pen) : 0xFFFFFFFFu);
        if (mn <= pen_order(shfl_f32(st.pen, l))) nskip |= 1ull << l;
      }
      const bool wrc = wr && lane < Bc;
      const uint32_t n_ins = (uint32_t)__popcll(__ballot(wrc && !found));
      const bool full = vcount + n_ins >= VCAP - VCAP / 8;
      if (!full && !__ballot(wrc && vslot == EMPTY)) {
        if (wrc && w == lane) {
          if (found) vis[vslot].pen = st.pen;  // lower the stored penalty (:623)
          else vis[vslot] = st;                // insert (:626)
        }
        vcount = __builtin_amdgcn_readfirstlane(vcount + (uint32_t)__popcll(__ballot(wrc && w == lane && !found)));
        __builtin_amdgcn_wave_barrier();
        // the same-key duplicates that are not skipped lower the entry, in lane order (each below
        // every earlier one: the last leaves the smallest)
        uint64_t dl = dup & bmask & ~nskip;
        while (dl) {
          const int l = first_lane(dl);
          dl &= dl - 1;
          if (lane == (uint32_t)l) vis[vslot].pen = st.pen;
          __builtin_amdgcn_wave_barrier();
        }
        uint64_t ml = __ballot(wrc && loser);
        while (ml) {
          const int l = first_lane(ml);
          ml &= ml - 1;
          KState kt;
          kt.node = shfl_u32(st.node, l);
          kt.jm = shfl_u32(st.jm, l);
          kt.pen = shfl_f32(st.pen, l);
          kt.packed = shfl_u32(st.packed, l);
          if (visited_check<VCAP>(vis, vcount, kt, P.exact_dedup != 0, err)) nskip |= 1ull << l;  // a loser's duplicate
        }
      } else {  // near-full table: the reference order, one state at a time
        nskip = 0;
        const uint64_t mw = __ballot(wr);
        for (uint32_t t = 0; t < Bc; ++t) {
          if (!((mw >> t) & 1ull)) continue;
          KState kt;
          kt.node = shfl_u32(st.node, t);
          kt.jm = shfl_u32(st.jm, t);
          kt.pen = shfl_f32(st.pen, t);
          kt.packed = shfl_u32(st.packed, t);
          if (visited_check<VCAP>(vis, vcount, kt, P.exact_dedup != 0, err)) nskip |= 1ull << t;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    PROF_ACC(4, t4);
    PROF_T(t5);
    // in-batch duplicates skipped above push nothing: the pushes' offsets without them
    const bool keep = alive && lane < Bc && !((nskip >> lane) & 1ull);
    const uint32_t cnt2 = keep ? x.count : 0u;
    const uint32_t incl2 = nskip ? wave_inclusive_sum(cnt2) : incl;
    const uint32_t excl2 = incl2 - cnt2;
    // ---- phase D: emissions (FIFO order), then pushes at tail + exclusive prefix
    uint64_t mem = __ballot(keep && node_has_out(nd));
    while (mem) {
      const int l = first_lane(mem);
      mem &= mem - 1;
      emit_state(P, EL, shfl_u32(st.jm, l) >> 16, shfl_f32(st.pen, l), shfl_u32(st.packed, l), shfl_u32(st.node, l),
                 err);
    }
    PROF_ACC(5, t5);
    PROF_T(t6);
    push_units<QCAP, FAC_UK, MAP>(P, reinterpret_cast<ExpScratch*>(claim), q, tail + excl2, st, nd, x, pr.cur_ch,
                                  keep && x.count != 0);
#if defined(FAC_DUP) && FAC_DUP == 4
    push_units<QCAP, FAC_UK, MAP>(P, reinterpret_cast<ExpScratch*>(claim), q, opq(tail + excl2), st, nd, x, opq(pr.cur_ch),
                             keep && x.count != 0);  // same entries rewritten
#endif
    __builtin_amdgcn_wave_barrier();
    tail += shfl_u32(incl2, Bc - 1);
    if (track_beam && lane < Bc) jp1 = max(jp1, (st.jm & 0xFFFFu) + 1u);
    head += Bc;
    popped += Bc;
    PROF_ACC(6, t6);
#ifdef FAC_PHASE_PROF
    prof_acc[8] += 1;  // batches
    prof_acc[14] += Bc;
    prof_acc[15] += B;
    prof_acc[16] += Bc <= 4 ? 1 : 0;  // constant indices: the accumulators stay in registers
    prof_acc[17] += Bc > 4 && Bc <= 16 ? 1 : 0;
    prof_acc[18] += Bc > 16 && Bc <= 40 ? 1 : 0;
    prof_acc[19] += Bc > 40 ? 1 : 0;
#endif
    if (any_err(err)) break;
  }

  PROF_T(t_fl);
  head_out = head;
  vcount_out = vcount;
  if (jbeam_out) {
    jbeam_out[0] = jbeam;
    jbeam_out[1] = track_beam ? shfl_u32(wave_inclusive_max(jp1), 63) : 0u;
  }
  // flush this window's best map (search.rs:1111-1118)
  wave_mem_fence();
  // a window that overflowed the frontier is spilled whole (re-run on a larger variant): no flush;
  // a cache build's representative is searched again by the main pass: no flush either
  if (EL.n && P.rc_mode != 2 && !(wave_or(err) & (ERR_EMIT | ERR_QUEUE | ERR_VISITED))) {
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(P.counters, (unsigned long long)EL.n);
    base = shfl_u64(base, 0);
    const uint64_t sb = S.byte_base + local_byte(P, S, start);
    for (uint32_t i = lane; i < EL.n; i += 64) {
      if (base + i >= P.out_cap) break;
      P.out[base + i] = match_record(P, S, start, sb, EL.buf[i]);
    }
  }
#ifdef FAC_PHASE_PROF
  PROF_ACC(21, t_fl);
  PROF_ACC(7, t_win);
#endif
  return tail;  // states pushed this window, the root included: the reference's queue.len()
}

// Key partition (Haystack::kparts): a start window belongs to part hash(its first two characters,
// folded as the keys fold them) mod parts. Every prefix-cache key extends its window's first two
// characters (keys hold >= 2), so a key's windows -- and its snapshot -- live in one part.
__device__ __forceinline__ bool kp_owned_chars(const SearchParams& P, uint32_t c0, uint32_t c1) {
  uint32_t h = (c0 * 0x9E3779B1u) ^ (c1 * 0x85EBCA6Bu);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h % P.kp_n == P.kp_r;
}
__device__ __forceinline__ bool window_owned_kp(const SearchParams& P, const SegDesc& S, uint64_t s, unsigned& err) {
  if (P.kp_n <= 1u) return true;
  const uint32_t c0 = text_char(P, S, s, err);
  const uint32_t c1 = s + 1 < S.n ? text_char(P, S, s + 1, err) : 0xFFFFFFFFu;
  return kp_owned_chars(P, c0, c1);
}

// 2-gram window skip (search.rs:535-553)
__device__ __forceinline__ bool window_skipped(const SearchParams& P, const SegDesc& S, uint64_t s, unsigned& err) {
  if (!P.window_skip) return false;
  const uint32_t ch = text_char(P, S, s, err);
  if (ch < 128u && !((P.first_bits[ch >> 5] >> (ch & 31u)) & 1u)) {
    if (s + 1 >= S.n) return true;
    const uint32_t nc = text_char(P, S, s + 1, err);
    if (nc < 128u && !((P.second_bits[nc >> 5] >> (nc & 31u)) & 1u)) return true;
  }
  return false;
}


__device__ __forceinline__ uint32_t find_seg(const SearchParams& P, uint64_t v) {
  uint32_t lo = 0, hi = P.n_segs;  // last k with prefix[k] <= v
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P.seg_prefix[mid] <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Prefix-cache key of a window: its first k (<= 8) chars (0x1FFFFF past the end of the text and
// in unused positions) and a 64-bit hash of them (top bit set: 0 marks an empty table slot). A
// snapshot stores the chars and a lookup compares them, so hash collisions only cost a cache miss.
// False: not cacheable (a char inside the text but beyond the resident halo).
struct RcChars {
  uint4 a, b;
};
constexpr uint32_t RC_PAD = 0x1FFFFFu;
// the window's first k chars (RC_PAD past the end of the text); false: a char inside the text but
// beyond the resident halo (not cacheable)
__device__ __forceinline__ bool rc_chars(const SearchParams& P, const SegDesc& S, uint64_t s, uint32_t k, uint32_t c[8]) {
  unsigned e2 = 0;
  bool ok = true;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) {
    c[i] = RC_PAD;
    if (i < k && s + i < S.n) {
      if (s + i >= S.avail) ok = false;
      else c[i] = text_char(P, S, s + i, e2);
    }
  }
  return ok;
}
// key of the first k of the chars c (the rest padded)
__device__ __forceinline__ uint64_t rc_hash_chars(const uint32_t c[8], uint32_t k, RcChars& ch) {
  uint32_t d[8];
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) d[i] = i < k ? c[i] : RC_PAD;
  ch.a = make_uint4(d[0], d[1], d[2], d[3]);
  ch.b = make_uint4(d[4], d[5], d[6], d[7]);
  uint64_t h = 0x632BE59BD9B4E019ull ^ k;
#pragma unroll
  for (uint32_t i = 0; i < 8; i += 2) {
    const uint64_t w = ((uint64_t)d[i + 1] << 21) | d[i];
    h = (h ^ w) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
  }
  h *= 0xD6E8FEB86659FD93ull;
  h ^= h >> 32;
  return h | (1ull << 63);
}
__device__ __forceinline__ bool rc_key(const SearchParams& P, const SegDesc& S, uint64_t s, uint32_t k, RcChars& ch,
                                       uint64_t& key) {
  uint32_t c[8];
  if (!rc_chars(P, S, s, k, c)) return false;
  key = rc_hash_chars(c, k, ch);
  return true;
}
__device__ __forceinline__ uint32_t rc_hash(uint64_t k) { return (uint32_t)k ^ (uint32_t)(k >> 32); }
constexpr uint32_t RC_PROBES = 32;
constexpr uint32_t RC_OCC = 1u << 31, RC_POPS_MASK = (1u << 22) - 1;
constexpr uint32_t RC_DONE = 0xFFFFFFFEu;  // rc_hits: window skipped or finished by its snapshot
constexpr uint32_t RC_REGION = 1024;       // main pass: windows per region of compacted open entries
__device__ __forceinline__ uint64_t rc_window_of(const SearchParams& P, uint64_t e) {  // entry -> window
  return (e / RC_REGION) * RC_REGION + P.rc_voff[e];
}
// exact lookup key: the first k chars as 16-bit units (0xFFFF pads; chars >= 0xFFFF are not encoded)
__device__ __forceinline__ uint4 rc_exact_key(const uint32_t c[8], uint32_t k) {
  uint32_t u[8];
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) u[i] = (i < k && c[i] != RC_PAD) ? (c[i] & 0xFFFFu) : 0xFFFFu;
  return make_uint4(u[0] | (u[1] << 16), u[2] | (u[3] << 16), u[4] | (u[5] << 16), u[6] | (u[7] << 16));
}
__device__ __forceinline__ uint32_t rc_key_hash(uint4 k) {
  uint64_t h = (((uint64_t)k.y << 32) | k.x) * 0x9E3779B97F4A7C15ull;
  h ^= (((uint64_t)k.w << 32) | k.z) + 0x632BE59BD9B4E019ull + (h >> 29);
  h *= 0xD6E8FEB86659FD93ull;
  return (uint32_t)(h >> 32) ^ (uint32_t)h;
}

// A window's prefix-cache hit (from the levels' exact-key lookup tables): off = EMPTY on a miss.
// Any level's snapshot resumes the window exactly; the deepest usable one leaves the least work.
// Probe order: a lookup starts at the shallowest level with k >= P.rc_kstart (the first sampled
// level; a k no level has = the deepest level) and goes deeper while the levels hit with an open snapshot: a key
// whose snapshot is final has no deeper snapshot (its builds stop at the final parent), and a deeper
// key that is not cached means its extensions are not either (they are counted on the same sampled
// windows; the rare exception -- a key that failed to build while an extension built from the
// shallower snapshot -- only costs that window some work). On a miss the shallower levels are
// probed, deepest first. C3 (vocabulary workload): 1.8 random lines per window instead of 2.9 when
// the deepest level came first (windows settle at 5 chars most often, and 53 M of them finally).
// one level's probe: 0 miss (or not probed), 1 hit with an open snapshot, 2 final, 3 unusable
__device__ __forceinline__ uint32_t rc_probe(const RcTable& T, const uint32_t* c, uint32_t enc, bool ok, uint64_t s,
                                             const SegDesc& S, uint32_t QCAP, uint32_t t, RcHit& h) {
  if (!(T.k <= enc && (ok || s + T.k <= S.avail))) return 0u;
  const uint4 want = rc_exact_key(c, T.k);
  uint32_t slot = rc_key_hash(want) & T.ct_mask;
  uint4 val = make_uint4(0u, 0u, 0u, 0u);
  bool hit = false;
  for (uint32_t p = 0; p < RC_PROBES; ++p, slot = (slot + 1) & T.ct_mask) {  // collisions probe on (rare)
    const uint4* e = T.ct + 2 * (size_t)slot;
    const uint4 k2 = e[0];
    val = e[1];
    if (!(val.w & RC_OCC)) break;
    if (k2.x == want.x && k2.y == want.y && k2.z == want.z && k2.w == want.w) {
      hit = true;
      break;
    }
  }
  if (!hit) return 0u;
  const uint32_t nq = val.z & 0xFFFFu;
  if (nq + 1u > QCAP) return 3u;
  h = RcHit{val.x, val.y, val.y + nq, ((val.w >> 22) & 0x1FFu) | (val.z & 0xFFFF0000u), val.w & RC_POPS_MASK, t};
  return nq ? 1u : 2u;
}
__device__ __forceinline__ RcHit rc_lookup(const SearchParams& P, const SegDesc& S, uint64_t s, uint32_t QCAP) {
  uint32_t kmax = 0;
  for (uint32_t t = 0; t < P.rc_ntab; ++t) kmax = max(kmax, P.rc_tab[t].k);
  uint32_t c[8];
  const bool ok = rc_chars(P, S, s, kmax, c);  // not cacheable past the halo at the deepest level:
  uint32_t enc = 8;                             // probe the levels whose keys stay inside it
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i)  // keys hold 16-bit units: a longer key would contain char i
    if (enc == 8 && c[i] != RC_PAD && c[i] >= 0xFFFFu) enc = i;
  // (every loop is unrolled over the level index, and the probe is a force-inlined function: a
  // dynamic index into the kernel argument's table array, or a lambda capturing the chars, made the
  // cache builds keep them in scratch, 76 -> 972 B per lane)
  const uint32_t n = P.rc_ntab;
  uint32_t st = 0;  // rc_tab is deepest first: the last level with k >= rc_kstart
#pragma unroll
  for (uint32_t t = 0; t < (uint32_t)kRcLevels; ++t)
    if (t < n && P.rc_tab[t].k >= P.rc_kstart) st = t;
  RcHit r{EMPTY, 0u, 0u, 0u, 0u};
  bool found = false, up = true;
#pragma unroll
  for (int t = kRcLevels - 1; t >= 0; --t) {  // st, then deeper while open
    if (!up || (uint32_t)t > st || (uint32_t)t >= n) continue;
    RcHit h{EMPTY, 0u, 0u, 0u, 0u};
    const uint32_t res = rc_probe(P.rc_tab[t], c, enc, ok, s, S, QCAP, (uint32_t)t, h);
    if (res == 1u || res == 2u) {
      r = h;
      found = true;
    }
    up = res == 1u;
  }
#pragma unroll
  for (uint32_t t = 0; t < (uint32_t)kRcLevels; ++t) {  // shallower levels, deepest first
    if (found || t <= st || t >= n) continue;
    RcHit h{EMPTY, 0u, 0u, 0u, 0u};
    const uint32_t res = rc_probe(P.rc_tab[t], c, enc, ok, s, S, QCAP, t, h);
    if (res == 1u || res == 2u) {
      r = h;
      found = true;
    }
  }
  return r;
}
// rc_lookup in two halves for rc_lookup_kernel: the start level and the deeper ones while open
// (found: a usable hit), then -- for the windows that found none -- the shallower levels. The
// kernel defers the second half of a wave's missing windows into full waves of them.
struct RcKey {
  uint32_t c[8];
  uint32_t enc;
  bool ok;
};
__device__ __forceinline__ uint32_t rc_start_level(const SearchParams& P) {
  uint32_t st = 0;  // rc_tab is deepest first: the last level with k >= rc_kstart
#pragma unroll
  for (uint32_t t = 0; t < (uint32_t)kRcLevels; ++t)
    if (t < P.rc_ntab && P.rc_tab[t].k >= P.rc_kstart) st = t;
  return st;
}
__device__ __forceinline__ void rc_key_of(const SearchParams& P, const SegDesc& S, uint64_t s, RcKey& K) {
  uint32_t kmax = 0;
  for (uint32_t t = 0; t < P.rc_ntab; ++t) kmax = max(kmax, P.rc_tab[t].k);
  K.ok = rc_chars(P, S, s, kmax, K.c);
  K.enc = 8;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i)
    if (K.enc == 8 && K.c[i] != RC_PAD && K.c[i] >= 0xFFFFu) K.enc = i;
}
__device__ __forceinline__ RcHit rc_lookup_deep(const SearchParams& P, const SegDesc& S, uint64_t s, uint32_t QCAP,
                                                const RcKey& K, uint32_t st, bool& found) {
  RcHit r{EMPTY, 0u, 0u, 0u, 0u};
  found = false;
  bool up = true;
#pragma unroll
  for (int t = kRcLevels - 1; t >= 0; --t) {  // st, then deeper while open
    if (!up || (uint32_t)t > st || (uint32_t)t >= P.rc_ntab) continue;
    RcHit h{EMPTY, 0u, 0u, 0u, 0u};
    const uint32_t res = rc_probe(P.rc_tab[t], K.c, K.enc, K.ok, s, S, QCAP, (uint32_t)t, h);
    if (res == 1u || res == 2u) {
      r = h;
      found = true;
    }
    up = res == 1u;
  }
  return r;
}
__device__ __forceinline__ RcHit rc_lookup_shallow(const SearchParams& P, const SegDesc& S, uint64_t s, uint32_t QCAP,
                                                   const RcKey& K, uint32_t st) {
  RcHit r{EMPTY, 0u, 0u, 0u, 0u};
  bool found = false;
#pragma unroll
  for (uint32_t t = 0; t < (uint32_t)kRcLevels; ++t) {  // shallower levels, deepest first
    if (found || t <= st || t >= P.rc_ntab) continue;
    RcHit h{EMPTY, 0u, 0u, 0u, 0u};
    const uint32_t res = rc_probe(P.rc_tab[t], K.c, K.enc, K.ok, s, S, QCAP, t, h);
    if (res == 1u || res == 2u) {
      r = h;
      found = true;
    }
  }
  return r;
}

// The cache builds' parent lookups, one thread per key ahead of the build (rc_bhits / rc_bpops): in
// the build kernel itself the lookup's registers and arrays raised the window loop's pressure (spills
// and a 972-byte scratch frame per lane).
__global__ __launch_bounds__(256) void rc_parent_kernel(SearchParams P, uint32_t qcap) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < P.total_windows;
       v += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t wid = P.win_list[v];
    const uint32_t kl = find_seg(P, wid);
    const SegDesc S = P.segs[kl];
    const uint64_t start = S.w_begin + (wid - P.seg_prefix[kl]);
    const RcHit hit = rc_lookup(P, S, start, qcap);
    P.rc_bhits[v] = make_uint4(hit.off, hit.head, hit.tail, hit.nv_nel);
    P.rc_bpops[v] = hit.pops;
  }
}

// Lookup table of a built level: every entry with a snapshot is inserted under its exact key (the
// chars from the snapshot header); keys holding a char >= 0xFFFF stay out (such windows resume
// from a shorter key).
__global__ __launch_bounds__(256) void rc_publish_kernel(SearchParams P, const uint64_t* reps, const uint4* pool,
                                                         const uint32_t* off, const uint32_t* count, uint32_t n_ent,
                                                         uint32_t k, uint4* ct, uint32_t mask) {
  for (uint32_t ent = blockIdx.x * blockDim.x + threadIdx.x; ent < n_ent; ent += gridDim.x * blockDim.x) {
    if (count[ent] == EMPTY) continue;
    const uint32_t o = off[ent];
    const uint4 h0 = pool[o], h1 = pool[o + 1];
    // the key: the first k chars of the representative window (the build's own window)
    const uint64_t wid = reps[ent];
    const uint32_t kl = find_seg(P, wid);
    const SegDesc S = P.segs[kl];
    uint32_t c[8];
    if (!rc_chars(P, S, S.w_begin + (wid - P.seg_prefix[kl]), k, c)) continue;
    bool enc = true;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) enc = enc && (i >= k || c[i] == RC_PAD || c[i] < 0xFFFFu);
    if (!enc) continue;
    const uint4 key = rc_exact_key(c, k);
    const uint32_t nq = h0.y - h0.x;  // {head, tail, nv, pops}, {ne}
    const uint4 val = make_uint4(o, h0.x, nq | (h1.x << 16), RC_OCC | (h0.z << 22) | min(h0.w, RC_POPS_MASK));
    uint32_t slot = rc_key_hash(key) & mask;
    for (uint32_t p = 0; p < RC_PROBES; ++p, slot = (slot + 1) & mask) {
      uint4* e = ct + 2 * (size_t)slot;
      if (atomicCAS(&e[1].w, 0u, val.w) == 0u) {  // read only by later launches
        e[0] = key;
        e[1].x = val.x;
        e[1].y = val.y;
        e[1].z = val.z;
        break;
      }
    }
  }
}

// Dense start-level bitmaps (P.rc_dense). Most windows' start-level snapshot is final without
// records (C2: 732 M of 1.07 G windows), and the lookup learns that from a random line of a lookup
// table of up to 256 MB. Over an alphabet of the A most frequent ASCII characters of such keys
// (A^k <= 2^24), a key of ranked characters has a dense index, and two bitmaps of at most 2 MB each
// (L2-resident) answer the common cases: bit F -- the key's snapshot is final with no records, so the
// window is done (a final snapshot is a property of the key: no window starting with it reads past
// it, and it holds no match); bit C -- the key has a snapshot at this level at all (clear: the probe
// would miss, so the window goes straight to the shallower levels). F is exact; C is a hint (a set
// bit whose key is not in the table only costs the probe). Keys with an unranked character, and
// windows too close to the text end or the halo (their chars read as RC_PAD), take the probes.
// A third bitmap, F4, holds bit F for level 1's shorter keys (k1 chars, the same ranks): a window
// whose k1-char key is final without records is done too (C2: the 178 M windows whose 5-char key
// is absent because its 4-char parent is final). The window list (dl_*_kernel) tests both.
// Words: [0, 32) rank bytes (0xFF: unranked), [32] A (0: off), [33] k, [34, 36) the sampled count
// (u64), [36] / [37] the level's final record-less ASCII keys / cached keys, [38] k1 (0: no F4),
// [64, 192) the histogram, [RC_DENSE_F, +2^19) bits F, [RC_DENSE_C, +2^19) bits C,
// [RC_DENSE_F4, +2^19) bits F4.
constexpr uint32_t RC_DENSE_LOG2 = 24, RC_DENSE_F = 256, RC_DENSE_C = RC_DENSE_F + (1u << (RC_DENSE_LOG2 - 5));
constexpr uint32_t RC_DENSE_F4 = RC_DENSE_C + (1u << (RC_DENSE_LOG2 - 5));
constexpr size_t RC_DENSE_WORDS = RC_DENSE_F4 + (1u << (RC_DENSE_LOG2 - 5));
__device__ __forceinline__ bool rc_dense_entry(const SearchParams& P, const uint64_t* reps, const uint4* pool,
                                               const uint32_t* off, const uint32_t* count, uint32_t ent, uint32_t k,
                                               uint32_t c[8], bool& fin_empty) {
  if (count[ent] == EMPTY) return false;
  const uint32_t o = off[ent];
  const uint4 h0 = pool[o], h1 = pool[o + 1];
  fin_empty = h0.y == h0.x && h1.x == 0u;  // rc_publish_kernel: nq = 0, ne = 0
  const uint64_t wid = reps[ent];
  const uint32_t kl = find_seg(P, wid);
  const SegDesc S = P.segs[kl];
  if (!rc_chars(P, S, S.w_begin + (wid - P.seg_prefix[kl]), k, c)) return false;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i)
    if (i < k && c[i] >= 128u) return false;  // RC_PAD included
  return true;
}
// character histogram of the level's final record-less keys (ASCII keys only)
__global__ __launch_bounds__(256) void rc_dense_hist_kernel(SearchParams P, const uint64_t* reps, const uint4* pool,
                                                            const uint32_t* off, const uint32_t* count, uint32_t n_ent,
                                                            uint32_t k, uint32_t* dense) {
  __shared__ uint32_t h[128];
  if (threadIdx.x < 128) h[threadIdx.x] = 0;
  __syncthreads();
  uint32_t n_fe = 0, n_cached = 0;
  for (uint32_t ent = blockIdx.x * blockDim.x + threadIdx.x; ent < n_ent; ent += gridDim.x * blockDim.x) {
    uint32_t c[8];
    bool fe = false;
    n_cached += count[ent] != EMPTY ? 1u : 0u;
    if (!rc_dense_entry(P, reps, pool, off, count, ent, k, c, fe) || !fe) continue;
    ++n_fe;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i)
      if (i < k) atomicAdd(&h[c[i]], 1u);  // LDS
  }
  __syncthreads();
  if (threadIdx.x < 128 && h[threadIdx.x]) atomicAdd(&dense[64 + threadIdx.x], h[threadIdx.x]);
  if (n_fe) atomicAdd(&dense[36], n_fe);
  if (n_cached) atomicAdd(&dense[37], n_cached);
}
// ranks by descending count (ties: lower character first), A = the most with A^k <= 2^24; one block
// of 128 threads, one character each
// (A = 0 -- no bitmaps -- when fewer than min_pm per mille of the cached keys are ASCII and final
// without records: C3 finishes 1.5 % of its windows through them, not worth the lookups' test)
__global__ __launch_bounds__(128) void rc_dense_rank_kernel(uint32_t k, uint32_t k1, uint32_t min_pm, uint32_t* dense) {
  __shared__ uint32_t h[128];
  const uint32_t ch = threadIdx.x;
  h[ch] = dense[64 + ch];
  __syncthreads();
  const uint32_t v = h[ch];
  uint32_t r = 0, used = 0;
  for (uint32_t o = 0; o < 128; ++o) {
    const uint32_t w = h[o];
    r += (w > v || (w == v && o < ch)) ? 1u : 0u;
    used += w ? 1u : 0u;
  }
  uint32_t A = 0;
  for (;;) {
    uint64_t p = 1;
    for (uint32_t i = 0; i < k && p <= (1ull << RC_DENSE_LOG2); ++i) p *= (uint64_t)(A + 1);
    if (A + 1 > used || p > (1ull << RC_DENSE_LOG2)) break;
    ++A;
  }
  if (A < 2 || (uint64_t)dense[36] * 1000u < (uint64_t)dense[37] * min_pm) A = 0;
  reinterpret_cast<uint8_t*>(dense)[ch] = (v && r < A) ? (uint8_t)r : (uint8_t)0xFF;
  if (ch == 0) {
    dense[32] = A;
    dense[33] = k;
    dense[38] = k1 < k ? k1 : 0u;
  }
}
// dense index of a key: its ranks as base-A digits, first character most significant (Horner), so
// the next window's index slides: (idx - r0 * A^(k-1)) * A + r_k (dl_tile)
__device__ __forceinline__ bool rc_dense_index(const uint8_t* rank, uint32_t A, uint32_t k, const uint32_t c[8],
                                               uint32_t& idx) {
  idx = 0;
  bool ok = true;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) {
    if (i >= k) continue;
    const uint32_t r = c[i] < 128u ? (uint32_t)rank[c[i]] : 0xFFu;
    ok = ok && r < A;
    idx = __umul24(idx, A) + (r < A ? r : 0u);
  }
  return ok;
}
// bits F (at f_off) and C (at c_off, 0: none) of a level's entries
__global__ __launch_bounds__(256) void rc_dense_fill_kernel(SearchParams P, const uint64_t* reps, const uint4* pool,
                                                            const uint32_t* off, const uint32_t* count, uint32_t n_ent,
                                                            uint32_t k, uint32_t* dense, uint32_t f_off, uint32_t c_off) {
  __shared__ uint8_t s_rank[128];
  if (threadIdx.x < 128) s_rank[threadIdx.x] = reinterpret_cast<const uint8_t*>(dense)[threadIdx.x];
  __syncthreads();
  const uint32_t A = dense[32];
  if (A == 0) return;
  for (uint32_t ent = blockIdx.x * blockDim.x + threadIdx.x; ent < n_ent; ent += gridDim.x * blockDim.x) {
    uint32_t c[8], idx = 0;
    bool fe = false;
    if (!rc_dense_entry(P, reps, pool, off, count, ent, k, c, fe) || !rc_dense_index(s_rank, A, k, c, idx)) continue;
    if (c_off) atomicOr(&dense[c_off + (idx >> 5)], 1u << (idx & 31u));
    if (fe) atomicOr(&dense[f_off + (idx >> 5)], 1u << (idx & 31u));
  }
}

// Prefix-cache keys: every `stride`-th window's key is inserted and counted (level 1: every window,
// sampled levels: a sample); the first inserter of a key is its representative. Counts saturate
// at `sat` (only "at least thr" is asked), so a frequent key is not one hot atomic per window.
// A key that finds no slot within `probes` stays uncounted (not cached).
// One level's count table (rc_count_kernel): keys of k chars, open addressing with `probes` slots
// A slot is one 64-bit word: the key hash with its low 4 bits replaced by the key's count (saturating
// at `sat` <= RC_CSAT), so an insert of a known key touches one line (rounds <= 3 kept the counts in
// an array of their own: a second random line per insert, C3 69 GB of count traffic per step). The
// representative (`rep`, by slot) is written by the sighting that brings the count to min(sat, 2):
// any window holding the key is a valid one, and keys seen once (most long keys) are never selected
// when sat >= 2, so they cost one line.
constexpr uint32_t RC_CSAT = 15;
__device__ __forceinline__ uint32_t rc_slot_count(unsigned long long w) { return (uint32_t)(w & 0xFull); }
struct RcCountTarget {
  unsigned long long* keys;
  uint64_t* rep;
  uint32_t mask;
  uint32_t k;  // 0: no table
};
__device__ __forceinline__ void rc_count_insert(const RcCountTarget& T, uint64_t k, uint64_t vid, uint32_t sat,
                                                uint32_t probes) {
  const uint32_t h = rc_hash(k);
  const unsigned long long tag = (k & ~0xFull) ? (k & ~0xFull) : 0x10ull;
  for (uint32_t p = 0; p < probes; ++p) {
    const uint32_t slot = (h + p) & T.mask;
    unsigned long long w = T.keys[slot];
    if (w == 0ull) {
      w = atomicCAS(&T.keys[slot], 0ull, tag | 1ull);
      if (w == 0ull) {
        if (sat <= 1u) T.rep[slot] = vid;
        return;
      }
    }
    if ((w & ~0xFull) == tag) {  // counted up to sat (a failed exchange means another sighting landed)
      while (rc_slot_count(w) < sat) {
        const unsigned long long old = atomicCAS(&T.keys[slot], w, w + 1ull);
        if (old == w) {
          if (rc_slot_count(w) == 1u) T.rep[slot] = vid;
          break;
        }
        w = old;
      }
      return;
    }
  }
}
// Up to three levels are counted in one pass over the windows (level 1; the sampled levels): their
// inserts go out together and the window's text is read once.
// The key part's start windows, listed in ascending order (kp_mask_kernel: one mask per 64 windows
// and a count per block of KP_CHUNK; dl_scan_kernel; dl_write_kernel writes each block's windows at
// its offset in window order). The count, lookup and cache-off searches then walk the part's windows
// only; the ownership test stays out of the window loops, whose registers it would crowd.
constexpr uint32_t KP_CHUNK = 4096;
__device__ __forceinline__ bool kp_owned_window(const SearchParams& P, uint64_t v) {
  unsigned err = 0;
  const uint32_t kl = find_seg(P, v);
  const SegDesc S = P.segs[kl];
  return window_owned_kp(P, S, S.w_begin + (v - P.seg_prefix[kl]), err);
}

// The windows the dense bitmaps leave open (bit F clear), listed in ascending order ahead of the
// main lookups, which then walk the list as they walk a key part's (P.kp_wlist; the source is the
// key part's list or every window): C2 lists 0.34 G of its 1.07 G windows. Per block of KP_CHUNK
// source windows one 64-bit mask per wave round (window b0 + 64 m + lane), the block's count, then a
// one-block scan and the writes.
// F-done test of one window (the lookup's dense check: chars past the text or the halo are RC_PAD,
// unranked)
__device__ __forceinline__ bool dl_window_done(const SearchParams& P, const uint8_t* rank, uint32_t A, uint32_t k, uint64_t v) {
  const uint32_t kl = find_seg(P, v);
  const SegDesc S = P.segs[kl];
  uint32_t c[8], idx = 0;
  (void)rc_chars(P, S, S.w_begin + (v - P.seg_prefix[kl]), k, c);
  if (rc_dense_index(rank, A, k, c, idx) && ((P.rc_dense[RC_DENSE_F + (idx >> 5)] >> (idx & 31u)) & 1u)) return true;
  const uint32_t k1 = P.rc_dense[38];
  return k1 && rc_dense_index(rank, A, k1, c, idx) && ((P.rc_dense[RC_DENSE_F4 + (idx >> 5)] >> (idx & 31u)) & 1u);
}
// a thread's 16 consecutive windows of a staged tile (ranks s_r, 0xFF unranked): bit w of the result
// set when window b0 + 16 t + w exists and the bitmaps do not finish it
template <uint32_t K>
__device__ __forceinline__ uint32_t dl_tile(const SearchParams& P, const uint8_t* s_r, uint32_t A, uint64_t b0, uint64_t last) {
  uint32_t rw[6];
#pragma unroll
  for (uint32_t x = 0; x < 6; ++x) rw[x] = reinterpret_cast<const uint32_t*>(s_r)[threadIdx.x * 4u + x];
  uint32_t r[16 + K - 1], bad = 0;
#pragma unroll
  for (uint32_t p = 0; p < 16 + K - 1; ++p) {
    const uint32_t v = (rw[p >> 2] >> ((p & 3u) * 8u)) & 0xFFu;
    bad |= v < A ? 0u : 1u << p;
    r[p] = v < A ? v : 0u;
  }
  uint32_t top = 1;  // A^(K-1)
#pragma unroll
  for (uint32_t i = 1; i < K; ++i) top = __umul24(top, A);
  uint32_t idx[16];
  uint32_t x = 0;
#pragma unroll
  for (uint32_t i = 0; i < K; ++i) x = __umul24(x, A) + r[i];
  idx[0] = x;
#pragma unroll
  for (uint32_t w = 1; w < 16; ++w) {
    x = __umul24(x - __umul24(r[w - 1], top), A) + r[w + K - 1];
    idx[w] = x;
  }
  const uint64_t q0 = b0 + threadIdx.x * 16ull;
  uint32_t okm = 0;
#pragma unroll
  for (uint32_t w = 0; w < 16; ++w) okm |= (((bad >> w) & ((1u << K) - 1u)) == 0u && q0 + w <= last) ? 1u << w : 0u;
  uint32_t bw[16];
#pragma unroll
  for (uint32_t w = 0; w < 16; ++w) bw[w] = ((okm >> w) & 1u) ? P.rc_dense[RC_DENSE_F + (idx[w] >> 5)] : 0u;
  uint32_t done = 0;
#pragma unroll
  for (uint32_t w = 0; w < 16; ++w) done |= (((okm >> w) & 1u) && ((bw[w] >> (idx[w] & 31u)) & 1u)) ? 1u << w : 0u;
  const uint32_t k1 = P.rc_dense[38];
  if (k1) {  // the k1-char prefix: the high digits of idx, idx / A^(K - k1)
    uint32_t D = 1;
    for (uint32_t i = k1; i < K; ++i) D = __umul24(D, A);
    const float inv = 1.0f / (float)D;
    const uint32_t m1 = (1u << k1) - 1u;
    uint32_t i4[16], ok4 = 0;
#pragma unroll
    for (uint32_t w = 0; w < 16; ++w) {
      uint32_t q = (uint32_t)((float)idx[w] * inv);  // exact below 2^24 up to one step
      if (__umul24(q, D) > idx[w]) --q;
      else if (__umul24(q + 1u, D) <= idx[w]) ++q;
      i4[w] = q;
      ok4 |= (!((done >> w) & 1u) && ((bad >> w) & m1) == 0u && q0 + w <= last) ? 1u << w : 0u;
    }
#pragma unroll
    for (uint32_t w = 0; w < 16; ++w) bw[w] = ((ok4 >> w) & 1u) ? P.rc_dense[RC_DENSE_F4 + (i4[w] >> 5)] : 0u;
#pragma unroll
    for (uint32_t w = 0; w < 16; ++w) done |= (((ok4 >> w) & 1u) && ((bw[w] >> (i4[w] & 31u)) & 1u)) ? 1u << w : 0u;
  }
  uint32_t pat = 0;
#pragma unroll
  for (uint32_t w = 0; w < 16; ++w) pat |= (q0 + w <= last && !((done >> w) & 1u)) ? 1u << w : 0u;
  return pat;
}
__global__ __launch_bounds__(256) void dl_mask_kernel(SearchParams P, unsigned long long* masks, uint32_t* bcount) {
  __shared__ uint8_t s_rank[128];
  __shared__ __attribute__((aligned(16))) uint8_t s_r[KP_CHUNK + 32];  // the tile's character ranks
  __shared__ uint32_t s_pat[256];
  __shared__ uint32_t s_n;
  if (threadIdx.x < 128) s_rank[threadIdx.x] = reinterpret_cast<const uint8_t*>(P.rc_dense)[threadIdx.x];
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const uint32_t A = P.rc_dense[32], k = P.rc_dense[33];
  const uint64_t b0 = (uint64_t)blockIdx.x * KP_CHUNK;
  const uint64_t last = min(b0 + KP_CHUNK, P.total_windows) - 1;
  const uint32_t kl = find_seg(P, b0);
  uint32_t n = 0;
  if (!P.kp_wlist && find_seg(P, last) == kl) {
    // one segment: stage the ranks of the tile's chars (coalesced), then 16 consecutive windows a
    // thread, their bitmap words loaded together
    const SegDesc S = P.segs[kl];
    const uint64_t s0 = S.w_begin + (b0 - P.seg_prefix[kl]);
    constexpr uint32_t kLoads = (KP_CHUNK + 32 + 255) / 256;
    uint32_t cs[kLoads];
    const uint64_t jmax = min(S.n, S.avail);
    if (S.ascii) {  // every load issued before the first is used
#pragma unroll
      for (uint32_t u = 0; u < kLoads; ++u) {
        const uint64_t j = s0 + threadIdx.x + u * 256u;
        cs[u] = j < jmax ? (uint32_t)P.utf8[S.text_base + j] : RC_PAD;
      }
#pragma unroll
      for (uint32_t u = 0; u < kLoads; ++u)
        if (P.case_insensitive && cs[u] - 'A' < 26u) cs[u] += 32u;
    } else {
#pragma unroll
      for (uint32_t u = 0; u < kLoads; ++u) {
        const uint64_t j = s0 + threadIdx.x + u * 256u;
        cs[u] = j < jmax ? P.text32[S.text_base + j] : RC_PAD;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kLoads; ++u) {
      const uint32_t q = threadIdx.x + u * 256u;
      if (q < KP_CHUNK + 32) s_r[q] = cs[u] < 128u ? s_rank[cs[u]] : (uint8_t)0xFF;
    }
    __syncthreads();
    uint32_t pat = 0;
    switch (k) {
      case 2: pat = dl_tile<2>(P, s_r, A, b0, last); break;
      case 3: pat = dl_tile<3>(P, s_r, A, b0, last); break;
      case 4: pat = dl_tile<4>(P, s_r, A, b0, last); break;
      case 5: pat = dl_tile<5>(P, s_r, A, b0, last); break;
      case 6: pat = dl_tile<6>(P, s_r, A, b0, last); break;
      case 7: pat = dl_tile<7>(P, s_r, A, b0, last); break;
      default: pat = dl_tile<8>(P, s_r, A, b0, last); break;
    }
    s_pat[threadIdx.x] = pat;
    __syncthreads();
    if (threadIdx.x < 64) {  // mask m: windows 64 m .. 64 m + 63 = threads 4 m .. 4 m + 3
      const uint32_t m = threadIdx.x;
      const unsigned long long mk = (unsigned long long)s_pat[4 * m] | ((unsigned long long)s_pat[4 * m + 1] << 16) |
                                    ((unsigned long long)s_pat[4 * m + 2] << 32) | ((unsigned long long)s_pat[4 * m + 3] << 48);
      masks[(uint64_t)blockIdx.x * (KP_CHUNK / 64) + m] = mk;
      n = (uint32_t)__popcll(mk);
    }
  } else {
    for (uint32_t r = 0; r < KP_CHUNK; r += 256) {
      const uint64_t i = b0 + r + threadIdx.x;
      const bool keep = i <= last && !dl_window_done(P, s_rank, A, k, P.kp_wlist ? P.kp_wlist[i] : i);
      const unsigned long long m = __ballot(keep);
      if (lane_id() == 0) {
        masks[(uint64_t)blockIdx.x * (KP_CHUNK / 64) + (r + threadIdx.x) / 64] = m;
        n += (uint32_t)__popcll(m);
      }
    }
  }
  if (n) atomicAdd(&s_n, n);  // LDS
  __syncthreads();
  if (threadIdx.x == 0) bcount[blockIdx.x] = s_n;
}
// the share of F-done windows, from 16384 spread over the windows (dense[34..35], u64): the lookups
// take the list only when it leaves enough out
__global__ __launch_bounds__(256) void rc_dense_sample_kernel(SearchParams P, uint64_t windows) {
  __shared__ uint8_t s_rank[128];
  if (threadIdx.x < 128) s_rank[threadIdx.x] = reinterpret_cast<const uint8_t*>(P.rc_dense)[threadIdx.x];
  __syncthreads();
  const uint32_t A = P.rc_dense[32], k = P.rc_dense[33];
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, ns = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i = g * windows / ns;
  const bool done = A && i < windows && dl_window_done(P, s_rank, A, k, P.kp_wlist ? P.kp_wlist[i] : i);
  const unsigned long long m = __ballot(done);
  if (lane_id() == 0 && m)
    atomicAdd(reinterpret_cast<unsigned long long*>(const_cast<uint32_t*>(P.rc_dense) + 34), (unsigned long long)__popcll(m));
}
__global__ __launch_bounds__(1024) void dl_scan_kernel(const uint32_t* bcount, uint64_t* boff, uint64_t nb,
                                                       unsigned long long* total) {
  __shared__ unsigned long long wsum[16];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  const uint64_t per = ((nb + 1023) / 1024 + 7) & ~7ull;  // 8-entry runs: 16-byte aligned loads
  const uint64_t a = min(nb, (uint64_t)t * per), b = min(nb, a + per);
  unsigned long long sum = 0;
  uint64_t i = a;
  for (; i + 8 <= b; i += 8) {
    const uint4 u0 = *reinterpret_cast<const uint4*>(bcount + i), u1 = *reinterpret_cast<const uint4*>(bcount + i + 4);
    sum += (unsigned long long)u0.x + u0.y + u0.z + u0.w + u1.x + u1.y + u1.z + u1.w;
  }
  for (; i < b; ++i) sum += bcount[i];
  unsigned long long x = sum;
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
    boff[i] = run;
    run += bcount[i];
  }
}
__global__ __launch_bounds__(256) void dl_write_kernel(SearchParams P, const unsigned long long* masks, const uint64_t* boff,
                                                       uint64_t* list) {
  __shared__ uint32_t s_pre[KP_CHUNK / 64];
  const unsigned long long* bm = masks + (uint64_t)blockIdx.x * (KP_CHUNK / 64);
  if (threadIdx.x < 64) {  // exclusive scan of the 64 masks' counts (one wave)
    const uint32_t c = (uint32_t)__popcll(bm[threadIdx.x]);
    uint32_t x = c;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (threadIdx.x >= (uint32_t)o) x += y;
    }
    s_pre[threadIdx.x] = x - c;
  }
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * KP_CHUNK, at = boff[blockIdx.x];
  const uint32_t lane = lane_id();
  for (uint32_t m = threadIdx.x / 64; m < KP_CHUNK / 64; m += 4) {
    const unsigned long long mk = bm[m];
    if (!((mk >> lane) & 1ull)) continue;
    const uint64_t i = b0 + 64ull * m + lane;
    list[at + s_pre[m] + prefix_below(mk)] = P.kp_wlist ? P.kp_wlist[i] : i;
  }
}

// The key part's windows as dl_mask_kernel's masks (then dl_scan_kernel / dl_write_kernel list them):
// one segment per block -- the tile's chars staged in LDS with coalesced loads, each wave testing 64
// consecutive windows per round (their two chars: consecutive LDS words); else window by window.
__global__ __launch_bounds__(256) void kp_mask_kernel(SearchParams P, unsigned long long* masks, uint32_t* bcount) {
  __shared__ uint32_t s_c[KP_CHUNK + 1];
  __shared__ uint32_t s_n;
  if (threadIdx.x == 0) s_n = 0;
  const uint64_t b0 = (uint64_t)blockIdx.x * KP_CHUNK;
  const uint64_t last = min(b0 + KP_CHUNK, P.total_windows) - 1;
  const uint32_t kl = find_seg(P, b0);
  const bool tile = find_seg(P, last) == kl;
  if (tile) {
    const SegDesc S = P.segs[kl];
    const uint64_t s0 = S.w_begin + (b0 - P.seg_prefix[kl]);
    constexpr uint32_t kLoads = (KP_CHUNK + 1 + 255) / 256;
    uint32_t cs[kLoads];
#pragma unroll
    for (uint32_t u = 0; u < kLoads; ++u) {  // window_owned_kp's chars: past the halo 0, past the text ~0
      const uint64_t j = s0 + threadIdx.x + u * 256u;
      uint32_t c = 0xFFFFFFFFu;
      if (j < S.n) c = j >= S.avail ? 0u : S.ascii ? (uint32_t)P.utf8[S.text_base + j] : P.text32[S.text_base + j];
      cs[u] = c;
    }
#pragma unroll
    for (uint32_t u = 0; u < kLoads; ++u) {
      const uint32_t q = threadIdx.x + u * 256u;
      uint32_t c = cs[u];
      if (S.ascii && P.case_insensitive && c - 'A' < 26u) c += 32u;
      if (q <= KP_CHUNK) s_c[q] = c;
    }
  }
  __syncthreads();
  uint32_t n = 0;
  for (uint32_t r = 0; r < KP_CHUNK; r += 256) {
    const uint32_t q = r + threadIdx.x;
    bool own = b0 + q <= last;
    if (own) own = tile ? kp_owned_chars(P, s_c[q], s_c[q + 1]) : kp_owned_window(P, b0 + q);
    const unsigned long long m = __ballot(own);
    if (lane_id() == 0) {
      masks[(uint64_t)blockIdx.x * (KP_CHUNK / 64) + q / 64] = m;
      n += (uint32_t)__popcll(m);
    }
  }
  if (n) atomicAdd(&s_n, n);  // LDS
  __syncthreads();
  if (threadIdx.x == 0) bcount[blockIdx.x] = s_n;
}

__global__ __launch_bounds__(256) void rc_count_kernel(SearchParams P, RcCountTarget t0, RcCountTarget t1,
                                                       RcCountTarget t2, uint32_t stride, uint32_t sat, uint32_t probes) {
  const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
  unsigned err = 0;
  const uint64_t ns = (P.total_windows + stride - 1) / stride;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gstride) {
    const uint64_t vid = P.kp_wlist ? P.kp_wlist[i * stride] : i * stride;  // a key part: its windows
    const uint32_t kl = find_seg(P, vid);
    const SegDesc S = P.segs[kl];
    const uint64_t start = S.w_begin + (vid - P.seg_prefix[kl]);
    if (window_skipped(P, S, start, err)) continue;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const RcCountTarget& T = t == 0 ? t0 : t == 1 ? t1 : t2;
      if (!T.k) continue;
      RcChars ch;
      uint64_t k;
      if (!rc_key(P, S, start, T.k, ch, k)) continue;
      rc_count_insert(T, k, vid, sat, probes);
    }
  }
}

// Level-0 keys are the level-1 keys' prefixes: inserted from the level-1 representatives (one per
// level-1 key, each the representative of its prefix too) instead of from every window.
__global__ __launch_bounds__(256) void rc_derive_kernel(SearchParams P, const uint64_t* reps, uint32_t n,
                                                        RcCountTarget T, uint32_t probes) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t vid = reps[i];
    const uint32_t kl = find_seg(P, vid);
    const SegDesc S = P.segs[kl];
    const uint64_t start = S.w_begin + (vid - P.seg_prefix[kl]);
    RcChars ch;
    uint64_t k;
    if (rc_key(P, S, start, T.k, ch, k)) rc_count_insert(T, k, vid, 1u, probes);
  }
}

// Entries of a level: the keys counted at least `thr` times, numbered without a contended counter
// (one same-address atomic per selected wave serialises at one L2 channel): per-block counts over
// contiguous slot ranges, an exclusive scan of the block counts, then the assignment. Every other
// slot maps to EMPTY (not cached: the lookup falls through to the next level).
__device__ __forceinline__ bool rc_selected(const unsigned long long* keys, uint32_t s, uint32_t thr) {
  const unsigned long long w = keys[s];
  return w != 0ull && rc_slot_count(w) >= thr;
}
__global__ __launch_bounds__(64) void rc_sel_count_kernel(const unsigned long long* keys, uint32_t n_slots,
                                                           uint32_t range, uint32_t thr, uint32_t* bcount) {
  __shared__ uint32_t tot;
  if (threadIdx.x == 0) tot = 0;
  __syncthreads();
  const uint32_t b0 = blockIdx.x * range, b1 = min(b0 + range, n_slots);
  uint32_t c = 0;
  for (uint32_t s = b0 + threadIdx.x; s < b1; s += blockDim.x) c += rc_selected(keys, s, thr) ? 1u : 0u;
  c = wave_inclusive_sum(c);
  if (lane_id() == 63) atomicAdd(&tot, c);
  __syncthreads();
  if (threadIdx.x == 0) bcount[blockIdx.x] = tot;
}
// one wave: exclusive scan of nb (<= 8192) block counts in place; n_ent = the total. Each lane
// scans 128 consecutive counts. The numbering kernels run while the level-1 build's persistent
// single-wave workgroups hold the CUs on the second stream, and every freed wave slot goes to the
// build's next workgroup first: a 4-wave workgroup queued there 10 ms, a 1-wave one does not.
__global__ __launch_bounds__(64) void rc_sel_scan_kernel(uint32_t* bcount, uint32_t nb, unsigned int* n_ent) {
  const uint32_t base = lane_id() * 128;
  uint32_t tot = 0;
  for (uint32_t i = 0; i < 128; ++i) tot += base + i < nb ? bcount[base + i] : 0u;
  const uint32_t incl = wave_inclusive_sum(tot);
  uint32_t run = incl - tot;
  if (lane_id() == 63) *n_ent = incl;
  for (uint32_t i = 0; i < 128 && base + i < nb; ++i) {
    const uint32_t v = bcount[base + i];
    bcount[base + i] = run;
    run += v;
  }
}
// val[slot] = the slot's entry (EMPTY: not selected); rep[entry] = the slot's representative window
__global__ __launch_bounds__(64) void rc_sel_assign_kernel(const unsigned long long* keys,
                                                            const uint64_t* rep_slot, uint32_t* val, uint64_t* rep,
                                                            const uint32_t* bbase, uint32_t n_slots, uint32_t range,
                                                            uint32_t thr, uint32_t max_ent) {
  __shared__ uint32_t run;
  if (threadIdx.x == 0) run = bbase[blockIdx.x];
  __syncthreads();
  const uint32_t b0 = blockIdx.x * range, b1 = min(b0 + range, n_slots);
  for (uint32_t s0 = b0; s0 < b1; s0 += blockDim.x) {
    const uint32_t s = s0 + threadIdx.x;
    const bool sel = s < b1 && rc_selected(keys, s, thr);
    const uint64_t m = __ballot(sel);
    uint32_t base = 0;
    if (m) {
      if (lane_id() == (uint32_t)first_lane(m)) base = atomicAdd(&run, (uint32_t)__popcll(m));  // LDS
      base = shfl_u32(base, first_lane(m));
    }
    if (s < b1) {
      uint32_t v = EMPTY;
      if (sel) {
        const uint32_t ent = base + prefix_below(m);
        if (ent < max_ent) {
          rep[ent] = rep_slot[s];
          v = ent;
        }
      }
      val[s] = v;
    }
  }
}

// A resumed window whose snapshot has an empty queue is finished: the snapshot's best list is its
// final best map. Each such lane writes its own window's records (one output atomic per wave);
// returns true for them.
__device__ __forceinline__ bool flush_final(const SearchParams& P, bool resumed, const RcHit& hit, uint32_t kl,
                                            uint64_t start, uint64_t vid, uint64_t& cached_lane,
                                            uint32_t& triv_lane) {
  const bool triv = resumed && hit.tail == hit.head && P.rc_lane_flush;
  if (!__ballot(triv)) return false;
  const uint32_t ne = triv ? (hit.nv_nel >> 16) : 0u;
  const uint32_t incl = wave_inclusive_sum(ne), tot = shfl_u32(incl, 63);
  unsigned long long base = 0;
  if (tot) {
    if (lane_id() == 0) base = atomicAdd(P.counters, (unsigned long long)tot);
    base = shfl_u64(base, 0);
  }
  if (triv) {
    const SegDesc S = P.segs[kl];
    const uint64_t sb = S.byte_base + local_byte(P, S, start);
    const uint4* src = P.rc_pool + hit.off + RC_HDR + (hit.nv_nel & 0xFFFFu);  // best list (nq == 0)
    for (uint32_t i = 0; i < ne; ++i) {
      const uint64_t o = base + incl - ne + i;
      if (o < P.out_cap) P.out[o] = match_record(P, S, start, sb, src[i]);
    }
    if (P.win_counts) P.win_counts[vid] = hit.tail;
    cached_lane += hit.pops;
    triv_lane += 1;
  }
  return triv;
}

// Per-window prefix-cache lookups of a main pass (P.rc_mode == 1), ahead of the search kernels:
// windows that are skipped or finished by their snapshot (flushed here) are done; the others' hits
// (or misses) are stored compacted per region of RC_REGION windows (entries rc_hits / rc_hit_pops /
// rc_voff, counts rc_region_cnt), so the searches read only the open windows (C2: 15 % of them).
// A wave takes whole regions from a work counter (counters[10]). Keeps the lookup's registers out of
// the search kernels.
__global__ __launch_bounds__(256) void rc_lookup_kernel(SearchParams P) {
  // per wave: region offsets of windows whose start-level chain found nothing, probed on the
  // shallower levels once 64 of them are queued (or at the region's end) -- a full wave's round trip
  // instead of one for every 64 windows that hold a few such lanes (C2: 17 % of windows, C3: 30 %)
  __shared__ uint16_t s_dq[4][128];
  __shared__ uint8_t s_rank[128];  // the dense bitmaps' character ranks (rc_dense_rank_kernel)
  uint16_t* dq = s_dq[threadIdx.x / 64];
  const uint32_t lane = lane_id();
  uint64_t cached_lane = 0;
  uint32_t res_lane = 0, triv_lane = 0;
  unsigned err = 0;
  const uint64_t n_reg = (P.total_windows + RC_REGION - 1) / RC_REGION;
  const uint32_t st = rc_start_level(P);
  const bool shallower = st + 1 < P.rc_ntab;
  const uint32_t dA = P.rc_dense ? P.rc_dense[32] : 0u, dk = P.rc_dense ? P.rc_dense[33] : 0u;
  if (dA) {
    if (threadIdx.x < 128) s_rank[threadIdx.x] = reinterpret_cast<const uint8_t*>(P.rc_dense)[threadIdx.x];
    __syncthreads();
  }
  for (;;) {
    unsigned long long rg = 0;
    if (lane == 0) rg = atomicAdd(P.counters + 10, 1ull);
    rg = shfl_u64(rg, 0);
    if (rg >= n_reg) break;
    const uint64_t rbase = rg * RC_REGION;
    uint32_t n_open = 0;  // wave-uniform
    uint32_t nq = 0;      // wave-uniform: deferred windows queued
    // a window's outcome: finished here (flush_final) or stored open for the searches
    // off: the window's offset from the region base (its voff), 0xFFFFFFFF for no window
    auto settle = [&](bool active, const RcHit& hit, uint32_t kl, uint64_t start, uint64_t v, uint32_t off) {
      const bool resumed = active && hit.off != EMPTY;
      res_lane += resumed ? 1u : 0u;
      if (P.lane_debug) {  // diagnostics: windows by the level they resume from (x final), misses, skips
        const uint32_t cat = !active ? 13u : !resumed ? 12u : hit.lvl * 2u + (hit.tail == hit.head ? 1u : 0u);
        for (uint32_t c = 0; c < 14; ++c) {
          const uint64_t m = __ballot(cat == c && off != 0xFFFFFFFFu);
          if (m && lane == 0) atomicAdd(&g_lk_dbg[c], (unsigned long long)__popcll(m));
        }
      }
      const bool fin = flush_final(P, resumed, hit, kl, start, v, cached_lane, triv_lane);
      const bool open = active && !fin;
      const uint64_t om = __ballot(open);
      if (open) {
        const uint64_t e = rbase + n_open + prefix_below(om);
        P.rc_hits[e] = make_uint4(hit.off, hit.head, hit.tail, hit.nv_nel);
        P.rc_hit_pops[e] = hit.pops;
        P.rc_voff[e] = off;
      }
      n_open += (uint32_t)__popcll(om);
    };
    auto drain = [&](bool all) {
      while (nq >= 64 || (all && nq > 0)) {
        const uint32_t take = min(nq, 64u);
        __builtin_amdgcn_wave_barrier();
        const bool act = lane < take;
        const uint32_t qo = act ? (uint32_t)dq[nq - take + lane] : 0u;
        __builtin_amdgcn_wave_barrier();
        nq -= take;
        uint32_t kl = 0;
        uint64_t start = 0;
        const uint64_t v = P.kp_wlist ? (act ? P.kp_wlist[rbase + qo] : rbase) : rbase + qo;
        const uint32_t off = act ? (uint32_t)(v - rbase) : 0xFFFFFFFFu;
        RcHit hit{EMPTY, 0u, 0u, 0u, 0u};
        if (act) {
          kl = find_seg(P, v);
          const SegDesc S = P.segs[kl];
          start = S.w_begin + (v - P.seg_prefix[kl]);
          RcKey K;
          rc_key_of(P, S, start, K);
          hit = rc_lookup_shallow(P, S, start, P.rc_qcap, K, st);
        }
        settle(act, hit, kl, start, v, off);
      }
    };
    for (uint32_t it = 0; it < RC_REGION; it += 64) {
      const uint64_t e = rbase + it + lane;  // whole waves iterate together (ballots, DPP scans)
      bool active = e < P.total_windows;
      // the window: the entry itself, or a key part's e-th window (ascending, so v >= e and the
      // stored offset v - rbase maps back through the searches' rc_window_of)
      const uint64_t v = (P.kp_wlist && active) ? P.kp_wlist[e] : e;
      uint32_t kl = 0;
      uint64_t start = 0;
      if (active) {
        kl = find_seg(P, v);
        const SegDesc S = P.segs[kl];
        start = S.w_begin + (v - P.seg_prefix[kl]);
        active = !window_skipped(P, S, start, err);
      }
      RcHit hit{EMPTY, 0u, 0u, 0u, 0u};
      bool found = false, done = false;
      if (active) {
        const SegDesc S = P.segs[kl];
        RcKey K;
        rc_key_of(P, S, start, K);
        uint32_t idx = 0;
        bool absent = false;
        if (dA && rc_dense_index(s_rank, dA, dk, K.c, idx)) {  // the dense bitmaps (rc_dense_fill_kernel)
          const uint32_t wf = P.rc_dense[RC_DENSE_F + (idx >> 5)], wc = P.rc_dense[RC_DENSE_C + (idx >> 5)];
          done = (wf >> (idx & 31u)) & 1u;
          absent = !((wc >> (idx & 31u)) & 1u);
        }
        if (!done && !absent) hit = rc_lookup_deep(P, S, start, P.rc_qcap, K, st, found);
      }
      if (P.lane_debug) {
        const uint64_t m = __ballot(done);
        if (m && lane == 0) atomicAdd(&g_lk_dbg[14], (unsigned long long)__popcll(m));
      }
      if (done) {  // final without records at the start level: nothing to write (flush_final's counts)
        res_lane += 1;
        triv_lane += 1;
        active = false;
      }
      const bool defer = active && !found && shallower;
      const uint64_t dm = __ballot(defer);
      if (defer) dq[nq + prefix_below(dm)] = (uint16_t)(it + lane);
      nq += (uint32_t)__popcll(dm);
      settle(active && !defer, hit, kl, start, v,
             (e < P.total_windows && !defer && !done) ? (uint32_t)(v - rbase) : 0xFFFFFFFFu);
      if (nq >= 64) drain(false);
    }
    drain(true);
    if (lane == 0) P.rc_region_cnt[rg] = n_open;
  }
  wave_add_counter(P.counters + 4, cached_lane);
  wave_add_counter(P.counters + 5, res_lane);
  wave_add_counter(P.counters + 6, triv_lane);
  if (err) atomicOr(reinterpret_cast<unsigned int*>(P.counters + 2), err);
}

// ---- Lane-serial search of small resumed windows ----
// After the prefix-cache lookups most unfinished windows need only a handful of pops, for which
// run_window spends a window prologue and whole 64-lane batches holding a few states. Here every
// lane runs one such window alone, in the reference's sequential order (search.rs:560-1089, the
// oracle's Searcher::run), resumed from its snapshot: the queue ring and the best list live in LDS
// (slot i of lane l at i * 64 + l). There is no dedup table: without a beam, dedup cannot change
// results, and a queue run without dedup is never shorter than the dedup queue at
// the same pop (every state it adds over the dedup run is pushed before it is popped), so a window
// whose dedup-free pending count never exceeds 2·beam never beams. A window that would (or that
// overflows the ring or the best list, reads past the resident halo, or exceeds the pop budget) is
// left to the wave kernel, which restarts it from its snapshot; finished windows write their
// records and are marked RC_DONE.
constexpr uint32_t LANE_RUN = 1u, LANE_OK = 2u, LANE_BAIL = 3u;
constexpr uint32_t LANE_CHUNK = 4096;
__device__ unsigned long long g_lane_dbg[8];  // diagnostics (FAC_RC_DEBUG): taken, finished, bailed, lane runs
// Lane ring entries are 12 bytes in three LDS planes (node, penalty, position word): the position word
// packs j_rel and me_rel (8 bits each) and the four edit counts (4 bits each). A state that does not
// fit sends its window back to the wave kernel.
__device__ __forceinline__ bool lane_pack(uint32_t jm, uint32_t pk, uint32_t& w) {
  const uint32_t jr = jm & 0xFFFFu, mr = jm >> 16;
  w = jr | (mr << 8) | ((pk & 0xFu) << 16) | (((pk >> 8) & 0xFu) << 20) | (((pk >> 16) & 0xFu) << 24) | ((pk >> 24) << 28);
  return jr < 256u && mr < 256u && ((pk & 0xF0F0F0F0u) == 0u);
}
__device__ __forceinline__ void lane_unpack(uint32_t w, uint32_t& jm, uint32_t& pk) {
  jm = (w & 0xFFu) | (((w >> 8) & 0xFFu) << 16);
  pk = ((w >> 16) & 0xFu) | (((w >> 20) & 0xFu) << 8) | (((w >> 24) & 0xFu) << 16) | ((w >> 28) << 24);
}
// Live dedup entries of the snapshot a beamed window resumed from (lv_n entries at pool word lv_off,
// the largest j below jlive): the window runs dedup-free, which cannot change results while no beam
// triggers -- except against the states popped before the snapshot, whose subtrees a beam may have
// pruned there. A popped state equal to such an entry with a stored penalty <= its own is skipped
// exactly as the reference's visited map would (search.rs:618-622); the entries are not updated (a
// later duplicate of a state expanded here only mirrors descendants that are all explored).
struct LiveDedup {
  uint32_t off, n, jlive;
};
__device__ __forceinline__ bool live_dup(const SearchParams& P, const LiveDedup& L, const KState& st) {
  if (L.n == 0 || (st.jm & 0xFFFFu) + 1u > L.jlive) return false;
  bool hit = false;
  for (uint32_t i = 0; i < L.n; i += 4) {  // four entries in flight (the checks are rare: C3 ~0.2 % of pops)
    uint4 e[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) e[u] = i + u < L.n ? P.rc_pool[L.off + i + u] : make_uint4(EMPTY, 0u, 0u, 0u);
    bool done = false;
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
      if (!done && e[u].x == st.node && e[u].y == st.jm && e[u].w == st.packed) {
        hit = __uint_as_float(e[u].z) <= st.pen;
        done = true;
      }
    if (done) break;
  }
  if (P.lane_debug) {
    atomicAdd(&g_live_dbg[0], 1ull);
    if (hit) atomicAdd(&g_live_dbg[1], 1ull);
  }
  return hit;
}

// The body of one lane-serial pop after its dedup decision (search.rs:629-1089): node ceiling,
// emission into the lane's best list, expansion pushed at the tail. LINEAR: the lane's states are
// a linear array (the cache build keeps its popped states for the dedup scans), else a ring.
template <uint32_t QL, uint32_t ELN, bool LINEAR>
__device__ __forceinline__ void lane_expand(const SearchParams& P, uint32_t* s_q, uint4* s_e, const SegDesc& S,
                                            uint64_t start, const KState& st, uint32_t& status, uint32_t& head,
                                            uint32_t& tail, uint32_t& nel, unsigned& err) {
  const uint32_t lane = lane_id();
  const bool fast = P.mef != 255u;
  // the state's reads go out together: node record, char filters, text at j and j + 1
  const DevNode nd = P.nodes[st.node];
  const uint4 aux = P.aux[st.node];
  const uint32_t j_rel = st.jm & 0xFFFFu, me_rel = st.jm >> 16;
  const uint64_t j = start + j_rel;
  uint32_t c0 = 0, c1 = 0;
  if (j < S.n) c0 = text_char(P, S, j, err);
  if (j + 1 < S.n) c1 = text_char(P, S, j + 1, err);
  if (st.pen > __fsub_rn(nd.prune_len, __fmul_rn(nd.prune_lw, P.thr))) return;  // :638-642
  if (err) {
    status = LANE_BAIL;
    return;
  }
  const uint32_t packed = st.packed, edits = edits_of(packed);
  if (node_has_out(nd)) {  // emission (:659-737) into the best list, first-found ties
    const uint2 orr = P.out_range[st.node];
    const uint32_t ins = packed & 0xFFu, del = (packed >> 8) & 0xFFu, sub = (packed >> 16) & 0xFFu, swp = packed >> 24;
    for (uint32_t i = orr.x; i < orr.y && status == LANE_RUN; ++i) {
      const uint32_t p = P.out_pat[i];
      const DevPattern pt = P.pats[p];
      bool ok;
      if (fast) {
        ok = edits <= P.mef;
      } else {  // within_limits (:151-169)
        const Lim m = pick_limits(P, pt.has_limits ? (int32_t)p : -1);
        ok = m.has ? (lim_le(m.l.edits, edits) && lim_le(m.l.ins, ins) && lim_le(m.l.del, del) &&
                      lim_le(m.l.sub, sub) && lim_le(m.l.swp, swp))
                   : (edits == 0);
      }
      if (!ok) continue;
      const float sim = __fmul_rn(__fdiv_rn(__fsub_rn(pt.glen, st.pen), pt.glen), pt.weight);  // :696-699
      if (sim < P.thr) continue;                                                              // :701
      uint32_t at = nel;
      for (uint32_t k = 0; k < nel; ++k) {
        const uint4 e = s_e[k * 64 + lane];
        if (e.x == me_rel && e.y == p) {
          at = k;
          if (sim > __uint_as_float(e.z)) s_e[k * 64 + lane] = make_uint4(me_rel, p, __float_as_uint(sim), packed);
          break;
        }
      }
      if (at == nel) {
        if (nel == ELN) status = LANE_BAIL;
        else s_e[(nel++) * 64 + lane] = make_uint4(me_rel, p, __float_as_uint(sim), packed);
      }
    }
    if (status != LANE_RUN) return;
  }
  const Prep pr = lane_prep(P, S, st, nd, start, c0, c1, nd.sb);
  auto push = [&](uint32_t node, uint32_t jm, float pen, uint32_t pk) {
    uint32_t w;
    if ((LINEAR ? tail >= QL : tail - head >= QL) || !lane_pack(jm, pk, w)) {
      status = LANE_BAIL;
      return false;
    }
    const uint32_t slot = (tail % QL) * 64 + lane;
    s_q[slot] = node;
    s_q[QL * 64 + slot] = __float_as_uint(pen);
    s_q[2 * QL * 64 + slot] = w;
    ++tail;
    return true;
  };
  const uint32_t eb = nd.edge_begin, ee = node_end(nd);
  const uint32_t j1 = j_rel + 1u, jm1 = j1 | (j1 << 16);
  // O(1) expansion (expand_fast: the wave kernel's decisions for a state whose similarity cannot drop
  // a substitution): the substitution / deletion sets come as edge masks, so only their set bits are
  // walked -- at the last edit the dead-end filters leave a few of a node's edges
  if (P.gt_fast && node_deg(nd) <= 64u &&
      (!(pr.flags & PF_SUB) || P.p_sub <= pr.remaining || no_subs(P, nd, pr.cur_ch, pr.remaining))) {
    uint64_t msub = 0, mdel = 0;
    uint32_t ex = 0u, xe = 0u;
    expand_fast(P, st, nd, pr, aux, msub, mdel, ex, xe);
    if (ex) {  // exact (:776-800); the exact edge leaves the substitution set
      msub &= ~(1ull << (63u - (ex >> 26)));
      if (!push(ex & CHILD26_MASK, jm1, st.pen, packed)) return;
    }
    while (msub) {  // substitutions (:803-874), edge order
      const uint32_t e = (uint32_t)__ffsll((unsigned long long)msub) - 1u;
      msub &= msub - 1;
      const DevEdge ed = P.edges[eb + e];
      const float penalty = __fmul_rn(P.p_sub, __fsub_rn(1.0f, similarity(P, ed.ch, pr.cur_ch)));
      if (!push(ed.next & EDGE_NEXT_MASK, jm1, __fadd_rn(st.pen, penalty), packed + 0x10000u)) return;
    }
    if (xe) {  // swap (:935-989): goto(goto(node, text[j+1]), text[j])
      uint64_t g2 = 0;
      bool ok = gt_get(P, GT_VALID | GT_GOTO | ((uint64_t)(xe & CHILD26_MASK) << 21) | pr.cur_ch, true, g2);
      if (ok && !fast) {  // within_limits_swap_ahead with node2's limits (:962-967)
        const Lim m = pick_limits(P, node_limits(P, (uint32_t)(g2 & CHILD26_MASK)));
        ok = m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.swp, packed >> 24)) : false;
      }
      if (ok) {
        const uint32_t j2 = j_rel + 2u;
        if (!push((uint32_t)(g2 & CHILD26_MASK), j2 | (j2 << 16), __fadd_rn(st.pen, P.p_swp), packed + 0x1000000u)) return;
      }
    }
    if ((pr.flags & PF_INS) && !push(st.node, j1 | (me_rel << 16), __fadd_rn(st.pen, P.p_ins), packed + 1u)) return;
    const float npen = __fadd_rn(st.pen, P.p_del);
    while (mdel) {  // deletions (:1035-1089), edge order
      const uint32_t e = (uint32_t)__ffsll((unsigned long long)mdel) - 1u;
      mdel &= mdel - 1;
      if (!push(P.edges[eb + e].next & EDGE_NEXT_MASK, st.jm, npen, packed + 0x100u)) return;
    }
    return;
  }
  // exact and swap successors through the goto table (first edge with the char, structs.rs:512-519);
  // a clear char-filter bit proves the lookup would miss
  int64_t ex = -1, x = -1;
  uint64_t gx = 0, gv = 0;
  const bool want_ex = (pr.flags & PF_EX) && filt_has(aux.z, pr.cur_ch);
  const bool want_x = (pr.flags & PF_SWAP) && filt_has(aux.z, pr.nch);
  if (gt_get(P, GT_VALID | GT_GOTO | ((uint64_t)st.node << 21) | pr.cur_ch, want_ex, gv)) ex = (int64_t)(gv & CHILD26_MASK);
  if (gt_get(P, GT_VALID | GT_GOTO | ((uint64_t)st.node << 21) | pr.nch, want_x, gx)) x = (int64_t)(gx & CHILD26_MASK);
  if (ex >= 0 && !push((uint32_t)ex, jm1, st.pen, packed)) return;  // exact (:776-800)
  // substitutions (:803-874), edge order, the exact edge excluded; none when similarity must be
  // positive and no edge can have it (no_subs)
  if ((pr.flags & PF_SUB) && !(P.p_sub > pr.remaining && no_subs(P, nd, pr.cur_ch, pr.remaining))) {
    bool ok = true;
    for (uint32_t e0 = eb; e0 < ee && ok; e0 += 4) {
      DevEdge ed[4];
      float sim[4];
      bool sbn[4];
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) ed[k] = e0 + k < ee ? P.edges[e0 + k] : DevEdge{0u, 0u};
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) sim[k] = similarity(P, ed[k].ch, pr.cur_ch);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k)
        sbn[k] = (pr.flags & PF_LAST) && (pr.flags & PF_NEXT) && e0 + k < ee && sb_has(P, ed[k].next & EDGE_NEXT_MASK, pr.next_ch);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        if (!ok || e0 + k >= ee) continue;
        const uint32_t child = ed[k].next & EDGE_NEXT_MASK;
        if (ex >= 0 && child == (uint32_t)ex) continue;
        if (sim[k] < P.min_sym) continue;
        const float penalty = __fmul_rn(P.p_sub, __fsub_rn(1.0f, sim[k]));
        if (penalty > pr.remaining) continue;
        if ((pr.flags & PF_LAST) && !(ed[k].next & EDGE_CHILD_OUTPUT) && !sbn[k]) continue;
        ok = push(child, jm1, __fadd_rn(st.pen, penalty), packed + 0x10000u);
      }
    }
    if (!ok) return;
  }
  if (x >= 0) {  // swap (:935-989): goto(goto(node, text[j+1]), text[j])
    int64_t node2 = -1;
    uint64_t g2 = 0;
    const bool want2 = ((gx >> 48) >> (ch_filt_bit(pr.cur_ch) & 15u)) & 1u;  // x's folded char filter
    if (gt_get(P, GT_VALID | GT_GOTO | ((uint64_t)x << 21) | pr.cur_ch, want2, g2)) node2 = (int64_t)(g2 & CHILD26_MASK);
    if (node2 >= 0 && !fast) {  // within_limits_swap_ahead with node2's limits (:962-967)
      const Lim m = pick_limits(P, node_limits(P, (uint32_t)node2));
      if (!(m.has ? (lim_lt(m.l.edits, edits) && lim_lt(m.l.swp, packed >> 24)) : false)) node2 = -1;
    }
    const uint32_t j2 = j_rel + 2u;
    if (node2 >= 0 && !push((uint32_t)node2, j2 | (j2 << 16), __fadd_rn(st.pen, P.p_swp), packed + 0x1000000u)) return;
  }
  if ((pr.flags & PF_INS) && !push(st.node, j1 | (me_rel << 16), __fadd_rn(st.pen, P.p_ins), packed + 1u)) return;  // :994-1029
  if (pr.flags & PF_DEL) {  // deletions (:1035-1089), edge order
    const float npen = __fadd_rn(st.pen, P.p_del);
    bool ok = true;
    for (uint32_t e0 = eb; e0 < ee && ok; e0 += 4) {
      DevEdge ed[4];
      bool sbc[4];
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) ed[k] = e0 + k < ee ? P.edges[e0 + k] : DevEdge{0u, 0u};
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k)
        sbc[k] = (pr.flags & PF_LAST) && (pr.flags & PF_CUR) && e0 + k < ee && sb_has(P, ed[k].next & EDGE_NEXT_MASK, pr.cur_ch);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        if (!ok || e0 + k >= ee) continue;
        if ((pr.flags & PF_LAST) && !(ed[k].next & EDGE_CHILD_OUTPUT) && !sbc[k]) continue;
        ok = push(ed[k].next & EDGE_NEXT_MASK, st.jm, npen, packed + 0x100u);
      }
    }
  }
}

template <uint32_t QL, uint32_t ELN>
__device__ __forceinline__ void lane_step(const SearchParams& P, uint32_t* s_q, uint4* s_e, const SegDesc& S, uint64_t start,
                                          const LiveDedup& lv, uint32_t& status, uint32_t& head, uint32_t& tail,
                                          uint32_t& nel, uint32_t& pops, unsigned& err) {
  const uint32_t lane = lane_id();
  if (head == tail) {
    status = LANE_OK;
    return;
  }
  if ((P.beam && tail - head > 2u * P.beam) || pops >= P.lane_popmax) {  // the beam could trigger (:577)
    status = LANE_BAIL;
    return;
  }
  const uint32_t slot = (head % QL) * 64 + lane;
  uint32_t jm0, pk0;
  lane_unpack(s_q[2 * QL * 64 + slot], jm0, pk0);
  ++head;
  ++pops;
  const KState st{s_q[slot], jm0, __uint_as_float(s_q[QL * 64 + slot]), pk0};
  if (live_dup(P, lv, st)) return;  // :618-622 against the snapshot's popped states
  lane_expand<QL, ELN, false>(P, s_q, s_e, S, start, st, status, head, tail, nel, err);
}

// Persistent lanes: a lane whose window finishes (or bails) takes the next listed window at once,
// so a wave is not held by its slowest window; the wave lists unfinished windows from the lookup
// results chunk by chunk as its idle lanes need them.
template <uint32_t QL, uint32_t ELN>
__global__ __launch_bounds__(64) void lane_window_kernel(SearchParams P) {
  __shared__ uint32_t s_q[3 * QL * 64];  // ring slot i of lane l at i * 64 + l, three planes
  // best lists in this workgroup's slice of the emit scratch (read only on emissions; keeping them out
  // of LDS lets more waves share a CU): entry i of lane l at i * 64 + l
  uint4* s_e = P.ebuf + (size_t)blockIdx.x * P.ecap;
  __shared__ uint64_t s_list[128];
  const uint32_t lane = lane_id();
  uint64_t popped_lane = 0, cached_lane = 0;
  uint32_t done_lane = 0;
  uint32_t nbuf = 0;          // wave-uniform: listed windows
  uint64_t cur = 0, ce = 0;   // wave-uniform: scan position and end of the current region's entries
  uint64_t rg_next = 0, rg_end = 0;  // wave-uniform: regions left of the current chunk
  bool chunks_done = false;   // wave-uniform
  uint32_t status = 0, head = 0, tail = 0, nel = 0, pops = 0, snap_pops = 0;
  LiveDedup lv{0u, 0u, 0u};
  uint64_t vid = 0, start = 0;
  SegDesc S{};
  unsigned err = 0;
  uint64_t trips = 0, started = 0;
  const uint64_t t_k0 = __builtin_amdgcn_s_memtime();
  for (;;) {
    const uint64_t idle = __ballot(status != LANE_RUN);
    const uint32_t n_idle = (uint32_t)__popcll(idle);
    while (nbuf < n_idle && !chunks_done) {  // list unfinished resumed windows whose snapshot fits
      if (cur >= ce) {  // the next region's open entries (rc_lookup_kernel)
        if (rg_next >= rg_end) {  // the next LANE_CHUNK windows' regions
          unsigned long long c = 0;
          if (lane == 0) c = atomicAdd(P.counters + 9, (unsigned long long)LANE_CHUNK);
          const uint64_t cb = shfl_u64(c, 0);
          if (cb >= P.total_windows) {
            chunks_done = true;
            break;
          }
          rg_next = cb / RC_REGION;
          rg_end = (min(cb + (uint64_t)LANE_CHUNK, P.total_windows) + RC_REGION - 1) / RC_REGION;
        }
        cur = rg_next * RC_REGION;
        ce = cur + P.rc_region_cnt[rg_next];
        ++rg_next;
        continue;
      }
      const uint64_t v = cur + lane;
      bool take = false;
      if (v < ce) {
        const uint4 h = P.rc_hits[v];
        take = h.x != RC_DONE && h.x != EMPTY && h.z - h.y <= QL && (h.w >> 16) <= ELN;
      }
      const uint64_t m = __ballot(take);
      if (take) s_list[nbuf + prefix_below(m)] = v;
      nbuf += (uint32_t)__popcll(m);
      cur += 64;
      __builtin_amdgcn_wave_barrier();
    }
    const uint32_t give = min(nbuf, n_idle);
    if (give == 0 && !__ballot(status == LANE_RUN)) break;
    const uint32_t r = prefix_below(idle);
    const bool starts = status != LANE_RUN && r < give;
    uint64_t next = 0;
    if (starts) next = s_list[r];
    if (give) {  // drop the handed-out entries from the list
      const uint32_t rest = nbuf - give;
      __builtin_amdgcn_wave_barrier();
      const uint64_t a0 = lane < rest ? s_list[give + lane] : 0ull;
      const uint64_t a1 = lane + 64 < rest ? s_list[give + lane + 64] : 0ull;
      __builtin_amdgcn_wave_barrier();
      if (lane < rest) s_list[lane] = a0;
      if (lane + 64 < rest) s_list[lane + 64] = a1;
      nbuf = rest;
      __builtin_amdgcn_wave_barrier();
    }
    if (starts) {  // resume the window from its snapshot
      vid = next;  // an open entry
      const uint4 h = P.rc_hits[vid];
      snap_pops = P.rc_hit_pops[vid];
      const uint64_t wid = rc_window_of(P, vid);
      const uint32_t kl = find_seg(P, wid);
      S = P.segs[kl];
      start = S.w_begin + (wid - P.seg_prefix[kl]);
      const uint32_t nq = h.z - h.y, nv = h.w & 0xFFFFu;
      nel = h.w >> 16;
      const uint4* src = P.rc_pool + h.x + RC_HDR;  // queue, dedup entries (unused), best list
      bool fits = true;
      for (uint32_t i = 0; i < nq; ++i) {
        const uint4 q = src[i];
        uint32_t w;
        fits = lane_pack(q.y, q.w, w) && fits;
        s_q[i * 64 + lane] = q.x;
        s_q[QL * 64 + i * 64 + lane] = q.z;
        s_q[2 * QL * 64 + i * 64 + lane] = w;
      }
      for (uint32_t i = 0; i < nel; ++i) s_e[i * 64 + lane] = src[nq + nv + i];
      // beamed engines: the snapshot's popped states still dedup (live_dup); a long list goes back
      const uint32_t jc = P.beam && nv ? P.rc_pool[h.x + 1].y : 0u;  // jcheck | ncheck << 16
      lv = LiveDedup{h.x + RC_HDR + nq, jc >> 16, jc & 0xFFFFu};
      head = 0;
      tail = nq;
      pops = 0;
      err = 0;
      status = fits ? LANE_RUN : LANE_BAIL;
      ++started;
    }
    ++trips;
    if (status == LANE_RUN) lane_step<QL, ELN>(P, s_q, s_e, S, start, lv, status, head, tail, nel, pops, err);
    const bool fin = status == LANE_OK, bail = status == LANE_BAIL;
    if (__ballot(fin || bail)) {  // finished windows write their records (one output atomic per wave)
      const uint32_t ne = fin ? nel : 0u;
      const uint32_t incl = wave_inclusive_sum(ne), tot = shfl_u32(incl, 63);
      unsigned long long base = 0;
      if (tot) {
        if (lane == 0) base = atomicAdd(P.counters, (unsigned long long)tot);
        base = shfl_u64(base, 0);
      }
      if (fin) {
        const uint64_t sb = S.byte_base + local_byte(P, S, start);
        for (uint32_t i = 0; i < ne; ++i) {
          const uint64_t o = base + incl - ne + i;
          if (o < P.out_cap) P.out[o] = match_record(P, S, start, sb, s_e[i * 64 + lane]);
        }
        P.rc_hits[vid] = make_uint4(RC_DONE, 0u, 0u, 0u);
        cached_lane += snap_pops;
        done_lane += 1;
      }
      if (fin || bail) {
        popped_lane += pops;
        status = 0u;
      }
    }
  }
  wave_add_counter(P.counters + 1, popped_lane);
  wave_add_counter(P.counters + 4, cached_lane);
  wave_add_counter(P.counters + 8, done_lane);
  if (P.lane_debug) {  // diagnostics (FAC_RC_DEBUG): windows started / finished, pop steps, cycles
    const uint32_t st = (uint32_t)wave_inclusive_sum((uint32_t)started), dn = wave_inclusive_sum(done_lane);
    if (lane == 63) {
      atomicAdd(&g_lane_dbg[0], (unsigned long long)st);
      atomicAdd(&g_lane_dbg[1], (unsigned long long)dn);
      atomicAdd(&g_lane_dbg[2], (unsigned long long)(st - dn));
      atomicAdd(&g_lane_dbg[4], trips);
      atomicAdd(&g_lane_dbg[6], __builtin_amdgcn_s_memtime() - t_k0);
      atomicAdd(&g_lane_dbg[7], 1ull);
    }
  }
}

// LK: the window prologue looks snapshots up itself (cache builds); otherwise a main pass with the
// prefix cache reads the hits rc_lookup_kernel stored.
template <uint32_t VCAP, uint32_t QCAP, bool MAP, bool LK, bool LIVE = false>
__device__ __forceinline__ void bfs_window_body(const SearchParams& P) {
  __shared__ KState s_vis[VCAP ? VCAP : 1];
  __shared__ KState s_live[LIVE ? LIVE_CAP : 1];
  __shared__ KState s_q[QCAP];
  __shared__ __attribute__((aligned(16))) uint32_t s_claim[claim_slots(VCAP)];
  const uint32_t lane = lane_id();
#ifdef FAC_PHASE_PROF
  const uint64_t t_life = __builtin_amdgcn_s_memtime();
  uint64_t t_grp = 0;  // group setup (lookups / hit loads) per 64 windows
  uint64_t prof_acc[kProf] = {};  // run_window's slots (per wave, in registers), 22: build epilogue, 32-36 its parts
#endif
  const uint32_t slot = slot_acquire(P);
  EmitList EL{P.ebuf + (size_t)slot * P.ecap, P.ecap, 0};
  uint4* bsel = (VCAP > 0 && P.bsel) ? P.bsel + (size_t)slot * P.bsel_stride : nullptr;
  uint64_t popped = 0, cached = 0;     // wave-uniform
  uint64_t cached_lane = 0;            // per lane: lane-flushed windows' snapshot pops
  unsigned long long pool_cur = 0, pool_end = 0;  // cache build: this wave's snapshot pool chunk
  uint32_t res_lane = 0, triv_lane = 0;  // per lane: resumed windows, of those lane-flushed
  uint32_t kept_snaps = 0;                // wave-uniform (lane 0's count): snapshots this cache build kept
  // dedup-commit claim sequence (phase C): fresh claims are >= 128, above any stale word the
  // expansion scratch leaves behind (<= 64)
  uint32_t cseq = 1;
  for (uint32_t i = lane_id(); i < claim_slots(VCAP); i += 64) s_claim[i] = 0u;
  __builtin_amdgcn_wave_barrier();
  unsigned err = 0;
  // chunks are handed out by a global work counter (counters[7]): waves that become resident late,
  // or draw cheap windows, take more chunks, so the launch ends when the work does (a static
  // grid-stride split idles every slot of a CU once its first-round workgroups finish)
  auto next_chunk = [&]() -> uint64_t {
    unsigned long long c = 0;
    if (lane == 0) c = atomicAdd(P.counters + 7, (unsigned long long)P.chunk);
    return shfl_u64(c, 0);
  };
  const uint64_t stride = (uint64_t)gridDim.x * P.chunk;
  // behind the lookups a chunk holds the open entries of each region it covers: one sub-range each
  const bool regions = !LK && P.rc_mode == 1 && !P.win_list;
  for (uint64_t cb0 = P.dyn_chunks ? next_chunk() : (uint64_t)blockIdx.x * P.chunk; cb0 < P.total_windows;
       cb0 = P.dyn_chunks ? next_chunk() : cb0 + stride) {
    const uint64_t ce0 = min(cb0 + (uint64_t)P.chunk, P.total_windows);
    for (uint64_t cb = cb0, cnext = cb0; cb < ce0 && !any_err(err); cb = cnext) {
    uint64_t ce = ce0;
    cnext = ce0;
    if (regions) {
      const uint64_t rg = cb / RC_REGION;
      cnext = min(ce0, (rg + 1) * RC_REGION);
      ce = min(cnext, rg * RC_REGION + P.rc_region_cnt[rg]);
      if (cb >= ce) continue;
    }
    // A main pass behind the lookups (and the lane kernel) finds most windows already RC_DONE:
    // one round of independent loads marks the chunk's 64-window groups that hold live windows,
    // and the rest are skipped without their dependent segment / hit / pops loads (C2 1 GiB: 6K
    // live windows out of 1G).
    uint64_t live_groups = ~0ull;
    if (!LK && P.rc_mode == 1 && !P.win_list && P.chunk > 256) {
      live_groups = 0ull;
      const uint32_t ng = (uint32_t)((ce - cb + 63) / 64);  // P.chunk <= 4096: at most 64 groups
      const uint32_t* hx = reinterpret_cast<const uint32_t*>(P.rc_hits);
      for (uint32_t g = 0; g < ng; g += 8) {
        uint32_t x[8];
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
          const uint64_t v = cb + (uint64_t)(g + q) * 64 + lane;
          x[q] = (g + q < ng && v < ce) ? hx[4 * v] : RC_DONE;
        }
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q)
          if (__ballot(x[q] != RC_DONE)) live_groups |= 1ull << (g + q);
      }
    }
    for (uint64_t v0 = cb; v0 < ce; v0 += 64) {
      if (!((live_groups >> ((v0 - cb) >> 6)) & 1ull)) continue;
#ifdef FAC_PHASE_PROF
      const uint64_t t_g0 = __builtin_amdgcn_s_memtime();
#endif
      const uint64_t v = v0 + lane;
      bool active = v < ce;
      uint32_t kl = 0;
      uint64_t start = 0, vid = 0, wid = 0;  // list id (an open entry behind the lookups) and window
      RcHit hit{EMPTY, 0u, 0u, 0u, 0u};  // prefix-cache snapshot of this lane's window
      if (active) {
        vid = P.win_list ? P.win_list[v] : v;
        wid = (!LK && P.rc_mode == 1) ? rc_window_of(P, vid) : vid;
        kl = find_seg(P, wid);
        const SegDesc S = P.segs[kl];
        start = S.w_begin + (wid - P.seg_prefix[kl]);
        if (!LK && P.rc_mode == 1) {  // skip decision and lookup made by rc_lookup_kernel
          const uint4 h = P.rc_hits[vid];
          hit = RcHit{h.x, h.y, h.z, h.w, P.rc_hit_pops[vid]};
          active = h.x != RC_DONE;
        } else {
          active = !window_skipped(P, S, start, err);
        }
      }
      if constexpr (LK)
        if (P.rc_mode != 0 && P.rc_ntab && active && P.rc_bhits) {  // rc_parent_kernel's lookup
          const uint4 h = P.rc_bhits[v];
          hit = RcHit{h.x, h.y, h.z, h.w, P.rc_bpops[v]};
        }
      if (LK && P.rc_mode == 1) {
        const bool resumed = active && hit.off != EMPTY;
        res_lane += resumed ? 1u : 0u;
        active = active && !flush_final(P, resumed, hit, kl, start, wid, cached_lane, triv_lane);
      }
      if (P.rc_mode == 2) {
        // a representative whose parent snapshot has an empty queue ends at the parent: its own
        // snapshot would hold the same best list, so the key stays uncached (lookups fall through)
        const bool done = active && hit.off != EMPTY && hit.tail == hit.head && !P.rc_keep_final;
        if (done) {
          P.rc_off[v] = EMPTY;
          P.rc_count[v] = EMPTY;
        }
        active = active && !done;
      }
      uint64_t m = __ballot(active);
#ifdef FAC_PHASE_PROF
      t_grp += __builtin_amdgcn_s_memtime() - t_g0;
#endif
      while (m) {
        const int l = first_lane(m);
        m &= m - 1;
        const uint32_t seg = shfl_u32(kl, l);
        const uint64_t st = shfl_u64(start, l);
        const SegDesc S = P.segs[seg];
        const uint64_t popped0 = popped;
        uint32_t qhead = 0, vcnt = 0, jbeam[2] = {0u, 0u};
        const RcHit rc{shfl_u32(hit.off, l), shfl_u32(hit.head, l), shfl_u32(hit.tail, l), shfl_u32(hit.nv_nel, l),
                       shfl_u32(hit.pops, l)};
#ifdef FAC_WIN_HIST
        const uint64_t t_w0 = __builtin_amdgcn_s_memtime();
#endif
        const uint32_t qlen =
            run_window<VCAP, QCAP, MAP, LIVE>(P, S, s_vis, s_q, s_claim, cseq, EL, st, rc, popped, cached, err, qhead,
                                              vcnt, s_live, jbeam, bsel
#ifdef FAC_PHASE_PROF
                                              , prof_acc
#endif
                                              );
#ifdef FAC_WIN_HIST
        if (lane == 0 && P.rc_mode != 2) {
          const uint32_t b = hist_bucket(popped - popped0);
          atomicAdd(&g_hist[b], 1ull);
          atomicAdd(&g_hist[6 + b], (unsigned long long)(popped - popped0));
          atomicAdd(&g_hist[12 + b], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_w0));
          atomicAdd(&g_hist[18 + b], rc.off != EMPTY ? 1ull : 0ull);
        }
#endif
        if (LK && P.rc_mode == 2) {  // cache build: entry = list position; what does not fit stays uncached
#ifdef FAC_PHASE_PROF
          struct EpAcc {
            uint64_t t;
            uint64_t& acc;
            __device__ ~EpAcc() { acc += __builtin_amdgcn_s_memtime() - t; }
          } ep_acc{__builtin_amdgcn_s_memtime(), prof_acc[22]};
#endif
#ifdef FAC_PHASE_PROF
          uint64_t t_ep = __builtin_amdgcn_s_memtime();
          auto ep_lap = [&](int slot) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            prof_acc[slot] += t - t_ep;
            t_ep = t;
          };
#define EP_LAP(i) ep_lap(i)
#else
#define EP_LAP(i)
#endif
          const uint32_t ent = (uint32_t)(v0 + (uint64_t)l);
          const uint32_t nq = qlen - qhead;
          // live dedup entries: a key is only met again at its own j, and every future state's j is
          // at least the smallest j in the queue (j never decreases along a path)
          uint32_t jmin = 0xFFFFu;
          for (uint32_t i = lane; i < nq; i += 64) jmin = min(jmin, s_q[(qhead + i) & (QCAP - 1)].jm & 0xFFFFu);
          jmin = wave_min_u32(jmin);
          auto live = [&](const KState& k) { return k.node != EMPTY && (k.jm & 0xFFFFu) >= jmin; };
          uint32_t nv = 0, jlive = 0;  // 1 + the largest j among the live entries (0: none)
          // each lane's VCAP/64 slots, their live bits kept; the entries are read from LDS again by the
          // writing passes below (held in registers, the 8 slots' 32 VGPRs made this the kernel's
          // register peak and pushed loop state into scratch)
          constexpr uint32_t NSL = VCAP ? VCAP / 64 : 1;
          uint32_t lmask = 0;
          if constexpr (VCAP > 0) {
#pragma unroll
            for (uint32_t u = 0; u < NSL; ++u) {
              const KState kvu = s_vis[u * 64 + lane];
              const bool lv = live(kvu);
              lmask |= (lv ? 1u : 0u) << u;
              nv += (uint32_t)__popcll(__ballot(lv));
              jlive = max(jlive, lv ? (kvu.jm & 0xFFFFu) + 1u : 0u);
            }
          }
          jlive = wave_inclusive_max(jlive);
          jlive = shfl_u32(jlive, 63);
          bool bad = (wave_or(err) & (ERR_QUEUE | ERR_VISITED | ERR_EMIT)) != 0 || EL.n > P.rc_emax || nv > P.rc_vmax;
          if (bad && lane == 0) {  // diagnostics (FAC_RC_DEBUG): why keys stay uncached
            const unsigned we = wave_or(err);
            atomicAdd(&g_bad[(we & ERR_QUEUE) ? 0 : (we & ERR_VISITED) ? 1 : (we & ERR_EMIT) ? 2 : EL.n > P.rc_emax ? 3 : 4], 1ull);
          }
          EP_LAP(32);
          const uint32_t words = RC_HDR + nq + nv + EL.n;
          // the wave carves snapshots out of its own pool chunk: one pool atomic per chunk, not per
          // snapshot (a same-address atomic per entry serialises the build at one L2 channel)
          if (!bad && pool_cur + words > pool_end) {
            const unsigned long long want = max((unsigned long long)words, (unsigned long long)P.rc_pool_chunk);
            unsigned long long c = 0;
            if (lane == 0) c = atomicAdd(P.rc_pool_used, want);
            pool_cur = shfl_u64(c, 0);
            pool_end = pool_cur + want;
          }
          const unsigned long long off = pool_cur;
          if (!bad) pool_cur += words;
          bad = bad || off + words > P.rc_pool_cap || off > 0xFFFFFFF0ull;
          EP_LAP(33);
          // (the key's chars are not stored: rc_publish_kernel reads them from the representative's text)
          uint4* dst = P.rc_pool + off + RC_HDR;  // after the header words
          for (uint32_t i = lane; i < nq && !bad; i += 64) {
            const KState k = s_q[(qhead + i) & (QCAP - 1)];
            dst[i] = make_uint4(k.node, k.jm, __float_as_uint(k.pen), k.packed);
          }
          EP_LAP(34);
          // compacted in slot order, the entries a resumed dedup-free run must still honour (j < jcheck)
          // first: ncheck of them
          const uint32_t jcheck = min(jlive, jbeam[0]);
          uint32_t ncheck = 0;
          if constexpr (VCAP > 0) {
            uint32_t at0 = 0;
            for (uint32_t pass = 0; pass < 2 && !bad; ++pass) {
#pragma unroll
              for (uint32_t u = 0; u < NSL; ++u) {
                const KState kvu = s_vis[u * 64 + lane];
                const bool chk = (kvu.jm & 0xFFFFu) + 1u <= jcheck;
                const bool occ = ((lmask >> u) & 1u) && (pass == 0 ? chk : !chk);
                const uint64_t m = __ballot(occ);
                if (occ) dst[nq + at0 + prefix_below(m)] = make_uint4(kvu.node, kvu.jm, __float_as_uint(kvu.pen), kvu.packed);
                at0 += (uint32_t)__popcll(m);
              }
              if (pass == 0) ncheck = at0;
            }
          }
          EP_LAP(35);
          for (uint32_t i = lane; i < EL.n && !bad; i += 64) dst[nq + nv + i] = EL.buf[i];
          if (lane == 0) {
            if (!bad) {
              // pops: those of the parent snapshot this build resumed from, plus its own
              P.rc_pool[off] = make_uint4(qhead, qlen, nv, (uint32_t)(popped - popped0) + rc.pops);
              // jcheck: dedup entries a resumed dedup-free run must still honour (j + 1 <= jcheck)
              P.rc_pool[off + 1] = make_uint4(EL.n, ncheck ? (jcheck | (ncheck << 16)) : 0u, jbeam[0], jbeam[1]);
            }
            P.rc_off[ent] = bad ? EMPTY : (uint32_t)off;
            P.rc_count[ent] = bad ? EMPTY : nq;
            kept_snaps += bad ? 0u : 1u;
          }
          (void)vcnt;
          err &= ~(ERR_QUEUE | ERR_VISITED | ERR_EMIT);
          __builtin_amdgcn_wave_barrier();
          EP_LAP(36);
#undef EP_LAP
          if (any_err(err)) break;
          continue;
        }
        const bool overflow = (wave_or(err) & (ERR_QUEUE | ERR_VISITED)) != 0;
        const uint64_t w_id = shfl_u64(wid, l);
        if (P.win_counts && !overflow && lane == 0) P.win_counts[w_id] = qlen;
        if (overflow) {  // frontier overflow: spill the window
          const uint64_t id = shfl_u64(vid, l);
          if (lane == 0) {
            const unsigned long long k = atomicAdd(P.counters + 3, 1ull);
            if (k < P.spill_cap) P.spill[k] = id;
            else err |= ERR_SPILL;
          }
          err &= ~(ERR_QUEUE | ERR_VISITED);
        }
        if (any_err(err)) break;
      }
      if (any_err(err)) break;
    }
    }  // sub-ranges
    if (any_err(err)) break;
  }
  if (lane == 0) atomicAdd(P.counters + 1, (unsigned long long)popped);
  if (lane == 0 && kept_snaps) atomicAdd(P.counters + 11, (unsigned long long)kept_snaps);  // sizes the lookup table
#ifdef FAC_PHASE_PROF
  if (lane == 0) {
    const int pb = P.rc_mode == 2 ? kProf : 0;
    for (int i = 0; i < kProf; ++i)
      if (i != 23 && i != 24) atomicAdd(&g_prof[pb + i], (unsigned long long)prof_acc[i]);
    atomicAdd(&g_prof[pb + 23], (unsigned long long)t_grp);
    atomicAdd(&g_prof[pb + 24], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_life));
  }
#endif
  if (lane == 0) cached_lane += cached;
  wave_add_counter(P.counters + 4, cached_lane);
  wave_add_counter(P.counters + 5, res_lane);
  wave_add_counter(P.counters + 6, triv_lane);
  const unsigned all = wave_or(err);
  if (lane == 0 && all) atomicOr(reinterpret_cast<unsigned int*>(P.counters + 2), all);
  slot_release(P, slot);
}

// one wavefront per workgroup; the dedup-free variants are held to <= 128 VGPRs (4 waves/SIMD),
// the dedup variants are bounded by LDS first
#ifndef FAC_BEAM_WAVES  // waves/SIMD the dedup variants are compiled for (VGPR budget); 0 = unbounded
// 3: <= 168 VGPRs (a few rare-path spills), matching the 11 workgroups/CU their LDS allows; unbounded
// they take ~175 VGPRs and 2 waves/SIMD (C3 kernel 133 -> 111 ms measured)
#define FAC_BEAM_WAVES 3
#endif
template <uint32_t VCAP, uint32_t QCAP, bool MAP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu((FAC_BEAM_WAVES && VCAP <= 512 && QCAP <= 256) ? (VCAP <= 256 ? FAC_BEAM_WAVES + 1 : FAC_BEAM_WAVES) : 1)))
void bfs_window_kernel(SearchParams P) {
  bfs_window_body<VCAP, QCAP, MAP, false>(P);
}
template <uint32_t QCAP, bool MAP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(QCAP <= 512 ? 4 : 1))) void bfs_window_kernel_nd(SearchParams P) {
  bfs_window_body<0, QCAP, MAP, false>(P);
}
// dedup-free first pass of a beamed engine (launch_pass): windows that would beam are spilled, the
// resumed snapshots' popped states still dedup (run_window LIVE)
#ifndef FAC_LIVE_WAVES  // waves/SIMD bfs_window_kernel_live is compiled for (VGPR budget)
#define FAC_LIVE_WAVES 4
#endif
template <uint32_t QCAP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FAC_LIVE_WAVES))) void bfs_window_kernel_live(SearchParams P) {
  bfs_window_body<0, QCAP, false, false, true>(P);
}
// prefix-cache build (P.rc_mode == 2): one representative window per key, popped up to the first
// state past the key; its own symbol so profiles separate it from the search launches
template <uint32_t QCAP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu((FAC_BEAM_WAVES && QCAP <= 256) ? FAC_BEAM_WAVES : 1)))
void rc_build_kernel(SearchParams P) {
  bfs_window_body<512, QCAP, false, true>(P);  // the prefix cache is off with mappings
}

// ------------------------------------------------------------------------------------------
// Bit-parallel pre-filter (prefilter.rs:247-435)
// ------------------------------------------------------------------------------------------

// transcode, ASCII fast path (prefilter.rs:253-260): ids[i] = ascii_id[byte]
__global__ void transcode_ascii_kernel(const uint8_t* __restrict__ utf8, uint64_t n, const uint8_t* __restrict__ ascii_id,
                                       uint8_t* __restrict__ ids) {
  const uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (i0 + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(utf8 + i0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
    for (int q = 0; q < 4; ++q) {
      uint32_t r = 0;
      for (int b = 0; b < 4; ++b) r |= (uint32_t)ascii_id[(w[q] >> (8 * b)) & 0x7Fu] << (8 * b);
      o[q] = r;
    }
    *reinterpret_cast<uint4*>(ids + i0) = make_uint4(o[0], o[1], o[2], o[3]);
  } else {
    for (uint64_t i = i0; i < n; ++i) ids[i] = ascii_id[utf8[i] & 0x7Fu];
  }
}

struct BitapParams {
  const uint8_t* ids;
  uint64_t n;
  const void* mask_t;      // [(alphabet+1)][n_words] transposed packed masks (uint32_t or uint64_t words)
  const void* top;         // per word: the top (match) bit of every pattern packed into it
  const uint32_t* k;       // per word: the edit budget shared by its patterns
  uint32_t n_words;
  uint32_t seg_len;        // text positions owned by one wave
  uint32_t* cover;         // coverage bitmap, 1 bit per grapheme
};

// Shift-AND over several patterns per automaton word: the patterns of one edit budget are packed
// side by side (pattern f in bits lo_f..top_f). Every recurrence of bitap_windows
// (prefilter.rs:410-435) only moves bits upwards by one, so a pattern's top bit carries into the next
// pattern's bit 0 only, and that bit is forced to 1 in every level (the `| 1` of the recurrence,
// here `| first`) -- level 0 ANDs the carried bit with the same mask bit as the forced one. Bits
// 0..m-1 of every field therefore evolve exactly as in a word of their own; the reference's bits at
// and above m never reach below m, so dropping them changes nothing observable.
template <typename W>
__device__ __forceinline__ W low_bits(uint32_t n) {
  return n >= sizeof(W) * 8 ? ~(W)0 : (((W)1 << n) - (W)1);
}

// Each lane runs one packed word over the wave's text segment. The state after `m + k` symbols no
// longer depends on the initial state, so a segment starts `m + k` symbols early from the
// reference's initial state and only reports ends inside its own range. Every hit of pattern f
// covers [end - m_f - k, end) in the bitmap; maximal runs of the bitmap are exactly the sorted +
// merged windows of prefilter.rs:334-342.
// W: the automaton word (uint32_t when every pattern has m <= 32: half the VALU work of uint64_t);
// KMAX: the largest edit budget (levels above a word's own k are computed but never read).
template <int KMAX, typename W>
__global__ __launch_bounds__(256) void bitap_kernel(BitapParams B) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t word_groups = (B.n_words + 63) / 64;
  const uint64_t seg = wave / word_groups;
  const uint32_t p = (wave % word_groups) * 64 + lane;
  const uint64_t a = seg * B.seg_len;
  if (a >= B.n) return;
  const uint64_t b = min(a + (uint64_t)B.seg_len, B.n);
  const bool live = p < B.n_words;
  const W top = live ? static_cast<const W*>(B.top)[p] : (W)0;
  const uint32_t k = live ? B.k[p] : 0;
  const W first = (W)(top << 1) | (W)1;  // bit 0 of every field
  W r[KMAX + 1];
  // initial state R[d] = (1 << d) - 1 per pattern (prefilter.rs:417), clipped to the field
#pragma unroll
  for (int d = 0; d <= KMAX; ++d) r[d] = 0;
  {
    uint32_t lo = 0;
    for (W t = top; t;) {
      const uint32_t hi = (uint32_t)__builtin_ctzll((unsigned long long)t);
      t &= t - 1;
      const uint32_t m = hi + 1 - lo;
#pragma unroll
      for (int d = 1; d <= KMAX; ++d) r[d] |= low_bits<W>(min((uint32_t)d, m)) << lo;
      lo = hi + 1;
    }
  }
  // Start 87 = 63 + 24 symbols early: from there on the automaton state equals the one obtained by
  // scanning from the text start (an alignment with <= k errors spans <= m + k symbols).
  const uint64_t warm = 63 + 24;
  const uint64_t s0 = a > warm ? a - warm : 0;
  // Symbols come in 64 at a time (lane l loads symbol i0 + l, broadcast by readlane) and each lane
  // issues the masks of 8 symbols before stepping through them, so the loop waits on one memory
  // round trip per 8 symbols instead of two per symbol.
  constexpr uint32_t U = 8;
  const W* mask_p = static_cast<const W*>(B.mask_t) + (live ? p : 0u);  // this lane's column
  for (uint64_t i0 = s0; i0 < b; i0 += 64) {
    const uint32_t cl = i0 + lane < b ? (uint32_t)B.ids[i0 + lane] : 0u;
    const uint32_t nsym = (uint32_t)min((uint64_t)64, b - i0);
    for (uint32_t u0 = 0; u0 < nsym; u0 += U) {
      W bcs[U];
#pragma unroll
      for (uint32_t q = 0; q < U; ++q) {
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cl, (int)(u0 + q));  // u0 + q < 64: wave-uniform
        bcs[q] = (live && u0 + q < nsym) ? mask_p[(size_t)c * B.n_words] : (W)0;
      }
      // the hits of the 8 symbols are kept and only looked at when one of them is set (rare): the
      // per-symbol path carries no segment-range compare and no divergent branch
      W hq[U];
#pragma unroll
      for (uint32_t q = 0; q < U; ++q) hq[q] = (W)0;
#pragma unroll
      for (uint32_t q = 0; q < U; ++q) {
        if (u0 + q >= nsym) break;
        const W bc = bcs[q];
        W prev_old = r[0];
        W prev_new = ((r[0] << 1) | first) & bc;
        r[0] = prev_new;
        W hit_level = (k == 0) ? prev_new : (W)0;
#pragma unroll
        for (int d = 1; d <= KMAX; ++d) {
          const W old = r[d];
          const W nv = ((old << 1) & bc) | ((prev_old | prev_new) << 1) | prev_old | first;
          r[d] = nv;  // levels above k are computed but never read
          prev_old = old;
          prev_new = nv;
          if ((uint32_t)d == k) hit_level = nv;
        }
        hq[q] = hit_level & top;  // R[k] subsumes the lower levels
      }
      W any = (W)0;
#pragma unroll
      for (uint32_t q = 0; q < U; ++q) any |= hq[q];
      if (live && any) {
#pragma unroll
        for (uint32_t q = 0; q < U; ++q) {
          W hits = hq[q];
          const uint64_t i = i0 + u0 + q;
          if (!hits || i < a) continue;  // ends before the segment belong to the previous wave
          const uint64_t end = i + 1;
          do {
            const uint32_t hi = (uint32_t)__builtin_ctzll((unsigned long long)hits);
            hits &= hits - 1;
            const W below = top & low_bits<W>(hi);  // tops of the fields under this one
            const uint32_t lo = below ? 64u - (uint32_t)__builtin_clzll((unsigned long long)below) : 0u;
            const uint64_t span = (uint64_t)(hi + 1 - lo) + k;
            const uint64_t ws = end > span ? end - span : 0;
            for (uint64_t x = ws; x < end;) {  // set bits [ws, end)
              const uint64_t w = x >> 5;
              const uint32_t l = (uint32_t)(x & 31);
              const uint32_t cnt = (uint32_t)min((uint64_t)(32 - l), end - x);
              const uint32_t bits = (cnt == 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u)) << l;
              atomicOr(B.cover + w, bits);
              x += cnt;
            }
          } while (hits);
        }
      }
    }
  }
}

// ---- Pigeonhole q-gram filter in front of the bitap scan (exact) ----
// A pattern of m symbols within k Levenshtein edits of a text window keeps at least one of k + 1
// disjoint pieces of itself untouched, i.e. that piece occurs verbatim in the window. Each piece
// contributes its first q symbols (q = min(4, shortest piece), >= 3) as a gram; qgram_scan_kernel
// looks every text position's 3- and 4-gram up in a small cache-resident table and lists the
// (position, pattern, piece offset) candidates. qgram_verify_kernel runs the pattern's own bitap
// recurrence (prefilter.rs:410-435) over the only ends the candidate allows -- piece at text t,
// pattern offset o: end in [t + m - o - k, t + m - o + k] -- starting m + k symbols early, where the
// automaton state no longer depends on where the scan began (bitap_kernel's warm-up), and sets the
// same coverage bits as bitap_kernel. Every hit of every gram-eligible pattern is thus found (and no
// other: the recurrence is exact), so the merged windows equal the full scan's.
struct QgramParams {
  // the text: symbol ids (ids mode), or an ASCII haystack's bytes read directly (bytes mode: the
  // grams are keyed by case-folded bytes, verify maps bytes to ids through aid); text position i is
  // buffer byte off + i (the buffer 16-byte aligned), and bytes at or past nsafe are never read
  const uint8_t* ids;
  uint64_t n;
  uint64_t nsafe;
  uint32_t off, bytes, ci;
  const uint8_t* aid;
  const uint2* tab;        // open addressing: {gram key, first entry << 8 | entries} (0: empty slot)
  uint32_t tab_mask;
  const uint2* ent;        // entries: {pattern << 8 | piece offset, m | k << 8} (one load per candidate)
  uint32_t use3, use4;     // gram lengths in use
  uint32_t use5;           // 4-gram probes screened by the 5-gram (pieces of >= 5 symbols)
  // candidates (text position << 24 | entry index): scan block b fills region b of cand (region
  // entries, rcnt[b] of them valid), and what does not fit goes to the overflow list ovf
  unsigned long long* cand;
  uint64_t region;
  uint32_t* rcnt;
  uint32_t nreg;
  unsigned long long* ovf;
  unsigned long long* n_ovf;
  uint64_t ovf_cap;
  const uint64_t* pmask;   // per pattern: [rows] symbol masks (bit j = the pattern's j-th symbol)
  const uint32_t* pm;      // per pattern: m | k << 8
  uint32_t rows;
  uint32_t* cover;
  const uint32_t* bits;    // QG_BITS_WORDS: screening bitmap of the grams (qgram_bit)
  const uint32_t* m16;     // every q-gram pattern m <= 16: [pattern][rows] 16-bit masks, m16_words words
  uint32_t m16_words;
  // stream windows (a batch of stream.rs windows searched by one pass over their union, the view):
  // window w is the text [wlo[w], whi[w]) of the view, sorted by wlo, overlapping only its neighbours;
  // its coverage goes to cover (w even) or cover2 (w odd), so same-parity windows never touch.
  // wtab[t >> QG_WSH]: the last window starting at or before that bucket's first position.
  uint32_t nwin;
  const uint64_t* wlo;
  const uint64_t* whi;
  const uint32_t* wtab;
  uint32_t* cover2;
  // wsh != 0: window w is [w << wsh, min(n, (w + 1) << wsh) + wov)) -- the crate's fixed-size cut,
  // bounds computed instead of loaded
  uint32_t wsh, wov;
};
constexpr uint32_t QG_WSH = 16;  // window-table buckets of 64 Ki positions
__host__ __device__ inline uint32_t qgram_key(uint32_t a, uint32_t b, uint32_t c, uint32_t d, bool q4) {
  return q4 ? (a | (b << 8) | (c << 16) | (d << 24)) : (a | (b << 8) | (c << 16) | 0xFF000000u);
}
__host__ __device__ inline uint32_t qgram_hash(uint32_t h) {  // murmur3 finalizer: every key bit reaches the low bits
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

__device__ __forceinline__ uint32_t qgram_find(const QgramParams& Q, uint32_t key) {  // 0: none
  uint32_t s = qgram_hash(key) & Q.tab_mask;
  for (;;) {
    const uint2 e = Q.tab[s];
    if (e.y == 0u) return 0u;
    if (e.x == key) return e.y;
    s = (s + 1) & Q.tab_mask;
  }
}

// The screening bitmap's hash (64 Kbit; the table probe behind it keeps qgram_hash). Built on the
// host, copied into LDS per block. Bit = the top 18 bits of P = key[0:24) * A for a 3-gram, of
// P + key[8:32) * B for a 4-gram: full-rate 24-bit multiplies (a 32-bit v_mul_lo is quarter rate, and
// the scan's VALU count bounds it); a position's 3- and 4-gram share P (their first three symbols), so
// the pair costs one multiply and one v_mad_u32_u24, and the scan reads the bit as byte hash >> 17,
// bit (hash >> 14) & 7 with no masking. 3-gram keys carry 0xFF as their fourth symbol (qgram_key).
// 256 Kbit: every false pass costs a queue round and a table probe (C5 scan per GiB, profiles/r05_scan:
// 64 / 128 / 256 Kbit 1.49 / 1.14 / 1.11 ms).
__host__ __device__ inline uint32_t qg_mul24(uint32_t a, uint32_t b) { return (a & 0xFFFFFFu) * (b & 0xFFFFFFu); }
constexpr uint32_t QG_HA = 0x9E3779u, QG_HB = 0x85EBCAu;
#ifndef FAC_QG_BITS_LOG
#define FAC_QG_BITS_LOG 18
#endif
constexpr uint32_t QG_BITS_LOG = FAC_QG_BITS_LOG;  // log2 of the bitmap's bits
__host__ __device__ inline uint32_t qgram_bit(uint32_t key) {
  const uint32_t p = qg_mul24(key, QG_HA);
  return ((key >> 24) == 0xFFu ? p : p + qg_mul24(key >> 8, QG_HB)) >> (32 - QG_BITS_LOG);
}
constexpr uint32_t QG_BITS_WORDS = (1u << QG_BITS_LOG) / 32;
// A piece of >= 5 symbols is screened by its first five (round 6): its table key stays the 4-gram,
// but its bit is qgram_bit5 of the 4-gram and the fifth symbol, so a text position whose 4-gram
// matches a piece while its fifth symbol does not (C5: most of the 34 M candidates per GiB of
// 4-gram screening -- random vocabulary words sharing four letters with a pattern piece) rarely
// passes, and the verify no longer runs for it. Exact: a true hit keeps a whole piece, whose first
// five symbols lie in the text.
constexpr uint32_t QG_HC = 0xC2B2AEu;
__host__ __device__ inline uint32_t qgram_bit5(uint32_t key4, uint32_t c5) {
  const uint32_t h4 = qg_mul24(key4, QG_HA) + qg_mul24(key4 >> 8, QG_HB);
  return (h4 + qg_mul24((key4 >> 16) | (c5 << 16), QG_HC)) >> (32 - QG_BITS_LOG);
}

// Candidates go to the block's own region of the list, reserved with an LDS counter: one global
// list counter took a same-address atomic per flush of a per-wave buffer, and those atomics
// serialised at one L2 channel (C5, 34 M candidates per GiB: 256-entry flushes 1.87 ms per GiB,
// 128-entry 3.68, one atomic per wave turn 175 ms; per-block regions 1.14; profiles/r05_scan). 16 waves
// per block share the screening bitmap: 32 KB + 1.5 KB per wave = 56 KB, 2 blocks = 32 waves per CU
// (8-wave blocks: 44 KB, 3 blocks = 24 waves, 1.09 against 1.00 ms per GiB).
#ifndef FAC_QG_WAVES
#define FAC_QG_WAVES 16
#endif
constexpr uint32_t QG_WAVES = FAC_QG_WAVES;
// The bitmap screens every position first: only the ~3 % that pass (C5) probe the table in global
// memory, 64 at a time from a per-wave LDS queue (one table round trip per 64 passing grams: probing
// where they stood cost a round trip per wave step, since some lane of 64 passes almost every one).
// Round 5: a thread's 32 grams (16 positions x 3-/4-gram, one 16-byte load) are screened together
// into a pass mask, and the passes join the queue in rounds of one per lane (one ballot per round)
// instead of a ballot per gram.
constexpr uint32_t QG_PQ = 128;  // per-wave probe queue (LDS): < 64 left after a drain + one round
// 4 buffer bytes from byte b (4-aligned), zero at and past nsafe
__device__ __forceinline__ uint32_t qg_word(const QgramParams& Q, uint64_t b) {
  if (b + 4 <= Q.nsafe) return reinterpret_cast<const uint32_t*>(Q.ids)[b >> 2];
  uint32_t w = 0;
  for (uint32_t u = 0; u < 4; ++u)
    if (b + u < Q.nsafe) w |= (uint32_t)Q.ids[b + u] << (8 * u);
  return w;
}
// ASCII case folding of four bytes < 0x80 (the engine's fold for ASCII haystacks, builder.cpp ascii_id)
__device__ __forceinline__ uint32_t qg_fold(uint32_t w) {
  const uint32_t t = w | 0x80808080u;
  const uint32_t up = ((t - 0x41414141u) & ~(t - 0x5B5B5B5Bu)) & 0x80808080u;  // bytes in 'A'..'Z'
  return w + (up >> 2);
}
// U3 / U4: 3- / 4-grams in use (C5: 4-grams only, so the 3-grams' bitmap reads are not issued)
template <bool U3, bool U4, bool U5>
__global__ __launch_bounds__(64 * QG_WAVES) void qgram_scan_kernel(QgramParams Q) {
  __shared__ uint32_t s_bits[QG_BITS_WORDS];
  __shared__ uint32_t s_cnt, s_fail;  // region entries reserved; the first reservation that did not fit
  __shared__ uint32_t s_pk[QG_WAVES][QG_PQ];
  __shared__ uint64_t s_pp[QG_WAVES][QG_PQ];
  for (uint32_t x = threadIdx.x; x < QG_BITS_WORDS; x += blockDim.x) s_bits[x] = Q.bits[x];
  if (threadIdx.x == 0) {
    s_cnt = 0;
    s_fail = (uint32_t)Q.region;
  }
  __syncthreads();
  unsigned long long* const reg = Q.cand + (uint64_t)blockIdx.x * Q.region;
  uint32_t* pk = s_pk[threadIdx.x / 64];
  uint64_t* pp = s_pp[threadIdx.x / 64];
  uint32_t nq = 0;  // wave-uniform
  auto drain = [&](bool all) {
    while (nq >= 64 || (all && nq > 0)) {
      const uint32_t take = min(nq, 64u), lane = lane_id();
      uint32_t h = 0;
      uint64_t pos = 0;
      __builtin_amdgcn_wave_barrier();
      if (lane < take) {
        pos = pp[nq - take + lane];
        h = qgram_find(Q, pk[nq - take + lane]);
      }
      __builtin_amdgcn_wave_barrier();
      nq -= take;
      const uint32_t cnt = h & 0xFFu;
      if (!__ballot(cnt)) continue;
      const uint32_t incl = wave_inclusive_sum(cnt), tot = shfl_u32(incl, 63);
      uint32_t r0 = 0;
      if (lane == 63) r0 = atomicAdd(&s_cnt, tot);
      r0 = shfl_u32(r0, 63);
      unsigned long long* dst = reg;
      uint64_t at = r0 + (incl - cnt), lim = Q.region;
      if ((uint64_t)r0 + tot > Q.region) {  // region full: the overflow list
        unsigned long long o0 = 0;
        if (lane == 63) {
          atomicMin(&s_fail, r0);
          o0 = atomicAdd(Q.n_ovf, (unsigned long long)tot);
        }
        dst = Q.ovf;
        at = shfl_u64(o0, 63) + (incl - cnt);
        lim = Q.ovf_cap;
      }
      for (uint32_t y = 0; y < cnt; ++y, ++at)
        if (at < lim) dst[at] = (pos << 24) | ((h >> 8) + y);
    }
  };
  // a thread takes 16 consecutive positions from one aligned 16-byte load plus the next word
  // (positions whose gram would cross the text's end are not looked up)
  const uint4* ids16 = reinterpret_cast<const uint4*>(Q.ids);
  const uint32_t* ids32 = reinterpret_cast<const uint32_t*>(Q.ids);
  const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(s_bits);
  const uint64_t nbuf = Q.off + Q.n;  // buffer bytes of the text
  const uint64_t n16 = (nbuf + 15) / 16;  // buffer sixteens
  // sixteens whose 20 bytes lie below nsafe: read with plain loads
  const uint64_t gdir = min(n16, Q.nsafe >= 20 ? (Q.nsafe - 20) / 16 + 1 : (uint64_t)0);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t lane64 = threadIdx.x % 64;
  uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x - lane64;  // whole waves iterate together
  auto turn = [&](uint64_t g, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4)
                  __attribute__((always_inline)) {
    if (Q.bytes && Q.ci) {
      w0 = qg_fold(w0);
      w1 = qg_fold(w1);
      w2 = qg_fold(w2);
      w3 = qg_fold(w3);
      w4 = qg_fold(w4);
    }
    // symbols j .. j + 3 of this thread's sixteen (value selects: a select of references became a
    // pointer array in scratch)
    auto gram4 = [w0, w1, w2, w3, w4](uint32_t j) -> uint32_t {
      const uint32_t q = j >> 2;
      uint32_t lo = w0, hi = w1;
      lo = q >= 1u ? w1 : lo;
      hi = q >= 1u ? w2 : hi;
      lo = q >= 2u ? w2 : lo;
      hi = q >= 2u ? w3 : hi;
      lo = q >= 3u ? w3 : lo;
      hi = q >= 3u ? w4 : hi;
      return __builtin_amdgcn_alignbyte(hi, lo, j & 3u);
    };
    // pass mask: bit 2j = the 4-gram at buffer byte 16g + j (text position 16g + j - off), bit
    // 2j + 1 = its 3-gram. Every bitmap read is unconditional (the text bounds are a mask applied
    // after), so the LDS reads go out in batches: per-gram conditions had made each a branch with its
    // own wait.
    uint32_t pm = 0;
    auto screen = [&](auto all_in) {  // all_in: every gram of the sixteen lies inside the text
#pragma unroll
      for (uint32_t j = 0; j < 16; ++j) {
        // qgram_bit of the 3-gram (h3) and the 4-gram (h4) at this position, qgram_bit5 (h5)
        const uint32_t k4 = gram4(j), h3 = qg_mul24(k4, QG_HA), h4 = h3 + qg_mul24(k4 >> 8, QG_HB);
        constexpr uint32_t sh = 32 - QG_BITS_LOG;
        if constexpr (U4) pm |= __builtin_amdgcn_ubfe(s_bytes[h4 >> (sh + 3)], (h4 >> sh) & 7u, 1u) << (2 * j);
        if constexpr (U5) {
          const uint32_t wq = (j + 4) >> 2;  // symbol j + 4: in w1..w4 (j + 4 <= 19)
          const uint32_t c5 = ((wq == 1u ? w1 : wq == 2u ? w2 : wq == 3u ? w3 : w4) >> (8 * ((j + 4) & 3u))) & 0xFFu;
          const uint32_t h5 = h4 + qg_mul24((k4 >> 16) | (c5 << 16), QG_HC);
          pm |= __builtin_amdgcn_ubfe(s_bytes[h5 >> (sh + 3)], (h5 >> sh) & 7u, 1u) << (2 * j);
        }
        if constexpr (U3) pm |= __builtin_amdgcn_ubfe(s_bytes[h3 >> (sh + 3)], (h3 >> sh) & 7u, 1u) << (2 * j + 1);
      }
      if (!all_in) {
        uint32_t ok = 0;
        for (uint32_t j = 0; j < 16; ++j) {
          const uint64_t i = 16 * g + j;
          if (i >= Q.off && i + 4 <= nbuf) ok |= 1u << (2 * j);
          if (i >= Q.off && i + 3 <= nbuf) ok |= 1u << (2 * j + 1);
        }
        pm &= ok;
      }
    };
    if (g < n16) {
      if (16 * g >= Q.off && 16 * g + 19 <= nbuf) screen(std::true_type{});
      else screen(std::false_type{});
    }
    // rounds: each lane's next pass joins the queue (in lane order within a round)
    for (;;) {
      const bool has = pm != 0;
      const uint64_t m = __ballot(has);
      if (!m) break;
      if (nq + 64 > QG_PQ) drain(false);
      if (has) {
        const uint32_t bit = (uint32_t)__builtin_ctz(pm);
        pm &= pm - 1;
        const uint32_t j = bit >> 1;
        const uint32_t k4 = gram4(j);
        const uint32_t at = nq + prefix_below(m);
        pk[at] = (bit & 1u) ? ((k4 & 0xFFFFFFu) | 0xFF000000u) : k4;
        pp[at] = 16 * g + j - Q.off;
      }
      nq += (uint32_t)__popcll(m);
    }
  };
  // Turns whose every sixteen reads directly: the next turn's loads are issued before this turn's
  // screening, unconditionally (past the direct range they read sixteen 0 and are not used) -- under
  // a branch, the load's join waited for it and the prefetch hid nothing. A full probe queue goes out
  // before the prefetch (loads retire in order: a wait on the probe would wait for the prefetch too).
  if (g0 + 64 <= gdir) {
    uint4 an = ids16[g0 + lane64];
    uint32_t xn = ids32[4 * (g0 + lane64) + 4];
    for (; g0 + 64 <= gdir; g0 += stride) {
      const uint32_t w0 = an.x, w1 = an.y, w2 = an.z, w3 = an.w, w4 = xn;
      if (nq >= 64) drain(false);
      const uint64_t gn = g0 + stride + lane64 < gdir ? g0 + stride + lane64 : 0;
      an = ids16[gn];
      xn = ids32[4 * gn + 4];
      turn(g0 + lane64, w0, w1, w2, w3, w4);
    }
  }
  // the text's last sixteens (no read at or past nsafe)
  for (; g0 < n16; g0 += stride) {
    const uint64_t g = g0 + lane64;
    if (nq >= 64) drain(false);
    turn(g, qg_word(Q, 16 * g), qg_word(Q, 16 * g + 4), qg_word(Q, 16 * g + 8), qg_word(Q, 16 * g + 12),
         qg_word(Q, 16 * g + 16));
  }
  drain(true);
  __syncthreads();
  if (threadIdx.x == 0) Q.rcnt[blockIdx.x] = min(s_cnt, s_fail);
}

// coverage [end - span, end) clipped to the text start wlo, as bitap_kernel (a hit: rare, kept out
// of the verify's unrolled symbol loop)
__device__ __attribute__((noinline)) void qgram_cover(uint32_t* cover, uint64_t wlo, uint64_t span, uint64_t end) {
  const uint64_t ws = end > wlo + span ? end - span : wlo;
  for (uint64_t y = ws; y < end;) {
    const uint64_t w = y >> 5;
    const uint32_t l = (uint32_t)(y & 31);
    const uint32_t cnt = (uint32_t)min((uint64_t)(32 - l), end - y);
    const uint32_t bits = (cnt == 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u)) << l;
    atomicOr(cover + w, bits);
    y += cnt;
  }
}

// W: the automaton word, uint32_t when every q-gram pattern has m <= 32 (half the 64-bit VALU work)
// One candidate (qgram_verify_kernel). LM: every q-gram pattern has m <= 16 and their masks fit in
// LDS (16-bit, pattern-major): the mask reads are LDS reads instead of L2 round trips.
// The text is [wlo, whi) of the view (the whole view, or one stream window of a batch): the
// recurrence starts from its initial state at wlo (prefilter.rs:415-418, a window's text begins
// there) or m + k symbols before the first end it reports, and coverage bits go to `cover`.
template <int KMAX, typename W, bool LM>
__device__ __forceinline__ void verify_one(const QgramParams& Q, unsigned long long cd, uint2 en, const uint8_t* s_aid,
                                           const uint16_t* s_m16, uint64_t wlo, uint64_t whi, uint32_t* cover) {
  const uint64_t t = cd >> 24;
  const uint32_t p = en.x >> 8, o = en.x & 0xFFu, m = en.y & 0xFFu, k = en.y >> 8;
  // ends the candidate allows, 1-based: [t + m - o - k, t + m - o + k], clipped to the text
  const int64_t lo = (int64_t)t + m - o - k, hi = (int64_t)t + m - o + k;
  const uint64_t e_min = (uint64_t)max<int64_t>((int64_t)wlo + 1, lo);
  const uint64_t e_max = (uint64_t)min<int64_t>((int64_t)whi, hi);
  if (e_min > e_max) return;
  const uint64_t warm = (uint64_t)m + k;
  const uint64_t s0 = e_min - 1 > wlo + warm ? e_min - 1 - warm : wlo;
  const uint64_t* mask = Q.pmask + (size_t)p * Q.rows;
  const uint16_t* mask16 = s_m16 + (size_t)p * Q.rows;  // LM: the pattern's masks in LDS
  const W top = (W)1 << (m - 1);
  W r[KMAX + 1];
#pragma unroll
  for (int d = 0; d <= KMAX; ++d) r[d] = d ? (((W)1 << d) - (W)1) : (W)0;  // prefilter.rs:415-418
  // the symbols [s0, e_max) in aligned 4-symbol words, up to 64 per pass, loaded together; their masks
  // 16 at a time (one round trip for the words and one per 16 masks: C5's candidates span ~23
  // symbols, three round trips instead of six); W = uint32_t reads the masks' low halves only
  // (text positions; buffer byte = position + off, both 4-aligned when base is: off % 4 folded in)
  const uint32_t* mask32 = reinterpret_cast<const uint32_t*>(mask);
  const uint32_t sh = Q.off & 3u;
  auto cover_end = [&](uint64_t end) { qgram_cover(cover, wlo, (uint64_t)m + k, end); };
  {
    // Short spans (every C5 candidate: m + 3k + 1 <= 23 symbols): the symbols [s0, e_max) from eight
    // words realigned to s0 (v_alignbyte), stepped exactly -- the general loop below runs whole
    // 16-symbol chunks from the aligned word before s0 (32 steps for C5's ~20; round 5: 941 VALU
    // instructions per candidate)
    const uint64_t ns = e_max - s0;
    const uint64_t wb = (s0 + sh) & ~3ull, bb = wb + (Q.off - sh);
    if (ns <= 28 && bb + 32 <= Q.nsafe) {
      const uint32_t* w32 = reinterpret_cast<const uint32_t*>(Q.ids) + (bb >> 2);
      uint32_t wd[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) wd[u] = w32[u];
      const uint32_t al = (uint32_t)(s0 + sh - wb);
      uint32_t sw[7];
#pragma unroll
      for (uint32_t u = 0; u < 7; ++u) sw[u] = __builtin_amdgcn_alignbyte(wd[u + 1], wd[u], al);
      const uint32_t nsym = (uint32_t)ns, t_end = (uint32_t)(e_min - 1 - s0);
#pragma unroll
      for (uint32_t t = 0; t < 28; ++t) {
        if (t >= nsym) continue;  // (not break: the loop must unroll -- sw is indexed by t)
        uint32_t sym = (sw[t >> 2] >> (8 * (t & 3u))) & 0xFFu;
        if (Q.bytes) sym = s_aid[sym & 0x7Fu];
        const W bc = LM ? (W)mask16[sym] : sizeof(W) == 4 ? (W)mask32[2 * sym] : (W)mask[sym];
        W prev_old = r[0];
        W prev_new = ((r[0] << 1) | (W)1) & bc;
        r[0] = prev_new;
        W hit = (k == 0) ? prev_new : (W)0;
#pragma unroll
        for (int d = 1; d <= KMAX; ++d) {
          const W old = r[d];
          const W nv = ((old << 1) & bc) | ((prev_old | prev_new) << 1) | prev_old | (W)1;
          r[d] = nv;
          prev_old = old;
          prev_new = nv;
          if ((uint32_t)d == k) hit = nv;
        }
        if (t >= t_end && (hit & top)) cover_end(s0 + t + 1);
      }
      return;
    }
  }
  // per pass, 32-bit bounds relative to the pass's first buffer word (u = 16c + v indexes its
  // symbols): symbols u in [u_lo, u_hi) are stepped, ends at u >= u_end report (a pass spans 64
  // symbols, so every bound fits; 64-bit compares per symbol cost as much as the recurrence)
  for (uint64_t base = (s0 + sh) & ~3ull; base < e_max + sh; base += 64) {  // buffer bytes - (off - sh)
    uint32_t wd[16];
    const uint64_t nw = min<uint64_t>(16, (e_max + sh - base + 3) / 4);
    const uint64_t bb = base + (Q.off - sh);  // the buffer byte of word 0 (4-aligned)
    if (bb + 64 <= Q.nsafe) {
      const uint32_t* w32 = reinterpret_cast<const uint32_t*>(Q.ids) + (bb >> 2);
#pragma unroll
      for (uint32_t u = 0; u < 16; ++u) wd[u] = u < nw ? w32[u] : 0u;
    } else {  // the text's end: no read at or past nsafe
      for (uint32_t u = 0; u < 16; ++u) wd[u] = u < nw ? qg_word(Q, bb + 4 * u) : 0u;
    }
    const int32_t u_lo = (int32_t)min<int64_t>((int64_t)(s0 + sh) - (int64_t)base, 64);
    const int32_t u_hi = (int32_t)min<uint64_t>(e_max + sh - base, 64);
    // end (1-based text position) of symbol u: base + u - sh + 1 >= e_min
    const int32_t u_end = (int32_t)max<int64_t>(-1, min<int64_t>((int64_t)(e_min + sh) - (int64_t)base - 1, 64));
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) {
      if ((int32_t)(16 * c) >= u_hi) break;
      W bcs[16];
#pragma unroll
      for (uint32_t v = 0; v < 16; ++v) {
        const int32_t u = (int32_t)(16 * c + v);
        uint32_t sym = (wd[4 * c + v / 4] >> (8 * (v % 4))) & 0xFFu;
        if (Q.bytes) sym = s_aid[sym & 0x7Fu];
        if (u >= u_lo && u < u_hi)
          bcs[v] = LM ? (W)mask16[sym] : sizeof(W) == 4 ? (W)mask32[2 * sym] : (W)mask[sym];
        else bcs[v] = (W)0;
      }
#pragma unroll
      for (uint32_t v = 0; v < 16; ++v) {
        const int32_t u = (int32_t)(16 * c + v);
        if (u >= u_hi) break;
        if (u < u_lo) continue;
        const W bc = bcs[v];
        W prev_old = r[0];
        W prev_new = ((r[0] << 1) | (W)1) & bc;
        r[0] = prev_new;
        W hit = (k == 0) ? prev_new : (W)0;
#pragma unroll
        for (int d = 1; d <= KMAX; ++d) {
          const W old = r[d];
          const W nv = ((old << 1) & bc) | ((prev_old | prev_new) << 1) | prev_old | (W)1;
          r[d] = nv;
          prev_old = old;
          prev_new = nv;
          if ((uint32_t)d == k) hit = nv;
        }
        if (u >= u_end && (hit & top)) cover_end(base + (uint64_t)u - sh + 1);
      }
    }
  }
}

// WIN: a batch of stream windows -- each candidate is verified for the window(s) holding its gram
// position (two in an overlap), with that window's bounds and coverage bitmap
template <int KMAX, typename W, bool LM, bool WIN>
__global__ __launch_bounds__(LM ? 512 : 256) void qgram_verify_kernel(QgramParams Q) {
  __shared__ uint8_t s_aid[128];  // bytes mode: byte -> symbol id
  extern __shared__ uint16_t s_m16[];  // LM: Q.m16_words 32-bit words of 16-bit masks
  if (Q.bytes)
    for (uint32_t i = threadIdx.x; i < 128; i += blockDim.x) s_aid[i] = Q.aid[i];
  if constexpr (LM)
    for (uint32_t i = threadIdx.x; i < Q.m16_words; i += blockDim.x) reinterpret_cast<uint32_t*>(s_m16)[i] = Q.m16[i];
  __syncthreads();
  // persistent: block b takes the scan's regions b, b + grid, ..., then (region nreg) the overflow list.
  // (Loading two candidates and their entries per thread before verifying either measured no faster:
  // 1.37 ms per GiB held to 128 VGPRs, 1.96 at 133 VGPRs, against 1.36; profiles/r05_scan.)
  for (uint32_t r = blockIdx.x; r <= Q.nreg; r += gridDim.x) {
    const unsigned long long* base = r < Q.nreg ? Q.cand + (uint64_t)r * Q.region : Q.ovf;
    const uint64_t cnt = r < Q.nreg ? (uint64_t)Q.rcnt[r] : min((uint64_t)*Q.n_ovf, Q.ovf_cap);
    for (uint64_t x = threadIdx.x; x < cnt; x += blockDim.x) {
      const unsigned long long cd = base[x];
      if constexpr (!WIN) {
        verify_one<KMAX, W, LM>(Q, cd, Q.ent[cd & 0xFFFFFFu], s_aid, s_m16, 0, Q.n, Q.cover);
      } else {
        const uint64_t t = cd >> 24;
        uint32_t w;
        if (Q.wsh) {
          w = (uint32_t)min(t >> Q.wsh, (uint64_t)(Q.nwin - 1));
        } else {
          w = Q.wtab[t >> QG_WSH];
          while (w + 1 < Q.nwin && Q.wlo[w + 1] <= t) ++w;
        }
        const uint2 en = Q.ent[cd & 0xFFFFFFu];
        for (uint32_t d = 0; d < 2; ++d) {  // the window holding t, then its predecessor if they overlap at t
          if (d > w) break;
          const uint32_t ww = w - d;
          const uint64_t lo = Q.wsh ? (uint64_t)ww << Q.wsh : Q.wlo[ww];
          const uint64_t hi = Q.wsh ? min(Q.n, lo + (1ull << Q.wsh) + Q.wov) : Q.whi[ww];
          if (t >= lo && t < hi) verify_one<KMAX, W, LM>(Q, cd, en, s_aid, s_m16, lo, hi, (ww & 1u) ? Q.cover2 : Q.cover);
        }
      }
    }
  }
}

// Maximal runs of set bits -> [start, end) windows (unordered; the host sorts them).
__global__ void runs_kernel(const uint32_t* __restrict__ cover, uint64_t n_words, uint64_t n,
                            unsigned long long* __restrict__ out, unsigned long long* __restrict__ count,
                            uint64_t cap) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n_words) return;
  const uint32_t cur = cover[w];
  const uint32_t prev_hi = w > 0 ? (cover[w - 1] >> 31) : 0u;
  uint32_t starts = cur & ~((cur << 1) | prev_hi);  // bit set, previous bit clear
  while (starts) {
    const uint32_t b = __ffs(starts) - 1;
    starts &= starts - 1;
    const uint64_t s = w * 32 + b;
    if (s >= n) break;
    uint64_t e;  // first clear bit at or after s
    uint64_t ww = w;
    uint32_t bits = cur | (b ? ((1u << b) - 1u) : 0u);
    for (;;) {
      const uint32_t inv = ~bits;
      if (inv) {
        e = ww * 32 + (uint64_t)__builtin_ctz(inv);
        break;
      }
      if (++ww >= n_words) {
        e = n_words * 32;
        break;
      }
      bits = cover[ww];
    }
    if (e > n) e = n;
    const unsigned long long idx = atomicAdd(count, 1ull);
    if (idx < cap) {
      out[2 * idx] = s;
      out[2 * idx + 1] = e;
    }
  }
}

#define HIP_TRY(x)                                          \
  do {                                                      \
    hipError_t _e = (x);                                    \
    if (_e != hipSuccess) {                                 \
      err = std::string(#x) + ": " + hipGetErrorString(_e); \
      return FAC_E_HIP;                                     \
    }                                                       \
  } while (0)

template <typename T>
int upload(const std::vector<T>& v, T** d, std::string& err) {
  *d = nullptr;
  const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
  HIP_TRY(hipMalloc((void**)d, bytes));
  if (!v.empty()) HIP_TRY(hipMemcpy(*d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return FAC_OK;
}

struct Variant {
  uint32_t vcap, qcap;  // vcap 0: no dedup table (unbeamed engines only)
};

// FAC_LDS_PAD (bytes of unused dynamic LDS per workgroup): occupancy experiments only
uint32_t lds_pad() {
  static const uint32_t v = [] {
    const char* e = diag_env("FAC_LDS_PAD");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
  }();
  return v;
}

template <uint32_t Q>
void launch_nd(uint32_t grid, hipStream_t s, const SearchParams& P) {
  if constexpr (Q == 256)
    if (P.beam && !P.has_map) {
      hipLaunchKernelGGL((bfs_window_kernel_live<Q>), dim3(grid), dim3(64), lds_pad(), s, P);
      return;
    }
  if (P.has_map) hipLaunchKernelGGL((bfs_window_kernel_nd<Q, true>), dim3(grid), dim3(64), lds_pad(), s, P);
  else hipLaunchKernelGGL((bfs_window_kernel_nd<Q, false>), dim3(grid), dim3(64), lds_pad(), s, P);
}

template <uint32_t V, uint32_t Q>
void launch_one(uint32_t grid, hipStream_t s, const SearchParams& P) {
  if (P.has_map) hipLaunchKernelGGL((bfs_window_kernel<V, Q, true>), dim3(grid), dim3(64), lds_pad(), s, P);
  else hipLaunchKernelGGL((bfs_window_kernel<V, Q, false>), dim3(grid), dim3(64), lds_pad(), s, P);
}

// LDS per wave: 16 B x (vcap + qcap) + vcap claim bytes
constexpr Variant kVariants[] = {{0, 128},   {0, 256},   {0, 512},     {256, 256},   {512, 256},
                                 {512, 512}, {1024, 1024}, {2048, 2048}, {4096, 4096}, {0, 8192}};

// cache-build ring: at least the root's pushes after the popped root and the main pass's ring
bool launch_rc_build(uint32_t need_q, uint32_t grid, hipStream_t s, const SearchParams& P) {
  if (need_q <= 256) hipLaunchKernelGGL((rc_build_kernel<256>), dim3(grid), dim3(64), 0, s, P);
  else if (need_q <= 512) hipLaunchKernelGGL((rc_build_kernel<512>), dim3(grid), dim3(64), 0, s, P);
  else if (need_q <= 1024) hipLaunchKernelGGL((rc_build_kernel<1024>), dim3(grid), dim3(64), 0, s, P);
  else if (need_q <= 2048) hipLaunchKernelGGL((rc_build_kernel<2048>), dim3(grid), dim3(64), 0, s, P);
  else if (need_q <= 4096) hipLaunchKernelGGL((rc_build_kernel<4096>), dim3(grid), dim3(64), 0, s, P);
  else return false;
  return true;
}

hipError_t launch_variant(const Variant& v, uint32_t grid, hipStream_t s, const SearchParams& P) {
  switch (v.vcap * 16384u + v.qcap) {
    case 0 * 16384u + 128: launch_nd<128>(grid, s, P); break;
    case 0 * 16384u + 256: launch_nd<256>(grid, s, P); break;
    case 0 * 16384u + 512: launch_nd<512>(grid, s, P); break;
    case 256 * 16384u + 256: launch_one<256, 256>(grid, s, P); break;
    case 512 * 16384u + 256: launch_one<512, 256>(grid, s, P); break;
    case 512 * 16384u + 512: launch_one<512, 512>(grid, s, P); break;
    case 1024 * 16384u + 1024: launch_one<1024, 1024>(grid, s, P); break;
    case 2048 * 16384u + 2048: launch_one<2048, 2048>(grid, s, P); break;
    case 4096 * 16384u + 4096: launch_one<4096, 4096>(grid, s, P); break;  // 136 KB LDS: one wave per CU
    default: launch_nd<8192>(grid, s, P); break;                          // 130 KB, dedup-free (unbeamed)
  }
  return hipGetLastError();
}

// first dedup-table size tried for beamed engines (FAC_BEAM_VCAP overrides; 256 / 512 / ...)
uint32_t default_beam_vcap() {
  const char* e = diag_env("FAC_BEAM_VCAP");
  return e ? (uint32_t)std::atoi(e) : 512u;
}

bool debug_poison() {
  static const bool v = [] {
    const char* e = diag_env("FAC_DEBUG_POISON");
    return e && e[0] == '1';
  }();
  return v;
}

// RAII scratch. Plain hipMalloc/hipFree: with the stream-ordered pool (hipMallocAsync /
// hipFreeAsync) on ROCm 7.2 the match counter of a recycled block intermittently came back short
// (reproduced 6/60 calls; 0/60 with hipMalloc), so the pool is not used.
// One pinned, device-mapped host word per host thread (kept for the thread's lifetime): kernels
// store small results there directly, with no copy to queue behind other streams' work.
// a device counter into the pinned host word (a kernel, not a D2H blit: see number_entries)
__global__ void word_kernel(const unsigned long long* src, unsigned int* dst) { *dst = (unsigned int)min(*src, 0xFFFFFFFFull); }

int pinned_word(unsigned int*& host, unsigned int*& dev, std::string& err) {
  thread_local struct Word {  // freed when the thread ends (streaming workers come and go)
    unsigned int* p = nullptr;
    ~Word() {
      if (p) (void)hipHostFree(p);
    }
  } word;
  unsigned int*& h = word.p;
  if (!h) {
    void* p = nullptr;
    const hipError_t e = hipHostMalloc(&p, 64, hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) {
      err = std::string("hipHostMalloc: ") + hipGetErrorString(e);
      return FAC_E_HIP;
    }
    h = static_cast<unsigned int*>(p);
  }
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    err = std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e);
    return FAC_E_HIP;
  }
  host = h;
  dev = static_cast<unsigned int*>(d);
  return FAC_OK;
}

struct DevBuf {
  void* p = nullptr;
  hipStream_t s = nullptr;
  void** slot = nullptr;  // engine scratch slot (kept across calls) or null (owned, freed here)
  size_t* slot_n = nullptr;
  ~DevBuf() { release(); }
  void bind(void** sp, size_t* sn) {
    slot = sp;
    slot_n = sn;
  }
  void release() {
    if (!p) return;
    if (slot) {  // the engine keeps it; the next user orders after us on its own stream
      (void)hipStreamSynchronize(s);
      p = nullptr;
      return;
    }
    (void)hipStreamSynchronize(s);
    (void)hipFree(p);
    p = nullptr;
  }
  hipError_t alloc(size_t bytes, hipStream_t stream) {
    bytes = std::max<size_t>(bytes, 16);
    if (slot) {
      p = nullptr;
      s = stream;
      if (*slot_n < bytes) {
        if (*slot) {
          (void)hipStreamSynchronize(stream);
          (void)hipFree(*slot);
          *slot = nullptr;
          *slot_n = 0;
        }
        const size_t want = bytes + bytes / 4;
        const hipError_t err = hipMalloc(slot, want);
        if (err != hipSuccess) return err;
        *slot_n = want;
      }
      p = *slot;
      return hipSuccess;
    }
    release();
    s = stream;
    return hipMalloc(&p, bytes);
  }
};

// Stream-ordered call scratch (call_scratch_take / give, pooled per thread and size class): the
// pre-filter's per-call buffers -- hipMalloc + hipFree of C5's 0.5 GB candidate list and 134 MB
// coverage bitmap per stream window stalled the device ~0.5 ms a window
struct PoolBuf {
  void* p = nullptr;
  hipStream_t s = nullptr;
  ~PoolBuf() {
    if (p) call_scratch_give(p, s);
  }
  hipError_t alloc(size_t bytes, hipStream_t stream) {
    if (p) call_scratch_give(p, s);
    s = stream;
    hipError_t e = hipSuccess;
    p = call_scratch_take(std::max<size_t>(bytes, 16), stream, &e);
    return e;
  }
};

struct Events {
  hipEvent_t a = nullptr, b = nullptr;
  ~Events() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
  }
};

thread_local ScratchSet* t_scratch = nullptr;  // scratch_bind

}  // namespace

void scratch_bind(ScratchSet* s) { t_scratch = s; }

void scratch_free(ScratchSet& s) {
  if (s.aux) {
    call_scratch_release_stream(s.aux);
    (void)hipStreamDestroy(s.aux);
    s.aux = nullptr;
  }
  for (int i = 0; i < ScratchSet::kSlots; ++i)
    if (s.p[i]) {
      (void)hipFree(s.p[i]);
      s.p[i] = nullptr;
      s.n[i] = 0;
    }
}

int aux_priority() {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return 0;
  return diag_env("FAC_L1_HIGH") ? greatest : least;
}

int upload_engine(Engine& e, std::string& err) {
  HIP_TRY(hipSetDevice(e.device));
  if (!e.stream) HIP_TRY(hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking));
  if (!e.aux_stream) HIP_TRY(hipStreamCreateWithPriority(&e.aux_stream, hipStreamNonBlocking, aux_priority()));
  int rc;
  if ((rc = upload(e.dnodes, &e.d_nodes, err))) return rc;
  if ((rc = upload(e.out_range, &e.d_out_range, err))) return rc;
  if ((rc = upload(e.node_pidx, &e.d_pidx, err))) return rc;
  if ((rc = upload(e.edges, &e.d_edges, err))) return rc;
  if ((rc = upload(e.out_pat, &e.d_out_pat, err))) return rc;
  if ((rc = upload(e.sb_edge, &e.d_sb_edge, err))) return rc;
  if ((rc = upload(e.gt, &e.d_gt, err))) return rc;
  if ((rc = upload(e.aux, &e.d_aux, err))) return rc;
  if ((rc = upload(e.pat_bytes, &e.d_pat_bytes, err))) return rc;
  if ((rc = upload(e.pats, &e.d_pats, err))) return rc;
  if ((rc = upload(e.sim_ascii, &e.d_sim_ascii, err))) return rc;
  if ((rc = upload(e.sim_keys, &e.d_sim_keys, err))) return rc;
  if ((rc = upload(e.sim_vals, &e.d_sim_vals, err))) return rc;
  if (e.has_map) {
    if ((rc = upload(e.edge_gid, &e.d_edge_gid, err))) return rc;
    std::vector<uint32_t> ag(e.ascii_gid, e.ascii_gid + 128);
    if ((rc = upload(ag, &e.d_ascii_gid, err))) return rc;
    if ((rc = upload(e.map_range, &e.d_map_range, err))) return rc;
    if ((rc = upload(e.map_ent, &e.d_map_ent, err))) return rc;
    if ((rc = upload(e.map_hay, &e.d_map_hay, err))) return rc;
  }
  if (e.bitap_ok) {
    // the packed masks depend on the per-call edit budgets: prefilter_windows builds them
    std::vector<uint8_t> aid(e.ascii_id, e.ascii_id + 128);
    if ((rc = upload(aid, &e.d_ascii_id, err))) return rc;
  }
  // Pageable hipMemcpy may return before the DMA lands and the engine's stream is non-blocking:
  // make the tables visible to every stream before the first launch.
  HIP_TRY(hipDeviceSynchronize());
  return FAC_OK;
}

void free_engine_device(Engine& e) {
  if (e.d_nodes == nullptr && e.stream == nullptr) return;
  (void)hipSetDevice(e.device);
  void* ptrs[] = {e.d_nodes, e.d_out_range, e.d_pidx, e.d_edges, e.d_out_pat, e.d_sb_edge, e.d_gt, e.d_aux, e.d_pat_bytes, e.d_pats, e.d_sim_ascii, e.d_sim_keys,
                  e.d_sim_vals, e.d_ascii_id, e.d_edge_gid, e.d_ascii_gid, e.d_map_range,
                  e.d_map_ent, e.d_map_hay};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  e.pf_cache.clear();
  for (int i = 0; i < Engine::kScratch; ++i)
    if (e.scratch_p[i]) {
      (void)hipFree(e.scratch_p[i]);
      e.scratch_p[i] = nullptr;
      e.scratch_n[i] = 0;
    }
  if (e.stream) {
    call_scratch_release_stream(e.stream);
    (void)hipStreamDestroy(e.stream);
  }
  e.stream = nullptr;
  if (e.aux_stream) {
    call_scratch_release_stream(e.aux_stream);
    (void)hipStreamDestroy(e.aux_stream);
  }
  e.aux_stream = nullptr;
  e.d_nodes = nullptr;
}

int stage_haystack(const Engine& e, const uint8_t* utf8, uint64_t len, Haystack& h, std::string& err,
                   int force_ascii, hipStream_t stream) {
  h.device = e.device;
  h.len = len;
  // force_ascii -2: the bytes are validated and classified on the device after the upload
  const bool check_on_device = force_ascii == -2;
  h.ascii = check_on_device ? false : force_ascii < 0 ? ascii_only(utf8, len) : force_ascii != 0;
  h.n = h.ascii ? len : 0;
  HIP_TRY(hipSetDevice(e.device));
  // All uploads go through one stream (the engine's, or the caller's) and are synchronized before
  // returning, so kernels on any stream see complete data (pageable copies may otherwise still be
  // in flight).
  hipStream_t st = stream ? stream : e.stream;
  HIP_TRY(hipMalloc((void**)&h.d_utf8, std::max<uint64_t>(len, 16)));
  h.own_utf8 = true;
  if (len) HIP_TRY(hipMemcpyAsync(h.d_utf8, utf8, len, hipMemcpyHostToDevice, st));
  // UTF-8 check / is_ascii, UAX #29 segmentation + folding on the device (stage_kernels.hip)
  if (int rc = stage_device(e, h, st, err, check_on_device ? -2 : h.ascii ? 1 : 0)) return rc;
  if (h.n > grapheme_limit()) return FAC_E_HAYSTACK_TOO_LARGE;
  HIP_TRY(hipStreamSynchronize(st));
  return FAC_OK;
}

int stage_haystack_device(const Engine& e, const uint8_t* d_utf8, uint64_t len, Haystack& h, std::string& err,
                          hipStream_t stream, int mode) {
  HIP_TRY(hipSetDevice(e.device));
  if (h.d_utf8 && h.own_utf8) HIP_TRY(hipFree(h.d_utf8));
  h.device = e.device;
  h.len = len;
  h.d_utf8 = const_cast<uint8_t*>(d_utf8);
  h.own_utf8 = false;
  h.base = 0;
  h.open_end = false;
  h.owned = UINT64_MAX;
  {
    std::lock_guard<std::mutex> lk(h.host_mu);
    h.host_ready = false;
    h.utf8.clear();
    h.starts.clear();
  }
  h.sym_ready = false;
  h.sym.clear();
  if (h.d_gid) HIP_TRY(hipFree(h.d_gid));
  h.d_gid = nullptr;
  h.gid_engine = nullptr;
  hipStream_t st = stream ? stream : e.stream;
  int rc = stage_device(e, h, st, err, mode);
  if (!rc) {
    const hipError_t se = hipStreamSynchronize(st);
    if (se != hipSuccess) {
      err = std::string("hipStreamSynchronize: ") + hipGetErrorString(se);
      rc = FAC_E_HIP;
    }
  }
  if (rc) {  // a failed restage leaves a valid empty haystack (no stale grapheme offsets over new bytes)
    h.failed_n = h.n;  // HaystackTooLarge reports the count
    h.ascii = true;
    h.len = 0;
    h.n = 0;
    h.d_utf8 = nullptr;
  }
  return rc;
}

// Bit-parallel pre-filter transcode of a Unicode haystack (prefilter.rs:262-280): symbol id of
// every folded grapheme, computed on first use (only pre-filtered searches need it).
int ensure_host(const Haystack& h, std::string& err) {
  std::lock_guard<std::mutex> lk(h.host_mu);
  if (h.host_ready) return FAC_OK;
  HIP_TRY(hipSetDevice(h.device));
  h.utf8.resize(h.len);
  if (h.len) HIP_TRY(hipMemcpy(h.utf8.data(), h.d_utf8, h.len, hipMemcpyDeviceToHost));
  if (!h.ascii) {
    h.starts.resize(h.n);
    if (h.n) HIP_TRY(hipMemcpy(h.starts.data(), h.d_off, h.n * 8, hipMemcpyDeviceToHost));
  }
  h.host_ready = true;
  return FAC_OK;
}

void ensure_symbols(const Engine& e, const Haystack& h) {
  if (h.ascii || h.sym_ready) return;
  std::string err;
  if (ensure_host(h, err)) return;
  h.sym.assign(h.n, 0);
  std::u32string g;
  const uint8_t* utf8 = h.utf8.data();
  for (uint64_t i = 0; i < h.n; ++i) {
    const uint64_t b = h.starts[i], en = i + 1 < h.n ? h.starts[i + 1] : h.len;
    fold_grapheme(utf8, b, en, e.case_insensitive, g);
    auto it = std::lower_bound(e.symbol_ids.begin(), e.symbol_ids.end(), std::make_pair(g, 0u));
    if (it != e.symbol_ids.end() && it->first == g) h.sym[i] = (uint8_t)it->second;
  }
  h.sym_ready = true;
}

void free_haystack(Haystack& h) {
  (void)hipSetDevice(h.device);
  if (h.d_utf8 && h.own_utf8) (void)hipFree(h.d_utf8);
  if (h.d_text32) (void)hipFree(h.d_text32);
  if (h.d_off) (void)hipFree(h.d_off);
  if (h.d_gid) (void)hipFree(h.d_gid);
  if (h.d_stage) (void)hipFree(h.d_stage);
  h.d_utf8 = nullptr;
  h.d_text32 = nullptr;
  h.d_off = nullptr;
  h.d_gid = nullptr;
  h.d_stage = nullptr;
  h.off_cap = 0;
  h.stage_cap = 0;
}

// Grapheme ids of a Unicode haystack for an engine with mappings (gs_text compared as whole
// folded graphemes, grapheme.rs:61-63): computed on the host on first use and uploaded.
int ensure_gids(const Engine& e, const Haystack& h, std::string& err) {
  if (h.ascii || (h.d_gid && h.gid_engine == &e)) return FAC_OK;
  if (int hrc = ensure_host(h, err)) return hrc;
  std::vector<uint32_t> gid(h.n, 0);
  std::u32string g;
  const uint8_t* utf8 = h.utf8.data();
  for (uint64_t i = 0; i < h.n; ++i) {
    const uint64_t b = h.starts[i], en = i + 1 < h.n ? h.starts[i + 1] : h.len;
    fold_grapheme(utf8, b, en, e.case_insensitive, g);
    auto it = e.gid_of.find(g);
    if (it != e.gid_of.end()) gid[i] = it->second;
  }
  HIP_TRY(hipSetDevice(h.device));
  if (h.d_gid) HIP_TRY(hipFree(h.d_gid));
  h.d_gid = nullptr;
  HIP_TRY(hipMalloc((void**)&h.d_gid, std::max<size_t>(gid.size() * sizeof(uint32_t), 16)));
  if (!gid.empty()) HIP_TRY(hipMemcpy(h.d_gid, gid.data(), gid.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  h.gid_engine = &e;
  return FAC_OK;
}

// One search over the windows of `segs_in` with a given beam (0 = none). exact_dedup: the dedup
// must be exact (beam, or auto-beam counting); counts (optional): per virtual window (non-empty
// segments concatenated) the number of states pushed, the reference's queue.len().
int launch_pass(const Engine& e, const Haystack& h, const std::vector<SegDesc>& segs_in, float thr,
                hipStream_t stream, uint32_t beam, bool exact_dedup, std::vector<uint32_t>* counts,
                MatchSink& out, fac_stats* stats, std::string& err) {
  const auto t_begin = std::chrono::steady_clock::now();
  auto host_ms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count(); };
  const bool timing = diag_env("FAC_TIMING") != nullptr;  // diagnostics: host wall-clock phases
  HIP_TRY(hipSetDevice(e.device));
  if (!stream) stream = e.stream;
  std::vector<SegDesc> segs;
  std::vector<uint64_t> prefix(1, 0);
  for (const SegDesc& s : segs_in) {
    SegDesc c = s;
    c.w_end = std::min(c.w_end, c.n);
    if (c.w_begin >= c.w_end) continue;
    segs.push_back(c);
    prefix.push_back(prefix.back() + (c.w_end - c.w_begin));
  }
  uint64_t windows = prefix.back();  // (a key part: its own windows, set once they are listed)
  if (windows == 0) return FAC_OK;

  SearchParams P{};
  P.nodes = e.d_nodes;
  P.edges = e.d_edges;
  P.out_pat = e.d_out_pat;
  P.out_range = e.d_out_range;
  P.node_pidx = e.d_pidx;
  P.sb_edge = e.d_sb_edge;
  P.gt = e.d_gt;
  P.gt_mask = e.gt_mask;
  P.gt_seed1 = e.gt_seed1;
  P.gt_seed2 = e.gt_seed2;
  P.gt_fast = (e.gt_fast && !diag_env("FAC_NO_FAST")) ? 1 : 0;  // env: A/B knob
  P.aux = e.d_aux;
  P.pats = e.d_pats;
  P.sim_ascii = e.d_sim_ascii;
  P.sim_keys = e.d_sim_keys;
  P.sim_vals = e.d_sim_vals;
  P.n_sim = (uint32_t)e.sim_keys.size();
  P.utf8 = h.d_utf8;
  P.text32 = h.d_text32;
  P.off = h.d_off;
  P.n_segs = (uint32_t)segs.size();
  P.total_windows = windows;
  P.case_insensitive = e.case_insensitive;
  P.thr = thr;
  P.out_shift = h.base;
  {  // search.rs:486-487, evaluated as two rounded f32 operations like the reference
    volatile float prod = e.nodes[0].prune_lw * thr;
    P.max_penalties = e.nodes[0].prune_len - prod;
  }
  P.p_ins = e.p_ins;
  P.p_del = e.p_del;
  P.p_sub = e.p_sub;
  P.p_swp = e.p_swp;
  P.min_sym = e.min_sym;
  P.mef = e.mef;
  P.has_glim = e.has_limits;
  P.glim = e.limits;
  P.has_pattern_limits = e.has_pattern_limits;
  P.beam = beam;
  P.exact_dedup = exact_dedup ? 1 : 0;
  P.dup_cut = diag_env("FAC_DUP_CUT") ? 1 : 0;
  P.kp_n = h.kparts;
  P.kp_r = h.kpart;
  P.window_skip = e.window_skip;
  P.has_map = e.has_map ? 1 : 0;
  if (e.has_map) {  // multi-character mappings: whole-grapheme ids (ensure_gids for Unicode text)
    const int grc = ensure_gids(e, h, err);
    if (grc) return grc;
    P.edge_gid = e.d_edge_gid;
    P.gid32 = h.d_gid;
    P.ascii_gid = e.d_ascii_gid;
    P.map_range = e.d_map_range;
    P.map_ent = e.d_map_ent;
    P.map_hay = e.d_map_hay;
  }
  std::memcpy(P.first_bits, e.first_bits, sizeof(P.first_bits));
  std::memcpy(P.second_bits, e.second_bits, sizeof(P.second_bits));
  P.chunk = 256;
  P.ecap = 1024;

  int cus = 256;
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e.device));
  // Variant ladder. A variant fits when one state's fan-out always fits the ring: for a beam,
  // after the selection (<= 2 bw pending, search.rs:577-589) plus one non-root state's pushes;
  // without one, only the single-state bound (overflowing windows spill to the next variant).
  const uint64_t fan_root = 3ull + e.max_map + 2ull * (e.nodes.empty() ? 0u : e.nodes[0].edge_end - e.nodes[0].edge_begin);
  const uint64_t fan_nr = 3ull + e.max_map + 2ull * e.max_degree_nonroot;
  auto fits = [&](const Variant& v) {
    if (P.beam) return v.vcap > 0 && fan_root + 1 <= v.qcap && 2ull * P.beam + fan_nr + 1 <= v.qcap;
    return (v.vcap > 0 || !exact_dedup) && fan_root + 1 <= v.qcap && fan_nr + 1 <= v.qcap;
  };
  const size_t nv = sizeof(kVariants) / sizeof(kVariants[0]);
  size_t vi = nv;
  // defaults (measured on MI355X): beamed -> 512-entry table + 256-entry ring
  // (12.8 KB LDS); unbeamed -> no table + 512-entry ring (a 128 ring cuts batches too often)
  for (size_t i = 0; i < nv && vi == nv; ++i)
    if (fits(kVariants[i]) && (P.beam          ? kVariants[i].vcap >= default_beam_vcap()
                               : exact_dedup ? kVariants[i].vcap >= 512 && kVariants[i].qcap >= 512
                                             : kVariants[i].vcap == 0 && kVariants[i].qcap >= 512))
      vi = i;
  for (size_t i = 0; i < nv && vi == nv; ++i)
    if (fits(kVariants[i])) vi = i;
  // Beamed main passes start dedup-free (no table: more windows per CU, no dedup work) and spill the
  // windows whose pending count would pass 2·bw to the dedup variants (run_window).
  // Not for the auto-beam count pass (exact queue.len() per window) or mappings.
  if (P.beam && !counts && !e.has_map && fan_root + 1 <= 256 && fan_nr + 1 <= 256 && !diag_env("FAC_NO_BEAM_BAIL"))
    for (size_t i = 0; i < nv; ++i)
      if (kVariants[i].vcap == 0 && kVariants[i].qcap == 256) vi = i;
  if (const char* fv = diag_env("FAC_VARIANT")) {  // tuning override "vcap,qcap"
    unsigned a = 0, b = 0;
    if (std::sscanf(fv, "%u,%u", &a, &b) == 2)
      for (size_t i = 0; i < nv; ++i)
        if (kVariants[i].vcap == a && kVariants[i].qcap == b && fits(kVariants[i])) vi = i;
  }
  if (vi == nv) {
    err = "beam width too large for the on-chip frontier";
    return FAC_E_UNSUPPORTED;
  }
  auto escalate = [&](size_t cur) {  // next variant for spilled windows
    const uint32_t want_v = std::max<uint32_t>(kVariants[cur].vcap * 2, 512);
    for (size_t i = cur + 1; i < nv; ++i)
      if (fits(kVariants[i]) && kVariants[i].vcap >= want_v && kVariants[i].qcap >= kVariants[cur].qcap) return i;
    // past the largest table: an unbeamed, non-exact engine may still trade the table for a
    // longer ring (dedup never changes unbeamed results)
    for (size_t i = cur + 1; i < nv; ++i)
      if (fits(kVariants[i]) && kVariants[i].vcap == 0 && kVariants[i].qcap > kVariants[cur].qcap) return i;
    return nv;
  };

  DevBuf d_segs, d_prefix, d_out, d_ebuf, d_cnt, d_list, d_spill;
  DevBuf d_rck, d_rcv, d_rcslot, d_rcb, d_rcrep, d_rcs, d_rcc, d_rcn;  // prefix cache, level 1 + pool
  DevBuf d_xk[kRcLevels - 1], d_xv[kRcLevels - 1], d_xslot[kRcLevels - 1], d_xrep[kRcLevels - 1],
      d_xc[kRcLevels - 1];  // prefix cache, sampled levels
  DevBuf d_ct[kRcLevels];  // prefix cache lookup tables ([kRcLevels - 1]: level 0)
  DevBuf d_l0k, d_l0v, d_l0slot, d_l0rep, d_l0c;  // prefix cache, level 0
  DevBuf d_hits, d_hitp;   // per-window lookups of the main pass
  DevBuf d_voff, d_rcnt;   // ... their windows and per-region counts
  DevBuf d_bhits, d_bpops; // prefix cache builds: the representatives' parent snapshots
  DevBuf d_slots, d_bsel;  // wave-slot rings (one per stream), beam-selection scratch
  DevBuf d_dense;          // the start level's dense key bitmaps
  ScratchSet* bound = t_scratch;  // a streaming worker's own set, else the engine's
  std::unique_lock<std::mutex> lease(bound ? bound->mu : e.scratch_mu, std::try_to_lock);
  void** scratch_p = bound ? bound->p : e.scratch_p;
  size_t* scratch_n = bound ? bound->n : e.scratch_n;
  if (lease.owns_lock()) {  // reuse the engine's scratch (no per-call hipMalloc of the 64 MB lists)
    std::vector<DevBuf*> bufs = {&d_segs, &d_prefix, &d_out, &d_ebuf, &d_cnt, &d_list, &d_spill,
                                 &d_rck,  &d_rcv,    &d_rcslot, &d_rcb, &d_rcrep, &d_rcs, &d_rcc, &d_rcn};
    for (int x = 0; x < kRcLevels - 1; ++x)
      for (DevBuf* b : {&d_xk[x], &d_xv[x], &d_xslot[x], &d_xrep[x], &d_xc[x]}) bufs.push_back(b);
    for (int x = 0; x < kRcLevels; ++x) bufs.push_back(&d_ct[x]);
    for (DevBuf* b : {&d_l0k, &d_l0v, &d_l0slot, &d_l0rep, &d_l0c}) bufs.push_back(b);
    bufs.push_back(&d_hits);
    bufs.push_back(&d_hitp);
    bufs.push_back(&d_voff);
    bufs.push_back(&d_rcnt);
    bufs.push_back(&d_slots);
    bufs.push_back(&d_bsel);
    bufs.push_back(&d_bhits);
    bufs.push_back(&d_bpops);
    bufs.push_back(&d_dense);
    static_assert(Engine::kScratch >= 31 + 5 * (kRcLevels - 1) + kRcLevels, "engine scratch slots");
    static_assert(ScratchSet::kSlots >= Engine::kScratch, "stream scratch slots");
    for (size_t i = 0; i < bufs.size(); ++i) bufs[i]->bind(&scratch_p[i], &scratch_n[i]);
  }
  HIP_TRY(d_segs.alloc(segs.size() * sizeof(SegDesc), stream));
  HIP_TRY(d_prefix.alloc(prefix.size() * sizeof(uint64_t), stream));
  if (timing) std::fprintf(stderr, "FAC_TIMING launch_pass setup before the segment upload %.3f ms\n", host_ms());
  HIP_TRY(hipMemcpyAsync(d_segs.p, segs.data(), segs.size() * sizeof(SegDesc), hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(d_prefix.p, prefix.data(), prefix.size() * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
  uint64_t out_cap = std::max<uint64_t>(4096, windows / 64);
  // beamed passes spill every window whose pending count passes 2 bw from the dedup-free first pass
  // (C3: ~5 % of its windows): a list too short re-runs the whole pass
  uint64_t spill_cap = std::max<uint64_t>(4096, windows / (P.beam ? 8 : 32));
  const uint32_t max_grid = (uint32_t)cus * 16;
  HIP_TRY(d_ebuf.alloc((size_t)max_grid * P.ecap * sizeof(uint4), stream));
  HIP_TRY(d_cnt.alloc(N_COUNTERS * sizeof(unsigned long long), stream));
  // wave slots: a ring of max_grid slots per stream a slot-using kernel runs on (this one, the
  // level-1 build's); beamed engines: each slot's beam-selection scratch, sized for 256-state rings
  // at max_grid slots (larger rings get fewer slots, still above their LDS-bound residency)
  HIP_TRY(d_slots.alloc(2 * ((size_t)max_grid + 2) * sizeof(unsigned int), stream));
  const size_t bsel_cap = P.beam ? (size_t)max_grid * bsel_stride(256) : 0;  // uint4
  if (P.beam) HIP_TRY(d_bsel.alloc(bsel_cap * sizeof(uint4), stream));
  P.sel_limit = 16;
  if (const char* sl = diag_env("FAC_SEL_LIMIT")) P.sel_limit = (uint32_t)std::strtoul(sl, nullptr, 10);
  P.beam_canonical = diag_env("FAC_BEAM_CANONICAL") ? 1 : 0;
  // before every bfs_window_body launch: the stream's slot ring reset, the launch's scratch stride
  auto prep_slots = [&](SearchParams& Q, hipStream_t s, uint32_t qcap, bool select) -> int {
    const size_t pool = s == stream ? 0 : 1;
    unsigned int* base = static_cast<unsigned int*>(d_slots.p) + pool * ((size_t)max_grid + 2);
    Q.slot_ring = base;
    Q.slot_ctr = base + max_grid;
    Q.n_slots = max_grid;
    Q.bsel = nullptr;
    Q.bsel_stride = 0;
    if (select && P.beam) {
      Q.bsel = static_cast<uint4*>(d_bsel.p);
      Q.bsel_stride = bsel_stride(qcap);
      Q.n_slots = (uint32_t)std::min<size_t>(max_grid, bsel_cap / Q.bsel_stride);
    }
    hipLaunchKernelGGL(slot_init_kernel, dim3(16), dim3(256), 0, s, Q.slot_ring, Q.slot_ctr, Q.n_slots);
    HIP_TRY(hipGetLastError());
    return FAC_OK;
  };
  HIP_TRY(d_out.alloc(out_cap * sizeof(fac_match), stream));
  HIP_TRY(d_spill.alloc(spill_cap * sizeof(uint64_t), stream));
  DevBuf d_counts;
  P.win_counts = nullptr;
  if (counts) {
    HIP_TRY(d_counts.alloc(windows * sizeof(uint32_t), stream));
    HIP_TRY(hipMemsetAsync(d_counts.p, 0, windows * sizeof(uint32_t), stream));  // skipped windows: 0
    P.win_counts = static_cast<uint32_t*>(d_counts.p);
  }
  Events ev;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  P.segs = static_cast<const SegDesc*>(d_segs.p);
  P.seg_prefix = static_cast<const uint64_t*>(d_prefix.p);
  P.win_list = nullptr;
  P.kp_wlist = nullptr;
  // a key part (Haystack::kparts): its windows listed in ascending order; from here on `windows`
  // counts them (the cache policy, lookups and searches see the part alone)
  PoolBuf d_kpl, d_kpc;
  if (P.kp_n > 1) {
    // masks (kp_mask_kernel), a one-block scan, the total through the pinned word, the list writes
    const uint64_t nb = (windows + KP_CHUNK - 1) / KP_CHUNK;
    const size_t mask_b = nb * (KP_CHUNK / 64) * 8, cnt_b = (nb * 4 + 7) & ~7ull;
    HIP_TRY(d_kpc.alloc(mask_b + cnt_b + nb * 8 + 8, stream));
    auto* masks = static_cast<unsigned long long*>(d_kpc.p);
    auto* bcount = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_kpc.p) + mask_b);
    auto* boff = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(d_kpc.p) + mask_b + cnt_b);
    auto* total = reinterpret_cast<unsigned long long*>(boff + nb);
    unsigned int* w_host = nullptr;
    unsigned int* w_dev = nullptr;
    if (int hrc = pinned_word(w_host, w_dev, err)) return hrc;
    P.total_windows = windows;
    hipLaunchKernelGGL(kp_mask_kernel, dim3((uint32_t)nb), dim3(256), 0, stream, P, masks, bcount);
    hipLaunchKernelGGL(dl_scan_kernel, dim3(1), dim3(1024), 0, stream, bcount, boff, nb, total);
    hipLaunchKernelGGL(word_kernel, dim3(1), dim3(1), 0, stream, total, w_dev);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(stream));
    const uint64_t tot = *reinterpret_cast<volatile unsigned int*>(w_host);
    HIP_TRY(d_kpl.alloc(std::max<uint64_t>(1, tot) * sizeof(uint64_t), stream));
    hipLaunchKernelGGL(dl_write_kernel, dim3((uint32_t)nb), dim3(256), 0, stream, P, masks, boff,
                       static_cast<uint64_t*>(d_kpl.p));
    HIP_TRY(hipGetLastError());
    windows = tot;
    P.total_windows = windows;
    P.kp_wlist = static_cast<const uint64_t*>(d_kpl.p);
    if (windows == 0) return FAC_OK;
  }

  int rc = FAC_OK;
  uint64_t retries = 0, launches = 0, popped = 0, cached_pops = 0, pass_windows = windows;
  unsigned long long cnt[N_COUNTERS] = {};
  float ms_total = 0.f, cache_ms = 0.f, lane_ms = 0.f;
  uint64_t lane_windows = 0, dense_done = 0;
  hipEvent_t ev_lane = nullptr;  // end of the lane-serial kernel (destroyed on return)
  struct EvGuard {
    hipEvent_t& e;
    ~EvGuard() {
      if (e) (void)hipEventDestroy(e);
    }
  } ev_lane_guard{ev_lane};

  // Prefix cache. Level 1: every window's key of K0 chars (4, else 3, else 2,
  // whichever first gives every snapshot at least 8 windows on average); rc_count_kernel inserts
  // the keys, rc_build_kernel searches one representative per key up to the first state that reads
  // past the key. Level 2: keys of K1 (> K0) chars, counted on a sample of the windows; keys seen at
  // least T times get a snapshot built by resuming their representative from its level-1 snapshot.
  // A window resumes from the deepest snapshot its prefix has. Skipped when the root emits (an empty
  // pattern), with mappings (whole-grapheme keys), or when the search is small.
  P.rc_mode = 0;
  P.rc_hits = nullptr;
  P.rc_hit_pops = nullptr;
  P.rc_voff = nullptr;
  P.rc_region_cnt = nullptr;
  P.rc_ntab = 0;
  P.rc_kstart = 0;
  P.live_nqmax = 0;
  P.rc_lane_flush = diag_env("FAC_RC_NO_LANE") ? 0 : 1;
  P.dyn_chunks = diag_env("FAC_STATIC_GRID") ? 0 : 1;
  const bool root_out = !e.nodes.empty() && e.nodes[0].out_end > e.nodes[0].out_begin;
  const char* rc_min = diag_env("FAC_RC_MIN");  // env knobs: tests force it on / pin K, A/B turns it off
  const char* kenv = diag_env("FAC_RC_K");
  std::vector<RcTable> tabs;      // built levels, ascending k: a build resumes its representatives from them
  RcTable L1{0u, 0u, nullptr, nullptr, nullptr, nullptr};
  uint32_t n_ent0 = 0, qbuild = 0;
  uint64_t ct_mult = 4, ct_mult2 = 4;  // lookup slots per entry: levels 0/1 by entries, sampled levels by kept snapshots
  unsigned int* dense_w_host = nullptr;  // the dense bitmaps' sampled share of finished windows
  unsigned int* dense_w_dev = nullptr;
  uint32_t dense_pm = 0;
  bool dense_list = false, dense_built = false;
  // after its build a level's entries are published into an exact-key lookup table (4 slots per
  // entry: a miss usually ends at the first probe)
  auto ct_slots = [&](uint32_t n_ent, uint64_t mult) {
    uint32_t cs = 1u << 12;
    while (cs < mult * n_ent && cs < (1u << 28)) cs <<= 1;
    return cs;
  };
  auto clear_ct = [&](uint32_t n_ent, DevBuf& ct, hipStream_t bs, uint64_t mult = 0) -> int {
    const uint32_t cs = ct_slots(n_ent, mult ? mult : ct_mult);
    HIP_TRY(ct.alloc((size_t)cs * 2 * sizeof(uint4), bs));
    HIP_TRY(hipMemsetAsync(ct.p, 0, (size_t)cs * 2 * sizeof(uint4), bs));
    return FAC_OK;
  };
  // (segments of < 1024 windows on average -- the pre-filter's merged windows -- share too few keys
  // for the cache's counts and builds: C5 212.7 vs 241.5 Gchars/s with it off, round 5 profiles/r05s)
  if (!root_out && !e.has_map && fan_root + 1 <= 4096 && kVariants[vi].qcap <= 4096 &&
      windows >= (rc_min ? std::strtoull(rc_min, nullptr, 10) : 4096ull) &&
      (rc_min || windows >= 1024ull * segs.size()) && !diag_env("FAC_NO_RC")) {
    auto env_u = [](const char* name, uint64_t dflt) {
      const char* v = diag_env(name);
      return v ? std::strtoull(v, nullptr, 10) : dflt;
    };
    const uint32_t kpin = kenv ? (uint32_t)std::min<unsigned long>(4, std::max<unsigned long>(2, std::strtoul(kenv, nullptr, 10))) : 0u;
    const uint32_t qmain = kVariants[vi].qcap, vmain = kVariants[vi].vcap;
    qbuild = std::max<uint32_t>((uint32_t)fan_root + 1, qmain);
    P.rc_vmax = vmain ? std::min<uint32_t>(256, vmain / 2) : 256;
    P.rc_emax = 64;
    // entries per level: fresh-word C3 selects more than 16 M 5-char keys (32 M: 448.7 -> 445.8 ms per
    // step, the vocabulary C3 unchanged, profiles/r04t)
    const uint64_t ent_cap = std::max<uint64_t>(1, env_u("FAC_RC_ENTRIES", 32ull << 20));
    const uint32_t max_ent = (uint32_t)std::min<uint64_t>(windows, ent_cap);
    // count tables: level-1 keys are few (one per distinct k-gram), so the table stays cache-sized
    const uint32_t cprobes = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(RC_PROBES, env_u("FAC_RC_CPROBES", RC_PROBES)));
    const uint32_t l1_log2 = (uint32_t)std::min<uint64_t>(24, std::max<uint64_t>(12, env_u("FAC_RC_SLOTS1", 24)));
    uint32_t slots = 1u << 12;
    while (slots < 4ull * max_ent && slots < (1u << l1_log2)) slots <<= 1;
    HIP_TRY(d_rck.alloc(slots * sizeof(unsigned long long), stream));
    HIP_TRY(d_rcv.alloc(slots * sizeof(uint32_t), stream));  // entries by slot
    HIP_TRY(d_rcslot.alloc(slots * sizeof(uint64_t), stream));
    HIP_TRY(d_rcb.alloc(8192 * sizeof(uint32_t), stream));
    HIP_TRY(d_rcrep.alloc(max_ent * sizeof(uint64_t), stream));
    HIP_TRY(d_rcc.alloc(2 * (size_t)max_ent * sizeof(uint32_t), stream));  // counts, then offsets
    HIP_TRY(d_rcn.alloc(4 * sizeof(unsigned long long), stream));  // keys, pool words used, level-2 entries
    L1 = RcTable{0u, slots - 1, static_cast<const unsigned long long*>(d_rck.p), static_cast<const uint32_t*>(d_rcv.p),
                 static_cast<uint32_t*>(d_rcc.p) + max_ent, static_cast<uint32_t*>(d_rcc.p)};
    P.rc_pool_used = static_cast<unsigned long long*>(d_rcn.p) + 1;
    HIP_TRY(hipEventRecord(ev.a, stream));
    HIP_TRY(hipMemsetAsync(d_rcn.p, 0, 4 * sizeof(unsigned long long), stream));
    const uint32_t cgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((windows + 255) / 256, (uint64_t)cus * env_u("FAC_RC_CGRID", 8)));

    // keys counted >= thr -> entries 0..n-1 (val by slot), reps by entry;
    // returns n (all selected keys; entries past max_ent stay uncached)
    auto number_entries = [&](const DevBuf& keys, const DevBuf& cv, const DevBuf& rslot, const DevBuf& rep,
                              uint32_t n_slots, uint32_t thr, uint32_t cap, unsigned int& n) -> int {
      const uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(8192, n_slots / 4096));
      const uint32_t range = (n_slots + nb - 1) / nb;  // n_slots and nb are powers of two: a multiple of 256
      // the count comes back through pinned host memory written by the scan kernel: a 4-byte D2H copy
      // is a blit workgroup that queued 9 ms behind the level-1 build's waves on the second stream
      unsigned int* n_host = nullptr;
      unsigned int* n_dev = nullptr;
      if (int hrc = pinned_word(n_host, n_dev, err)) return hrc;
      *reinterpret_cast<volatile unsigned int*>(n_host) = 0u;
      // single-wave workgroups throughout (see rc_sel_scan_kernel)
      hipLaunchKernelGGL(rc_sel_count_kernel, dim3(nb), dim3(64), 0, stream,
                         static_cast<const unsigned long long*>(keys.p), n_slots, range, thr, static_cast<uint32_t*>(d_rcb.p));
      hipLaunchKernelGGL(rc_sel_scan_kernel, dim3(1), dim3(64), 0, stream, static_cast<uint32_t*>(d_rcb.p), nb, n_dev);
      hipLaunchKernelGGL(rc_sel_assign_kernel, dim3(nb), dim3(64), 0, stream,
                         static_cast<const unsigned long long*>(keys.p), static_cast<const uint64_t*>(rslot.p),
                         static_cast<uint32_t*>(cv.p),
                         static_cast<uint64_t*>(rep.p), static_cast<const uint32_t*>(d_rcb.p), n_slots, range, thr, cap);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipStreamSynchronize(stream));
      n = *reinterpret_cast<volatile unsigned int*>(n_host);
      return FAC_OK;
    };
    uint32_t n_ent1 = 0;
    uint64_t l1_keys = 0;
    // Level 0: keys one char shorter than level 1's, every window, built from the root; the level-1
    // build then resumes its representatives from them and pops only the last key char's states
    // (the root pop, its beam and the first chars' states are shared by every level-1 key). Counted
    // in the level-1 pass; used when level 1 keeps its first key length.
    RcTable L0{0u, 0u, nullptr, nullptr, nullptr, nullptr};
    n_ent0 = 0;
    const bool want_l0 = !diag_env("FAC_NO_RC_L0");
    auto target = [](const DevBuf& keys, const DevBuf& rep, uint32_t n_slots, uint32_t k) {
      return RcCountTarget{static_cast<unsigned long long*>(keys.p), static_cast<uint64_t*>(rep.p), n_slots - 1, k};
    };
    // Level-1 keys are counted on every stride1-th window, about 32 M windows in all (a power of two,
    // at most 16): a key that only unsampled windows hold stays uncached, and its windows resume from
    // level 0 (the prefixes of the sampled keys; the lookups reach it last) or from the root. Measured
    // per step against counting every window: C3 (stride 4; 0.3 M windows fall back) 92.4 -> 89.8 ms,
    // C2 1 GiB (stride 16) 105.5 -> 88.7 ms; strides 8 / 16 on C3 gave 90.0 / 93.3 ms.
    uint32_t stride1 = 1;
    while (stride1 < 16 && windows / (2ull * stride1) >= (1ull << 25)) stride1 *= 2;
    stride1 = (uint32_t)std::max<uint64_t>(1, env_u("FAC_RC_STRIDE1", stride1));
    for (uint32_t k = kpin ? kpin : 4u; k >= (kpin ? kpin : 2u); --k) {
      P.rc_k = k;
      HIP_TRY(hipMemsetAsync(d_rck.p, 0, slots * sizeof(unsigned long long), stream));
      const uint32_t k0 = std::max<uint64_t>(2, std::min<uint64_t>(k - 1, env_u("FAC_RC_L0K", k - 1)));  // knob: A/B
      const bool l0 = want_l0 && k >= 3 && L0.k == 0;  // the first key length only
      RcCountTarget t1{nullptr, nullptr, 0u, 0u};
      if (l0) {
        HIP_TRY(d_l0k.alloc(slots * sizeof(unsigned long long), stream));
        HIP_TRY(d_l0v.alloc(slots * sizeof(uint32_t), stream));
        HIP_TRY(d_l0slot.alloc(slots * sizeof(uint64_t), stream));
        HIP_TRY(hipMemsetAsync(d_l0k.p, 0, slots * sizeof(unsigned long long), stream));
        t1 = target(d_l0k, d_l0slot, slots, k0);
        L0.k = k0;
      }
      hipLaunchKernelGGL(rc_count_kernel, dim3(cgrid), dim3(256), 0, stream, P, target(d_rck, d_rcslot, slots, k),
                         RcCountTarget{nullptr, nullptr, 0u, 0u}, RcCountTarget{nullptr, nullptr, 0u, 0u},
                         stride1, 1u, cprobes);
      HIP_TRY(hipGetLastError());
      unsigned int n_keys = 0;
      if (int nrc = number_entries(d_rck, d_rcv, d_rcslot, d_rcrep, slots, 1u, max_ent, n_keys)) return nrc;
      l1_keys = n_keys;
      if (n_keys == 0) break;
      if (!kpin && 8ull * n_keys > (windows + stride1 - 1) / stride1) continue;  // too little reuse: fewer chars per key
      n_ent1 = std::min(n_keys, max_ent);
      L1.k = k;
      // lookups start at the first sampled level (rc_lookup); FAC_RC_DEEPEST (A/B): a start no level
      // reaches, so st stays at the deepest level and the shallower ones follow deepest first
      P.rc_kstart = diag_env("FAC_RC_DEEPEST") ? 0xFFFFFFFFu : k + 1;
      if (l0) {  // level-0 keys from the level-1 representatives
        hipLaunchKernelGGL(rc_derive_kernel, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n_ent1 + 255) / 256, cus * 8))), dim3(256),
                           0, stream, P, static_cast<const uint64_t*>(d_rcrep.p), n_ent1, t1, cprobes);
        HIP_TRY(hipGetLastError());
        const uint32_t max_ent0 = std::min<uint32_t>(n_ent1, max_ent);
        HIP_TRY(d_l0rep.alloc(max_ent0 * sizeof(uint64_t), stream));
        HIP_TRY(d_l0c.alloc(2 * (size_t)max_ent0 * sizeof(uint32_t), stream));
        unsigned int n0 = 0;
        if (int nrc = number_entries(d_l0k, d_l0v, d_l0slot, d_l0rep, slots, 1u, max_ent0, n0)) return nrc;
        n_ent0 = std::min(n0, max_ent0);
        L0 = RcTable{k0, slots - 1, static_cast<const unsigned long long*>(d_l0k.p),
                     static_cast<const uint32_t*>(d_l0v.p), static_cast<uint32_t*>(d_l0c.p) + max_ent0,
                     static_cast<uint32_t*>(d_l0c.p)};
      }
      break;
    }
    if (!n_ent0) L0.k = 0;
    // sampled levels: frequent long prefixes, ascending key lengths (FAC_RC_LEVELS, e.g. "6" or
    // "5,7"; FAC_RC_K2 = k pins one level, 0 turns them off)
    std::vector<uint32_t> ks;
    if (const char* k2e = diag_env("FAC_RC_K2")) {
      const uint32_t k2 = (uint32_t)std::strtoul(k2e, nullptr, 10);
      if (k2) ks.push_back(std::min<uint32_t>(8, k2));
    } else {
      const char* le = diag_env("FAC_RC_LEVELS");
      // with the lane-serial kernel an 8-char level no longer pays (C3 156 -> 147 ms); one-edit
      // engines finish most windows within 5 chars, and a 6-char level costs them more in counts
      // and lookup probes than it saves (C2 1 GiB: 266 -> 188 ms per step with "5" alone)
      // beamed engines (the reference's select_nth_unstable_by order): 5 and 7 chars, built exactly
      // (measured C3: "5,6" 257.7, "5,7" with keys seen >= 4 times 214.9 ms per step; after the
      // selects became calls, "5,7" / "5,6,7" at >= 2 sightings 151.8 / 151.1; profiles/r03/sweep_levels.txt;
      // at the final round-3 kernels "5,6,7" 147.1-147.8 against "5,7" 149.0-149.7 over five runs each,
      // profiles/r03ah, r03ai)
      std::string spec = le ? le : (e.mef <= 1u ? "5" : P.beam ? "5,6,7" : "5,6");
      for (size_t a = 0; a < spec.size();) {
        const size_t b = spec.find(',', a);
        const uint32_t k = (uint32_t)std::strtoul(spec.substr(a, b == std::string::npos ? std::string::npos : b - a).c_str(), nullptr, 10);
        if (k && (ks.empty() || k > ks.back()) && k <= 8 && ks.size() < (size_t)kRcLevels - 2) ks.push_back(k);
        if (b == std::string::npos) break;
        a = b + 1;
      }
    }
    // Snapshot pool and the level-1 build go first: the level-1 build runs on the engine's second
    // stream while the sampled levels are counted on this one (the counts only need level 1's k).
    // The pool is sized for every key the levels could select (up to the budget); a build that runs
    // out of pool leaves the remaining keys uncached.
    const uint64_t samples_est = windows >= env_u("FAC_RC_MIN2", 1ull << 20) ? (windows + std::max<uint64_t>(1, env_u("FAC_RC_STRIDE2", 2)) - 1) / std::max<uint64_t>(1, env_u("FAC_RC_STRIDE2", 2)) : 0;
    const uint64_t max_ent2_est = std::min<uint64_t>(samples_est, ent_cap);
    const uint64_t worst = RC_HDR + std::min(qmain, qbuild) + P.rc_vmax + P.rc_emax;
    hipStream_t bstream = stream;  // the level-1 build's stream
    hipEvent_t l1_done = nullptr;
    struct EvDel {
      hipEvent_t& e;
      ~EvDel() {
        if (e) (void)hipEventDestroy(e);
      }
    } l1_done_guard{l1_done};
    // (Dedup-free "live" builds of the sampled levels -- every key whose build would beam left
    // uncached, inexact snapshots -- lost to the exact builds with the reference's beam order: C3 537
    // vs 258 ms per step; removed in round 5, git history keeps them.)
    // 4 slots per entry, the sampled levels' per kept snapshot (C3: 5.9 M of 8.2 M 5-char entries kept).
    // 2 per entry cost C2 76.0 vs 71.0 ms (profiles/r04ab); 4 for the sampled levels: C2 71.1 vs 73.5,
    // C4 16.45 vs 17.39, C3 135.9 vs 136.8 against 2 (profiles/r04ac)
    ct_mult = std::max<uint64_t>(1, std::min<uint64_t>(8, env_u("FAC_RC_CT_MULT", 4)));
    ct_mult2 = std::max<uint64_t>(1, std::min<uint64_t>(8, env_u("FAC_RC_CT_MULT2", 4)));
    auto build = [&](const RcTable& T, uint32_t n_ent, const uint64_t* reps, hipStream_t bs, bool cleared = false) -> int {
      SearchParams Q = P;
      Q.rc_mode = 2;
      Q.rc_k = T.k;
      Q.rc_ntab = 0;
      for (size_t t = tabs.size(); t-- > 0 && T.k > tabs[t].k;)  // levels below T, deepest first
        Q.rc_tab[Q.rc_ntab++] = tabs[t];
      Q.rc_off = const_cast<uint32_t*>(T.off);
      Q.rc_count = const_cast<uint32_t*>(T.count);
      Q.rc_keep_final = (n_ent0 && T.k == L1.k) ? 1 : 0;  // main lookups skip level 0
      Q.win_list = reps;
      Q.total_windows = n_ent;
      // list chunks of up to 64 representatives: their parent lookups go out together
      Q.chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(64, n_ent / (4ull * max_grid)));
      Q.win_counts = nullptr;
      Q.ebuf = static_cast<uint4*>(d_ebuf.p);
      Q.out = static_cast<fac_match*>(d_out.p);
      Q.out_cap = out_cap;
      Q.spill = static_cast<uint64_t*>(d_spill.p);
      Q.spill_cap = spill_cap;
      Q.counters = static_cast<unsigned long long*>(d_cnt.p);
      if (!cleared) HIP_TRY(hipMemsetAsync(Q.counters, 0, N_COUNTERS * sizeof(unsigned long long), bs));
      uint32_t grid = std::min<uint32_t>(n_ent, max_grid);
      if (bs != stream && !diag_env("FAC_L1_PERSIST")) {
        // beside the sampled-level counts: one chunk per workgroup, so workgroup slots free up all
        // along the build and the counts (higher-priority stream) are not held back to its end
        Q.dyn_chunks = 0;
        grid = (uint32_t)std::min<uint64_t>((n_ent + Q.chunk - 1) / Q.chunk, 0x7FFFFFFFull);
      }
      Q.rc_bhits = nullptr;
      Q.rc_bpops = nullptr;
      if (Q.rc_ntab > 0) {  // the representatives' parent snapshots (rc_parent_kernel)
        // (each level allocates: the slot keeps the largest, and a level's build is ordered after the
        // previous one's on this stream or waits for it through l1_done)
        HIP_TRY(d_bhits.alloc((size_t)n_ent * sizeof(uint4), bs));
        HIP_TRY(d_bpops.alloc((size_t)n_ent * sizeof(uint32_t), bs));
        Q.rc_bhits = static_cast<uint4*>(d_bhits.p);
        Q.rc_bpops = static_cast<uint32_t*>(d_bpops.p);
        uint32_t qk0 = 256;
        while (qk0 < qbuild) qk0 <<= 1;
        hipLaunchKernelGGL(rc_parent_kernel, dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n_ent + 255) / 256, (uint64_t)cus * 8))),
                           dim3(256), 0, bs, Q, qk0);
        HIP_TRY(hipGetLastError());
      }
      uint32_t qk = 256;  // launch_rc_build's ring
      while (qk < qbuild) qk <<= 1;
      if (int src = prep_slots(Q, bs, qk, true)) return src;
      launch_rc_build(qbuild, grid, bs, Q);
      const hipError_t le = hipGetLastError();
      if (le != hipSuccess) {
        err = std::string("kernel launch: ") + hipGetErrorString(le);
        return FAC_E_HIP;
      }
      return FAC_OK;
    };
    // n_size: the entries the table is sized for (the snapshots the build kept, when known)
    auto publish = [&](RcTable& T, uint32_t n_ent, const uint64_t* reps, DevBuf& ct, hipStream_t bs,
                       bool cleared = false, uint32_t n_size = 0xFFFFFFFFu, uint64_t mult = 0) -> int {
      if (n_size == 0xFFFFFFFFu) n_size = n_ent;
      if (!mult) mult = ct_mult;
      const uint32_t cs = ct_slots(n_size, mult);
      if (!cleared) {
        if (int crc = clear_ct(n_size, ct, bs, mult)) return crc;
      }
      hipLaunchKernelGGL(rc_publish_kernel, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n_ent + 255) / 256, cus * 8))),
                         dim3(256), 0, bs, P, reps, static_cast<const uint4*>(P.rc_pool), T.off, T.count, n_ent, T.k,
                         static_cast<uint4*>(ct.p), cs - 1);
      HIP_TRY(hipGetLastError());
      T.ct = static_cast<const uint4*>(ct.p);
      T.ct_mask = cs - 1;
      return FAC_OK;
    };
    if (n_ent1) {
      const uint64_t n_all = n_ent0 + n_ent1 + (uint64_t)ks.size() * max_ent2_est;
      const uint64_t budget = env_u("FAC_RC_POOL_MB", 16384ull) << 20;
      // per-wave pool chunks: about a quarter of the expected pool (~40 words a snapshot) spread over
      // the building waves, at least one worst snapshot; + one partly used chunk per wave and level
      const uint64_t grids = std::min<uint64_t>(n_ent0, max_grid) + std::min<uint64_t>(n_ent1, max_grid) +
                             (uint64_t)ks.size() * std::min<uint64_t>(max_ent2_est, max_grid);
      P.rc_pool_chunk = (uint32_t)std::max<uint64_t>(worst, std::min<uint64_t>(RC_POOL_CHUNK, n_all * 40 / (4 * grids)));
      const uint64_t pool_words = std::max<uint64_t>(1024, std::min<uint64_t>(n_all * worst, budget / sizeof(uint4))) +
                                  grids * P.rc_pool_chunk;
      HIP_TRY(d_rcs.alloc(pool_words * sizeof(uint4), stream));
      P.rc_pool = static_cast<uint4*>(d_rcs.p);
      P.rc_pool_cap = pool_words;
      if (!diag_env("FAC_RC_ONE_STREAM")) {
        // the lowest priority: the sampled-level counts beside it come first. A streaming worker's
        // scratch set has its own (only that worker's thread uses it), so two windows in flight do
        // not queue their builds behind each other; the engine's is created with its tables.
        if (bound && !bound->aux) HIP_TRY(hipStreamCreateWithPriority(&bound->aux, hipStreamNonBlocking, aux_priority()));
        HIP_TRY(hipEventCreateWithFlags(&l1_done, hipEventDisableTiming));
        bstream = bound ? bound->aux : e.aux_stream;
      }
    }
    // launched once the sampled levels' count tables are cleared (a fill queued behind the build's
    // persistent waves would hold the counts back)
    bool l1_launched = false;
    auto launch_l1 = [&]() -> int {
      if (l1_launched || !n_ent1) return FAC_OK;
      l1_launched = true;
      // the build's counters are cleared here: a fill queued on the second stream behind the
      // sampled-level count kernel's workgroups started the build 2.6 ms late
      HIP_TRY(hipMemsetAsync(d_cnt.p, 0, N_COUNTERS * sizeof(unsigned long long), stream));
      if (int crc = clear_ct(n_ent1, d_ct[0], stream)) return crc;  // likewise the lookup table
      if (n_ent0) {  // level 0 first (same stream), the level-1 build resumes from it
        HIP_TRY(hipMemsetAsync(d_cnt.p, 0, N_COUNTERS * sizeof(unsigned long long), stream));
        if (int crc = clear_ct(n_ent0, d_ct[kRcLevels - 1], stream)) return crc;
      }
      if (bstream != stream) {
        HIP_TRY(hipEventRecord(l1_done, stream));  // everything so far (counts, pool, clears) first
        HIP_TRY(hipStreamWaitEvent(bstream, l1_done, 0));
      }
      if (n_ent0) {
        int brc = build(L0, n_ent0, static_cast<const uint64_t*>(d_l0rep.p), bstream, true);
        if (brc) return brc;
        if ((brc = publish(L0, n_ent0, static_cast<const uint64_t*>(d_l0rep.p), d_ct[kRcLevels - 1], bstream, true))) return brc;
        tabs.push_back(L0);
        HIP_TRY(hipMemsetAsync(d_cnt.p, 0, N_COUNTERS * sizeof(unsigned long long), bstream));
      }
      int brc = build(L1, n_ent1, static_cast<const uint64_t*>(d_rcrep.p), bstream, true);
      if (brc) return brc;
      if ((brc = publish(L1, n_ent1, static_cast<const uint64_t*>(d_rcrep.p), d_ct[0], bstream, true))) return brc;
      if (bstream != stream) HIP_TRY(hipEventRecord(l1_done, bstream));
      tabs.push_back(L1);
      return FAC_OK;
    };
    // Sampled levels: every 2nd window's key, kept when seen twice. With a single sampled level
    // (one-edit engines, whose windows mostly end within 5 chars) about 8-32 M windows are sampled
    // (stride a power of two, at most 32: C2's 1 G windows still sample 32 M) and every sampled key
    // is kept; keys numbered past the entry budget (ent_cap, 16 M) stay uncached, which is exact: C2 1 GiB 88.8 -> 71.0 ms,
    // C4 18.9 -> 17.6 ms per step with the same lane / wave work (the keys that matter are frequent);
    // C4 at stride 16 (8 M samples) against 4 (32 M): 17.7 -> 16.6 ms, C2 at stride 64: no change.
    // Two levels (C3) stay at 2 / 2: strides 3 / 4 or threshold 1 measured slower.
    uint32_t s2 = 2;
    if (ks.size() == 1)
      while (s2 < 32 && windows / (2ull * s2) >= (1ull << 23)) s2 *= 2;
    const uint32_t stride2 = (uint32_t)std::max<uint64_t>(1, env_u("FAC_RC_STRIDE2", s2));
    // the sampled levels' counts run beside the level-0/1 builds and have slack until the level-1
    // build ends: fewer workgroups leave the builds more of the CUs. Measured: two sampled levels
    // (C3) 2 per CU (-2 ms against 8), one level (C2, whose builds are shorter) 4 per CU (-2 ms)
    const uint32_t cgrid2 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((windows + 255) / 256,
        (uint64_t)cus * env_u("FAC_RC_CGRID2", ks.size() >= 2 ? 2 : 4)));
    // (beamed engines: keys seen >= 4 times while the selects were inlined into the window loop and
    // the builds spilled registers; >= 2 since: C3 162.0 -> 151.8 ms, profiles/r03/sweep_levels.txt)
    // (keys seen >= 3 times measured slower once the small build variant made the builds cheaper:
    // the lane and wave kernels took more than the builds saved, profiles/r04k)
    const uint32_t thr2 = (uint32_t)std::min<uint64_t>(RC_CSAT, std::max<uint64_t>(1, env_u("FAC_RC_T2", s2 > 2 ? 1 : 2)));
    std::vector<RcTable> Lx;        // sampled levels, ascending k
    std::vector<uint32_t> n_entx;   // their entries
    std::vector<size_t> xbuf;       // their count-table buffers
    if (n_ent1 && windows >= env_u("FAC_RC_MIN2", 1ull << 20)) {
      const uint64_t samples = (windows + stride2 - 1) / stride2;
      const uint32_t l2_log2 = (uint32_t)std::min<uint64_t>(27, std::max<uint64_t>(12, env_u("FAC_RC_SLOTS2", 27)));
      uint32_t slots2 = 1u << 12;
      while (slots2 < 2ull * samples && slots2 < (1u << l2_log2)) slots2 <<= 1;
      const uint32_t thr_t = thr2;
      const uint32_t max_ent2 = (uint32_t)std::min<uint64_t>(samples, ent_cap);
      std::vector<uint32_t> kk;  // the levels to count; buffers x = position in kk
      for (uint32_t k2 : ks)
        if (k2 > L1.k) kk.push_back(k2);
      for (size_t x = 0; x < kk.size(); ++x) {  // every level's tables cleared before the level-1 build
        HIP_TRY(d_xk[x].alloc(slots2 * sizeof(unsigned long long), stream));
        HIP_TRY(d_xv[x].alloc(slots2 * sizeof(uint32_t), stream));  // entries by slot
        HIP_TRY(d_xslot[x].alloc(slots2 * sizeof(uint64_t), stream));
        HIP_TRY(d_xrep[x].alloc(max_ent2 * sizeof(uint64_t), stream));
        HIP_TRY(d_xc[x].alloc(2 * (size_t)max_ent2 * sizeof(uint32_t), stream));
        HIP_TRY(hipMemsetAsync(d_xk[x].p, 0, slots2 * sizeof(unsigned long long), stream));
      }
      if (int lrc = launch_l1()) return lrc;
      for (size_t x = 0; x < kk.size(); ++x) {
        const uint32_t k2 = kk[x];
        // levels are counted three per pass over the sampled windows: with three levels in two passes
        // the second pass ran after the first one's numbering and held the sampled builds back behind
        // the level-1 build (C3, r03aj)
        if (x % 3 == 0) {
          const RcCountTarget none{nullptr, nullptr, 0u, 0u};
          const RcCountTarget t1 = x + 1 < kk.size() ? target(d_xk[x + 1], d_xslot[x + 1], slots2, kk[x + 1]) : none;
          const RcCountTarget t2 = x + 2 < kk.size() ? target(d_xk[x + 2], d_xslot[x + 2], slots2, kk[x + 2]) : none;
          hipLaunchKernelGGL(rc_count_kernel, dim3(cgrid2), dim3(256), 0, stream, P,
                             target(d_xk[x], d_xslot[x], slots2, k2), t1, t2, stride2, thr_t, cprobes);
          HIP_TRY(hipGetLastError());
        }
        unsigned int nk2 = 0;
        if (int nrc = number_entries(d_xk[x], d_xv[x], d_xslot[x], d_xrep[x], slots2, thr_t, max_ent2, nk2)) return nrc;
        const uint32_t ne = std::min(nk2, max_ent2);
        if (ne == 0) continue;
        Lx.push_back(RcTable{k2, slots2 - 1, static_cast<const unsigned long long*>(d_xk[x].p),
                             static_cast<const uint32_t*>(d_xv[x].p), static_cast<uint32_t*>(d_xc[x].p) + max_ent2,
                             static_cast<uint32_t*>(d_xc[x].p)});
        n_entx.push_back(ne);
        xbuf.push_back(x);
      }
    }
    if (int lrc = launch_l1()) return lrc;  // no sampled levels
    if (n_ent1) {
      if (bstream != stream) HIP_TRY(hipStreamWaitEvent(stream, l1_done, 0));  // level 1 built and published
      for (size_t x = 0; x < Lx.size(); ++x) {
        int brc = build(Lx[x], n_entx[x], static_cast<const uint64_t*>(d_xrep[xbuf[x]].p), stream, false);
        if (brc) return brc;
        // the lookup table is sized for the snapshots the build kept (C3: 5.9 M of 8.2 M 5-char entries,
        // 0.6 M of 5.8 M 7-char ones), read back through the pinned word: tables 4x smaller to clear
        // and to probe
        uint32_t kept = n_entx[x];
        if (!diag_env("FAC_RC_CT_ENTRIES")) {
          unsigned int* w_host = nullptr;
          unsigned int* w_dev = nullptr;
          if (int hrc = pinned_word(w_host, w_dev, err)) return hrc;
          hipLaunchKernelGGL(word_kernel, dim3(1), dim3(1), 0, stream, static_cast<const unsigned long long*>(d_cnt.p) + 11, w_dev);
          HIP_TRY(hipGetLastError());
          HIP_TRY(hipStreamSynchronize(stream));
          const uint32_t got = *reinterpret_cast<volatile unsigned int*>(w_host);
          kept = std::min<uint32_t>(kept, got);
        }
        if ((brc = publish(Lx[x], n_entx[x], static_cast<const uint64_t*>(d_xrep[xbuf[x]].p), d_ct[1 + x], stream, false,
                           kept, ct_mult2))) return brc;
        // the first sampled level is where the main lookups start (P.rc_kstart = level 1's k + 1)
        if (x == 0 && P.rc_kstart == L1.k + 1 && !P.win_counts && P.rc_lane_flush && !diag_env("FAC_RC_NO_DENSE")) {
          HIP_TRY(d_dense.alloc(RC_DENSE_WORDS * sizeof(uint32_t), stream));
          HIP_TRY(hipMemsetAsync(d_dense.p, 0, RC_DENSE_WORDS * sizeof(uint32_t), stream));
          uint32_t* dn = static_cast<uint32_t*>(d_dense.p);
          const uint64_t* reps = static_cast<const uint64_t*>(d_xrep[xbuf[x]].p);
          const dim3 dg(std::max<uint32_t>(1, std::min<uint32_t>((n_entx[x] + 255) / 256, cus * 4)));
          hipLaunchKernelGGL(rc_dense_hist_kernel, dg, dim3(256), 0, stream, P, reps, static_cast<const uint4*>(P.rc_pool),
                             Lx[x].off, Lx[x].count, n_entx[x], Lx[x].k, dn);
          const bool f4 = n_ent1 && L1.k < Lx[x].k && !diag_env("FAC_RC_NO_DENSE4");
          hipLaunchKernelGGL(rc_dense_rank_kernel, dim3(1), dim3(128), 0, stream, Lx[x].k, f4 ? L1.k : 0u,
                             (uint32_t)env_u("FAC_RC_DENSE_KEYS", 50), dn);
          hipLaunchKernelGGL(rc_dense_fill_kernel, dg, dim3(256), 0, stream, P, reps, static_cast<const uint4*>(P.rc_pool),
                             Lx[x].off, Lx[x].count, n_entx[x], Lx[x].k, dn, RC_DENSE_F, RC_DENSE_C);
          if (f4)  // level 1 (built and published: the stream waited for it above)
            hipLaunchKernelGGL(rc_dense_fill_kernel, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n_ent1 + 255) / 256, cus * 4))),
                               dim3(256), 0, stream, P, static_cast<const uint64_t*>(d_rcrep.p),
                               static_cast<const uint4*>(P.rc_pool), L1.off, L1.count, n_ent1, L1.k, dn, RC_DENSE_F4, 0u);
          HIP_TRY(hipGetLastError());
          P.rc_dense = dn;
          dense_built = true;
        }
        tabs.push_back(Lx[x]);
      }
      if (P.rc_dense) {  // the share of windows the dense bitmaps finish, read after the sync below
        if (int hrc = pinned_word(dense_w_host, dense_w_dev, err)) return hrc;
        hipLaunchKernelGGL(rc_dense_sample_kernel, dim3(64), dim3(256), 0, stream, P, windows);
        hipLaunchKernelGGL(word_kernel, dim3(1), dim3(1), 0, stream,
                           reinterpret_cast<const unsigned long long*>(P.rc_dense + 34), dense_w_dev);
        HIP_TRY(hipGetLastError());
      }
      // the lookups probe deepest first and stop at the first hit: level 0 is reached only by the
      // windows whose level-1 key the sampled count missed
      P.rc_ntab = 0;
      for (size_t t = tabs.size(); t-- > 0;) P.rc_tab[P.rc_ntab++] = tabs[t];
      P.rc_mode = 1;
    }
    HIP_TRY(hipEventRecord(ev.b, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    HIP_TRY(hipEventElapsedTime(&cache_ms, ev.a, ev.b));
    if (P.rc_dense) {
      // F-done windows among 16384 sampled: below FAC_RC_DENSE_OFF per mille the bitmaps are dropped
      // (their test costs the lookup more than it saves), from FAC_RC_DENSE_LIST per mille the lookups
      // walk the list of the others (dl_*_kernel)
      dense_pm = (uint32_t)((uint64_t)*reinterpret_cast<volatile unsigned int*>(dense_w_host) * 1000 / 16384);
      const uint32_t off_pm = (uint32_t)env_u("FAC_RC_DENSE_OFF", 50), list_pm = (uint32_t)env_u("FAC_RC_DENSE_LIST", 250);
      if (dense_pm < off_pm) P.rc_dense = nullptr;
      dense_list = dense_pm >= list_pm;
    }
    if (P.rc_mode == 1 && diag_env("FAC_RC_DEBUG")) {  // diagnostics: keys, pool use, cached entries
      unsigned long long rcn[2] = {0, 0};
      HIP_TRY(hipMemcpy(rcn, d_rcn.p, sizeof(rcn), hipMemcpyDeviceToHost));
      auto cached_of = [&](const RcTable& T, uint32_t ne, uint64_t& qsum) -> uint64_t {
        std::vector<uint32_t> cntv(ne);
        if (ne && hipMemcpy(cntv.data(), T.count, ne * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) return 0;
        uint64_t c = 0;
        for (uint32_t v : cntv)
          if (v != EMPTY) ++c, qsum += v;
        return c;
      };
      uint64_t q1 = 0;
      const uint64_t c1 = cached_of(L1, n_ent1, q1);
      std::string lv;
      for (size_t x = 0; x < Lx.size(); ++x) {
        uint64_t q = 0;
        const uint64_t c = cached_of(Lx[x], n_entx[x], q);
        char b[160];
        std::snprintf(b, sizeof(b), " | k=%u entries=%u cached=%llu mean_queue=%.1f", Lx[x].k, n_entx[x],
                      (unsigned long long)c, c ? (double)q / c : 0.0);
        lv += b;
      }
      {
        unsigned long long gb[8];
        HIP_TRY(hipMemcpyFromSymbol(gb, HIP_SYMBOL(g_bad), sizeof(gb)));
        std::fprintf(stderr, "FAC_RC uncached keys: queue %llu visited %llu emit %llu best %llu vmax %llu\n", gb[0], gb[1],
                     gb[2], gb[3], gb[4]);
        std::memset(gb, 0, sizeof(gb));
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_bad), gb, sizeof(gb)));
      }
      uint64_t q0 = 0;
      const uint64_t c0 = n_ent0 ? cached_of(L0, n_ent0, q0) : 0;
      std::fprintf(stderr, "FAC_RC windows=%llu L0 k=%u entries=%u cached=%llu mean_queue=%.1f | L1 k=%u keys=%llu cached=%llu "
                   "mean_queue=%.1f%s | pool %.1f MB\n",
                   (unsigned long long)windows, L0.k, n_ent0, (unsigned long long)c0, c0 ? (double)q0 / c0 : 0.0, L1.k,
                   (unsigned long long)l1_keys, (unsigned long long)c1, c1 ? (double)q1 / c1 : 0.0, lv.c_str(),
                   rcn[1] * 16.0 / 1e6);
    }
  }
  const double t_cache = host_ms();
  double t_dev = 0.0;
  // Main-pass chunk behind the prefix cache. Unbeamed windows left after the lookups and the lane
  // kernel are few and cheap, and a wave's turn costs a hand-out atomic plus the group prescan, so
  // chunks grow to 16 turns per wave (up to 4096 windows; C2 1 GiB: wave kernel 51 -> 4.5 ms).
  // Beamed searches keep 256: their remaining windows are heavy and balance matters more (C3: 256
  // -> 2048 costs 0.7 ms).
  // lane-serial kernel over the open entries (P.total_windows of them, in regions)
  auto launch_lane = [&]() -> int {
    // one wave per workgroup; each takes its best lists from its own emit-scratch slice
    const uint32_t lgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((windows + LANE_CHUNK - 1) / LANE_CHUNK, (uint64_t)max_grid));
    static_assert(16 * 64 <= 1024, "lane best lists must fit the emit scratch slice (P.ecap >= 1024)");
    // 12-state rings by default: 10 KB of LDS, so 16 waves per CU instead of 12 with 16 states, and the
    // windows that need 13-16 states (the ones that held a wave longest) go to the dedup-free pass.
    // C3: lane 13.6 -> 7.1 ms, wave 41.0 -> 45.0 ms (133.5 vs 135.7 per step); fresh words 447.5 vs
    // 442.4 (profiles/r04ab/r04ag.txt). Round 2: 16 states against 8, lane 19 + wave 37 ms vs 6 + 58.
    // (The 8-, 16- and 32-state variants were removed in round 5; git history keeps them.)
    hipLaunchKernelGGL((lane_window_kernel<12, 8>), dim3(lgrid), dim3(64), 0, stream, P);
    HIP_TRY(hipGetLastError());
    return FAC_OK;
  };
  auto lane_debug_line = [&](float lms) -> int {
    if (!diag_env("FAC_RC_DEBUG")) return FAC_OK;
    unsigned long long d[8];
    HIP_TRY(hipMemcpyFromSymbol(d, HIP_SYMBOL(g_lane_dbg), sizeof(d)));
    std::fprintf(stderr, "FAC_LANE taken=%llu finished=%llu bailed=%llu ms=%.3f popmax=%u trips=%llu run_cycles=%llu "
                 "wave_cycles=%llu rounds=%llu\n", d[0], d[1], d[2], lms, P.lane_popmax, d[4], d[5], d[6], d[7]);
    std::memset(d, 0, sizeof(d));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_lane_dbg), d, sizeof(d)));
    return FAC_OK;
  };
  // Few windows (the pre-filter's merged windows, small slices): chunks shrink until every wave slot
  // gets two, down to one window -- 256-window chunks left C5's re-search of ~20 K windows per GiB to
  // ~70 waves, 3.2 ms per stream window (round 5, profiles/r05b)
  const uint64_t base_chunk = std::min<uint64_t>(256, std::max<uint64_t>(1, pass_windows / (2ull * max_grid)));
  const uint64_t rc_auto = P.beam ? base_chunk
                                  : std::min<uint64_t>(4096, std::max<uint64_t>(base_chunk, pass_windows / (16ull * max_grid)));
  const uint32_t rc_chunk = (uint32_t)std::min<unsigned long>(4096, std::max<unsigned long>(1,
      diag_env("FAC_RC_CHUNK") ? std::strtoul(diag_env("FAC_RC_CHUNK"), nullptr, 10) : rc_auto));
  PoolBuf d_dl, d_dlm;     // the windows the dense bitmaps leave open (dl_*_kernel) and their masks
  bool kp_listed = false;  // the main pass walks the key part's window list (no prefix cache)
  if (P.rc_mode == 0 && P.kp_wlist) {
    P.win_list = P.kp_wlist;
    kp_listed = true;
  }
  for (;;) {
    if (pass_windows == 0) break;
    // spilled windows are few and heavy: one per block turn; behind the prefix-cache lookups most
    // windows are done, so chunks are larger (fewer hand-out atomics; the group prescan skips them)
    P.chunk = kp_listed ? (uint32_t)base_chunk : P.win_list ? 1u : (P.rc_mode == 1 ? rc_chunk : (uint32_t)base_chunk);
    P.total_windows = pass_windows;
    const uint64_t want = (pass_windows + P.chunk - 1) / P.chunk;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, max_grid));
    P.ebuf = static_cast<uint4*>(d_ebuf.p);
    P.out = static_cast<fac_match*>(d_out.p);
    P.out_cap = out_cap;
    P.spill = static_cast<uint64_t*>(d_spill.p);
    P.spill_cap = spill_cap;
    P.counters = static_cast<unsigned long long*>(d_cnt.p);
    HIP_TRY(hipMemsetAsync(d_cnt.p, 0, N_COUNTERS * sizeof(unsigned long long), stream));
    if (debug_poison()) HIP_TRY(hipMemsetAsync(d_out.p, 0xAB, out_cap * sizeof(fac_match), stream));
    if (P.rc_mode == 1 && !P.win_list) {  // every window's lookup (+ flush of finished windows) first
      uint64_t lk_windows = pass_windows;
      if (P.rc_dense && dense_list && !diag_env("FAC_RC_NO_DENSE_LIST")) {  // the windows bit F leaves open, listed
        const uint64_t nb = (lk_windows + KP_CHUNK - 1) / KP_CHUNK;
        const size_t mask_b = nb * (KP_CHUNK / 64) * 8, cnt_b = (nb * 4 + 7) & ~7ull;
        HIP_TRY(d_dlm.alloc(mask_b + cnt_b + nb * 8 + 8, stream));
        auto* masks = static_cast<unsigned long long*>(d_dlm.p);
        auto* bcount = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_dlm.p) + mask_b);
        auto* boff = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(d_dlm.p) + mask_b + cnt_b);
        unsigned int* w_host = nullptr;
        unsigned int* w_dev = nullptr;
        if (int hrc = pinned_word(w_host, w_dev, err)) return hrc;
        P.total_windows = lk_windows;
        hipLaunchKernelGGL(dl_mask_kernel, dim3((uint32_t)nb), dim3(256), 0, stream, P, masks, bcount);
        auto* total = reinterpret_cast<unsigned long long*>(boff + nb);
        hipLaunchKernelGGL(dl_scan_kernel, dim3(1), dim3(1024), 0, stream, bcount, boff, nb, total);
        hipLaunchKernelGGL(word_kernel, dim3(1), dim3(1), 0, stream, total, w_dev);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(stream));
        const uint64_t listed = *reinterpret_cast<volatile unsigned int*>(w_host);
        HIP_TRY(d_dl.alloc(std::max<uint64_t>(1, listed) * sizeof(uint64_t), stream));
        hipLaunchKernelGGL(dl_write_kernel, dim3((uint32_t)nb), dim3(256), 0, stream, P, masks, boff,
                           static_cast<uint64_t*>(d_dl.p));
        HIP_TRY(hipGetLastError());
        P.kp_wlist = static_cast<const uint64_t*>(d_dl.p);
        lk_windows = listed;
        dense_done += pass_windows - listed;
      }
      // the open windows' hits, compacted per region (entries: n_reg * RC_REGION at most)
      const uint64_t n_reg = std::max<uint64_t>(1, (lk_windows + RC_REGION - 1) / RC_REGION);
      P.total_windows = lk_windows;
      HIP_TRY(d_hits.alloc(n_reg * RC_REGION * sizeof(uint4), stream));
      HIP_TRY(d_hitp.alloc(n_reg * RC_REGION * sizeof(uint32_t), stream));
      HIP_TRY(d_voff.alloc(n_reg * RC_REGION * sizeof(uint32_t), stream));
      HIP_TRY(d_rcnt.alloc(n_reg * sizeof(uint32_t), stream));
      P.rc_hits = static_cast<uint4*>(d_hits.p);
      P.rc_hit_pops = static_cast<uint32_t*>(d_hitp.p);
      P.rc_voff = static_cast<uint32_t*>(d_voff.p);
      P.rc_region_cnt = static_cast<uint32_t*>(d_rcnt.p);
      P.rc_qcap = kVariants[vi].qcap;
      HIP_TRY(hipEventRecord(ev.a, stream));
      P.lane_debug = diag_env("FAC_RC_DEBUG") ? 1 : 0;
      // one region per wave turn, up to 32 waves per CU (7 fit: SGPR-bound)
      hipLaunchKernelGGL(rc_lookup_kernel, dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n_reg + 3) / 4, (uint64_t)cus * 8))),
                         dim3(256), 0, stream, P);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipEventRecord(ev.b, stream));
      P.total_windows = n_reg * RC_REGION;  // the searches run over entries
      // small unfinished windows: one lane each (lane_window_kernel); the rest stay for the wave kernel
      const bool lane_on = !diag_env("FAC_NO_LANE") && !P.win_counts && !P.has_map;  // beamed: exact_dedup is set, bail-outs keep it exact
      if (lane_on) {
        if (!ev_lane) HIP_TRY(hipEventCreate(&ev_lane));
        P.lane_debug = diag_env("FAC_RC_DEBUG") ? 1 : 0;
        P.lane_popmax = (uint32_t)std::max<unsigned long>(1, diag_env("FAC_LANE_POPS") ? std::strtoul(diag_env("FAC_LANE_POPS"), nullptr, 10) : 32ul);
        P.live_nqmax = diag_env("FAC_LIVE_NQMAX") ? (uint32_t)std::strtoul(diag_env("FAC_LIVE_NQMAX"), nullptr, 10) : 0u;
        if (int lrc = launch_lane()) return lrc;
        HIP_TRY(hipEventRecord(ev_lane, stream));
      }
      HIP_TRY(hipEventSynchronize(lane_on ? ev_lane : ev.b));
      float lms = 0.f;
      HIP_TRY(hipEventElapsedTime(&lms, ev.a, ev.b));
      cache_ms += lms;
      if (P.lane_debug) {
        unsigned long long d[16];
        HIP_TRY(hipMemcpyFromSymbol(d, HIP_SYMBOL(g_lk_dbg), sizeof(d)));
        std::string lv;
        for (uint32_t t = 0; t < P.rc_ntab; ++t) {
          char b[96];
          std::snprintf(b, sizeof(b), " k=%u: open %llu final %llu |", P.rc_tab[t].k, d[2 * t], d[2 * t + 1]);
          lv += b;
        }
        uint32_t dk[2] = {0, 0};  // the start level's cached keys: ASCII and final without records, all
        if (dense_built) HIP_TRY(hipMemcpy(dk, static_cast<uint32_t*>(d_dense.p) + 36, sizeof(dk), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "FAC_LK%s miss %llu skipped %llu dense-final %llu unlisted %llu (sampled %u per mille; keys %u of %u)\n",
                     lv.c_str(), d[12], d[13], d[14], (unsigned long long)dense_done, dense_pm, dk[0], dk[1]);
        std::memset(d, 0, sizeof(d));
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_lk_dbg), d, sizeof(d)));
      }
      if (lane_on) {
        HIP_TRY(hipEventElapsedTime(&lms, ev.b, ev_lane));
        lane_ms += lms;
        if (int drc = lane_debug_line(lms)) return drc;
      }
    }
    if (int src = prep_slots(P, stream, kVariants[vi].qcap, kVariants[vi].vcap > 0)) {
      rc = src;
      break;
    }
    HIP_TRY(hipEventRecord(ev.a, stream));
    const hipError_t le = launch_variant(kVariants[vi], grid, stream, P);
    if (le != hipSuccess) {
      err = std::string("kernel launch: ") + hipGetErrorString(le);
      rc = FAC_E_HIP;
      break;
    }
    HIP_TRY(hipEventRecord(ev.b, stream));
    HIP_TRY(hipMemcpyAsync(cnt, d_cnt.p, N_COUNTERS * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    ms_total += ms;
    launches += 1;
    popped += cnt[1];
    cached_pops += cnt[4];
    lane_windows += cnt[8];
    if (diag_env("FAC_RC_DEBUG") && P.rc_mode == 1)
    {
      std::fprintf(stderr, "FAC_RC launch windows=%llu resumed=%llu lane_flushed=%llu lane_searched=%llu popped=%llu\n",
                   (unsigned long long)pass_windows, cnt[5], cnt[6], cnt[8], cnt[1]);
      unsigned long long d[12];
      HIP_TRY(hipMemcpyFromSymbol(d, HIP_SYMBOL(g_live_dbg), sizeof(d)));
      std::fprintf(stderr, "FAC_LIVE lane checks=%llu hits=%llu | wave checks=%llu hits=%llu windows with/without live entries=%llu/%llu"
                   " | spills=%llu spill_pops=%llu spill_snapq=%llu spill_pushed=%llu spill_ring_intact=%llu\n",
                   d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], d[10]);
      std::memset(d, 0, sizeof(d));
      HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_live_dbg), d, sizeof(d)));
    }
#ifdef FAC_WIN_HIST
    {
      unsigned long long h[24];
      HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_hist), sizeof(h)));
      for (int b = 0; b < 6; ++b)
        std::fprintf(stderr, "FAC_HIST variant=%u,%u bucket=%d windows=%llu pops=%llu cycles=%llu resumed=%llu\n",
                     kVariants[vi].vcap, kVariants[vi].qcap, b, h[b], h[6 + b], h[12 + b], h[18 + b]);
      std::memset(h, 0, sizeof(h));
      HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_hist), h, sizeof(h)));
    }
#endif
#ifdef FAC_PHASE_PROF
    {
      unsigned long long pr[2 * kProf];
      HIP_TRY(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_prof), sizeof(pr)));
      for (int m = 0; m < 2; ++m) {
        const unsigned long long* q = pr + kProf * m;
        std::fprintf(stderr, "FAC_PROF %s variant=%u,%u beam_select=%llu phaseA=%llu wide=%llu phaseB=%llu phaseC=%llu "
                     "emit=%llu push=%llu window_total=%llu batches=%llu [B: prep=%llu units=%llu finish=%llu] "
                     "states: per-edge=%llu fast=%llu committed=%llu loaded=%llu Bc<=4:%llu <=16:%llu <=40:%llu >40:%llu "
                     "main_popped=%llu prologue=%llu flush=%llu build_epilogue=%llu group_setup=%llu wave_life=%llu "
                     "cuts: beam=%llu ring=%llu key_end=%llu dup=%llu wide=%llu dup_lanes=%llu full_batches=%llu "
                     "epilogue: scan=%llu pool=%llu queue=%llu dedup=%llu tail=%llu prologue: clear=%llu load=%llu\n",
                     m ? "builds" : "main", kVariants[vi].vcap, kVariants[vi].qcap, q[0], q[1], q[2], q[3], q[4], q[5],
                     q[6], q[7], q[8], q[9], q[10], q[11], q[12], q[13], q[14], q[15], q[16], q[17], q[18], q[19], cnt[1],
                     q[20], q[21], q[22], q[23], q[24], q[25], q[26], q[27], q[28], q[29], q[30], q[31],
                     q[32], q[33], q[34], q[35], q[36], q[37], q[38]);
      }
      std::memset(pr, 0, sizeof(pr));
      HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), pr, sizeof(pr)));
    }
#endif
    const unsigned flags = (unsigned)cnt[2];
    if (flags & ERR_HALO) {
      err = "haystack shard does not hold the halo its windows need";
      rc = FAC_E_INVALID;
      break;
    }
    // buffer growth: the whole pass is re-run (its counters were reset)
    if (flags & ERR_EMIT) {
      if (P.ecap < (1u << 20)) {
        P.ecap *= 8;
        HIP_TRY(d_ebuf.alloc((size_t)max_grid * P.ecap * sizeof(uint4), stream));
        ++retries;
        continue;
      }
      err = "per-window match list exceeded capacity";
      rc = FAC_E_CAPACITY;
      break;
    }
    if ((flags & ERR_SPILL) || cnt[3] > spill_cap) {
      spill_cap = std::max<uint64_t>(cnt[3], spill_cap * 2);
      HIP_TRY(d_spill.alloc(spill_cap * sizeof(uint64_t), stream));
      ++retries;
      continue;
    }
    if (cnt[0] > out_cap) {
      out_cap = cnt[0];
      HIP_TRY(d_out.alloc(out_cap * sizeof(fac_match), stream));
      ++retries;
      continue;
    }
    t_dev = host_ms();
    if (cnt[0]) {
      const int arc = sink_append_device(out, static_cast<const fac_match*>(d_out.p), cnt[0], stream, err);
      if (arc) return arc;
    }
    HIP_TRY(hipStreamSynchronize(stream));
    if (cnt[3] == 0) break;
    // windows that overflowed this variant's frontier: re-run just those on the next one
    const size_t nx = escalate(vi);
    if (nx == nv) {
      err = "per-window frontier exceeded the on-chip capacity";
      rc = FAC_E_CAPACITY;
      break;
    }
    vi = nx;
    pass_windows = cnt[3];
    std::swap(d_list.p, d_spill.p);
    std::swap(d_list.s, d_spill.s);
    std::swap(d_list.slot, d_spill.slot);
    std::swap(d_list.slot_n, d_spill.slot_n);
    if (!d_spill.p || spill_cap < pass_windows) {
      HIP_TRY(d_spill.alloc(std::max<uint64_t>(spill_cap, pass_windows) * sizeof(uint64_t), stream));
      spill_cap = std::max<uint64_t>(spill_cap, pass_windows);
    }
    P.win_list = static_cast<const uint64_t*>(d_list.p);
    kp_listed = false;
    ++retries;
  }
  if (timing)
    std::fprintf(stderr, "FAC_TIMING setup+cache %.2f ms, search %.2f ms, records D2H %.2f ms (host wall clock)\n", t_cache,
                 t_dev - t_cache, host_ms() - t_dev);
  if (counts && rc == FAC_OK) {
    counts->resize(windows);
    HIP_TRY(hipMemcpyAsync(counts->data(), d_counts.p, windows * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
  }
  if (stats) {
    stats->kernel_ms += ms_total;
    stats->kernel_launches += launches;
    stats->cache_ms += cache_ms;
    stats->states_cached += cached_pops;
    stats->lane_ms += lane_ms;
    stats->lane_windows += lane_windows;
    stats->windows += windows;
    stats->states_popped += popped;
    stats->graphemes = h.n;
    stats->bytes = h.len;
    stats->retries += retries;
  }
  return rc;
}

// search_unsorted_impl for a list of (sub)haystacks (search.rs:418-1119). With auto_beam and no
// explicit beam (search.rs:1096-1103) the beam switches on after the first window at which the
// running total of queue.len() exceeds the budget; the total runs per search_raw call, i.e. per
// segment (the pre-filter re-searches every merged window with its own call). Two passes
// reproduce it exactly: pass 1 searches every window unbeamed with exact dedup and records each
// window's queue.len(); per segment the switch window w* is the first whose running total exceeds
// the budget; pass-1 matches of windows <= w* are kept and the windows after w* are re-searched
// with the auto-beam width.
int launch_search_sink(const Engine& e, const Haystack& h, const std::vector<SegDesc>& segs_in, float thr,
                       hipStream_t stream, uint64_t ab_prefix, MatchSink& out, fac_stats* stats, std::string& err) {
  const uint32_t beam = (uint32_t)std::min<uint64_t>(e.beam_width, 0xFFFFFFFFull);
  if (!(e.has_auto_beam && e.beam_width == 0))
    return launch_pass(e, h, segs_in, thr, stream, beam, beam != 0, nullptr, out, stats, err);
  const uint32_t ab_beam = (uint32_t)std::min<uint64_t>(e.ab_width, 0xFFFFFFFFull);
  // a shard whose earlier shards already crossed the budget is beamed from its first window
  if (ab_prefix > e.ab_budget) return launch_pass(e, h, segs_in, thr, stream, ab_beam, true, nullptr, out, stats, err);
  std::vector<SegDesc> segs;
  for (const SegDesc& s : segs_in) {
    SegDesc c = s;
    c.w_end = std::min(c.w_end, c.n);
    if (c.w_begin < c.w_end) segs.push_back(c);
  }
  std::vector<uint32_t> counts;
  std::vector<fac_match> pass1;
  MatchSink s1;
  s1.vec = &pass1;
  int rc = launch_pass(e, h, segs, thr, stream, 0, true, &counts, s1, stats, err);
  if (rc) return rc;
  std::vector<SegDesc> tails;          // windows after each segment's switch window
  std::vector<std::pair<uint64_t, uint64_t>> keep;  // per segment: [byte_base, cut byte) of pass 1
  if (!h.ascii)
    if (int hrc = ensure_host(h, err)) return hrc;
  uint64_t v = 0;
  for (const SegDesc& c : segs) {
    uint64_t total = ab_prefix, cut_w = c.w_end;  // first window searched with the beam
    for (uint64_t w = c.w_begin; w < c.w_end; ++w, ++v) {
      total += counts[v];
      if (cut_w == c.w_end && total > e.ab_budget) cut_w = w + 1;
    }
    const uint64_t cut_local = cut_w >= c.n ? c.hay_len
                               : c.ascii    ? cut_w
                                            : h.starts[c.text_base + cut_w] - c.byte_base;
    keep.push_back({c.byte_base, c.byte_base + cut_local});
    if (cut_w < c.w_end) {
      SegDesc t = c;
      t.w_begin = cut_w;
      tails.push_back(t);
    }
  }
  // segments cover disjoint byte ranges: attribute each pass-1 match by its start byte (records
  // carry the shard's global shift h.base)
  std::vector<size_t> order(segs.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return segs[a].byte_base < segs[b].byte_base; });
  std::vector<fac_match> kept;
  for (const fac_match& m : pass1) {
    const uint64_t st = m.start - h.base;
    size_t lo = 0, hi = order.size();
    while (hi - lo > 1) {
      const size_t mid = (lo + hi) / 2;
      if (segs[order[mid]].byte_base <= st) lo = mid;
      else hi = mid;
    }
    const auto& k = keep[order[lo]];
    if (st >= k.first && st < k.second) kept.push_back(m);
  }
  if ((rc = sink_append_host(out, kept.data(), kept.size(), stream, err))) return rc;
  if (tails.empty()) return FAC_OK;
  return launch_pass(e, h, tails, thr, stream, ab_beam, true, nullptr, out, stats, err);
}

int launch_search(const Engine& e, const Haystack& h, const std::vector<SegDesc>& segs, float thr,
                  hipStream_t stream, std::vector<fac_match>& out, fac_stats* stats, std::string& err) {
  out.clear();
  MatchSink s;
  s.vec = &out;
  return launch_search_sink(e, h, segs, thr, stream, 0, s, stats, err);
}

int auto_beam_total(const Engine& e, const Haystack& h, const std::vector<SegDesc>& segs, float thr,
                    hipStream_t stream, uint64_t& total, std::string& err) {
  std::vector<uint32_t> counts;
  std::vector<fac_match> recs;
  MatchSink s;
  s.vec = &recs;
  const int rc = launch_pass(e, h, segs, thr, stream, 0, true, &counts, s, nullptr, err);
  total = 0;
  for (uint32_t c : counts) total += c;
  return rc;
}

// The pre-filter's device tables for the edit budgets ks (PfTables), built once per engine, ks and
// mode: the packed full-scan words and the q-gram path's tables (want_bytes: keyed by case-folded
// bytes when the q-gram path takes every pattern). Host work and uploads measured 0.41 ms per C5
// stream window when rebuilt per call.
int pf_tables(const Engine& e, const std::vector<uint32_t>& ks, bool want_bytes, const PfTables*& out, std::string& err) {
  const bool qgram_on = !diag_env("FAC_NO_QGRAM");
  std::lock_guard<std::mutex> lk(e.pf_mu);
  for (const auto& t : e.pf_cache)
    if (t->ks == ks && t->want_bytes == want_bytes && t->qgram_on == qgram_on) {
      out = t.get();
      return FAC_OK;
    }
  auto T = std::make_unique<PfTables>();
  T->ks = ks;
  T->want_bytes = want_bytes;
  T->qgram_on = qgram_on;
  const uint32_t np = (uint32_t)e.bp_m.size();
  const uint32_t rows = e.alphabet + 1;
  auto upload_raw = [&](const void* src, size_t bytes, void*& dst) -> int {
    HIP_TRY(hipMalloc(&dst, std::max<size_t>(bytes, 16)));
    if (bytes) HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return FAC_OK;
  };
  // Pigeonhole q-gram path (qgram_scan_kernel / qgram_verify_kernel) for the patterns whose k + 1
  // pieces are at least 3 symbols long; the rest go through the full bitap scan.
  std::vector<uint8_t> qlen(np, 0);
  std::vector<std::pair<uint32_t, uint32_t>> grams;  // (gram key, pattern << 8 | piece offset)
  std::vector<uint32_t> gram5;                       // per gram: its piece's fifth symbol (0xFFFF: none)
  if (qgram_on && rows <= 256) {
    std::vector<uint32_t> sym(64);
    // 5-gram screens only when no piece is screened by its 3-gram: 3-grams pass so often that they
    // make most candidates, and the extra screen then costs more than it removes (C5: 33.0 M
    // candidates per GiB either way, scan 1.02 -> 1.16 ms per GiB)
    bool any3 = false;
    for (uint32_t i = 0; i < np; ++i) any3 = any3 || (e.bp_m[i] <= 63 && e.bp_m[i] / (ks[i] + 1) == 3);
    for (uint32_t i = 0; i < np; ++i) {
      const uint32_t m = e.bp_m[i], k = ks[i], L = m / (k + 1);
      if (L < 3 || m > 63) continue;
      bool one = true;  // every pattern position is exactly one symbol
      for (uint32_t j = 0; j < m; ++j) {
        uint32_t hits = 0;
        for (uint32_t c = 0; c < rows; ++c)
          if ((e.bp_mask[(size_t)i * rows + c] >> j) & 1ull) sym[j] = c, ++hits;
        one = one && hits == 1;
      }
      if (!one) continue;
      const bool five = L >= 5 && !any3 && !diag_env("FAC_QG_NO5");
      const uint32_t q = std::min<uint32_t>(4, L);
      qlen[i] = (uint8_t)(five ? 5 : q);
      for (uint32_t r = 0; r <= k; ++r) {
        const uint32_t o = (uint32_t)((uint64_t)r * m / (k + 1));
        grams.push_back({qgram_key(sym[o], sym[o + 1], sym[o + 2], q == 4 ? sym[o + 3] : 0u, q == 4), (i << 8) | o});
      }
    }
    std::sort(grams.begin(), grams.end());
    for (const auto& g : grams) {  // (after the sort: gram5 follows grams' order)
      const uint32_t i = g.second >> 8, o = g.second & 0xFFu;
      if (qlen[i] != 5) {
        gram5.push_back(0xFFFFu);
        continue;
      }
      uint32_t c = 0;
      for (uint32_t cc = 0; cc < rows; ++cc)
        if ((e.bp_mask[(size_t)i * rows + cc] >> (o + 4)) & 1ull) c = cc;
      gram5.push_back(c);
    }
    for (size_t a = 0, b; a < grams.size(); a = b) {  // at most 255 entries per gram (table word)
      for (b = a; b < grams.size() && grams[b].first == grams[a].first; ++b) {}
      if (b - a > 255) {
        std::fill(qlen.begin(), qlen.end(), 0);
        grams.clear();
        gram5.clear();
        break;
      }
    }
  }
  // Pack the full-scan patterns into automaton words: patterns of one edit budget, longest first,
  // each into the first word with room (first-fit decreasing); 32-bit words when every pattern fits.
  std::vector<uint32_t> order;
  for (uint32_t i = 0; i < np; ++i)
    if (!qlen[i]) order.push_back(i);
  uint32_t mmax = 0;
  for (uint32_t i : order) mmax = std::max(mmax, e.bp_m[i]);
  const bool w32 = mmax <= 32;
  const uint32_t wbits = w32 ? 32u : 64u;
  std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    return ks[x] != ks[y] ? ks[x] < ks[y] : (e.bp_m[x] != e.bp_m[y] ? e.bp_m[x] > e.bp_m[y] : x < y);
  });
  std::vector<uint32_t> wk, wused;                   // per word: edit budget, bits used
  std::vector<std::pair<uint32_t, uint32_t>> place(np);  // pattern -> (word, bit offset)
  uint32_t k_first_word = 0;                         // words of the current budget start here
  for (uint32_t idx = 0; idx < (uint32_t)order.size(); ++idx) {
    const uint32_t i = order[idx], m = e.bp_m[i];
    if (idx && ks[i] != ks[order[idx - 1]]) k_first_word = (uint32_t)wk.size();
    uint32_t w = k_first_word;
    while (w < wk.size() && wused[w] + m > wbits) ++w;
    if (w == wk.size()) {
      wk.push_back(ks[i]);
      wused.push_back(0);
    }
    place[i] = {w, wused[w]};
    wused[w] += m;
  }
  const uint32_t nw = (uint32_t)wk.size();
  T->nw = nw;
  T->w32 = w32;
  for (uint32_t i : order) T->kmax = std::max(T->kmax, ks[i]);
  // Every pattern on the q-gram path: an ASCII text's bytes are read by the scan itself, so its grams
  // are keyed by each id's folded ASCII char (0x80: none, never in the text)
  T->bytes = want_bytes && nw == 0 && !grams.empty();
  if (T->bytes) {
    uint8_t byte_of_id[256];
    std::memset(byte_of_id, 0x80, sizeof(byte_of_id));
    for (uint32_t b = 0; b < 128; ++b) {
      const uint32_t id = e.ascii_id[b];
      if (id && byte_of_id[id] == 0x80) byte_of_id[id] = (uint8_t)(e.case_insensitive && b - 'A' < 26u ? b + 32u : b);
    }
    std::vector<std::pair<std::pair<uint32_t, uint32_t>, uint32_t>> g5(grams.size());
    for (size_t x = 0; x < grams.size(); ++x) {
      const uint32_t k = grams[x].first, q4 = (k >> 24) != 0xFFu;
      g5[x] = {{qgram_key(byte_of_id[k & 0xFFu], byte_of_id[(k >> 8) & 0xFFu], byte_of_id[(k >> 16) & 0xFFu],
                          q4 ? byte_of_id[k >> 24] : 0u, q4), grams[x].second},
               gram5[x] == 0xFFFFu ? 0xFFFFu : (uint32_t)byte_of_id[gram5[x]]};
    }
    std::sort(g5.begin(), g5.end());
    for (size_t x = 0; x < g5.size(); ++x) {
      grams[x] = g5[x].first;
      gram5[x] = g5[x].second;
    }
  }
  std::vector<uint64_t> pmask((size_t)rows * nw, 0), ptop(nw, 0);
  for (uint32_t i : order) {
    const uint32_t w = place[i].first, off = place[i].second;
    ptop[w] |= 1ull << (off + e.bp_m[i] - 1);
    for (uint32_t c = 0; c < rows; ++c) pmask[(size_t)c * nw + w] |= e.bp_mask[(size_t)i * rows + c] << off;
  }
  if (w32) {
    std::vector<uint32_t> m32(pmask.begin(), pmask.end()), t32(ptop.begin(), ptop.end());
    if (int rc = upload_raw(m32.data(), m32.size() * 4, T->pmask)) return rc;
    if (int rc = upload_raw(t32.data(), t32.size() * 4, T->ptop)) return rc;
  } else {
    if (int rc = upload_raw(pmask.data(), pmask.size() * 8, T->pmask)) return rc;
    if (int rc = upload_raw(ptop.data(), ptop.size() * 8, T->ptop)) return rc;
  }
  if (int rc = upload_raw(wk.data(), wk.size() * 4, T->wk)) return rc;
  if (!grams.empty()) {
    T->q = true;
    std::vector<uint2> ent(grams.size());
    std::vector<std::pair<uint32_t, uint32_t>> keys;  // (key, first entry << 8 | entries)
    for (size_t a = 0, b; a < grams.size(); a = b) {
      for (b = a; b < grams.size() && grams[b].first == grams[a].first; ++b) {
        const uint32_t i = grams[b].second >> 8;
        ent[b] = make_uint2(grams[b].second, e.bp_m[i] | (ks[i] << 8));
      }
      keys.push_back({grams[a].first, (uint32_t)(a << 8) | (uint32_t)(b - a)});
    }
    uint32_t ts = 64;
    while (ts < 2 * keys.size()) ts <<= 1;
    std::vector<uint2> tab(ts, make_uint2(0u, 0u));
    for (const auto& kv : keys) {
      uint32_t sl = qgram_hash(kv.first) & (ts - 1);
      while (tab[sl].y) sl = (sl + 1) & (ts - 1);
      tab[sl] = make_uint2(kv.first, kv.second);
    }
    std::vector<uint32_t> qbits(QG_BITS_WORDS, 0u);  // the scan's screening bitmap
    for (size_t x = 0; x < grams.size(); ++x) {
      const uint32_t b = gram5[x] == 0xFFFFu ? qgram_bit(grams[x].first) : qgram_bit5(grams[x].first, gram5[x]);
      qbits[b >> 5] |= 1u << (b & 31u);
    }
    std::vector<uint32_t> pm(np, 0);
    for (uint32_t i = 0; i < np; ++i)
      if (qlen[i]) {
        pm[i] = e.bp_m[i] | (ks[i] << 8);
        T->kq = std::max(T->kq, ks[i]);
        T->mq = std::max(T->mq, e.bp_m[i]);
        (qlen[i] == 5 ? T->use5 : qlen[i] == 4 ? T->use4 : T->use3) = 1u;
        T->n_qpat += 1;
      }
    T->ts = ts;
    T->n_grams = grams.size();
    T->n_keys = keys.size();
    if (int rc = upload_raw(tab.data(), tab.size() * sizeof(uint2), T->tab)) return rc;
    if (int rc = upload_raw(ent.data(), ent.size() * sizeof(uint2), T->ent)) return rc;
    if (int rc = upload_raw(e.bp_mask.data(), e.bp_mask.size() * 8, T->qmask)) return rc;
    if (int rc = upload_raw(pm.data(), pm.size() * 4, T->qpm)) return rc;
    if (int rc = upload_raw(qbits.data(), qbits.size() * 4, T->qbits)) return rc;
    // m <= 16 everywhere and a table within the 64 KB of dynamic LDS a block takes (two blocks per
    // CU, C5: 1 000 patterns x 27 rows = 54 KB): verify reads its masks from LDS
    const size_t n16 = ((size_t)np * rows + 1) & ~(size_t)1;
    if (T->mq <= 16 && n16 * 2 <= (64u << 10) - 256 && !diag_env("FAC_QGRAM_NO_LDS")) {
      std::vector<uint16_t> m16(n16, 0);
      for (size_t i = 0; i < (size_t)np * rows; ++i) m16[i] = (uint16_t)e.bp_mask[i];
      if (int rc = upload_raw(m16.data(), n16 * 2, T->m16)) return rc;
      T->m16_words = (uint32_t)(n16 / 2);
    }
  }
  out = T.get();
  e.pf_cache.push_back(std::move(T));
  return FAC_OK;
}

// qgram_verify_kernel for the tables' edit budget and mask layout: LDS masks in persistent blocks (two
// per CU), else global masks, 32- or 64-bit automaton words
template <bool WIN>
void launch_qverify(const PfTables& T, const QgramParams& Q, dim3 vg, hipStream_t stream) {
  const uint32_t kq = T.kq;
  if (T.m16) {
    const size_t lds = (size_t)T.m16_words * 4;
    if (kq <= 1) hipLaunchKernelGGL((qgram_verify_kernel<1, uint32_t, true, WIN>), vg, dim3(512), lds, stream, Q);
    else if (kq <= 2) hipLaunchKernelGGL((qgram_verify_kernel<2, uint32_t, true, WIN>), vg, dim3(512), lds, stream, Q);
    else if (kq <= 4) hipLaunchKernelGGL((qgram_verify_kernel<4, uint32_t, true, WIN>), vg, dim3(512), lds, stream, Q);
    else if (kq <= 8) hipLaunchKernelGGL((qgram_verify_kernel<8, uint32_t, true, WIN>), vg, dim3(512), lds, stream, Q);
    else hipLaunchKernelGGL((qgram_verify_kernel<24, uint32_t, true, WIN>), vg, dim3(512), lds, stream, Q);
  } else if (T.mq <= 32) {
    if (kq <= 1) hipLaunchKernelGGL((qgram_verify_kernel<1, uint32_t, false, WIN>), vg, dim3(256), 0, stream, Q);
    else if (kq <= 2) hipLaunchKernelGGL((qgram_verify_kernel<2, uint32_t, false, WIN>), vg, dim3(256), 0, stream, Q);
    else if (kq <= 4) hipLaunchKernelGGL((qgram_verify_kernel<4, uint32_t, false, WIN>), vg, dim3(256), 0, stream, Q);
    else if (kq <= 8) hipLaunchKernelGGL((qgram_verify_kernel<8, uint32_t, false, WIN>), vg, dim3(256), 0, stream, Q);
    else hipLaunchKernelGGL((qgram_verify_kernel<24, uint32_t, false, WIN>), vg, dim3(256), 0, stream, Q);
  } else {
    if (kq <= 1) hipLaunchKernelGGL((qgram_verify_kernel<1, uint64_t, false, WIN>), vg, dim3(256), 0, stream, Q);
    else if (kq <= 2) hipLaunchKernelGGL((qgram_verify_kernel<2, uint64_t, false, WIN>), vg, dim3(256), 0, stream, Q);
    else if (kq <= 4) hipLaunchKernelGGL((qgram_verify_kernel<4, uint64_t, false, WIN>), vg, dim3(256), 0, stream, Q);
    else if (kq <= 8) hipLaunchKernelGGL((qgram_verify_kernel<8, uint64_t, false, WIN>), vg, dim3(256), 0, stream, Q);
    else hipLaunchKernelGGL((qgram_verify_kernel<24, uint64_t, false, WIN>), vg, dim3(256), 0, stream, Q);
  }
}

int prefilter_windows(const Engine& e, const Haystack& h, const SegDesc& view, const std::vector<uint32_t>& ks,
                      hipStream_t stream, std::vector<std::pair<uint64_t, uint64_t>>& windows, fac_stats* stats,
                      std::string& err) {
  return prefilter_windows_ex(e, h, view, ks, stream, nullptr, windows, nullptr, stats, err);
}

// wins (optional): a batch of stream windows, [lo, hi) text positions of the view sorted by lo,
// each overlapping only its neighbours and not adjacent to the next-but-one (lo[w + 2] > hi[w]).
// Every window's bitap windows are its own -- the automaton starts at its lo, its coverage stays in
// it -- from one scan of the view; run_win receives each merged window's stream window. Returns
// FAC_E_UNSUPPORTED when some pattern needs the packed full scan (not window-aware).
int prefilter_windows_ex(const Engine& e, const Haystack& h, const SegDesc& view, const std::vector<uint32_t>& ks,
                         hipStream_t stream, const std::vector<std::pair<uint64_t, uint64_t>>* wins,
                         std::vector<std::pair<uint64_t, uint64_t>>& windows, std::vector<uint32_t>* run_win,
                         fac_stats* stats, std::string& err) {
  windows.clear();
  if (run_win) run_win->clear();
  HIP_TRY(hipSetDevice(e.device));
  if (!stream) stream = e.stream;
  const uint64_t n = view.n;
  if (n == 0) return FAC_OK;
  // An ASCII text whose bytes lie 16-byte aligned can be read by the q-gram scan itself, with no
  // transcode pass (0.66 ms per GiB at C5), when the q-gram path takes every pattern (pf_tables)
  const uint8_t* vb = h.d_utf8 + view.text_base;
  const bool want_bytes = view.ascii && ((uintptr_t)h.d_utf8 & 15u) == 0 && !diag_env("FAC_QGRAM_IDS");
  const PfTables* T = nullptr;
  if (int rc = pf_tables(e, ks, want_bytes, T, err)) return rc;
  const uint32_t nw = T->nw;
  const bool win = wins && !wins->empty();
  if (win && (nw != 0 || !T->q)) return FAC_E_UNSUPPORTED;  // the packed full scan has no window bounds
  PoolBuf d_ids, d_cover, d_runs, d_cnt, d_cover2, d_wlo, d_whi, d_wtab;
  if (!T->bytes) {  // the text's symbol ids (prefilter.rs:253-260)
    HIP_TRY(d_ids.alloc(n + 80, stream));  // padded: the scan's 16-byte loads and next word, verify's 64-symbol passes
    if (view.ascii) {  // transcode, ASCII text (prefilter.rs:253-258): one byte per grapheme
      const uint64_t threads = (n + 15) / 16;
      hipLaunchKernelGGL(transcode_ascii_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, stream, vb, n,
                         e.d_ascii_id, static_cast<uint8_t*>(d_ids.p));
      HIP_TRY(hipGetLastError());
    } else {
      ensure_symbols(e, h);
      HIP_TRY(hipMemcpyAsync(d_ids.p, h.sym.data() + view.text_base, n, hipMemcpyHostToDevice, stream));
    }
  }
  const uint64_t n_words = (n + 31) / 32;
  HIP_TRY(d_cover.alloc(n_words * 4, stream));
  HIP_TRY(hipMemsetAsync(d_cover.p, 0, n_words * 4, stream));
  std::vector<uint64_t> wlo, whi;
  std::vector<uint32_t> wtab;
  if (win) {  // the batch's window bounds and bucket table (QgramParams::wtab)
    const size_t nwin = wins->size();
    wlo.resize(nwin);
    whi.resize(nwin);
    for (size_t w = 0; w < nwin; ++w) {
      wlo[w] = (*wins)[w].first;
      whi[w] = std::min<uint64_t>((*wins)[w].second, n);
    }
    wtab.resize((size_t)((n >> QG_WSH) + 1));
    uint32_t w = 0;
    for (size_t b = 0; b < wtab.size(); ++b) {
      while (w + 1 < nwin && wlo[w + 1] <= ((uint64_t)b << QG_WSH)) ++w;
      wtab[b] = w;
    }
    HIP_TRY(d_cover2.alloc(n_words * 4, stream));
    HIP_TRY(hipMemsetAsync(d_cover2.p, 0, n_words * 4, stream));
    HIP_TRY(d_wlo.alloc(nwin * 8, stream));
    HIP_TRY(d_whi.alloc(nwin * 8, stream));
    HIP_TRY(d_wtab.alloc(wtab.size() * 4, stream));
    HIP_TRY(hipMemcpyAsync(d_wlo.p, wlo.data(), nwin * 8, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(d_whi.p, whi.data(), nwin * 8, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(d_wtab.p, wtab.data(), wtab.size() * 4, hipMemcpyHostToDevice, stream));
  }
  Events ev;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  HIP_TRY(hipEventRecord(ev.a, stream));
  BitapParams B{};
  B.ids = static_cast<const uint8_t*>(d_ids.p);
  B.n = n;
  B.mask_t = T->pmask;
  B.top = T->ptop;
  B.k = static_cast<const uint32_t*>(T->wk);
  B.n_words = nw;
  B.seg_len = 4096;
  B.cover = static_cast<uint32_t*>(d_cover.p);
  const uint64_t segs = (n + B.seg_len - 1) / B.seg_len;
  const uint64_t waves = segs * ((nw + 63) / 64);
  const uint32_t kmax = T->kmax;
  const dim3 bgrid((uint32_t)std::max<uint64_t>(1, (waves + 3) / 4));
  if (nw == 0) {
    // every pattern takes the q-gram path
  } else if (T->w32) {
    if (kmax == 0) hipLaunchKernelGGL((bitap_kernel<0, uint32_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax == 1) hipLaunchKernelGGL((bitap_kernel<1, uint32_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax == 2) hipLaunchKernelGGL((bitap_kernel<2, uint32_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax <= 4) hipLaunchKernelGGL((bitap_kernel<4, uint32_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax <= 8) hipLaunchKernelGGL((bitap_kernel<8, uint32_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax <= 16) hipLaunchKernelGGL((bitap_kernel<16, uint32_t>), bgrid, dim3(256), 0, stream, B);
    else hipLaunchKernelGGL((bitap_kernel<24, uint32_t>), bgrid, dim3(256), 0, stream, B);
  } else {
    if (kmax <= 1) hipLaunchKernelGGL((bitap_kernel<1, uint64_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax <= 2) hipLaunchKernelGGL((bitap_kernel<2, uint64_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax <= 4) hipLaunchKernelGGL((bitap_kernel<4, uint64_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax <= 8) hipLaunchKernelGGL((bitap_kernel<8, uint64_t>), bgrid, dim3(256), 0, stream, B);
    else if (kmax <= 16) hipLaunchKernelGGL((bitap_kernel<16, uint64_t>), bgrid, dim3(256), 0, stream, B);
    else hipLaunchKernelGGL((bitap_kernel<24, uint64_t>), bgrid, dim3(256), 0, stream, B);
  }
  HIP_TRY(hipGetLastError());
  PoolBuf d_qcand, d_qn, d_qovf, d_qrcnt;
  if (T->q) {
    HIP_TRY(d_qn.alloc(8, stream));
    QgramParams Q{};
    Q.ids = static_cast<const uint8_t*>(d_ids.p);
    Q.n = n;
    Q.nsafe = n + 80;
    if (T->bytes) {
      Q.ids = reinterpret_cast<const uint8_t*>((uintptr_t)vb & ~(uintptr_t)15);
      Q.off = (uint32_t)(vb - Q.ids);
      Q.nsafe = (uint64_t)(h.d_utf8 + h.len - Q.ids);
      Q.bytes = 1;
      Q.ci = e.case_insensitive ? 1u : 0u;
      Q.aid = e.d_ascii_id;
    }
    Q.tab = static_cast<const uint2*>(T->tab);
    Q.tab_mask = T->ts - 1;
    Q.ent = static_cast<const uint2*>(T->ent);
    Q.use3 = T->use3;
    Q.use4 = T->use4;
    Q.use5 = T->use5;
    Q.n_ovf = static_cast<unsigned long long*>(d_qn.p);
    Q.pmask = static_cast<const uint64_t*>(T->qmask);
    Q.pm = static_cast<const uint32_t*>(T->qpm);
    Q.rows = e.alphabet + 1;
    Q.cover = static_cast<uint32_t*>(d_cover.p);
    Q.bits = static_cast<const uint32_t*>(T->qbits);
    Q.m16 = static_cast<const uint32_t*>(T->m16);
    Q.m16_words = T->m16_words;
    if (win) {
      Q.nwin = (uint32_t)wlo.size();
      Q.wlo = static_cast<const uint64_t*>(d_wlo.p);
      Q.whi = static_cast<const uint64_t*>(d_whi.p);
      Q.wtab = static_cast<const uint32_t*>(d_wtab.p);
      Q.cover2 = static_cast<uint32_t*>(d_cover2.p);
      // the fixed-size cut (window w at w * 2^sh, its text 2^sh + ov bytes): bounds by arithmetic
      if (wlo.size() > 1 && wlo[0] == 0 && (wlo[1] & (wlo[1] - 1)) == 0 && wlo[1] >= 64 && whi[0] > wlo[1]) {
        const uint32_t sh = (uint32_t)__builtin_ctzll(wlo[1]);
        const uint64_t ov = whi[0] - wlo[1];
        bool uni = ov < (1ull << 31);
        for (size_t w = 0; w < wlo.size() && uni; ++w)
          uni = wlo[w] == ((uint64_t)w << sh) && whi[w] == std::min<uint64_t>(n, wlo[w] + (1ull << sh) + ov);
        if (uni) {
          Q.wsh = sh;
          Q.wov = (uint32_t)ov;
        }
      }
    }
    int cus = 256;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e.device));
    // two full resident rounds of scan blocks (2 per CU at 56 KB of LDS): the scan strides over the
    // text, so every block does the same work, and a grid of 8 per CU ran 2.7 rounds (the last one 2/3
    // full); one round left the verify's 2 persistent blocks per CU 1.5 regions each (1.21 vs 1.15 ms)
    // instantiations by the gram kinds in use (3-grams alone, 4-grams, 5-gram screens, or mixed)
    const uint32_t qk = (Q.use3 ? 1u : 0u) | (Q.use4 ? 2u : 0u) | (Q.use5 ? 4u : 0u);
    const void* scan_fns[8] = {reinterpret_cast<const void*>(&qgram_scan_kernel<true, false, false>),
                               reinterpret_cast<const void*>(&qgram_scan_kernel<true, false, false>),
                               reinterpret_cast<const void*>(&qgram_scan_kernel<false, true, false>),
                               reinterpret_cast<const void*>(&qgram_scan_kernel<true, true, false>),
                               reinterpret_cast<const void*>(&qgram_scan_kernel<false, false, true>),
                               reinterpret_cast<const void*>(&qgram_scan_kernel<true, false, true>),
                               reinterpret_cast<const void*>(&qgram_scan_kernel<false, true, true>),
                               reinterpret_cast<const void*>(&qgram_scan_kernel<true, true, true>)};
    const void* scan_fn = scan_fns[qk];
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, scan_fn, 64 * QG_WAVES, 0) != hipSuccess || per_cu < 1)
      per_cu = 1;
    const uint32_t sgrid =
        (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 8191) / 8192, (uint64_t)cus * (uint64_t)per_cu * 2));
    // regions of 1/16 of a block's positions (C5 fills ~half); the overflow list is checked after
    Q.nreg = sgrid;
    Q.region = std::max<uint64_t>(256, (n / sgrid + 15) / 16);
    HIP_TRY(d_qcand.alloc(Q.region * sgrid * 8, stream));
    HIP_TRY(d_qrcnt.alloc((size_t)sgrid * 4, stream));
    Q.cand = static_cast<unsigned long long*>(d_qcand.p);
    Q.rcnt = static_cast<uint32_t*>(d_qrcnt.p);
    uint64_t ocap = 1 << 20;
    unsigned long long nc = 0;  // overflow entries
    for (;;) {  // candidates: one scan, again with room for all of them if the overflow list overflowed
      HIP_TRY(d_qovf.alloc(ocap * 8, stream));
      Q.ovf = static_cast<unsigned long long*>(d_qovf.p);
      Q.ovf_cap = ocap;
      HIP_TRY(hipMemsetAsync(d_qn.p, 0, 8, stream));
      switch (qk) {
        case 2: hipLaunchKernelGGL((qgram_scan_kernel<false, true, false>), dim3(sgrid), dim3(64 * QG_WAVES), 0, stream, Q); break;
        case 3: hipLaunchKernelGGL((qgram_scan_kernel<true, true, false>), dim3(sgrid), dim3(64 * QG_WAVES), 0, stream, Q); break;
        case 4: hipLaunchKernelGGL((qgram_scan_kernel<false, false, true>), dim3(sgrid), dim3(64 * QG_WAVES), 0, stream, Q); break;
        case 5: hipLaunchKernelGGL((qgram_scan_kernel<true, false, true>), dim3(sgrid), dim3(64 * QG_WAVES), 0, stream, Q); break;
        case 6: hipLaunchKernelGGL((qgram_scan_kernel<false, true, true>), dim3(sgrid), dim3(64 * QG_WAVES), 0, stream, Q); break;
        case 7: hipLaunchKernelGGL((qgram_scan_kernel<true, true, true>), dim3(sgrid), dim3(64 * QG_WAVES), 0, stream, Q); break;
        default: hipLaunchKernelGGL((qgram_scan_kernel<true, false, false>), dim3(sgrid), dim3(64 * QG_WAVES), 0, stream, Q); break;
      }
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemcpyAsync(&nc, d_qn.p, 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      if (nc <= ocap) break;
      // which candidates overflow depends on wave timing (a block's first failed reservation varies
      // by up to one drain, 64 x 255 entries): regrow with headroom so the re-scan fits
      ocap = nc + nc / 4 + (uint64_t)sgrid * 64 * 255;
    }
    if (diag_env("FAC_TIMING")) {
      std::vector<uint32_t> rc(sgrid);
      HIP_TRY(hipMemcpyAsync(rc.data(), d_qrcnt.p, (size_t)sgrid * 4, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      uint64_t tot = nc, mx = 0;
      for (uint32_t c : rc) tot += c, mx = std::max<uint64_t>(mx, c);
      std::fprintf(stderr, "FAC_QGRAM text %llu symbols, %llu candidates (%llu overflow, region %llu, fullest %llu), use3 %u use4 %u use5 %u\n",
                   (unsigned long long)n, (unsigned long long)tot, nc, (unsigned long long)Q.region,
                   (unsigned long long)mx, Q.use3, Q.use4, Q.use5);
    }
    {
      const dim3 vg((uint32_t)std::min<uint64_t>(sgrid + 1, (uint64_t)cus * (T->m16 ? 2 : 8)));
      if (Q.nwin) launch_qverify<true>(*T, Q, vg, stream);
      else launch_qverify<false>(*T, Q, vg, stream);
      HIP_TRY(hipGetLastError());
    }
    if (diag_env("FAC_RC_DEBUG"))
      std::fprintf(stderr, "FAC_QGRAM patterns=%zu/%zu grams=%zu keys=%zu candidates=%llu full-scan words=%u bytes=%d\n",
                   T->n_qpat, e.bp_m.size(), T->n_grams, T->n_keys, nc, nw, (int)T->bytes);
  }
  // maximal runs of each bitmap (with windows: cover holds the even windows', cover2 the odd ones';
  // same-parity windows are not adjacent, so no run spans two of them)
  std::vector<uint32_t> par[2];  // the windows of each parity, ascending lo
  if (win)
    for (uint32_t w = 0; w < (uint32_t)wlo.size(); ++w) par[w & 1].push_back(w);
  std::vector<std::tuple<uint64_t, uint64_t, uint32_t>> runs;  // (start, end, stream window)
  const int npass = win ? 2 : 1;
  PoolBuf d_runs2;
  PoolBuf* rbuf[2] = {&d_runs, &d_runs2};
  uint64_t cap[2] = {1u << 16, 1u << 16};
  HIP_TRY(d_cnt.alloc(16, stream));
  for (;;) {  // both bitmaps' runs in one round trip; again with room for all of them if a list overflowed
    HIP_TRY(hipMemsetAsync(d_cnt.p, 0, 16, stream));
    for (int pass = 0; pass < npass; ++pass) {
      const uint32_t* cov = static_cast<const uint32_t*>(pass ? d_cover2.p : d_cover.p);
      HIP_TRY(rbuf[pass]->alloc(cap[pass] * 16, stream));
      hipLaunchKernelGGL(runs_kernel, dim3((uint32_t)((n_words + 255) / 256)), dim3(256), 0, stream, cov, n_words, n,
                         static_cast<unsigned long long*>(rbuf[pass]->p), static_cast<unsigned long long*>(d_cnt.p) + pass,
                         cap[pass]);
      HIP_TRY(hipGetLastError());
    }
    unsigned long long c[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(c, d_cnt.p, 16, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    bool again = false;
    for (int pass = 0; pass < npass; ++pass)
      if (c[pass] > cap[pass]) {
        cap[pass] = c[pass];
        again = true;
      }
    if (again) continue;
    std::vector<unsigned long long> buf[2];
    for (int pass = 0; pass < npass; ++pass) {
      buf[pass].resize(2 * c[pass]);
      if (c[pass]) HIP_TRY(hipMemcpyAsync(buf[pass].data(), rbuf[pass]->p, c[pass] * 16, hipMemcpyDeviceToHost, stream));
    }
    HIP_TRY(hipEventRecord(ev.b, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    for (int pass = 0; pass < npass; ++pass)
      for (uint64_t i = 0; i < c[pass]; ++i) {
        const uint64_t r0 = buf[pass][2 * i], r1 = buf[pass][2 * i + 1];
        uint32_t w = 0xFFFFFFFFu;
        if (win) {  // the window of this bitmap's parity whose [lo, hi) holds the run
          const auto& v = par[pass];
          auto it = std::upper_bound(v.begin(), v.end(), r0, [&](uint64_t x, uint32_t ww) { return x < wlo[ww]; });
          if (it != v.begin() && r0 < whi[*(it - 1)]) w = *(it - 1);
          if (w == 0xFFFFFFFFu) {
            err = "internal: a pre-filter run outside every stream window";
            return FAC_E_INTERNAL;
          }
        }
        runs.emplace_back(r0, r1, w);
      }
    break;
  }
  std::sort(runs.begin(), runs.end(), [](const auto& x, const auto& y) {
    return std::get<2>(x) != std::get<2>(y) ? std::get<2>(x) < std::get<2>(y) : std::get<0>(x) < std::get<0>(y);
  });
  windows.resize(runs.size());
  if (run_win) run_win->resize(runs.size());
  for (size_t r = 0; r < runs.size(); ++r) {
    windows[r] = {std::get<0>(runs[r]), std::get<1>(runs[r])};
    if (run_win) (*run_win)[r] = std::get<2>(runs[r]);
  }
  if (stats) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    stats->prefilter_ms += ms;
  }
  return FAC_OK;
}


// ---- Diagnostics: the beam cut alone (tests) ----------------------------------------------------
// One wave per key array: the array becomes a ring of states (node = original index, pen = key) at a
// rotated head, then beam_select_lds (ring of 256, the LDS claim-word scratch) or beam_select (ring of
// 1024 in LDS, the global per-wave scratch) keeps bw states; perm[i] = the node of the i-th survivor,
// i < bw -- compared by the tests with the oracle's select_nth_unstable_by (oracle.cpp rsel).
template <uint32_t QCAP, bool LDS>
__global__ __launch_bounds__(64) void diag_select_kernel(const float* keys, const uint64_t* offs, uint32_t bw,
                                                         uint32_t limit, uint4* bsel, uint32_t* perm) {
  __shared__ KState q[QCAP];
  __shared__ uint32_t claim[512];
  const uint32_t lane = lane_id();
  const uint32_t a = blockIdx.x;
  const uint64_t b = offs[a], P = offs[a + 1] - b;
  const uint32_t head = (a * 37u) & (QCAP - 1u);
  for (uint32_t i = lane; i < 512u; i += 64u) claim[i] = 0u;
  for (uint32_t i = lane; i < (uint32_t)P; i += 64u) q[(head + i) & (QCAP - 1u)] = KState{i, 0u, keys[b + i], 0u};
  wave_mem_fence();
  uint32_t tail = head + (uint32_t)P;
  if constexpr (LDS) beam_select_lds<QCAP>(q, head, tail, bw, claim, limit);
  else beam_select<QCAP>(q, head, tail, bw, bsel + (size_t)a * bsel_stride(QCAP), limit);
  wave_mem_fence();
  for (uint32_t i = lane; i < bw; i += 64u) perm[(size_t)a * bw + i] = q[(head + i) & (QCAP - 1u)].node;
}

int diag_beam_select(const float* keys, const uint64_t* offs, uint64_t count, uint32_t bw, int32_t lds,
                     int32_t sel_limit, uint32_t* perm, std::string& err) {
  const uint32_t cap = lds ? 256u : 1024u;
  if (bw == 0 || count == 0 || count > (1u << 20)) {
    err = "diag_beam_select: bw and count must be in [1, 2^20]";
    return FAC_E_INVALID;
  }
  for (uint64_t a = 0; a < count; ++a) {  // the kernels' preconditions: 2 bw < P <= ring
    const uint64_t P = offs[a + 1] - offs[a];
    if (offs[a + 1] < offs[a] || P <= 2ull * bw || P > cap) {
      err = "diag_beam_select: every array needs 2*bw < len <= " + std::to_string(cap);
      return FAC_E_INVALID;
    }
  }
  const uint64_t nk = offs[count];
  std::vector<float> hk(keys, keys + nk);
  std::vector<uint64_t> ho(offs, offs + count + 1);
  float* dk = nullptr;
  uint64_t* dof = nullptr;
  uint32_t* dp = nullptr;
  uint4* db = nullptr;
  int rc = upload(hk, &dk, err);
  if (!rc) rc = upload(ho, &dof, err);
  auto cleanup = [&] {
    (void)hipFree(dk);
    (void)hipFree(dof);
    (void)hipFree(dp);
    (void)hipFree(db);
  };
  if (rc) {
    cleanup();
    return rc;
  }
  auto run = [&]() -> int {
    HIP_TRY(hipMalloc((void**)&dp, count * bw * sizeof(uint32_t)));
    if (!lds) HIP_TRY(hipMalloc((void**)&db, count * bsel_stride(1024) * sizeof(uint4)));
    const uint32_t lim = sel_limit < 0 ? 16u : (uint32_t)sel_limit;
    if (lds) hipLaunchKernelGGL((diag_select_kernel<256, true>), dim3((uint32_t)count), dim3(64), 0, 0, dk, dof, bw, lim, db, dp);
    else hipLaunchKernelGGL((diag_select_kernel<1024, false>), dim3((uint32_t)count), dim3(64), 0, 0, dk, dof, bw, lim, db, dp);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(perm, dp, count * bw * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return FAC_OK;
  };
  rc = run();
  cleanup();
  return rc;
}

}  // namespace fac
