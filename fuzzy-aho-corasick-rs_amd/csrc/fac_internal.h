// fac_internal.h — host/device data layout of the MI355X fuzzy Aho–Corasick engine.
//
// The reference keeps a `Vec<Node>` of 112-byte nodes, each owning two heap `Vec`s and a
// hash map (structs.rs:249-281). On MI355X the automaton is flattened into structure-of-arrays
// tables that stay L2-resident (≈1-5 MB at 10K patterns) and are read with wave-uniform loads:
//
//   DevNode[N]   32 B  prune_len, prune_len_over_weight, edge_begin, degree | has-output, and the
//                      node's single-ASCII-byte edge map (structs.rs:471-493): one load per pop
//   out_range[N]  8 B  output range (read on emission only); node_pidx[N] 4 B pattern_index
//   DevEdge[E]    8 B  first code point | target node + (child-has-output, single-byte) flag bits
//   sb_edge[E]   16 B  sb_bits of each edge's child (one parent edge per node: loads in parallel
//                      with the edge record instead of after it)
//   out_pat[O]    4 B  output pattern ids (own + fail-merged, builder.rs:235,264-268)
//   DevPattern[P]32 B  grapheme_len as f32, weight, per-pattern limits
//   sim_ascii  64 KiB  128x128 f32 similarity table (structs.rs:36-48) + sorted non-ASCII pairs
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>

#include "../../include/fac.h"

namespace fac {

// ---------------------------------------------------------------- unicode.cpp
uint32_t utf8_decode(const uint8_t* s, uint64_t n, uint64_t& i);
bool utf8_valid(const uint8_t* s, uint64_t n, bool* ascii = nullptr);  // ascii: also whether every byte < 0x80
uint64_t utf8_valid_prefix(const uint8_t* s, uint64_t n);
void segment_graphemes(const uint8_t* s, uint64_t n, std::vector<uint64_t>& starts);
int lower_full(uint32_t cp, uint32_t out[3]);
void fold_grapheme(const uint8_t* s, uint64_t b, uint64_t e, bool ci, std::u32string& out);
uint32_t fold_first_char(const uint8_t* s, uint64_t b, uint64_t e, bool ci);

// ---------------------------------------------------------------- device layout
constexpr uint32_t EDGE_SINGLE_BYTE = 1u << 31;
constexpr uint32_t EDGE_CHILD_OUTPUT = 1u << 30;
constexpr uint32_t EDGE_NEXT_MASK = (1u << 30) - 1;
constexpr uint32_t CHILD26_MASK = (1u << 26) - 1;  // node ids are < 2^26 (builder limit)

// goto table entry: kv = GT_VALID | kind << 47 | node << 21 | char; val by kind:
//   GT_GOTO: first edge of `node` whose first char is `char`: child | edge index << 32 | own-single-byte << 40
//   GT_SB:   bit i = child of edge i has a single-byte edge labelled `char` (char < 128)
constexpr uint64_t GT_VALID = 1ull << 63;
constexpr uint64_t GT_GOTO = 0, GT_SB = 1ull << 47;
// 2-choice cuckoo table of 16 B entries {kv, val}: a key lives at gt_slot(kv, seed1) or
// gt_slot(kv, seed2); lookups read both slots, no probing
__host__ __device__ inline uint32_t gt_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// both cuckoo slots from one 32-bit hash: a base hash of (node, char) shared by the GOTO and SB
// keys of that pair (the SB hash is an affine step away), low bits and the 16-bit rotation
__host__ __device__ inline uint32_t gt_base(uint32_t node, uint32_t ch, uint64_t seed) {
  return gt_mix32(((node << 21) | ch) ^ gt_mix32((node >> 11) ^ (uint32_t)seed));
}
// char filters (Engine::aux, GOTO values bits 48-63): one bit per hashed code point, a clear bit
// proves the (node, char) lookup would miss
__host__ __device__ inline uint32_t ch_filt_bit(uint32_t c) { return (c * 0x9E3779B1u) >> 27; }
__host__ __device__ inline uint32_t filt_fold16(uint32_t f) { return (f | (f >> 16)) & 0xFFFFu; }
__host__ __device__ inline uint32_t gt_kind_hash(uint32_t base, bool sb) {
  return sb ? base * 0x9E3779B1u + 0x7F4A7C15u : base;
}
__host__ __device__ inline void gt_slots_h(uint32_t h, uint32_t mask, uint32_t& s1, uint32_t& s2) {
  s1 = h & mask;
  s2 = ((h >> 16) | (h << 16)) & mask;
}
__host__ __device__ inline void gt_slots(uint64_t kv, uint64_t seed, uint32_t mask, uint32_t& s1, uint32_t& s2) {
  const uint32_t node = (uint32_t)((kv >> 21) & ((1u << 26) - 1)), ch = (uint32_t)(kv & ((1u << 21) - 1));
  gt_slots_h(gt_kind_hash(gt_base(node, ch, seed), (kv & GT_SB) != 0), mask, s1, s2);
}
constexpr int32_t LIM_NONE = -1;

struct U32StrHash {
  size_t operator()(const std::u32string& s) const {
    uint64_t h = 1469598103934665603ull;
    for (char32_t c : s) h = (h ^ (uint64_t)c) * 1099511628211ull;
    return (size_t)h;
  }
};

// host-side node (builder, host bookkeeping)
struct HostNode {
  float prune_len;
  float prune_lw;
  uint32_t edge_begin, edge_end;
  uint32_t out_begin, out_end;
  int32_t pidx;  // pattern_index (first pattern touching the node), -1 = None
};

// device node: one 32 B load gives everything a pop needs
constexpr uint32_t NODE_HAS_OUT = 1u << 31;
constexpr uint32_t NODE_DUP_CH = 1u << 30;     // two of the node's edges share a first char
constexpr uint32_t NODE_ASCII_EDGE = 1u << 29; // some edge's first char is ASCII
constexpr uint32_t NODE_DEG_MASK = (1u << 24) - 1;
struct alignas(16) DevNode {
  float prune_len;
  float prune_lw;
  uint32_t edge_begin;
  uint32_t degf;  // degree | NODE_HAS_OUT
  uint4 sb;       // 128-bit map of the node's single-ASCII-byte edge chars (structs.rs:471-493)
};
static_assert(sizeof(DevNode) == 32, "DevNode layout");

struct DevEdge {
  uint32_t ch;    // first char of the folded grapheme
  uint32_t next;  // target | EDGE_CHILD_OUTPUT | EDGE_SINGLE_BYTE
};

struct DevLimits {
  int32_t ins, del, sub, swp, edits;  // LIM_NONE = None
};

struct alignas(16) DevPattern {
  float glen;    // grapheme_len as f32 (search.rs:696)
  float weight;  // Pattern::weight
  int32_t has_limits;
  DevLimits lim;
};
static_assert(sizeof(DevPattern) == 32, "DevPattern layout");

// Dedup entry / queued state, 16 B. j and matched_end are stored relative to the window start
// (matched_start == start for every state of a window).
struct alignas(16) KState {
  uint32_t node;
  uint32_t jm;     // j_rel | me_rel << 16
  float pen;
  uint32_t packed;  // ins | del << 8 | sub << 16 | swp << 24 (structs.rs:173-176)
};

// A (sub)haystack searched as if it were the whole `haystack` argument of search_raw: the prefilter
// re-searches merged windows as independent slices (prefilter.rs:346-350), shards of one haystack
// keep the global length but only own a window range, and batches hold several haystacks.
struct SegDesc {
  uint64_t text_base;  // ascii: byte index of local grapheme 0 in `utf8`; unicode: grapheme index
  uint64_t n;          // text_len of the (sub)haystack (search.rs:440)
  uint64_t avail;      // local graphemes resident (>= every j the windows can reach, else ERR_HALO)
  uint64_t hay_len;    // byte length of the (sub)haystack (end_byte when me >= n, search.rs:672-676)
  uint64_t byte_base;  // global byte offset of local byte 0 (added to every output offset)
  uint64_t w_begin, w_end;  // local start windows to search
  uint32_t ascii;      // 1: grapheme == byte (AsciiGraphemes), 0: Unicode graphemes
  uint32_t pad;
};

// one prefix-cache level: open-addressing table of key hashes -> entry -> snapshot
struct RcTable {
  uint32_t k;                        // key chars
  uint32_t mask;                     // slots - 1
  const unsigned long long* keys;    // 0 = empty slot
  const uint32_t* val;               // entry of each slot (EMPTY: not cached)
  const uint32_t* off;               // snapshot offset of each entry (pool words)
  const uint32_t* count;             // queued states of each entry (EMPTY: not cached)
  // lookup table of the built entries (rc_publish_kernel): 32-byte slots {exact key: the k chars as
  // 16-bit units, padded with 0xFFFF; snapshot offset, head, queue length | best entries << 16,
  // occupied | dedup entries << 22 | pops}
  const uint4* ct;
  uint32_t ct_mask;                  // lookup slots - 1
};

constexpr int N_COUNTERS = 12;  // SearchParams::counters (8: lane-searched windows, 9: lane work counter, 10: lookup
                                // regions, 11: snapshots a cache build kept)
constexpr int kRcLevels = 5;   // prefix-cache levels: level 0 (under level 1), level 1, up to 3 sampled levels

struct SearchParams {
  // automaton
  const DevNode* nodes;
  const DevEdge* edges;
  const uint32_t* out_pat;
  const uint2* out_range;
  const int32_t* node_pidx;
  // O(1) expansion tables (builder.cpp "goto table"): (node, char) -> first edge / child maps
  const uint4* gt;            // cuckoo slots {kv lo, kv hi, val lo, val hi}
  uint32_t gt_mask;           // slot count - 1
  unsigned long long gt_seed1, gt_seed2;
  int32_t gt_fast;            // similarity can never drop a substitution when p_sub <= remaining
  // per node {child-has-output mask lo, hi (degree <= 64), child char filter, grandchild single-byte
  // char filter}: the filters (bit ch_filt_bit(c)) gate goto-table lookups that would miss
  const uint4* aux;
  const uint4* sb_edge;
  const DevPattern* pats;
  const float* sim_ascii;
  const uint64_t* sim_keys;  // (a << 32 | b), sorted
  const float* sim_vals;
  uint32_t n_sim;
  // haystack storage
  const uint8_t* utf8;     // raw bytes (ascii segments read graphemes from here)
  const uint32_t* text32;  // folded first code point per grapheme (unicode segments)
  const uint64_t* off;     // global byte offset per grapheme (unicode segments)
  const SegDesc* segs;
  const uint64_t* seg_prefix;  // exclusive prefix of (w_end - w_begin), n_segs + 1 entries
  uint32_t n_segs;
  uint64_t total_windows;
  int32_t case_insensitive;
  // scoring
  float thr;
  float max_penalties;
  float p_ins, p_del, p_sub, p_swp;
  float min_sym;
  uint32_t mef;  // MAX_EDITS_FAST (1..6) or 255
  int32_t has_glim;
  DevLimits glim;
  int32_t has_pattern_limits;
  uint32_t beam;  // 0 = None
  int32_t window_skip;
  uint32_t first_bits[4], second_bits[4];
  // work distribution / outputs
  uint32_t chunk;
  uint32_t ecap;            // per-wave emission list capacity
  uint4* ebuf;              // per-wave emission scratch (slice = the wave's slot)
  // wave slots (bfs_window_body): a launch may have more workgroups than resident waves (the
  // one-chunk-per-workgroup level-1 build), so per-wave global scratch is indexed by a slot taken
  // from a free ring when the wave starts and returned when it ends (slot_ctr: taken, returned)
  unsigned int* slot_ring;
  unsigned int* slot_ctr;
  uint32_t n_slots;
  uint4* bsel;              // beamed engines: the beam selection's scratch (bsel_stride per slot)
  uint32_t bsel_stride;
  uint32_t sel_limit;       // select.rs partition rounds before median_of_medians (16; tests lower it)
  int32_t beam_canonical;   // diagnostics (FAC_BEAM_CANONICAL): rounds 1-2's canonical tie rule
  fac_match* out;
  uint64_t out_cap;
  uint64_t out_shift;       // added to every record's start/end (global byte of a shard's byte 0)
  unsigned long long* counters;  // [0] matches, [1] states popped, [2] error flags, [3] spilled windows,
                                 // [4] pops replayed from snapshots, [5] windows resumed from a snapshot,
                                 // [6] of those, finished by the snapshot alone (empty queue),
                                 // [7] next window chunk (dynamic chunk hand-out)
  int32_t rc_lane_flush;         // resumed windows with an empty queue are flushed lane-parallel
  int32_t dyn_chunks;            // 1: chunks from the work counter; 0: static grid-stride
  uint32_t lane_popmax;           // lane_window_kernel: pops after which a window goes back to the wave kernel
  uint32_t live_nqmax;            // bfs_window_kernel_live: windows resuming with a longer queue go straight to the
                                  // exact variant (0: none)
  int32_t lane_debug;             // lane_window_kernel: diagnostics counters (FAC_RC_DEBUG)
  // window list mode (re-run of spilled windows) and the spill list of capacity overflows
  const uint64_t* win_list;  // null: virtual windows 0..total_windows; else list of virtual ids
  uint64_t* spill;           // virtual ids of windows that overflowed this variant's LDS frontier
  uint64_t spill_cap;
  // auto-beam pass 1 (search.rs:1096-1103): per window queue.len() under exact dedup
  uint32_t* win_counts;  // null: not recorded
  int32_t exact_dedup;   // dedup must be exact (beam, or counting for auto-beam)
  int32_t dup_cut;       // diagnostics (FAC_DUP_CUT=1): cut a batch at an in-batch duplicate instead of resolving it
  // prefix cache (launch_pass): a state at j reads text[j] and text[j + 1], so the
  // pops before the first state with j >= rc_k - 1 depend only on the window's first rc_k chars;
  // windows sharing them resume from one snapshot (queue, dedup entries, best list, counters)
  // Two levels: short keys for every window, long keys for the frequent prefixes only; a lookup
  // takes the deepest hit (rc_tab[0] first). A level-2 build resumes its representatives from
  // level-1 snapshots.
  int32_t rc_mode;                  // 0 off, 1 use the cache, 2 build it (win_list = representatives)
  uint32_t rc_k;                    // key chars of the level being collected / built (2..8)
  uint32_t rc_ntab;                 // tables a lookup consults (0..kRcLevels), deepest first
  uint32_t rc_kstart;               // rc_lookup's first probe: the shallowest level with k >= this (0: the
                                    // shallowest level; a k no level has, 0xFFFFFFFF: the deepest level)
  uint4* rc_bhits;                  // cache build: each key's parent snapshot (rc_parent_kernel), as rc_hits
  uint32_t* rc_bpops;               // ... and its pops
  RcTable rc_tab[kRcLevels];
  uint32_t rc_vmax, rc_emax;        // dedup / best-list entries a snapshot may hold
  uint4* rc_pool;                   // snapshots: header x4, queue, dedup entries, best list
  unsigned long long rc_pool_cap;   // pool words (uint4)
  unsigned long long* rc_pool_used; // bump allocator
  uint32_t rc_pool_chunk;           // pool words a building wave takes at a time
  uint32_t rc_qcap;                 // main pass ring: snapshots with more queued states are not resumed
  uint4* rc_hits;                   // main pass: per window {offset | RC_DONE, head, tail, nv | ne << 16}
  uint32_t* rc_hit_pops;            // ... and the snapshot's pops
  // main pass: rc_hits / rc_hit_pops hold only the windows the lookups leave open, compacted per
  // region of RC_REGION windows (entries [r * RC_REGION, + rc_region_cnt[r])); rc_voff = the window
  // of each entry as its offset in the region
  uint32_t* rc_voff;
  uint32_t* rc_region_cnt;
  uint32_t* rc_off;                 // build: snapshot offset of each entry (pool words)
  uint32_t* rc_count;               // build: queued states of each entry (EMPTY: not cached)
  int32_t rc_keep_final;            // build: snapshot a key whose parent is final too (its level is
                                    // looked up without the parent's: level 1 over level 0)
  // multi-character mappings (search.rs:776-780, 883-922, 945-961; builder.rs:383-442). With
  // has_map, exact and swap transitions compare whole folded graphemes (ids, 0 = not in the
  // engine's grapheme dictionary): edge_gid per edge, text gids per grapheme (gid32 for Unicode
  // segments, ascii_gid[folded byte] for ASCII ones)
  int32_t has_map;
  const uint32_t* edge_gid;
  const uint32_t* gid32;
  const uint32_t* ascii_gid;  // 128 entries
  const uint2* map_range;     // per node [begin, end) into map_ent
  const uint4* map_ent;       // {hay begin (into map_hay), hay length, next node, penalty bits}
  const uint32_t* map_hay;    // haystack-side grapheme ids
  // key partition of the haystack's start windows (Haystack::kparts / kpart), last: fields added
  // in the middle moved every later kernel argument and changed the window kernels' allocation
  uint32_t kp_n, kp_r;
  // the key part's start windows, ascending (rc_count_kernel / rc_lookup_kernel walk them; the
  // lookup stores each open window as its list region's base + offset, so the searches' entry ->
  // window mapping needs no list)
  const uint64_t* kp_wlist;
  // dense start-level key bitmaps (rc_dense_*_kernel, search_kernels.hip): rank table, alphabet size,
  // "final without records" and "cached" bits over the keys of ranked characters; null: none
  const uint32_t* rc_dense;
};

constexpr unsigned ERR_QUEUE = 1u, ERR_VISITED = 2u, ERR_EMIT = 4u, ERR_HALO = 8u, ERR_OUT = 16u, ERR_SPILL = 32u;

// ---------------------------------------------------------------- engine
// The pre-filter's device tables for one set of edit budgets (search_kernels.hip prefilter_windows):
// the packed full-scan words and the q-gram path's gram table, screening bitmap and pattern masks.
// Built on a call's first use and kept by the engine (they depend on the engine and ks alone).
struct PfTables {
  std::vector<uint32_t> ks;
  bool want_bytes = false;  // the key: built for a byte-reading scan (if the q-gram path takes every pattern),
  bool qgram_on = true;     // and the FAC_NO_QGRAM knob's state
  bool bytes = false;       // the grams keyed by case-folded bytes (else by symbol ids)
  uint32_t nw = 0, kmax = 0;  // packed full scan: automaton words, largest edit budget
  bool w32 = true;
  void *pmask = nullptr, *ptop = nullptr, *wk = nullptr;
  bool q = false;           // q-gram path in use
  uint32_t ts = 0, use3 = 0, use4 = 0, use5 = 0, kq = 0, mq = 0;
  size_t n_qpat = 0, n_grams = 0, n_keys = 0;
  void *tab = nullptr, *ent = nullptr, *qmask = nullptr, *qpm = nullptr, *qbits = nullptr;
  void* m16 = nullptr;      // every q-gram pattern m <= 16: 16-bit masks [pattern][rows] for LDS
  uint32_t m16_words = 0;
  ~PfTables() {
    for (void* p : {pmask, ptop, wk, tab, ent, qmask, qpm, qbits, m16})
      if (p) (void)hipFree(p);
  }
};

struct Engine {
  int device = 0;
  hipStream_t stream = nullptr;
  // prefix cache: level-1 build beside the sampled-level counts (lowest priority; created with the
  // engine's tables; a streaming worker's ScratchSet has its own)
  hipStream_t aux_stream = nullptr;
  fac_config cfg{};
  bool case_insensitive = false;
  bool has_limits = false;
  DevLimits limits{LIM_NONE, LIM_NONE, LIM_NONE, LIM_NONE, LIM_NONE};
  bool has_pattern_limits = false;
  uint32_t max_edits_fast = 0;
  uint32_t mef = 255;
  uint64_t beam_width = 0;
  bool has_auto_beam = false;
  uint64_t ab_budget = 0, ab_width = 0;
  float p_ins, p_del, p_sub, p_swp, min_sym;
  // host tables
  std::vector<HostNode> nodes;
  std::vector<DevNode> dnodes;
  std::vector<uint2> out_range;
  std::vector<int32_t> node_pidx;
  std::vector<DevEdge> edges;
  std::vector<uint32_t> out_pat;
  std::vector<uint4> sb_bits;
  std::vector<uint4> sb_edge;
  std::vector<uint4> gt;  // goto table (cuckoo slots)
  uint32_t gt_mask = 0;
  uint64_t gt_seed1 = 0, gt_seed2 = 0;
  bool gt_fast = false;
  std::vector<uint4> aux;  // SearchParams::aux
  std::vector<uint32_t> pat_bytes;  // Pattern::len (bytes, structs.rs:628-630) for ranking
  std::vector<DevPattern> pats;
  std::vector<float> sim_ascii;
  std::vector<uint64_t> sim_keys;
  std::vector<float> sim_vals;
  uint32_t max_degree = 0;
  uint32_t max_degree_nonroot = 0;
  uint32_t max_glen = 0;
  uint64_t max_match_graphemes = 0;
  bool window_skip = false;
  uint32_t first_bits[4] = {0, 0, 0, 0}, second_bits[4] = {0, 0, 0, 0};
  // prefilter (prefilter.rs:69-93)
  bool bitap_ok = false;
  float edit_cost_mult = 0.f;
  uint8_t ascii_id[128] = {0};
  std::vector<std::pair<std::u32string, uint32_t>> symbol_ids;  // sorted by key
  // multi-character mappings (builder.rs:383-442); has_map = the precomputed table is non-empty
  bool has_map = false;
  std::unordered_map<std::u32string, uint32_t, U32StrHash> gid_of;  // folded grapheme -> id (1-based)
  std::vector<uint32_t> edge_gid;   // per edge
  uint32_t ascii_gid[128] = {0};    // id of each (folded) ASCII byte, 0 = none
  std::vector<uint2> map_range;     // per node
  std::vector<uint4> map_ent;
  std::vector<uint32_t> map_hay;
  uint32_t max_map = 0;             // most mapping transitions at one node (<= 64)
  uint32_t alphabet = 0;
  std::vector<uint32_t> bp_m;
  std::vector<float> bp_weight;
  std::vector<int64_t> bp_k_limit;  // -1 = None
  std::vector<uint64_t> bp_mask;    // P x (alphabet+1)
  // device copies
  DevNode* d_nodes = nullptr;
  DevEdge* d_edges = nullptr;
  uint32_t* d_out_pat = nullptr;
  uint2* d_out_range = nullptr;
  int32_t* d_pidx = nullptr;
  uint4* d_sb_edge = nullptr;
  uint4* d_gt = nullptr;
  uint4* d_aux = nullptr;
  uint32_t* d_pat_bytes = nullptr;
  DevPattern* d_pats = nullptr;
  float* d_sim_ascii = nullptr;
  uint64_t* d_sim_keys = nullptr;
  float* d_sim_vals = nullptr;
  uint8_t* d_ascii_id = nullptr;
  uint32_t* d_edge_gid = nullptr;
  uint32_t* d_ascii_gid = nullptr;
  uint2* d_map_range = nullptr;
  uint4* d_map_ent = nullptr;
  uint32_t* d_map_hay = nullptr;
  std::mutex mu;  // guards lazily grown scratch below
  // per-engine device scratch of the search launcher, reused across calls by whichever call holds
  // scratch_mu (a concurrent call on the same engine allocates its own)
  mutable std::mutex scratch_mu;
  mutable std::mutex pf_mu;  // guards pf_cache
  mutable std::vector<std::unique_ptr<PfTables>> pf_cache;
  static constexpr int kScratch = 64;
  mutable void* scratch_p[kScratch] = {};
  mutable size_t scratch_n[kScratch] = {};
};

struct Haystack {
  bool ascii = true;
  uint64_t len = 0;  // bytes
  uint64_t n = 0;    // graphemes
  // shard of a larger haystack (fac_haystack_stage_shard): output offsets are shifted by `base`
  // (global byte of local byte 0); `open_end`: the text continues past the resident bytes, which
  // hold only the halo (j == n / end-of-text logic never applies); start windows [0, owned)
  uint64_t base = 0;
  bool open_end = false;
  uint64_t owned = UINT64_MAX;
  // key partition (fac_haystack_set_key_partition): only the start windows whose first two
  // characters hash to part (of parts) are searched -- a strong-scaling split of one haystack that
  // keeps every window of a prefix on one GPU, so each GPU's prefix cache covers whole keys
  uint32_t kparts = 1, kpart = 0;
  uint8_t* d_utf8 = nullptr;
  bool own_utf8 = true;          // false: the caller's device bytes (fac_haystack_stage_device)
  uint32_t* d_text32 = nullptr;  // Unicode only
  uint64_t* d_off = nullptr;     // Unicode only
  uint64_t off_cap = 0;          // entries d_off / d_text32 hold (kept when staged again)
  void* d_stage = nullptr;       // staging scratch (stage_device), kept when staged again
  size_t stage_cap = 0;
  // host copies, fetched from the device on first use (ensure_host): the UTF-8 bytes (pre-filter
  // slices re-decide is_ascii; host transcodes) and the grapheme byte starts (Unicode only)
  mutable std::vector<uint8_t> utf8;
  mutable std::vector<uint64_t> starts;
  mutable bool host_ready = false;
  mutable std::mutex host_mu;
  mutable std::vector<uint8_t> sym;  // prefilter symbol ids per grapheme (Unicode only, lazy)
  mutable bool sym_ready = false;
  mutable uint32_t* d_gid = nullptr;  // grapheme ids (Unicode, engines with mappings; lazy)
  mutable const void* gid_engine = nullptr;
  int device = 0;
  uint64_t failed_n = 0;  // graphemes counted by a failed restage (stage_haystack_device), for the error
};

// Where a search delivers its records: a host vector (internal callers), a pooled pinned host
// buffer handed to the C ABI caller (fac_search_staged / fac_search_raw: no page faults on the
// D2H, result_alloc below), or the caller's device buffer (fac_search_staged_device: records stay
// in HBM for the RCCL gather). `n` counts every record; with a device buffer only the first
// dev_cap are written.
struct MatchSink {
  std::vector<fac_match>* vec = nullptr;
  fac_match* pinned = nullptr;
  uint64_t pinned_cap = 0;
  fac_match* dev = nullptr;
  uint64_t dev_cap = 0;
  uint64_t n = 0;
};
// result buffers (api.cpp): large ones come from a pool of pinned host buffers that
// fac_matches_free returns to the pool; small ones are malloc'd. result_free takes either.
fac_match* result_alloc(uint64_t n_records);
void result_free(void* p);
int sink_append_device(MatchSink& s, const fac_match* d_src, uint64_t cnt, hipStream_t stream, std::string& err);
int sink_append_host(MatchSink& s, const fac_match* src, uint64_t cnt, hipStream_t stream, std::string& err);

// builder.cpp
int build_engine(const fac_pattern* pats, uint64_t n, const fac_config* cfg, Engine& e, std::string& err);
// a node's children (folded graphemes, insertion order) -> their transitions-map iteration order
std::vector<uint32_t> transitions_order(const std::vector<std::u32string>& children);
// search_kernels.hip
int launch_search(const Engine& e, const Haystack& h, const std::vector<SegDesc>& segs, float thr,
                  hipStream_t stream, std::vector<fac_match>& out, fac_stats* stats, std::string& err);
// ab_prefix: the running auto-beam total (queue.len() summed) of the windows before this call's
// first window, for a shard of one haystack (search.rs:1096-1103); 0 for a whole search
int launch_search_sink(const Engine& e, const Haystack& h, const std::vector<SegDesc>& segs, float thr,
                       hipStream_t stream, uint64_t ab_prefix, MatchSink& sink, fac_stats* stats, std::string& err);
// auto-beam pass 1 alone: sum of queue.len() over the windows of `segs` searched unbeamed
int auto_beam_total(const Engine& e, const Haystack& h, const std::vector<SegDesc>& segs, float thr,
                    hipStream_t stream, uint64_t& total, std::string& err);
// diagnostics knobs: FAC_* environment variables are honoured only with FAC_DIAGNOSTICS=1 set, so
// a stray variable in a user's environment never changes the search path
const char* diag_env(const char* name);
// the host copies of a staged haystack (Haystack::utf8, ::starts), fetched once from the device
int ensure_host(const Haystack& h, std::string& err);
// largest grapheme count a haystack may have (u32::MAX, search.rs:198-201; lowered only by the
// diagnostics knob FAC_GRAPHEME_LIMIT so tests can reach SearchError::HaystackTooLarge)
uint64_t grapheme_limit();
// A set of lazily grown device scratch buffers for the search launcher. The engine owns one (leased
// by whichever call gets it first); a streaming search owns one per in-flight window, bound to the
// worker thread that searches it (scratch_bind) so concurrent windows never hipMalloc per call.
struct ScratchSet {
  static constexpr int kSlots = 64;
  std::mutex mu;
  void* p[kSlots] = {};
  size_t n[kSlots] = {};
  hipStream_t aux = nullptr;  // this set's low-priority second stream (prefix-cache level-1 build)
};
void scratch_bind(ScratchSet* s);  // this thread's searches use `s` (nullptr: the engine's)
void scratch_free(ScratchSet& s);
// Short-lived call scratch (rank kernels, stream-window record buffers), one process-wide pool: a
// block given back on stream s is handed out again only for work on s (same device), whose order
// makes the reuse safe without the device-wide synchronisation a hipFree implies (a per-call
// hipMalloc/hipFree stalled every other stream once per stream window). At most 2 GiB / 64 blocks
// are kept (oldest freed first); fac_trim_scratch / fac_engine_free release them.
void* call_scratch_take(size_t bytes, hipStream_t s, hipError_t* e);
void call_scratch_give(void* p, hipStream_t s);
void call_scratch_trim();                         // frees every kept block
void call_scratch_release_stream(hipStream_t s);  // before the library destroys stream s

// stream.cpp: the WindowReader state (stream.rs:77-159), the windows in flight and the matches
// ready to hand out. Windows are cut on the host and searched by `depth` worker threads, each with
// its own HIP stream and scratch: window k + 1's upload, segmentation and search overlap window k's
// (double buffering); results are handed out in window order.
struct StreamTask;
struct StreamWorker;
struct StreamCore {
  const Engine* e = nullptr;
  float threshold = 0.f;
  uint64_t window = 256 * 1024;  // DEFAULT_WINDOW (stream.rs:61)
  uint64_t overlap = 1;
  std::vector<uint8_t> buf;
  uint64_t base = 0, total = 0;
  uint64_t carry = 0;  // bytes the last window left in the buffer (its text after the commit point)
  uint64_t valid_end = 0;  // stream offset up to which the bytes are known valid UTF-8 (a character boundary)
  bool done = false;
  StreamTask* pending = nullptr;  // windows cut but not yet dispatched (one batch)
  std::vector<fac_match> ready;
  std::vector<uint8_t> ready_text;  // matched bytes of `ready`, concatenated
  static constexpr uint32_t depth = 2;
  StreamWorker* workers[depth] = {};
  std::vector<StreamTask*> inflight;  // window order
  uint64_t seq = 0;
  uint64_t handed = 0;  // commit point of the last window whose matches were handed out
  int failed = 0;
  std::string fail_msg;
};

StreamCore* stream_open(const Engine& e, float threshold, uint64_t window);
int stream_feed(StreamCore& s, const uint8_t* data, uint64_t len, bool eof, std::string& err);
void stream_close(StreamCore* s);
uint64_t stream_committed(const StreamCore& s);  // commit point of the windows handed out so far
// staging of the bytes at h.d_utf8 on the device (stage_kernels.hip): mode -2 checks the UTF-8 and
// decides is_ascii, 0 stages Unicode graphemes, 1 ASCII (asynchronous after its count sync)
int stage_device(const Engine& e, Haystack& h, hipStream_t st, std::string& err, int mode);
// graphemes of a staged haystack that start before byte b (a grapheme boundary), synchronously on st
int graphemes_before(const Haystack& h, uint64_t b, hipStream_t st, uint64_t& out, std::string& err);
void ensure_symbols(const Engine& e, const Haystack& h);
int apply_matches(const Engine& e, std::vector<fac_match>& v, int order, int overlap, const uint64_t* unique_ids,
                  std::string& err);
// stream.rs window_matches' tail on the device (rank_kernels.hip): the n raw records of one window
// at d_a (d_b: scratch of n) ranked sorted().non_overlapping(), those starting before `commit` bytes
// into the window (which starts at byte byte_base of the staged text) rebased to stream offset `base`
// and written to d_out; *n_owned their count (FAC_E_OUTPUT_CAPACITY if it exceeds cap)
int window_owned_device(const Engine& e, fac_match* d_a, fac_match* d_b, uint64_t n, uint64_t byte_base, uint64_t commit,
                        uint64_t base, hipStream_t s, fac_match* d_out, uint64_t cap, uint64_t* n_owned, std::string& err);
// A stream window of a batch: its text starts at staged byte byte_base, it owns the matches starting
// before commit bytes into it, and byte_base maps to stream offset base. A batch's ASCII segments
// carry their window in the bits of SegDesc::byte_base from kWinTagShift up, so every record's start
// and end come back tagged (the kernels only add byte offsets to byte_base for ASCII text).
struct WinOwn {
  uint64_t byte_base, commit, base;
};
constexpr uint32_t kWinTagShift = 40;
void windows_owned_host(const Engine& e, std::vector<fac_match>& recs, const std::vector<WinOwn>& wins,
                        std::vector<fac_match>& out);
// api.cpp: a batch of stream windows (g_begin, g_end, commit_bytes, base) x n of a whole staged ASCII
// haystack searched in one pass; FAC_E_UNSUPPORTED when the batch does not qualify (see there)
int stream_windows_batch(const Engine& e, const Haystack& h, const uint64_t* wins, uint64_t n_windows, float threshold,
                         bool prefilter, hipStream_t st, std::vector<fac_match>& owned, fac_stats* stats, std::string& err);
// merged bitap windows (prefilter.rs:319-342) of a text view of a staged haystack (view.ascii:
// bytes [text_base, text_base + n) of h.d_utf8; else graphemes [text_base, text_base + n)); windows
// in the view's local grapheme coordinates
// diagnostics: beam_select(_lds) alone on key arrays (tests; fac_diag_beam_select)
int diag_beam_select(const float* keys, const uint64_t* offs, uint64_t count, uint32_t bw, int32_t lds,
                     int32_t sel_limit, uint32_t* perm, std::string& err);
int prefilter_windows(const Engine& e, const Haystack& h, const SegDesc& view, const std::vector<uint32_t>& ks,
                      hipStream_t stream, std::vector<std::pair<uint64_t, uint64_t>>& windows, fac_stats* stats,
                      std::string& err);
// the same for a batch of stream windows of the view (wins: [lo, hi) text positions, sorted, each
// overlapping only its neighbours): one scan of the view, every window's merged bitap windows as if
// its text were searched alone; run_win = each merged window's stream window. FAC_E_UNSUPPORTED
// when the tables need the packed full scan.
int prefilter_windows_ex(const Engine& e, const Haystack& h, const SegDesc& view, const std::vector<uint32_t>& ks,
                         hipStream_t stream, const std::vector<std::pair<uint64_t, uint64_t>>* wins,
                         std::vector<std::pair<uint64_t, uint64_t>>& windows, std::vector<uint32_t>* run_win,
                         fac_stats* stats, std::string& err);
// force_ascii: -1 decide from the bytes (search.rs:196), 0 Unicode graphemes, 1 ASCII bytes (a
// shard of a haystack whose global is_ascii is already known)
int stage_haystack(const Engine& e, const uint8_t* utf8, uint64_t len, Haystack& h, std::string& err,
                   int force_ascii = -1, hipStream_t stream = nullptr);
// search_raw's staging of bytes already in device memory (borrowed, not copied): the UTF-8 check,
// is_ascii, segmentation and folding on the device; h may hold buffers of an earlier staging.
// mode -2: decide is_ascii from the bytes; 1 / 0: ASCII / Unicode graphemes as given (a shard of a
// haystack whose global is_ascii is known; Unicode bytes are UTF-8 checked)
int stage_haystack_device(const Engine& e, const uint8_t* d_utf8, uint64_t len, Haystack& h, std::string& err,
                          hipStream_t stream, int mode = -2);
// start byte of the n-th grapheme counted from the end of s[0, len) (UAX #29, the whole text's
// segmentation; stream.rs:134-139 grapheme_indices(true).rev().nth(n - 1)); false if it has fewer
bool nth_grapheme_from_end(const uint8_t* s, uint64_t len, uint64_t n, uint64_t& off);
// shard planning (unicode.cpp): p is a grapheme boundary whose segmentation does not depend on
// anything before it (previous char ASCII and not CR, char at p neither Extend, ZWJ nor SpacingMark;
// or the char at p starts a cluster in every context: GCB Other, not ExtPict, no InCB class, and
// the previous char is not Prepend)
bool safe_cut(const uint8_t* s, uint64_t n, uint64_t p);
// str::is_ascii (search.rs:196), eight bytes at a time
bool ascii_only(const uint8_t* s, uint64_t n);
void free_haystack(Haystack& h);
int upload_engine(Engine& e, std::string& err);
void free_engine_device(Engine& e);

}  // namespace fac
