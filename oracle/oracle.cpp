// oracle/oracle.cpp — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from the
// product path (`fuzzy-aho-corasick-rs_amd/`). Only `tests/`, `__graft_entry__.smoke()` and
// `bench.py`'s `cpu_baseline` leg may load this library, and only as the checker / CPU baseline.
//
// A single-threaded CPU restatement of the reference crate's hot path
// (kakserpom/fuzzy-aho-corasick-rs v0.5.0, mounted at /root/reference), following the cited lines:
//
//   builder   src/builder.rs:181-484   trie, fail-link output merge, reach-based prune coefficients,
//                                      effective limits, max_edits_fast
//   similarity src/builder.rs:492-526, src/structs.rs:30-92 (default table, get, max_off_diagonal)
//   search    src/search.rs:418-1119   per-start-window FIFO BFS with dedup, node ceiling, emission,
//                                      exact / substitution / swap / insertion / deletion fan-out,
//                                      beam prune, auto-beam
//   limits    src/search.rs:84-169     within_limits_* family
//   prefilter src/prefilter.rs:161-435 bitap build, transcode, k_for, window merge + re-search
//
// Deliberate, documented deviations (see DESIGN.md "Oracle"):
//   * Edge order. The reference iterates `Node.transitions` in hashbrown order (builder.rs:336-341),
//     which cannot be reproduced without a Rust toolchain. Edges here are kept in insertion order
//     (order in which the child grapheme was first inserted). Unbeamed match sets do not depend on
//     it; edit-count tie-breaks and beam ties do.
//   * Beam ties. `select_nth_unstable_by` (search.rs:584) leaves ties at the cut unspecified. The
//     oracle uses the canonical rule: keep the `bw` smallest by (penalty total order, queue
//     position) and keep the survivors in their queue order — one legal outcome of the reference's
//     partial selection.
//   * Output order: sorted by (start, end, pattern) instead of hash-bucket order (the reference
//     documents raw output as unordered, search.rs:1105-1110).
//
// Grapheme segmentation and case folding are NOT done here: the caller (Python test harness, using
// the `regex` module's UAX #29 `\X`) passes already-segmented, already-folded graphemes, which keeps
// this restatement independent of the product's generated Unicode tables.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace {

constexpr int LIM_NONE = -1;

struct Limits {  // FuzzyLimits (structs.rs:293-299); -1 = None
  int ins = LIM_NONE, del = LIM_NONE, sub = LIM_NONE, swp = LIM_NONE, edits = LIM_NONE;
};

struct Pattern {  // structs.rs:598-610 (only what the hot path reads)
  uint32_t glen = 0;
  float weight = 1.f;
  bool has_limits = false;
  Limits lim;
  std::vector<std::u32string> graphemes;  // folded graphemes
};

struct Edge {  // structs.rs:186-229
  uint32_t first_char;
  uint32_t next;
  bool single_byte;
};

struct Node {  // structs.rs:249-281
  std::vector<Edge> edges;
  std::vector<uint32_t> output;
  float prune_len = 0.f, prune_lw = 0.f;
  int64_t pattern_index = -1;
  uint32_t fail = 0;
  std::map<std::u32string, uint32_t> transitions;  // lookup only; iteration uses `order`
  std::vector<std::u32string> order;               // insertion order of transition keys
};

struct Similarity {  // structs.rs:9-14, 30-54, 82-92
  float ascii[128][128];
  std::map<std::pair<uint32_t, uint32_t>, float> map;
  float get(uint32_t a, uint32_t b) const {
    if (a < 128 && b < 128) return ascii[a][b];
    auto it = map.find({a, b});
    return it == map.end() ? 0.f : it->second;
  }
  float max_off_diagonal() const {  // structs.rs:61-76
    float m = 0.f;
    for (int i = 0; i < 128; ++i)
      for (int j = 0; j < 128; ++j)
        if (i != j) m = std::fmax(m, ascii[i][j]);
    for (auto& kv : map)
      if (kv.first.first != kv.first.second) m = std::fmax(m, kv.second);
    return m;
  }
};

struct MapT {  // MappingTransition (structs.rs:235-242)
  std::vector<std::u32string> hay;  // haystack graphemes to consume (folded)
  uint32_t next;                    // node reached by the pattern-side walk
  float penalty;                    // substitution * (1 - score)
};

struct Engine {
  std::vector<Node> nodes;
  // multi-character mappings: rules as configured (folded sides, score), and the precomputed
  // per-node transitions (builder.rs:383-442); has_mappings = !self.mappings.is_empty()
  std::vector<std::tuple<std::vector<std::u32string>, std::vector<std::u32string>, float>> map_rules;
  std::vector<std::vector<MapT>> mappings;
  bool has_mappings = false;
  std::vector<Pattern> patterns;
  Similarity sim;
  bool has_limits = false;
  Limits limits;  // effective limits (builder.rs:289-329)
  float p_ins, p_del, p_sub, p_swp;
  bool case_insensitive = false;
  bool has_pattern_limits = false;
  uint32_t max_edits_fast = 0;
  size_t beam_width = 0;  // 0 = None
  bool has_auto_beam = false;
  size_t ab_budget = 0, ab_width = 0;
  int beam_rule = 2;  // g_beam_rule at build time
  float min_symbol_similarity = 0.f;
  // prefilter (prefilter.rs:69-93)
  bool bitap_ok = false;
  std::map<std::u32string, uint32_t> symbol_ids;
  uint8_t ascii_id[128];
  float edit_cost_mult = 0.f;
  struct BP { uint32_t m; float weight; std::vector<uint64_t> mask; bool has_k_limit; size_t k_limit; };
  std::vector<BP> bitap;
};

struct Match {
  uint64_t start, end;
  uint32_t pattern;
  float similarity;
  uint8_t ins, del, sub, swp, edits;
};

// Restatement modes (orc_set_modes). Edge order: 0 = insertion order, 1 = the iteration order of
// the reference's `FxHashMap<String, u32>` transitions (FxHasher + hashbrown, below). Beam rule:
// 0 = canonical (penalty, queue position), 1 = the same with ties at the cut broken towards the
// LATEST queue position (tie-sensitivity diagnostic only), 2 = core's select_nth_unstable_by, 3 = the
// same with round 3's defective early exit (stop at index == mid after the equal-to-ancestor split;
// diagnostics only: profiles/beam_ties.py measures what the fix changed).
int g_edge_order = 1;
int g_beam_rule = 2;
int g_sel_limit = 16;  // select.rs partition_at_index_loop's round limit (tests lower it to reach median_of_medians)

// ------------------------------------------------------------------------------------------
// FxHashMap<String, u32> iteration order (builder.rs:208-214 inserts, :336-342 iterates)
// ------------------------------------------------------------------------------------------
// The crate's own FxHasher (structs.rs:95-156) over `impl Hash for str` = write(bytes) then
// write_u8(0xff) (core::hash::Hasher::write_str).
uint64_t fx_hash_str(const std::string& s) {
  const uint64_t K = 0x517cc1b727220a95ull;
  uint64_t h = 0;
  auto add = [&](uint64_t i) { h = (((h << 5) | (h >> 59)) ^ i) * K; };
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data());
  size_t n = s.size();
  while (n >= 8) {
    uint64_t w = 0;
    for (int b = 0; b < 8; ++b) w |= (uint64_t)p[b] << (8 * b);
    add(w);
    p += 8;
    n -= 8;
  }
  if (n >= 4) {
    uint32_t w = 0;
    for (int b = 0; b < 4; ++b) w |= (uint32_t)p[b] << (8 * b);
    add(w);
    p += 4;
    n -= 4;
  }
  for (size_t b = 0; b < n; ++b) add(p[b]);
  add(0xff);
  return h;
}

std::string utf8_of(const std::u32string& g) {
  std::string o;
  for (char32_t c : g) {
    if (c < 0x80) o += (char)c;
    else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 0x3F)); }
    else if (c < 0x10000) {
      o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F));
    } else {
      o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 0x3F));
      o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F));
    }
  }
  return o;
}

// hashbrown's RawTable as std's HashMap uses it on x86-64 (SSE2 groups of 16 control bytes),
// restricted to what an insert-only map does: `insert` = reserve(1) (grow when growth_left == 0,
// to capacity max(items + 1, full_capacity + 1), re-inserting the old buckets in index order) then
// the first EMPTY control byte along the triangular group probe from h1 = hash & bucket_mask
// (fix_insert_slot for tables smaller than a group). Iteration visits full buckets in index order.
struct SwissOrder {
  std::vector<int> slot;       // bucket -> item (-1 = EMPTY)
  std::vector<uint64_t> hash;  // item -> hash
  size_t items = 0, growth_left = 0;
  size_t buckets() const { return slot.size(); }
  static size_t cap_of_mask(size_t mask) { return mask < 8 ? mask : ((mask + 1) / 8) * 7; }
  static size_t buckets_for(size_t cap) {
    if (cap < 8) return cap < 4 ? 4 : 8;  // (String, u32) entries: hashbrown's small-table minimum is 3
    size_t adj = cap * 8 / 7, b = 1;
    while (b < adj) b <<= 1;
    return b;
  }
  bool ctrl_empty(size_t i) const {  // control byte i of [0, buckets + 16): real, padding or mirror
    const size_t nb = buckets(), m = std::max<size_t>(nb, 16);
    if (i < nb) return slot[i] < 0;
    if (i >= m) return slot[i - m] < 0;
    return true;  // the EMPTY padding of a table smaller than one group
  }
  size_t find_insert_slot(uint64_t h) const {
    const size_t mask = buckets() - 1;
    size_t pos = (size_t)h & mask, stride = 0;
    for (;;) {
      for (size_t bit = 0; bit < 16; ++bit)
        if (ctrl_empty(pos + bit)) {
          size_t idx = (pos + bit) & mask;
          if (slot[idx] >= 0)  // fix_insert_slot: first EMPTY of the aligned group at 0
            for (idx = 0; slot[idx] >= 0; ++idx) {}
          return idx;
        }
      stride += 16;
      pos = (pos + stride) & mask;
    }
  }
  void insert(uint64_t h) {
    const int id = (int)hash.size();
    hash.push_back(h);
    if (growth_left == 0) {
      const size_t full_cap = slot.empty() ? 0 : cap_of_mask(buckets() - 1);
      const size_t nb = buckets_for(std::max(items + 1, full_cap + 1));
      std::vector<int> old;
      old.swap(slot);
      slot.assign(nb, -1);
      for (int it : old)
        if (it >= 0) slot[find_insert_slot(hash[(size_t)it])] = it;
      growth_left = cap_of_mask(nb - 1) - items;
    }
    slot[find_insert_slot(h)] = id;
    --growth_left;
    ++items;
  }
  std::vector<int> iteration_order() const {
    std::vector<int> o;
    for (int it : slot)
      if (it >= 0) o.push_back(it);
    return o;
  }
};

// The children of one node in the reference's `transitions.iter()` order, given their insertion order.
std::vector<std::u32string> hashbrown_order(const std::vector<std::u32string>& inserted) {
  SwissOrder t;
  for (auto& g : inserted) t.insert(fx_hash_str(utf8_of(g)));
  std::vector<std::u32string> o;
  for (int it : t.iteration_order()) o.push_back(inserted[(size_t)it]);
  return o;
}

// ------------------------------------------------------------------------------------------
// core::slice::select_nth_unstable_by (Rust >= 1.81: introselect with the ipnsort partition),
// restated for the beam (search.rs:584-587). is_less(a, b) = a.penalties.total_cmp(&b.penalties)
// == Less. core/src/slice/select.rs: partition_at_index, partition_at_index_loop,
// median_of_medians, median_of_ninthers, ninther, median_idx, min_index, max_index;
// core/src/slice/sort/shared/pivot.rs: choose_pivot, median3_rec, median3;
// core/src/slice/sort/unstable/quicksort.rs: partition, partition_lomuto_branchless_cyclic
// (State is 28 bytes <= 96); core/src/slice/sort/shared/smallsort.rs: insertion_sort_shift_left.
// ------------------------------------------------------------------------------------------
namespace rsel {
template <typename T, typename L>
void insertion_sort_shift_left(T* v, size_t len, size_t offset, L& is_less) {
  for (size_t i = offset; i < len; ++i) {
    if (!is_less(v[i], v[i - 1])) continue;
    T tmp = v[i];
    size_t j = i;
    for (;;) {
      v[j] = v[j - 1];
      --j;
      if (j == 0 || !is_less(tmp, v[j - 1])) break;
    }
    v[j] = tmp;
  }
}
template <typename T, typename L>
size_t median3(const T* v, size_t a, size_t b, size_t c, L& is_less) {
  const bool x = is_less(v[a], v[b]), y = is_less(v[a], v[c]);
  if (x == y) {
    const bool z = is_less(v[b], v[c]);
    return (z ^ x) ? c : b;
  }
  return a;
}
template <typename T, typename L>
size_t median3_rec(const T* v, size_t a, size_t b, size_t c, size_t n, L& is_less) {
  if (n * 8 >= 64) {
    const size_t n8 = n / 8;
    a = median3_rec(v, a, a + n8 * 4, a + n8 * 7, n8, is_less);
    b = median3_rec(v, b, b + n8 * 4, b + n8 * 7, n8, is_less);
    c = median3_rec(v, c, c + n8 * 4, c + n8 * 7, n8, is_less);
  }
  return median3(v, a, b, c, is_less);
}
template <typename T, typename L>
size_t choose_pivot(const T* v, size_t len, L& is_less) {  // len >= 8
  const size_t d8 = len / 8, a = 0, b = d8 * 4, c = d8 * 7;
  if (len < 64) return median3(v, a, b, c, is_less);
  return median3_rec(v, a, b, c, d8, is_less);
}
// partition_lomuto_branchless_cyclic over w[0..m) against `pivot`: elements are taken in the order
// w[1], ..., w[m-1], w[0] (w[0] is held in the gap value); each is written to w[num_lt] and the
// previous occupant of w[num_lt] moves into the gap left by the previous element.
template <typename T, typename L>
size_t lomuto_cyclic(T* w, size_t m, const T& pivot, L& is_less) {
  if (m == 0) return 0;
  const T gap_value = w[0];
  size_t gap = 0, num_lt = 0;
  for (size_t r = 1; r < m; ++r) {
    const bool lt = is_less(w[r], pivot);
    w[gap] = w[num_lt];
    w[num_lt] = w[r];
    gap = r;
    num_lt += lt;
  }
  const bool lt = is_less(gap_value, pivot);
  w[gap] = w[num_lt];
  w[num_lt] = gap_value;
  return num_lt + lt;
}
template <typename T, typename L>
size_t partition(T* v, size_t len, size_t pivot, L& is_less) {
  if (len == 0) return 0;
  std::swap(v[0], v[pivot]);
  const T p = v[0];
  const size_t num_lt = lomuto_cyclic(v + 1, len - 1, p, is_less);
  std::swap(v[0], v[num_lt]);
  return num_lt;
}
template <typename T, typename L>
size_t min_index(const T* v, size_t len, L& is_less) {
  size_t acc = 0;
  for (size_t i = 1; i < len; ++i)
    if (is_less(v[i], v[acc])) acc = i;
  return acc;
}
template <typename T, typename L>
size_t max_index(const T* v, size_t len, L& is_less) {
  size_t acc = 0;
  for (size_t i = 1; i < len; ++i)
    if (is_less(v[acc], v[i])) acc = i;
  return acc;
}
template <typename T, typename L>
size_t median_idx(const T* v, L& is_less, size_t a, size_t b, size_t c) {
  if (is_less(v[c], v[a])) std::swap(a, c);
  if (is_less(v[c], v[b])) return c;
  if (is_less(v[b], v[a])) return a;
  return b;
}
template <typename T, typename L>
void ninther(T* v, L& is_less, size_t a, size_t b, size_t c, size_t d, size_t e, size_t f, size_t g, size_t h,
             size_t i) {
  b = median_idx(v, is_less, a, b, c);
  h = median_idx(v, is_less, g, h, i);
  if (is_less(v[h], v[b])) std::swap(b, h);
  if (is_less(v[f], v[d])) std::swap(d, f);
  if (is_less(v[e], v[d])) {
    // the middle triple's median is d
  } else if (is_less(v[f], v[e])) {
    d = f;
  } else {
    if (is_less(v[e], v[b])) std::swap(v[e], v[b]);
    else if (is_less(v[h], v[e])) std::swap(v[e], v[h]);
    return;
  }
  if (is_less(v[d], v[b])) d = b;
  else if (is_less(v[h], v[d])) d = h;
  std::swap(v[d], v[e]);
}
template <typename T, typename L>
void median_of_medians(T* v, size_t len, L& is_less, size_t k);
template <typename T, typename L>
size_t median_of_ninthers(T* v, size_t len, L& is_less) {
  const size_t frac = len <= 1024 ? len / 12 : (len <= 128 * 1024 ? len / 64 : len / 1024);
  const size_t pivot = frac / 2, lo = len / 2 - pivot, hi = frac + lo, gap = (len - 9 * frac) / 4;
  size_t a = lo - 4 * frac - gap, b = hi + gap;
  for (size_t i = lo; i < hi; ++i) {
    ninther(v, is_less, a, i - frac, b, a + 1, i, b + 1, a + 2, i + frac, b + 2);
    a += 3;
    b += 3;
  }
  median_of_medians(v + lo, frac, is_less, pivot);
  return partition(v, len, lo + pivot, is_less);
}
template <typename T, typename L>
void median_of_medians(T* v, size_t len, L& is_less, size_t k) {
  for (;;) {
    if (len <= 16) {
      if (len >= 2) insertion_sort_shift_left(v, len, 1, is_less);
      return;
    }
    if (k == len - 1) { std::swap(v[max_index(v, len, is_less)], v[k]); return; }
    if (k == 0) { std::swap(v[min_index(v, len, is_less)], v[k]); return; }
    const size_t p = median_of_ninthers(v, len, is_less);
    if (p == k) return;
    if (p > k) {
      len = p;
    } else {
      v += p + 1;
      len -= p + 1;
      k -= p + 1;
    }
  }
}
template <typename T, typename L>
void partition_at_index_loop(T* v, size_t len, size_t index, L& is_less) {
  int limit = g_sel_limit;
  const T* ancestor = nullptr;
  T anc_copy{};
  for (;;) {
    if (len <= 16) {
      if (len >= 2) insertion_sort_shift_left(v, len, 1, is_less);
      return;
    }
    if (limit == 0) {
      median_of_medians(v, len, is_less, index);
      return;
    }
    --limit;
    const size_t pivot_pos = choose_pivot(v, len, is_less);
    if (ancestor && !is_less(*ancestor, v[pivot_pos])) {
      auto le = [&](const T& a, const T& b) { return !is_less(b, a); };
      const size_t mid = partition(v, len, pivot_pos, le) + 1;
      if (index < mid || (g_beam_rule == 3 && index == mid)) return;  // core: `if mid > index { return; }`
      v += mid;
      len -= mid;
      index -= mid;
      ancestor = nullptr;
      continue;
    }
    const size_t mid = partition(v, len, pivot_pos, is_less);
    if (mid < index) {
      anc_copy = v[mid];  // the pivot stays at v[mid] for the rest of the call
      ancestor = &anc_copy;
      v += mid + 1;
      len -= mid + 1;
      index -= mid + 1;
    } else if (mid > index) {
      len = mid;
    } else {
      return;
    }
  }
}
template <typename T, typename L>
void select_nth_unstable_by(T* v, size_t len, size_t index, L is_less) {  // partition_at_index
  if (index >= len) std::abort();
  if (index == len - 1) std::swap(v[max_index(v, len, is_less)], v[index]);
  else if (index == 0) std::swap(v[min_index(v, len, is_less)], v[index]);
  else partition_at_index_loop(v, len, index, is_less);
}
}  // namespace rsel

// ------------------------------------------------------------------------------------------
// Builder (builder.rs:181-484)
// ------------------------------------------------------------------------------------------
void default_similarity(Similarity& s) {  // builder.rs:492-526 + structs.rs:36-48
  for (int i = 0; i < 128; ++i)
    for (int j = 0; j < 128; ++j) s.ascii[i][j] = (i == j) ? 1.f : 0.f;
  const char* vowels = "aeiou";
  auto is_vowel = [&](char c) { return std::strchr(vowels, c) != nullptr; };
  for (char a = 'a'; a <= 'z'; ++a)
    for (char b = 'a'; b <= 'z'; ++b) {
      if (a == b) continue;
      if (is_vowel(a) && is_vowel(b)) s.ascii[(int)a][(int)b] = 0.6f;
      if (!is_vowel(a) && !is_vowel(b)) s.ascii[(int)a][(int)b] = 0.4f;
    }
  s.ascii['o']['0'] = 0.6f; s.ascii['0']['o'] = 0.6f;
  s.ascii['l']['1'] = 0.7f; s.ascii['1']['l'] = 0.7f;
  s.ascii['i']['1'] = 0.6f; s.ascii['1']['i'] = 0.6f;
  s.ascii['s']['5'] = 0.5f; s.ascii['5']['s'] = 0.5f;
}

size_t k_from_limits(const Limits& l, bool& bounded) {  // prefilter.rs:388-405
  bounded = true;
  if (l.edits != LIM_NONE) {
    bool swaps_forbidden = l.swp == 0;
    return swaps_forbidden ? (size_t)l.edits : 2 * (size_t)l.edits;
  }
  if (l.ins == LIM_NONE || l.del == LIM_NONE || l.sub == LIM_NONE || l.swp == LIM_NONE) {
    bounded = false;
    return 0;
  }
  return (size_t)l.ins + l.del + l.sub + 2 * (size_t)l.swp;
}

void build_bitap(Engine& e) {  // prefilter.rs:161-245
  e.bitap_ok = false;
  if (e.has_mappings) return;  // :162-165
  if (e.patterns.empty()) return;
  float max_sim = e.sim.max_off_diagonal();
  float p_sub_min = e.p_sub * (1.0f - max_sim);
  float mults[4] = {1.0f / e.p_ins, 1.0f / e.p_del, 1.0f / p_sub_min, 2.0f / e.p_swp};
  for (float m : mults)
    if (!std::isfinite(m) || m <= 0.0f) return;
  float ecm = 0.0f;
  for (float m : mults) ecm = std::fmax(ecm, m);  // fold(0.0, f32::max)
  e.edit_cost_mult = ecm;
  e.symbol_ids.clear();
  std::vector<std::vector<uint32_t>> pat_ids;
  e.bitap.clear();
  for (auto& p : e.patterns) {
    size_t m = p.graphemes.size();
    if (m == 0 || m > 63) return;
    std::vector<uint32_t> ids;
    for (auto& g : p.graphemes) {
      uint32_t next_id = (uint32_t)e.symbol_ids.size() + 1;
      auto it = e.symbol_ids.find(g);
      uint32_t id;
      if (it == e.symbol_ids.end()) { e.symbol_ids[g] = next_id; id = next_id; } else id = it->second;
      if (id > 255) return;
      ids.push_back(id);
    }
    Engine::BP bp;
    bp.m = (uint32_t)m;
    bp.weight = p.weight;
    const Limits* app = p.has_limits ? &p.lim : (e.has_limits ? &e.limits : nullptr);
    bp.has_k_limit = false;
    bp.k_limit = 0;
    if (app) {
      bool bounded;
      size_t k = k_from_limits(*app, bounded);
      if (bounded) { bp.has_k_limit = true; bp.k_limit = k; }
    }
    e.bitap.push_back(bp);
    pat_ids.push_back(ids);
  }
  for (int b = 0; b < 128; ++b) {
    uint32_t ch = (uint32_t)b;
    if (e.case_insensitive && ch >= 'A' && ch <= 'Z') ch += 32;
    std::u32string key(1, ch);
    auto it = e.symbol_ids.find(key);
    e.ascii_id[b] = it == e.symbol_ids.end() ? 0 : (uint8_t)it->second;
  }
  size_t alphabet = e.symbol_ids.size();
  for (size_t i = 0; i < e.bitap.size(); ++i) {
    e.bitap[i].mask.assign(alphabet + 1, 0);
    for (size_t k = 0; k < pat_ids[i].size(); ++k) e.bitap[i].mask[pat_ids[i][k]] |= 1ull << k;
  }
  e.bitap_ok = true;
}

void build(Engine& e) {
  auto& nodes = e.nodes;
  nodes.clear();
  nodes.emplace_back();
  for (size_t i = 0; i < e.patterns.size(); ++i) {  // builder.rs:195-237
    size_t cur = 0;
    for (auto& g : e.patterns[i].graphemes) {
      size_t next;
      auto it = nodes[cur].transitions.find(g);
      if (it != nodes[cur].transitions.end()) {
        next = it->second;
      } else {
        next = nodes.size();
        nodes[cur].transitions[g] = (uint32_t)next;
        nodes[cur].order.push_back(g);
        nodes.emplace_back();
      }
      if (nodes[next].pattern_index < 0) nodes[next].pattern_index = (int64_t)i;  // :227
      cur = next;
    }
    nodes[cur].output.push_back((uint32_t)i);  // :235
  }
  // fail links + output merge (builder.rs:239-276), BFS by depth
  std::vector<uint32_t> queue;
  for (auto& g : nodes[0].order) {
    uint32_t c = nodes[0].transitions[g];
    nodes[c].fail = 0;
    queue.push_back(c);
  }
  for (size_t qi = 0; qi < queue.size(); ++qi) {
    uint32_t current = queue[qi];
    for (auto& g : nodes[current].order) {
      uint32_t next = nodes[current].transitions[g];
      uint32_t fail = nodes[current].fail;
      while (fail != 0 && nodes[fail].transitions.find(g) == nodes[fail].transitions.end())
        fail = nodes[fail].fail;
      auto it = nodes[fail].transitions.find(g);
      uint32_t fallback = it == nodes[fail].transitions.end() ? 0 : it->second;
      nodes[next].fail = fallback;
      std::vector<uint32_t> fo = nodes[fallback].output;
      for (uint32_t entry : fo)
        if (std::find(nodes[next].output.begin(), nodes[next].output.end(), entry) ==
            nodes[next].output.end())
          nodes[next].output.push_back(entry);
      queue.push_back(next);
    }
  }
  // effective limits (builder.rs:289-329): e.has_limits/e.limits already hold the global limits
  e.has_pattern_limits = false;
  if (!e.has_limits) {
    Limits m;
    bool any = false;
    for (auto& p : e.patterns) {
      if (!p.has_limits) continue;
      any = true;
      if (p.lim.edits != LIM_NONE) m.edits = std::max(m.edits == LIM_NONE ? 0 : m.edits, p.lim.edits);
      if (p.lim.ins != LIM_NONE) m.ins = std::max(m.ins == LIM_NONE ? 0 : m.ins, p.lim.ins);
      if (p.lim.del != LIM_NONE) m.del = std::max(m.del == LIM_NONE ? 0 : m.del, p.lim.del);
      if (p.lim.sub != LIM_NONE) m.sub = std::max(m.sub == LIM_NONE ? 0 : m.sub, p.lim.sub);
      if (p.lim.swp != LIM_NONE) m.swp = std::max(m.swp == LIM_NONE ? 0 : m.swp, p.lim.swp);
    }
    if (any) { e.has_limits = true; e.limits = m; }
  }
  for (auto& p : e.patterns) e.has_pattern_limits |= p.has_limits;
  // edges (builder.rs:336-342): the transitions map's iteration order (or insertion order, mode 0)
  e.beam_rule = g_beam_rule;
  for (auto& nd : nodes) {
    nd.edges.clear();
    if (g_edge_order == 1) nd.order = hashbrown_order(nd.order);
    for (auto& g : nd.order) {
      uint32_t fc = g.empty() ? 0 : g[0];
      bool single = g.size() == 1 && g[0] < 0x80;  // g.len() == 1 (UTF-8 bytes)
      nd.edges.push_back({fc, nd.transitions[g], single});
    }
  }
  // reach fixpoint (builder.rs:348-381)
  size_t nn = nodes.size();
  std::vector<size_t> rl(nn, 0);
  std::vector<float> rw(nn, 0.f);
  for (size_t i = 0; i < nn; ++i)
    for (uint32_t p : nodes[i].output) {
      rl[i] = std::max(rl[i], (size_t)e.patterns[p].glen);
      rw[i] = std::fmax(rw[i], e.patterns[p].weight);
    }
  bool changed = true;
  while (changed) {
    changed = false;
    for (size_t ii = nn; ii-- > 0;) {
      size_t bl = rl[ii];
      float bw = rw[ii];
      for (auto& ed : nodes[ii].edges) {
        bl = std::max(bl, rl[ed.next]);
        bw = std::fmax(bw, rw[ed.next]);
      }
      if (bl > rl[ii] || bw > rw[ii]) { rl[ii] = bl; rw[ii] = bw; changed = true; }
    }
  }
  for (size_t i = 0; i < nn; ++i) {
    float len = (float)rl[i];
    nodes[i].prune_len = len;
    nodes[i].prune_lw = len / rw[i];
  }
  // max_edits_fast (builder.rs:451-468)
  if (e.has_pattern_limits) e.max_edits_fast = 255;
  else if (!e.has_limits) e.max_edits_fast = 0;
  else {
    const Limits& l = e.limits;
    if (l.edits != LIM_NONE && l.ins == LIM_NONE && l.del == LIM_NONE && l.sub == LIM_NONE &&
        l.swp == LIM_NONE)
      e.max_edits_fast = (uint32_t)l.edits;
    else
      e.max_edits_fast = 255;
  }
  // multi-character mapping transitions (builder.rs:383-442): each rule in both directions; from
  // every node, walk the pattern side through the trie and record a jump consuming the haystack side
  e.mappings.assign(nn, {});
  e.has_mappings = false;
  if (!e.map_rules.empty()) {
    std::vector<std::tuple<std::vector<std::u32string>, std::vector<std::u32string>, float>> directed;
    for (auto& r : e.map_rules) {
      const auto& ga = std::get<0>(r);
      const auto& gb = std::get<1>(r);
      if (ga.empty() || gb.empty() || ga == gb) continue;
      const float penalty = e.p_sub * (1.0f - std::get<2>(r));
      directed.emplace_back(ga, gb, penalty);
      directed.emplace_back(gb, ga, penalty);
    }
    for (size_t start = 0; start < nn; ++start)
      for (auto& d : directed) {
        size_t cur = start;
        bool ok = true;
        for (auto& g : std::get<0>(d)) {
          auto it = nodes[cur].transitions.find(g);
          if (it == nodes[cur].transitions.end()) { ok = false; break; }
          cur = it->second;
        }
        if (ok) {
          e.mappings[start].push_back({std::get<1>(d), (uint32_t)cur, std::get<2>(d)});
          e.has_mappings = true;
        }
      }
  }
  build_bitap(e);
}

// ------------------------------------------------------------------------------------------
// Search (search.rs:418-1119)
// ------------------------------------------------------------------------------------------
struct State {  // structs.rs:166-179
  uint32_t node, j, ms, me;
  float pen;
  uint8_t edits;
  uint32_t packed;
};

inline bool lim_lt(int max, int v) { return max == LIM_NONE || v < max; }
inline bool lim_le(int max, int v) { return max == LIM_NONE || v <= max; }

struct Searcher {
  const Engine& e;
  explicit Searcher(const Engine& en) : e(en) {}

  const Limits* node_limits(uint32_t node) const {  // search.rs:67-71
    int64_t pi = e.nodes[node].pattern_index;
    if (pi < 0) return nullptr;
    const Pattern& p = e.patterns[(size_t)pi];
    return p.has_limits ? &p.lim : nullptr;
  }
  const Limits* pick(const Limits* l) const { return l ? l : (e.has_limits ? &e.limits : nullptr); }
  bool ins_ahead(const Limits* l, int edits, int ins) const {  // :87-99
    const Limits* m = pick(l);
    return m ? (lim_lt(m->edits, edits) && lim_lt(m->ins, ins)) : false;
  }
  bool del_ahead(const Limits* l, int edits, int del) const {  // :103-115
    const Limits* m = pick(l);
    return m ? (lim_lt(m->edits, edits) && lim_lt(m->del, del)) : false;
  }
  bool swp_ahead(const Limits* l, int edits, int swp) const {  // :119-130
    const Limits* m = pick(l);
    return m ? (lim_lt(m->edits, edits) && lim_lt(m->swp, swp)) : false;
  }
  bool subst(const Limits* l, int edits, int sub) const {  // :134-146
    const Limits* m = pick(l);
    return m ? (lim_lt(m->edits, edits) && lim_lt(m->sub, sub)) : (edits == 0 && sub == 0);
  }
  bool within(const Limits* l, int edits, int ins, int del, int sub, int swp) const {  // :151-169
    const Limits* m = pick(l);
    if (!m) return edits == 0 && ins == 0 && del == 0 && sub == 0 && swp == 0;
    return lim_le(m->edits, edits) && lim_le(m->ins, ins) && lim_le(m->del, del) &&
           lim_le(m->sub, sub) && lim_le(m->swp, swp);
  }
  float similarity(uint32_t a, uint32_t b) const { return a == b ? 1.0f : e.sim.get(a, b); }  // :76-82

  static int64_t find_no_mappings(const Node& n, uint32_t ch) {  // structs.rs:512-519
    for (auto& ed : n.edges)
      if (ed.first_char == ch) return ed.next;
    return -1;
  }
  // Node::find_transition (structs.rs:452-464): a one-byte grapheme takes the first single-byte
  // edge with that char; anything longer is a transitions-map lookup of the whole grapheme
  static int64_t find_transition(const Node& n, const std::u32string& g) {
    if (g.size() == 1 && g[0] < 0x80) {
      for (auto& ed : n.edges)
        if (ed.first_char == g[0] && ed.single_byte) return ed.next;
      return -1;
    }
    auto it = n.transitions.find(g);
    return it == n.transitions.end() ? -1 : (int64_t)it->second;
  }
  static bool has_matching_edge_char(const Node& n, uint32_t ch) {  // structs.rs:471-475
    for (auto& ed : n.edges)
      if (ed.first_char == ch && ed.single_byte) return true;
    return false;
  }
  static __uint128_t single_char_edge_bits(const Node& n) {  // structs.rs:482-493
    __uint128_t bits = 0;
    for (auto& ed : n.edges)
      if (ed.single_byte && ed.first_char < 128) bits |= (__uint128_t)1 << ed.first_char;
    return bits;
  }

  // Dedup key (search.rs:30-50); matched_start is kept for fidelity although it equals `start`.
  struct Key {
    uint32_t node, j, ms, me, packed;
    bool operator==(const Key& o) const {
      return node == o.node && j == o.j && ms == o.ms && me == o.me && packed == o.packed;
    }
  };
  struct KeyHash {  // FxHasher rounds (structs.rs:101-109) over the reference's write sequence
    size_t operator()(const Key& k) const {
      const uint64_t K = 0x517cc1b727220a95ull;
      uint64_t h = 0;
      auto add = [&](uint64_t i) { h = (((h << 5) | (h >> 59)) ^ i) * K; };
      add((uint64_t)k.node | ((uint64_t)k.j << 32));
      add((uint64_t)k.ms | ((uint64_t)k.me << 32));
      add((uint64_t)k.packed);
      return (size_t)h;
    }
  };

  uint64_t states_popped = 0, states_pushed = 0;
  uint64_t* deg_hist = nullptr;  // optional diagnostics: [0..64] degree of expanded states, [65..] per-edits
  uint64_t* batch_hist = nullptr;

  // `text_chars`, grapheme byte offsets (nullptr = identity), haystack byte length.
  uint32_t w_begin = 0, w_end = 0xFFFFFFFFu;  // start-window range (sharding diagnostics)

  // gt: the folded grapheme strings (gs_text), required when the engine has mappings
  void run(const uint32_t* tc, const uint64_t* off, uint32_t n, uint64_t hay_len, float thr,
           std::vector<Match>& out, const std::u32string* gt = nullptr) {
    out.clear();
    if (n == 0) return;
    const bool MAPPINGS = e.has_mappings;  // search.rs:204, 303
    const uint32_t mef = e.max_edits_fast == 0 || e.max_edits_fast > 6 ? 255 : e.max_edits_fast;
    const bool fast = mef != 255;
    const uint32_t text_len = n;
    auto OFF = [&](uint32_t i) -> uint64_t { return off ? off[i] : (uint64_t)i; };

    std::map<std::pair<uint64_t, uint32_t>, size_t> best_idx;  // per window (start fixed): (end,pattern) -> idx
    std::vector<State> queue;
    queue.reserve(e.beam_width ? e.beam_width : 128);
    std::unordered_map<Key, float, KeyHash> visited;
    visited.reserve(256);

    const Node& root = e.nodes[0];
    const float max_penalties = root.prune_len - root.prune_lw * thr;  // :486-487
    const float min_sym = e.min_symbol_similarity;

    bool ws = false;  // :504-521
    __uint128_t first_bits = 0, second_bits = 0;
    if (mef == 1 && !MAPPINGS && root.output.empty()) {  // :505 (WINDOW_SKIP && !MAPPINGS)
      first_bits = single_char_edge_bits(root);
      bool child_output = false;
      for (auto& ed : root.edges) {
        const Node& ch = e.nodes[ed.next];
        __uint128_t cb = single_char_edge_bits(ch);
        second_bits |= cb;
        first_bits |= cb;
        if (!ch.output.empty()) child_output = true;
      }
      ws = !child_output;
    }

    size_t effective_beam = e.beam_width;  // 0 = None
    size_t states_expanded = 0;

    for (uint32_t start = w_begin; start < text_len && start < w_end; ++start) {
      if (ws) {  // :535-553
        uint32_t ch = tc[start];
        if (ch < 128 && !((first_bits >> ch) & 1)) {
          uint32_t nx = start + 1;
          if (nx >= text_len) continue;
          uint32_t nch = tc[nx];
          if (nch < 128 && !((second_bits >> nch) & 1)) continue;
        }
      }
      queue.clear();
      visited.clear();
      best_idx.clear();
      size_t window_first_out = out.size();
      queue.push_back({0, start, start, start, 0.f, 0, 0});
      size_t q_idx = 0;
      size_t horizon[3] = {SIZE_MAX, SIZE_MAX, SIZE_MAX};  // diagnostics: pops before the first j + 1 - start >= 4, 5, 6
      size_t win_pops = 0;
      while (q_idx < queue.size()) {
        if (effective_beam) {  // :577-589
          size_t bw = effective_beam;
          size_t remaining = queue.size() - q_idx;
          if (remaining > bw * 2) {
            if (e.beam_rule >= 2) {
              rsel::select_nth_unstable_by(queue.data() + q_idx, remaining, bw - 1, [](const State& a, const State& b) {
                return total_order_bits(a.pen) < total_order_bits(b.pen);
              });
              queue.resize(q_idx + bw);
            } else {
              beam_select(queue, q_idx, bw, e.beam_rule == 1);
            }
          }
        }
        State st = queue[q_idx];
        if (deg_hist) {
          deg_hist[73] = std::max<uint64_t>(deg_hist[73], queue.size() - q_idx);
          for (int h = 0; h < 3; ++h)
            if (horizon[h] == SIZE_MAX && st.j + 1 - start >= (uint32_t)(4 + h)) horizon[h] = win_pops;
          ++win_pops;
        }
        ++q_idx;
        ++states_popped;
        Key key{st.node, st.j, st.ms, st.me, st.packed};
        auto vit = visited.find(key);  // :618-628
        if (vit != visited.end()) {
          if (vit->second <= st.pen) continue;
          vit->second = st.pen;
        } else {
          visited.emplace(key, st.pen);
        }
        const Node& nd = e.nodes[st.node];
        if (st.pen > nd.prune_len - nd.prune_lw * thr) continue;  // :638-642
        if (deg_hist) {
          deg_hist[std::min<size_t>(nd.edges.size(), 64)]++;
          deg_hist[65 + std::min<uint32_t>(st.edits, 7)]++;
        }
        const float remaining = max_penalties - st.pen;            // :648
        const Limits* nlim = e.has_pattern_limits ? node_limits(st.node) : nullptr;
        const uint8_t edits = st.edits;
        const uint32_t pc = st.packed;
        if (!nd.output.empty()) {  // :659-737
          uint8_t ins = pc & 0xFF, del = (pc >> 8) & 0xFF, sub = (pc >> 16) & 0xFF, swp = (pc >> 24) & 0xFF;
          uint64_t sb = st.ms < text_len ? OFF(st.ms) : 0;
          uint64_t eb = st.me < text_len ? OFF(st.me) : hay_len;
          for (uint32_t p : nd.output) {
            if (fast) {
              if (edits > mef) continue;
            } else {
              const Pattern& P = e.patterns[p];
              if (!within(P.has_limits ? &P.lim : nullptr, edits, ins, del, sub, swp)) continue;
            }
            float total = (float)e.patterns[p].glen;
            float sim = (total - st.pen) / total * e.patterns[p].weight;
            if (sim < thr) continue;
            auto bk = std::make_pair(eb, p);  // start_byte is fixed within a window
            auto bi = best_idx.find(bk);
            if (bi == best_idx.end()) {
              best_idx.emplace(bk, out.size());
              out.push_back({sb, eb, p, sim, ins, del, sub, swp, edits});
            } else if (sim > out[bi->second].similarity) {
              out[bi->second] = {sb, eb, p, sim, ins, del, sub, swp, edits};
            }
          }
        }
        const bool is_last_edit = fast && (uint32_t)edits + 1 >= mef;  // :742
        const uint32_t j = st.j;
        const uint32_t current_ch = j < text_len ? tc[j] : 0;
        if (j < text_len) {
          bool have_next = false;
          uint32_t next_ch = 0;
          if (is_last_edit && (!fast || edits < mef) && j + 1 < text_len) { have_next = true; next_ch = tc[j + 1]; }
          const uint32_t ms_next = st.me == st.ms ? j : st.ms;
          int64_t exact_next = MAPPINGS ? find_transition(nd, gt[j])           // :776-780
                                        : find_no_mappings(nd, current_ch);
          if (exact_next >= 0) {
            queue.push_back({(uint32_t)exact_next, j + 1, ms_next, j + 1, st.pen, edits, pc});
            ++states_pushed;
          }
          bool subst_ok = fast ? (edits < mef) : subst(nlim, edits, (uint8_t)(pc >> 16));  // :803-811
          if (subst_ok) {
            for (auto& ed : nd.edges) {  // :814-874
              if (exact_next >= 0 && ed.next == (uint32_t)exact_next) continue;
              float sim = similarity(ed.first_char, current_ch);
              if (sim < min_sym) continue;
              float penalty = e.p_sub * (1.0f - sim);
              if (penalty > remaining) continue;
              if (is_last_edit) {
                const Node& child = e.nodes[ed.next];
                if (child.output.empty() && (!have_next || !has_matching_edge_char(child, next_ch))) continue;
              }
              queue.push_back({ed.next, j + 1, ms_next, j + 1, st.pen + penalty, (uint8_t)(edits + 1), pc + 0x10000});
              ++states_pushed;
            }
            if (MAPPINGS)  // 1b) multi-character mappings (:883-922)
              for (const MapT& mt : e.mappings[st.node]) {
                const uint32_t hlen = (uint32_t)mt.hay.size();
                if ((uint64_t)j + hlen > text_len) continue;
                bool hay_matches = true;
                for (uint32_t k = 0; k < hlen && hay_matches; ++k) hay_matches = gt[j + k] == mt.hay[k];
                if (!hay_matches) continue;
                const float np = st.pen + mt.penalty;
                if (np > max_penalties) continue;
                queue.push_back({mt.next, j + hlen, ms_next, j + hlen, np, (uint8_t)(edits + 1), pc + 0x10000});
                ++states_pushed;
              }
          }
          // swap :935-989
          if (j + 1 < text_len && e.p_swp <= remaining && (!fast || edits < mef)) {
            uint32_t nch = have_next ? next_ch : tc[j + 1];
            int64_t x = MAPPINGS ? find_transition(nd, gt[j + 1]) : find_no_mappings(nd, nch);  // :945-961
            int64_t node2 = x < 0 ? -1
                            : MAPPINGS ? find_transition(e.nodes[(size_t)x], gt[j])
                                       : find_no_mappings(e.nodes[(size_t)x], current_ch);
            if (node2 >= 0 && (fast || swp_ahead(node_limits((uint32_t)node2), edits, (uint8_t)(pc >> 24)))) {
              queue.push_back({(uint32_t)node2, j + 2, st.ms, j + 2, st.pen + e.p_swp, (uint8_t)(edits + 1), pc + 0x1000000});
              ++states_pushed;
            }
          }
          // insertion :994-1029
          if ((st.ms != st.me || st.ms != j) && e.p_ins <= remaining &&
              (fast ? edits < mef : ins_ahead(nlim, edits, (uint8_t)(pc & 0xFF))) &&
              !(is_last_edit && nd.output.empty() && (!have_next || !has_matching_edge_char(nd, next_ch)))) {
            queue.push_back({st.node, j + 1, st.ms, st.me, st.pen + e.p_ins, (uint8_t)(edits + 1), pc + 1});
            ++states_pushed;
          }
        }
        // deletion :1035-1089
        if (e.p_del <= remaining && (fast ? edits < mef : del_ahead(nlim, edits, (uint8_t)((pc >> 8) & 0xFF)))) {
          bool have_cur = is_last_edit && j < text_len;
          for (auto& ed : nd.edges) {
            if (is_last_edit) {
              const Node& child = e.nodes[ed.next];
              if (child.output.empty() && (!have_cur || !has_matching_edge_char(child, current_ch))) continue;
            }
            queue.push_back({ed.next, j, st.ms, st.me, st.pen + e.p_del, (uint8_t)(edits + 1), pc + 0x100});
            ++states_pushed;
          }
        }
      }
      (void)window_first_out;
      if (deg_hist) {  // diagnostics: per-window maxima (pending queue, distinct visited keys)
        deg_hist[74] = std::max<uint64_t>(deg_hist[74], visited.size());
        deg_hist[75] += visited.size();
        deg_hist[76] += 1;
        for (int h = 0; h < 3; ++h) deg_hist[77 + h] += horizon[h] == SIZE_MAX ? win_pops : horizon[h];
      }
      if (e.has_auto_beam && effective_beam == 0) {  // :1096-1103
        states_expanded += queue.size();
        if (states_expanded > e.ab_budget) effective_beam = e.ab_width;
      }
    }
    std::sort(out.begin(), out.end(), [](const Match& a, const Match& b) {
      if (a.start != b.start) return a.start < b.start;
      if (a.end != b.end) return a.end < b.end;
      return a.pattern < b.pattern;
    });
  }

  static uint32_t total_order_bits(float f) {  // f32::total_cmp as an unsigned key
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  }
  // Canonical beam: keep the bw smallest by (penalty total order, position), stable; `latest`
  // breaks ties at the cut towards the latest positions instead (diagnostic).
  static void beam_select(std::vector<State>& q, size_t q_idx, size_t bw, bool latest) {
    size_t n = q.size() - q_idx;
    std::vector<uint64_t> keys(n);
    for (size_t i = 0; i < n; ++i)
      keys[i] = ((uint64_t)total_order_bits(q[q_idx + i].pen) << 32) | (uint64_t)(latest ? n - 1 - i : i);
    std::vector<uint64_t> tmp = keys;
    std::nth_element(tmp.begin(), tmp.begin() + (bw - 1), tmp.end());
    uint64_t cut = tmp[bw - 1];
    size_t w = q_idx;
    for (size_t i = 0; i < n; ++i)
      if (keys[i] <= cut) q[w++] = q[q_idx + i];
    q.resize(q_idx + bw);
  }
};

// Unit-cost bitap over a u8 id stream (prefilter.rs:410-435).
void bitap_windows(const std::vector<uint64_t>& mask, size_t m, size_t k, const uint8_t* ids, size_t n,
                   std::vector<std::pair<size_t, size_t>>& out) {
  uint64_t match_bit = 1ull << (m - 1);
  std::vector<uint64_t> r(k + 1), nr(k + 1);
  for (size_t d = 0; d <= k; ++d) r[d] = (d >= 64 ? ~0ull : ((1ull << d) - 1));
  size_t span = m + k;
  for (size_t i = 0; i < n; ++i) {
    uint64_t bc = mask[ids[i]];
    nr[0] = ((r[0] << 1) | 1) & bc;
    for (size_t d = 1; d <= k; ++d)
      nr[d] = ((r[d] << 1) & bc) | ((r[d - 1] | nr[d - 1]) << 1) | r[d - 1] | 1;
    if (nr[k] & match_bit) {
      size_t end = i + 1;
      out.push_back({end >= span ? end - span : 0, end});
    }
    std::swap(r, nr);
  }
}

thread_local uint64_t g_deg_hist[80];  // diagnostics only (degree / edits histogram of expanded states); per thread: the CPU baseline runs the oracle on several threads

// Staging for a (sub)haystack: ASCII fast path or caller-provided global graphemes.
struct Staged {
  std::vector<uint32_t> tc;
  std::vector<std::u32string> gt;  // folded grapheme strings (engines with mappings only)
  std::vector<uint64_t> off;  // empty = identity
  uint64_t len = 0;
};

bool is_ascii(const uint8_t* p, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i)
    if (p[i] & 0x80) return false;
  return true;
}

struct Text {  // full haystack + its global segmentation (used when not ASCII)
  const uint8_t* utf8;
  uint64_t len;
  uint32_t n;            // grapheme count (non-ASCII path)
  const uint32_t* goff;  // [n+1] offsets into cps
  const uint32_t* cps;   // folded code points of each grapheme
  const uint64_t* boff;  // [n] grapheme byte offsets
};

// search_raw on bytes [b0, b1) of the text; grapheme range [g0, g1) used when non-ASCII.
void search_raw_slice(const Engine& e, const Text& t, uint64_t b0, uint64_t b1, uint32_t g0, uint32_t g1,
                      float thr, std::vector<Match>& out, uint64_t* popped, uint32_t w_begin = 0,
                      uint32_t w_end = 0xFFFFFFFFu) {
  Staged s;
  s.len = b1 - b0;
  if (is_ascii(t.utf8 + b0, s.len)) {  // search.rs:196-203, grapheme.rs:76-125
    s.tc.resize(s.len);
    for (uint64_t i = 0; i < s.len; ++i) {
      uint8_t b = t.utf8[b0 + i];
      if (e.case_insensitive && b >= 'A' && b <= 'Z') b += 32;
      s.tc[i] = b;
    }
    if (e.has_mappings)  // gs_text (grapheme.rs:100-109)
      for (uint64_t i = 0; i < s.len; ++i) s.gt.emplace_back(1, (char32_t)s.tc[i]);
  } else {  // search.rs:296-302 (global segmentation restricted to the slice)
    uint32_t n = g1 - g0;
    s.tc.resize(n);
    s.off.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t g = g0 + i;
      s.tc[i] = t.goff[g + 1] > t.goff[g] ? t.cps[t.goff[g]] : 0;
      s.off[i] = t.boff[g] - b0;
      if (e.has_mappings) s.gt.emplace_back(t.cps + t.goff[g], t.cps + t.goff[g + 1]);  // grapheme.rs:61-63
    }
  }
  if (s.tc.size() > 0xFFFFFFFFull) { out.clear(); return; }
  Searcher S(e);
  S.deg_hist = g_deg_hist;
  S.w_begin = w_begin;
  S.w_end = w_end;
  S.run(s.tc.data(), s.off.empty() ? nullptr : s.off.data(), (uint32_t)s.tc.size(), s.len, thr, out,
        s.gt.empty() ? nullptr : s.gt.data());
  if (popped) *popped += S.states_popped;
  for (auto& m : out) { m.start += b0; m.end += b0; }
}

}  // namespace

namespace {
int total_cmp(float a, float b) {  // f32::total_cmp
  int32_t x, y;
  std::memcpy(&x, &a, 4);
  std::memcpy(&y, &b, 4);
  x ^= (int32_t)(((uint32_t)(x >> 31)) >> 1);
  y ^= (int32_t)(((uint32_t)(y >> 31)) >> 1);
  return x < y ? -1 : (x > y ? 1 : 0);
}
template <typename T>
int cmp3(T a, T b) { return a < b ? -1 : (a > b ? 1 : 0); }
// <[T]>::binary_search_by as in Rust >= 1.82 (the crate is edition 2024): on equal keys it returns
// the index the halving loop settles on, not necessarily the first
template <typename F>
std::pair<bool, size_t> rust_binary_search_by(size_t len, F f) {
  size_t size = len;
  if (size == 0) return {false, 0};
  size_t base = 0;
  while (size > 1) {
    const size_t half = size / 2, mid = base + half;
    if (f(mid) <= 0) base = mid;  // cmp != Greater
    size -= half;
  }
  const int c = f(base);
  if (c == 0) return {true, base};
  return {false, base + (c < 0 ? 1 : 0)};
}
}  // namespace

// ==========================================================================================
// C ABI (ctypes)
// ==========================================================================================
extern "C" {

struct orc_config {
  int32_t case_insensitive;
  int32_t has_limits;
  int32_t lim[5];  // ins, del, sub, swp, edits; -1 = None
  float p_ins, p_del, p_sub, p_swp;
  uint64_t beam_width;  // 0 = none
  int32_t has_auto_beam;
  uint64_t ab_budget, ab_width;
  float min_symbol_similarity;
  int32_t custom_similarity;      // 1 = use sim_ascii + sim_pairs below
  const float* sim_ascii;         // 128*128
  uint64_t n_sim_pairs;
  const uint32_t* sim_pair_ab;    // 2*n
  const float* sim_pair_val;      // n
  // mapping rules (builder.rs:116-132), sides already segmented + folded by the caller:
  // rule r's side a = graphemes [side_off[2r], side_off[2r+1]), side b = [side_off[2r+1], side_off[2r+2])
  uint64_t n_map;
  const uint32_t* map_side_off;  // 2*n_map + 1
  const uint32_t* map_g_off;     // graphemes + 1, into map_cps
  const uint32_t* map_cps;
  const float* map_score;        // n_map
};

struct orc_match {
  uint64_t start, end;
  uint32_t pattern;
  float similarity;
  uint8_t ins, del, sub, swp, edits, pad[3];
};

// patterns: n_patterns; per pattern: glen[i] graphemes (also the folded grapheme count),
// weight[i], lim_flag[i] (1 = has limits), lim[i*5..]; graphemes as flat cps with offsets.
void* orc_build(const orc_config* cfg, uint64_t n_patterns, const uint32_t* glen, const float* weight,
                const int32_t* lim_flag, const int32_t* lim, const uint32_t* pg_off /* n_patterns+1 */,
                const uint32_t* g_off /* total_graphemes+1 */, const uint32_t* cps) {
  Engine* e = new Engine();
  e->case_insensitive = cfg->case_insensitive != 0;
  e->has_limits = cfg->has_limits != 0;
  if (e->has_limits) {
    e->limits.ins = cfg->lim[0]; e->limits.del = cfg->lim[1]; e->limits.sub = cfg->lim[2];
    e->limits.swp = cfg->lim[3]; e->limits.edits = cfg->lim[4];
  }
  e->p_ins = cfg->p_ins; e->p_del = cfg->p_del; e->p_sub = cfg->p_sub; e->p_swp = cfg->p_swp;
  e->beam_width = cfg->beam_width;
  e->has_auto_beam = cfg->has_auto_beam != 0;
  e->ab_budget = cfg->ab_budget; e->ab_width = cfg->ab_width;
  e->min_symbol_similarity = cfg->min_symbol_similarity;
  if (cfg->custom_similarity) {
    for (int i = 0; i < 128; ++i)
      for (int j = 0; j < 128; ++j) e->sim.ascii[i][j] = cfg->sim_ascii[i * 128 + j];
    for (uint64_t k = 0; k < cfg->n_sim_pairs; ++k)
      e->sim.map[{cfg->sim_pair_ab[2 * k], cfg->sim_pair_ab[2 * k + 1]}] = cfg->sim_pair_val[k];
  } else {
    default_similarity(e->sim);
  }
  e->patterns.resize(n_patterns);
  for (uint64_t i = 0; i < n_patterns; ++i) {
    Pattern& p = e->patterns[i];
    p.glen = glen[i];
    p.weight = weight[i];
    p.has_limits = lim_flag[i] != 0;
    if (p.has_limits) {
      p.lim.ins = lim[i * 5 + 0]; p.lim.del = lim[i * 5 + 1]; p.lim.sub = lim[i * 5 + 2];
      p.lim.swp = lim[i * 5 + 3]; p.lim.edits = lim[i * 5 + 4];
    }
    for (uint32_t g = pg_off[i]; g < pg_off[i + 1]; ++g)
      p.graphemes.emplace_back(cps + g_off[g], cps + g_off[g + 1]);
  }
  for (uint64_t r = 0; r < cfg->n_map; ++r) {
    std::vector<std::u32string> side[2];
    for (int k = 0; k < 2; ++k)
      for (uint32_t g = cfg->map_side_off[2 * r + k]; g < cfg->map_side_off[2 * r + k + 1]; ++g)
        side[k].emplace_back(cfg->map_cps + cfg->map_g_off[g], cfg->map_cps + cfg->map_g_off[g + 1]);
    e->map_rules.emplace_back(side[0], side[1], cfg->map_score[r]);
  }
  build(*e);
  return e;
}

void orc_free(void* h) { delete static_cast<Engine*>(h); }

// Restatement modes for engines built afterwards (see g_edge_order / g_beam_rule); -1 keeps a mode.
// The oracle's transitions-map order for one node's children (see hashbrown_order), for tests.
void orc_edge_order(const uint32_t* cps, const uint64_t* off, uint64_t n, uint32_t* order) {
  SwissOrder t;
  for (uint64_t i = 0; i < n; ++i) t.insert(fx_hash_str(utf8_of(std::u32string(cps + off[i], cps + off[i + 1]))));
  std::vector<int> o = t.iteration_order();
  for (uint64_t i = 0; i < n; ++i) order[i] = (uint32_t)o[i];
}

// rsel::select_nth_unstable_by over n f32 keys (total_cmp), for tests: perm[i] = the original index
// of the element at position i afterwards.
void orc_select_nth(const float* keys, uint64_t n, uint64_t index, uint32_t* perm) {
  struct E { float k; uint32_t i; };
  std::vector<E> v(n);
  for (uint64_t i = 0; i < n; ++i) v[i] = {keys[i], (uint32_t)i};
  rsel::select_nth_unstable_by(v.data(), (size_t)n, (size_t)index, [](const E& a, const E& b) {
    return Searcher::total_order_bits(a.k) < Searcher::total_order_bits(b.k);
  });
  for (uint64_t i = 0; i < n; ++i) perm[i] = v[i].i;
}

// The same over `count` arrays (array a = keys[offs[a] .. offs[a+1]), its own index[a]); perm is laid
// out like keys. Returns the number of arrays whose result violates select_nth_unstable_by's
// post-condition (every element before index <= v[index] <= every element after), for tests.
uint64_t orc_select_nth_batch(const float* keys, const uint64_t* offs, uint64_t count, const uint64_t* index,
                              uint32_t* perm) {
  uint64_t bad = 0;
  for (uint64_t a = 0; a < count; ++a) {
    const uint64_t b = offs[a], n = offs[a + 1] - b;
    orc_select_nth(keys + b, n, index[a], perm + b);
    const uint32_t* p = perm + b;
    const uint32_t kv = Searcher::total_order_bits(keys[b + p[index[a]]]);
    bool ok = true;
    for (uint64_t i = 0; i < n && ok; ++i) {
      const uint32_t k = Searcher::total_order_bits(keys[b + p[i]]);
      ok = i < index[a] ? k <= kv : k >= kv;
    }
    bad += ok ? 0 : 1;
  }
  return bad;
}

// sel_limit: select.rs's 16 partition rounds before median_of_medians (tests only).
void orc_set_modes(int32_t edge_order, int32_t beam_rule, int32_t sel_limit) {
  if (edge_order >= 0) g_edge_order = edge_order;
  if (beam_rule >= 0) g_beam_rule = beam_rule;
  if (sel_limit >= 0) g_sel_limit = sel_limit;
}
uint64_t* orc_deg_hist() { return g_deg_hist; }

uint64_t orc_num_nodes(void* h) { return static_cast<Engine*>(h)->nodes.size(); }
uint32_t orc_max_edits_fast(void* h) { return static_cast<Engine*>(h)->max_edits_fast; }
int32_t orc_prefilter_active(void* h) { return static_cast<Engine*>(h)->bitap_ok ? 1 : 0; }

// Full search_raw (search.rs:187-395) or Prefiltered::raw (prefilter.rs:146-155).
// For non-ASCII text the caller supplies the global grapheme segmentation (folded).
int32_t orc_search_windows(void* h, const uint8_t* utf8, uint64_t len, uint32_t n_graphemes, const uint32_t* goff,
                           const uint32_t* cps, const uint64_t* boff, float threshold, int32_t use_prefilter,
                           orc_match** out, uint64_t* n_out, uint64_t* states_popped, uint32_t w_begin,
                           uint32_t w_end);

int32_t orc_search(void* h, const uint8_t* utf8, uint64_t len, uint32_t n_graphemes, const uint32_t* goff,
                   const uint32_t* cps, const uint64_t* boff, float threshold, int32_t use_prefilter,
                   orc_match** out, uint64_t* n_out, uint64_t* states_popped) {
  return orc_search_windows(h, utf8, len, n_graphemes, goff, cps, boff, threshold, use_prefilter, out, n_out,
                            states_popped, 0, 0xFFFFFFFFu);
}

// search_raw restricted to start windows [w_begin, w_end) (no prefilter): the per-rank work of a
// sharded search; the union over a partition of [0, n) equals search_raw.
int32_t orc_search_windows(void* h, const uint8_t* utf8, uint64_t len, uint32_t n_graphemes, const uint32_t* goff,
                           const uint32_t* cps, const uint64_t* boff, float threshold, int32_t use_prefilter,
                           orc_match** out, uint64_t* n_out, uint64_t* states_popped, uint32_t w_begin,
                           uint32_t w_end) {
  const Engine& e = *static_cast<Engine*>(h);
  Text t{utf8, len, n_graphemes, goff, cps, boff};
  bool ascii = is_ascii(utf8, len);
  uint32_t n = ascii ? (uint32_t)len : n_graphemes;
  std::vector<Match> res;
  uint64_t popped = 0;
  if (ascii && len > 0xFFFFFFFFull) return 1;  // HaystackTooLarge
  if (!use_prefilter || !e.bitap_ok) {
    search_raw_slice(e, t, 0, len, 0, ascii ? 0 : n, threshold, res, &popped, w_begin, w_end);
  } else {
    // prefilter.rs:304-374
    std::vector<size_t> ks;
    bool fallback = false;
    for (auto& bp : e.bitap) {  // k_for :285-302
      float nf = (float)bp.m;
      float p_max = nf * (1.0f - threshold / bp.weight);
      size_t k_pen = 0;
      if (p_max <= 0.0f) k_pen = 0;
      else {
        float kf = std::floor(p_max * e.edit_cost_mult);
        k_pen = kf >= 1.8446744e19f ? SIZE_MAX : (kf != kf ? 0 : (size_t)kf);  // Rust `as usize` saturates, NaN -> 0
      }
      size_t k = bp.has_k_limit ? std::min(k_pen, bp.k_limit) : k_pen;
      if (k > 24) { fallback = true; break; }
      ks.push_back(k);
    }
    if (fallback) {
      search_raw_slice(e, t, 0, len, 0, ascii ? 0 : n, threshold, res, &popped);
    } else {
      std::vector<uint8_t> ids(n);
      if (ascii) {
        for (uint64_t i = 0; i < len; ++i) ids[i] = e.ascii_id[utf8[i]];
      } else {
        for (uint32_t g = 0; g < n; ++g) {
          std::u32string key(cps + goff[g], cps + goff[g + 1]);
          auto it = e.symbol_ids.find(key);
          ids[g] = it == e.symbol_ids.end() ? 0 : (uint8_t)it->second;
        }
      }
      std::vector<std::pair<size_t, size_t>> windows;
      for (size_t i = 0; i < e.bitap.size(); ++i)
        bitap_windows(e.bitap[i].mask, e.bitap[i].m, ks[i], ids.data(), n, windows);
      if (!windows.empty()) {
        std::sort(windows.begin(), windows.end());
        std::vector<std::pair<size_t, size_t>> merged;
        for (auto& w : windows) {
          if (!merged.empty() && w.first <= merged.back().second)
            merged.back().second = std::max(merged.back().second, w.second);
          else
            merged.push_back(w);
        }
        std::map<std::tuple<uint64_t, uint64_t, uint32_t>, Match> best;
        for (auto& w : merged) {
          size_t gs = w.first, ge = std::min(w.second, (size_t)n);
          uint64_t bs = ascii ? gs : boff[gs];
          uint64_t be = ascii ? ge : (ge < n ? boff[ge] : len);
          std::vector<Match> part;
          search_raw_slice(e, t, bs, be, (uint32_t)gs, (uint32_t)ge, threshold, part, &popped);
          for (auto& m : part) {
            auto key = std::make_tuple(m.start, m.end, m.pattern);
            auto it = best.find(key);
            if (it == best.end()) best.emplace(key, m);
            else if (m.similarity > it->second.similarity) it->second = m;
          }
        }
        for (auto& kv : best) res.push_back(kv.second);
      }
    }
  }
  *n_out = res.size();
  *out = (orc_match*)std::malloc(sizeof(orc_match) * (res.size() ? res.size() : 1));
  for (size_t i = 0; i < res.size(); ++i) {
    orc_match& o = (*out)[i];
    std::memset(&o, 0, sizeof(o));
    o.start = res[i].start; o.end = res[i].end; o.pattern = res[i].pattern; o.similarity = res[i].similarity;
    o.ins = res[i].ins; o.del = res[i].del; o.sub = res[i].sub; o.swp = res[i].swp; o.edits = res[i].edits;
  }
  if (states_popped) *states_popped = popped;
  return 0;
}

void orc_matches_free(orc_match* m) { std::free(m); }

// FuzzyMatches::apply (matches.rs:7-19): ranking by `order` (0 Unsorted, 1 Default :24-38, 2 Greedy
// :43-57, 3 CoverageWeighted :64-81), then overlap resolution by `overlap` (0 Keep, 1 NonOverlapping
// :86-113, 2 NonOverlappingUnique :117-149). pat_len[p] = Pattern::len() in bytes (structs.rs:628-630);
// uid[p] = the uniqueness key of pattern p (custom_unique_id or automatic index, never equal across
// kinds). Kept matches are compacted to the front in the reference's final order; returns the count.

uint64_t orc_apply(orc_match* m, uint64_t n, int32_t order, int32_t overlap, const uint64_t* pat_len,
                   const uint64_t* uid) {
  std::vector<orc_match> v(m, m + n);
  auto tail = [](const orc_match& l, const orc_match& r) {  // .then start, end, pattern_index
    int c = cmp3(l.start, r.start);
    if (!c) c = cmp3(l.end, r.end);
    if (!c) c = cmp3(l.pattern, r.pattern);
    return c;
  };
  if (order == 1) {
    std::sort(v.begin(), v.end(), [&](const orc_match& l, const orc_match& r) {
      int c = total_cmp(r.similarity, l.similarity);
      if (!c) c = cmp3(pat_len[r.pattern], pat_len[l.pattern]);
      if (!c) c = cmp3(r.end - r.start, l.end - l.start);  // text.len()
      if (!c) c = tail(l, r);
      return c < 0;
    });
  } else if (order == 2) {
    std::sort(v.begin(), v.end(), [&](const orc_match& l, const orc_match& r) {
      int c = cmp3(pat_len[r.pattern], pat_len[l.pattern]);
      if (!c) c = total_cmp(r.similarity, l.similarity);
      if (!c) c = tail(l, r);
      return c < 0;
    });
  } else if (order == 3) {
    auto score = [&](const orc_match& x) {  // similarity * similarity * len as f32, in that order
      volatile float s2 = x.similarity * x.similarity;
      return (float)(s2 * (float)pat_len[x.pattern]);
    };
    std::sort(v.begin(), v.end(), [&](const orc_match& l, const orc_match& r) {
      int c = total_cmp(score(r), score(l));
      if (!c) c = total_cmp(r.similarity, l.similarity);
      if (!c) c = tail(l, r);
      return c < 0;
    });
  }
  if (overlap == 1 || overlap == 2) {
    std::vector<std::pair<uint64_t, uint64_t>> occupied;
    std::set<uint64_t> used;
    std::vector<orc_match> kept;
    for (const orc_match& x : v) {
      if (overlap == 2 && used.count(uid[x.pattern])) continue;
      const auto r = rust_binary_search_by(occupied.size(), [&](size_t i) { return cmp3(occupied[i].first, x.start); });
      const size_t pos = r.second;
      const bool prev_ok = pos == 0 || occupied[pos - 1].second <= x.start;
      const bool next_ok = pos == occupied.size() || occupied[pos].first >= x.end;
      if (prev_ok && next_ok) {
        if (overlap == 2) used.insert(uid[x.pattern]);
        occupied.insert(occupied.begin() + (std::ptrdiff_t)pos, {x.start, x.end});
        kept.push_back(x);
      }
    }
    // sort_unstable_by_key(start): equal starts (empty spans only) keep an unspecified order
    std::stable_sort(kept.begin(), kept.end(), [](const orc_match& a, const orc_match& b) { return a.start < b.start; });
    v.swap(kept);
  }
  std::copy(v.begin(), v.end(), m);
  return v.size();
}

// Merged bitap windows (prefilter.rs:319-342) for diagnostics; -1 = full-search fallback.
int64_t orc_prefilter_windows(void* h, const uint8_t* utf8, uint64_t len, uint32_t n_graphemes, const uint32_t* goff,
                              const uint32_t* cps, float threshold, uint64_t* out, uint64_t cap) {
  const Engine& e = *static_cast<Engine*>(h);
  if (!e.bitap_ok) return -1;
  bool ascii = is_ascii(utf8, len);
  uint32_t n = ascii ? (uint32_t)len : n_graphemes;
  std::vector<size_t> ks;
  for (auto& bp : e.bitap) {
    float nf = (float)bp.m;
    float p_max = nf * (1.0f - threshold / bp.weight);
    size_t k_pen = 0;
    if (!(p_max <= 0.0f)) {
      float kf = std::floor(p_max * e.edit_cost_mult);
      k_pen = kf >= 1.8446744e19f ? SIZE_MAX : (kf != kf ? 0 : (size_t)kf);
    }
    size_t k = bp.has_k_limit ? std::min(k_pen, bp.k_limit) : k_pen;
    if (k > 24) return -1;
    ks.push_back(k);
  }
  std::vector<uint8_t> ids(n);
  for (uint32_t g = 0; g < n; ++g) {
    if (ascii) { ids[g] = e.ascii_id[utf8[g]]; continue; }
    std::u32string key(cps + goff[g], cps + goff[g + 1]);
    auto it = e.symbol_ids.find(key);
    ids[g] = it == e.symbol_ids.end() ? 0 : (uint8_t)it->second;
  }
  std::vector<std::pair<size_t, size_t>> windows, merged;
  for (size_t i = 0; i < e.bitap.size(); ++i) bitap_windows(e.bitap[i].mask, e.bitap[i].m, ks[i], ids.data(), n, windows);
  std::sort(windows.begin(), windows.end());
  for (auto& w : windows) {
    if (!merged.empty() && w.first <= merged.back().second) merged.back().second = std::max(merged.back().second, w.second);
    else merged.push_back(w);
  }
  for (size_t i = 0; i < merged.size() && i < cap; ++i) { out[2 * i] = merged[i].first; out[2 * i + 1] = merged[i].second; }
  return (int64_t)merged.size();
}

// Standalone bitap over an id stream with an explicit mask (for the brute-force DP check,
// examples/bitap_prototype.rs:21-56). Writes match END positions (1-based exclusive) into ends.
uint64_t orc_bitap_ends(const uint8_t* pattern, uint64_t m, const uint8_t* text, uint64_t n, uint64_t k,
                        uint64_t* ends) {
  std::vector<uint64_t> mask(256, 0);
  for (uint64_t i = 0; i < m; ++i) mask[pattern[i]] |= 1ull << i;
  std::vector<std::pair<size_t, size_t>> w;
  bitap_windows(mask, m, k, text, n, w);
  for (size_t i = 0; i < w.size(); ++i) ends[i] = w[i].second;
  return w.size();
}

}  // extern "C"
