// builder.cpp — host construction of the device automaton tables.
//
// Mirrors FuzzyAhoCorasickBuilder::build (src/builder.rs:181-484) and emits the flat
// structure-of-arrays layout of fac_internal.h instead of the reference's per-node Vecs/maps:
//   * graphemes are interned to ids and the trie is one (node, grapheme-id) -> child hash map;
//   * each node's children are ordered like the reference's `transitions.iter()` (builder.rs:
//     336-342): the crate's FxHasher over the grapheme's UTF-8 bytes (structs.rs:95-156) placed by
//     hashbrown's SSE2 group probing as std's HashMap inserts them (edge_order below);
//   * fail links exist only to merge suffix-pattern outputs (builder.rs:239-276); they are not
//     uploaded, because the search never follows them;
//   * prune coefficients come from the reach-len / reach-weight pass (builder.rs:344-381).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <unordered_map>

#include "fac_internal.h"

namespace fac {
namespace {

struct U32Hash {
  size_t operator()(const std::u32string& s) const {
    uint64_t h = 1469598103934665603ull;
    for (char32_t c : s) h = (h ^ (uint64_t)c) * 1099511628211ull;
    return (size_t)h;
  }
};

void default_similarity(std::vector<float>& t) {  // builder.rs:492-526, structs.rs:36-48
  t.assign(128 * 128, 0.f);
  for (int i = 0; i < 128; ++i) t[i * 128 + i] = 1.f;
  auto vowel = [](int c) { return c == 'a' || c == 'e' || c == 'i' || c == 'o' || c == 'u'; };
  for (int a = 'a'; a <= 'z'; ++a)
    for (int b = 'a'; b <= 'z'; ++b) {
      if (a == b) continue;
      if (vowel(a) == vowel(b)) t[a * 128 + b] = vowel(a) ? 0.6f : 0.4f;
    }
  const struct { char a, b; float s; } ocr[] = {{'o', '0', 0.6f}, {'l', '1', 0.7f}, {'i', '1', 0.6f},
                                                {'s', '5', 0.5f}};
  for (auto& o : ocr) {
    t[o.a * 128 + o.b] = o.s;
    t[o.b * 128 + o.a] = o.s;
  }
}

// Hash of a `String` key under the crate's FxHasher: `Hash for str` writes the bytes, then 0xff
// (structs.rs:101-156; core::hash::Hasher::write_str).
uint64_t fx_str_hash(const std::u32string& g) {
  std::string u;
  for (char32_t c : g) {  // UTF-8
    if (c < 0x80) {
      u.push_back((char)c);
    } else if (c < 0x800) {
      u.push_back((char)(0xC0 | (c >> 6)));
      u.push_back((char)(0x80 | (c & 0x3F)));
    } else if (c < 0x10000) {
      u.push_back((char)(0xE0 | (c >> 12)));
      u.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      u.push_back((char)(0x80 | (c & 0x3F)));
    } else {
      u.push_back((char)(0xF0 | (c >> 18)));
      u.push_back((char)(0x80 | ((c >> 12) & 0x3F)));
      u.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      u.push_back((char)(0x80 | (c & 0x3F)));
    }
  }
  uint64_t h = 0;
  auto mix = [&h](uint64_t word) { h = ((h << 5) | (h >> 59)) ^ word, h *= 0x517cc1b727220a95ull; };
  size_t i = 0;
  for (; i + 8 <= u.size(); i += 8) {
    uint64_t w;
    std::memcpy(&w, u.data() + i, 8);  // little-endian host, like u64::from_le_bytes
    mix(w);
  }
  if (i + 4 <= u.size()) {
    uint32_t w;
    std::memcpy(&w, u.data() + i, 4);
    mix(w);
    i += 4;
  }
  for (; i < u.size(); ++i) mix((uint8_t)u[i]);
  mix(0xff);
  return h;
}

// Iteration order of an insert-only std HashMap (hashbrown RawTable, x86-64 SSE2: 16 control bytes
// per group) after inserting `hashes` in order: a table of 2^b buckets holds at most b < 3 ? 2^b - 1 :
// 2^b * 7 / 8 items; inserting into a full one first moves every item, in bucket order, into the
// next size (4, 8, 16, ... buckets); an item goes to the first EMPTY control byte along the
// triangular probe over 16-byte groups from hash & mask (control bytes past the buckets mirror the
// first 16; a small table's padding bytes are EMPTY, and a hit there falls back to the first EMPTY
// bucket). Returns item indices in bucket order.
std::vector<uint32_t> edge_order(const std::vector<uint64_t>& hashes) {
  std::vector<int32_t> bucket;  // -1 = EMPTY
  size_t items = 0;
  auto capacity = [](size_t nb) { return nb < 16 ? nb - 1 : nb / 8 * 7; };  // bucket_mask_to_capacity
  auto place = [&bucket](uint64_t hsh) -> size_t {
    const size_t nb = bucket.size(), mask = nb - 1, mirror_at = std::max<size_t>(nb, 16);
    size_t pos = (size_t)hsh & mask;
    for (size_t stride = 16;; pos = (pos + stride) & mask, stride += 16)
      for (size_t k = 0; k < 16; ++k) {
        const size_t c = pos + k;  // control byte index
        const bool empty = c < nb ? bucket[c] < 0 : c >= mirror_at ? bucket[c - mirror_at] < 0 : true;
        if (!empty) continue;
        size_t idx = c & mask;
        if (bucket[idx] >= 0)
          for (idx = 0; bucket[idx] >= 0; ++idx) {}
        return idx;
      }
  };
  for (size_t it = 0; it < hashes.size(); ++it) {
    if (bucket.empty() || items == capacity(bucket.size())) {
      const size_t want = bucket.empty() ? 1 : capacity(bucket.size()) + 1;  // max(items + 1, cap + 1)
      size_t nb = want < 4 ? 4 : want < 8 ? 8 : 0;
      if (!nb) {
        nb = 1;
        while (nb < want * 8 / 7) nb <<= 1;
      }
      std::vector<int32_t> old;
      old.swap(bucket);
      bucket.assign(nb, -1);
      for (int32_t o : old)
        if (o >= 0) bucket[place(hashes[(size_t)o])] = o;
    }
    bucket[place(hashes[it])] = (int32_t)it;
    ++items;
  }
  std::vector<uint32_t> order;
  for (int32_t b : bucket)
    if (b >= 0) order.push_back((uint32_t)b);
  return order;
}

int32_t lim_max(int32_t acc, int32_t v) {
  if (v == LIM_NONE) return acc;
  return std::max(acc == LIM_NONE ? 0 : acc, v);
}

DevLimits to_dev(const fac_limits& l) { return {l.insertions, l.deletions, l.substitutions, l.swaps, l.edits}; }

bool lim_ok(int32_t v) { return v == LIM_NONE || (v >= 0 && v <= 255); }

}  // namespace

std::vector<uint32_t> transitions_order(const std::vector<std::u32string>& children) {
  std::vector<uint64_t> hs;
  for (auto& g : children) hs.push_back(fx_str_hash(g));
  return edge_order(hs);
}

int build_engine(const fac_pattern* pats, uint64_t np, const fac_config* cfg, Engine& e, std::string& err) {
  e.cfg = *cfg;
  e.device = cfg->device;
  e.case_insensitive = cfg->case_insensitive != 0;
  e.p_ins = cfg->penalty_insertion;
  e.p_del = cfg->penalty_deletion;
  e.p_sub = cfg->penalty_substitution;
  e.p_swp = cfg->penalty_swap;
  e.min_sym = cfg->min_symbol_similarity;
  e.beam_width = cfg->beam_width;
  e.has_auto_beam = cfg->has_auto_beam != 0;
  e.ab_budget = cfg->auto_beam_budget;
  e.ab_width = cfg->auto_beam_width;
  if (cfg->n_mappings > 0 && !cfg->mappings) { err = "NULL mappings"; return FAC_E_INVALID; }
  if (e.has_auto_beam && e.ab_width == 0 && e.beam_width == 0) {
    err = "auto_beam width must be >= 1";
    return FAC_E_INVALID;
  }
  e.has_limits = cfg->has_limits != 0;
  if (e.has_limits) {
    e.limits = to_dev(cfg->limits);
    const fac_limits& l = cfg->limits;
    if (!lim_ok(l.insertions) || !lim_ok(l.deletions) || !lim_ok(l.substitutions) || !lim_ok(l.swaps) ||
        !lim_ok(l.edits)) {
      err = "limits must be 0..255 or None";
      return FAC_E_INVALID;
    }
  }

  // ---- patterns: segment, fold, intern graphemes (builder.rs:195-205, structs.rs:660-754)
  std::unordered_map<std::u32string, uint32_t, U32Hash> gid_of;
  std::vector<std::u32string> gstr;
  std::vector<std::vector<uint32_t>> pat_gids(np);
  e.pats.resize(np);
  std::vector<uint64_t> starts;
  std::u32string folded;
  e.pat_bytes.assign(np, 0);
  for (uint64_t i = 0; i < np; ++i) {
    const uint8_t* s = reinterpret_cast<const uint8_t*>(pats[i].utf8);
    uint64_t len = pats[i].len;
    e.pat_bytes[i] = (uint32_t)std::min<uint64_t>(len, 0xFFFFFFFFull);
    if (len && !s) { err = "NULL pattern"; return FAC_E_INVALID; }
    if (!utf8_valid(s, len)) { err = "pattern is not valid UTF-8"; return FAC_E_INVALID; }
    segment_graphemes(s, len, starts);
    for (size_t g = 0; g < starts.size(); ++g) {
      uint64_t b = starts[g], en = g + 1 < starts.size() ? starts[g + 1] : len;
      fold_grapheme(s, b, en, e.case_insensitive, folded);
      auto it = gid_of.find(folded);
      uint32_t id;
      if (it == gid_of.end()) {
        id = (uint32_t)gstr.size();
        gid_of.emplace(folded, id);
        gstr.push_back(folded);
      } else {
        id = it->second;
      }
      pat_gids[i].push_back(id);
    }
    DevPattern& dp = e.pats[i];
    dp.glen = (float)starts.size();
    dp.weight = pats[i].weight;
    dp.has_limits = pats[i].has_limits != 0;
    dp.lim = dp.has_limits ? to_dev(pats[i].limits) : DevLimits{LIM_NONE, LIM_NONE, LIM_NONE, LIM_NONE, LIM_NONE};
    e.max_glen = std::max<uint32_t>(e.max_glen, (uint32_t)starts.size());
    if (dp.has_limits) {
      const fac_limits& l = pats[i].limits;
      if (!lim_ok(l.insertions) || !lim_ok(l.deletions) || !lim_ok(l.substitutions) || !lim_ok(l.swaps) ||
          !lim_ok(l.edits)) {
        err = "limits must be 0..255 or None";
        return FAC_E_INVALID;
      }
    }
  }

  // ---- trie (builder.rs:207-237)
  std::unordered_map<uint64_t, uint32_t> go;  // (node << 32 | gid) -> child
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> kids(1);  // (gid, child), insertion order
  std::vector<int32_t> pidx(1, -1);
  std::vector<std::vector<uint32_t>> output(1);
  for (uint64_t i = 0; i < np; ++i) {
    uint32_t cur = 0;
    for (uint32_t g : pat_gids[i]) {
      uint64_t key = ((uint64_t)cur << 32) | g;
      auto it = go.find(key);
      uint32_t next;
      if (it == go.end()) {
        next = (uint32_t)kids.size();
        go.emplace(key, next);
        kids[cur].push_back({g, next});
        kids.emplace_back();
        pidx.push_back(-1);
        output.emplace_back();
      } else {
        next = it->second;
      }
      if (pidx[next] < 0) pidx[next] = (int32_t)i;
      cur = next;
    }
    output[cur].push_back((uint32_t)i);
  }
  const size_t nn = kids.size();
  if (nn > (size_t)CHILD26_MASK) { err = "automaton too large (more than 2^26 nodes)"; return FAC_E_UNSUPPORTED; }
  // edges in the reference's transitions-map iteration order (builder.rs:336-342); diagnostics
  // knob FAC_EDGE_INSERTION keeps insertion order (A/B measurements only)
  if (!diag_env("FAC_EDGE_INSERTION")) {
    std::vector<uint64_t> gh(gstr.size());
    for (size_t g = 0; g < gstr.size(); ++g) gh[g] = fx_str_hash(gstr[g]);
    std::vector<uint64_t> hs;
    std::vector<std::pair<uint32_t, uint32_t>> tmp;
    for (auto& k : kids) {
      if (k.size() < 2) continue;
      hs.clear();
      for (auto& c : k) hs.push_back(gh[c.first]);
      tmp.clear();
      for (uint32_t i : edge_order(hs)) tmp.push_back(k[i]);
      k.swap(tmp);
    }
  }

  // ---- fail links, used only to merge outputs (builder.rs:239-276); BFS by depth
  {
    std::vector<uint32_t> fail(nn, 0), queue;
    queue.reserve(nn);
    for (auto& k : kids[0]) queue.push_back(k.second);
    for (size_t qi = 0; qi < queue.size(); ++qi) {
      uint32_t cur = queue[qi];
      for (auto& k : kids[cur]) {
        uint32_t g = k.first, next = k.second;
        uint32_t f = fail[cur];
        while (f != 0 && go.find(((uint64_t)f << 32) | g) == go.end()) f = fail[f];
        auto it = go.find(((uint64_t)f << 32) | g);
        uint32_t fb = it == go.end() ? 0 : it->second;
        fail[next] = fb;
        for (uint32_t p : output[fb])
          if (std::find(output[next].begin(), output[next].end(), p) == output[next].end())
            output[next].push_back(p);
        queue.push_back(next);
      }
    }
  }

  // ---- multi-character mappings (builder.rs:383-442): every rule in both directions; from every
  // node the pattern side is walked through the trie (whole folded graphemes) and, when it is a
  // path, a transition consuming the haystack side is recorded. Haystack-side graphemes join the
  // grapheme dictionary so text graphemes can be compared by id.
  auto intern = [&](const std::u32string& g) -> uint32_t {
    auto it = gid_of.find(g);
    if (it != gid_of.end()) return it->second;
    const uint32_t id = (uint32_t)gstr.size();
    gid_of.emplace(g, id);
    gstr.push_back(g);
    return id;
  };
  e.map_range.assign(nn, uint2{0, 0});
  e.map_ent.clear();
  e.map_hay.clear();
  e.has_map = false;
  e.max_map = 0;
  uint32_t max_map_hay = 1;
  if (cfg->n_mappings > 0) {
    auto fold_side = [&](const char* p, uint64_t len, std::vector<uint32_t>& out) -> bool {
      const uint8_t* u = reinterpret_cast<const uint8_t*>(p);
      if (len && !u) return false;
      if (!utf8_valid(u, len)) return false;
      segment_graphemes(u, len, starts);
      out.clear();
      for (size_t g = 0; g < starts.size(); ++g) {
        fold_grapheme(u, starts[g], g + 1 < starts.size() ? starts[g + 1] : len, e.case_insensitive, folded);
        out.push_back(intern(folded));
      }
      return true;
    };
    struct Directed { std::vector<uint32_t> pat, hay; float penalty; };
    std::vector<Directed> directed;
    std::vector<uint32_t> ga, gb;
    for (uint64_t r = 0; r < cfg->n_mappings; ++r) {
      const fac_mapping& m = cfg->mappings[r];
      if (!fold_side(m.a, m.a_len, ga) || !fold_side(m.b, m.b_len, gb)) {
        err = "mapping is not valid UTF-8";
        return FAC_E_INVALID;
      }
      if (ga.empty() || gb.empty() || ga == gb) continue;
      volatile float one_minus = 1.0f - m.score;  // substitution * (1 - score), two rounded ops
      const float penalty = e.p_sub * one_minus;
      directed.push_back({ga, gb, penalty});
      directed.push_back({gb, ga, penalty});
    }
    for (size_t start = 0; start < nn; ++start) {
      e.map_range[start].x = (uint32_t)e.map_ent.size();
      for (const Directed& d : directed) {
        uint32_t cur = (uint32_t)start;
        bool ok = true;
        for (uint32_t g : d.pat) {
          auto it = go.find(((uint64_t)cur << 32) | g);
          if (it == go.end()) { ok = false; break; }
          cur = it->second;
        }
        if (!ok) continue;
        uint32_t f;
        std::memcpy(&f, &d.penalty, 4);
        e.map_ent.push_back(uint4{(uint32_t)e.map_hay.size(), (uint32_t)d.hay.size(), cur, f});
        for (uint32_t g : d.hay) e.map_hay.push_back(g + 1);
        max_map_hay = std::max<uint32_t>(max_map_hay, (uint32_t)d.hay.size());
      }
      e.map_range[start].y = (uint32_t)e.map_ent.size();
      e.max_map = std::max(e.max_map, e.map_range[start].y - e.map_range[start].x);
    }
    e.has_map = !e.map_ent.empty();
    if (e.max_map > 64) {
      err = "more than 64 mapping transitions at one trie node";
      return FAC_E_UNSUPPORTED;
    }
  }
  e.gid_of.clear();
  e.edge_gid.clear();
  std::memset(e.ascii_gid, 0, sizeof(e.ascii_gid));
  if (e.has_map) {  // ids are 1-based: 0 is "not a known grapheme" and matches no edge
    for (size_t i = 0; i < gstr.size(); ++i) e.gid_of.emplace(gstr[i], (uint32_t)i + 1);
    for (uint32_t b = 0; b < 128; ++b) {  // gs_text of an ASCII byte (grapheme.rs:100-109)
      const uint32_t c = (e.case_insensitive && b >= 'A' && b <= 'Z') ? b + 32 : b;
      auto it = e.gid_of.find(std::u32string(1, (char32_t)c));
      e.ascii_gid[b] = it == e.gid_of.end() ? 0u : it->second;
    }
  }

  // ---- effective limits (builder.rs:289-329), has_pattern_limits, max_edits_fast (:444-468)
  e.has_pattern_limits = false;
  for (auto& p : e.pats) e.has_pattern_limits |= p.has_limits != 0;
  if (!e.has_limits && e.has_pattern_limits) {
    DevLimits m{LIM_NONE, LIM_NONE, LIM_NONE, LIM_NONE, LIM_NONE};
    for (auto& p : e.pats) {
      if (!p.has_limits) continue;
      m.edits = lim_max(m.edits, p.lim.edits);
      m.ins = lim_max(m.ins, p.lim.ins);
      m.del = lim_max(m.del, p.lim.del);
      m.sub = lim_max(m.sub, p.lim.sub);
      m.swp = lim_max(m.swp, p.lim.swp);
    }
    e.has_limits = true;
    e.limits = m;
  }
  if (e.has_pattern_limits) e.max_edits_fast = 255;
  else if (!e.has_limits) e.max_edits_fast = 0;
  else if (e.limits.edits != LIM_NONE && e.limits.ins == LIM_NONE && e.limits.del == LIM_NONE &&
           e.limits.sub == LIM_NONE && e.limits.swp == LIM_NONE)
    e.max_edits_fast = (uint32_t)e.limits.edits;
  else
    e.max_edits_fast = 255;
  // search.rs:204-248 dispatch: 1..=6 specialise, everything else (incl. 0) is the 255 path
  e.mef = (e.max_edits_fast >= 1 && e.max_edits_fast <= 6) ? e.max_edits_fast : 255;

  // ---- flat tables
  e.nodes.assign(nn, HostNode{});
  e.edges.clear();
  e.out_pat.clear();
  e.sb_bits.assign(nn, uint4{0, 0, 0, 0});
  e.max_degree = 0;
  e.max_degree_nonroot = 0;
  for (size_t i = 0; i < nn; ++i) {
    HostNode& d = e.nodes[i];
    d.edge_begin = (uint32_t)e.edges.size();
    for (auto& k : kids[i]) {
      const std::u32string& g = gstr[k.first];
      uint32_t fc = g.empty() ? 0 : (uint32_t)g[0];
      bool single = g.size() == 1 && g[0] < 0x80;  // grapheme byte length == 1 (builder.rs:340)
      uint32_t nx = k.second;
      if (!output[nx].empty()) nx |= EDGE_CHILD_OUTPUT;
      if (single) nx |= EDGE_SINGLE_BYTE;
      e.edges.push_back({fc, nx});
      if (e.has_map) e.edge_gid.push_back(k.first + 1);
      if (single && fc < 128) (&e.sb_bits[i].x)[fc >> 5] |= 1u << (fc & 31);
    }
    d.edge_end = (uint32_t)e.edges.size();
    e.max_degree = std::max(e.max_degree, d.edge_end - d.edge_begin);
    if (i) e.max_degree_nonroot = std::max(e.max_degree_nonroot, d.edge_end - d.edge_begin);
    d.out_begin = (uint32_t)e.out_pat.size();
    for (uint32_t p : output[i]) e.out_pat.push_back(p);
    d.out_end = (uint32_t)e.out_pat.size();
    d.pidx = pidx[i];
  }
  e.sb_edge.resize(e.edges.size());
  for (size_t k = 0; k < e.edges.size(); ++k) e.sb_edge[k] = e.sb_bits[e.edges[k].next & EDGE_NEXT_MASK];
  // reach fixpoint (builder.rs:348-381): children always have larger ids than their parent in a
  // freshly built trie, so one reverse pass reaches the fixpoint.
  std::vector<uint64_t> rl(nn, 0);
  std::vector<float> rw(nn, 0.f);
  for (size_t i = 0; i < nn; ++i)
    for (uint32_t p : output[i]) {
      rl[i] = std::max<uint64_t>(rl[i], (uint64_t)e.pats[p].glen);
      rw[i] = std::fmax(rw[i], e.pats[p].weight);
    }
  for (size_t i = nn; i-- > 0;)
    for (auto& k : kids[i]) {
      rl[i] = std::max(rl[i], rl[k.second]);
      rw[i] = std::fmax(rw[i], rw[k.second]);
    }
  for (size_t i = 0; i < nn; ++i) {
    float len = (float)rl[i];
    e.nodes[i].prune_len = len;
    e.nodes[i].prune_lw = len / rw[i];
  }

  // ---- device node records (fac_internal.h): 32 B per node + side tables
  e.dnodes.resize(nn);
  e.out_range.resize(nn);
  e.node_pidx.resize(nn);
  for (size_t i = 0; i < nn; ++i) {
    const HostNode& h = e.nodes[i];
    const uint32_t deg = h.edge_end - h.edge_begin;
    if (deg > NODE_DEG_MASK) { err = "node degree too large"; return FAC_E_UNSUPPORTED; }
    // edge-set flags for the substitution shortcut: an ASCII first char among the edges, two edges
    // sharing a first char
    uint32_t fl = 0;
    std::vector<uint32_t> chs;
    for (uint32_t a = h.edge_begin; a < h.edge_end; ++a) {
      if (e.edges[a].ch < 128u) fl |= NODE_ASCII_EDGE;
      chs.push_back(e.edges[a].ch);
    }
    std::sort(chs.begin(), chs.end());
    if (std::adjacent_find(chs.begin(), chs.end()) != chs.end()) fl |= NODE_DUP_CH;
    e.dnodes[i] = DevNode{h.prune_len, h.prune_lw, h.edge_begin,
                          deg | fl | (h.out_end != h.out_begin ? NODE_HAS_OUT : 0u), e.sb_bits[i]};
    e.out_range[i] = uint2{h.out_begin, h.out_end};
    e.node_pidx[i] = h.pidx;
  }

  // ---- similarity (structs.rs:30-54)
  if (cfg->similarity_ascii) {
    e.sim_ascii.assign(cfg->similarity_ascii, cfg->similarity_ascii + 128 * 128);
    std::vector<std::pair<uint64_t, float>> pr;
    for (uint64_t k = 0; k < cfg->n_similarity_pairs; ++k) {
      uint32_t a = cfg->similarity_pairs[2 * k], b = cfg->similarity_pairs[2 * k + 1];
      if (a < 128 && b < 128) continue;  // lives in the ASCII table
      pr.push_back({((uint64_t)a << 32) | b, cfg->similarity_pair_values[k]});
    }
    std::stable_sort(pr.begin(), pr.end(), [](auto& x, auto& y) { return x.first < y.first; });
    e.sim_keys.clear();
    e.sim_vals.clear();
    for (size_t k = 0; k < pr.size(); ++k) {
      if (!e.sim_keys.empty() && e.sim_keys.back() == pr[k].first) { e.sim_vals.back() = pr[k].second; continue; }
      e.sim_keys.push_back(pr[k].first);
      e.sim_vals.push_back(pr[k].second);
    }
  } else {
    default_similarity(e.sim_ascii);
  }
  // 128 more entries after the table: for each ASCII text char b, the largest similarity any other
  // ASCII edge char a has to it (table[a][b], a != b): the kernels' no-substitution test
  e.sim_ascii.resize(128 * 128 + 128, 0.0f);
  for (uint32_t b = 0; b < 128; ++b) {
    float m = 0.0f;
    for (uint32_t a = 0; a < 128; ++a)
      if (a != b) m = std::fmax(m, e.sim_ascii[a * 128 + b]);
    e.sim_ascii[128 * 128 + b] = m;
  }

  // ---- 2-gram window skip (search.rs:504-521)
  std::memset(e.first_bits, 0, sizeof(e.first_bits));
  std::memset(e.second_bits, 0, sizeof(e.second_bits));
  e.window_skip = false;
  if (e.mef == 1 && !e.has_map && output[0].empty()) {  // search.rs:505 (WINDOW_SKIP && !MAPPINGS)
    bool child_output = false;
    uint32_t f[4] = {e.sb_bits[0].x, e.sb_bits[0].y, e.sb_bits[0].z, e.sb_bits[0].w};
    uint32_t s2[4] = {0, 0, 0, 0};
    for (auto& k : kids[0]) {
      const uint4& cb = e.sb_bits[k.second];
      const uint32_t c[4] = {cb.x, cb.y, cb.z, cb.w};
      for (int w = 0; w < 4; ++w) { s2[w] |= c[w]; f[w] |= c[w]; }
      if (!output[k.second].empty()) child_output = true;
    }
    if (!child_output) {
      e.window_skip = true;
      std::memcpy(e.first_bits, f, sizeof(f));
      std::memcpy(e.second_bits, s2, sizeof(s2));
    }
  }

  // ---- max_match_graphemes (stream.rs:213-253): longest pattern + edits x longest mapping side
  {
    uint64_t max_edits = 0;
    auto edits_of = [](const DevLimits& l) -> uint64_t {
      if (l.edits != LIM_NONE) return (uint64_t)l.edits;
      auto z = [](int32_t v) { return v == LIM_NONE ? 0ull : (uint64_t)v; };
      return z(l.ins) + z(l.del) + z(l.sub) + z(l.swp);
    };
    for (auto& p : e.pats) {
      const DevLimits* l = p.has_limits ? &p.lim : (e.has_limits ? &e.limits : nullptr);
      max_edits = std::max<uint64_t>(max_edits, l ? edits_of(*l) : 0);
    }
    e.max_match_graphemes = (uint64_t)e.max_glen + max_edits * (uint64_t)max_map_hay;
    if (e.max_match_graphemes + 4 > 0xFFFFu) {
      err = "pattern length + edit budget exceeds the 16-bit window span";
      return FAC_E_UNSUPPORTED;
    }
  }

  // ---- O(1) expansion tables: (node, char) goto entries and child single-byte maps for nodes of
  // degree <= 64, plus each node's child-has-output mask (used by the kernels' fast path)
  {
    e.aux.assign(nn, uint4{0, 0, 0, 0});
    for (size_t i = 0; i < nn; ++i)
      for (uint32_t m = e.nodes[i].edge_begin; m < e.nodes[i].edge_end; ++m)
        e.aux[i].z |= 1u << ch_filt_bit(e.edges[m].ch);
    std::vector<std::pair<uint64_t, uint64_t>> ent;  // (kv, val)
    std::unordered_map<uint64_t, size_t> at;         // kv -> index in ent
    auto put = [&](uint64_t kv) -> uint64_t& {
      auto it = at.find(kv);
      if (it != at.end()) return ent[it->second].second;
      at.emplace(kv, ent.size());
      ent.push_back({kv, 0ull});
      return ent.back().second;
    };
    for (size_t i = 0; i < nn; ++i) {
      const HostNode& h = e.nodes[i];
      const uint32_t deg = h.edge_end - h.edge_begin;
      for (uint32_t k = 0; k < deg; ++k) {  // goto entries for every node (swap resolution)
        const DevEdge& ed = e.edges[h.edge_begin + k];
        const uint32_t child = ed.next & EDGE_NEXT_MASK;
        const uint64_t key = ((uint64_t)i << 21) | ed.ch;
        const bool existed = at.count(GT_VALID | GT_GOTO | key) != 0;
        uint64_t& g = put(GT_VALID | GT_GOTO | key);
        if (!existed)  // first edge with this first char; the child's folded char filter on top
          g = child | ((uint64_t)std::min<uint32_t>(k, 255) << 32) | ((uint64_t)filt_fold16(e.aux[child].z) << 48);
        if (ed.next & EDGE_SINGLE_BYTE) g |= 1ull << 40;
        if (deg > 64) continue;  // child maps only for the fast path's nodes
        if (ed.next & EDGE_CHILD_OUTPUT) (k < 32 ? e.aux[i].x : e.aux[i].y) |= 1u << (k & 31u);
        const HostNode& c = e.nodes[child];
        for (uint32_t m = c.edge_begin; m < c.edge_end; ++m) {
          const DevEdge& ce = e.edges[m];
          if ((ce.next & EDGE_SINGLE_BYTE) && ce.ch < 128) {
            put(GT_VALID | GT_SB | ((uint64_t)i << 21) | ce.ch) |= 1ull << k;
            e.aux[i].w |= 1u << ch_filt_bit(ce.ch);
          }
        }
      }
    }
    // cuckoo placement (load <= ~0.4): random-walk eviction, reseed / grow on failure
    uint32_t ns = 16;
    while (ns * 2 < ent.size() * 5) ns <<= 1;
    uint64_t rng = 0x2545F4914F6CDD1Dull;
    auto next_rand = [&]() {
      rng ^= rng << 13;
      rng ^= rng >> 7;
      rng ^= rng << 17;
      return rng;
    };
    for (int attempt = 0;; ++attempt) {
      if (attempt > 0 && attempt % 4 == 0) ns <<= 1;
      e.gt_mask = ns - 1;
      e.gt_seed1 = next_rand();
      e.gt_seed2 = next_rand();
      e.gt.assign(ns, uint4{0, 0, 0, 0});
      bool ok = true;
      for (auto& kvv : ent) {
        uint64_t kv = kvv.first, val = kvv.second;
        uint32_t pos = 0;
        bool placed = false;
        for (int kick = 0; kick < 500 && !placed; ++kick) {
          uint32_t p1, p2;
          gt_slots(kv, e.gt_seed1, e.gt_mask, p1, p2);
          for (uint32_t p : {p1, p2}) {
            if (e.gt[p].x == 0 && e.gt[p].y == 0) {
              e.gt[p] = uint4{(uint32_t)kv, (uint32_t)(kv >> 32), (uint32_t)val, (uint32_t)(val >> 32)};
              placed = true;
              break;
            }
          }
          if (placed) break;
          pos = (next_rand() & 1) ? p1 : p2;  // evict one occupant and re-place it
          const uint4 old = e.gt[pos];
          e.gt[pos] = uint4{(uint32_t)kv, (uint32_t)(kv >> 32), (uint32_t)val, (uint32_t)(val >> 32)};
          kv = ((uint64_t)old.y << 32) | old.x;
          val = ((uint64_t)old.w << 32) | old.z;
        }
        if (!placed) {
          ok = false;
          break;
        }
      }
      if (ok) break;
    }
    bool sims01 = true;  // every similarity in [0, 1]: p_sub * (1 - sim) in [0, p_sub]
    for (float v : e.sim_ascii) sims01 = sims01 && v >= 0.0f && v <= 1.0f;
    for (float v : e.sim_vals) sims01 = sims01 && v >= 0.0f && v <= 1.0f;
    // with mappings the exact/swap transitions compare whole graphemes: per-edge path only
    e.gt_fast = sims01 && e.min_sym <= 0.0f && e.p_sub >= 0.0f && !e.has_map;
  }

  // ---- bitap pre-filter tables (prefilter.rs:161-245)
  e.bitap_ok = false;
  do {
    if (np == 0 || e.has_map) break;  // prefilter.rs:162-165: mappings are not unit edits
    float max_sim = 0.f;  // structs.rs:61-76
    for (int i = 0; i < 128; ++i)
      for (int j = 0; j < 128; ++j)
        if (i != j) max_sim = std::fmax(max_sim, e.sim_ascii[i * 128 + j]);
    for (size_t k = 0; k < e.sim_keys.size(); ++k)
      if ((e.sim_keys[k] >> 32) != (e.sim_keys[k] & 0xFFFFFFFFull)) max_sim = std::fmax(max_sim, e.sim_vals[k]);
    float p_sub_min = e.p_sub * (1.0f - max_sim);
    float mults[4] = {1.0f / e.p_ins, 1.0f / e.p_del, 1.0f / p_sub_min, 2.0f / e.p_swp};
    bool ok = true;
    for (float m : mults)
      if (!std::isfinite(m) || m <= 0.0f) ok = false;
    if (!ok) break;
    float ecm = 0.f;
    for (float m : mults) ecm = std::fmax(ecm, m);
    std::unordered_map<uint32_t, uint32_t> sym_of_gid;  // gid -> symbol id
    std::vector<std::vector<uint32_t>> ids(np);
    for (uint64_t i = 0; i < np && ok; ++i) {
      size_t m = pat_gids[i].size();
      if (m == 0 || m > 63) { ok = false; break; }
      for (uint32_t g : pat_gids[i]) {
        auto it = sym_of_gid.find(g);
        uint32_t id;
        if (it == sym_of_gid.end()) {
          id = (uint32_t)sym_of_gid.size() + 1;
          sym_of_gid.emplace(g, id);
        } else {
          id = it->second;
        }
        if (id > 255) { ok = false; break; }
        ids[i].push_back(id);
      }
    }
    if (!ok) break;
    e.edit_cost_mult = ecm;
    e.alphabet = (uint32_t)sym_of_gid.size();
    e.symbol_ids.clear();
    for (auto& kv : sym_of_gid) e.symbol_ids.push_back({gstr[kv.first], kv.second});
    std::sort(e.symbol_ids.begin(), e.symbol_ids.end());
    std::memset(e.ascii_id, 0, sizeof(e.ascii_id));
    for (int b = 0; b < 128; ++b) {
      uint32_t ch = (uint32_t)b;
      if (e.case_insensitive && ch >= 'A' && ch <= 'Z') ch += 32;
      std::u32string key(1, (char32_t)ch);
      auto it = gid_of.find(key);
      if (it != gid_of.end()) {
        auto s = sym_of_gid.find(it->second);
        if (s != sym_of_gid.end()) e.ascii_id[b] = (uint8_t)s->second;
      }
    }
    e.bp_m.assign(np, 0);
    e.bp_weight.assign(np, 0.f);
    e.bp_k_limit.assign(np, -1);
    e.bp_mask.assign(np * (e.alphabet + 1), 0);
    for (uint64_t i = 0; i < np; ++i) {
      e.bp_m[i] = (uint32_t)ids[i].size();
      e.bp_weight[i] = e.pats[i].weight;
      const DevLimits* l = e.pats[i].has_limits ? &e.pats[i].lim : (e.has_limits ? &e.limits : nullptr);
      if (l) {  // k_from_limits (prefilter.rs:388-405)
        if (l->edits != LIM_NONE) e.bp_k_limit[i] = l->swp == 0 ? l->edits : 2 * (int64_t)l->edits;
        else if (l->ins != LIM_NONE && l->del != LIM_NONE && l->sub != LIM_NONE && l->swp != LIM_NONE)
          e.bp_k_limit[i] = (int64_t)l->ins + l->del + l->sub + 2 * (int64_t)l->swp;
      }
      for (size_t k = 0; k < ids[i].size(); ++k) e.bp_mask[i * (e.alphabet + 1) + ids[i][k]] |= 1ull << k;
    }
    e.bitap_ok = true;
  } while (false);
  return FAC_OK;
}

}  // namespace fac
