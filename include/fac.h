/* fac.h — C ABI of the MI355X-native fuzzy Aho–Corasick engine (libfac.so).
 *
 * Drop-in boundary for the hot path of kakserpom/fuzzy-aho-corasick-rs v0.5.0 (reference at
 * /root/reference). Everything public in the crate funnels through one crate-private seam,
 *
 *     pub(crate) fn search_raw(&'a self, haystack: &'a str, similarity_threshold: f32)
 *         -> Result<FuzzyMatches<'a>, SearchError>                       (src/search.rs:187-191)
 *
 * plus the engine constructor `FuzzyAhoCorasickBuilder::build` (src/builder.rs:181) and the
 * pre-filter wrapper `Prefiltered::search` (src/prefilter.rs:135-155). The entry points below are
 * exactly what a Rust `extern "C"` block (or any FFI) would bind to replace those; see
 * INTEGRATION.md for the binding a maintainer would add. Plain pointers and sizes only; no C++ or
 * torch types cross this boundary. All functions are reentrant; an engine is immutable after
 * fac_build and may be shared across host threads (structs.rs:528-567).
 *
 * Return codes (SearchError is #[non_exhaustive], src/error.rs:7-17, so new codes follow the
 * reference's own convention):
 *   FAC_OK                      0
 *   FAC_E_HAYSTACK_TOO_LARGE    1   SearchError::HaystackTooLarge{graphemes} (search.rs:198-201)
 *   FAC_E_INVALID             100   bad argument (NULL, invalid UTF-8, beam_width == 0, ...)
 *   FAC_E_UNSUPPORTED         101   configuration outside the GPU path (> 64 mapping transitions
 *                                   at one node, > 2^26 nodes, ...) — never a silent CPU fallback
 *   FAC_E_HIP                 102   HIP runtime error (fac_last_error() has the text)
 *   FAC_E_NO_DEVICE           103   no usable MI355X (gfx950) device
 *   FAC_E_OOM                 104   host or device allocation failure
 *   FAC_E_CAPACITY            105   a per-window device work buffer overflowed even after the
 *                                   automatic retries (pathological input)
 *   FAC_E_OUTPUT_CAPACITY     106   the caller's device output buffer is too small; *n_out holds
 *                                   the record count needed (fac_search_staged_ex)
 *   FAC_E_INTERNAL            107   unexpected internal error (fac_last_error() has the text)
 *
 * Diagnostics: the library reads FAC_* environment knobs (kernel variants, prefix-cache levels,
 * FAC_GRAPHEME_LIMIT, ...) only when FAC_DIAGNOSTICS=1 is set; otherwise the search path depends
 * on the arguments alone.
 */
#ifndef FAC_H
#define FAC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FAC_OK 0
#define FAC_E_HAYSTACK_TOO_LARGE 1
#define FAC_E_INVALID 100
#define FAC_E_UNSUPPORTED 101
#define FAC_E_HIP 102
#define FAC_E_NO_DEVICE 103
#define FAC_E_OOM 104
#define FAC_E_CAPACITY 105
#define FAC_E_OUTPUT_CAPACITY 106
#define FAC_E_INTERNAL 107

#define FAC_LIMIT_NONE (-1)

/* FuzzyLimits (src/structs.rs:293-299), already finalized (structs.rs:319-335):
 * each field is a count 0..255 or FAC_LIMIT_NONE. */
typedef struct fac_limits {
  int32_t insertions;
  int32_t deletions;
  int32_t substitutions;
  int32_t swaps;
  int32_t edits;
} fac_limits;

/* One Pattern (src/structs.rs:598-610). `custom_unique_id` only matters for host-side
 * overlap resolution and is not passed. */
typedef struct fac_pattern {
  const char* utf8; /* pattern text, valid UTF-8 */
  uint64_t len;     /* bytes */
  float weight;     /* Pattern::weight, default 1.0 */
  int32_t has_limits;
  fac_limits limits; /* per-pattern limits, finalized; used iff has_limits */
} fac_pattern;

/* One multi-character mapping rule (a, b, score), builder.rs:30-31, 116-132: either side may
 * stand in for the other at penalty substitution * (1 - score), counted as one substitution. */
typedef struct fac_mapping {
  const char* a; /* UTF-8 */
  uint64_t a_len;
  const char* b; /* UTF-8 */
  uint64_t b_len;
  float score;
} fac_mapping;

/* Builder state (src/builder.rs:22-33, FuzzyPenalties structs.rs:370-393). */
typedef struct fac_config {
  int32_t case_insensitive;
  int32_t has_limits;   /* FuzzyAhoCorasickBuilder::fuzzy(...) called */
  fac_limits limits;    /* finalized global limits */
  float penalty_insertion;
  float penalty_deletion;
  float penalty_substitution;
  float penalty_swap;
  uint64_t beam_width;  /* 0 = None (exact exploration) */
  int32_t has_auto_beam;
  uint64_t auto_beam_budget;
  uint64_t auto_beam_width;
  float min_symbol_similarity;
  /* Custom Similarity (structs.rs:30-54); NULL = the crate's DEFAULT_SIMILARITY
   * (builder.rs:492-526). similarity_ascii is a 128x128 row-major table indexed [a][b];
   * the pair list holds entries with a or b >= 128. */
  const float* similarity_ascii;
  uint64_t n_similarity_pairs;
  const uint32_t* similarity_pairs; /* 2*n code points (a, b) */
  const float* similarity_pair_values;
  /* Multi-character mappings (builder.rs:108-132, mapping / mapping_scored): applied
   * bidirectionally; precomputed per trie node like builder.rs:383-442. */
  uint64_t n_mappings;
  const struct fac_mapping* mappings;
  int32_t device; /* HIP device ordinal for this engine's tables */
} fac_config;

/* Owned match record: the crate's OwnedMatch/StreamMatch POD (src/stream.rs:719-745), 32 bytes,
 * identical on host, device and the RCCL wire. `start`/`end` are byte offsets into the haystack;
 * the host rebuilds `text = haystack[start..end]`. */
typedef struct fac_match {
  uint64_t start;
  uint64_t end;
  uint32_t pattern_index;
  float similarity;
  uint8_t insertions;
  uint8_t deletions;
  uint8_t substitutions;
  uint8_t swaps;
  uint8_t edits;
  uint8_t pad[3];
} fac_match;

/* Per-call device statistics (filled when the pointer is non-NULL). */
typedef struct fac_stats {
  double kernel_ms;        /* HIP-event time of the window search kernel(s) on the call's stream */
  double prefilter_ms;     /* HIP-event time of the bitap scan + window merge (0 if unused) */
  uint64_t kernel_launches;
  uint64_t windows;        /* start windows searched */
  uint64_t states_popped;  /* BFS states popped by the search kernel (work diagnostic) */
  uint64_t graphemes;      /* haystack graphemes */
  uint64_t bytes;          /* haystack UTF-8 bytes */
  uint64_t retries;        /* capacity retries */
  double cache_ms;         /* HIP-event time of the prefix cache: key counts, snapshot builds, per-window lookups */
  uint64_t states_cached;  /* pops replayed from prefix-cache snapshots (not in states_popped) */
  double lane_ms;          /* HIP-event time of the lane-serial search of small resumed windows */
  uint64_t lane_windows;   /* windows finished by the lane-serial kernel */
} fac_stats;

typedef struct fac_engine fac_engine;
typedef struct fac_haystack fac_haystack;

/* Last error text of the calling thread ("" if none). */
const char* fac_last_error(void);

/* FuzzyAhoCorasickBuilder::build (builder.rs:181-484): builds the trie, fail-link output merge
 * and prune coefficients on the host and uploads the device tables to cfg->device. */
int fac_build(const fac_pattern* patterns, uint64_t n_patterns, const fac_config* cfg,
              fac_engine** out);
void fac_engine_free(fac_engine* engine);
/* Frees the device blocks the library keeps for reuse between calls (per-call scratch of the
 * pre-filter, ranking and stream windows; at most 2 GiB are kept, fac_engine_free trims too). */
void fac_trim_scratch(void);

/* FuzzyAhoCorasick::search_raw (search.rs:187-395): best-per-(start,end,pattern) matches at or
 * above `threshold`, unordered. *out is allocated by the library (fac_matches_free). On
 * FAC_E_HAYSTACK_TOO_LARGE, *err_graphemes receives the grapheme count. */
int fac_search_raw(const fac_engine* engine, const uint8_t* utf8, uint64_t len, float threshold,
                   fac_match** out, uint64_t* n_out, uint64_t* err_graphemes);
void fac_matches_free(fac_match* matches);

/* FuzzyAhoCorasick::with_prefilter + Prefiltered (prefilter.rs:113-155). */
int fac_prefilter_active(const fac_engine* engine);
int fac_search_prefiltered(const fac_engine* engine, const uint8_t* utf8, uint64_t len,
                           float threshold, fac_match** out, uint64_t* n_out,
                           uint64_t* err_graphemes);

/* FuzzyAhoCorasick::max_match_graphemes (stream.rs:213-253). */
uint64_t fac_max_match_graphemes(const fac_engine* engine);

/* Device-resident haystacks (bench / sharded multi-GPU). fac_haystack_stage performs the
 * search_raw staging (is_ascii, grapheme segmentation + folding, search.rs:196-203/296-302)
 * and uploads the result to the engine's device; the staged haystack can then be searched
 * repeatedly with no host->device traffic. */
int fac_haystack_stage(const fac_engine* engine, const uint8_t* utf8, uint64_t len,
                       fac_haystack** out, uint64_t* err_graphemes);
/* search_raw's staging of UTF-8 bytes that are already in device memory (`d_utf8`, a device
 * pointer on the engine's device; borrowed, not copied: keep it alive and unchanged while the
 * haystack is used): the UTF-8 check (the C ABI's stand-in for `&str`), is_ascii, UAX #29
 * segmentation and folding, all on the device (search.rs:196-203, 296-302), ordered on `stream`
 * (a hipStream_t; NULL = the engine's) and complete on return. `*hay`: NULL to create a haystack,
 * or one returned earlier by this function for the same engine, whose device buffers are then
 * reused (staging again per search costs no allocation). Errors as fac_haystack_stage; on error
 * `*hay` is left as passed. */
int fac_haystack_stage_device(const fac_engine* engine, const uint8_t* d_utf8, uint64_t len, void* stream,
                              fac_haystack** hay, uint64_t* err_graphemes);
uint64_t fac_haystack_graphemes(const fac_haystack* hay);
/* Byte start of every staged grapheme (the device segmentation's result, for tests / hosts that
 * map windows to bytes). Writes up to `cap` entries, returns the grapheme count. */
uint64_t fac_haystack_grapheme_starts(const fac_haystack* hay, uint64_t* out, uint64_t cap);
void fac_haystack_free(fac_haystack* hay);

/* Search start windows [window_begin, window_end) of a staged haystack (window_end is clamped
 * to the grapheme count). Searching every window reproduces search_raw; disjoint window ranges
 * give disjoint match sets (the best-map key holds the start byte), which is how the host shards
 * one haystack across GPUs. `stream` is a hipStream_t (NULL = the engine's stream). */
int fac_search_staged(const fac_engine* engine, const fac_haystack* hay, uint64_t window_begin,
                      uint64_t window_end, float threshold, void* stream, fac_match** out,
                      uint64_t* n_out, fac_stats* stats);

/* Extended staged search. Records go to the host (*out, fac_matches_free) or, with device_out set,
 * straight into that device buffer of device_cap records on the engine's device (no host copy: the
 * multi-GPU gather sends them over RCCL from there); *n_out is the record count either way, and
 * FAC_E_OUTPUT_CAPACITY means the buffer was too small (grow it to *n_out and search again).
 * auto_beam_prefix: for a shard of one haystack, the running auto-beam total (sum of queue.len())
 * of every window before this shard (search.rs:1096-1103; fac_auto_beam_total), 0 otherwise. */
typedef struct fac_search_args {
  uint64_t window_begin;
  uint64_t window_end;
  float threshold;
  void* stream;
  uint64_t auto_beam_prefix;
  void* device_out;
  uint64_t device_cap;
} fac_search_args;
int fac_search_staged_ex(const fac_engine* engine, const fac_haystack* hay, const fac_search_args* args,
                         fac_match** out, uint64_t* n_out, fac_stats* stats);

/* Auto-beam pass 1 alone (search.rs:1096-1103): the sum of queue.len() over the start windows
 * [window_begin, window_end) searched unbeamed. A sharded search of an auto-beam engine exchanges
 * these totals so every shard switches the beam on at the same global window as search_raw. */
int fac_auto_beam_total(const fac_engine* engine, const fac_haystack* hay, uint64_t window_begin, uint64_t window_end,
                        float threshold, void* stream, uint64_t* total);

/* Sharding one haystack over n_shards GPUs. fac_shard_plan cuts the bytes into
 * contiguous shards at grapheme boundaries whose segmentation needs no left context (any byte of
 * an ASCII haystack; otherwise after an ASCII non-CR character, before a character that is not
 * Extend/ZWJ/SpacingMark; host-only, no device needed) and returns plan = {a, b, e, flags}: the shard owns the start windows of
 * bytes [a, b) and must stage bytes [a, e), e = b plus max_match_graphemes() + 2 graphemes (the
 * stream overlap of stream.rs:256-258 and the text[j+1] lookahead; max_match_graphemes is
 * fac_max_match_graphemes(engine)), flags bit 0 = global is_ascii,
 * bit 1 = the text continues past e. is_ascii: the haystack's is_ascii if known, -1 to compute it.
 * fac_haystack_stage_shard stages such a slice: searched with fac_search_staged[_ex] it yields
 * exactly the records search_raw of the whole haystack yields for the owned start windows, at
 * global byte offsets (slice offset + base). */
int fac_shard_plan(uint64_t max_match_graphemes, const uint8_t* utf8, uint64_t len, int32_t is_ascii, uint64_t n_shards,
                   uint64_t shard, uint64_t plan[4]);
int fac_haystack_stage_shard(const fac_engine* engine, const uint8_t* utf8, uint64_t len, uint64_t owned_bytes,
                             int32_t global_ascii, int32_t open_end, uint64_t base, fac_haystack** out,
                             uint64_t* err_graphemes);
/* fac_haystack_stage_shard for a shard whose bytes [a, e) are already in device memory (`d_utf8`,
 * borrowed like fac_haystack_stage_device's, which it otherwise follows: staging on the device,
 * ordered on `stream`, complete on return; `*hay` NULL or a haystack this function staged before,
 * restaged in place). The grapheme mode is the global is_ascii; a Unicode shard's bytes are UTF-8
 * checked on the device. Replaces nothing in the reference: it is the per-step staging of the
 * sharded search_raw (search.rs:196-203, 296-302 on each rank's slice). */
int fac_haystack_stage_shard_device(const fac_engine* engine, const uint8_t* d_utf8, uint64_t len, uint64_t owned_bytes,
                                    int32_t global_ascii, int32_t open_end, uint64_t base, void* stream, fac_haystack** hay,
                                    uint64_t* err_graphemes);
/* start windows a staged haystack owns (all of them unless it is a shard) */
uint64_t fac_haystack_owned_windows(const fac_haystack* hay);
/* Strong-scaling split by key instead of by position: searches of `hay` cover only the start windows
 * whose first two (folded) characters hash to `part` of `parts` (parts = 1: all). Every window of a
 * prefix lands in one part, so each GPU's prefix cache holds whole keys -- a position
 * shard of 1/N shares its keys with every other shard and rebuilds them. The union of the parts'
 * records is the whole haystack's search_raw (windows are independent). FAC_E_UNSUPPORTED for
 * auto_beam engines (a running count over windows in order, search.rs:1096-1103). */
int fac_haystack_set_key_partition(const fac_engine* engine, fac_haystack* hay, uint32_t parts, uint32_t part);

/* One streaming window on the device (stream.rs:262-297 window_matches): the graphemes
 * [g_begin, g_end) of a staged haystack are searched as the window's text (Prefiltered::search if
 * `prefilter`, else search), ranked sorted().non_overlapping() (matches.rs), and the matches the
 * window owns (start byte < commit_bytes, relative to the window) are returned at absolute offsets
 * base + window offset. */
int fac_stream_window_staged(const fac_engine* engine, const fac_haystack* hay, uint64_t g_begin, uint64_t g_end,
                             uint64_t commit_bytes, uint64_t base, float threshold, int32_t prefilter, void* stream,
                             fac_match** out, uint64_t* n_out, fac_stats* stats);

/* fac_stream_window_staged with the owned records left in HBM (no host round trip): the window's
 * raw records are ranked sorted().non_overlapping() on the device and the owned ones (start before
 * the commit point) written, rebased to the stream offset `base`, to device_out (room for device_cap
 * records). *n_out = the owned count; FAC_E_OUTPUT_CAPACITY when it exceeds device_cap (nothing is
 * written then; grow the buffer and call again). For the multi-GPU gather of C5 (stream.rs:378-429). */
int fac_stream_window_staged_device(const fac_engine* engine, const fac_haystack* hay, uint64_t g_begin, uint64_t g_end,
                                    uint64_t commit_bytes, uint64_t base, float threshold, int32_t prefilter, void* stream,
                                    void* device_out, uint64_t device_cap, uint64_t* n_out, fac_stats* stats);

/* A batch of streaming windows (stream.rs:262-297 window_matches for each; the crate cuts them
 * DEFAULT_WINDOW = 256 KiB apart, stream.rs:65): windows[4 w .. 4 w + 3] = (g_begin, g_end,
 * commit_bytes, base) of window w, ascending g_begin, each overlapping only its neighbours. Every
 * window is searched as its own text exactly like fac_stream_window_staged_device; on an ASCII
 * haystack the batch is one pre-filter pass over the windows' union (each window's bitap automaton
 * starting at its first byte) and one search launch over every window's segments, then per-window
 * ranking and commit cut. The owned records of all windows go to device_out in window order;
 * *n_out = their count (FAC_E_OUTPUT_CAPACITY when it exceeds device_cap). */
int fac_stream_windows_staged_device(const fac_engine* engine, const fac_haystack* hay, const uint64_t* windows,
                                     uint64_t n_windows, float threshold, int32_t prefilter, void* stream, void* device_out,
                                     uint64_t device_cap, uint64_t* n_out, fac_stats* stats);

/* Prefiltered::raw on a staged haystack (prefilter.rs:146-155, 304-374): the bitap scan and the
 * window merge run on the device-resident text, each merged window is re-searched as its own
 * sub-haystack, results are best-per-(start, end, pattern) and sorted. Falls back to the full
 * search exactly where the reference does (no bitap filter, or some pattern needs k > 24). */
int fac_search_staged_prefiltered(const fac_engine* engine, const fac_haystack* hay, float threshold,
                                  void* stream, fac_match** out, uint64_t* n_out, fac_stats* stats);

/* FuzzyMatches::apply (matches.rs:7-149) on the device: rank `n` raw records in place by `order`
 * (0 Unsorted, 1 Default, 2 Greedy, 3 CoverageWeighted; matches.rs:23-81) and resolve overlaps by
 * `overlap` (0 Keep, 1 NonOverlapping, 2 NonOverlappingUnique; matches.rs:83-149). `unique_ids`
 * (NULL = the pattern index) maps a pattern index to its uniqueness key for overlap 2 (distinct keys
 * for custom_unique_id and automatic ids). The surviving records are compacted to the front of
 * `matches`, their count written to `n_out`. */
int fac_matches_apply(const fac_engine* engine, fac_match* matches, uint64_t n, int32_t order, int32_t overlap,
                      const uint64_t* unique_ids, uint64_t* n_out);

/* Streaming search (stream.rs:77-297): feed the input in the reader's read() pieces; windows
 * of `window_bytes` (0 = the crate's 256 KiB) are cut, searched (sorted + non-overlapping) and
 * their owned matches returned with absolute byte offsets, exactly like search_stream. Two windows
 * are searched at a time on two HIP streams (the next window's upload and search overlap the
 * current one's); matches are still returned in stream order. Each feed
 * returns the matches completed so far (`*out`, free with fac_matches_free) and their matched
 * bytes concatenated in the same order (`*text`, match i has end - start bytes; free with
 * fac_buffer_free). Pass eof = 1 (data may be empty) once the input has ended. */
typedef struct fac_stream fac_stream;
int fac_stream_open(const fac_engine* engine, float threshold, uint64_t window_bytes, fac_stream** out);
int fac_stream_feed(fac_stream* stream, const uint8_t* data, uint64_t len, int32_t eof, fac_match** out,
                    uint64_t* n_out, uint8_t** text, uint64_t* text_len);
uint64_t fac_stream_total(const fac_stream* stream);
/* Commit point of the windows whose matches were handed out so far: every match still to come
 * starts at or after this offset (the streaming replace copies the text before it through). */
uint64_t fac_stream_committed(const fac_stream* stream);
void fac_stream_close(fac_stream* stream);
void fac_buffer_free(void* p);

/* Diagnostics: the merged candidate windows (grapheme ranges [start, end)) of the bitap
 * pre-filter for `threshold` (prefilter.rs:319-342). Returns the window count (writes up to `cap`
 * pairs into `out`), or -1 if the pre-filter would fall back to a full search. */
int64_t fac_prefilter_windows(const fac_engine* engine, const uint8_t* utf8, uint64_t len, float threshold,
                              uint64_t* out, uint64_t cap);

/* Engine introspection (tests / diagnostics). */
uint64_t fac_engine_num_nodes(const fac_engine* engine);
uint32_t fac_engine_max_edits_fast(const fac_engine* engine);

/* Host-side UTF-8 staging helpers exposed for tests: extended grapheme cluster segmentation
 * (UAX #29) and per-grapheme first-code-point folding. Writes up to `cap` entries. */
uint64_t fac_segment_graphemes(const uint8_t* utf8, uint64_t len, uint64_t* starts, uint64_t cap);
uint32_t fac_fold_first_char(const uint8_t* utf8, uint64_t len, int32_t case_insensitive);

/* Host-side builder helper exposed for tests: the order in which the reference iterates a trie
 * node's `transitions: FxHashMap<String, u32>` (builder.rs:336-342; FxHasher structs.rs:95-156 +
 * std's hashbrown) given the children's graphemes in insertion order (code points: grapheme i is
 * cps[off[i] .. off[i+1])). Writes the n insertion indices in iteration order to `order`. */
void fac_edge_order(const uint32_t* cps, const uint64_t* off, uint64_t n, uint32_t* order);

/* Diagnostics (tests): the device beam cut alone. Array a holds keys[offs[a] .. offs[a+1]) as the
 * penalties of a queue's pending states (2*bw < length <= 256 for lds != 0, <= 1024 otherwise); the
 * kernel keeps bw of them exactly as the search's beam does -- the reference's
 * `queue[q_idx..].select_nth_unstable_by(bw - 1, total_cmp)` + `truncate(q_idx + bw)`
 * (search.rs:584-587) -- and writes the survivors' original indices, in queue order, to
 * perm[a*bw .. a*bw + bw). sel_limit < 0: core's 16 partition rounds. Uses device 0. */
int fac_diag_beam_select(const float* keys, const uint64_t* offs, uint64_t count, uint32_t bw, int32_t lds,
                         int32_t sel_limit, uint32_t* perm);

#ifdef __cplusplus
}
#endif

#endif /* FAC_H */
