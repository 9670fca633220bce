"""GPU tests of the round-2 paths: halo-sliced shard staging (fac_shard_plan +
fac_haystack_stage_shard), device-resident record output (fac_search_staged_ex), device stream
windows (fac_stream_window_staged, the C5 driver's unit of work), SearchError::HaystackTooLarge
through the C ABI, and the FAC_DIAGNOSTICS gate on the library's tuning knobs."""
import os
import subprocess
import sys

import numpy as np
import pytest

from fuzzy_aho_corasick import FuzzyAhoCorasickBuilder as B, FuzzyLimits as L, HaystackTooLarge, SearchOptions as O
from fuzzy_aho_corasick import workloads as W
from fuzzy_aho_corasick.engine import StagedHaystack
from oracle_harness import OracleEngine

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def recs_key(recs):
    return sorted((int(r["start"]), int(r["end"]), int(r["pattern_index"]), int(np.float32(r["similarity"]).view(np.uint32)),
                   int(r["edits"])) for r in recs)


def rows_key(rows):
    return sorted((r[0], r[1], r[2], int(np.float32(r[3]).view(np.uint32)), r[8]) for r in rows)


def _c3_slice(nbytes):
    wl = W.config("c3", nbytes)
    return wl, W.builder_for(wl).device(0)


@pytest.mark.parametrize("config,nbytes,shards", [("c3", 96 << 10, (2, 3, 5)), ("c2", 256 << 10, (2, 4))])
def test_shards_union_equals_whole(config, nbytes, shards):
    """Each shard stages only its owned bytes + halo; the union of the shards' records (at global
    offsets) equals the whole haystack's search_raw on every field. The slices are large enough for
    the prefix cache (>= 4096 windows per shard) and the C3 engine is beamed."""
    wl = W.config(config, nbytes)
    eng = W.builder_for(wl).device(0).build(wl.patterns)
    whole = StagedHaystack(eng, wl.haystack)
    want = rows_key(whole.search_windows(wl.threshold)[0])
    assert len(want) > 20
    for n in shards:
        got = []
        for r in range(n):
            sh = StagedHaystack.shard(eng, wl.haystack, n, r)
            assert sh.owned_windows <= sh.graphemes
            got += sh.search_windows(wl.threshold)[0]
        assert rows_key(got) == want, (config, n)


@pytest.mark.parametrize("config,nbytes,n", [("c3", 96 << 10, 3), ("c2", 256 << 10, 4)])
def test_device_staged_shards_equal_host_staged(config, nbytes, n):
    """bench.py --shard's per-step staging: each rank's shard bytes [a, e) held in HBM and staged on
    the device (fac_haystack_stage_shard_device, global is_ascii, owned windows counted on the
    device), restaged in place twice: the same graphemes, owned windows and records as the host-staged
    shard, and the union over the shards == the whole haystack. A Unicode shard that is all ASCII
    still stages as graphemes ("\r\n" is one cluster) when the whole haystack is not ASCII."""
    import torch
    from fuzzy_aho_corasick import _native
    wl = W.config(config, nbytes)
    eng = W.builder_for(wl).device(0).build(wl.patterns)
    want = rows_key(StagedHaystack(eng, wl.haystack).search_windows(wl.threshold)[0])
    got = []
    for r in range(n):
        plan = _native.shard_plan(eng.max_match_graphemes(), wl.haystack, n, r)
        host = StagedHaystack.shard(eng, wl.haystack, n, r)
        dev = torch.from_numpy(np.frombuffer(wl.haystack, np.uint8)[plan[0]:plan[2]].copy()).cuda()
        sh = StagedHaystack.shard_from_device(eng, dev.data_ptr(), plan)
        for _ in range(2):
            sh = StagedHaystack.shard_from_device(eng, dev.data_ptr(), plan, reuse=sh)
            assert (sh.graphemes, sh.owned_windows) == (host.graphemes, host.owned_windows)
            rows = sh.search_windows(wl.threshold)[0]
            assert rows_key(rows) == rows_key(host.search_windows(wl.threshold)[0])
        got += rows
    assert rows_key(got) == want and len(want) > 20
    # an ASCII-only shard of a Unicode haystack: graphemes, not bytes
    data = ("ab\r\ncd " * 50 + "école \r\n" * 50).encode()
    plan = _native.shard_plan(eng.max_match_graphemes(), data, 2, 0)
    assert plan[3] is False
    dev = torch.from_numpy(np.frombuffer(data, np.uint8)[plan[0]:plan[2]].copy()).cuda()
    sh = StagedHaystack.shard_from_device(eng, dev.data_ptr(), plan)
    host = StagedHaystack.shard(eng, data, 2, 0)
    assert (sh.graphemes, sh.owned_windows) == (host.graphemes, host.owned_windows)


@pytest.mark.parametrize("config,nbytes,parts", [("c3", 96 << 10, (2, 3, 8)), ("c2", 256 << 10, (2, 5)), ("c3", 5000, (3,))])
def test_key_partitions_union_equals_whole(config, nbytes, parts):
    """fac_haystack_set_key_partition (bench.py's key-split strong scaling): the parts' start windows
    (by a hash of their first two characters) are disjoint and cover the haystack, so the union of
    the parts' records equals the whole haystack's search_raw on every field -- with the prefix cache
    (each part counts, builds and looks up only its own keys; the C3 engine is beamed) and without it
    (5000 bytes: fewer than 4096 windows), restaged in place between searches like the bench step."""
    import torch
    wl = W.config(config, nbytes)
    eng = W.builder_for(wl).device(0).build(wl.patterns)
    want = rows_key(StagedHaystack(eng, wl.haystack).search_windows(wl.threshold)[0])
    assert len(want) >= 1
    dev = torch.from_numpy(np.frombuffer(wl.haystack, np.uint8).copy()).cuda()
    for n in parts:
        got, sizes = [], []
        for r in range(n):
            sh = StagedHaystack.from_device(eng, dev.data_ptr(), len(wl.haystack)).set_key_partition(n, r)
            for _ in range(2):
                sh = StagedHaystack.from_device(eng, dev.data_ptr(), len(wl.haystack), reuse=sh)
                rows = sh.search_windows(wl.threshold)[0]
            got += rows
            sizes.append(len(rows))
        assert rows_key(got) == want, (config, n)
        assert len(want) < 20 or min(sizes) > 0, sizes
    ab = B().fuzzy(L().edits(1)).auto_beam(1000, 2).device(0).build(["needle"])
    with pytest.raises(Exception):
        StagedHaystack(ab, b"a needle here").set_key_partition(2, 0)


def test_key_partitions_with_dense_window_lists(monkeypatch):
    """Key parts of a C2 slice with the sampled level forced on, so the dense bitmaps' list is built from
    the key part's list (dl_mask_kernel's per-window path over P.kp_wlist): the parts' union == the whole
    search, with the bitmaps on and off."""
    import torch
    monkeypatch.setenv("FAC_RC_MIN2", "1")
    wl = W.config("c2", 4 << 20)
    eng = W.builder_for(wl).device(0).build(wl.patterns)
    want = rows_key(StagedHaystack(eng, wl.haystack).search_windows(wl.threshold)[0])
    assert len(want) >= 100
    dev = torch.from_numpy(np.frombuffer(wl.haystack, np.uint8).copy()).cuda()
    for dense in (True, False):
        if not dense:
            monkeypatch.setenv("FAC_RC_NO_DENSE", "1")
        for n in (2, 3):
            got = []
            for r in range(n):
                sh = StagedHaystack.from_device(eng, dev.data_ptr(), len(wl.haystack)).set_key_partition(n, r)
                got += sh.search_windows(wl.threshold)[0]
            assert rows_key(got) == want, (dense, n)


def test_empty_unicode_shard_stages_on_device():
    """A short Unicode text over many ranks leaves the last shards empty (plan (len, len, len, ...)):
    staging such a shard fresh from device memory must not touch the unallocated staging scratch
    (graphemes_before on an empty haystack), and gives the host-staged shard's (empty) result."""
    import torch
    from fuzzy_aho_corasick import _native
    eng = B().fuzzy(L().edits(1)).device(0).build(["é"])
    data = "éé".encode()  # 4 bytes: shards 6 and 7 of 8 are (4, 4, 4)
    n = 8
    empty = 0
    for r in range(n):
        plan = _native.shard_plan(eng.max_match_graphemes(), data, n, r)
        host = StagedHaystack.shard(eng, data, n, r)
        dev = torch.from_numpy(np.frombuffer(data, np.uint8)[plan[0]:plan[2]].copy()).cuda()
        sh = StagedHaystack.shard_from_device(eng, dev.data_ptr() if plan[2] > plan[0] else 0, plan)
        assert (sh.graphemes, sh.owned_windows) == (host.graphemes, host.owned_windows), (r, plan)
        assert rows_key(sh.search_windows(0.5)[0]) == rows_key(host.search_windows(0.5)[0])
        empty += plan[0] == plan[2]
    assert empty > 0


def test_search_device_equals_host_records():
    wl, b = _c3_slice(64 << 10)
    eng = b.build(wl.patterns)
    st = StagedHaystack(eng, wl.haystack)
    host = st.search_windows_records(wl.threshold)[0]
    t, n, _ = st.search_device(wl.threshold)
    dev = t.cpu().numpy().view(host.dtype)
    assert n == len(host) > 10
    assert recs_key(dev) == recs_key(host)
    st._dev_out = st._dev_out[:64]  # too small: the call grows it (FAC_E_OUTPUT_CAPACITY) and retries
    t2, n2, _ = st.search_device(wl.threshold)
    assert n2 == n and recs_key(t2.cpu().numpy().view(host.dtype)) == recs_key(host)


def test_auto_beam_prefix_matches_whole():
    """A later shard given the running auto-beam total of the windows before it switches the beam on
    exactly where search_raw of the whole haystack does (search.rs:1096-1103)."""
    hay = ("a needle in a haystakc, fuzzy automatn; ecole Москва école nedle " * 60).strip()
    pats = ["needle", "haystack", "fuzzy", "automaton", "école", "Москва"]
    b = B().fuzzy(L().edits(2)).case_insensitive(True).auto_beam(3000, 3).device(0)
    eng = b.build(pats)
    data = hay.encode()
    whole = rows_key(StagedHaystack(eng, data).search_windows(0.7)[0])
    assert whole == rows_key(OracleEngine(b, pats).raw_rows(hay, 0.7))
    got, prefix = [], 0
    for r in range(3):
        sh = StagedHaystack.shard(eng, data, 3, r)
        t, n, _ = sh.search_device(0.7, auto_beam_prefix=prefix)
        got += list(t.cpu().numpy().view(_match_dtype()))
        prefix += sh.auto_beam_total(0.7)
    assert recs_key(np.array(got, dtype=_match_dtype())) == whole


def _match_dtype():
    from fuzzy_aho_corasick._native import MATCH_DTYPE
    return MATCH_DTYPE


def _sparse_c5(nbytes, every):
    rng = W.XorShift(5).numpy()
    pats = W._words(rng, [W.ASCII_LOWER], 200, 10, 16, True)
    hay = W._haystack(W.XorShift(6).numpy(), [W.ASCII_LOWER], pats, nbytes, 1, every)
    return pats, hay


@pytest.mark.parametrize("prefilter", [True, False])
def test_stream_windows_on_device_equal_whole_input(prefilter):
    """C5's unit of work: device-resident stream windows (window text = its bytes + overlap, searched,
    ranked sorted().non_overlapping(), owned matches kept; stream.rs:262-297) over a sparse input
    equal the whole input's sorted().non_overlapping() search (the reference's own streaming
    property, tests.rs:1058-1062), checked against the oracle."""
    pats, hay = _sparse_c5(1 << 20, 8 << 10)
    b = B().fuzzy(L().edits(1)).device(0)
    eng = b.build(pats)
    orc = OracleEngine(b, pats)
    text = hay.decode()
    opts = O().threshold(0.85).sorted().non_overlapping()
    whole = (orc.with_prefilter().search(text, opts) if prefilter else orc.search(text, opts))
    want = sorted((m.start, m.end, m.pattern_index, m.sim_bits()) for m in whole)
    assert len(want) > 50
    overlap = eng.max_match_graphemes() + 1
    st = StagedHaystack(eng, hay)
    import torch
    from fuzzy_aho_corasick._native import MATCH_DTYPE
    for win in (64 << 10, 200 << 10, 100_003):  # (100 003: windows at unaligned byte offsets)
        got = []
        # and fac_stream_window_staged_device (bench.py --config c5 at N > 1): every window's owned
        # records appended in HBM to one buffer, started tiny so it must grow, gathered from there
        dev = torch.empty(64, dtype=torch.uint8, device="cuda")
        n = 0
        for c in range(0, len(hay), win):
            c1 = min(len(hay), c + win)
            recs, _ = st.stream_window(c, min(len(hay), c1 + overlap), c1 - c, c, 0.85, prefilter)
            got += [(int(r["start"]), int(r["end"]), int(r["pattern_index"]),
                     int(np.float32(r["similarity"]).view(np.uint32))) for r in recs]
            dev, k, _ = st.stream_window_device(c, min(len(hay), c1 + overlap), c1 - c, c, 0.85, prefilter, dev, n)
            assert k == len(recs)
            n += k
        assert sorted(got) == want, win
        drecs = dev[: n * 32].cpu().numpy().view(MATCH_DTYPE)
        assert [tuple(r) for r in drecs] == [tuple(r) for r in np.concatenate(
            [st.stream_window(c, min(len(hay), min(len(hay), c + win) + overlap), min(len(hay), c + win) - c, c, 0.85,
                              prefilter)[0] for c in range(0, len(hay), win)])], win


def _window_cuts(n, win, overlap):
    return [(c, min(n, min(n, c + win) + overlap), min(n, c + win) - c, c) for c in range(0, n, win)]


@pytest.mark.parametrize("prefilter", [True, False])
def test_stream_window_batches_equal_single_windows(prefilter):
    """fac_stream_windows_staged_device (bench.py C5 at the crate's 256 KiB windows, stream.rs:65):
    a batch of stream windows searched in one pre-filter pass over their union and one search launch
    gives every window exactly what fac_stream_window_staged_device gives it alone -- records, order
    and fields -- including matches planted across window boundaries (in the overlaps, where two
    windows verify the same candidate with different automaton starts) and windows at unaligned byte
    offsets; and the union over the windows equals the whole input's sorted().non_overlapping()
    search by the oracle."""
    import torch
    from fuzzy_aho_corasick._native import MATCH_DTYPE
    pats, hay = _sparse_c5(1 << 20, 3 << 10)
    b = B().fuzzy(L().edits(1)).device(0)
    eng = b.build(pats)
    overlap = eng.max_match_graphemes() + 1
    # plant needles straddling the cuts of the 8 KiB windows
    ba = bytearray(hay)
    win = 8 << 10
    for i, c in enumerate(range(win, len(ba) - 64, win)):
        p = pats[i % len(pats)].encode()
        at = c - len(p) // 2 - (i % 5)
        ba[at - 1: at + len(p) + 1] = b" " + p + b" "
    hay = bytes(ba)
    st = StagedHaystack(eng, hay)
    orc = OracleEngine(b, pats)
    orc = orc.with_prefilter() if prefilter else orc
    opts = O().threshold(0.85).sorted().non_overlapping()
    want = []  # the oracle, window by window (window_matches: sorted().non_overlapping(), start < commit)
    for (g0, g1, commit, base) in _window_cuts(len(hay), win, overlap):
        want += [(base + m.start, base + m.end, m.pattern_index, m.sim_bits())
                 for m in orc.search(hay[g0:g1].decode(), opts) if m.start < commit]
    want.sort()
    assert len(want) > 300
    for w in (win, 100_003, 256 << 10):
        cuts = _window_cuts(len(hay), w, overlap)
        single = [st.stream_window(*c, 0.85, prefilter)[0] for c in cuts]
        single = np.concatenate(single) if single else np.zeros(0, MATCH_DTYPE)
        for batch in (len(cuts), 7):
            dev = torch.empty(64, dtype=torch.uint8, device="cuda")
            n = 0
            for a in range(0, len(cuts), batch):
                dev, k, _ = st.stream_windows_device(cuts[a: a + batch], 0.85, prefilter, dev, n)
                n += k
            got = dev[: n * 32].cpu().numpy().view(MATCH_DTYPE)
            assert [tuple(r) for r in got] == [tuple(r) for r in single], (w, batch)
        if w == win:
            key = sorted((int(r["start"]), int(r["end"]), int(r["pattern_index"]),
                          int(np.float32(r["similarity"]).view(np.uint32))) for r in single)
            assert key == want


def test_dense_window_list_across_segments(monkeypatch, capfd):
    """The dense bitmaps' window list (dl_mask_kernel) over a batch of stream windows: 100 003-byte
    windows make segments whose boundaries fall inside the list's 4096-window blocks, so blocks take
    the window-by-window path as well as the staged-tile one. Prefix cache and sampled level forced on:
    records == bitmaps off == cache off, and windows are left out of the lookups (FAC_RC_DEBUG)."""
    import re
    import torch
    from fuzzy_aho_corasick._native import MATCH_DTYPE
    pats, hay = _sparse_c5(3 << 20, 3 << 10)
    eng = B().fuzzy(L().edits(1)).device(0).build(pats)
    st = StagedHaystack(eng, hay)
    cuts = _window_cuts(len(hay), 100_003, eng.max_match_graphemes() + 1)
    monkeypatch.setenv("FAC_RC_MIN", "1")
    monkeypatch.setenv("FAC_RC_MIN2", "1")

    def run():
        dev = torch.empty(64, dtype=torch.uint8, device="cuda")
        dev, k, _ = st.stream_windows_device(cuts, 0.85, False, dev, 0)
        return [tuple(r) for r in dev[: k * 32].cpu().numpy().view(MATCH_DTYPE)]

    monkeypatch.setenv("FAC_RC_DEBUG", "1")
    capfd.readouterr()
    dense = run()
    err = capfd.readouterr().err
    monkeypatch.delenv("FAC_RC_DEBUG")
    m = re.findall(r"unlisted (\d+)", err)
    assert m and int(m[-1]) > 0, err[-2000:]
    monkeypatch.setenv("FAC_RC_NO_DENSE", "1")
    plain = run()
    monkeypatch.delenv("FAC_RC_NO_DENSE")
    monkeypatch.setenv("FAC_NO_RC", "1")
    off = run()
    assert len(dense) > 100 and dense == plain == off


@pytest.mark.parametrize("unicode_tail", [False, True])
def test_search_stream_batches_match_oracle_emulation(unicode_tail):
    """search_stream over fac_stream_* with many windows per batch (stream.cpp: an ASCII batch staged
    once and searched in one launch, each window its own text) == the crate's WindowReader (64 KiB
    reads) + per-window sorted().non_overlapping() search replayed on the CPU oracle; fed in 4 MiB
    pieces, the windows are cut as the 64 KiB reads would cut them. With a Unicode tail the last
    batch takes the per-window path."""
    import io
    from stream_emulation import stream_rows
    pats, hay = _sparse_c5(2 << 20, 2 << 10)
    if unicode_tail:
        hay = hay + ("école " + pats[3] + " Москва ").encode() * 2000
    b = B().fuzzy(L().edits(1)).device(0)
    eng = b.build(pats)
    got = sorted((m.start, m.end, m.pattern_index, int(np.float32(m.similarity).view(np.uint32)), m.text)
                 for m in eng.stream_matches(io.BytesIO(hay), 0.85))
    want = sorted(stream_rows(OracleEngine(b, pats), hay, 0.85, eng.max_match_graphemes() + 1))
    assert len(want) > 500
    assert got == want


def test_haystack_too_large_is_reported(monkeypatch):
    """search_raw's SearchError::HaystackTooLarge{graphemes} (search.rs:198-201, error.rs:13-16)
    crosses the C ABI as return code 1 with the grapheme count; the u32::MAX limit is lowered by the
    FAC_GRAPHEME_LIMIT diagnostics knob so the path can be reached."""
    monkeypatch.setenv("FAC_GRAPHEME_LIMIT", "100")
    eng = B().fuzzy(L().edits(1)).device(0).build(["hello"])
    with pytest.raises(HaystackTooLarge) as ei:
        eng.search("x" * 101)
    assert ei.value.graphemes == 101
    with pytest.raises(HaystackTooLarge) as ei:
        eng.search("é" * 150)
    assert ei.value.graphemes == 150
    assert len(eng.search("hello " * 16, O().threshold(0.9))) == 16  # 96 graphemes: fine


def test_knobs_need_diagnostics_mode():
    """FAC_* knobs change the kernel path only with FAC_DIAGNOSTICS=1 (fac.h): a stray FAC_NO_RC in a
    user's environment leaves the prefix cache on."""
    code = ("import sys; sys.path.insert(0, 'fuzzy-aho-corasick-rs_amd');"
            "from fuzzy_aho_corasick import workloads as W;"
            "from fuzzy_aho_corasick.engine import StagedHaystack;"
            "wl = W.config('c2', 64 << 10); e = W.builder_for(wl).device(0).build(wl.patterns);"
            "print(StagedHaystack(e, wl.haystack).search_windows(wl.threshold)[1].states_cached)")
    out = {}
    for diag in ("0", "1"):
        env = dict(os.environ, FAC_NO_RC="1", FAC_DIAGNOSTICS=diag)
        r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        out[diag] = int(r.stdout.strip().splitlines()[-1])
    assert out["0"] > 0 and out["1"] == 0


# ---- streaming replace (tests.rs:1153-1273), on the double-buffered device stream

def _needle_engine():
    return B().fuzzy(L().edits(1)).case_insensitive(True).device(0).build(["needle"])


def _replace(eng, text, cb, window=0, parallel=False):
    import io
    out = io.BytesIO()
    if parallel:
        n = eng.replace_stream_parallel(io.BytesIO(text.encode()), out, 4, 0.8, cb)
    else:
        n = eng.replace_stream(io.BytesIO(text.encode()), out, 0.8, cb, window=window)
    s = out.getvalue().decode()
    assert n == len(out.getvalue())
    return s


@pytest.mark.parametrize("parallel", [False, True])
def test_replace_stream_small_cases(parallel):  # tests.rs:1153-1183, 1240-1259
    eng = _needle_engine()
    x = lambda m: "X"  # noqa: E731
    assert _replace(eng, "a needle b", x, parallel=parallel) == "a X b"
    assert _replace(eng, "needle b", x, parallel=parallel) == "X b"
    assert _replace(eng, "a needle", x, parallel=parallel) == "a X"
    assert _replace(eng, "needle needle", x, parallel=parallel) == "X X"
    assert _replace(eng, "a neeedle b", x, parallel=parallel) == "a X b"  # one insertion
    assert _replace(eng, "nothing here", x, parallel=parallel) == "nothing here"
    assert _replace(eng, "", x, parallel=parallel) == ""
    assert _replace(eng, "a needle b", lambda m: None, parallel=parallel) == "a needle b"


@pytest.mark.parametrize("window", [0, 4096, 64 << 10])
def test_replace_stream_matches_whole_input(window):  # tests.rs:1186-1237
    eng = _needle_engine()
    filler = "the quick brown fox " * 50
    text = ""
    while len(text) < 600_000:
        text += filler + "needle "
    truth = eng.replace(text, O().threshold(0.8), lambda m: f"<{m.pattern_index}>")
    got = _replace(eng, text, lambda m: f"<{m.pattern_index}>", window=window)
    assert got == truth and "<0>" in got
    assert _replace(eng, text, lambda m: f"<{m.pattern_index}>", parallel=True) == truth


def test_fuzzy_replacer_replace_stream():  # tests.rs:1262-1273
    import io
    r = B().case_insensitive(True).fuzzy(L().edits(1)).device(0).build_replacer([("hello", "hi"), ("world", "earth")])
    out = io.BytesIO()
    r.replace_stream(io.BytesIO(b"hell0 w0rld!"), out, 0.8)
    assert out.getvalue().decode() == "hi earth!"


def test_stream_many_windows_in_order():
    """The double-buffered stream hands windows out in stream order: tiny windows (thousands of
    cuts, two in flight) give the same matches, in the same order, as the whole-input ranking."""
    import io
    eng = _needle_engine()
    text = ("fox needle " + "x" * 40 + " nedle ") * 800
    truth = [(m.start, m.end) for m in eng.search(text, O().threshold(0.8).sorted().non_overlapping())]
    got = [(m.start, m.end) for m in eng.stream_matches(io.BytesIO(text.encode()), 0.8, window=512)]
    assert got == truth and len(got) == 1600


@pytest.mark.gpu
def test_device_utf8_check_matches_python():
    """fac_haystack_stage checks the bytes on the device (seg_tile_kernel: per 64-byte thread range, from
    its first non-continuation byte) and decides search.rs:196's is_ascii there: accepted exactly when
    Python's strict decoder (like Rust's str::from_utf8: no overlongs, surrogates, > U+10FFFF,
    truncations or stray continuation bytes) accepts, with invalid sequences planted at and around
    the 64-byte range and 16 KiB tile boundaries; accepted haystacks search like the oracle."""
    import random
    from fuzzy_aho_corasick import DeviceError
    from fuzzy_aho_corasick._native import FAC_E_INVALID
    rng = random.Random(0x0757)
    eng = B().fuzzy(L().edits(1)).device(0).build(["héllo", "wörld", "ab"])
    bad = [b"\x80", b"\xbf\xbf", b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf0\x80\x80\x80",
           b"\xf4\x90\x80\x80", b"\xf8\x88\x80\x80\x80", b"\xff", b"\xc3", b"\xe2\x82", b"\xf0\x9f\x98",
           b"\x80\x80\x80\x80\x80", b"\xc3\xa9\x80"]
    cps = [0x41, 0x7A, 0x20, 0xE9, 0x3B1, 0x20AC, 0x4E2D, 0xFFFD, 0x1F600, 0x10FFFF, 0xD7FF, 0xE000]

    def text(nbytes):
        out = bytearray()
        while len(out) < nbytes:
            out += chr(rng.choice(cps)).encode("utf-8")
        return bytes(out)

    checked = 0
    for trial in range(160):
        base = text(rng.choice([40, 255, 256, 300, 700, 1500, 5000, 17000]))
        data = base
        if trial % 4:  # plant an invalid (or, cut mid-sequence, sometimes valid) piece
            piece = rng.choice(bad)
            at = rng.choice([0, 1, 63, 64, 65, 127, 128, 255, 256, 257, 511, 512, 16383, 16384, 16385, len(base) - 1, len(base),
                             rng.randrange(len(base) + 1)])
            at = max(0, min(len(base), at))
            data = base[:at] + piece + base[at:]
        try:
            data.decode("utf-8")
            ok = True
        except UnicodeDecodeError:
            ok = False
        if ok:
            st = StagedHaystack(eng, data)
            assert st.graphemes == len(data.decode("utf-8")) or not data.isascii(), trial
            checked += 1
        else:
            with pytest.raises(DeviceError) as ei:
                StagedHaystack(eng, data)
            assert ei.value.code == FAC_E_INVALID, trial
    assert checked >= 30
    for hay in ("plain ascii héllo wörld " * 40, "ascii only hello world ab " * 20):
        want = sorted((m.start, m.end, m.pattern_index) for m in OracleEngine(
            B().fuzzy(L().edits(1)), ["héllo", "wörld", "ab"]).search_raw(hay, 0.8))
        got = sorted((m.start, m.end, m.pattern_index) for m in eng.search_raw(hay, 0.8))
        assert len(got) > 0 and got == want


def test_device_utf8_check_inside_long_runs():
    """64-byte ranges with no resync code point within 1 KiB (long combining / emoji ZWJ /
    regional-indicator runs) are segmented by seg_hard_kernel, which decodes leniently; the UTF-8
    check must still cover their bytes. Invalid pieces planted inside and right after > 1 KiB runs
    are refused on both staging paths (host bytes and device bytes, incl. a restage of a live
    haystack, which is left empty and usable), exactly when Python's strict decoder refuses."""
    import random
    import torch
    from fuzzy_aho_corasick import DeviceError
    from fuzzy_aho_corasick._native import FAC_E_INVALID
    rng = random.Random(0x1057)
    eng = B().fuzzy(L().edits(1)).device(0).build(["héllo", "wörld", "ab"])
    runs = ["́", "‍\U0001F469", "\U0001F1EB\U0001F1F7", "̈́", "\U0001F3FB"]
    bad = [b"\x80", b"\xff", b"\xc0\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xc3", b"\xe2\x82", b"\xf0\x9f\x98",
           b"\xe0\x80\x80"]
    st = None
    refused = 0
    for trial in range(60):
        run = rng.choice(runs) * rng.choice([400, 700, 1500, 9000])
        head = "ab héllo " + ("a" if trial % 2 else "\U0001F468")
        data = (head + run).encode("utf-8")
        at = rng.choice([len(data) // 2, len(data) - 1, len(data), 1100 + rng.randrange(64), 16384, 16385])
        at = min(at, len(data))
        data = data[:at] + rng.choice(bad) + data[at:] + (rng.choice(runs) * 30 + " wörld").encode("utf-8")
        try:
            data.decode("utf-8")
            ok = True
        except UnicodeDecodeError:
            ok = False
        dev = torch.from_numpy(np.frombuffer(data + b"\0", dtype=np.uint8).copy()).to("cuda")
        if ok:
            StagedHaystack(eng, data)
            st = StagedHaystack.from_device(eng, dev.data_ptr(), len(data), reuse=st)
            continue
        refused += 1
        with pytest.raises(DeviceError) as ei:
            StagedHaystack(eng, data)
        assert ei.value.code == FAC_E_INVALID, trial
        with pytest.raises(DeviceError) as ei:
            st = StagedHaystack.from_device(eng, dev.data_ptr(), len(data), reuse=st)
        assert ei.value.code == FAC_E_INVALID, trial
        if st is not None:  # the failed restage left an empty haystack: searching it finds nothing
            assert st.graphemes == 0
            assert len(st.search_windows(0.8)[0]) == 0
        del dev
    assert refused >= 40
