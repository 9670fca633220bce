"""The two toolchain algorithms the reference's beamed results depend on, each
restated three times and cross-checked on the CPU:

* the trie edge order: iteration order of `Node.transitions: FxHashMap<String, u32>`
  (builder.rs:336-342) = the crate's FxHasher (structs.rs:95-156) + std's hashbrown table — a
  Python restatement below, the oracle's (oracle.cpp hashbrown_order) and the product builder's
  (builder.cpp edge_order, exported as fac_edge_order);
* the beam cut `select_nth_unstable_by(bw - 1, total_cmp)` (search.rs:584-587) = core's introselect
  (Rust >= 1.81) — a Python restatement below against the oracle's (oracle.cpp rsel); the GPU's
  lane-parallel form of the cyclic Lomuto partition (search_kernels.hip sel_partition) is checked
  here against the sequential one. GPU == oracle on beamed searches is in test_gpu_parity.py.

No Rust toolchain exists in this image, so these pin the restatements to each other, not to rustc
("parity unpinned; deterministic restatement").
"""
import ctypes
import os
import random
import struct

import numpy as np
import pytest

import oracle_harness as OH

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# ---------------------------------------------------------------------------------------------
# FxHasher + hashbrown (x86-64 SSE2 groups of 16), insert-only
# ---------------------------------------------------------------------------------------------
M64 = (1 << 64) - 1


def fx_hash_str(b: bytes) -> int:
    h = 0

    def add(w):
        nonlocal h
        h = ((((h << 5) | (h >> 59)) & M64) ^ w) * 0x517CC1B727220A95 & M64

    i = 0
    while len(b) - i >= 8:
        add(int.from_bytes(b[i:i + 8], "little"))
        i += 8
    if len(b) - i >= 4:
        add(int.from_bytes(b[i:i + 4], "little"))
        i += 4
    for x in b[i:]:
        add(x)
    add(0xFF)
    return h


def hashbrown_order(keys):
    """Insertion indices of `keys` (bytes) in HashMap iteration order after inserting them in order."""
    hashes = [fx_hash_str(k) for k in keys]
    ctrl = []  # bucket -> item or None
    items = 0

    def cap(nb):
        return nb - 1 if nb < 8 + 1 else nb // 8 * 7

    def find(h):
        nb = len(ctrl)
        mask, width = nb - 1, max(nb, 16)
        pos, stride = h & mask, 0
        while True:
            for k in range(16):
                c = pos + k
                empty = (ctrl[c] is None) if c < nb else (ctrl[c - width] is None) if c >= width else True
                if empty:
                    idx = c & mask
                    if ctrl[idx] is not None:
                        idx = next(i for i in range(nb) if ctrl[i] is None)
                    return idx
            stride += 16
            pos = (pos + stride) & mask

    for it, h in enumerate(hashes):
        if not ctrl or items == cap(len(ctrl)):
            want = 1 if not ctrl else cap(len(ctrl)) + 1
            if want < 8:
                nb = 4 if want < 4 else 8
            else:
                nb = 1
                while nb < want * 8 // 7:
                    nb <<= 1
            old, ctrl = ctrl, [None] * nb
            for o in old:
                if o is not None:
                    ctrl[find(hashes[o])] = o
        ctrl[find(h)] = it
        items += 1
    return [o for o in ctrl if o is not None]


def _children(rng, n):
    alphabet = [chr(c) for c in list(range(0x61, 0x7B)) + list(range(0xE0, 0x100)) + list(range(0x3B1, 0x3CA))
                + list(range(0x430, 0x450)) + list(range(0x100, 0x180))] + ["é", "\U0001F600", "ab", "é́", "abcdefghij"]
    return rng.sample(alphabet, n)


def _edge_order_lib(lib_fn, children):
    cps, off = [], [0]
    for g in children:
        cps += [ord(c) for c in g]
        off.append(len(cps))
    out = (ctypes.c_uint32 * max(1, len(children)))()
    lib_fn((ctypes.c_uint32 * max(1, len(cps)))(*cps), (ctypes.c_uint64 * len(off))(*off), len(children), out)
    return list(out[:len(children)])


@pytest.mark.parametrize("seed", range(6))
def test_edge_order_three_restatements_agree(seed):
    from fuzzy_aho_corasick import _native
    lib = _native.lib
    lib.fac_edge_order.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64,
                                   ctypes.POINTER(ctypes.c_uint32)]
    OH._lib.orc_edge_order.argtypes = lib.fac_edge_order.argtypes
    rng = random.Random(seed)
    for n in list(range(1, 40)) + [57, 64, 100, 113, 150]:
        ch = _children(rng, n)
        py = hashbrown_order([g.encode() for g in ch])
        assert sorted(py) == list(range(n))
        assert _edge_order_lib(OH._lib.orc_edge_order, ch) == py, (n, ch)
        assert _edge_order_lib(lib.fac_edge_order, ch) == py, (n, ch)


def test_edge_order_small_tables_wrap():
    # 3 children: 4 buckets, probing wraps through the group's EMPTY padding to bucket 0
    for ch in (["a", "b", "c"], ["z", "y", "x"], ["é", "e", "е"]):
        assert _edge_order_lib(OH._lib.orc_edge_order, ch) == hashbrown_order([g.encode() for g in ch])


# ---------------------------------------------------------------------------------------------
# core::slice::select_nth_unstable_by
# ---------------------------------------------------------------------------------------------
def _tkey(f):
    u = struct.unpack("<I", struct.pack("<f", f))[0]
    return (~u & 0xFFFFFFFF) if u & 0x80000000 else (u | 0x80000000)


def py_select(keys, index, limit0=16):
    """select.rs partition_at_index with is_less = total_cmp == Less, on (key, original index)."""
    v = [(_tkey(k), i) for i, k in enumerate(keys)]
    lt = lambda a, b: a[0] < b[0]  # noqa: E731

    def insertion(lo, hi):
        for i in range(lo + 1, hi):
            if not lt(v[i], v[i - 1]):
                continue
            tmp, j = v[i], i
            while True:
                v[j] = v[j - 1]
                j -= 1
                if j == lo or not lt(tmp, v[j - 1]):
                    break
            v[j] = tmp

    def median3(a, b, c):
        x, y = lt(v[a], v[b]), lt(v[a], v[c])
        if x == y:
            return c if (lt(v[b], v[c]) ^ x) else b
        return a

    def median3_rec(a, b, c, n):
        if n * 8 >= 64:
            n8 = n // 8
            a = median3_rec(a, a + n8 * 4, a + n8 * 7, n8)
            b = median3_rec(b, b + n8 * 4, b + n8 * 7, n8)
            c = median3_rec(c, c + n8 * 4, c + n8 * 7, n8)
        return median3(a, b, c)

    def choose_pivot(lo, n):
        d8 = n // 8
        if n < 64:
            return median3(lo, lo + 4 * d8, lo + 7 * d8) - lo
        return median3_rec(lo, lo + 4 * d8, lo + 7 * d8, d8) - lo

    def partition(lo, n, pp, less):
        v[lo], v[lo + pp] = v[lo + pp], v[lo]
        piv = v[lo]
        w0, m = lo + 1, n - 1
        nl = 0
        if m:
            gv, gap = v[w0], 0
            for r in range(1, m):
                x = v[w0 + r]
                l_ = less(x, piv)
                v[w0 + gap] = v[w0 + nl]
                v[w0 + nl] = x
                gap = r
                nl += l_
            l_ = less(gv, piv)
            v[w0 + gap] = v[w0 + nl]
            v[w0 + nl] = gv
            nl += l_
        v[lo], v[lo + nl] = v[lo + nl], v[lo]
        return nl

    def median_idx(a, b, c):
        if lt(v[c], v[a]):
            a, c = c, a
        if lt(v[c], v[b]):
            return c
        if lt(v[b], v[a]):
            return a
        return b

    def ninther(a, b, c, d, e, f, g, h, i):
        b = median_idx(a, b, c)
        h = median_idx(g, h, i)
        if lt(v[h], v[b]):
            b, h = h, b
        if lt(v[f], v[d]):
            d, f = f, d
        if lt(v[e], v[d]):
            pass
        elif lt(v[f], v[e]):
            d = f
        else:
            if lt(v[e], v[b]):
                v[e], v[b] = v[b], v[e]
            elif lt(v[h], v[e]):
                v[e], v[h] = v[h], v[e]
            return
        if lt(v[d], v[b]):
            d = b
        elif lt(v[h], v[d]):
            d = h
        v[d], v[e] = v[e], v[d]

    def mom(lo, n, k):
        while True:
            if n <= 16:
                insertion(lo, lo + n)
                return
            if k == n - 1 or k == 0:
                acc = lo
                for i in range(lo + 1, lo + n):
                    if (lt(v[acc], v[i]) if k else lt(v[i], v[acc])):
                        acc = i
                v[acc], v[lo + k] = v[lo + k], v[acc]
                return
            frac = n // 12 if n <= 1024 else (n // 64 if n <= 128 * 1024 else n // 1024)
            pivot = frac // 2
            l0 = n // 2 - pivot
            hi = frac + l0
            gap = (n - 9 * frac) // 4
            a, b = l0 - 4 * frac - gap, hi + gap
            for i in range(l0, hi):
                ninther(lo + a, lo + i - frac, lo + b, lo + a + 1, lo + i, lo + b + 1, lo + a + 2, lo + i + frac, lo + b + 2)
                a += 3
                b += 3
            mom(lo + l0, frac, pivot)
            p = partition(lo, n, l0 + pivot, lt)
            if p == k:
                return
            if p > k:
                n = p
            else:
                lo, n, k = lo + p + 1, n - p - 1, k - p - 1

    n = len(v)
    if index == n - 1:
        acc = 0
        for i in range(1, n):
            if lt(v[acc], v[i]):
                acc = i
        v[acc], v[index] = v[index], v[acc]
    elif index == 0:
        acc = 0
        for i in range(1, n):
            if lt(v[i], v[acc]):
                acc = i
        v[acc], v[0] = v[0], v[acc]
    else:
        lo, n_, idx, limit, anc = 0, n, index, limit0, None
        while True:
            if n_ <= 16:
                insertion(lo, lo + n_)
                break
            if limit == 0:
                mom(lo, n_, idx)
                break
            limit -= 1
            pp = choose_pivot(lo, n_)
            if anc is not None and not lt(anc, v[lo + pp]):
                mid = partition(lo, n_, pp, lambda a, b: not lt(b, a)) + 1
                if idx < mid:  # core: `if mid > index { return; }`
                    break
                lo, n_, idx, anc = lo + mid, n_ - mid, idx - mid, None
                continue
            mid = partition(lo, n_, pp, lt)
            if mid < idx:
                anc = v[lo + mid]
                lo, n_, idx = lo + mid + 1, n_ - mid - 1, idx - mid - 1
            elif mid > idx:
                n_ = mid
            else:
                break
    return [i for _, i in v]


def _orc_select(keys, index):
    OH._lib.orc_select_nth.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint32)]
    out = (ctypes.c_uint32 * len(keys))()
    OH._lib.orc_select_nth((ctypes.c_float * len(keys))(*keys), len(keys), index, out)
    return list(out)


def _beam_like_keys(rng, n):
    # penalties like the beam sees: sums of a few discrete edit costs, many ties
    costs = np.array([0.0, 0.5199999809, 0.5719999671, 0.8579999804, 0.9099999666, 1.4299999475], np.float32)
    k = rng.integers(0, len(costs), size=(n, 2))
    return [float(np.float32(costs[a]) + np.float32(costs[b])) for a, b in k]


@pytest.mark.parametrize("limit", [16, 2, 0])
def test_select_oracle_matches_python_restatement(limit):
    OH.set_modes(sel_limit=limit)
    try:
        rng = np.random.default_rng(17 + limit)
        for t in range(300):
            n = int(rng.choice([3, 17, 40, 63, 64, 65, 129, 200, 300, 511, 512, 600, 1100]))
            keys = (_beam_like_keys(rng, n) if t % 3 else
                    [float(x) for x in rng.integers(0, [2, 5, 1000][t % 3 + (t // 3) % 2], size=n).astype(np.float32)])
            index = int(rng.integers(0, max(1, (n - 1) // 2))) if t % 5 else (0 if t % 2 else 63 % n)
            got = _orc_select(keys, index)
            want = py_select(keys, index, limit)
            assert got == want, (n, index, limit)
            kk = [_tkey(keys[i]) for i in got]  # and it is a selection
            assert all(x <= kk[index] for x in kk[:index]) and all(x >= kk[index] for x in kk[index + 1:])
    finally:
        OH.set_modes(sel_limit=16)


# VERDICT r03 / ADVICE r03: after the equal-to-ancestor split core continues while `index == mid`
# (`if mid > index { return; }`, select.rs partition_at_index_loop); rounds <= 3 stopped there and left
# a larger element at `index`. This array (keys {0..5}, index 29) was an invalid selection then.
_REPRO_INDEX_EQ_MID = [3.0, 1.0, 5.0, 5.0, 1.0, 3.0, 5.0, 5.0, 4.0, 3.0, 0.0, 4.0, 2.0, 0.0, 1.0, 3.0, 4.0, 3.0, 3.0,
                       5.0, 4.0, 2.0, 3.0, 3.0, 0.0, 0.0, 3.0, 2.0, 3.0, 1.0, 1.0, 0.0, 2.0, 4.0, 2.0, 2.0, 3.0, 5.0,
                       2.0, 3.0]


def _is_selection(keys, perm, index):
    kk = [_tkey(keys[i]) for i in perm]
    return all(x <= kk[index] for x in kk[:index]) and all(x >= kk[index] for x in kk[index + 1:])


def test_select_index_equal_to_mid_regression():
    keys = _REPRO_INDEX_EQ_MID
    got = _orc_select(keys, 29)
    assert got == py_select(keys, 29)
    assert _is_selection(keys, got, 29)
    assert sorted(keys[i] for i in got[:30]) == sorted(keys)[:30]


_BEAM_COSTS = np.array([0.0, 0.5199999809, 0.5719999671, 0.8579999804, 0.9099999666, 1.4299999475], np.float32)


def _beam_batch(seed, count, nmax=600):
    """`count` beam events like the search's: bw in {2, 8, 64}, pending max(17, 2 bw + 1) .. 600,
    penalties sums of two discrete edit costs (many ties). Returns keys (f32), offsets, indices."""
    rng = np.random.default_rng(seed)
    bw = rng.choice(np.array([2, 8, 64]), size=count)
    lo = np.maximum(17, 2 * bw + 1)
    n = lo + (rng.random(count) * (nmax + 1 - lo)).astype(np.int64)
    offs = np.zeros(count + 1, np.uint64)
    offs[1:] = np.cumsum(n)
    k = rng.integers(0, len(_BEAM_COSTS), size=(int(offs[-1]), 2))
    keys = (_BEAM_COSTS[k[:, 0]] + _BEAM_COSTS[k[:, 1]]).astype(np.float32)
    return keys, offs, (bw - 1).astype(np.uint64)


def _orc_select_batch(keys, offs, index):
    fn = OH._lib.orc_select_nth_batch
    fn.restype = ctypes.c_uint64
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    perm = np.zeros(len(keys), np.uint32)
    bad = fn(keys.ctypes.data, offs.ctypes.data, len(offs) - 1, index.ctypes.data, perm.ctypes.data)
    return perm, int(bad)


def _selection_violations(keys, offs, index, perm):
    """select_nth_unstable_by's post-condition checked with numpy (independently of the oracle):
    v[..i] <= v[i] <= v[i+1..] under total_cmp, per array. Returns the number of arrays violating it."""
    tk = keys.view(np.int32).astype(np.int64)
    tk = np.where(tk < 0, tk ^ 0x7FFFFFFF, tk)  # f32::total_cmp as a signed integer order
    starts = offs[:-1].astype(np.int64)
    seg = np.repeat(np.arange(len(starts)), np.diff(offs).astype(np.int64))
    v = tk[starts[seg] + perm.astype(np.int64)]  # keys in selected order
    pos = np.arange(len(v)) - starts[seg]
    piv = v[starts + index.astype(np.int64)][seg]
    bad = ((pos < index[seg].astype(np.int64)) & (v > piv)) | ((pos > index[seg].astype(np.int64)) & (v < piv))
    return int(np.count_nonzero(np.bincount(seg, weights=bad, minlength=len(starts))))


@pytest.mark.parametrize("limit", [16, 1, 0])
def test_select_postcondition_oracle_100k(limit):
    """>= 100 000 beam events per round limit (16 = core's; 1 and 0 reach median_of_medians early)."""
    OH.set_modes(sel_limit=limit)
    try:
        for chunk in range(5):
            keys, offs, index = _beam_batch(1000 * limit + chunk, 20000)
            perm, bad = _orc_select_batch(keys, offs, index)
            assert bad == 0
            assert _selection_violations(keys, offs, index, perm) == 0
            # and a permutation of each array
            seg = np.repeat(np.arange(len(offs) - 1), np.diff(offs).astype(np.int64))
            order = np.lexsort((perm, seg))
            assert np.array_equal(perm[order], np.arange(len(perm)) - offs[:-1].astype(np.int64)[seg])
    finally:
        OH.set_modes(sel_limit=16)


def _py_chunk(args):
    seed, count, limit = args
    OH.set_modes(sel_limit=limit)
    keys, offs, index = _beam_batch(seed, count)
    perm, bad = _orc_select_batch(keys, offs, index)
    mism = inval = 0
    for a in range(count):
        b, e = int(offs[a]), int(offs[a + 1])
        kl = keys[b:e].tolist()
        got = py_select(kl, int(index[a]), limit)
        mism += got != perm[b:e].tolist()
        inval += not _is_selection(kl, got, int(index[a]))
    return mism, inval, bad


def test_select_postcondition_python_100k():
    """The Python restatement on 100 000 beam events (70 000 at core's limit, 15 000 each at limits 1
    and 0): a valid selection every time, and the oracle's permutation exactly."""
    import multiprocessing as mp
    jobs = [(50_000 + i, 5000, 16) for i in range(14)] + [(60_000 + i, 5000, l) for i in range(3) for l in (1, 0)]
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(_py_chunk, jobs)
    assert sum(r[0] for r in res) == 0, "python restatement != oracle"
    assert sum(r[1] for r in res) == 0, "python restatement: invalid selection"
    assert sum(r[2] for r in res) == 0, "oracle: invalid selection"


def _lomuto_serial(w, lt):
    w = list(w)
    m = len(w)
    gv, gap, nl = w[0], 0, 0
    for r in range(1, m):
        x = w[r]
        l_ = lt(x)
        w[gap] = w[nl]
        w[nl] = x
        gap = r
        nl += l_
    l_ = lt(gv)
    w[gap] = w[nl]
    w[nl] = gv
    return w, nl + l_


def _lomuto_closed(w, lt):
    """search_kernels.hip sel_partition's lane-parallel form."""
    m = len(w)
    e = [None] + w[1:] + [w[0]]
    is_lt = [None] + [lt(e[r]) for r in range(1, m + 1)]
    L = [0] * (m + 2)
    for r in range(1, m + 1):
        L[r + 1] = L[r] + is_lt[r]
    F = L[m + 1]
    out = [None] * m
    for r in range(1, m + 1):
        if is_lt[r]:
            out[L[r]] = e[r]
    for p in range(F, m):
        if p == F and not is_lt[m]:
            out[p] = e[m]
            continue
        r = p + 1
        while is_lt[r - 1]:
            r = L[r] + 1
        out[p] = e[r - 1]
    return out, F


def test_cyclic_lomuto_closed_form():
    rng = random.Random(5)
    for _ in range(20000):
        m = rng.randint(1, 70)
        w = [(rng.randint(0, rng.choice([1, 3, 20])), i) for i in range(m)]
        piv = rng.randint(0, 20)
        lt = lambda x: x[0] < piv  # noqa: E731
        assert _lomuto_serial(w, lt) == _lomuto_closed(w, lt)
