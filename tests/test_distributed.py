"""World-size-2 tests of the multi-rank path: shard the start windows of one haystack across two
processes, gather the 32-byte Match records to rank 0 with torch.distributed, and check the union
equals the single-process search. CPU variant: gloo + the oracle as the per-rank compute; GPU
variant: gloo for the exchange, both ranks' searches on cuda:0 through the C ABI."""
import os
import socket
import sys
import tempfile

import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PATTERNS = ["needle", "haystack", "fuzzy", "automaton", "école", "Москва"]
HAY = ("a needle in a haystakc, fuzzy automatn; ecole Москва école nedle " * 40).strip()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, use_gpu, out_path):
    sys.path[:0] = [os.path.join(REPO, "fuzzy-aho-corasick-rs_amd"), os.path.join(REPO, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from fuzzy_aho_corasick import FuzzyAhoCorasickBuilder, FuzzyLimits
    from fuzzy_aho_corasick.distributed import gather_rows, shard_bounds

    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = FuzzyAhoCorasickBuilder().fuzzy(FuzzyLimits().edits(1)).case_insensitive(True).device(0)
    if use_gpu:
        staged = b.build(PATTERNS).stage(HAY.encode("utf-8"))
        a, e = shard_bounds(staged.graphemes, world, rank)
        rows, _ = staged.search_windows(0.7, a, e)
        full = staged.search_windows(0.7)[0] if rank == 0 else None
    else:
        from oracle_harness import OracleEngine, graphemes
        eng = OracleEngine(b, PATTERNS)
        n = len(graphemes(HAY))
        a, e = shard_bounds(n, world, rank)
        rows = eng.raw_rows(HAY, 0.7, windows=(a, e))
        full = eng.raw_rows(HAY, 0.7) if rank == 0 else None
    got = gather_rows(rows, torch.device("cpu"))
    if rank == 0:
        with open(out_path, "w") as f:
            f.write(repr((sorted(got), sorted(full))))
    dist.barrier()
    dist.destroy_process_group()


def _run(use_gpu):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.txt")
        mp.spawn(_worker, args=(2, _free_port(), use_gpu, out), nprocs=2, join=True)
        got, full = eval(open(out).read())
    assert got == full and len(full) > 10


def test_shard_bounds_partition():
    sys.path.insert(0, os.path.join(REPO, "fuzzy-aho-corasick-rs_amd"))
    from fuzzy_aho_corasick.distributed import shard_bounds
    for n in (0, 1, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            rs = [shard_bounds(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


def test_two_rank_gloo_shard_and_gather_cpu():
    _run(False)


@pytest.mark.gpu
def test_two_rank_gloo_shard_and_gather_gpu():
    _run(True)


def _rec_worker(rank, world, port, out_path):
    sys.path[:0] = [os.path.join(REPO, "fuzzy-aho-corasick-rs_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import numpy as np
    import torch
    import torch.distributed as dist
    from fuzzy_aho_corasick._native import MATCH_DTYPE
    from fuzzy_aho_corasick.distributed import gather_records
    dist.init_process_group("gloo", rank=rank, world_size=world)
    recs = np.zeros(3 + rank, dtype=MATCH_DTYPE)
    recs["start"] = np.arange(len(recs)) + 100 * rank
    recs["end"] = recs["start"] + 5
    recs["pattern_index"] = rank
    recs["similarity"] = np.float32(0.5 + rank / 8)
    got = gather_records(recs, torch.device("cpu"))
    if rank == 0:
        with open(out_path, "w") as f:
            f.write(repr([(int(r["start"]), int(r["end"]), int(r["pattern_index"]), float(r["similarity"])) for r in got]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_gather_records_cpu():
    """The bench's record-array gather (32-byte fac_match structs as bytes over the collective)."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.txt")
        mp.spawn(_rec_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        got = eval(open(out).read())
    want = [(i, i + 5, 0, 0.5) for i in range(3)] + [(100 + i, 105 + i, 1, 0.625) for i in range(4)]
    assert got == want
