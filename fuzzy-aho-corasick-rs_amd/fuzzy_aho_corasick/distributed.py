"""Multi-GPU search: one process per GPU (torch.distributed; backend "nccl" = RCCL on ROCm).

Start windows are independent and the best-map key holds the start byte (search.rs:444, 694), so
the path shards with no data-path collective; the only exchange is the final gather of the
32-byte Match records (the crate's OwnedMatch POD, stream.rs:719-745) to rank 0:
  * batch mode (C4): every rank searches its own haystack;
  * shard mode (C2/C3 on N GPUs): every rank stages only its slice of one haystack — the bytes
    whose start windows it owns plus a halo of max_match_graphemes() + 2 graphemes, cut at
    context-free grapheme boundaries (fac_shard_plan) — and keeps the global is_ascii, so the
    union of the shards' records is search_raw's result on the whole haystack.

The gather (`gather_device`) is an all_gather of the u64 record counts followed by point-to-point
sends of each rank's count x 32 B straight from its HBM record buffer to rank 0's (batched
isend/irecv: each peer has a direct xGMI link to rank 0). No rank receives records it does not
need and nothing is padded. The reference's parallel analogue is search_stream_parallel
(stream.rs:378-429), which fans windows out to threads and funnels their matches to one callback.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ._native import MATCH_DTYPE

REC_BYTES = 32
Row = Tuple[int, int, int, float, int, int, int, int, int]


def shard_bounds(n_windows: int, world: int, rank: int) -> Tuple[int, int]:
    """Even split of the start windows [0, n) into `world` contiguous ranges."""
    base, extra = divmod(n_windows, world)
    a = rank * base + min(rank, extra)
    return a, a + base + (1 if rank < extra else 0)


def stream_share_windows(total: int, block: int, share_index: int, overlap: int,
                         n_shares: int = 8, window: int = None) -> List[Tuple[int, int, int, int]]:
    """C5's cut of a stream of `total` bytes = total / block repeats of one `block`-byte block (SURVEY
    §8(d)): the stream is split into `n_shares` contiguous shares (one per GPU of the 8-GPU node;
    GPU g takes share g, so a run on fewer GPUs keeps each GPU's work: weak scaling), and the share
    into windows cut at block and share boundaries and every `window` bytes (None: blocks only; the
    crate's DEFAULT_WINDOW is 256 KiB, stream.rs:65 -- its WindowReader fed 64 KiB reads cuts windows
    of window + overlap bytes that commit `window` bytes each, :102-158, which is this cut shifted by
    the overlap). A window is searched exactly like stream.rs window_matches (:262-297): its text
    is its bytes plus `overlap` following bytes (max_match_graphemes() + 1 of an ASCII stream,
    :256-258, clipped at the stream's end), and it owns the matches starting in its bytes. The block
    is resident once as block || block[:overlap], so every window is a contiguous slice of it:
    returns (g_begin, g_end, commit, base) = the slice [g_begin, g_end) of that buffer, the owned byte
    count, the window's stream offset."""
    share = total // n_shares
    lo, hi = share_index * share, ((share_index + 1) * share if share_index + 1 < n_shares else total)
    out = []
    c = lo
    while c < hi:
        c1 = min(hi, (c // block + 1) * block)
        if window:
            c1 = min(c1, c + window)
        o = c % block
        end = min(total, c1 + overlap)
        out.append((o, o + (end - c), c1 - c, c))
        c = c1
    return out


def _wire_device(group) -> torch.device:
    """Where collective buffers live: HBM for RCCL, host memory for gloo (CPU tests)."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_device(recs: torch.Tensor, n: int, dst: int = 0, group=None) -> Optional[torch.Tensor]:
    """Gather every rank's `n` records (a uint8 tensor of >= n * 32 bytes, in HBM for RCCL) to
    rank `dst`: all_gather of the counts, then one batched isend/irecv per peer carrying exactly
    count * 32 bytes. Returns the concatenation in rank order on `dst` (a uint8 tensor on the wire
    device), None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    wire = _wire_device(group)
    cnt = torch.tensor([n], dtype=torch.int64, device=wire)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    mine = recs[: n * REC_BYTES]
    if mine.device != wire:
        mine = mine.to(wire)
    if rank != dst:
        if n:
            dist.batch_isend_irecv([dist.P2POp(dist.isend, mine.contiguous(), dist.get_global_rank(group, dst)
                                               if group is not None else dst, group)])[0].wait()
        return None
    offs = np.concatenate([[0], np.cumsum(counts)]) * REC_BYTES
    out = torch.empty(int(offs[-1]), dtype=torch.uint8, device=wire)
    if n:
        out[offs[rank]: offs[rank] + n * REC_BYTES].copy_(mine)
    ops = []
    for r in range(world):
        if r == rank or counts[r] == 0:
            continue
        src = dist.get_global_rank(group, r) if group is not None else r
        ops.append(dist.P2POp(dist.irecv, out[offs[r]: offs[r + 1]], src, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return out


def records_to_tensor(recs: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).reshape(-1))


def tensor_to_records(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(MATCH_DTYPE)


def gather_records(recs: np.ndarray, dst: int = 0, group=None) -> Optional[np.ndarray]:
    """gather_device for a host NumPy array of 32-byte records (MATCH_DTYPE)."""
    t = records_to_tensor(recs)
    got = gather_device(t, len(recs), dst, group)
    return None if got is None else tensor_to_records(got)


def gather_rows(rows: Sequence[Row], dst: int = 0, group=None) -> Optional[List[Row]]:
    """gather_records for row tuples (start, end, pattern, sim, ins, del, sub, swp, edits)."""
    recs = np.zeros(len(rows), dtype=MATCH_DTYPE)
    if rows:
        cols = list(zip(*rows))
        for name, col in zip(("start", "end", "pattern_index", "similarity", "insertions", "deletions",
                              "substitutions", "swaps", "edits"), cols):
            recs[name] = col
    got = gather_records(recs, dst, group)
    if got is None:
        return None
    return [(int(r["start"]), int(r["end"]), int(r["pattern_index"]), float(r["similarity"]), int(r["insertions"]),
             int(r["deletions"]), int(r["substitutions"]), int(r["swaps"]), int(r["edits"])) for r in got]


def check_grapheme_total(owned_graphemes: int, group=None) -> None:
    """search_raw refuses a haystack of more than u32::MAX graphemes (search.rs:198-201); a sharded
    haystack is refused the same way, on the global count."""
    from .structs import HaystackTooLarge
    t = torch.tensor([owned_graphemes], dtype=torch.int64, device=_wire_device(group))
    dist.all_reduce(t, group=group)
    total = int(t.item())
    if total > 0xFFFFFFFF:
        raise HaystackTooLarge(total)


def auto_beam_prefix(staged, threshold: float, group=None) -> int:
    """Running auto-beam total (search.rs:1096-1103) of every window before this rank's shard: each
    rank counts its own windows unbeamed (fac_auto_beam_total), the totals are all-gathered and the
    exclusive prefix is this rank's starting total."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    t = torch.tensor([staged.auto_beam_total(threshold)], dtype=torch.int64, device=_wire_device(group))
    totals = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(totals, t, group=group)
    return int(sum(int(x.item()) for x in totals[:rank]))


def sharded_search(engine, data: bytes, threshold: float, group=None, staged=None, is_ascii: int = -1):
    """search_raw of one haystack across the group's ranks (one GPU each): every rank stages its
    halo-sliced shard, searches its start windows with the records left in HBM and sends them to
    rank 0, which returns the full raw result as a NumPy record array (None on other ranks)."""
    from .engine import StagedHaystack
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if staged is None:
        staged = StagedHaystack.shard(engine, data, world, rank, is_ascii)
    check_grapheme_total(staged.owned_windows, group)
    prefix = 0
    b = engine.builder
    if b._auto_beam is not None and b._beam_width is None:
        prefix = auto_beam_prefix(staged, threshold, group)
    recs, n, _ = staged.search_device(threshold, auto_beam_prefix=prefix)
    got = gather_device(recs, n, 0, group)
    return None if got is None else tensor_to_records(got)
