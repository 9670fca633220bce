"""Multi-GPU search: one process per GPU (torch.distributed; backend "nccl" = RCCL on ROCm).

Start windows are independent and the best-map key holds the start byte (search.rs:444, 694), so
the path shards with no data-path collective; the only exchange is the final gather of the
32-byte Match records (the crate's OwnedMatch POD, stream.rs:719-745) to rank 0:
  * batch mode  (C4): every rank searches its own haystack;
  * shard mode (C2/C3 on N GPUs): every rank searches the start windows [a_r, b_r) of one
    haystack (`shard_bounds`), keeping the global length so `j == n` / end-byte logic is unchanged.
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

REC = struct.Struct("<QQIf5B3x")  # fac_match, 32 bytes
assert REC.size == 32

Row = Tuple[int, int, int, float, int, int, int, int, int]


def shard_bounds(n_windows: int, world: int, rank: int) -> Tuple[int, int]:
    """Even split of the start windows [0, n) into `world` contiguous ranges."""
    base, extra = divmod(n_windows, world)
    a = rank * base + min(rank, extra)
    return a, a + base + (1 if rank < extra else 0)


def pack_rows(rows: Sequence[Row]) -> torch.Tensor:
    buf = bytearray(REC.size * len(rows))
    for i, r in enumerate(rows):
        REC.pack_into(buf, i * REC.size, *r)
    return torch.frombuffer(buf, dtype=torch.uint8) if buf else torch.zeros(0, dtype=torch.uint8)


def unpack_rows(t: torch.Tensor, n: int) -> List[Row]:
    data = bytes(t[: n * REC.size].cpu().numpy().tobytes())
    return [REC.unpack_from(data, i * REC.size) for i in range(n)]


def gather_rows(rows: Sequence[Row], device: torch.device, dst: int = 0, group=None) -> Optional[List[Row]]:
    """Gather every rank's Match records to `dst`: all_gather of the counts, then an all_gather of
    the records padded to the largest count (the volume is KBs-MBs; one collective each)."""
    world = dist.get_world_size(group)
    n = torch.tensor([len(rows)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    cap = max(1, max(counts)) * REC.size
    mine = torch.zeros(cap, dtype=torch.uint8, device=device)
    packed = pack_rows(rows)
    if packed.numel():
        mine[: packed.numel()] = packed.to(device)
    bufs = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(bufs, mine, group=group)
    if dist.get_rank(group) != dst:
        return None
    out: List[Row] = []
    for b, c in zip(bufs, counts):
        out.extend(unpack_rows(b, c))
    return out


def gather_records(recs, device: torch.device, dst: int = 0, group=None):
    """gather_rows for a NumPy array of 32-byte records (fac_match): the records travel as bytes,
    rank `dst` receives one concatenated array."""
    import numpy as np
    from ._native import MATCH_DTYPE
    world = dist.get_world_size(group)
    n = torch.tensor([len(recs)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    cap = max(1, max(counts)) * REC.size
    mine = torch.zeros(cap, dtype=torch.uint8, device=device)
    if len(recs):
        mine[: len(recs) * REC.size] = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8)).to(device)
    bufs = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(bufs, mine, group=group)
    if dist.get_rank(group) != dst:
        return None
    parts = [b[: c * REC.size].cpu().numpy().view(MATCH_DTYPE) for b, c in zip(bufs, counts)]
    return np.concatenate(parts) if parts else np.zeros(0, dtype=MATCH_DTYPE)


def sharded_search(staged, threshold: float, device: torch.device, group=None) -> Optional[List[Row]]:
    """Search one staged haystack across the group's ranks; rank 0 receives the full raw result
    (identical to search_raw on the whole haystack)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    a, b = shard_bounds(staged.graphemes, world, rank)
    rows, _ = staged.search_windows(threshold, a, b)
    return gather_rows(rows, device, 0, group)
