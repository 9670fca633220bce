#!/usr/bin/env python3
"""bench.py — haystack Gchars/s of the MI355X fuzzy Aho–Corasick engine (BASELINE.json metric).

Workload (default): BASELINE.json configs[2] — edits=2, beam_width=64, 10K patterns,
case-insensitive Unicode graphemes, one MI355X per rank — on seeded synthetic data
(fuzzy_aho_corasick/workloads.py, SURVEY.md §8(d) generator). A "step" is one pass of the hot path
(FuzzyAhoCorasick::search_raw over every start window of the rank's device-resident haystack) with
the 32-byte Match records delivered to rank 0's host memory: at N = 1 straight D2H, at N > 1 sent
from each rank's HBM to rank 0 over RCCL (counts all-gather + point-to-point sends) and then D2H.

Modes:
  default (weak scaling, the C4 batch layout): every rank owns its own haystack of the size;
  --shard (strong scaling): one haystack; every rank stages only its halo-sliced shard;
  --config c5: the 100 GiB streaming run (100 x a 1 GiB block, pre-filter on): each GPU processes
    its 1/8 share (12.5 GiB) as device-resident stream windows (stream.rs window_matches).

    python bench.py [--gpus N --steps K --warmup W --config c3 --mib 256 --shard]

`--gpus N` with N > 1 outside torchrun re-launches this script under torch.distributed.run with N
ranks (before any GPU call); under torchrun, --gpus must equal WORLD_SIZE.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "fuzzy-aho-corasick-rs_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
DEFAULT_MIB = {"c1": 1, "c2": 1024, "c3": 256, "c4": 128, "c5": 1024}  # C2: the 1 GB of BASELINE configs[1]
# CPU baseline samples: prefixes of the same haystack for the all-cores leg
CPU_PREFIX_MIB = {"c1": 1, "c2": 64, "c3": 16, "c4": 64, "c5": 64}
WORKLOAD = {
    "c1": "exact, 16 ASCII patterns",
    "c2": "edits=1, 1K ASCII patterns",
    "c3": "edits=2, beam_width=64, 10K patterns, case-insensitive Unicode graphemes",
    "c4": "edits=1, 1K ASCII patterns (C2 engine), one 128 MiB haystack per GPU (seeds 40..47)",
    "c5": "streaming, edits=1, 1K patterns (10-16), threshold 0.85, bitap prefilter, 1/8 of 100 GiB per GPU",
}
METRIC = "haystack Gchars/s at edits<=2, 10K patterns; 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=["c1", "c2", "c3", "c4", "c5", "stream"])
    ap.add_argument("--mib", type=float, default=None, help="haystack MiB per rank (c5: block MiB)")
    ap.add_argument("--shard", action="store_true", help="strong scaling: shard one haystack over the ranks")
    ap.add_argument("--end-to-end", action="store_true",
                    help="time search_raw from host bytes: staging (H2D, UTF-8 check, segmentation) -> records")
    ap.add_argument("--prestaged", action="store_true",
                    help="diagnostic: stage the haystack once before the timed steps (search only)")
    ap.add_argument("--gib", type=float, default=100.0, help="c5: total stream GiB (each GPU takes 1/8)")
    ap.add_argument("--window-kib", type=float, default=256.0,
                    help="c5: stream window bytes (KiB; the crate's DEFAULT_WINDOW, stream.rs:65); 0: one window per 1 GiB block")
    ap.add_argument("--vocab", type=int, default=50_000,
                    help="filler words drawn from a fixed vocabulary of this many random words; 0: fresh random words")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="single-thread CPU baseline sample budget")
    ap.add_argument("--cpu-min-mib", type=float, default=None,
                    help="single-thread CPU baseline: at least this many MiB of the haystack (default 2)")
    ap.add_argument("--no-fresh-diag", action="store_true",
                    help="skip every extra diagnostics leg: fresh_words (c2/c3 at N=1: the same config on SURVEY "
                         "§8(d)'s fresh-word generator), strong_emulated (N=1: the --shard step of every shard of "
                         "N in {2,4,8} timed one after another on this GPU), strong (N>1: the --shard step measured "
                         "beside the weak one), and the default run's c2 / c5 legs")
    ap.add_argument("--cpu-threads", type=int, default=16, help="all-cores CPU baseline threads (box share: 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=None, help="default: profiles/traffic_<config>.json")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/gather plumbing only (gloo, no GPU, no search): for CPU tests of --gpus N")
    return ap.parse_args()


def relaunch(args) -> int:
    """Run this script under torch.distributed.run with args.gpus ranks (this process has touched no
    GPU), wait, and return its exit code."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def sources_sha() -> str:
    """Hash of the kernel and host sources (csrc/): a traffic.json measured on other sources is stale."""
    h = hashlib.sha256()
    d = os.path.join(REPO, "fuzzy-aho-corasick-rs_amd", "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".cpp", ".h", ".inc")):
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus is not None and args.gpus > 1:
        sys.exit(relaunch(args))
    world = int(world_env or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with --nproc-per-node {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    if args.dry_run:
        return run_dry(args, world, rank)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))  # RCCL on ROCm
    if args.config == "c5":
        return run_c5(args, world, rank, local)
    if args.config == "stream":
        return run_stream(args, world, rank, local)

    from fuzzy_aho_corasick import workloads as W
    from fuzzy_aho_corasick.engine import StagedHaystack
    from fuzzy_aho_corasick.distributed import gather_device

    mib = args.mib if args.mib is not None else DEFAULT_MIB[args.config]
    nbytes = int(mib * (1 << 20))
    vocab = args.vocab or None
    if args.config == "c4":  # C2 engine, haystack seeds 40..47
        wl = W.config("c4", nbytes, hay_seed=40 + (0 if args.shard else rank), vocab=vocab)
    else:
        base_seed = {"c1": 1, "c2": 2, "c3": 3}[args.config]
        # weak scaling: every rank builds the same engine and owns a different haystack of equal size
        wl = W.config(args.config, nbytes, seed=base_seed,
                      hay_seed=base_seed + 1000 + (0 if args.shard else 101 * rank), vocab=vocab)
    engine = W.builder_for(wl).device(local).build(wl.patterns)
    stream = torch.cuda.current_stream().cuda_stream
    # default step = search_raw on device-resident input: the UTF-8 bytes are uploaded
    # once (H2D reported apart); every step stages them on the device (UTF-8 check, is_ascii, UAX #29
    # segmentation + folding: fac_haystack_stage_device), searches every start window and delivers
    # the records. --shard: each rank holds its halo-sliced shard's bytes [a, e) in HBM and stages
    # them the same way in every step (fac_haystack_stage_shard_device), so the strong-scaling step
    # is the N = 1 step's work split over the ranks. --prestaged (diagnostic) stages once outside the
    # timed steps.
    device_staging = not (args.prestaged or args.end_to_end)
    dev_hay, h2d_ms, plan = None, None, None
    if device_staging:
        import numpy as np
        from fuzzy_aho_corasick import _native
        lo, hi = 0, len(wl.haystack)
        if args.shard:  # fac_shard_plan on the host bytes, once: (a, b, e, global is_ascii, open end)
            plan = _native.shard_plan(engine.max_match_graphemes(), wl.haystack, world, rank)
            lo, hi = plan[0], plan[2]
        torch.cuda.synchronize()
        t = time.perf_counter()
        dev_hay = torch.from_numpy(np.frombuffer(wl.haystack, dtype=np.uint8)[lo:hi].copy()).to(torch.device("cuda", local))
        torch.cuda.synchronize()
        h2d_ms = (time.perf_counter() - t) * 1e3
        if args.shard:
            staged = StagedHaystack.shard_from_device(engine, dev_hay.data_ptr(), plan, stream)
        else:
            staged = StagedHaystack.from_device(engine, dev_hay.data_ptr(), len(wl.haystack), stream)
    else:
        staged = StagedHaystack(engine, wl.haystack)
    windows = staged.owned_windows  # graphemes this rank searches per step
    host_buf = [None]  # rank 0: pinned landing buffer of the gathered records
    stage_ms = [0.0]

    def step():
        if args.end_to_end:  # search_raw from host bytes: staging (H2D, UTF-8 check, segmentation + fold) + search
            hs = StagedHaystack(engine, wl.haystack)
            rows, st = hs.search_windows_records(wl.threshold, stream=stream)
            del hs
            return len(rows), st
        hs = staged
        if device_staging:  # synchronous: its kernels are done on return
            t = time.perf_counter()
            if args.shard:
                hs = StagedHaystack.shard_from_device(engine, dev_hay.data_ptr(), plan, stream, reuse=staged)
            else:
                hs = StagedHaystack.from_device(engine, dev_hay.data_ptr(), len(wl.haystack), stream, reuse=staged)
            stage_ms[0] += (time.perf_counter() - t) * 1e3
        if world == 1:  # records D2H into the library's pooled pinned buffers
            rows, st = (hs.search_prefiltered_records(wl.threshold, stream=stream) if wl.prefilter
                        else hs.search_windows_records(wl.threshold, stream=stream))
            return len(rows), st
        recs, n, st = hs.search_device(wl.threshold, stream=stream)
        got = gather_device(recs, n, 0)  # RCCL: counts all-gather + point-to-point sends to rank 0
        if got is not None:
            if host_buf[0] is None or host_buf[0].numel() < got.numel():
                host_buf[0] = torch.empty(int(got.numel() * 1.25) + 4096, dtype=torch.uint8, pin_memory=True)
            host_buf[0][: got.numel()].copy_(got)
            return got.numel() // 32, st
        return n, st

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stage_ms[0] = 0.0
    t0 = time.perf_counter()
    acc = dict(kernel_ms=0.0, lane_ms=0.0, cache_ms=0.0, prefilter_ms=0.0, launches=0, popped=0, cached=0,
               lane_windows=0, matches=0)
    for _ in range(args.steps):
        nrec, st = step()
        acc["kernel_ms"] += st.kernel_ms
        acc["lane_ms"] += st.lane_ms
        acc["cache_ms"] += st.cache_ms
        acc["prefilter_ms"] += st.prefilter_ms
        acc["launches"] += st.kernel_launches
        acc["popped"] += st.states_popped
        acc["cached"] += st.states_cached
        acc["lane_windows"] += st.lane_windows
        acc["matches"] += nrec
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    total_graphemes = windows * args.steps
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        g = torch.tensor([windows], device="cuda", dtype=torch.int64)
        dist.all_reduce(g)
        total_graphemes = int(g.item()) * args.steps

    value = total_graphemes / elapsed / 1e9
    K = max(1, args.steps)
    # Roofline of the whole step: this rank's algorithmic bytes (its haystack's UTF-8
    # bytes read once + 32 B per record written) over the device time of every kernel of the step —
    # prefix-cache counts/builds/publishes and lookups, the lane-serial and the wave kernels (HIP events
    # on the search streams), or the bitap scan + re-search for the pre-filter.
    step_dev_ms = (acc["cache_ms"] + acc["lane_ms"] + acc["kernel_ms"] + acc["prefilter_ms"] + stage_ms[0]) / K
    rank_bytes = staged.owned_bytes if args.shard else len(wl.haystack)
    recs_rank = acc["matches"] / K / (world if world > 1 else 1)
    bytes_step = rank_bytes + 32 * recs_rank
    achieved = bytes_step / (step_dev_ms / 1e3) / 1e9 if step_dev_ms > 0 else 0.0
    traffic, traffic_note = load_traffic(args, mib)

    fresh = strong = legs = None
    if (world == 1 and args.config in ("c2", "c3") and args.vocab and device_staging and not args.no_fresh_diag):
        fresh = fresh_words_diag(args, engine, nbytes, local, stream)
    if args.config in ("c2", "c3", "c4") and device_staging and not args.shard and not args.no_fresh_diag:
        base_hay = wl.haystack if world == 1 else base_haystack(args, nbytes, vocab)
        if world == 1:  # every shard of N in {2, 4, 8} on this GPU, one after another
            strong = strong_emulated(engine, base_hay, wl.threshold, local, stream, elapsed / args.steps * 1e3)
        else:  # the --shard step on the same ranks, beside the weak one
            strong = strong_measured(engine, base_hay, wl.threshold, world, rank, local, stream, args.steps)
        del base_hay
    if world == 1 and args.config == "c3" and device_staging and not args.no_fresh_diag and args.mib is None:
        legs = default_legs(args, local)  # C2 (1 GiB) and C5 (one GPU's 12.5 GiB share) in the driver's run

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        min_mib = args.cpu_min_mib if args.cpu_min_mib is not None else 2.0  # at least 2 MiB single-thread
        cpu = cpu_baseline(wl, args.cpu_seconds, args.cpu_threads, int(min_mib * (1 << 20)))

    if rank == 0:
        wave_ms = acc["kernel_ms"] / K
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "Gchars/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.shard else "weak",
            "vs_baseline": None,
            "dtype": "u32 code points / f32 penalties",
            "data": "synthetic (seeded xorshift generator, SURVEY.md §8(d)): random words of 2-12 chars "
                    + (f"drawn from a fixed {args.vocab}-word random vocabulary" if args.vocab else "(every word fresh)")
                    + ", separated by ' ', one planted pattern with 0..edits random edits every 4 KiB",
            "config": {
                "workload": f"{args.config}: " + WORKLOAD[args.config],
                "patterns": len(wl.patterns),
                "haystack_bytes_per_gpu": rank_bytes,
                "graphemes_per_gpu": windows,
                "threshold": wl.threshold,
                "filler_vocabulary": args.vocab or "fresh",
                "timed_step": timed_step_desc(args),
                "parallelism": (f"shard{world} (strong: one {len(wl.haystack)}-byte haystack, halo-sliced shards)"
                                if args.shard else f"dp{world} (weak: one haystack per GPU)")
                               + (", RCCL gather of Match records to rank 0" if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_note,
                "kernel": "whole search_raw step: staging (seg_tile + write_tile, synchronous) + prefix-cache "
                          "count/build/publish + rc_lookup + lane_window + bfs_window kernels" if not wl.prefilter else
                          "pre-filter (q-gram scan + verify / packed bitap) + runs + re-search",
                "avg_kernel_ms": step_dev_ms,
                "algorithmic_bytes_per_launch": bytes_step,
                "wave_kernel_only": {"kernel": "bfs_window_kernel", "avg_ms": wave_ms,
                                     "frac": (bytes_step / (wave_ms / 1e3) / 1e9 / HBM_PEAK_GBS) if wave_ms > 0 else None},
            },
            "cpu_baseline": cpu,
            "diagnostics": {
                "matches_per_step": acc["matches"] / K,
                "states_popped_per_step": acc["popped"] / K,
                "states_per_second": acc["popped"] / max(1e-9, acc["kernel_ms"] / 1e3),
                "kernel_launches": acc["launches"],
                "search_kernel_ms_per_step": wave_ms,
                "lane_kernel_ms_per_step": acc["lane_ms"] / K,
                "lane_windows_per_step": acc["lane_windows"] / K,
                "prefilter_ms_per_step": acc["prefilter_ms"] / K,
                "prefix_cache_ms_per_step": acc["cache_ms"] / K,
                "staging_ms_per_step": stage_ms[0] / K,
                "h2d_ms_once": h2d_ms,
                "states_from_prefix_cache_per_step": acc["cached"] / K,
                "sources_sha": sources_sha(),
                "fresh_words": fresh,
                ("strong_emulated" if world == 1 else "strong"): strong,
                **(legs or {}),
            },
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def timed_step_desc(args) -> str:
    """What one timed step covers (the line's config.timed_step)."""
    if args.end_to_end:
        return "search_raw from host bytes (H2D + staging + search + records)"
    if args.prestaged:
        return "search only (haystack staged before the timed steps)"
    return ("search_raw on device-resident bytes: device staging (UTF-8 check, is_ascii, UAX #29 segmentation + "
            "folding" + (" of the rank's halo-sliced shard" if args.shard else "") + ") + search + records"
            + (" gathered to rank 0 over RCCL" if args.gpus and args.gpus > 1 else ""))


def fresh_words_diag(args, engine, nbytes, local, stream, steps=2):
    """The same engine and size on SURVEY.md §8(d)'s generator taken literally (every filler word
    fresh, bench.py --vocab 0): device-resident bytes, the same timed step (device staging + search +
    records D2H), `steps` steps after one warm-up. Reported beside the headline."""
    import numpy as np
    import torch
    from fuzzy_aho_corasick import workloads as W
    from fuzzy_aho_corasick.engine import StagedHaystack
    base_seed = {"c2": 2, "c3": 3}[args.config]
    wl = W.config(args.config, nbytes, seed=base_seed, hay_seed=base_seed + 1000, vocab=None)
    dev = torch.from_numpy(np.frombuffer(wl.haystack, dtype=np.uint8).copy()).to(torch.device("cuda", local))
    staged = StagedHaystack.from_device(engine, dev.data_ptr(), len(wl.haystack), stream)
    n = 0

    def step():
        hs = StagedHaystack.from_device(engine, dev.data_ptr(), len(wl.haystack), stream, reuse=staged)
        rows, st = hs.search_windows_records(wl.threshold, stream=stream)
        return len(rows), st

    step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    cache = lane = kern = 0.0
    for _ in range(steps):
        n, st = step()
        cache += st.cache_ms
        lane += st.lane_ms
        kern += st.kernel_ms
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    out = {"value": staged.owned_windows / dt / 1e9, "unit": "Gchars/s", "ms_per_step": dt * 1e3, "steps": steps,
           "matches_per_step": n, "haystack_bytes": len(wl.haystack), "graphemes": staged.owned_windows,
           "prefix_cache_ms_per_step": cache / steps, "lane_kernel_ms_per_step": lane / steps,
           "search_kernel_ms_per_step": kern / steps,
           "data": "every filler word fresh (SURVEY.md §8(d) generator), same seeds otherwise"}
    del staged, dev
    return out


def base_haystack(args, nbytes, vocab):
    """Rank 0's haystack of the config (the one --shard splits)."""
    from fuzzy_aho_corasick import workloads as W
    if args.config == "c4":
        return W.config("c4", nbytes, hay_seed=40, vocab=vocab).haystack
    base_seed = {"c1": 1, "c2": 2, "c3": 3}[args.config]
    return W.config(args.config, nbytes, seed=base_seed, hay_seed=base_seed + 1000, vocab=vocab).haystack


def shard_steps(engine, hay, n, r, local, stream, world=1):
    """The --shard step on shard r of n of `hay`: the shard's bytes [a, e) resident in HBM, staged on
    the device (fac_haystack_stage_shard_device) and searched in every step, records to rank 0 (RCCL
    gather at world > 1, else D2H). Returns (the staged shard, step(threshold), the device bytes,
    [records of the last step])."""
    import numpy as np
    import torch
    from fuzzy_aho_corasick import _native
    from fuzzy_aho_corasick.engine import StagedHaystack
    from fuzzy_aho_corasick.distributed import gather_device
    plan = _native.shard_plan(engine.max_match_graphemes(), hay, n, r)
    a, e = plan[0], plan[2]
    dev = torch.from_numpy(np.frombuffer(hay, dtype=np.uint8)[a:e].copy()).to(torch.device("cuda", local))
    staged = StagedHaystack.shard_from_device(engine, dev.data_ptr() if e > a else 0, plan, stream)
    nrec = [0]

    def step(threshold):
        hs = StagedHaystack.shard_from_device(engine, dev.data_ptr() if e > a else 0, plan, stream, reuse=staged)
        if world == 1:
            rows, _ = hs.search_windows_records(threshold, stream=stream)
            nrec[0] = len(rows)
            return
        recs, k, _ = hs.search_device(threshold, stream=stream)
        got = gather_device(recs, k, 0)
        nrec[0] = got.numel() // 32 if got is not None else k

    return staged, step, dev, nrec


def key_part_steps(engine, hay, n, r, local, stream, world=1):
    """The key-split step on part r of n of `hay`: the whole haystack resident in HBM and staged on
    the device in every step (fac_haystack_stage_device), searching only the start windows whose first
    two characters hash to part r (fac_haystack_set_key_partition), records to rank 0 (RCCL gather at
    world > 1, else D2H). Same return shape as shard_steps."""
    import numpy as np
    import torch
    from fuzzy_aho_corasick.engine import StagedHaystack
    from fuzzy_aho_corasick.distributed import gather_device
    dev = torch.from_numpy(np.frombuffer(hay, dtype=np.uint8).copy()).to(torch.device("cuda", local))
    staged = StagedHaystack.from_device(engine, dev.data_ptr(), len(hay), stream).set_key_partition(n, r)
    nrec = [0]

    def step(threshold):
        hs = StagedHaystack.from_device(engine, dev.data_ptr(), len(hay), stream, reuse=staged)
        if world == 1:
            rows, _ = hs.search_windows_records(threshold, stream=stream)
            nrec[0] = len(rows)
            return
        recs, k, _ = hs.search_device(threshold, stream=stream)
        got = gather_device(recs, k, 0)
        nrec[0] = got.numel() // 32 if got is not None else k

    return staged, step, dev, nrec


def _time_shard(engine, hay, n, r, local, stream, steps, threshold, world=1, keys=False):
    import torch
    import torch.distributed as dist
    staged, step, dev, nrec = (key_part_steps if keys else shard_steps)(engine, hay, n, r, local, stream, world=world)
    step(threshold)  # warm-up
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step(threshold)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    out = (dt, staged.owned_windows if not keys else staged.graphemes / n, nrec[0], staged.owned_bytes)
    del staged, dev
    return out


def strong_emulated(engine, hay, threshold, local, stream, full_ms, ns=(2, 4, 8), steps=3):
    """Strong scaling of the headline, estimated on one GPU: for N in `ns`, every part
    r of N of the same haystack is staged from HBM and searched, one part after another; an N-GPU step
    takes the slowest part's time (+ the record gather), so predicted_speedup = the N = 1 step /
    max_rank_ms. Two splits: "shards" (bench.py --shard: contiguous byte ranges + halo, fac_shard_plan,
    each shard staging only its bytes) and "keys" (fac_haystack_set_key_partition: every rank stages
    the whole haystack and searches the start windows whose first two characters hash to its part, so
    a prefix-cache key is built once, on one GPU, for all its windows)."""
    out = {"method": "every part of N timed alone on this GPU (device staging + search + records D2H), predicted "
                     "N-GPU step = the slowest part; the RCCL gather excluded",
           "n1_ms": full_ms}
    for keys in (False, True):
        res = {}
        for n in ns:
            ms = []
            for r in range(n):
                dt, w, k, b = _time_shard(engine, hay, n, r, local, stream, steps, threshold, keys=keys)
                ms.append(dt / steps * 1e3)
            res[str(n)] = {"max_rank_ms": max(ms), "min_rank_ms": min(ms), "sum_rank_ms": sum(ms),
                           "predicted_speedup": full_ms / max(ms), "rank_ms": [round(x, 2) for x in ms]}
        out["keys" if keys else "shards"] = res
    return out


def strong_measured(engine, hay, threshold, world, rank, local, stream, steps):
    """At N > 1 (default weak run): one haystack over the same ranks, timed like the headline (barrier +
    synchronize on both sides, max over ranks), split both ways -- "shards" (--shard: contiguous byte
    ranges) and "keys" (fac_haystack_set_key_partition); value = the haystack's windows / that time."""
    import torch
    import torch.distributed as dist
    out = {}
    for keys in (False, True):
        dt, w, k, b = _time_shard(engine, hay, world, rank, local, stream, steps, threshold, world=world, keys=keys)
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        g = torch.tensor([float(w)], device="cuda", dtype=torch.float64)
        dist.all_reduce(g)
        dt = float(t.item())
        out["keys" if keys else "shards"] = {
            "value": float(g.item()) * steps / dt / 1e9, "unit": "Gchars/s", "ms_per_step": dt / steps * 1e3,
            "steps": steps, "haystack_bytes": len(hay), "records_per_step": k,
            "step": ("every rank stages the whole haystack on the device and searches its key part "
                     "(fac_haystack_set_key_partition)" if keys else
                     "--shard: every rank stages its halo-sliced shard on the device and searches it")
                    + ", records gathered to rank 0 over RCCL"}
    return out


def default_legs(args, local):
    """The default run's extra configs (measured by the driver's own run): C2 (edits 1,
    1K ASCII patterns, 1 GiB, the C2 step) and C5 (one GPU's 12.5 GiB share of the 100 GiB stream)."""
    import numpy as np
    import torch
    from fuzzy_aho_corasick import workloads as W
    from fuzzy_aho_corasick.engine import StagedHaystack
    out = {}
    stream = torch.cuda.current_stream().cuda_stream
    t0 = time.perf_counter()
    wl = W.config("c2", DEFAULT_MIB["c2"] << 20, seed=2, hay_seed=1002)
    eng = W.builder_for(wl).device(local).build(wl.patterns)
    dev = torch.from_numpy(np.frombuffer(wl.haystack, dtype=np.uint8).copy()).to(torch.device("cuda", local))
    staged = StagedHaystack.from_device(eng, dev.data_ptr(), len(wl.haystack), stream)
    gen_s = time.perf_counter() - t0
    acc = dict(cache=0.0, lane=0.0, kern=0.0, n=0)

    def step():
        hs = StagedHaystack.from_device(eng, dev.data_ptr(), len(wl.haystack), stream, reuse=staged)
        rows, st = hs.search_windows_records(wl.threshold, stream=stream)
        return len(rows), st

    step()
    torch.cuda.synchronize()
    steps = 5
    t = time.perf_counter()
    for _ in range(steps):
        n, st = step()
        acc["n"] = n
        acc["cache"] += st.cache_ms
        acc["lane"] += st.lane_ms
        acc["kern"] += st.kernel_ms
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    alg = len(wl.haystack) + 32 * acc["n"]
    out["c2"] = {"value": staged.owned_windows / dt / 1e9, "unit": "Gchars/s", "ms_per_step": dt * 1e3, "steps": steps,
                 "workload": "c2: " + WORKLOAD["c2"], "haystack_bytes": len(wl.haystack), "matches_per_step": acc["n"],
                 "prefix_cache_ms_per_step": acc["cache"] / steps, "lane_kernel_ms_per_step": acc["lane"] / steps,
                 "search_kernel_ms_per_step": acc["kern"] / steps,
                 "roofline_frac_step": alg / dt / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": alg,
                 "setup_s": gen_s, "timed_step": timed_step_desc(args)}
    del staged, dev, eng, wl
    torch.cuda.empty_cache()
    c5 = c5_measure(args, 1, 0, local, steps=2, warmup=1, gib=100.0)
    c5.pop("_wl")
    out["c5"] = {k: c5[k] for k in ("value", "unit", "ms_per_step", "steps", "bytes_per_gpu", "stream_windows_per_gpu",
                                    "window_bytes", "batches_per_step", "matches_per_step", "prefilter_ms_per_step",
                                    "research_kernel_ms_per_step", "roofline_frac_kernels", "roofline_frac_step",
                                    "setup_s", "workload")}
    return out


def load_traffic(args, mib):
    """PMC traffic per step (profiles/make_traffic.py) if it was measured on this config, size and
    these sources; else (None, why)."""
    path = args.traffic_json or os.path.join(REPO, "profiles", f"traffic_{args.config}.json")
    if not os.path.exists(path):
        return None, f"no {os.path.relpath(path, REPO)}"
    tj = json.load(open(path))
    if tj.get("sources_sha") != sources_sha():
        return None, f"{os.path.relpath(path, REPO)} is stale (sources {tj.get('sources_sha')} != {sources_sha()})"
    if tj.get("config") != args.config or abs(tj.get("mib", -1) - mib) > 1e-6 or args.shard or args.vocab != 50_000:
        return None, f"{os.path.relpath(path, REPO)} was measured on another workload"
    return tj.get("hbm_bytes_per_step"), tj.get("source")


def c5_measure(args, world, rank, local, steps, warmup, gib):
    """C5: a `gib` GiB stream = repeats of one deterministic 1 GiB block (1 needle per
    MiB), resident once in HBM as block || block[:halo]. GPU g processes its contiguous 1/8 of the
    stream as windows cut at block and share boundaries, each searched on the device exactly like
    stream.rs window_matches: the window's text (its bytes plus max_match_graphemes() + 1 of
    overlap, stream.rs:256-258) through Prefiltered::search, ranked sorted().non_overlapping(), and
    the matches starting before the commit point kept, at absolute offsets. Returns the timing dict
    (every rank; elapsed is the max over ranks)."""
    import torch
    import torch.distributed as dist
    from fuzzy_aho_corasick import workloads as W
    from fuzzy_aho_corasick.engine import StagedHaystack
    from fuzzy_aho_corasick.distributed import gather_device, stream_share_windows
    from fuzzy_aho_corasick._native import MATCH_DTYPE

    t_setup = time.perf_counter()
    block_bytes = int((args.mib if (args.mib is not None and args.config == "c5") else DEFAULT_MIB["c5"]) * (1 << 20))
    wl = W.config("c5", block_bytes, seed=5)
    block = wl.haystack
    engine = W.builder_for(wl).device(local).build(wl.patterns)
    overlap = engine.max_match_graphemes() + 1  # stream_overlap (stream.rs:256-258); ASCII: bytes
    B = len(block)
    staged = StagedHaystack(engine, block + block[:overlap])
    total = int(gib * (1 << 30)) // B * B  # whole blocks
    # this GPU's 1/8 of the stream (weak scaling: rank r takes share r)
    window_bytes = int(args.window_kib * 1024) if args.window_kib else None  # None: 1 GiB block windows
    windows = stream_share_windows(total, B, rank, overlap, window=window_bytes)
    processed_rank = sum(w[2] for w in windows)
    # batches: the windows of one block pass (contiguous in the resident block), one batched call each
    batches, cur = [], []
    for w in windows:
        if cur and w[0] < cur[-1][0]:
            batches.append(cur)
            cur = []
        cur.append(w)
    if cur:
        batches.append(cur)
    stream = torch.cuda.current_stream().cuda_stream
    setup_s = time.perf_counter() - t_setup

    dev_recs = [torch.empty(1 << 20, dtype=torch.uint8, device=torch.device("cuda", local))]

    def step():
        # every window's owned records (stream.rs:262-297) appended in HBM in stream order, then at
        # N > 1 one RCCL gather to rank 0 from there, at N = 1 one copy to host memory
        pf_ms, k_ms, n = 0.0, 0.0, 0
        for bw in batches:
            dev_recs[0], got, st = staged.stream_windows_device(bw, wl.threshold, True, dev_recs[0], n, stream=stream)
            n += got
            pf_ms += st.prefilter_ms
            k_ms += st.kernel_ms
        if world > 1:
            gathered = gather_device(dev_recs[0], n, 0)
            return (gathered.numel() // 32 if gathered is not None else 0), pf_ms, k_ms
        recs = dev_recs[0][: n * 32].cpu().numpy().view(MATCH_DTYPE)
        return len(recs), pf_ms, k_ms

    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    matches = pf = km = 0
    for _ in range(steps):
        n, a, b = step()
        matches += n
        pf += a
        km += b
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    pr = torch.tensor([processed_rank], dtype=torch.int64, device="cuda")
    if world > 1:
        dist.all_reduce(pr)
    processed = int(pr.item()) * steps
    K = max(1, steps)
    dev_ms = (pf + km) / K
    bytes_step = processed_rank + 32 * matches / K / world
    out = {"value": processed / elapsed / 1e9, "unit": "Gchars/s", "ms_per_step": elapsed / steps * 1e3, "steps": steps,
           "elapsed_s": elapsed, "bytes_per_gpu": processed_rank, "stream_bytes": total,
           "stream_windows_per_gpu": len(windows), "window_bytes": window_bytes or B, "overlap": overlap, "block_bytes": B,
           "batches_per_step": len(batches),
           "matches_per_step": matches / K, "prefilter_ms_per_step": pf / K, "research_kernel_ms_per_step": km / K,
           "dev_ms": dev_ms, "algorithmic_bytes": bytes_step,
           "roofline_frac_kernels": (bytes_step / (dev_ms / 1e3) / 1e9 / HBM_PEAK_GBS) if dev_ms > 0 else None,
           "roofline_frac_step": bytes_step / (elapsed / steps) / 1e9 / HBM_PEAK_GBS,
           "setup_s": setup_s, "workload": "c5: " + WORKLOAD["c5"], "patterns": len(wl.patterns),
           "threshold": wl.threshold, "_wl": wl}
    del staged, engine
    return out


def run_c5(args, world, rank, local):
    """C5 line (--config c5): c5_measure at the requested stream size, CPU baseline on rank 0 at N = 1."""
    r = c5_measure(args, world, rank, local, args.steps, args.warmup, args.gib)
    wl = r.pop("_wl")
    traffic, traffic_note = load_traffic(args, args.gib * 1024)  # c5 traffic is keyed by the stream size
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        min_mib = args.cpu_min_mib if args.cpu_min_mib is not None else 2.0  # at least 2 MiB single-thread
        cpu = cpu_baseline(wl, args.cpu_seconds, args.cpu_threads, int(min_mib * (1 << 20)))
    if rank == 0:
        achieved = r["algorithmic_bytes"] / (r["dev_ms"] / 1e3) / 1e9 if r["dev_ms"] > 0 else 0.0
        print(json.dumps({
            "metric": METRIC, "value": r["value"], "unit": "Gchars/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": r["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8 haystack bytes / u32 bitap words",
            "data": f"synthetic: {r['stream_bytes'] / (1 << 30):g} GiB stream = repeats of one {r['block_bytes']}-byte block "
                    "(SURVEY.md §8(d) generator, 1 planted needle per MiB), resident in HBM",
            "config": {"workload": r["workload"], "patterns": r["patterns"],
                       "stream_bytes": r["stream_bytes"], "bytes_per_gpu": r["bytes_per_gpu"],
                       "stream_windows_per_gpu": r["stream_windows_per_gpu"], "window_bytes": r["window_bytes"],
                       "batches_per_step": r["batches_per_step"],
                       "window_overlap_graphemes": r["overlap"], "threshold": r["threshold"],
                       "parallelism": f"dp{world} (each GPU its 1/8 of the stream; RCCL gather of Match records)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_note,
                         "kernel": "pre-filter (q-gram scan + per-candidate bitap verify; packed bitap scan for "
                                   "patterns with pieces < 3 symbols) + runs_kernel + re-search of the merged windows",
                         "avg_kernel_ms": r["dev_ms"], "algorithmic_bytes_per_launch": r["algorithmic_bytes"]},
            "cpu_baseline": cpu,
            "diagnostics": {"matches_per_step": r["matches_per_step"], "prefilter_ms_per_step": r["prefilter_ms_per_step"],
                            "research_kernel_ms_per_step": r["research_kernel_ms_per_step"], "sources_sha": sources_sha()},
        }), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


class _RepeatReader:
    """An in-memory reader of `total` bytes: repeats of `block` (io.RawIOBase-like read(n))."""

    def __init__(self, block: bytes, total: int):
        self.block, self.total, self.pos = memoryview(block), total, 0

    def read(self, n: int) -> bytes:
        n = min(n, self.total - self.pos)
        if n <= 0:
            return b""
        o = self.pos % len(self.block)
        take = min(n, len(self.block) - o)
        self.pos += take
        return bytes(self.block[o:o + take])


def stream_measure(local, gib, steps, warmup=1):
    """The product's streaming API itself (FuzzyAhoCorasick::search_stream, stream.rs:319-335, over
    fac_stream_*): an in-memory reader of `gib` GiB (repeats of C5's 1 GiB block, SURVEY §8(d)
    generator) read in READ_CHUNK pieces, windows of the crate's 256 KiB cut as its WindowReader
    does, each searched without the pre-filter (the crate's search_stream has none), ranked and cut
    at its commit point; every match delivered to the callback. Host bytes in, matches out: H2D
    copies inside the timed region."""
    from fuzzy_aho_corasick import workloads as W
    t0 = time.perf_counter()
    wl = W.config("c5", 1 << 30, seed=5)
    engine = W.builder_for(wl).device(local).build(wl.patterns)
    total = int(gib * (1 << 30))
    setup_s = time.perf_counter() - t0
    hits = [0]

    def on_match(m):
        hits[0] += 1

    for _ in range(warmup):
        engine.search_stream(_RepeatReader(wl.haystack, min(total, 1 << 30)), wl.threshold, on_match)
    hits[0] = 0
    t = time.perf_counter()
    for _ in range(steps):
        n = engine.search_stream(_RepeatReader(wl.haystack, total), wl.threshold, on_match)
        assert n == total
    dt = (time.perf_counter() - t) / steps
    return {"value": total / dt / 1e9, "unit": "Gchars/s", "ms_per_step": dt * 1e3, "steps": steps,
            "stream_bytes": total, "matches_per_step": hits[0] / steps, "setup_s": setup_s,
            "workload": "search_stream (fac_stream_*) over an in-memory reader of C5 data, 256 KiB windows, "
                        "no pre-filter (as the crate's search_stream), edits=1, 1K patterns (10-16), threshold 0.85",
            "timed": "host bytes -> window cuts -> batched H2D + search + per-window ranking -> matches to a callback"}


def run_stream(args, world, rank, local):
    """--config stream: stream_measure on this rank (N > 1: every rank its own stream, weak)."""
    import torch.distributed as dist
    r = stream_measure(local, args.gib if args.gib != 100.0 else 8.0, args.steps, args.warmup)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": r["value"] * world, "unit": "Gchars/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": r["ms_per_step"],
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8 haystack bytes",
                          "data": "synthetic: repeats of C5's 1 GiB block (SURVEY.md §8(d) generator), in host memory",
                          "config": {"workload": r["workload"], "stream_bytes_per_gpu": r["stream_bytes"],
                                     "window_bytes": 256 * 1024, "timed_step": r["timed"]},
                          "diagnostics": {"matches_per_step": r["matches_per_step"], "sources_sha": sources_sha()}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_dry(args, world, rank):
    """Plumbing check without a GPU: the same launch, barrier / max-over-ranks timing and record
    gather to rank 0 (gloo). Default: every rank contributes synthetic records. With --shard: the
    real shard path on a small haystack of the config (--mib, default 1/32 MiB) -- fac_shard_plan
    cuts it, every rank searches only its owned windows of its halo-sliced piece with the CPU oracle
    (test infrastructure standing in for the GPU search), the records are gathered to rank 0, which
    checks the union against the oracle's search of the whole haystack."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from fuzzy_aho_corasick._native import MATCH_DTYPE
    from fuzzy_aho_corasick.distributed import gather_records, gather_rows
    if world > 1:
        dist.init_process_group("gloo")
    parity = None
    if args.shard:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from fuzzy_aho_corasick import _native
        from fuzzy_aho_corasick import workloads as W
        from oracle_harness import OracleEngine, graphemes  # test infrastructure (dry run only)
        nbytes = int((args.mib if args.mib is not None else 1 / 32) * (1 << 20))
        seed = {"c1": 1, "c2": 2, "c3": 3, "c4": 2, "c5": 5}[args.config]
        wl = W.config(args.config, nbytes, seed=seed, hay_seed=seed + 1000)
        if args.config == "c3":  # the dry run's oracle is single-threaded: a slice of the 10K patterns
            wl.patterns = wl.patterns[:500]
        orc = OracleEngine(W.builder_for(wl), wl.patterns)
        mmg = max(len(graphemes(p)) for p in wl.patterns) + wl.edits
        a, b, e, asc, _ = _native.shard_plan(mmg, wl.haystack, world, rank)
        piece = wl.haystack[a:e]
        owned = (b - a) if asc else len(graphemes(piece[: b - a].decode("utf-8")))
        rows = orc.raw_rows(piece, wl.threshold, windows=(0, owned)) if b > a else []
        mine = [(s + a, en + a) + tuple(r) for (s, en, *r) in rows]
    recs = np.zeros(1000 + rank, dtype=MATCH_DTYPE)
    recs["start"] = np.arange(len(recs)) + (rank << 32)
    got = 0
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if args.shard:
            g = gather_rows(mine) if world > 1 else mine
        else:
            g = gather_records(recs, 0) if world > 1 else recs
        got = len(g) if g is not None else 0
    elapsed = time.perf_counter() - t0
    if args.shard and rank == 0:
        parity = sorted(g) == sorted(orc.raw_rows(wl.haystack, wl.threshold))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        cfg = {"workload": "dry-run", "records_gathered_per_step": got, "timed_step": timed_step_desc(args)}
        if args.shard:
            cfg.update(workload=f"dry-run shard: {args.config} slice of {len(wl.haystack)} bytes, {len(wl.patterns)} patterns, "
                                "oracle compute", shard_union_equals_whole=parity)
        print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "Gchars/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": elapsed / max(1, args.steps) * 1e3,
                          "higher_is_better": True, "scaling": "strong" if args.shard else "weak", "vs_baseline": None,
                          "dtype": "none",
                          "data": "dry run: launcher, shard plan and record-gather plumbing, no GPU search",
                          "config": cfg}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(wl, budget_s, threads, min_bytes=0):
    """The CPU restatement (oracle/, test infrastructure) timed on the host cores on bounded prefixes
    of the same haystack: one thread on a prefix sized to ~budget_s (and at least min_bytes), and `threads` threads
    (start-range sharding, like search_stream_parallel, stream.rs:378-429) on SURVEY §8(d)'s prefix
    (C2/C4/C5: 64 MiB, C3: 16 MiB; shortened if it would take more than ~20 s)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_harness import OracleEngine, PreparedText  # test infrastructure, baseline leg only
    from fuzzy_aho_corasick import workloads as W

    orc = OracleEngine(W.builder_for(wl), wl.patterns)

    def prefix(nbytes):
        s = wl.haystack[:nbytes]
        while s and (s[-1] & 0xC0) == 0x80:
            s = s[:-1]
        if s and s[-1] >= 0xC0:
            s = s[:-1]
        return s

    size, rate = 1 << 14, None
    while True:
        pt = PreparedText(orc, prefix(size))
        t = time.perf_counter()
        pt.search(wl.threshold, prefilter=wl.prefilter)
        dt = time.perf_counter() - t
        rate = pt.n / dt
        if (dt * 4 > budget_s and len(pt.data) >= min_bytes) or size >= len(wl.haystack):
            break
        grow = min(8.0, max(2.0, budget_s / max(dt, 1e-3) / 2))
        if dt * 4 > budget_s:  # the budget is spent but the sample is below min_bytes: straight to it
            grow = max(grow, min_bytes / max(1, len(pt.data)) * 1.01)
        size = min(len(wl.haystack), int(size * grow))
    one = {"value": rate / 1e9, "unit": "Gchars/s", "cores": 1, "kind": "port",
           "sample": f"first {len(pt.data)} bytes ({pt.n} graphemes) of the same haystack, {dt:.1f} s, "
                     "oracle/ CPU restatement of the reference algorithm, single thread"}
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    want = CPU_PREFIX_MIB[wl.name] << 20
    est = want / max(1.0, len(pt.data) / dt) / threads  # seconds at linear scaling
    nbytes = int(want if est <= 20 else want * 20 / est)
    big = PreparedText(orc, prefix(nbytes))
    t = time.perf_counter()
    big.search(wl.threshold, prefilter=wl.prefilter, threads=threads)
    dt_all = time.perf_counter() - t
    one["all_cores"] = {"value": big.n / dt_all / 1e9, "unit": "Gchars/s", "cores": threads, "kind": "port",
                        "sample": f"first {len(big.data)} bytes ({big.n} graphemes), {dt_all:.1f} s, {threads} threads, "
                                  "start windows split into contiguous ranges (prefilter: whole-text per thread "
                                  "slices)" if wl.prefilter else
                                  f"first {len(big.data)} bytes ({big.n} graphemes), {dt_all:.1f} s, {threads} threads, "
                                  "start windows split into contiguous ranges"}
    return one


if __name__ == "__main__":
    main()
