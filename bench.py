#!/usr/bin/env python3
"""bench.py — haystack Gchars/s of the MI355X fuzzy Aho–Corasick engine (BASELINE.json metric).

Workload (default): BASELINE.json configs[2] — edits=2, beam_width=64, 10K patterns,
case-insensitive Unicode graphemes, one MI355X per rank — on seeded synthetic data
(fuzzy_aho_corasick/workloads.py, SURVEY.md §8(d) generator). A "step" is one pass of the hot path
(FuzzyAhoCorasick::search_raw over every start window of the rank's staged haystack, device
resident) plus, for N > 1, the RCCL gather of the 32-byte Match records to rank 0. Weak scaling:
each rank owns its own haystack of the same size (the C4 batch layout).

    python bench.py [--gpus N --steps K --warmup W --config c3 --mib 16]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "fuzzy-aho-corasick-rs_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
DEFAULT_MIB = {"c1": 1, "c2": 1024, "c3": 256, "c4": 128, "c5": 256}  # C2: the 1 GB of BASELINE configs[1]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=["c1", "c2", "c3", "c4", "c5"])
    ap.add_argument("--mib", type=float, default=None, help="haystack MiB per rank per step")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")  # RCCL on ROCm
    torch.cuda.set_device(local)

    from fuzzy_aho_corasick import workloads as W
    from fuzzy_aho_corasick.engine import StagedHaystack

    mib = args.mib if args.mib is not None else DEFAULT_MIB[args.config]
    nbytes = int(mib * (1 << 20))
    base_seed = {"c1": 1, "c2": 2, "c3": 3, "c4": 40, "c5": 5}[args.config]
    # weak scaling: every rank builds the same engine and owns a different haystack of equal size
    wl = W.config(args.config, nbytes, seed=base_seed, hay_seed=base_seed + 1000 + 101 * rank)
    engine = W.builder_for(wl).device(local).build(wl.patterns)
    staged = StagedHaystack(engine, wl.haystack)
    graphemes = staged.graphemes
    stream = torch.cuda.current_stream().cuda_stream

    from fuzzy_aho_corasick.distributed import gather_records
    dev = torch.device("cuda", local)

    def step():  # records stay 32-byte structs (MATCH_DTYPE), as search_raw's Vec<OwnedMatch>
        if wl.prefilter:  # C5: bitap pre-filter + re-search of the merged windows (prefilter.rs:304-374)
            rows, st = staged.search_prefiltered_records(wl.threshold, stream=stream)
        else:
            rows, st = staged.search_windows_records(wl.threshold, stream=stream)
        if world > 1:  # gather the 32 B Match records to rank 0 over RCCL (xGMI)
            gather_records(rows, dev)
        return rows, st

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms, launches, matches, popped, prefilter_ms, cache_ms, cached = 0.0, 0, 0, 0, 0.0, 0.0, 0
    lane_ms, lane_windows = 0.0, 0
    for _ in range(args.steps):
        rows, st = step()
        prefilter_ms += st.prefilter_ms
        cache_ms += st.cache_ms
        cached += st.states_cached
        kernel_ms += st.kernel_ms
        lane_ms += st.lane_ms
        lane_windows += st.lane_windows
        launches += st.kernel_launches
        matches += len(rows)
        popped += st.states_popped
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        g = torch.tensor([graphemes], device="cuda", dtype=torch.int64)
        dist.all_reduce(g)
        total_graphemes = int(g.item()) * args.steps
    else:
        total_graphemes = graphemes * args.steps

    value = total_graphemes / elapsed / 1e9
    # the search proper: the wave kernel's launches plus the lane-serial kernel that takes the small
    # resumed windows off it (one launch per step when the prefix cache is on)
    avg_kernel_s = (kernel_ms + lane_ms) / max(1, launches) / 1e3
    bytes_per_launch = len(wl.haystack) + 32 * (matches / max(1, args.steps))
    kernel_name = "bfs_window_kernel + lane_window_kernel" if lane_ms > 0 else "bfs_window_kernel"
    if prefilter_ms > kernel_ms:  # C5: the bitap scan dominates; 1 B/char in
        kernel_name = "bitap_kernel (+transcode, runs)"
        avg_kernel_s = prefilter_ms / max(1, args.steps) / 1e3
        bytes_per_launch = len(wl.haystack)
    achieved = bytes_per_launch / avg_kernel_s / 1e9 if avg_kernel_s > 0 else 0.0
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("config") == args.config and abs(tj.get("mib", -1) - mib) < 1e-6:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(wl, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "haystack Gchars/s at edits<=2, 10K patterns; 1/2/4/8 MI355X",
            "value": value,
            "unit": "Gchars/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 code points / f32 penalties",
            "data": "synthetic (seeded xorshift generator, SURVEY.md §8(d)); random words + planted fuzzy patterns",
            "config": {
                "workload": f"{args.config}: " + {
                    "c1": "exact, 16 ASCII patterns",
                    "c2": "edits=1, 1K ASCII patterns",
                    "c3": "edits=2, beam_width=64, 10K patterns, case-insensitive Unicode graphemes",
                    "c4": "edits=1, 1K ASCII patterns, one haystack per GPU",
                    "c5": "edits=1, 1K patterns (10-16), threshold 0.85, bitap prefilter",
                }[args.config],
                "patterns": len(wl.patterns),
                "haystack_bytes_per_gpu": len(wl.haystack),
                "graphemes_per_gpu": graphemes,
                "threshold": wl.threshold,
                "parallelism": f"dp{world} (weak: one haystack per GPU, RCCL gather of Match records)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": kernel_name,
                "avg_kernel_ms": avg_kernel_s * 1e3,
                "algorithmic_bytes_per_launch": bytes_per_launch,
            },
            "cpu_baseline": cpu,
            "diagnostics": {
                "matches_per_step": matches / max(1, args.steps),
                "states_popped_per_step": popped / max(1, args.steps),
                "states_per_second": popped / max(1e-9, kernel_ms / 1e3),
                "kernel_launches": launches,
                "search_kernel_ms_per_step": kernel_ms / max(1, args.steps),
                "lane_kernel_ms_per_step": lane_ms / max(1, args.steps),
                "lane_windows_per_step": lane_windows / max(1, args.steps),
                "prefilter_ms_per_step": prefilter_ms / max(1, args.steps),
                "prefix_cache_ms_per_step": cache_ms / max(1, args.steps),
                "states_from_prefix_cache_per_step": cached / max(1, args.steps),
            },
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(wl, budget_s):
    """CPU restatement (oracle/, single thread) timed on a bounded prefix of the same workload."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_harness import OracleEngine  # test infrastructure, baseline leg only
    from fuzzy_aho_corasick import workloads as W

    orc = OracleEngine(W.builder_for(wl), wl.patterns)
    size = 1 << 14
    while True:
        sample = wl.haystack[:size]
        while sample and (sample[-1] & 0xC0) == 0x80:
            sample = sample[:-1]
        if sample and sample[-1] >= 0xC0:
            sample = sample[:-1]
        text = sample.decode("utf-8")
        from oracle_harness import graphemes as segs
        n_g = len(sample) if sample.isascii() else len(segs(text))
        t = time.perf_counter()
        orc.raw_rows(sample, wl.threshold, prefilter=wl.prefilter)
        dt = time.perf_counter() - t
        if dt * 4 > budget_s or size >= len(wl.haystack):
            break
        size = min(len(wl.haystack), int(size * min(8.0, max(2.0, budget_s / max(dt, 1e-3) / 2))))
    return {"value": n_g / dt / 1e9, "unit": "Gchars/s", "cores": 1, "kind": "port",
            "sample": f"first {len(sample)} bytes ({n_g} graphemes) of the same haystack, {dt:.1f} s, "
                      f"oracle/ CPU restatement, single thread"}


if __name__ == "__main__":
    main()
