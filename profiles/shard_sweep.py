"""Strong-scaling policy sweep (round 6): the C3 haystack's shards of N (fac_shard_plan, staged from HBM
every step like bench.py --shard) timed one after another on one GPU under prefix-cache knob settings
(FAC_DIAGNOSTICS=1 knobs, read at each call), beside the whole haystack under the same setting.

    python profiles/shard_sweep.py [N] [setting ...]   setting: NAME=VAL[;NAME=VAL] or 'default'
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fuzzy-aho-corasick-rs_amd")]
os.environ["FAC_DIAGNOSTICS"] = "1"

import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from fuzzy_aho_corasick import workloads as W  # noqa: E402
from fuzzy_aho_corasick.engine import StagedHaystack  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    settings = sys.argv[2:] or ["default"]
    wl = W.config("c3", 256 << 20, seed=3, hay_seed=1003)
    eng = W.builder_for(wl).device(0).build(wl.patterns)
    stream = torch.cuda.current_stream().cuda_stream
    dev = torch.from_numpy(np.frombuffer(wl.haystack, dtype=np.uint8).copy()).cuda()
    staged = StagedHaystack.from_device(eng, dev.data_ptr(), len(wl.haystack), stream)
    base_env = {k: v for k, v in os.environ.items()}
    for s in settings:
        os.environ.clear()
        os.environ.update(base_env)
        if s != "default":
            for kv in s.split(";"):
                k, v = kv.split("=", 1)
                os.environ[k] = v

        def whole():
            hs = StagedHaystack.from_device(eng, dev.data_ptr(), len(wl.haystack), stream, reuse=staged)
            return len(hs.search_windows_records(wl.threshold, stream=stream)[0])

        whole()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            nrec = whole()
        torch.cuda.synchronize()
        full_ms = (time.perf_counter() - t) / 3 * 1e3
        ms = []
        for r in range(n):
            dt, w, k, b = bench._time_shard(eng, wl.haystack, n, r, 0, stream, 3, wl.threshold)
            ms.append(dt / 3 * 1e3)
        print(json.dumps({"setting": s, "n": n, "n1_ms": round(full_ms, 2), "records": nrec,
                          "max_rank_ms": round(max(ms), 2), "speedup_vs_this_n1": round(full_ms / max(ms), 2),
                          "rank_ms": [round(x, 2) for x in ms]}), flush=True)


if __name__ == "__main__":
    main()
