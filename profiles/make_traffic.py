"""Build profiles/traffic.json from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of
`bench.py --config CFG --mib MIB --steps STEPS --warmup 0 --no-cpu-baseline`.

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): on gfx950
FETCH_SIZE reports half of the fetched bytes of a wide streaming read -> x2 (an upper bound for
non-streaming reads); WRITE_SIZE as reported. Both counters are in kB, per kernel dispatch.

Every kernel of the timed step is summed (prefix-cache counts / numbering / builds / publishes,
lookups, the lane-serial and the wave kernel, buffer fills; bitap + runs + re-search for the
pre-filter) — the same set bench.py's whole-step roofline times. The one-off staging kernels
(segmentation, compaction, fold, transcode), which run once before the timed steps, are excluded.
The result is stamped with bench.sources_sha() of the csrc/ tree it was measured on; bench.py
refuses a traffic.json whose stamp differs from the running sources.

usage: python profiles/make_traffic.py CFG MIB STEPS FETCH.csv WRITE.csv [SOURCES_SHA]
(SOURCES_SHA: the bench line's diagnostics.sources_sha of the measured run; default: this tree's)
"""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

# kernels that run once per staged haystack (before the timed loop), not per step
STAGING = ("validate_kernel", "seg_chunk_kernel", "seg_hard_kernel", "unit_count_kernel", "unit_scan_kernel",
           "unit_write_kernel", "fold_kernel", "transcode_ascii_kernel")


def is_staging(name):
    base = name.replace("(anonymous namespace)", "").split("(")[0].split("<")[0].split("::")[-1]
    return "rocprim" in name or base.startswith(STAGING)


def per_kernel_kb(path):
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if is_staging(name):
            continue
        out[name] = out.get(name, 0.0) + float(r["Counter_Value"])
    if not out:
        raise SystemExit(f"no kernel rows in {path}")
    return out


def short(name):
    name = name.replace("fac::(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def main():
    from bench import sources_sha
    cfg, mib, steps, fetch_csv, write_csv = sys.argv[1], float(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    fetch = per_kernel_kb(fetch_csv)
    write = per_kernel_kb(write_csv)
    names = sorted(set(fetch) | set(write), key=lambda n: -(2 * fetch.get(n, 0) + write.get(n, 0)))
    per_kernel = {short(n): {"FETCH_SIZE_kB_per_step": fetch.get(n, 0.0) / steps,
                             "WRITE_SIZE_kB_per_step": write.get(n, 0.0) / steps,
                             "hbm_bytes_per_step": (2 * fetch.get(n, 0.0) + write.get(n, 0.0)) * 1024.0 / steps}
                  for n in names}
    fetch_kb = sum(fetch.values()) / steps
    write_kb = sum(write.values()) / steps
    out = {
        "config": cfg,
        "mib": mib,
        "steps_measured": steps,
        "sources_sha": sys.argv[6] if len(sys.argv) > 6 else sources_sha(),
        "kernel": "every kernel of the step (staging excluded)",
        "FETCH_SIZE_kB_per_step": fetch_kb,
        "WRITE_SIZE_kB_per_step": write_kb,
        "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md HBM/rocprofv3 section; upper bound for "
                      "non-streaming reads); WRITE_SIZE as reported; kB = 1024 B",
        "hbm_bytes_per_step": (2.0 * fetch_kb + write_kb) * 1024.0,
        "per_kernel": per_kernel,
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                  f"python3 bench.py --config {cfg} --mib {mib:g} --steps {steps} --warmup 0 --no-cpu-baseline",
    }
    json.dump(out, open(os.path.join(HERE, "traffic.json"), "w"), indent=1)
    print(json.dumps(out)[:2000])


if __name__ == "__main__":
    main()
