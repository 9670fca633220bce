"""Build profiles/traffic.json from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of
`bench.py --config CFG --mib MIB --steps STEPS --warmup 0 --no-cpu-baseline`.

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): on gfx950
FETCH_SIZE reports half of the fetched bytes of a wide streaming read -> x2 (an upper bound for
non-streaming reads); WRITE_SIZE as reported. Both counters are in kB, per kernel dispatch.

Every kernel of the timed step is summed (the device staging of search_raw -- UTF-8 check,
segmentation, folding -- then prefix-cache counts / numbering / builds / publishes, lookups, the
lane-serial and the wave kernel, buffer fills; bitap + runs + re-search for the pre-filter) — the
same set bench.py's whole-step roofline times. The staging kernels also run once before the timed
steps (bench.py stages the haystack to size its windows), so theirs are averaged per dispatch; C5
stages its block once and searches stream windows: there they are excluded. The result is stamped
with bench.sources_sha() of the csrc/ tree it was measured on and written to
profiles/traffic_<CFG>.json; bench.py refuses one whose stamp differs from the running sources.

usage: python profiles/make_traffic.py CFG MIB STEPS FETCH.csv WRITE.csv [SOURCES_SHA]
(SOURCES_SHA: the bench line's diagnostics.sources_sha of the measured run; default: this tree's)
"""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

# search_raw's device staging (one dispatch each per staging; bmp_tables_kernel once per process)
STAGING = ("ascii_or_kernel", "seg_tile_kernel", "seg_hard_kernel", "recount_kernel", "unit_scan_kernel",
           "write_tile_kernel", "bmp_tables_kernel", "transcode_ascii_kernel")


def is_staging(name):
    base = name.replace("(anonymous namespace)", "").split("(")[0].split("<")[0].split("::")[-1]
    return "rocprim" in name or base.startswith(STAGING)


def per_kernel_kb(path, cfg, steps):
    """kB per step by kernel: totals / steps; staging kernels: per dispatch (C5: excluded)."""
    tot, disp = {}, {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        tot[name] = tot.get(name, 0.0) + float(r["Counter_Value"])
        disp[name] = disp.get(name, 0) + 1
    if not tot:
        raise SystemExit(f"no kernel rows in {path}")
    out = {}
    for name, v in tot.items():
        if is_staging(name):
            if cfg == "c5" or "bmp_tables" in name:
                continue
            out[name] = v / disp[name]
        else:
            out[name] = v / steps
    return out


def short(name):
    name = name.replace("fac::(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def main():
    from bench import sources_sha
    cfg, mib, steps, fetch_csv, write_csv = sys.argv[1], float(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    fetch = per_kernel_kb(fetch_csv, cfg, steps)
    write = per_kernel_kb(write_csv, cfg, steps)
    names = sorted(set(fetch) | set(write), key=lambda n: -(2 * fetch.get(n, 0) + write.get(n, 0)))
    per_kernel = {short(n): {"FETCH_SIZE_kB_per_step": fetch.get(n, 0.0),
                             "WRITE_SIZE_kB_per_step": write.get(n, 0.0),
                             "hbm_bytes_per_step": (2 * fetch.get(n, 0.0) + write.get(n, 0.0)) * 1024.0}
                  for n in names}
    fetch_kb = sum(fetch.values())
    write_kb = sum(write.values())
    out = {
        "config": cfg,
        "mib": mib,
        "steps_measured": steps,
        "sources_sha": sys.argv[6] if len(sys.argv) > 6 else sources_sha(),
        "kernel": "every kernel of the step" + (" (the block's one-off staging excluded)" if cfg == "c5" else
                                                 " (device staging of search_raw included)"),
        "FETCH_SIZE_kB_per_step": fetch_kb,
        "WRITE_SIZE_kB_per_step": write_kb,
        "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md HBM/rocprofv3 section; upper bound for "
                      "non-streaming reads); WRITE_SIZE as reported; kB = 1024 B",
        "hbm_bytes_per_step": (2.0 * fetch_kb + write_kb) * 1024.0,
        "per_kernel": per_kernel,
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                  f"python3 bench.py --config {cfg} --mib {mib:g} --steps {steps} --warmup 0 --no-cpu-baseline",
    }
    json.dump(out, open(os.path.join(HERE, f"traffic_{cfg}.json"), "w"), indent=1)
    print(json.dumps(out)[:2000])


if __name__ == "__main__":
    main()
