"""Build profiles/traffic.json from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of
`bench.py --config CFG --mib MIB`. Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM /
rocprofv3 section): on gfx950 FETCH_SIZE reports half of the fetched bytes -> x2 (an upper bound
for non-streaming reads); WRITE_SIZE as reported. Both counters are in kB, per kernel launch.

usage: python profiles/make_traffic.py CFG MIB FETCH.csv WRITE.csv [TARGET_MIB [KERNEL_SUBSTR]]

KERNEL_SUBSTR may list several kernels separated by commas (e.g.
"bfs_window_kernel,lane_window_kernel"): their per-launch averages are summed, matching bench.py's
roofline, which times the wave kernel and the lane-serial kernel together (one launch each per step).

TARGET_MIB (optional) scales a measurement taken on a smaller launch linearly to the bench launch
(windows are i.i.d.; checked: 8, 32 and 256 MiB C3 launches give the same bytes per grapheme).
"""
import csv
import json
import os
import sys


def per_launch_kb(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {kernel} rows in {path}")
    return sum(vals) / len(vals), next(r["Kernel_Name"] for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"])


def main():
    cfg, mib, fetch_csv, write_csv = sys.argv[1], float(sys.argv[2]), sys.argv[3], sys.argv[4]
    target = float(sys.argv[5]) if len(sys.argv) > 5 else mib
    kernels = (sys.argv[6] if len(sys.argv) > 6 else "bfs_window_kernel,lane_window_kernel").split(",")
    fetch_kb = write_kb = 0.0
    names = []
    for kernel in kernels:
        f, name = per_launch_kb(fetch_csv, kernel)
        w, _ = per_launch_kb(write_csv, kernel)
        fetch_kb += f
        write_kb += w
        names.append(name)
    name = " + ".join(names)
    scale = target / mib
    out = {
        "config": cfg,
        "mib": target,
        "measured_at_mib": mib,
        "scale": scale,
        "kernel": name,
        "FETCH_SIZE_kB_per_launch": fetch_kb,
        "WRITE_SIZE_kB_per_launch": write_kb,
        "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md HBM/rocprofv3 section; upper bound for "
                      "non-streaming reads); WRITE_SIZE as reported; kB = 1024 B",
        "hbm_bytes_per_launch": (2.0 * fetch_kb + write_kb) * 1024.0 * scale,
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                  f"python3 bench.py --config {cfg} --mib {mib:g} --steps 2 --warmup 0 --no-cpu-baseline",
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "traffic.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
