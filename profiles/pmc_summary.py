"""Per-kernel sums of rocprofv3 --pmc counter_collection CSVs (one row per dispatch and counter):
python profiles/pmc_summary.py pmc1.csv [pmc2.csv ...]"""
import csv
import re
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("fac::(anonymous namespace)::", "").replace("void ", "")
        n = re.sub(r"\(.*", "", n)[:40]
        if "rocprim" in n:
            n = "rocprim"
        tot[n][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[n].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
keys = sorted({c for d in tot.values() for c in d})
for n, d in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    print(f"{n} ({len(calls[n])} dispatches)")
    for c in keys:
        if c in d:
            print(f"    {c:24s} {d[c]:.4g}")
    w = d.get("SQ_WAVE_CYCLES", 0)
    if w:
        print("    wait %.2f  issue-stall %.2f  active %.2f (of wave cycles)" % (
            d.get("SQ_WAIT_ANY", 0) / w, d.get("SQ_WAIT_INST_ANY", 0) / w, d.get("SQ_ACTIVE_INST_ANY", 0) / w))
    if d.get("TCC_HIT_sum", 0) + d.get("TCC_MISS_sum", 0):
        print("    L2 hit rate %.3f" % (d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])))
