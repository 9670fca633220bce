"""One C3 step's kernels on their queues (start/end/duration ms from the step's first kernel), from a
rocprofv3 --kernel-trace --output-format csv run: python profiles/step_timeline.py run_kernel_trace.csv
A step starts at its device staging (ascii_or_kernel), or, for pre-staged runs, at a level-1 count
(rc_count_kernel) that follows a search kernel; the last complete step is printed."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'] for r in rows]
def prev_kernel(i):  # the last kernel before i that is not a runtime fill / copy
    for j in range(i - 1, -1, -1):
        if '__amd_rocclr' not in names[j]:
            return names[j]
    return ''


starts = [i for i, n in enumerate(names) if 'ascii_or_kernel' in n]
if len(starts) < 2:  # a shard staged in Unicode mode (no is_ascii pass): its segmentation starts the step
    starts = [i for i, n in enumerate(names) if 'seg_tile_kernel' in n]
if len(starts) < 2:
    starts = [i for i, n in enumerate(names) if 'rc_count_kernel' in n and 'window_kernel' in prev_kernel(i)]
a, b = (starts[-2], starts[-1]) if len(starts) >= 2 else (starts[-1], len(rows))
seg = rows[a:b]
t0 = int(seg[0]['Start_Timestamp'])
for r in seg:
    n = r['Kernel_Name'].replace('fac::(anonymous namespace)::', '').replace('void ', '')
    n = re.sub(r'\(.*', '', n)[:40]
    if 'copy' in n:
        continue
    s = (int(r['Start_Timestamp']) - t0) / 1e6
    e = (int(r['End_Timestamp']) - t0) / 1e6
    if 'fill' in n and e - s < 0.1:
        continue
    print(f"{n:40s} q{r['Queue_Id'][-1]} {s:8.2f} {e:8.2f} {e - s:7.2f}")
