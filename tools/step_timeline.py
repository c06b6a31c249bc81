"""Kernel timeline of the last steps of a rocprofv3 kernel trace: every kernel's start offset, its
duration and the idle gap before it, per step (a step starts at each launch of `first_kernel`).
usage: python tools/step_timeline.py <kernel_trace.csv> <first_kernel_substring> [steps]"""
import csv
import sys

path, first = sys.argv[1], sys.argv[2]
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = []
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("eon::", "").split("(")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.replace("void ", "")))
rows.sort()
starts = [i for i, r in enumerate(rows) if first in r[2]]
for k in range(max(0, len(starts) - nsteps), len(starts)):
    i0 = starts[k]
    i1 = starts[k + 1] if k + 1 < len(starts) else len(rows)
    t0, busy_end, busy = rows[i0][0], rows[i0][0], 0.0
    print(f"step {k}: {i1 - i0} kernels")
    for s, e, n in rows[i0:i1]:
        gap = max(0, s - busy_end)
        print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap / 1e3:7.1f}  {n[:70]}")
        busy += max(0, e - max(s, busy_end))
        busy_end = max(busy_end, e)
    print(f"  span {(busy_end - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
