"""Exposure analysis of a rocprofv3 kernel trace: for the last `window_ms` of the trace, the time
during which a given critical kernel is NOT running, attributed to the kernels that are.

usage: python tools/timeline.py <kernel_trace.csv> [critical_kernel] [window_ms]
"""
import collections
import csv
import sys

path = sys.argv[1]
crit = sys.argv[2] if len(sys.argv) > 2 else "k_piece_sum"
win_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = list(csv.DictReader(open(path)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[-40:]
end = max(r["e"] for r in rows)
t0 = end - win_ms * 1e6 if win_ms else min(r["s"] for r in rows)
win = [r for r in rows if r["s"] >= t0]
ev = sorted([(r["s"], 1, r["n"]) for r in win] + [(r["e"], -1, r["n"]) for r in win])
active = collections.Counter()
last, idle, crit_on = t0, 0.0, 0.0
exposed = collections.defaultdict(float)
for t, d, n in ev:
    dt = (t - last) / 1e6
    if dt > 0:
        names = [k for k, v in active.items() if v > 0]
        if not names:
            idle += dt
        elif any(crit in k for k in names):
            crit_on += dt
        else:
            for k in names:
                exposed[k] += dt / len(names)
    active[n] += d
    last = t
print(f"window {(end - t0) / 1e6:.1f} ms: {crit} active {crit_on:.1f} ms, idle {idle:.1f} ms, "
      f"exposed {sum(exposed.values()):.1f} ms")
for k, v in sorted(exposed.items(), key=lambda kv: -kv[1])[:15]:
    print(f"  {k:42s} {v:8.1f}")
