"""Gaps in piece-sum activity of the last `window_ms` of a rocprofv3 kernel trace, with the kernels
active in each gap: python tools/gaps.py <kernel_trace.csv> [window_ms] [min_gap_ms]"""
import collections
import csv
import sys

path = sys.argv[1]
win = float(sys.argv[2]) if len(sys.argv) > 2 else 900
min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
rows = list(csv.DictReader(open(path)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("eon::", "").split("(")[0].replace("void ", "")
    r["n"] = "rocprim" if ("rocprim" in n or "trampoline" in n) else n
end = max(r["e"] for r in rows)
t0 = end - win * 1e6
rows = sorted([r for r in rows if r["s"] >= t0], key=lambda r: r["s"])
ps = sorted((r["s"], r["e"]) for r in rows if "piece_sum" in r["n"])
merged = []
for s, e in ps:
    if merged and s <= merged[-1][1]:
        merged[-1][1] = max(merged[-1][1], e)
    else:
        merged.append([s, e])
prev, total = t0, 0.0
for s, e in merged + [[end, end]]:
    if s - prev > min_gap * 1e6:
        ks = collections.Counter()
        for r in rows:
            a, b = max(r["s"], prev), min(r["e"], s)
            if b > a:
                ks[r["n"][:28]] += (b - a) / 1e6
        total += (s - prev) / 1e6
        print(f"gap @{(prev - t0) / 1e6:7.1f} len {(s - prev) / 1e6:6.2f} ms:",
              ", ".join(f"{k} {v:.1f}" for k, v in ks.most_common(6)))
    prev = max(prev, e)
print(f"piece-sum active {sum(e - s for s, e in merged) / 1e6:.1f} ms, gaps {total:.1f} ms")
