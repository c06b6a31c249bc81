#!/usr/bin/env python3
"""Timeline of one steady-state prove of a rocprofv3 kernel trace (tools/gpu_trace.sh): the
period between the 2nd and 3rd k_p2_quotient launches, cut into phases where the set of running
kernels (short names) is unchanged; consecutive phases with the same dominant kernel are merged,
and device-idle stretches are listed as "IDLE".  Shows where the device waits on the host (the
Fiat-Shamir transcript, exchanges) in a prove.

usage: python tools/phases.py <kernel_trace.csv> [min_ms]
"""
import collections
import csv
import sys


def short(kernel: str) -> str:
    n = kernel.replace("(anonymous namespace)::", "").replace("eon::", "").split("(")[0].replace("void ", "")
    return n.split("<")[0]


def main(path: str, min_ms: float) -> None:
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"], r["n"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])
    quot = sorted((r for r in rows if r["n"] == "k_p2_quotient"), key=lambda r: r["s"])
    if len(quot) < 3:
        raise SystemExit("need a trace of at least three proves (bench.py --steps 1 --warmup 1)")
    a, b = quot[1]["s"], quot[2]["s"]
    win = [(max(r["s"], a), min(r["e"], b), r["n"]) for r in rows if r["e"] > a and r["s"] < b]
    events = sorted([(s, 1, n) for s, _, n in win] + [(e, -1, n) for _, e, n in win])
    active = collections.Counter()
    last = a
    phases = []  # (start, duration, dominant label)
    for t, d, n in events:
        dt = (t - last) / 1e6
        if dt > 0:
            names = sorted(k for k, v in active.items() if v > 0)
            label = "IDLE" if not names else ("k_piece_sum" if "k_piece_sum29" in names else names[0])
            if phases and phases[-1][2] == label:
                phases[-1][1] += dt
            else:
                phases.append([(last - a) / 1e6, dt, label])
        active[n] += d
        last = t
    print(f"prove period {(b - a) / 1e6:.1f} ms (t = 0 at k_p2_quotient)")
    totals = collections.Counter()
    for s, dt, label in phases:
        totals[label] += dt
        if dt >= min_ms:
            print(f"  @{s:8.2f} {dt:7.2f} ms  {label}")
    print("totals:", ", ".join(f"{k} {v:.1f}" for k, v in totals.most_common(12)))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.3)
