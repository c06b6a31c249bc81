#!/usr/bin/env python3
"""Exposure of one steady-state prove period of a rocprofv3 kernel trace (tools/gpu_trace.sh):
the period between the 2nd and 3rd k_p2_quotient launches (one prove), the time k_piece_sum* is
active, and the time each other kernel runs while no piece sum does.

usage: python tools/exposure.py <kernel_trace.csv>
"""
import collections
import csv
import sys


def short_name(kernel: str) -> str:
    return (kernel.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            .replace("eon::", ""))


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["n"] = short_name(r["Kernel_Name"])
    quot = sorted((r for r in rows if "k_p2_quotient" in r["n"]), key=lambda r: r["s"])
    if len(quot) < 3:
        raise SystemExit("need a trace of at least three proves (bench.py --steps 1 --warmup 1)")
    a, b = quot[1]["s"], quot[2]["s"]
    # clip every launch to the period [a, b)
    win = [(max(r["s"], a), min(r["e"], b), r["n"]) for r in rows if r["e"] > a and r["s"] < b]
    events = sorted([(s, 1, n) for s, _, n in win] + [(e, -1, n) for _, e, n in win])
    active = collections.Counter()
    last, idle, piece = a, 0.0, 0.0
    exposed = collections.defaultdict(float)
    for t, d, n in events:
        dt = (t - last) / 1e6
        if dt > 0:
            names = [k for k, v in active.items() if v > 0]
            if not names:
                idle += dt
            elif any("k_piece_sum" in k for k in names):
                piece += dt
            else:
                for k in names:
                    exposed[k] += dt / len(names)
        active[n] += d
        last = t
    print(f"period {(b - a) / 1e6:.1f} ms: piece active {piece:.1f}, idle {idle:.1f}, "
          f"exposed {sum(exposed.values()):.1f}")
    for k, v in sorted(exposed.items(), key=lambda kv: -kv[1])[:25]:
        print(f"  {k[:45]:45s} {v:7.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
