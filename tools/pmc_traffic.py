"""Turns two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM traffic of one
kernel.  Counters are in KB (x1024).  `bytes_per_launch` is the RAW sum FETCH_SIZE + WRITE_SIZE:
the guide's x2 on FETCH_SIZE is calibrated for wide coalesced streaming reads (16 B per lane),
and the MSM piece sums' reads are scattered 16/64-byte table gathers, for which it over-counts
(DESIGN.md section 4); the x2 figure is kept beside it as `bytes_per_launch_x2_streaming`, an
upper bound.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <workload | bench.json> <out.json>
(a bench.json argument supplies config.workload from that bench line)
"""

import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and kernel in r.get("Kernel_Name", ""):
                key = r.get("Dispatch_Id")
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return vals


def main():
    fdir, wdir, kernel, workload, out = sys.argv[1:6]
    if workload.endswith(".json"):
        txt = open(workload).read()
        workload = json.loads(txt[txt.index("{"):])["config"]["workload"]
    fetch = per_dispatch(fdir, "FETCH_SIZE", kernel)
    write = per_dispatch(wdir, "WRITE_SIZE", kernel)
    if not fetch or not write:
        raise SystemExit(f"no counter rows for {kernel}: fetch={len(fetch)} write={len(write)}")
    f_kb = sum(fetch.values()) / len(fetch)
    w_kb = sum(write.values()) / len(write)
    res = {
        "kernel": kernel,
        "workload": workload,
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "fetch_size_kb_per_launch": f_kb,
        "write_size_kb_per_launch": w_kb,
        "bytes_per_launch": int(f_kb * 1024 + w_kb * 1024),
        "bytes_per_launch_x2_streaming": int(2 * f_kb * 1024 + w_kb * 1024),
        "correction": "bytes = (FETCH_SIZE + WRITE_SIZE) * 1024, raw: the x2 streaming-read correction of "
                      "FETCH_SIZE does not apply to scattered 16/64-B gathers (bytes_per_launch_x2_streaming "
                      "applies it, an upper bound)",
        "commit": os.environ.get("EON_COMMIT", "unknown"),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
