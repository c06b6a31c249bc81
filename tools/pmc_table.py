"""Per-kernel PMC table from several rocprofv3 --pmc passes (each its own run directory): the
per-dispatch mean of every counter for the dispatches of one kernel, plus the derived ratios used
in DESIGN.md §4 (stall breakdown, L2 hit rate, corrected HBM bytes).

usage: python tools/pmc_table.py <kernel-substring> <out.json> <pass_dir> [<pass_dir> ...]
Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles;
FETCH_SIZE / WRITE_SIZE are KB, FETCH_SIZE halves wide streaming reads on gfx950 (x2).
"""

import csv
import glob
import json
import sys


def collect(d, kernel):
    per = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r.get("Kernel_Name", ""):
                continue
            c = r["Counter_Name"]
            per.setdefault(c, {})
            k = r.get("Dispatch_Id")
            per[c][k] = per[c].get(k, 0.0) + float(r["Counter_Value"])
    return {c: (sum(v.values()) / len(v), len(v)) for c, v in per.items()}


def main():
    kernel, out = sys.argv[1], sys.argv[2]
    tab, disp = {}, {}
    for d in sys.argv[3:]:
        for c, (mean, n) in collect(d, kernel).items():
            tab[c] = mean
            disp[c] = n
    if not tab:
        raise SystemExit(f"no counter rows for {kernel}")
    g = tab.get
    der = {}
    if g("SQ_WAVE_CYCLES"):
        wc = g("SQ_WAVE_CYCLES")
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA"):
            if g(c) is not None:
                der[c + "/WAVE_CYCLES"] = round(g(c) / wc, 4)
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
        der["L2 hit rate"] = round(g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")), 4)
    if g("FETCH_SIZE") is not None:
        der["FETCH bytes x2 (GB per launch)"] = round(2 * g("FETCH_SIZE") * 1024 / 1e9, 3)
    if g("WRITE_SIZE") is not None:
        der["WRITE bytes (GB per launch)"] = round(g("WRITE_SIZE") * 1024 / 1e9, 3)
    if g("TA_BUSY_avr") is not None and g("TA_DATA_STALLED_BY_TC_CYCLES_sum") is not None:
        der["TA data stalled by TC / TA busy (sum over TAs)"] = g("TA_DATA_STALLED_BY_TC_CYCLES_sum")
    res = {"kernel": kernel, "dispatches": disp, "per_dispatch_mean": tab, "derived": der}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
