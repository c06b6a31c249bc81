"""Instruction mix of a kernel's basic blocks in a gfx950 assembly listing.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude --cuda-device-only -S \
        plonky3_eon_amd/csrc/msm.hip -o /tmp/msm.s
    python tools/isa_count.py /tmp/msm.s k_piece_sum29 [--blocks N] [--costs profiles/r06/s4/ubench_isa2.txt]

Prints the N largest basic blocks of the first function whose symbol contains the substring,
each with its VALU / SALU / memory / s_nop counts and the VALU mnemonic histogram of the largest
one -- the per-addition instruction count of a straight-line loop body.
With --costs (tools/ubench_isa2 output: SIMD cycles per wave-instruction at 4 waves per SIMD) every
block also gets its issue cycles (VOP3 ~4.8, VOP2 ~2.8, s_nop ~1 -- the pads are hidden by the
other waves -- unlisted VALU at the VOP3 cost).
"""

from __future__ import annotations

import argparse
import collections
import re


def blocks(lines):
    cur, name = [], "entry"
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("//"):
            continue
        if re.match(r"^[.\w$]+:", s):
            if cur:
                yield name, cur
            name, cur = s.split(":")[0], []
            continue
        if s.startswith("."):
            continue
        op = s.split()[0]
        cur.append(op)
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op == "s_endpgm":
            yield name, cur
            name, cur = name + "+", []
    if cur:
        yield name, cur


def classify(op: str) -> str:
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


VOP2 = ("v_add_u32_e32", "v_sub_u32_e32", "v_and_b32_e32", "v_ashrrev_i32_e32", "v_lshrrev_b32_e32",
        "v_lshlrev_b32_e32", "v_mov_b32_e32", "v_or_b32_e32", "v_xor_b32_e32", "v_cndmask_b32_e32",
        "v_subrev_u32_e32")


def load_costs(path):
    """op -> cycles at 4 waves per SIMD from tools/ubench_isa2 JSON lines."""
    import json

    c = {}
    for ln in open(path):
        ln = ln.strip()
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        if d["waves_per_simd"] == 4 and "+" not in d["op"]:
            c[d["op"].split()[0]] = d["simd_cycles_per_wave_instr"]
    return c


def cost_of(op, costs):
    base = op.split("_e32")[0].split("_e64")[0].split("_sdwa")[0]
    if op.startswith("s_nop"):
        return 1.0
    if not op.startswith("v_"):
        return 0.0
    if base in costs and "cndmask" not in base:
        return costs[base]
    if op in VOP2 or op.endswith("_e32"):
        return costs.get("v_sub_u32", 2.8)
    return costs.get("v_mad_u64_u32", 4.8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--costs", default=None)
    a = ap.parse_args()
    costs = load_costs(a.costs) if a.costs else None
    text = open(a.asm).read().splitlines()
    start = next(i for i, ln in enumerate(text) if re.match(r"^_Z\w*" + re.escape(a.kernel) + r"\w*:", ln))
    end = next(i for i in range(start, len(text)) if text[i].startswith(".Lfunc_end"))
    bbs = sorted(blocks(text[start:end]), key=lambda b: -len(b[1]))[: a.blocks]
    print(f"{text[start].split(':')[0]}: {end - start} lines")
    for name, ops in bbs:
        c = collections.Counter(classify(o) for o in ops)
        cyc = "  issue %.0f cyc" % sum(cost_of(o, costs) for o in ops) if costs else ""
        print(f"  {name:24s} {len(ops):6d} instr  " + "  ".join(f"{k} {v}" for k, v in sorted(c.items())) + cyc)
    name, ops = bbs[0]
    hist = collections.Counter(o for o in ops if o.startswith("v_"))
    print(f"VALU mnemonics of {name}:")
    for op, n in hist.most_common():
        print(f"  {op:28s} {n}")


if __name__ == "__main__":
    main()
