#!/usr/bin/env python3
"""Summarise tools/pmc_c3.sh for the C3 cluster kernel (wmvc_cluster_lc_kernel<5>, the
2^24-slot launches of tools/bench_c3.py): VALU wave-instructions per slot, the VALU
issue utilisation, and (pass 2) the instruction mix.

Peak issue rate (MI355X_MICROARCH.md, "Wave scheduling": a SIMD-32 issues a wave64
VALU instruction over 2 cycles): 4 SIMDs x 256 CUs / 2 = 512 wave-instructions per
cycle. Measured on this chip (tools/valu_peak.hip, 8 waves per SIMD of independent
chains, the same counters): v_xor_b32 / v_add_u32 reach 0.79 of it, v_mul_lo_u32 and
v_bcnt_u32_b32 0.48 (twice the issue cost of a plain 32-bit op).
GRBM_GUI_ACTIVE is summed over the 8 XCDs (the guide's DVFS note): active cycles =
GRBM_GUI_ACTIVE / 8.
usage: python tools/pmc_c3_summary.py <p1 counter_collection.csv> [<p2 csv>] <out.json>"""
import collections
import csv
import json
import sys

PEAK = 512  # wave64 VALU instructions per cycle, chip-wide


def per_dispatch(path):
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if "wmvc_cluster_lc_kernel" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


args = sys.argv[1:]
out_path = args[-1]
d1 = per_dispatch(args[0])
top = max(c["SQ_INSTS_VALU"] for c in d1.values())
big = sorted(d for d in d1 if d1[d]["SQ_INSTS_VALU"] > top / 2)  # the 2^24-slot launches
slots = 1 << 24
out = {"kernel": "wmvc_cluster_lc_kernel<5>", "slots": slots, "dispatches": len(big),
       "peak_wave_instr_per_cycle": PEAK, "per_dispatch": []}
for d in big:
    c = d1[d]
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    out["per_dispatch"].append({
        "SQ_INSTS_VALU": c["SQ_INSTS_VALU"], "SQ_INSTS_SALU": c["SQ_INSTS_SALU"], "SQ_WAVES": c["SQ_WAVES"],
        "SQ_ACTIVE_INST_VALU": c.get("SQ_ACTIVE_INST_VALU"), "active_cycles": cycles,
        "valu_issue_util": c["SQ_INSTS_VALU"] / (PEAK * cycles),
        "valu_wave_instr_per_slot": c["SQ_INSTS_VALU"] / slots})
pd = out["per_dispatch"]
out["valu_wave_instr_per_slot"] = sum(x["valu_wave_instr_per_slot"] for x in pd) / len(pd)
out["valu_issue_util"] = sum(x["valu_issue_util"] for x in pd) / len(pd)
if len(args) > 2:
    d2 = per_dispatch(args[1])
    big2 = [d for d in d2 if d2[d].get("SQ_INSTS_VALU_INT32", 1) > 0]
    big2 = sorted(big2, key=lambda d: -sum(d2[d].values()))[:len(big)]
    mix = collections.defaultdict(float)
    for d in big2:
        for k, v in d2[d].items():
            mix[k] += v / len(big2)
    out["mix_per_dispatch"] = dict(mix)
    out["mix_per_slot"] = {k: v / slots for k, v in mix.items()}
json.dump(out, open(out_path, "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "per_dispatch"}))
