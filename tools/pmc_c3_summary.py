#!/usr/bin/env python3
"""Summarise the SQ/GRBM counter pass of tools/pmc_c3.sh for the C3 cluster kernel
(wmvc_cluster_lc_kernel<5>, the 2^24-slot launches of tools/bench_c3.py): VALU
wave-instructions per slot and the VALU issue utilisation. Peak issue rate: each of a
CU's 4 SIMDs issues one wave64 VALU instruction per 4 cycles (MI355X_MICROARCH.md, vector
issue cost; the pure-VALU trace kernel reaches 98 % of it), so the chip peak is
256 x 4 / 4 = 256 wave-instructions per cycle. GRBM_GUI_ACTIVE is
summed over the 8 XCDs (the guide's DVFS note): active cycles = GRBM_GUI_ACTIVE / 8.
usage: python tools/pmc_c3_summary.py <counter_collection.csv> <out.json>"""
import csv
import collections
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
disp = collections.defaultdict(dict)
grid = {}
for r in rows:
    if "wmvc_cluster_lc_kernel" not in r["Kernel_Name"]:
        continue
    d = int(r["Dispatch_Id"])
    disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    grid[d] = int(r["Grid_Size"])
top = max(c["SQ_INSTS_VALU"] for c in disp.values())
big = [d for d in disp if disp[d]["SQ_INSTS_VALU"] > top / 2]  # the 2^24-slot launches (same grid as 2^21)
slots = 1 << 24
out = {"kernel": "wmvc_cluster_lc_kernel<5>", "slots": slots, "dispatches": len(big), "per_dispatch": []}
for d in sorted(big):
    c = disp[d]
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    out["per_dispatch"].append({
        "SQ_INSTS_VALU": c["SQ_INSTS_VALU"], "SQ_INSTS_SALU": c["SQ_INSTS_SALU"], "SQ_WAVES": c["SQ_WAVES"],
        "active_cycles": cycles,
        "valu_issue_util": c["SQ_INSTS_VALU"] / (256.0 * cycles),
        "valu_wave_instr_per_slot": c["SQ_INSTS_VALU"] / slots})
pd = out["per_dispatch"]
out["valu_wave_instr_per_slot"] = sum(x["valu_wave_instr_per_slot"] for x in pd) / len(pd)
out["valu_issue_util"] = sum(x["valu_issue_util"] for x in pd) / len(pd)
out["peak_wave_instr_per_cycle"] = 256
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "per_dispatch"}))
