"""Fold two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of bench.py into
per-launch HBM bytes of the REF step kernel -> profiles/pmc_c2.json.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE
is exact for 16 B/lane streaming stores. Both counters are in KB.
usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <replicas> <slots_per_launch> <out.json> [kernel_substring]
(kernel_substring default "ref_": the REF step kernel, tiled or lag)
"""
import csv
import glob
import json
import statistics
import sys


def per_dispatch(d, counter, kernel_sub="ref_"):
    """Counter value per dispatch of the headline launch: the step kernel dispatches
    with the largest grid (bench.py also times single-window launches)."""
    rows = []
    for path in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name") or ""
                if kernel_sub in name and (row.get("Counter_Name") or "") == counter:
                    rows.append(row)
    if not rows:
        return []
    gmax = max(int(r["Grid_Size"]) for r in rows)
    vals = {}
    for r in rows:
        if int(r["Grid_Size"]) == gmax:
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(r.get("Counter_Value") or 0)
    return list(vals.values())


def main():
    fdir, wdir, n, slots, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    ks = sys.argv[6] if len(sys.argv) > 6 else "ref_"
    f = per_dispatch(fdir, "FETCH_SIZE", ks)
    w = per_dispatch(wdir, "WRITE_SIZE", ks)
    if not f or not w:
        raise SystemExit(f"no {ks} rows (fetch {len(f)}, write {len(w)})")
    fk, wk = statistics.median(f), statistics.median(w)
    res = {"replicas": n, "slots_per_launch": slots, "kernel": ks, "dispatches": [len(f), len(w)],
           "fetch_size_kb_median": fk, "write_size_kb_median": wk,
           "hbm_read_bytes_per_launch": 2 * fk * 1024, "hbm_write_bytes_per_launch": wk * 1024,
           "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
           "alg_bytes_per_launch": slots * (4 * n + 8) / 8,
           "note": "FETCH_SIZE doubled per the gfx950 correction (MI355X_MICROARCH.md HBM section)"}
    res["traffic_over_alg"] = res["hbm_bytes_per_launch"] / res["alg_bytes_per_launch"]
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
