#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace (run_kernel_trace.csv) around the last step
kernels of a pipelined bench run: every kernel's hardware queue, start, end and duration
(µs from the first listed kernel), the synthetic-trace kernels left out. Shows whether
the exchange kernels of step t run beside the step kernel of t + 1 and what sits between
two step kernels.  usage: python tools/trace_timeline.py <run_kernel_trace.csv> [rows]"""
import csv
import sys


def main():
    path = sys.argv[1]
    limit = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    lag = [r for r in rows if "ref_lag_kernel" in r["Kernel_Name"]]
    print("step (lag) kernels", len(lag))
    t0 = int(lag[-6]["Start_Timestamp"]) - 1 if len(lag) >= 6 else int(rows[0]["Start_Timestamp"])
    sel = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and "trace_kernel" not in r["Kernel_Name"]]
    base = int(sel[0]["Start_Timestamp"])
    for r in sel[:limit]:
        name = r["Kernel_Name"].split("(")[0].replace("rg::", "").replace("void ", "")[:40]
        s = (int(r["Start_Timestamp"]) - base) / 1000
        e = (int(r["End_Timestamp"]) - base) / 1000
        print(f"{name:42s} q{r['Queue_Id']:>3} {s:9.1f} {e:9.1f} {e - s:8.1f}")


if __name__ == "__main__":
    main()
