"""Per-step kernel table of the LAST ``steps`` optimiser steps of a rocprofv3 kernel trace (the bench's timed
window), launches grouped by kernel name and grid: calls per step and average duration.
    python tools/trace_tail.py gpurun_out/<tag>/trace_C4/run_kernel_trace.csv [steps] [anchor-kernel]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
anchor = sys.argv[3] if len(sys.argv) > 3 else "k_build_rays"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
first = idx[-steps]
tail = rows[first:]
agg = defaultdict(list)
for r in tail:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lnr::", "")
    key = (name[:70], r["Grid_Size_X"], r["Grid_Size_Y"])
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for key, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    s = sum(v) / steps
    tot += s
    print(f"{key[0]:70s} grid {key[1]:>9s}x{key[2]:<3s} {len(v) / steps:5.2f}/step {sum(v) / len(v):8.1f} us  {s:8.1f} us/step")
span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3 / steps
print(f"kernel time per step {tot:.1f} us; wall per step {span:.1f} us")
