"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, average us, share; plus the per-step sum.
    python tools/kstats.py gpurun_out/r3/prof_1/run_kernel_stats.csv [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
tot = 0.0
for r in rows:
    n, avg = int(r["Calls"]), float(r["AverageNs"]) / 1000
    tot += n * avg
    print(f"{r['Name'][:78]:78s} {n:5d} {avg:9.2f} us {float(r['Percentage']):6.2f}%")
print(f"kernel time per step (all calls / {steps}): {tot / steps:.1f} us")
