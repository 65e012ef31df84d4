"""Per-kernel average durations of every tools/exp_variants.sh run (gpurun_out/exp/<tag>/**/run_kernel_stats.csv),
side by side.  python tools/exp_summary.py [pattern]"""
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("lnr::", "")
    return name.replace("PosFromRays", "R").replace("PosFromArray", "A")[:34]


def main(pat=""):
    tabs = {}
    for f in sorted(glob.glob("gpurun_out/exp/*/**/*kernel_stats.csv", recursive=True)):
        tag = f.split(os.sep)[2]
        if pat not in tag:
            continue
        tabs[tag] = {short(r["Name"]): (float(r["AverageNs"]) / 1e3, int(r["Calls"])) for r in csv.DictReader(open(f))}
    names = sorted({k for t in tabs.values() for k in t}, key=lambda k: -max(t.get(k, (0, 0))[0] for t in tabs.values()))
    print(f"{'kernel (avg us)':36s}" + "".join(f"{t[:14]:>15s}" for t in tabs))
    for k in names[:18]:
        print(f"{k:36s}" + "".join(f"{tabs[t].get(k, (0, 0))[0]:15.1f}" for t in tabs))
    for t in tabs:
        out = glob.glob(f"gpurun_out/exp/{t}/out.txt")
        if out:
            print(t, [l for l in open(out[0]).read().splitlines() if "ms/step" in l][-1:])


if __name__ == "__main__":
    main(*sys.argv[1:])
