"""Compare per-kernel average durations across experiment variants (gpurun_out/exp/*/run_kernel_stats.csv)."""
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("lnr::", "").replace("PosFromRays", "R").replace("PosFromArray", "A")
    return name[:48]


def load(path):
    out = {}
    for row in csv.DictReader(open(path)):
        out[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3)
    return out


def main(root="gpurun_out/exp"):
    vs = sorted(glob.glob(os.path.join(root, "*", "run_kernel_stats.csv")))
    data = {os.path.basename(os.path.dirname(v)): load(v) for v in vs}
    names = sorted({k for d in data.values() for k in d}, key=lambda k: -max(d.get(k, (0, 0))[1] for d in data.values()))
    tags = list(data)
    print(f"{'kernel (avg us)':50s}" + "".join(f"{t[-14:]:>16s}" for t in tags))
    for k in names:
        print(f"{k:50s}" + "".join(f"{data[t].get(k, (0, float('nan')))[1]:16.1f}" for t in tags))
    for t in tags:
        out = os.path.join(root, t, "out.txt")
        lines = [l for l in open(out) if "ms/step" in l] if os.path.exists(out) else []
        print(t, lines[-1].strip() if lines else "")


if __name__ == "__main__":
    main(*sys.argv[1:])
