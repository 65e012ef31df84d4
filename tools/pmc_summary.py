"""Average PMC counter values per kernel from tools/pmc.sh output (gpurun_out/pmc/*/run_counter_collection.csv)."""
import collections
import csv
import glob
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("lnr::", "")
    return name.replace("PosFromRays", "R").replace("PosFromArray", "A")[:40]


def main(root="gpurun_out/pmc"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/*/*counter_collection.csv"):
        per = collections.defaultdict(float)
        for row in csv.DictReader(open(f)):
            key = (short(row["Kernel_Name"]), row["Dispatch_Id"], row["Counter_Name"])
            per[key] += float(row["Counter_Value"])
        for (k, _, c), v in per.items():
            acc[k][c].append(v)
    for k in sorted(acc):
        vals = {c: sum(v) / len(v) for c, v in acc[k].items()}
        print(k)
        print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))


if __name__ == "__main__":
    main(*sys.argv[1:])
