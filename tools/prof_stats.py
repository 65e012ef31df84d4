"""Summarise a rocprofv3 rocpd database (``-d DIR -o run`` writes DIR/run_results.db) into the
``--stats`` kernel CSV layout: Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs.

    python tools/prof_stats.py gpurun_out/prof/run_results.db > profiles/rNN_....csv
"""
import csv
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, s, a, lo, hi in rows:
        w.writerow([name, n, int(s), round(a, 1), round(100.0 * s / tot, 3), int(lo), int(hi)])


if __name__ == "__main__":
    main(sys.argv[1])
