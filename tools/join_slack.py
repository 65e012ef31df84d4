"""Side-stream join slack from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``): for every
launch of a side-stream kernel (default ``k_count_opaque``, forked at the step's start and joined before
the field kernel, step.py), the time from its end to the start of the next main-stream kernel that waits
for it (default ``k_sigma_fwd_tiles``, the field kernel's first launch).  Negative slack would mean the
join stalled the step.  Also the side kernel's own trace durations (dispatch to end).

    python tools/join_slack.py gpurun_out/.../run_kernel_trace.csv [side_kernel] [joined_kernel]
"""
import csv
import json
import sys


def main(path, side="k_count_opaque", joined="k_sigma_fwd_tiles"):
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or ""
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    ev.sort()
    slack, dur = [], []
    starts_joined = [s for s, e, n in ev if joined in n]
    for s, e, n in ev:
        if side not in n:
            continue
        dur.append((e - s) / 1e3)
        nxt = next((t for t in starts_joined if t >= s), None)
        if nxt is not None:
            slack.append((nxt - e) / 1e3)
    if not slack:
        print(json.dumps(dict(error=f"no {side} / {joined} pairs in {path}")))
        return
    slack.sort()
    dur.sort()
    out = dict(side=side, joined=joined, launches=len(slack), slack_us_min=slack[0],
               slack_us_p5=slack[len(slack) // 20], slack_us_median=slack[len(slack) // 2],
               stalls=sum(1 for x in slack if x < 0), side_dur_us_median=dur[len(dur) // 2], side_dur_us_max=dur[-1])
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
