"""What a graph-replayed step saves and what capturing costs (host wall time per step_window call with a
device sync after each call, so the numbers are per-step latency): eager pipelined steps, the first call
of each graph variant (an eager step + the capture), and replays.  For choosing when the Optimizer's
windows (32 iterations in the north-star driver) should capture.  GPU only; prints JSON lines.

    python tools/graph_cost.py [C1|C2]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from loner_amd import step as S_  # noqa: E402
from loner_amd import synthetic as syn  # noqa: E402
from loner_amd.rays import RayWindow  # noqa: E402


def main(config="C1"):
    n_kf, rpk, S = (1, 512, 64) if config == "C1" else (16, 512, 512)
    scans = syn.make_window("quad", n_kf, seed=1)
    wc = syn.world_cube("quad")
    win = RayWindow(scans, wc, syn.SENSORS["quad"]["ray_range"], n_lidar=rpk, strategy="RANDOM")
    out = {}
    for graph in (False, True):
        st = S_.FieldState(S_.StepConfig(n_samples=S), device="cuda:0")
        eng = S_.StepEngine(st, win.n_slots, seed=3)
        eng.use_graph = graph
        times = []
        for g in range(1, 41):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.step_window(win, global_step=g)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        if graph:
            out["graph_first_calls_ms"] = [round(t, 3) for t in times[:4]]
            out["graph_captures"] = len(eng._graphs)
            steady = sorted(times[10:])
            out["graph_replay_ms_median"] = steady[len(steady) // 2]
        else:
            steady = sorted(times[10:])
            out["eager_ms_median"] = steady[len(steady) // 2]
    out["config"] = config
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
