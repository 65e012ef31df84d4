"""GPU box: the data-parallel step's own overhead at world size 1 over RCCL (the bucketed all-reduces,
or the sharded optimiser's reduce-scatters, per-range Adam and shadow all-gathers, and their stream
waits; no peer traffic) against the plain step, C2 shape.

    python tools/dp_overhead.py            plain, all-reduce hook, ZeRO-1 hooks, plain again
    python tools/dp_overhead.py dp|zero    one of the hooked runs alone (for a kernel trace)
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(allreduce, steps=50, warmup=10, zero_hooks=None):
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    kind = "quad"
    scans = syn.make_window(kind, 16, seed=1000)
    win = RayWindow(scans, syn.world_cube(kind), syn.SENSORS[kind]["ray_range"], n_lidar=512, strategy="RANDOM",
                    device="cuda:0")
    st = S_.FieldState(S_.StepConfig(n_samples=512), device="cuda:0")
    extra = dict(zero=(0, 1), **zero_hooks) if zero_hooks else {}
    eng = S_.StepEngine(st, win.n_slots, seed=1, allreduce=allreduce, **extra)
    for i in range(warmup):
        eng.step_window(win, global_step=i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        eng.step_window(win, global_step=i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))

    def allreduce(t, async_op=False):
        return dist.all_reduce(t, async_op=async_op)

    zh = dict(reduce_scatter=lambda o, i, async_op=False: dist.reduce_scatter_tensor(o, i, async_op=async_op),
              all_gather=lambda o, i, async_op=False: dist.all_gather_into_tensor(o, i, async_op=async_op))
    if "dp" in sys.argv[1:]:  # the data-parallel run alone (for a kernel trace)
        print(json.dumps({"ms_per_step_rccl_world1": run(allreduce)}))
        dist.destroy_process_group()
        return
    if "zero" in sys.argv[1:]:
        print(json.dumps({"ms_per_step_zero_rccl_world1": run(allreduce, zero_hooks=zh)}))
        dist.destroy_process_group()
        return
    plain = run(None)
    dp = run(allreduce)
    zero = run(allreduce, zero_hooks=zh)
    plain2 = run(None)
    print(json.dumps({"config": "C2", "ms_per_step_plain": [plain, plain2], "ms_per_step_allreduce_rccl_world1": dp,
                      "ms_per_step_zero_rccl_world1": zero, "backend": dist.get_backend()}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
