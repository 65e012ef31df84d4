"""Turn a tools/gpu_check.sh run (gpurun_out/) into committed profile files:

    profiles/<tag>_bench_<cfg>.json            the bench line (plain run)
    profiles/<tag>_bench_<cfg>_under_rocprof.json
    profiles/<tag>_bench_<cfg>_kernel_stats.csv rocprofv3 --kernel-trace --stats summary
    profiles/<tag>_traffic_<cfg>.json           PMC HBM bytes per launch for the hash-grid backward
    profiles/<tag>_mfma_<cfg>.json              PMC MFMA busy fraction of the sigma-MLP kernels

Traffic per the MI355X guide's HBM section: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, FETCH_SIZE
doubled on gfx950 (it counts 128-B requests as 64 B), averaged per dispatch and summed over the
backward stage's kernels per step, over the steps after the bench's warmup (the first steps run the
full backward until the live switch's probe lands).

    python tools/refresh_profiles.py r01 C2 [source dir, default gpurun_out]
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BWD_KERNELS = ("k_bwd_col_totals", "k_bwd_live_flags", "k_bwd_live_list", "k_bwd_count_live", "k_bwd_chunk_sums",
               "k_bwd_scan_rows", "k_bwd_scan_buckets", "k_bwd_scatter_rows", "k_bwd_scatter", "k_denc_level_max",
               "k_bwd_accum", "k_bwd_finalize", "k_bwd_accum_units", "k_bwd_finalize_units", "k_bwd_accum_buckets",
               "k_bwd_units")


def _short(name):
    return name.split("(")[0].replace("void ", "").replace("lnr::", "").strip()


def _base(name):
    return _short(name).split("<")[0]


def _timed_rows(paths_mults, warmup):
    """Rows (short kernel name, bytes) of the steps after the bench's warmup: a step ends with its Adam
    (k_adam), so the dispatches after the warmup-th k_adam are the timed and profiled steps.  Returns
    (steps counted, {name: [bytes, dispatch ids]})."""
    out = collections.defaultdict(lambda: [0.0, set()])
    n_steps = None
    for path, mult in paths_mults:
        rows = list(csv.DictReader(open(path)))
        adam = sorted({int(r["Dispatch_Id"]) for r in rows if _base(r["Kernel_Name"]) == "k_adam"})
        cut = adam[warmup - 1] if 0 < warmup <= len(adam) else -1
        n = len(adam) - (warmup if 0 < warmup <= len(adam) else 0)
        n_steps = n if n_steps is None else min(n_steps, n)
        for r in rows:
            if int(r["Dispatch_Id"]) > cut:
                e = out[_short(r["Kernel_Name"])]
                e[0] += mult * float(r["Counter_Value"]) * 1024
                e[1].add((path, r["Dispatch_Id"]))
    return max(n_steps or 0, 1), out


MLP_KERNELS = ("k_sigma_fwd_tiles", "k_field_wave", "k_mlp_bwd_tiles")
N_SIMD = 256 * 4  # 256 CUs x 4 SIMDs


def mfma_busy(path):
    """Per sigma-MLP kernel: mean SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE per dispatch, and the
    busy fraction MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs).  GRBM_GUI_ACTIVE is the sum over the
    8 XCDs (MI355X_MICROARCH.md, DVFS give-back) and reads high on dispatches under ~0.3 ms, so the
    fraction is a lower bound there."""
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for row in csv.DictReader(open(path)):
        key = next((k for k in MLP_KERNELS if k in row["Kernel_Name"]), None)
        if key is None:
            continue
        tot[key][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[key].add(row["Dispatch_Id"])
    out = {}
    for k, c in tot.items():
        nd = len(disp[k])
        busy, active = c["SQ_VALU_MFMA_BUSY_CYCLES"] / nd, c["GRBM_GUI_ACTIVE"] / nd
        out[k] = {"SQ_VALU_MFMA_BUSY_CYCLES": busy, "GRBM_GUI_ACTIVE": active,
                  "mfma_busy_frac": busy / (active / 8 * N_SIMD) if active else None}
    return out


OGM_KERNELS = ("k_ogm_grad", "k_sum_replicas", "k_sgd")


def step_traffic(fetch_csv, write_csv, warmup):
    """Per kernel: HBM bytes per optimiser step from the --pmc passes over bench.py, over the steps after the
    warmup (the timed and profiled steps), FETCH_SIZE doubled on gfx950."""
    n_steps, rows = _timed_rows(((fetch_csv, 2.0), (write_csv, 1.0)), warmup)
    # (torch's own kernels are the bench's instrumentation around its profiled steps -- the dL/dsigma zero
    # counts -- and the live switch's probe, not the step)
    out = {k: {"bytes_per_step": v[0] / n_steps, "dispatches": len(v[1]) // 2} for k, v in rows.items()
           if not k.startswith("at::")}
    return n_steps, out


def main(tag, cfg, src=None):
    out = os.path.join(ROOT, src or "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(out, "bench.json"), os.path.join(prof, f"{tag}_bench_{cfg}.json"))
    shutil.copy(os.path.join(out, "bench_prof.json"), os.path.join(prof, f"{tag}_bench_{cfg}_under_rocprof.json"))
    stats = glob.glob(os.path.join(out, "prof", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_bench_{cfg}_kernel_stats.csv"))
    bench = json.load(open(os.path.join(out, "bench.json")))
    warmup = int(bench.get("warmup", 10))
    f = glob.glob(os.path.join(out, "pmc", "FETCH_SIZE", "*counter_collection.csv"))
    w = glob.glob(os.path.join(out, "pmc", "WRITE_SIZE", "*counter_collection.csv"))
    if f and w:
        n_steps, rows = _timed_rows(((f[0], 2.0), (w[0], 1.0)), warmup)
        kern = {k: {"bytes_per_step": v[0] / n_steps, "dispatches": len(v[1]) // 2} for k, v in rows.items()
                if _base(k) in BWD_KERNELS}
        total = sum(v["bytes_per_step"] for v in kern.values())
        alg = (bench.get("backward_stage") or {}).get("algorithmic_bytes_per_launch")
        rec = {"stage": "hash-grid backward, every kernel of the stage, per step (one launch of the stage per step)",
               "config": cfg, "steps_profiled": n_steps, "hbm_bytes_per_launch": total,
               "algorithmic_bytes_per_launch": alg, "ratio_to_algorithmic": total / alg if alg else None,
               "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving, validated per access pattern in profiles/r04_fetch_calibration.json); the steps after the bench's warmup",
               "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["bytes_per_step"]))}
        json.dump(rec, open(os.path.join(prof, f"{tag}_traffic_{cfg}.json"), "w"), indent=1)
        print(f"backward traffic {total / 1e9:.3f} GB per step vs algorithmic {(alg or 0) / 1e9:.3f} GB")
    f = glob.glob(os.path.join(out, "pmc_step", "FETCH_SIZE", "*counter_collection.csv"))
    w = glob.glob(os.path.join(out, "pmc_step", "WRITE_SIZE", "*counter_collection.csv"))
    if f and w:
        n_steps, kern = step_traffic(f[0], w[0], warmup)
        total = sum(v["bytes_per_step"] for v in kern.values())
        alg = bench["roofline"].get("step_algorithmic_bytes")
        rec = {"what": "HBM bytes per optimiser step, every kernel of the step (rocprofv3 --pmc FETCH_SIZE and "
                       "WRITE_SIZE passes over the bench command)", "config": cfg, "steps_profiled": n_steps,
               "hbm_bytes_per_step": total, "step_algorithmic_bytes": alg,
               "ratio_to_algorithmic": total / alg if alg else None,
               "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving, validated per access pattern in profiles/r04_fetch_calibration.json)",
               "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["bytes_per_step"]))}
        json.dump(rec, open(os.path.join(prof, f"{tag}_traffic_{cfg}_step.json"), "w"), indent=1)
        print(f"step traffic {total / 1e9:.3f} GB per step vs algorithmic {(alg or 0) / 1e9:.3f} GB")
    m = glob.glob(os.path.join(out, "pmc", "MFMA", "*counter_collection.csv"))
    if m:
        kern = mfma_busy(m[0])
        rec = {"kernels": kern, "config": cfg,
               "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs)"}
        json.dump(rec, open(os.path.join(prof, f"{tag}_mfma_{cfg}.json"), "w"), indent=1)
        print("mfma busy", {k: round(v["mfma_busy_frac"] or 0.0, 4) for k, v in kern.items()})
    # texture-addresser busy of the encode (tools/pmc_l2req.sh pass l2b): TA_BUSY_avr per TA instance over the
    # GPU-active cycles of one XCD (GRBM_GUI_ACTIVE sums the 8 XCDs)
    t = glob.glob(os.path.join(out, "pmcl2", "l2b", "*counter_collection.csv"))
    if t:
        tot = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for row in csv.DictReader(open(t[0])):
            if "k_hashgrid_fwd" not in row["Kernel_Name"]:
                continue
            tot[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        ta = sum(tot["TA_BUSY_avr"].values()) / max(len(tot["TA_BUSY_avr"]), 1)
        gr = sum(tot["GRBM_GUI_ACTIVE"].values()) / max(len(tot["GRBM_GUI_ACTIVE"]), 1)
        rec = {"kernel": "k_hashgrid_fwd", "config": cfg, "dispatches": len(tot["TA_BUSY_avr"]),
               "TA_BUSY_avr": ta, "GRBM_GUI_ACTIVE": gr, "ta_busy_frac": ta / (gr / 8) if gr else None,
               "formula": "TA_BUSY_avr / (GRBM_GUI_ACTIVE / 8 XCDs)"}
        json.dump(rec, open(os.path.join(prof, f"{tag}_ta_{cfg}.json"), "w"), indent=1)
        print("encode TA busy", rec["ta_busy_frac"])
    for sub, name in (("pmcl2", "l2req"), ("pmcb", "pmc")):
        f = os.path.join(out, sub, "summary.txt")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(prof, f"{tag}_{name}_{cfg}.txt"))


if __name__ == "__main__":
    main(*sys.argv[1:])
