"""The north-star driver's depth-L1 metric files (examples/fdt_optimize_implicit_map.py:548-562 and
:645-677), written in the reference's format so the evaluation scripts that read them keep working:

    <log>/metrics/l1_test.csv, l1_eval.csv   header ``global_step,min,max,mean,rmse``, one row per
                                            repetition (created, header only, before the loop)
    <log>/metrics_test/l1_<step>.yaml        ``min: ...`` / ``max: ...`` / ``mean: ...`` / ``rmse: ...``
    <log>/metrics_eval/l1_<step>.yaml        (no trailing newline; ``w+``: overwritten per step)

The per-scan L1 values arrive as one tensor (the reference ``torch.hstack``s the per-scan
``compute_l1_depth`` results); the statistics and their text are formed from a torch tensor as the
reference forms them (the YAML gets a 0-d tensor's format, the CSV the numpy scalar's), so the files
match byte for byte for the same values on the same device.
"""
import csv
import os

import torch

HEADER = ["global_step", "min", "max", "mean", "rmse"]


class L1MetricsLog:
    """``L1MetricsLog(log_dir)`` creates ``metrics/`` and both CSVs with their header (:548-562);
    ``write(kind, global_step, l1s)`` appends one repetition's statistics for ``kind`` in
    ("test", "eval") and writes its YAML (:645-677)."""

    def __init__(self, log_dir):
        self.log_dir = str(log_dir)
        os.makedirs(os.path.join(self.log_dir, "metrics"), exist_ok=True)
        for kind in ("test", "eval"):
            with open(self.csv_path(kind), "w") as f:
                csv.writer(f).writerow(HEADER)

    def csv_path(self, kind):
        return os.path.join(self.log_dir, "metrics", f"l1_{kind}.csv")

    def yaml_path(self, kind, global_step):
        return os.path.join(self.log_dir, f"metrics_{kind}", f"l1_{global_step}.yaml")

    def write(self, kind, global_step, l1s):
        if kind not in ("test", "eval"):
            raise ValueError(f"kind must be 'test' or 'eval', got {kind!r}")
        if isinstance(l1s, (list, tuple)) and l1s and isinstance(l1s[0], torch.Tensor):
            t = torch.hstack([x.reshape(-1) for x in l1s])
        else:
            t = l1s if isinstance(l1s, torch.Tensor) else torch.as_tensor(l1s)
        lo, hi, mean, rmse = t.min(), t.max(), t.mean(), torch.sqrt(torch.mean(t ** 2))
        os.makedirs(os.path.dirname(self.yaml_path(kind, global_step)), exist_ok=True)
        with open(self.yaml_path(kind, global_step), "w+") as f:
            f.write(f"min: {lo}\nmax: {hi}\nmean: {mean}\nrmse: {rmse}")
        with open(self.csv_path(kind), "a") as f:
            csv.writer(f).writerow([global_step] + [v.cpu().numpy() for v in (lo, hi, mean, rmse)])
        return dict(min=float(lo), max=float(hi), mean=float(mean), rmse=float(rmse))
