"""Build the HIP C-ABI library ``loner_amd/_lib/libloner_amd.so`` for gfx950 (in-tree, so the
built .so travels to the GPU box with the repo snapshot).

    python -m loner_amd.build [--jobs N] [--force]

Plain hipcc, one object per translation unit, then a shared link.  No torch types cross the
boundary: the library exports exactly the symbols declared in ``include/loner_amd.h``.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libloner_amd.so")
OBJDIR = os.path.join(ROOT, "build", "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("LONER_ARCH", "gfx950")
# -ffp-contract=off: elementwise fp32 math rounds after every op, like the reference's torch ops.
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-ffp-contract=off", "-Wall",
         "-Wno-unused-function", "-I", os.path.join(ROOT, "include")]


# Per-file flags.  The hash-grid kernels keep global loads in flight across LDS-only barriers;
# SLP-packed f32 math (v_pk_*) needs its loaded operands copied into register pairs, and those
# copies wait for the loads before the barrier.
# rgb_train.hip: MFMA results in VGPRs (the colour-head backward's VALU reads every one of them; the default
# heuristic put them in AGPRs and paid a v_accvgpr_read per value).
FILE_FLAGS = {"hashgrid_bwd.hip": ["-fno-slp-vectorize"], "rgb_train.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
              "field.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _deps():
    return sorted(glob.glob(os.path.join(CSRC, "*.hpp")) + [os.path.join(ROOT, "include", "loner_amd.h")])


def _compile(src, objdir=OBJDIR, extra=(), file_flags=None):
    obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
    newest_dep = max(os.path.getmtime(p) for p in _deps() + [src])
    if os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj, ""
    ff = FILE_FLAGS if file_flags is None else file_flags
    cmd = [HIPCC, *FLAGS, *ff.get(os.path.basename(src), []), *extra, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj, r.stderr


def build(jobs=8, force=False, verbose=False, defines=(), out=None):
    """Build the library.  ``defines``/``out``: an experiment variant (-D flags) linked to ``out``
    with its own object directory (tools/exp_variants.py); the default build has neither.  A define
    ``FLAGS@<file>.hip@<flag>@<flag>...`` adds compiler flags for one source file instead."""
    lib_path = out or LIB
    objdir = OBJDIR if not defines else os.path.join(
        ROOT, "build", "obj_" + "_".join(sorted(defines)).lower().replace("@", "_").replace("-", "").replace("=", ""))
    file_flags = {k: list(v) for k, v in FILE_FLAGS.items()}
    for d in defines:
        if d.startswith("FLAGS@"):
            f, *fl = d.split("@")[1:]
            file_flags.setdefault(f, []).extend(fl)
    extra = [f"-D{d}" for d in defines if not d.startswith("FLAGS@")]
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    if force:
        for o in glob.glob(os.path.join(objdir, "*.o")):
            os.remove(o)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, objdir, extra, file_flags), srcs))
    objs = [o for o, _ in results]
    if verbose:
        for o, err in results:
            if err.strip():
                print(f"[{os.path.basename(o)}]\n{err}", file=sys.stderr)
    if os.path.exists(lib_path) and os.path.getmtime(lib_path) >= max(os.path.getmtime(o) for o in objs):
        return lib_path
    tmp = lib_path + ".tmp"  # linked aside, then renamed: a reader never sees a half-written library
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, lib_path)
    return lib_path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(a.jobs, a.force, a.verbose))


if __name__ == "__main__":
    main()
