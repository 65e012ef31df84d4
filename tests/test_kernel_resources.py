"""Register spills of the built gfx950 kernels (CPU only: reads the code objects inside
loner_amd/_lib/libloner_amd.so, nothing runs on a GPU).

The library's .hip_fatbin section holds one clang offload bundle per translation unit; each gfx950
code object's AMDGPU metadata note carries every kernel's .vgpr_spill_count.  No kernel of the
benched step may spill; the allowlist names the few that do, off that path:
  * k_bwd_accum with the fused Adam epilogue (<*, true>): the record-balanced accumulate only takes
    the epilogue above 2^17 samples, where the step keeps Adam separate (step.FUSED_ADAM_MAX_N);
  * the two-samples-per-thread encodes (k_hashgrid_fwd<*, 2, false, 1>): of plain positions, and of rays
    with a live mask (one VGPR since that encode can count the backward's records of live samples); a
    live encode takes it only with LONER_ENC_LIVE_LPB=1 or an odd level count (default: <*, 1, false, 2>).
A spill the allowlist does not name fails here: 20 spilled VGPRs went unnoticed in the C2
accumulate for a while (the epilogue used to be a runtime branch of the same kernel)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "loner_amd", "_lib", "libloner_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"
ALLOWED = [
    r"^_ZN3lnr11k_bwd_accumILb[01]ELb1E",
    r"^_ZN3lnr14k_hashgrid_fwdINS_12PosFromArrayELi2ELb0ELi1E(E|Lb0ELb0EE)",
    r"^_ZN3lnr14k_hashgrid_fwdINS_11PosFromRaysELi2ELb0ELi1E(E|Lb0ELb0EE)",
]
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernel_spills(tmp_path):
    """kernel symbol -> (vgpr_spill_count, sgpr_spill_count) over every code object in the library."""
    fb = tmp_path / "fatbin.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", LIB, str(tmp_path / "copy.so")],
                   check=True, capture_output=True)
    data = fb.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = {}
    for i, o in enumerate(offs):
        part = tmp_path / f"b{i}.bin"
        part.write_bytes(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
        co = tmp_path / f"d{i}.co"
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                       capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
        for block in notes.split("- .agpr_count")[1:]:
            name = re.search(r"\.name:\s+(\S+)", block).group(1)
            v = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", block).group(1))
            s = int(re.search(r"\.sgpr_spill_count:\s+(\d+)", block).group(1))
            out[name] = (v, s)
    return out


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(f"{LLVM}/clang-offload-bundler"),
                    reason="library not built or ROCm LLVM tools absent")
def test_no_unexpected_vgpr_spills(tmp_path):
    spills = kernel_spills(tmp_path)
    assert len(spills) > 100, f"only {len(spills)} kernels found in the library's code objects"
    for must in ("k_bwd_accumILb0ELb0E", "k_bwd_scatter_rows", "k_hashgrid_fwd", "k_mlp_bwd_tiles",
                 "k_sigma_fwd_tiles", "k_sampler_wave", "k_adam"):
        assert any(must in k for k in spills), f"{must} not found"
    bad = {k: v for k, (v, _) in spills.items() if v and not any(re.search(p, k) for p in ALLOWED)}
    assert not bad, f"kernels spilling VGPRs outside the allowlist: {bad}"
