"""Digest of a few training steps (C2 shape: 16 keyframes x 512 rays x 512 samples, synthetic quad
window): sha256 of the fp32 parameters, the Adam moments and the last step's loss after K steps.  Run
once per library build (LONER_AMD_LIB=...) to check that an experiment variant changes no bit.

    LONER_AMD_LIB=loner_amd/_lib/variants/x.so python tools/lib_digest.py [steps]
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from loner_amd import _lib as L  # noqa: E402
from loner_amd import step as S_  # noqa: E402
from loner_amd import synthetic as syn  # noqa: E402
from loner_amd.rays import RayWindow  # noqa: E402


def main(steps=3):
    steps = int(steps)
    scans = syn.make_window("quad", 16, seed=1)
    win = RayWindow(scans, syn.world_cube("quad"), syn.SENSORS["quad"]["ray_range"], n_lidar=512, strategy="RANDOM")
    st = S_.FieldState(S_.StepConfig(n_samples=512), device="cuda:0")
    eng = S_.StepEngine(st, win.n_slots, seed=3)
    loss = None
    for g in range(1, steps + 1):
        loss = eng.step_window(win, global_step=g)
    eng.drop_prefetch()
    torch.cuda.synchronize()

    def sha(t):
        return hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()[:16]

    print(json.dumps(dict(lib=os.path.basename(L.LIB_PATH), steps=steps, params=sha(st.params), m=sha(st.m),
                          v=sha(st.v), loss=sha(loss) if torch.is_tensor(loss) else None)))


if __name__ == "__main__":
    main(*sys.argv[1:])
