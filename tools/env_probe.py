"""GPU probe: fused 3-D kernel time at 512^3 under several settings of the per-launch environment
knobs (MVTV_F3D_IH, MVTV_F3D_STRIP, MVTV_F3D_WG), all inside ONE process so every setting sees the
same buffer placement. usage: python tools/env_probe.py "" "MVTV_F3D_IH=16" "MVTV_F3D_STRIP=0" ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import multivartv_amd as mv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402

KNOBS = ("MVTV_F3D_IH", "MVTV_F3D_STRIP", "MVTV_F3D_WG", "MVTV_F3D_XCD")
m = [512] * 3
y = towers(m)
P = mv.Problem(m, y, deltas=[(1.0 + 2e-4) / v for v in m], order=mv.ORDER_CPP, device=0)
P.state_set(np.full(y.size, y.mean()), None, 0.2)
del y
P.run(1.0, fixed_iters=2)
for rep in range(2):
    for setting in sys.argv[1:] or [""]:
        for k in KNOBS:
            os.environ.pop(k, None)
        for kv in setting.split():
            k, v = kv.split("=")
            os.environ[k] = v
        P.timing(True)
        P.run(1.0, fixed_iters=10)
        t = P.timings()["admm_fused"]
        P.timing(False)
        print(f"rep {rep} [{setting or 'default'}]: admm_fused {t['ms'] / t['launches']:.4f} ms", flush=True)
P.close()
