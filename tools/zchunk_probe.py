"""GPU probe: fused 3-D kernel time at 512^3 for several dim-2 chunkings (MVTV_F3D_WG = target
workgroup count) inside ONE process, so every setting sees the same buffer placement."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import multivartv_amd as mv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402

m = [512] * 3
y = towers(m)
P = mv.Problem(m, y, deltas=[(1.0 + 2e-4) / v for v in m], order=mv.ORDER_CPP, device=0)
P.state_set(np.full(y.size, y.mean()), None, 0.2)
del y
P.run(1.0, fixed_iters=2)
settings = [int(v) for v in (sys.argv[1:] or ["4096", "2508", "5016", "8151", "3762", "4096"])]
for rep in range(2):
    for wg in settings:
        os.environ["MVTV_F3D_WG"] = str(wg)
        P.timing(True)
        P.run(1.0, fixed_iters=10)
        t = P.timings()["admm_fused"]
        P.timing(False)
        print(f"rep {rep} MVTV_F3D_WG={wg}: admm_fused {t['ms'] / t['launches']:.4f} ms", flush=True)
P.close()
