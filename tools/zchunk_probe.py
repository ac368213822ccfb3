"""GPU probe: fused 3-D kernel time for several dim-2 chunkings (MVTV_F3D_WG = target workgroup count)
inside ONE process, so every setting sees the same buffer placement. Probe build only
(make PROBES=1 OUT=...; MVTV_LIB_PATH=.../libmvtv.so).
usage: zchunk_probe.py SIZE|MxMxM WG [WG ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import multivartv_amd as mv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402

arg = sys.argv[1] if len(sys.argv) > 1 else "512"
m = [int(v) for v in arg.split("x")] if "x" in arg else [int(arg)] * 3
size = m[0]
y = towers(m)
P = mv.Problem(m, y, deltas=[(1.0 + 2e-4) / v for v in m], order=mv.ORDER_CPP, device=0)
P.state_set(np.full(y.size, y.mean()), None, 0.2)
del y
P.run(1.0, fixed_iters=2)
settings = [int(v) for v in (sys.argv[2:] or ["4096", "2508", "5016", "8151", "3762", "4096"])]
reps = 20 if int(np.prod(m)) <= 256 ** 3 else 10
for rep in range(2):
    for wg in settings:
        os.environ["MVTV_F3D_WG"] = str(wg)
        P.timing(True)
        P.run(1.0, fixed_iters=reps)
        t = P.timings()["admm_fused"]
        P.timing(False)
        print(f"mesh {arg} rep {rep} MVTV_F3D_WG={wg}: admm_fused {t['ms'] / t['launches']:.4f} ms, "
              f"{t['bytes_per_launch'] / (t['ms'] / t['launches'] * 1e-3) / 1e9:.0f} GB/s", flush=True)
P.close()
