"""GPU probe: per-launch time of the fused 3-D kernel at 512^3 under the two pairings of the z and
g_u ping-pong buffers, inside ONE process (same allocations). Each run is one ADMM iteration, so
consecutive runs alternate the buffer parity; MVTV_ZFLIP=1 (MVTV_GFLIP=1) for one run moves z (g_u)
to the other buffer, which shifts that ping-pong by one against the run index. usage: python tools/zflip_probe.py [iters per phase]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import multivartv_amd as mv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
m = [512] * 3
y = towers(m)
P = mv.Problem(m, y, deltas=[(1.0 + 2e-4) / v for v in m], order=mv.ORDER_CPP, device=0)
P.state_set(np.full(y.size, y.mean()), None, 0.2)
del y
P.run(1.0, fixed_iters=2)


def phase(name):
    ts = []
    for _ in range(n):
        P.timing(True)
        P.run(1.0, fixed_iters=1)
        t = P.timings()["admm_fused"]
        P.timing(False)
        ts.append(t["ms"] / t["launches"])
    even, odd = np.mean(ts[0::2]), np.mean(ts[1::2])
    print(f"{name}: " + " ".join(f"{v:.2f}" for v in ts) + f"  | even {even:.3f} odd {odd:.3f} mean {np.mean(ts):.3f}",
          flush=True)


def flip(knob):
    os.environ[knob] = "1"
    P.run(1.0, fixed_iters=1)
    os.environ.pop(knob)


for rep in range(2):
    phase(f"rep {rep} start")
    flip("MVTV_ZFLIP")   # z to the other buffer: other pairing of z and g
    phase(f"rep {rep} z flipped")
    flip("MVTV_GFLIP")   # g_u to the other buffer as well
    phase(f"rep {rep} z+g flipped")
    flip("MVTV_ZFLIP")
    phase(f"rep {rep} g flipped")
    flip("MVTV_GFLIP")
P.close()
