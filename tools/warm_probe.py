"""GPU probe: fused-kernel and DCT launch times of the 512^3 bench problem in consecutive chunks
of ADMM iterations from a cold process (does the box need time before it reaches steady state?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import multivartv_amd as mv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402

m = [512] * 3
y = towers(m)
P = mv.Problem(m, y, deltas=[(1.0 + 2e-4) / v for v in m], order=mv.ORDER_CPP, device=0)
P.state_set(np.full(y.size, y.mean()), None, 0.2)
del y
t0 = time.perf_counter()
for c in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    P.timing(True)
    P.run(1.0, fixed_iters=20)
    t = P.timings()
    P.timing(False)
    f = t["admm_fused"]
    d = t["dct"]
    print(f"t={time.perf_counter() - t0:6.2f}s chunk {c}: admm_fused {f['ms'] / f['launches']:.3f} ms, "
          f"dct {d['ms'] / d['launches']:.3f} ms", flush=True)
P.close()
