"""GPU probe: fused 3-D kernel time per node for meshes whose dim 0 is / is not a multiple of the
63-column interior of a k_admm3d tile (512 = 8 x 63 + 8 leaves a 9th, nearly idle x-tile)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import multivartv_amd as mv
from multivartv_amd.synth import towers

for m in ([512] * 3, [504] * 3, [512] * 3, [504] * 3):
    y = towers(m)
    # Python block order without deltas: 7 blocks, no dim-0-first mixed-partial rule (unequal m allowed)
    P = mv.Problem(m, y, deltas=None, order=mv.ORDER_PY, device=0)
    P.state_set(np.full(y.size, y.mean()), None, 0.2)
    del y
    P.run(1.0, fixed_iters=2, pcg_rtol=1e-6, theta_solver=mv.SOLVER_PCG)
    P.timing(True)
    P.run(1.0, fixed_iters=6, pcg_rtol=1e-6, theta_solver=mv.SOLVER_PCG)
    t = P.timings()["admm_fused"]
    ms = t["ms"] / max(1, t["launches"])
    N = m[0] * m[1] * m[2]
    print(f"{m}: admm_fused {ms:.3f} ms, {ms * 1e6 / N:.3f} ns/node, launches {t['launches']}", flush=True)
    P.close()
