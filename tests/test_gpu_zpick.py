"""pick_zpair (mvtv_capi.cpp): the placement-aware choice of the fused 3-D kernel's z buffer pair moves
the edge state between physical buffers and nothing else. A 256^3 problem (2^24 nodes, the smallest that
takes the pick) runs 3 iterations, then 2 more resumed from the resident state, in fresh processes with
the pick on, off and forced down its failure path; theta, rho and the residual norms must be identical
bit for bit, for variant B (U_EXPLICIT start) and variant A (theta_old tracked)."""
import json
import os
import subprocess
import sys

import pytest

pytest.importorskip("multivartv_amd")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import hashlib, json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import multivartv_amd as mv
from multivartv_amd.synth import towers
variant = int(sys.argv[2])
m = [256, 256, 256]
y = towers(m)
with mv.Problem(m, y, deltas=[(1 + 2e-4) / 256] * 3, order=mv.ORDER_CPP) as P:
    P.state_set(np.full(y.size, y.mean()), None, 0.2)
    kw = dict(variant=variant, theta_solver=mv.SOLVER_SPECTRAL, ymean=float(y.mean()))
    s1 = P.run(2.0, fixed_iters=3, **kw)
    s2 = P.run(2.0, fixed_iters=2, **kw)
    th, _, rho = P.state_get(want_u=False)
print(json.dumps(dict(h=hashlib.sha256(th.tobytes()).hexdigest(), rho=rho, r=[s1["r_norm"], s2["r_norm"]],
                      s=[s1["s_norm"], s2["s_norm"]])))
"""


@pytest.mark.parametrize("variant", [0, 1])
def test_zpick_on_off_fail_identical(variant):
    out = {}
    for mode in ("0", "1", "fail"):
        env = dict(os.environ, MVTV_ZPICK=mode)
        r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, str(variant)], env=env, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out[mode] = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["0"] == out["1"] == out["fail"]
