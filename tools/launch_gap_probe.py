"""Small-mesh launch-gap probe: ADMM it/s of the asynchronous loop at 2-D / 3-D
config shapes with per-launch HIP events off and on, and the summed kernel time, in one process.
Usage: python tools/launch_gap_probe.py [--steps 400] [--mesh 1024x1024 ...]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multivartv_amd as mv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--mesh", nargs="*", default=["1024x1024", "2048x2048", "256x256x256"])
    a = ap.parse_args()
    for spec in a.mesh:
        m = [int(v) for v in spec.split("x")]
        y = towers(m)
        deltas = [(1.0 + 2e-4) / v for v in m]
        with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
            P.state_set(np.full(y.size, y.mean()), None, 0.2)
            P.run(1.0, fixed_iters=20)
            res = {}
            for ev in (False, True, False):
                P.timing(ev)
                steps = a.steps if len(m) == 2 else a.steps // 10
                t0 = time.perf_counter()
                P.run(1.0, fixed_iters=steps)
                dt = time.perf_counter() - t0
                tm = P.timings() if ev else None
                P.timing(False)
                key = "events" if ev else "plain"
                res[key] = steps / dt
                if tm:
                    ksum = sum(v["ms"] for v in tm.values()) / steps
                    res["kernel_ms_per_iter"] = ksum
            print(f"{spec}: it/s plain {res['plain']:.1f}, with events {res['events']:.1f}; "
                  f"wall {1e3 / res['plain']:.4f} ms/iter, kernels {res['kernel_ms_per_iter']:.4f} ms/iter", flush=True)


if __name__ == "__main__":
    main()
