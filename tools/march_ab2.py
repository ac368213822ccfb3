"""A/B of probe settings for the k_march 3-D solve at 512^3 (same process, interleaved): each argument is a
comma-separated list of NAME=VALUE probe variables (empty = defaults). Needs the probe build."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multivartv_amd as mv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402


def main():
    m = [int(v) for v in os.environ.get("AB_MESH", "512x512x512").split("x")]
    settings = sys.argv[1:] or [""]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    steps = max(10, int(2e9 // y.size))
    keys = set()
    for st in settings:
        for kv in filter(None, st.split(",")):
            keys.add(kv.split("=")[0])
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        th0 = np.full(y.size, y.mean())
        for rep in range(3):
            for st in settings:
                for k in keys:
                    os.environ.pop(k, None)
                for kv in filter(None, st.split(",")):
                    k, v = kv.split("=")
                    os.environ[k] = v
                P.state_set(th0, None, 0.2)
                P.run(1.0, fixed_iters=3)
                t0 = time.perf_counter()
                P.run(1.0, fixed_iters=steps)
                rate = steps / (time.perf_counter() - t0)
                P.timing(True)
                P.run(1.0, fixed_iters=steps)
                tm = P.timings()
                P.timing(False)
                ks = {k: round(v["ms"] / max(1, v["launches"]), 4) for k, v in tm.items() if v["launches"]}
                print(f"{'x'.join(map(str, m))} rep {rep} [{st or 'default'}]: {rate:.2f} it/s  {ks}", flush=True)


if __name__ == "__main__":
    main()
