"""Same-process A/B of the k_march 3-D solve (dim 2 first, marching dim-0 transforms + dim-1 Thomas) against the
five-pass solve (MVTV_MARCH=0): ADMM it/s without events and the per-kernel times with them, interleaved.
Needs the probe build (make PROBES=1 OUT=../lib_probe; MVTV_LIB_PATH=.../lib_probe/libmvtv.so)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multivartv_amd as mv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402


def main():
    meshes = [[int(v) for v in s.split("x")] for s in (sys.argv[1:] or ["256x256x256", "512x512x512"])]
    for m in meshes:
        y = towers(m)
        deltas = [(1.0 + 2e-4) / v for v in m]
        steps = max(10, int(2e9 // y.size))
        with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
            th0 = np.full(y.size, y.mean())
            for rep in range(3):
                for off in ("0", "1"):
                    if off == "1":
                        os.environ.pop("MVTV_MARCH", None)
                    else:
                        os.environ["MVTV_MARCH"] = "1"
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
                    print(f"{'x'.join(map(str, m))} rep {rep} {'five-pass' if off == '1' else 'march    '}: "
                          f"{rate:.2f} it/s  {ks}", flush=True)


if __name__ == "__main__":
    main()
