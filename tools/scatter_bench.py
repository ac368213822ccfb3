"""Throughput of the scattered-data setup (create_cache_objects on the GPU, mvtv_problem_set_scattered):
n uniform points in [0,1]^3 onto a 256^3 create_mesh grid. Prints one JSON line per size with the
wall time of the call (host buffers in, so PCIe included) and, under rocprofv3 --kernel-trace, the
kernels can be read separately (k_nearest, rocPRIM's radix sort, k_run_sums)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import multivartv_amd as mv  # noqa: E402


def main():
    m = [256, 256, 256]
    N = int(np.prod(m))
    axes = [np.linspace(-1e-4, 1 + 1e-4, mj) for mj in m]
    with mv.Problem(m, np.zeros(N)) as P:
        for n in (1 << 22, 1 << 24, 1 << 26):
            rng = np.random.default_rng(n)
            x = np.asfortranarray(rng.uniform(0, 1, size=(n, 3)))
            y = rng.standard_normal(n)
            P.set_scattered(axes, x[:1024], y[:1024])   # warm-up (rocPRIM kernels loaded)
            t0 = time.perf_counter()
            idx = P.set_scattered(axes, x, y)
            t1 = time.perf_counter()
            P.nearest(axes, x)
            t2 = time.perf_counter()
            print(json.dumps({"n": n, "nodes": N, "set_scattered_s": round(t1 - t0, 4), "nearest_s": round(t2 - t1, 4),
                              "points_per_s_setup": round(n / (t1 - t0), 1), "idx_max": int(idx.max())}),
                  flush=True)


if __name__ == "__main__":
    main()
