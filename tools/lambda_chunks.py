"""Config 4 (2D 2048^2, 32 lambdas) on ONE GPU: the lambda grid in K contiguous chunks
(cold start at each chunk head, cv.lambda_path's throughput form), the chunks run one after another
or concurrently (one mvtv_problem = one HIP stream per chunk, one host thread each; the C calls
release the GIL). Prints one JSON line per K: wall seconds, ADMM iterations/s over all chunks."""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multivartv_amd as mv  # noqa: E402
from multivartv_amd import synth  # noqa: E402


def main():
    m = [2048, 2048]
    N = m[0] * m[1]
    y = synth.towers(m)
    deltas = [(1 + 2e-4) / mj for mj in m]
    lams = np.exp(np.linspace(np.log(1.0), np.log(1e-3), 32))
    fixed = int(os.environ.get("FIXED", "60"))
    for K in (1, 2, 4, 8):
        probs = [mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) for _ in range(K)]
        chunks = np.array_split(lams, K)
        its = [0] * K

        def work(i):
            _, _, st = probs[i].path(chunks[i], np.full(N, y.mean()), chunks[i][0] / 5, want_thetas=False,
                                     fixed_iters=fixed)
            its[i] = sum(s["iters"] for s in st)

        work(0)   # warm-up (plans, lazily allocated buffers)
        t0 = time.perf_counter()
        th = [threading.Thread(target=work, args=(i,)) for i in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        print(json.dumps({"chunks": K, "lambdas": len(lams), "fixed_iters": fixed, "wall_s": round(wall, 4),
                          "admm_iters": sum(its), "iters_per_s": round(sum(its) / wall, 1)}), flush=True)
        for p in probs:
            p.close()


if __name__ == "__main__":
    main()
