"""Diagnostic: 2-rank slab ADMM on one GPU vs the one-GPU solver, iteration by iteration."""
import os, socket, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multivartv_amd as mv
from multivartv_amd import slab
from multivartv_amd.synth import towers

M = [16, 16, 16]


def ref(k):
    y = towers(M)
    deltas = [(1.0 + 2e-4) / v for v in M]
    with mv.Problem(M, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        th, _, rho, st = P.admm(1.0, np.full(y.size, y.mean()), u=np.zeros(P.E), rho=0.2, fixed_iters=k)
        x = P.solve_spectral(0.2, y)
    return th, x


def rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y = towers(M)
    deltas = [(1.0 + 2e-4) / v for v in M]
    b = slab.plane_bounds(M[-1], world)
    pl = int(np.prod(M[:-1]))
    S = slab.SlabADMM(M, y[b[rank] * pl:b[rank + 1] * pl], deltas, y.mean(), device=0)
    out = []
    for k in (1, 2, 3):
        S.run(1.0, fixed_iters=k)
        out.append(S.theta_owned())
    q.put((rank, out))
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted((q.get(timeout=100) for _ in ps), key=lambda t: t[0])
    [p.join() for p in ps]
    th1, x = ref(1)
    print("solve-only vs theta1 ref:", np.abs(x - th1).max())
    for i, k in enumerate((1, 2, 3)):
        thk, _ = ref(k)
        full = np.concatenate([r[1][i] for r in res])
        d = np.abs(full - thk).reshape(M[::-1])
        print(k, "max diff", d.max(), "per plane:", np.round(d.max(axis=(1, 2)), 12).tolist())
