"""Diagnostic: pieces of the distributed spectral solve with 2 ranks on one GPU."""
import os, socket, sys
import ctypes as C
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multivartv_amd as mv
from multivartv_amd import slab, _lib
from multivartv_amd.synth import towers

M = [16, 16, 16]


def rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y = towers(M)
    deltas = [(1.0 + 2e-4) / v for v in M]
    b = slab.plane_bounds(M[-1], world)
    pl = int(np.prod(M[:-1]))
    S = slab.SlabADMM(M, y[b[rank] * pl:b[rank + 1] * pl], deltas, y.mean(), device=0)
    P = S.P
    res = {}
    # (a) transpose round trip of a pattern
    pat = np.arange(P.N, dtype=np.float64) + 1000.0 * rank
    P.state_set(pat, np.zeros(P.E), 0.2)
    for s_ in range(S.G):
        S._copy(slab.THETA, S.glo * pl + s_ * S.chunk, S.nz, S.chunk, pl, S.chunk, S.sendbuf, 1, ext_offset=s_ * S.nz * S.chunk)
    res["send"] = S.sendbuf.numpy().copy()
    S.T.alltoall(S.linebuf, S.sendbuf, S.a2a_out, S.a2a_in)
    res["lines"] = S.linebuf.numpy().copy()
    S.T.alltoall(S.sendbuf, S.linebuf, S.a2a_in, S.a2a_out)
    for s_ in range(S.G):
        S._copy(slab.THETA, S.glo * pl + s_ * S.chunk, S.nz, S.chunk, pl, S.chunk, S.sendbuf, 0, ext_offset=s_ * S.nz * S.chunk)
    th, _, _ = P.state_get(want_u=False)
    res["rt"] = float(np.abs(th - pat).max())
    res["pat"] = pat[S.glo * pl:(S.glo + S.nz) * pl]
    q.put((rank, res, S.a2a_in.tolist(), S.a2a_out.tolist(), S.glo, S.nz))
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
    pl = 256
    full = np.concatenate([r[1]["pat"] for r in res]).reshape(16, pl)   # [z][q]
    for r in res:
        print("rank", r[0], "a2a_in", r[2], "a2a_out", r[3], "glo", r[4], "nz", r[5], "roundtrip err", r[1]["rt"])
        lines = r[1]["lines"].reshape(16, 128)
        expect = full[:, r[0] * 128:(r[0] + 1) * 128]
        print("  lines ok:", np.array_equal(lines, expect), "send[:4]", r[1]["send"][:4], "lines[:4]", lines[0, :4], "expect", expect[0, :4])
