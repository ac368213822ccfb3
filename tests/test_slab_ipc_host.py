"""The inter-process transport's host side (mvtv_comm_create_ipc: shared-memory rendezvous, rank-ordered host
all-reduce) across real processes, gloo for the segment name. No GPU: the all-reduce of host values touches no
device, and a communicator that never ran a slab loop holds no device mapping."""
import os
import socket

import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from multivartv_amd import slab
        c = slab.Comm.ipc(0)
        assert (c.rank, c.size) == (rank, world)
        outs = []
        for k in range(5):   # every all-reduce reuses the slots: the barriers keep rounds apart
            v = np.array([0.1 * (rank + 1) + k, 1e16 if rank == 0 else 1.0, -1e16 if rank == world - 1 else 0.0])
            outs.append(c.allreduce_host(v).tolist())
        c.close()
        q.put((rank, outs, None))
    except Exception as e:  # noqa: BLE001 (reported to the parent)
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ipc_host_allreduce_rank_ordered(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, _, err in res:
        assert err is None, err
    for k in range(5):
        want = []
        for i in range(3):   # the rank-ordered sum, as every rank computes it
            acc = 0.0
            for r in range(world):
                acc += [0.1 * (r + 1) + k, 1e16 if r == 0 else 1.0, -1e16 if r == world - 1 else 0.0][i]
            want.append(acc)
        for _, outs, _ in res:
            assert outs[k] == want   # bit-identical on every rank


def test_ipc_bad_arguments():
    from multivartv_amd import _lib, slab
    import ctypes as C
    h = C.c_void_p()
    L = _lib.lib()
    assert L.mvtv_comm_create_ipc(b"no-slash", 2, 0, 0, C.byref(h)) == _lib.MVTV_BAD_ARG
    assert L.mvtv_comm_create_ipc(b"/x", 17, 0, 0, C.byref(h)) == _lib.MVTV_BAD_ARG
    assert L.mvtv_comm_create_ipc(b"/x", 2, 2, 0, C.byref(h)) == _lib.MVTV_BAD_ARG
    # one rank: the segment is created and unlinked at once, the host all-reduce is the identity
    name = f"/mvtv_test_{os.getpid()}".encode()
    assert L.mvtv_comm_create_ipc(name, 1, 0, 0, C.byref(h)) == _lib.MVTV_OK
    c = slab.Comm(h)
    assert c.allreduce_host([1.5, 2.5]).tolist() == [1.5, 2.5]
    c.close()
    assert not os.path.exists("/dev/shm" + name.decode())
