"""One mesh decomposed over ranks: slab-parallel ADMM (SURVEY §8e, config 5 / the metric at 2-8 GPUs).

The mesh is cut along its slowest dimension (dim p-1, contiguous in the column-major layout): rank r
owns planes [floor(m r / G), floor(m (r+1) / G)) plus one ghost plane below and above
(mvtv_problem_create_slab). The whole variant-B loop of a rank (rcpp-code/MultivarTV/src/solvers.cpp:
110-133) runs inside libmvtv (``mvtv_slab_run``, csrc/mvtv_slab.cpp) with its collectives on the
problem's HIP stream and the adapt_step / stopping decisions taken on the device:

  theta-solve   cosine transforms along dims 0..p-2 on the owned planes (the last pass writes the
                all-to-all buffer directly), all-to-all, forward / divide / inverse along dim p-1,
                all-to-all back (the first inverse pass reads the buffer directly);
  theta halo    both ghost planes;
  edges         p = 3: the fused edge-update + gather pass on the owned planes; p = 4: edge update,
                z ghost plane, gather;
  all-reduce    the 7 partial sums into the device control block;
  z halo        (p = 3) the new z's last owned plane -> rank+1 (the next chunk-start recompute).

Transports (``Comm``): RCCL over xGMI, one process per GPU (``Comm.rccl``; the 128-byte unique id goes
through torch.distributed); an inter-process group over HIP IPC memory (``Comm.ipc``: one process per rank,
the ranks on one GPU or on peer GPUs of a node, device-to-device copies out of the peer's buffer, ordered
through a shared-memory rendezvous; host-synchronous collectives); or an in-process loopback group
(``Comm.local_group``): every rank on its own host thread, transfers as device copies, so a G-rank
decomposition is rehearsed on one GPU.
"""
from __future__ import annotations

import ctypes as _C
import os
import threading

import numpy as np

from . import _lib

_L = _lib.lib


class SlabDesc(_C.Structure):
    _fields_ = [("m_global", _C.c_int64), ("z_begin", _C.c_int64), ("z_end", _C.c_int64),
                ("ghost_lo", _C.c_int32), ("ghost_hi", _C.c_int32)]


_dp = _C.POINTER(_C.c_double)
_SIGS = {
    "mvtv_problem_create_slab": (_C.c_int, [_C.POINTER(_lib.ProblemDesc), _C.POINTER(SlabDesc), _C.POINTER(_C.c_void_p)]),
    "mvtv_comm_unique_id": (_C.c_int, [_C.c_char_p]),
    "mvtv_comm_create_rccl": (_C.c_int, [_C.c_char_p, _C.c_int32, _C.c_int32, _C.c_int32, _C.POINTER(_C.c_void_p)]),
    "mvtv_comm_create_local": (_C.c_int, [_C.c_int32, _C.POINTER(_C.c_void_p)]),
    "mvtv_comm_create_ipc": (_C.c_int, [_C.c_char_p, _C.c_int32, _C.c_int32, _C.c_int32, _C.POINTER(_C.c_void_p)]),
    "mvtv_comm_destroy": (None, [_C.c_void_p]),
    "mvtv_comm_rank": (_C.c_int32, [_C.c_void_p]),
    "mvtv_comm_size": (_C.c_int32, [_C.c_void_p]),
    "mvtv_slab_run": (_C.c_int, [_C.c_void_p, _C.c_void_p, _C.POINTER(_lib.AdmmOpts), _C.c_double, _C.c_double,
                                 _C.c_double, _C.POINTER(_lib.AdmmStats)]),
    "mvtv_sync": (_C.c_int, [_C.c_void_p]),
    "mvtv_comm_allreduce_host": (_C.c_int, [_C.c_void_p, _dp, _C.c_int32]),
    "mvtv_comm_library": (_C.c_char_p, []),
}
_lib.SIGNATURES.update(_SIGS)
if _lib._LIB is not None:   # library already loaded: register the new signatures
    for _n in _SIGS:
        _f = getattr(_lib._LIB, _n)
        _f.restype, _f.argtypes = _lib.SIGNATURES[_n]


def plane_bounds(m_last: int, world: int):
    """Contiguous plane ranges floor(m r / G) (the split mvtv_slab_run assumes); every rank owns >= 1 plane."""
    if m_last < world:
        raise ValueError(f"{m_last} planes cannot be split over {world} ranks")
    return np.array([(m_last * r) // world for r in range(world + 1)], dtype=np.int64)


class Comm:
    """A transport of mvtv_slab_run (an mvtv_comm handle)."""

    def __init__(self, h, kind="local"):
        self._h = h
        self.kind = kind   # "rccl", "ipc" or "local"
        self.rank = int(_L().mvtv_comm_rank(h))
        self.size = int(_L().mvtv_comm_size(h))

    @classmethod
    def rccl(cls, device: int, group=None):
        """RCCL communicator over the ranks of torch.distributed's (default) group, one process per GPU."""
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        buf = [None]
        if rank == 0:
            raw = _C.create_string_buffer(128)
            _lib._check(_L().mvtv_comm_unique_id(raw))
            buf[0] = bytes(raw.raw)
        dist.broadcast_object_list(buf, src=0, group=group)
        h = _C.c_void_p()
        _lib._check(_L().mvtv_comm_create_rccl(buf[0], world, rank, device, _C.byref(h)))
        return cls(h, "rccl")

    @classmethod
    def rccl_single(cls, device: int):
        """A one-rank RCCL communicator (no torch.distributed needed)."""
        raw = _C.create_string_buffer(128)
        _lib._check(_L().mvtv_comm_unique_id(raw))
        h = _C.c_void_p()
        _lib._check(_L().mvtv_comm_create_rccl(raw.raw, 1, 0, device, _C.byref(h)))
        return cls(h, "rccl")

    @classmethod
    def ipc(cls, device: int, group=None):
        """Inter-process group over HIP IPC memory across the ranks of torch.distributed's (default) group
        (any backend: only a segment name is broadcast). Works where RCCL refuses, e.g. several ranks on one GPU."""
        import uuid

        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        buf = [f"/mvtv_{os.getpid()}_{uuid.uuid4().hex[:12]}" if rank == 0 else None]
        dist.broadcast_object_list(buf, src=0, group=group)
        h = _C.c_void_p()
        _lib._check(_L().mvtv_comm_create_ipc(buf[0].encode(), world, rank, device, _C.byref(h)))
        return cls(h, "ipc")

    @classmethod
    def local_group(cls, n: int):
        """n loopback handles of one in-process group (run each rank on its own thread)."""
        hs = (_C.c_void_p * n)()
        _lib._check(_L().mvtv_comm_create_local(n, hs))
        return [cls(_C.c_void_p(hs[i])) for i in range(n)]

    def allreduce_host(self, vals):
        """Sum of a few host doubles over the RCCL or ipc communicator (blocking)."""
        v = np.ascontiguousarray(np.asarray(vals, dtype=np.float64).ravel())
        _lib._check(_L().mvtv_comm_allreduce_host(self._h, v.ctypes.data_as(_dp), v.size))
        return v

    @staticmethod
    def library():
        """The file RCCL was resolved from (ROCm's librccl, on libmvtv's HIP runtime)."""
        return (_L().mvtv_comm_library() or b"").decode()

    def close(self):
        if getattr(self, "_h", None):
            _L().mvtv_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Slab(_lib.Problem):
    """A Problem created with mvtv_problem_create_slab (same wrapper, different constructor)."""

    def __init__(self, m_local, oty_local, deltas, order, device, m_global, zb, ze, glo, ghi, w_local=None):
        p = len(m_local)
        self.m, self.p = [int(v) for v in m_local], p
        self.N = int(np.prod(m_local))
        d = _lib.ProblemDesc()
        d.p = p
        for j in range(4):
            d.m[j] = self.m[j] if j < p else 1
            d.deltas[j] = float(deltas[j]) if j < p else 0.0
        d.block_order = order
        d.weighted = 1
        self.deltas = [float(v) for v in deltas]
        self.order, self.weighted, self.device = order, True, device
        self._oty = _lib._f64(oty_local, self.N)
        self._w = None if w_local is None else _lib._f64(w_local, self.N)
        d.oty = _lib._ptr(self._oty)
        d.wdiag = None if self._w is None else _lib._ptr(self._w)
        d.device = device
        sd = SlabDesc()
        sd.m_global, sd.z_begin, sd.z_end, sd.ghost_lo, sd.ghost_hi = m_global, zb, ze, glo, ghi
        h = _C.c_void_p()
        _lib._check(_L().mvtv_problem_create_slab(_C.byref(d), _C.byref(sd), _C.byref(h)))
        self._h = h
        self.E = int(_L().mvtv_problem_edges(h))
        self.nb = int(_L().mvtv_problem_blocks(h))


class SlabADMM:
    """Variant-B ADMM on one rank's slab of a mesh fit (p >= 2; m_j <= 4096 for j < p - 1, the last dimension
    any length over >= 2 ranks).

    ``oty_owned``: O^T y on the owned planes (= y for lattice data, W y for a diagonal W). ``ymean``: theta_0
    (the global mean of y, rcpp…/solvers.cpp:207). ``comm``: a :class:`Comm` (its rank / size fix the slab).
    ``w_owned``: diag(W) = diag(O^T O) on the owned planes (None: W = I). With W the theta-solve is PCG with the
    spectral preconditioner of mean(W) I + rho D^T D, distributed like the direct solve.
    """

    def __init__(self, m, oty_owned, deltas, ymean, comm: Comm, device=None, order=_lib.ORDER_CPP, w_owned=None):
        self.m = [int(v) for v in m]
        p = len(self.m)
        if p < 2:
            raise ValueError("slab decomposition needs p >= 2")
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        self.comm = comm
        G, r = comm.size, comm.rank
        self.G, self.r = G, r
        self.mg = self.m[-1]
        self.bounds = plane_bounds(self.mg, G)
        self.zb, self.ze = int(self.bounds[r]), int(self.bounds[r + 1])
        self.nz = self.ze - self.zb
        self.glo, self.ghi = int(self.zb > 0), int(self.ze < self.mg)
        self.plane = int(np.prod(self.m[:-1]))
        m_local = self.m[:-1] + [self.nz + self.glo + self.ghi]
        oty_local = np.zeros(int(np.prod(m_local)))
        own = slice(self.glo * self.plane, (self.glo + self.nz) * self.plane)
        oty_local[own] = np.asarray(oty_owned, dtype=np.float64)
        w_local = None
        if w_owned is not None:   # ghost planes: never read as W (the operator is formed on owned nodes only)
            w_local = np.ones(int(np.prod(m_local)))
            w_local[own] = np.asarray(w_owned, dtype=np.float64)
        self.P = _Slab(m_local, oty_local, deltas, order, device, self.mg, self.zb, self.ze, self.glo, self.ghi,
                       w_local)
        self.ymean = float(ymean)

    def run(self, lam, rho0=None, fixed_iters=0, tol=1e-4, max_counter=3000, pcg_rtol=None, pcg_max_iter=None):
        """admm_update B from theta_0 = mean(y), u_0 = 0, rho_0 = lambda/5 (or rho0); collective. Stats dict."""
        o = _lib.default_opts(_lib.VARIANT_RCPP, fixed_iters=int(fixed_iters), tol=float(tol),
                              max_counter=int(max_counter), pcg_rtol=pcg_rtol, pcg_max_iter=pcg_max_iter)
        st = _lib.AdmmStats()
        r0 = lam / 5.0 if rho0 is None else float(rho0)
        s = _L().mvtv_slab_run(self.P._h, self.comm._h, _C.byref(o), float(lam), self.ymean, r0, _C.byref(st))
        if s not in (_lib.MVTV_OK, _lib.MVTV_MAXITER):
            _lib._check(s)
        return st.as_dict()

    def theta_owned(self):
        th, _, _ = self.P.state_get(want_u=False)
        return th[self.glo * self.plane:(self.glo + self.nz) * self.plane]

    def close(self):
        self.P.close()


def run_local_group(m, y, deltas, lam, world, device=0, w=None, theta0=None, **run_kw):
    """Rehearse a `world`-rank decomposition of one mesh in this process (loopback transport, one host thread
    per rank, every slab on `device`). ``w``: diag(W) over the mesh (O^T y = w y), None for W = I; ``theta0``:
    None for mean(y). Returns (stats of every rank, theta assembled from the owned planes)."""
    comms = Comm.local_group(world)
    b = plane_bounds(int(m[-1]), world)
    pl = int(np.prod(m[:-1]))
    y = np.asarray(y, dtype=np.float64)
    oty = y if w is None else np.asarray(w, dtype=np.float64) * y
    t0 = float(y.mean()) if theta0 is None else float(theta0)
    ranks = [SlabADMM(m, oty[b[r] * pl:b[r + 1] * pl], deltas, t0, comms[r], device=device,
                      w_owned=None if w is None else np.asarray(w, dtype=np.float64)[b[r] * pl:b[r + 1] * pl])
             for r in range(world)]
    out, err = [None] * world, [None] * world

    def work(r):
        try:
            out[r] = ranks[r].run(lam, **run_kw)
        except Exception as e:   # noqa: BLE001 (re-raised below)
            err[r] = e

    threads = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for e in err:
        if e is not None:
            raise e
    theta = np.concatenate([s.theta_owned() for s in ranks])
    for s in ranks:
        s.close()
    for c in comms:
        c.close()
    return out, theta
