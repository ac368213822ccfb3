"""One mesh decomposed over ranks: slab-parallel ADMM (SURVEY §8e, config 5 / the metric at 2-8 GPUs).

The mesh is cut along its slowest dimension (dim p-1, contiguous in the column-major layout):
rank r owns planes [z_r, z_{r+1}) plus one ghost plane below and above (mvtv_problem_create_slab).
Per ADMM iteration of the reference's variant B (rcpp-code/MultivarTV/src/solvers.cpp:110-133):

  theta-solve   spectral, exact (W = I): DCT along dims 0..p-2 on the owned planes (local),
                an all-to-all transpose so each rank holds full dim-(p-1) lines of 1/G of the
                (dims 0..p-2) lines, forward/divide/inverse along dim p-1, the transpose back,
                inverse DCT along dims p-2..0 (local);
  theta halo    first owned plane -> rank-1's upper ghost (D theta reads theta at z+1);
  edge update   on the owned planes; 4 partial sums;
  edge halo     last owned plane of every block -> rank+1's lower ghost (D^T reads z-1);
  gather        on the owned planes; 3 partial sums;
  all-reduce    the 7 sums (one collective), then every rank takes the same adapt_step /
                stopping decision (bit-identical inputs).

Transport: torch.distributed. With the "nccl" backend (RCCL over xGMI) the exchange buffers are
device tensors and the line chunks are transformed in place in the receive buffer; with "gloo"
they are host arrays staged through the library's device scratch (used by the CPU-driven tests
and single-GPU rehearsals with several ranks on one card). Every numerical step runs in libmvtv.
"""
from __future__ import annotations

import math
import os

import numpy as np

from . import _lib

_L = _lib.lib


class _Slab(_lib.Problem):
    """A Problem created with mvtv_problem_create_slab (same wrapper, different constructor)."""

    def __init__(self, m_local, oty_local, deltas, order, device, m_global, zb, ze, glo, ghi):
        import ctypes as C
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
        self._w = None
        d.oty = _lib._ptr(self._oty)
        d.wdiag = None
        d.device = device
        sd = SlabDesc()
        sd.m_global, sd.z_begin, sd.z_end, sd.ghost_lo, sd.ghost_hi = m_global, zb, ze, glo, ghi
        h = C.c_void_p()
        _lib._check(_L().mvtv_problem_create_slab(C.byref(d), C.byref(sd), C.byref(h)))
        self._h = h
        self.E = int(_L().mvtv_problem_edges(h))
        self.nb = int(_L().mvtv_problem_blocks(h))


import ctypes as _C  # noqa: E402


class SlabDesc(_C.Structure):
    _fields_ = [("m_global", _C.c_int64), ("z_begin", _C.c_int64), ("z_end", _C.c_int64),
                ("ghost_lo", _C.c_int32), ("ghost_hi", _C.c_int32)]


_dp = _C.POINTER(_C.c_double)
_lib.SIGNATURES.update({
    "mvtv_problem_create_slab": (_C.c_int, [_C.POINTER(_lib.ProblemDesc), _C.POINTER(SlabDesc), _C.POINTER(_C.c_void_p)]),
    "mvtv_slab_solve_fwd": (_C.c_int, [_C.c_void_p, _C.c_double, _C.c_double, _C.c_double]),
    "mvtv_slab_solve_mid": (_C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_int64, _C.c_int64, _C.c_double]),
    "mvtv_slab_solve_inv": (_C.c_int, [_C.c_void_p]),
    "mvtv_slab_init": (_C.c_int, [_C.c_void_p]),
    "mvtv_slab_edge": (_C.c_int, [_C.c_void_p, _C.c_int32, _C.c_double, _C.c_double, _C.c_double, _dp]),
    "mvtv_slab_gather": (_C.c_int, [_C.c_void_p, _C.c_int32, _C.c_double, _C.c_double, _dp]),
    "mvtv_copy2d": (_C.c_int, [_C.c_void_p, _C.c_int32, _C.c_int64, _C.c_int64, _C.c_int64, _C.c_int64, _C.c_int64,
                               _C.c_void_p, _C.c_int32]),
    "mvtv_scratch": (_C.c_void_p, [_C.c_void_p, _C.c_int64]),
    "mvtv_sync": (_C.c_int, [_C.c_void_p]),
})
if _lib._LIB is not None:   # library already loaded: register the new signatures
    for _n in ("mvtv_problem_create_slab", "mvtv_slab_solve_fwd", "mvtv_slab_solve_mid", "mvtv_slab_solve_inv",
               "mvtv_slab_init", "mvtv_slab_edge", "mvtv_slab_gather", "mvtv_copy2d", "mvtv_scratch", "mvtv_sync"):
        _f = getattr(_lib._LIB, _n)
        _f.restype, _f.argtypes = _lib.SIGNATURES[_n]

THETA, EDGES, SCRATCH = 0, 1, 2
U_EXPLICIT, U_FROM_Z = 0, 1


def plane_bounds(m_last: int, world: int):
    """Contiguous plane ranges, as even as possible (every rank owns at least one plane)."""
    if m_last < world:
        raise ValueError(f"{m_last} planes cannot be split over {world} ranks")
    return np.linspace(0, m_last, world + 1).round().astype(np.int64)


class _Transport:
    """Neighbour plane exchange, 7-value all-reduce and the all-to-all transpose over torch.distributed."""

    def __init__(self, dist, group, device):
        import torch
        self.torch, self.dist, self.group = torch, dist, group
        self.world = dist.get_world_size(group) if dist else 1
        self.rank = dist.get_rank(group) if dist else 0
        self.on_device = bool(dist) and dist.get_backend(group) == "nccl"
        self.dev = torch.device("cuda", device) if self.on_device else torch.device("cpu")

    def empty(self, n):
        return self.torch.empty(int(n), dtype=self.torch.float64, device=self.dev)

    def ptr(self, t):
        return _C.c_void_p(t.data_ptr())

    def sync(self):
        if self.on_device:
            self.torch.cuda.synchronize(self.dev)

    def exchange(self, sends, recvs):
        """sends / recvs: lists of (peer, tensor); matched point-to-point."""
        if not self.dist or (not sends and not recvs):
            return
        ops = [self.dist.P2POp(self.dist.isend, t, peer, self.group) for peer, t in sends]
        ops += [self.dist.P2POp(self.dist.irecv, t, peer, self.group) for peer, t in recvs]
        for w in self.dist.batch_isend_irecv(ops):
            w.wait()
        self.sync()

    def allreduce(self, vals):
        if not self.dist:
            return np.asarray(vals, dtype=np.float64)
        t = self.torch.tensor(np.asarray(vals, dtype=np.float64), device=self.dev)
        self.dist.all_reduce(t, group=self.group)
        return t.cpu().numpy()

    def alltoall(self, out, inp, out_splits, in_splits):
        if not self.dist:
            out.copy_(inp)
            return
        self.dist.all_to_all_single(out, inp, output_split_sizes=[int(v) for v in out_splits],
                                    input_split_sizes=[int(v) for v in in_splits], group=self.group)
        self.sync()


class SlabADMM:
    """Variant-B ADMM on this rank's slab of a mesh fit (W = I, power-of-two m_j, p >= 2).

    ``oty_owned``: O^T y on the owned planes (= y for lattice data). ``ymean``: the global mean
    of y (theta_0 = mean(y), rcpp…/solvers.cpp:207). Construction is collective.
    """

    def __init__(self, m, oty_owned, deltas, ymean, group=None, device=None, order=_lib.ORDER_CPP):
        try:
            import torch.distributed as dist
            dist = dist if (dist.is_available() and dist.is_initialized() and group is not False) else None
        except ImportError:
            dist = None
        self.m = [int(v) for v in m]
        p = len(self.m)
        if p < 2:
            raise ValueError("slab decomposition needs p >= 2")
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        self.T = _Transport(dist, None if group is False else group, device)
        G, r = self.T.world, self.T.rank
        self.G, self.r = G, r
        self.mg = self.m[-1]
        self.bounds = plane_bounds(self.mg, G)
        self.zb, self.ze = int(self.bounds[r]), int(self.bounds[r + 1])
        self.nz = self.ze - self.zb
        self.glo, self.ghi = int(self.zb > 0), int(self.ze < self.mg)
        self.plane = int(np.prod(self.m[:-1]))
        self.lines = self.plane
        if self.lines % G or (self.lines // G) & (self.lines // G - 1):
            raise ValueError("the (dims 0..p-2) line count must split into power-of-two chunks over the ranks")
        self.chunk = self.lines // G
        m_local = self.m[:-1] + [self.nz + self.glo + self.ghi]
        oty_local = np.zeros(int(np.prod(m_local)))
        oty_local[self.glo * self.plane:(self.glo + self.nz) * self.plane] = np.asarray(oty_owned, dtype=np.float64)
        self.P = _Slab(m_local, oty_local, deltas, order, device, self.mg, self.zb, self.ze, self.glo, self.ghi)
        self.N = float(np.prod(self.m))
        # global edge count E = sum over blocks of prod_j (m_j - [j in S'])
        self.E = 0.0
        for _, sp, _ in self.P.block_info():
            self.E += float(np.prod([mj - ((sp >> j) & 1) for j, mj in enumerate(self.m)]))
        self.ymean = float(ymean)
        nzs = np.diff(self.bounds)
        self.a2a_in = nzs[r] * self.chunk * np.ones(G, dtype=np.int64)     # to every rank: my planes x its chunk
        self.a2a_out = nzs * self.chunk                                       # from rank s: its planes x my chunk
        self.sendbuf = self.T.empty(self.nz * self.lines)
        self.linebuf = self.T.empty(self.mg * self.chunk)
        pl = self.plane
        self.gbuf = {k: self.T.empty(pl) for k in ("th_up_s", "th_up_r", "th_dn_s", "th_dn_r")}
        self.ebuf = {k: self.T.empty(self.P.nb * pl) for k in ("s", "r")}
        if not self.T.on_device:
            self.scratch = _L().mvtv_scratch(self.P._h, self.mg * self.chunk)
            if not self.scratch:
                raise MemoryError("mvtv_scratch")

    # ---- library <-> exchange buffers --------------------------------------------------------------
    def _copy(self, what, offset, rows, width, lib_pitch, ext_pitch, tensor, to_ext, ext_offset=0):
        ptr = _C.c_void_p(tensor.data_ptr() + 8 * int(ext_offset))
        _lib._check(_L().mvtv_copy2d(self.P._h, what, int(offset), int(rows), int(width), int(lib_pitch),
                                     int(ext_pitch), ptr, int(to_ext)))

    def _theta_halo(self, down=True):
        """Ghost planes of theta: upper ghost from rank+1 (always), lower ghost from rank-1 (down=True)."""
        pl, r, G = self.plane, self.r, self.G
        sends, recvs = [], []
        if r > 0:   # my first owned plane is rank-1's upper ghost
            self._copy(THETA, self.glo * pl, 1, pl, pl, pl, self.gbuf["th_up_s"], 1)
            sends.append((r - 1, self.gbuf["th_up_s"]))
        if r < G - 1:
            recvs.append((r + 1, self.gbuf["th_up_r"]))
        if down:
            if r < G - 1:   # my last owned plane is rank+1's lower ghost
                self._copy(THETA, (self.glo + self.nz - 1) * pl, 1, pl, pl, pl, self.gbuf["th_dn_s"], 1)
                sends.append((r + 1, self.gbuf["th_dn_s"]))
            if r > 0:
                recvs.append((r - 1, self.gbuf["th_dn_r"]))
        self.T.exchange(sends, recvs)
        if r < G - 1:
            self._copy(THETA, (self.glo + self.nz) * pl, 1, pl, pl, pl, self.gbuf["th_up_r"], 0)
        if down and r > 0:
            self._copy(THETA, 0, 1, pl, pl, pl, self.gbuf["th_dn_r"], 0)

    def _edge_halo(self):
        """Lower ghost plane of every edge block from rank-1 (D^T reads the anchors at z-1)."""
        pl, r, G, N, nb = self.plane, self.r, self.G, self.P.N, self.P.nb
        sends, recvs = [], []
        if r < G - 1:
            self._copy(EDGES, (self.glo + self.nz - 1) * pl, nb, pl, N, pl, self.ebuf["s"], 1)
            sends.append((r + 1, self.ebuf["s"]))
        if r > 0:
            recvs.append((r - 1, self.ebuf["r"]))
        self.T.exchange(sends, recvs)
        if r > 0:
            self._copy(EDGES, 0, nb, pl, N, pl, self.ebuf["r"], 0)

    def _solve(self, ca, cb, sigma):
        P, pl, G = self.P, self.plane, self.G
        _lib._check(_L().mvtv_slab_solve_fwd(P._h, ca, cb, sigma))
        # transpose: to rank s, my owned planes x its line chunk
        for s in range(G):
            self._copy(THETA, self.glo * pl + s * self.chunk, self.nz, self.chunk, pl, self.chunk, self.sendbuf, 1,
                       ext_offset=s * self.nz * self.chunk)
        self.T.alltoall(self.linebuf, self.sendbuf, self.a2a_out, self.a2a_in)
        q0 = self.r * self.chunk
        if self.T.on_device:
            _lib._check(_L().mvtv_slab_solve_mid(P._h, self.T.ptr(self.linebuf), q0, self.chunk, sigma))
        else:
            n = self.mg * self.chunk
            self._copy(SCRATCH, 0, 1, n, n, n, self.linebuf, 0)
            _lib._check(_L().mvtv_slab_solve_mid(P._h, _C.c_void_p(self.scratch), q0, self.chunk, sigma))
            self._copy(SCRATCH, 0, 1, n, n, n, self.linebuf, 1)
        self.T.alltoall(self.sendbuf, self.linebuf, self.a2a_in, self.a2a_out)
        for s in range(G):
            self._copy(THETA, self.glo * pl + s * self.chunk, self.nz, self.chunk, pl, self.chunk, self.sendbuf, 0,
                       ext_offset=s * self.nz * self.chunk)
        _lib._check(_L().mvtv_slab_solve_inv(P._h))

    def theta_owned(self):
        th, _, _ = self.P.state_get(want_u=False)
        return th[self.glo * self.plane:(self.glo + self.nz) * self.plane]

    def run(self, lam, rho0=None, fixed_iters=0, tol=1e-4, max_counter=3000, timer=None):
        """admm_update B from theta_0 = mean(y), u_0 = 0, rho_0 = lambda/5 (or rho0). Returns stats."""
        P = self.P
        rho = lam / 5.0 if rho0 is None else float(rho0)
        P.state_set(np.full(P.N, self.ymean), np.zeros(P.E), rho)
        self._theta_halo(down=True)
        _lib._check(_L().mvtv_slab_init(P._h))
        red3 = (_C.c_double * 3)()
        _lib._check(_L().mvtv_slab_gather(P._h, U_EXPLICIT, 0.0, 1.0, red3))
        mode, c_prev, t_z, sigma = U_EXPLICIT, 1.0, 0.0, rho
        dual = primal = 1.0
        eps_d = eps_p = tol
        counter, it, status = 1, 0, 0
        red4 = (_C.c_double * 4)()
        sqN, sqE = math.sqrt(self.N), math.sqrt(self.E)
        if timer:
            timer("start")
        while True:
            if fixed_iters > 0:
                if it >= fixed_iters:
                    break
            elif not (dual > eps_d or primal > eps_p):
                break
            self._solve(rho, rho * c_prev, sigma)
            self._theta_halo(down=False)
            t_new = lam / rho if rho != 0.0 else math.inf
            _lib._check(_L().mvtv_slab_edge(P._h, mode, t_z, c_prev, t_new, red4))
            self._edge_halo()
            _lib._check(_L().mvtv_slab_gather(P._h, U_FROM_Z, t_new, c_prev, red3))
            R = self.T.allreduce([red4[0], red4[1], red4[2], red3[0], red3[1], red3[2]])
            mode, t_z = U_FROM_Z, t_new
            it += 1
            counter += 1
            # rcpp-code/MultivarTV/src/solvers.cpp:117-125 (the library's host loop, mvtv_capi.cpp)
            dual = abs(rho) * math.sqrt(R[4])
            primal = math.sqrt(R[0])
            eps_d = tol * (sqN + math.sqrt(R[3]))
            eps_p = tol * (sqE + max(math.sqrt(R[1]), math.sqrt(R[2])))
            c_next, rho_next = 1.0, rho
            if primal > 10 * dual:
                rho_next, c_next = 2.0 * rho, 1.0 / 2.0
            elif dual > 10 * primal:
                rho_next, c_next = 1.0 / 2.0 * rho, 2.0
            c_prev, rho, sigma = c_next, rho_next, rho_next
            if fixed_iters <= 0 and counter > max_counter:
                status = 1
                break
        if timer:
            timer("stop")
        return {"iters": it, "rho": rho, "r_norm": primal, "s_norm": dual, "eps_pri": eps_p, "eps_dual": eps_d,
                "status": status}

    def close(self):
        self.P.close()
