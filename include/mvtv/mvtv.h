/*
 * mvtv.h — C ABI of the MI355X-native mesh-TV ADMM solver (libmvtv.so).
 *
 * This is the drop-in boundary for the reference's ADMM hot path. Every entry
 * point replaces one reference interface (cited as path:line under
 * /root/reference) and uses only plain pointers, sizes and PODs: no Armadillo,
 * Rcpp or torch types. Host buffers are caller-owned; device buffers are owned
 * by the opaque mvtv_problem handle (one handle per GPU; handles are
 * thread-safe with respect to each other, a single handle is not).
 *
 * Layouts (identical to the reference):
 *   theta  [N]  mesh values, column-major, dim 0 fastest (cpp-code/utils.cpp:40-52)
 *   u      [E]  scaled dual, blocks concatenated in the D row order of the
 *               caller (C++ create_D: all-ones block first; Python create_D:
 *               b = 1..), each block a column-major reduced grid
 *               (cpp-code/utils.cpp:103-134, 245-269; code/utils.py:138-149)
 *
 * Errors never cross the ABI as exceptions: every call returns mvtv_status and
 * leaves a message readable through mvtv_last_error() (thread-local).
 */
#ifndef MVTV_MVTV_H
#define MVTV_MVTV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVTV_MAX_DIMS 4
#define MVTV_MAX_BLOCKS 15

typedef enum mvtv_status {
    MVTV_OK = 0,
    MVTV_MAXITER = 1,        /* A: "Failed to converge!" (cpp-code/solvers.cpp:122-124); B: max_counter break (rcpp…/solvers.cpp:129-132) */
    MVTV_BAD_ARG = 2,
    MVTV_DIM_MISMATCH = 3,   /* reference's mixed-partial product fails for this mesh */
    MVTV_HIP_ERROR = 4,
    MVTV_NO_DEVICE = 5,
    MVTV_OUT_OF_MEMORY = 6,
    MVTV_PCG_NOT_CONVERGED = 7 /* only reported when opts.pcg_strict != 0 */
} mvtv_status;

/* Which reference implementation's ADMM semantics to follow. */
typedef enum mvtv_variant {
    MVTV_VARIANT_RCPP = 0,   /* B: rcpp-code/MultivarTV/src/solvers.cpp:96-136 (released package) */
    MVTV_VARIANT_CPP = 1,    /* A: cpp-code/solvers.cpp:90-130 (int rho, theta-change stop) */
    MVTV_VARIANT_PY = 2      /* C: code/solvers.py:53-76 (fixed rho = lambda, threshold 1) */
} mvtv_variant;

/* Row-block order of D. */
typedef enum mvtv_block_order {
    MVTV_ORDER_CPP = 0,      /* C++ create_D: [all-ones, w=1] + b=1..2^p-2 (cpp-code/utils.cpp:245-269) */
    MVTV_ORDER_PY = 1        /* Python create_D: b=1..2^p-1 unweighted, or b=1..2^p-2 weighted (code/utils.py:138-149) */
} mvtv_block_order;

/* Replaces the mbs_cache / mbs_one_inits bundles (rcpp…/solvers.hpp:30-50,
 * cpp-code/solvers.hpp:25-43): instead of sparse O, D, D^T D the problem is the
 * mesh shape, the block weights and the diagonal W = O^T O with O^T y. */
typedef struct mvtv_problem_desc {
    int32_t p;                       /* 1..4 dimensions */
    int64_t m[MVTV_MAX_DIMS];        /* mesh points per dimension (each >= 2) */
    int32_t block_order;             /* mvtv_block_order */
    int32_t weighted;                /* 1: w_b = prod_{j not in b} deltas_j; 0: every w = 1 */
    double deltas[MVTV_MAX_DIMS];    /* mesh widths (create_deltas, rcpp…/utils.cpp:256-263) */
    const double* oty;               /* [N] O^T y (required) */
    const double* wdiag;             /* [N] diag(O^T O), or NULL for W = I (mesh == data) */
    int32_t device;                  /* HIP device ordinal */
} mvtv_problem_desc;

typedef struct mvtv_admm_opts {
    int32_t variant;        /* mvtv_variant */
    double tol;             /* <= 0: variant default (B 1e-4 rcpp…/solvers.hpp:19; A 1e-3 cpp-code/solvers.hpp:14; C 1e-3) */
    int32_t max_counter;    /* <= 0: variant default (B 3000, A 2000, C 1000000 — the reference's C guard is dead) */
    int32_t fixed_iters;    /* > 0: run exactly this many iterations, stopping test disabled (trajectory / bench mode) */
    double sigma;           /* solve-matrix scalar W + sigma D^T D at entry; NaN: variant default (B rho, A lambda, C lambda) */
    double ymean;           /* mean(y): A and C initialise theta_old from it (cpp-code/solvers.cpp:103, code/solvers.py:63) */
    double pcg_rtol;        /* <= 0: 1e-10 (relative to ||b||) */
    int32_t pcg_max_iter;   /* <= 0: 20000 */
    int32_t pcg_strict;     /* != 0: report MVTV_PCG_NOT_CONVERGED when a theta-solve stops at pcg_max_iter */
    int32_t verbose;        /* != 0: print "Lambda= .., Counter = .." like rcpp…/solvers.cpp:134 */
    int32_t theta_solver;   /* mvtv_theta_solver: how spsolve(spcrosses, b) (rcpp…/solvers.cpp:113) is replaced */
} mvtv_admm_opts;

/* theta-solve of (W + sigma D^T D) theta = b. The reference factorises with SuperLU every
 * iteration (rcpp…/solvers.cpp:113, cpp-code/solvers.cpp:116, code/solvers.py:72). */
typedef enum mvtv_theta_solver {
    MVTV_SOLVER_AUTO = 0,      /* SPECTRAL where it is exact; else PCG_SPECTRAL on the same meshes; else PCG */
    MVTV_SOLVER_PCG = 1,       /* Jacobi-PCG on the 3^p-point stencil, warm-started, pcg_rtol */
    MVTV_SOLVER_SPECTRAL = 2,  /* direct: cosine transforms + a tridiagonal solve along the last dim. Exact for
                                  W = I (mesh == data) with every m_j <= 4096 (FFT plans for lengths with prime
                                  factors 2, 3, 5, 7, Bluestein's chirp-z for any other); MVTV_BAD_ARG otherwise */
    MVTV_SOLVER_PCG_SPECTRAL = 3 /* PCG preconditioned by S (mean(W) I + sigma D^T D) S, its middle factor inverted
                                  exactly by cosine transforms, S = I or a Jacobi-like diagonal scaling when W varies
                                  strongly against sigma D^T D's diagonal: for W != I (scattered data, CV folds) on
                                  the meshes SPECTRAL accepts */
} mvtv_theta_solver;

typedef struct mvtv_admm_stats {
    int32_t iters;          /* ADMM iterations executed */
    int32_t status;         /* mvtv_status of the run */
    double r_norm, s_norm;  /* last primal / dual residual norms */
    double eps_pri, eps_dual;
    double rho;             /* final rho (after the last adaptation) */
    double dtheta_max;      /* last max|theta - theta_old| (A, C) */
    int64_t pcg_iters;      /* total PCG iterations */
    int32_t pcg_iters_max;  /* max PCG iterations in one theta-solve */
    int32_t pcg_unconverged;/* theta-solves that hit pcg_max_iter */
    double seconds;         /* wall time of the call */
    int32_t theta_solver;   /* the solver that ran (MVTV_SOLVER_PCG or MVTV_SOLVER_SPECTRAL) */
} mvtv_admm_stats;

typedef struct mvtv_problem mvtv_problem;

/* ---- library -------------------------------------------------------------------- */
const char* mvtv_version(void);
const char* mvtv_status_string(int32_t status);
const char* mvtv_last_error(void);
int32_t mvtv_device_count(void);
void mvtv_default_opts(mvtv_admm_opts* opts, int32_t variant);

/* ---- problem (replaces create_cache_objects / fill_cache / use_cache,
 *      rcpp…/solvers.cpp:36-69; cpp-code/solvers.cpp:31-62) ------------------------ */
mvtv_status mvtv_problem_create(const mvtv_problem_desc* desc, mvtv_problem** out);
void mvtv_problem_destroy(mvtv_problem* prob);
int64_t mvtv_problem_nodes(const mvtv_problem* prob);   /* N = ntheta (rcpp…/solvers.hpp:36) */
int64_t mvtv_problem_edges(const mvtv_problem* prob);   /* E = rowsD (rcpp…/solvers.hpp:35) */
int32_t mvtv_problem_blocks(const mvtv_problem* prob);
/* block k's binary code, effective difference set S' (bit j = dim j) and weight */
mvtv_status mvtv_problem_block_info(const mvtv_problem* prob, int32_t k, int32_t* code, int32_t* sprime, double* weight);
/* new O^T y and W for the same mesh (CV folds re-run create_cache_objects, rcpp…/solvers.cpp:347-348) */
mvtv_status mvtv_problem_set_data(mvtv_problem* prob, const double* oty, const double* wdiag);
/* 1 if MVTV_SOLVER_SPECTRAL applies to this problem (W = I, every m_j <= 4096), else 0 */
int32_t mvtv_problem_spectral_ok(const mvtv_problem* prob);

/* ---- the hot path ------------------------------------------------------------------ */
/* Drop-in for admm_update:
 *   B: void admm_update(vec y, mbs_one_inits, vec& theta_init, double lambda, bool verbose,
 *                       vec& u_init, double& rho_init, admm_out&)   rcpp…/solvers.hpp:100
 *   A: vec admm_update(vec y, mbs_one_inits, vec* theta_init, double lambda)  cpp-code/solvers.hpp:85
 *   C: the while-loop of mbs_one                                     code/solvers.py:53-76
 * theta_inout [N]: theta_init in, theta out. u_inout [E]: u_init in / u out, or NULL for the
 * variant's own u0 (B 0, A and C 1/lambda) with u not returned. rho_inout: rho_init in /
 * rho out (B; A and C derive rho from lambda and return the final one). */
mvtv_status mvtv_admm(mvtv_problem* prob, const mvtv_admm_opts* opts, double lambda,
                      double* theta_inout, double* u_inout, double* rho_inout, mvtv_admm_stats* stats);

/* Resident form of the same loop for callers that keep the state in HBM across calls
 * (lambda paths with warm start rcpp…/solvers.cpp:212-220, benchmarks). */
mvtv_status mvtv_state_set(mvtv_problem* prob, const double* theta, const double* u, double rho);
mvtv_status mvtv_state_get(mvtv_problem* prob, double* theta, double* u, double* rho);
mvtv_status mvtv_admm_run(mvtv_problem* prob, const mvtv_admm_opts* opts, double lambda, mvtv_admm_stats* stats);
/* mbs_path's lambda loop (rcpp…/solvers.cpp:204-222) in one call: from theta_init [N], the variant's
 * u0 and rho_init, the ADMM state (theta, u, rho) is carried on the device from each lambda to the
 * next (:217-219). thetas_out [n_lambda x N] (may be NULL): theta after each lambda, lambda-major.
 * rhos_out, stats [n_lambda] (may be NULL). The state stays resident (mvtv_state_get reads the last).
 * Returns MVTV_MAXITER when some lambda hit max_counter (the loop goes on, as B breaks and goes on). */
mvtv_status mvtv_path(mvtv_problem* prob, const mvtv_admm_opts* opts, const double* lambdas, int32_t n_lambda,
                      const double* theta_init, double rho_init, double* thetas_out, double* rhos_out,
                      mvtv_admm_stats* stats);
/* fitted values O theta for n points given their mesh index (fill_output_mbs_one, rcpp…/solvers.cpp:73) */
mvtv_status mvtv_fitted(mvtv_problem* prob, const int64_t* mesh_index, int64_t n, double* fitted);

/* ---- scattered data on the device ----------------------------------------------------
 * axes: the mesh's sorted axis values, m[0] values of dim 0, then m[1] of dim 1, ... (the linspace
 * axes of create_mesh, rcpp…/utils.cpp:234-254; mesh rows in column-major order). data: n x p,
 * column-major (arma::mat). mesh_index_out [n] (may be NULL): the column-major mesh node of each
 * point, i.e. the column of the 1 in row i of O. */
/* nearest1 / nearest_interp_matrix (rcpp…/utils.cpp:267-304): first nearest mesh row per point */
mvtv_status mvtv_nearest(mvtv_problem* prob, const double* axes, const double* data, int64_t n,
                         int64_t* mesh_index_out);
/* create_cache_objects (rcpp…/solvers.cpp:36-44) on the device: O from mvtv_nearest, then
 * W = diag(O^T O) and O^T y (summed per node in data order) installed as the problem's data, as by
 * mvtv_problem_set_data (W = I when every node holds exactly one point). */
mvtv_status mvtv_problem_set_scattered(mvtv_problem* prob, const double* axes, const double* data, int64_t n,
                                       const double* y, int64_t* mesh_index_out);
/* mbs_predict (rcpp…/solvers.cpp:161-165): O(data) theta of the resident state, fits [n] */
mvtv_status mvtv_predict(mvtv_problem* prob, const double* axes, const double* data, int64_t n, double* fits);

/* ---- operators (inits.D*theta, inits.Dt*v, spcrosses*x, spsolve(spcrosses, b):
 *      rcpp…/solvers.cpp:112-126) ----------------------------------------------------- */
mvtv_status mvtv_apply_D(mvtv_problem* prob, const double* theta, double* d_out);        /* [N] -> [E] */
mvtv_status mvtv_apply_Dt(mvtv_problem* prob, const double* v, double* g_out);           /* [E] -> [N] */
mvtv_status mvtv_apply_A(mvtv_problem* prob, double sigma, const double* x, double* q_out); /* (W + sigma D^T D) x */
mvtv_status mvtv_solve(mvtv_problem* prob, double sigma, const double* b, double* x_inout,
                       double rtol, int32_t max_iter, int32_t* iters, double* relres);
/* lam_max_pinv (rcpp…/utils.cpp:306-355, called by create_lambdas rcpp…/solvers.cpp:186-200):
 * 5 ||D x||_inf with x from the reference's CG on D^T D x = O^T y (relative stop 1e-4, at most
 * min(N, 2000) iterations), its recurrences reproduced step by step on the GPU. */
mvtv_status mvtv_lambda_max(mvtv_problem* prob, double* out, int32_t* iters);
/* lam_max_pinv of variant A (cpp-code/utils.cpp:354-404, called by create_lambdas cpp-code/solvers.cpp:
 * 179-192): ||D x||_inf with x from cg(D^T D, O^T y): x0 = mean(O^T y), absolute stop ||r|| < 0.01, at most
 * 500 iterations (N < 400) or 100 */
mvtv_status mvtv_lambda_max_cpp(mvtv_problem* prob, double* out, int32_t* iters);
/* direct theta-solve (I + sigma D^T D) x = b by cosine transforms (MVTV_SOLVER_SPECTRAL) */
mvtv_status mvtv_solve_spectral(mvtv_problem* prob, double sigma, const double* b, double* x_out);

/* ---- slab decomposition of one mesh over ranks (the metric at 2-8 GPUs) ---------
 * Rank r holds planes [z_begin, z_end) of the last dimension plus one ghost plane below (unless
 * z_begin = 0) and above (unless z_end = m_global); desc->m[p-1] counts owned + ghost planes and
 * desc->oty (and desc->wdiag, if any) cover them (ghost values are not used). Rank r owns planes
 * [floor(m r / G), floor(m (r+1) / G)). mvtv_slab_run is the whole variant-B loop of one rank
 * (rcpp…/solvers.cpp:110-133) with its collectives on a communication stream: the substructured line solves'
 * two all-to-alls of 2 and 2 numbers per line (each block's two recursion sums, then its two carries), halo
 * planes of theta and of the edge state, one 7-value all-reduce per iteration feeding the device-side
 * adapt_step / stopping decision. With W != I (desc->wdiag)
 * the theta-solve is PCG with the spectral preconditioner of mean(W) I + sigma D^T D (opts pcg_rtol,
 * pcg_max_iter, pcg_strict as mvtv_admm_run), distributed: a halo of the search direction per iteration and
 * one all-reduce per dot product; the loop then polls once per ADMM iteration. Supported: variant B, W = I
 * or diagonal, u0 = 0, m_j <= 4096 for j < p - 1; the last dimension any length when G >= 2 (its line solves
 * are substructured over the ranks; each rank's plane count must be 1..64 segments of <= 32 rows, e.g. any
 * count <= 64 or with a divisor in 2..32 giving <= 64 segments: checked on every rank before the first
 * collective, MVTV_BAD_ARG on all of them otherwise), <= 4096 when G = 1. */
typedef struct mvtv_slab_desc {
    int64_t m_global;          /* planes of dim p-1 in the whole mesh */
    int64_t z_begin, z_end;    /* owned planes */
    int32_t ghost_lo, ghost_hi;
} mvtv_slab_desc;
typedef struct mvtv_comm mvtv_comm;
mvtv_status mvtv_problem_create_slab(const mvtv_problem_desc* desc, const mvtv_slab_desc* slab, mvtv_problem** out);
/* RCCL transport (one process per GPU): rank 0 makes the id, every rank passes the same 128 bytes. The first
 * mvtv_slab_run on a communicator with MVTV_RCCL_SPLIT=1 splits off a second RCCL communicator (ncclCommSplit,
 * collective) for the halos, so they can run beside the critical-path collectives issued on the problem's stream; the
 * ranks all-reduce the split's outcome before use and all keep one communicator unless every split succeeded.
 * Without it (the default) every collective goes on the communication stream. */
mvtv_status mvtv_comm_unique_id(uint8_t* id128);
mvtv_status mvtv_comm_create_rccl(const uint8_t* id128, int32_t nranks, int32_t rank, int32_t device, mvtv_comm** out);
/* in-process loopback group of nranks handles (comms[0..nranks-1]): each rank's mvtv_slab_run on its own
 * host thread, transfers as device copies (rehearsal of the decomposition on one GPU) */
mvtv_status mvtv_comm_create_local(int32_t nranks, mvtv_comm** comms);
/* inter-process group over HIP IPC memory (one process per rank; the ranks' devices one GPU or peers of one
 * node): transfers are device-to-device copies out of the sender's buffer (hipIpcOpenMemHandle), ordered through
 * a POSIX shared-memory rendezvous segment `name` ("/..."; rank 0 creates it, every rank passes the same name,
 * it is unlinked once all nranks <= 16 have attached). Host-synchronous inside each collective (no overlap of
 * the z halo): the multi-process path without RCCL, e.g. several ranks on one GPU, where RCCL refuses. Waits give
 * up after MVTV_IPC_TIMEOUT seconds (default 300) or when a peer's loop failed. */
mvtv_status mvtv_comm_create_ipc(const char* name, int32_t nranks, int32_t rank, int32_t device, mvtv_comm** out);
void mvtv_comm_destroy(mvtv_comm* comm);
int32_t mvtv_comm_rank(const mvtv_comm* comm);
int32_t mvtv_comm_size(const mvtv_comm* comm);
/* sum of n <= 64 host doubles over an RCCL or ipc communicator, in place (the global residual all-reduce of
 * independent fits); blocking */
mvtv_status mvtv_comm_allreduce_host(mvtv_comm* comm, double* vals, int32_t n);
/* the file RCCL was resolved from (ROCm's librccl, which shares libmvtv's HIP runtime); "" when RCCL is
 * unavailable */
const char* mvtv_comm_library(void);
/* admm_update B from theta = theta0 on every node, u = 0, rho = rho0 (rcpp…/solvers.cpp:207-209); collective
 * over the communicator. stats hold the global norms; theta of the owned planes: mvtv_state_get (ghosts
 * included, planes as desc->m) */
mvtv_status mvtv_slab_run(mvtv_problem* prob, mvtv_comm* comm, const mvtv_admm_opts* opts, double lambda,
                          double theta0, double rho0, mvtv_admm_stats* stats);
mvtv_status mvtv_sync(mvtv_problem* prob);

/* ---- instrumentation (HIP events on the solver's stream) ---------------------------- */
typedef enum mvtv_kernel_id {
    MVTV_K_EDGE_UPDATE = 0,   /* D theta, soft-threshold, dual update, |r|,|D theta|,|alpha| */
    MVTV_K_GATHER = 1,        /* D^T alpha, D^T u and the dual-residual norms */
    MVTV_K_PCG_INIT = 2,      /* b and r0 = b - A theta */
    MVTV_K_PCG_APPLY = 3,     /* q = A p, p.q */
    MVTV_K_PCG_UPDATE = 4,    /* x += a p, r -= a q, r.z */
    MVTV_K_PCG_DIRECTION = 5, /* p = z + b p */
    MVTV_K_REDUCE = 6,        /* partial-sum finalisation / PCG scalars */
    MVTV_K_OTHER = 7,
    MVTV_K_PCG_FUSED = 8,     /* 3-D fused Chronopoulos-Gear iteration: p, A p, r, A M^-1 r, x in one pass */
    MVTV_K_DCT_FIRST = 9,     /* spectral solve, first pass: b formed on load, DCT along dim 0 */
    MVTV_K_DCT = 10,          /* spectral solve, other passes (DCT / divide / inverse DCT along one dim) */
    MVTV_K_ADMM_FUSED = 11,   /* 3-D: edge update + D^T gather in one pass over the edge state */
    MVTV_K_GATHER4B = 12,     /* 4-D two-pass gather, second pass (the first is MVTV_K_GATHER) */
    MVTV_K_DCT_FOLD = 13,     /* spectral solve, first pass from the folded s (b = oty + s; + D^T u after a rho change) */
    MVTV_K_ADMM_FUSED4 = 14,  /* 4-D: edge update + the gather's first pass in one pass over the edge state */
    MVTV_K_COUNT = 15
} mvtv_kernel_id;
mvtv_status mvtv_timing_enable(mvtv_problem* prob, int32_t on);
mvtv_status mvtv_timing_get(mvtv_problem* prob, int32_t kernel_id, double* total_ms, int64_t* launches,
                            double* bytes_per_launch);
const char* mvtv_kernel_name(int32_t kernel_id);

#ifdef __cplusplus
}
#endif
#endif /* MVTV_MVTV_H */
