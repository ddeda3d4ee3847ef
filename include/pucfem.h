/*
 * pucfem.h -- C ABI of libpucfem.so, the MI355X (gfx950) hot path of the
 * PUC-Fluidsimulation-Project Stokes/squirmer time-stepping core.
 *
 * The reference (TobiasHoffmannP/PUC-Fluidsimulation-Project, pure Python/NumPy)
 * has no FFI layer: its de-facto interface is a set of module-level functions plus
 * the np.linalg.solve call sites.  Each entry point below names the
 * reference code it replaces (file:line into /root/reference).  The Python host
 * (puc-fluidsimulation-project_amd/_lib.py) binds these with ctypes; INTEGRATION.md
 * shows the binding.
 *
 * Conventions
 *   - Every function returns int: 0 = ok, < 0 = error (PUCFEM_E*); the message is in
 *     pucfem_last_error(ctx) (or pucfem_last_error(NULL) for context-free calls).
 *   - Plain pointers and sizes only.  The library COPIES every input buffer; the caller
 *     keeps ownership.  Output buffers are caller-allocated.
 *   - Node / triangle numbering at the ABI is always the CALLER's (reference) numbering,
 *     0-based.  The library renumbers internally for locality and partitioning.
 *   - A context is bound to one HIP device (or none: device = PUCFEM_HOST_ONLY builds the
 *     host-side operators only, for CPU tests) and is NOT thread-safe.  Calls are
 *     synchronous at the ABI level; device streams are internal.
 *   - fp64 throughout, except the fp32-coordinate assembly of poisson.py / heatEq.py
 *     (poisson.py:40, :100-146), reproduced bit-for-bit on the host.
 */
#ifndef PUCFEM_H
#define PUCFEM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PUCFEM_ABI_VERSION 1
#define PUCFEM_HOST_ONLY (-1)
#define PUCFEM_UNIQUE_ID_BYTES 128

enum pucfem_status {
  PUCFEM_OK = 0,
  PUCFEM_EINVAL = -1,   /* bad argument / shape */
  PUCFEM_EHIP = -2,     /* HIP runtime error (no device, launch failure, ...) */
  PUCFEM_ENOCONV = -3,  /* iterative solver hit maxit without reaching rtol */
  PUCFEM_ESTATE = -4,   /* call out of order (e.g. step before build) */
  PUCFEM_ENCCL = -5,    /* RCCL error */
  PUCFEM_ENOMEM = -6,
  PUCFEM_ENODEV = -7    /* compute call on a host-only context */
};

/* which reference script's step loop the context runs */
enum pucfem_scheme {
  PUCFEM_STOKES_COLOR = 0, /* StokesColor.py:537-586  (Stokes + semi-Lagrangian dye) */
  PUCFEM_STOKES_FOOD = 1,  /* StokesFood.py:441-505   (Stokes + tracer capture)     */
  PUCFEM_HEAT = 2,         /* heatEq.py:304-325       (backward-Euler diffusion)    */
  PUCFEM_POISSON = 3       /* poisson.py:218-285      (steady Poisson)              */
};

typedef struct pucfem_params {
  int32_t scheme;      /* enum pucfem_scheme */
  int32_t nstrips;     /* y-strips of the node ordering / partition; 0 = auto */
  double dt;           /* DT  (StokesColor.py:43, StokesFood.py:42, heatEq.py:304) */
  double nu;           /* v   (kinematic viscosity, StokesColor.py:39) */
  double rtol_visc;    /* CG rtol, viscous solve  (replaces LU at StokesColor.py:544-545) */
  double rtol_pres;    /* CG rtol, pressure solve (replaces LU at StokesColor.py:555,569) */
  double rtol_lin;     /* BiCGStab rtol, heat / Poisson literal operators */
  int32_t maxit_visc, maxit_pres, maxit_lin;
  int32_t warm_start;  /* 1: start each solve from the previous step's solution */
  int32_t sl_k;        /* PointLocator k (StokesColor.py:324), 10 */
  double capture_radius; /* StokesFood.py:50-51, 0.28 */
  double center_x, center_y; /* squirmer centre (0.5, 0.5) */
  int32_t precond;     /* pressure solve: 0 = Jacobi-CG, 1 = geometric-multigrid-preconditioned CG
                          (needs pucfem_set_hierarchy) */
  int32_t mg_degree;   /* Chebyshev smoothing steps per level, pre and post (2) */
  double mg_ratio;     /* Chebyshev interval [lmax / mg_ratio, lmax] (10) */
  int32_t mg_post;     /* post-smoothing steps (0: same as mg_degree) */
  int32_t mg_single;   /* 1: fp32 V-cycle (values, vectors, halos) inside the fp64 CG */
  int64_t mg_rep_nodes; /* multi-rank: coarse levels up to this many nodes are replicated (0: 1000000) */
  int32_t mg_f32_vals; /* fp32 cycle: 0 = level operators stored in fp16 when every value is representable
                          (arithmetic stays fp32), 1 = all stored in fp32, 2 = the finest in fp32 and
                          the coarser levels in fp16 */
  int32_t idx32;       /* 0 = int16 column deltas for square operators whose band fits, 1 = int32 columns */
  int32_t proj_k;      /* pressure solves (multigrid path): initial guess = A-orthogonal projection onto a
                          basis of up to proj_k directions spanning the recent solutions of the same solve
                          (Fischer 1998, deferred basis update, re-seeded when full; 3..32, 0 = off: warm
                          start from the previous solution) */
  int32_t proj_k_visc; /* the same for the two components of the viscous solve (0 = off: warm start u^n
                          plus an extrapolation of the last viscous increments) */
  int32_t mg_kind;     /* smoother polynomial: 0/1 = Chebyshev (first kind) on [lmax / mg_ratio, lmax],
                          4 = Chebyshev of the fourth kind on [0, lmax] (Lottes 2022; no mg_ratio) */
  int32_t solver_path; /* 0 = auto; 1 = multi-kernel iterative solves on every mesh (no dense inverses and no
                          one-workgroup CG on small meshes: the large-mesh code path, for parity tests) */
  int32_t assembled;   /* 0 = auto: with a multigrid hierarchy of >= 2 levels, the rows of nodes inside the
                          coarse mesh's triangles are matrix-free lattice stencils (per-face constants) and only
                          the nodes on coarse edges / vertices keep stored SELL rows; 1 = stored SELL operators
                          for every row */
  int32_t dye_scheme;  /* STOKES_COLOR dye update: 0 = semi-Lagrangian (StokesColor.py:347-389); 1 = implicit
                          FEM advection-diffusion (scripts/good_visualization.py:700-718: consistent mass +
                          convection + diffusion, the periodic penalty restated as its exact merged limit,
                          BiCGStab); single rank */
  double dye_diffusivity; /* D of the implicit variant (good_visualization.py:404: 1e-3) */
  int32_t assembly;    /* 0 = auto: on a context bound to a device, the node-triangle incidence, the stiffness
                          pattern and the K / Gx / Gy / lumped-mass values of every level (buildStiffnessMatrix,
                          buildLumpedMassMatrix and the divergence / gradient coefficients, StokesColor.py:98-128,
                          130-284) are assembled on the device, bit-identical to the host assembly; 1 = host C++ */
  int32_t proj_shared; /* 1 = the two pressure solves of a step project onto ONE basis of up to proj_k
                          directions that collects the solutions of both (the same merged operator: one
                          A-orthonormal basis serves both); 0 = a basis per solve */
} pucfem_params;

/* per-step diagnostics, the values the reference prints (StokesColor.py:586, StokesFood.py:505) */
typedef struct pucfem_step_stats {
  double max_div_star;   /* max |div u*|          */
  double max_final_div;  /* max |div u^{n+1}|     */
  double mix_I, mix_mu, mix_var; /* mixing_index (StokesColor.py:391-403) over marker==0 */
  int64_t eaten;         /* StokesFood: sum(tracer_status) */
  int32_t it_visc, it_p, it_p2; /* CG iterations of the three solves */
  int32_t sl_notfound;   /* nodes that kept c[n] because PointLocator.find returned None */
} pucfem_step_stats;

/* fields exchanged with pucfem_set_field / pucfem_get_field (reference numbering) */
enum pucfem_field {
  PUCFEM_F_U = 0,         /* u      (N,2) row-major */
  PUCFEM_F_USTAR = 1,     /* u_star (N,2) */
  PUCFEM_F_P = 2,         /* p      (N)   zero-mean gauge */
  PUCFEM_F_P2 = 3,        /* p2     (N) */
  PUCFEM_F_DIV_STAR = 4,  /* div_u_star (N) */
  PUCFEM_F_DIV_U = 5,     /* div_u      (N) (before the 2nd projection) */
  PUCFEM_F_FINAL_DIV = 6, /* final_div  (N) */
  PUCFEM_F_C = 7,         /* dye c  (N) */
  PUCFEM_F_SCALAR = 8,    /* heat u / Poisson f (N) */
  PUCFEM_F_TRACERS = 9,   /* tracer_points (n_tr,2); set_field defines n_tr */
  PUCFEM_F_STATUS = 10    /* tracer_status (n_tr) as 0.0 / 1.0 */
};

/* operators for pucfem_apply / pucfem_solve / pucfem_host_get_csr */
enum pucfem_op {
  PUCFEM_OP_K = 0,      /* stiffness K (StokesColor.py:98-128), y = K x */
  PUCFEM_OP_VISC = 1,   /* A_visc (StokesColor.py:471-475) */
  PUCFEM_OP_PRES = 2,   /* periodic-merged pressure operator P^T K P (+ identity slave rows) */
  PUCFEM_OP_GX = 3,     /* lumped gradient coefficients (StokesColor.py:224-263), x-part */
  PUCFEM_OP_GY = 4,
  PUCFEM_OP_DIV = 5,    /* calculate_divergence (StokesColor.py:130-165): x = u (N,2), y = div (N) */
  PUCFEM_OP_GRAD = 6,   /* calculate_gradiant  (StokesColor.py:224-263): x = p (N), y = (N,2) */
  PUCFEM_OP_LIT = 7,    /* literal heat operator I + DT*A (heatEq.py:305) or Poisson A (poisson.py:253-278) */
  PUCFEM_OP_MCONS = 8,  /* consistent mass of the implicit dye variant (StokesColor.py:286-312; host CSR only) */
  PUCFEM_OP_MLUMP = 9,  /* lumped mass M (StokesColor.py:266-284) as a diagonal (host CSR only) */
  PUCFEM_OP_ASUM = 10   /* area_sum of calculate_divergence (StokesColor.py:151-163) as a diagonal (host CSR only) */
};

/* ---- library / context ---------------------------------------------------------- */
int pucfem_abi_version(void);
const char* pucfem_last_error(const void* ctx);
int pucfem_device_count(int32_t* n);
int pucfem_ctx_create(int32_t device, void** out_ctx);
/* multi-GPU: one process per GPU; rank/world from torch.distributed, unique id from
   rank 0's pucfem_rccl_unique_id broadcast over the control plane. */
int pucfem_rccl_unique_id(uint8_t* out_id /* PUCFEM_UNIQUE_ID_BYTES */);
int pucfem_ctx_create_dist(int32_t device, int32_t rank, int32_t world, const uint8_t* unique_id,
                           void** out_ctx);
/* world = 1 with a real unique id creates an RCCL communicator of one rank: the context then runs the
   multi-rank data path (all-reduced dots, broadcasts, the dye range exchange) through RCCL on one GPU.
   A unique id that starts with the 16 bytes "PUCFEM-LOCALCOMM" selects the in-process test backend:
   `world` contexts created from host threads of ONE process exchange data with device-to-device
   copies instead of RCCL (multi-rank validation on a one-GPU machine). */
int pucfem_ctx_destroy(void* ctx);

/* ---- mesh + boundary conditions (replaces readNode/readEle globals, StokesColor.py:437-464) */
int pucfem_mesh_upload(void* ctx, int64_t n_nodes, const double* xy /* N x 2 */,
                       const int32_t* markers, int64_t n_tris, const int32_t* tris /* T x 3 */,
                       int32_t coord_fp32 /* 1: poisson/heat fp32 coordinates (poisson.py:40) */);
/* periodic pairs (master, slave):
   kind 0 = operator pairs: filtered pairs of StokesColor.py:449-457 / poisson.py:242-253
   kind 1 = BC-copy pairs: makePerBCU (StokesColor.py:429-431) / reapply_periodic_u (heatEq.py:298-301,
            UNFILTERED).  Sequential semantics (u[s] = u[m] in list order) are preserved. */
int pucfem_set_pairs(void* ctx, int32_t kind, int64_t n_pairs, const int64_t* pairs /* P x 2 */);
/* Dirichlet nodes and values, applied in list order (makeDirBCU StokesColor.py:405-427,
   reapply_dirchlect_u heatEq.py:282-295, Dirichlet rows poisson.py:258-278). ncomp = 2 (Stokes) or 1. */
int pucfem_set_dirichlet(void* ctx, int64_t n, const int32_t* nodes, const double* values, int32_t ncomp);
/* Poisson load g(centroid) per triangle, evaluated by the host in the reference's dtype
   (poisson.py:135-144, g = 50 sin(3y) in fp32). */
int pucfem_set_source(void* ctx, int64_t n_tris, const float* g_tri);
/* Multigrid hierarchy: the uploaded mesh must be `levels` red refinements (pucfem_refine) of this
   coarse mesh; the library rebuilds the intermediate levels and checks the result bit for bit. */
int pucfem_set_hierarchy(void* ctx, int64_t n_nodes0, const double* xy0, const int32_t* markers0,
                         int64_t n_tris0, const int32_t* tris0, int32_t levels);
int pucfem_build_operators(void* ctx, const pucfem_params* params);

/* ---- fields ---------------------------------------------------------------------- */
int pucfem_set_field(void* ctx, int32_t field, const double* buf, int64_t count);
int pucfem_get_field(void* ctx, int32_t field, double* buf, int64_t count);

/* ---- time stepping: nsteps iterations of the scheme's loop body ------------------- */
/* Within one call, single-rank StokesColor with the semi-Lagrangian dye runs each step's dye tail
   (final divergence, advection, mixing sums) on a second stream overlapped with the next step's
   solves (PUCFEM_SL_OVERLAP=0: one stream); the call returns with all of it complete, so fields and
   stats read afterwards are those of the last step, as with one stream. */
int pucfem_step(void* ctx, int32_t nsteps, pucfem_step_stats* stats /* nsteps entries or NULL */);

/* ---- unit operations (reference-named shims and parity tests) --------------------- */
int pucfem_apply(void* ctx, int32_t op, const double* x, double* y);
/* op VISC: b,x are (N,2) (both velocity components, StokesColor.py:544-545);
   op PRES: b = b_p (N) as formed at StokesColor.py:554, x = zero-mean p;
   op LIT : heat / Poisson literal system. */
int pucfem_solve(void* ctx, int32_t op, const double* b, double* x, double rtol, int32_t maxit,
                 int32_t* iters);
/* advect_semilagrange (StokesColor.py:347-389): c_out = SL(c, u, dt); notfound may be NULL */
int pucfem_sl_advect(void* ctx, const double* c, const double* u, double dt, double* c_out,
                     int32_t* notfound);
/* tracer step (StokesFood.py:482-499) on the tracers held in the context, with u given */
int pucfem_tracer_step(void* ctx, const double* u, double dt, int32_t nsteps);
/* makePerBCU / makeDirBCU (StokesColor.py:405-431) on a host velocity u (N,2), in place, through the
   device's boundary kernels: which bit 0 = makePerBCU (slave <- master copies), bit 1 = makeDirBCU
   (walls and squirmer surface); both: the periodic copies first, as the step applies them.
   Single-rank Stokes contexts; the step's state is not touched (scratch buffers). */
int pucfem_apply_bc(void* ctx, int32_t which, double* u);
/* One implicit FEM dye step (scripts/good_visualization.py:700-718) on a context built with
   dye_scheme = 1: c_out = A^-1 (M c) with A = M + dt (C_u + D K) + diag(dt M_lumped div u), periodic
   pairs merged, then c[slave] = c[master]; c, c_out (N), u (N,2) in caller order; iters: BiCGStab
   iterations (may be NULL).  The step's state is not touched. */
int pucfem_dye_step(void* ctx, const double* c, const double* u, double* c_out, int32_t* iters);
/* mixing_index (StokesColor.py:391-403) over marker==0 nodes: out = (I, mu, var) */
int pucfem_mixing_index(void* ctx, const double* c, double* out3);
/* mixing_index(c, mass, mask) (StokesColor.py:391-403) with arbitrary node weights w (N, caller order): the
   reference's c[mask], mass[mask] is w = mass on the mask and 0 elsewhere (repeated mask entries count
   repeatedly); out = (I, mu, var) */
int pucfem_mixing_index_w(void* ctx, const double* c, const double* w, double* out3);

/* ---- measurement ------------------------------------------------------------------ */
/* HIP-event timing of each kernel class (bench.py roofline): the events are taken by each launch's own
   dispatch, on the stream the kernel runs on.  on: 0 off, 1 every class, 2 every class but 5-7 (the
   classes with a share of the step; the roofline kernel is the largest of them) */
int pucfem_timing_enable(void* ctx, int32_t on);
/* kernel classes: 0 = multigrid Chebyshev smoother on the finest level (k_cheb), 1 = CG SpMV+direction
   (k_cg_dir), 2 = CG update (k_cg_upd), 3 = gradient projection (k_grad_proj), 4 = semi-Lagrangian (k_sl),
   5 = multigrid residual on the finest level (k_resid), 6 = restriction from the finest level,
   7 = prolongation to the finest level (k_transfer), 8 = the semi-Lagrangian second pass (k_sl_slow: general
   locate and rank count of the rows off the lattice fast path), 9 = the viscous Chebyshev step over the whole
   grid (k_vcheb), 10 = two finest-level smoothing steps (k_cheb_pair), 11 = divergence (k_div), 12 = two
   viscous Chebyshev steps on the face rows (k_vcheb_pair), 13 = viscous right-hand side and warm start
   (k_visc_prep), 14 / 15 = the pressure projection's multi-dot and combination passes (k_mdot2, k_pcomb) */
int pucfem_timing_get(void* ctx, int32_t kclass, double* total_ms, int64_t* launches,
                      double* bytes_per_launch);
int pucfem_sync(void* ctx);
/* cumulative launches and algorithmic bytes of one kernel class (the classes of pucfem_timing_get) over EVERY
   launch since the context's creation, timed or not (launches of a solve after its convergence, which do no
   work, are taken back): with the timed launches' rate, bench.py weighs the classes over the whole timed
   window.  Measurement only. */
int pucfem_class_counters(void* ctx, int32_t kclass, int64_t* launches, double* bytes);
/* cumulative counters of the calling thread / context since its creation (bench.py's step roofline):
   launches = kernel launches issued by this thread through the library; bytes = the algorithmic bytes of
   the context's launched kernels (each vector counted once per row it is read or written, stored operators
   per entry; kernels launched after their solve had converged, which do no work, are not counted) --
   the HBM floor of the work the steps did.  Replaces nothing in the reference (measurement only). */
int pucfem_counters(void* ctx, int64_t* launches, double* bytes);
/* micro-benchmark of the pressure CG's SpMV + direction kernel (k_cg_dir; the round-1 roofline kernel,
   kept for A/B measurements) on the pressure operator: variant 0 plain loop, 1 unrolled, 2 non-temporal,
   3 unrolled + non-temporal; average ms/launch */
int pucfem_bench_dir(void* ctx, int32_t variant, int32_t nblocks, int32_t iters, double* ms_out);
/* timing of one kernel on the context's finest-level data (bench.py's roofline cross-check):
   kernel 0 = k_cheb general step (fp32 V-cycle), 1 = k_resid, 2 = k_cg_dir<1> of the pressure CG.
   ms_batch: `iters` back-to-back launches between two events, per launch; ms_each: the average of
   per-launch dispatch events (hipExtLaunchKernelGGL); bytes: algorithmic bytes per launch.
   kernel + 16*F: F untimed launches of a coarse level's smoother follow every timed launch
   (ms_batch then includes them; ms_each still times the kernel's own launches) */
int pucfem_bench_kernel(void* ctx, int32_t kernel, int32_t iters, double* ms_batch, double* ms_each, double* bytes);
/* sizes of the internal operators: out[0]=N, [1]=T, [2]=nnz(P), [3]=nnz(Pp), [4]=n_own,
   [5]=n_ghost, [6]=padded SELL entries (P), [7]=padded SELL entries (Pp), [8]=n_pairs, [9]=n_dirichlet,
   [10]=storage flags (bit 0: P has int16 columns, bit 1: Pp has int16 columns, bit 2: the finest
   V-cycle operator is stored in fp16), [11]=multigrid levels (0: none) */
int pucfem_info(void* ctx, int64_t* out12);
/* which code path the step runs (for tests of the production path): out[0] viscous solve (0 dense inverse,
   1 one-workgroup CG, 2 multi-kernel CG), [1] pressure solve (0 dense, 1 one-workgroup CG, 2 multi-kernel
   Jacobi CG, 3 multigrid-preconditioned CG), [2] projection bases re-seeded so far, [3] / [4] current
   basis sizes of the two pressure solves, [5] extrapolation order of the viscous warm start in use,
   [6] projection basis capacity (0: off), [7] bit 0: the operators are lattice stencils on the face
   interiors (pucfem_params.assembled = 0 with a hierarchy; clear: every row is a stored SELL row),
   bit 1: the semi-Lagrangian point location uses the lattice locator (else per-triangle records),
   bit 7: pressure PCG iterations ran in the single-reduction (Chronopoulos-Gear) form */
int pucfem_path_info(void* ctx, int64_t* out8);
/* multi-rank data flow of the last step: out[0] dye values this rank received in the wide halo before
   the semi-Lagrangian step, out[1] the values a full all-gather of the dye would have received
   (N - n_own), out[2] values all-reduced for the StokesFood tracers (3 x tracers), out[3] the data-path
   backend (0 none: single rank, 1 LocalComm test backend, 2 RCCL) */
int pucfem_comm_info(void* ctx, int64_t* out4);
/* Communicator self-test on the library stream (RCCL's first contact in a run): sum and max all-reduces
   of 8 values and one grouped ring exchange (rank -> rank + 1; a send to itself on one rank), checked
   against their known results: out = (|sum err|, |max err|, |recv err|, backend 1 LocalComm / 2 RCCL).
   The replaced reference sites are the dot products inside the np.linalg.solve calls
   (StokesColor.py:544-545, 555, 569), which become all-reduced CG dots on multi-rank runs. */
int pucfem_comm_selftest(void* ctx, double* out4);
/* unit probe of the single-reduction PCG's scalar kernel (k_cgcg_coef, the multi-rank pressure solve of
   StokesColor.py:555,569): one launch on the context's stream from the given 8 reduced values red8, <b, b> bb,
   the state sc5 (alpha, beta, gamma of the last iteration, alpha_(it-1), gamma_(it-1)) and iteration `it`;
   ctl_out[2] receives the control word ({0, 0} continue, {1, k} converged at iteration k, {2, it} maxit,
   {3, it} not finite), sc_out5 the new state.  Test infrastructure (tests/test_gpu_parity.py). */
int pucfem_cgcg_coef_probe(void* ctx, const double* red8, double bb, const double* sc5, double tol2, int32_t it,
                           int32_t maxit, double rho0, int32_t* ctl_out, double* sc_out5);
/* cumulative data-path traffic of this rank's communicator (zeros without one): out[0] all-reduce calls,
   [1] all-reduced values, [2] point-to-point sends, [3] bytes sent, [4] grouped launches (group_start),
   [5] broadcasts (DESIGN.md §7's per-step counts; measurement only) */
int pucfem_comm_counters(void* ctx, int64_t* out6);
/* The viscous Chebyshev iteration's interval for the Jacobi-scaled A_visc (StokesColor.py:471-475):
   out2 = [lo, hi], lo = max(1 - R, 1 / max_i a_ii), hi = 1 + R, R the Gershgorin radius.  Every
   eigenvalue lies inside (tests/test_host_assembly.py checks it against scipy's eigensolver). */
int pucfem_visc_interval(void* ctx, double* out2);
/* The pressure multigrid's smoothing interval on one level (0 = coarsest .. levels) of a single-rank context:
   the Chebyshev smoother of D^-1 A runs on [lmax / mg_ratio, lmax] (the np.linalg.solve sites
   StokesColor.py:555,569 it preconditions).  out4 = [lmax in use, the device power iteration's Rayleigh
   quotient (0: estimated on the host), the host 30-step power iteration's quotient on the level's fp64
   operator (computed by this call), the host Gershgorin bound]; lmax = min(Gershgorin, 1.1 x quotient). */
int pucfem_mg_lmax(void* ctx, int32_t level, double* out4);
/* The pressure solves' projected initial guesses (successive right-hand sides, pucfem_params.proj_k; the solves
   replace np.linalg.solve at StokesColor.py:555,569): out4 = [bases re-seeded so far, bases restarted by the guess
   monitor (a projected guess > 50x worse than the best of its basis' last 8), the last projected guess's relative residual
   |b - A x0| / |b| of basis 1 and of basis 2 (0: none yet)]. */
int pucfem_proj_info(void* ctx, double* out4);

/* ---- host-only (no device needed) ---------------------------------------------------- */
/* Red refinement, `levels` times.  Call with xy_out == NULL to get sizes. */
int pucfem_refine(int64_t n_nodes, const double* xy, const int32_t* markers, int64_t n_tris,
                  const int32_t* tris, int32_t levels, int64_t* n_nodes_out, int64_t* n_tris_out,
                  double* xy_out, int32_t* markers_out, int32_t* tris_out);
/* The host-assembled operator of this rank in the CALLER's numbering (rows owned by this rank,
   global column ids).  Call with col == NULL to get nnz.  For CPU tests of the assembly. */
int pucfem_host_get_csr(void* ctx, int32_t op, int64_t* n_rows, int64_t* nnz, int64_t* rowptr,
                        int64_t* col, double* val);
/* Host reference of the lattice face stencils (CPU tests of the index arithmetic and the per-face
   coefficients; single-rank contexts with lattice operators).  Rows of face-interior nodes of the output
   level are written, every other entry of y is NaN.  kind 0: K x, 1: Gx x0 + Gy x1 (x is (N, 2), the
   divergence numerator), 2: S A_visc S x, 3: the level's periodic-merged pressure operator (any level),
   5: prolongation from level-1 into level (x on level-1), 6: restriction from level into level-1.
   Vectors in the caller numbering of their level (level = the multigrid level, 0 = the coarse mesh). */
int pucfem_host_lattice_apply(void* ctx, int32_t level, int32_t kind, const double* x, double* y);
/* Partition plan for (rank, world) computed on a host-only context (pucfem_ctx_create(-1)):
   owned rows (caller numbering) in internal order, then the ghost ids; send lists per peer.
   Sizes first (arrays NULL), then contents. */
int pucfem_host_partition(void* ctx, int32_t rank, int32_t world, int64_t* n_own, int64_t* n_ghost,
                          int64_t* owned, int64_t* ghosts, int32_t* ghost_owner,
                          int64_t* n_send, int64_t* send_ids, int32_t* send_peer);

#ifdef __cplusplus
}
#endif
#endif /* PUCFEM_H */
