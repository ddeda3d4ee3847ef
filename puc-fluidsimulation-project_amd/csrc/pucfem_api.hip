// libpucfem C ABI (include/pucfem.h): context, device memory, solver orchestration, RCCL halo /
// all-reduce, and the Stokes / heat / Poisson step loops.  One HIP stream per context; every
// kernel of a step is enqueued back to back and the host synchronises only to poll CG
// convergence (once per chunk of iterations) and to return results.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <memory>
#include <numeric>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>
#include <future>
#include <map>

#include "pucfem.h"
#include "pucfem_comm.hpp"
#include "pucfem_host.hpp"
#include "pucfem_kernels.hpp"
#include "pucfem_kernels_impl.hpp"

using namespace pucfem;
using namespace pucfem::dev;

// Kernel launches of this thread (pucfem_counters): every launch of the library goes through
// hipLaunchKernelGGL (redefined here to count) or Ctx::klaunch.
namespace {
thread_local int64_t g_nlaunch = 0;
}
#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(kernelName, ...) \
  do {                                      \
    ++g_nlaunch;                            \
    hipLaunchKernelGGLInternal((kernelName), __VA_ARGS__); \
  } while (0)

// LocalComm reduction (fixed rank order -> identical result on every rank)
__global__ void pucfem::k_comm_reduce(int world, int is_max, size_t n, const double* const* bufs, double* out) {
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) {
    double a = bufs[0][i];
    for (int r = 1; r < world; ++r) a = is_max ? fmax(a, bufs[r][i]) : a + bufs[r][i];
    out[i] = a;
  }
}

namespace {

constexpr int64_t DENSE_MAX = 1500;  // small-mesh direct-solve threshold (mesh_fine: 1,067 nodes)
static_assert(DENSE_MAX <= dev::DENSE_LDS, "the dense solves stage their vectors in LDS");

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(x)                                                                                 \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess)                                                                         \
      throw Error(PUCFEM_EHIP, std::string(#x) + ": " + hipGetErrorString(e_));                   \
  } while (0)
#define NCCLCHK(x)                                                                                \
  do {                                                                                            \
    ncclResult_t r_ = (x);                                                                        \
    if (r_ != ncclSuccess) throw Error(PUCFEM_ENCCL, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)
#define KCHK() HIPCHK(hipGetLastError())

std::string g_err;  // errors of context-free calls

struct DevSell {
  int64_t* off = nullptr;
  int32_t* w = nullptr;
  int32_t* col = nullptr;
  int16_t* c16 = nullptr;  // int16 column deltas (square operators whose band fits), else null
  int64_t nslices = 0, nrows = 0, nnz = 0, padded = 0;
  int32_t wrap = 0;        // c16 modulus (local vector length)
  int32_t* rows = nullptr; // row list (lattice operators: the skeleton rows), else null
  int64_t n_own = 0;       // owned rows of the vector space (0: nrows)
  // deep halos (Sell::gk0): slices [nslices, nslices_g) hold ghost rows one layer out, which the launches that
  // compute them redundantly (step pairs, residuals, last smoothing steps on W > 1 ranks) include: with_ghosts()
  int64_t nslices_g = 0;
  SellDev view() const { return SellDev{off, w, col, nslices, nrows, c16, wrap, rows, n_own ? n_own : nrows}; }
  bool has_ghost_rows() const { return nslices_g > nslices; }
  DevSell with_ghosts() const {
    DevSell d = *this;
    if (nslices_g > nslices) d.nslices = nslices_g;
    return d;
  }
  // after a row-listed upload of S: the own rows' slices only by default, the ghost rows' ones behind with_ghosts()
  void ghost_slices(const pucfem::Sell& S) {
    if (S.gk0 < 0) return;
    nslices_g = S.nslices;
    nslices = S.nslices_own;
    nrows = S.nrows - (int64_t)S.grow.size();
  }
  double idx_bytes() const { return c16 ? 2.0 : 4.0; }  // per stored entry
  double row_bytes() const { return rows ? 4.0 : 0.0; }  // per row (the row list)
  int64_t own() const { return n_own ? n_own : nrows; }   // rows of the vector space
};

// A lattice operator's face part on the host (pucfem_lattice.hpp): the FaceDev image and its work
// items.  Partial-producing launches cap the face blocks (the partial arrays hold MAXB blocks in all;
// at L7 every item still gets its own block), the others give every item a block.
constexpr int32_t FACE_PART_BLOCKS = MAXB - 8192;
struct HFace {
  FaceDev d{};
  int32_t items = 0;
  int64_t rows = 0;  // face-interior rows (algorithmic bytes)
  FaceDev part() const {
    FaceDev f = d;
    f.nb = std::min(items, FACE_PART_BLOCKS);
    return f;
  }
  FaceDev full() const {
    FaceDev f = d;
    f.nb = items;
    return f;
  }
};
// f(std::true_type) when A carries int16 columns, f(std::false_type) otherwise: one launch site
// instantiates both SpMV variants
template <class F>
void with_c16(const DevSell& A, F&& f) {
  if (A.c16) f(std::true_type{});
  else f(std::false_type{});
}

struct Red {  // a (possibly globally reduced) partial array
  const double* p;
  int nb;
  int stride;
};

struct Timer {
  bool on = false;
  uint32_t mask = ~0u;  // timed kernel classes
  std::vector<hipEvent_t> pool;
  struct Pend { int cls; hipEvent_t a, b; double bytes; bool keep = false; };  // (cls < 0: not accounted)
  std::vector<Pend> pend;
  // classes: 0 k_cheb (finest), 1 k_cg_dir, 2 k_cg_upd, 3 k_grad_proj, 4 k_sl, 5 k_resid (finest), 6 / 7 the
  // finest level's restriction / prolongation, 8 k_sl_slow, 9 k_vcheb (whole-grid steps), 10 k_cheb_pair,
  // 11 k_div, 12 k_vcheb_pair, 13 k_visc_prep, 14 k_mdot2, 15 k_pcomb
  static constexpr int NCLS = 16;
  double ms[NCLS] = {};
  double bytes[NCLS] = {};
  int64_t n[NCLS] = {};
  hipEvent_t get() {
    if (pool.empty())  // in batches: the samples stay pending until their solve's test is read
      for (int k = 0; k < 256; ++k) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        pool.push_back(e);
      }
    hipEvent_t e = pool.back();
    pool.pop_back();
    return e;
  }
  size_t done = 0;  // samples accounted so far (the absolute index of pend[0])
  size_t mark() const { return done + pend.size(); }
  void account(const Pend& p) {
    if (p.cls >= 0) {
      float t = 0;
      HIPCHK(hipEventElapsedTime(&t, p.a, p.b));
      ms[p.cls] += t;
      bytes[p.cls] += p.bytes;
      n[p.cls]++;
    }
    pool.push_back(p.a);
    pool.push_back(p.b);
  }
  void flush() {
    for (auto& p : pend) {
      HIPCHK(hipEventSynchronize(p.b));
      account(p);
    }
    done += pend.size();
    pend.clear();
  }
  // account the finished samples before absolute index `limit` without waiting: called while the GPU runs the
  // work just enqueued, so the host's event reads overlap it (a blocking flush after a solve's convergence
  // read idled the GPU ~0.12 ms per pressure solve, r10x trace)
  void flush_ready(size_t limit) {
    size_t i = 0;
    for (; i < pend.size() && done + i < limit; ++i)
      if (hipEventQuery(pend[i].b) != hipSuccess) break;
    for (size_t k = 0; k < i; ++k) account(pend[k]);
    pend.erase(pend.begin(), pend.begin() + (std::ptrdiff_t)i);
    done += i;
  }
  // drop the pending samples from absolute index k on (launches that found the solve converged and returned
  // without work: counting them would credit their bytes to a near-zero duration)
  // (samples marked `keep` stay: a gated gradient projection behind the read that found the solve converged)
  void drop_from(size_t k) {
    size_t w = k > done ? k - done : 0;
    for (size_t i = w; i < pend.size(); ++i) {
      if (pend[i].keep) {
        pend[w++] = pend[i];
        continue;
      }
      pool.push_back(pend[i].a);
      pool.push_back(pend[i].b);
    }
    if (w < pend.size()) pend.resize(w);
  }
  ~Timer() {
    for (auto e : pool) (void)hipEventDestroy(e);
    for (auto& p : pend) {
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
  }
};

template <typename T>
struct MgBufs {
  T *Aval = nullptr, *Prval = nullptr, *Rval = nullptr, *dinv = nullptr;
  T *x = nullptr, *x2 = nullptr, *b = nullptr, *d = nullptr, *res = nullptr, *sendbuf = nullptr;
  // fp16 copy of the level operator's values (fp32 cycle, when every value is representable): the
  // smoother and residual stream 2 B per entry instead of 4, arithmetic stays fp32
  _Float16* Aval16 = nullptr;
  template <class F>
  void with_vals(F&& f) const {
    if constexpr (std::is_same<T, float>::value) {
      if (Aval16) {
        f((const _Float16*)Aval16);
        return;
      }
    }
    f((const T*)Aval);
  }
  double val_bytes() const { return Aval16 ? 2.0 : (double)sizeof(T); }
};

// face-interior node -> its macro face (the deep halos' face-stencil ghost rows, face_ghost_rows)
struct FaceLookup {
  std::vector<std::pair<i64, i32>> starts;  // (first interior node, face), ascending
  LocalPlan full;                           // the level's whole range: to_local = the global id
  void init(const Macro& M, const LatticeLevel& LL) {
    starts.clear();
    for (i64 f = 0; f < M.nf; ++f)
      if (LL.face_start[f] >= 0) starts.push_back({LL.face_start[f], (i32)f});
    std::sort(starts.begin(), starts.end());
    full.r0 = 0;
    full.r1 = (i64)LL.type.size();
    full.n_own = full.r1;
  }
  // face-interior node g -> (face, offset t)
  void find(i64 g, i32& f, i32& t) const {
    auto it = std::upper_bound(starts.begin(), starts.end(), std::make_pair(g, (i32)INT32_MAX));
    --it;
    f = it->second;
    t = (i32)(g - it->first);
  }
};
GhostRowFn face_ghost_rows(const Macro& M, const LatticeLevel& LL, const FaceLookup& FL, const std::vector<i32>* dof,
                           int l, double dtnu) {
  return [&M, &LL, &FL, dof, l, dtnu](i32 g, std::vector<i32>& cols, std::vector<double>& vals) -> bool {
    if (LL.F == 0 || LL.type[g] != 0) return false;
    i32 f, t;
    FL.find(g, f, t);
    std::vector<lat::FaceTab> tab;
    lattice_tabs(M, LL, {f}, 0, FL.full, dof, tab);
    std::vector<double> rec;
    lattice_coefs(M, {f}, l, dtnu, rec);
    const i32 n = LL.n;
    i32 i, j, nb[6];
    bool in[6];
    lat::coords(t, n, 1.0f / (float)(n - 1), i, j);
    lat::neighbours(tab[0], n, t, i, j, nb, in);
    cols.assign({g, nb[0], nb[1], nb[2], nb[3], nb[4], nb[5]});
    const double kab = rec[lat::C_KAB], kac = rec[lat::C_KAC], kbc = rec[lat::C_KBC];
    vals.assign({rec[lat::C_KD], kab, kab, kac, kac, kbc, kbc});
    return true;
  };
}
double face_dinv(const Macro& M, const LatticeLevel& LL, const FaceLookup& FL, int l, i64 g) {
  i32 f, t;
  FL.find(g, f, t);
  std::vector<double> rec;
  lattice_coefs(M, {f}, l, 0.0, rec);
  return rec[lat::C_DINV];
}

// One level of the geometric multigrid hierarchy (pressure preconditioner).  Level 0 is the
// coarsest (the caller's base mesh, solved densely), the last level is the simulation mesh.
struct MgLevel {
  HostMesh mesh;            // coarse levels only (the finest is Ctx::mesh)
  std::vector<i32> ea, eb;  // edge endpoints of the level below (midpoint parents), caller numbering
  Ordering ord;
  Csr P, Pp, Pr, R;         // pattern, merged pressure operator, prolongation from l-1, restriction to l-1
  std::vector<i32> dof, master_of, slave_of;
  std::vector<std::pair<i64, i64>> pairs;
  std::vector<i64> rs;      // partition of this level's internal ids
  LocalPlan lp;
  double lmax = 2.0;
  double lam_dev = 0.0;  // the device power iteration's last Rayleigh quotient (0: not run; pucfem_mg_lmax)
  // device
  Sell sA, sPr, sR;         // host SELL images (built with the plans, also on host-only contexts)
  DevSell dA, dPr, dR;
  MgBufs<double> f64;       // the V-cycle's values and vectors: one of the two sets is allocated
  MgBufs<float> f32;        // (fp32 = the mixed-precision cycle, prm.mg_single)
  int32_t* dsend = nullptr;
  i64 nsend = 0, nloc = 0;
  // multi-rank runs: coarse levels of <= mg_rep_nodes nodes are REPLICATED (every rank holds and
  // smooths the whole level, no halos); the restriction into the finest replicated level computes
  // the rows of the strip partition (rs) and an all-gather (broadcast group) completes the vector
  bool rep = false;
  // deep halos (W > 1, lattice, PUCFEM_DEEP_HALO): the plan's ghosts reach two layers out (make_local_plan2's G2) and
  // the operator's SELL carries the ghost rows one layer out (g1, global ids) behind DevSell::with_ghosts().  Then
  // - a step pair runs its first step on those rows too (one exchange of x for two steps; pairs at W > 1),
  // - res_deep: the residual runs on them too, so the restriction reads no exchanged residual,
  // - the post-smoothing's last step runs on them (x and d exchanged before it, as x alone was), so its output is
  //   current at the ghosts the next consumer gathers: z for the PCG's A z (finest), x for the prolongation into
  //   the finer level (xc_deep, on that finer level: its prolongation's coarse columns lie in own + G1).
  // Every rank takes the same path (the flags are all-reduced at build).
  // - pr_deep: the prolongation into this level also runs on its ghost rows (x there is current since the exchange
  //   before the residual), its coarse columns in level l - 1's own + G1 rows: the post-smoothing's first pair needs
  //   no exchange of x.
  std::vector<i32> g1;
  bool deep = false, res_deep = false, xc_deep = false, pr_deep = false;
  FaceLookup flook;  // (deep lattice levels) face-interior node -> face
  i64 r_r0 = 0;  // first row of this level's restriction operator (rows live on level l-1)
  i64 own0(int rank) const { return rep ? 0 : rs[rank]; }
  // lattice face parts (Ctx::lattice): the faces whose interiors are this rank's rows of this level,
  // their tables (plain: K / G / A_visc; merged: the periodic-merged pressure operator) and records;
  // the prolongation into this level gathers the same faces on level l-1 (pr_tab2, merged), the
  // restriction into level l-1 writes the faces of its rows [r_r0, r_r0 + nr) (r_tab, bases from
  // r_r0) from this level's nodes (r_tab2, plain)
  LatticeLevel latl;
  std::vector<i32> lf_faces, r_faces;
  std::vector<lat::FaceTab> lf_plain, lf_merged, pr_tab2, r_tab, r_tab2;
  std::vector<double> lf_coef;
  HFace hA, hPr, hR;  // level operator (merged), prolongation into / restriction from this level
};
template <typename T> MgBufs<T>& bufs(MgLevel& L);
template <> MgBufs<double>& bufs<double>(MgLevel& L) { return L.f64; }
template <> MgBufs<float>& bufs<float>(MgLevel& L) { return L.f32; }

void spmv_on(hipStream_t st, const DevSell& A, const FaceDev& fc, const double* val, const double* x, double* y);
// k_mdot2 / k_pcomb for basis size m (0..PROJ_MAX): one instance per size, picked from a table (every
// instance has the same signature, so the launch goes through Ctx::klaunch like any other kernel)
using Mdot2K = decltype(&k_mdot2<0>);
using PcombK = decltype(&k_pcomb<0>);
template <int... M>
constexpr std::array<Mdot2K, sizeof...(M)> mdot2_table(std::integer_sequence<int, M...>) {
  return {&k_mdot2<M>...};
}
template <int... M>
constexpr std::array<PcombK, sizeof...(M)> pcomb_table(std::integer_sequence<int, M...>) {
  return {&k_pcomb<M>...};
}
Mdot2K mdot2_kernel(int m) {
  static constexpr auto tab = mdot2_table(std::make_integer_sequence<int, PROJ_MAX + 1>{});
  if (m < 0 || m > PROJ_MAX) throw Error(PUCFEM_EINVAL, "projection basis size out of range");
  return tab[m];
}
PcombK pcomb_kernel(int m) {
  static constexpr auto tab = pcomb_table(std::make_integer_sequence<int, PROJ_MAX>{});
  if (m < 0 || m >= PROJ_MAX) throw Error(PUCFEM_EINVAL, "projection basis size out of range");
  return tab[m];
}

struct Ctx {
  std::string err;
  int device = -1;
  bool host_only = true;
  int rank = 0, world = 1;
  // the data-path communicator: RCCL (or the LocalComm test backend) on multi-rank runs; also RCCL on a
  // ONE-rank context created from a real unique id (pucfem_ctx_create_dist with world 1), which then
  // takes every multi-rank code path -- all-reduces, broadcasts, the dye range exchange -- through RCCL
  std::unique_ptr<Comm> comm;
  bool dist() const { return comm != nullptr; }
  hipStream_t st = nullptr;
  std::vector<void*> allocs;
  Timer timer;
  // algorithmic bytes of the launched kernels (pucfem_counters: the step's HBM floor): each vector
  // counted once per row it is read or written, stored operators per entry; launches that find their
  // solve already converged (no work) are taken back once the host learns the iteration count
  double algo_bytes = 0.0;
  // per kernel class (Timer's classes), every launch timed or not: launches and algorithmic bytes
  // (pucfem_class_counters: bench.py weighs the classes over the whole timed window with them)
  double cls_bytes[Timer::NCLS] = {};
  int64_t cls_n[Timer::NCLS] = {};
  struct ByteMark {  // the counters at one point (launches after a solve's convergence are taken back)
    double total;
    double cb[Timer::NCLS];
    int64_t cn[Timer::NCLS];
  };
  ByteMark bmark_now() const {
    ByteMark m{algo_bytes, {}, {}};
    for (int k = 0; k < Timer::NCLS; ++k) {
      m.cb[k] = cls_bytes[k];
      m.cn[k] = cls_n[k];
    }
    return m;
  }
  void bmark_restore(const ByteMark& m) {
    algo_bytes = m.total;
    for (int k = 0; k < Timer::NCLS; ++k) {
      cls_bytes[k] = m.cb[k];
      cls_n[k] = m.cn[k];
    }
  }

  // ---- inputs
  HostMesh mesh;
  bool has_mesh = false;
  std::vector<std::pair<i64, i64>> op_pairs, bc_pairs;
  std::vector<i32> dir_nodes;
  std::vector<double> dir_vals;
  int dir_ncomp = 0;
  std::vector<float> g_tri;
  pucfem_params prm{};
  bool built = false;

  // ---- host structures (internal numbering)
  Ordering ord;
  Csr P, Pp, Lit;
  Assembly as;
  std::vector<double> litb, Kv;
  std::vector<i64> row_start;
  LocalPlan lp;
  Sell sP, sPp, sLit;
  std::vector<i32> dof, slave_of, master_of;  // global internal ids
  i64 n_free = 0;
  int scheme = 0;

  // ---- device operators
  DevSell dP, dPp, dLit;
  double *dK = nullptr, *dGx = nullptr, *dGy = nullptr, *dKv = nullptr, *dKp = nullptr, *dLitv = nullptr;
  double *dsv = nullptr, *dsp = nullptr, *dlit_dinv = nullptr;
  double *das1 = nullptr, *dmp = nullptr, *dwmix = nullptr;
  uint8_t* ddir = nullptr;
  int32_t *dslave_of = nullptr, *dmaster_of = nullptr;
  int32_t *dcdst = nullptr, *dcsrc = nullptr, *ddnode = nullptr;
  double *ddval = nullptr, *dbctmp = nullptr;
  int32_t *dbcsrc = nullptr, *dbcdir = nullptr;  // dense path: k_dense_mv2_bc's row maps
  int ncopy = 0, ndir = 0;
  bool bc_gather = true;  // some copy source is also written: k_bc_gather saves the sources first
  int32_t* dsend = nullptr;
  double* dsendbuf = nullptr;
  i64 nsend = 0;

  // ---- device fields (local: n_own + n_ghost)
  i64 nloc = 0;
  double *ux = nullptr, *uy = nullptr, *usx = nullptr, *usy = nullptr, *p = nullptr, *p2 = nullptr;
  double *yp = nullptr, *yp2 = nullptr, *yvx = nullptr, *yvy = nullptr;
  double *div_star = nullptr, *div_u = nullptr, *final_div = nullptr, *braw = nullptr, *bh = nullptr;
  double *bvx = nullptr, *bvy = nullptr;
  double *cg_r[2] = {nullptr, nullptr}, *cg_pa[2] = {nullptr, nullptr}, *cg_pb[2] = {nullptr, nullptr},
         *cg_q[2] = {nullptr, nullptr};
  double *part_a = nullptr, *part_b = nullptr, *part_c = nullptr, *part_d = nullptr;
  double* scal = nullptr;
  int* ctl = nullptr;
  int* h_ctl = nullptr;  // pinned
  double* redbuf = nullptr;  // small buffers for all-reduced scalars (64 x 8)
  double* vals = nullptr;    // per-step diagnostic slots (16)
  double* scalar = nullptr;  // heat u / poisson f
  double* litw[10] = {};     // BiCGStab workspace
  double* bicg_sc = nullptr;
  double* h_pinned = nullptr;

  // ---- full-mesh replica (SL, tracers)
  double *mx = nullptr, *my = nullptr;
  int32_t* mtri = nullptr;
  GridDev cgrid{}, tgrid{};
  LocDev lgrid{};
  // implicit FEM dye variant (prm.dye_scheme == 1, good_visualization.py:700-718)
  bool dye_impl = false;
  DevSell dDye{};              // the merged (Pp) pattern, every row stored
  DyeDev dye{};
  double *dDyeVal = nullptr, *dDyeM = nullptr, *dDyeW = nullptr, *dDyeDinv = nullptr, *dDyeB = nullptr;
  int64_t* dDyeDiag = nullptr;  // SELL slot of each row's diagonal
  int32_t *dDyeSrow = nullptr, *dDyeSk = nullptr, *dDyeSc = nullptr;
  int64_t* dDyeSptr = nullptr;
  int32_t dye_nsrow = 0;
  int last_dye_it = 0;
  bool lmax_dev = false;            // the finest level's lmax: power iteration on the device
  // multi-rank dye replica: a wide halo instead of an all-gather (dye_halo)
  std::vector<double> strip_ylo, strip_yhi;  // per strip (internal order): the y extent of its nodes
  std::vector<i64> rank_s0, rank_s1;         // per rank: its strips [s0, s1)
  std::vector<double> rank_ylo, rank_yhi;    // per rank: the y extent of its nodes
  double tri_hy = 0.0;                       // largest y extent of a triangle
  double* part_u = nullptr;                  // back-traced y range partials (1 - min, max)
  double *yr_own = nullptr, *yr_all = nullptr;  // this rank's (1 - min, max); every rank's (2 W)
  std::vector<double> h_yr;
  double* trv = nullptr;                     // multi-rank tracer velocities (3 x ntr, all-reduced)
  int32_t* dghost_global = nullptr;          // lp.ghost_global on the device
  i64 dye_halo_values = 0;                   // values received by the last dye_halo (diagnostics)
  std::vector<double> lmax_dinv;    // its D^-1 (host, Gershgorin pass)
  DyeOp dyeop;  // host data of the implicit dye operator (built with the host operators)
  LatLocDev llgrid{};  // lattice locator (lat_sl): replaces lgrid's records on lattice hierarchies
  bool lat_sl = false;
  double* part_sl = nullptr;  // k_sl partials, 3 x SLB
  int32_t* sl_queue = nullptr; // k_sl -> k_sl_slow: rows off the lattice fast path (mesh.N)
  int32_t* sl_qcnt = nullptr; // per wave of k_sl: queued entries (SLB * BS / 64)
  int32_t* sl_qoff = nullptr; // k_sl_qscan: the queues' first entry numbers (SLB * BS / 64 + 1)
  bool has_cgrid = false, has_tgrid = false;
  double *c_full = nullptr, *c_new = nullptr, *ufx = nullptr, *ufy = nullptr;
  int32_t* dnotfound = nullptr;
  int32_t ntr = 0;
  double *trx = nullptr, *try_ = nullptr, *trs = nullptr, *d_eaten = nullptr;
  // iteration count of the last solve per `which` slot (the next solve's first host check): 0 viscous,
  // 1 / 2 the two pressure solves of a step, 3 / 4 standalone viscous / pressure solves (pucfem_solve)
  int last_it[6] = {0, 0, 0, 0, 0, 0};
  bool solved_before[6] = {false, false, false, false, false, false};  // last_it[which] holds a real count
  // per slot: whether each of the last 8 solves that followed a solve of <= 1 iteration passed at its
  // initial guess (bit 0 the latest) -- pcg_mg's pre-check policy
  unsigned zero_hist[6] = {0u, 0u, 0u, 0u, 0u, 0u};
  bool lds_attr[3] = {false, false, false};  // k_cg_block<NR>: dynamic-LDS attribute set on this device
  double* solve_tmp = nullptr;  // pucfem_solve scratch (4 x nloc): standalone solves never touch the step state
  int* dits = nullptr;  // per-step iteration counts written by single-workgroup solves (no host sync)
  int cur_step = 0;
  bool block_cg = true;  // small operators: whole CG in one workgroup
  // small meshes (N <= DENSE_MAX, one rank): both linear solves are dense direct solves with
  // precomputed inverses -- the reference's np.linalg.solve, factorised once instead of per call
  bool dense = false;
  double *dVinv = nullptr, *dPinv = nullptr;
  // small literal operators (heat / Poisson, N <= DENSE_MAX): the inverse of the literal operator
  // (heatEq.py:321 / poisson.py:283 solve with it every step: np.linalg.solve, factorised once here)
  double* dLitInv = nullptr;
  // small meshes: one StokesColor/StokesFood step captured once into a hipGraph and replayed
  bool graph_mode = false;
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  // and GK = 8 consecutive steps in one graph (PUCFEM_GRAPH_STEPS, measurement knob; 1 = one step per replay): one
  // launch per 8 steps, whose ~8 us between replays (r14u trace) the steps inside a graph do not pay; the same bits
  // (test_graph_of_k_steps_equals_single_step_graph).  mesh_fine 12.3-12.6k -> 13.1-13.5k steps/s (r14x; with the
  // step's earlier 13 launches, 8-step graphs measured slower, r14b)
  int gk = std::getenv("PUCFEM_GRAPH_STEPS") ? std::max(1, std::min(64, std::atoi(std::getenv("PUCFEM_GRAPH_STEPS")))) : 8;
  hipGraphExec_t gexec_k = nullptr;
  hipGraph_t graph_k = nullptr;
  double* gstats = nullptr;
  // the replayed step's records: a device ring of GRING steps (k_stats_ring), copied out per call / full ring
  static constexpr int GRING = 1024;
  double* gring = nullptr;
  int* gcount = nullptr;
  bool gcapture = false;  // (the step being captured)
  // the captured step's record appended by k_mix2's reducing block (PUCFEM_RING_FOLD=0, measurement knob: k_stats_ring)
  bool ring_fold = !(std::getenv("PUCFEM_RING_FOLD") && std::atoi(std::getenv("PUCFEM_RING_FOLD")) == 0);
  bool ring_in_mix = false;
  // the captured step's fork (PUCFEM_GRAPH_FORK=1, measurement knob, off): a side stream and its events, made before
  // the capture (prep_fork).  The same bits, but the graph's cross-stream edges cost more than the overlap gains:
  // mesh_fine 10.0k steps/s forked against 12.5k in one chain (r14q)
  hipStream_t st_fk = nullptr;
  hipEvent_t ev_fk = nullptr, ev_fj = nullptr;
  bool fork_pend = false;
  void prep_fork() {
    if (st_fk || !(std::getenv("PUCFEM_GRAPH_FORK") && std::atoi(std::getenv("PUCFEM_GRAPH_FORK")) != 0)) return;
    HIPCHK(hipStreamCreateWithFlags(&st_fk, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&ev_fk, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_fj, hipEventDisableTiming));
  }
  void fork_join() {
    if (!fork_pend) return;
    HIPCHK(hipStreamWaitEvent(st, ev_fj, 0));
    fork_pend = false;
  }

  // ---- lattice operators (pucfem_lattice.hpp): multigrid hierarchies with faces of interior nodes
  bool lattice = false;
  // deep halos on W > 1 ranks (MgLevel::deep; PUCFEM_DEEP_HALO=0 keeps one-layer halos and single smoothing steps,
  // a test / measurement knob)
  bool deep_halo = !(std::getenv("PUCFEM_DEEP_HALO") && std::atoi(std::getenv("PUCFEM_DEEP_HALO")) == 0);
  bool z_cur = false;  // the finest level's last smoothing step wrote z at the ghost rows one layer out too
  // PUCFEM_DEEP_MASK (diagnostic knob, default all): 1 multigrid step pairs, 2 residual rows, 4 last smoothing step
  // (+ the skipped z / x exchanges), 8 prolongation rows, 16 the viscous first pair -- each use of the ghost rows
  int deep_mask = std::getenv("PUCFEM_DEEP_MASK") ? std::atoi(std::getenv("PUCFEM_DEEP_MASK")) : 31;
  Macro macro;
  LatticeLevel lat_fine;  // the finest level's layout until build_mg_host moves it into mg.back()
  HFace fK, fVisc, fP;  // finest level: K / Gx / Gy (plain table), scaled A_visc (plain), pressure (merged)
  // Gershgorin radius of the Jacobi-scaled A_visc, max_i sum_{j != i} |a_ij| / sqrt(a_ii a_jj): its spectrum
  // lies in [1 - visc_R, 1 + visc_R] (the Chebyshev viscous solve's interval)
  double visc_R = 1.0, visc_lo = 0.0;
  int visc_solver = 0;  // 0 = Chebyshev iteration when visc_R < 0.25 (multi-kernel path), 1 = CG
  // a-posteriori check of the Chebyshev bound (vcheb): the last step of a solve also reduces |r_{k}|^2 of
  // the iterate it starts from (k = K - 1), copied to h_pinned[32 ..]; the next solve compares it with
  // |r_0| / T_k(sigma) -- a spectrum outside [visc_lo, 1 + visc_R] (a wrong interval) breaks the bound.  A
  // violation switches the viscous solves to the CG (visc_check_fail counts them, pucfem_path_info)
  struct ViscCheck {
    bool pending = false;
    int nr = 0;
    double bound2[2] = {0.0, 0.0}, floor2[2] = {0.0, 0.0};
  } vcc;
  int visc_check_fail = 0;
  // step pairs of the viscous Chebyshev solve (k_vcheb_pair, single rank with a face part): PUCFEM_VISC_PAIR=0
  // runs every step as its own k_vcheb (a measurement knob); the pair's third x buffer and second d
  // buffer are allocated on first use
  bool visc_pair = !(std::getenv("PUCFEM_VISC_PAIR") && std::atoi(std::getenv("PUCFEM_VISC_PAIR")) == 0);
  int64_t visc_pairs = 0;  // pairs launched (pucfem_path_info)
  // step pairs of the finest level's smoothing in the fp32 V-cycle (k_cheb_pair, single rank):
  // PUCFEM_MG_PAIR=0 runs every step as its own k_cheb (a measurement knob); a third x buffer and a second
  // d buffer of the finest level are allocated on first use
  bool mg_pair = !(std::getenv("PUCFEM_MG_PAIR") && std::atoi(std::getenv("PUCFEM_MG_PAIR")) == 0);
  // PUCFEM_MG_PAIR_LEVELS (measurement knob): the step pairs on the finest k levels (default 1: the finest only)
  int mg_pair_levels = std::getenv("PUCFEM_MG_PAIR_LEVELS") ? std::max(1, std::atoi(std::getenv("PUCFEM_MG_PAIR_LEVELS"))) : 1;
  int64_t mg_pairs = 0;
  float* mgp_x = nullptr;
  float* mgp_d = nullptr;
  double* dwsk = nullptr;  // scaled A_visc skeleton column weights
  static FaceDev nof() { return FaceDev{}; }

  // ---- multigrid
  HostMesh coarse;
  int mg_levels = 0;  // refinements from `coarse` to `mesh` (0: no hierarchy given)
  bool use_mg = false;
  std::vector<MgLevel> mg;
  double* dKp_raw = nullptr;        // unscaled finest pressure operator on sPp
  double* dAinv = nullptr;          // dense pseudo-inverse of the coarse-solve level's operator (replicated)
  float* dAinv32 = nullptr;         // its fp32 copy (the fp32 V-cycle, when that level is not the coarsest)
  // The V-cycle's dense coarse solve runs on level mg_dense_l: 0 (the coarsest, mesh_fine's 1,067 nodes), or with
  // PUCFEM_MG_DENSE_LEVEL=1 (measurement knob) on level 1: the ~3.6k-node level's 8 latency-bound launches per V-cycle
  // and the coarsest's dense solve replaced by one fp32 dense product.  At L7: 238 -> 214 launches per step, the
  // window +0.3 %, steady +0.6 % (within the spread), but the per-step parity margin at L7 5.7x / 7.5x -> 3.6x / 5.2x
  // (the iterates take another path to the tolerance) and setup +1 s (r12f / r12g): off.
  int mg_dense_l = 0;
  std::future<std::vector<double>> dense_fut;  // level mg_dense_l > 0: its inverse, computed beside the rest of setup
  bool mg_single = false;                        // fp32 V-cycle
  double* z = nullptr;              // preconditioned residual (finest; the fp64 V-cycle's)
  // the fp32 V-cycle's z: its last smoothing step computes in fp32, so z is fp32-exact -- stored as such,
  // the direction kernel gathers 4 B per point instead of 8 and p = z + beta p_old is the same
  float* z32 = nullptr;
  // successive right-hand sides: per pressure solve (which = 1: p, 2: p2) an A-orthonormal basis of
  // up to proj_k solution directions, the projected guess x0 and the new direction
  // (which = 3, 4: the viscous solve's x and y components, proj_k_visc directions each)
  int proj_k = 0, proj_k_visc = 0;
  ProjT* projX[5] = {};
  i64 ldx = 0;  // column-major basis (PUCFEM_PROJ_TILED=0): the vectors' stride, nloc rounded up to even
  // the basis of slot w: its ld argument (tiled: the capacity) and the offset of its vector i
  i64 pld(int w) const { return PUCFEM_PROJ_TILED ? (w <= 2 ? proj_k : proj_k_visc) : ldx; }
  i64 pcol(int w, int i) const { return PUCFEM_PROJ_TILED ? 64 * (i64)i : (i64)i * ldx; }
  double* proj_x0[5] = {};
  int proj_m[5] = {0, 0, 0, 0, 0};
  // Deferred update (project_guess): after a solve only v = y - x0 and A v are formed; the next
  // guess of the same solve orthogonalises v against X, appends it and projects the new right-hand
  // side in one multi-dot and one combination pass over X.  h_coef (pinned) receives each guess's
  // coefficients, read at the next guess to track the coordinates of the recent solutions in the
  // basis (re-seeding a full basis, proj_reseed).  PUCFEM_PROJ_KEEP (measurement knob, 2..16,
  // default 16): seeds kept.
  static constexpr int NCOEF = 2 * PROJ_MAX + 4;
  double* h_coef = nullptr;
  ProjT* projXalt[5] = {};
  struct ProjHist {
    std::vector<std::vector<double>> sols;  // coordinates of the last solutions
    std::vector<double> gamma;              // coordinates of the last guess x0
    int coef_m = -1;                        // h_coef holds a guess over coef_m directions (-1: none)
  } proj_hist[5];
  int proj_keep = std::getenv("PUCFEM_PROJ_KEEP")
                      ? std::max(2, std::min(PROJ_KEEP_MAX, std::atoi(std::getenv("PUCFEM_PROJ_KEEP"))))
                      : 16;
  double *proj_part = nullptr, *proj_d = nullptr, *proj_coef = nullptr;
  double* dqm = nullptr;  // re-seed coefficients (QMat) on the device
  bool proj_pend[5] = {false, false, false, false, false};  // v / A v wait for the next guess
  double *pv[5] = {}, *pav[5] = {};
  // Pressure directions left pending (one rank, lattice, multigrid, shared-basis-free or shared): after a solve
  // the projection update's v = y - x0 and A v = r0 - r_final are not stored; the next solve's k_mdot2 /
  // k_pcomb form them from y, x0, pav (r0) and cg_r[0] (r_final) -- the same values, 60 B/row of k_diff2_fin
  // saved for 24 B/row more in those passes -- and the gradient projection gathers the solution y through
  // the merged (slave -> master) face tables and SELL columns instead of a separate p = y with the slaves
  // copied (p_s = p_m exactly, so the same values).  proj_materialize() stores a pending direction
  // (k_diff2) before anything could overwrite its inputs.
  bool p_from_y = false;
  DevSell dPm;  // dP with merged columns (the gradient's gathers of y)
  bool pend_otf[5] = {};
  const double* pend_y[5] = {};
  // the solve after a projected guess accumulates its correction v = sum alpha_k p_k in pv[slot] (k_cg_upd's
  // vacc; k_pcomb clears it with the guess): pend_acc -- the pending / stored v is that accumulator, not y - x0
  bool pend_acc[5] = {};
  // the accumulated v of slot is zero (its solve passed at the guess: no update ran, so the accumulator, which the
  // first update starts instead of a cleared buffer, was not written); k_mdot2 / k_pcomb then read no v
  bool pend_vzero[5] = {};
  double* cg_vacc = nullptr;  // pcg_mg's accumulator of the current solve (null: none)
  // keep: a slot whose pending direction stays (its r_final is the one cg_r[0] still holds)
  void proj_materialize(int keep = 0) {
    for (int w = 1; w <= 2; ++w) {
      if (!pend_otf[w] || w == keep) continue;
      const i64 n = lp.n_own;
      algo_bytes += 48.0 * (double)n;
      hipLaunchKernelGGL(k_diff2, dim3(grid_ew(n)), dim3(BS), 0, st, n, pend_y[w], (const double*)proj_x0[w],
                         pend_acc[w] ? (double*)nullptr : pv[w],
                         (const double*)pav[w], (const double*)cg_r[0], pav[w]);
      KCHK();
      pend_otf[w] = false;
    }
  }
  // viscous warm start u^n + a polynomial extrapolation of the increments u* - u of the last steps:
  // dvinc[0..1] the last (x, y), [2..3] the one before, [4..5] the one before that, ...;
  // PUCFEM_VISC_EXTRAP (measurement knob): the order, 0 (off) .. VINC_MAX, default 5 (round 2, L7 driver
  // command with the Chebyshev solve: 77 / 71 / 67 viscous steps per 20 steps for orders 3 / 4 / 5,
  // 106.1 / 107.0 / 107.2 steps/s, r5e; orders 6 / 7: 64 steps, within the spread, r6e; L7, 40 steps,
  // round 1: viscous iterations per step 5 / 4 / 3 / 2-3 for orders 0-3, 17.47 / 16.82 / 16.12 /
  // 15.75 ms per step)
  float* dvinc[2 * VINC_MAX] = {};
  int have_vinc = 0;
  int visc_extrap = std::getenv("PUCFEM_VISC_EXTRAP") ? std::max(0, std::min(VINC_MAX, std::atoi(std::getenv("PUCFEM_VISC_EXTRAP")))) : 5;
  // the operator a basis is A-orthonormal for: the pressure solves' unscaled merged operator (null
  // space: constants on the free dofs, cleared from new directions) or the Jacobi-scaled A_visc
  struct ProjOp {
    const DevSell* A;
    const double* val;
    const int32_t* null_free;  // master_of (free rows: < 0) when the operator has the constants' null space
    int kmax;
    FaceDev fc;
  };
  ProjOp proj_op(int which) const {
    return which <= 2 ? ProjOp{&dPp, dKp_raw, dmaster_of, proj_k, fP.full()}
                      : ProjOp{&dP, dKv, nullptr, proj_k_visc, fVisc.full()};
  }
  float* r32 = nullptr;             // fp32 copy of the CG residual: the fp32 V-cycle's right-hand side

  ~Ctx() {
    if (!host_only) {
      if (st) (void)hipStreamSynchronize(st);
      if (gexec) (void)hipGraphExecDestroy(gexec);
      if (graph) (void)hipGraphDestroy(graph);
      if (gexec_k) (void)hipGraphExecDestroy(gexec_k);
      if (graph_k) (void)hipGraphDestroy(graph_k);
      if (st_fk) (void)hipStreamDestroy(st_fk);
      if (ev_fk) (void)hipEventDestroy(ev_fk);
      if (ev_fj) (void)hipEventDestroy(ev_fj);
      for (void* a : allocs) (void)hipFree(a);
      if (h_ctl) (void)hipHostFree(h_ctl);
      if (h_coef) (void)hipHostFree(h_coef);
      if (h_pinned) (void)hipHostFree(h_pinned);
      if (h_yr_pin) (void)hipHostFree(h_yr_pin);
      if (ev_yr) (void)hipEventDestroy(ev_yr);
      for (int k = 0; k < 2; ++k) {
        if (stage[k]) (void)hipHostFree(stage[k]);
        if (stage_ev[k]) (void)hipEventDestroy(stage_ev[k]);
      }
      comm.reset();
      if (st_sl) (void)hipStreamSynchronize(st_sl);
      if (ev_u) (void)hipEventDestroy(ev_u);
      if (ev_sl) (void)hipEventDestroy(ev_sl);
      if (ev_gate) (void)hipEventDestroy(ev_gate);
      if (ev_wait) (void)hipEventDestroy(ev_wait);
      if (st_sl) (void)hipStreamDestroy(st_sl);
      if (st) (void)hipStreamDestroy(st);
    }
  }

  template <class T>
  T* dalloc(i64 n) {
    if (n <= 0) n = 1;
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, sizeof(T) * (size_t)n));
    HIPCHK(hipMemsetAsync(p, 0, sizeof(T) * (size_t)n, st));
    allocs.push_back(p);
    return (T*)p;
  }
  template <class T>
  T* upload(const std::vector<T>& v) {
    T* p = dalloc<T>((i64)v.size());
    if (!v.empty()) h2d(p, v.data(), sizeof(T) * v.size());
    return p;
  }
  // Setup copies of large pageable arrays through two pinned staging buffers (double-buffered; the host
  // side of every chunk copied by the host threads): a pageable hipMemcpy moved 3 GB of device-assembly
  // results in 0.66 s at L7.  h2d is ordered on st like hipMemcpyAsync; d2h returns with the data in dst.
  static constexpr size_t STAGE_BYTES = size_t(64) << 20;
  char* stage[2] = {nullptr, nullptr};
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  bool stage_busy[2] = {false, false};
  void stage_wait(int k) {
    if (!stage[k]) {
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&stage[k]), STAGE_BYTES));
      HIPCHK(hipEventCreateWithFlags(&stage_ev[k], hipEventDisableTiming));
    }
    if (stage_busy[k]) HIPCHK(hipEventSynchronize(stage_ev[k]));
    stage_busy[k] = false;
  }
  static void host_copy(char* dst, const char* src, size_t len) {
    parallel_for((i64)len, [&](i64 a, i64 b) { std::memcpy(dst + a, src + a, (size_t)(b - a)); });
  }
  void h2d(void* dst, const void* src, size_t bytes) {
    if (bytes < (size_t(8) << 20)) {
      HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
      return;
    }
    for (size_t off = 0, i = 0; off < bytes; off += STAGE_BYTES, ++i) {
      const size_t len = std::min(STAGE_BYTES, bytes - off);
      const int k = (int)(i & 1);
      stage_wait(k);
      host_copy(stage[k], static_cast<const char*>(src) + off, len);
      HIPCHK(hipMemcpyAsync(static_cast<char*>(dst) + off, stage[k], len, hipMemcpyHostToDevice, st));
      HIPCHK(hipEventRecord(stage_ev[k], st));
      stage_busy[k] = true;
    }
  }
  void d2h(void* dst, const void* src, size_t bytes) {
    if (bytes < (size_t(8) << 20)) {
      HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      return;
    }
    size_t prev_off = 0, prev_len = 0;
    int prev_k = -1;
    for (size_t off = 0, i = 0; off < bytes; off += STAGE_BYTES, ++i) {
      const size_t len = std::min(STAGE_BYTES, bytes - off);
      const int k = (int)(i & 1);
      stage_wait(k);
      HIPCHK(hipMemcpyAsync(stage[k], static_cast<const char*>(src) + off, len, hipMemcpyDeviceToHost, st));
      HIPCHK(hipEventRecord(stage_ev[k], st));
      stage_busy[k] = true;
      if (prev_k >= 0) {  // the previous chunk, while this one is in flight
        stage_wait(prev_k);
        host_copy(static_cast<char*>(dst) + prev_off, stage[prev_k], prev_len);
      }
      prev_off = off;
      prev_len = len;
      prev_k = k;
    }
    if (prev_k >= 0) {
      stage_wait(prev_k);
      host_copy(static_cast<char*>(dst) + prev_off, stage[prev_k], prev_len);
    }
  }
  // int16 column deltas for a square operator's SELL (prm.idx32 = 0 and the band fits); nloc: the
  // local vector length (owned + ghost), the wrap modulus
  void attach_c16(const Sell& S, i64 nloc, DevSell& D) {
    if (!S.rows.empty()) return;  // row lists (lattice skeleton rows): int32 columns
    std::vector<int16_t> c16;
    if (!prm.idx32 && sell_col16(S, nloc, c16)) {
      D.c16 = upload(c16);
      D.wrap = (int32_t)nloc;
    }
  }
  // operator assembly on the device (prm.assembly 0 on a context bound to a device)
  bool dev_asm() const { return !host_only && prm.assembly == 0; }
  void need_dev() const {
    if (host_only) throw Error(PUCFEM_ENODEV, "compute call on a host-only context");
  }
  void need_built() const {
    if (!built) throw Error(PUCFEM_ESTATE, "pucfem_build_operators has not been called");
  }

  static int nb_for(i64 nslices) { return (int)std::max<i64>(1, std::min<i64>(EWB, (nslices + 3) / 4)); }
  // grid of the V-cycle kernels that produce no partials (more waves in flight than MAXB blocks)
  int mg_nb_max = 16384;
  int nb_mg(i64 nslices) const { return (int)std::max<i64>(1, std::min<i64>(mg_nb_max, (nslices + 3) / 4)); }
  int nb_rows(i64 n) const { return nb_for((n + 63) / 64); }
  // semi-Lagrangian grid: latency-bound gathers want more waves in flight than MAXB blocks give
  // PUCFEM_SL_BLOCKS (measurement knob): a cap on k_sl's grid below SLB (fewer resident waves beside the main
  // stream's kernels; the rows per block grow, the per-wave queue follows them)
  int sl_cap = std::getenv("PUCFEM_SL_BLOCKS") ? std::max(8, std::min(SLB, std::atoi(std::getenv("PUCFEM_SL_BLOCKS"))))
                                               : SLB;
  // PUCFEM_SL_LDS (measurement knob): dynamic LDS bytes requested by the k_sl launches (unused by the kernel): caps
  // the k_sl blocks resident per CU (160 KB / bytes), leaving wave slots and registers to the main stream
  size_t sl_lds = std::getenv("PUCFEM_SL_LDS") ? (size_t)std::max(0, std::min(65536, std::atoi(std::getenv("PUCFEM_SL_LDS"))))
                                               : 0;
  // PUCFEM_SL_WAVE (measurement knob): the lattice locator's second pass -- 2 (default) the numbered list
  // (k_sl_qscan + k_sl_wq + k_sl_qsum), 1 k_sl_wave (each wave its own queue), 0 k_sl_slow (one lane per point)
  int sl_wave_mode = std::getenv("PUCFEM_SL_WAVE") ? std::atoi(std::getenv("PUCFEM_SL_WAVE")) : 2;
  bool sl_wave = sl_wave_mode != 0;
  int nb_sl(i64 n) const {
    if (sl_rec_wave(n)) return (int)((n + BS / 64 - 1) / (BS / 64));  // k_sl_rec_wave: a wave per row
    return (int)std::max<i64>(1, std::min<i64>(sl_cap, (n + 4 * 64 - 1) / (4 * 64)));
  }
  // the record locator on a small mesh (mesh.1, mesh_fine): one wave per row in one launch instead of k_sl queueing
  // every row for k_sl_slow's one lane per point (PUCFEM_SL_WAVE=0 keeps the two passes)
  bool sl_rec_wave(i64 n) const { return !lat_sl && sl_wave && n <= SLB * (BS / 64); }
  static int grid_ew(i64 n) { return (int)std::max<i64>(1, std::min<i64>(2048, (n + BS - 1) / BS)); }
  // A grid-stride kernel whose grid holds more blocks than the chip keeps resident runs its work in two rounds of
  // equal blocks, the second on part of the chip (k_mdot2 at 96 VGPRs: 5 blocks per CU resident, 1,280 of its 2,048);
  // fit_grid gives the resident count (hipOccupancy..., cached per kernel) for such a grid.  With PUCFEM_FIT_GRID=1
  // (measurement knob, off) k_mdot2 keeps its 2,048 blocks' rows and partials as virtual blocks run by a grid of
  // nb / ceil(nb / resident) blocks: the same bits, and no faster (461 vs 465 us, r14g: 1,024 blocks of two units at
  // 4 blocks per CU).  Capping the grid itself made k_mdot2 442 -> 397 us, but its partials then group other rows, the
  // projection's guesses differ in their last bits and with them where each production solve stops below rtol: the
  // L7 per-step margins went 5.7x / 7.5x -> 2.8x / 2.6x (r14d / r14e), so the plain grid stays.
  bool fit_grid_on = std::getenv("PUCFEM_FIT_GRID") && std::atoi(std::getenv("PUCFEM_FIT_GRID")) != 0;
  std::map<const void*, int> resident_blocks;
  int n_cu = 0;
  int fit_grid(const void* kern, int nb) {
    if (!fit_grid_on) return nb;
    auto it = resident_blocks.find(kern);
    if (it == resident_blocks.end()) {
      if (n_cu == 0) {
        int d = 0;
        HIPCHK(hipGetDevice(&d));
        HIPCHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, d));
      }
      int per = 0;
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, BS, 0));
      it = resident_blocks.emplace(kern, std::max(1, per) * std::max(1, n_cu)).first;
    }
    return std::max(1, std::min(nb, it->second));
  }

  // ------------------------------------------------------------------ timing helpers
  // Launch on the library stream.  When timing (cls >= 0), the start / stop events are taken by the
  // kernel's dispatch itself (hipExtLaunchKernelGGL): the sample is the kernel's own duration, as
  // rocprofv3 reports it, without the command-processor gap a separately recorded event adds.
  size_t kl_lds = 0;  // dynamic LDS of the launch (0 but around the k_sl launches with PUCFEM_SL_LDS)
  template <typename... KArgs, typename... Args>
  void klaunch(int cls, double bytes, void (*kernel)(KArgs...), dim3 g, dim3 b, Args... args) {
    algo_bytes += bytes;
    if (cls >= 0) {
      cls_bytes[cls] += bytes;
      ++cls_n[cls];
    }
    if (timer.on && cls >= 0 && ((timer.mask >> cls) & 1u)) {
      hipEvent_t a = timer.get(), e = timer.get();
      ++g_nlaunch;
      hipExtLaunchKernelGGL(kernel, g, b, kl_lds, st, a, e, 0, args...);
      timer.pend.push_back({cls, a, e, bytes});
      if (timer.pend.size() > 4096) timer.flush();  // bounded number of live events
    } else {
      hipLaunchKernelGGL(kernel, g, b, kl_lds, st, args...);
    }
  }
  // The solvers' host reads (convergence tests, |r_0|) wait by polling the event instead of a blocking
  // synchronize: a blocking wait that outlasts the runtime's short active spin sleeps on an interrupt, and
  // its wake-up left the GPU idle ~0.1 ms after every pressure solve (r10x trace: 124 us before each
  // k_grad_proj).  PUCFEM_SPIN_WAIT=0 keeps the blocking calls (measurement knob).
  bool spin_wait = !(std::getenv("PUCFEM_SPIN_WAIT") && std::atoi(std::getenv("PUCFEM_SPIN_WAIT")) == 0);
  int spin_us = std::getenv("PUCFEM_SPIN_US") ? std::max(0, std::atoi(std::getenv("PUCFEM_SPIN_US"))) : 500;
  hipEvent_t ev_wait = nullptr;
  void wait_event(hipEvent_t e) {
    if (!spin_wait) {
      HIPCHK(hipEventSynchronize(e));
      return;
    }
    // a bounded spin (the solvers' reads wait tens of microseconds): a longer wait blocks, so no host core
    // stays pinned beside other ranks' and the setup's threads
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0;; ++k) {
      const hipError_t q = hipEventQuery(e);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) HIPCHK(q);
      if ((k & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) {
        HIPCHK(hipEventSynchronize(e));
        return;
      }
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    }
  }
  void sync_st() {  // hipStreamSynchronize(st) for the solvers' reads
    if (!spin_wait) {
      HIPCHK(hipStreamSynchronize(st));
      return;
    }
    if (!ev_wait) HIPCHK(hipEventCreateWithFlags(&ev_wait, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ev_wait, st));
    wait_event(ev_wait);
  }

  // k_sl over rows [row0, row0 + n) of the full replica c (cout: the new values), either locator
  void sl_launch(int nb, i64 row0, i64 n, const double* vx, const double* vy, double dt, const double* cf, double* cn,
                 const double* w, int32_t* nf, RedOut ro = RedOut{}) {
    const MeshDev M{mx, my, mtri, mesh.T};
    struct LdsScope {  // (reset on unwind)
      size_t& v;
      LdsScope(size_t& x, size_t n) : v(x) { v = n; }
      ~LdsScope() { v = 0; }
    } lds_scope(kl_lds, sl_lds);
    if (lat_sl) {
      // per row: coordinates 16, u 16, c 8 (the departure triangle's vertices lie near the row: their
      // coordinate and c lines are the rows' own), home face 4, lattice cell entries 8 and fast-accept
      // radii 8 (two triangles per node), the mixing weight 8, c_new written 8
      const double sl_bytes = (16.0 + 16.0 + 8.0 + 4.0 + 8.0 + 8.0 + (w ? 8.0 : 0.0) + 8.0) * (double)n;
      klaunch(4, sl_bytes, k_sl<LatLocDev>, dim3(nb), dim3(BS), M, llgrid, (int64_t)row0, (int64_t)n, vx,
              vy, dt, cf, cn, w, nf, part_sl, sl_queue, sl_qcnt);
      kl_lds = 0;  // (the knob's LDS is k_sl's alone: k_sl_slow has static LDS of its own)
      // the queued rows: one wave per point (k_sl_wave, on k_sl's grid), or -- with the fused reductions (a
      // measurement knob) or PUCFEM_SL_WAVE=0 -- k_sl_slow on k_sl's grid, one lane per point
      if (sl_wave_mode == 2 && !ro.out) {
        const int32_t nq = nb * (BS / 64);
        if (nq > QSCAN_BS * QSCAN_PER) throw Error(PUCFEM_ESTATE, "k_sl grid larger than k_sl_qscan covers");
        hipLaunchKernelGGL(k_sl_qscan, dim3(1), dim3(QSCAN_BS), 0, st, (const int32_t*)sl_qcnt, nq, sl_qoff);
        KCHK();
        klaunch(8, 0.0, k_sl_wq, dim3(nb), dim3(BS), M, llgrid, cgrid, (int64_t)row0, (int64_t)n, (int32_t)nb, vx, vy,
                dt, cf, cn, nf, sl_queue, (const int32_t*)sl_qoff, nq);
        KCHK();
        hipLaunchKernelGGL(k_sl_qsum, dim3(nb), dim3(BS), 0, st, (int64_t)row0, (int64_t)n, (const double*)cn, w,
                           part_sl, (const int32_t*)sl_queue, (const int32_t*)sl_qcnt);
      } else if (sl_wave && !ro.out)
        klaunch(8, 0.0, k_sl_wave, dim3(nb), dim3(BS), M, llgrid, cgrid, (int64_t)row0, (int64_t)n, vx, vy, dt, cf, cn,
                w, nf, part_sl, (const int32_t*)sl_queue, (const int32_t*)sl_qcnt);
      else
        klaunch(8, 0.0, k_sl_slow<LatLocDev>, dim3(nb), dim3(BS), M, llgrid, cgrid, (int64_t)row0, (int64_t)n, vx, vy,
                dt, cf, cn, w, nf, part_sl, (const int32_t*)sl_queue, (const int32_t*)sl_qcnt, ro);
    } else if (sl_rec_wave(n)) {
      kl_lds = 0;
      klaunch(4, 8.0 * 6 * (double)n, k_sl_rec_wave, dim3(nb), dim3(BS), M, lgrid, cgrid, (int64_t)row0, (int64_t)n, vx,
              vy, dt, cf, cn, w, nf, part_sl, ro);
    } else {
      klaunch(4, 8.0 * 6 * (double)n, k_sl<LocDev>, dim3(nb), dim3(BS), M, lgrid, (int64_t)row0, (int64_t)n, vx, vy,
              dt, cf, cn, w, nf, part_sl, sl_queue, sl_qcnt);
      kl_lds = 0;
      klaunch(8, 0.0, k_sl_slow<LocDev>, dim3(nb), dim3(BS), M, lgrid, cgrid, (int64_t)row0, (int64_t)n, vx, vy, dt,
              cf, cn, w, nf, part_sl, (const int32_t*)sl_queue, (const int32_t*)sl_qcnt, ro);
    }
  }



  // ------------------------------------------------------------------ fused reductions
  // The step's partial-producing kernels reduce their own partials (RedOut: the last block to finish
  // sums them, pucfem_kernels.hpp) instead of a k_reduce launch after them.  One ticket counter per
  // launch site (a site's launches are ordered on its stream; the dye stream's sites have their own).
  // Off by default (PUCFEM_FUSED_RED=1 turns it on, a measurement knob): at L7 the fused path ran 101.4
  // steps/s against 107.2 with k_reduce (r8a/r8b, same box type): under streaming load each block's
  // write-through partial store and returned ticket (two memory round trips in the block's tail) cost
  // 10-25 us per producer launch, more than the 9-14 us k_reduce launch they remove.
  enum { CNT_VCHEB, CNT_INIT, CNT_RZ, CNT_DIR, CNT_UPD, CNT_DIV, CNT_MDOT, CNT_MIX, CNT_SL, CNT_DYE_DIV = 16,
         CNT_DYE_SL, CNT_DYE_MIX, CNT_N = 32 };
  unsigned* dcnt = nullptr;
  bool fused_red = std::getenv("PUCFEM_FUSED_RED") && std::atoi(std::getenv("PUCFEM_FUSED_RED")) != 0;
  RedOut ro(double* out, int cnt, int nv, int stride = MAXB, unsigned maxmask = 0u, double* out1 = nullptr) const {
    if (!fused_red || !dcnt) return RedOut{};
    return RedOut{out, out1, dcnt + cnt, nv, stride, maxmask};
  }
  // after a fused reduction into out[0..nv): the all-reduce across ranks
  void red_done(double* out, int nv, bool is_max) {
    if (dist()) comm->allreduce(out, nv, is_max, st);
  }
  RedOut ro_rz{};  // the finest level's last smoothing step (<r, z>), set by pcg_mg around precondition()

  // ------------------------------------------------------------------ communication
  // partials of a producer kernel -> nv final values in redbuf slot `slot` (one 1-block kernel, then
  // the all-reduce across ranks): consumers read one scalar instead of re-reducing up to MAXB
  // partials in each of their blocks
  // the dye stream's reductions run in 256-thread blocks: a 1,024-thread block needs 16 free wave slots on
  // one CU, which the main stream's kernels rarely leave (the k_sl sums waited ~270 us for a CU, r10a)
  bool red_small = false;
  void launch_reduce(const double* part, int nb, int stride, int nv, bool is_max, double* out) {
    // one block per value (k_reduce_t)
    if (red_small)
      hipLaunchKernelGGL(k_reduce_t<256>, dim3(std::max(1, nv)), dim3(256), 0, st, part, nb, stride, nv,
                         is_max ? 1 : 0, out);
    else
      hipLaunchKernelGGL(k_reduce, dim3(std::max(1, nv)), dim3(RB), 0, st, part, nb, stride, nv, is_max ? 1 : 0, out);
  }
  Red reduce_global(double* part, int nb, int nv, bool is_max, int slot) {
    double* buf = redbuf + 8 * slot;
    launch_reduce(part, nb, MAXB, nv, is_max, buf);
    KCHK();
    if (dist()) comm->allreduce(buf, nv, is_max, st);
    return Red{buf, 1, 1};
  }
  // reduce partials into vals[slot..slot+nv) (+ all-reduce)
  void reduce_into(double* part, int nb, int nv, bool is_max, int slot, int stride = MAXB) {
    launch_reduce(part, nb, stride, nv, is_max, vals + slot);
    KCHK();
    if (dist())
      comm->allreduce(vals + slot, nv, is_max, st);
  }
  // refresh the ghost entries of up to two local vectors
  void halo(double* a, double* b = nullptr) { halo_lp(lp, dsend, dsendbuf, nsend, a, b); }
  template <typename T>
  void halo_lp(const LocalPlan& P, const int32_t* sidx, T* sbuf, i64 ns, T* a, T* b = nullptr) {
    if (!dist() || (P.send_peer.empty() && P.recv_peer.empty())) return;
    if (ns > 0) {
      hipLaunchKernelGGL(k_pack<T>, dim3(grid_ew(ns)), dim3(BS), 0, st, ns, sidx, a, b, sbuf);
      KCHK();
    }
    comm->group_start();
    for (size_t k = 0; k < P.send_peer.size(); ++k) {
      comm->send(sbuf + P.send_off[k], P.send_cnt[k], P.send_peer[k], st);
      if (b) comm->send(sbuf + ns + P.send_off[k], P.send_cnt[k], P.send_peer[k], st);
    }
    for (size_t k = 0; k < P.recv_peer.size(); ++k) {
      comm->recv(a + P.n_own + P.recv_off[k], P.recv_cnt[k], P.recv_peer[k], st);
      if (b) comm->recv(b + P.n_own + P.recv_off[k], P.recv_cnt[k], P.recv_peer[k], st);
    }
    comm->group_end(st);
  }
  template <typename T>
  void mg_halo(MgLevel& L, T* a, T* b = nullptr) {  // (two vectors: one grouped exchange; sendbuf holds 2 nsend)
    if (&L == &mg.back()) halo_lp(lp, dsend, bufs<T>(L).sendbuf, nsend, a, b);
    else halo_lp(L.lp, L.dsend, bufs<T>(L).sendbuf, L.nsend, a, b);
  }
  // Before the semi-Lagrangian step on W > 1 ranks: refresh the dye replica where this step's
  // back-traced points can reach -- the strips within dt max|u_y| + (largest triangle height) of each
  // rank's own y extent -- with point-to-point copies of contiguous internal-id ranges (every rank's
  // own segment is current: its SL wrote it).  Replaces the all-gather of the whole field (SURVEY.md
  // §8e: the departure distance bounds the gather).
  // The wide halo in two halves.  dye_range_start: every rank's range of back-traced y (StokesColor.py:361-372),
  // all-gathered as a max-reduction of a 2 W vector holding (1 - min, max) in each rank's slot, copied to pinned
  // host memory behind an event.  dye_halo_exchange: once that copy has landed, the point-to-point copies of the
  // strip ranges each rank reads.  The step (stokes_step) queues the first half at its end and the second half at
  // the next step, after that step's viscous solve, whose host round trip has seen the copy land -- no blocking
  // read of its own (round 5 synchronised the stream here every step).
  double* h_yr_pin = nullptr;  // 2 W (pinned)
  hipEvent_t ev_yr = nullptr;
  void dye_range_start(const double* vy, double dt) {
    const i64 n = lp.n_own;
    const int nb = nb_rows(n);
    if (!h_yr_pin) {
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h_yr_pin), sizeof(double) * 2 * world));
      HIPCHK(hipEventCreateWithFlags(&ev_yr, hipEventDisableTiming));
    }
    hipLaunchKernelGGL(k_yrange, dim3(nb), dim3(BS), 0, st, n, my + lp.r0, vy, dt, part_u);
    KCHK();
    hipLaunchKernelGGL(k_reduce, dim3(2), dim3(RB), 0, st, part_u, nb, MAXB, 2, 1, yr_own);
    hipLaunchKernelGGL(k_place2, dim3(1), dim3(64), 0, st, world, rank, (const double*)yr_own, yr_all);
    KCHK();
    comm->allreduce(yr_all, 2 * (size_t)world, true, st);
    HIPCHK(hipMemcpyAsync(h_yr_pin, yr_all, sizeof(double) * 2 * world, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(ev_yr, st));
  }
  void dye_halo_exchange() {
    wait_event(ev_yr);  // (at the step's use: long complete, a query)
    std::copy(h_yr_pin, h_yr_pin + 2 * world, h_yr.begin());
    const i64 S = (i64)strip_ylo.size();
    auto need = [&](int j, i64& a, i64& b) {  // internal-id range rank j reads: the strips that meet
      // its back-traced y range widened by a triangle height (the located triangle's vertices)
      const double lo = (1.0 - h_yr[2 * j]) - tri_hy - 1e-9, hi = h_yr[2 * j + 1] + tri_hy + 1e-9;
      i64 sa = 0, sb = S;
      while (sa < S && strip_yhi[sa] < lo) ++sa;
      while (sb > sa && strip_ylo[sb - 1] > hi) --sb;
      a = ord.strip_ptr[sa];
      b = ord.strip_ptr[sb];
    };
    const i64 o0 = row_start[rank], o1 = row_start[rank + 1];
    dye_halo_values = 0;
    comm->group_start();
    for (int j = 0; j < world; ++j) {
      if (j == rank) continue;
      i64 a, b;
      need(j, a, b);
      a = std::max(a, o0);
      b = std::min(b, o1);
      if (b > a) comm->send(c_full + a, (size_t)(b - a), j, st);
    }
    i64 a0, b0;
    need(rank, a0, b0);
    for (int j = 0; j < world; ++j) {
      if (j == rank) continue;
      const i64 a = std::max(a0, row_start[j]), b = std::min(b0, row_start[j + 1]);
      if (b > a) {
        comm->recv(c_full + a, (size_t)(b - a), j, st);
        dye_halo_values += b - a;
      }
    }
    comm->group_end(st);
  }
  // full replica <- every rank's owned segment (internal numbering is rank-contiguous)
  void allgather_full(double* full) {
    if (!dist()) return;
    comm->group_start();
    for (int r = 0; r < world; ++r) {
      const i64 o = row_start[r], n = row_start[r + 1] - row_start[r];
      comm->bcast(full + o, n, r, st);
    }
    comm->group_end(st);
  }

  // ------------------------------------------------------------------ CG
  template <int NR>
  int cg(const DevSell& A, const HFace& hf, const double* val, double* const y[NR], const double* const b[NR],
         double tol, int maxit, int which) {
    if (!dist() && block_cg && !hf.items && A.nrows <= (int64_t)CGB_THREADS * CGB_MAXR) {
      const size_t vec = (size_t)NR * A.nrows * sizeof(double);
      const size_t mat = (size_t)A.padded * (sizeof(double) + sizeof(int32_t));
      const bool mat_lds = vec + mat <= (size_t)150 * 1024;
      const size_t lds = vec + (mat_lds ? mat : 0);
      // the attribute is per device and function: set it once per context (a context is bound to one
      // device; a second context on the same device sets it again, which is harmless)
      if (!lds_attr[NR]) {
        HIPCHK(hipFuncSetAttribute((const void*)k_cg_block<NR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   150 * 1024));
        lds_attr[NR] = true;
      }
      int* slot = dits ? dits + 3 * cur_step + which : nullptr;
      hipLaunchKernelGGL((k_cg_block<NR>), dim3(1), dim3(CGB_THREADS), lds, st, A.view(), val, y[0],
                         NR > 1 ? y[1] : (double*)nullptr, b[0], NR > 1 ? b[1] : (const double*)nullptr, tol * tol,
                         maxit, mat_lds ? 1 : 0, ctl, slot);
      KCHK();
      if (dits) return -1;  // collected after the step loop
      HIPCHK(hipMemcpyAsync(h_ctl, ctl, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (h_ctl[0] == 3) throw Error(PUCFEM_ENOCONV, "CG residual is not finite");
      if (h_ctl[0] != 1) throw Error(PUCFEM_ENOCONV, "CG did not converge within maxit=" + std::to_string(maxit));
      return h_ctl[1];
    }
    // multi-kernel Jacobi-scaled CG with the direction updated in place (k_cgr_*): an iteration is
    // the SpMV with its three dots, the update (y, r, p) with the exact <r, r>, and the control test
    const FaceDev fc = hf.part();
    const int nb = grid_part(fc, A);
    CgVecs<NR> v;
    for (int c = 0; c < NR; ++c) {
      v.y[c] = y[c];
      v.b[c] = b[c];
      v.r[c] = cg_r[c];
      v.po[c] = cg_pa[c];  // the direction p
      v.pn[c] = cg_pb[c];
      v.q[c] = cg_q[c];
    }
    auto halo_p = [&]() {
      if (NR == 2) halo(cg_pa[0], cg_pa[1]);
      else halo(cg_pa[0]);
    };
    if (NR == 2) halo(y[0], y[1]);
    else halo(y[0]);
    HIPCHK(hipMemsetAsync(ctl, 0, 2 * sizeof(int), st));
    algo_bytes += (8.0 + A.idx_bytes()) * (double)A.nnz + A.row_bytes() * (double)A.nrows + 32.0 * NR * (double)A.own();
    with_c16(A, [&](auto c16) {
      hipLaunchKernelGGL((k_cg_init<NR, decltype(c16)::value>), dim3(nb), dim3(BS), 0, st, A.view(), fc, val, v,
                         lp.n_ghost, part_a, part_b, (float*)nullptr, 1, RedOut{});
    });
    KCHK();
    Red rr = reduce_global(part_a, nb, NR, false, 0);
    Red bb = reduce_global(part_b, nb, NR, false, 1);
    const double tol2 = tol * tol;
    hipLaunchKernelGGL(k_cgr_ctl, dim3(1), dim3(64), 0, st, rr.p, bb.p, tol2, ctl, 0, maxit, NR);
    KCHK();
    halo_p();
    // algorithmic bytes: dir gathers p once per row and reads r, writes q; upd reads y, p, r, q and
    // writes y, r, p
    const double bytes_dir =
        (8.0 + A.idx_bytes()) * (double)A.nnz + A.row_bytes() * (double)A.nrows + 24.0 * NR * (double)A.own();
    const double bytes_upd = 56.0 * NR * (double)A.own();
    int it = 0;
    // host convergence checks: the first after as many iterations as the last solve took (the control
    // test after each update lets the check see convergence without a further launch)
    int chunk = std::max(1, std::min(maxit + 1, last_it[which] > 0 ? last_it[which] : 4));
    std::vector<ByteMark> bmark;  // the byte counters at the start of each iteration of the current chunk
    for (;;) {
      const int it0 = it;
      bmark.clear();
      for (int k = 0; k < chunk; ++k, ++it) {
        bmark.push_back(bmark_now());
        // HIP-event timing samples every 8th iteration (bounded event count for long solves)
        const bool samp = (it & 7) == 0;
        with_c16(A, [&](auto c16) {
          klaunch(samp ? 1 : -1, bytes_dir, k_cgr_dir<NR, decltype(c16)::value>, dim3(nb), dim3(BS), A.view(), fc,
                  val, v, (const int*)ctl, part_c);
        });
        KCHK();
        Red dots = reduce_global(part_c, nb, 3 * NR, false, 2);
        klaunch(samp ? 2 : -1, bytes_upd, k_cgr_upd<NR>, dim3(nb_rows(A.own())), dim3(BS), v, A.own(),
                (const double*)dots.p, (const double*)rr.p, (const int*)ctl, part_a);
        KCHK();
        rr = reduce_global(part_a, nb_rows(A.own()), NR, false, 0);
        hipLaunchKernelGGL(k_cgr_ctl, dim3(1), dim3(64), 0, st, rr.p, bb.p, tol2, ctl, it + 1, maxit, NR);
        KCHK();
        halo_p();
      }
      HIPCHK(hipMemcpyAsync(h_ctl, ctl, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (timer.on) timer.flush();
      // iterations from the converged one on were launched but did no work
      if (h_ctl[0] && h_ctl[1] >= it0 && h_ctl[1] < it) bmark_restore(bmark[h_ctl[1] - it0]);
      if (h_ctl[0]) break;
      chunk = std::max(1, std::min(64, it / 8));
    }
    last_it[which] = h_ctl[1];
    if (h_ctl[0] == 3) throw Error(PUCFEM_ENOCONV, "CG residual is not finite (iteration " + std::to_string(h_ctl[1]) + ")");
    if (h_ctl[0] != 1)
      throw Error(PUCFEM_ENOCONV, "CG did not converge within maxit=" + std::to_string(maxit));
    return h_ctl[1];
  }

  // Chebyshev iteration for the Jacobi-scaled viscous system (k_vcheb), both components at once in the
  // interleaved (dbl2) vectors: y (warm start, overwritten only through the buffers) and b; the converged
  // iterate is returned in *out (y itself or one of the x buffers).  Target: the CG's test
  // <r, r> <= tol^2 <b, b> per component, met through the a-priori residual bound of the interval (below).
  // fin (optional): the viscous finish (k_visc_fin: u* = S y, the fp32 increment u* - u) for the solve's
  // last step to do in place of its x_out; *fin_done tells whether it did
  struct ViscFin {
    const double* s;
    const double* u[2];
    double* us[2];
    float* inc[2];
  };
  // the interleaved vectors of the viscous Chebyshev solve (allocated with the operators): the start / x
  // buffers, b, and the fp32 increments d (a step pair writes its d to the second buffer)
  dbl2 *vx2[3] = {nullptr, nullptr, nullptr}, *vb2 = nullptr;
  flt2* vd2[2] = {nullptr, nullptr};
  // halo of an interleaved vector (both components of each ghost row)
  void halo2(dbl2* a, dbl2* b = nullptr) {  // (b: a second interleaved vector in the same grouped exchange)
    const LocalPlan& P = lp;
    if (!dist() || (P.send_peer.empty() && P.recv_peer.empty())) return;
    if (nsend > 0) {
      hipLaunchKernelGGL(k_pack<dbl2>, dim3(grid_ew(nsend)), dim3(BS), 0, st, nsend, dsend, (const dbl2*)a,
                         (const dbl2*)b, reinterpret_cast<dbl2*>(dsendbuf));
      KCHK();
    }
    comm->group_start();
    for (size_t k = 0; k < P.send_peer.size(); ++k) {
      comm->send(dsendbuf + 2 * P.send_off[k], 2 * P.send_cnt[k], P.send_peer[k], st);
      if (b) comm->send(dsendbuf + 2 * (nsend + P.send_off[k]), 2 * P.send_cnt[k], P.send_peer[k], st);
    }
    for (size_t k = 0; k < P.recv_peer.size(); ++k) {
      comm->recv(reinterpret_cast<double*>(a + P.n_own + P.recv_off[k]), 2 * P.recv_cnt[k], P.recv_peer[k], st);
      if (b) comm->recv(reinterpret_cast<double*>(b + P.n_own + P.recv_off[k]), 2 * P.recv_cnt[k], P.recv_peer[k], st);
    }
    comm->group_end(st);
  }
  // PUCFEM_VISC_SPEC=0 (measurement knob): no speculative finish ahead of the |r_0| round trip (see vcheb)
  bool visc_spec = !(std::getenv("PUCFEM_VISC_SPEC") && std::atoi(std::getenv("PUCFEM_VISC_SPEC")) == 0);
  int vcheb(const DevSell& A, const HFace& hf, const double* val, dbl2* y, const dbl2* b, double tol, int maxit,
            int which, dbl2** out, const ViscFin* vfin = nullptr, bool* fin_done = nullptr) {
    constexpr int NR = 2;
    if (fin_done) *fin_done = false;
    const FaceDev fc = hf.part();
    const int nb = grid_part(fc, A);
    // step pairs (k_vcheb_pair): a face part of lattice size <= VP_HALO.  On W > 1 ranks only the solve's first pair
    // (0, 1), whose first step also runs on the ghost rows one layer out (deep halos: x and b exchanged two layers
    // out together, one exchange for the two steps); later pairs would need d exchanged too, so single steps
    const bool deepv = dist() && A.has_ghost_rows() && use_mg && mg.back().deep && (deep_mask & 16);
    const DevSell Ag = A.with_ghosts();  // (= A without ghost rows)
    const int nbs = nb_for(Ag.nslices);  // a pair's SELL grids (its first launch covers the ghost rows)
    const bool pairs_ok = visc_pair && hf.items > 0 && fc.n <= VP_HALO &&
                          nbs + hf.items <= MAXB;  // (the check's partials of both halves)
    const bool pairs = pairs_ok && !dist();
    dbl2* xa = y;
    dbl2* xb = vx2[1];
    dbl2* xc = vx2[2];  // step pairs: x_{a+2}
    flt2* dcur = vd2[0];  // the fp32 increments d (in place for single steps)
    flt2* dalt = vd2[1];  // step pairs: d_{a+2}
    HIPCHK(hipMemsetAsync(ctl, 0, 2 * sizeof(int), st));
    const bool pair0 = (pairs || (pairs_ok && deepv)) && !ro(redbuf, CNT_VCHEB, 2 * NR).out;
    if (pair0 && deepv) halo2(xa, const_cast<dbl2*>(b));  // (b's ghosts: the first step on the ghost rows)
    else halo2(xa);
    // the interval [visc_lo, 1 + visc_R]: theta its centre, delta its half-width
    const double hi = 1.0 + visc_R, lo = visc_lo;
    const double theta = 0.5 * (hi + lo), delta = 0.5 * (hi - lo), sigma = theta / delta, tol2 = tol * tol;
    // algorithmic bytes: x gathered once, b, d (fp32; not at the first step) read, d and x_out written
    const double bytes = (8.0 + A.idx_bytes()) * (double)A.nnz + A.row_bytes() * (double)A.nrows +
                         32.0 * NR * (double)A.own();
    // One step: x_out = x_in + d, d = c1 d + c2 (b - A^ x_in); the first step also yields |r_0| and |b|.
    auto step = [&](int it, double c1, double c2, bool check = false, bool fin = false) {
      ChebVecs2 v{};
      v.xin = xa;
      v.xout = xb;
      v.b = b;
      v.d = dcur;
      if (fin) {
        v.s = vfin->s;
        for (int c = 0; c < NR; ++c) {
          v.u[c] = vfin->u[c];
          v.us[c] = vfin->us[c];
          v.inc[c] = vfin->inc[c];
        }
      }
      // timing class 9; the first step reads no d (4 B/row per right-hand side less)
      // step 0 reduces its own partials (fused): |r_0|^2 into redbuf[0 .. NR), |b|^2 into redbuf[NR .. 2 NR)
      const RedOut r0 = it == 0 ? ro(redbuf, CNT_VCHEB, 2 * NR) : RedOut{};
      double* pb = it == 0 ? (r0.out ? part_a + NR * MAXB : part_b) : (double*)nullptr;
      // check: the post-check's |r_it|^2 partials (part_c)
      double* pr = it == 0 ? part_a : (check ? part_c : (double*)nullptr);
      with_c16(A, [&](auto c16) {
        // fin: + s, u read and u*, the increment written - d, x_out
        klaunch(9, (it == 0 ? bytes - 4.0 * NR * (double)A.own() : bytes) + (fin ? 12.0 * NR * (double)A.own() : 0.0),
                k_vcheb<decltype(c16)::value>, dim3(nb),
                dim3(BS), A.view(), fc, val, v, c1, c2, it == 0 ? 1 : 0, (const int*)ctl, pr, pb, r0);
      });
      KCHK();
      if (fin) return;  // the solve's output is u* (haloed by viscous()), x_out was not written
      halo2(xb);
      std::swap(xa, xb);
    };
    // Two steps a, a + 1 in three launches: the skeleton rows' step a (k_vcheb on the SELL part alone),
    // both steps on the face interiors (k_vcheb_pair: x_{a+1} in LDS), the skeleton rows' step a + 1.
    // check: the |r_{a+1}|^2 partials of both halves in part_c (SELL blocks first); fin: step a + 1 is
    // the solve's last and writes u* and the increment.
    const double bytes_sk = (8.0 + A.idx_bytes()) * (double)A.nnz + A.row_bytes() * (double)A.nrows +
                            32.0 * NR * (double)(A.own() - hf.rows);
    // first: the pair is the solve's steps 0 and 1: step 0 reads no d and both halves write the |r_0|^2 /
    // |b|^2 partials (part_a / part_b: the SELL blocks at their block indices, the face items after them)
    auto pair_step = [&](double c1a, double c2a, double c1b, double c2b, bool check, bool fin, bool first = false) {
      FaceDev fs = fc;
      fs.nb = 0;
      ChebVecs2 v1{}, v2{};
      VPairVecs p{};
      v1.xin = xa;
      v1.xout = xb;
      v1.b = b;
      v1.d = dcur;
      v2.xin = xb;
      v2.xout = xc;
      v2.b = b;
      v2.d = dcur;
      v2.dout = dalt;
      p.xa = xa;
      p.xb = xb;
      p.xc = xc;
      p.b = b;
      p.da = dcur;
      p.dc = dalt;
      if (fin) {
        v2.s = p.s = vfin->s;
        for (int c = 0; c < NR; ++c) {
          v2.u[c] = p.u[c] = vfin->u[c];
          v2.us[c] = p.us[c] = vfin->us[c];
          v2.inc[c] = p.inc[c] = vfin->inc[c];
        }
      }
      // face rows: x_a, b, d_a read, x_{a+2}, d_{a+2} written (fin: + s, u read, u*, the increment
      // written - x, d), x_{a+1} written at the rows next to the skeleton (3 (n - 3) per face)
      const double bnd_rows = fc.n > 3 ? 3.0 * (fc.n - 3) * (double)fc.nf : 0.0;
      const double bytes_f = (32.0 * NR + (fin ? 12.0 * NR : 0.0)) * (double)hf.rows + 8.0 * NR * bnd_rows;
      const double fin_sk = fin ? 12.0 * NR * (double)(A.own() - hf.rows) : 0.0;
      double* pc = check ? part_c : nullptr;
      with_c16(A, [&](auto c16) {
        klaunch(-1, bytes_sk - (first ? 4.0 * NR * (double)(A.own() - hf.rows) : 0.0), k_vcheb<decltype(c16)::value>,
                dim3(nbs), dim3(BS), Ag.view(), fs, val, v1, c1a, c2a, first ? 1 : 0, (const int*)ctl,
                first ? part_a : (double*)nullptr, first ? part_b : (double*)nullptr, RedOut{});
        KCHK();
        if (first && dye_gate == 3) dye_tail_release();
        klaunch(12, bytes_f - (first ? 4.0 * NR * (double)hf.rows : 0.0), k_vcheb_pair, dim3(hf.items), dim3(BS), fc, p,
                c1a, c2a, c1b, c2b, (const int*)ctl, pc, (int32_t)nbs, first ? 1 : 0,
                first ? part_a : (double*)nullptr, first ? part_b : (double*)nullptr);
        KCHK();
        if (first && dye_gate == 4) dye_tail_release();
        klaunch(-1, bytes_sk + fin_sk, k_vcheb<decltype(c16)::value>, dim3(nbs), dim3(BS), A.view(), fs, val, v2,
                c1b, c2b, 0, (const int*)ctl, pc, (double*)nullptr, RedOut{});
        KCHK();
      });
      ++visc_pairs;
      if (fin) return;
      // x_{a+2} is current; x_a, x_{a+1} are free
      dbl2* t = xa;
      xa = xc;
      xc = xb;
      xb = t;
      std::swap(dcur, dalt);
      if (dist()) halo2(xa);  // (W > 1: the next single step gathers x_{a+2}'s ghosts)
    };
    // Step 0 gives r_0 = b - A^ x_0.  The residual polynomial of the Chebyshev iteration on an interval
    // holding the spectrum is bounded by 1 / T_k(sigma) there, so |r_k| <= |r_0| / T_k(sigma): the step
    // count K that meets the CG's test |r_K| <= rtol |b| is known after step 0, and steps 1 .. K-1 run with
    // no residual checks, no reductions and no host round trip.  (The bound is rigorous for the interval
    // [visc_lo, 1 + visc_R], which tests/test_host_assembly.py checks against the spectrum; the
    // adaptive test it replaces needed one extra step per solve to see the passing residual.)
    // With step pairs the solve starts with the pair (0, 1) -- one face pass where step 0 and a single step
    // 1 took two -- and the step count K decides the rest: K <= 2 is done (the finish runs as k_visc_fin),
    // K = 3 / 4 add a single step / a pair with the finish.  Without pairs: step 0 alone.
    double rho_old = 1.0 / sigma;
    int done = 1;
    int nb0 = nb;  // the first step's partial count
    if (pair0) {
      const double rho = 1.0 / (2.0 * sigma - rho_old);
      pair_step(0.0, 1.0 / theta, rho * rho_old, 2.0 * rho / delta, true, false, true);
      rho_old = rho;
      done = 2;
      nb0 = nbs + (int)hf.items;
    } else {
      step(0, 0.0, 1.0 / theta);
    }
    Red rr{redbuf, 1, 1}, bb{redbuf + NR, 1, 1};
    if (!pair0 && ro(redbuf, CNT_VCHEB, 2 * NR).out) {
      red_done(redbuf, 2 * NR, false);
    } else {
      rr = reduce_global(part_a, nb0, NR, false, 0);
      bb = reduce_global(part_b, nb0, NR, false, 1);
    }
    HIPCHK(hipMemcpyAsync(h_pinned, rr.p, NR * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h_pinned + 8, bb.p, NR * sizeof(double), hipMemcpyDeviceToHost, st));
    hipEvent_t have_r0 = timer.get();
    HIPCHK(hipEventRecord(have_r0, st));
    // while the host waits for |r_0|, the GPU already runs the steps the last solve certainly needed
    // (one fewer than its count): the round trip hides behind them
    // (step pairs: two steps per pass while at least two are due)
    auto pair_coefs = [&](double& c1a, double& c2a, double& c1b, double& c2b) {
      const double ra = 1.0 / (2.0 * sigma - rho_old), rb = 1.0 / (2.0 * sigma - ra);
      c1a = ra * rho_old;
      c2a = 2.0 * ra / delta;
      c1b = rb * ra;
      c2b = 2.0 * rb / delta;
      rho_old = rb;
    };
    auto advance = [&](int upto) {
      while (done < upto) {
        if (pairs && upto - done >= 2) {
          double c1a, c2a, c1b, c2b;
          pair_coefs(c1a, c2a, c1b, c2b);
          pair_step(c1a, c2a, c1b, c2b, false, false);
          done += 2;
          continue;
        }
        const double rho = 1.0 / (2.0 * sigma - rho_old);
        step(done, rho * rho_old, 2.0 * rho / delta);
        rho_old = rho;
        ++done;
      }
    };
    // with step pairs only whole pairs go ahead of the round trip, and at least the last two steps
    // wait for it (so that they can run as one pair with the finish)
    advance(pair0 ? 2 + 2 * std::max(0, (last_it[which] - 4) / 2)
                  : (pairs ? 1 + 2 * std::max(0, (last_it[which] - 3) / 2) : std::max(1, last_it[which] - 1)));
    // the last solve took at most two steps (past the transient: always): the finish from x_2 (k_visc_fin, as
    // viscous() would launch it) goes ahead of the round trip, so the GPU works while the host waits; it stands
    // when the count is again at most two and is rewritten by the solve's real last step (or by viscous() from
    // x_0 when x_0 passes) otherwise
    const bool spec_fin = pair0 && vfin && visc_spec && done == 2 && last_it[which] <= 2 && fin_done;
    if (spec_fin) {
      const i64 n = A.own();
      algo_bytes += 64.0 * (double)n;  // s, x_2, u read; u*, the fp32 increment written
      hipLaunchKernelGGL(k_visc_fin, dim3(grid_ew(n)), dim3(BS), 0, st, (int64_t)n, vfin->s, (const dbl2*)xa,
                         vfin->u[0], vfin->u[1], vfin->us[0], vfin->us[1], vfin->inc[0], vfin->inc[1]);
      KCHK();
    }
    wait_event(have_r0);
    timer.pool.push_back(have_r0);
    if (vcc.pending) {  // the previous solve's post-check (its copy preceded step 0 on the stream)
      vcc.pending = false;
      for (int c = 0; c < vcc.nr; ++c)
        if (!(h_pinned[32 + c] <= vcc.bound2[c] * 1.0201 + vcc.floor2[c])) {
          ++visc_check_fail;
          visc_solver = 1;  // the interval does not hold the spectrum: CG from the next solve on
        }
    }
    int K = 1;  // x_1 exists now; x_0 (y) is the answer when r_0 already passes
    bool pass0 = true;
    for (int c = 0; c < NR; ++c) {
      const double r0 = h_pinned[c], bn = h_pinned[8 + c];
      if (!std::isfinite(r0) || !std::isfinite(bn)) throw Error(PUCFEM_ENOCONV, "Chebyshev residual is not finite");
      if (r0 <= tol2 * bn) continue;
      pass0 = false;
      // smallest k with T_k(sigma) >= |r_0| / (rtol |b|)
      const double need = std::sqrt(r0 / (tol2 * bn));
      double tm = 1.0, tk = sigma;
      int k = 1;
      while (tk < need && k < maxit) {
        const double tn = 2.0 * sigma * tk - tm;
        tm = tk;
        tk = tn;
        ++k;
      }
      if (tk < need) throw Error(PUCFEM_ENOCONV, "Chebyshev iteration would not converge within maxit=" + std::to_string(maxit));
      K = std::max(K, k);
    }
    if (pass0 && (done == 1 || (pair0 && done == 2))) {  // y itself passes (the first pair left it intact)
      *out = y;
      last_it[which] = 0;
      return 0;
    }
    // the a-posteriori check of the next solve: |r_kc|^2 (kc = K - 1, reduced from part_c) against
    // |r_0| / T_kc(sigma)
    auto post_check = [&](int kc, int nck) {
      hipLaunchKernelGGL(k_reduce, dim3(NR), dim3(RB), 0, st, (const double*)part_c, nck, MAXB, NR, 0, redbuf + 48);
      KCHK();
      if (dist()) comm->allreduce(redbuf + 48, NR, false, st);
      HIPCHK(hipMemcpyAsync(h_pinned + 32, redbuf + 48, NR * sizeof(double), hipMemcpyDeviceToHost, st));
      double tm = 1.0, tk = sigma;  // T_kc(sigma)
      for (int k = 1; k < kc; ++k) {
        const double tn = 2.0 * sigma * tk - tm;
        tm = tk;
        tk = tn;
      }
      vcc.pending = true;
      vcc.nr = NR;
      for (int c = 0; c < NR; ++c) {
        vcc.bound2[c] = h_pinned[c] / (tk * tk);
        vcc.floor2[c] = 1e-28 * h_pinned[8 + c];  // rounding: |r| ~ 1e-14 |b| is as far as it resolves
      }
    };
    if (pair0 && done >= K) {  // the first pair did it (x_2, or more steps already launched)
      if (K >= 2) post_check(1, nbs + (int)hf.items);  // |r_1|^2: the first pair's check partials
      if (spec_fin) *fin_done = true;  // (the finish from x_2 = xa ran: k_visc_fin's launch, its values)
      *out = xa;
      last_it[which] = std::max(K, 1);
      return done;
    }
    if (done < K) {
      // the last step also reduces |r_{K-1}|^2 (its input's residual) for the a-posteriori check; with
      // step pairs it is the second step of a pair when an even number of steps is left
      const bool fuse = vfin != nullptr;
      const bool last_pair = pairs && (K - done) % 2 == 0;
      advance(last_pair ? K - 2 : K - 1);
      int kc, nck;
      if (last_pair) {
        double c1a, c2a, c1b, c2b;
        pair_coefs(c1a, c2a, c1b, c2b);
        pair_step(c1a, c2a, c1b, c2b, true, fuse);
        kc = done + 1;
        done += 2;
        nck = nbs + (int)hf.items;
      } else {
        const double rho = 1.0 / (2.0 * sigma - rho_old);
        step(done, rho * rho_old, 2.0 * rho / delta, true, fuse);
        rho_old = rho;
        kc = done;
        ++done;
        nck = nb;
      }
      if (fuse) *fin_done = true;
      post_check(kc, nck);
    }
    advance(K);  // (steps beyond K, already launched, only reduce the residual further)
    *out = xa;  // x_done, done >= K
    last_it[which] = K;
    return done;
  }

  // ------------------------------------------------------------------ multigrid V-cycle / PCG
  // Polynomial smoothing (deg steps) for D^-1 A: Chebyshev on [lmax / mg_ratio, lmax] (mg_kind 1), or
  // the fourth-kind Chebyshev recurrence on [0, lmax] (mg_kind 4, Lottes 2022: d_0 = 4/(3 lmax) D^-1 r,
  // d_i = (2i-1)/(2i+3) d_(i-1) + (8i+4)/((2i+3) lmax) D^-1 r_i).  Both are d = c1 d + c2 D^-1 (b - A x),
  // x += d with step-dependent scalars.
  // x_in (nullable: zero initial guess) -> returns the buffer holding the result; with zout the
  // last step writes its result (in fp64) to zout instead and nullptr is returned.
  // launch grids of a lattice operator: its face blocks, then the SELL blocks (launches that write
  // partials stay within MAXB blocks)
  // The SELL blocks come first and their count is a multiple of 8, so the face blocks' hardware ids
  // keep their XCD (id % 8) for the XCD-aware item order of face_rows.
  static int sell_blocks(int nb, const FaceDev& f) {
    if (!f.nb) return nb;
    return std::min((nb + 7) & ~7, (MAXB - f.nb) & ~7);
  }
  static int grid_part(const FaceDev& f, const DevSell& A) { return f.nb + sell_blocks(nb_for(A.nslices), f); }
  int grid_full(const FaceDev& f, const DevSell& A) const {
    return f.nb + (f.nb ? (nb_mg(A.nslices) + 7) & ~7 : nb_mg(A.nslices));
  }

  template <typename T, typename TB>
  // toz: the last step writes the preconditioned residual (z32 in the fp32 cycle, z in the fp64 one)
  // last_g (deep halos): the last step also runs on the ghost rows one layer out (x and d exchanged before it)
  // xin_cur (deep halos): xin's ghosts (two layers) are current, the first step needs no exchange
  T* mg_smooth(MgLevel& L, const DevSell& A, const HFace& hf, MgBufs<T>& B, const TB* b, T* xin, T* xa, T* xb,
               bool tozr, const double* rdot, double* part, int deg, bool last_g = false, bool xin_cur = false) {
    const double lmax = L.lmax, lmin = lmax / prm.mg_ratio;
    const double theta = 0.5 * (lmax + lmin), delta = 0.5 * (lmax - lmin), sigma = theta / delta;
    double rho_old = 1.0 / sigma;
    T* cur = xin;
    deg = std::max(1, deg);
    const bool finest = &L == &mg.back();
    // the step coefficients: d = c1 d + c2 Dinv (b - A x)
    std::vector<double> c1s(deg), c2s(deg);
    for (int k = 0; k < deg; ++k) {
      double c1 = 0.0, c2 = 1.0 / theta;
      if (prm.mg_kind == 4) {
        c1 = k == 0 ? 0.0 : (2.0 * k - 1.0) / (2.0 * k + 3.0);
        c2 = k == 0 ? 4.0 / (3.0 * lmax) : (8.0 * k + 4.0) / ((2.0 * k + 3.0) * lmax);
      } else if (k > 0) {
        const double rho = 1.0 / (2.0 * sigma - rho_old);
        c1 = rho * rho_old;
        c2 = 2.0 * rho / delta;
        rho_old = rho;
      }
      c1s[k] = c1;
      c2s[k] = c2;
    }
    // step pairs (k_cheb_pair) on the finest level of the fp32 cycle, one rank: two steps per pass on the
    // face interiors; not the step that writes z / the <r, z> partials
    bool pairs = false;
    // deep halos (W > 1): a pair's first step also runs on the ghost rows one layer out, so a pair needs one
    // exchange (x, two layers) where two single steps needed two -- pairs on every partitioned level
    const bool dg = dist() && L.deep && (deep_mask & 1);
    if constexpr (std::is_same<T, float>::value && std::is_same<TB, float>::value)
      // (one rank: the finest level only; pairs on L6 / L5 too measured neutral to -0.7 %, r10m)
      pairs = mg_pair && hf.items > 0 && hf.d.n <= VP_HALO &&
              (dist() ? dg : (int)(&mg.back() - &L) < mg_pair_levels);
    if (pairs && !mgp_x) {  // (sized for the finest level: every pair level uses them in turn)
      mgp_x = dalloc<float>(mg.back().nloc);
      mgp_d = dalloc<float>(mg.back().nloc);
    }
    T* dcur = B.d;  // the current d (a pair writes its d to the other buffer)
    double c20 = 0.0;
    for (int k = 0; k < deg; ++k) {
      const double c1 = c1s[k], c2 = c2s[k];
      // zero initial guess and >= 2 steps: step 0 is folded into step 1 (mode 2; b's ghosts are
      // current, see vcycle)
      const bool fuse = cur == nullptr && k == 0 && deg >= 2;
      if (fuse) {
        c20 = c2;
        continue;
      }
      const int mode = (cur == nullptr && k == 0) ? 0 : (cur == nullptr ? 2 : 1);
      if constexpr (std::is_same<T, float>::value && std::is_same<TB, float>::value) {
        const bool next_last = k + 1 == deg - 1;
        // (W > 1: a general-step pair only where d_a is not read, c1 = 0: d is not exchanged before it)
        if (pairs && mode != 0 && k + 1 < deg && !(next_last && (tozr || rdot || last_g)) &&
            (!dg || mode == 2 || c1 == 0.0)) {
          if (dg && mode == 1 && !(xin_cur && cur == xin)) mg_halo(L, cur);  // x_a two layers out: the first step
                                                                              // runs on the ghost rows
          // steps k, k + 1: x_a = cur (mode 1) -> x_{a+1} in p1 (skeleton rows, the face rows next to
          // them) -> x_{a+2} in p2; d_a = dcur -> d_{a+2} in the other d buffer
          float* p1 = mode == 2 ? xa : (cur == xa ? xb : xa);
          float* p2 = mode == 2 ? xb : mgp_x;
          if (mode == 1 && cur == mgp_x) {  // (cur is the extra buffer after an earlier pair)
            p1 = xa;
            p2 = xb;
          }
          float* dn = dcur == B.d ? mgp_d : B.d;
          FaceDev fs = hf.full();
          fs.nb = 0;
          const int nbs = nb_mg(A.nslices);
          const DevSell Ag = dg ? A.with_ghosts() : A;  // the first SELL launch: + the ghost rows one layer out
          const int nbg = nb_mg(Ag.nslices);
          // skeleton rows: the SELL part of a k_cheb step (bytes as in the single step, SELL rows only)
          const double sk_row = (mode == 1 ? 3.0 * sizeof(T) : 1.0 * sizeof(T)) + sizeof(TB) + 2.0 * sizeof(T);
          const double bytes_sk = (B.val_bytes() + A.idx_bytes()) * (double)A.nnz +
                                  (double)A.nrows * (sk_row + A.row_bytes());
          const double bytes_sk1 = (B.val_bytes() + A.idx_bytes()) * (double)A.nnz +
                                   (double)A.nrows * (5.0 * sizeof(T) + sizeof(TB) + A.row_bytes());
          // face rows: x_a and d_a (mode 1) and b read once, x_{a+2} and d_{a+2} written, x_{a+1} at the
          // 3 (n - 3) rows per face next to the skeleton
          const double bnd_rows = hf.d.n > 3 ? 3.0 * (hf.d.n - 3) * (double)hf.d.nf : 0.0;
          const double bytes_f = (double)hf.rows * ((mode == 1 ? 8.0 : 0.0) + 4.0 + 8.0) + 4.0 * bnd_rows;
          MgPairVecs pv{(const float*)b, (const float*)B.dinv, (const float*)cur, p1, p2, (const float*)dcur, dn};
          B.with_vals([&](auto* val) {
            using VT = std::remove_const_t<std::remove_pointer_t<decltype(val)>>;
            with_c16(A, [&](auto c16) {
              constexpr bool C = decltype(c16)::value;
              klaunch(-1, bytes_sk, k_cheb<T, TB, T, VT, C, 1>, dim3(nbg), dim3(BS), Ag.view(), fs, val,
                      (const T*)B.dinv, b, (const T*)(mode == 1 ? cur : nullptr), p1, dcur, c1, c2, c20, mode,
                      (const int*)ctl, (const double*)nullptr, (double*)nullptr, RedOut{}, (T*)nullptr);
              KCHK();
              if (mode == 1)
                klaunch(finest ? 10 : -1, bytes_f, k_cheb_pair<1>, dim3(hf.items), dim3(BS), hf.full(), pv, (float)c1, (float)c2,
                        (float)c20, (float)c1s[k + 1], (float)c2s[k + 1], (const int*)ctl);
              else
                klaunch(finest ? 10 : -1, bytes_f, k_cheb_pair<2>, dim3(hf.items), dim3(BS), hf.full(), pv, (float)c1, (float)c2,
                        (float)c20, (float)c1s[k + 1], (float)c2s[k + 1], (const int*)ctl);
              KCHK();
              klaunch(-1, bytes_sk1, k_cheb<T, TB, T, VT, C, 1>, dim3(nbs), dim3(BS), A.view(), fs, val,
                      (const T*)B.dinv, b, (const T*)p1, p2, dcur, c1s[k + 1], c2s[k + 1], c20, 1, (const int*)ctl,
                      (const double*)nullptr, (double*)nullptr, RedOut{}, dn);
              KCHK();
            });
          });
          ++mg_pairs;
          cur = p2;
          dcur = dn;
          ++k;
          continue;
        }
      }
      T* out = (cur == xa) ? xb : xa;
      const bool last = k == deg - 1;
      // the last step on the ghost rows one layer out too (deep halos): x two layers out and d one layer out
      const bool gl = last && last_g && dist() && L.deep;
      if (mode == 1) {
        if (gl) mg_halo(L, cur, dcur);
        else if (!(xin_cur && cur == xin && k == 0)) mg_halo(L, cur);
      }
      const DevSell& As = gl ? A.with_ghosts() : A;
      const bool timed = finest && mode != 0;
      const double* rd = last ? rdot : nullptr;
      const bool toz = last && tozr;
      if (toz) z_cur = gl;
      const FaceDev fc = rd ? hf.part() : hf.full();
      // (the grid of the own rows also with the ghost rows, whose slices its SELL blocks share: the <r, z> partials
      // keep the block count the PCG's reduction reads)
      const int nb = rd ? grid_part(fc, A) : grid_full(fc, A);
      const T* xi = mode == 1 ? cur : nullptr;
      // algorithmic bytes: matrix (value + column) per entry; per row x_in (mode 1) or b and dinv
      // (mode 2) gathered once, b, dinv, d read (mode 1), d and x_out written, <r, z>'s r; face rows
      // read no matrix and no dinv (per-face constants)
      const double rd_row = (mode == 1 ? 3.0 * sizeof(T) : 1.0 * sizeof(T)) + sizeof(TB) + (rd ? 8.0 : 0.0);
      const double rd_face = (mode == 1 ? 2.0 * sizeof(T) : 0.0) + sizeof(TB) + (rd ? 8.0 : 0.0);
      const double wr_row = 2.0 * sizeof(T);
      const double bytes = (B.val_bytes() + A.idx_bytes()) * (double)A.nnz +
                           (double)A.nrows * (rd_row + wr_row + A.row_bytes()) + (double)hf.rows * (rd_face + wr_row);
      B.with_vals([&](auto* val) {
        using VT = std::remove_const_t<std::remove_pointer_t<decltype(val)>>;
        with_c16(A, [&](auto c16) {
          constexpr bool C = decltype(c16)::value;
          T* zo = nullptr;
          if constexpr (std::is_same<T, float>::value) zo = z32;
          else zo = z;
          if (toz)
            klaunch(timed ? 0 : -1, bytes, k_cheb<T, TB, T, VT, C, 1>, dim3(nb), dim3(BS), As.view(), fc, val,
                    (const T*)B.dinv, b, xi, zo, dcur, c1, c2, c20, mode, (const int*)ctl, rd, part,
                    rd ? ro_rz : RedOut{}, (T*)nullptr);
          else if (finest)
            klaunch(timed ? 0 : -1, bytes, k_cheb<T, TB, T, VT, C, 1>, dim3(nb), dim3(BS), As.view(), fc, val,
                    (const T*)B.dinv, b, xi, out, dcur, c1, c2, c20, mode, (const int*)ctl, rd, part, RedOut{},
                    (T*)nullptr);
          else
            klaunch(-1, bytes, k_cheb<T, TB, T, VT, C, 0>, dim3(nb), dim3(BS), As.view(), fc, val, (const T*)B.dinv, b,
                    xi, out, dcur, c1, c2, c20, mode, (const int*)ctl, rd, part, RedOut{}, (T*)nullptr);
        });
      });
      KCHK();
      cur = toz ? nullptr : out;
    }
    return cur;
  }
  // z = M^-1 r on level l (b = r_l); the finest level passes rdot = r for the <r, z> partials and
  // writes z (fp64) directly from its last smoothing step
  // (every level smooths with the finest level's degrees: fewer steps on the latency-bound coarse levels
  // cost more pressure iterations than their launches save, round 3 r8e / r8f)
  template <typename T, typename TB>
  T* vcycle(int l, const TB* b, const double* rdot, double* part) {
    MgLevel& L = mg[l];
    MgBufs<T>& B = bufs<T>(L);
    const bool finest = l == (int)mg.size() - 1;
    const DevSell& A = finest ? dPp : L.dA;
    const HFace& hf = finest ? fP : L.hA;
    T* xa = B.x;
    T* xb = B.x2;
    if (l == mg_dense_l) {
      if constexpr (std::is_same<T, TB>::value) {
        // coarse solve: dense pseudo-inverse (replicated on every rank of a multi-rank run)
        const i64 N0 = (i64)L.ord.new2old.size();
        const dim3 g((unsigned)std::min<i64>(4096, (N0 + 3) / 4));
        if (std::is_same<T, float>::value && dAinv32) {
          algo_bytes += 4.0 * (double)N0 * (double)N0 + 2.0 * sizeof(T) * (double)N0;
          hipLaunchKernelGGL((k_dense_mv<T, float>), g, dim3(BS), 0, st, N0, (const float*)dAinv32, b, xa, ctl);
        } else {
          algo_bytes += 8.0 * (double)N0 * (double)N0 + 2.0 * sizeof(T) * (double)N0;
          hipLaunchKernelGGL(k_dense_mv<T>, g, dim3(BS), 0, st, N0, (const double*)dAinv, b, xa, ctl);
        }
        KCHK();
        return xa;
      } else {
        throw Error(PUCFEM_ESTATE, "multigrid hierarchy has a single level");
      }
    }
    const int pre = prm.mg_degree;
    if constexpr (std::is_same<T, TB>::value) {
      // coarse levels: the fused first smoothing step reads b at ghost columns
      if (pre >= 2) mg_halo(L, const_cast<T*>(b));
    }
    T* x = mg_smooth<T, TB>(L, A, hf, B, b, nullptr, xa, xb, false, nullptr, nullptr, pre);
    mg_halo(L, x);
    // residual: matrix entries, x gathered once, b read, res written; deep halos: also on the ghost rows one layer
    // out, which the restriction gathers (no exchange of the residual)
    const bool rg = dist() && L.res_deep && (deep_mask & 2);
    const DevSell& Ar = rg ? A.with_ghosts() : A;
    const double bytes_res = (B.val_bytes() + A.idx_bytes()) * (double)A.nnz + A.row_bytes() * (double)A.nrows +
                             (double)A.own() * (2.0 * sizeof(T) + sizeof(TB));
    const FaceDev fr = hf.full();
    B.with_vals([&](auto* val) {
      using VT = std::remove_const_t<std::remove_pointer_t<decltype(val)>>;
      with_c16(A, [&](auto c16) {
        if (finest)
          klaunch(5, bytes_res, k_resid<T, TB, VT, decltype(c16)::value, 1>, dim3(grid_full(fr, Ar)), dim3(BS),
                  Ar.view(), fr, val, b, (const T*)x, B.res, (const int*)ctl);
        else
          klaunch(-1, bytes_res, k_resid<T, TB, VT, decltype(c16)::value, 0>, dim3(grid_full(fr, Ar)), dim3(BS),
                  Ar.view(), fr, val, b, (const T*)x, B.res, (const int*)ctl);
      });
    });
    KCHK();
    if (!rg) mg_halo(L, B.res);
    MgLevel& C = mg[l - 1];
    MgBufs<T>& CB = bufs<T>(C);
    const bool gather = C.rep && !L.rep && dist();  // into the finest replicated level
    T* cb = gather ? CB.b + L.r_r0 : CB.b;
    // restriction: entries (value + column), fine residual read once, coarse rhs written
    const FaceDev frs = L.hR.full(), fpr = L.hPr.full();
    klaunch(finest ? 6 : -1,
            (double)(sizeof(T) + 4) * (double)L.dR.nnz + L.dR.row_bytes() * (double)L.dR.nrows +
                (double)sizeof(T) * (double)(A.own() + L.dR.nrows + L.hR.rows),
            k_transfer<T>, dim3(grid_full(frs, L.dR)), dim3(BS), L.dR.view(), frs, (const T*)B.Rval, (const T*)B.res,
            cb, 0, (const int*)ctl);
    KCHK();
    if (gather) {
      comm->group_start();
      for (int r = 0; r < world; ++r) comm->bcast(CB.b + C.rs[r], C.rs[r + 1] - C.rs[r], r, st);
      comm->group_end(st);
    }
    T* xc = vcycle<T, T>(l - 1, CB.b, nullptr, nullptr);
    if (!(dist() && L.xc_deep && (deep_mask & 4))) mg_halo(C, xc);  // (xc_deep: level l - 1's last step wrote its ghosts one layer out)
    // prolongation: entries, coarse x read once, fine x read + written; pr_deep: also on this level's ghost rows (x
    // there is current since the exchange before the residual), so the post-smoothing starts without an exchange
    const bool pg = dist() && L.pr_deep && (deep_mask & 8) && ((deep_mask & 4) || C.rep);
    const DevSell& Apr = pg ? L.dPr.with_ghosts() : L.dPr;
    klaunch(finest ? 7 : -1,
            (double)(sizeof(T) + 4) * (double)L.dPr.nnz + L.dPr.row_bytes() * (double)L.dPr.nrows +
                (double)sizeof(T) * (double)(2 * A.own() + L.dR.nrows + L.hR.rows),
            k_transfer<T>, dim3(grid_full(fpr, Apr)), dim3(BS), Apr.view(), fpr, (const T*)B.Prval, (const T*)xc,
            x, 1, (const int*)ctl);
    KCHK();
    T* other = (x == xa) ? xb : xa;
    const int post = prm.mg_post > 0 ? prm.mg_post : prm.mg_degree;
    // the last step on the ghost rows one layer out where its consumer gathers them: the prolongation into level
    // l + 1 (xc_deep), and z for the PCG's A z on the finest level -- there the ghost rows must repeat the owners'
    // arithmetic bit for bit (the outer fp64 PCG needs w = A z of ONE vector z: its recurrences s = A p and
    // r = b - A y hold only then), which face_ghost_rows ensures: face-interior ghost rows are their face stencils
    const bool last_g = dist() && L.deep && (deep_mask & 4) && (finest || mg[l + 1].xc_deep);
    return mg_smooth<T, TB>(L, A, hf, B, b, x, x, other, finest, rdot, part, post, last_g, pg);
  }
  // z = M^-1 r (finest level), <r, z> partials in part_d + 2 MAXB.  The fp32 cycle reads r32 (owned
  // rows written by k_cg_init / k_cg_upd; its ghosts are exchanged by the cycle); the fp64 one r itself
  void precondition(double* rz_part = nullptr) {
    if (!rz_part) rz_part = part_d + 2 * MAXB;
    z_cur = false;
    if (mg_single) {
      vcycle<float, float>((int)mg.size() - 1, r32, cg_r[0], rz_part);
    } else {
      halo(cg_r[0]);
      vcycle<double, double>((int)mg.size() - 1, cg_r[0], cg_r[0], rz_part);
    }
  }
  // Chronopoulos-Gear PCG (k_cgcg_*): the multi-rank pressure solves, one all-reduce per iteration instead of three;
  // PUCFEM_CGCG=1 / 0 forces it on / off (measurement and test knob: the single-rank path keeps the standard form,
  // 24 B/row less per iteration)
  int cgcg_env = std::getenv("PUCFEM_CGCG") ? std::atoi(std::getenv("PUCFEM_CGCG")) : -1;
  bool use_cgcg() const { return cgcg_env >= 0 ? cgcg_env != 0 : dist(); }
  double* part_cc = nullptr;  // CGCG_NV x MAXB partials
  double* cgcg_sc = nullptr;  // k_cgcg_coef's scalars (8)
  int64_t cgcg_iters = 0;     // iterations run in the single-reduction form (pucfem_path_info bit 7)
  // preconditioned CG on the unscaled merged pressure operator (finest level = dPp / dKp_raw)
  // prm.proj_shared: both pressure solves of a step project onto ONE basis (the same merged operator, so
  // one A-orthonormal basis serves both) that collects the solutions of both -- slot 1 for both; else a
  // basis per solve.  Separate bases stop improving at 16 directions; a shared one keeps improving up to
  // PROJ_MAX = 32 (r8l: 72 -> 63 pressure iterations over the driver window, +2 % steps/s)
  // PUCFEM_PCG_TRACE=1 (diagnostic): the relative residual of every pressure PCG iteration on stderr (a host
  // round trip per iteration)
  bool pcg_trace = false;  // (read at every solve)
  long n_pcg_traced = 0;
  void trace_pcg(int which, int it) {
    double h[5];
    HIPCHK(hipMemcpyAsync(h, redbuf, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h + 1, redbuf + 8, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h + 2, redbuf + 32, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h + 3, ctl, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    int cc[2];
    std::memcpy(cc, h + 3, sizeof(cc));
    if (it == 0) ++n_pcg_traced;
    std::fprintf(stderr, "[pcg] solve %ld (slot %d) it %d |r|/|b| %.3e <r,z> %.3e ctl %d/%d\n", n_pcg_traced, which, it,
                 std::sqrt(h[0] / h[1]), h[2], cc[0], cc[1]);
  }
  // PUCFEM_PROJ_SPMV=1 (diagnostic knob): the projection update's A v by an SpMV of v = y - x0 instead of the
  // CG's residuals r0 - r_final (no pending directions)
  bool proj_spmv = std::getenv("PUCFEM_PROJ_SPMV") && std::atoi(std::getenv("PUCFEM_PROJ_SPMV")) != 0;
  // the PCG's initial <r, r> and <b, b> beside the control word (k_conv / k_reduce_conv write them at iteration
  // 0; pcg_mg's control reads bring them along): the projected guess's quality, h_note() after a solve
  double* ctl_note() const { return reinterpret_cast<double*>(ctl + 2); }
  double guess_rel() const {
    const double* h = reinterpret_cast<const double*>(h_ctl + 2);
    return h[1] > 0.0 ? std::sqrt(h[0] / h[1]) : 0.0;
  }
  // Guess monitor (round 5).  A projection basis whose A-orthonormality has decayed (rounding of the fp32 basis
  // through repeated re-seeds; with 12 directions, re-seeded every solve, steady L7 steps went from 0-1 to 5
  // iterations per solve, r11g) gives guesses orders of magnitude worse than the last ones while the flow
  // changes smoothly; the decay builds up over a few solves (r11h: 5e-8 -> 1e-4 of b in ~4 solves).  When a
  // projected guess's relative residual exceeds 50x the best of the last 8 projected guesses of its basis (and
  // 10x the tolerance), the basis restarts from the next solution (Fischer's restart).  Healthy steady guesses
  // spread over ~10x (2.6e-8 .. 2.9e-7 at L7, r11e); in the start-up transient they fall step by step.
  static constexpr int GUESS_HIST = 8;
  double guess_last[5] = {0, 0, 0, 0, 0};
  double guess_hist[5][GUESS_HIST] = {};
  int guess_n[5] = {0, 0, 0, 0, 0};
  int64_t n_restart = 0;
  bool guess_decayed(int slot, double g) {
    double best = 0.0;
    const int k = std::min(guess_n[slot], GUESS_HIST);
    for (int i = 0; i < k; ++i) best = i == 0 ? guess_hist[slot][i] : std::min(best, guess_hist[slot][i]);
    guess_hist[slot][guess_n[slot] % GUESS_HIST] = g;
    ++guess_n[slot];
    guess_last[slot] = g;
    return k > 0 && g > 50.0 * best && g > 10.0 * prm.rtol_pres;
  }
  void proj_restart(int slot) {
    proj_m[slot] = 0;
    proj_pend[slot] = false;
    pend_otf[slot] = false;
    pend_acc[slot] = false;
    pend_vzero[slot] = false;
    proj_hist[slot] = ProjHist{};
    guess_n[slot] = 0;
    ++n_restart;
  }
  bool proj_shared = false;  // prm.proj_shared (PUCFEM_PROJ_SHARED=0/1 overrides it: a measurement knob)
  int proj_slot(int which) const { return proj_shared && which == 2 ? 1 : which; }
  int pcg_mg(double* y, const double* b, double tol, int maxit, int which) {
    const FaceDev fc = fP.part();
    const int nb = grid_part(fc, dPp);  // also the grid of the V-cycle's last smoothing step (<r, z> partials)
    const i64 n = dPp.own();
    const int nbu = nb_rows(n);
    CgVecs<1> v;
    v.y[0] = y;
    v.b[0] = b;
    v.r[0] = z;  // the gathered "r" of k_cg_dir is the preconditioned residual
    v.zf[0] = z32;  // (in fp32 from the fp32 V-cycle)
    v.po[0] = cg_pa[0];
    v.pn[0] = cg_pb[0];
    v.q[0] = cg_q[0];
    CgVecs<1> vi = v;
    vi.r[0] = cg_r[0];
    halo(y);
    HIPCHK(hipMemsetAsync(ctl, 0, 2 * sizeof(int), st));
    float* r32o = mg_single ? r32 : nullptr;
    // the projection's update takes A (y - x0) = r0 - r_final from the CG's residuals: k_cg_init
    // keeps r0 in pav (its "first direction" output; pcg_mg's directions live elsewhere)
    const bool keep_r0 = proj_k > 0 && (which == 1 || which == 2);
    if (keep_r0) vi.po[0] = pav[proj_slot(which)];
    algo_bytes += (8.0 + dPp.idx_bytes()) * (double)dPp.nnz + dPp.row_bytes() * (double)dPp.nrows +
                  (24.0 + (mg_single ? 4.0 : 0.0) + (keep_r0 ? 8.0 : 0.0)) * (double)n;
    // fused reductions: <r, r> -> redbuf slot 0, <b, b> -> slot 1 (as k_reduce would place them)
    const RedOut ri = ro(redbuf, CNT_INIT, 2, MAXB, 0u, redbuf + 8);
    with_c16(dPp, [&](auto c16) {
      hipLaunchKernelGGL((k_cg_init<1, decltype(c16)::value>), dim3(nb), dim3(BS), 0, st, dPp.view(), fc, dKp_raw, vi,
                         lp.n_ghost, part_a, ri.out ? part_a + MAXB : part_b, r32o, keep_r0 ? 1 : 0, ri);
    });
    KCHK();
    Red rr{redbuf, 1, 1}, bb{redbuf + 8, 1, 1};
    const double tol2 = tol * tol;
    // single rank with k_reduce: the reduction of <b, b> (and, per iteration, of <r, r>) also runs the
    // convergence test (k_reduce_conv: one launch instead of k_reduce + k_conv; multi-rank runs test after
    // the all-reduce)
    const bool merged_conv = !dist() && !ri.out;
    if (ri.out) {
      red_done(redbuf, 1, false);
      red_done(redbuf + 8, 1, false);
    } else {
      rr = reduce_global(part_a, nb, 1, false, 0);
      if (merged_conv) {
        hipLaunchKernelGGL(k_reduce_conv, dim3(1), dim3(RB), 0, st, (const double*)part_b, nb, MAXB, redbuf + 8,
                           (const double*)rr.p, (const double*)(redbuf + 8), tol2, ctl, 0, ctl_note());
        KCHK();
      } else {
        bb = reduce_global(part_b, nb, 1, false, 1);
      }
    }
    const RedOut rdir = ro(redbuf + 16, CNT_DIR, 1), rupd = ro(redbuf, CNT_UPD, 1);
    // (iteration, first timing sample): samples from the converged iteration on are dropped
    std::vector<std::pair<int, size_t>> marks;
    std::vector<std::pair<int, ByteMark>> bmarks;  // (iteration, the byte counters at its start) of the current chunk
    if (!merged_conv) {
      hipLaunchKernelGGL(k_conv, dim3(1), dim3(64), 0, st, rr.p, bb.p, tol2, ctl, 0, 1, ctl_note());
      KCHK();
    }
    // direction: z (4 B in the fp32 cycle) and p_old gathered once, p and q written
    const double bytes_dir = (8.0 + dPp.idx_bytes()) * (double)dPp.nnz + dPp.row_bytes() * (double)dPp.nrows +
                             (mg_single ? 28.0 : 32.0) * (double)n;
    const double bytes_upd = (48.0 + (mg_single ? 4.0 : 0.0)) * (double)n;  // + the fp32 r copy
    // the single-reduction form: w = A z (z gathered once, r and s_old read, w written), the update (z, w, p, s,
    // y, r read; p, s, y, r written; the fp32 r copy, the accumulated correction)
    const bool cgcg = use_cgcg();
    const double zb = mg_single ? 4.0 : 8.0;
    const double bytes_w = (8.0 + dPp.idx_bytes()) * (double)dPp.nnz + dPp.row_bytes() * (double)dPp.nrows +
                           (zb + 24.0) * (double)n;
    const double bytes_cu = (zb + 72.0 + (mg_single ? 4.0 : 0.0) + (cg_vacc ? 16.0 : 0.0)) * (double)n;
    const double* rho0 = rr.p;  // the initial <r, r> (k_cgcg_coef's rho at iteration 0)
    int it = 0;
    // an iteration = V-cycle, direction, update, convergence test (k_conv): the host checks right
    // after a test, so a solve that converges at a check launches no V-cycle after it.  The first
    // check comes one iteration before the last solve's count (a no-op iteration costs more than a
    // check's round trip), then every iteration while the solve is short.  Past the start-up transient
    // the projected guess often passes the test itself (0 iterations): when the last solve took at most
    // one iteration and, of the last 8 such solves, at least 2 passed at their guess, the host reads the
    // initial test before launching any (one round trip, where an iteration of early-exiting launches --
    // the V-cycle's ~70 -- costs ~0.3 ms of GPU time; in the start-up transient, where no solve passes at
    // its guess, the round trip would only idle the GPU: +0.25 ms per step in the driver window, r10b)
    pcg_trace = std::getenv("PUCFEM_PCG_TRACE") && std::atoi(std::getenv("PUCFEM_PCG_TRACE")) != 0;
    if (pcg_trace) trace_pcg(which, 0);
    const bool seen = solved_before[which];
    solved_before[which] = true;
    int chunk = std::max(1, std::min(maxit + 1, !seen ? 4 : (last_it[which] > 1 ? last_it[which] - 1 : 1)));
    bool done0 = false;
    const bool eligible = seen && last_it[which] <= 1;
    if (eligible && __builtin_popcount(zero_hist[which] & 0xffu) >= 2) {
      read_ctl();
      done0 = h_ctl[0] != 0;
    }
    for (bool first = true; !done0; first = false) {
      if (!first) marks.clear();  // the previous chunk's samples are flushed
      bmarks.clear();
      for (int k = 0; k < chunk; ++k, ++it) {
        marks.push_back({it, timer.mark()});  // this iteration's V-cycle works iff not converged at it
        bmarks.push_back({it, bmark_now()});
        if (cgcg) {  // single-reduction iteration (k_cgcg_*)
          ++cgcg_iters;
          precondition(part_cc + 3 * MAXB);
          if (!z_cur) {  // (deep halos: the last smoothing step wrote z's ghosts one layer out, bit for bit)
            if (mg_single) mg_halo(mg.back(), z32);
            else halo(z);
          }
          with_c16(dPp, [&](auto c16) {
            if (mg_single)
              klaunch(1, bytes_w, k_cgcg_w<decltype(c16)::value, true>, dim3(nb), dim3(BS), dPp.view(), fc,
                      (const double*)dKp_raw, (const double*)nullptr, (const float*)z32, (const double*)cg_r[0],
                      it > 0 ? (const double*)cg_q[0] : (const double*)nullptr, cg_pb[0], part_cc, (const int*)ctl);
            else
              klaunch(1, bytes_w, k_cgcg_w<decltype(c16)::value, false>, dim3(nb), dim3(BS), dPp.view(), fc,
                      (const double*)dKp_raw, (const double*)z, (const float*)nullptr, (const double*)cg_r[0],
                      it > 0 ? (const double*)cg_q[0] : (const double*)nullptr, cg_pb[0], part_cc, (const int*)ctl);
          });
          KCHK();
          launch_reduce(part_cc, nb, MAXB, CGCG_NV, false, redbuf + 64);
          KCHK();
          if (dist()) comm->allreduce(redbuf + 64, CGCG_NV, false, st);
          hipLaunchKernelGGL(k_cgcg_coef, dim3(1), dim3(64), 0, st, (const double*)(redbuf + 64), (const double*)bb.p,
                             cgcg_sc, tol2, ctl, it, maxit, (const double*)rho0);
          KCHK();
          if (mg_single)
            klaunch(2, bytes_cu - (cg_vacc && it == 0 ? 8.0 * (double)n : 0.0), k_cgcg_upd<true>, dim3(nb), dim3(BS),
                    (int64_t)n, (const double*)nullptr,
                    (const float*)z32, (const double*)cg_pb[0], cg_pa[0], cg_q[0], y, cg_r[0], r32o, cg_vacc,
                    (const double*)cgcg_sc, (const int*)ctl, it, part_cc);
          else
            klaunch(2, bytes_cu - (cg_vacc && it == 0 ? 8.0 * (double)n : 0.0), k_cgcg_upd<false>, dim3(nb), dim3(BS),
                    (int64_t)n, (const double*)z,
                    (const float*)nullptr, (const double*)cg_pb[0], cg_pa[0], cg_q[0], y, cg_r[0], r32o, cg_vacc,
                    (const double*)cgcg_sc, (const int*)ctl, it, part_cc);
          KCHK();
          if (pcg_trace) trace_pcg(which, it + 1);
          continue;
        }
        if (dye_gate == 1 && which == 1) dye_tail_release();
        ro_rz = ro(redbuf + 32, CNT_RZ, 1);
        precondition();
        ro_rz = RedOut{};
        Red rz{redbuf + 32, 1, 1};
        if (ro(redbuf + 32, CNT_RZ, 1).out) red_done(redbuf + 32, 1, false);
        else rz = reduce_global(part_d + 2 * MAXB, nb, 1, false, 4);
        if (!z_cur) {
          if (mg_single) mg_halo(mg.back(), z32);
          else halo(z);
        }
        with_c16(dPp, [&](auto c16) {
          if (mg_single)
            klaunch(1, bytes_dir, k_cg_dir<1, 8, true, decltype(c16)::value, true>, dim3(nb), dim3(BS), dPp.view(), fc,
                    (const double*)dKp_raw, v, lp.n_ghost, rz.p, rz.nb, rz.stride, bb.p, bb.nb, bb.stride, scal, ctl,
                    it, maxit, tol2, part_c, rr.p, rr.nb, rr.stride, rdir);
          else
            klaunch(1, bytes_dir, k_cg_dir<1, 8, true, decltype(c16)::value>, dim3(nb), dim3(BS), dPp.view(), fc,
                    (const double*)dKp_raw, v, lp.n_ghost, rz.p, rz.nb, rz.stride, bb.p, bb.nb, bb.stride, scal, ctl,
                    it, maxit, tol2, part_c, rr.p, rr.nb, rr.stride, rdir);
        });
        KCHK();
        Red pq{redbuf + 16, 1, 1};
        if (rdir.out) red_done(redbuf + 16, 1, false);
        else pq = reduce_global(part_c, nb, 1, false, 2);
        CgVecs<1> vu = v;
        vu.r[0] = cg_r[0];
        klaunch(2, bytes_upd + (cg_vacc ? (it == 0 ? 8.0 : 16.0) * (double)n : 0.0), k_cg_upd<1>, dim3(nbu), dim3(BS),
                vu, n, pq.p, pq.nb, pq.stride, (const double*)scal, (const int*)ctl, part_a, r32o, rupd, cg_vacc,
                it == 0 ? 1 : 0);
        KCHK();
        if (rupd.out) rr = Red{redbuf, 1, 1}, red_done(redbuf, 1, false);
        else if (!merged_conv) rr = reduce_global(part_a, nbu, 1, false, 0);
        if (merged_conv) {
          rr = Red{redbuf, 1, 1};
          hipLaunchKernelGGL(k_reduce_conv, dim3(1), dim3(RB), 0, st, (const double*)part_a, nbu, MAXB, redbuf,
                             (const double*)redbuf, (const double*)bb.p, tol2, ctl, it + 1);
        } else {
          hipLaunchKernelGGL(k_conv, dim3(1), dim3(64), 0, st, rr.p, bb.p, tol2, ctl, it + 1, 1);
        }
        KCHK();
        std::swap(v.po[0], v.pn[0]);
        if (pcg_trace) trace_pcg(which, it + 1);
      }
      // the samples before this chunk, while the GPU runs it (this chunk's stay pending until its test is read)
      if (timer.on && !marks.empty()) timer.flush_ready(marks.front().second);
      read_ctl(it >= last_it[which]);
      if (timer.on && h_ctl[0])  // iterations from the converged one on launched kernels that did no work
        for (auto& mk : marks)
          if (mk.first >= h_ctl[1]) {
            timer.drop_from(mk.second);
            break;
          }
      if (h_ctl[0])  // the bytes of the iterations that found the solve converged did not move
        for (auto& bm : bmarks)
          if (bm.first >= h_ctl[1]) {
            bmark_restore(bm.second);
            break;
          }
      if (h_ctl[0]) break;
      chunk = it < 8 ? 1 : std::min(16, it / 4);
    }
    last_it[which] = h_ctl[1];
    if (eligible) zero_hist[which] = (zero_hist[which] << 1) | (h_ctl[1] == 0 ? 1u : 0u);
    if (h_ctl[0] == 3) throw Error(PUCFEM_ENOCONV, "MG-PCG residual is not finite (iteration " + std::to_string(h_ctl[1]) + ")");
    if (h_ctl[0] != 1) throw Error(PUCFEM_ENOCONV, "MG-PCG did not converge within maxit=" + std::to_string(maxit));
    return h_ctl[1];
  }

  // ------------------------------------------------------------------ building blocks of the step
  // makePerBCU + makeDirBCU on owned rows: the interleaved velocity (a = its x components, b = a + 1), or with
  // b null one plain vector (the heat / Poisson scalar)
  void bc(double* a, double* b) {
    const int vs = b ? VS : 1;
    if (ncopy == 0 && ndir == 0) return;
    const int nb = (int)std::min<i64>(1024, std::max<i64>(1, (ncopy + ndir + BS - 1) / BS));
    if (bc_gather && ncopy > 0) {
      hipLaunchKernelGGL(k_bc_gather, dim3(std::min(1024, (ncopy + BS - 1) / BS)), dim3(BS), 0, st, ncopy, dcsrc,
                         dbctmp, dir_ncomp, a, b, vs);
      KCHK();
    }
    hipLaunchKernelGGL(k_bc_apply, dim3(nb), dim3(BS), 0, st, ncopy, dcdst, dcsrc,
                       bc_gather ? (const double*)dbctmp : nullptr, ndir, ddnode, ddval, dir_ncomp, a, b, vs);
    KCHK();
  }
  // halo of the interleaved velocity u / u* (component pointers)
  void halo_v(double* vx) { halo2(reinterpret_cast<dbl2*>(vx)); }
  // PUCFEM_VISC_FUSE_FIN=0 (measurement knob): k_visc_fin as its own launch after the solve
  bool visc_fuse_fin = !(std::getenv("PUCFEM_VISC_FUSE_FIN") && std::atoi(std::getenv("PUCFEM_VISC_FUSE_FIN")) == 0);
  bool dense_bc = !(std::getenv("PUCFEM_DENSE_BC") && std::atoi(std::getenv("PUCFEM_DENSE_BC")) == 0);
  int viscous(int& iters) {  // StokesColor.py:540-547
    const i64 n = lp.n_own;
    if (dense) {  // u* = A_visc^-1 (u + DT * 0)
      // (PUCFEM_DENSE_BC=0, measurement knob: the BCs in their own launch)
      if (dbcsrc && dense_bc && dir_ncomp == 2) {  // (velocity BCs: both components copied / set)
        hipLaunchKernelGGL(k_dense_mv2_bc, dim3((int)std::min<i64>(2048, (n + 3) / 4)), dim3(BS), 0, st, n, dVinv, ux,
                           uy, usx, usy, (const int32_t*)dbcsrc, (const int32_t*)dbcdir, (const double*)ddval,
                           dir_ncomp);
        KCHK();
      } else {
        hipLaunchKernelGGL(k_dense_mv2, dim3((int)std::min<i64>(2048, (n + 3) / 4)), dim3(BS), 0, st, n, dVinv, ux, uy,
                           usx, usy);
        KCHK();
        bc(usx, usy);
      }
      iters = 0;
      return 0;
    }
    const bool ext = dvinc[0] != nullptr && !proj_k_visc;
    VincDev vd{};
    vd.order = ext ? std::min(have_vinc, visc_extrap) : 0;
    for (int k = 0; k < 2 * VINC_MAX; ++k) vd.d[k] = dvinc[k];
    const bool proj = proj_k_visc > 0;
    // the Chebyshev iteration (interleaved vectors); the CG (SoA vectors) when the interval is too wide, the
    // post-check failed, the operator is small enough for the one-workgroup CG, or the projection guess of
    // the viscous solve is on (a measurement knob whose bases hold SoA vectors)
    const bool cheb = visc_solver == 0 && visc_R < 0.25 && !proj &&
                      !(!dist() && block_cg && !fVisc.items && dP.nrows <= (int64_t)CGB_THREADS * CGB_MAXR);
    // (k_visc_prep folded into the solve's first step was measured 9 % slower in round 3, r9i: the window
    // recomputes the start's 64 B/row of inputs on 25 % more rows, so the fusion saved no bytes)
    // (folded into the previous step's second k_grad_proj, which holds the final u in registers: bit-identical,
    // ~50 us less kernel time per step, yet 0.4-1.4 % slower in four A/B pairs with and without the dye
    // overlap, r11s; not kept)
    // u, s, the increments read; b, y written
    const double prep_bytes = (56.0 + 8.0 * vd.order) * (double)n;
    if (cheb)
      klaunch(13, prep_bytes, k_visc_prep<true>, dim3(grid_ew(n)), dim3(BS), (int64_t)n, (const double*)dsv,
              (const double*)ux, (const double*)uy, reinterpret_cast<double*>(vb2),
              (double*)nullptr, reinterpret_cast<double*>(vx2[0]), (double*)nullptr, vd);
    else
      klaunch(13, prep_bytes, k_visc_prep<false>, dim3(grid_ew(n)), dim3(BS), (int64_t)n, (const double*)dsv,
              (const double*)ux, (const double*)uy, bvx, bvy, yvx, yvy, vd);
    KCHK();
    // with the extrapolated start the solve's last Chebyshev step also does k_visc_fin's work
    const int last = 2 * (visc_extrap - 1);
    bool fin_done = false;
    if (cheb) {
      ViscFin vf{};
      const bool fuse = ext && visc_fuse_fin;
      if (fuse) vf = ViscFin{dsv, {ux, uy}, {usx, usy}, {dvinc[last], dvinc[last + 1]}};
      dbl2* yo = vx2[0];  // the converged iterate (one of the solve's buffers)
      iters = vcheb(dP, fVisc, dKv, vx2[0], vb2, prm.rtol_visc, prm.maxit_visc, 0, &yo, fuse ? &vf : nullptr,
                    &fin_done);
      if (!fin_done) {  // u* = S y (and the increment)
        algo_bytes += (ext ? 64.0 : 40.0) * (double)n;  // s, y (, u) read; u* (, the fp32 increment) written
        hipLaunchKernelGGL(k_visc_fin, dim3(grid_ew(n)), dim3(BS), 0, st, (int64_t)n, (const double*)dsv,
                           (const dbl2*)yo, (const double*)ux, (const double*)uy, usx, usy,
                           ext ? dvinc[last] : (float*)nullptr, ext ? dvinc[last + 1] : (float*)nullptr);
      }
    } else {
      proj_materialize();  // (the CG's vectors include cg_r[0], a pending pressure direction's input)
      double* y[2] = {yvx, yvy};
      const double* b[2] = {bvx, bvy};
      if (proj) {  // the warm start u^n is replaced by the projection onto earlier solutions
        project_guess(3, bvx, yvx);
        project_guess(4, bvy, yvy);
      }
      iters = cg<2>(dP, fVisc, dKv, y, b, prm.rtol_visc, prm.maxit_visc, 0);
      if (proj) {
        project_update(3, yvx);
        project_update(4, yvy);
      }
      if (ext) {
        algo_bytes += 64.0 * (double)n;  // s, y, u read; u*, the fp32 increment written
        hipLaunchKernelGGL(k_visc_fin_soa, dim3(grid_ew(n)), dim3(BS), 0, st, (int64_t)n, (const double*)dsv,
                           (const double*)yvx, (const double*)yvy, (const double*)ux, (const double*)uy, usx, usy,
                           dvinc[last], dvinc[last + 1]);
      } else {
        algo_bytes += 40.0 * (double)n;
        hipLaunchKernelGGL(k_cg_fin, dim3(grid_ew(n)), dim3(BS), 0, st, n, 2, dsv, yvx, yvy, usx, usy,
                           (const int32_t*)nullptr, VS);
      }
    }
    if (ext) {  // the new increment replaces the oldest: (d1, d2, d3) <- (new, d1, d2)
      for (int k = last; k >= 2; k -= 2) {
        std::swap(dvinc[k], dvinc[k - 2]);
        std::swap(dvinc[k + 1], dvinc[k - 1]);
      }
      have_vinc = std::min(have_vinc + 1, visc_extrap);
    }
    KCHK();
    bc(usx, usy);
    halo_v(usx);
    return 0;
  }
  // grid of k_div (its partials: max |div|, sum braw)
  int div_grid() const { return grid_part(fK.part(), dP); }
  void div(const double* ax, const double* ay, double* out, bool rhs, double* part = nullptr, RedOut r = RedOut{}) {
    const FaceDev fc = fK.part();
    with_c16(dP, [&](auto c16) {
      // ux, uy gathered once; div (when stored) and braw (the pressure rhs) written
      klaunch(11,
              (16.0 + dP.idx_bytes()) * (double)dP.nnz + dP.row_bytes() * (double)dP.nrows +
                  (16.0 + (out ? 8.0 : 0.0) + (rhs ? 8.0 : 0.0)) * (double)lp.n_own,
              k_div<decltype(c16)::value, true>, dim3(div_grid()), dim3(BS), dP.view(), fc, (const double*)dGx,
              (const double*)dGy, ax, ay, (const double*)das1, out, (const double*)dmp, -(1.0 / prm.dt),
              rhs ? braw : (double*)nullptr, part ? part : part_d, r);
    });
    KCHK();
  }
  // sb_fused: the preceding k_div reduced sum(braw) into redbuf slot 3 itself (div_rhs)
  // PUCFEM_RHS_FUSE=0 (measurement knob): the pressure right-hand side always in its own pass (k_pres_rhs)
  bool rhs_fuse = !(std::getenv("PUCFEM_RHS_FUSE") && std::atoi(std::getenv("PUCFEM_RHS_FUSE")) == 0);
  int pressure(double* yst, double* pout, int which, bool sb_fused = false) {  // StokesColor.py:554-555 (restated)
    if (dye_gate >= 2 && which == 1) dye_tail_release();  // (gates 3 / 4 when the viscous solve ran no pair)
    const int nb = div_grid();
    Red sb{redbuf + 24, 1, 1};
    if (!sb_fused) sb = reduce_global(part_d + MAXB, nb, 1, false, 3);
    const i64 n = lp.n_own;
    const double* sc = (use_mg || dense) ? nullptr : dsp;  // MG and dense paths solve the unscaled system
    const bool proj = use_mg && proj_k > 0 && (which == 1 || which == 2);
    // with a projected guess k_mdot2 (the first pass over the rows) forms the right-hand side itself
    const bool rhs_in_mdot = proj && rhs_fuse && !sc && proj_pend[proj_slot(which)];
    if (dense) {  // small meshes: right-hand side, dense solve and p in one launch (k_dense_pres)
      algo_bytes += 8.0 * (double)n * (double)n + 48.0 * (double)n;
      hipLaunchKernelGGL(k_dense_pres, dim3((int)std::min<i64>(2048, (n + 3) / 4)), dim3(BS), 0, st, n,
                         (const double*)dPinv, (const double*)braw, (const int32_t*)dslave_of,
                         (const int32_t*)dmaster_of, sb.p, sb.nb, 1.0 / (double)n_free, yst, pout);
      KCHK();
      halo(pout);
      return 0;
    }
    if (!rhs_in_mdot) {
      algo_bytes += 24.0 * (double)n;  // braw, slave_of, master_of read; bh written
      hipLaunchKernelGGL(k_pres_rhs, dim3(grid_ew(n)), dim3(BS), 0, st, n, braw, dslave_of, dmaster_of, sc,
                         sb.p, sb.nb, 1.0 / (double)n_free, bh);
      KCHK();
    }
    if (!prm.warm_start) HIPCHK(hipMemsetAsync(yst, 0, sizeof(double) * nloc, st));
    const RhsIn rin{braw, dslave_of, sb.p, 1.0 / (double)n_free, bh};
    const bool projected = proj && project_guess(proj_slot(which), bh, yst, rhs_in_mdot ? &rin : nullptr);
    const bool acc = projected && !proj_spmv;  // the CG accumulates v (k_pcomb cleared pv)
    int it;
    if (dense) {
      hipLaunchKernelGGL(k_dense_mv<double>, dim3((int)std::min<i64>(2048, (n + 3) / 4)), dim3(BS), 0, st, n, dPinv, bh, yst,
                         (const int*)nullptr);
      KCHK();
      it = 0;
    } else if (use_mg) {
      // separate bases: the other slot's pending direction reads the r_final this solve overwrites
      proj_materialize(proj ? proj_slot(which) : 0);
      cg_vacc = acc ? pv[proj_slot(which)] : nullptr;
      it = pcg_mg(yst, bh, prm.rtol_pres, prm.maxit_pres, which);
      cg_vacc = nullptr;
      // (the projection update and the finish in one pass: sc is null on the multigrid path)
      if (proj) {
        const int slot = proj_slot(which);
        pend_acc[slot] = acc;
        pend_vzero[slot] = acc && it == 0;
        if (proj_spmv) {
          project_update(slot, yst);  // A v by an SpMV of the stored v
        } else if (p_from_y && proj_m[slot] > 0) {  // the direction stays pending (the next solve forms it)
          pend_otf[slot] = true;
          pend_y[slot] = yst;
          proj_pend[slot] = true;
        } else {
          project_update(slot, yst, bh, cg_r[0], pout);
        }
        if (projected && guess_decayed(slot, guess_rel())) proj_restart(slot);
      }
    } else {
      double* y[1] = {yst};
      const double* b[1] = {bh};
      it = cg<1>(dPp, HFace{}, dKp, y, b, prm.rtol_pres, prm.maxit_pres, which);
    }
    if (use_mg && proj && p_from_y) {  // p stays in y: the gradient gathers y's ghosts
      halo(yst);
      return it;
    }
    if (!(use_mg && proj) || proj_spmv) {
      algo_bytes += (20.0 + (sc ? 8.0 : 0.0)) * (double)n;  // master_of, y (, s) read; p written
      hipLaunchKernelGGL(k_cg_fin, dim3(grid_ew(n)), dim3(BS), 0, st, n, 1, sc, yst, (const double*)nullptr, pout,
                         (double*)nullptr, dmaster_of);
      KCHK();
    }
    halo(pout);
    return it;
  }
  // Successive right-hand sides (Fischer 1998) with a deferred update.
  // Guess for the right-hand side b: x0 = sum_i <X_i, b> X_i, the A-projection of the new solution
  // onto span X (X A-orthonormal).  Before it, the last solve's direction v = y - x0 (with A v) is
  // A-orthogonalised against X, cleared of the operator's null space and appended:
  //   X_m = s (v - mu 1_free - sum_i c_i X_i),  c_i = <X_i, A v>,  s = (<v, A v> - |c|^2)^-1/2,
  //   <X_m, b> = s (<v, b> - mu sum_free b - sum_i c_i <X_i, b>),
  // so one multi-dot pass over X (dots with b and A v, k_mdot2) and one combination pass (X_m and
  // x0 together, k_pcomb) do both: 2m + 9 vector passes per solve where a separate update took
  // 4m + 15.  A full basis is re-seeded first (proj_reseed).  With an empty basis the solve keeps
  // its warm start (x0 = 0).
  // returns whether a guess was projected (false: the first solve of the basis keeps its warm start)
  // rin: the right-hand side b is formed (and stored) by k_mdot2 from the divergence instead of read
  bool project_guess(int which, const double* b, double* y, const RhsIn* rin = nullptr) {
    const i64 n = lp.n_own;
    const ProjOp op = proj_op(which);
    ProjHist& H = proj_hist[which];
    proj_coords(which);
    int m = proj_m[which];
    if (!proj_pend[which]) {  // first solve: no direction yet
      HIPCHK(hipMemsetAsync(proj_x0[which], 0, sizeof(double) * n, st));
      H.gamma.clear();
      return false;
    }
    const int nb = grid_ew(n);
    const RedOut rmd = ro(proj_d, CNT_MDOT, 2 * m + 4);
    // virtual blocks: nb blocks' rows and partials on a grid the chip holds at once (not with the fused reduction)
    int nbp = nb, nvb = 0;
    if (!rmd.out) {
      const int res = fit_grid((const void*)mdot2_kernel(m), nb);
      if (res < nb) {
        const int per = (nb + res - 1) / res;
        nbp = (nb + per - 1) / per;
        nvb = nb;
      }
    }
    // k_mdot2: X (fp32), b, A v, v read
    const bool otf = pend_otf[which];
    // a pending direction: A v from the residuals; v accumulated (pend_acc) or y - x0 (the first direction)
    const bool vdiff = otf && !pend_acc[which];
    const bool vz0 = pend_vzero[which];  // (v = 0: neither v nor y - x0 is read)
    const double* vp = vz0 ? nullptr : (const double*)pv[which];
    const PendDir pd = otf ? PendDir{vz0 ? nullptr : pend_y[which], (const double*)proj_x0[which], (const double*)cg_r[0],
                                     pend_acc[which] ? vp : nullptr}
                           : PendDir{nullptr, nullptr, nullptr, nullptr};
    // (rin: braw and slave_of read and b written instead of b read)
    klaunch(14,
            (4.0 * m + 24.0 + (otf ? 8.0 : 0.0) + (vdiff ? 8.0 : 0.0) - (vz0 ? 8.0 : 0.0) + (rin ? 12.0 : 0.0)) *
                (double)n,
            mdot2_kernel(m), dim3(nbp), dim3(BS), (int64_t)n,
            (const ProjT*)projX[which], (int64_t)pld(which), b, (const double*)pav[which], vp,
            op.null_free, proj_part, rmd, pd, rin ? *rin : RhsIn{}, nvb);
    if (!rmd.out) launch_reduce(proj_part, nb, MAXB, 2 * m + 4, false, proj_d);
    KCHK();
    if (dist()) comm->allreduce(proj_d, 2 * m + 4, false, st);
    QMat qm{};
    int kq = m;
    if (m == op.kmax) kq = proj_reseed(which, m, qm);  // full: X' = Q X, the dots follow as Q a, Q c
    hipLaunchKernelGGL(k_pcoef, dim3(1), dim3(64), 0, st, (const double*)proj_d, m, (const double*)dqm,
                       m == op.kmax ? kq : -1,
                       1.0 / (double)n_free, proj_coef);
    KCHK();
    HIPCHK(hipMemcpyAsync(h_coef + which * NCOEF, proj_coef, sizeof(double) * NCOEF, hipMemcpyDeviceToHost, st));
    // k_pcomb: X, v read; the new direction, y and x0 written (not x0 when the coming solve accumulates its
    // correction: the first update starts the accumulator, so it needs no clearing either)
    const bool acc_next = which <= 2 && !proj_spmv;
    klaunch(15, (4.0 * kq + (acc_next ? 24.0 : 32.0) + (vdiff ? 8.0 : 0.0) - (vz0 ? 8.0 : 0.0)) * (double)n,
            pcomb_kernel(kq), dim3(nb), dim3(BS), (int64_t)n,
            (const ProjT*)projX[which], (int64_t)pld(which), (const double*)proj_coef, vp,
            op.null_free, projX[which] + pcol(which, kq), y, acc_next ? (double*)nullptr : proj_x0[which],
            vdiff ? pend_y[which] : (const double*)nullptr, (double*)nullptr);
    pend_vzero[which] = false;
    KCHK();
    pend_otf[which] = false;
    H.coef_m = kq;
    proj_m[which] = kq + 1;
    proj_pend[which] = false;
    return true;
  }
  // coordinates bookkeeping: the last guess's coefficients (h_coef, copied with it; read after the
  // solve's host synchronisation) give the last solution y = x0 + v in the basis,
  // [gamma_i + c_i, 1 / s], and the last guess x0, [a_i, alpha_new]
  void proj_coords(int which) {
    ProjHist& H = proj_hist[which];
    if (H.coef_m < 0) return;
    const int m = H.coef_m;
    const double* K = h_coef + which * NCOEF;  // a (m), c (m), s, mu, alpha_new
    std::vector<double> y(m + 1, 0.0);
    for (int i = 0; i < m; ++i) y[i] = (i < (int)H.gamma.size() ? H.gamma[i] : 0.0) + K[m + i];
    y[m] = K[2 * m] > 0.0 ? 1.0 / K[2 * m] : 0.0;
    H.sols.push_back(std::move(y));
    if ((int)H.sols.size() > PROJ_KEEP_MAX) H.sols.erase(H.sols.begin());
    H.gamma.assign(K, K + m);
    H.gamma.push_back(K[2 * m + 2]);
    H.coef_m = -1;
  }
  // Full basis: re-seed it with the span of the last solutions and the last guess x0 (the pending
  // direction v then completes the span of the last solution).  In an A-orthonormal basis A-inner
  // products are coordinate dot products, so a Gram-Schmidt of the coordinate rows gives the new
  // basis' coefficients Q, X' = Q X (k_reseed, one pass over X).  Two Gram-Schmidt passes:
  // successive solutions are nearly parallel, one pass leaves Q orthogonal only to eps / |residual|,
  // and a basis that is not A-orthonormal makes the projection formula wrong, not just weaker;
  // seeds within 1e-6 of the span of the earlier ones add only their coordinates' noise.  Fischer's
  // restart (drop everything) costs a run of solves of 7, 5, 4, 3 iterations where the full basis
  // gives 1-2.  Returns the new basis size (<= kmax - 1).
  int64_t n_reseed = 0;  // full bases re-seeded so far (pucfem_path_info)
  int proj_reseed(int which, int m, QMat& qm) {
    ProjHist& H = proj_hist[which];
    ++n_reseed;
    const int cap = std::min(proj_keep, m - 1);
    std::vector<std::vector<double>> seeds;
    const int nh = std::min<int>((int)H.sols.size(), cap - 1);
    for (int k = (int)H.sols.size() - nh; k < (int)H.sols.size(); ++k) seeds.push_back(H.sols[k]);
    seeds.push_back(H.gamma);
    for (auto& v : seeds) v.resize(m, 0.0);
    std::vector<std::vector<double>> Q, R(seeds.size());
    for (size_t a = 0; a < seeds.size(); ++a) {
      std::vector<double> w = seeds[a];
      const double n0 = std::sqrt(std::inner_product(w.begin(), w.end(), w.begin(), 0.0));
      R[a].assign(PROJ_KEEP_MAX, 0.0);
      for (int pass = 0; pass < 2; ++pass)
        for (size_t b2 = 0; b2 < Q.size(); ++b2) {
          const double d = std::inner_product(w.begin(), w.end(), Q[b2].begin(), 0.0);
          R[a][b2] += d;
          for (int j = 0; j < m; ++j) w[j] -= d * Q[b2][j];
        }
      const double nw = std::sqrt(std::inner_product(w.begin(), w.end(), w.begin(), 0.0));
      if (nw > 1e-6 * n0 && nw > 0.0 && (int)Q.size() < cap) {
        R[a][Q.size()] = nw;
        for (double& x : w) x /= nw;
        Q.push_back(std::move(w));
      }
    }
    const int kq = (int)Q.size();
    for (int i = 0; i < kq; ++i)
      for (int j = 0; j < m; ++j) qm.q[i][j] = Q[i][j];
    // (pageable source: the copy is staged before the call returns)
    HIPCHK(hipMemcpyAsync(dqm, &qm, sizeof(QMat), hipMemcpyHostToDevice, st));
    const i64 n = lp.n_own;
    algo_bytes += 4.0 * (double)(m + kq) * (double)n;
    hipLaunchKernelGGL(k_reseed, dim3(grid_ew(n)), dim3(BS), 0, st, n, (const ProjT*)projX[which], pld(which), m,
                       (const double*)dqm, kq,
                       projXalt[which]);
    KCHK();
    std::swap(projX[which], projXalt[which]);
    H.sols.clear();
    for (int a = 0; a + 1 < (int)seeds.size(); ++a) H.sols.emplace_back(R[a].begin(), R[a].begin() + kq);
    H.gamma.assign(R.back().begin(), R.back().begin() + kq);
    return kq;
  }
  // after a solve: the new direction v = y - x0 and A v, for the next guess.  b, r_final (optional):
  // the solve's right-hand side and final CG residual, with its initial residual r0 = b - A x0 saved
  // in pav[which]: then A v = r0 - r_final (A y = b - r_final for the first direction, whose solve
  // started from the warm start with x0 = 0) instead of an SpMV -- exact up to the CG recurrence's
  // rounding drift.
  // pfin (with r_final): also the pressure solve's finish p = y with the slaves copied from their masters
  // (k_cg_fin's work, unscaled), in the same pass
  void project_update(int which, const double* y, const double* b = nullptr, const double* r_final = nullptr,
                      double* pfin = nullptr) {
    const i64 n = lp.n_own;
    const ProjOp op = proj_op(which);
    double *v = pv[which], *av = pav[which];
    if (r_final) {  // v = y - x0 (unless the solve accumulated it) and A v = r0 - r_final in one pass
      const bool whole = proj_m[which] == 0;
      double* vout = pend_acc[which] ? nullptr : v;
      if (pfin) {
        algo_bytes += (vout ? 68.0 : 52.0) * (double)n;  // + master_of read, p written
        hipLaunchKernelGGL(k_diff2_fin, dim3(grid_ew(n)), dim3(BS), 0, st, (int64_t)n, y,
                           (const double*)proj_x0[which], vout, whole ? b : (const double*)av, r_final, av,
                           (const int32_t*)dmaster_of, pfin);
      } else {
        algo_bytes += (vout ? 48.0 : 24.0) * (double)n;
        hipLaunchKernelGGL(k_diff2, dim3(grid_ew(n)), dim3(BS), 0, st, n, y, (const double*)proj_x0[which], vout,
                           whole ? b : (const double*)av, r_final, av);
      }
      KCHK();
    } else {
      hipLaunchKernelGGL(k_diff, dim3(grid_ew(n)), dim3(BS), 0, st, n, y, proj_x0[which], v);
      KCHK();
      halo(v);
      spmv_on(st, *op.A, op.fc, op.val, v, av);
    }
    proj_pend[which] = true;
  }
  // k_div with the pressure right-hand side; max |div| into maxout (a vals slot, or scratch), sum(braw)
  // into redbuf slot 3 (pressure's sb) -- fused when enabled (returns whether it was)
  bool div_rhs(const double* ax, const double* ay, double* out, double* maxout) {
    const RedOut r = ro(maxout, CNT_DIV, 2, MAXB, 1u, redbuf + 24);
    div(ax, ay, out, true, nullptr, r);
    if (!r.out) return false;
    if (maxout != redbuf + 40) red_done(maxout, 1, true);  // (redbuf slot 5: an unrecorded maximum)
    red_done(redbuf + 24, 1, false);
    return true;
  }
  // pp: p, or with p_from_y the pressure solve's y (gathered through the merged tables and columns)
  // gate (optional): the PCG's control word -- the projection runs only if the solve has finished by then
  double grad_proj(const double* pp, int mode, const int* gate = nullptr) {
    const FaceDev fc = p_from_y ? fP.full() : fK.full();
    const DevSell& A = p_from_y ? dPm : dP;
    const double bytes = (16.0 + A.idx_bytes()) * (double)A.nnz + A.row_bytes() * (double)A.nrows + 40.0 * (double)lp.n_own;
    with_c16(A, [&](auto c16) {
      klaunch(3, bytes, k_grad_proj<decltype(c16)::value>, dim3(grid_full(fc, A)), dim3(BS), A.view(), fc,
              (const double*)dGx, (const double*)dGy, pp, (const double*)das1, prm.dt, mode, (const uint8_t*)ddir,
              (const double*)usx, (const double*)usy, ux, uy, gate);
    });
    KCHK();
    return bytes;
  }
  // small meshes: the first projection with the velocity BCs (k_grad_proj_bc; the faces are empty there)
  int32_t* dspos = nullptr;  // the projection operator's (slice, lane) position of each row
  // (the position map is built before any graph capture: an allocation inside a captured step is not allowed)
  void prep_grad_proj_bc() {
    if (!dense || !dbcsrc || dspos) return;
    const DevSell& A = p_from_y ? dPm : dP;
    const int nb = (int)std::max<i64>(1, std::min<i64>(1024, (A.nslices * 64 + BS - 1) / BS));
    dspos = dalloc<int32_t>(std::max<i64>(1, lp.n_own));
    hipLaunchKernelGGL(k_sell_pos, dim3(nb), dim3(BS), 0, st, A.view(), dspos);
    KCHK();
  }
  void grad_proj_bc(const double* pp) {
    const DevSell& A = p_from_y ? dPm : dP;
    const int nb = (int)std::max<i64>(1, std::min<i64>(1024, (A.nslices * 64 + BS - 1) / BS));
    algo_bytes += (16.0 + A.idx_bytes()) * (double)A.nnz + A.row_bytes() * (double)A.nrows + 40.0 * (double)lp.n_own;
    with_c16(A, [&](auto c16) {
      hipLaunchKernelGGL(k_grad_proj_bc<decltype(c16)::value>, dim3(nb), dim3(BS), 0, st, A.view(), (const double*)dGx,
                         (const double*)dGy, pp, (const double*)das1, prm.dt, (const double*)usx, ux,
                         (const int32_t*)dbcsrc, (const int32_t*)dbcdir, (const int32_t*)dspos, (const double*)ddval,
                         dir_ncomp);
    });
    KCHK();
  }
  // The gradient projection after a pressure solve, enqueued behind the solve's convergence reads and gated on its
  // control word (PUCFEM_GP_GATE, default on): when the read finds the solve converged the GPU has been running the
  // projection during the host's round trip (the r13g trace: ~50 us idle before each k_grad_proj), and when it finds
  // it not converged the launch did nothing and the next read enqueues it again.  Single rank, multigrid path with
  // p kept in y (nothing is launched between the solve's last read and the projection there).
  struct GpGate {
    bool on = false, done = false;
    const double* pp = nullptr;
    int mode = 0;
    double bytes = 0.0;
  } gp_gate;
  // a pressure solve with the gated projection armed (disarmed if the solve throws)
  int gated_pressure(const GpGate& g, double* yst, double* pout, int which, bool sb_fused) {
    gp_gate = g;
    try {
      return pressure(yst, pout, which, sb_fused);
    } catch (...) {
      gp_gate = GpGate{};
      throw;
    }
  }
  // after the solve: whether the gated projection ran (then its bytes are counted here)
  bool gp_gate_end() {
    const bool d = gp_gate.done;
    if (d) {
      algo_bytes += gp_gate.bytes;
      cls_bytes[3] += gp_gate.bytes;
      ++cls_n[3];
    }
    gp_gate = GpGate{};
    return d;
  }
  bool gp_gate_env = !(std::getenv("PUCFEM_GP_GATE") && std::atoi(std::getenv("PUCFEM_GP_GATE")) == 0);
  // the PCG's control-word read (h_ctl), with the gated projection behind it
  // arm: enqueue the gated projection behind this read (pcg_mg: when the solve has reached the last solve's count, so
  // that a read unlikely to find it converged adds no launch that does nothing)
  void read_ctl(bool arm = true) {
    HIPCHK(hipMemcpyAsync(h_ctl, ctl, 6 * sizeof(int), hipMemcpyDeviceToHost, st));  // (+ the note)
    if (!gp_gate.on || !arm) {
      sync_st();
      return;
    }
    if (!ev_wait) HIPCHK(hipEventCreateWithFlags(&ev_wait, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ev_wait, st));
    sl_join();  // (the dye tail reads u)
    const size_t np = timer.pend.size();
    const double b = grad_proj(gp_gate.pp, gp_gate.mode, ctl);
    const bool timed = timer.on && timer.pend.size() == np + 1;
    if (timed) timer.pend.back().keep = true;
    // its bytes are counted by the caller once the solve has returned (the solve takes back the counts of launches
    // behind its converged iteration)
    algo_bytes -= b;
    cls_bytes[3] -= b;
    --cls_n[3];
    gp_gate.bytes = b;
    wait_event(ev_wait);
    if (h_ctl[0]) {
      gp_gate.done = true;
      gp_gate.on = false;
    } else if (timed) {
      timer.pend[np].cls = -1;  // (the launch found the solve unfinished: no sample)
    }
  }

  // side stream of the overlapped dye advection (stokes_step)
  hipStream_t st_sl = nullptr;
  int sl_prio = 0;  // (PUCFEM_STREAM_PRIO: the side stream's priority)
  bool sl_prio_on = false;
  hipEvent_t ev_u = nullptr, ev_sl = nullptr;
  bool sl_overlap = true, sl_pending = false;
  double* part_mx = nullptr;  // k_mix2 partials (part_b belongs to the solvers of the main stream)
  double* part_fd = nullptr;  // final-divergence partials (part_d: the main stream's)
  struct StreamSwap {  // run the enclosed launches on the other stream (restored on unwind)
    hipStream_t &a, &b;
    StreamSwap(hipStream_t& x, hipStream_t& y) : a(x), b(y) { std::swap(a, b); }
    ~StreamSwap() { std::swap(a, b); }
  };
  // order the main stream after the pending dye advection
  void sl_join() {
    dye_tail_release();
    if (!sl_pending) return;
    HIPCHK(hipStreamWaitEvent(st, ev_sl, 0));
    sl_pending = false;
  }

  // one StokesColor / StokesFood step (StokesColor.py:537-586, StokesFood.py:441-505)
  RedOut sl_ro{};
  // The dye tail of a step (final-divergence record, semi-Lagrangian advection, mixing sums, its part of
  // the step record) on the side stream, after the main stream's event `gate`.  (Round 3 measured the
  // tail enqueued after the next step's viscous solve instead, beside the pressure solve: the time moved
  // between the streams, the step rate stayed, r8j.)
  // (round 4 measured the tail released after the next step's first viscous step and after its viscous
  // solve: neutral, r10f; it is released at the end of the step)
  hipEvent_t ev_gate = nullptr;
  // PUCFEM_DYE_GATE (measurement knob): where the semi-Lagrangian part of the tail (advection, mixing sums, the
  // record) is released -- 0 with the final-divergence record at the end of the step (default), 1 at the first
  // V-cycle of the next step's first pressure solve (beside its latency-bound coarse levels), 2 at the start of that
  // pressure solve, 3 / 4 after the first SELL launch / the face kernel of the next viscous solve's first pair
  int dye_gate = std::getenv("PUCFEM_DYE_GATE") ? std::atoi(std::getenv("PUCFEM_DYE_GATE")) : 0;
  bool slb_pend = false;     // the semi-Lagrangian part waits for its release (dye_gate > 0)
  double* slb_rec = nullptr;
  struct SmallRed {  // (reset on unwind)
    bool& f;
    explicit SmallRed(bool& x) : f(x) { f = true; }
    ~SmallRed() { f = false; }
  };
  void dye_tail(double* rec) {
    HIPCHK(hipEventRecord(ev_gate, st));
    HIPCHK(hipStreamWaitEvent(st_sl, ev_gate, 0));
    {
      StreamSwap sw(st, st_sl);
      SmallRed small_red(red_small);
      if (dye_gate == 0 && dye_sl_first) dye_tail_sl(rec, false);
      const RedOut rf = ro(vals + 1, CNT_DYE_DIV, 1, MAXB, 1u);
      div(ux, uy, nullptr, false, part_fd, rf);  // (the final div field is computed when read)
      if (!rf.out) reduce_into(part_fd, div_grid(), 1, true, 1);  // max |final div|
      if (dye_gate == 0 && !dye_sl_first) dye_tail_sl(rec);
      if (dye_gate == 0 && dye_sl_first) {
        hipLaunchKernelGGL(k_stats, dim3(1), dim3(64), 0, st, vals, rec, 6);
        KCHK();
      }
    }
    if (dye_gate == 0) {
      HIPCHK(hipEventRecord(ev_sl, st_sl));
      sl_pending = true;
    } else {
      slb_pend = true;
      slb_rec = rec;
    }
  }
  // PUCFEM_DYE_SL_FIRST=1 (measurement knob): the tail's semi-Lagrangian part before its final-divergence record
  bool dye_sl_first = std::getenv("PUCFEM_DYE_SL_FIRST") && std::atoi(std::getenv("PUCFEM_DYE_SL_FIRST")) != 0;
  // the semi-Lagrangian part of the tail (launched on st_sl: the caller swapped the streams); stats: the step
  // record after it (else the caller writes it)
  void dye_tail_sl(double* rec, bool stats = true) {
    const int nb = nb_sl(lp.n_own);
    const RedOut rs = ro(vals + 2, CNT_DYE_SL, 3, SLB);
    sl_launch(nb, lp.r0, lp.n_own, ux, uy, prm.dt, c_full, c_new, dwmix, nullptr, rs);
    KCHK();
    std::swap(c_full, c_new);
    if (!rs.out) reduce_into(part_sl, nb, 3, false, 2, SLB);  // sum wc, sum w, not-found
    const int nbm = nb_rows(lp.n_own);
    algo_bytes += 16.0 * (double)lp.n_own;  // c, w
    const RedOut rm = ro(vals + 5, CNT_DYE_MIX, 1);
    hipLaunchKernelGGL(k_mix2, dim3(nbm), dim3(BS), 0, st, lp.r0, lp.n_own, c_full, dwmix, vals + 2, 1, 1,
                       part_mx, rm);
    KCHK();
    if (!rm.out) reduce_into(part_mx, nbm, 1, false, 5);
    if (!stats) return;
    hipLaunchKernelGGL(k_stats, dim3(1), dim3(64), 0, st, vals, rec, 6);
    KCHK();
  }
  // release a deferred semi-Lagrangian part (dye_gate > 0): behind the main stream's work so far
  void dye_tail_release() {
    if (!slb_pend) return;
    slb_pend = false;
    HIPCHK(hipEventRecord(ev_gate, st));
    HIPCHK(hipStreamWaitEvent(st_sl, ev_gate, 0));
    {
      StreamSwap sw(st, st_sl);
      SmallRed small_red(red_small);
      dye_tail_sl(slb_rec);
    }
    HIPCHK(hipEventRecord(ev_sl, st_sl));
    sl_pending = true;
  }
  // W > 1, StokesColor: the second half of a step's dye tail (dye_range_start queued the first at its end): the
  // wide halo, the semi-Lagrangian advection of the owned rows, the mixing sums and the rest of the step record.
  // It reads the step's final u and c; the next step's viscous solve writes neither, and its first write to u (the
  // gradient projection) follows in stream order.
  bool tail_pend = false;
  double* tail_rec = nullptr;
  void dye_tail_dist() {
    if (!tail_pend) return;
    tail_pend = false;
    dye_halo_exchange();
    const int nb = nb_sl(lp.n_own);
    sl_ro = ro(vals + 2, CNT_SL, 3, SLB);
    sl_launch(nb, lp.r0, lp.n_own, ux, uy, prm.dt, c_full, c_new, dwmix, nullptr, sl_ro);
    KCHK();
    // (the replica keeps its halo values; k_mix2 copies the new owned segment into it)
    if (sl_ro.out) red_done(vals + 2, 3, false);
    else reduce_into(part_sl, nb, 3, false, 2, SLB);  // sum wc, sum w, not-found
    sl_ro = RedOut{};
    const int nbm = nb_rows(lp.n_own);
    algo_bytes += 16.0 * (double)lp.n_own;
    const RedOut rm = ro(vals + 5, CNT_MIX, 1);
    hipLaunchKernelGGL(k_mix2, dim3(nbm), dim3(BS), 0, st, lp.r0, lp.n_own, (const double*)c_new, dwmix, vals + 2, 1, 1,
                       part_mx, rm, c_full);
    KCHK();
    if (rm.out) red_done(vals + 5, 1, false);
    else reduce_into(part_mx, nbm, 1, false, 5);
    hipLaunchKernelGGL(k_stats, dim3(1), dim3(64), 0, st, vals, tail_rec, 4);
    KCHK();
  }
  void stokes_step(double* rec, int32_t* its) {
    int itv = 0;
    ring_in_mix = false;
    viscous(itv);
    dye_tail_dist();  // (W > 1: the previous step's dye tail)
    // max |div u*| -> vals[0]; the div u* field itself is computed when read (pucfem_get_field): nothing in the
    // step reads it, and its 8 B/row store is a quarter of the kernel's bytes
    const bool f1 = div_rhs(usx, usy, nullptr, vals);
    if (!f1) reduce_into(part_d, div_grid(), 1, true, 0);
    const bool gpg = gp_gate_env && use_mg && proj_k > 0 && p_from_y && !dist() && !proj_spmv;
    // (a solve that throws leaves no gated projection armed for later calls: gated_pressure resets it on unwind)
    const int itp = gated_pressure(GpGate{gpg, false, yp, 0, 0.0}, yp, p, 1, f1);
    const bool gp1 = gp_gate_end();
    sl_join();  // the previous step's dye advection still reads u: it must finish before u is rewritten
    if (dense && dspos && dense_bc && dir_ncomp == 2 && !gp1 && (p_from_y ? fP : fK).rows == 0) {
      grad_proj_bc(p_from_y ? yp : p);  // (the BCs inside the projection: small meshes)
    } else {
      if (!gp1) grad_proj(p_from_y ? yp : p, 0);
      bc(ux, uy);
    }
    halo_v(ux);
    const bool f2 = div_rhs(ux, uy, div_u, redbuf + 40);  // (its max is not recorded: scratch slot 5)
    const int itp2 = gated_pressure(GpGate{gpg, false, yp2, 1, 0.0}, yp2, p2, 2, f2);
    const bool gp2 = gp_gate_end();
    if (!gp2) grad_proj(p_from_y ? yp2 : p2, 1);
    halo_v(ux);
    // single-rank explicit dye: the final-divergence record and the advection of this step (they read
    // the final u and c, write final_div, c_new and their own partials) run on a side stream,
    // overlapped with the next step's viscous solve and first pressure solve; the main stream waits
    // for them before its next write to u (sl_join above)
    const bool ovl = sl_overlap && scheme == PUCFEM_STOKES_COLOR && !dye_impl && !graph_mode && !dist();
    if (!ovl) {
      const RedOut r = ro(vals + 1, CNT_DIV, 1, MAXB, 1u);
      // captured small-mesh step (fused reductions): the final-divergence record on a forked branch of the graph, beside
      // the semi-Lagrangian advection (both read u and write their own partials); joined before the step record
      const bool fork = gcapture && r.out && !dye_impl && st_fk != nullptr && scheme == PUCFEM_STOKES_COLOR;
      if (fork) {
        HIPCHK(hipEventRecord(ev_fk, st));
        HIPCHK(hipStreamWaitEvent(st_fk, ev_fk, 0));
        {
          StreamSwap sw(st, st_fk);
          div(ux, uy, nullptr, false, nullptr, r);
        }
        HIPCHK(hipEventRecord(ev_fj, st_fk));
        fork_pend = true;
      } else {
        div(ux, uy, dye_impl ? final_div : nullptr, false, nullptr, r);  // (the implicit dye reads it)
      }
      if (r.out) red_done(vals + 1, 1, true);
      else reduce_into(part_d, div_grid(), 1, true, 1);  // max |final div|
    }
    if (ovl) {
      if (!st_sl) {
        // (stream priorities and CU masks for the side stream were measured and changed nothing or lost,
        // rounds 2-3: r4d, r6c)
        // PUCFEM_SL_CUMASK=k (measurement knob, 1..7): the side stream on k of every 8 CUs (mask bits i with
        // i % 8 < k), the rest left to the main stream's small launches
        const int cuk = std::getenv("PUCFEM_SL_CUMASK") ? std::atoi(std::getenv("PUCFEM_SL_CUMASK")) : 0;
        if (cuk > 0 && cuk < 8) {
          int d = 0, ncu = 0;
          HIPCHK(hipGetDevice(&d));
          HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d));
          std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
          for (int i = 0; i < ncu; ++i)
            if (i % 8 < cuk) mask[(size_t)i / 32] |= 1u << (i % 32);
          HIPCHK(hipExtStreamCreateWithCUMask(&st_sl, (uint32_t)mask.size(), mask.data()));
        } else if (sl_prio_on) {
          HIPCHK(hipStreamCreateWithPriority(&st_sl, hipStreamNonBlocking, sl_prio));
        } else {
          HIPCHK(hipStreamCreateWithFlags(&st_sl, hipStreamNonBlocking));
        }
        HIPCHK(hipEventCreateWithFlags(&ev_u, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_sl, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_gate, hipEventDisableTiming));
      }
      hipLaunchKernelGGL(k_stats, dim3(1), dim3(64), 0, st, vals, rec, 1);  // max |div u*|
      KCHK();
      dye_tail(rec);
    } else if (scheme == PUCFEM_STOKES_COLOR) {
      const int nb = nb_sl(lp.n_own);
      if (dye_impl) {
        last_dye_it = dye_step(ux, uy, final_div, c_full, c_new);
        hipLaunchKernelGGL(k_wsum, dim3(nb), dim3(BS), 0, st, lp.r0, lp.n_own, (const double*)c_new,
                           (const double*)dwmix, part_sl);
      } else if (dist()) {
        // W > 1: the back-traced ranges now, the rest of the tail at the next step (dye_tail_dist)
        hipLaunchKernelGGL(k_stats, dim3(1), dim3(64), 0, st, vals, rec, 3);  // max |div u*|, max |final div|
        KCHK();
        dye_range_start(uy, prm.dt);
        tail_pend = true;
        tail_rec = rec;
        its[0] = itv;
        its[1] = itp;
        its[2] = itp2;
        return;
      } else {
        sl_ro = ro(vals + 2, CNT_SL, 3, SLB);
        sl_launch(nb, lp.r0, lp.n_own, ux, uy, prm.dt, c_full, c_new, dwmix, nullptr, sl_ro);
      }
      KCHK();
      // fixed buffers inside a captured graph: k_mix2 copies the new values back instead of a swap
      const bool mix_copy = graph_mode && !dye_impl;
      if (graph_mode && dye_impl) {
        HIPCHK(hipMemcpyAsync(c_full + lp.r0, c_new + lp.r0, sizeof(double) * lp.n_own, hipMemcpyDeviceToDevice, st));
      } else if (!mix_copy) {
        std::swap(c_full, c_new);
      }
      if (sl_ro.out) red_done(vals + 2, 3, false);
      else reduce_into(part_sl, nb, 3, false, 2, SLB);  // sum wc, sum w, not-found
      sl_ro = RedOut{};
      const int nbm = nb_rows(lp.n_own);
      algo_bytes += 16.0 * (double)lp.n_own;
      fork_join();  // (k_mix2's reducing block writes the step record, which holds the final divergence)
      const RedOut rm = ro(vals + 5, CNT_MIX, 1);
      // (captured small-mesh step with the fused reduction: k_mix2's reducing block appends the step record)
      ring_in_mix = gcapture && rm.out && !ovl && ring_fold;
      hipLaunchKernelGGL(k_mix2, dim3(nbm), dim3(BS), 0, st, lp.r0, lp.n_own, mix_copy ? (const double*)c_new : c_full,
                         dwmix, vals + 2, 1, 1, part_mx, rm, mix_copy ? c_full : (double*)nullptr, (const double*)vals,
                         ring_in_mix ? gring : (double*)nullptr, ring_in_mix ? gcount : (int*)nullptr, 7);
      KCHK();
      if (rm.out) red_done(vals + 5, 1, false);
      else reduce_into(part_mx, nbm, 1, false, 5);
    } else {
      tracer_advance(prm.dt);
    }
    fork_join();
    if (!ovl) {
      if (gcapture) {
        if (!ring_in_mix) hipLaunchKernelGGL(k_stats_ring, dim3(1), dim3(64), 0, st, vals, gring, gcount, 7);
      } else {
        hipLaunchKernelGGL(k_stats, dim3(1), dim3(64), 0, st, vals, rec, 7);
      }
      KCHK();
    }
    its[0] = itv;
    its[1] = itp;
    its[2] = itp2;
  }

  // the finest multigrid level's lmax (lmax_estimate's power iteration, on the device operator):
  // min(Gershgorin bound gersh, 1.1 x 30 steps of x <- D^-1 A x / |D^-1 A x|)
  double lmax_device(double gersh, double* lam_out) {
    const i64 n = lp.n_own;
    struct Scratch {  // setup scratch: freed on return, not kept with the context
      double* p = nullptr;
      Scratch(i64 m) { HIPCHK(hipMalloc(&p, sizeof(double) * (size_t)std::max<i64>(1, m))); }
      ~Scratch() { (void)hipFree(p); }
    } xt(nloc), yt(nloc), dt(n);
    double *x = xt.p, *y = yt.p, *dinv = dt.p;
    std::vector<double> x0;  // (global row index: a partitioned run iterates the single-rank vector)
    host_alloc_fresh(x0, n);
    parallel_for(n, [&](i64 i0, i64 i1) {
      for (i64 i = i0; i < i1; ++i) x0[i] = 1.0 + 0.5 * std::sin((double)(lp.r0 + i));
    });
    h2d(dinv, lmax_dinv.data() + lp.r0, sizeof(double) * n);
    h2d(x, x0.data(), sizeof(double) * n);
    const int nb = nb_rows(n), ge = grid_ew(n);
    double lam = 0.0;
    for (int it = 0; it < 30; ++it) {
      halo(x);
      spmv_on(st, dPp, fP.full(), dKp_raw, x, y);
      hipLaunchKernelGGL(k_vmul, dim3(ge), dim3(BS), 0, st, n, (const double*)y, dinv, y);
      hipLaunchKernelGGL(k_dot2, dim3(nb), dim3(BS), 0, st, n, (const double*)x, (const double*)x, (const double*)y,
                         (const double*)y, part_a);
      hipLaunchKernelGGL(k_reduce, dim3(2), dim3(RB), 0, st, part_a, nb, MAXB, 2, 0, redbuf);
      KCHK();
      if (dist()) comm->allreduce(redbuf, 2, false, st);
      HIPCHK(hipMemcpyAsync(h_pinned, redbuf, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      const double nx = h_pinned[0], ny = h_pinned[1];
      lam = std::sqrt(ny / nx);
      hipLaunchKernelGGL(k_axpbypcz, dim3(ge), dim3(BS), 0, st, n, (const double*)nullptr, (const double*)y,
                         (const double*)nullptr, (const double*)nullptr, (const double*)nullptr, (const double*)nullptr,
                         1.0 / std::sqrt(ny), 0.0, 0.0, x);
      KCHK();
    }
    HIPCHK(hipStreamSynchronize(st));
    lmax_dinv.clear();
    lmax_dinv.shrink_to_fit();
    *lam_out = lam;
    return std::min(gersh, 1.1 * lam);
  }

  // a coarse multigrid level's lmax: lmax_estimate's 30-step power iteration on the level's device operator
  // (its V-cycle values: fp32 in the fp32 cycle) instead of on the host, min(Gershgorin bound gersh, 1.1 lam);
  // a partitioned level exchanges its halo before each product and all-reduces the norms
  template <typename T>
  double lmax_level_device(MgLevel& L, double gersh) {
    MgBufs<T>& B = bufs<T>(L);
    const i64 n = L.lp.n_own, r0 = L.own0(rank);
    std::vector<T> x0;
    host_alloc_fresh(x0, n);
    parallel_for(n, [&](i64 i0, i64 i1) {
      for (i64 i = i0; i < i1; ++i) x0[i] = (T)(1.0 + 0.5 * std::sin((double)(r0 + i)));
    });
    h2d(B.x, x0.data(), sizeof(T) * n);
    HIPCHK(hipMemsetAsync(B.b, 0, sizeof(T) * L.nloc, st));
    HIPCHK(hipMemsetAsync(ctl, 0, 2 * sizeof(int), st));
    const FaceDev fr = L.hA.full();
    const DevSell& A = L.dA;
    const int nb = nb_rows(n), ge = grid_ew(n);
    double lam = 0.0;
    for (int it = 0; it < 30; ++it) {
      mg_halo(L, B.x);
      B.with_vals([&](auto* val) {
        using VT = std::remove_const_t<std::remove_pointer_t<decltype(val)>>;
        with_c16(A, [&](auto c16) {
          hipLaunchKernelGGL((k_resid<T, T, VT, decltype(c16)::value, 0>), dim3(grid_full(fr, A)), dim3(BS), 0, st,
                             A.view(), fr, val, (const T*)B.b, (const T*)B.x, B.res, (const int*)ctl);
        });
      });
      hipLaunchKernelGGL(k_pow_step<T>, dim3(nb), dim3(BS), 0, st, (int64_t)n, (const T*)B.x, (const T*)B.res,
                         (const T*)B.dinv, B.x2, part_a);
      hipLaunchKernelGGL(k_reduce, dim3(2), dim3(RB), 0, st, part_a, nb, MAXB, 2, 0, redbuf);
      KCHK();
      if (dist() && !L.rep) comm->allreduce(redbuf, 2, false, st);
      HIPCHK(hipMemcpyAsync(h_pinned, redbuf, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      const double nx = h_pinned[0], ny = h_pinned[1];
      lam = std::sqrt(ny / nx);
      hipLaunchKernelGGL(k_pow_scale<T>, dim3(ge), dim3(BS), 0, st, (int64_t)n, (const T*)B.x2, 1.0 / std::sqrt(ny),
                         B.x);
      KCHK();
    }
    HIPCHK(hipStreamSynchronize(st));
    L.lam_dev = lam;
    return std::min(gersh, 1.1 * lam);
  }

  // implicit dye step (good_visualization.py:700-718) from cin with velocity (vx, vy) and its lumped
  // divergence dv into cout: assemble the merged operator, rhs = M c, BiCGStab from c, periodic copies
  int dye_step(const double* vx, const double* vy, const double* dv, const double* cin, double* cout) {
    const i64 n = lp.n_own;
    hipLaunchKernelGGL(k_dye_w, dim3(grid_ew(mesh.T)), dim3(BS), 0, st, MeshDev{mx, my, mtri, mesh.T}, vx, vy, dDyeW);
    hipLaunchKernelGGL(k_dye_assemble, dim3(grid_ew(dye.nslots)), dim3(BS), 0, st, dye, (const double*)dDyeW, dv,
                       prm.dt, prm.dye_diffusivity, dDyeVal);
    hipLaunchKernelGGL(k_dye_dinv, dim3(grid_ew(n)), dim3(BS), 0, st, n, (const int64_t*)dDyeDiag,
                       (const double*)dDyeVal, dDyeDinv);
    KCHK();
    with_c16(dDye, [&](auto c16) {
      hipLaunchKernelGGL(k_spmv<decltype(c16)::value>, dim3(nb_for(dDye.nslices)), dim3(BS), 0, st, dDye.view(), nof(),
                         (const double*)dDyeM, cin, dDyeB);
    });
    KCHK();
    if (dye_nsrow > 0) {
      hipLaunchKernelGGL(k_dye_rhs_fix, dim3(std::min(256, (dye_nsrow + BS - 1) / BS)), dim3(BS), 0, st, dye_nsrow,
                         (const int32_t*)dDyeSrow, (const int64_t*)dDyeSptr, (const int32_t*)dDyeSk,
                         (const int32_t*)dDyeSc, dye, (const double*)dDyeW, dv, prm.dt, prm.dye_diffusivity, cin, dDyeB);
      KCHK();
    }
    HIPCHK(hipMemcpyAsync(cout, cin, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
    const int it = bicgstab(cout, dDyeB, std::max(prm.rtol_lin, 1e-13), prm.maxit_lin, &dDye, dDyeVal, dDyeDinv);
    if (ncopy > 0) {  // c[slave] = c[master] (good_visualization.py:715-716)
      if (bc_gather) {
        hipLaunchKernelGGL(k_bc_gather, dim3(std::min(1024, (ncopy + BS - 1) / BS)), dim3(BS), 0, st, ncopy, dcsrc,
                           dbctmp, 1, cout, cout, 1);
        KCHK();
      }
      hipLaunchKernelGGL(k_bc_apply, dim3(std::min(1024, (ncopy + BS - 1) / BS)), dim3(BS), 0, st, ncopy, dcdst, dcsrc,
                         bc_gather ? (const double*)dbctmp : nullptr, 0, ddnode, ddval, 1, cout, cout, 1);
      KCHK();
    }
    return it;
  }

  void tracer_advance(double dt) {
    if (ntr == 0) {
      HIPCHK(hipMemsetAsync(vals + 6, 0, sizeof(double), st));
      return;
    }
    if (!has_tgrid) throw Error(PUCFEM_ESTATE, "tracer grid not built (scheme is not STOKES_FOOD)");
    double *fx = ux, *fy = uy;
    if (dist()) {
      // no replica of u: each rank interpolates the tracers in its own triangles from its owned and
      // ghost values (placed at their global ids), then one all-reduce of 3 x ntr values hands every
      // rank all the velocities (StokesFood's 488 tracers: ~12 KB per step instead of the whole u)
      hipLaunchKernelGGL(k_unstride, dim3(grid_ew(lp.n_own)), dim3(BS), 0, st, lp.n_own, (const double*)ux, VS,
                         ufx + lp.r0);
      hipLaunchKernelGGL(k_unstride, dim3(grid_ew(lp.n_own)), dim3(BS), 0, st, lp.n_own, (const double*)uy, VS,
                         ufy + lp.r0);
      if (lp.n_ghost > 0) {
        hipLaunchKernelGGL(k_scatter_ghosts, dim3(grid_ew(lp.n_ghost)), dim3(BS), 0, st, lp.n_ghost,
                           (const int32_t*)dghost_global, (const double*)(ux + VS * lp.n_own), ufx, VS);
        hipLaunchKernelGGL(k_scatter_ghosts, dim3(grid_ew(lp.n_ghost)), dim3(BS), 0, st, lp.n_ghost,
                           (const int32_t*)dghost_global, (const double*)(uy + VS * lp.n_own), ufy, VS);
      }
      hipLaunchKernelGGL(k_tracer_vel, dim3((ntr + BS - 1) / BS), dim3(BS), 0, st, MeshDev{mx, my, mtri, mesh.T},
                         tgrid, (const double*)ufx, (const double*)ufy, ntr, (const double*)trx, (const double*)try_,
                         (int64_t)lp.r0, (int64_t)lp.r1, trv);
      KCHK();
      comm->allreduce(trv, 3 * (size_t)ntr, false, st);
      hipLaunchKernelGGL(k_tracer_move, dim3(1), dim3(BS), 0, st, ntr, trx, try_, trs, (const double*)trv, dt,
                         prm.center_x, prm.center_y, prm.capture_radius, vals + 6);
      KCHK();
      return;
    }
    hipLaunchKernelGGL(k_tracer, dim3(1), dim3(BS), 0, st, MeshDev{mx, my, mtri, mesh.T}, tgrid, fx, fy, ntr, trx,
                       try_, trs, dt, prm.center_x, prm.center_y, prm.capture_radius, vals + 6);
    KCHK();
  }

  // ------------------------------------------------------------------ literal operators (heat / Poisson)
  // Jacobi-preconditioned BiCGStab on the literal operator (heat / Poisson) or, given A / av / dinv,
  // on another fully stored SELL operator (the implicit dye system)
  int bicgstab(double* x, const double* b, double tol, int maxit, const DevSell* A = nullptr,
               const double* av = nullptr, const double* dinv_op = nullptr) {
    const i64 n = lp.n_own;
    const int nb = nb_rows(n), ge = grid_ew(n);
    double *r = litw[0], *rh = litw[1], *pp = litw[2], *v = litw[3], *s = litw[4], *t = litw[5], *ph = litw[6],
           *sh = litw[7];
    const DevSell& AA = A ? *A : dLit;
    const double* AV = A ? av : dLitv;
    const double* dlit_dinv = A ? dinv_op : this->dlit_dinv;
    auto spmv = [&](const double* in, double* out) {
      with_c16(AA, [&](auto c16) {
        hipLaunchKernelGGL(k_spmv<decltype(c16)::value>, dim3(nb_for(AA.nslices)), dim3(BS), 0, st, AA.view(), nof(),
                           AV, in, out);
      });
      KCHK();
    };
    spmv(x, t);
    hipLaunchKernelGGL(k_axpbypcz, dim3(ge), dim3(BS), 0, st, n, (const double*)nullptr, b, (const double*)nullptr,
                       (const double*)t, (const double*)nullptr, (const double*)nullptr, 1.0, -1.0, 0.0, r);
    KCHK();
    HIPCHK(hipMemcpyAsync(rh, r, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemsetAsync(pp, 0, sizeof(double) * n, st));
    HIPCHK(hipMemsetAsync(v, 0, sizeof(double) * n, st));
    const double init[8] = {1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    HIPCHK(hipMemcpyAsync(bicg_sc, init, sizeof(init), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_dot2, dim3(nb), dim3(BS), 0, st, n, b, b, (const double*)r, (const double*)r, part_a);
    KCHK();
    hipLaunchKernelGGL(k_reduce, dim3(2), dim3(RB), 0, st, part_a, nb, MAXB, 2, 0, bicg_sc + 8);
    KCHK();
    HIPCHK(hipMemcpyAsync(h_pinned, bicg_sc + 8, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const double bb = h_pinned[0];
    double rr = h_pinned[1];
    const double tol2 = tol * tol * bb;
    int it = 0;
    while (!(rr <= tol2)) {
      if (it >= maxit || !std::isfinite(rr)) throw Error(PUCFEM_ENOCONV, "BiCGStab did not converge");
      hipLaunchKernelGGL(k_dot2, dim3(nb), dim3(BS), 0, st, n, rh, r, (const double*)nullptr, (const double*)nullptr, part_a);
      hipLaunchKernelGGL(k_bicg_scalar, dim3(1), dim3(BS), 0, st, 0, part_a, nb, bicg_sc);
      hipLaunchKernelGGL(k_bicg_p, dim3(ge), dim3(BS), 0, st, n, r, pp, v, dlit_dinv, ph, bicg_sc);
      spmv(ph, v);
      hipLaunchKernelGGL(k_dot2, dim3(nb), dim3(BS), 0, st, n, rh, v, (const double*)nullptr, (const double*)nullptr, part_a);
      hipLaunchKernelGGL(k_bicg_scalar, dim3(1), dim3(BS), 0, st, 1, part_a, nb, bicg_sc);
      hipLaunchKernelGGL(k_bicg_s, dim3(ge), dim3(BS), 0, st, n, r, v, dlit_dinv, s, sh, bicg_sc);
      spmv(sh, t);
      hipLaunchKernelGGL(k_dot2, dim3(nb), dim3(BS), 0, st, n, t, s, (const double*)t, (const double*)t, part_a);
      hipLaunchKernelGGL(k_bicg_scalar, dim3(1), dim3(BS), 0, st, 2, part_a, nb, bicg_sc);
      hipLaunchKernelGGL(k_bicg_x, dim3(ge), dim3(BS), 0, st, n, x, ph, sh, s, t, r, bicg_sc);
      hipLaunchKernelGGL(k_dot2, dim3(nb), dim3(BS), 0, st, n, r, r, (const double*)nullptr, (const double*)nullptr, part_a);
      hipLaunchKernelGGL(k_reduce, dim3(1), dim3(RB), 0, st, part_a, nb, MAXB, 1, 0, bicg_sc + 5);
      KCHK();
      HIPCHK(hipMemcpyAsync(h_pinned, bicg_sc + 5, sizeof(double), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      rr = h_pinned[0];
      ++it;
    }
    return it;
  }
};

Ctx* C(void* p) { return static_cast<Ctx*>(p); }

void spmv_on(hipStream_t st, const DevSell& A, const FaceDev& fc, const double* val, const double* x, double* y) {
  with_c16(A, [&](auto c16) {
    hipLaunchKernelGGL(k_spmv<decltype(c16)::value>, dim3(Ctx::grid_part(fc, A)), dim3(BS), 0, st, A.view(),
                       fc, val, x, y);
  });
}

template <class F>
int guard(void* ctx, F&& f) {
  try {
    f();
    return PUCFEM_OK;
  } catch (const Error& e) {
    (ctx ? C(ctx)->err : g_err) = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    (ctx ? C(ctx)->err : g_err) = "out of host memory";
    return PUCFEM_ENOMEM;
  } catch (const std::exception& e) {
    (ctx ? C(ctx)->err : g_err) = e.what();
    return PUCFEM_EINVAL;
  }
}

// const char* overload first: a check inside a hot loop must not build a std::string per call
inline void require(bool ok, const char* msg) {
  if (!ok) throw Error(PUCFEM_EINVAL, msg);
}
inline void require(bool ok, const std::string& msg) {
  if (!ok) throw Error(PUCFEM_EINVAL, msg);
}

// ------------------------------------------------------------------ multigrid hierarchy (host)
// min(Gershgorin bound, 1.1 x 30-step power iteration) of D^-1 A; rows in fixed chunks (threads),
// the norms summed per chunk and then in chunk order: the same value on every machine.  power = false:
// the Gershgorin bound only, with D^-1 in *dinv_out (the finest level's power iteration then runs on
// the device, Ctx::lmax_device)
double lmax_estimate(const Csr& A, bool power = true, std::vector<double>* dinv_out = nullptr,
                     double* lam_out = nullptr) {
  const i64 n = A.nrows;
  std::vector<double> dinv(n), x(power ? n : 0), y(power ? n : 0);
  std::vector<double> cg(PAR_CHUNKS, 0.0), cx(PAR_CHUNKS), cy(PAR_CHUNKS);
  parallel_chunks(n, [&](int ch, i64 r0, i64 r1) {
    for (i64 r = r0; r < r1; ++r) {
      double d = 1.0, s = 0.0;
      for (i64 k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k) {
        if (A.col[k] == r) d = A.val[k];
        s += std::fabs(A.val[k]);
      }
      dinv[r] = 1.0 / d;
      cg[ch] = std::max(cg[ch], s / d);
    }
  });
  double gersh = 0.0;
  for (double g : cg) gersh = std::max(gersh, g);
  if (!power) {
    if (dinv_out) dinv_out->swap(dinv);
    return gersh;
  }
  parallel_for(n, [&](i64 i0, i64 i1) {
    for (i64 i = i0; i < i1; ++i) x[i] = 1.0 + 0.5 * std::sin((double)i);
  });
  double lam = 0.0;
  for (int it = 0; it < 30; ++it) {
    parallel_chunks(n, [&](int ch, i64 r0, i64 r1) {
      double nx = 0.0, ny = 0.0;
      for (i64 r = r0; r < r1; ++r) {
        double a = 0.0;
        for (i64 k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k) a += A.val[k] * x[A.col[k]];
        y[r] = dinv[r] * a;
        nx += x[r] * x[r];
        ny += y[r] * y[r];
      }
      cx[ch] = nx;
      cy[ch] = ny;
    });
    double nx = 0.0, ny = 0.0;
    for (int ch = 0; ch < PAR_CHUNKS; ++ch) {
      nx += cx[ch];
      ny += cy[ch];
    }
    lam = std::sqrt(ny / nx);
    const double inv = 1.0 / std::sqrt(ny);
    parallel_for(n, [&](i64 r0, i64 r1) {
      for (i64 r = r0; r < r1; ++r) x[r] = y[r] * inv;
    });
  }
  if (lam_out) *lam_out = lam;
  return std::min(gersh, 1.1 * lam);
}

// wall time per setup phase on stderr (PUCFEM_SETUP_TIMING=1)
struct SetupClock {
  bool on = std::getenv("PUCFEM_SETUP_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[setup] %-34s %8.3f s\n", what, std::chrono::duration<double>(n - t).count());
    t = n;
  }
};

void assemble_device(Ctx& c, const HostMesh& m, const Ordering& ord, Csr& P, Assembly& A);

// the red refinements of the hierarchy (host only: levels' meshes and their midpoint parents); build()
// runs it on a thread beside the finest level's assembly and pressure merge, which do not touch c.mg
void mg_refine(Ctx& c) {
  const int Lv = c.mg_levels;
  c.mg[0].mesh = c.coarse;
  for (int l = 1; l <= Lv; ++l) {
    HostMesh tmp;
    red_refine(c.mg[l - 1].mesh, tmp, &c.mg[l].ea, &c.mg[l].eb);
    if (l < Lv) {
      c.mg[l].mesh = std::move(tmp);
    } else {
      require(tmp.N == c.mesh.N && tmp.T == c.mesh.T && tmp.x == c.mesh.x && tmp.y == c.mesh.y &&
                  tmp.tri == c.mesh.tri,
              "the uploaded mesh is not the red refinement of the hierarchy's coarse mesh");
    }
  }
}
double diag_of(const Csr& A, const std::vector<double>& val, i64 g);
// the dense pseudo-inverse of a coarse level's merged operator, constants regularised on the free dofs
static std::vector<double> dense_coarse_inverse(const MgLevel& L0) {
  const i64 n0 = L0.mesh.N;
  require(n0 <= 8192, "multigrid coarse level too large for the dense coarse solve (<= 8192 nodes)");
  std::vector<double> D(n0 * n0, 0.0);
  const Csr& A = L0.Pp;
  double dsum = 0.0;
  i64 nf = 0;
  for (i64 r = 0; r < n0; ++r) {
    for (i64 k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k) D[r * n0 + A.col[k]] += A.val[k];
    if (L0.master_of[r] < 0) {
      dsum += diag_of(A, A.val, r);
      ++nf;
    }
  }
  const double cc = dsum / (double)nf / (double)nf;
  for (i64 i = 0; i < n0; ++i)
    if (L0.master_of[i] < 0)
      for (i64 j = 0; j < n0; ++j)
        if (L0.master_of[j] < 0) D[i * n0 + j] += cc;
  require(spd_inverse(D, n0), "coarse operator is not SPD after regularisation");
  return D;
}

void build_mg_host(Ctx& c, SetupClock& clk) {  // (after mg_refine)
  const int Lv = c.mg_levels;
  for (int l = 0; l < Lv; ++l) {
    MgLevel& L = c.mg[l];
    if (c.lattice) lattice_ordering(L.mesh, c.macro, l, L.ord, L.latl);
    else make_ordering_cuts(L.mesh, c.ord.cuts, L.ord);
    Assembly A;
    if (c.dev_asm()) {
      assemble_device(c, L.mesh, L.ord, L.P, A);
    } else {
      Incidence inc;
      build_incidence(L.mesh, L.ord, inc);
      build_pattern(L.mesh, L.ord, L.P, &inc);
      assemble_stokes(L.mesh, L.ord, L.P, A, &inc);
    }
    L.pairs = level_pairs(L.mesh, 1.0, 1e-6, 1.0);
    const i64 n = L.mesh.N;
    L.dof.resize(n);
    for (i64 i = 0; i < n; ++i) L.dof[i] = (i32)i;
    L.master_of.assign(n, -1);
    L.slave_of.assign(n, -1);
    for (auto& pr : L.pairs) {
      const i32 mi = L.ord.old2new[pr.first], si = L.ord.old2new[pr.second];
      require(L.master_of[si] < 0 && L.dof[mi] == mi && L.slave_of[si] < 0, "multigrid level has chained pairs");
      L.dof[si] = mi;
      L.master_of[si] = mi;
      L.slave_of[mi] = si;
    }
    build_pressure(L.P, A.K, L.dof, L.slave_of, L.Pp);
    L.P = Csr();  // only the merged operator is needed on coarse levels
  }
  clk.mark("  mg: coarse level operators");
  // the level of the dense coarse solve; level 1's inverse (~3.6k rows: ~1.5 s of host work) runs beside the rest of
  // setup from here
  c.mg_dense_l = 0;
  if (const char* e = std::getenv("PUCFEM_MG_DENSE_LEVEL"))
    c.mg_dense_l = std::max(0, std::min(std::min(1, Lv - 1), std::atoi(e)));
  if (c.mg_dense_l > 0)
    c.dense_fut = std::async(std::launch::async, [&c] { return dense_coarse_inverse(c.mg[c.mg_dense_l]); });
  MgLevel& F = c.mg[Lv];
  F.ord = c.ord;
  if (c.lattice) F.latl = std::move(c.lat_fine);
  F.dof = c.dof;
  F.master_of = c.master_of;
  // the transfers of every level (serial builders, one thread per level) and the lmax estimates (each
  // parallel inside) read only what the level operators above produced: they run concurrently
  // the finest level's power iteration runs on the device at the end of build() (every rank its strip:
  // halos before the products, the two norms all-reduced)
  // PUCFEM_LMAX_HOST=1 (measurement knob): every level's power iteration on the host's fp64 operator
  c.lmax_dev = !c.host_only && !(std::getenv("PUCFEM_LMAX_HOST") && std::atoi(std::getenv("PUCFEM_LMAX_HOST")));
  {
    ThreadGroup g;  // joined on every exit path; a level's exception reaches the caller from join()
    for (int l = 1; l <= Lv; ++l)
      g.spawn([&c, l] {
        MgLevel& L = c.mg[l];
        const MgLevel& C = c.mg[l - 1];
        build_prolongation(C.mesh.N, L.ea, L.eb, L.ord, C.ord, C.dof, L.master_of, L.Pr);
        transpose(L.Pr, C.mesh.N, L.R);
      });
    std::exception_ptr e0;
    try {
      for (int l = 0; l <= Lv; ++l)  // (device power iterations: the Gershgorin bound here, the rest in build())
        c.mg[l].lmax = l == Lv && c.lmax_dev ? lmax_estimate(c.Pp, false, &c.lmax_dinv)
                                             : lmax_estimate(l == Lv ? c.Pp : c.mg[l].Pp, !(c.lmax_dev && l >= 1));
    } catch (...) {
      e0 = std::current_exception();
    }
    clk.mark("  mg: lmax estimates (host)");
    g.join();
    if (e0) std::rethrow_exception(e0);
  }
  clk.mark("  mg: transfers (joined)");
}

// ------------------------------------------------------------------ operator build
double diag_of(const Csr& A, const std::vector<double>& val, i64 g) {
  for (i64 k = A.rowptr[g]; k < A.rowptr[g + 1]; ++k)
    if (A.col[k] == g) return val[k];
  return 1.0;
}

// binary SELL image: int64 nslices, nrows, padded; int64 slice_off[nslices+1]; int32 slice_w[nslices];
// int32 col[padded]; double val[padded]
void dump_sell(const char* path, const Sell& S, const std::vector<double>& val) {
  FILE* f = std::fopen(path, "wb");
  require(f != nullptr, std::string("cannot write ") + path);
  const int64_t h[3] = {S.nslices, S.nrows, S.padded};
  std::fwrite(h, sizeof(h), 1, f);
  std::fwrite(S.slice_off.data(), sizeof(int64_t), S.slice_off.size(), f);
  std::fwrite(S.slice_w.data(), sizeof(int32_t), S.slice_w.size(), f);
  std::fwrite(S.col.data(), sizeof(int32_t), S.col.size(), f);
  std::fwrite(val.data(), sizeof(double), val.size(), f);
  std::fclose(f);
}

// fp16 image of operator values for the fp32 V-cycle: null when disabled (prm.mg_f32_vals 1: every
// level, 2: the finest level) or when some value is not a finite fp16 (|v| >= 65504)
_Float16* upload_f16(Ctx& c, const std::vector<double>& v, bool finest) {
  if (c.prm.mg_f32_vals == 1 || (c.prm.mg_f32_vals == 2 && finest)) return nullptr;
  std::vector<_Float16> h(v.size());
  for (size_t k = 0; k < v.size(); ++k) {
    if (!(std::fabs(v[k]) < 65504.0)) return nullptr;
    h[k] = (_Float16)v[k];
  }
  return c.upload(h);
}

template <typename T>
T* upload_as(Ctx& c, const std::vector<double>& v) {
  if constexpr (std::is_same<T, double>::value) {
    return c.upload(v);
  } else {
    std::vector<T> w(v.begin(), v.end());
    return c.upload(w);
  }
}

// ------------------------------------------------------------------ device assembly
// Scratch device buffer of one setup phase (freed on scope exit, not kept with the context).
template <class T>
struct DevTmp {
  T* p = nullptr;
  explicit DevTmp(i64 n, hipStream_t st) {
    HIPCHK(hipMalloc(&p, sizeof(T) * (size_t)std::max<i64>(1, n)));
    HIPCHK(hipMemsetAsync(p, 0, sizeof(T) * (size_t)std::max<i64>(1, n), st));
  }
  DevTmp(const std::vector<T>& v, hipStream_t st) : DevTmp((i64)v.size(), st) {
    if (!v.empty()) HIPCHK(hipMemcpyAsync(p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, st));
  }
  ~DevTmp() { (void)hipFree(p); }
  DevTmp(const DevTmp&) = delete;
  DevTmp& operator=(const DevTmp&) = delete;
  void get(std::vector<T>& v, i64 n, hipStream_t st) const {
    v.resize((size_t)n);
    if (n > 0) HIPCHK(hipMemcpyAsync(v.data(), p, sizeof(T) * (size_t)n, hipMemcpyDeviceToHost, st));
  }
  // through the context's pinned staging buffers (returns with the data on the host)
  void get(std::vector<T>& v, i64 n, Ctx& c) const {
    host_alloc_fresh(v, (size_t)n);
    if (n > 0) c.d2h(v.data(), p, sizeof(T) * (size_t)n);
  }
};

// The stiffness pattern P and the K / Gx / Gy / lumped-mass / area-sum values of a mesh assembled on the
// device (pucfem_kernels_impl.hpp k_inc_* / k_pat_* / k_asm): the same arrays pucfem_host.cpp's
// build_incidence + build_pattern + assemble_stokes produce, bit for bit (tests/test_gpu_assembly.py).
// Only the two prefix sums (row counts -> offsets) run on the host.
void assemble_device(Ctx& c, const HostMesh& m, const Ordering& ord, Csr& P, Assembly& A) {
  hipStream_t st = c.st;
  const i64 N = m.N, T = m.T;
  SetupClock ck;  // (PUCFEM_SETUP_TIMING: the phases inside)
  const int nb = (int)std::min<i64>(16384, std::max<i64>(1, (3 * T + BS - 1) / BS));
  const int nbr = (int)std::min<i64>(16384, std::max<i64>(1, (N + BS - 1) / BS));
  DevTmp<i32> dtri(m.tri, st), dold2new(ord.old2new, st);
  DevTmp<double> dx(m.x, st), dy(m.y, st);
  if (ck.on) {
    HIPCHK(hipStreamSynchronize(st));
    ck.mark("  asm: mesh upload");
  }
  // incidence
  DevTmp<i32> cnt(N, st);
  hipLaunchKernelGGL(k_inc_count, dim3(nb), dim3(BS), 0, st, 3 * T, (const i32*)dtri.p, (const i32*)dold2new.p, cnt.p);
  KCHK();
  std::vector<i32> hc;
  cnt.get(hc, N, st);
  HIPCHK(hipStreamSynchronize(st));
  std::vector<i64> ptr(N + 1, 0);
  for (i64 i = 0; i < N; ++i) ptr[i + 1] = ptr[i] + hc[i];
  DevTmp<i64> dptr(ptr, st);
  DevTmp<i32> cur(N, st), itri(ptr[N], st), err(1, st);
  hipLaunchKernelGGL(k_inc_fill, dim3(nb), dim3(BS), 0, st, 3 * T, (const i32*)dtri.p, (const i32*)dold2new.p,
                     (const i64*)dptr.p, cur.p, itri.p);
  KCHK();
  hipLaunchKernelGGL(k_inc_sort, dim3(nbr), dim3(BS), 0, st, N, (const i64*)dptr.p, itri.p, err.p);
  KCHK();
  // pattern
  hipLaunchKernelGGL(k_pat_count, dim3(nbr), dim3(BS), 0, st, N, (const i64*)dptr.p, (const i32*)itri.p,
                     (const i32*)dtri.p, (const i32*)dold2new.p, cnt.p);
  KCHK();
  int herr = 0;
  HIPCHK(hipMemcpyAsync(&herr, err.p, sizeof(int), hipMemcpyDeviceToHost, st));
  cnt.get(hc, N, st);
  HIPCHK(hipStreamSynchronize(st));
  require(herr == 0, "device assembly: a node has more than 32 incident triangles (use assembly = 1)");
  P.nrows = N;
  P.rowptr.assign(N + 1, 0);
  for (i64 i = 0; i < N; ++i) P.rowptr[i + 1] = P.rowptr[i] + hc[i];
  const i64 nnz = P.rowptr[N];
  DevTmp<i64> drow(P.rowptr, st);
  DevTmp<i32> dcol(nnz, st);
  hipLaunchKernelGGL(k_pat_fill, dim3(nbr), dim3(BS), 0, st, N, (const i64*)dptr.p, (const i32*)itri.p,
                     (const i32*)dtri.p, (const i32*)dold2new.p, (const i64*)drow.p, dcol.p);
  KCHK();
  // values
  DevTmp<double> K(nnz, st), Gx(nnz, st), Gy(nnz, st), M(N, st), as(N, st);
  hipLaunchKernelGGL(k_asm, dim3(nbr), dim3(BS), 0, st, N, (const i64*)dptr.p, (const i32*)itri.p, (const i32*)dtri.p,
                     (const i32*)dold2new.p, (const double*)dx.p, (const double*)dy.p, (const i64*)drow.p,
                     (const i32*)dcol.p, K.p, Gx.p, Gy.p, M.p, as.p);
  KCHK();
  if (ck.on) {
    HIPCHK(hipStreamSynchronize(st));
    ck.mark("  asm: incidence, pattern, values (device)");
  }
  dcol.get(P.col, nnz, c);
  P.val.clear();
  K.get(A.K, nnz, c);
  Gx.get(A.Gx, nnz, c);
  Gy.get(A.Gy, nnz, c);
  M.get(A.M, N, c);
  as.get(A.asum, N, c);
  HIPCHK(hipStreamSynchronize(st));
  ck.mark("  asm: downloads");
}

// device values and work vectors of every multigrid level in the V-cycle's type T.
// kp_vals: the finest operator's SELL values (fp64, = dKp_raw), reused for fp64 cycles.
template <typename T>
void mg_alloc(Ctx& c, const std::vector<double>& kp_vals) {
  const int Lv = c.mg_levels;
  std::vector<double> tmp;
  for (int l = 0; l <= Lv; ++l) {
    MgLevel& L = c.mg[l];
    MgBufs<T>& B = bufs<T>(L);
    const Csr& A = l == Lv ? c.Pp : L.Pp;
    const i64 n = L.lp.n_own;
    L.nloc = n + L.lp.n_ghost;
    // 1 / diag on owned AND ghost rows (the fused first smoothing step evaluates x1 = c Dinv b at
    // gathered columns)
    std::vector<double> dv(L.nloc);
    const i64 r0 = L.own0(c.rank);
    parallel_for(n, [&](i64 i0, i64 i1) {
      for (i64 i = i0; i < i1; ++i) dv[i] = 1.0 / diag_of(A, A.val, r0 + i);
    });
    for (i64 k = 0; k < L.lp.n_ghost; ++k) dv[n + k] = 1.0 / diag_of(A, A.val, L.lp.ghost_global[k]);
    if (L.deep && c.lattice && L.latl.F > 0 && !L.flook.starts.empty()) {
      // deep halos: every face-interior row's 1 / diag is its face record's (the face kernels' value), so the ghost
      // rows' steps repeat the owners' arithmetic (face_ghost_rows)
      for (size_t q = 0; q < L.lf_faces.size(); ++q) {
        const double di = L.lf_coef[q * lat::NCOEF + lat::C_DINV];
        const i64 b0 = L.latl.face_start[L.lf_faces[q]] - r0;
        for (i64 t = 0; t < L.latl.F; ++t) dv[b0 + t] = di;
      }
      for (i64 k = 0; k < L.lp.n_ghost; ++k) {
        const i32 g = L.lp.ghost_global[k];
        if (L.latl.type[g] == 0) dv[n + k] = face_dinv(c.macro, L.latl, L.flook, l, g);
      }
    }
    B.dinv = upload_as<T>(c, dv);
    if (l < Lv) {
      const Sell& S = L.sA;
      sell_values_x(A, r0, S, A.val, tmp);
      L.dA = DevSell{c.upload(S.slice_off), c.upload(S.slice_w), c.upload(S.col), nullptr, S.nslices, S.nrows,
                     S.rows.empty() ? A.rowptr[r0 + n] - A.rowptr[r0] : S.nnz, S.padded, 0};
      if (!S.rows.empty()) L.dA.rows = c.upload(S.rows);
      L.dA.n_own = n;
      L.dA.ghost_slices(S);
      c.attach_c16(S, L.nloc, L.dA);
      B.Aval = upload_as<T>(c, tmp);
      if constexpr (std::is_same<T, float>::value) B.Aval16 = upload_f16(c, tmp, false);
      L.nsend = (i64)L.lp.send_local.size();
      L.dsend = c.upload(L.lp.send_local);
      B.sendbuf = c.dalloc<T>(std::max<i64>(1, 2 * L.nsend));  // (two vectors per exchange: x and d)
    } else {
      if constexpr (std::is_same<T, double>::value) {
        B.Aval = c.dKp_raw;
      } else {
        B.Aval = upload_as<T>(c, kp_vals);
        B.Aval16 = upload_f16(c, kp_vals, true);
      }
      B.sendbuf = c.dalloc<T>(std::max<i64>(1, 2 * (i64)c.lp.send_local.size()));
    }
    if (l >= 1) {
      const Sell& S = L.sPr;
      sell_values_x(L.Pr, r0, S, L.Pr.val, tmp);
      L.dPr = DevSell{c.upload(S.slice_off), c.upload(S.slice_w), c.upload(S.col), nullptr, S.nslices, S.nrows,
                      S.rows.empty() ? L.Pr.rowptr[r0 + n] - L.Pr.rowptr[r0] : S.nnz, S.padded};
      if (!S.rows.empty()) L.dPr.rows = c.upload(S.rows);
      L.dPr.n_own = n;
      L.dPr.ghost_slices(S);
      B.Prval = upload_as<T>(c, tmp);
      const Sell& R = L.sR;
      sell_values_x(L.R, L.r_r0, R, L.R.val, tmp);
      L.dR = DevSell{c.upload(R.slice_off), c.upload(R.slice_w), c.upload(R.col), nullptr, R.nslices, R.nrows,
                     R.rows.empty() ? L.R.rowptr[L.r_r0 + R.nrows] - L.R.rowptr[L.r_r0] : R.nnz, R.padded};
      if (!R.rows.empty()) L.dR.rows = c.upload(R.rows);
      B.Rval = upload_as<T>(c, tmp);
    }
    for (T** f : {&B.x, &B.x2, &B.b, &B.d, &B.res}) *f = c.dalloc<T>(L.nloc);
  }
}


// Host half of the semi-Lagrangian / replica setup (build): node and triangle tables in internal
// numbering, the centroid grid, the lattice locator's tables, the initial dye.  It reads only the mesh,
// the ordering, the macro mesh and the finest lattice level, which nothing writes after the multigrid
// hierarchy exists, so build() runs it on a thread beside the operator uploads and SELL fills
// (round 4: ~1.3 s of L7 setup off the critical path); the uploads and kernels stay on the caller.
struct SlPrep {
  std::vector<double> X, Y, cx, cy, xy, c0;
  std::vector<i32> tri, home;
  Grid G, TG, MG;
  std::vector<lat::SlFace> sf;
  std::vector<uint32_t> cells;
  bool lat_sl = false;
};
void sl_prep(const Ctx& c, bool food, SlPrep& P) {
  SetupClock ck;  // (its own thread: the marks interleave with build()'s)
  const HostMesh& m = c.mesh;
  const i64 N = m.N;
  host_alloc_fresh(P.X, N);
  host_alloc_fresh(P.Y, N);
  parallel_for(N, [&](i64 g0, i64 g1) {
    for (i64 g = g0; g < g1; ++g) {
      P.X[g] = m.x[c.ord.new2old[g]];
      P.Y[g] = m.y[c.ord.new2old[g]];
    }
  });
  host_alloc_fresh(P.tri, 3 * m.T);
  parallel_for(3 * m.T, [&](i64 k0, i64 k1) {
    for (i64 k = k0; k < k1; ++k) P.tri[k] = c.ord.old2new[m.tri[k]];
  });
  // PointLocator centroids (StokesColor.py:321): (x1 + x2 + x3) / 3
  host_alloc_fresh(P.cx, m.T);
  host_alloc_fresh(P.cy, m.T);
  parallel_for(m.T, [&](i64 t0, i64 t1) {
    for (i64 t = t0; t < t1; ++t) {
      const i32 a = m.tri[3 * t], b = m.tri[3 * t + 1], d = m.tri[3 * t + 2];
      P.cx[t] = (m.x[a] + m.x[b] + m.x[d]) / 3;
      P.cy[t] = (m.y[a] + m.y[b] + m.y[d]) / 3;
    }
  });
  ck.mark("  sl: node / triangle tables, centroids");
  build_centroid_grid(P.cx, P.cy, 2.0, P.G);
  ck.mark("  sl: centroid grid");
  if (food) build_tri_grid(P.X, P.Y, P.tri, 4.0, P.TG);  // tracer location (StokesFood only)
  host_alloc_fresh(P.xy, 2 * (size_t)N);
  parallel_for(N, [&](i64 i0, i64 i1) {
    for (i64 i = i0; i < i1; ++i) {
      P.xy[2 * i] = P.X[i];
      P.xy[2 * i + 1] = P.Y[i];
    }
  });
  // semi-Lagrangian point location: on a lattice hierarchy the lattice locator (no per-triangle
  // records); PUCFEM_SL_RECORDS=1 forces the record locator (measurement / cross-check knob)
  P.lat_sl = c.lattice && !c.mg.empty() && !(std::getenv("PUCFEM_SL_RECORDS") && std::atoi(std::getenv("PUCFEM_SL_RECORDS")));
  if (P.lat_sl) {
    try {
      lattice_locator(c.macro, c.mg.back().latl, m, c.ord, P.sf, P.cells);
    } catch (const std::exception&) {
      P.lat_sl = false;  // a hierarchy not numbered face by face: the record locator
    }
  }
  ck.mark("  sl: xy, lattice locator");
  if (P.lat_sl) {
    build_tri_grid(c.macro.x, c.macro.y, c.macro.tri, 0.25, P.MG, 1e-6);
    // home faces: the macro face of every face-interior row (the first face tried)
    const LatticeLevel& LL = c.mg.back().latl;
    host_alloc_fresh(P.home, N);
    std::fill(P.home.begin(), P.home.end(), -1);
    parallel_for(c.macro.nf, [&](i64 f0, i64 f1) {
      for (i64 f = f0; f < f1; ++f)
        for (i64 k = 0; k < LL.F; ++k) P.home[LL.face_start[f] + k] = (i32)f;
    }, 1);
  }
  // initial dye c = 1[x < 0.5] (StokesColor.py:493-495)
  host_alloc_fresh(P.c0, N);
  parallel_for(N, [&](i64 g0, i64 g1) {
    for (i64 g = g0; g < g1; ++g) P.c0[g] = m.x[c.ord.new2old[g]] < 0.5 ? 1.0 : 0.0;
  });
  ck.mark("  sl: home faces, initial dye");
}

// Deep halos: a ghost row one layer out that is a macro-face interior node goes into the SELL as its face stencil --
// the node, then its six neighbours in lat::neighbours' order (the merged table's: slave columns are their masters),
// with the face record's coefficients -- so that a launch computing it does the owner's face-kernel arithmetic bit
// for bit (the stored row would sum the same terms in column order, and the assembled values agree with the
// records only to rounding); its 1 / diag is the record's too (face_dinv, mg_alloc).  This is what lets a rank use
// the ghost rows' results in place of exchanged values where the outer PCG needs one vector (z).
void build(Ctx& c) {
  SetupClock clk;
  require(c.has_mesh, "mesh not uploaded");
  const pucfem_params& prm = c.prm;
  c.scheme = prm.scheme;
  require(prm.scheme >= 0 && prm.scheme <= 3, "bad scheme");
  const bool stokes = prm.scheme == PUCFEM_STOKES_COLOR || prm.scheme == PUCFEM_STOKES_FOOD;
  const bool literal = !stokes;
  require(!(literal && c.dist()), "heat / Poisson literal operators run on one rank");
  require(!stokes || prm.sl_k == KNN, "sl_k must be 10 (PointLocator.find default)");
  HostMesh& m = c.mesh;
  // PUCFEM_PLAN_EMULATE="rank,world" (diagnostic, host-only contexts): build rank `rank`'s plans and deep-halo
  // flags of a `world`-rank run on the host (no communicator: nothing steps); with PUCFEM_DEEP_REPORT=1 the flags'
  // checks are reported
  if (const char* e = std::getenv("PUCFEM_PLAN_EMULATE")) {
    if (c.host_only && !c.dist()) {
      int r = 0, w = 1;
      if (std::sscanf(e, "%d,%d", &r, &w) == 2 && w > 1 && r >= 0 && r < w) {
        c.rank = r;
        c.world = w;
      }
    }
  }
  // lattice operators: a multigrid hierarchy of >= 2 red refinements (face interiors exist)
  c.lattice = stokes && prm.precond == 1 && c.mg_levels >= 2 && prm.assembled == 0;
  c.dye_impl = prm.scheme == PUCFEM_STOKES_COLOR && prm.dye_scheme == 1;
  require(prm.dye_scheme == 0 || prm.dye_scheme == 1, "dye_scheme must be 0 (semi-Lagrangian) or 1 (implicit)");
  require(!c.dye_impl || !c.dist(), "the implicit dye variant runs on one rank");
  if (c.lattice) {
    build_macro(c.coarse, prm.nstrips, c.mg_levels, c.macro);
    lattice_ordering(m, c.macro, c.mg_levels, c.ord, c.lat_fine);
  } else {
    make_ordering(m, prm.nstrips, c.ord);
  }
  clk.mark("ordering");
  // the multigrid hierarchy's refinements on a thread beside the finest assembly and pressure merge
  ThreadGroup refg;
  if (stokes && prm.precond == 1 && c.mg_levels > 0) {
    c.mg.clear();
    c.mg.resize(c.mg_levels + 1);
    refg.spawn([&c] { mg_refine(c); });
  }
  if (c.dev_asm()) {
    assemble_device(c, m, c.ord, c.P, c.as);
    clk.mark("pattern + assembly (device)");
  } else {
    Incidence inc;
    build_incidence(m, c.ord, inc);
    build_pattern(m, c.ord, c.P, &inc);
    clk.mark("pattern");
    assemble_stokes(m, c.ord, c.P, c.as, &inc);
  }
  const i64 N = m.N;

  // periodic pressure merge maps (internal numbering)
  c.dof.resize(N);
  for (i64 i = 0; i < N; ++i) c.dof[i] = (i32)i;
  c.slave_of.assign(N, -1);
  c.master_of.assign(N, -1);
  if (stokes) {
    for (auto& pr : c.op_pairs) {
      const i32 mi = c.ord.old2new[pr.first], si = c.ord.old2new[pr.second];
      require(c.master_of[si] < 0, "duplicate periodic slave: the pressure restatement needs unique slaves");
      require(c.dof[mi] == mi && c.slave_of[si] < 0, "chained periodic pairs are not supported for Stokes");
      c.dof[si] = mi;
      c.master_of[si] = mi;
      c.slave_of[mi] = si;
    }
    c.n_free = N - (i64)c.op_pairs.size();
    build_pressure(c.P, c.as.K, c.dof, c.slave_of, c.Pp);
    if (c.dye_impl) build_dye(m, c.ord, c.P, c.Pp, c.dof, c.dyeop);
  }
  c.use_mg = stokes && prm.precond == 1 && c.mg_levels > 0;
  clk.mark("assembly + pressure merge");
  refg.join();
  clk.mark("  mg: refinements (joined)");
  if (c.use_mg) build_mg_host(c, clk);
  if (literal) {
    assemble_literal(m, c.ord, c.g_tri, c.op_pairs, c.dir_nodes, c.dir_vals,
                     prm.scheme == PUCFEM_HEAT ? prm.dt : -1.0, c.Lit, c.litb);
  }
  clk.mark("multigrid hierarchy (host)");
  // the semi-Lagrangian tables' host half, beside everything up to the SL uploads below
  SlPrep slp;
  ThreadGroup slg;
  if (stokes) slg.spawn([&c, &slp, &prm] { sl_prep(c, prm.scheme == PUCFEM_STOKES_FOOD, slp); });
  // A_visc on P (StokesColor.py:471-475)
  std::vector<uint8_t> isdir(N, 0);
  for (i32 d : c.dir_nodes) isdir[c.ord.old2new[d]] = 1;
  const double dtnu = prm.dt * prm.nu;
  host_alloc_fresh(c.Kv, c.P.nnz());
  parallel_for(N, [&](i64 r0, i64 r1) {
    for (i64 r = r0; r < r1; ++r)
      for (i64 k = c.P.rowptr[r]; k < c.P.rowptr[r + 1]; ++k) {
        const i32 j = c.P.col[k];
        if (isdir[r]) c.Kv[k] = (j == r) ? 1.0 : 0.0;
        else if (isdir[j]) c.Kv[k] = 0.0;
        else c.Kv[k] = (j == r) ? 1.0 + dtnu * c.as.K[k] : dtnu * c.as.K[k];
      }
  });
  if (stokes) {  // spectral interval of the Jacobi-scaled A_visc (Ctx::visc_R, Ctx::visc_lo)
    std::vector<double> dg;
    host_alloc_fresh(dg, N);
    parallel_for(N, [&](i64 r0, i64 r1) {
      for (i64 r = r0; r < r1; ++r) dg[r] = diag_of(c.P, c.Kv, r);
    });
    std::vector<double> cr(PAR_CHUNKS, 0.0), cd(PAR_CHUNKS, 0.0);
    parallel_chunks(N, [&](int ch, i64 r0, i64 r1) {
      double R = 0.0, dmax = 0.0;
      for (i64 r = r0; r < r1; ++r) {
        double sr = 0.0;
        for (i64 k = c.P.rowptr[r]; k < c.P.rowptr[r + 1]; ++k)
          if (c.P.col[k] != r) sr += std::fabs(c.Kv[k]) / std::sqrt(dg[r] * dg[c.P.col[k]]);
        R = std::max(R, sr);
        dmax = std::max(dmax, dg[r]);
      }
      cr[ch] = R;
      cd[ch] = dmax;
    });
    c.visc_R = *std::max_element(cr.begin(), cr.end());
    // A_visc = I + DT nu K on the free rows (K PSD), identity on the Dirichlet rows: its eigenvalues are
    // >= 1, so the scaled x^T S A S x >= |S x|^2 >= |x|^2 / max_i a_ii (a rigorous lower end, tighter
    // than Gershgorin's 1 - R)
    c.visc_lo = std::max(1.0 - c.visc_R, 1.0 / *std::max_element(cd.begin(), cd.end()));
    if (const char* e = std::getenv("PUCFEM_VISC_SOLVER")) c.visc_solver = std::atoi(e);  // 1: CG (measurement)
    // test knob: a deliberately wrong (too short) interval [visc_lo, 1 + s R], for the post-check's test
    if (const char* e = std::getenv("PUCFEM_VISC_R_SCALE")) c.visc_R *= std::atof(e);
  }
  clk.mark("A_visc");
  // partition + local plan
  if (stokes) partition_rows(c.P, c.ord, c.world, c.row_start);
  else c.row_start = {0, N};
  std::vector<const Csr*> pats;
  if (stokes) pats = {&c.P, &c.Pp};
  else pats = {&c.P, &c.Lit};
  if (!c.use_mg) {
    make_local_plan(pats, c.row_start, c.rank, c.lp);
  } else {
    // every level cut at the same strips (y-cuts) as the finest partition
    const int Lv = c.mg_levels;
    std::vector<i64> cut(c.world + 1);
    for (int r = 0; r <= c.world; ++r)
      cut[r] = std::lower_bound(c.ord.strip_ptr.begin(), c.ord.strip_ptr.end(), c.row_start[r]) - c.ord.strip_ptr.begin();
    for (int l = 0; l <= Lv; ++l) {
      MgLevel& L = c.mg[l];
      L.rs.resize(c.world + 1);
      for (int r = 0; r <= c.world; ++r) L.rs[r] = L.ord.strip_ptr[cut[r]];
    }
    // replicated coarse levels (multi-rank): level 0 always, then every level up to mg_rep_nodes
    // default 1M: at L7 L5 (894k) and below are replicated.  Counted at W = 8 (tools/comm_probe.py, r8n):
    // grouped exchanges per PCG iteration 25 -> 17, per step 264-385 -> 184-265, for each rank smoothing
    // the whole L5 (latency-bound launches either way: ~11 against ~6 us)
    const i64 rep_max = prm.mg_rep_nodes > 0 ? prm.mg_rep_nodes : 1000000;
    for (int l = 0; l < Lv; ++l) c.mg[l].rep = c.dist() && (l == 0 || c.mg[l].mesh.N <= rep_max);
    for (int l = 1; l < Lv; ++l) c.mg[l].rep = c.mg[l].rep && c.mg[l - 1].rep;
    for (int l = 0; l <= Lv; ++l) {
      MgLevel& L = c.mg[l];
      if (L.rep) {  // the whole level on every rank: a single-rank plan (no ghosts)
        const std::vector<i64> full = {0, (i64)L.mesh.N};
        make_local_plan2({{&L.Pp, &full}}, full, 0, L.lp);
        continue;
      }
      std::vector<PatRows> pr;
      pr.push_back({l == Lv ? &c.Pp : &L.Pp, &L.rs});
      if (l >= 1) pr.push_back({&L.R, &c.mg[l - 1].rs});
      if (l < Lv) pr.push_back({&c.mg[l + 1].Pr, &c.mg[l + 1].rs});
      if (l == Lv) pr.push_back({&c.P, &L.rs});
      // deep halos on the partitioned lattice levels (Ctx::deep_halo): the ghost rows one layer out of the level
      // operator (the finest level: of the pressure and the K / A_visc patterns) and their columns
      std::vector<const Csr*> deep;
      if (c.deep_halo && c.lattice && c.world > 1) {
        deep.push_back(l == Lv ? &c.Pp : &L.Pp);
        if (l == Lv) deep.push_back(&c.P);
      }
      make_local_plan2(pr, L.rs, c.rank, L.lp, deep.empty() ? nullptr : &deep, deep.empty() ? nullptr : &L.g1);
      L.deep = !deep.empty();
    }
    c.lp = c.mg[Lv].lp;
    // lattice operators: SELL rows for the skeleton (macro edge / vertex nodes) only
    auto skel = [&](const LatticeLevel& LL, i64 r0, i64 n) {
      std::vector<i32> rows;
      for (i64 i = 0; i < n; ++i)
        if (LL.type[r0 + i] != 0) rows.push_back((i32)i);
      return rows;
    };
    for (int l = 0; l <= Lv; ++l) {  // host SELL images; resolving every column validates the plans
      MgLevel& L = c.mg[l];
      const i64 o0 = L.own0(c.rank);
      if (l < Lv) {
        if (c.lattice) build_sell_rows(L.Pp, o0, skel(L.latl, o0, L.lp.n_own), L.lp, L.sA);
        else build_sell_x(L.Pp, o0, L.lp.n_own, L.lp, L.sA, true);
        if (L.deep) {
          L.flook.init(c.macro, L.latl);
          const GhostRowFn fn = face_ghost_rows(c.macro, L.latl, L.flook, &L.dof, l, prm.dt * prm.nu);
          sell_append_ghost_rows(L.Pp, L.g1, L.lp, L.sA, nullptr, c.lattice ? &fn : nullptr);
        }
      }
      if (l >= 1) {
        const MgLevel& C = c.mg[l - 1];
        if (c.lattice) build_sell_rows(L.Pr, o0, skel(L.latl, o0, L.lp.n_own), C.lp, L.sPr);
        else build_sell_x(L.Pr, o0, L.lp.n_own, C.lp, L.sPr);
        // restriction rows: the coarse level's owned rows; into a replicated level from a
        // distributed one, this rank's strip rows of it (completed by the all-gather)
        const bool gather = C.rep && !L.rep;
        L.r_r0 = gather ? C.rs[c.rank] : C.own0(c.rank);
        const i64 nr = gather ? C.rs[c.rank + 1] - C.rs[c.rank] : C.lp.n_own;
        if (c.lattice) build_sell_rows(L.R, L.r_r0, skel(C.latl, L.r_r0, nr), L.lp, L.sR);
        else build_sell_x(L.R, L.r_r0, nr, L.lp, L.sR);
      }
    }
    // deep halos: which consumers can read the ghost rows one layer out instead of an exchange (every column
    // they gather outside the rank's rows must be one of them); all-reduced over the ranks at the upload
    for (int l = 1; l <= Lv; ++l) {
      MgLevel& L = c.mg[l];
      MgLevel& C = c.mg[l - 1];
      if (!L.deep) continue;
      const i64 lo = L.own0(c.rank), hi = lo + L.lp.n_own;
      auto in_g1 = [](const std::vector<i32>& g1, i32 g) { return std::binary_search(g1.begin(), g1.end(), g); };
      // the restriction's rows (on level l - 1) gather this level's residual
      const bool gather = C.rep && !L.rep;
      const i64 nr = gather ? C.rs[c.rank + 1] - C.rs[c.rank] : C.lp.n_own;
      bool ok = true;
      for (i64 r = L.r_r0; r < L.r_r0 + nr && ok; ++r)
        for (i64 k = L.R.rowptr[r]; k < L.R.rowptr[r + 1]; ++k) {
          const i32 j = L.R.col[k];
          if ((j < lo || j >= hi) && !in_g1(L.g1, j)) {
            ok = false;
            break;
          }
        }
      L.res_deep = ok;
      // the prolongation into this level gathers level l - 1's result: its ghosts one layer out suffice
      ok = C.deep && !C.rep;
      const i64 clo = C.own0(c.rank), chi = clo + C.lp.n_own;
      for (i64 r = lo; r < hi && ok; ++r)
        for (i64 k = L.Pr.rowptr[r]; k < L.Pr.rowptr[r + 1]; ++k) {
          const i32 j = L.Pr.col[k];
          if ((j < clo || j >= chi) && !in_g1(C.g1, j)) {
            ok = false;
            break;
          }
        }
      L.xc_deep = ok;
      // ... and on this level's ghost rows too (pr_deep): their coarse columns in level l - 1's own + G1 rows, or
      // any, from a replicated level l - 1 (whose every value every rank holds)
      ok = L.xc_deep || C.rep;
      for (size_t k = 0; k < L.lp.ghost_global.size() && ok; ++k) {
        const i32 r = L.lp.ghost_global[k];
        for (i64 e = L.Pr.rowptr[r]; e < L.Pr.rowptr[r + 1]; ++e) {
          const i32 j = L.Pr.col[e];
          if (!C.rep && (j < clo || j >= chi) && !in_g1(C.g1, j)) {
            ok = false;
            break;
          }
        }
      }
      L.pr_deep = ok;
      if (std::getenv("PUCFEM_DEEP_REPORT") && c.rank == 0) {  // (diagnostic: which rows fail the prolongation check)
        i64 bad_rows = 0, bad_g1 = 0;
        i32 ex = -1, exc = -1;
        for (const i32 r : L.lp.ghost_global) {
          bool bad = false;
          for (i64 e = L.Pr.rowptr[r]; e < L.Pr.rowptr[r + 1]; ++e) {
            const i32 j = L.Pr.col[e];
            if (!C.rep && (j < clo || j >= chi) && !in_g1(C.g1, j)) {
              bad = true;
              exc = j;
            }
          }
          if (bad) {
            ++bad_rows;
            bad_g1 += in_g1(L.g1, r) ? 1 : 0;
            ex = r;
          }
        }
        std::fprintf(stderr, "[deep] level %d: res %d xc %d pr %d; ghost rows failing the prolongation check %lld "
                     "(%lld of them G1), e.g. row %d (type %d) -> coarse %d (type %d)\n", l, (int)L.res_deep,
                     (int)L.xc_deep, (int)L.pr_deep, (long long)bad_rows, (long long)bad_g1, ex,
                     ex >= 0 ? (int)L.latl.type[ex] : -1, exc, exc >= 0 ? (int)C.latl.type[exc] : -1);
      }
      if (L.pr_deep)  // the prolongation's SELL: + every ghost row of this level (rows in this level's plan)
        sell_append_ghost_rows(L.Pr, L.lp.ghost_global, C.lp, L.sPr, &L.lp);
    }
    if (c.lattice) {  // face tables and coefficient records of every level (pucfem_lattice.hpp)
      const double dtnu = prm.dt * prm.nu;
      for (int l = 0; l <= Lv; ++l) {
        MgLevel& L = c.mg[l];
        const i64 o0 = L.own0(c.rank);
        L.lf_faces = lattice_faces(c.macro, L.latl, o0, L.lp.n_own);
        lattice_tabs(c.macro, L.latl, L.lf_faces, -1, L.lp, nullptr, L.lf_plain);
        lattice_tabs(c.macro, L.latl, L.lf_faces, -1, L.lp, &L.dof, L.lf_merged);
        lattice_coefs(c.macro, L.lf_faces, l, dtnu, L.lf_coef);
        if (l >= 1) {
          MgLevel& C = c.mg[l - 1];
          lattice_tabs(c.macro, C.latl, L.lf_faces, -1, C.lp, &C.dof, L.pr_tab2);
          const bool gather = C.rep && !L.rep;
          const i64 nr = gather ? C.rs[c.rank + 1] - C.rs[c.rank] : C.lp.n_own;
          L.r_faces = lattice_faces(c.macro, C.latl, L.r_r0, nr);
          lattice_tabs(c.macro, C.latl, L.r_faces, L.r_r0, C.lp, nullptr, L.r_tab);
          lattice_tabs(c.macro, L.latl, L.r_faces, -1, L.lp, nullptr, L.r_tab2);
        }
      }
    }
  }
  if (stokes && c.dist()) {  // wide-halo tables of the dye replica (Ctx::dye_halo)
    const i64 S = (i64)c.ord.strip_ptr.size() - 1;
    c.strip_ylo.assign(S, INFINITY);
    c.strip_yhi.assign(S, -INFINITY);
    for (i64 s = 0; s < S; ++s)
      for (i64 g = c.ord.strip_ptr[s]; g < c.ord.strip_ptr[s + 1]; ++g) {
        const double y = m.y[c.ord.new2old[g]];
        c.strip_ylo[s] = std::min(c.strip_ylo[s], y);
        c.strip_yhi[s] = std::max(c.strip_yhi[s], y);
      }
    c.rank_ylo.assign(c.world, INFINITY);
    c.rank_yhi.assign(c.world, -INFINITY);
    for (int r = 0; r < c.world; ++r)
      for (i64 g = c.row_start[r]; g < c.row_start[r + 1]; ++g) {
        const double y = m.y[c.ord.new2old[g]];
        c.rank_ylo[r] = std::min(c.rank_ylo[r], y);
        c.rank_yhi[r] = std::max(c.rank_yhi[r], y);
      }
    double hy = 0.0;
    for (i64 t = 0; t < m.T; ++t) {
      const double a = m.y[m.tri[3 * t]], b = m.y[m.tri[3 * t + 1]], d = m.y[m.tri[3 * t + 2]];
      hy = std::max(hy, std::max({a, b, d}) - std::min({a, b, d}));
    }
    c.tri_hy = hy;
  }
  clk.mark("partition, plans, level tables");
  if (c.lattice) {
    const LatticeLevel& LL = c.mg.back().latl;
    std::vector<i32> rows;
    for (i64 i = 0; i < c.lp.n_own; ++i)
      if (LL.type[c.lp.r0 + i] != 0) rows.push_back((i32)i);
    build_sell_rows(c.P, c.lp.r0, rows, c.lp, c.sP);
    build_sell_rows(c.Pp, c.lp.r0, rows, c.lp, c.sPp);
    if (c.use_mg && c.mg.back().deep) {  // deep halos: the finest level's ghost rows (pressure, A_visc / K)
      MgLevel& F = c.mg.back();
      F.flook.init(c.macro, F.latl);
      const GhostRowFn fn = face_ghost_rows(c.macro, F.latl, F.flook, &F.dof, c.mg_levels, prm.dt * prm.nu);
      sell_append_ghost_rows(c.Pp, F.g1, c.lp, c.sPp, nullptr, &fn);
      sell_append_ghost_rows(c.P, F.g1, c.lp, c.sP);
    }
  } else {
    build_sell(c.P, c.lp, c.sP);
    if (stokes) build_sell(c.Pp, c.lp, c.sPp);
  }
  if (literal) build_sell(c.Lit, c.lp, c.sLit);
  c.built = true;
  // tooling hook (tools/spmv_lab.hip --real): the pressure operator's SELL image
  if (const char* path = std::getenv("PUCFEM_DUMP_SELL")) {
    if (stokes) {
      std::vector<double> v;
      sell_values(c.Pp, c.lp, c.sPp, c.Pp.val, v);
      dump_sell(path, c.sPp, v);
    }
  }
  if (clk.on) {  // slice widths of the skeleton SELLs (PUCFEM_SETUP_TIMING): > 14 runs the generic entry loop
    for (const auto* S : {&c.sP, &c.sPp}) {
      std::map<int, i64> h;
      for (i32 w : S->slice_w) ++h[w];
      std::fprintf(stderr, "[setup] SELL %s: %lld slices, widths", S == &c.sP ? "P (K, G)" : "Pp (pressure)",
                   (long long)S->nslices);
      for (auto& kv : h) std::fprintf(stderr, " %d:%lld", kv.first, (long long)kv.second);
      std::fprintf(stderr, "\n");
    }
  }
  clk.mark("SELL images");
  if (c.host_only) return;

  // ---------------------------------------------------------------- device upload
  LocalPlan& lp = c.lp;
  const i64 no = lp.n_own;
  c.nloc = no + lp.n_ghost;
  auto dsell = [&](const Sell& S, const Csr& A, DevSell& D) {
    D.off = c.upload(S.slice_off);
    D.w = c.upload(S.slice_w);
    D.col = c.upload(S.col);
    c.attach_c16(S, c.nloc, D);
    D.nslices = S.nslices;
    D.nrows = S.nrows;
    D.padded = S.padded;
    D.nnz = S.rows.empty() ? A.rowptr[lp.r1] - A.rowptr[lp.r0] : S.nnz;
    if (!S.rows.empty()) D.rows = c.upload(S.rows);
    D.n_own = lp.n_own;
    D.ghost_slices(S);
  };
  std::vector<double> tmp;
  dsell(c.sP, c.P, c.dP);
  sell_values(c.P, lp, c.sP, c.as.K, tmp);
  c.dK = c.upload(tmp);
  sell_values(c.P, lp, c.sP, c.as.Gx, tmp);
  c.dGx = c.upload(tmp);
  sell_values(c.P, lp, c.sP, c.as.Gy, tmp);
  c.dGy = c.upload(tmp);
  if (c.dye_impl) {  // implicit dye operator on the merged pattern, every row stored
    const DyeOp& D = c.dyeop;
    Sell S;
    build_sell(c.Pp, lp, S);
    dsell(S, c.Pp, c.dDye);
    const i64 nnzp = c.Pp.nnz();
    std::vector<double> eid(nnzp);
    for (i64 e = 0; e < nnzp; ++e) eid[e] = (double)(e + 1);
    sell_values(c.Pp, lp, S, eid, tmp);
    std::vector<i32> slot2e(S.padded);
    for (i64 q = 0; q < S.padded; ++q) slot2e[q] = tmp[q] > 0.0 ? (i32)(tmp[q] - 1.0) : -1;
    std::vector<double> mm(nnzp, 0.0);  // merged consistent mass, identity slave rows
    for (i64 e = 0; e < nnzp; ++e) {
      if (D.eptr[e] == D.eptr[e + 1]) mm[e] = 1.0;
      for (i64 z = D.eptr[e]; z < D.eptr[e + 1]; ++z) mm[e] += D.mc[D.ek[z]];
    }
    sell_values(c.Pp, lp, S, mm, tmp);
    c.dDyeM = c.upload(tmp);
    std::vector<i64> dslot(N);
    for (i64 r = 0; r < N; ++r) {
      const i64 e = c.Pp.find(r, (i32)r);
      require(e >= 0, "dye operator: a row without a diagonal");
      dslot[r] = S.slice_off[r / 64] + (e - c.Pp.rowptr[r]) * 64 + r % 64;
    }
    c.dDyeDiag = c.upload(dslot);
    c.dye = DyeDev{c.upload(slot2e), c.upload(D.eptr), c.upload(D.ek), c.upload(D.mc), c.upload(c.as.K),
                   c.upload(D.cptr), c.upload(D.cw), c.upload(D.diag_row), c.upload(c.dof), c.upload(c.as.M), S.padded};
    c.dye_nsrow = (int32_t)D.srow.size();
    if (c.dye_nsrow > 0) {
      c.dDyeSrow = c.upload(D.srow);
      c.dDyeSptr = c.upload(D.sptr);
      c.dDyeSk = c.upload(D.sk);
      c.dDyeSc = c.upload(D.sc);
    }
    c.dDyeVal = c.dalloc<double>(S.padded);
    c.dDyeW = c.dalloc<double>(3 * m.T);
    c.dDyeDinv = c.dalloc<double>(c.nloc);
    c.dDyeB = c.dalloc<double>(c.nloc);
  }
  clk.mark("device: K, G, dye operator");
  // Jacobi symmetric scaling S A S: s_g = 1 / sqrt(a_gg); the scaled values s_r a_rk s_col go straight into
  // the SELL image (only the skeleton rows on lattice hierarchies)
  auto scaling = [&](const Csr& A, const std::vector<double>& val, std::vector<double>& sg) {
    host_alloc_fresh(sg, N);
    parallel_for(N, [&](i64 g0, i64 g1) {
      for (i64 g = g0; g < g1; ++g) sg[g] = 1.0 / std::sqrt(diag_of(A, val, g));
    });
  };
  auto local_vec = [&](const std::vector<double>& g) {  // owned + ghost entries of a global vector
    std::vector<double> v;
    host_alloc_fresh(v, c.nloc);
    parallel_for(no, [&](i64 i0, i64 i1) { std::memcpy(v.data() + i0, g.data() + lp.r0 + i0, sizeof(double) * (i1 - i0)); });
    for (i64 k = 0; k < lp.n_ghost; ++k) v[no + k] = g[lp.ghost_global[k]];
    return v;
  };
  {
    std::vector<double> sg;
    scaling(c.P, c.Kv, sg);
    sell_values_fn(c.P, lp.r0, c.sP, [&](i64 r, i64 k) { return sg[r] * c.Kv[k] * sg[c.P.col[k]]; }, tmp);
    c.dKv = c.upload(tmp);
    c.dsv = c.upload(local_vec(sg));  // (k_visc_prep forms 1 / s itself)
    if (c.lattice) {  // scaled A_visc, skeleton columns: s_j, 0 for Dirichlet columns (StokesColor.py:473-475)
      std::vector<double> w = local_vec(sg);
      for (i64 i = 0; i < no; ++i)
        if (isdir[lp.r0 + i]) w[i] = 0.0;
      for (i64 k = 0; k < lp.n_ghost; ++k)
        if (isdir[lp.ghost_global[k]]) w[no + k] = 0.0;
      c.dwsk = c.upload(w);
    }
  }
  clk.mark("  dev: scaled A_visc");
  if (stokes) {
    dsell(c.sPp, c.Pp, c.dPp);
    if (!c.lattice) {  // the Jacobi-scaled pressure operator (Jacobi-CG and the SELL unit op; a lattice hierarchy
                       // always runs the multigrid PCG on the unscaled one)
      std::vector<double> sg;
      scaling(c.Pp, c.Pp.val, sg);
      sell_values_fn(c.Pp, lp.r0, c.sPp, [&](i64 r, i64 k) { return sg[r] * c.Pp.val[k] * sg[c.Pp.col[k]]; }, tmp);
      c.dKp = c.upload(tmp);
      c.dsp = c.upload(local_vec(sg));
    }
  }
  if (c.use_mg) {
    sell_values(c.Pp, lp, c.sPp, c.Pp.val, tmp);
    c.dKp_raw = c.upload(tmp);
    c.z = c.dalloc<double>(c.nloc);
    c.z32 = c.dalloc<float>(c.nloc);

    c.r32 = c.dalloc<float>(c.nloc);
    c.mg_single = c.prm.mg_single != 0;
    if (c.mg_single) mg_alloc<float>(c, tmp);
    else mg_alloc<double>(c, tmp);
    clk.mark("  dev: pressure SELL, level values");
    if (c.lattice) {  // the face parts of every lattice operator (pucfem_lattice.hpp)
      auto mkface = [&](const std::vector<lat::FaceTab>& tab, const std::vector<lat::FaceTab>* tab2, const double* coef,
                        const float* coef32, int l, int l2, int op) {
        HFace h;
        const i32 n = 1 << l, F = lat::interior_count(n);
        if (tab.empty() || F == 0) return h;
        h.d.tab = c.upload(tab);
        h.d.tab2 = tab2 ? c.upload(*tab2) : nullptr;
        h.d.coef = coef;
        h.d.coef32 = coef32;
        h.d.wsk = op == 1 ? c.dwsk : nullptr;
        h.d.nf = (int32_t)tab.size();
        h.d.n = n;
        h.d.F = F;
        h.d.cpf = (F + BS * FACE_RPT - 1) / (BS * FACE_RPT);
        h.d.n2 = l2 >= 0 ? 1 << l2 : 0;
        h.d.rinv = 1.0f / (float)(n - 1);
        h.d.nb = 0;
        h.d.op = op;
        h.items = h.d.nf * h.d.cpf;
        h.rows = (i64)h.d.nf * F;
        return h;
      };
      const int Lv = c.mg_levels;
      for (int l = 0; l <= Lv; ++l) {
        MgLevel& L = c.mg[l];
        const double* coef = c.upload(L.lf_coef);
        const float* coef32 = c.upload(std::vector<float>(L.lf_coef.begin(), L.lf_coef.end()));
        if (l < Lv) {
          L.hA = mkface(L.lf_merged, nullptr, coef, coef32, l, -1, 0);
        } else {
          c.fP = mkface(L.lf_merged, nullptr, coef, coef32, l, -1, 0);
          c.fK = mkface(L.lf_plain, nullptr, coef, coef32, l, -1, 0);
          c.fVisc = mkface(L.lf_plain, nullptr, coef, coef32, l, -1, 1);
        }
        if (l >= 1) {
          L.hPr = mkface(L.lf_plain, &L.pr_tab2, nullptr, nullptr, l, l - 1, 0);
          L.hR = mkface(L.r_tab, &L.r_tab2, nullptr, nullptr, l - 1, l, 0);
        }
      }
    }
    clk.mark("  dev: lattice face tables");
    // coarse solve: dense pseudo-inverse of the merged operator, constants regularised on the free dofs
    {
      const std::vector<double> D =
          c.dense_fut.valid() ? c.dense_fut.get() : dense_coarse_inverse(c.mg[c.mg_dense_l]);
      c.dAinv = c.upload(D);
      if (c.mg_dense_l > 0) c.dAinv32 = c.upload(std::vector<float>(D.begin(), D.end()));
    }
  }
  if (c.dist() && c.use_mg) {  // deep-halo flags: every rank takes the same exchanges (a flag off anywhere is off)
    const size_t nl = c.mg.size();
    std::vector<double> off(4 * nl);
    for (size_t l = 0; l < nl; ++l) {
      off[4 * l] = c.mg[l].deep ? 0.0 : 1.0;
      off[4 * l + 1] = c.mg[l].res_deep ? 0.0 : 1.0;
      off[4 * l + 2] = c.mg[l].xc_deep ? 0.0 : 1.0;
      off[4 * l + 3] = c.mg[l].pr_deep ? 0.0 : 1.0;
    }
    DevTmp<double> t(off, c.st);
    c.comm->allreduce(t.p, off.size(), true, c.st);
    t.get(off, off.size(), c.st);
    HIPCHK(hipStreamSynchronize(c.st));
    for (size_t l = 0; l < nl; ++l) {
      MgLevel& L = c.mg[l];
      L.deep = L.deep && off[4 * l] == 0.0;
      L.res_deep = L.deep && L.res_deep && off[4 * l + 1] == 0.0;
      L.xc_deep = l > 0 && c.mg[l - 1].deep && L.xc_deep && off[4 * l + 2] == 0.0;
      L.pr_deep = l > 0 && L.deep && (L.xc_deep || c.mg[l - 1].rep) && L.pr_deep && off[4 * l + 3] == 0.0;
      if (std::getenv("PUCFEM_DEEP_REPORT") && c.rank == 0)  // (diagnostic: tools/comm_probe.py)
        std::fprintf(stderr, "[deep] level %zu: rep %d deep %d res %d xc %d pr %d  own %lld ghosts %lld g1 %zu\n", l,
                     (int)L.rep, (int)L.deep, (int)L.res_deep, (int)L.xc_deep, (int)L.pr_deep, (long long)L.lp.n_own,
                     (long long)L.lp.n_ghost, L.g1.size());
    }
  }
  c.block_cg = c.prm.solver_path != 1;
  c.dense = stokes && !c.dist() && N <= DENSE_MAX && c.prm.precond != 1 && c.prm.solver_path != 1;
  // the small-mesh step is ~20 latency-bound launches replayed from a graph: its reductions finish inside their
  // producers (RedOut, the last block reduces) instead of a k_reduce launch after each (PUCFEM_FUSED_RED=0 keeps them)
  if (c.dense && !std::getenv("PUCFEM_FUSED_RED")) c.fused_red = true;
  clk.mark("device: A_visc, pressure, multigrid");
  // successive-RHS projections (multi-kernel CG paths only: the dense and one-workgroup solves of
  // small meshes need no better start)
  // (a basis needs room for the re-seeded span and one new direction: at least 3)
  auto proj_size = [](int k) { return k <= 0 ? 0 : std::max(3, std::min(k, (int)PROJ_MAX)); };
  c.proj_k = c.use_mg && !c.dense ? proj_size(c.prm.proj_k) : 0;
  c.proj_shared = c.prm.proj_shared != 0;
  if (const char* e = std::getenv("PUCFEM_PROJ_SHARED")) c.proj_shared = std::atoi(e) != 0;
  // pending pressure directions and the gradient on y (Ctx::p_from_y): lattice operators, the multigrid PCG
  // with the projection, the explicit dye; PUCFEM_P_FROM_Y=0 keeps the stored form (a measurement knob: the
  // same values either way).  Partitioned runs exchange y's halo instead of p's.
  c.p_from_y = stokes && c.lattice && c.use_mg && c.proj_k > 0 && !c.dye_impl && c.dP.c16 == nullptr && !c.proj_spmv &&
               !(std::getenv("PUCFEM_P_FROM_Y") && std::atoi(std::getenv("PUCFEM_P_FROM_Y")) == 0);
  if (c.p_from_y) {  // dP with every column mapped to its periodic master (the dof map), in local ids
    std::vector<i32> colm(c.sP.col.size());
    const i64 nl = (i64)c.nloc;
    bool ok = true;
    for (size_t e = 0; e < colm.size() && ok; ++e) {
      const i32 j = c.sP.col[e];
      colm[e] = j;
      if (j < 0 || j >= nl) continue;
      const i32 g = j < no ? (i32)(lp.r0 + j) : lp.ghost_global[j - no];
      const i32 mg = c.dof[g];
      if (mg == g) continue;
      if (mg >= lp.r0 && mg < lp.r1) {
        colm[e] = (i32)(mg - lp.r0);
      } else {
        auto it = std::lower_bound(lp.ghost_global.begin(), lp.ghost_global.end(), mg);
        if (it == lp.ghost_global.end() || *it != mg) ok = false;  // a master outside the local columns
        else colm[e] = (i32)(no + (it - lp.ghost_global.begin()));
      }
    }
    // every rank takes the same path: a rank whose merged columns reach outside its local columns would
    // halo p while its neighbours send y (whose slave entries are not copies of their masters)
    if (c.dist()) {
      std::vector<double> bad(1, ok ? 0.0 : 1.0);
      DevTmp<double> t(bad, c.st);
      c.comm->allreduce(t.p, 1, true, c.st);
      t.get(bad, 1, c.st);
      HIPCHK(hipStreamSynchronize(c.st));
      ok = bad[0] == 0.0;
    }
    c.p_from_y = ok;
    if (ok) {
      c.dPm = c.dP;
      c.dPm.col = c.upload(colm);
    }
  }
  const bool block_visc = !c.dist() && c.block_cg && no <= (i64)CGB_THREADS * CGB_MAXR;
  c.proj_k_visc = stokes && !c.dense && !block_visc ? proj_size(c.prm.proj_k_visc) : 0;
  c.ldx = (c.nloc + 1) & ~(i64)1;
  for (int w = 1; w <= 4; ++w) {
    const int k = w <= 2 ? c.proj_k : c.proj_k_visc;
    if (k > 0) {
      const i64 pn = PUCFEM_PROJ_TILED ? (c.nloc + 63) / 64 * 64 * k : (i64)k * c.ldx;
      c.projX[w] = c.dalloc<ProjT>(pn);
      c.proj_x0[w] = c.dalloc<double>(c.nloc);
      c.projXalt[w] = c.dalloc<ProjT>(pn);  // re-seeding target
    }
  }
  if (stokes && !c.dense && !block_visc && c.proj_k_visc == 0 && c.visc_extrap > 0)
    for (int k = 0; k < 2 * c.visc_extrap; ++k) c.dvinc[k] = c.dalloc<float>(c.nloc);
  if (c.proj_k > 0 || c.proj_k_visc > 0) {
    for (int w = 1; w <= 4; ++w)
      if (c.projX[w]) {
        c.pv[w] = c.dalloc<double>(c.nloc);
        c.pav[w] = c.dalloc<double>(c.nloc);
      }
    c.proj_part = c.dalloc<double>((i64)Ctx::NCOEF * MAXB);
    c.dqm = c.dalloc<double>((i64)sizeof(QMat) / (i64)sizeof(double));
    c.proj_d = c.dalloc<double>(Ctx::NCOEF);
    c.proj_coef = c.dalloc<double>(Ctx::NCOEF);
  }
  if (c.dense) {
    // A_visc^-1 and the pseudo-inverse of the merged pressure operator (constants on the free dofs
    // regularised, as for the multigrid coarse level)
    std::vector<double> Dv(N * N, 0.0), Dp(N * N, 0.0);
    for (i64 r = 0; r < N; ++r) {
      for (i64 k = c.P.rowptr[r]; k < c.P.rowptr[r + 1]; ++k) Dv[r * N + c.P.col[k]] = c.Kv[k];
      for (i64 k = c.Pp.rowptr[r]; k < c.Pp.rowptr[r + 1]; ++k) Dp[r * N + c.Pp.col[k]] += c.Pp.val[k];
    }
    double dsum = 0.0;
    for (i64 r = 0; r < N; ++r)
      if (c.master_of[r] < 0) dsum += Dp[r * N + r];
    const double cc = dsum / (double)c.n_free / (double)c.n_free;
    for (i64 i = 0; i < N; ++i)
      if (c.master_of[i] < 0)
        for (i64 j = 0; j < N; ++j)
          if (c.master_of[j] < 0) Dp[i * N + j] += cc;
    require(spd_inverse(Dv, N), "A_visc is not SPD");
    require(spd_inverse(Dp, N), "regularised pressure operator is not SPD");
    c.dVinv = c.upload(Dv);
    c.dPinv = c.upload(Dp);
  }
  if (literal && !c.dist() && N <= DENSE_MAX && c.prm.solver_path != 1) {
    std::vector<double> D(N * N, 0.0);
    for (i64 r = 0; r < N; ++r)
      for (i64 k = c.Lit.rowptr[r]; k < c.Lit.rowptr[r + 1]; ++k) D[r * N + c.Lit.col[k]] += c.Lit.val[k];
    require(lu_inverse(D, N), "literal operator is singular");
    c.dLitInv = c.upload(D);
  }
  if (literal) {
    dsell(c.sLit, c.Lit, c.dLit);
    sell_values(c.Lit, lp, c.sLit, c.Lit.val, tmp);
    c.dLitv = c.upload(tmp);
    std::vector<double> dinv(N);
    for (i64 g = 0; g < N; ++g) dinv[g] = 1.0 / diag_of(c.Lit, c.Lit.val, g);
    c.dlit_dinv = c.upload(dinv);
  }
  clk.mark("device: projections, dense");
  // per-row data
  {
    std::vector<double> as1, mp, wm;
    std::vector<uint8_t> df;
    std::vector<i32> so, mo;
    host_alloc_fresh(as1, no);
    host_alloc_fresh(mp, no);
    host_alloc_fresh(wm, no);
    host_alloc_fresh(df, no);
    host_alloc_fresh(so, no);
    host_alloc_fresh(mo, no);
    parallel_for(no, [&](i64 i0, i64 i1) {
      for (i64 i = i0; i < i1; ++i) {
        const i64 g = lp.r0 + i;
        as1[i] = c.as.asum[g] + 1e-12;
        mp[i] = c.as.M[g] + 1e-12;
        wm[i] = m.mk[c.ord.new2old[g]] == 0 ? c.as.M[g] : 0.0;
        df[i] = isdir[g];
        so[i] = c.slave_of[g] >= 0 ? to_local(lp, c.slave_of[g]) : -1;
        mo[i] = c.master_of[g] >= 0 ? to_local(lp, c.master_of[g]) : -1;
        require(so[i] < (i32)no && mo[i] < (i32)no, "periodic partner on another rank");
      }
    });
    c.das1 = c.upload(as1);
    c.dmp = c.upload(mp);
    c.dwmix = c.upload(wm);
    c.ddir = c.upload(df);
    c.dslave_of = c.upload(so);
    c.dmaster_of = c.upload(mo);
  }
  clk.mark("  dev: per-row data");
  // BC lists: sequential copy semantics resolved symbolically (caller numbering), then local
  {
    std::vector<i64> src(N);
    for (i64 i = 0; i < N; ++i) src[i] = i;
    for (auto& pr : c.bc_pairs) src[pr.second] = src[pr.first];
    std::vector<i32> cd, cs;
    for (i64 o = 0; o < N; ++o)
      if (src[o] != o) {
        const i64 g = c.ord.old2new[o];
        if (g < lp.r0 || g >= lp.r1) continue;
        const i64 gs = c.ord.old2new[src[o]];
        require(gs >= lp.r0 && gs < lp.r1, "periodic BC source on another rank");
        cd.push_back((i32)(g - lp.r0));
        cs.push_back((i32)(gs - lp.r0));
      }
    // Dirichlet: last occurrence wins (sequential semantics), owned nodes only
    std::vector<i64> last(N, -1);
    for (size_t k = 0; k < c.dir_nodes.size(); ++k) last[c.dir_nodes[k]] = (i64)k;
    std::vector<i32> dn;
    std::vector<double> dv;
    for (size_t k = 0; k < c.dir_nodes.size(); ++k) {
      if (last[c.dir_nodes[k]] != (i64)k) continue;
      const i64 g = c.ord.old2new[c.dir_nodes[k]];
      if (g < lp.r0 || g >= lp.r1) continue;
      dn.push_back((i32)(g - lp.r0));
      for (int q = 0; q < c.dir_ncomp; ++q) dv.push_back(c.dir_vals[c.dir_ncomp * k + q]);
    }
    // a copy into a Dirichlet node is overwritten by its Dirichlet value: drop it, so the write sets
    // are disjoint
    {
      std::vector<char> written(no, 0);
      for (i32 d : dn) written[d] = 1;
      std::vector<i32> cd2, cs2;
      for (size_t k = 0; k < cd.size(); ++k)
        if (!written[cd[k]]) {
          cd2.push_back(cd[k]);
          cs2.push_back(cs[k]);
        }
      cd.swap(cd2);
      cs.swap(cs2);
      for (i32 d : cd) written[d] = 1;
      c.bc_gather = false;
      for (i32 sidx : cs) c.bc_gather = c.bc_gather || written[sidx];
    }
    c.ncopy = (int)cd.size();
    c.ndir = (int)dn.size();
    c.dcdst = c.upload(cd);
    c.dcsrc = c.upload(cs);
    c.ddnode = c.upload(dn);
    c.ddval = c.upload(dv);
    c.dbctmp = c.dalloc<double>(2 * std::max(1, c.ncopy));
    c.dspos = nullptr;  // (k_grad_proj_bc's position map follows the operators: rebuilt at the next step call)
    c.dbcsrc = c.dbcdir = nullptr;
    if (c.dense) {  // k_dense_mv2_bc's per-row maps
      std::vector<i32> bsrc(no), bdir(no, -1);
      for (i64 i = 0; i < no; ++i) bsrc[i] = (i32)i;
      for (size_t k = 0; k < cd.size(); ++k) bsrc[cd[k]] = cs[k];
      for (size_t k = 0; k < dn.size(); ++k) bdir[dn[k]] = (i32)k;
      c.dbcsrc = c.upload(bsrc);
      c.dbcdir = c.upload(bdir);
    }
  }
  clk.mark("  dev: BC lists");
  // halo plan
  c.nsend = (i64)lp.send_local.size();
  c.dsend = c.upload(lp.send_local);
  c.dsendbuf = c.dalloc<double>(4 * std::max<i64>(1, c.nsend));  // (two interleaved vectors: halo2(x, b))
  // fields + workspace
  for (double** f : {&c.p, &c.p2, &c.yp, &c.yp2, &c.yvx, &c.yvy, &c.div_star, &c.div_u, &c.final_div, &c.braw,
                     &c.bh, &c.bvx, &c.bvy, &c.scalar})
    *f = c.dalloc<double>(c.nloc);
  // u and u*: interleaved (x, y) pairs (VS); ux / usx point at the pairs, uy / usy at their y components
  c.ux = c.dalloc<double>(2 * c.nloc);
  c.uy = c.ux + 1;
  c.usx = c.dalloc<double>(2 * c.nloc);
  c.usy = c.usx + 1;
  for (int q = 0; q < 2; ++q) {
    c.cg_r[q] = c.dalloc<double>(c.nloc);
    c.cg_pa[q] = c.dalloc<double>(c.nloc);
    c.cg_pb[q] = c.dalloc<double>(c.nloc);
    c.cg_q[q] = c.dalloc<double>(c.nloc);
  }
  if (stokes && !c.dense) {  // the viscous Chebyshev solve's interleaved vectors
    for (auto& x : c.vx2) x = c.dalloc<dbl2>(c.nloc);
    c.vb2 = c.dalloc<dbl2>(c.nloc);
    for (auto& d : c.vd2) d = c.dalloc<flt2>(c.nloc);
  }
  // 6 MAXB: the recurrence CG direction kernel writes 3 dots per right-hand side
  for (double** f : {&c.part_a, &c.part_b, &c.part_c, &c.part_d}) *f = c.dalloc<double>(6 * MAXB);
  c.part_sl = c.dalloc<double>(3 * SLB);
  c.part_mx = c.dalloc<double>(MAXB);
  c.part_fd = c.dalloc<double>(2 * MAXB);
  if (const char* e = std::getenv("PUCFEM_SL_OVERLAP")) c.sl_overlap = std::atoi(e) != 0;  // 0: one stream
  c.part_u = c.dalloc<double>(2 * MAXB);
  c.yr_own = c.dalloc<double>(2);
  c.yr_all = c.dalloc<double>(2 * c.world);
  c.h_yr.assign(2 * c.world, 0.0);
  if (stokes) {
    c.sl_queue = c.dalloc<int32_t>(m.N);
    c.sl_qcnt = c.dalloc<int32_t>(SLB * BS / 64);
    c.sl_qoff = c.dalloc<int32_t>(SLB * BS / 64 + 1);
  }
  c.scal = c.dalloc<double>(32);
  c.part_cc = c.dalloc<double>(CGCG_NV * MAXB);
  c.cgcg_sc = c.dalloc<double>(8);
  c.ctl = c.dalloc<int>(8);  // [0..1] the control word, bytes 8..23: the PCG's initial <r, r>, <b, b> (k_conv's note)
  c.redbuf = c.dalloc<double>(8 * 64);
  c.dcnt = c.dalloc<unsigned>(Ctx::CNT_N);
  c.vals = c.dalloc<double>(16);
  c.bicg_sc = c.dalloc<double>(16);
  if (literal || c.dye_impl) {
    for (int q = 0; q < 9; ++q) c.litw[q] = c.dalloc<double>(c.nloc);
  }
  clk.mark("device: per-row data, BCs, halo, workspace");
  // full-mesh replica in internal numbering (the host half: sl_prep, on its thread since the hierarchy)
  if (!stokes) sl_prep(c, false, slp);
  slg.join();
  clk.mark("SL: host tables (joined)");
  {
    const std::vector<double>&X = slp.X, &Y = slp.Y;
    const std::vector<i32>& tri = slp.tri;
    c.mx = c.upload(X);
    c.my = c.upload(Y);
    c.mtri = c.upload(tri);
    auto dgrid = [&](const Grid& G, GridDev& D, bool pts) {
      D.nx = G.nx;
      D.ny = G.ny;
      D.x0 = G.x0;
      D.y0 = G.y0;
      D.hx = G.hx;
      D.hy = G.hy;
      D.start = c.upload(G.cell_start);
      D.item = c.upload(G.item);
      D.px = pts ? c.upload(G.px) : nullptr;
      D.py = pts ? c.upload(G.py) : nullptr;
    };
    if (stokes) {  // PointLocator centroids (StokesColor.py:321), their grid (sl_prep)
      const std::vector<double>&cx = slp.cx, &cy = slp.cy;
      const Grid& G = slp.G;
      dgrid(G, c.cgrid, true);
      c.has_cgrid = true;
      if (prm.scheme == PUCFEM_STOKES_FOOD) {  // tracer location (StokesFood only)
        dgrid(slp.TG, c.tgrid, false);
        c.has_tgrid = true;
      }
      clk.mark("SL: centroid / triangle grids");
      // fast-accept radii (k-NN of every centroid among the centroids, of every vertex among the
      // centroids): on the device (k_knn_radius2, bit-identical to the host's knn_radius2, which
      // PUCFEM_KNN_HOST=1 selects -- the cross-check of tests/test_gpu_parity.py)
      const bool knn_host = std::getenv("PUCFEM_KNN_HOST") && std::atoi(std::getenv("PUCFEM_KNN_HOST"));
      const bool knn_ok = (i64)G.item.size() - 1 >= KNN && (i64)G.item.size() >= KNN + 1;
      std::vector<float> rho2;
      const float* drho2 = nullptr;
      const float* drv2 = nullptr;
      if (knn_host || !knn_ok) {
        rho2 = centroid_knn_radius2(G, cx, cy, KNN);
        drho2 = c.upload(rho2);
        clk.mark("SL: centroid 10-NN radii");
        drv2 = c.upload(knn_radius2(G, X, Y, KNN + 1, false));
      } else {
        float* r2 = c.dalloc<float>(m.T);
        hipLaunchKernelGGL(k_knn_radius2, dim3((unsigned)std::min<i64>(65536, (m.T + BS - 1) / BS)), dim3(BS), 0, c.st,
                           c.cgrid, c.cgrid.px, c.cgrid.py, c.cgrid.item, (int64_t)m.T, KNN, 1, r2);
        KCHK();
        float* v2 = c.dalloc<float>(N);
        hipLaunchKernelGGL(k_knn_radius2, dim3((unsigned)std::min<i64>(65536, (N + BS - 1) / BS)), dim3(BS), 0, c.st,
                           c.cgrid, (const double*)c.mx, (const double*)c.my, (const int32_t*)nullptr, (int64_t)N,
                           KNN + 1, 0, v2);
        KCHK();
        drho2 = r2;
        drv2 = v2;
        clk.mark("SL: centroid 10-NN radii");
      }
      const double2* dxy = reinterpret_cast<const double2*>(c.upload(slp.xy));
      clk.mark("SL: vertex 11-NN radii");
      const int probe = std::getenv("PUCFEM_SL_PROBE") ? std::atoi(std::getenv("PUCFEM_SL_PROBE")) : 0;
      c.lat_sl = slp.lat_sl;  // the lattice locator (sl_prep decided), else the record locator below
      if (c.lat_sl) {
        GridDev mg{};
        dgrid(slp.MG, mg, false);
        c.llgrid = LatLocDev{mg.nx, mg.ny, mg.x0, mg.y0, 1.0 / mg.hx, 1.0 / mg.hy, mg.start, mg.item,
                             reinterpret_cast<const lat::SlFace*>(c.upload(slp.sf)), c.upload(slp.cells), dxy,
                             drho2, drv2, c.upload(slp.home), nullptr, c.mg.back().latl.n, probe};
        // zero-velocity rows (walls): the answer for the row's own node, once
        int32_t* dself = c.dalloc<int32_t>(N);
        hipLaunchKernelGGL(k_sl_self<LatLocDev>, dim3(2048), dim3(BS), 0, c.st, MeshDev{c.mx, c.my, c.mtri, m.T},
                           c.llgrid, c.cgrid, (int64_t)N, dself);
        KCHK();
        c.llgrid.self = dself;
      } else {
        // inflated-bbox grid (~1 triangle per cell) + packed records
        Grid LG;
        build_tri_grid(X, Y, tri, 1.0, LG, 1e-6);
        // records in node order: position p holds triangle p2t[p], sorted by smallest vertex id
        std::vector<i32> p2t(m.T), t2p(m.T), vmin(m.T);
        for (i64 t = 0; t < m.T; ++t) {
          p2t[t] = (i32)t;
          vmin[t] = std::min(tri[3 * t], std::min(tri[3 * t + 1], tri[3 * t + 2]));
        }
        std::stable_sort(p2t.begin(), p2t.end(), [&](i32 a, i32 b) { return vmin[a] < vmin[b]; });
        for (i64 p = 0; p < m.T; ++p) t2p[p2t[p]] = (i32)p;
        if (rho2.empty()) {  // the device radii, in triangle order, for the record permutation below
          rho2.resize(m.T);
          HIPCHK(hipMemcpyAsync(rho2.data(), drho2, sizeof(float) * m.T, hipMemcpyDeviceToHost, c.st));
          HIPCHK(hipStreamSynchronize(c.st));
        }
        std::vector<int32_t> rec(4 * (size_t)m.T);  // SlTri records (pucfem_kernels_impl.hpp)
        std::vector<float> rho2p(m.T);
        for (i64 p = 0; p < m.T; ++p) {
          const i64 t = p2t[p];
          for (int v = 0; v < 3; ++v) rec[4 * p + v] = tri[3 * t + v];
          rec[4 * p + 3] = (int32_t)t;
          rho2p[p] = rho2[t];
        }
        for (i64 cl = 0; cl + 1 < (i64)LG.cell_start.size(); ++cl) {
          auto b0 = LG.item.begin() + LG.cell_start[cl], b1 = LG.item.begin() + LG.cell_start[cl + 1];
          for (auto it = b0; it != b1; ++it) *it = t2p[*it];
          std::sort(b0, b1);
        }
        GridDev lg{};
        dgrid(LG, lg, false);
        c.lgrid = LocDev{lg.nx, lg.ny, lg.x0, lg.y0, lg.hx, lg.hy, lg.start, lg.item,
                         reinterpret_cast<const int4*>(c.upload(rec)), dxy, c.upload(rho2p), drv2, probe};
      }
    }
    c.c_full = c.dalloc<double>(N);
    c.c_new = c.dalloc<double>(N);
    c.dnotfound = c.dalloc<int32_t>(no);
    if (c.dist()) {
      c.ufx = c.dalloc<double>(N);
      c.ufy = c.dalloc<double>(N);
      if (c.lp.n_ghost > 0) c.dghost_global = c.upload(c.lp.ghost_global);
    }
  }
  // initial state: u = 0 then makeDirBCU (StokesColor.py:482-483); c = 1[x < 0.5] (:493-495)
  if (stokes) {
    c.bc(c.ux, c.uy);
    c.halo_v(c.ux);
    HIPCHK(hipMemcpyAsync(c.c_full, slp.c0.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
  }
  HIPCHK(hipStreamSynchronize(c.st));
  clk.mark("SL: locator / self table, initial state");
  if (c.use_mg && c.lmax_dev) {
    MgLevel& F = c.mg[c.mg_levels];
    F.lmax = c.lmax_device(F.lmax, &F.lam_dev);
    clk.mark("finest lmax (device power iteration)");
    for (int l = 1; l < c.mg_levels; ++l)
      c.mg[l].lmax = c.mg_single ? c.lmax_level_device<float>(c.mg[l], c.mg[l].lmax)
                                 : c.lmax_level_device<double>(c.mg[l], c.mg[l].lmax);
    clk.mark("coarse lmax (device power iterations)");
  }
}

}  // namespace

// =====================================================================================================
extern "C" {

int pucfem_abi_version(void) { return PUCFEM_ABI_VERSION; }

const char* pucfem_last_error(const void* ctx) {
  return ctx ? static_cast<const Ctx*>(ctx)->err.c_str() : g_err.c_str();
}

int pucfem_device_count(int32_t* n) {
  return guard(nullptr, [&] {
    int k = 0;
    HIPCHK(hipGetDeviceCount(&k));
    *n = k;
  });
}

int pucfem_ctx_create(int32_t device, void** out) {
  return guard(nullptr, [&] {
    auto c = std::make_unique<Ctx>();
    c->device = device;
    c->host_only = device < 0;
    if (const char* e = std::getenv("PUCFEM_MG_BLOCKS")) c->mg_nb_max = std::max(1, std::atoi(e));  // tuning knob
    if (!c->host_only) {
      HIPCHK(hipSetDevice(device));
      // PUCFEM_STREAM_PRIO=1 (measurement knob): the main stream at the highest priority, the dye side stream at the
      // lowest (the dispatcher then hands freed slots to the main stream's blocks first)
      if (std::getenv("PUCFEM_STREAM_PRIO") && std::atoi(std::getenv("PUCFEM_STREAM_PRIO")) != 0) {
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&c->st, hipStreamNonBlocking, hi));
        c->sl_prio = lo;
        c->sl_prio_on = true;
      } else {
        HIPCHK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
      }
      HIPCHK(hipHostMalloc((void**)&c->h_ctl, 8 * sizeof(int), hipHostMallocDefault));
      HIPCHK(hipHostMalloc((void**)&c->h_coef, 5 * Ctx::NCOEF * sizeof(double), hipHostMallocDefault));
      HIPCHK(hipHostMalloc((void**)&c->h_pinned, 64 * sizeof(double), hipHostMallocDefault));
    }
    *out = c.release();
  });
}

int pucfem_rccl_unique_id(uint8_t* out) {
  return guard(nullptr, [&] {
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == PUCFEM_UNIQUE_ID_BYTES, "unique id size");
    std::memcpy(out, &id, sizeof(id));
  });
}

int pucfem_ctx_create_dist(int32_t device, int32_t rank, int32_t world, const uint8_t* uid, void** out) {
  void* p = nullptr;
  int rc = pucfem_ctx_create(device, &p);
  if (rc) return rc;
  rc = guard(p, [&] {
    Ctx& c = *C(p);
    require(world >= 1 && rank >= 0 && rank < world, "bad rank / world");
    c.rank = rank;
    c.world = world;
    static const char kLocal[] = "PUCFEM-LOCALCOMM";
    const bool local = std::memcmp(uid, kLocal, sizeof(kLocal) - 1) == 0;
    if (!c.host_only && (world > 1 || !local)) {
      if (local) {
        // test backend: W ranks as W contexts (host threads) of one process
        c.comm = std::make_unique<LocalComm>(std::string((const char*)uid, PUCFEM_UNIQUE_ID_BYTES), world, rank);
      } else {
        ncclUniqueId id;
        std::memcpy(&id, uid, sizeof(id));
        try {
          c.comm = std::make_unique<NcclComm>(world, id, rank);
        } catch (const std::exception& e) {
          throw Error(PUCFEM_ENCCL, e.what());
        }
      }
    }
  });
  if (rc) {
    g_err = C(p)->err;
    delete C(p);
    return rc;
  }
  *out = p;
  return 0;
}

int pucfem_ctx_destroy(void* ctx) {
  return guard(nullptr, [&] { delete C(ctx); });
}

int pucfem_mesh_upload(void* ctx, int64_t N, const double* xy, const int32_t* mk, int64_t T, const int32_t* tris,
                       int32_t coord_fp32) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    require(N > 0 && T > 0 && xy && mk && tris, "empty mesh");
    HostMesh& m = c.mesh;
    m.N = N;
    m.T = T;
    m.x.resize(N);
    m.y.resize(N);
    for (i64 i = 0; i < N; ++i) {
      m.x[i] = xy[2 * i];
      m.y[i] = xy[2 * i + 1];
    }
    m.mk.assign(mk, mk + N);
    m.tri.assign(tris, tris + 3 * T);
    bool ok = true;
    for (i64 k = 0; k < 3 * T; ++k) ok &= m.tri[k] >= 0 && m.tri[k] < N;
    require(ok, "triangle index out of range");
    m.fp32 = coord_fp32 != 0;
    c.has_mesh = true;
    c.built = false;
  });
}

int pucfem_set_pairs(void* ctx, int32_t kind, int64_t n, const int64_t* pairs) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    require(c.has_mesh, "mesh first");
    auto& v = kind == 0 ? c.op_pairs : c.bc_pairs;
    v.clear();
    for (i64 k = 0; k < n; ++k) {
      require(pairs[2 * k] >= 0 && pairs[2 * k] < c.mesh.N && pairs[2 * k + 1] >= 0 && pairs[2 * k + 1] < c.mesh.N,
              "pair index out of range");
      v.push_back({pairs[2 * k], pairs[2 * k + 1]});
    }
    c.built = false;
  });
}

int pucfem_set_dirichlet(void* ctx, int64_t n, const int32_t* nodes, const double* values, int32_t ncomp) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    require(c.has_mesh, "mesh first");
    require(ncomp == 1 || ncomp == 2, "ncomp must be 1 or 2");
    c.dir_nodes.assign(nodes, nodes + n);
    for (i32 d : c.dir_nodes) require(d >= 0 && d < c.mesh.N, "Dirichlet node out of range");
    c.dir_vals.assign(values, values + ncomp * n);
    c.dir_ncomp = ncomp;
    c.built = false;
  });
}

int pucfem_set_hierarchy(void* ctx, int64_t N0, const double* xy0, const int32_t* mk0, int64_t T0,
                         const int32_t* tris0, int32_t levels) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    require(levels >= 0 && levels <= 12, "levels in [0, 12]");
    require(N0 > 0 && T0 > 0, "empty coarse mesh");
    HostMesh& m = c.coarse;
    m.N = N0;
    m.T = T0;
    m.x.resize(N0);
    m.y.resize(N0);
    for (i64 i = 0; i < N0; ++i) {
      m.x[i] = xy0[2 * i];
      m.y[i] = xy0[2 * i + 1];
    }
    m.mk.assign(mk0, mk0 + N0);
    m.tri.assign(tris0, tris0 + 3 * T0);
    for (i64 k = 0; k < 3 * T0; ++k) require(m.tri[k] >= 0 && m.tri[k] < N0, "coarse triangle index out of range");
    c.mg_levels = levels;
    c.built = false;
  });
}

int pucfem_set_source(void* ctx, int64_t T, const float* g) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    require(c.has_mesh && T == c.mesh.T, "source must have one value per triangle");
    c.g_tri.assign(g, g + T);
    c.built = false;
  });
}

int pucfem_build_operators(void* ctx, const pucfem_params* prm) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.prm = *prm;
    c.built = false;
    if (c.gexec) {
      (void)hipGraphExecDestroy(c.gexec);
      (void)hipGraphDestroy(c.graph);
      c.gexec = nullptr;
      c.graph = nullptr;
      c.graph_mode = false;
    }
    if (c.gexec_k) {
      (void)hipGraphExecDestroy(c.gexec_k);
      (void)hipGraphDestroy(c.graph_k);
      c.gexec_k = nullptr;
      c.graph_k = nullptr;
    }
    build(c);
  });
}

// ---- fields
int pucfem_set_field(void* ctx, int32_t field, const double* buf, int64_t count) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    const i64 N = c.mesh.N, no = c.lp.n_own;
    auto own2 = [&](double* a, double*) {  // (the interleaved velocity: a = its pairs)
      require(count == 2 * N, "field must be (N, 2)");
      std::vector<double> xy(2 * no);
      for (i64 i = 0; i < no; ++i) {
        const i64 o = c.ord.new2old[c.lp.r0 + i];
        xy[2 * i] = buf[2 * o];
        xy[2 * i + 1] = buf[2 * o + 1];
      }
      HIPCHK(hipMemcpyAsync(a, xy.data(), sizeof(double) * 2 * no, hipMemcpyHostToDevice, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      c.halo_v(a);
    };
    auto own1 = [&](double* a) {
      require(count == N, "field must be (N,)");
      std::vector<double> x(no);
      for (i64 i = 0; i < no; ++i) x[i] = buf[c.ord.new2old[c.lp.r0 + i]];
      HIPCHK(hipMemcpyAsync(a, x.data(), sizeof(double) * no, hipMemcpyHostToDevice, c.st));
      c.halo(a);
    };
    switch (field) {
      case PUCFEM_F_U:
        own2(c.ux, c.uy);
        c.have_vinc = 0;  // a new state: no last viscous increment
        break;
      case PUCFEM_F_USTAR: own2(c.usx, c.usy); break;
      case PUCFEM_F_SCALAR: own1(c.scalar); break;
      case PUCFEM_F_C: {
        require(count == N, "c must be (N,)");
        std::vector<double> x(N);
        for (i64 g = 0; g < N; ++g) x[g] = buf[c.ord.new2old[g]];
        HIPCHK(hipMemcpyAsync(c.c_full, x.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
        break;
      }
      case PUCFEM_F_TRACERS: {
        require(count % 2 == 0, "tracers must be (n, 2)");
        const i64 n = count / 2;
        if (n != c.ntr) {
          c.ntr = (int32_t)n;
          c.trx = c.dalloc<double>(n);
          c.try_ = c.dalloc<double>(n);
          c.trs = c.dalloc<double>(n);
          if (c.dist()) c.trv = c.dalloc<double>(3 * n);
        }
        std::vector<double> x(n), y(n);
        for (i64 k = 0; k < n; ++k) {
          x[k] = buf[2 * k];
          y[k] = buf[2 * k + 1];
        }
        HIPCHK(hipMemcpyAsync(c.trx, x.data(), sizeof(double) * n, hipMemcpyHostToDevice, c.st));
        HIPCHK(hipMemcpyAsync(c.try_, y.data(), sizeof(double) * n, hipMemcpyHostToDevice, c.st));
        HIPCHK(hipMemsetAsync(c.trs, 0, sizeof(double) * n, c.st));
        break;
      }
      case PUCFEM_F_STATUS:
        require(count == c.ntr, "status must match the tracer count");
        HIPCHK(hipMemcpyAsync(c.trs, buf, sizeof(double) * count, hipMemcpyHostToDevice, c.st));
        break;
      default: throw Error(PUCFEM_EINVAL, "field cannot be set");
    }
    HIPCHK(hipStreamSynchronize(c.st));
  });
}

int pucfem_get_field(void* ctx, int32_t field, double* buf, int64_t count) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    const i64 N = c.mesh.N, no = c.lp.n_own;
    auto get2 = [&](const double* a, const double*) {  // (the interleaved velocity)
      require(count == 2 * N, "field is (N, 2)");
      std::vector<double> xy(2 * no);
      HIPCHK(hipMemcpyAsync(xy.data(), a, sizeof(double) * 2 * no, hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      for (i64 i = 0; i < no; ++i) {
        const i64 o = c.ord.new2old[c.lp.r0 + i];
        buf[2 * o] = xy[2 * i];
        buf[2 * o + 1] = xy[2 * i + 1];
      }
    };
    auto get1 = [&](const double* a) {
      require(count == N, "field is (N,)");
      std::vector<double> x(no);
      HIPCHK(hipMemcpyAsync(x.data(), a, sizeof(double) * no, hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      for (i64 i = 0; i < no; ++i) buf[c.ord.new2old[c.lp.r0 + i]] = x[i];
    };
    switch (field) {
      case PUCFEM_F_U: get2(c.ux, c.uy); break;
      case PUCFEM_F_USTAR: get2(c.usx, c.usy); break;
      case PUCFEM_F_P:  // with p_from_y the step keeps p in y (slaves not copied): p formed when read
      case PUCFEM_F_P2: {
        double* pf = field == PUCFEM_F_P ? c.p : c.p2;
        if (c.p_from_y) {
          const i64 n = c.lp.n_own;
          hipLaunchKernelGGL(k_cg_fin, dim3(Ctx::grid_ew(n)), dim3(BS), 0, c.st, n, 1, (const double*)nullptr,
                             (const double*)(field == PUCFEM_F_P ? c.yp : c.yp2), (const double*)nullptr, pf,
                             (double*)nullptr, (const int32_t*)c.dmaster_of);
          KCHK();
        }
        get1(pf);
        break;
      }
      case PUCFEM_F_DIV_STAR:  // computed from u* when read (the step records only its max)
        if (c.scheme == PUCFEM_STOKES_COLOR || c.scheme == PUCFEM_STOKES_FOOD) c.div(c.usx, c.usy, c.div_star, false);
        get1(c.div_star);
        break;
      case PUCFEM_F_DIV_U: get1(c.div_u); break;
      case PUCFEM_F_FINAL_DIV:  // likewise from u (the implicit dye variant keeps its own copy)
        if ((c.scheme == PUCFEM_STOKES_COLOR || c.scheme == PUCFEM_STOKES_FOOD) && !c.dye_impl)
          c.div(c.ux, c.uy, c.final_div, false);
        get1(c.final_div);
        break;
      case PUCFEM_F_SCALAR: get1(c.scalar); break;
      case PUCFEM_F_C: {
        require(count == N, "c is (N,)");
        c.allgather_full(c.c_full);  // multi-rank: collective (every rank reads c), the full field
        std::vector<double> x(N);
        HIPCHK(hipMemcpyAsync(x.data(), c.c_full, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipStreamSynchronize(c.st));
        for (i64 g = 0; g < N; ++g) buf[c.ord.new2old[g]] = x[g];
        break;
      }
      case PUCFEM_F_TRACERS: {
        require(count == 2 * (i64)c.ntr, "tracers are (n, 2)");
        std::vector<double> x(c.ntr), y(c.ntr);
        HIPCHK(hipMemcpyAsync(x.data(), c.trx, sizeof(double) * c.ntr, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipMemcpyAsync(y.data(), c.try_, sizeof(double) * c.ntr, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipStreamSynchronize(c.st));
        for (i64 k = 0; k < c.ntr; ++k) {
          buf[2 * k] = x[k];
          buf[2 * k + 1] = y[k];
        }
        break;
      }
      case PUCFEM_F_STATUS:
        require(count == c.ntr, "status is (n,)");
        HIPCHK(hipMemcpyAsync(buf, c.trs, sizeof(double) * count, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipStreamSynchronize(c.st));
        break;
      default: throw Error(PUCFEM_EINVAL, "unknown field");
    }
  });
}

// ---- stepping
int pucfem_step(void* ctx, int32_t nsteps, pucfem_step_stats* stats) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(nsteps >= 0, "nsteps < 0");
    if (nsteps == 0) return;
    if (c.scheme == PUCFEM_STOKES_COLOR || c.scheme == PUCFEM_STOKES_FOOD) {
      double* rec = c.dalloc<double>(8 * (i64)nsteps);
      int* dits = c.dalloc<int>(3 * (i64)nsteps);
      std::vector<int32_t> its(3 * (size_t)nsteps);
      if (c.dense && !c.timer.on && !c.dye_impl) {
        // direct-solve small-mesh path: every step is the same sequence of ~25 launches with no
        // host synchronisation -> capture it once (and GK steps of it once), replay them
        // capture `count` consecutive steps into one graph (the steps' buffers are fixed in graph mode)
        auto capture = [&](int count, hipGraph_t& gr, hipGraphExec_t& ex) {
          int32_t tmp[3];
          HIPCHK(hipStreamBeginCapture(c.st, hipStreamCaptureModeThreadLocal));
          try {
            c.gcapture = true;
            for (int k = 0; k < count; ++k) c.stokes_step(c.gstats, tmp);
            c.gcapture = false;
          } catch (...) {
            c.gcapture = false;
            c.fork_pend = false;
            hipGraph_t g;
            (void)hipStreamEndCapture(c.st, &g);
            c.graph_mode = c.gexec != nullptr;
            throw;
          }
          HIPCHK(hipStreamEndCapture(c.st, &gr));
          HIPCHK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
        };
        c.prep_grad_proj_bc();
        c.prep_fork();
        if (!c.gexec) {
          c.gstats = c.dalloc<double>(8);
          c.gring = c.dalloc<double>(8 * (i64)Ctx::GRING);
          c.gcount = c.dalloc<int>(1);
          HIPCHK(hipStreamSynchronize(c.st));
          c.graph_mode = true;
          capture(1, c.graph, c.gexec);
        }
        if (!c.gexec_k && c.gk > 1 && nsteps >= c.gk) capture(c.gk, c.graph_k, c.gexec_k);
        HIPCHK(hipMemsetAsync(c.gcount, 0, sizeof(int), c.st));
        for (int s = 0, k = 0; s < nsteps;) {
          int d = 1;
          if (c.gexec_k && nsteps - s >= c.gk && k + c.gk <= Ctx::GRING) {
            HIPCHK(hipGraphLaunch(c.gexec_k, c.st));
            d = c.gk;
          } else {
            HIPCHK(hipGraphLaunch(c.gexec, c.st));
          }
          s += d;
          k += d;
          if (k == Ctx::GRING || s == nsteps) {  // the ring's records -> this call's records
            HIPCHK(hipMemcpyAsync(rec + 8 * (s - k), c.gring, sizeof(double) * 8 * k, hipMemcpyDeviceToDevice, c.st));
            if (s < nsteps) HIPCHK(hipMemsetAsync(c.gcount, 0, sizeof(int), c.st));
            k = 0;
          }
        }
      } else {
        c.graph_mode = c.gexec != nullptr;  // once captured, keep c in its fixed buffer
        c.dits = dits;
        c.prep_grad_proj_bc();
        try {
          for (int s = 0; s < nsteps; ++s) {
            c.cur_step = s;
            c.stokes_step(rec + 8 * s, its.data() + 3 * s);
          }
          c.proj_materialize();  // (no direction stays pending between API calls)
          c.dye_tail_dist();     // (nor a dye tail: the last step's, now)
          c.sl_join();
        } catch (...) {
          c.dits = nullptr;
          if (c.sl_pending) (void)hipStreamSynchronize(c.st_sl);
          c.sl_pending = false;
          c.slb_pend = false;
          c.tail_pend = false;
          throw;
        }
        c.dits = nullptr;
      }
      std::vector<double> h(8 * (size_t)nsteps);
      std::vector<int> hd(3 * (size_t)nsteps);
      HIPCHK(hipMemcpyAsync(h.data(), rec, sizeof(double) * h.size(), hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipMemcpyAsync(hd.data(), dits, sizeof(int) * hd.size(), hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      if (c.timer.on) c.timer.flush();
      for (void* q : {(void*)rec, (void*)dits}) {
        HIPCHK(hipFree(q));
        c.allocs.erase(std::find(c.allocs.begin(), c.allocs.end(), q));
      }
      for (size_t k = 0; k < its.size(); ++k)
        if (its[k] < 0) {
          if (hd[k] < 0) throw Error(PUCFEM_ENOCONV, "single-workgroup CG did not converge (step " +
                                                         std::to_string(k / 3) + ")");
          its[k] = hd[k];
        }
      if (stats)
        for (int s = 0; s < nsteps; ++s) {
          pucfem_step_stats& o = stats[s];
          const double* r = h.data() + 8 * s;
          o.max_div_star = r[0];
          o.max_final_div = r[1];
          o.mix_I = r[2];
          o.mix_mu = r[3];
          o.mix_var = r[4];
          o.eaten = (int64_t)std::llround(r[5]);
          o.sl_notfound = (int32_t)std::llround(r[6]);
          o.it_visc = its[3 * s];
          o.it_p = its[3 * s + 1];
          o.it_p2 = its[3 * s + 2];
        }
    } else if (c.scheme == PUCFEM_HEAT) {
      // heatEq.py:321-325: u = solve(A, u + DT*b*0); reapply_periodic_u; reapply_dirchlect_u
      const i64 n = c.lp.n_own;
      for (int s = 0; s < nsteps; ++s) {
        int it = 0;
        if (c.dLitInv) {  // small mesh: u = A^-1 u (one launch, no host synchronisation)
          hipLaunchKernelGGL(k_dense_mv<double>, dim3((int)std::min<i64>(2048, (n + 3) / 4)), dim3(BS), 0, c.st, n,
                             (const double*)c.dLitInv, (const double*)c.scalar, c.litw[8], (const int*)nullptr);
          KCHK();
          std::swap(c.scalar, c.litw[8]);
        } else {
          HIPCHK(hipMemcpyAsync(c.litw[8], c.scalar, sizeof(double) * n, hipMemcpyDeviceToDevice, c.st));
          it = c.bicgstab(c.scalar, c.litw[8], c.prm.rtol_lin, c.prm.maxit_lin);
        }
        c.bc(c.scalar, nullptr);
        if (stats) {
          std::memset(&stats[s], 0, sizeof(pucfem_step_stats));
          stats[s].it_visc = it;
        }
      }
      HIPCHK(hipStreamSynchronize(c.st));
    } else {
      // poisson.py:283-285: f = solve(A, b)
      HIPCHK(hipMemcpyAsync(c.bh, c.litb.data(), sizeof(double) * c.lp.n_own, hipMemcpyHostToDevice, c.st));
      HIPCHK(hipMemsetAsync(c.scalar, 0, sizeof(double) * c.lp.n_own, c.st));
      int it = 0;
      if (c.dLitInv) {
        hipLaunchKernelGGL(k_dense_mv<double>, dim3((int)std::min<i64>(2048, (c.lp.n_own + 3) / 4)), dim3(BS), 0, c.st,
                           (int64_t)c.lp.n_own, (const double*)c.dLitInv, (const double*)c.bh, c.scalar,
                           (const int*)nullptr);
        KCHK();
      } else {
        it = c.bicgstab(c.scalar, c.bh, c.prm.rtol_lin, c.prm.maxit_lin);
      }
      HIPCHK(hipStreamSynchronize(c.st));
      if (stats) {
        std::memset(&stats[0], 0, sizeof(pucfem_step_stats));
        stats[0].it_visc = it;
      }
    }
  });
}

// ---- unit operations (single rank)
int pucfem_apply(void* ctx, int32_t op, const double* x, double* y) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(!c.dist(), "pucfem_apply is single-rank");
    const i64 N = c.mesh.N;
    auto perm_in = [&](const double* src, int ncomp, double* d0, double* d1) {
      std::vector<double> a(N), b(N);
      for (i64 g = 0; g < N; ++g) {
        const i64 o = c.ord.new2old[g];
        a[g] = src[ncomp * o];
        if (ncomp > 1) b[g] = src[ncomp * o + 1];
      }
      HIPCHK(hipMemcpyAsync(d0, a.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
      if (ncomp > 1) HIPCHK(hipMemcpyAsync(d1, b.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
    };
    auto perm_out = [&](double* dst, int ncomp, const double* d0, const double* d1) {
      std::vector<double> a(N), b(N);
      HIPCHK(hipMemcpyAsync(a.data(), d0, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
      if (ncomp > 1) HIPCHK(hipMemcpyAsync(b.data(), d1, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      for (i64 g = 0; g < N; ++g) {
        const i64 o = c.ord.new2old[g];
        dst[ncomp * o] = a[g];
        if (ncomp > 1) dst[ncomp * o + 1] = b[g];
      }
    };
    double *t0 = c.cg_pa[0], *t1 = c.cg_pa[1], *o0 = c.cg_q[0], *o1 = c.cg_q[1];
    switch (op) {
      case PUCFEM_OP_K:
      case PUCFEM_OP_GX:
      case PUCFEM_OP_GY: {
        perm_in(x, 1, t0, nullptr);
        require(op == PUCFEM_OP_K || !c.lattice, "Gx / Gy alone are not applied on lattice operators (use DIV / GRAD)");
        const double* v = op == PUCFEM_OP_K ? c.dK : op == PUCFEM_OP_GX ? c.dGx : c.dGy;
        spmv_on(c.st, c.dP, c.fK.full(), v, t0, o0);
        KCHK();
        perm_out(y, 1, o0, nullptr);
        break;
      }
      case PUCFEM_OP_PRES: {
        require(c.dKp || c.dKp_raw, "no pressure operator (scheme is not Stokes)");
        if (c.lattice) {  // the unscaled merged operator (the multigrid path's)
          perm_in(x, 1, t0, nullptr);
          spmv_on(c.st, c.dPp, c.fP.full(), c.dKp_raw, t0, o0);
          KCHK();
          perm_out(y, 1, o0, nullptr);
          break;
        }
        perm_in(x, 1, t0, nullptr);
        // unscaled action: S^-1 A^ S^-1 x
        std::vector<double> s(N);
        HIPCHK(hipMemcpyAsync(s.data(), c.dsp, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipStreamSynchronize(c.st));
        std::vector<double> a(N), xs(N);
        for (i64 g = 0; g < N; ++g) xs[g] = x[c.ord.new2old[g]] / s[g];
        HIPCHK(hipMemcpyAsync(t0, xs.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
        spmv_on(c.st, c.dPp, FaceDev{}, c.dKp, t0, o0);
        KCHK();
        HIPCHK(hipMemcpyAsync(a.data(), o0, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipStreamSynchronize(c.st));
        for (i64 g = 0; g < N; ++g) y[c.ord.new2old[g]] = a[g] / s[g];
        break;
      }
      case PUCFEM_OP_LIT: {
        require(c.dLitv, "no literal operator (scheme is Stokes)");
        perm_in(x, 1, t0, nullptr);
        spmv_on(c.st, c.dLit, FaceDev{}, c.dLitv, t0, o0);
        KCHK();
        perm_out(y, 1, o0, nullptr);
        break;
      }
      case PUCFEM_OP_DIV: {
        perm_in(x, 2, t0, t1);
        with_c16(c.dP, [&](auto c16) {
          hipLaunchKernelGGL((k_div<decltype(c16)::value, false>), dim3(c.div_grid()), dim3(BS), 0, c.st, c.dP.view(),
                             c.fK.part(), c.dGx, c.dGy, t0, t1, c.das1, o0, c.dmp, -1.0, (double*)nullptr, c.part_d, RedOut{});
        });
        KCHK();
        perm_out(y, 1, o0, nullptr);
        break;
      }
      case PUCFEM_OP_GRAD: {
        perm_in(x, 1, t0, nullptr);
        with_c16(c.dP, [&](auto c16) {
          hipLaunchKernelGGL(k_grad<decltype(c16)::value>, dim3(c.grid_full(c.fK.full(), c.dP)), dim3(BS), 0, c.st,
                             c.dP.view(), c.fK.full(), c.dGx, c.dGy, t0, c.das1, o0, o1);
        });
        KCHK();
        perm_out(y, 2, o0, o1);
        break;
      }
      case PUCFEM_OP_VISC: {
        // unscaled A_visc x = S^-1 A^ S^-1 x
        std::vector<double> s(N), xs(N), a(N);
        HIPCHK(hipMemcpyAsync(s.data(), c.dsv, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipStreamSynchronize(c.st));
        for (i64 g = 0; g < N; ++g) xs[g] = x[c.ord.new2old[g]] / s[g];
        HIPCHK(hipMemcpyAsync(t0, xs.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
        spmv_on(c.st, c.dP, c.fVisc.full(), c.dKv, t0, o0);
        KCHK();
        HIPCHK(hipMemcpyAsync(a.data(), o0, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipStreamSynchronize(c.st));
        for (i64 g = 0; g < N; ++g) y[c.ord.new2old[g]] = a[g] / s[g];
        break;
      }
      default: throw Error(PUCFEM_EINVAL, "unknown op");
    }
  });
}

int pucfem_solve(void* ctx, int32_t op, const double* b, double* x, double rtol, int32_t maxit, int32_t* iters) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(!c.dist(), "pucfem_solve is single-rank");
    const i64 N = c.mesh.N;
    int it = 0;
    // standalone solves run on scratch buffers with their own iteration-hint slots (3, 4) and no
    // projection basis: a context that is stepping keeps u, p, the warm starts and the bases intact
    if (!c.solve_tmp) c.solve_tmp = c.dalloc<double>(4 * c.nloc);
    double *s0 = c.solve_tmp, *s1 = s0 + c.nloc, *s2 = s1 + c.nloc, *s3 = s2 + c.nloc;
    if (op == PUCFEM_OP_VISC) {
      // rhs = b (as u^n, initial guess b): the viscous CG without BCs
      std::vector<double> bxy(2 * N);  // (k_visc_prep reads u interleaved: s0 / s0 + 1 over 2 N of scratch)
      for (i64 g = 0; g < N; ++g) {
        bxy[2 * g] = b[2 * c.ord.new2old[g]];
        bxy[2 * g + 1] = b[2 * c.ord.new2old[g] + 1];
      }
      HIPCHK(hipMemcpyAsync(s0, bxy.data(), sizeof(double) * 2 * N, hipMemcpyHostToDevice, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      hipLaunchKernelGGL(k_visc_prep<false>, dim3(Ctx::grid_ew(N)), dim3(BS), 0, c.st, N, c.dsv, s0, s0 + 1,
                         c.bvx, c.bvy, c.yvx, c.yvy, VincDev{});
      KCHK();
      double* y[2] = {c.yvx, c.yvy};
      const double* bb[2] = {c.bvx, c.bvy};
      it = c.cg<2>(c.dP, c.fVisc, c.dKv, y, bb, rtol, maxit, 3);
      hipLaunchKernelGGL(k_cg_fin, dim3(Ctx::grid_ew(N)), dim3(BS), 0, c.st, N, 2, c.dsv, c.yvx, c.yvy, s2, s3,
                         (const int32_t*)nullptr);
      KCHK();
      std::vector<double> ox(N), oy(N);
      HIPCHK(hipMemcpyAsync(ox.data(), s2, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipMemcpyAsync(oy.data(), s3, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      for (i64 g = 0; g < N; ++g) {
        x[2 * c.ord.new2old[g]] = ox[g];
        x[2 * c.ord.new2old[g] + 1] = oy[g];
      }
    } else if (op == PUCFEM_OP_PRES) {
      require(c.dKp || c.dKp_raw, "no pressure operator");
      // b = b_p: braw = (M + 1e-12) * b_p, then the same path as the step (slot 4: no projection)
      std::vector<double> mp(N), br(N);
      HIPCHK(hipMemcpyAsync(mp.data(), c.dmp, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      double sum = 0.0;
      for (i64 g = 0; g < N; ++g) {
        br[g] = mp[g] * b[c.ord.new2old[g]];
        sum += br[g];
      }
      HIPCHK(hipMemcpyAsync(c.braw, br.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
      std::vector<double> part(4 * MAXB, 0.0);
      part[MAXB] = sum;
      HIPCHK(hipMemcpyAsync(c.part_d, part.data(), sizeof(double) * part.size(), hipMemcpyHostToDevice, c.st));
      // pressure() reduces part_d + MAXB over nb_for(dP) blocks: only entry 0 is non-zero
      HIPCHK(hipMemsetAsync(s0, 0, sizeof(double) * c.nloc, c.st));
      pucfem_params save = c.prm;
      c.prm.rtol_pres = rtol;
      c.prm.maxit_pres = maxit;
      try {
        it = c.pressure(s0, s1, 4);
      } catch (...) {
        c.prm = save;
        throw;
      }
      c.prm = save;
      std::vector<double> o(N);
      HIPCHK(hipMemcpyAsync(o.data(), s1, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      for (i64 g = 0; g < N; ++g) x[c.ord.new2old[g]] = o[g];
    } else if (op == PUCFEM_OP_LIT) {
      require(c.dLitv, "no literal operator");
      std::vector<double> bb(N), x0(N);
      for (i64 g = 0; g < N; ++g) {
        bb[g] = b[c.ord.new2old[g]];
        x0[g] = x[c.ord.new2old[g]];
      }
      HIPCHK(hipMemcpyAsync(c.bh, bb.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
      HIPCHK(hipMemcpyAsync(c.scalar, x0.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
      it = c.bicgstab(c.scalar, c.bh, rtol, maxit);
      std::vector<double> o(N);
      HIPCHK(hipMemcpyAsync(o.data(), c.scalar, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
      HIPCHK(hipStreamSynchronize(c.st));
      for (i64 g = 0; g < N; ++g) x[c.ord.new2old[g]] = o[g];
    } else {
      throw Error(PUCFEM_EINVAL, "op cannot be solved");
    }
    if (iters) *iters = it;
  });
}

int pucfem_sl_advect(void* ctx, const double* cin, const double* u, double dt, double* cout, int32_t* notfound) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(!c.dist() && c.has_cgrid, "sl_advect needs a single-rank Stokes context");
    const i64 N = c.mesh.N;
    std::vector<double> a(N), bxy(2 * N);
    for (i64 g = 0; g < N; ++g) {
      const i64 o = c.ord.new2old[g];
      a[g] = cin[o];
      bxy[2 * g] = u[2 * o];
      bxy[2 * g + 1] = u[2 * o + 1];
    }
    // u as the step stores it (interleaved pairs) in scratch: the step's state stays untouched
    if (!c.solve_tmp) c.solve_tmp = c.dalloc<double>(4 * c.nloc);
    double *cf = c.litw[0] ? c.litw[0] : c.cg_pa[0], *cn = c.cg_pb[0], *tx = c.solve_tmp, *ty = tx + 1;
    HIPCHK(hipMemcpyAsync(cf, a.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(tx, bxy.data(), sizeof(double) * 2 * N, hipMemcpyHostToDevice, c.st));
    const int nb = c.nb_sl(N);
    c.sl_launch(nb, 0, N, tx, ty, dt, cf, cn, c.dwmix, c.dnotfound);
    KCHK();
    std::vector<double> o(N);
    std::vector<int32_t> nf(N);
    HIPCHK(hipMemcpyAsync(o.data(), cn, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipMemcpyAsync(nf.data(), c.dnotfound, sizeof(int32_t) * N, hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipStreamSynchronize(c.st));
    for (i64 g = 0; g < N; ++g) {
      cout[c.ord.new2old[g]] = o[g];
      if (notfound) notfound[c.ord.new2old[g]] = nf[g];
    }
  });
}

int pucfem_apply_bc(void* ctx, int32_t which, double* u) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(!c.dist() && (c.scheme == PUCFEM_STOKES_COLOR || c.scheme == PUCFEM_STOKES_FOOD),
            "apply_bc needs a single-rank Stokes context");
    require(which >= 1 && which <= 3, "apply_bc: which must be 1 (periodic), 2 (Dirichlet) or 3 (both)");
    const i64 N = c.mesh.N;
    std::vector<double> bx(N), by(N);
    for (i64 g = 0; g < N; ++g) {
      bx[g] = u[2 * c.ord.new2old[g]];
      by[g] = u[2 * c.ord.new2old[g] + 1];
    }
    double *tx = c.cg_q[0], *ty = c.cg_q[1];  // scratch (the step's state stays untouched)
    HIPCHK(hipMemcpyAsync(tx, bx.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(ty, by.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
    const int ncopy = (which & 1) ? c.ncopy : 0, ndir = (which & 2) ? c.ndir : 0;
    if (ncopy + ndir > 0) {
      if (c.bc_gather && ncopy > 0) {
        hipLaunchKernelGGL(k_bc_gather, dim3(std::min(1024, (ncopy + BS - 1) / BS)), dim3(BS), 0, c.st, ncopy,
                           c.dcsrc, c.dbctmp, c.dir_ncomp, tx, ty, 1);
        KCHK();
      }
      const int nb = (int)std::min<i64>(1024, std::max<i64>(1, (ncopy + ndir + BS - 1) / BS));
      hipLaunchKernelGGL(k_bc_apply, dim3(nb), dim3(BS), 0, c.st, ncopy, c.dcdst, c.dcsrc,
                         c.bc_gather ? (const double*)c.dbctmp : nullptr, ndir, c.ddnode, c.ddval, c.dir_ncomp, tx, ty,
                         1);
      KCHK();
    }
    HIPCHK(hipMemcpyAsync(bx.data(), tx, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipMemcpyAsync(by.data(), ty, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipStreamSynchronize(c.st));
    for (i64 g = 0; g < N; ++g) {
      u[2 * c.ord.new2old[g]] = bx[g];
      u[2 * c.ord.new2old[g] + 1] = by[g];
    }
  });
}

int pucfem_dye_step(void* ctx, const double* cin, const double* u, double* cout, int32_t* iters) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(c.dye_impl, "dye_step needs a context built with dye_scheme = 1 (implicit)");
    const i64 N = c.mesh.N;
    std::vector<double> a(N), bxy(2 * N);
    for (i64 g = 0; g < N; ++g) {
      const i64 o = c.ord.new2old[g];
      a[g] = cin[o];
      bxy[2 * g] = u[2 * o];
      bxy[2 * g + 1] = u[2 * o + 1];
    }
    // u as the step stores it (interleaved pairs) in scratch: the step's state stays untouched
    if (!c.solve_tmp) c.solve_tmp = c.dalloc<double>(4 * c.nloc);
    double *tx = c.solve_tmp, *ty = tx + 1, *cf = c.cg_pa[0], *cn = c.cg_pb[0], *dv = c.litw[8];
    HIPCHK(hipMemcpyAsync(cf, a.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(tx, bxy.data(), sizeof(double) * 2 * N, hipMemcpyHostToDevice, c.st));
    c.div(tx, ty, dv, false);
    const int it = c.dye_step(tx, ty, dv, cf, cn);
    HIPCHK(hipMemcpyAsync(a.data(), cn, sizeof(double) * N, hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipStreamSynchronize(c.st));
    for (i64 g = 0; g < N; ++g) cout[c.ord.new2old[g]] = a[g];
    if (iters) *iters = it;
  });
}

int pucfem_tracer_step(void* ctx, const double* u, double dt, int32_t nsteps) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(!c.dist(), "tracer_step unit op is single-rank");
    require(c.has_tgrid, "tracer_step needs a STOKES_FOOD context (the tracer grid)");
    const i64 N = c.mesh.N;
    std::vector<double> bxy(2 * N);  // (u interleaved, as the step stores it)
    for (i64 g = 0; g < N; ++g) {
      bxy[2 * g] = u[2 * c.ord.new2old[g]];
      bxy[2 * g + 1] = u[2 * c.ord.new2old[g] + 1];
    }
    HIPCHK(hipMemcpyAsync(c.ux, bxy.data(), sizeof(double) * 2 * N, hipMemcpyHostToDevice, c.st));
    for (int s = 0; s < nsteps; ++s) c.tracer_advance(dt);
    HIPCHK(hipStreamSynchronize(c.st));
  });
}

// (I, mu, var) of c with the node weights w (device, internal order) over the N nodes of a single-rank
// context: the two weighted sums, then the weighted variance about mu (k_mix2), then k_stats
static void mixing_on(Ctx& c, const double* cin, const double* w, double* out3) {
  const i64 N = c.mesh.N;
  std::vector<double> a(N);
  for (i64 g = 0; g < N; ++g) a[g] = cin[c.ord.new2old[g]];
  double* cf = c.cg_pa[0];
  HIPCHK(hipMemcpyAsync(cf, a.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
  const int nb = c.nb_rows(N);
  // part_a[0..] = sum w c (the second dot, w w, is not used)
  hipLaunchKernelGGL(k_dot2, dim3(nb), dim3(BS), 0, c.st, N, w, (const double*)cf, w, w, c.part_a);
  KCHK();
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(RB), 0, c.st, c.part_a, nb, MAXB, 1, 0, c.vals + 2);
  std::vector<double> ones(N, 1.0);
  double* on = c.cg_pb[0];
  HIPCHK(hipMemcpyAsync(on, ones.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
  hipLaunchKernelGGL(k_dot2, dim3(nb), dim3(BS), 0, c.st, N, w, (const double*)on, (const double*)nullptr,
                     (const double*)nullptr, c.part_b);
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(RB), 0, c.st, c.part_b, nb, MAXB, 1, 0, c.vals + 3);
  hipLaunchKernelGGL(k_mix2, dim3(nb), dim3(BS), 0, c.st, (int64_t)0, N, cf, w, c.vals + 2, 1, 1, c.part_c, RedOut{});
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(RB), 0, c.st, c.part_c, nb, MAXB, 1, 0, c.vals + 5);
  HIPCHK(hipMemsetAsync(c.vals + 6, 0, 2 * sizeof(double), c.st));
  double* rec = c.vals + 8;
  hipLaunchKernelGGL(k_stats, dim3(1), dim3(64), 0, c.st, c.vals, rec, 7);
  KCHK();
  double h[8];
  HIPCHK(hipMemcpyAsync(h, rec, sizeof(double) * 7, hipMemcpyDeviceToHost, c.st));
  HIPCHK(hipStreamSynchronize(c.st));
  out3[0] = h[2];
  out3[1] = h[3];
  out3[2] = h[4];
}

int pucfem_mixing_index(void* ctx, const double* cin, double* out3) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(!c.dist(), "mixing_index unit op is single-rank");
    mixing_on(c, cin, c.dwmix, out3);
  });
}

int pucfem_mixing_index_w(void* ctx, const double* cin, const double* w, double* out3) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(!c.dist(), "mixing_index unit op is single-rank");
    require(w != nullptr, "mixing_index_w: weights");
    const i64 N = c.mesh.N;
    std::vector<double> a(N);
    for (i64 g = 0; g < N; ++g) a[g] = w[c.ord.new2old[g]];
    double* dw = c.cg_q[0];
    HIPCHK(hipMemcpyAsync(dw, a.data(), sizeof(double) * N, hipMemcpyHostToDevice, c.st));
    mixing_on(c, cin, dw, out3);
  });
}

// ---- measurement
int pucfem_timing_enable(void* ctx, int32_t on) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    HIPCHK(hipStreamSynchronize(c.st));
    c.timer.flush();
    require(on >= 0 && on <= 2, "timing mode");
    c.timer.on = on != 0;
    // mode 2: the kernel classes with a share of the step (the roofline kernel is the largest of them); mode 1
    // adds the finest level's residual and transfers
    c.timer.mask = on == 2 ? ~((1u << 5) | (1u << 6) | (1u << 7)) : ~0u;
    for (int k = 0; k < Timer::NCLS; ++k) {
      c.timer.ms[k] = 0;
      c.timer.bytes[k] = 0;
      c.timer.n[k] = 0;
    }
  });
}

int pucfem_timing_get(void* ctx, int32_t k, double* ms, int64_t* n, double* bytes) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    require(k >= 0 && k < Timer::NCLS, "kernel class");
    if (!c.host_only) {
      HIPCHK(hipStreamSynchronize(c.st));
      c.timer.flush();
    }
    *ms = c.timer.ms[k];
    *n = c.timer.n[k];
    *bytes = c.timer.n[k] ? c.timer.bytes[k] / (double)c.timer.n[k] : 0.0;
  });
}

int pucfem_counters(void* ctx, int64_t* launches, double* bytes) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    *launches = g_nlaunch;
    *bytes = c.algo_bytes;
  });
}

int pucfem_class_counters(void* ctx, int32_t kclass, int64_t* launches, double* bytes) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    require(kclass >= 0 && kclass < Timer::NCLS, "kernel class out of range");
    *launches = c.cls_n[kclass];
    *bytes = c.cls_bytes[kclass];
  });
}

int pucfem_sync(void* ctx) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    if (!c.host_only) {
      HIPCHK(hipStreamSynchronize(c.st));
    }
  });
}

int pucfem_info(void* ctx, int64_t* o) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    o[0] = c.mesh.N;
    o[1] = c.mesh.T;
    o[2] = c.P.nnz();
    o[3] = c.Pp.nnz();
    o[4] = c.lp.n_own;
    o[5] = c.lp.n_ghost;
    o[6] = c.sP.padded;
    o[7] = c.sPp.padded;
    o[8] = (int64_t)c.op_pairs.size();
    o[9] = (int64_t)c.dir_nodes.size();
    o[10] = (c.dP.c16 ? 1 : 0) | (c.dPp.c16 ? 2 : 0) | (!c.mg.empty() && c.mg.back().f32.Aval16 ? 4 : 0);
    o[11] = (int64_t)c.mg.size();
  });
}

int pucfem_path_info(void* ctx, int64_t* o) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    for (int k = 0; k < 8; ++k) o[k] = 0;
    const bool stokes = c.scheme == PUCFEM_STOKES_COLOR || c.scheme == PUCFEM_STOKES_FOOD;
    if (!stokes) return;
    const bool block = !c.dist() && c.block_cg && c.lp.n_own <= (i64)CGB_THREADS * CGB_MAXR;
    o[0] = c.dense ? 0 : (block ? 1 : 2);
    o[1] = c.dense ? 0 : (c.use_mg ? 3 : (block ? 1 : 2));
    o[2] = c.n_reseed;
    o[3] = c.proj_m[1];
    o[4] = c.proj_m[2];
    o[5] = c.dvinc[0] && !c.proj_k_visc ? std::min(c.have_vinc, c.visc_extrap) : 0;
    o[6] = c.proj_k;
    o[7] = (c.lattice ? 1 : 0) | (c.lat_sl ? 2 : 0) |
           (!c.dense && !block && c.visc_solver == 0 && c.visc_R < 0.25 ? 4 : 0) | (c.visc_check_fail ? 8 : 0) |
           (c.visc_pairs ? 16 : 0) | (c.mg_pairs ? 32 : 0) | (c.p_from_y ? 64 : 0) | (c.cgcg_iters ? 128 : 0);
  });
}

int pucfem_mg_lmax(void* ctx, int32_t level, double* o) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    require(c.use_mg && level >= 0 && level <= c.mg_levels, "level of a multigrid hierarchy");
    require(!c.dist(), "a single-rank context (the host estimate iterates the whole level)");
    const MgLevel& L = c.mg[level];
    const Csr& A = level == c.mg_levels ? c.Pp : L.Pp;
    double lam = 0.0;
    o[0] = L.lmax;
    o[1] = L.lam_dev;
    o[3] = lmax_estimate(A, false);
    lmax_estimate(A, true, nullptr, &lam);
    o[2] = lam;
  });
}

int pucfem_proj_info(void* ctx, double* o) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    o[0] = (double)c.n_reseed;
    o[1] = (double)c.n_restart;
    o[2] = c.guess_last[1];
    o[3] = c.guess_last[2];
  });
}

int pucfem_visc_interval(void* ctx, double* o) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    require(c.scheme == PUCFEM_STOKES_COLOR || c.scheme == PUCFEM_STOKES_FOOD, "a Stokes context");
    o[0] = c.visc_lo;
    o[1] = 1.0 + c.visc_R;
  });
}

int pucfem_comm_info(void* ctx, int64_t* o) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    o[0] = c.dist() ? c.dye_halo_values : 0;
    o[1] = c.dist() ? c.mesh.N - c.lp.n_own : 0;
    o[2] = c.dist() ? 3 * (int64_t)c.ntr : 0;
    o[3] = !c.comm ? 0 : (dynamic_cast<NcclComm*>(c.comm.get()) ? 2 : 1);
  });
}

int pucfem_comm_counters(void* ctx, int64_t* o) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    for (int k = 0; k < 6; ++k) o[k] = 0;
    if (!c.comm) return;
    o[0] = c.comm->n_allreduce;
    o[1] = c.comm->v_allreduce;
    o[2] = c.comm->n_msg;
    o[3] = c.comm->b_msg;
    o[4] = c.comm->n_group;
    o[5] = c.comm->n_bcast;
  });
}

// Communicator self-test on the library stream: an all-reduce (sum and max) of 8 values and one grouped
// ring exchange (send to rank + 1, receive from rank - 1; on one rank a send to itself), checked on the
// device values.  out[0] = |sum - expected|, out[1] = |max - expected|, out[2] = |received - expected|,
// out[3] = backend (1 LocalComm, 2 RCCL).
int pucfem_comm_selftest(void* ctx, double* out4) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    require(c.dist(), "comm_selftest needs a context created by pucfem_ctx_create_dist with a communicator");
    const int W = c.world, R = c.rank;
    constexpr int n = 8;
    std::vector<double> h(3 * n);
    for (int k = 0; k < n; ++k) {
      h[k] = (R + 1) * (k + 1.0);      // sum over ranks: (k + 1) W (W + 1) / 2
      h[n + k] = R + 0.25 * k;         // max over ranks: W - 1 + 0.25 k
      h[2 * n + k] = 1000.0 * R + k;   // sent to rank + 1
    }
    double* d = c.dalloc<double>(4 * n);
    HIPCHK(hipMemcpyAsync(d, h.data(), sizeof(double) * 3 * n, hipMemcpyHostToDevice, c.st));
    c.comm->allreduce(d, n, false, c.st);
    c.comm->allreduce(d + n, n, true, c.st);
    c.comm->group_start();
    c.comm->send(d + 2 * n, n, (R + 1) % W, c.st);
    c.comm->recv(d + 3 * n, n, (R + W - 1) % W, c.st);
    c.comm->group_end(c.st);
    std::vector<double> g(4 * n);
    HIPCHK(hipMemcpyAsync(g.data(), d, sizeof(double) * 4 * n, hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipStreamSynchronize(c.st));
    double e0 = 0, e1 = 0, e2 = 0;
    const int from = (R + W - 1) % W;
    for (int k = 0; k < n; ++k) {
      e0 = std::max(e0, std::fabs(g[k] - (k + 1.0) * W * (W + 1) / 2.0));
      e1 = std::max(e1, std::fabs(g[n + k] - (W - 1 + 0.25 * k)));
      e2 = std::max(e2, std::fabs(g[3 * n + k] - (1000.0 * from + k)));
    }
    out4[0] = e0;
    out4[1] = e1;
    out4[2] = e2;
    out4[3] = dynamic_cast<NcclComm*>(c.comm.get()) ? 2 : 1;
  });
}

int pucfem_cgcg_coef_probe(void* ctx, const double* red8, double bb, const double* sc5, double tol2, int32_t it,
                           int32_t maxit, double rho0, int32_t* ctl_out, double* sc_out5) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    std::vector<double> h(24, 0.0);
    for (int k = 0; k < 8; ++k) h[k] = red8[k];
    h[8] = bb;
    h[9] = rho0;
    for (int k = 0; k < 5; ++k) h[16 + k] = sc5[k];
    DevTmp<double> d(h, c.st);
    DevTmp<int> ctl(std::vector<int>{0, 0}, c.st);
    hipLaunchKernelGGL(k_cgcg_coef, dim3(1), dim3(64), 0, c.st, (const double*)d.p, (const double*)(d.p + 8), d.p + 16,
                       tol2, ctl.p, (int)it, (int)maxit, (const double*)(d.p + 9));
    KCHK();
    std::vector<int> hc;
    std::vector<double> out;
    ctl.get(hc, 2, c.st);
    d.get(out, 24, c.st);
    HIPCHK(hipStreamSynchronize(c.st));
    ctl_out[0] = hc[0];
    ctl_out[1] = hc[1];
    for (int k = 0; k < 5; ++k) sc_out5[k] = out[16 + k];
  });
}

// ---- host-only
int pucfem_refine(int64_t N, const double* xy, const int32_t* mk, int64_t T, const int32_t* tris, int32_t levels,
                  int64_t* N_out, int64_t* T_out, double* xy_out, int32_t* mk_out, int32_t* tris_out) {
  return guard(nullptr, [&] {
    require(levels >= 0 && levels <= 12, "levels in [0, 12]");
    if (!xy_out) {  // sizes only: N' = N + E, T' = 4T, E = (3T + Eb) / 2 with Eb doubling per level
      std::vector<std::pair<i32, i32>> es(3 * (size_t)T);
      for (i64 t = 0; t < T; ++t)
        for (int e = 0; e < 3; ++e) {
          const i32 a = tris[3 * t + e], b = tris[3 * t + (e + 1) % 3];
          es[3 * t + e] = {std::min(a, b), std::max(a, b)};
        }
      std::sort(es.begin(), es.end());
      i64 Eb = 0;
      for (size_t i = 0; i < es.size();) {
        size_t j = i;
        while (j < es.size() && es[j] == es[i]) ++j;
        if (j - i == 1) ++Eb;
        i = j;
      }
      i64 n = N, t = T;
      for (int l = 0; l < levels; ++l) {
        n += (3 * t + Eb) / 2;
        t *= 4;
        Eb *= 2;
      }
      *N_out = n;
      *T_out = t;
      return;
    }
    HostMesh a;
    a.N = N;
    a.T = T;
    a.x.resize(N);
    a.y.resize(N);
    for (i64 i = 0; i < N; ++i) {
      a.x[i] = xy[2 * i];
      a.y[i] = xy[2 * i + 1];
    }
    a.mk.assign(mk, mk + N);
    a.tri.assign(tris, tris + 3 * T);
    for (int l = 0; l < levels; ++l) {
      HostMesh b;
      red_refine(a, b);
      a = std::move(b);
    }
    *N_out = a.N;
    *T_out = a.T;
    if (xy_out) {
      for (i64 i = 0; i < a.N; ++i) {
        xy_out[2 * i] = a.x[i];
        xy_out[2 * i + 1] = a.y[i];
      }
      std::copy(a.mk.begin(), a.mk.end(), mk_out);
      std::copy(a.tri.begin(), a.tri.end(), tris_out);
    }
  });
}

int pucfem_host_get_csr(void* ctx, int32_t op, int64_t* n_rows, int64_t* nnz, int64_t* rowptr, int64_t* col,
                        double* val) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    const Csr* A = nullptr;
    const std::vector<double>* v = nullptr;
    if (op >= 100) {  // multigrid level matrices (CPU tests): 100 + 3 l + {0: Pp_l, 1: Pr_l, 2: R_l}
      const int l = (op - 100) / 3, kind = (op - 100) % 3;
      require(c.use_mg && l >= 0 && l <= c.mg_levels, "no such multigrid level");
      const int Lv = c.mg_levels;
      const MgLevel& L = c.mg[l];
      require(kind == 0 || l >= 1, "level 0 has no transfer operators");
      const Csr& M = kind == 0 ? (l == Lv ? c.Pp : L.Pp) : kind == 1 ? L.Pr : L.R;
      const Ordering& ro = kind == 2 ? c.mg[l - 1].ord : L.ord;
      const Ordering& co = kind == 1 ? c.mg[l - 1].ord : L.ord;
      *n_rows = M.nrows;
      *nnz = M.nnz();
      if (!col) return;
      i64 k = 0;
      rowptr[0] = 0;
      std::vector<std::pair<i64, double>> tmp;
      for (i64 o = 0; o < M.nrows; ++o) {
        const i64 g = ro.old2new[o];
        tmp.clear();
        for (i64 e = M.rowptr[g]; e < M.rowptr[g + 1]; ++e) tmp.push_back({co.new2old[M.col[e]], M.val[e]});
        std::sort(tmp.begin(), tmp.end());
        for (auto& t : tmp) {
          col[k] = t.first;
          val[k] = t.second;
          ++k;
        }
        rowptr[o + 1] = k;
      }
      return;
    }
    if (op == PUCFEM_OP_MLUMP || op == PUCFEM_OP_ASUM) {  // diagonals, owned rows in caller numbering
      const std::vector<double>& d = op == PUCFEM_OP_MLUMP ? c.as.M : c.as.asum;
      require(!d.empty(), "operator not built for this scheme");
      std::vector<i64> rows;
      for (i64 g = c.lp.r0; g < c.lp.r1; ++g) rows.push_back(c.ord.new2old[g]);
      std::sort(rows.begin(), rows.end());
      *n_rows = (i64)rows.size();
      *nnz = (i64)rows.size();
      if (!col) return;
      rowptr[0] = 0;
      for (size_t r = 0; r < rows.size(); ++r) {
        col[r] = rows[r];
        val[r] = d[c.ord.old2new[rows[r]]];
        rowptr[r + 1] = (i64)r + 1;
      }
      return;
    }
    switch (op) {
      case PUCFEM_OP_K: A = &c.P; v = &c.as.K; break;
      case PUCFEM_OP_MCONS:
        require(c.dye_impl, "the consistent mass exists on dye_scheme = 1 contexts");
        A = &c.P;
        v = &c.dyeop.mc;
        break;
      case PUCFEM_OP_GX: A = &c.P; v = &c.as.Gx; break;
      case PUCFEM_OP_GY: A = &c.P; v = &c.as.Gy; break;
      case PUCFEM_OP_VISC: A = &c.P; v = &c.Kv; break;
      case PUCFEM_OP_PRES: A = &c.Pp; v = &c.Pp.val; break;
      case PUCFEM_OP_LIT: A = &c.Lit; v = &c.Lit.val; break;
      default: throw Error(PUCFEM_EINVAL, "op has no CSR");
    }
    require(A->nrows > 0, "operator not built for this scheme");
    const LocalPlan& lp = c.lp;
    // owned rows in caller numbering, ascending
    std::vector<i64> rows;
    for (i64 g = lp.r0; g < lp.r1; ++g) rows.push_back(c.ord.new2old[g]);
    std::sort(rows.begin(), rows.end());
    i64 total = 0;
    for (i64 o : rows) {
      const i64 g = c.ord.old2new[o];
      total += A->rowptr[g + 1] - A->rowptr[g];
    }
    *n_rows = (i64)rows.size();
    *nnz = total;
    if (!col) return;
    i64 k = 0;
    rowptr[0] = 0;
    std::vector<std::pair<i64, double>> tmp;
    for (size_t r = 0; r < rows.size(); ++r) {
      const i64 g = c.ord.old2new[rows[r]];
      tmp.clear();
      for (i64 e = A->rowptr[g]; e < A->rowptr[g + 1]; ++e) tmp.push_back({c.ord.new2old[A->col[e]], (*v)[e]});
      std::sort(tmp.begin(), tmp.end());
      for (auto& t : tmp) {
        col[k] = t.first;
        val[k] = t.second;
        ++k;
      }
      rowptr[r + 1] = k;
    }
  });
}

int pucfem_host_lattice_apply(void* ctx, int32_t level, int32_t kind, const double* x, double* y) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    require(c.lattice && !c.dist(), "needs a single-rank context with lattice operators");
    const int Lv = c.mg_levels;
    require(level >= 0 && level <= Lv, "level out of range");
    require(kind >= 0 && kind <= 6 && kind != 4, "kind");
    require(kind >= 3 || level == Lv, "kinds 0-2 are finest-level operators");
    require(kind < 5 || level >= 1, "transfers need level >= 1");
    MgLevel& L = c.mg[level];
    const int in_l = kind == 5 ? level - 1 : level, out_l = kind == 6 ? level - 1 : level;
    const Ordering& oin = c.mg[in_l].ord;
    const Ordering& oout = c.mg[out_l].ord;
    const i64 nin = (i64)oin.new2old.size(), nout = (i64)oout.new2old.size();
    const int ncomp = kind == 1 ? 2 : 1;
    std::vector<double> x0(nin), x1(ncomp > 1 ? nin : 0), yv(nout, NAN);
    for (i64 g = 0; g < nin; ++g) {
      const i64 o = oin.new2old[g];
      x0[g] = x[ncomp * o];
      if (ncomp > 1) x1[g] = x[ncomp * o + 1];
    }
    const int n = 1 << level;
    std::vector<double> wsk;
    if (kind == 2) {
      std::vector<uint8_t> isdir(c.mesh.N, 0);
      for (i32 d : c.dir_nodes) isdir[c.ord.old2new[d]] = 1;
      wsk.resize(c.mesh.N);
      for (i64 g = 0; g < c.mesh.N; ++g) wsk[g] = isdir[g] ? 0.0 : 1.0 / std::sqrt(diag_of(c.P, c.Kv, g));
    }
    if (kind <= 2) {
      lattice_apply_host(kind, n, L.lf_plain, L.lf_coef, x0.data(), ncomp > 1 ? x1.data() : nullptr,
                         kind == 2 ? wsk.data() : nullptr, yv.data());
    } else if (kind == 3) {
      lattice_apply_host(0, n, L.lf_merged, L.lf_coef, x0.data(), nullptr, nullptr, yv.data());
    } else if (kind == 5) {
      lattice_apply_host(3, n, L.lf_plain, L.lf_coef, x0.data(), nullptr, nullptr, yv.data(), &L.pr_tab2, n / 2);
    } else {
      lattice_apply_host(4, n / 2, L.r_tab, L.lf_coef, x0.data(), nullptr, nullptr, yv.data(), &L.r_tab2, n);
    }
    for (i64 g = 0; g < nout; ++g) y[oout.new2old[g]] = yv[g];
  });
}

int pucfem_host_partition(void* ctx, int32_t rank, int32_t world, int64_t* n_own, int64_t* n_ghost, int64_t* owned,
                          int64_t* ghosts, int32_t* ghost_owner, int64_t* n_send, int64_t* send_ids,
                          int32_t* send_peer) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_built();
    require(rank >= 0 && rank < world, "bad rank");
    std::vector<i64> rs;
    partition_rows(c.P, c.ord, world, rs);
    LocalPlan lp;
    std::vector<const Csr*> pats = {&c.P};
    if (c.Pp.nrows) pats.push_back(&c.Pp);
    // PUCFEM_HOST_PLAN_DEEP=1 (test knob): the deep-halo plan of the W > 1 multigrid runs (make_local_plan2 with the
    // patterns' ghost rows one layer out and their columns), as Ctx builds it for the finest level
    const char* deep_env = std::getenv("PUCFEM_HOST_PLAN_DEEP");
    if (deep_env && std::atoi(deep_env) != 0) {
      std::vector<PatRows> pr;
      for (const Csr* A : pats) pr.push_back({A, &rs});
      make_local_plan2(pr, rs, rank, lp, &pats);
    } else {
      make_local_plan(pats, rs, rank, lp);
    }
    *n_own = lp.n_own;
    *n_ghost = lp.n_ghost;
    *n_send = (i64)lp.send_local.size();
    if (!owned) return;
    for (i64 i = 0; i < lp.n_own; ++i) owned[i] = c.ord.new2old[lp.r0 + i];
    for (i64 k = 0; k < lp.n_ghost; ++k) {
      ghosts[k] = c.ord.new2old[lp.ghost_global[k]];
      ghost_owner[k] = lp.ghost_owner[k];
    }
    for (size_t q = 0; q < lp.send_peer.size(); ++q)
      for (i64 k = 0; k < lp.send_cnt[q]; ++k) {
        const i64 idx = lp.send_off[q] + k;
        send_ids[idx] = c.ord.new2old[lp.r0 + lp.send_local[idx]];
        send_peer[idx] = lp.send_peer[q];
      }
  });
}


// ---- kernel micro-benchmark (tools/spmv_variants.py): k_cg_dir variants on the pressure operator
int pucfem_bench_dir(void* ctx, int32_t variant, int32_t nblocks, int32_t iters, double* ms_out) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(c.dKp && !c.lattice, "needs a Stokes context with SELL operators");
    const DevSell& A = c.dPp;
    const int nb = nblocks > 0 ? std::min(nblocks, MAXB) : Ctx::nb_for(A.nslices);
    CgVecs<1> v;
    v.y[0] = c.yp;
    v.b[0] = c.bh;
    v.r[0] = c.cg_r[0];
    v.po[0] = c.cg_pa[0];
    v.pn[0] = c.cg_pb[0];
    v.q[0] = c.cg_q[0];
    std::vector<double> ones(c.nloc, 1.0);
    HIPCHK(hipMemcpyAsync(c.cg_r[0], ones.data(), sizeof(double) * c.nloc, hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(c.cg_pa[0], ones.data(), sizeof(double) * c.nloc, hipMemcpyHostToDevice, c.st));
    const double sc[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
    HIPCHK(hipMemcpyAsync(c.scal, sc, sizeof(sc), hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(c.part_a, sc, sizeof(double), hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemsetAsync(c.ctl, 0, 2 * sizeof(int), c.st));
    auto launch = [&]() {
      switch (variant) {
        case 0: hipLaunchKernelGGL((k_cg_dir<1, 0, false, false>), dim3(nb), dim3(BS), 0, c.st, A.view(), FaceDev{}, c.dKp, v, (int64_t)0, c.part_a, 1, 1, c.part_a, 1, 1, c.scal, c.ctl, 1, 1 << 30, 0.0, c.part_c); break;
        case 1: hipLaunchKernelGGL((k_cg_dir<1, 8, false, false>), dim3(nb), dim3(BS), 0, c.st, A.view(), FaceDev{}, c.dKp, v, (int64_t)0, c.part_a, 1, 1, c.part_a, 1, 1, c.scal, c.ctl, 1, 1 << 30, 0.0, c.part_c); break;
        case 2: hipLaunchKernelGGL((k_cg_dir<1, 0, true, false>), dim3(nb), dim3(BS), 0, c.st, A.view(), FaceDev{}, c.dKp, v, (int64_t)0, c.part_a, 1, 1, c.part_a, 1, 1, c.scal, c.ctl, 1, 1 << 30, 0.0, c.part_c); break;
        case 3: hipLaunchKernelGGL((k_cg_dir<1, 8, true, false>), dim3(nb), dim3(BS), 0, c.st, A.view(), FaceDev{}, c.dKp, v, (int64_t)0, c.part_a, 1, 1, c.part_a, 1, 1, c.scal, c.ctl, 1, 1 << 30, 0.0, c.part_c); break;
        default: require(A.c16 != nullptr, "variant 4 needs int16 columns");
                 hipLaunchKernelGGL((k_cg_dir<1, 8, true, true>), dim3(nb), dim3(BS), 0, c.st, A.view(), FaceDev{}, c.dKp, v, (int64_t)0, c.part_a, 1, 1, c.part_a, 1, 1, c.scal, c.ctl, 1, 1 << 30, 0.0, c.part_c); break;
      }
      KCHK();
    };
    launch();
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(hipEventRecord(a, c.st));
    for (int k = 0; k < iters; ++k) launch();
    HIPCHK(hipEventRecord(b, c.st));
    HIPCHK(hipEventSynchronize(b));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *ms_out = ms / iters;
  });
}

int pucfem_bench_kernel(void* ctx, int32_t kernel, int32_t iters, double* ms_batch, double* ms_each, double* bytes) {
  return guard(ctx, [&] {
    Ctx& c = *C(ctx);
    c.need_dev();
    c.need_built();
    require(c.use_mg && c.mg_single && iters > 0, "bench_kernel needs a multigrid context with the fp32 V-cycle");
    MgLevel& L = c.mg.back();
    MgBufs<float>& B = L.f32;
    const DevSell& A = c.dPp;
    // kernel / 16 = untimed launches of a coarse level's smoother between the timed launches (how the
    // per-launch events behave when other kernels run in between, as inside a step)
    // kernel / 256 = 1: the host waits for every launch before it submits the next (the GPU is idle
    // when each launch's packet arrives)
    const bool idle = (kernel / 256) & 1;
    kernel %= 256;
    const int nfill = kernel / 16;
    kernel %= 16;
    const FaceDev ff = c.fP.full(), fpt = c.fP.part();
    const int nb_mg = c.grid_full(ff, A), nb = Ctx::grid_part(fpt, A);
    CgVecs<1> v;
    v.y[0] = c.yp;
    v.b[0] = c.bh;
    v.r[0] = c.z;
    v.po[0] = c.cg_pa[0];
    v.pn[0] = c.cg_pb[0];
    v.q[0] = c.cg_q[0];
    double by = 0.0;
    // scalar state of k_cg_dir: beta = 1, never converged
    const double sc[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
    double* one = c.redbuf + 8 * 60;
    HIPCHK(hipMemcpyAsync(c.scal, sc, sizeof(sc), hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(one, sc, sizeof(double), hipMemcpyHostToDevice, c.st));
    int* ctl0 = reinterpret_cast<int*>(c.redbuf + 8 * 61);
    HIPCHK(hipMemsetAsync(ctl0, 0, 4 * sizeof(int), c.st));
    auto launch = [&](hipEvent_t a, hipEvent_t e) {
      with_c16(A, [&](auto c16) {
        constexpr bool C16 = decltype(c16)::value;
        SellDev none = A.view();
        none.nslices = 0;
        switch (kernel) {
          case 3:  // the face part alone
            hipExtLaunchKernelGGL(k_cheb<float, float, float, float, C16, 2>, dim3(ff.nb + 8), dim3(BS), 0, c.st, a, e, 0,
                                  none, ff, (const float*)B.Aval, (const float*)B.dinv, (const float*)c.r32,
                                  (const float*)B.x, B.x2, B.d, 0.3, 0.7, 0.0, 1, (const int*)nullptr,
                                  (const double*)nullptr, (double*)nullptr, RedOut{},
                                  (float*)nullptr);
            break;
          case 4:  // the SELL (skeleton) part alone
            hipExtLaunchKernelGGL(k_cheb<float, float, float, float, C16, 2>, dim3(c.nb_mg(A.nslices)), dim3(BS), 0, c.st,
                                  a, e, 0, A.view(), FaceDev{}, (const float*)B.Aval, (const float*)B.dinv,
                                  (const float*)c.r32, (const float*)B.x, B.x2, B.d, 0.3, 0.7, 0.0, 1,
                                  (const int*)nullptr, (const double*)nullptr, (double*)nullptr, RedOut{},
                                  (float*)nullptr);
            break;
          case 5:  // k_cg_dir, the face part alone
            hipExtLaunchKernelGGL(k_cg_dir<1, 8, true, C16>, dim3(fpt.nb + 8), dim3(BS), 0, c.st, a, e, 0, none, fpt,
                                  (const double*)c.dKp_raw, v, c.lp.n_ghost, (const double*)one, 1, 1,
                                  (const double*)one, 1, 1, c.scal, ctl0, 1, 1 << 30, 0.0, c.part_c,
                                  (const double*)nullptr, 0, 0, RedOut{});
            break;
          case 6:  // k_cg_dir, the SELL (skeleton) part alone
            hipExtLaunchKernelGGL(k_cg_dir<1, 8, true, C16>, dim3(Ctx::nb_for(A.nslices)), dim3(BS), 0, c.st, a, e, 0,
                                  A.view(), FaceDev{}, (const double*)c.dKp_raw, v, c.lp.n_ghost, (const double*)one,
                                  1, 1, (const double*)one, 1, 1, c.scal, ctl0, 1, 1 << 30, 0.0, c.part_c,
                                  (const double*)nullptr, 0, 0, RedOut{});
            break;
          case 0:
            hipExtLaunchKernelGGL(k_cheb<float, float, float, float, C16, 2>, dim3(nb_mg), dim3(BS), 0, c.st, a, e, 0,
                                  A.view(), ff, (const float*)B.Aval, (const float*)B.dinv, (const float*)c.r32,
                                  (const float*)B.x, B.x2, B.d, 0.3, 0.7, 0.0, 1, (const int*)nullptr,
                                  (const double*)nullptr, (double*)nullptr, RedOut{},
                                  (float*)nullptr);
            break;
          case 1:
            hipExtLaunchKernelGGL(k_resid<float, float, float, C16, 2>, dim3(nb_mg), dim3(BS), 0, c.st, a, e, 0, A.view(),
                                  ff, (const float*)B.Aval, (const float*)c.r32, (const float*)B.x, B.res,
                                  (const int*)nullptr);
            break;
          case 12:  // k_cheb_pair<1> (two smoothing steps on the face rows, general start)
          case 13:  // k_cheb_pair<2> (the fused first two steps from x = 0, then the third)
            if (c.mgp_x && c.fP.items > 0) {
              const HFace& hf = c.fP;
              MgPairVecs pv{(const float*)c.r32, (const float*)B.dinv, (const float*)B.x, B.x2, c.mgp_x,
                            (const float*)B.d, c.mgp_d};
              if (kernel == 12)
                hipExtLaunchKernelGGL(k_cheb_pair<1>, dim3(hf.items), dim3(BS), 0, c.st, a, e, 0, hf.full(), pv, 0.3f,
                                      0.7f, 0.0f, 0.3f, 0.7f, (const int*)nullptr);
              else
                hipExtLaunchKernelGGL(k_cheb_pair<2>, dim3(hf.items), dim3(BS), 0, c.st, a, e, 0, hf.full(), pv, 0.3f,
                                      0.7f, 0.5f, 0.3f, 0.7f, (const int*)nullptr);
            }
            break;
          case 15:  // k_reseed: the pressure basis (all proj_k vectors) into PROJ_KEEP_MAX new ones (scratch target)
            if (c.proj_k > 0 && c.dqm) {
              const i64 n = c.lp.n_own;
              hipExtLaunchKernelGGL(k_reseed, dim3(Ctx::grid_ew(n)), dim3(BS), 0, c.st, a, e, 0, (int64_t)n,
                                    (const ProjT*)c.projX[1], (int64_t)c.pld(1), c.proj_k, (const double*)c.dqm,
                                    (int)PROJ_KEEP_MAX, c.projXalt[1]);
            }
            break;
          case 14:  // k_vcheb_pair (two viscous Chebyshev steps on the face rows, general start)
            if (c.vx2[2] && c.fVisc.items > 0) {
              VPairVecs p{};
              p.xa = c.vx2[0];
              p.xb = c.vx2[1];
              p.xc = c.vx2[2];
              p.b = c.vb2;
              p.da = c.vd2[0];
              p.dc = c.vd2[1];
              hipExtLaunchKernelGGL(k_vcheb_pair, dim3(c.fVisc.items), dim3(BS), 0, c.st, a, e, 0, c.fVisc.part(), p,
                                    0.3, 0.7, 0.3, 0.7, (const int*)ctl0, (double*)nullptr, 0, 0, (double*)nullptr,
                                    (double*)nullptr);
            }
            break;
          case 7:   // k_div as in the step (interleaved u, the pressure rhs, partials)
          case 8:   // its face part alone
          case 9:   // its SELL (skeleton) part alone
          case 10:  // k_div on interleaved (x, y) pairs
          case 11:  // the same, face part alone
            with_c16(c.dP, [&](auto d16) {
              constexpr bool D16 = decltype(d16)::value;
              const FaceDev fd = c.fK.part();
              SellDev dv = c.dP.view();
              if (kernel == 8 || kernel == 11) dv.nslices = 0;
              const int g = kernel == 8 || kernel == 11 ? fd.nb + 8 : kernel == 9 ? c.div_grid() - fd.nb : c.div_grid();
              const FaceDev fk = kernel == 9 ? FaceDev{} : fd;
              const bool aos = true;  // (the step's u is interleaved: 7-9 on u itself, 10-11 on a viscous buffer)
              const double* xa = kernel >= 10 ? reinterpret_cast<const double*>(c.vx2[0]) : (const double*)c.ux;
              if (aos)
                hipExtLaunchKernelGGL(k_div<D16, true>, dim3(g), dim3(BS), 0, c.st, a, e, 0, dv, fk, (const double*)c.dGx,
                                      (const double*)c.dGy, xa, (const double*)nullptr, (const double*)c.das1,
                                      (double*)nullptr, (const double*)c.dmp, -1.0, c.braw, c.part_d, RedOut{});
              else
                hipExtLaunchKernelGGL(k_div<D16, false>, dim3(g), dim3(BS), 0, c.st, a, e, 0, dv, fk,
                                      (const double*)c.dGx, (const double*)c.dGy, xa, (const double*)c.uy,
                                      (const double*)c.das1, (double*)nullptr, (const double*)c.dmp, -1.0, c.braw,
                                      c.part_d, RedOut{});
            });
            break;
          default:
            hipExtLaunchKernelGGL(k_cg_dir<1, 8, true, C16>, dim3(nb), dim3(BS), 0, c.st, a, e, 0, A.view(), fpt,
                                  (const double*)c.dKp_raw, v, c.lp.n_ghost, (const double*)one, 1, 1,
                                  (const double*)one, 1, 1, c.scal, ctl0, 1, 1 << 30, 0.0, c.part_c,
                                  (const double*)nullptr, 0, 0, RedOut{});
        }
      });
      KCHK();
    };
    // face rows read no matrix (and the smoother no dinv: 24 B instead of 28)
    const double fr = (double)c.fP.rows, sk = (double)A.nrows, rb = A.row_bytes();
    switch (kernel) {
      case 0: by = (4.0 + A.idx_bytes()) * (double)A.nnz + (28.0 + rb) * sk + 24.0 * fr; break;
      case 3: by = 24.0 * fr; break;
      case 4: by = (4.0 + A.idx_bytes()) * (double)A.nnz + (28.0 + rb) * sk; break;
      case 5: by = 32.0 * fr; break;
      case 6: by = (8.0 + A.idx_bytes()) * (double)A.nnz + (32.0 + rb) * sk; break;
      case 1: by = (4.0 + A.idx_bytes()) * (double)A.nnz + (12.0 + rb) * sk + 12.0 * fr; break;
      case 7:
      case 10:
        by = (16.0 + c.dP.idx_bytes()) * (double)c.dP.nnz + c.dP.row_bytes() * (double)c.dP.nrows + 24.0 * (double)c.lp.n_own;
        break;
      case 8:
      case 11: by = 24.0 * (double)c.fK.rows; break;
      case 12: by = 20.0 * (double)c.fP.rows; break;  // x_a, d_a, b read; x_{a+2}, d_{a+2} written (fp32)
      case 13: by = 12.0 * (double)c.fP.rows; break;  // b read; x_{a+2}, d_{a+2} written
      case 14: by = 64.0 * (double)c.fVisc.rows; break;  // x_a, b, d_a read; x_{a+2}, d_{a+2} written
      case 15: by = 4.0 * (c.proj_k + PROJ_KEEP_MAX) * (double)c.lp.n_own; break;  // the basis read, the new one written
      case 9: by = (16.0 + c.dP.idx_bytes()) * (double)c.dP.nnz + (c.dP.row_bytes() + 24.0) * (double)c.dP.nrows; break;
      default: by = (8.0 + A.idx_bytes()) * (double)A.nnz + (32.0 + rb) * sk + 32.0 * fr;
    }
    MgLevel& Lc = c.mg[c.mg.size() >= 3 ? c.mg.size() - 3 : 0];
    auto fill = [&] {
      for (int f = 0; f < nfill; ++f) {
        with_c16(Lc.dA, [&](auto c16) {
          constexpr bool C16 = decltype(c16)::value;
          hipLaunchKernelGGL((k_cheb<float, float, float, float, C16, 0>), dim3(c.grid_full(Lc.hA.full(), Lc.dA)), dim3(BS),
                             0, c.st, Lc.dA.view(), Lc.hA.full(), (const float*)Lc.f32.Aval, (const float*)Lc.f32.dinv,
                             (const float*)Lc.f32.b, (const float*)nullptr, Lc.f32.x2, Lc.f32.d, 0.3, 0.7, 0.0, 2,
                             (const int*)nullptr, (const double*)nullptr, (double*)nullptr, RedOut{});
        });
        KCHK();
      }
    };
    launch(nullptr, nullptr);
    hipEvent_t ea, eb;
    HIPCHK(hipEventCreate(&ea));
    HIPCHK(hipEventCreate(&eb));
    HIPCHK(hipEventRecord(ea, c.st));
    for (int k = 0; k < iters; ++k) {
      launch(nullptr, nullptr);
      fill();
    }
    HIPCHK(hipEventRecord(eb, c.st));
    HIPCHK(hipEventSynchronize(eb));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ea, eb));
    *ms_batch = ms / iters;
    std::vector<hipEvent_t> ev(2 * (size_t)iters);
    for (auto& x : ev) HIPCHK(hipEventCreate(&x));
    for (int k = 0; k < iters; ++k) {
      launch(ev[2 * k], ev[2 * k + 1]);
      fill();
      if (idle) HIPCHK(hipStreamSynchronize(c.st));
    }
    HIPCHK(hipEventSynchronize(ev.back()));
    double tot = 0.0;
    for (int k = 0; k < iters; ++k) {
      HIPCHK(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
      tot += ms;
    }
    *ms_each = tot / iters;
    for (auto& x : ev) (void)hipEventDestroy(x);
    (void)hipEventDestroy(ea);
    (void)hipEventDestroy(eb);
    *bytes = by;
  });
}

}  // extern "C"
