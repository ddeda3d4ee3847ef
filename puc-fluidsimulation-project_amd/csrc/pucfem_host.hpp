// Host-side runtime of libpucfem: mesh refinement, node ordering, operator assembly,
// partition / halo plan and the SELL-64 device layout.  Pure C++ (no HIP), so it is
// exercised by the CPU test-suite through a host-only context.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <memory>
#include <string>
#include <algorithm>
#include <thread>
#include <utility>
#include <functional>
#include <vector>

#include <sys/mman.h>

#include "pucfem_lattice.hpp"

namespace pucfem {

using i32 = int32_t;
using i64 = int64_t;

// ----------------------------------------------------------------------------- host threading
// Threads that are joined on every exit path (a failed spawn unwinds through the destructor instead of
// destroying joinable threads, which would terminate the process) and whose exceptions reach the caller:
// join() rethrows the first one.
struct ThreadGroup {
  std::vector<std::thread> th;
  std::vector<std::shared_ptr<std::exception_ptr>> err;  // one heap slot per thread (stable while spawning)
  template <class F>
  void spawn(F&& f) {
    auto slot = std::make_shared<std::exception_ptr>();
    err.push_back(slot);
    th.emplace_back([slot, f = std::forward<F>(f)]() mutable {
      try {
        f();
      } catch (...) {
        *slot = std::current_exception();
      }
    });
  }
  void wait() {
    for (auto& t : th)
      if (t.joinable()) t.join();
  }
  void join() {
    wait();
    for (auto& e : err)
      if (*e) std::rethrow_exception(*e);
  }
  ~ThreadGroup() { wait(); }
};
// host threads for the setup's parallel loops: PUCFEM_HOST_THREADS, else OMP_NUM_THREADS, else the cgroup's
// CPU quota (cgroup v2 cpu.max), else the hardware threads; at most 64.  (A GPU box shows hundreds of
// hardware threads to a process whose quota is 16 CPUs: 64 threads per loop there only add spawns and
// throttling.)
inline int host_threads() {
  static const int n = [] {
    auto env = [](const char* k) {
      const char* e = std::getenv(k);
      return e ? std::atoi(e) : 0;
    };
    int t = env("PUCFEM_HOST_THREADS");
    if (t <= 0) t = env("OMP_NUM_THREADS");
    if (t <= 0) {
      if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long long period = 0;
        if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
          t = (int)std::max(1LL, std::atoll(q) / period);
        std::fclose(f);
      }
    }
    const int hw = (int)std::thread::hardware_concurrency();
    if (t <= 0) t = hw > 0 ? hw : 1;
    if (hw > 0) t = std::min(t, hw);
    return std::max(1, std::min(t, 64));
  }();
  return n;
}
// f(r0, r1) over a split of [0, n) into contiguous ranges, one thread each (up to host_threads(), and one
// per `grain` items: loops over heavy items -- faces, SELL slices, chunks -- pass a small grain)
template <class F>
void parallel_for(i64 n, F&& f, i64 grain = 4096) {
  const int nt = (int)std::max<i64>(1, std::min<i64>({(i64)host_threads(), n / std::max<i64>(1, grain) + 1}));
  if (nt == 1) {
    f((i64)0, n);
    return;
  }
  ThreadGroup g;
  for (int w = 0; w < nt; ++w) g.spawn([&, w] { f(n * w / nt, n * (w + 1) / nt); });
  g.join();
}
// v = n value-initialised elements (the old contents are dropped, whatever the capacity) for a large array
// the setup fills next: a fresh allocation is advised onto transparent huge pages first (first-touch
// zero-fill of 4 KiB pages ran at ~1.6 GB/s, half the rate on 2 MiB pages)
template <class T>
void host_alloc_fresh(std::vector<T>& v, size_t n) {
  v.clear();
  if (n * sizeof(T) >= (size_t(32) << 20) && v.capacity() < n) {
    std::vector<T>().swap(v);
    v.reserve(n);
    const uintptr_t HP = uintptr_t(1) << 21;
    const uintptr_t a = (reinterpret_cast<uintptr_t>(v.data()) + HP - 1) & ~(HP - 1);
    const uintptr_t e = reinterpret_cast<uintptr_t>(v.data()) + n * sizeof(T);
    if (e > a) (void)madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);
  }
  v.resize(n);
}
// f(chunk, r0, r1) over PAR_CHUNKS fixed chunks of [0, n) (independent of the machine's thread
// count: per-chunk partial sums combined in chunk order are reproducible everywhere)
constexpr int PAR_CHUNKS = 64;
template <class F>
void parallel_chunks(i64 n, F&& f) {
  const int nt = (int)std::max<i64>(1, std::min<i64>({PAR_CHUNKS, (i64)host_threads(), n / 4096 + 1}));
  auto run = [&](int w) {
    for (int ch = w; ch < PAR_CHUNKS; ch += nt) f(ch, n * ch / PAR_CHUNKS, n * (ch + 1) / PAR_CHUNKS);
  };
  if (nt == 1) {
    run(0);
    return;
  }
  ThreadGroup g;
  for (int w = 0; w < nt; ++w) g.spawn([&run, w] { run(w); });
  g.join();
}

struct HostMesh {
  i64 N = 0, T = 0;
  std::vector<double> x, y;  // caller numbering
  std::vector<i32> mk;       // Triangle boundary markers (0 interior, 1 outer, 2 inner body)
  std::vector<i32> tri;      // T*3, caller numbering, CCW
  bool fp32 = false;         // coordinates are the fp32 values of poisson.py:40
};

// Red refinement: every triangle -> 4, edge midpoints appended after the old nodes in
// (min, max) edge order; boundary-edge midpoints inherit the boundary marker.
void red_refine(const HostMesh& in, HostMesh& out, std::vector<i32>* edge_a = nullptr,
                std::vector<i32>* edge_b = nullptr);

// CSR pattern / matrix with column ids in the INTERNAL (new) numbering.
struct Csr {
  i64 nrows = 0;
  std::vector<i64> rowptr;
  std::vector<i32> col;
  std::vector<double> val;
  i64 nnz() const { return nrows ? rowptr[nrows] : 0; }
  i64 find(i64 r, i32 c) const {
    for (i64 k = rowptr[r]; k < rowptr[r + 1]; ++k)
      if (col[k] == c) return k;
    return -1;
  }
};

// Internal node order: y-strips (so periodic partners x=0 <-> x=1 share a strip and a rank),
// x-sorted inside a strip.  Ranks own contiguous strip ranges.
struct Ordering {
  std::vector<i32> new2old, old2new;
  std::vector<i64> strip_ptr;  // size S+1, internal-index start of each strip
  std::vector<double> cuts;    // S-1 increasing y values separating the strips
};
// y-strips holding equal node counts (cuts between distinct y values, so nodes of equal y -- the
// periodic partners -- share a strip), x-sorted inside a strip
void make_ordering(const HostMesh& m, int nstrips, Ordering& ord);
// the given strips (cut values) for every level of a hierarchy, so a node keeps its strip -- and its
// rank -- on every level it appears on
void make_ordering_cuts(const HostMesh& m, const std::vector<double>& cuts, Ordering& ord);
int auto_strips(i64 N);

// Node-adjacency pattern (incl. diagonal) in internal numbering, sorted columns.
// node -> incident triangles (internal ids; ascending triangle ids per node)
struct Incidence {
  std::vector<i64> ptr;
  std::vector<i32> tri;
};
void build_incidence(const HostMesh& m, const Ordering& ord, Incidence& I);
void build_pattern(const HostMesh& m, const Ordering& ord, Csr& P, const Incidence* I = nullptr);

struct Assembly {
  std::vector<double> K;     // on P (StokesColor.py:98-128), reference triangle order
  std::vector<double> Gx, Gy;// on P: lumped gradient/divergence coefficients (StokesColor.py:130-263)
  std::vector<double> M;     // lumped mass (StokesColor.py:266-284), internal numbering
  std::vector<double> asum;  // area_sum of calculate_divergence (|det| >= 1e-14 only)
};
void assemble_stokes(const HostMesh& m, const Ordering& ord, const Csr& P, Assembly& A, const Incidence* I = nullptr);

// poisson.py:100-146 in fp32 arithmetic (bit-exact), fp64 accumulation, then the literal
// periodic row-merge (poisson.py:187-213) and Dirichlet rows (poisson.py:258-278).
// Returns a CSR in internal numbering with its own pattern, plus the RHS.
void assemble_literal(const HostMesh& m, const Ordering& ord, const std::vector<float>& g_tri,
                      const std::vector<std::pair<i64, i64>>& op_pairs_old,
                      const std::vector<i32>& dir_nodes_old, const std::vector<double>& dir_vals,
                      double heat_dt /* <= 0: Poisson A; > 0: I + dt*A */, Csr& A,
                      std::vector<double>& b);

// P^T K P with identity slave rows (the well-posed pressure operator).
void build_pressure(const Csr& P, const std::vector<double>& K, const std::vector<i32>& dof,
                    const std::vector<i32>& slave_of, Csr& Pp);

// Partition of the internal index range into `world` contiguous strip ranges, balanced by nnz.
void partition_rows(const Csr& P, const Ordering& ord, int world, std::vector<i64>& row_start);

// Periodic (master, slave) pairs of a multigrid level (caller numbering): left x~0 node with the
// right x~L node of nearest y (ties: lowest index), masters on y=0|H dropped (StokesColor.py:449-457).
std::vector<std::pair<i64, i64>> level_pairs(const HostMesh& m, double L, double tol, double H);

// Prolongation level c -> level f (f = red refinement of c): rows = fine internal ids, cols = coarse
// internal ids mapped through the coarse periodic dof map; copies weight 1, edge midpoints 1/2+1/2;
// fine periodic slaves get empty rows (their merged value lives on the master).
void build_prolongation(i64 Nc, const std::vector<i32>& edge_a, const std::vector<i32>& edge_b,
                        const Ordering& of, const Ordering& oc, const std::vector<i32>& dof_c,
                        const std::vector<i32>& master_of_f, Csr& P);
void transpose(const Csr& A, i64 ncols, Csr& At);
// Dense inverse of a (regularised) SPD matrix, row-major n x n, by Cholesky.  Returns false if not SPD.
bool spd_inverse(std::vector<double>& A, i64 n);
// general dense inverse (LU with partial pivoting), in place; false when singular
bool lu_inverse(std::vector<double>& A, i64 n);

// Local view of one rank: owned rows [r0, r1) + sorted ghost list, local column ids.
struct LocalPlan {
  i64 r0 = 0, r1 = 0, n_own = 0, n_ghost = 0;
  std::vector<i32> ghost_global;        // internal ids, sorted
  std::vector<i32> ghost_owner;
  std::vector<i32> recv_peer;           // peers we receive from, ascending
  std::vector<i64> recv_off, recv_cnt;  // into the ghost region
  std::vector<i32> send_peer;
  std::vector<i64> send_off, send_cnt;
  std::vector<i32> send_local;          // owned local ids to pack, per peer contiguous
};
// patterns: every pattern whose columns must be resolved (P, Pp, ...)
void make_local_plan(const std::vector<const Csr*>& pats, const std::vector<i64>& row_start, int rank,
                     LocalPlan& lp);
// general form: each pattern reads THIS level's vectors through its columns, but its rows may be
// partitioned by another level's ranges (restriction rows live on the coarse level, ...)
struct PatRows {
  const Csr* A;
  const std::vector<i64>* rows;  // owner ranges of A's rows
};
// deep (optional): operator patterns (rows partitioned by row_start) whose rows ONE layer out -- the ghost rows
// adjacent to a rank's rows, "G1" -- the rank computes redundantly (Ctx: step pairs, residuals and last smoothing
// steps on W > 1 ranks with one exchange where two were needed).  Their columns ("G2") join the ghost set of every
// rank (and so the send lists), and g1_out receives this rank's G1 rows (sorted global ids).
void make_local_plan2(const std::vector<PatRows>& pats, const std::vector<i64>& row_start, int rank,
                      LocalPlan& lp, const std::vector<const Csr*>* deep = nullptr, std::vector<i32>* g1_out = nullptr);

// SELL-64: slices of 64 rows, per-slice width = max row length, entries column-major
// inside a slice (lane = row) so a wave's loads are contiguous.
struct Sell {
  i64 nrows = 0, nslices = 0, padded = 0;
  std::vector<i64> slice_off;  // nslices+1, entry offsets
  std::vector<i32> slice_w;
  std::vector<i32> col;        // local column ids
  // row list (lattice operators: the skeleton rows only), local output indices, padded to nslices*64
  // with -1; empty: slice s holds rows s*64 .. s*64+63
  std::vector<i32> rows;
  i64 nnz = 0;  // stored (unpadded) entries of the listed rows (build_sell_rows)
  // ghost rows appended by sell_append_ghost_rows (deep halos): entries k >= gk0 of `rows` are ghost rows, whose
  // operator rows are A's rows grow[k - gk0] (global ids; their `rows` entries are the local ghost indices);
  // nslices_own slices hold the rank's own rows (-1: no ghost rows)
  i64 gk0 = -1, nslices_own = -1;
  std::vector<i32> grow;
  // values of the ghost slices' entries when some ghost rows are not A's rows as stored (a face-interior row in its
  // face stencil's order and coefficients: the owner's arithmetic, bit for bit), laid out like col from
  // slice_off[nslices_own]; empty: every ghost row is A's row
  std::vector<double> gval;
  i64 global_row(i64 r0, i64 k) const { return gk0 >= 0 && k >= gk0 ? (i64)grow[k - gk0] : r0 + (i64)rows[k]; }
};
// SELL of the rows `rows` (offsets from r0 into A's rows; they are also the local output indices),
// columns resolved in `cols`; int32 columns only (rows are not contiguous)
void build_sell_rows(const Csr& A, i64 r0, const std::vector<i32>& rows, const LocalPlan& cols, Sell& S);
void sell_values_rows(const Csr& A, i64 r0, const Sell& S, const std::vector<double>& val, std::vector<double>& out);
// append the rows `grows` (global ids, each a ghost of `cols`) to a row-listed SELL as whole slices of their own:
// local output index = the ghost's local id, columns resolved in `cols`
// (rows_plan: the plan holding the rows as ghosts, when it is not the columns' -- a transfer between two levels)
// custom (optional): a ghost row's entries (global columns, values) in place of A's row when it returns true
using GhostRowFn = std::function<bool(i32 g, std::vector<i32>& cols, std::vector<double>& vals)>;
void sell_append_ghost_rows(const Csr& A, const std::vector<i32>& grows, const LocalPlan& cols, Sell& S,
                            const LocalPlan* rows_plan = nullptr, const GhostRowFn* custom = nullptr);
// the SELL image of A's rows in S (rows r0 + k, or r0 + S.rows[k]) with entry values f(r, e) computed in
// place (r: the row's global index, e: its CSR entry) -- no full-length value array for a SELL that
// holds only the lattice skeleton's rows
template <class F>
void sell_values_fn(const Csr& A, i64 r0, const Sell& S, F&& f, std::vector<double>& out) {
  out.assign(S.padded, 0.0);
  parallel_for(S.nslices, [&](i64 s0, i64 s1) {
    for (i64 s = s0; s < s1; ++s)
      for (i64 l = 0; l < 64; ++l) {
        const i64 k = s * 64 + l;
        if (S.rows.empty() ? k >= S.nrows : S.rows[k] < 0) continue;  // (row lists: padding lanes are -1)
        if (!S.gval.empty() && S.gk0 >= 0 && k >= S.gk0)
          throw std::runtime_error("sell_values_fn: ghost rows with their own values (use sell_values_rows)");
        const i64 r = S.rows.empty() ? r0 + k : S.global_row(r0, k);
        const i64 b = A.rowptr[r], len = A.rowptr[r + 1] - b;
        for (i64 e = 0; e < len; ++e) out[S.slice_off[s] + e * 64 + l] = f(r, b + e);
      }
  }, 64);
}

// ----------------------------------------------------------------------------- lattice layout
// Macro primitives (the coarse mesh of a red-refinement hierarchy: faces, edges, vertices), their
// strips and their order (pucfem_lattice.hpp).
struct Macro {
  i64 nv = 0, ne = 0, nf = 0;
  std::vector<double> x, y;     // coarse coordinates
  std::vector<i32> tri;         // 3 nf: A, B, C of every face (the coarse mesh's triangles, CCW)
  std::vector<i32> ev;          // 2 ne: edge endpoints (lo < hi)
  std::vector<i32> fe;          // 3 nf: edge ids of AB, AC, BC
  int S = 1;                    // strips
  std::vector<double> cuts;     // S - 1 increasing y values
  // strip-major order: per strip its faces, then its edges, then its vertices (x-sorted); pos_* the
  // position of a primitive in its kind's order, strip_* the first position of each strip (S + 1)
  std::vector<i32> order_f, order_e, order_v;
  std::vector<i32> strip_f, strip_e, strip_v;
};
// strips: 0 = auto; weights of the strip balance: interior / edge nodes at level `lw`
void build_macro(const HostMesh& coarse, int strips, int lw, Macro& M);

struct LatticeLevel {
  int l = 0;
  i32 n = 1, F = 0;               // segments per macro edge, interior nodes per face
  std::vector<i64> face_start;    // per face id: internal id of its first interior node
  std::vector<i64> edge_start;    // per edge id: internal id of its node k = 1 (from the lo endpoint)
  std::vector<i64> vert_start;    // per vertex id
  std::vector<uint8_t> type;      // per internal id: 0 face interior, 1 macro edge, 2 macro vertex
  // global internal id of point k (1..n-1, from the lo endpoint) of edge e
  i64 edge_node(i32 e, i32 k) const { return edge_start[e] + k - 1; }
};
// The internal ordering of level l of the hierarchy (ml = the coarse mesh red-refined l times):
// strip-major; in a strip the face interiors (lattice layout), the edges, the vertices.  Fills
// ord (new2old, old2new, strip_ptr, cuts) and LL.  Throws if a node is not on the lattice.
void lattice_ordering(const HostMesh& ml, const Macro& M, int l, Ordering& ord, LatticeLevel& LL);

// Face tables of one rank at one level: faces whose interiors are rows [r0, r0 + nrows) of the level
// (internal ids), local indices through the plan `lp` (owned + ghosts); dof: the periodic master map
// of the level (internal ids; null: the plain, unmerged table).  Returns the local face list (face ids).
std::vector<i32> lattice_faces(const Macro& M, const LatticeLevel& LL, i64 r0, i64 nrows);
void lattice_tabs(const Macro& M, const LatticeLevel& LL, const std::vector<i32>& faces, i64 row0,
                  const LocalPlan& lp, const std::vector<i32>* dof, std::vector<lat::FaceTab>& out);
// Coefficient records (lat::NCOEF doubles per face of `faces`) at level l
void lattice_coefs(const Macro& M, const std::vector<i32>& faces, int l, double dtnu, std::vector<double>& out);
// Implicit FEM dye advection-diffusion (scripts/good_visualization.py:700-718): the per-entry data of
// A = M + dt (C_u + D K) + diag(G) on the stiffness pattern P and of its periodic-merged form on Pp.
// mc: the consistent mass of every P entry (build_mass_and_convection, StokesColor.py:286-312,
// accumulated in triangle order); cptr / cw: per P entry the convection weights that sum into it,
// w index 3 t + j (triangle t, its vertex j = the column), ascending t; diag_row: the row of a
// diagonal P entry, else -1; eptr / ek: per Pp entry the P entries folded into it (the pair rows
// summed, slave columns onto the master's).  Triangles with |det| < 1e-14 contribute nothing.
// srow / sptr / sk / sc: the merged rows that hold P entries in a slave's column, with those entries
// and their slave columns (the right-hand side term of a dye field that is not periodic at the pairs).
struct DyeOp {
  std::vector<double> mc;
  std::vector<i64> cptr;
  std::vector<i32> cw;
  std::vector<i32> diag_row;
  std::vector<i64> eptr;
  std::vector<i32> ek;
  std::vector<i32> srow;
  std::vector<i64> sptr;
  std::vector<i32> sk, sc;
};
void build_dye(const HostMesh& m, const Ordering& ord, const Csr& P, const Csr& Pp, const std::vector<i32>& dof,
               DyeOp& D);

// Point location on the finest level of a lattice hierarchy (the semi-Lagrangian step): one SlFace per
// macro face (frame, face table in global internal ids of `ord`, corners, first fine triangle) and the
// cell table, per cell (i, j, s) of a face (lat::cell_index) the fine triangle's offset in its face
// and the rotation of its stored vertex order: (offset << 2) | rotation.  Built from face 0 and checked
// against the mesh's triangles on every face (throws if a face is numbered differently).
void lattice_locator(const Macro& M, const LatticeLevel& LL, const HostMesh& m, const Ordering& ord,
                     std::vector<lat::SlFace>& faces, std::vector<uint32_t>& cells);
// Host reference of the face stencils (CPU tests of the index arithmetic and the coefficients):
// kind 0 y = K x (K-type stencil), 1 = the lumped divergence numerator Gx ux + Gy uy (x: 2 vectors,
// x0 and x1), 2 = A_visc scaled (wsk: skeleton weights), 3 = prolongation rows (x0 on the coarse level
// through tab2, n2 = n / 2), 4 = restriction rows (x0 on the fine level through tab2, n2 = 2 n); writes
// the face rows of y only.
void lattice_apply_host(int kind, int n, const std::vector<lat::FaceTab>& tab, const std::vector<double>& coef,
                        const double* x0, const double* x1, const double* wsk, double* y,
                        const std::vector<lat::FaceTab>* tab2 = nullptr, int n2 = 0);
// rows [r0, r1) of `A` (global internal ids) -> local SELL; values extracted with sell_values().
void build_sell(const Csr& A, const LocalPlan& lp, Sell& S);
void sell_values(const Csr& A, const LocalPlan& lp, const Sell& S, const std::vector<double>& val,
                 std::vector<double>& out);
// int16 image of a square operator's SELL columns: col - (first row of the slice), taken modulo
// nloc (the local vector length) into [-32768, 32767], so ghost columns appended after the owned
// rows are reached from the first rows by wrapping below 0; rows past nrows point at the slice's
// first row.  false (out untouched) when some column is out of range.
bool sell_col16(const Sell& S, i64 nloc, std::vector<int16_t>& out);
// rows [r0, r0 + n) of A, columns resolved in `cols` (another level's plan)
// pad_self: padding entries point at their own row (square operators: keeps the band, see
// sell_col16); otherwise at column 0
void build_sell_x(const Csr& A, i64 r0, i64 n, const LocalPlan& cols, Sell& S, bool pad_self = false);
void sell_values_x(const Csr& A, i64 r0, const Sell& S, const std::vector<double>& val, std::vector<double>& out);
i32 to_local(const LocalPlan& lp, i32 g);

// Uniform grid of items (centroids / triangle bboxes) for the device point searches.
struct Grid {
  i32 nx = 1, ny = 1;
  double x0 = 0, y0 = 0, hx = 1, hy = 1;
  std::vector<i32> cell_start;  // nx*ny+1
  std::vector<i32> item;        // triangle ids
  std::vector<double> px, py;   // centroid coordinates per entry (centroid grid only)
};
void build_centroid_grid(const std::vector<double>& cx, const std::vector<double>& cy, double per_cell, Grid& G);
// per query point i: the squared distance to its k-th nearest centroid of the centroid grid G (self:
// the points are G's own centroids, and item i itself is skipped), rounded down to fp32; +inf when
// there are fewer than k
std::vector<float> knn_radius2(const Grid& G, const std::vector<double>& qx, const std::vector<double>& qy, int k,
                               bool self);
// per triangle t: the squared distance from its centroid to its k-th nearest OTHER centroid (G is
// the centroid grid of cx, cy), rounded down to fp32; +inf when there are fewer than k others
std::vector<float> centroid_knn_radius2(const Grid& G, const std::vector<double>& cx, const std::vector<double>& cy,
                                        int k);
// inflate > 0: each bbox grows by inflate * (its extent) + 1e-14 on every side, so a point that a
// rounding-sensitive weight test accepts on a triangle's edge is still listed with that triangle
void build_tri_grid(const std::vector<double>& x, const std::vector<double>& y, const std::vector<i32>& tri,
                    double per_cell, Grid& G, double inflate = 0.0);

}  // namespace pucfem
