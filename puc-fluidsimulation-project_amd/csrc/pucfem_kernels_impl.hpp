// Device kernels of libpucfem -- see pucfem_kernels.hpp for the layout / reduction conventions.
// Included by pucfem_api.hip (single translation unit for the device code).
#pragma once
#include <type_traits>

#include "pucfem_kernels.hpp"

namespace pucfem {
namespace dev {

// row-group sizes of face kernels (rows per thread loaded together, face_rows_k): compile-time, so A/B
// builds (tools/build_variant.sh) can measure them; the defaults are the measured choices
#ifndef PUCFEM_INIT_K
#define PUCFEM_INIT_K 2
#endif
#ifndef PUCFEM_VCHEB_K
#define PUCFEM_VCHEB_K 2
#endif
#ifndef PUCFEM_DIV_K
#define PUCFEM_DIV_K 2
#endif
// launch bounds of the gather kernels (k_cg_dir, k_vcheb, k_vcheb_pair, k_div, k_grad_proj, k_sl):
// PUCFEM_GATHER_WAVES = w > 0 asks for >= w waves per SIMD (a register cap), 0: the compiler's choice
#ifndef PUCFEM_GATHER_WAVES
#define PUCFEM_GATHER_WAVES 0
#endif
#if PUCFEM_GATHER_WAVES > 0
#define LB_GATHER __launch_bounds__(BS, PUCFEM_GATHER_WAVES)
#else
#define LB_GATHER __launch_bounds__(BS)
#endif
#ifndef PUCFEM_GRADP_K
#define PUCFEM_GRADP_K 4
#endif

// SELL row dot product (defined with the multigrid kernels below)
template <bool C16, typename T, typename VT, typename G>
__device__ __forceinline__ T sell_row_dot_g(const SellDev& A, const VT* __restrict__ val, const G& gx, int64_t s,
                                            int lane);

// ----------------------------------------------------------------------------- lattice face rows
// fn(F, lf, t, i, j) for the interior rows of the face part that block b of nbf runs (work items: chunks
// of BS consecutive rows of one face; the item index is block-uniform, so the face table entry and
// the coefficient record are scalar loads)
template <class Fn>
__device__ __forceinline__ void face_rows(const FaceDev& fc, int32_t b, int32_t nbf, Fn&& fn) {
  const int32_t items = fc.nf * fc.cpf;
  // one block per item (launches without partials): consecutive chunks of a face run on one XCD
  // (blocks are dealt round-robin over the 8 XCDs), so the rows a chunk shares with its neighbours
  // stay in that XCD's L2
  if (nbf == items && items >= 8 * 64) {
    // XCD x = b % 8 runs blocks x, x + 8, ...: K_x = items / 8 (+1 for x < items % 8) of them, which
    // take the x-th contiguous range of items (a bijection of [0, items))
    const int32_t x = b & 7, q = items >> 3, rem = items & 7;
    b = x * q + (x < rem ? x : rem) + (b >> 3);
    nbf = items + 1;  // one item, no further iteration
  }
  for (int32_t it = b; it < items; it += nbf) {
    const int32_t lf = it / fc.cpf;
    const int32_t t0 = (it - lf * fc.cpf) * (BS * FACE_RPT) + (int32_t)threadIdx.x;
    const lat::FaceTab F = fc.tab[lf];
    for (int32_t r = 0; r < FACE_RPT; ++r) {
      const int32_t t = t0 + r * BS;
      if (t < fc.F) {
        int32_t i, j;
        lat::coords(t, fc.n, fc.rinv, i, j);
        fn(F, lf, t, i, j);
      }
    }
  }
}

// The same work items as face_rows, handed to fn in groups of K rows of one thread (rows t0 + r BS):
// fn(F, lf, t[K], i[K], j[K], ok[K]) loads every row of the group before computing any, so the
// group's memory round trips overlap.  Rows past the face end are clamped to its last row (valid
// addresses; ok = false: not stored).
template <int K, class Fn>
__device__ __forceinline__ void face_rows_k(const FaceDev& fc, int32_t b, int32_t nbf, Fn&& fn) {
  static_assert(FACE_RPT % K == 0, "group size divides the rows per thread");
  const int32_t items = fc.nf * fc.cpf;
  if (nbf == items && items >= 8 * 64) {  // XCD-grouped item order (face_rows)
    const int32_t x = b & 7, q = items >> 3, rem = items & 7;
    b = x * q + (x < rem ? x : rem) + (b >> 3);
    nbf = items + 1;
  }
  for (int32_t it = b; it < items; it += nbf) {
    const int32_t lf = it / fc.cpf;
    const int32_t t0 = (it - lf * fc.cpf) * (BS * FACE_RPT) + (int32_t)threadIdx.x;
    const lat::FaceTab F = fc.tab[lf];
#pragma unroll
    for (int32_t g = 0; g < FACE_RPT; g += K) {
      if (t0 + g * BS >= fc.F) break;
      int32_t t[K], i[K], j[K];
      bool ok[K];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        const int32_t tt = t0 + (g + r) * BS;
        ok[r] = tt < fc.F;
        t[r] = ok[r] ? tt : fc.F - 1;
        lat::coords(t[r], fc.n, fc.rinv, i[r], j[r]);
      }
      fn(F, lf, t, i, j, ok);
    }
  }
}

// entries of an interior row of a stiffness-type face operator: a[0] the row's own, a[1 + k] its
// neighbour k (lat::neighbours order).  op 0: K (every level's operator, the merged pressure
// operator with the merged table); op 1: the Jacobi-scaled A_visc, S A S with s_f inside the face
// and the skeleton columns' s_j (0 for Dirichlet columns, StokesColor.py:473-475) from fc.wsk
template <typename T>
__device__ __forceinline__ void face_kcoefs(const FaceDev& fc, int32_t lf, const int32_t (&nb)[6],
                                            const bool (&in)[6], T (&a)[7]) {
  if constexpr (std::is_same<T, float>::value) {
    const float* c = fc.coef32 + lf * lat::NCOEF;
    a[0] = c[lat::C_KD];
    a[1] = a[2] = c[lat::C_KAB];
    a[3] = a[4] = c[lat::C_KAC];
    a[5] = a[6] = c[lat::C_KBC];
  } else {
    const double* c = fc.coef + lf * lat::NCOEF;
    const double k3[3] = {c[lat::C_KAB], c[lat::C_KAC], c[lat::C_KBC]};
    if (fc.op == 1) {
      const double vs = c[lat::C_VS], g = vs * c[lat::C_DTNU];
      a[0] = vs * c[lat::C_VD] * vs;
#pragma unroll
      // (under a branch: loading wsk at every neighbour cost the viscous pair 308 -> 353 us, r12e)
      for (int k = 0; k < 6; ++k) a[1 + k] = (g * k3[k >> 1]) * (in[k] ? vs : fc.wsk[nb[k]]);
    } else {
      a[0] = c[lat::C_KD];
#pragma unroll
      for (int k = 0; k < 6; ++k) a[1 + k] = k3[k >> 1];
    }
  }
}

// the lumped gradient stencil of an interior row applied to x: (sum_j Gx_ij x_j, sum_j Gy_ij x_j)
__device__ __forceinline__ void face_grad(const double* c, const int32_t (&nb)[6], const double* __restrict__ x,
                                          double& gx, double& gy) {
  const double d1 = x[nb[1]] - x[nb[0]], d2 = x[nb[2]] - x[nb[3]], d3 = x[nb[4]] - x[nb[5]];
  gx = c[lat::C_G1X] * d1 + c[lat::C_G2X] * d2 + c[lat::C_G3X] * d3;
  gy = c[lat::C_G1Y] * d1 + c[lat::C_G2Y] * d2 + c[lat::C_G3Y] * d3;
}
// the same from the six neighbour values v[k] = x[nb[k]] (loaded beforehand)
__device__ __forceinline__ void face_grad_v(const double* c, const double (&v)[6], double& gx, double& gy) {
  const double d1 = v[1] - v[0], d2 = v[2] - v[3], d3 = v[4] - v[5];
  gx = c[lat::C_G1X] * d1 + c[lat::C_G2X] * d2 + c[lat::C_G3X] * d3;
  gy = c[lat::C_G1Y] * d1 + c[lat::C_G2Y] * d2 + c[lat::C_G3Y] * d3;
}

// ----------------------------------------------------------------------------- SpMV
// y = A x over owned rows (generic; unit `pucfem_apply`, residuals).
template <bool C16>
__global__ __launch_bounds__(BS) void k_spmv(SellDev A, FaceDev fc, const double* __restrict__ val,
                                             const double* __restrict__ x, double* __restrict__ y) {
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    face_rows(fc, role.idx, fc.nb, [&](const lat::FaceTab& F, int32_t lf, int32_t t, int32_t i, int32_t j) {
      int32_t nb[6];
      bool in[6];
      lat::neighbours(F, fc.n, t, i, j, nb, in);
      double a[7];
      face_kcoefs(fc, lf, nb, in, a);
      double acc = a[0] * x[F.base + t];
#pragma unroll
      for (int k = 0; k < 6; ++k) acc += a[1 + k] * x[nb[k]];
      stnt(y + F.base + t, acc);
    });
    return;
  }
  int64_t s0, s1;
  block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
  const int lane = threadIdx.x & 63, wv = wave_id();
  for (int64_t s = s0 + wv; s < s1; s += 4) {
    const int64_t off = A.off[s];
    const int w = A.w[s];
    const int64_t row = sell_row(A, s, lane);
    const int32_t base = (int32_t)(s * 64);
    double acc = 0.0;
    for (int k = 0; k < w; ++k) {
      const int64_t e = off + (int64_t)k * 64 + lane;
      acc += val[e] * x[sell_col<C16, false>(A, e, base)];
    }
    if (row >= 0) stnt(y + row, acc);
  }
}

// ----------------------------------------------------------------------------- CG (Jacobi-scaled)
// The solver works on A^ = S A S (S = diag(1/sqrt(a_ii))), so Jacobi-PCG is plain CG on A^.
// Per iteration two kernels:
//   dir: beta = rr/rr_prev; p_new = r + beta p_old (recomputed at the gathered columns, so no
//        separate direction pass); q = A^ p_new; partial <p_new, q>
//   upd: alpha = rr/<p,q>; y += alpha p; r -= alpha q; partial <r, r>
// scal layout (doubles): [0..NR) rr_prev slot 0, [4..4+NR) rr_prev slot 1, [8..8+NR) bb, [12..12+NR) rr_cur
// ctl layout (ints):    [0] 0 running / 1 converged / 2 maxit, [1] iterations
template <int NR>
struct CgVecs {
  double* y[NR];
  double* r[NR];
  double* po[NR];
  double* pn[NR];
  double* q[NR];
  const double* b[NR];
  const float* zf[NR];  // k_cg_dir<..., ZF = true>: the gathered residual in fp32 (the fp32 V-cycle's z)
};
// the residual k_cg_dir gathers: r (fp64) or, ZF, the fp32-exact preconditioned residual
template <bool ZF, int NR>
__device__ __forceinline__ double cg_rg(const CgVecs<NR>& v, int c, int64_t j) {
  if constexpr (ZF) return (double)v.zf[c][j];
  else return v.r[c][j];
}

// r32 (optional): fp32 copy of r for the mixed-precision V-cycle, whose right-hand side is only
// ever used in fp32 (bit-identical to converting inside the cycle, at half the bytes per read)
// write_p: also p = r into v.po (the first direction of k_cgr_dir / k_cgr_upd)
template <int NR, bool C16>
__global__ __launch_bounds__(BS) void k_cg_init(SellDev A, FaceDev fc, const double* __restrict__ val, CgVecs<NR> v,
                                                int64_t n_ghost, double* part_rr, double* part_bb,
                                                float* __restrict__ r32 = nullptr, int write_p = 0,
                                                RedOut ro = RedOut{}) {
  __shared__ double sh[4];
  double rr[NR], bb[NR];
#pragma unroll
  for (int c = 0; c < NR; ++c) rr[c] = bb[c] = 0.0;
  auto finish = [&](int64_t row, const double (&acc)[NR]) {
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      const double b = v.b[c][row];
      const double r = b - acc[c];
      stnt(v.r[c] + row, r);
      if (r32) stnt(r32 + row, (float)r);
      if (write_p) stnt(v.po[c] + row, r);
      rr[c] += r * r;
      bb[c] += b * b;
    }
  };
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    // groups of K rows per thread, every gathered value of a group loaded first (face_rows_k)
    constexpr int K = face_k(NR == 1 ? PUCFEM_INIT_K : 2);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      int32_t nb[K][6];
      bool in[K][6];
#pragma unroll
      for (int r = 0; r < K; ++r) lat::neighbours(F, fc.n, t[r], i[r], j[r], nb[r], in[r]);
      double a[K][7];
#pragma unroll
      for (int r = 0; r < K; ++r) face_kcoefs(fc, lf, nb[r], in[r], a[r]);
      double yv[K][NR][7];
#pragma unroll
      for (int r = 0; r < K; ++r) {
#pragma unroll
        for (int c = 0; c < NR; ++c) {
          yv[r][c][6] = v.y[c][F.base + t[r]];
#pragma unroll
          for (int k = 0; k < 6; ++k) yv[r][c][k] = v.y[c][nb[r][k]];
        }
      }
#pragma unroll
      for (int r = 0; r < K; ++r) {
        if (!ok[r]) continue;
        double acc[NR];
#pragma unroll
        for (int c = 0; c < NR; ++c) {
          acc[c] = a[r][0] * yv[r][c][6];
#pragma unroll
          for (int k = 0; k < 6; ++k) acc[c] += a[r][1 + k] * yv[r][c][k];
        }
        finish(F.base + t[r], acc);
      }
    });
  } else {
    int64_t s0, s1;
    block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
    const int lane = threadIdx.x & 63, wv = wave_id();
    for (int64_t s = s0 + wv; s < s1; s += 4) {
      const int64_t off = A.off[s];
      const int w = A.w[s];
      const int64_t row = sell_row(A, s, lane);
      const int32_t base = (int32_t)(s * 64);
      double acc[NR];
#pragma unroll
      for (int c = 0; c < NR; ++c) acc[c] = 0.0;
      // every column / value load of the slice before the gathers (k_cg_dir's form), summed in k order
      by_width(w, [&](auto wc) {
        constexpr int WN = decltype(wc)::value;
        if constexpr (WN > 0) {
          int32_t cj[WN];
          double av[WN];
#pragma unroll
          for (int k = 0; k < WN; ++k) {
            const int64_t e = off + (int64_t)k * 64 + lane;
            av[k] = val[e];
            cj[k] = sell_col<C16, false>(A, e, base);
          }
#pragma unroll
          for (int k = 0; k < WN; ++k) {
#pragma unroll
            for (int c = 0; c < NR; ++c) acc[c] += av[k] * v.y[c][cj[k]];
          }
        } else {
          for (int k = 0; k < w; ++k) {
            const int64_t e = off + (int64_t)k * 64 + lane;
            const double a = val[e];
            const int32_t j = sell_col<C16, false>(A, e, base);
#pragma unroll
            for (int c = 0; c < NR; ++c) acc[c] += a * v.y[c][j];
          }
        }
      });
      if (row >= 0) finish(row, acc);
    }
  }
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    const double t = block_sum(rr[c], sh);
    const double u = block_sum(bb[c], sh);
    if (threadIdx.x == 0) {
      if (ro.out) {  // fused reduction: <r, r> values 0 .. NR-1, <b, b> values NR .. 2 NR - 1 of part_rr
        red_part(ro, part_rr, c, t);
        red_part(ro, part_rr, NR + c, u);
      } else {
        part_rr[c * MAXB + blockIdx.x] = t;
        part_bb[c * MAXB + blockIdx.x] = u;
      }
    }
  }
  red_finish(ro, part_rr, sh);
}

// One SELL slice of q = A^ (r + beta p_old): WMAX > 0 unrolls the entry loop (all index/value
// loads issued before the dependent gathers); NT streams the matrix with non-temporal loads so it
// does not evict the gathered vectors from L2 / MALL.
template <int NR, int WMAX, bool NT, bool C16, bool ZF = false>
__device__ __forceinline__ void dir_slice(const SellDev& A, const double* __restrict__ val, const CgVecs<NR>& v,
                                          const double (&beta)[NR], bool first, int64_t s, int lane,
                                          double (&pq)[NR]) {
  const int64_t off = A.off[s];
  const int w = A.w[s];
  const int64_t row = sell_row(A, s, lane);
  const int32_t base = (int32_t)(s * 64);
  double acc[NR];
#pragma unroll
  for (int c = 0; c < NR; ++c) acc[c] = 0.0;
  auto generic = [&]() {
    for (int k = 0; k < w; ++k) {
      const int64_t e = off + (int64_t)k * 64 + lane;
      const double a = NT ? ldnt(val + e) : val[e];
      const int32_t j = sell_col<C16, NT>(A, e, base);
#pragma unroll
      for (int c = 0; c < NR; ++c) acc[c] += a * (cg_rg<ZF>(v, c, j) + beta[c] * (first ? 0.0 : v.po[c][j]));
    }
  };
  if constexpr (WMAX > 0) {
    by_width(w, [&](auto wc) {
      constexpr int WN = decltype(wc)::value;
      if constexpr (WN > 0) {
        int32_t cj[WN];
        double a[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          cj[k] = sell_col<C16, NT>(A, e, base);
          a[k] = NT ? ldnt(val + e) : val[e];
        }
#pragma unroll
        for (int k = 0; k < WN; ++k) {
#pragma unroll
          for (int c = 0; c < NR; ++c) acc[c] += a[k] * (cg_rg<ZF>(v, c, cj[k]) + beta[c] * (first ? 0.0 : v.po[c][cj[k]]));
        }
      } else {
        generic();
      }
    });
  } else {
    generic();
  }
  if (row >= 0) {
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      const double p = cg_rg<ZF>(v, c, row) + beta[c] * (first ? 0.0 : v.po[c][row]);
      stnt(v.pn[c] + row, p);
      stnt(v.q[c] + row, acc[c]);
      pq[c] += p * acc[c];
    }
  }
}

#ifndef PUCFEM_DIR_K1
#define PUCFEM_DIR_K1 2
#endif
#ifndef PUCFEM_DIR_K2
#define PUCFEM_DIR_K2 1
#endif
template <int NR, int WMAX, bool NT, bool C16, bool ZF = false>
__global__ LB_GATHER void k_cg_dir(SellDev A, FaceDev fc, const double* __restrict__ val, CgVecs<NR> v,
                                               int64_t n_ghost, const double* part_rr, int nb_rr, int stride_rr,
                                               const double* part_bb, int nb_bb, int stride_bb, double* scal,
                                               int* ctl, int it, int maxit, double tol2, double* part_pq,
                                               const double* part_cv = nullptr, int nb_cv = 0, int stride_cv = 0,
                                               RedOut ro = RedOut{}) {
  // part_rr: numerator of beta (<r,r> for CG, <r,z> for preconditioned CG); part_cv (if given):
  // <r,r> for the convergence test; part_bb: <b,b>.
  __shared__ double sh[4];
  if (ctl[0]) return;
  double rr[NR], bb[NR], beta[NR];
  bool conv = true, bad = false;
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    rr[c] = reduce_partials(part_rr + c * stride_rr, nb_rr, sh);
    bb[c] = it == 0 ? reduce_partials(part_bb + c * stride_bb, nb_bb, sh) : scal[8 + c];
    const double cv = part_cv ? reduce_partials(part_cv + c * stride_cv, nb_cv, sh) : rr[c];
    conv = conv && (cv <= tol2 * bb[c]);
    bad = bad || !isfinite(rr[c]) || !isfinite(cv);
  }
  if (conv || bad || it >= maxit) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      ctl[0] = conv ? 1 : (bad ? 3 : 2);
      ctl[1] = it;
    }
    return;
  }
#pragma unroll
  for (int c = 0; c < NR; ++c) beta[c] = it == 0 ? 0.0 : rr[c] / scal[(it & 1) * 4 + c];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      scal[((it + 1) & 1) * 4 + c] = rr[c];
      scal[12 + c] = rr[c];
      if (it == 0) scal[8 + c] = bb[c];
    }
  }
  double pq[NR];
#pragma unroll
  for (int c = 0; c < NR; ++c) pq[c] = 0.0;
  // the first iteration's direction is r itself: p_old is neither read nor needed (k_cg_init does not
  // clear it; a uniform branch skips its loads)
  const bool first = it == 0;
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    // groups of K rows per thread, every load of the group first (face_rows_k)
    constexpr int K = face_k(NR == 1 ? PUCFEM_DIR_K1 : PUCFEM_DIR_K2);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      int32_t nb[K][6];
      bool in[K][6];
#pragma unroll
      for (int r = 0; r < K; ++r) lat::neighbours(F, fc.n, t[r], i[r], j[r], nb[r], in[r]);
      double a[K][7];
#pragma unroll
      for (int r = 0; r < K; ++r) face_kcoefs(fc, lf, nb[r], in[r], a[r]);
      double rv[K][NR][7], pv[K][NR][7];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        const int64_t row = F.base + t[r];
#pragma unroll
        for (int c = 0; c < NR; ++c) {
          rv[r][c][6] = cg_rg<ZF>(v, c, row);
          pv[r][c][6] = first ? 0.0 : v.po[c][row];
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            rv[r][c][k] = cg_rg<ZF>(v, c, nb[r][k]);
            pv[r][c][k] = first ? 0.0 : v.po[c][nb[r][k]];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < K; ++r) {
        if (!ok[r]) continue;
        const int64_t row = F.base + t[r];
#pragma unroll
        for (int c = 0; c < NR; ++c) {
          double g[6];
#pragma unroll
          for (int k = 0; k < 6; ++k) g[k] = rv[r][c][k] + beta[c] * pv[r][c][k];
          const double p = rv[r][c][6] + beta[c] * pv[r][c][6];
          double q = a[r][0] * p;
#pragma unroll
          for (int k = 0; k < 6; ++k) q += a[r][1 + k] * g[k];
          stnt(v.pn[c] + row, p);
          stnt(v.q[c] + row, q);
          pq[c] += p * q;
        }
      }
    });
  } else {
    int64_t s0, s1;
    block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
    const int lane = threadIdx.x & 63, wv = wave_id();
    for (int64_t s = s0 + wv; s < s1; s += 4) dir_slice<NR, WMAX, NT, C16, ZF>(A, val, v, beta, first, s, lane, pq);
  }
  for (int64_t g = A.n_own + (int64_t)blockIdx.x * BS + threadIdx.x; g < A.n_own + n_ghost;
       g += (int64_t)gridDim.x * BS) {
#pragma unroll
    for (int c = 0; c < NR; ++c) v.pn[c][g] = cg_rg<ZF>(v, c, g) + beta[c] * (first ? 0.0 : v.po[c][g]);
  }
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    const double t = block_sum(pq[c], sh);
    if (threadIdx.x == 0) red_part(ro, part_pq, c, t);
  }
  red_finish(ro, part_pq, sh);
}

template <int NR>
__global__ __launch_bounds__(BS) void k_cg_upd(CgVecs<NR> v, int64_t nrows, const double* part_pq, int nb_pq,
                                               int stride_pq, const double* scal, const int* ctl, double* part_rr,
                                               float* __restrict__ r32 = nullptr, RedOut ro = RedOut{},
                                               double* __restrict__ vacc = nullptr, int vfirst = 0) {
  // vacc (NR = 1, optional): the correction sum_k alpha_k p_k accumulated beside y (the projection's v);
  // vfirst: the solve's first update, which starts the sum (no read of the buffer)
  __shared__ double sh[4];
  if (ctl[0]) return;
  double alpha[NR], rr[NR];
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    const double pq = reduce_partials(part_pq + c * stride_pq, nb_pq, sh);
    alpha[c] = scal[12 + c] / pq;
    rr[c] = 0.0;
  }
  int64_t r0, r1;
  block_rows(nrows, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      const double pi = v.pn[c][i];
      stnt(v.y[c] + i, v.y[c][i] + alpha[c] * pi);
      if (NR == 1 && vacc) stnt(vacc + i, vfirst ? alpha[c] * pi : vacc[i] + alpha[c] * pi);
      const double r = v.r[c][i] - alpha[c] * v.q[c][i];
      stnt(v.r[c] + i, r);
      if (NR == 1 && r32) stnt(r32 + i, (float)r);
      rr[c] += r * r;
    }
  }
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    const double t = block_sum(rr[c], sh);
    if (threadIdx.x == 0) red_part(ro, part_rr, c, t);
  }
  red_finish(ro, part_rr, sh);
}

// ----------------------------------------------------------------------------- single-reduction PCG
// Chronopoulos-Gear PCG (one all-reduce per iteration, the multi-rank pressure solves; PUCFEM_CGCG=1 forces it on
// one rank).  Iteration i, from r_i, p_(i-1), s_(i-1) = A p_(i-1):
//   z_i = M r_i (the V-cycle; its last smoothing step writes the <r_i, z_i> partials),  w_i = A z_i  (k_cgcg_w),
//   ONE reduction of the 8 values [rho_i, <r_i, s_(i-1)>, <s_(i-1), s_(i-1)>  (k_cgcg_upd of iteration i-1, exact),
//                                  gamma_i = <r_i, z_i>, delta_i = <w_i, z_i>, <r_i, w_i>, <w_i, w_i>, <w_i, s_(i-1)>]
//   beta = gamma_i / gamma_(i-1), alpha = gamma_i / (delta_i - beta gamma_i / alpha_(i-1))      (k_cgcg_coef),
//   p_i = z_i + beta p_(i-1), s_i = w_i + beta s_(i-1), y += alpha p_i, r_(i+1) = r_i - alpha s_i  (k_cgcg_upd).
// The convergence test of r_(i+1) comes from the same reduction: rho_(i+1) = rho_i - 2 alpha <r_i, s_i> +
// alpha^2 <s_i, s_i>, with <r_i, s_i> = <r_i, w_i> + beta <r_i, s_(i-1)> and <s_i, s_i> = <w_i, w_i> +
// 2 beta <w_i, s_(i-1)> + beta^2 <s_(i-1), s_(i-1)> -- exact dots, one step of recurrence (relative error
// ~eps rho_i / rho_(i+1)); rho_i itself is the exact lagged value.  Per iteration against the three reductions of
// the standard form: one all-reduce instead of three, 24 B/row more (s, w).
// Partial layout: value v at part[v * MAXB + block], one grid (nb blocks) for all producers.
constexpr int CGCG_NV = 8;
template <bool C16, bool ZF>
__global__ LB_GATHER void k_cgcg_w(SellDev A, FaceDev fc, const double* __restrict__ val, const double* __restrict__ z,
                                   const float* __restrict__ zf, const double* __restrict__ r,
                                   const double* __restrict__ s_old, double* __restrict__ w, double* part,
                                   const int* ctl) {
  __shared__ double sh[4];
  if (ctl[0]) return;
  auto zg = [&](int64_t j) -> double {
    if constexpr (ZF) return (double)zf[j];
    else return z[j];
  };
  double d[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // delta, <r, w>, <w, w>, <w, s_old>
  auto finish = [&](int64_t row, double q) {
    stnt(w + row, q);
    d[0] += zg(row) * q;
    d[1] += r[row] * q;
    d[2] += q * q;
    if (s_old) d[3] += q * s_old[row];
  };
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    constexpr int K = face_k(PUCFEM_DIR_K1);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      int32_t nb[K][6];
      bool in[K][6];
#pragma unroll
      for (int q = 0; q < K; ++q) lat::neighbours(F, fc.n, t[q], i[q], j[q], nb[q], in[q]);
      double a[K][7];
#pragma unroll
      for (int q = 0; q < K; ++q) face_kcoefs(fc, lf, nb[q], in[q], a[q]);
      double zv[K][7];
#pragma unroll
      for (int q = 0; q < K; ++q) {
        zv[q][6] = zg(F.base + t[q]);
#pragma unroll
        for (int k = 0; k < 6; ++k) zv[q][k] = zg(nb[q][k]);
      }
#pragma unroll
      for (int q = 0; q < K; ++q) {
        if (!ok[q]) continue;
        double acc = a[q][0] * zv[q][6];
#pragma unroll
        for (int k = 0; k < 6; ++k) acc += a[q][1 + k] * zv[q][k];
        finish(F.base + t[q], acc);
      }
    });
  } else {
    int64_t s0, s1;
    block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
    const int lane = threadIdx.x & 63, wv = wave_id();
    for (int64_t sl = s0 + wv; sl < s1; sl += 4) {
      const int64_t off = A.off[sl];
      const int wd = A.w[sl];
      const int64_t row = sell_row(A, sl, lane);
      const int32_t base = (int32_t)(sl * 64);
      double acc = 0.0;
      by_width(wd, [&](auto wc) {
        constexpr int WN = decltype(wc)::value;
        if constexpr (WN > 0) {
          int32_t cj[WN];
          double av[WN];
#pragma unroll
          for (int k = 0; k < WN; ++k) {
            const int64_t e = off + (int64_t)k * 64 + lane;
            cj[k] = sell_col<C16, false>(A, e, base);
            av[k] = val[e];
          }
#pragma unroll
          for (int k = 0; k < WN; ++k) acc += av[k] * zg(cj[k]);
        } else {
          for (int k = 0; k < wd; ++k) {
            const int64_t e = off + (int64_t)k * 64 + lane;
            acc += val[e] * zg(sell_col<C16, false>(A, e, base));
          }
        }
      });
      if (row >= 0) finish(row, acc);
    }
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const double t = block_sum(d[v], sh);
    if (threadIdx.x == 0) part[(4 + v) * MAXB + blockIdx.x] = t;
  }
}

// the scalars of iteration `it` from the 8 reduced values (red8; bb: <b, b>); state sc: [0] alpha_it, [1] beta_it,
// [2] gamma_it, [3] alpha_(it-1), [4] gamma_(it-1).  ctl: {1, it} when rho_it passes (no update), {1, it + 1} when
// the recurrence rho_(it+1) passes (the update of `it` completes the solve), {3, it} not finite, {2, it} maxit
__global__ void k_cgcg_coef(const double* __restrict__ red8, const double* __restrict__ bb, double* sc, double tol2,
                            int* ctl, int it, int maxit, const double* rho0) {
  if (threadIdx.x != 0 || blockIdx.x != 0 || ctl[0]) return;
  const double rho = it == 0 ? rho0[0] : red8[0];
  const double rs_old = it == 0 ? 0.0 : red8[1], ss_old = it == 0 ? 0.0 : red8[2];
  const double gamma = red8[3], delta = red8[4], rw = red8[5], ww = red8[6], ws = it == 0 ? 0.0 : red8[7];
  const double b2 = bb[0];
  if (!isfinite(rho) || !isfinite(gamma) || !isfinite(delta)) {
    ctl[0] = 3;
    ctl[1] = it;
    return;
  }
  if (rho <= tol2 * b2) {
    ctl[0] = 1;
    ctl[1] = it;
    return;
  }
  if (it >= maxit) {
    ctl[0] = 2;
    ctl[1] = it;
    return;
  }
  const double beta = it == 0 ? 0.0 : gamma / sc[4];
  const double alpha = it == 0 ? gamma / delta : gamma / (delta - beta * gamma / sc[3]);
  const double rs = rw + beta * rs_old, ss = ww + 2.0 * beta * ws + beta * beta * ss_old;
  const double rho1 = rho - 2.0 * alpha * rs + alpha * alpha * ss;
  sc[0] = alpha;
  sc[1] = beta;
  sc[3] = alpha;
  sc[4] = gamma;
  // the recurrence's estimate decides only when it is resolved: its rounding error is ~eps (rho + 2 |alpha rs| +
  // alpha^2 ss), so a value within a few of those (or negative, from cancellation) says nothing about the accepted
  // iterate -- the next iteration's exact lagged rho decides then
  const double floor1 = 16.0 * 2.220446049250313e-16 * (rho + 2.0 * fabs(alpha * rs) + alpha * alpha * ss);
  if (rho1 > floor1 && rho1 <= tol2 * b2) {
    ctl[0] = 1;
    ctl[1] = it + 1;
  }
}

// the update of iteration `it` (skipped when the solve converged before it); partials of rho_(it+1),
// <r_(it+1), s_it>, <s_it, s_it> into values 0..2 of part (the next iteration's exact lagged values)
template <bool ZF>
__global__ __launch_bounds__(BS) void k_cgcg_upd(int64_t n, const double* __restrict__ z, const float* __restrict__ zf,
                                                 const double* __restrict__ w, double* __restrict__ p,
                                                 double* __restrict__ s, double* __restrict__ y, double* __restrict__ r,
                                                 float* __restrict__ r32, double* __restrict__ vacc,
                                                 const double* __restrict__ sc, const int* ctl, int it, double* part) {
  __shared__ double sh[4];
  if (ctl[0] && ctl[1] <= it) return;
  const double alpha = sc[0], beta = sc[1];
  const bool first = it == 0;
  double d0 = 0.0, d1 = 0.0, d2 = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
    double zi;
    if constexpr (ZF) zi = (double)zf[i];
    else zi = z[i];
    const double pi = zi + (first ? 0.0 : beta * p[i]);
    const double si = w[i] + (first ? 0.0 : beta * s[i]);
    stnt(p + i, pi);
    stnt(s + i, si);
    stnt(y + i, y[i] + alpha * pi);
    if (vacc) stnt(vacc + i, first ? alpha * pi : vacc[i] + alpha * pi);
    const double rn = r[i] - alpha * si;
    stnt(r + i, rn);
    if (r32) stnt(r32 + i, (float)rn);
    d0 += rn * rn;
    d1 += rn * si;
    d2 += si * si;
  }
  const double t0 = block_sum(d0, sh), t1 = block_sum(d1, sh), t2 = block_sum(d2, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = t0;
    part[MAXB + blockIdx.x] = t1;
    part[2 * MAXB + blockIdx.x] = t2;
  }
}

// ----------------------------------------------------------------------------- solution projection
// Successive right-hand sides (Fischer 1998): the pressure solves of consecutive steps keep an
// A-orthonormal basis X of their recent solution directions; the initial guess is the A-orthogonal
// projection of the new solution onto span X, x0 = sum_i <X_i, b> X_i.  X: m vectors at stride ld.
constexpr int PROJ_MAX = 32;
// Storage of the basis vectors: fp32.  The guess only has to start the CG close to the solution (its
// relative residual is 1e-6 .. 1e-5 against the solve's rtol 1e-8), and rounding the A-orthonormal
// directions to fp32 perturbs their A-inner products by ~1e-7, below that; the dots and the
// combinations are formed in fp64.  Halves the two passes over the basis (2 m vector reads per solve).
#ifdef PUCFEM_PROJ_F64
using ProjT = double;  // (A/B variant: the basis in fp64)
#else
using ProjT = float;
#endif
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef float flt2 __attribute__((ext_vector_type(2)));

// Basis layout.  PUCFEM_PROJ_TILED (default): tiles of 64 rows, inside a tile each of the basis' kcap vectors holds
// 64 consecutive values -- element (i, r) at ((r / 64) kcap + i) 64 + r % 64, ld = kcap: a wave's 64 rows of all
// vectors are one contiguous block (one DRAM stream instead of one per vector), a new vector's 64 values one
// 256-B segment.  0: column-major, (i, r) at i ld + r, ld = the vector stride
#ifndef PUCFEM_PROJ_TILED
#define PUCFEM_PROJ_TILED 1
#endif
__host__ __device__ __forceinline__ int64_t pxi(int i, int64_t r, int64_t ld) {
#if PUCFEM_PROJ_TILED
  return (((r >> 6) * ld + i) << 6) + (r & 63);
#else
  return (int64_t)i * ld + r;
#endif
}
// basis re-seeding: out_i = sum_j q[i][j] X_j (i < kq <= PROJ_KEEP_MAX, j < m), one pass over X.
// Q: the re-seed coefficients in device memory, row-major [PROJ_KEEP_MAX][PROJ_MAX] (block-uniform loads)
constexpr int PROJ_KEEP_MAX = 16;
struct QMat {
  double q[PROJ_KEEP_MAX][PROJ_MAX];
};
// The re-seed coefficients are staged in LDS once per block (uniform loads of all 16 x 32 of them per row from
// device memory: 1.18 ms at L7 in-step, r10z; isolated 0.77 ms with LDS, r11q, where all 32 basis loads issued first
// and then the sums took 1.93 ms); the per-row operations and their order are unchanged
__global__ __launch_bounds__(BS) void k_reseed(int64_t n, const ProjT* __restrict__ X, int64_t ld, int m,
                                               const double* __restrict__ Q, int kq, ProjT* __restrict__ out) {
  __shared__ double q[PROJ_KEEP_MAX * PROJ_MAX];
  for (int t = threadIdx.x; t < PROJ_KEEP_MAX * PROJ_MAX; t += BS) q[t] = Q[t];
  __syncthreads();
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) {
    double acc[PROJ_KEEP_MAX];
#pragma unroll
    for (int i = 0; i < PROJ_KEEP_MAX; ++i) acc[i] = 0.0;
    for (int j = 0; j < m; ++j) {
      const double x = (double)X[pxi(j, r, ld)];
#pragma unroll
      for (int i = 0; i < PROJ_KEEP_MAX; ++i) acc[i] += q[i * PROJ_MAX + j] * x;
    }
#pragma unroll
    for (int i = 0; i < PROJ_KEEP_MAX; ++i)
      if (i < kq) out[pxi(i, r, ld)] = (ProjT)acc[i];
  }
}

// deferred projection update + guess (Ctx::project_guess), pass 1: partial dots of the M basis
// vectors with b and A v, and <v, b>, <v, A v>, the sums of v and b over the free (non-slave) rows
// (master_of null: no null space, zero); stride MAXB per value, order
// [<X_i, b> (M), <X_i, A v> (M), <v, b>, <v, A v>, sum_free v, sum_free b].  One instance per M:
// the M loads of a row are unconditional (all in flight together); grid-stride rows keep the
// resident waves on one compact window of every vector.
// The last solve's direction may still be pending: then A v = r0 - r_final is formed here from the solve's initial
// and final residuals (av holds r0, D.rf the final one) -- the operations k_diff2_fin would have stored, so the
// same values -- instead of being read.  v itself is the CG's accumulated correction sum_k alpha_k p_k
// (k_cg_upd's vacc, D.v) after a projected guess: the same vector as y - x0 in exact arithmetic, but y - x0
// formed from the two stored fp64 vectors carries their rounding, whose A-norm is not small against a
// correction of ~1e-8 of y (at L7, A x of a rounded smooth field has a relative noise of ~1e-8 of b): A v
// from the residuals then does not match that v, the new direction is mis-normalised and the basis decays
// (driver-window rtol 5e-8 runs went from 0-1 to 6 iterations per solve, profiles/r11_projection.txt).
// Without D.v (the first direction, whose guess was 0): v = D.y - D.x0.
// the pressure right-hand side formed in k_mdot2 from the divergence (k_pres_rhs's operations on the unscaled
// multigrid path: slaves merged into their masters, zero at slave rows, the mean over the free rows removed) and
// stored for the solve; braw null: k_mdot2 reads the stored b
struct RhsIn {
  const double* braw;
  const int32_t* slave_of;
  const double* sum;  // sum of braw (a reduced scalar)
  double inv_nfree;
  double* bh;
};
struct PendDir {
  const double* y;   // the last solve's solution (with x0; used when v is null)
  const double* x0;  // its guess
  const double* rf;  // its final residual (null: A v was stored in av)
  const double* v;   // its accumulated correction (null: y - x0, or the stored v)
};
// Virtual blocks (nvb > 0): the rows and partials are those of a grid of nvb blocks (virtual block vb: rows
// vb BS + t + k nvb BS, its partials at index vb), run by a smaller grid whose blocks take virtual blocks vb =
// blockIdx.x, + gridDim.x, ... one after another -- the same sums in the same order, so the same bits, on a grid the
// chip holds at once (at 96 VGPRs 1,280 of the 2,048 blocks are resident: the rest ran as a second, partial round)
template <int M>
__global__ __launch_bounds__(BS) void k_mdot2(int64_t n, const ProjT* __restrict__ X, int64_t ld,
                                              const double* __restrict__ b, const double* __restrict__ av,
                                              const double* __restrict__ v, const int32_t* __restrict__ master_of,
                                              double* part, RedOut ro, PendDir D, RhsIn R = RhsIn{}, int nvb = 0) {
  constexpr int NA = 2 * M + 4;
  __shared__ double sh[NA][4];
  const double mean = R.braw ? R.sum[0] * R.inv_nfree : 0.0;
  const int V = nvb > 0 ? nvb : (int)gridDim.x;
  const int64_t step = (int64_t)V * BS;
  for (int vb = blockIdx.x; vb < V; vb += gridDim.x) {
  double acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = 0.0;
  for (int64_t r = (int64_t)vb * BS + threadIdx.x; r < n; r += step) {
    double br;
    if (R.braw) {  // (k_pres_rhs's row)
      if (master_of[r] >= 0) {
        br = 0.0;
      } else {
        br = R.braw[r];
        if (R.slave_of[r] >= 0) br += R.braw[R.slave_of[r]];
        br = br - mean;
      }
      stnt(R.bh + r, br);
    } else {
      br = b[r];
    }
    const double ar = D.rf ? av[r] - D.rf[r] : av[r];
    const double vr = D.v ? D.v[r] : (D.y ? D.y[r] - D.x0[r] : (v ? v[r] : 0.0));  // (all null: v = 0)
    ProjT x[M > 0 ? M : 1];
#pragma unroll
    for (int i = 0; i < M; ++i) x[i] = X[pxi(i, r, ld)];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      acc[i] += (double)x[i] * br;
      acc[M + i] += (double)x[i] * ar;
    }
    acc[2 * M] += vr * br;
    acc[2 * M + 1] += vr * ar;
    if (master_of && master_of[r] < 0) {
      acc[2 * M + 2] += vr;
      acc[2 * M + 3] += br;
    }
  }
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const double t = wave_sum(acc[i]);
    if ((threadIdx.x & 63) == 0) sh[i][threadIdx.x >> 6] = t;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NA; i += BS) {
    const double t = (sh[i][0] + sh[i][1]) + (sh[i][2] + sh[i][3]);
    if (nvb > 0) part[(int64_t)i * MAXB + vb] = t;  // (virtual blocks: the plain partials, no fused reduction)
    else red_part(ro, part, i, t);
  }
  __syncthreads();  // (sh is reused by the next virtual block)
  }
  red_finish(ro, part, sh[0], true);  // (several waves stored partials)
}

// pass 1 -> coefficients (one thread).  D: the reduced dots of k_mdot2 over m vectors; kq >= 0: the
// basis was re-seeded, X' = Q X (kq rows), so <X'_i, .> = Q <X, .>.  Out (m' = kq or m):
// [a (m'), c (m'), s, mu, alpha] with a_i = <X_i, b>, c_i = <X_i, A v>,
// s = (<v, A v> - |c|^2)^-1/2 (0 when v lies in span X to 1e-10 relative: a null direction),
// mu = sum_free v / n_free, alpha = <X_m, b> = s (<v, b> - mu sum_free b - <c, a>).
__global__ void k_pcoef(const double* __restrict__ D, int m, const double* __restrict__ Q, int kq, double inv_nfree,
                        double* K) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int mp = kq >= 0 ? kq : m;
  double q = 0.0, ca = 0.0;
  for (int i = 0; i < mp; ++i) {
    double a = 0.0, c = 0.0;
    if (kq >= 0) {
      for (int j = 0; j < m; ++j) {
        a += Q[i * PROJ_MAX + j] * D[j];
        c += Q[i * PROJ_MAX + j] * D[m + j];
      }
    } else {
      a = D[i];
      c = D[m + i];
    }
    K[i] = a;
    K[mp + i] = c;
    q += c * c;
    ca += c * a;
  }
  const double vb = D[2 * m], vav = D[2 * m + 1], vs = D[2 * m + 2], bs = D[2 * m + 3];
  const double den = vav - q;
  const double s = den > 1e-10 * vav && den > 0.0 ? 1.0 / sqrt(den) : 0.0;
  const double mu = vs * inv_nfree;
  K[2 * mp] = s;
  K[2 * mp + 1] = mu;
  K[2 * mp + 2] = s * (vb - mu * bs - ca);
}

// pass 2: the new direction X_M = s (v - mu 1_free - sum_i c_i X_i) and the guess
// x0 = sum_i a_i X_i + alpha X_M (written to y, and to x0 when given), one pass over the M basis vectors.
// v: the stored or accumulated direction, or with yp non-null v = yp - x0 (the first direction) from the last
// solve's solution and its guess, each row read before this row's new values are written.  vz (optional): the
// next solve's correction accumulator, cleared (it may be v's buffer: each row reads v first)
template <int M>
__global__ __launch_bounds__(BS) void k_pcomb(int64_t n, const ProjT* __restrict__ X, int64_t ld,
                                              const double* __restrict__ K, const double* v,
                                              const int32_t* __restrict__ master_of, ProjT* __restrict__ xm_out,
                                              double* y, double* x0, const double* yp, double* vz) {
  double ka[M > 0 ? M : 1], kc[M > 0 ? M : 1];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    ka[i] = K[i];
    kc[i] = K[M + i];
  }
  const double s = K[2 * M], mu = K[2 * M + 1], alpha = K[2 * M + 2];
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) {
    ProjT x[M > 0 ? M : 1];
#pragma unroll
    for (int i = 0; i < M; ++i) x[i] = X[pxi(i, r, ld)];
    const double vr = yp ? yp[r] - x0[r] : (v ? v[r] : 0.0);  // (both null: v = 0)
    double sa = 0.0, sc = 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      sa += ka[i] * (double)x[i];
      sc += kc[i] * (double)x[i];
    }
    const double xm = s * (vr - ((master_of && master_of[r] < 0) ? mu : 0.0) - sc);
    const double g = sa + alpha * xm;
    stnt(xm_out + pxi(0, r, ld), (ProjT)xm);  // (xm_out: the basis at the new vector's column)
    stnt(y + r, g);
    if (x0) stnt(x0 + r, g);
    if (vz) stnt(vz + r, 0.0);
  }
}

__global__ void k_diff(int64_t n, const double* __restrict__ a, const double* __restrict__ b, double* __restrict__ out) {
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) stnt(out + r, a[r] - b[r]);
}

// out = a - b (when out is given) and out2 = a2 - b2 (out2 may alias a2: each row reads before it writes)
__global__ void k_diff2(int64_t n, const double* __restrict__ a, const double* __restrict__ b, double* __restrict__ out,
                        const double* a2, const double* __restrict__ b2, double* out2) {
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) {
    const double x2 = a2[r], y2 = b2[r];
    if (out) stnt(out + r, a[r] - b[r]);
    stnt(out2 + r, x2 - y2);
  }
}

// k_diff2 and the pressure solve's finish (k_cg_fin with master_of, unscaled) in one pass: the projection's
// v = y - x0 (when v is given; else v is the CG's accumulated correction) and A v = a2 - r_final, and p = y with
// every periodic slave row copied from its master
__global__ void k_diff2_fin(int64_t n, const double* __restrict__ y, const double* __restrict__ x0,
                            double* __restrict__ v, const double* a2, const double* __restrict__ rf, double* av,
                            const int32_t* __restrict__ master_of, double* __restrict__ p) {
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) {
    const double yr = y[r], a = a2[r], f = rf[r];
    const int32_t m = master_of[r];
    const double pr = m >= 0 ? y[m] : yr;
    if (v) stnt(v + r, yr - x0[r]);
    stnt(av + r, a - f);
    p[r] = pr;
  }
}

// ----------------------------------------------------------------------------- CG, direction updated in place
// Jacobi-scaled CG (no preconditioner: the viscous solve, the Jacobi pressure path) with the direction
// formed in the update kernel instead of at the direction kernel's gathered columns: the SpMV then
// gathers one vector per right-hand side (p) instead of two (r and p_old).  beta needs <r_new, r_new>
// before r_new exists; it comes from the recurrence <r - a q, r - a q> = rr - 2 a <r, q> + a^2 <q, q>
// with the direction kernel's dots (relative error ~ eps * rr / rr_new, ~1e-12 here); the convergence
// test keeps the exact <r_new, r_new> of the update's partials, and so does the next alpha.
//   dir: q = A^ p; partials <p, q>, <r, q>, <q, q>          (stride MAXB, [c], [NR + c], [2 NR + c])
//   upd: a = rr / <p, q>; y += a p; r -= a q; p = r + b p; partial <r, r>
template <int NR, bool C16>
__global__ __launch_bounds__(BS) void k_cgr_dir(SellDev A, FaceDev fc, const double* __restrict__ val, CgVecs<NR> v,
                                                const int* ctl, double* part) {
  __shared__ double sh[4];
  if (ctl[0]) return;
  double pq[NR], rq[NR], qq[NR];
#pragma unroll
  for (int c = 0; c < NR; ++c) pq[c] = rq[c] = qq[c] = 0.0;
  auto finish = [&](int c, double p, double r, double q, int64_t row) {
    stnt(v.q[c] + row, q);
    pq[c] += p * q;
    rq[c] += r * q;
    qq[c] += q * q;
  };
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    constexpr int K = face_k(NR == 1 ? 4 : 2);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      int32_t nb[K][6];
      bool in[K][6];
#pragma unroll
      for (int r = 0; r < K; ++r) lat::neighbours(F, fc.n, t[r], i[r], j[r], nb[r], in[r]);
      double a[K][7];
#pragma unroll
      for (int r = 0; r < K; ++r) face_kcoefs(fc, lf, nb[r], in[r], a[r]);
      double pv[K][NR][7], rv[K][NR];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        const int64_t row = F.base + t[r];
#pragma unroll
        for (int c = 0; c < NR; ++c) {
          pv[r][c][6] = v.po[c][row];
          rv[r][c] = v.r[c][row];
#pragma unroll
          for (int k = 0; k < 6; ++k) pv[r][c][k] = v.po[c][nb[r][k]];
        }
      }
#pragma unroll
      for (int r = 0; r < K; ++r) {
        if (!ok[r]) continue;
#pragma unroll
        for (int c = 0; c < NR; ++c) {
          double q = a[r][0] * pv[r][c][6];
#pragma unroll
          for (int k = 0; k < 6; ++k) q += a[r][1 + k] * pv[r][c][k];
          finish(c, pv[r][c][6], rv[r][c], q, F.base + t[r]);
        }
      }
    });
  } else {
    int64_t s0, s1;
    block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
    const int lane = threadIdx.x & 63, wv = wave_id();
    for (int64_t s = s0 + wv; s < s1; s += 4) {
      const int64_t row = sell_row(A, s, lane);
      const int64_t rr = row >= 0 ? row : 0;
      double acc[NR], pr[NR], rr_[NR];
#pragma unroll
      for (int c = 0; c < NR; ++c) {
        pr[c] = v.po[c][rr];
        rr_[c] = v.r[c][rr];
      }
      if constexpr (NR == 1) {
        acc[0] = sell_row_dot_g<C16, double>(A, val, [&](int32_t j) { return v.po[0][j]; }, s, lane);
      } else {
        const int64_t off = A.off[s];
        const int w = A.w[s];
        const int32_t base = (int32_t)(s * 64);
#pragma unroll
        for (int c = 0; c < NR; ++c) acc[c] = 0.0;
        by_width(w, [&](auto wc) {
          constexpr int WN = decltype(wc)::value;
          if constexpr (WN > 0) {
            int32_t cj[WN];
            double av[WN];
#pragma unroll
            for (int k = 0; k < WN; ++k) {
              const int64_t e = off + (int64_t)k * 64 + lane;
              cj[k] = sell_col<C16>(A, e, base);
              av[k] = ldnt(val + e);
            }
#pragma unroll
            for (int k = 0; k < WN; ++k) {
#pragma unroll
              for (int c = 0; c < NR; ++c) acc[c] += av[k] * v.po[c][cj[k]];
            }
          } else {
            for (int k = 0; k < w; ++k) {
              const int64_t e = off + (int64_t)k * 64 + lane;
              const double av = ldnt(val + e);
              const int32_t j = sell_col<C16>(A, e, base);
#pragma unroll
              for (int c = 0; c < NR; ++c) acc[c] += av * v.po[c][j];
            }
          }
        });
      }
      if (row >= 0) {
#pragma unroll
        for (int c = 0; c < NR; ++c) finish(c, pr[c], rr_[c], acc[c], row);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    const double t1 = block_sum(pq[c], sh);
    const double t2 = block_sum(rq[c], sh);
    const double t3 = block_sum(qq[c], sh);
    if (threadIdx.x == 0) {
      part[(int64_t)c * MAXB + blockIdx.x] = t1;
      part[(int64_t)(NR + c) * MAXB + blockIdx.x] = t2;
      part[(int64_t)(2 * NR + c) * MAXB + blockIdx.x] = t3;
    }
  }
}

// dots: the reduced [<p, q> (NR), <r, q> (NR), <q, q> (NR)]; rr: the reduced exact <r, r> (NR)
template <int NR>
__global__ __launch_bounds__(BS) void k_cgr_upd(CgVecs<NR> v, int64_t nrows, const double* __restrict__ dots,
                                                const double* __restrict__ rr, const int* ctl, double* part_rr) {
  __shared__ double sh[4];
  if (ctl[0]) return;
  double alpha[NR], beta[NR], acc[NR];
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    const double r0 = rr[c], pq = dots[c], rq = dots[NR + c], qq = dots[2 * NR + c];
    alpha[c] = r0 / pq;
    const double r1 = r0 - 2.0 * alpha[c] * rq + alpha[c] * alpha[c] * qq;
    beta[c] = r0 > 0.0 ? fmax(r1, 0.0) / r0 : 0.0;
    acc[c] = 0.0;
  }
  int64_t r0, r1;
  block_rows(nrows, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      const double p = v.po[c][i], q = v.q[c][i];
      stnt(v.y[c] + i, v.y[c][i] + alpha[c] * p);
      const double r = v.r[c][i] - alpha[c] * q;
      stnt(v.r[c] + i, r);
      stnt(v.po[c] + i, r + beta[c] * p);
      acc[c] += r * r;
    }
  }
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    const double t = block_sum(acc[c], sh);
    if (threadIdx.x == 0) part_rr[(int64_t)c * MAXB + blockIdx.x] = t;
  }
}

// ----------------------------------------------------------------------------- Chebyshev iteration (viscous)
// The Jacobi-scaled A_visc (unit diagonal) has its spectrum inside the Gershgorin interval [1 - R, 1 + R]
// with R = max_i sum_{j != i} |A^_ij| (~0.02: A_visc = I + DT nu K, condition ~1.04), so the Chebyshev
// iteration on that interval converges at a guaranteed rate (T_k(1 / R) ~ (2 / R)^k / 2: ~100x per step)
// with no inner products.  One kernel per step:
//   r = b - A^ x_in;  d = c1 d + c2 r;  x_out = x_in + d;  partial <r, r> (and <b, b> at the first step)
// Only the first step writes partials (<r_0, r_0>, <b, b>); the host derives the step count K from the
// residual bound |r_K| <= |r_0| / T_K(sigma) (Ctx::vcheb) and runs steps 1 .. K-1 without reductions.
// first: c1 = 0 (d is not read).
// d, the Chebyshev increment, is stored in fp32: x_out = x_in + d takes the fp64 value, and the next
// step's d = c1 d + c2 r only damps the stored one (c1 < 1), so the rounding perturbs the polynomial by
// ~1e-7 of a shrinking correction -- 16 of the 80 B/row saved
// The solver's vectors interleave the x and y components of u (dbl2: one 16-B gather per neighbour where
// the two components were two 8-B gathers; round 4 lab, tools/vlayout_lab.hip: the face-row step 215 ->
// 170 us warm, 252 -> 221 us cold at L7 size); u and u* themselves stay SoA.
// (dbl2 / flt2: the 16-B / 8-B vector types defined with ProjT above)
struct ChebVecs2 {
  const dbl2* xin;
  dbl2* xout;
  const dbl2* b;
  const flt2* d;
  // non-null: the new d goes here instead of in place (the skeleton half of a step pair, k_vcheb_pair)
  flt2* dout;
  // the solve's last step with k_visc_fin folded in (us[0] non-null): instead of d and x_out it writes
  // u* = s x_out and the fp32 increment u* - u (the same operations as k_visc_fin: bit-identical)
  const double* s;
  const double* u[2];
  double* us[2];
  float* inc[2];
};
template <bool C16>
__global__ LB_GATHER void k_vcheb(SellDev A, FaceDev fc, const double* __restrict__ val, ChebVecs2 v,
                                              double c1, double c2, int first, const int* ctl, double* part_rr,
                                              double* part_bb, RedOut ro = RedOut{}) {
  __shared__ double sh[4];
  if (ctl[0]) return;
  double rr[2] = {0.0, 0.0}, bb[2] = {0.0, 0.0};
  const bool fin = v.us[0] != nullptr;
  flt2* dout = v.dout ? v.dout : const_cast<flt2*>(v.d);
  // row: r = b - A^ x (both components), d = c1 d + c2 r, x_out = x + d
  // own: the row adds to the partials (not a ghost row one layer out, deep halos)
  auto finish = [&](int64_t row, dbl2 ax, dbl2 x0, dbl2 br, flt2 dr, bool own = true) {
    const double r0 = br.x - ax.x, r1 = br.y - ax.y;
    const double dn0 = first ? c2 * r0 : c1 * (double)dr.x + c2 * r0;
    const double dn1 = first ? c2 * r1 : c1 * (double)dr.y + c2 * r1;
    if (fin) {
      const double s = v.s[row];
      const double a0 = s * (x0.x + dn0), a1 = s * (x0.y + dn1);
      stnt(reinterpret_cast<dbl2*>(v.us[0]) + row, dbl2{a0, a1});  // (interleaved u*)
      stnt(v.inc[0] + row, (float)(a0 - v.u[0][VS * row]));
      stnt(v.inc[1] + row, (float)(a1 - v.u[1][VS * row]));
    } else {
      const flt2 dn = {(float)dn0, (float)dn1};
      const dbl2 xo = {x0.x + dn0, x0.y + dn1};
      stnt(dout + row, dn);
      stnt(v.xout + row, xo);
    }
    if (!own) return;
    rr[0] += r0 * r0;
    rr[1] += r1 * r1;
    bb[0] += br.x * br.x;
    bb[1] += br.y * br.y;
  };
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    constexpr int K = face_k(PUCFEM_VCHEB_K);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      int32_t nb[K][6];
      bool in[K][6];
#pragma unroll
      for (int r = 0; r < K; ++r) lat::neighbours(F, fc.n, t[r], i[r], j[r], nb[r], in[r]);
      double a[K][7];
#pragma unroll
      for (int r = 0; r < K; ++r) face_kcoefs(fc, lf, nb[r], in[r], a[r]);
      dbl2 xv[K][7], bv[K];
      flt2 dv[K];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        const int64_t row = F.base + t[r];
        xv[r][6] = v.xin[row];
        bv[r] = v.b[row];
        dv[r] = first ? flt2{0.0f, 0.0f} : v.d[row];
#pragma unroll
        for (int k = 0; k < 6; ++k) xv[r][k] = v.xin[nb[r][k]];
      }
#pragma unroll
      for (int r = 0; r < K; ++r) {
        if (!ok[r]) continue;
        double ax0 = a[r][0] * xv[r][6].x, ax1 = a[r][0] * xv[r][6].y;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          ax0 += a[r][1 + k] * xv[r][k].x;
          ax1 += a[r][1 + k] * xv[r][k].y;
        }
        finish(F.base + t[r], dbl2{ax0, ax1}, xv[r][6], bv[r], dv[r]);
      }
    });
  } else {
    int64_t s0, s1;
    block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
    const int lane = threadIdx.x & 63, wv = wave_id();
    for (int64_t s = s0 + wv; s < s1; s += 4) {
      const int64_t row = sell_row(A, s, lane);
      const int64_t rw = row >= 0 ? row : 0;
      const dbl2 x0 = v.xin[rw], br = v.b[rw];
      const flt2 dr = first ? flt2{0.0f, 0.0f} : v.d[rw];
      double acc0 = 0.0, acc1 = 0.0;
      const int64_t off = A.off[s];
      const int w = A.w[s];
      const int32_t base = (int32_t)(s * 64);
      by_width(w, [&](auto wc) {
        constexpr int WN = decltype(wc)::value;
        if constexpr (WN > 0) {
          int32_t cj[WN];
          double av[WN];
#pragma unroll
          for (int k = 0; k < WN; ++k) {
            const int64_t e = off + (int64_t)k * 64 + lane;
            cj[k] = sell_col<C16>(A, e, base);
            av[k] = ldnt(val + e);
          }
#pragma unroll
          for (int k = 0; k < WN; ++k) {
            const dbl2 xj = v.xin[cj[k]];
            acc0 += av[k] * xj.x;
            acc1 += av[k] * xj.y;
          }
        } else {
          for (int k = 0; k < w; ++k) {
            const int64_t e = off + (int64_t)k * 64 + lane;
            const double av = ldnt(val + e);
            const dbl2 xj = v.xin[sell_col<C16>(A, e, base)];
            acc0 += av * xj.x;
            acc1 += av * xj.y;
          }
        }
      });
      if (row >= 0) finish(row, dbl2{acc0, acc1}, x0, br, dr, row < A.n_own);
    }
  }
  if (!part_rr) return;  // steps after the first: no residual norms needed (the step count is known)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const double t1 = block_sum(rr[c], sh);
    const double t2 = part_bb ? block_sum(bb[c], sh) : 0.0;
    if (threadIdx.x == 0) {
      if (ro.out) {  // fused reduction: |r_0|^2 values 0 .. 1, |b|^2 values 2 .. 3 of part_rr
        red_part(ro, part_rr, c, t1);
        red_part(ro, part_rr, 2 + c, t2);
      } else {
        part_rr[(int64_t)c * MAXB + blockIdx.x] = t1;
        if (part_bb) part_bb[(int64_t)c * MAXB + blockIdx.x] = t2;
      }
    }
  }
  red_finish(ro, part_rr, sh);
}

// Step pairs (temporal blocking through LDS): a block owns one work item (BS * FACE_RPT consecutive rows of
// one face) and runs step a on its rows and on their in-face neighbours (every in-face neighbour of lattice
// row t lies within n - 1 offsets of t: the window [t0 - n, t1 + n)), keeping x_{a+1} in LDS, then step
// a + 1 on its own rows.  The skeleton rows run their two steps in k_vcheb launches (SELL part only) before
// and after; the face kernel writes x_{a+1} at its rows next to the skeleton, which the second one gathers.
// Row for row k_vcheb's operations in k_vcheb's order (d rounded to fp32 between the steps): bit-identical
// to two single steps.
struct VPairVecs {
  const dbl2* xa;  // x_a (every row)
  dbl2* xb;        // x_{a+1}: read at skeleton rows, written at the face rows next to the skeleton
  dbl2* xc;        // x_{a+2}
  const dbl2* b;
  const flt2* da;  // d_a
  flt2* dc;        // d_{a+2}
  // the solve's last step (us[0] non-null): u* = s x_{a+2} and the fp32 increment instead of xc, dc
  const double* s;
  const double* u[2];
  double* us[2];
  float* inc[2];
};
constexpr int VP_HALO = 256;  // window rows on each side: n <= VP_HALO (lattice size of the face)
// A step pair's second-step neighbour: from the LDS window (in-face neighbour; lw clamped into the window), else
// the global x_{a+1} at a skeleton row.  The LDS value is read unconditionally and the global one under the
// branch: written as `in ? lds[lw] : glob[g]`, the compiler merges the two loads into one generic (flat) load of
// a selected address, which is slower than ds_read for every row although only the rows next to the skeleton
// take the global path.
// (the empty asm pins the LDS value in registers before the branch, so the loads cannot be merged)
__device__ __forceinline__ void pin_reg(float& x) { asm("" : "+v"(x)); }
__device__ __forceinline__ void pin_reg(dbl2& x) { asm("" : "+v"(x.x), "+v"(x.y)); }
template <typename T>
__device__ __forceinline__ T pair_nbr(const T* lds, int32_t lw, const T* glob, int64_t g, bool in) {
#ifdef PUCFEM_PAIR_SELECT_LOAD  // (A/B: the merged form)
  return in ? lds[lw] : glob[g];
#else
  T x = lds[lw];
  pin_reg(x);
  if (!in) x = glob[g];
  return x;
#endif
}
constexpr int VP_W = BS * FACE_RPT + 2 * VP_HALO;
constexpr int VP_WK = (VP_W + BS - 1) / BS;
#ifndef PUCFEM_VP_G
#define PUCFEM_VP_G 1
#endif
constexpr int VP_G = PUCFEM_VP_G;  // rows of a thread loaded together (compile-time: an A/B knob)
static_assert(VP_WK % VP_G == 0, "the window rows of a thread go in groups");
// first: step a is the solve's step 0 (d_a is not read: c1a = 0) and the block also writes the partials of
// |r_0|^2 and |b|^2 over its own rows into part_r0 / part_b0 (values c at c * MAXB + part_off + block, as
// k_vcheb's first step does for the skeleton rows at their own block indices)
__global__ LB_GATHER void k_vcheb_pair(FaceDev fc, VPairVecs v, double c1a, double c2a, double c1b,
                                                   double c2b, const int* ctl, double* part_rr, int32_t part_off,
                                                   int first = 0, double* part_r0 = nullptr,
                                                   double* part_b0 = nullptr) {
  __shared__ dbl2 lx[VP_W];
  __shared__ double sh[4];
  if (ctl[0]) return;
  const int32_t items = fc.nf * fc.cpf;
  int32_t it = blockIdx.x;
  if ((int32_t)gridDim.x == items && items >= 8 * 64) {  // XCD-grouped item order (face_rows)
    const int32_t x = it & 7, q = items >> 3, rem = items & 7;
    it = x * q + (x < rem ? x : rem) + (it >> 3);
  }
  const int32_t lf = it / fc.cpf;
  const lat::FaceTab F = fc.tab[lf];
  const int32_t n = fc.n;
  const int32_t t0 = (it - lf * fc.cpf) * (BS * FACE_RPT), t1 = min(t0 + BS * FACE_RPT, fc.F);
  const int32_t w0 = max(0, t0 - n), nw = min(fc.F, t1 + n) - w0;
  const bool fin = v.us[0] != nullptr;
  // step a on the window; b and the fp32 d_{a+1} of the rows stay in registers for step a + 1.  Rows
  // go in groups of VP_G with every load of the group first (k_vcheb's row groups); a row past the
  // window is clamped to the window's first row (a valid address; not stored)
  dbl2 bt[VP_WK];
  flt2 dt[VP_WK];
  double r00 = 0.0, r01 = 0.0, b00 = 0.0, b01 = 0.0;  // (first) |r_0|^2, |b|^2 over the block's own rows
#pragma unroll
  for (int k0 = 0; k0 < VP_WK; k0 += VP_G) {
    if (k0 * BS >= nw) break;
    int32_t nb[VP_G][6];
    bool in[VP_G][6], ok[VP_G];
    int64_t row[VP_G];
    dbl2 xv[VP_G][7], br[VP_G];
    flt2 dr[VP_G];
#pragma unroll
    for (int r = 0; r < VP_G; ++r) {
      const int32_t w = (int32_t)threadIdx.x + (k0 + r) * BS;
      ok[r] = w < nw;
      const int32_t t = w0 + (ok[r] ? w : 0);
      int32_t i, j;
      lat::coords(t, n, fc.rinv, i, j);
      lat::neighbours(F, n, t, i, j, nb[r], in[r]);
      row[r] = F.base + t;
      xv[r][6] = v.xa[row[r]];
#pragma unroll
      for (int q = 0; q < 6; ++q) xv[r][q] = v.xa[nb[r][q]];
      br[r] = v.b[row[r]];
      dr[r] = first ? flt2{0.0f, 0.0f} : v.da[row[r]];
    }
#pragma unroll
    for (int r = 0; r < VP_G; ++r) {
      double a[7];
      face_kcoefs(fc, lf, nb[r], in[r], a);
      const int32_t w = (int32_t)threadIdx.x + (k0 + r) * BS;
      double ax0 = a[0] * xv[r][6].x, ax1 = a[0] * xv[r][6].y;
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        ax0 += a[1 + q] * xv[r][q].x;
        ax1 += a[1 + q] * xv[r][q].y;
      }
      const double ra0 = br[r].x - ax0, ra1 = br[r].y - ax1;
      // (k_vcheb's first step: dn = c2 r; the general form with c1a = 0 and d = 0 is the same value)
      const double dn0 = first ? c2a * ra0 : c1a * (double)dr[r].x + c2a * ra0;
      const double dn1 = first ? c2a * ra1 : c1a * (double)dr[r].y + c2a * ra1;
      if (ok[r]) lx[w] = dbl2{xv[r][6].x + dn0, xv[r][6].y + dn1};
      if (first && ok[r] && w0 + w >= t0 && w0 + w < t1) {
        r00 += ra0 * ra0;
        r01 += ra1 * ra1;
        b00 += br[r].x * br[r].x;
        b01 += br[r].y * br[r].y;
      }
      bt[k0 + r] = br[r];
      dt[k0 + r] = flt2{(float)dn0, (float)dn1};
    }
  }
  __syncthreads();
  // step a + 1 on the item's own rows (in groups as above)
  double rr0 = 0.0, rr1 = 0.0;
#pragma unroll
  for (int k0 = 0; k0 < VP_WK; k0 += VP_G) {
    if (k0 * BS >= nw) break;
    int32_t nb[VP_G][6];
    bool in[VP_G][6], ok[VP_G];
    int32_t wr[VP_G];
    dbl2 xv[VP_G][7];
#pragma unroll
    for (int r = 0; r < VP_G; ++r) {
      const int32_t w = (int32_t)threadIdx.x + (k0 + r) * BS;
      ok[r] = w < nw && w0 + w >= t0 && w0 + w < t1;
      wr[r] = ok[r] ? w : t0 - w0;
      const int32_t t = w0 + wr[r];
      int32_t i, j;
      lat::coords(t, n, fc.rinv, i, j);
      lat::neighbours(F, n, t, i, j, nb[r], in[r]);
      xv[r][6] = lx[wr[r]];
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const int32_t lw = min(max(nb[r][q] - F.base - w0, 0), nw - 1);
        xv[r][q] = pair_nbr(lx, lw, v.xb, nb[r][q], in[r][q]);
      }
    }
#pragma unroll
    for (int r = 0; r < VP_G; ++r) {
      if (!ok[r]) continue;
      double a[7];
      face_kcoefs(fc, lf, nb[r], in[r], a);
      const int64_t row = F.base + w0 + wr[r];
      bool bnd = false;
#pragma unroll
      for (int q = 0; q < 6; ++q) bnd = bnd || !in[r][q];
      double ax0 = a[0] * xv[r][6].x, ax1 = a[0] * xv[r][6].y;
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        ax0 += a[1 + q] * xv[r][q].x;
        ax1 += a[1 + q] * xv[r][q].y;
      }
      const double rs0 = bt[k0 + r].x - ax0, rs1 = bt[k0 + r].y - ax1;
      const double dn0 = c1b * (double)dt[k0 + r].x + c2b * rs0;
      const double dn1 = c1b * (double)dt[k0 + r].y + c2b * rs1;
      if (bnd) v.xb[row] = xv[r][6];
      if (fin) {
        const double s = v.s[row];
        const double au0 = s * (xv[r][6].x + dn0), au1 = s * (xv[r][6].y + dn1);
        stnt(reinterpret_cast<dbl2*>(v.us[0]) + row, dbl2{au0, au1});  // (interleaved u*)
        stnt(v.inc[0] + row, (float)(au0 - v.u[0][VS * row]));
        stnt(v.inc[1] + row, (float)(au1 - v.u[1][VS * row]));
      } else {
        stnt(v.dc + row, flt2{(float)dn0, (float)dn1});
        stnt(v.xc + row, dbl2{xv[r][6].x + dn0, xv[r][6].y + dn1});
      }
      rr0 += rs0 * rs0;
      rr1 += rs1 * rs1;
    }
  }
  if (first && part_r0) {  // |r_0|^2 and |b|^2 partials of the solve's step 0
    const double p0 = block_sum(r00, sh), p1 = block_sum(r01, sh);
    const double q0 = block_sum(b00, sh), q1 = block_sum(b01, sh);
    if (threadIdx.x == 0) {
      part_r0[part_off + blockIdx.x] = p0;
      part_r0[(int64_t)MAXB + part_off + blockIdx.x] = p1;
      part_b0[part_off + blockIdx.x] = q0;
      part_b0[(int64_t)MAXB + part_off + blockIdx.x] = q1;
    }
  }
  if (!part_rr) return;  // |r_{a+1}|^2 partials for the a-posteriori check
  const double ta = block_sum(rr0, sh);
  const double tb = block_sum(rr1, sh);
  if (threadIdx.x == 0) {
    part_rr[part_off + blockIdx.x] = ta;
    part_rr[(int64_t)MAXB + part_off + blockIdx.x] = tb;
  }
}

// the recurrence CG's control after an update: converged (1), maxit (2), not finite (3); it = the
// iterations done
__global__ void k_cgr_ctl(const double* rr, const double* bb, double tol2, int* ctl, int it, int maxit, int nr) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && ctl[0] == 0) {
    bool conv = true, bad = false;
    for (int c = 0; c < nr; ++c) {
      conv = conv && rr[c] <= tol2 * bb[c];
      bad = bad || !isfinite(rr[c]);
    }
    if (conv || bad || it >= maxit) {
      ctl[0] = conv ? 1 : (bad ? 3 : 2);
      ctl[1] = it;
    }
  }
}

// CG convergence test right after the residual update: ctl = (1, it) when <r_c, r_c> <= tol2 <b_c, b_c>
// for every right-hand side c < nr, so the host's check after an iteration sees it (and a V-cycle
// or direction kernel launched after it returns at once).  k_cg_dir would find the same at
// iteration it; a NaN is left to it.
// note (optional): rr[0] and bb[0] copied there (the PCG's initial residual, read with the control word)
__global__ void k_conv(const double* rr, const double* bb, double tol2, int* ctl, int it, int nr,
                       double* note = nullptr) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && note) {
    note[0] = rr[0];
    note[1] = bb[0];
  }
  if (threadIdx.x == 0 && blockIdx.x == 0 && ctl[0] == 0) {
    bool conv = true;
    for (int c = 0; c < nr; ++c) conv = conv && rr[c] <= tol2 * bb[c];
    if (conv) {
      ctl[0] = 1;
      ctl[1] = it;
    }
  }
}

// x = S y; slaves (master_of >= 0) take their master's value (p_s = p_m).
// (xs: the element stride of x0 / x1 -- VS when they are the interleaved velocity's components)
__global__ void k_cg_fin(int64_t n, int nr, const double* __restrict__ s, const double* y0, const double* y1,
                         double* x0, double* x1, const int32_t* __restrict__ master_of, int xs = 1) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    int64_t j = i;
    if (master_of && master_of[i] >= 0) j = master_of[i];
    const double sj = s ? s[j] : 1.0;
    x0[xs * i] = sj * y0[j];
    if (nr > 1) x1[xs * i] = sj * y1[j];
  }
}

// viscous preparation: b^ = S u (rhs), y0 = S^-1 u (warm start x0 = u^n), StokesColor.py:540-545
// warm start u^n + a polynomial extrapolation of the viscous increment u* - u from the last steps
// (it changes smoothly from step to step): d = (d_1x, d_1y, d_2x, ...) the last `order` increments,
// newest first; u^n + d_1 (order 1), + 2 d_1 - d_2 (2), + 3 d_1 - 3 d_2 + d_3 (3), and the binomial
// rows 4 d_1 - 6 d_2 + 4 d_3 - d_4 (4), 5 d_1 - 10 d_2 + 10 d_3 - 5 d_4 + d_5 (5), ... (6, 7)
// The increments are stored in fp32: they only shape the warm start, which the solve corrects to its
// rtol (1e-12 relative residual); an fp32-rounded increment moves the start by ~1e-7 of the increment,
// far below the extrapolation's own error.  Halves the increments' share of k_visc_prep / k_visc_fin.
constexpr int VINC_MAX = 7;  // highest extrapolation order
struct VincDev {
  const float* d[2 * VINC_MAX];
  int order;
};
// the warm start's unscaled value at row i (u + the extrapolated increment), both components
__device__ __forceinline__ void visc_start(const VincDev& D, int64_t i, double a, double b, double& ga, double& gb) {
  ga = a;
  gb = b;
  double e[2 * VINC_MAX];
#pragma unroll
  for (int k = 0; k < 2 * VINC_MAX; ++k) e[k] = k < 2 * D.order ? (double)D.d[k][i] : 0.0;
  if (D.order == 1) {
    ga += e[0];
    gb += e[1];
  } else if (D.order == 2) {
    ga += 2.0 * e[0] - e[2];
    gb += 2.0 * e[1] - e[3];
  } else if (D.order == 3) {
    ga += 3.0 * (e[0] - e[2]) + e[4];
    gb += 3.0 * (e[1] - e[3]) + e[5];
  } else if (D.order == 4) {
    ga += 4.0 * (e[0] + e[4]) - 6.0 * e[2] - e[6];
    gb += 4.0 * (e[1] + e[5]) - 6.0 * e[3] - e[7];
  } else if (D.order == 5) {
    ga += 5.0 * (e[0] - e[6]) + 10.0 * (e[4] - e[2]) + e[8];
    gb += 5.0 * (e[1] - e[7]) + 10.0 * (e[5] - e[3]) + e[9];
  } else if (D.order == 6) {
    ga += 6.0 * (e[0] + e[8]) - 15.0 * (e[2] + e[6]) + 20.0 * e[4] - e[10];
    gb += 6.0 * (e[1] + e[9]) - 15.0 * (e[3] + e[7]) + 20.0 * e[5] - e[11];
  } else if (D.order == 7) {
    ga += 7.0 * (e[0] - e[10]) + 21.0 * (e[8] - e[2]) + 35.0 * (e[4] - e[6]) + e[12];
    gb += 7.0 * (e[1] - e[11]) + 21.0 * (e[9] - e[3]) + 35.0 * (e[5] - e[7]) + e[13];
  }
}
// the viscous right-hand side b = s u and the warm start y = sq (u + extrapolated increment); AOS: b and y
// interleaved (the Chebyshev solve's dbl2 vectors: bx, yx point at them, by, yy unused), else SoA (the CG)
// (the start's scale 1 / s is computed here: the same correctly rounded division as the host's, 8 B/row less than
// reading a stored copy)
template <bool AOS>
__global__ void k_visc_prep(int64_t n, const double* __restrict__ s, const double* ux, const double* uy, double* bx,
                            double* by, double* yx, double* yy, VincDev D) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    const double a = ux[VS * i] + 0.0, b = uy[VS * i] + 0.0;  // rhs = u + DT * b_force, b_force = 0
    const double si = s[i], sq = 1.0 / si;
    double ga, gb;
    visc_start(D, i, a, b, ga, gb);
    if constexpr (AOS) {
      stnt(reinterpret_cast<dbl2*>(bx) + i, dbl2{si * a, si * b});
      stnt(reinterpret_cast<dbl2*>(yx) + i, dbl2{sq * ga, sq * gb});
    } else {
      stnt(bx + i, si * a);
      stnt(by + i, si * b);
      stnt(yx + i, sq * ga);
      stnt(yy + i, sq * gb);
    }
  }
}
// the same from SoA y (the viscous CG's vectors)
__global__ void k_visc_fin_soa(int64_t n, const double* __restrict__ s, const double* __restrict__ yx,
                               const double* __restrict__ yy, const double* __restrict__ ux,
                               const double* __restrict__ uy, double* __restrict__ usx, double* __restrict__ usy,
                               float* __restrict__ dx, float* __restrict__ dy) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    const double a = s[i] * yx[i], b = s[i] * yy[i];
    stnt(reinterpret_cast<dbl2*>(usx) + i, dbl2{a, b});  // (usy = usx + 1: interleaved)
    stnt(dx + i, (float)(a - ux[VS * i]));
    stnt(dy + i, (float)(b - uy[VS * i]));
  }
}
// u* = S y (both components, y interleaved) and, with dx non-null, the increment u* - u for the next
// step's warm start
__global__ void k_visc_fin(int64_t n, const double* __restrict__ s, const dbl2* __restrict__ y,
                           const double* __restrict__ ux, const double* __restrict__ uy, double* __restrict__ usx,
                           double* __restrict__ usy, float* __restrict__ dx, float* __restrict__ dy) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    const dbl2 yi = y[i];
    const double a = s[i] * yi.x, b = s[i] * yi.y;
    stnt(reinterpret_cast<dbl2*>(usx) + i, dbl2{a, b});  // (usy = usx + 1: interleaved)
    if (dx) {
      stnt(dx + i, (float)(a - ux[VS * i]));
      stnt(dy + i, (float)(b - uy[VS * i]));
    }
  }
}

// ----------------------------------------------------------------------------- div / grad
// calculate_divergence (StokesColor.py:130-165) in operator form: div = (Gx ux + Gy uy) / (area_sum + 1e-12)
// into div (null: only its max |div| partials -- the step's div(u*) and final div fields are computed when
// read, pucfem_get_field).
// Optionally the pressure RHS of the row-scaled system: braw = (M + 1e-12) * (-(1/DT) * div)
// (StokesColor.py:554 with A_pressure = K / (M + 1e-12)).  Partials: [0] max|div|, [1] sum(braw).
// AOS: ux points at interleaved (x, y) pairs (uy unused): one 16-B gather per neighbour
template <bool C16, bool AOS = false>
__global__ LB_GATHER void k_div(SellDev A, FaceDev fc, const double* __restrict__ gx,
                                            const double* __restrict__ gy, const double* __restrict__ ux,
                                            const double* __restrict__ uy, const double* __restrict__ as1,
                                            double* __restrict__ div, const double* __restrict__ mp, double negidt,
                                            double* __restrict__ braw, double* part, RedOut ro = RedOut{}) {
  __shared__ double sh[4];
  double mx = 0.0, sb = 0.0;
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    // interior rows: the lumped divergence of the face's stencil; area_sum = lumped mass there
    // groups of 2 rows per thread, the 24 gathered values of a group loaded first
    constexpr int K = face_k(PUCFEM_DIV_K);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      const double* c = fc.coef + lf * lat::NCOEF;
      double vx[K][6], vy[K][6];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        int32_t nb[6];
        bool in[6];
        lat::neighbours(F, fc.n, t[r], i[r], j[r], nb, in);
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          if constexpr (AOS) {
            const dbl2 q = reinterpret_cast<const dbl2*>(ux)[nb[k]];
            vx[r][k] = q.x;
            vy[r][k] = q.y;
          } else {
            vx[r][k] = ux[nb[k]];
            vy[r][k] = uy[nb[k]];
          }
        }
      }
      const double as = c[lat::C_AS1];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        if (!ok[r]) continue;
        double ax, ay, bx, by;
        face_grad_v(c, vx[r], ax, ay);
        face_grad_v(c, vy[r], bx, by);
        const int64_t row = F.base + t[r];
        const double d = (ax + by) / as;
        if (div) stnt(div + row, d);
        mx = fmax(mx, fabs(d));
        if (braw) {
          const double b = as * (negidt * d);
          stnt(braw + row, b);
          sb += b;
        }
      }
    });
  } else {
    int64_t s0, s1;
    block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
    const int lane = threadIdx.x & 63, wv = wave_id();
    for (int64_t s = s0 + wv; s < s1; s += 4) {
      const int64_t off = A.off[s];
      const int w = A.w[s];
      const int64_t row = sell_row(A, s, lane);
      const int32_t base = (int32_t)(s * 64);
      double acc = 0.0;
      by_width(w, [&](auto wc) {
        constexpr int WN = decltype(wc)::value;
        if constexpr (WN > 0) {
          int32_t cj[WN];
          double ax[WN], ay[WN];
#pragma unroll
          for (int k = 0; k < WN; ++k) {
            const int64_t e = off + (int64_t)k * 64 + lane;
            cj[k] = sell_col<C16>(A, e, base);
            ax[k] = ldnt(gx + e);
            ay[k] = ldnt(gy + e);
          }
#pragma unroll
          for (int k = 0; k < WN; ++k) {
            if constexpr (AOS) {
              const dbl2 q = reinterpret_cast<const dbl2*>(ux)[cj[k]];
              acc += ax[k] * q.x + ay[k] * q.y;
            } else {
              acc += ax[k] * ux[cj[k]] + ay[k] * uy[cj[k]];
            }
          }
        } else {
          for (int k = 0; k < w; ++k) {
            const int64_t e = off + (int64_t)k * 64 + lane;
            const int32_t j = sell_col<C16>(A, e, base);
            if constexpr (AOS) {
              const dbl2 q = reinterpret_cast<const dbl2*>(ux)[j];
              acc += ldnt(gx + e) * q.x + ldnt(gy + e) * q.y;
            } else {
              acc += ldnt(gx + e) * ux[j] + ldnt(gy + e) * uy[j];
            }
          }
        }
      });
      if (row >= 0) {
        const double d = acc / as1[row];
        if (div) stnt(div + row, d);
        mx = fmax(mx, fabs(d));
        if (braw) {
          const double b = mp[row] * (negidt * d);
          stnt(braw + row, b);
          sb += b;
        }
      }
    }
  }
  const double t = block_max(mx, sh);
  const double u = block_sum(sb, sh);
  if (threadIdx.x == 0) {
    red_part(ro, part, 0, t);
    red_part(ro, part, 1, u);
  }
  red_finish(ro, part, sh);
}

// pressure RHS of the merged, range-projected, scaled system (oracle PressureSolver.rhs):
// b^_i = s_i * (b~_i - mean), b~_m = braw_m + braw_s, b~_s = 0.
__global__ void k_pres_rhs(int64_t n, const double* __restrict__ braw, const int32_t* __restrict__ slave_of,
                           const int32_t* __restrict__ master_of, const double* __restrict__ s,
                           const double* part_sum, int nb, double inv_nfree, double* __restrict__ bh) {
  __shared__ double sh[4];
  const double mean = reduce_partials(part_sum, nb, sh) * inv_nfree;
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    double b;
    if (master_of[i] >= 0) {
      b = 0.0;
    } else {
      b = braw[i];
      if (slave_of[i] >= 0) b += braw[slave_of[i]];
      b = s ? s[i] * (b - mean) : (b - mean);
    }
    stnt(bh + i, b);
  }
}

// Specialised on the mode, so each row body is one basic block: the row's u* (mode 0) or u (mode 1) loads
// issue with the gathers (4-row groups on the face interiors).
template <int MODE, bool C16>
__device__ __forceinline__ void grad_proj_body(const SellDev& A, const FaceDev& fc, const double* __restrict__ gx,
                                               const double* __restrict__ gy, const double* __restrict__ p,
                                               const double* __restrict__ as1, double dt,
                                               const uint8_t* __restrict__ dirflag, const double* usx,
                                               const double* usy, double* ux, double* uy) {
  // (u, u* interleaved: bx / ux point at the pairs, by / uy are their y components)
  const double* bx = MODE == 0 ? usx : ux;
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    // interior rows are never Dirichlet nodes
    constexpr int K = face_k(PUCFEM_GRADP_K);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      const double* c = fc.coef + lf * lat::NCOEF;
      double v[K][6], ox[K], oy[K];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        int32_t nb[6];
        bool in[6];
        lat::neighbours(F, fc.n, t[r], i[r], j[r], nb, in);
#pragma unroll
        for (int k = 0; k < 6; ++k) v[r][k] = p[nb[k]];
        const dbl2 o = reinterpret_cast<const dbl2*>(bx)[F.base + t[r]];
        ox[r] = o.x;
        oy[r] = o.y;
      }
      const double d = c[lat::C_AS1];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        if (!ok[r]) continue;
        double ax, ay;
        face_grad_v(c, v[r], ax, ay);
        const int64_t row = F.base + t[r];
        stnt(reinterpret_cast<dbl2*>(ux) + row, dbl2{ox[r] - dt * (ax / d), oy[r] - dt * (ay / d)});
      }
    });
    return;
  }
  int64_t s0, s1;
  block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
  const int lane = threadIdx.x & 63, wv = wave_id();
  for (int64_t s = s0 + wv; s < s1; s += 4) {
    const int64_t off = A.off[s];
    const int w = A.w[s];
    const int64_t row = sell_row(A, s, lane);
    const int32_t base = (int32_t)(s * 64);
    const int64_t rr = row >= 0 ? row : 0;
    const dbl2 o = reinterpret_cast<const dbl2*>(bx)[rr];
    const double ox = o.x, oy = o.y, d = as1[rr];
    const bool dirichlet = MODE == 1 && dirflag[rr] != 0;
    double ax = 0.0, ay = 0.0;
    by_width(w, [&](auto wc) {
      constexpr int WN = decltype(wc)::value;
      if constexpr (WN > 0) {
        int32_t cj[WN];
        double vx[WN], vy[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          cj[k] = sell_col<C16>(A, e, base);
          vx[k] = ldnt(gx + e);
          vy[k] = ldnt(gy + e);
        }
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          const double pj = p[cj[k]];
          ax += vx[k] * pj;
          ay += vy[k] * pj;
        }
      } else {
        for (int k = 0; k < w; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          const double pj = p[sell_col<C16>(A, e, base)];
          ax += ldnt(gx + e) * pj;
          ay += ldnt(gy + e) * pj;
        }
      }
    });
    if (row >= 0 && !dirichlet) stnt(reinterpret_cast<dbl2*>(ux) + row, dbl2{ox - dt * (ax / d), oy - dt * (ay / d)});
  }
}

// projection u = u* - DT grad p (mode 0, all rows, StokesColor.py:561-562) or the masked second
// projection u[interior] -= DT grad p2 (mode 1, StokesColor.py:572-573).
template <bool C16>
__global__ LB_GATHER void k_grad_proj(SellDev A, FaceDev fc, const double* __restrict__ gx,
                                                  const double* __restrict__ gy, const double* __restrict__ p,
                                                  const double* __restrict__ as1, double dt, int mode,
                                                  const uint8_t* __restrict__ dirflag, const double* usx,
                                                  const double* usy, double* ux, double* uy,
                                                  const int* gate = nullptr) {
  if (gate && gate[0] == 0) return;  // (gated on the PCG's control word: the solve has not finished)
  if (mode == 0) grad_proj_body<0, C16>(A, fc, gx, gy, p, as1, dt, dirflag, usx, usy, ux, uy);
  else grad_proj_body<1, C16>(A, fc, gx, gy, p, as1, dt, dirflag, usx, usy, ux, uy);
}

// gradient only (calculate_gradiant, StokesColor.py:224-263) for the unit op
template <bool C16>
__global__ __launch_bounds__(BS) void k_grad(SellDev A, FaceDev fc, const double* __restrict__ gx,
                                             const double* __restrict__ gy, const double* __restrict__ p,
                                             const double* __restrict__ as1, double* outx, double* outy) {
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    face_rows(fc, role.idx, fc.nb, [&](const lat::FaceTab& F, int32_t lf, int32_t t, int32_t i, int32_t j) {
      int32_t nb[6];
      bool in[6];
      lat::neighbours(F, fc.n, t, i, j, nb, in);
      const double* c = fc.coef + lf * lat::NCOEF;
      double ax, ay;
      face_grad(c, nb, p, ax, ay);
      stnt(outx + F.base + t, ax / c[lat::C_AS1]);
      stnt(outy + F.base + t, ay / c[lat::C_AS1]);
    });
    return;
  }
  int64_t s0, s1;
  block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
  const int lane = threadIdx.x & 63, wv = wave_id();
  for (int64_t s = s0 + wv; s < s1; s += 4) {
    const int64_t off = A.off[s];
    const int w = A.w[s];
    const int64_t row = sell_row(A, s, lane);
    const int32_t base = (int32_t)(s * 64);
    double ax = 0.0, ay = 0.0;
    for (int k = 0; k < w; ++k) {
      const int64_t e = off + (int64_t)k * 64 + lane;
      const double pj = p[sell_col<C16, false>(A, e, base)];
      ax += gx[e] * pj;
      ay += gy[e] * pj;
    }
    if (row >= 0) {
      outx[row] = ax / as1[row];
      outy[row] = ay / as1[row];
    }
  }
}

// ----------------------------------------------------------------------------- boundary conditions
// makePerBCU then makeDirBCU (StokesColor.py:405-431) / reapply_periodic_u + reapply_dirchlect_u
// (heatEq.py:282-301).
// Boundary conditions on owned rows, multi-block: copies u[dst] = u_old[src] (makePerBCU, sources
// resolved to pre-copy values on the host), then Dirichlet values (makeDirBCU).  The host drops the
// copies whose destination is a Dirichlet node (the Dirichlet value wins), so the two write sets are
// disjoint; when a source is also written, k_bc_gather first saves the sources in tmp (a separate
// launch orders every read before any write), else tmp is null and k_bc_apply reads u directly.
// (vs: the element stride of u0 / u1 -- VS for the interleaved velocity, 1 for a plain vector)
__global__ void k_bc_gather(int ncopy, const int32_t* __restrict__ csrc, double* __restrict__ tmp, int ncomp,
                            const double* __restrict__ u0, const double* __restrict__ u1, int vs) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ncopy; k += gridDim.x * blockDim.x) {
    tmp[2 * k] = u0[(int64_t)vs * csrc[k]];
    if (ncomp > 1) tmp[2 * k + 1] = u1[(int64_t)vs * csrc[k]];
  }
}
__global__ void k_bc_apply(int ncopy, const int32_t* __restrict__ cdst, const int32_t* __restrict__ csrc,
                           const double* tmp, int ndir, const int32_t* __restrict__ dnode,
                           const double* __restrict__ dval, int ncomp, double* u0, double* u1, int vs) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ncopy + ndir; k += gridDim.x * blockDim.x) {
    if (k < ncopy) {
      const int64_t d = (int64_t)vs * cdst[k], sidx = (int64_t)vs * csrc[k];
      const double a = tmp ? tmp[2 * k] : u0[sidx];
      const double b = ncomp > 1 ? (tmp ? tmp[2 * k + 1] : u1[sidx]) : 0.0;
      u0[d] = a;
      if (ncomp > 1) u1[d] = b;
    } else {
      const int j = k - ncopy;
      const int64_t d = (int64_t)vs * dnode[j];
      u0[d] = dval[ncomp * j];
      if (ncomp > 1) u1[d] = dval[ncomp * j + 1];
    }
  }
}

// ----------------------------------------------------------------------------- semi-Lagrangian
struct MeshDev {
  const double* x;      // full mesh, internal numbering
  const double* y;
  const int32_t* tri;   // T*3 internal node ids, reference triangle order
  int64_t T;
};
struct GridDev {
  int32_t nx, ny;
  double x0, y0, hx, hy;
  const int32_t* start;
  const int32_t* item;
  const double* px;
  const double* py;
};

__device__ __forceinline__ int32_t gcell(double v, double v0, double hv, int32_t n) {
  const double f = floor((v - v0) / hv);
  if (!(f >= 0.0)) return 0;
  if (f >= (double)n) return n - 1;
  return (int32_t)f;
}
// Squared distance from query q to its k-th nearest grid point (the semi-Lagrangian fast-accept radii,
// pucfem_host.cpp knn_radius2 restated for the device, operation for operation, so the tables are
// bit-identical): ring search over the grid cells, ascending k smallest distances, stop once every
// unvisited cell is farther than the k-th; rounded DOWN to fp32.  Query e: (qx[e], qy[e]); its own id
// qid[e] (self: the grid point with that id is skipped; qid null: id e) and out[id].
constexpr int KNN_MAX = 16;
__global__ __launch_bounds__(BS) void k_knn_radius2(GridDev G, const double* __restrict__ qx,
                                                    const double* __restrict__ qy, const int32_t* __restrict__ qid,
                                                    int64_t nq, int k, int self, float* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * BS + threadIdx.x; e < nq; e += (int64_t)gridDim.x * BS) {
    const double x = qx[e], y = qy[e];
    const int32_t id = qid ? qid[e] : (int32_t)e;
    double best[KNN_MAX];
    for (int p = 0; p < k; ++p) best[p] = INFINITY;
    const int32_t ci = gcell(x, G.x0, G.hx, G.nx), cj = gcell(y, G.y0, G.hy, G.ny);
    for (int32_t r = 0;; ++r) {
      const int32_t jlo = max(cj - r, 0), jhi = min(cj + r, G.ny - 1);
      for (int32_t j = jlo; j <= jhi; ++j) {
        const bool edge = j == cj - r || j == cj + r;
        for (int32_t i = ci - r; i <= ci + r; i += (edge || r == 0) ? 1 : 2 * r) {
          if (i < 0 || i >= G.nx) continue;
          const int64_t c = (int64_t)j * G.nx + i;
          for (int32_t q = G.start[c]; q < G.start[c + 1]; ++q) {
            if (self && G.item[q] == id) continue;
            const double dx = G.px[q] - x, dy = G.py[q] - y, d = dx * dx + dy * dy;
            if (d >= best[k - 1]) continue;
            int p = k - 1;
            while (p > 0 && best[p - 1] > d) {
              best[p] = best[p - 1];
              --p;
            }
            best[p] = d;
          }
        }
      }
      double dmin = INFINITY;
      if (ci - r > 0) dmin = fmin(dmin, x - (G.x0 + (ci - r) * G.hx));
      if (ci + r < G.nx - 1) dmin = fmin(dmin, G.x0 + (ci + r + 1) * G.hx - x);
      if (cj - r > 0) dmin = fmin(dmin, y - (G.y0 + (cj - r) * G.hy));
      if (cj + r < G.ny - 1) dmin = fmin(dmin, G.y0 + (cj + r + 1) * G.hy - y);
      if (dmin == INFINITY || (dmin > 0 && best[k - 1] < dmin * dmin * (1.0 - 1e-9))) break;
    }
    float f = (float)best[k - 1];
    if ((double)f > best[k - 1]) f = nextafterf(f, 0.0f);
    out[id] = f;
  }
}

__device__ __forceinline__ bool knn_less(double d, int32_t i, double bd, int32_t bi) {
  return d < bd || (d == bd && i < bi);
}

// Point location for the semi-Lagrangian step (PointLocator.find, StokesColor.py:314-345).
// The reference takes the k=10 nearest centroids in (distance, id) order and returns the first
// whose barycentric weights are all >= 0.  Restated exactly, without sorting 10 candidates:
//   1. every triangle that passes the weight test for q has q inside it up to rounding, so it is
//      listed in q's cell of the inflated-bbox grid L; among those that pass, take the one with the
//      smallest (d^2, id) key T*.  A triangle whose weights are all >= SL_MARGIN contains q with a
//      margin no other triangle's test can reach, so the scan stops at it;
//   2. T* is the answer iff fewer than 10 centroids have a key below T*'s (its rank is < 10).  Fast
//      accept: every such centroid c has |c - c_T*| <= 2 R (R = |q - c_T*|), so 4 R^2 below the
//      squared distance from c_T* to its 10th nearest other centroid (rho2, precomputed) bounds the
//      rank by 9.  Otherwise they are counted over the centroid-grid cells meeting [q - R, q + R]^2.
// Otherwise no triangle among the 10 nearest passes and the reference keeps c[n].
// Records are stored in node order (triangles sorted by their smallest vertex id), not in the
// mesh's triangle order, and hold vertex ids only (16 B: a, b, d and the mesh's triangle id, which
// the (distance, id) keys keep); the vertex coordinates come from one interleaved (x, y) array in
// node order, which neighbouring triangles share.  Cells list record positions.
struct LocDev {
  int32_t nx, ny;
  double x0, y0, hx, hy;
  const int32_t* start;  // nx*ny+1
  const int32_t* item;   // record positions, ascending per cell
  const int4* rec;       // per position: vertex ids a b d, triangle id
  const double2* xy;     // node coordinates (internal numbering)
  // per position: squared distance from the centroid to the 10th nearest other centroid (rounded down)
  const float* rho2;
  const float* rv2;  // per node: squared distance to its (KNN + 1)-th nearest centroid (rounded down)
  // measurement knob (PUCFEM_SL_PROBE): bit 0 = accept T* without the rank count, bit 1 = not-found
  // output 2 for the rows k_sl_slow finished (pucfem_sl_advect)
  int32_t probe;
};
struct SlTri {
  double x1, y1, x2, y2, x3, y3;
  int32_t a, b, d, id;
};
__device__ __forceinline__ SlTri sl_tri(const LocDev& L, int32_t pos) {
  const int4 m = L.rec[pos];
  const double2 p = L.xy[m.x], q = L.xy[m.y], s = L.xy[m.z];
  return SlTri{p.x, p.y, q.x, q.y, s.x, s.y, m.x, m.y, m.z, m.w};
}
constexpr double SL_MARGIN = 1e-6;

// rank test of the best passing triangle (id best, squared centroid distance bestd, fast-accept
// radius rho2): true iff fewer than KNN centroids have a (d^2, id) key below it
__device__ __forceinline__ bool sl_rank_ok(const GridDev& G, double qx, double qy, double bestd, int32_t best,
                                           float rho2, int32_t probe) {
  if (4.0 * bestd * (1.0 + 1e-9) < (double)rho2 || (probe & 1)) return true;
  const double R = sqrt(bestd) * (1.0 + 1e-9) + 1e-300;
  const int32_t i0 = gcell(qx - R, G.x0, G.hx, G.nx), i1 = gcell(qx + R, G.x0, G.hx, G.nx);
  const int32_t j0 = gcell(qy - R, G.y0, G.hy, G.ny), j1 = gcell(qy + R, G.y0, G.hy, G.ny);
  int cnt = 0;
  for (int32_t j = j0; j <= j1; ++j) {
    const int32_t f0 = G.start[(int64_t)j * G.nx + i0], f1 = G.start[(int64_t)j * G.nx + i1 + 1];
    for (int32_t e = f0; e < f1; ++e) {  // cells i0..i1 of row j are one contiguous entry range
      const double dx = G.px[e] - qx, dy = G.py[e] - qy;
      const double d = dx * dx + dy * dy;
      if (knn_less(d, G.item[e], bestd, best) && ++cnt >= KNN) return false;
    }
  }
  return true;
}

// the reference's weight test (StokesColor.py:325-333) and centroid distance of one candidate
__device__ __forceinline__ bool sl_test(const SlTri& r, double qx, double qy, double& d, bool& margin) {
  const double x1 = r.x1, y1 = r.y1, x2 = r.x2, y2 = r.y2, x3 = r.x3, y3 = r.y3;
  const double det = (x2 - x1) * (y3 - y1) - (x3 - x1) * (y2 - y1);
  if (!(fabs(det) >= 1e-14)) return false;
  const double w1 = ((x2 - qx) * (y3 - qy) - (x3 - qx) * (y2 - qy)) / det;
  const double w2 = ((x3 - qx) * (y1 - qy) - (x1 - qx) * (y3 - qy)) / det;
  const double w3 = 1.0 - w1 - w2;
  if (!(w1 >= 0.0 && w2 >= 0.0 && w3 >= 0.0)) return false;
  // centroid as StokesColor.py:321 / the centroid grid: (x1 + x2 + x3) / 3 in fp64
  const double dx = (x1 + x2 + x3) / 3.0 - qx, dy = (y1 + y2 + y3) / 3.0 - qy;
  d = dx * dx + dy * dy;
  margin = w1 >= SL_MARGIN && w2 >= SL_MARGIN && w3 >= SL_MARGIN;
  return true;
}

// Locate step (the rank test follows in k_sl_slow): the passing triangle with the smallest
// (d^2, id) key (false: none passes), its d^2 and its fast-accept radius.
// Record locator: the records listed in q's cell of the inflated-bbox grid.
__device__ __forceinline__ bool sl_best(const LocDev& L, int32_t, double qx, double qy, SlTri& out, double& bestd,
                                        float& rho2) {
  const int32_t ci = gcell(qx, L.x0, L.hx, L.nx), cj = gcell(qy, L.y0, L.hy, L.ny);
  const int64_t cell = (int64_t)cj * L.nx + ci;
  int32_t best = 0x7fffffff, bpos = -1;
  bestd = INFINITY;
  const int32_t e1 = L.start[cell + 1];
  for (int32_t e = L.start[cell]; e < e1; ++e) {
    const int32_t pos = L.item[e];
    const SlTri r = sl_tri(L, pos);
    double d;
    bool margin;
    if (sl_test(r, qx, qy, d, margin)) {
      if (knn_less(d, r.id, bestd, best)) {
        bestd = d;
        best = r.id;
        bpos = pos;
        out = r;
      }
      if (margin) break;
    }
  }
  if (bpos < 0) return false;
  rho2 = L.rho2[bpos];
  return true;
}

// Lattice locator (Ctx::lattice): the finest mesh is the coarse mesh red-refined L times, so the
// candidates of the weight test are found arithmetically instead of from per-triangle records: the
// macro faces listed in q's cell of a grid over the coarse triangles (inflated bboxes), q's lattice
// coordinates (u, v) = n M (q - A) in each, and the cells (i, j, s) whose closure holds (u, v) up to
// SL_LDEL lattice units (one cell away from edges, more only within 1e-7 of a lattice line, where the
// reference's weight test can pass in several triangles).  The rotation stored in the cell table
// gives the triangle's vertices in the mesh's own order, so the weight test and the (d^2, id) keys
// are the record locator's, bit for bit.
struct LatLocDev {
  int32_t nx, ny;
  double x0, y0, ihx, ihy;       // macro grid: origin, inverse cell sizes
  const int32_t* start;          // macro grid cells -> face ids
  const int32_t* item;
  const lat::SlFace* face;
  const uint32_t* cell;          // per lattice cell (lat::cell_index): (offset in face << 2) | rotation
  const double2* xy;             // node coordinates (internal numbering)
  const float* rho2;             // per triangle id
  const float* rv2;              // per node, as LocDev::rv2
  const int32_t* home;           // per row (internal id): its macro face (face-interior rows), else -1
  // per row: the triangle the locator returns for the row's own node (a zero velocity: walls), -1 when
  // none is accepted (k_sl_self, once at build); null until then
  const int32_t* self;
  int32_t n, probe;
};
constexpr double SL_LDEL = 1e-7;

// one lattice cell of face S as an SlTri (vertices in the mesh's stored order: the cell's list
// rotated by the table's rotation; selects, not a dynamically indexed array, which would live in LDS)
__device__ __forceinline__ SlTri sl_cell(const LatLocDev& L, const lat::SlFace& S, int32_t i, int32_t j, int32_t s) {
  const uint32_t ent = L.cell[lat::cell_index(L.n, i, j, s)];
  const int32_t rot = (int32_t)(ent & 3u);
  int32_t pi[3], pj[3];
  lat::cell_vertices(i, j, s, pi, pj);
  const int32_t c0 = lat::vertex(S.tab, S.va, S.vb, S.vc, L.n, pi[0], pj[0]);
  const int32_t c1 = lat::vertex(S.tab, S.va, S.vb, S.vc, L.n, pi[1], pj[1]);
  const int32_t c2 = lat::vertex(S.tab, S.va, S.vb, S.vc, L.n, pi[2], pj[2]);
  const int32_t v0 = rot == 0 ? c0 : (rot == 1 ? c1 : c2);
  const int32_t v1 = rot == 0 ? c1 : (rot == 1 ? c2 : c0);
  const int32_t v2 = rot == 0 ? c2 : (rot == 1 ? c0 : c1);
  const double2 p = L.xy[v0], q = L.xy[v1], w = L.xy[v2];
  return SlTri{p.x, p.y, q.x, q.y, w.x, w.y, v0, v1, v2, (int32_t)(S.t0 + (int64_t)(ent >> 2))};
}

// q strictly inside one cell of face S (by SL_LDEL lattice units, hence inside the face and in no
// other triangle's weight test): that cell; its key d is the reference's, exactly
__device__ __forceinline__ bool sl_inner(const LatLocDev& L, const lat::SlFace& S, double qx, double qy, SlTri& out,
                                         double& bestd, double& u, double& v) {
  const int32_t n = L.n;
  const double dx = qx - S.ax, dy = qy - S.ay;
  u = (double)n * (S.m00 * dx + S.m01 * dy);
  v = (double)n * (S.m10 * dx + S.m11 * dy);
  const double fu = floor(u), fv = floor(v);
  const double a = u - fu, b = v - fv;
  const int32_t s = a + b > 1.0 ? 1 : 0;
  const bool inner = s == 0 ? (a >= SL_LDEL && b >= SL_LDEL && a + b <= 1.0 - SL_LDEL)
                            : (a <= 1.0 - SL_LDEL && b <= 1.0 - SL_LDEL && a + b >= 1.0 + SL_LDEL);
  if (!(inner && fu >= 0.0 && fv >= 0.0 && fu + fv <= (double)(n - 1 - s))) return false;
  out = sl_cell(L, S, (int32_t)fu, (int32_t)fv, s);
  // the weights are >= SL_LDEL up to rounding: the weight test passes; only its det guard remains
  const double det = (out.x2 - out.x1) * (out.y3 - out.y1) - (out.x3 - out.x1) * (out.y2 - out.y1);
  if (!(fabs(det) >= 1e-14)) return false;
  const double ex = (out.x1 + out.x2 + out.x3) / 3.0 - qx, ey = (out.y1 + out.y2 + out.y3) / 3.0 - qy;
  bestd = ex * ex + ey * ey;
  return true;
}

// Lattice locator.  Common case: q lies inside a macro face and inside one lattice cell by more than
// SL_LDEL, so no other triangle can pass the weight test: that cell alone is tested.  Otherwise every
// cell of every candidate face whose closure holds q up to SL_LDEL is tested, as the record locator
// tests every record of its grid cell.
__device__ __forceinline__ bool sl_best(const LatLocDev& L, int32_t home, double qx, double qy, SlTri& out,
                                        double& bestd, float& rho2) {
  double u, v;
  if (home >= 0 && sl_inner(L, L.face[home], qx, qy, out, bestd, u, v)) {
    rho2 = L.rho2[out.id];
    return true;
  }
  // cells of the macro grid by multiplication: a point within rounding of a cell line may land in
  // either cell, and both list every face whose (inflated) bbox holds it
  const double gx = floor((qx - L.x0) * L.ihx), gy = floor((qy - L.y0) * L.ihy);
  const int32_t ci = !(gx >= 0.0) ? 0 : (gx >= (double)L.nx ? L.nx - 1 : (int32_t)gx);
  const int32_t cj = !(gy >= 0.0) ? 0 : (gy >= (double)L.ny ? L.ny - 1 : (int32_t)gy);
  const int64_t gc = (int64_t)cj * L.nx + ci;
  const int32_t n = L.n;
  const double dn = (double)n;
  int32_t best = 0x7fffffff;
  bestd = INFINITY;
  bool done = false;
  const int32_t e1 = L.start[gc + 1];
  for (int32_t e = L.start[gc]; e < e1 && !done; ++e) {
    const lat::SlFace& S = L.face[L.item[e]];
    {
      SlTri r;
      double d;
      if (sl_inner(L, S, qx, qy, r, d, u, v)) {
        if (knn_less(d, r.id, bestd, best)) {
          bestd = d;
          best = r.id;
          out = r;
        }
        break;
      }
    }
    if (!(u >= -SL_LDEL && v >= -SL_LDEL && u + v <= dn + SL_LDEL)) continue;
    const int32_t i0 = min(max((int32_t)floor(u), 0), n - 1), j0 = min(max((int32_t)floor(v), 0), n - 1);
    for (int32_t j = max(j0 - 1, 0); j <= j0 + 1 && !done; ++j)
      for (int32_t i = max(i0 - 1, 0); i <= i0 + 1 && i + j <= n - 1 && !done; ++i) {
        const double a = u - i, b = v - j;
        for (int32_t s = 0; s < 2 && !done; ++s) {
          const bool near = s == 0 ? (a >= -SL_LDEL && b >= -SL_LDEL && a + b <= 1.0 + SL_LDEL)
                                   : (i + j <= n - 2 && a <= 1.0 + SL_LDEL && b <= 1.0 + SL_LDEL && a + b >= 1.0 - SL_LDEL);
          if (!near) continue;
          const SlTri r = sl_cell(L, S, i, j, s);
          double d;
          bool margin;
          if (sl_test(r, qx, qy, d, margin)) {
            if (knn_less(d, r.id, bestd, best)) {
              bestd = d;
              best = r.id;
              out = r;
            }
            done = margin;
          }
        }
      }
  }
  if (best == 0x7fffffff) return false;
  rho2 = L.rho2[best];
  return true;
}

__device__ __forceinline__ double pdx(double a, double b) {  // StokesColor.py:353-357
  double d = a - b;
  if (d > 0.5) d -= 1.0;
  if (d < -0.5) d += 1.0;
  return d;
}

// back-traced point of row i (StokesColor.py:361-372): x mod 1, y clamped into (0, 1)
__device__ __forceinline__ void sl_point(const MeshDev& M, int64_t g, double vx, double vy, double dt, double& xb,
                                         double& yb) {
  xb = py_mod1(M.x[g] - dt * vx * 1.0);
  yb = M.y[g] - dt * vy * 1.0;
  if (yb < 0.0) yb = 1e-12;
  if (yb > 1.0) yb = 1.0 - 1e-12;
}
// interpolation in the located triangle with periodic x differences (StokesColor.py:374-386)
__device__ __forceinline__ double sl_value(const SlTri& r, double xb, double yb, const double* __restrict__ c) {
  const double x1 = r.x1, y1 = r.y1, x2 = r.x2, y2 = r.y2, x3 = r.x3, y3 = r.y3;
  const double det = pdx(x2, x1) * (y3 - y1) - pdx(x3, x1) * (y2 - y1);
  const double w1 = (pdx(x2, xb) * (y3 - yb) - pdx(x3, xb) * (y2 - yb)) / det;
  const double w2 = (pdx(x3, xb) * (y1 - yb) - pdx(x1, xb) * (y3 - yb)) / det;
  const double w3 = 1.0 - w1 - w2;
  return w1 * c[r.a] + w2 * c[r.b] + w3 * c[r.d];
}

// Lattice fast path, in two stages so that k_sl can overlap one row's second stage with the next row's
// first.  Stage 1 (sl_lat_cell): q strictly inside a cell of its row's home face, else of the first face
// of q's macro-grid cell holding q so -> the cell triangle's vertices and id (false: the general
// locate of k_sl_slow decides).  Stage 2 (sl_lat_value): with the triangle's coordinates, field values
// and radii loaded (all issued together), the det guard, the rank settled by a fast accept (sl_fast's
// tests) and the interpolated value (false: k_sl_slow decides).  Scalars only (a struct here ends in
// scratch memory).
__device__ __forceinline__ bool sl_lat_cell(const LatLocDev& L, int32_t home, double qx, double qy, int32_t& v0,
                                            int32_t& v1, int32_t& v2, int32_t& id) {
  const int32_t n = L.n;
  int32_t f = -1;
  double fu = 0.0, fv = 0.0;
  int32_t s = 0;
  auto inner = [&](int32_t cand) {
    const lat::SlFace& S = L.face[cand];
    const double dx = qx - S.ax, dy = qy - S.ay;
    const double u = (double)n * (S.m00 * dx + S.m01 * dy), v = (double)n * (S.m10 * dx + S.m11 * dy);
    fu = floor(u);
    fv = floor(v);
    const double a = u - fu, b = v - fv;
    s = a + b > 1.0 ? 1 : 0;
    const bool in = s == 0 ? (a >= SL_LDEL && b >= SL_LDEL && a + b <= 1.0 - SL_LDEL)
                           : (a <= 1.0 - SL_LDEL && b <= 1.0 - SL_LDEL && a + b >= 1.0 + SL_LDEL);
    return in && fu >= 0.0 && fv >= 0.0 && fu + fv <= (double)(n - 1 - s);
  };
  if (home >= 0 && inner(home)) {
    f = home;
  } else {
    const double gx = floor((qx - L.x0) * L.ihx), gy = floor((qy - L.y0) * L.ihy);
    const int32_t ci = !(gx >= 0.0) ? 0 : (gx >= (double)L.nx ? L.nx - 1 : (int32_t)gx);
    const int32_t cj = !(gy >= 0.0) ? 0 : (gy >= (double)L.ny ? L.ny - 1 : (int32_t)gy);
    const int64_t gc = (int64_t)cj * L.nx + ci;
    const int32_t e1 = L.start[gc + 1];
    for (int32_t e = L.start[gc]; e < e1; ++e) {
      const int32_t cand = L.item[e];
      if (cand != home && inner(cand)) {
        f = cand;
        break;
      }
    }
    if (f < 0) return false;
  }
  const lat::SlFace& S = L.face[f];
  const int32_t i = (int32_t)fu, j = (int32_t)fv;
  const uint32_t ent = L.cell[lat::cell_index(n, i, j, s)];
  const int32_t rot = (int32_t)(ent & 3u);
  int32_t pi[3], pj[3];
  lat::cell_vertices(i, j, s, pi, pj);
  const int32_t c0 = lat::vertex(S.tab, S.va, S.vb, S.vc, n, pi[0], pj[0]);
  const int32_t c1 = lat::vertex(S.tab, S.va, S.vb, S.vc, n, pi[1], pj[1]);
  const int32_t c2 = lat::vertex(S.tab, S.va, S.vb, S.vc, n, pi[2], pj[2]);
  v0 = rot == 0 ? c0 : (rot == 1 ? c1 : c2);
  v1 = rot == 0 ? c1 : (rot == 1 ? c2 : c0);
  v2 = rot == 0 ? c2 : (rot == 1 ? c0 : c1);
  id = (int32_t)(S.t0 + (int64_t)(ent >> 2));
  return true;
}
// stage 2 on the loaded values: P1..P3 the vertex coordinates, f1..f3 the field values, rho2 the
// triangle's fast-accept radius, rv1..rv3 the vertices' radii
__device__ __forceinline__ bool sl_lat_value(int32_t probe, double qx, double qy, double2 P1, double2 P2, double2 P3,
                                             double f1, double f2, double f3, float rho2, float rv1, float rv2,
                                             float rv3, double& cn) {
  const double x1 = P1.x, y1 = P1.y, x2 = P2.x, y2 = P2.y, x3 = P3.x, y3 = P3.y;
  // the weights are >= SL_LDEL up to rounding: the weight test passes; only its det guard remains
  const double det0 = (x2 - x1) * (y3 - y1) - (x3 - x1) * (y2 - y1);
  if (!(fabs(det0) >= 1e-14)) return false;
  const double ex = (x1 + x2 + x3) / 3.0 - qx, ey = (y1 + y2 + y3) / 3.0 - qy;
  const double bestd = ex * ex + ey * ey;
  if (!(4.0 * bestd * (1.0 + 1e-9) < (double)rho2 || (probe & 1))) {
    const double d1 = (x1 - qx) * (x1 - qx) + (y1 - qy) * (y1 - qy);
    const double d2 = (x2 - qx) * (x2 - qx) + (y2 - qy) * (y2 - qy);
    const double d3 = (x3 - qx) * (x3 - qx) + (y3 - qy) * (y3 - qy);
    const bool k1 = d1 <= d2 && d1 <= d3, k2 = !k1 && d2 <= d3;
    const double rr = sqrt(k1 ? d1 : (k2 ? d2 : d3)) + sqrt(bestd);
    if (!(rr * rr * (1.0 + 1e-9) < (double)(k1 ? rv1 : (k2 ? rv2 : rv3)))) return false;
  }
  // interpolation (StokesColor.py:374-386)
  const double det = pdx(x2, x1) * (y3 - y1) - pdx(x3, x1) * (y2 - y1);
  const double w1 = (pdx(x2, qx) * (y3 - qy) - pdx(x3, qx) * (y2 - qy)) / det;
  const double w2 = (pdx(x3, qx) * (y1 - qy) - pdx(x1, qx) * (y3 - qy)) / det;
  const double w3 = 1.0 - w1 - w2;
  cn = w1 * f1 + w2 * f2 + w3 * f3;
  return true;
}

// Fast accepts of the rank test (T* among the KNN nearest centroids); every centroid whose key is
// below T*'s lies within R = |q - c_T*| of q.  (1) they lie within 2R of c_T*: fewer than KNN when
// 2R is below the distance from c_T* to its KNN-th nearest other centroid (rho2) -- settles points
// near the centroid; (2) they and c_T* lie within |q - v| + R of T*'s vertex v nearest to q: fewer
// than KNN + 1 in all when that is below the distance from v to its (KNN + 1)-th nearest centroid
// (rv2) -- settles points near vertices and edges, where back-traced points of slow flow gather.
template <class LOC>
__device__ __forceinline__ bool sl_fast(const LOC& L, const SlTri& r, double qx, double qy, double bestd, float rho2) {
  if (4.0 * bestd * (1.0 + 1e-9) < (double)rho2 || (L.probe & 1)) return true;
  const double d1 = (r.x1 - qx) * (r.x1 - qx) + (r.y1 - qy) * (r.y1 - qy);
  const double d2 = (r.x2 - qx) * (r.x2 - qx) + (r.y2 - qy) * (r.y2 - qy);
  const double d3 = (r.x3 - qx) * (r.x3 - qx) + (r.y3 - qy) * (r.y3 - qy);
  const bool k1 = d1 <= d2 && d1 <= d3, k2 = !k1 && d2 <= d3;
  const double rr = sqrt(k1 ? d1 : (k2 ? d2 : d3)) + sqrt(bestd);
  return rr * rr * (1.0 + 1e-9) < (double)L.rv2[k1 ? r.a : (k2 ? r.b : r.d)];
}

// advect_semilagrange (StokesColor.py:347-389) + PointLocator.find (:314-345) for the owned
// nodes; c is the full replica, cout receives the owned segment [row0, row0 + n).
// Partials (stride SLB): [0] sum w c, [1] sum w (mixing, marker==0 nodes), [2] not-found count.
// Two passes.  k_sl finishes the points of the lattice fast path (q strictly inside a cell of its
// row's home face, rank settled by a fast accept: all but ~36k of L7's 14.2M rows, ~0.25 % -- ~35k
// departure points inside the squirmer, which no triangle holds, and ~800 rank counts, r12n) with a
// small register footprint; the rest are queued, and the second pass runs the general locate and the
// centroid rank count: lattice locator k_sl_qscan + k_sl_wq + k_sl_qsum (one numbered list, a wave per
// point; k_sl_wave / k_sl_slow by PUCFEM_SL_WAVE), record locator k_sl_slow.  The record locator has no
// fast path: k_sl queues every row (or k_sl_rec_wave runs both passes on small meshes).
// The queue is per wave and deterministic: wave w of block b writes its k-th entry into slot
// k % 64 of the (k / 64)-th 64-row slice it processed (entries never outrun the rows they come from);
// k_sl_slow block b runs the same waves' queues and adds its partial sums to block b's, so the
// reductions keep a fixed order.
template <class LOC>
__global__ LB_GATHER void k_sl(MeshDev M, LOC L, int64_t row0, int64_t n,
                                           const double* __restrict__ ux, const double* __restrict__ uy, double dt,
                                           const double* __restrict__ c, double* __restrict__ cout,
                                           const double* __restrict__ wmix, int32_t* notfound, double* part,
                                           int32_t* __restrict__ queue, int32_t* __restrict__ qcnt) {
  constexpr bool LAT = std::is_same<LOC, LatLocDev>::value;
  __shared__ double sh[4];
  double swc = 0.0, sw = 0.0, nnf = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t qn = 0;
  int64_t i = r0 + threadIdx.x;
  // LAT: a software pipeline over the thread's rows i, i + BS, ...: stage A (the row's coordinates,
  // velocity and home face) loaded two rows ahead, stage B (departure point, face, cell -> the cell
  // triangle: sl_lat_cell) one row ahead, stage C (the triangle's coordinates, field values and radii
  // -> the value: sl_lat_value) on the current row, its loads issued before the next row's stage B so
  // that the two dependent chains overlap.  Row i's operations are those of one pass, in one pass's order.
  // (the row's own coordinates from the locator's interleaved table, whose lines the vertex loads of
  // the departure triangles, near the row, then find in L2: 16 B/row less than M.x, M.y beside it)
  double ax_ = 0.0, ay_ = 0.0, avx = 0.0, avy = 0.0;  // stage A of row i + BS
  int32_t ah = -1;
  int32_t bm = 0, b0 = 0, b1 = 0, b2 = 0, bid = 0;  // stage B of row i: mode 0 queue, 1 cell, 2 self
  double bqx = 0.0, bqy = 0.0;
  // (generic lambdas: instantiated for the lattice locator only)
  auto stage_a = [&](const auto& LL, int64_t r) {
    const double2 P = LL.xy[row0 + r];
    ax_ = P.x;
    ay_ = P.y;
    avx = ux[VS * r];
    avy = uy[VS * r];
    ah = LL.home[row0 + r];
  };
  auto stage_b = [&](const auto& LL, int64_t r) {  // from the stage A values
    double xb = py_mod1(ax_ - dt * avx * 1.0);
    double yb = ay_ - dt * avy * 1.0;
    if (yb < 0.0) yb = 1e-12;
    if (yb > 1.0) yb = 1.0 - 1e-12;
    bqx = xb;
    bqy = yb;
    // (the stage's outputs assigned from locals: through references the mode and id end in scratch)
    int32_t m = 2, t0 = 0, t1 = 0, t2 = 0, tid = 0;
    if (avx == 0.0 && avy == 0.0 && LL.self) {
      // q is the row's own node (no-slip walls): on lattice lines, where several triangles pass the
      // weight test; the answer for this q was settled once at build
      tid = LL.self[row0 + r];
    } else {
      m = sl_lat_cell(LL, ah, xb, yb, t0, t1, t2, tid) ? 1 : 0;
    }
    bm = m;
    b0 = t0;
    b1 = t1;
    b2 = t2;
    bid = tid;
  };
  if constexpr (LAT) {
    if (i < r1) {
      stage_a(L, i);
      stage_b(L, i);
      if (i + BS < r1) stage_a(L, i + BS);
    }
  }
  for (; i < r1; i += BS) {
    const int64_t g = row0 + i;
    bool done = false;
    double cn = 0.0;
    if constexpr (LAT) {
      const int32_t cm = bm, cid = bid;
      const double qx = bqx, qy = bqy;
      // stage C loads of row i
      double2 P1{0.0, 0.0}, P2{0.0, 0.0}, P3{0.0, 0.0};
      double f1 = 0.0, f2 = 0.0, f3 = 0.0;
      float rho2 = 0.0f, rv1 = 0.0f, rv2 = 0.0f, rv3 = 0.0f;
      if (cm == 1) {
        P1 = L.xy[b0];
        P2 = L.xy[b1];
        P3 = L.xy[b2];
        f1 = c[b0];
        f2 = c[b1];
        f3 = c[b2];
        rho2 = L.rho2[cid];
        rv1 = L.rv2[b0];
        rv2 = L.rv2[b1];
        rv3 = L.rv2[b2];
      }
      // stage B of row i + BS, stage A of row i + 2 BS
      if (i + BS < r1) {
        stage_b(L, i + BS);
        if (i + 2 * BS < r1) stage_a(L, i + 2 * BS);
      }
      if (cm == 2) {
        const int32_t t = cid;
        if (t >= 0) {
          const int32_t va = M.tri[3 * (int64_t)t], vb = M.tri[3 * (int64_t)t + 1], vc = M.tri[3 * (int64_t)t + 2];
          const SlTri r{M.x[va], M.y[va], M.x[vb], M.y[vb], M.x[vc], M.y[vc], va, vb, vc, t};
          cn = sl_value(r, qx, qy, c);
        } else {
          cn = c[g];
          nnf += 1.0;
        }
        if (notfound) notfound[i] = t >= 0 ? 0 : 1;
        done = true;
      } else if (cm == 1) {
        done = sl_lat_value(L.probe, qx, qy, P1, P2, P3, f1, f2, f3, rho2, rv1, rv2, rv3, cn);
        if (done && notfound) notfound[i] = 0;
      }
    }
    const uint64_t m = __ballot(!done);
    if (!done) {
      const int32_t p = qn + __popcll(m & ((1ull << lane) - 1ull));
      queue[r0 + (int64_t)(BS / 64 * (p >> 6) + wv) * 64 + (p & 63)] = (int32_t)i;
    }
    qn += __popcll(m);
    const double w = wmix ? wmix[i] : 0.0;
    sw += w;
    if (done) {
      stnt(cout + g, cn);
      swc += w * cn;
    }
  }
  if (lane == 0) qcnt[BS / 64 * blockIdx.x + wv] = qn;
  const double a = block_sum(swc, sh), b = block_sum(sw, sh), d = block_sum(nnf, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = a;
    part[SLB + blockIdx.x] = b;
    part[2 * SLB + blockIdx.x] = d;
  }
}

// second pass: the queued points -- general locate, fast accepts, centroid rank count (same grid as k_sl)
template <class LOC>
__global__ __launch_bounds__(BS) void k_sl_slow(MeshDev M, LOC L, GridDev G, int64_t row0, int64_t n,
                                                const double* __restrict__ ux, const double* __restrict__ uy, double dt,
                                                const double* __restrict__ c, double* __restrict__ cout,
                                                const double* __restrict__ wmix, int32_t* notfound, double* part,
                                                const int32_t* __restrict__ queue, const int32_t* __restrict__ qcnt,
                                                RedOut ro = RedOut{}) {
  __shared__ double sh[4];
  double swc = 0.0, nnf = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int32_t cnt = qcnt[BS / 64 * blockIdx.x + wv];
  for (int32_t p = lane; p < cnt; p += 64) {
    const int64_t i = queue[r0 + (int64_t)(BS / 64 * (p >> 6) + wv) * 64 + (p & 63)], g = row0 + i;
    double xb, yb;
    sl_point(M, g, ux[VS * i], uy[VS * i], dt, xb, yb);
    SlTri r;
    double bestd;
    float rho2;
    const bool cand = sl_best(L, -1, xb, yb, r, bestd, rho2);
    const bool ok = cand && (sl_fast(L, r, xb, yb, bestd, rho2) || sl_rank_ok(G, xb, yb, bestd, r.id, 0.0f, 0));
    double cn;
    if (ok) {
      cn = sl_value(r, xb, yb, c);
    } else {
      cn = c[g];
      nnf += 1.0;
    }
    stnt(cout + g, cn);
    if (notfound) notfound[i] = ok ? ((L.probe & 2) ? 2 : 0) : 1;  // probe bit 1: mark the slow rows
    swc += (wmix ? wmix[i] : 0.0) * cn;
  }
  const double a = block_sum(swc, sh), d = block_sum(nnf, sh);
  if (threadIdx.x == 0) {  // k_sl's partials of this block (the same grid) plus this pass's
    if (ro.out) {
      red_part(ro, part, 0, part[blockIdx.x] + a);
      red_part(ro, part, 1, part[SLB + blockIdx.x]);
      red_part(ro, part, 2, part[2 * SLB + blockIdx.x] + d);
    } else {
      part[blockIdx.x] += a;
      part[2 * SLB + blockIdx.x] += d;
    }
  }
  red_finish(ro, part, sh);
}

// ---- k_sl_wave: the second pass of the lattice locator with ONE WAVE PER QUEUED POINT.  k_sl_slow ran a queued
// point's general locate (every candidate cell of every macro face listed in q's macro-grid cell, up to ~20 x 18
// dependent coordinate loads) and its centroid rank count serially in one lane, on k_sl's full 8,192-block grid:
// at L7 796 points (0.006 % of the rows, r12n) took 290 us per step, the latency of the slowest lane.  Here the
// wave's 64 lanes test the candidates together (the answer is the passing triangle with the smallest (d^2, id)
// key: a margin / inner pass is the only passing triangle, so the sequential scan's early exits never change it),
// then count the centroids below it together (ballots; the sequential count's early exit only saves work), and
// lane 0 writes the value -- the same arithmetic per candidate, so the same bits as k_sl_slow.
// Work: k_sl's grid, block b adding its points' contributions to block b's partials (the sums' order is fixed).
// (d, id) key minimum over the wave (every lane gets it)
__device__ __forceinline__ void wave_min_key(double& d, int32_t& id) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double od = __shfl_xor(d, o, 64);
    const int32_t oi = __shfl_xor(id, o, 64);
    if (knn_less(od, oi, d, id)) {
      d = od;
      id = oi;
    }
  }
}
// the general lattice locate of one point by a whole wave (sl_best with home = -1): false when no cell passes
__device__ __forceinline__ bool sl_best_wave(const LatLocDev& L, double qx, double qy, SlTri& out, double& bestd,
                                             float& rho2) {
  const int lane = threadIdx.x & 63;
  const double gx = floor((qx - L.x0) * L.ihx), gy = floor((qy - L.y0) * L.ihy);
  const int32_t ci = !(gx >= 0.0) ? 0 : (gx >= (double)L.nx ? L.nx - 1 : (int32_t)gx);
  const int32_t cj = !(gy >= 0.0) ? 0 : (gy >= (double)L.ny ? L.ny - 1 : (int32_t)gy);
  const int64_t gc = (int64_t)cj * L.nx + ci;
  const int32_t n = L.n;
  const double dn = (double)n;
  const int32_t e0 = L.start[gc], e1 = L.start[gc + 1];
  double md = INFINITY;
  int32_t mid = 0x7fffffff;
  SlTri mine{};
  // candidate k = (face e0 + k / 18, cell k % 18): 3 rows j x 3 columns i x 2 orientations s around (u, v), the
  // sequential scan's cells; cell 0 of a face also reports its inner cell.  Chunks of 64 candidates, in the scan's
  // order, until one holds an inner cell or a margin pass (the only passing triangle then: the scan stops there too)
  const int32_t total = (e1 - e0) * 18;
  for (int32_t base = 0; base < total; base += 64) {
    const int32_t k = base + lane;
    bool hit = false;
    if (k < total) {
      const lat::SlFace& S = L.face[L.item[e0 + k / 18]];
      const int32_t c = k % 18;
      SlTri r;
      double d, u, v;
      if (sl_inner(L, S, qx, qy, r, d, u, v)) {
        hit = true;
        if (c == 0 && knn_less(d, r.id, md, mid)) {
          md = d;
          mid = r.id;
          mine = r;
        }
      } else if (u >= -SL_LDEL && v >= -SL_LDEL && u + v <= dn + SL_LDEL) {
        const int32_t i0 = min(max((int32_t)floor(u), 0), n - 1), j0 = min(max((int32_t)floor(v), 0), n - 1);
        const int32_t j = max(j0 - 1, 0) + c / 6, i = max(i0 - 1, 0) + (c / 2) % 3, s = c & 1;
        const double a = u - i, b = v - j;
        const bool near = !(j > j0 + 1 || i > i0 + 1 || i + j > n - 1) &&
                          (s == 0 ? (a >= -SL_LDEL && b >= -SL_LDEL && a + b <= 1.0 + SL_LDEL)
                                  : (i + j <= n - 2 && a <= 1.0 + SL_LDEL && b <= 1.0 + SL_LDEL && a + b >= 1.0 - SL_LDEL));
        if (near) {
          r = sl_cell(L, S, i, j, s);
          bool margin;
          if (sl_test(r, qx, qy, d, margin)) {
            hit = margin;
            if (knn_less(d, r.id, md, mid)) {
              md = d;
              mid = r.id;
              mine = r;
            }
          }
        }
      }
    }
    if (__ballot(hit)) break;
  }
  double bd = md;
  int32_t bid = mid;
  wave_min_key(bd, bid);
  if (bid == 0x7fffffff) return false;
  const uint64_t own = __ballot(md == bd && mid == bid);
  const int src = __ffsll((unsigned long long)own) - 1;  // (one lane holds the winning cell; ties are one triangle)
  out.x1 = __shfl(mine.x1, src, 64);
  out.y1 = __shfl(mine.y1, src, 64);
  out.x2 = __shfl(mine.x2, src, 64);
  out.y2 = __shfl(mine.y2, src, 64);
  out.x3 = __shfl(mine.x3, src, 64);
  out.y3 = __shfl(mine.y3, src, 64);
  out.a = __shfl(mine.a, src, 64);
  out.b = __shfl(mine.b, src, 64);
  out.d = __shfl(mine.d, src, 64);
  out.id = bid;
  bestd = bd;
  rho2 = L.rho2[bid];
  return true;
}
// sl_rank_ok by a whole wave: the centroids below (bestd, best) counted over the lanes (same result).  The grid rows
// of the box [q - R, q + R] are flattened into one entry range (each row's cells are one contiguous entry range; a
// wave scan of their lengths), so the lanes load entries of every row at once instead of one row after another
__device__ __forceinline__ bool sl_rank_ok_wave(const GridDev& G, double qx, double qy, double bestd, int32_t best) {
  const int lane = threadIdx.x & 63;
  const double R = sqrt(bestd) * (1.0 + 1e-9) + 1e-300;
  const int32_t i0 = gcell(qx - R, G.x0, G.hx, G.nx), i1 = gcell(qx + R, G.x0, G.hx, G.nx);
  const int32_t j0 = gcell(qy - R, G.y0, G.hy, G.ny), j1 = gcell(qy + R, G.y0, G.hy, G.ny);
  const int32_t nrow = j1 - j0 + 1;
  int cnt = 0;
  if (nrow > 64) {  // (a box taller than a wave: row after row)
    for (int32_t j = j0; j <= j1; ++j) {
      const int32_t f0 = G.start[(int64_t)j * G.nx + i0], f1 = G.start[(int64_t)j * G.nx + i1 + 1];
      for (int32_t e = f0; e < f1; e += 64) {
        bool below = false;
        if (e + lane < f1) {
          const double dx = G.px[e + lane] - qx, dy = G.py[e + lane] - qy;
          below = knn_less(dx * dx + dy * dy, G.item[e + lane], bestd, best);
        }
        cnt += __popcll(__ballot(below));
        if (cnt >= KNN) return false;
      }
    }
    return true;
  }
  int32_t f0 = 0, len = 0;
  if (lane < nrow) {
    const int64_t rb = (int64_t)(j0 + lane) * G.nx;
    f0 = G.start[rb + i0];
    len = G.start[rb + i1 + 1] - f0;
  }
  int32_t incl = len;  // inclusive scan of the row lengths
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  const int32_t total = __shfl(incl, 63, 64), excl = incl - len;
  for (int32_t base = 0; base < total; base += 64) {
    const int32_t t = base + lane;
    int32_t e = -1;
    for (int32_t r = 0; r < nrow; ++r) {  // (uniform loop: every lane shuffles)
      const int32_t ex = __shfl(excl, r, 64), ln = __shfl(len, r, 64), st = __shfl(f0, r, 64);
      if (t >= ex && t < ex + ln) e = st + (t - ex);
    }
    bool below = false;
    if (e >= 0) {
      const double dx = G.px[e] - qx, dy = G.py[e] - qy;
      below = knn_less(dx * dx + dy * dy, G.item[e], bestd, best);
    }
    cnt += __popcll(__ballot(below));
    if (cnt >= KNN) return false;
  }
  return true;
}
__global__ __launch_bounds__(BS) void k_sl_wave(MeshDev M, LatLocDev L, GridDev G, int64_t row0, int64_t n,
                                                const double* __restrict__ ux, const double* __restrict__ uy, double dt,
                                                const double* __restrict__ c, double* __restrict__ cout,
                                                const double* __restrict__ wmix, int32_t* notfound, double* part,
                                                const int32_t* __restrict__ queue, const int32_t* __restrict__ qcnt) {
  // k_sl's grid: block b runs the queues of k_sl's block b, wave w that of its wave w, one point at a time with the
  // whole wave (the in-step trace of a 1,024-wave grid taking k_sl's blocks in turn: 2.0 ms, r13d -- its few
  // long-lived blocks waited for wave slots beside the main stream)
  __shared__ double sh[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  const int32_t cnt = qcnt[BS / 64 * blockIdx.x + wv];
  double swc = 0.0, nnf = 0.0;
  for (int32_t p = 0; p < cnt; ++p) {
    const int64_t i = queue[r0 + (int64_t)(BS / 64 * (p >> 6) + wv) * 64 + (p & 63)], g = row0 + i;
    double xb, yb;
    sl_point(M, g, ux[VS * i], uy[VS * i], dt, xb, yb);
    SlTri r;
    double bestd;
    float rho2;
    const bool cand = sl_best_wave(L, xb, yb, r, bestd, rho2);
    const bool ok = cand && (sl_fast(L, r, xb, yb, bestd, rho2) || sl_rank_ok_wave(G, xb, yb, bestd, r.id));
    double cn;
    if (ok) {
      cn = sl_value(r, xb, yb, c);
    } else {
      cn = c[g];
      nnf += 1.0;
    }
    if (lane == 0) {
      stnt(cout + g, cn);
      if (notfound) notfound[i] = ok ? ((L.probe & 2) ? 2 : 0) : 1;
    }
    swc += (wmix ? wmix[i] : 0.0) * cn;
  }
  // k_sl's partials of this block plus this pass's (lane 0 of each wave carries its wave's sums)
  const double a = block_sum(lane == 0 ? swc : 0.0, sh), d = block_sum(lane == 0 ? nnf : 0.0, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] += a;
    part[2 * SLB + blockIdx.x] += d;
  }
}

// ---- The second pass over ONE numbered list (round 6).  k_sl_wave on k_sl's grid runs each wave's own queue one
// point after another, and the queued points cluster: at L7 ~35k departure points inside the squirmer (not found)
// plus ~800 rank counts (r12n) come from the few row blocks around the body, so a handful of waves ran hundreds of
// points each: 981 us per step in the window (r13g; k_sl_slow's one lane per point: 290 us, r12t).  Here
//   k_sl_qscan  numbers the entries of every per-wave queue (an exclusive scan of k_sl's wave counts, one block),
//   k_sl_wq     lets wave w of a large grid take the entries p = w, w + (number of waves), ... of that numbering:
//               the queue holding p by a 64-ary search of the offsets, the locate faces first (sl_best_wave2) and
//               the rank count by the whole wave; lane 0 writes c_new and marks a not-found entry by complementing
//               its row index in the queue,
//   k_sl_qsum   adds the queued rows' contributions to k_sl's block partials in k_sl_slow's order (lane p % 64 of
//               the wave that queued entry p), so the sums are k_sl_slow's, bit for bit.
constexpr int QSCAN_BS = 256;
constexpr int QSCAN_PER = (SLB * (BS / 64) + QSCAN_BS - 1) / QSCAN_BS;  // entries per thread (128 at SLB = 8192)
// one block of 256 threads (a 1,024-thread block waited for a whole CU's wave slots beside the main stream: 79 us with
// a loop of dependent loads per thread, r14z; 168 us with them issued together, r14k): wave w scans entries
// [w 64 QSCAN_PER, (w + 1) 64 QSCAN_PER) in chunks of 64 consecutive entries (one per lane), every load issued first
__global__ __launch_bounds__(QSCAN_BS) void k_sl_qscan(const int32_t* __restrict__ qcnt, int32_t nq,
                                                       int32_t* __restrict__ qoff) {
  __shared__ int32_t ws[QSCAN_BS / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int32_t base = wv * 64 * QSCAN_PER;
  int32_t v[QSCAN_PER];
#pragma unroll
  for (int k = 0; k < QSCAN_PER; ++k) {
    const int32_t e = base + k * 64 + lane;
    v[k] = e < nq ? qcnt[e] : 0;
  }
  int32_t run = 0;  // this wave's total before chunk k
#pragma unroll
  for (int k = 0; k < QSCAN_PER; ++k) {
    int32_t incl = v[k];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    const int32_t tot = __shfl(incl, 63, 64);
    v[k] = run + incl - v[k];  // (exclusive, within the wave)
    run += tot;
  }
  if (lane == 0) ws[wv] = run;
  __syncthreads();
  int32_t wb = 0;
  for (int k = 0; k < wv; ++k) wb += ws[k];
#pragma unroll
  for (int k = 0; k < QSCAN_PER; ++k) {
    const int32_t e = base + k * 64 + lane;
    if (e < nq) qoff[e] = wb + v[k];
  }
  if (threadIdx.x == 0) {
    int32_t t = 0;
    for (int k = 0; k < QSCAN_BS / 64; ++k) t += ws[k];
    qoff[nq] = t;
  }
}
// the general lattice locate of one point by a whole wave, faces first: the lanes take the candidate faces of q's
// macro-grid cell (sl_inner: an inner cell is the only passing triangle), then the cells around (u, v) of every face
// whose closure holds q up to SL_LDEL -- the candidates the sequential scan tests, with the same arithmetic each (it
// stops early only at a pass that is the only passing triangle): two rounds of dependent loads per 64 faces where
// sl_best_wave's 64-candidate chunks (3.6 faces each) took one round per chunk
__device__ __forceinline__ bool sl_best_wave2(const LatLocDev& L, double qx, double qy, SlTri& out, double& bestd,
                                              float& rho2) {
  const int lane = threadIdx.x & 63;
  const double gx = floor((qx - L.x0) * L.ihx), gy = floor((qy - L.y0) * L.ihy);
  const int32_t ci = !(gx >= 0.0) ? 0 : (gx >= (double)L.nx ? L.nx - 1 : (int32_t)gx);
  const int32_t cj = !(gy >= 0.0) ? 0 : (gy >= (double)L.ny ? L.ny - 1 : (int32_t)gy);
  const int64_t gc = (int64_t)cj * L.nx + ci;
  const int32_t n = L.n;
  const double dn = (double)n;
  const int32_t e0 = L.start[gc], e1 = L.start[gc + 1];
  double md = INFINITY;
  int32_t mid = 0x7fffffff;
  SlTri mine{};
  for (int32_t base = e0; base < e1; base += 64) {
    const int32_t e = base + lane;
    bool inner = false, near = false;
    double u = 0.0, v = 0.0;
    int32_t fi = 0;
    if (e < e1) {
      fi = L.item[e];
      SlTri r;
      double d;
      if (sl_inner(L, L.face[fi], qx, qy, r, d, u, v)) {
        inner = true;
        if (knn_less(d, r.id, md, mid)) {
          md = d;
          mid = r.id;
          mine = r;
        }
      } else {
        near = u >= -SL_LDEL && v >= -SL_LDEL && u + v <= dn + SL_LDEL;
      }
    }
    if (__ballot(inner)) break;
    const uint64_t nm = __ballot(near);
    const int32_t ncand = 18 * __popcll(nm);
    bool stop = false;
    for (int32_t t0 = 0; t0 < ncand; t0 += 64) {
      const int32_t t = t0 + lane;
      int32_t fl = 0;  // the lane that holds candidate t's face: the (t / 18)-th near face
      if (t < ncand) {
        uint64_t m = nm;
        for (int32_t k = t / 18; k > 0; --k) m &= m - 1;
        fl = __ffsll((unsigned long long)m) - 1;
      }
      const double fu = __shfl(u, fl, 64), fv = __shfl(v, fl, 64);
      const int32_t ff = __shfl(fi, fl, 64);
      bool hit = false;
      if (t < ncand) {
        const int32_t c = t % 18;
        const int32_t i0 = min(max((int32_t)floor(fu), 0), n - 1), j0 = min(max((int32_t)floor(fv), 0), n - 1);
        const int32_t j = max(j0 - 1, 0) + c / 6, i = max(i0 - 1, 0) + (c / 2) % 3, s = c & 1;
        const double a = fu - i, b = fv - j;
        const bool cnear = !(j > j0 + 1 || i > i0 + 1 || i + j > n - 1) &&
                           (s == 0 ? (a >= -SL_LDEL && b >= -SL_LDEL && a + b <= 1.0 + SL_LDEL)
                                   : (i + j <= n - 2 && a <= 1.0 + SL_LDEL && b <= 1.0 + SL_LDEL && a + b >= 1.0 - SL_LDEL));
        if (cnear) {
          const SlTri r = sl_cell(L, L.face[ff], i, j, s);
          double d;
          bool margin;
          if (sl_test(r, qx, qy, d, margin)) {
            hit = margin;
            if (knn_less(d, r.id, md, mid)) {
              md = d;
              mid = r.id;
              mine = r;
            }
          }
        }
      }
      if (__ballot(hit)) {
        stop = true;
        break;
      }
    }
    if (stop) break;
  }
  double bd = md;
  int32_t bid = mid;
  wave_min_key(bd, bid);
  if (bid == 0x7fffffff) return false;
  const int src = __ffsll((unsigned long long)__ballot(md == bd && mid == bid)) - 1;
  out.x1 = __shfl(mine.x1, src, 64);
  out.y1 = __shfl(mine.y1, src, 64);
  out.x2 = __shfl(mine.x2, src, 64);
  out.y2 = __shfl(mine.y2, src, 64);
  out.x3 = __shfl(mine.x3, src, 64);
  out.y3 = __shfl(mine.y3, src, 64);
  out.a = __shfl(mine.a, src, 64);
  out.b = __shfl(mine.b, src, 64);
  out.d = __shfl(mine.d, src, 64);
  out.id = bid;
  bestd = bd;
  rho2 = L.rho2[bid];
  return true;
}
__global__ __launch_bounds__(BS) void k_sl_wq(MeshDev M, LatLocDev L, GridDev G, int64_t row0, int64_t n, int32_t nb_sl,
                                              const double* __restrict__ ux, const double* __restrict__ uy, double dt,
                                              const double* __restrict__ c, double* __restrict__ cout,
                                              int32_t* notfound, int32_t* __restrict__ queue,
                                              const int32_t* __restrict__ qoff, int32_t nq) {
  const int lane = threadIdx.x & 63;
  const int32_t nw = (int32_t)gridDim.x * (BS / 64);
  const int32_t total = qoff[nq];
  const int64_t nsl = (n + 63) / 64;
  for (int32_t p = (int32_t)blockIdx.x * (BS / 64) + (int32_t)(threadIdx.x >> 6); p < total; p += nw) {
    // the queue holding entry p: the last q < nq with qoff[q] <= p (qoff[0] = 0), 64 offsets per round
    int32_t lo = 0, hi = nq, qlo = 0;
    while (hi - lo > 1) {
      const int32_t step = (hi - lo + 63) / 64, idx = lo + lane * step;
      const int32_t qv = idx < hi ? qoff[idx] : 0x7fffffff;
      const uint64_t m = __ballot(qv <= p);  // (lane 0: qoff[lo] <= p)
      const int last = 63 - __clzll((long long)m);
      qlo = __shfl(qv, last, 64);
      lo += last * step;
      hi = min(lo + step, hi);
    }
    const int32_t bq = lo / (BS / 64), wq = lo % (BS / 64), k = p - qlo;
    const int64_t r0 = ((nsl * bq) / nb_sl) * 64;  // block_rows of k_sl's block bq
    const int64_t e = r0 + (int64_t)((BS / 64) * (k >> 6) + wq) * 64 + (k & 63);
    const int32_t i = queue[e];
    const int64_t g = row0 + i;
    double xb, yb;
    sl_point(M, g, ux[VS * i], uy[VS * i], dt, xb, yb);
    SlTri r;
    double bestd;
    float rho2;
    const bool cand = sl_best_wave2(L, xb, yb, r, bestd, rho2);
    const bool ok = cand && (sl_fast(L, r, xb, yb, bestd, rho2) || sl_rank_ok_wave(G, xb, yb, bestd, r.id));
    const double cn = ok ? sl_value(r, xb, yb, c) : c[g];
    if (lane == 0) {
      stnt(cout + g, cn);
      if (notfound) notfound[i] = ok ? ((L.probe & 2) ? 2 : 0) : 1;
      if (!ok) queue[e] = ~i;
    }
  }
}
__global__ __launch_bounds__(BS) void k_sl_qsum(int64_t row0, int64_t n, const double* __restrict__ cout,
                                                const double* __restrict__ wmix, double* part,
                                                const int32_t* __restrict__ queue, const int32_t* __restrict__ qcnt) {
  __shared__ double sh[4];
  double swc = 0.0, nnf = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int32_t cnt = qcnt[BS / 64 * blockIdx.x + wv];
  for (int32_t p = lane; p < cnt; p += 64) {
    const int32_t e = queue[r0 + (int64_t)(BS / 64 * (p >> 6) + wv) * 64 + (p & 63)];
    const bool nf = e < 0;
    const int32_t i = nf ? ~e : e;
    const double cn = cout[row0 + i];
    if (nf) nnf += 1.0;
    swc += (wmix ? wmix[i] : 0.0) * cn;
  }
  const double a = block_sum(swc, sh), d = block_sum(nnf, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] += a;
    part[2 * SLB + blockIdx.x] += d;
  }
}

// Record locator (meshes without a red-refinement hierarchy: mesh.1, mesh_fine), whose k_sl has no fast path and
// queued every row for k_sl_slow's one lane per point: one wave per ROW instead, in one launch (k_sl_rec_wave), the
// records of q's grid cell tested by the lanes together (the passing record with the smallest (d^2, id) key, as
// sl_best's scan returns it) and the rank count as k_sl_wave's.  Same arithmetic per candidate: the same bits.
__device__ __forceinline__ bool sl_best_wave(const LocDev& L, double qx, double qy, SlTri& out, double& bestd,
                                             float& rho2) {
  const int lane = threadIdx.x & 63;
  const int32_t ci = gcell(qx, L.x0, L.hx, L.nx), cj = gcell(qy, L.y0, L.hy, L.ny);
  const int64_t cell = (int64_t)cj * L.nx + ci;
  const int32_t e0 = L.start[cell], e1 = L.start[cell + 1];
  double md = INFINITY;
  int32_t mid = 0x7fffffff, mpos = -1;
  SlTri mine{};
  for (int32_t base = e0; base < e1; base += 64) {  // (chunks until a margin pass, the only passing record then)
    const int32_t e = base + lane;
    bool hit = false;
    if (e < e1) {
      const int32_t pos = L.item[e];
      const SlTri r = sl_tri(L, pos);
      double d;
      bool margin;
      if (sl_test(r, qx, qy, d, margin)) {
        hit = margin;
        if (knn_less(d, r.id, md, mid)) {
          md = d;
          mid = r.id;
          mpos = pos;
          mine = r;
        }
      }
    }
    if (__ballot(hit)) break;
  }
  double bd = md;
  int32_t bid = mid;
  wave_min_key(bd, bid);
  if (bid == 0x7fffffff) return false;
  const int src = __ffsll((unsigned long long)__ballot(md == bd && mid == bid)) - 1;
  out.x1 = __shfl(mine.x1, src, 64);
  out.y1 = __shfl(mine.y1, src, 64);
  out.x2 = __shfl(mine.x2, src, 64);
  out.y2 = __shfl(mine.y2, src, 64);
  out.x3 = __shfl(mine.x3, src, 64);
  out.y3 = __shfl(mine.y3, src, 64);
  out.a = __shfl(mine.a, src, 64);
  out.b = __shfl(mine.b, src, 64);
  out.d = __shfl(mine.d, src, 64);
  out.id = bid;
  bestd = bd;
  rho2 = L.rho2[__shfl(mpos, src, 64)];
  return true;
}
// one row per wave (row = 4 blockIdx + wave); partials of the block's rows (its four waves in order) at the block's
// index, as k_sl + k_sl_slow leave them: [0] sum w c, [1] sum w, [2] not-found count
__global__ __launch_bounds__(BS) void k_sl_rec_wave(MeshDev M, LocDev L, GridDev G, int64_t row0, int64_t n,
                                                    const double* __restrict__ ux, const double* __restrict__ uy,
                                                    double dt, const double* __restrict__ c, double* __restrict__ cout,
                                                    const double* __restrict__ wmix, int32_t* notfound, double* part,
                                                    RedOut ro = RedOut{}) {
  __shared__ double sw_[3][BS / 64];
  __shared__ double sh[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * (BS / 64) + wv;
  double swc = 0.0, sw = 0.0, nnf = 0.0;
  if (i < n) {
    const int64_t g = row0 + i;
    double xb, yb;
    sl_point(M, g, ux[VS * i], uy[VS * i], dt, xb, yb);
    SlTri r;
    double bestd;
    float rho2;
    const bool cand = sl_best_wave(L, xb, yb, r, bestd, rho2);
    const bool ok = cand && (sl_fast(L, r, xb, yb, bestd, rho2) || sl_rank_ok_wave(G, xb, yb, bestd, r.id));
    double cn;
    if (ok) {
      cn = sl_value(r, xb, yb, c);
    } else {
      cn = c[g];
      nnf = 1.0;
    }
    if (lane == 0) {
      stnt(cout + g, cn);
      if (notfound) notfound[i] = ok ? ((L.probe & 2) ? 2 : 0) : 1;
    }
    const double w = wmix ? wmix[i] : 0.0;
    sw = w;
    swc = w * cn;
  }
  if (lane == 0) {
    sw_[0][wv] = swc;
    sw_[1][wv] = sw;
    sw_[2][wv] = nnf;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      double a = 0.0;
      for (int k = 0; k < BS / 64; ++k) a += sw_[v][k];
      if (ro.out) red_part(ro, part, v, a);
      else part[(int64_t)v * SLB + blockIdx.x] = a;
    }
  }
  red_finish(ro, part, sh);
}

// the locator's answer for every row's own node (q = its node after the x wrap: zero velocity), once
// at build: the triangle id, or -1 when no triangle is accepted
template <class LOC>
__global__ __launch_bounds__(BS) void k_sl_self(MeshDev M, LOC L, GridDev G, int64_t n, int32_t* __restrict__ out) {
  for (int64_t g = (int64_t)blockIdx.x * BS + threadIdx.x; g < n; g += (int64_t)gridDim.x * BS) {
    double xb, yb;
    sl_point(M, g, 0.0, 0.0, 0.0, xb, yb);
    SlTri r;
    double bestd;
    float rho2;
    const bool cand = sl_best(L, -1, xb, yb, r, bestd, rho2);
    const bool ok = cand && (sl_fast(L, r, xb, yb, bestd, rho2) || sl_rank_ok(G, xb, yb, bestd, r.id, 0.0f, 0));
    out[g] = ok ? r.id : -1;
  }
}

// ----------------------------------------------------------------------------- implicit dye variant
// scripts/good_visualization.py:700-718 (build_mass_and_convection, StokesColor.py:286-312).
// Per triangle t the convection weights w[3 t + j] = area/3 <u_c, grad_j>: u_c the vertex mean of u,
// grad_j = (y_{j+1} - y_{j+2}, x_{j+2} - x_{j+1}) / (2 |det|); C[i][j] is their sum over the triangles
// holding i and j, independent of i.  Degenerate triangles (|det| < 1e-14) contribute nothing.
__global__ __launch_bounds__(BS) void k_dye_w(MeshDev M, const double* __restrict__ ux, const double* __restrict__ uy,
                                              double* __restrict__ w) {
  for (int64_t t = (int64_t)blockIdx.x * BS + threadIdx.x; t < M.T; t += (int64_t)gridDim.x * BS) {
    const int32_t a = M.tri[3 * t], b = M.tri[3 * t + 1], d = M.tri[3 * t + 2];
    const double x1 = M.x[a], y1 = M.y[a], x2 = M.x[b], y2 = M.y[b], x3 = M.x[d], y3 = M.y[d];
    const double det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2);
    double w0 = 0.0, w1 = 0.0, w2 = 0.0;
    if (fabs(det) >= 1e-14) {
      const double area = 0.5 * fabs(det), den = 2 * fabs(det);
      const double ucx = ((ux[VS * a] + ux[VS * b]) + ux[VS * d]) / 3.0,
                   ucy = ((uy[VS * a] + uy[VS * b]) + uy[VS * d]) / 3.0;
      w0 = (area / 3) * (ucx * ((y2 - y3) / den) + ucy * ((x3 - x2) / den));
      w1 = (area / 3) * (ucx * ((y3 - y1) / den) + ucy * ((x1 - x3) / den));
      w2 = (area / 3) * (ucx * ((y1 - y2) / den) + ucy * ((x2 - x1) / den));
    }
    w[3 * t] = w0;
    w[3 * t + 1] = w1;
    w[3 * t + 2] = w2;
  }
}

// The merged operator's SELL values: slot -> Pp entry e (-1: padding, value 0); e's P entries k each
// give (M_k + dt (C_k + D K_k)) (+ G of the row's master on a diagonal, G = dt M_lumped div u); the
// slave rows of Pp (no P entries) are identity rows.
struct DyeDev {
  const int32_t* slot2e;
  const int64_t* eptr;
  const int32_t* ek;
  const double* mc;
  const double* kv;
  const int64_t* cptr;
  const int32_t* cw;
  const int32_t* diag_row;
  const int32_t* dof;
  const double* ml;
  int64_t nslots;
};
__global__ __launch_bounds__(BS) void k_dye_assemble(DyeDev D, const double* __restrict__ w,
                                                     const double* __restrict__ div, double dt, double diff,
                                                     double* __restrict__ val) {
  for (int64_t q = (int64_t)blockIdx.x * BS + threadIdx.x; q < D.nslots; q += (int64_t)gridDim.x * BS) {
    const int32_t e = D.slot2e[q];
    double v = 0.0;
    if (e >= 0) {
      const int64_t k0 = D.eptr[e], k1 = D.eptr[e + 1];
      if (k0 == k1) v = 1.0;
      for (int64_t z = k0; z < k1; ++z) {
        const int32_t k = D.ek[z];
        double ck = 0.0;
        for (int64_t y = D.cptr[k]; y < D.cptr[k + 1]; ++y) ck += w[D.cw[y]];
        double a = D.mc[k] + dt * (ck + diff * D.kv[k]);
        const int32_t r = D.diag_row[k];
        if (r >= 0) {
          const int32_t m = D.dof[r];
          a = a + dt * (D.ml[m] * div[m]);
        }
        v += a;
      }
    }
    val[q] = v;
  }
}
// rhs of a dye field that is not periodic at the pairs: the penalty's limit keeps
// x_s = x_m - delta_s, delta_s = (c_m - c_s) / 2, which adds (A_k - 2 M_k) delta_s to the merged row
// of every P entry k in a slave's column (rhs = P^T (M c + A delta) with M c taken on merged columns)
__global__ void k_dye_rhs_fix(int32_t nrows, const int32_t* __restrict__ srow, const int64_t* __restrict__ sptr,
                              const int32_t* __restrict__ sk, const int32_t* __restrict__ sc, DyeDev D,
                              const double* __restrict__ w, const double* __restrict__ div, double dt, double diff,
                              const double* __restrict__ c, double* __restrict__ rhs) {
  for (int32_t q = blockIdx.x * BS + threadIdx.x; q < nrows; q += gridDim.x * BS) {
    double add = 0.0;
    for (int64_t z = sptr[q]; z < sptr[q + 1]; ++z) {
      const int32_t k = sk[z], s = sc[z];
      const double delta = (c[D.dof[s]] - c[s]) / 2;
      double ck = 0.0;
      for (int64_t y = D.cptr[k]; y < D.cptr[k + 1]; ++y) ck += w[D.cw[y]];
      double a = D.mc[k] + dt * (ck + diff * D.kv[k]);
      const int32_t r = D.diag_row[k];
      if (r >= 0) {
        const int32_t m = D.dof[r];
        a = a + dt * (D.ml[m] * div[m]);
      }
      add += (a - 2.0 * D.mc[k]) * delta;
    }
    rhs[srow[q]] += add;
  }
}
__global__ void k_dye_dinv(int64_t n, const int64_t* __restrict__ diag_slot, const double* __restrict__ val,
                           double* __restrict__ dinv) {
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS)
    dinv[r] = 1.0 / val[diag_slot[r]];
}
// mixing partials of a dye field (the k_sl partial layout): [0] sum w c, [1] sum w, [2] 0
__global__ __launch_bounds__(BS) void k_wsum(int64_t row0, int64_t n, const double* __restrict__ c,
                                             const double* __restrict__ wmix, double* part) {
  __shared__ double sh[4];
  double swc = 0.0, sw = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
    const double w = wmix[i];
    swc += w * c[row0 + i];
    sw += w;
  }
  const double a = block_sum(swc, sh), b = block_sum(sw, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = a;
    part[SLB + blockIdx.x] = b;
    part[2 * SLB + blockIdx.x] = 0.0;
  }
}

// mixing_index second pass (StokesColor.py:399-401): partial sum w (c - mu)^2, mu from pass 1.
// copy_to (non-null): also copies the owned segment of c there (the new dye into the replica: one launch less than
// a separate device copy before the sums)
// (small-mesh graph: with the fused reduction, the block that reduced also appends the step record to the ring --
// k_stats_ring's work, after the value it reduced -- when ring is given; vals: the step's values)
__device__ __forceinline__ void stats_body(const double* vals, double* out, int parts);
__global__ __launch_bounds__(BS) void k_mix2(int64_t row0, int64_t n, const double* __restrict__ c,
                                             const double* __restrict__ wmix, const double* part1, int nb1,
                                             int stride1, double* part, RedOut ro = RedOut{},
                                             double* __restrict__ copy_to = nullptr, const double* vals = nullptr,
                                             double* ring = nullptr, int* count = nullptr, int parts = 0) {
  __shared__ double sh[4];
  const double swc = reduce_partials(part1, nb1, sh);
  const double sw = reduce_partials(part1 + stride1, nb1, sh);
  const double mu = swc / sw;
  double acc = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
    const double ci = c[row0 + i];
    if (copy_to) copy_to[row0 + i] = ci;
    const double d = ci - mu;
    acc += wmix[i] * (d * d);
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) red_part(ro, part, 0, t);
  if (red_finish(ro, part, sh) && ring && threadIdx.x == 0) {  // (thread 0 stored the reduced value itself)
    const int k = count[0];
    stats_body(vals, ring + 8 * (int64_t)k, parts);
    count[0] = k + 1;
  }
}

// ----------------------------------------------------------------------------- tracers
// StokesFood.py:482-499: LinearTriInterpolator (matplotlib plane coefficients, NaN outside the
// mesh), forward Euler, x mod 1, sticky capture.  One thread per tracer; full-mesh u replica.
// LinearTriInterpolator at one point (StokesFood.py:482-487, matplotlib TrapezoidMapTriFinder +
// plane coefficients): the first triangle of the point's grid cell whose three orientation tests pass
// (-1: outside the mesh); the interpolated velocity when u is given
__device__ __forceinline__ int32_t tracer_locate(const MeshDev& M, const GridDev& G, double px, double py) {
  if (!(isfinite(px) && isfinite(py))) return -1;
  const int32_t ci = gcell(px, G.x0, G.hx, G.nx), cj = gcell(py, G.y0, G.hy, G.ny);
  const bool inside = px >= G.x0 && px <= G.x0 + G.nx * G.hx && py >= G.y0 && py <= G.y0 + G.ny * G.hy;
  if (!inside) return -1;
  const int64_t c = (int64_t)cj * G.nx + ci;
  for (int32_t e = G.start[c]; e < G.start[c + 1]; ++e) {
    const int32_t t = G.item[e];
    const int32_t a = M.tri[3 * t], b = M.tri[3 * t + 1], d = M.tri[3 * t + 2];
    const double x1 = M.x[a], y1 = M.y[a], x2 = M.x[b], y2 = M.y[b], x3 = M.x[d], y3 = M.y[d];
    const double o1 = (x2 - x1) * (py - y1) - (y2 - y1) * (px - x1);
    const double o2 = (x3 - x2) * (py - y2) - (y3 - y2) * (px - x2);
    const double o3 = (x1 - x3) * (py - y3) - (y1 - y3) * (px - x3);
    if (o1 >= 0.0 && o2 >= 0.0 && o3 >= 0.0) return t;
  }
  return -1;
}
// (vs: the element stride of ux / uy)
__device__ __forceinline__ void tracer_interp(const MeshDev& M, int32_t t, const double* __restrict__ ux,
                                              const double* __restrict__ uy, int vs, double px, double py, double& vx,
                                              double& vy) {
  const int32_t a = M.tri[3 * t], b = M.tri[3 * t + 1], d = M.tri[3 * t + 2];
  const double x0 = M.x[a], y0 = M.y[a];
  const double s1x = M.x[b] - x0, s1y = M.y[b] - y0, s2x = M.x[d] - x0, s2y = M.y[d] - y0;
  const double nz = s1x * s2y - s1y * s2x;
  double zv[2];
  const double* uu[2] = {ux, uy};
#pragma unroll
  for (int q = 0; q < 2; ++q) {  // Triangulation::calculate_plane_coefficients
    const double z0 = uu[q][(int64_t)vs * a];
    const double s1z = uu[q][(int64_t)vs * b] - z0, s2z = uu[q][(int64_t)vs * d] - z0;
    const double nx = s1y * s2z - s1z * s2y;
    const double ny = s1z * s2x - s1x * s2z;
    const double pa = -nx / nz, pb = -ny / nz;
    const double pc = (nx * x0 + ny * y0 + nz * z0) / nz;
    zv[q] = pa * px + pb * py + pc;
  }
  vx = zv[0];
  vy = zv[1];
}
// forward Euler, x mod 1, sticky capture (StokesFood.py:488-499)
__device__ __forceinline__ double tracer_move(double* tx, double* ty, double* status, int32_t k, double vx, double vy,
                                              double dt, double cx, double cy, double capture) {
  const double px = tx[k], py = ty[k];
  double nx_ = px + vx * dt, ny_ = py + vy * dt;
  nx_ = py_mod(nx_, 1.0);
  tx[k] = nx_;
  ty[k] = ny_;
  const double ddx = nx_ - cx, ddy = ny_ - cy;
  const double dist = sqrt(ddx * ddx + ddy * ddy);
  if (dist <= capture) status[k] = 1.0;
  return status[k];
}

__global__ void k_tracer(MeshDev M, GridDev G, const double* __restrict__ ux, const double* __restrict__ uy,
                         int32_t ntr, double* tx, double* ty, double* status, double dt, double cx, double cy,
                         double capture, double* eaten_out) {
  __shared__ double sh[4];
  double eaten = 0.0;
  for (int32_t k = threadIdx.x; k < ntr; k += blockDim.x) {
    const double px = tx[k], py = ty[k];
    double vx = NAN, vy = NAN;
    const int32_t found = tracer_locate(M, G, px, py);
    if (found >= 0) tracer_interp(M, found, ux, uy, VS, px, py, vx, vy);
    eaten += tracer_move(tx, ty, status, k, vx, vy, dt, cx, cy, capture);
  }
  const double t = block_sum(eaten, sh);
  if (threadIdx.x == 0) *eaten_out = t;
}

// multi-rank tracer step, part 1: every rank interpolates the tracers whose triangle it owns (its
// first vertex is one of the rank's rows: the other two are then owned or ghosts, filled into the
// global-index arrays fx / fy); tv[3k..3k+2] = (vx, vy, 1) there, zeros elsewhere -- summed over ranks
__global__ void k_tracer_vel(MeshDev M, GridDev G, const double* __restrict__ fx, const double* __restrict__ fy,
                             int32_t ntr, const double* tx, const double* ty, int64_t own0, int64_t own1, double* tv) {
  for (int32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < ntr; k += gridDim.x * blockDim.x) {
    const double px = tx[k], py = ty[k];
    double vx = 0.0, vy = 0.0, f = 0.0;
    const int32_t t = tracer_locate(M, G, px, py);
    if (t >= 0 && M.tri[3 * t] >= own0 && M.tri[3 * t] < own1) {
      tracer_interp(M, t, fx, fy, 1, px, py, vx, vy);  // (plain full replicas)
      f = 1.0;
    }
    tv[3 * k] = vx;
    tv[3 * k + 1] = vy;
    tv[3 * k + 2] = f;
  }
}
// part 2 (after the all-reduce, identical on every rank): the move with the owner's velocity (NaN
// where no rank holds the tracer: outside the mesh)
__global__ void k_tracer_move(int32_t ntr, double* tx, double* ty, double* status, const double* tv, double dt,
                              double cx, double cy, double capture, double* eaten_out) {
  __shared__ double sh[4];
  double eaten = 0.0;
  for (int32_t k = threadIdx.x; k < ntr; k += blockDim.x) {
    const bool found = tv[3 * k + 2] > 0.5;
    eaten += tracer_move(tx, ty, status, k, found ? tv[3 * k] : NAN, found ? tv[3 * k + 1] : NAN, dt, cx, cy, capture);
  }
  const double t = block_sum(eaten, sh);
  if (threadIdx.x == 0) *eaten_out = t;
}
// ghost values of a local vector into their global positions of a full-size array
// (vs: the element stride of v)
__global__ void k_scatter_ghosts(int64_t ng, const int32_t* __restrict__ ghost_global, const double* __restrict__ v,
                                 double* __restrict__ full, int vs) {
  for (int64_t k = (int64_t)blockIdx.x * BS + threadIdx.x; k < ng; k += (int64_t)gridDim.x * BS)
    full[ghost_global[k]] = v[vs * k];
}
// out[i] = v[vs * i] (a strided component into a plain vector)
__global__ void k_unstride(int64_t n, const double* __restrict__ v, int vs, double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = v[vs * i];
}

// ----------------------------------------------------------------------------- device assembly
// buildStiffnessMatrix / buildLumpedMassMatrix / the lumped divergence and gradient coefficients
// (StokesColor.py:98-128, 130-284) on the device, row-parallel.  Every row gathers
// its incident triangles in ascending triangle order -- the order in which the reference's scatter
// loops add to each entry -- with pucfem_host.cpp assemble_stokes's arithmetic (no contraction), so
// the values are the host assembly's (and the sequential scatter's) bit for bit.
constexpr int ASM_MAXDEG = 32;  // incident triangles per node (red refinement keeps the coarse degrees)

// node -> number of incident triangles (internal node ids)
__global__ void k_inc_count(int64_t n3, const int32_t* __restrict__ tri, const int32_t* __restrict__ old2new,
                            int32_t* cnt) {
  for (int64_t q = (int64_t)blockIdx.x * BS + threadIdx.x; q < n3; q += (int64_t)gridDim.x * BS)
    atomicAdd(cnt + old2new[tri[q]], 1);
}
// node -> incident triangles (any order; k_inc_sort orders them)
__global__ void k_inc_fill(int64_t n3, const int32_t* __restrict__ tri, const int32_t* __restrict__ old2new,
                           const int64_t* __restrict__ ptr, int32_t* cur, int32_t* __restrict__ itri) {
  for (int64_t q = (int64_t)blockIdx.x * BS + threadIdx.x; q < n3; q += (int64_t)gridDim.x * BS) {
    const int32_t v = old2new[tri[q]];
    itri[ptr[v] + atomicAdd(cur + v, 1)] = (int32_t)(q / 3);
  }
}
// ascending triangle ids per node (insertion sort of the node's short list); err[0] = 1 when a node has
// more than ASM_MAXDEG triangles
__global__ void k_inc_sort(int64_t n, const int64_t* __restrict__ ptr, int32_t* __restrict__ itri, int* err) {
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) {
    const int64_t b = ptr[r], e = ptr[r + 1];
    if (e - b > ASM_MAXDEG) err[0] = 1;
    for (int64_t k = b + 1; k < e; ++k) {
      const int32_t t = itri[k];
      int64_t m = k;
      while (m > b && itri[m - 1] > t) {
        itri[m] = itri[m - 1];
        --m;
      }
      itri[m] = t;
    }
  }
}
// the sorted distinct vertices (internal ids) of row r's incident triangles; an isolated node keeps
// a diagonal entry (build_pattern)
__device__ __forceinline__ int asm_row_cols(int64_t r, const int64_t* __restrict__ ptr, const int32_t* __restrict__ itri,
                                            const int32_t* __restrict__ tri, const int32_t* __restrict__ old2new,
                                            int32_t (&c)[3 * ASM_MAXDEG]) {
  int len = 0;
  const int64_t b = ptr[r], e = min(ptr[r + 1], b + ASM_MAXDEG);
  for (int64_t q = b; q < e; ++q) {
    const int64_t t = itri[q];
    for (int j = 0; j < 3; ++j) {
      const int32_t v = old2new[tri[3 * t + j]];
      int m = len;
      while (m > 0 && c[m - 1] > v) --m;
      if (m > 0 && c[m - 1] == v) continue;
      for (int k = len; k > m; --k) c[k] = c[k - 1];
      c[m] = v;
      ++len;
    }
  }
  if (len == 0) c[len++] = (int32_t)r;
  return len;
}
__global__ void k_pat_count(int64_t n, const int64_t* __restrict__ ptr, const int32_t* __restrict__ itri,
                            const int32_t* __restrict__ tri, const int32_t* __restrict__ old2new, int32_t* __restrict__ cnt) {
  int32_t c[3 * ASM_MAXDEG];
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS)
    cnt[r] = asm_row_cols(r, ptr, itri, tri, old2new, c);
}
__global__ void k_pat_fill(int64_t n, const int64_t* __restrict__ ptr, const int32_t* __restrict__ itri,
                           const int32_t* __restrict__ tri, const int32_t* __restrict__ old2new,
                           const int64_t* __restrict__ rowptr, int32_t* __restrict__ col) {
  int32_t c[3 * ASM_MAXDEG];
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) {
    const int len = asm_row_cols(r, ptr, itri, tri, old2new, c);
    for (int k = 0; k < len; ++k) col[rowptr[r] + k] = c[k];
  }
}
// values of row r on the pattern (K, Gx, Gy, lumped mass M, area_sum), assemble_stokes's loop
__global__ void k_asm(int64_t n, const int64_t* __restrict__ ptr, const int32_t* __restrict__ itri,
                      const int32_t* __restrict__ tri, const int32_t* __restrict__ old2new, const double* __restrict__ x,
                      const double* __restrict__ y, const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                      double* __restrict__ K, double* __restrict__ Gx, double* __restrict__ Gy, double* __restrict__ M,
                      double* __restrict__ asum) {
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) {
    const int64_t b = rowptr[r], e = rowptr[r + 1];
    double m = 0.0, as = 0.0;
    for (int64_t q = ptr[r]; q < ptr[r + 1]; ++q) {
      const int64_t t = itri[q];
      const int32_t o[3] = {tri[3 * t], tri[3 * t + 1], tri[3 * t + 2]};
      const int32_t nn[3] = {old2new[o[0]], old2new[o[1]], old2new[o[2]]};
      const double x1 = x[o[0]], y1 = y[o[0]], x2 = x[o[1]], y2 = y[o[1]], x3 = x[o[2]], y3 = y[o[2]];
      const double det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2);  // StokesColor.py:277-283
      const double area = 0.5 * fabs(det);
      for (int i = 0; i < 3; ++i)
        if (nn[i] == r) m += area / 3.0;
      if (fabs(det) < 1e-14) continue;  // StokesColor.py:113, :146, :239
      const double yd[3] = {y2 - y3, y3 - y1, y1 - y2};
      const double xd[3] = {x3 - x2, x1 - x3, x2 - x1};
      const double den = 2 * fabs(det);
      const double inv2A = 1.0 / det;  // StokesColor.py:149 / :241
      const double a3 = area / 3.0;
      for (int i = 0; i < 3; ++i) {
        if (nn[i] != r) continue;
        as += a3;
        for (int j = 0; j < 3; ++j) {
          int64_t k = b;
          while (k < e && col[k] != nn[j]) ++k;
          K[k] += (yd[i] * yd[j] + xd[i] * xd[j]) / den;  // StokesColor.py:120-126
          Gx[k] += (yd[j] * inv2A) * a3;
          Gy[k] += (xd[j] * inv2A) * a3;
        }
      }
    }
    M[r] = m;
    asum[r] = as;
  }
}

// ----------------------------------------------------------------------------- misc
// 1-block reduction of nv partial arrays (sum or max) into out[0..nv): the consumers of a producer
// kernel's partials read one scalar.  RB threads, each with RU independent loads in flight (the
// partials are L2 / MALL misses; a dependent load chain per thread would take nb / RB round trips).
// Fixed combination order: deterministic for a given nb.  Block b reduces values b, b + grid, ...: a
// launch over nv blocks reduces every value at once (the projection's 2 m + 4 dots were 68 reductions
// in a row in one block, ~150 us), with the same per-value order as a one-block launch.
constexpr int RB = 1024, RU = 8;
template <int RB>
__global__ __launch_bounds__(RB) void k_reduce_t(const double* part, int nb, int stride, int nv, int is_max, double* out) {
  __shared__ double sh[RB / 64];
  for (int v = blockIdx.x; v < nv; v += gridDim.x) {
    const double* p = part + (int64_t)v * stride;
    double a[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) a[u] = 0.0;  // partial maxima are of |.|, >= 0
    for (int b0 = threadIdx.x; b0 < nb; b0 += RB * RU) {
      double t[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) t[u] = b0 + u * RB < nb ? p[b0 + u * RB] : 0.0;
#pragma unroll
      for (int u = 0; u < RU; ++u) a[u] = is_max ? fmax(a[u], t[u]) : a[u] + t[u];
    }
    double x = a[0];
#pragma unroll
    for (int u = 1; u < RU; ++u) x = is_max ? fmax(x, a[u]) : x + a[u];
    x = is_max ? wave_max(x) : wave_sum(x);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      double y = sh[0];
      for (int w = 1; w < RB / 64; ++w) y = is_max ? fmax(y, sh[w]) : y + sh[w];
      out[v] = y;
    }
  }
}
// one sum (k_reduce_t's order) into out[0], then k_conv's test on rr / bb (either may be out): the PCG's
// reduction of <r, r> and its convergence test in one launch (single rank: no all-reduce in between)
__global__ __launch_bounds__(RB) void k_reduce_conv(const double* part, int nb, int stride, double* out,
                                                    const double* rr, const double* bb, double tol2, int* ctl,
                                                    int it, double* note = nullptr) {
  __shared__ double sh[RB / 64];
  double a[RU];
#pragma unroll
  for (int u = 0; u < RU; ++u) a[u] = 0.0;
  for (int b0 = threadIdx.x; b0 < nb; b0 += RB * RU) {
    double t[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) t[u] = b0 + u * RB < nb ? part[b0 + u * RB] : 0.0;
#pragma unroll
    for (int u = 0; u < RU; ++u) a[u] += t[u];
  }
  double x = a[0];
#pragma unroll
  for (int u = 1; u < RU; ++u) x += a[u];
  x = wave_sum(x);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    double y = sh[0];
    for (int w = 1; w < RB / 64; ++w) y += sh[w];
    out[0] = y;
    if (note) {  // (k_conv's note)
      note[0] = rr[0];
      note[1] = bb[0];
    }
    if (ctl[0] == 0 && rr[0] <= tol2 * bb[0]) {  // k_conv
      ctl[0] = 1;
      ctl[1] = it;
    }
  }
}
// the step's reductions: 1,024 threads (RB)
constexpr auto k_reduce = k_reduce_t<RB>;

template <typename T>
__global__ void k_pack(int64_t n, const int32_t* __restrict__ idx, const T* __restrict__ a, const T* __restrict__ b,
                       T* __restrict__ out) {
  for (int64_t k = (int64_t)blockIdx.x * BS + threadIdx.x; k < n; k += (int64_t)gridDim.x * BS) {
    out[k] = a[idx[k]];
    if (b) out[n + k] = b[idx[k]];
  }
}

// per-step diagnostics -> stats record.
// vals: [0] max|div*| [1] max|final div| [2] sum w c [3] sum w [4] not-found [5] sum w (c-mu)^2 [6] eaten
// out : [0] max|div*| [1] max|final div| [2] I [3] mu [4] var [5] eaten [6] not-found
// parts & 1: max |div u*| out[0]; & 2: max |final div| out[1]; & 4: the dye records out[2..6]
// (2 and 4 are written by the side stream when the dye advection overlaps the next step)
__device__ __forceinline__ void stats_body(const double* vals, double* out, int parts) {
  {
    if (parts & 1) out[0] = vals[0];
    if (parts & 2) out[1] = vals[1];
    if (parts & 4) {
      const double W = vals[3];
      const double mu = vals[2] / W, var = vals[5] / W;
      out[2] = var / (mu * (1 - mu) + 1e-16);  // StokesColor.py:402
      out[3] = mu;
      out[4] = var;
      out[5] = vals[6];
      out[6] = vals[4];
    }
  }
}
__global__ void k_stats(const double* vals, double* out, int parts) {
  if (threadIdx.x == 0) stats_body(vals, out, parts);
}
// a replayed small-mesh step (Ctx::graph_mode): the record goes to slot *count of a device ring and the count moves
// on (one copy of the ring per pucfem_step call instead of a device copy per step)
__global__ void k_stats_ring(const double* vals, double* ring, int* count, int parts) {
  if (threadIdx.x == 0) {
    const int k = count[0];
    stats_body(vals, ring + 8 * (int64_t)k, parts);
    count[0] = k + 1;
  }
}

// ----------------------------------------------------------------------------- BiCGStab pieces (literal operators)
// a multigrid level's power iteration (Ctx::lmax_level_device): y = D^-1 A x from res = 0 - A x (k_resid with
// b = 0), partial sums of x.x and y.y (stride MAXB, the k_dot2 layout)
template <typename T>
__global__ __launch_bounds__(BS) void k_pow_step(int64_t n, const T* __restrict__ x, const T* __restrict__ res,
                                                 const T* __restrict__ dinv, T* __restrict__ y, double* part) {
  __shared__ double sh[4];
  double sx = 0.0, sy = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
    const T yi = dinv[i] * -res[i];
    y[i] = yi;
    sx += (double)x[i] * (double)x[i];
    sy += (double)yi * (double)yi;
  }
  const double t1 = block_sum(sx, sh), t2 = block_sum(sy, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = t1;
    part[MAXB + blockIdx.x] = t2;
  }
}
template <typename T>
__global__ void k_pow_scale(int64_t n, const T* __restrict__ y, double s, T* __restrict__ x) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) x[i] = (T)(s * (double)y[i]);
}
__global__ __launch_bounds__(BS) void k_dot2(int64_t n, const double* a, const double* b, const double* c,
                                             const double* d, double* part) {
  __shared__ double sh[4];
  double s1 = 0.0, s2 = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
    s1 += a[i] * b[i];
    if (c) s2 += c[i] * d[i];
  }
  const double t1 = block_sum(s1, sh), t2 = block_sum(s2, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = t1;
    part[MAXB + blockIdx.x] = t2;
  }
}
// generic: z = a*x + b*y + c*w with coefficients read from device scalars (sign flags on the host)
// partial (1 - min, max) of the back-traced y of the rows (StokesColor.py:362-366: y - dt u_y, clamped
// into [1e-12, 1 - 1e-12]; both in [0, 1], as k_reduce's maxima start at 0); part[b] = 1 - min,
// part[MAXB + b] = max
__global__ __launch_bounds__(BS) void k_yrange(int64_t n, const double* __restrict__ y, const double* __restrict__ vy,
                                               double dt, double* part) {
  __shared__ double sh[4];
  double lo = 0.0, hi = 0.0;  // lo holds 1 - min
  int64_t r0, r1;
  block_rows(n, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
    double yb = y[i] - dt * vy[VS * i] * 1.0;
    if (yb < 0.0) yb = 1e-12;
    if (yb > 1.0) yb = 1.0 - 1e-12;
    lo = fmax(lo, 1.0 - yb);
    hi = fmax(hi, yb);
  }
  const double a = block_max(lo, sh), b = block_max(hi, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = a;
    part[MAXB + blockIdx.x] = b;
  }
}
// out[2 W] = -inf except this rank's slot (the all-gather of one pair as a max all-reduce)
__global__ void k_place2(int world, int rank, const double* v, double* out) {
  for (int i = threadIdx.x; i < 2 * world; i += blockDim.x) out[i] = i / 2 == rank ? v[i % 2] : -INFINITY;
}
// partial max |v| (block max over the block's rows)
__global__ __launch_bounds__(BS) void k_absmax(int64_t n, const double* __restrict__ v, double* part) {
  __shared__ double sh[4];
  double m = 0.0;
  int64_t r0, r1;
  block_rows(n, r0, r1);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) m = fmax(m, fabs(v[i]));
  const double t = block_max(m, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}
__global__ void k_vmul(int64_t n, const double* a, const double* b, double* out) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = a[i] * b[i];
}
__global__ void k_axpbypcz(int64_t n, const double* ca, const double* x, const double* cb, const double* y,
                           const double* cc, const double* w, double sa, double sb, double sc, double* z) {
  const double a = sa * (ca ? *ca : 1.0), b = sb * (cb ? *cb : 1.0), c = sc * (cc ? *cc : 1.0);
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    double v = a * x[i];
    if (y) v += b * y[i];
    if (w) v += c * w[i];
    z[i] = v;
  }
}
__global__ void k_mul(int64_t n, const double* a, const double* b, double* z) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) z[i] = a[i] * b[i];
}
// scalar bookkeeping of BiCGStab; sc layout: [0] rho_old [1] alpha [2] omega [3] beta [4] rho [5] rr [6] tmp
__global__ __launch_bounds__(BS) void k_bicg_scalar(int stage, const double* part, int nb, double* sc) {
  __shared__ double sh[4];
  const double d1 = reduce_partials(part, nb, sh);
  const double d2 = reduce_partials(part + MAXB, nb, sh);
  if (threadIdx.x != 0) return;
  if (stage == 0) {  // d1 = <r^, r>, d2 = <r, r>
    sc[3] = (d1 / sc[0]) * (sc[1] / sc[2]);
    sc[4] = d1;
    sc[5] = d2;
  } else if (stage == 1) {  // d1 = <r^, v>
    sc[1] = sc[4] / d1;
  } else if (stage == 2) {  // d1 = <t, s>, d2 = <t, t>
    sc[2] = d1 / d2;
    sc[0] = sc[4];
  } else if (stage == 3) {  // d2 = <r, r>
    sc[5] = d2;
  }
}


// p = r + beta (p - omega v); ph = Dinv p
__global__ void k_bicg_p(int64_t n, const double* r, double* p, const double* v, const double* dinv, double* ph,
                         const double* sc) {
  const double beta = sc[3], omega = sc[2];
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    const double pv = r[i] + beta * (p[i] - omega * v[i]);
    p[i] = pv;
    ph[i] = dinv[i] * pv;
  }
}
// s = r - alpha v; sh = Dinv s
__global__ void k_bicg_s(int64_t n, const double* r, const double* v, const double* dinv, double* s, double* sh,
                         const double* sc) {
  const double alpha = sc[1];
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    const double sv = r[i] - alpha * v[i];
    s[i] = sv;
    sh[i] = dinv[i] * sv;
  }
}
// x += alpha ph + omega sh; r = s - omega t
__global__ void k_bicg_x(int64_t n, double* x, const double* ph, const double* sh, const double* s,
                         const double* t, double* r, const double* sc) {
  const double alpha = sc[1], omega = sc[2];
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    x[i] = x[i] + alpha * ph[i] + omega * sh[i];
    r[i] = s[i] - omega * t[i];
  }
}


// ----------------------------------------------------------------------------- multigrid (pressure)
// sum_k A[row, k] x[col_k] for one SELL slice lane: entry loop unrolled to WMAX (index / value loads
// issued before the dependent gathers), matrix streamed with non-temporal loads.
// VT: the stored value type (fp16 in the mixed-precision V-cycle, widened to T for the arithmetic).
// s must be wave-uniform (see wave_id); entries are summed in k order for every width.
template <bool C16, typename T, typename VT, typename G>
__device__ __forceinline__ T sell_row_dot_g(const SellDev& A, const VT* __restrict__ val, const G& gx, int64_t s,
                                            int lane) {
  const int64_t off = A.off[s];
  const int w = A.w[s];
  const int32_t base = (int32_t)(s * 64);
  T acc = 0;
  by_width(w, [&](auto wc) {
    constexpr int WN = decltype(wc)::value;
    if constexpr (WN > 0) {
      int32_t cj[WN];
      VT a[WN];
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        const int64_t e = off + (int64_t)k * 64 + lane;
        cj[k] = sell_col<C16>(A, e, base);
        a[k] = ldnt(val + e);
      }
#pragma unroll
      for (int k = 0; k < WN; ++k) acc += (T)a[k] * gx(cj[k]);
    } else {
      for (int k = 0; k < w; ++k) {
        const int64_t e = off + (int64_t)k * 64 + lane;
        acc += (T)ldnt(val + e) * gx(sell_col<C16>(A, e, base));
      }
    }
  });
  return acc;
}
template <bool C16, typename T, typename VT>
__device__ __forceinline__ T sell_row_dot(const SellDev& A, const VT* __restrict__ val, const T* __restrict__ x,
                                          int64_t s, int lane) {
  return sell_row_dot_g<C16, T>(A, val, [x](int32_t j) { return x[j]; }, s, lane);
}

// Chebyshev smoothing step of the Jacobi-preconditioned smoother on A x = b (pucfem_api.hip
// mg_smooth), mode
//   0: first step from x = 0:  d = c2 Dinv b, x_out = d
//   1: general step:           d = c1 d + c2 Dinv (b - A x_in), x_out = x_in + d
//   2: steps 1 and 2 fused:    x1 = c20 Dinv b is recomputed at the gathered columns (b and Dinv
//                              carry ghost entries), then step 2 as mode 1 with d = x1 -- bit-identical
//                              to modes 0 + 1 and one pass over the level's vectors cheaper
// rdot != null: partial <rdot, x_out> (the <r, z> of the preconditioned CG).
// T: the V-cycle's storage/arithmetic type (float in the mixed-precision cycle, double otherwise);
// TB: the right-hand side (the CG residual, double, on the finest level); TO: the output (double
// for the final step that writes the preconditioned residual z).
// LV: a level tag with no effect on the code (1: the finest level, 2: pucfem_bench_kernel), so that
// profilers report the finest level's launches apart from the coarser levels' ones.
// One Chebyshev step specialised on the mode and on whether <rdot, x_out> is accumulated: the row body
// is one basic block, so every load of a row -- the gathered x (or b and dinv), the row's b, d and
// rdot -- issues before the first use.  (With a runtime mode the row streams b / d sat behind the
// gathers' branch: two dependent round trips per row.)  Face rows run in groups of 4 per thread with
// all loads of the group first.
template <int MODE, bool RD, typename T, typename TB, typename TO, typename VT, bool C16>
__device__ __forceinline__ void cheb_body(const SellDev& A, const FaceDev& fc, const VT* __restrict__ val,
                                          const T* __restrict__ dinv, const TB* __restrict__ b,
                                          const T* __restrict__ xin, TO* __restrict__ xout, T* __restrict__ d,
                                          T tc1, T tc2, T tc20, const double* __restrict__ rdot, double& acc_rz,
                                          T* __restrict__ dout) {
  // the step's row update from A x (ax), the row's 1 / diag, b and (mode 1) x_in and d
  auto finish = [&](int64_t row, T ax, T di, T brow, T xrow, T drow, double rrow) {
    T dn, xo;
    if constexpr (MODE == 0) {
      dn = tc2 * di * brow;
      xo = dn;
    } else {
      const T x1 = MODE == 2 ? tc20 * di * brow : xrow;
      const T d1 = MODE == 2 ? x1 : drow;
      dn = tc1 * d1 + tc2 * di * (brow - ax);
      xo = x1 + dn;
    }
    stnt((dout ? dout : d) + row, dn);
    stnt(xout + row, (TO)xo);
    if constexpr (RD) acc_rz += rrow * (double)xo;
  };
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    constexpr int K = face_k(4);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      int32_t nb[K][6];
      bool in[K][6];
#pragma unroll
      for (int r = 0; r < K; ++r) lat::neighbours(F, fc.n, t[r], i[r], j[r], nb[r], in[r]);
      T a[7];
      face_kcoefs(fc, lf, nb[0], in[0], a);
      const T di = std::is_same<T, float>::value ? (T)fc.coef32[lf * lat::NCOEF + lat::C_DINV]
                                                 : (T)fc.coef[lf * lat::NCOEF + lat::C_DINV];
      T g[K][7], brow[K], xrow[K], drow[K];
      double rrow[K];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        const int64_t row = F.base + t[r];
        brow[r] = (T)b[row];
        xrow[r] = drow[r] = (T)0;
        rrow[r] = 0.0;
        if constexpr (MODE == 1) {
          xrow[r] = xin[row];
          drow[r] = d[row];
#pragma unroll
          for (int k = 0; k < 6; ++k) g[r][k] = xin[nb[r][k]];
        } else if constexpr (MODE == 2) {
          // x1 = c20 Dinv b at the gathered columns (skeleton columns: their own dinv)
#pragma unroll
          for (int k = 0; k < 6; ++k) g[r][k] = tc20 * (in[r][k] ? di : dinv[nb[r][k]]) * (T)b[nb[r][k]];
        }
        if constexpr (RD) rrow[r] = rdot[row];
      }
#pragma unroll
      for (int r = 0; r < K; ++r) {
        if (!ok[r]) continue;
        const int64_t row = F.base + t[r];
        T ax = 0;
        if constexpr (MODE == 1) {
          ax = a[0] * xrow[r];
#pragma unroll
          for (int k = 0; k < 6; ++k) ax += a[1 + k] * g[r][k];
        } else if constexpr (MODE == 2) {
          ax = a[0] * (tc20 * di * brow[r]);
#pragma unroll
          for (int k = 0; k < 6; ++k) ax += a[1 + k] * g[r][k];
        }
        finish(row, ax, di, brow[r], xrow[r], drow[r], rrow[r]);
      }
    });
  } else {
    int64_t s0, s1;
    block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
    const int lane = threadIdx.x & 63, wv = wave_id();
    for (int64_t s = s0 + wv; s < s1; s += 4) {
      const int64_t row = sell_row(A, s, lane);
      const int64_t rr = row >= 0 ? row : 0;
      const T brow = (T)b[rr], di = dinv[rr];
      const T xrow = MODE == 1 ? xin[rr] : (T)0, drow = MODE == 1 ? d[rr] : (T)0;
      // (ghost rows one layer out -- deep halos, row >= n_own -- add nothing to <rdot, x_out>)
      const double rrow = RD && row < A.n_own ? rdot[rr] : 0.0;
      T ax = 0;
      if constexpr (MODE == 1) ax = sell_row_dot<C16>(A, val, xin, s, lane);
      else if constexpr (MODE == 2)
        ax = sell_row_dot_g<C16, T>(A, val, [=](int32_t j) { return tc20 * dinv[j] * (T)b[j]; }, s, lane);
      if (row >= 0) finish(row, ax, di, brow, xrow, drow, rrow);
    }
  }
}

template <typename T, typename TB, typename TO, typename VT, bool C16, int LV = 0>
__global__ __launch_bounds__(BS) void k_cheb(SellDev A, FaceDev fc, const VT* __restrict__ val,
                                             const T* __restrict__ dinv, const TB* __restrict__ b,
                                             const T* __restrict__ xin, TO* __restrict__ xout, T* __restrict__ d,
                                             double c1, double c2, double c20, int mode, const int* ctl,
                                             const double* __restrict__ rdot, double* part, RedOut ro = RedOut{},
                                             T* __restrict__ dout = nullptr) {
  __shared__ double sh[4];
  if (ctl && ctl[0]) return;
  const T tc1 = (T)c1, tc2 = (T)c2, tc20 = (T)c20;
  double acc_rz = 0.0;
#define PUCFEM_CHEB(M, R) \
  cheb_body<M, R, T, TB, TO, VT, C16>(A, fc, val, dinv, b, xin, xout, d, tc1, tc2, tc20, rdot, acc_rz, dout)
  if (mode == 1) {
    if (rdot) PUCFEM_CHEB(1, true);
    else PUCFEM_CHEB(1, false);
  } else if (mode == 2) {
    if (rdot) PUCFEM_CHEB(2, true);
    else PUCFEM_CHEB(2, false);
  } else {
    if (rdot) PUCFEM_CHEB(0, true);
    else PUCFEM_CHEB(0, false);
  }
#undef PUCFEM_CHEB
  if (rdot) {
    const double t = block_sum(acc_rz, sh);
    if (threadIdx.x == 0) red_part(ro, part, 0, t);
    red_finish(ro, part, sh);
  }
}

// Two smoothing steps of the fp32 V-cycle's finest level on the face interiors in one pass (the viscous
// k_vcheb_pair's scheme: step a on the item's rows and their in-face neighbours, x_{a+1} in LDS, step a + 1
// on the item's rows; the skeleton rows run in k_cheb launches on the SELL part alone before and after,
// and this kernel writes x_{a+1} at the face rows next to the skeleton for the second of them).  Step a is
// mode MA of cheb_body (1: general, 2: the fused first two steps from x = 0), step a + 1 mode 1; the
// arithmetic per row is cheb_body's, so the result is bit-identical to two k_cheb launches.
struct MgPairVecs {
  const float* b;
  const float* dinv;  // 1 / diag at skeleton columns (mode 2)
  const float* xa;    // x_a (mode 1)
  float* xb;          // x_{a+1}: read at skeleton rows, written at the face rows next to the skeleton
  float* xc;          // x_{a+2}
  const float* da;    // d_a (mode 1)
  float* dc;          // d_{a+2}
};
template <int MA>
__global__ __launch_bounds__(BS) void k_cheb_pair(FaceDev fc, MgPairVecs v, float c1a, float c2a, float c20, float c1b,
                                                  float c2b, const int* ctl) {
  __shared__ float lx[VP_W];
  if (ctl && ctl[0]) return;
  const int32_t items = fc.nf * fc.cpf;
  int32_t it = blockIdx.x;
  if ((int32_t)gridDim.x == items && items >= 8 * 64) {  // XCD-grouped item order (face_rows)
    const int32_t x = it & 7, q = items >> 3, rem = items & 7;
    it = x * q + (x < rem ? x : rem) + (it >> 3);
  }
  const int32_t lf = it / fc.cpf;
  const lat::FaceTab F = fc.tab[lf];
  const int32_t n = fc.n;
  const int32_t t0 = (it - lf * fc.cpf) * (BS * FACE_RPT), t1 = min(t0 + BS * FACE_RPT, fc.F);
  const int32_t w0 = max(0, t0 - n), nw = min(fc.F, t1 + n) - w0;
  const float di = fc.coef32[lf * lat::NCOEF + lat::C_DINV];
  float a[7];
  {
    int32_t nb0[6];
    bool in0[6];
    int32_t i, j;
    lat::coords(t0, n, fc.rinv, i, j);
    lat::neighbours(F, n, t0, i, j, nb0, in0);
    face_kcoefs(fc, lf, nb0, in0, a);  // (the K stencil: one set per face)
  }
  float bt[VP_WK], dt[VP_WK];
#pragma unroll
  for (int k = 0; k < VP_WK; ++k) {
    const int32_t w = (int32_t)threadIdx.x + k * BS;
    bt[k] = dt[k] = 0.0f;
    if (w < nw) {
      const int32_t t = w0 + w;
      int32_t i, j, nb[6];
      bool in[6];
      lat::coords(t, n, fc.rinv, i, j);
      lat::neighbours(F, n, t, i, j, nb, in);
      const int64_t row = F.base + t;
      const float brow = v.b[row];
      float g[6], x1, d1, ax;
      if constexpr (MA == 1) {
        x1 = v.xa[row];
        d1 = v.da[row];
#pragma unroll
        for (int q = 0; q < 6; ++q) g[q] = v.xa[nb[q]];
        ax = a[0] * x1;
      } else {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          // (a skeleton neighbour's 1 / diag; loaded for every neighbour at a clamped address -- the row's own
          // entry when in-face -- instead of under a branch per neighbour: 92 -> 86 us isolated, r12d)
          const float dv = v.dinv[in[q] ? row : nb[q]];
          g[q] = c20 * (in[q] ? di : dv) * v.b[nb[q]];
        }
        ax = a[0] * (c20 * di * brow);
        x1 = c20 * di * brow;
        d1 = x1;
      }
#pragma unroll
      for (int q = 0; q < 6; ++q) ax += a[1 + q] * g[q];
      const float dn = c1a * d1 + c2a * di * (brow - ax);
      lx[w] = x1 + dn;
      bt[k] = brow;
      dt[k] = dn;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < VP_WK; ++k) {
    const int32_t w = (int32_t)threadIdx.x + k * BS;
    const int32_t t = w0 + w;
    if (w < nw && t >= t0 && t < t1) {
      int32_t i, j, nb[6];
      bool in[6];
      lat::coords(t, n, fc.rinv, i, j);
      lat::neighbours(F, n, t, i, j, nb, in);
      const int64_t row = F.base + t;
      const float xr = lx[w];
      float ax = a[0] * xr;
      bool bnd = false;
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const int32_t lw = min(max(nb[q] - F.base - w0, 0), nw - 1);
        ax += a[1 + q] * pair_nbr(lx, lw, v.xb, nb[q], in[q]);
        bnd = bnd || !in[q];
      }
      const float dn = c1b * dt[k] + c2b * di * (bt[k] - ax);
      if (bnd) v.xb[row] = xr;
      stnt(v.dc + row, dn);
      stnt(v.xc + row, xr + dn);
    }
  }
}

// res = b - A x
template <typename T, typename TB, typename VT, bool C16, int LV = 0>
__global__ __launch_bounds__(BS) void k_resid(SellDev A, FaceDev fc, const VT* __restrict__ val,
                                              const TB* __restrict__ b, const T* __restrict__ x,
                                              T* __restrict__ res, const int* ctl) {
  if (ctl && ctl[0]) return;
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    constexpr int K = face_k(4);  // groups of K rows per thread, every load first (face_rows_k)
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      int32_t nb[K][6];
      bool in[K][6];
#pragma unroll
      for (int r = 0; r < K; ++r) lat::neighbours(F, fc.n, t[r], i[r], j[r], nb[r], in[r]);
      T a[7];
      face_kcoefs(fc, lf, nb[0], in[0], a);
      T xv[K][7], bv[K];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        const int64_t row = F.base + t[r];
        xv[r][6] = x[row];
        bv[r] = (T)b[row];
#pragma unroll
        for (int k = 0; k < 6; ++k) xv[r][k] = x[nb[r][k]];
      }
#pragma unroll
      for (int r = 0; r < K; ++r) {
        if (!ok[r]) continue;
        T ax = a[0] * xv[r][6];
#pragma unroll
        for (int k = 0; k < 6; ++k) ax += a[1 + k] * xv[r][k];
        stnt(res + F.base + t[r], bv[r] - ax);
      }
    });
    return;
  }
  int64_t s0, s1;
  block_slices_n(A.nslices, role.nsk, role.idx, s0, s1);
  const int lane = threadIdx.x & 63, wv = wave_id();
  for (int64_t s = s0 + wv; s < s1; s += 4) {
    const int64_t row = sell_row(A, s, lane);
    const T ax = sell_row_dot<C16>(A, val, x, s, lane);
    if (row >= 0) stnt(res + row, (T)b[row] - ax);
  }
}

// Specialised on the direction (prolongation adds), so a row body is one basic block with every load of a
// 4-row group first.  Prolongation: v = (x[pa] + x[pb]) / 2 with pa = pb at the coarse lattice points
// (exact: (a + a) / 2 = a), so the four parity cases of (i, j) are one branch-free body instead of four
// divergent ones.
template <bool ADD, typename T>
__device__ __forceinline__ void transfer_body(const SellDev& M, const FaceDev& fc, const T* __restrict__ val,
                                              const T* __restrict__ x, T* __restrict__ y) {
  const BlockRole role = block_role(fc.nb);
  if (role.face) {
    const int32_t n2 = fc.n2;
    constexpr int K = face_k(4);
    face_rows_k<K>(fc, role.idx, fc.nb,
                   [&](const lat::FaceTab& F, int32_t lf, const int32_t (&t)[K], const int32_t (&i)[K],
                       const int32_t (&j)[K], const bool (&ok)[K]) {
      const lat::FaceTab G = fc.tab2[lf];
      if constexpr (ADD) {
        T xa[K], xb[K], yr[K];
#pragma unroll
        for (int r = 0; r < K; ++r) {
          const int32_t i0 = i[r] >> 1, i1 = (i[r] + 1) >> 1, j0 = j[r] >> 1, j1 = (j[r] + 1) >> 1;
          const bool ie = !(i[r] & 1), je = !(j[r] & 1);
          // even/even: the coarse point; even j: along i; even i: along j; odd/odd: the diagonal
          const int32_t pa = lat::point(G, n2, i0, (ie || je) ? j0 : j1);
          const int32_t pb = lat::point(G, n2, ie ? i0 : i1, je ? j0 : (ie ? j1 : j0));
          xa[r] = x[pa];
          xb[r] = x[pb];
          yr[r] = y[F.base + t[r]];
        }
#pragma unroll
        for (int r = 0; r < K; ++r)
          if (ok[r]) stnt(y + F.base + t[r], yr[r] + (T)0.5 * (xa[r] + xb[r]));
      } else {
        T v[K][7];
#pragma unroll
        for (int r = 0; r < K; ++r) {
          const int32_t I = 2 * i[r], J = 2 * j[r];
          v[r][0] = x[lat::point(G, n2, I, J)];
          v[r][1] = x[lat::point(G, n2, I - 1, J)];
          v[r][2] = x[lat::point(G, n2, I + 1, J)];
          v[r][3] = x[lat::point(G, n2, I, J - 1)];
          v[r][4] = x[lat::point(G, n2, I, J + 1)];
          v[r][5] = x[lat::point(G, n2, I + 1, J - 1)];
          v[r][6] = x[lat::point(G, n2, I - 1, J + 1)];
        }
#pragma unroll
        for (int r = 0; r < K; ++r) {
          if (!ok[r]) continue;
          const T h = v[r][1] + v[r][2] + v[r][3] + v[r][4] + v[r][5] + v[r][6];
          stnt(y + F.base + t[r], v[r][0] + (T)0.5 * h);
        }
      }
    });
    return;
  }
  int64_t s0, s1;
  block_slices_n(M.nslices, role.nsk, role.idx, s0, s1);
  const int lane = threadIdx.x & 63, wv = wave_id();
  for (int64_t s = s0 + wv; s < s1; s += 4) {
    const int64_t off = M.off[s];
    const int w = M.w[s];
    const int64_t row = sell_row(M, s, lane);
    const T yr = ADD && row >= 0 ? y[row] : (T)0;
    T acc = 0;
    // every column / value load of the slice before the gathers (widths 1-14 unrolled), summed in k order
    by_width(w, [&](auto wc) {
      constexpr int WN = decltype(wc)::value;
      if constexpr (WN > 0) {
        int32_t cj[WN];
        T av[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          cj[k] = M.col[e];
          av[k] = val[e];
        }
        T xv[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) xv[k] = x[cj[k]];
#pragma unroll
        for (int k = 0; k < WN; ++k) acc += av[k] * xv[k];
      } else {
        for (int k = 0; k < w; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          acc += val[e] * x[M.col[e]];
        }
      }
    });
    if (row >= 0) stnt(y + row, ADD ? yr + acc : acc);
  }
}

// y = T x (restriction) or y += T x (prolongation, add = 1).  Face part: prolongation rows are the
// fine level's interior nodes (linear interpolation from the coarse lattice, fc.tab2 = the coarse
// level's merged table); restriction rows the coarse level's interior nodes (the transpose: the
// fine node on top with weight 1 and its six midpoint neighbours with 1/2, all fine interior nodes).
template <typename T>
__global__ __launch_bounds__(BS) void k_transfer(SellDev M, FaceDev fc, const T* __restrict__ val,
                                                 const T* __restrict__ x, T* __restrict__ y, int add, const int* ctl) {
  if (ctl && ctl[0]) return;
  if (add) transfer_body<true>(M, fc, val, x, y);
  else transfer_body<false>(M, fc, val, x, y);
}

// coarse solve: y = Ainv x (dense, n x n row-major fp64, replicated); one wave per row
template <typename T, typename MT = double>
__global__ __launch_bounds__(BS) void k_dense_mv(int64_t n, const MT* __restrict__ Ainv, const T* __restrict__ x,
                                                 T* __restrict__ y, const int* ctl) {
  if (ctl && ctl[0]) return;
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += (int64_t)gridDim.x * 4) {
    const MT* a = Ainv + row * n;
    double acc = 0.0;
    for (int64_t j = lane; j < n; j += 64) acc += a[j] * (double)x[j];
    acc = wave_sum(acc);
    if (lane == 0) y[row] = (T)acc;
  }
}

// out[i] = full[idx[i]] (local owned + ghost entries from a replicated vector)
template <typename T>
__global__ void k_gather(int64_t n, const int32_t* __restrict__ idx, const T* __restrict__ full, T* __restrict__ out,
                         const int* ctl) {
  if (ctl && ctl[0]) return;
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = full[idx[i]];
}


// ----------------------------------------------------------------------------- small-mesh CG
// The whole CG solve in ONE workgroup of 1024 threads (16 waves) for operators of <= 4096 rows
// (mesh_fine: 1,067): the search direction lives in LDS, y / r / q of a thread's rows in
// registers, and -- when it fits -- the SELL matrix is staged into LDS once, so an iteration is
// an LDS-resident SpMV plus two block reductions (no kernel boundaries, no host round trips).
constexpr int CGB_THREADS = 1024;
constexpr int CGB_MAXR = 4;  // rows per thread -> n <= 4096

__device__ __forceinline__ double bsum1024(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < 16; ++w) t += red[w];
  return t;
}

template <int NR>
__global__ __launch_bounds__(CGB_THREADS) void k_cg_block(SellDev A, const double* __restrict__ val, double* y0,
                                                          double* y1, const double* b0, const double* b1,
                                                          double tol2, int maxit, int mat_lds, int* ctl,
                                                          int* it_out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ double red[16];
  const int n = (int)A.nrows;
  const int tid = threadIdx.x;
  double* p = lds;                                     // NR * n
  const int64_t pad = A.off[A.nslices];
  double* mval = lds + NR * n;                         // pad (if mat_lds)
  int32_t* mcol = reinterpret_cast<int32_t*>(mval + (mat_lds ? pad : 0));
  if (mat_lds) {
    for (int64_t e = tid; e < pad; e += CGB_THREADS) {
      mval[e] = val[e];
      mcol[e] = A.col[e];
    }
  }
  double* yv[2] = {y0, y1};
  const double* bv[2] = {b0, b1};
  double y[NR][CGB_MAXR], r[NR][CGB_MAXR], q[NR][CGB_MAXR];
  __syncthreads();
  // r = b - A y ; p = r
  double rr[NR], bb[NR];
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    rr[c] = 0.0;
    bb[c] = 0.0;
#pragma unroll
    for (int k = 0; k < CGB_MAXR; ++k) {
      const int i = tid + k * CGB_THREADS;
      y[c][k] = i < n ? yv[c][i] : 0.0;
    }
  }
  // stage y in p (the SpMV gathers from LDS)
#pragma unroll
  for (int c = 0; c < NR; ++c)
#pragma unroll
    for (int k = 0; k < CGB_MAXR; ++k) {
      const int i = tid + k * CGB_THREADS;
      if (i < n) p[c * n + i] = y[c][k];
    }
  __syncthreads();
  auto spmv = [&](double (&out)[NR][CGB_MAXR]) {
#pragma unroll
    for (int k = 0; k < CGB_MAXR; ++k) {
      const int i = tid + k * CGB_THREADS;
#pragma unroll
      for (int c = 0; c < NR; ++c) out[c][k] = 0.0;
      if (i < n) {
        const int64_t s = i >> 6;
        const int lane = i & 63;
        const int64_t off = A.off[s];
        const int w = A.w[s];
        for (int kk = 0; kk < w; ++kk) {
          const int64_t e = off + (int64_t)kk * 64 + lane;
          const double a = mat_lds ? mval[e] : val[e];
          const int32_t j = mat_lds ? mcol[e] : A.col[e];
#pragma unroll
          for (int c = 0; c < NR; ++c) out[c][k] += a * p[c * n + j];
        }
      }
    }
  };
  spmv(q);
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    double a = 0.0, bsq = 0.0;
#pragma unroll
    for (int k = 0; k < CGB_MAXR; ++k) {
      const int i = tid + k * CGB_THREADS;
      const double bi = i < n ? bv[c][i] : 0.0;
      r[c][k] = i < n ? bi - q[c][k] : 0.0;
      a += r[c][k] * r[c][k];
      bsq += bi * bi;
    }
    rr[c] = bsum1024(a, red);
    bb[c] = bsum1024(bsq, red);
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NR; ++c)
#pragma unroll
    for (int k = 0; k < CGB_MAXR; ++k) {
      const int i = tid + k * CGB_THREADS;
      if (i < n) p[c * n + i] = r[c][k];
    }
  __syncthreads();
  int it = 0;
  int status = 0;
  for (;;) {
    bool conv = true, bad = false;
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      conv = conv && (rr[c] <= tol2 * bb[c]);
      bad = bad || !isfinite(rr[c]);
    }
    if (conv || bad || it >= maxit) {
      status = conv ? 1 : (bad ? 3 : 2);
      break;
    }
    spmv(q);
    double alpha[NR], beta[NR];
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      double a = 0.0;
#pragma unroll
      for (int k = 0; k < CGB_MAXR; ++k) {
        const int i = tid + k * CGB_THREADS;
        if (i < n) a += p[c * n + i] * q[c][k];
      }
      alpha[c] = rr[c] / bsum1024(a, red);
    }
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      double a = 0.0;
#pragma unroll
      for (int k = 0; k < CGB_MAXR; ++k) {
        const int i = tid + k * CGB_THREADS;
        if (i < n) {
          y[c][k] += alpha[c] * p[c * n + i];
          r[c][k] -= alpha[c] * q[c][k];
          a += r[c][k] * r[c][k];
        }
      }
      const double rn = bsum1024(a, red);
      beta[c] = rn / rr[c];
      rr[c] = rn;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NR; ++c)
#pragma unroll
      for (int k = 0; k < CGB_MAXR; ++k) {
        const int i = tid + k * CGB_THREADS;
        if (i < n) p[c * n + i] = r[c][k] + beta[c] * p[c * n + i];
      }
    __syncthreads();
    ++it;
  }
#pragma unroll
  for (int c = 0; c < NR; ++c)
#pragma unroll
    for (int k = 0; k < CGB_MAXR; ++k) {
      const int i = tid + k * CGB_THREADS;
      if (i < n) yv[c][i] = y[c][k];
    }
  if (tid == 0) {
    ctl[0] = status;
    ctl[1] = it;
    if (it_out) *it_out = status == 1 ? it : -it - 1;
  }
}


// dense 2-RHS matvec (small-mesh direct viscous solve): y0 = A x0, y1 = A x1; one wave per row
// (x0 / x1 and y0 / y1: the interleaved velocity's components, stride VS)
// small meshes (Ctx::dense): a pressure solve of StokesColor.py:554-555 in ONE launch -- the restated right-hand side
// (k_pres_rhs: each master row takes its slave's entry, the free rows' mean is removed, slave rows are 0) formed at
// every column from braw and the reduced sum, the dense pseudo-inverse product (k_dense_mv), and p = y with every
// slave taking its master's value (k_cg_fin) -- the same operations in the same order as the three launches it
// replaces, so the same bits
// The right-hand side is formed once per block into LDS (n <= DENSE_LDS), so a row's loop issues only its
// independent matrix loads (the column-wise formation took three dependent loads per column and row: 13 us per
// solve on mesh_fine, r14c)
constexpr int DENSE_LDS = 1536;
__global__ __launch_bounds__(BS) void k_dense_pres(int64_t n, const double* __restrict__ Pinv,
                                                   const double* __restrict__ braw, const int32_t* __restrict__ slave_of,
                                                   const int32_t* __restrict__ master_of, const double* part_sum, int nb,
                                                   double inv_nfree, double* __restrict__ y, double* __restrict__ p) {
  __shared__ double sh[4];
  __shared__ double bl[DENSE_LDS];
  const double mean = reduce_partials(part_sum, nb, sh) * inv_nfree;
  for (int64_t j = threadIdx.x; j < n; j += BS) {
    double b;
    if (master_of[j] >= 0) {
      b = 0.0;
    } else {
      b = braw[j];
      if (slave_of[j] >= 0) b += braw[slave_of[j]];
      b = b - mean;
    }
    bl[j] = b;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += (int64_t)gridDim.x * 4) {
    const double* a = Pinv + row * n;
    double acc = 0.0;
    for (int64_t j = lane; j < n; j += 64) acc += a[j] * bl[j];
    acc = wave_sum(acc);
    if (lane == 0) {
      y[row] = acc;
      if (master_of[row] < 0) {
        p[row] = 1.0 * acc;
        if (slave_of[row] >= 0) p[slave_of[row]] = 1.0 * acc;
      }
    }
  }
}

// (x0, x1 staged in LDS once per block, n <= DENSE_LDS)
__global__ __launch_bounds__(BS) void k_dense_mv2(int64_t n, const double* __restrict__ Ainv, const double* __restrict__ x0,
                                                  const double* __restrict__ x1, double* __restrict__ y0,
                                                  double* __restrict__ y1) {
  __shared__ double xl[2 * DENSE_LDS];
  for (int64_t j = threadIdx.x; j < n; j += BS) {
    xl[2 * j] = x0[VS * j];
    xl[2 * j + 1] = x1[VS * j];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += (int64_t)gridDim.x * 4) {
    const double* a = Ainv + row * n;
    double s0 = 0.0, s1 = 0.0;
    for (int64_t j = lane; j < n; j += 64) {
      const double v = a[j];
      s0 += v * xl[2 * j];
      s1 += v * xl[2 * j + 1];
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if (lane == 0) {
      y0[VS * row] = s0;
      y1[VS * row] = s1;
    }
  }
}

// Small meshes (Ctx::dense): the first gradient projection (grad_proj_body, mode 0, SELL rows) and the velocity BCs
// after it (Ctx::bc) in one launch -- a Dirichlet row takes its value, a periodic copy row the projection of its
// source row (from the source's SELL entries at its slice position spos[src]: the same operations in the same order,
// so the value k_bc_apply copies), every other row its own.  One thread per (slice, lane).
__global__ __launch_bounds__(BS) void k_sell_pos(SellDev A, int32_t* __restrict__ spos) {
  for (int64_t t = (int64_t)blockIdx.x * BS + threadIdx.x; t < A.nslices * 64; t += (int64_t)gridDim.x * BS) {
    const int64_t row = sell_row(A, t >> 6, (int)(t & 63));
    if (row >= 0) spos[row] = (int32_t)t;
  }
}
template <bool C16>
__global__ __launch_bounds__(BS) void k_grad_proj_bc(SellDev A, const double* __restrict__ gx,
                                                     const double* __restrict__ gy, const double* __restrict__ p,
                                                     const double* __restrict__ as1, double dt, const double* usx,
                                                     double* ux, const int32_t* __restrict__ bsrc,
                                                     const int32_t* __restrict__ bdir, const int32_t* __restrict__ spos,
                                                     const double* __restrict__ dval, int ncomp) {
  for (int64_t t = (int64_t)blockIdx.x * BS + threadIdx.x; t < A.nslices * 64; t += (int64_t)gridDim.x * BS) {
    const int64_t row = sell_row(A, t >> 6, (int)(t & 63));
    if (row < 0) continue;
    const int32_t dj = bdir[row];
    if (dj >= 0) {
      reinterpret_cast<dbl2*>(ux)[row] = dbl2{dval[ncomp * dj], dval[ncomp * dj + 1]};
      continue;
    }
    const int32_t src = bsrc[row];
    const int64_t pos = src == row ? t : (int64_t)spos[src];
    const int64_t ss = pos >> 6;
    const int lane = (int)(pos & 63);
    const int64_t off = A.off[ss];
    const int w = A.w[ss];
    const int32_t base = (int32_t)(ss * 64);
    const dbl2 o = reinterpret_cast<const dbl2*>(usx)[src];
    const double d = as1[src];
    double ax = 0.0, ay = 0.0;
    for (int k = 0; k < w; ++k) {
      const int64_t e = off + (int64_t)k * 64 + lane;
      const double pj = p[sell_col<C16>(A, e, base)];
      ax += ldnt(gx + e) * pj;
      ay += ldnt(gy + e) * pj;
    }
    reinterpret_cast<dbl2*>(ux)[row] = dbl2{o.x - dt * (ax / d), o.y - dt * (ay / d)};
  }
}

// k_dense_mv2 with the velocity BCs of the solve's result (Ctx::bc) in the same launch: a Dirichlet row takes its
// value, a periodic copy row the product of its source's matrix row (the source's value before the BCs, which is what
// k_bc_apply copies: write sets are disjoint, chained sources are read before the writes), every other row its own
// product -- the same values bit for bit without k_bc_apply's launch (bsrc: the row whose product the row takes,
// bdir: the Dirichlet entry or -1)
__global__ __launch_bounds__(BS) void k_dense_mv2_bc(int64_t n, const double* __restrict__ Ainv,
                                                     const double* __restrict__ x0, const double* __restrict__ x1,
                                                     double* __restrict__ y0, double* __restrict__ y1,
                                                     const int32_t* __restrict__ bsrc, const int32_t* __restrict__ bdir,
                                                     const double* __restrict__ dval, int ncomp) {
  // (ncomp = 2: the velocity BCs set and copy both components)
  __shared__ double xl[2 * DENSE_LDS];
  for (int64_t j = threadIdx.x; j < n; j += BS) {
    xl[2 * j] = x0[VS * j];
    xl[2 * j + 1] = x1[VS * j];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += (int64_t)gridDim.x * 4) {
    const int32_t d = bdir[row];
    if (d >= 0) {
      if (lane == 0) {
        y0[VS * row] = dval[ncomp * d];
        y1[VS * row] = dval[ncomp * d + 1];
      }
      continue;
    }
    const double* a = Ainv + (int64_t)bsrc[row] * n;
    double s0 = 0.0, s1 = 0.0;
    for (int64_t j = lane; j < n; j += 64) {
      const double v = a[j];
      s0 += v * xl[2 * j];
      s1 += v * xl[2 * j + 1];
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if (lane == 0) {
      y0[VS * row] = s0;
      y1[VS * row] = s1;
    }
  }
}

}  // namespace dev
}  // namespace pucfem
