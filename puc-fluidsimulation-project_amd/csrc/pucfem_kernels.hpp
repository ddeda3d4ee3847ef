// Device kernels of libpucfem (gfx950 / CDNA4, wave64).
//
// Layout: every operator is SELL-64 -- one 64-row slice per wavefront, lane = row, entries
// column-major inside the slice so each `col`/`val` load of a wave is one contiguous 256 / 512 B
// segment.  A block (256 threads = 4 waves) owns a CONTIGUOUS range of slices (good L2 reuse of
// the gathered vector on the block's XCD).  Reductions are deterministic: each block writes one
// partial per value; the consumer kernel re-reduces the partial array in a fixed order in every
// block (no atomics, identical scalars in all blocks, bit-reproducible run to run).
//
// Compiled with -ffp-contract=off: the semi-Lagrangian / tracer / divergence formulas are the
// reference's, operation for operation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pucfem_lattice.hpp"

namespace pucfem {
namespace dev {

constexpr int BS = 256;     // threads per block
// max blocks of a partial-producing launch (= partial stride): a lattice kernel's full grid (one block per
// 1,024-row face item, dealt XCD-contiguously, plus the skeleton SELL blocks: ~15.3k at L7) fits, so the
// kernels that produce partials get the same item mapping as the others
constexpr int MAXB = 32768;
constexpr int EWB = 8192;   // max blocks of a row-wise (SELL / elementwise) grid
constexpr int KNN = 10;     // PointLocator k (StokesColor.py:324)
// max blocks (= partial stride) of the semi-Lagrangian kernel.  At L7 a block of 8192 runs ~1,700 rows: shorter-lived
// blocks free wave slots sooner for the main stream's kernels beside the dye stream (4096 -> 8192: k_sl 600 -> 520 us
// in-step, driver window +0.5-1 %, steps 100-119 +1.5-2 %; 6144 / 10240 / 16384 measured too, r11x / r11y)
#ifndef PUCFEM_SLB
#define PUCFEM_SLB 8192
#endif
constexpr int SLB = PUCFEM_SLB;
// Velocity storage: u and u* are interleaved (x, y) pairs (one 16-B gather per neighbour in k_div, the tracers and
// the dye weights); kernels take the component pointers ux = u2, uy = u2 + 1 and index them at VS * i
constexpr int VS = 2;
#ifndef PUCFEM_FACE_RPT
#define PUCFEM_FACE_RPT 4
#endif
constexpr int FACE_RPT = PUCFEM_FACE_RPT; // face-interior rows per thread of a lattice work item (BS * FACE_RPT rows of one face)
// row-group size of a face kernel (face_rows_k): the kernel's choice, at most the rows per thread
constexpr int face_k(int k) { return k < FACE_RPT ? k : FACE_RPT; }

struct SellDev {
  const int64_t* off;  // nslices+1
  const int32_t* w;    // nslices
  const int32_t* col;  // padded entries
  int64_t nslices, nrows;
  const int16_t* c16;  // same entries as int16 deltas from the slice's first row (band fits), or null
  int32_t wrap;        // c16: a decoded index below 0 wraps by this (the local length; ghosts at the end)
  // row list (lattice operators: the skeleton rows), nslices * 64 local output indices, -1 padded;
  // null: slice s holds rows s * 64 .. s * 64 + 63 (< nrows)
  const int32_t* rows;
  int64_t n_own;       // owned rows of the vectors the operator acts on (their ghosts follow)
};
// output row of lane `lane` of slice s, or -1
__device__ __forceinline__ int64_t sell_row(const SellDev& A, int64_t s, int lane) {
  const int64_t r = s * 64 + lane;
  if (A.rows) return A.rows[r];
  return r < A.nrows ? r : -1;
}

// The face-interior part of a lattice operator (pucfem_lattice.hpp): the last `nb` blocks of a launch
// run the interior rows of the rank's faces (chunks of BS * FACE_RPT consecutive rows of one face, so a
// block's face table entry and coefficients are uniform: scalar loads), the first blocks run the
// skeleton rows through the SELL (dispatched first: their rows are longer and their gathers slower, so
// they overlap the face blocks instead of trailing them).  nb = 0: no face part (plain SELL operators).
struct FaceDev {
  const lat::FaceTab* tab;   // row side: one entry per face
  const lat::FaceTab* tab2;  // transfers: the same faces on the other level (the gathered vector)
  const double* coef;        // lat::NCOEF doubles per record
  const float* coef32;
  const double* wsk;         // viscous (op 1): skeleton column weights s_j (0: Dirichlet column)
  int32_t nf, n, F, cpf;     // faces, lattice size, interior nodes per face, BS * FACE_RPT-row chunks per face
  int32_t n2;                // transfers: lattice size of the gathered level
  float rinv;                // 1 / (n - 1)
  int32_t nb;                // blocks on the face part
  int32_t op;                // 0 = stiffness-type stencil (K, merged pressure, level operators), 1 = scaled A_visc
};

template <class T>
__device__ __forceinline__ T ldnt(const T* p) {
  return __builtin_nontemporal_load(p);
}
// Non-temporal (streaming) store of a kernel's output vector: the lattice kernels' gathers keep the
// L2 busy with the input vectors, and ordinary stores of the outputs allocate L2 lines that then have
// to be written back; the streaming store halves the time of a gather kernel with two fp64 outputs
// (tools/face_lab.hip: 119 -> 61 us for the 14M-row direction kernel, the same bytes as a pure copy).
// (Write-through sc1 stores instead were measured 5 % slower at L7, round 3 r9b.)
template <class T>
__device__ __forceinline__ void stnt(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}
// column of entry e of the slice whose first row is `base`.  C16: the operator's band fits int16, so
// the index stream is 2 B/entry instead of 4 (strip ordering keeps every neighbour within a few
// strips of its row); NT: streamed with non-temporal loads (the gathered vector keeps L2 / MALL).
template <bool C16, bool NT = true>
__device__ __forceinline__ int32_t sell_col(const SellDev& A, int64_t e, int32_t base) {
  if constexpr (C16) {
    const int32_t j = base + (int32_t)(NT ? ldnt(A.c16 + e) : A.c16[e]);
    return j + ((j >> 31) & A.wrap);
  }
  else return NT ? ldnt(A.col + e) : A.col[e];
}

// ----------------------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
// result valid in every thread; `sh` must hold >= 4 doubles
__device__ __forceinline__ double block_sum(double v, double* sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return ((sh[0] + sh[1]) + (sh[2] + sh[3]));
}
__device__ __forceinline__ double block_max(double v, double* sh) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmax(fmax(sh[0], sh[1]), fmax(sh[2], sh[3]));
}
// Sum of `nb` partials at stride 1 starting at p (fixed order -> identical in every block).
// nb == 1 (a k_reduce scalar slot, the usual case): the value itself, no block barrier, so the
// consumers' scalar loads issue together
__device__ __forceinline__ double reduce_partials(const double* p, int nb, double* sh) {
  if (nb == 1) return p[0];
  double a = 0.0;
  for (int i = threadIdx.x; i < nb; i += BS) a += p[i];
  return block_sum(a, sh);
}
__device__ __forceinline__ double reduce_partials_max(const double* p, int nb, double* sh) {
  if (nb == 1) return fmax(0.0, p[0]);
  double a = 0.0;
  for (int i = threadIdx.x; i < nb; i += BS) a = fmax(a, p[i]);
  return block_max(a, sh);
}

// ---- in-kernel reduction of a launch's per-block partials (replaces the one-block k_reduce launch
// that followed every partial-producing kernel, and its kernel boundary).  Every block's thread 0
// stores the block's partials write-through (agent-scope relaxed atomic stores: `sc1`, no L2 copy
// kept), drains them (s_waitcnt vmcnt(0)) and draws a ticket from an agent-scope counter; the block
// drawing the last ticket reads every partial with `sc1` loads (agent-scope relaxed atomic loads, so no
// stale L1 / L2 line can serve them) in block order, reduces them in a fixed order, writes the values
// and resets the counter.  MI355X_MICROARCH.md "inter-workgroup visibility": the R1 counter form
// (every handed-off byte stored sc1 and drained before the ticket, every load of it sc1).
// Deterministic: for a given grid the combination order is fixed, whichever block finishes last.
struct RedOut {
  double* out;       // value v -> out[v]; null: no in-kernel reduction (the partials stay for k_reduce)
  double* out1;      // non-null: value 1 -> out1[0] instead (k_div: a max and a sum with different homes)
  unsigned* cnt;     // ticket counter, 0 between launches
  int nv;            // values
  int stride;        // partial stride (value v of block b at part[v * stride + b])
  unsigned maxmask;  // bit v: value v is a maximum (of values >= 0), else a sum
};
__device__ __forceinline__ void red_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double red_load(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Called by every thread of every block after thread 0 stored the block's partials with red_store
// (and, as every block must, with no early return before it).  sh: >= 4 doubles of LDS.
// all_waves: partials were stored by several waves (each drains its stores before the barrier).
// returns true in the block that reduced (the last one to finish), after its thread 0 stored the values
__device__ __forceinline__ bool red_finish(const RedOut& R, const double* part, double* sh, bool all_waves = false) {
  if (!R.out) return false;
  __shared__ int last;
  if (all_waves) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's partials have left the CU
    // acquire-release ticket: this block's partials are released with it, and the last block acquires
    // every other block's (the HIP memory model's guarantee, not only the sc1 stores' hardware behaviour)
    const unsigned t = __hip_atomic_fetch_add(R.cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every thread of the last block reads after the ticket
  const int nb = gridDim.x;
  for (int v = 0; v < R.nv; ++v) {
    const bool mx = (R.maxmask >> v) & 1u;
    const double* p = part + (int64_t)v * R.stride;
    double a = 0.0;
    for (int i = threadIdx.x; i < nb; i += BS) {
      const double x = red_load(p + i);
      a = mx ? fmax(a, x) : a + x;
    }
    const double r = mx ? block_max(a, sh) : block_sum(a, sh);
    if (threadIdx.x == 0) {
      if (v == 1 && R.out1) R.out1[0] = r;
      else R.out[v] = r;
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(R.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}
// thread 0: partial of value v of this block (stride R.stride when fused, else MAXB: the k_reduce layout)
__device__ __forceinline__ void red_part(const RedOut& R, double* part, int v, double x) {
  if (R.out) red_store(part + (int64_t)v * R.stride + blockIdx.x, x);
  else part[(int64_t)v * MAXB + blockIdx.x] = x;
}

// wave index inside the block as a wave-uniform (scalar) value: slice indices derived from it stay
// in SGPRs, so per-slice offsets / widths are scalar loads and width branches are uniform
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

template <int N>
struct Wn {
  static constexpr int value = N;
};
// f(Wn<w>{}) for the common SELL slice widths -- straight-line code in which every index / value
// load of the slice issues before the dependent gathers (widths 1-14: transfer rows are 1-9 wide,
// merged periodic-master stencil rows wider than the 7-entry ones) -- and f(Wn<0>{}) (a runtime-width loop) otherwise.  w must be wave-uniform.
template <class F>
__device__ __forceinline__ void by_width(int w, F&& f) {
  switch (w) {
    case 1: f(Wn<1>{}); break;
    case 2: f(Wn<2>{}); break;
    case 3: f(Wn<3>{}); break;
    case 4: f(Wn<4>{}); break;
    case 5: f(Wn<5>{}); break;
    case 6: f(Wn<6>{}); break;
    case 7: f(Wn<7>{}); break;
    case 8: f(Wn<8>{}); break;
    case 9: f(Wn<9>{}); break;
    case 10: f(Wn<10>{}); break;
    case 11: f(Wn<11>{}); break;
    case 12: f(Wn<12>{}); break;
    case 13: f(Wn<13>{}); break;
    case 14: f(Wn<14>{}); break;
    default: f(Wn<0>{}); break;
  }
}

// slice range of this block
__device__ __forceinline__ void block_slices(int64_t nslices, int64_t& s0, int64_t& s1) {
  const int64_t nb = gridDim.x, b = blockIdx.x;
  s0 = (nslices * b) / nb;
  s1 = (nslices * (b + 1)) / nb;
}
// slice range of block b of the nb blocks that run the SELL rows
__device__ __forceinline__ void block_slices_n(int64_t nslices, int64_t nb, int64_t b, int64_t& s0, int64_t& s1) {
  s0 = (nslices * b) / nb;
  s1 = (nslices * (b + 1)) / nb;
}
// Roles in a launch of face blocks (nbf of them: lattice face rows, face_rows / face_rows_k) and skeleton
// blocks (the other nsk = gridDim.x - nbf: SELL slices, block_slices_n).  The skeleton blocks are
// latency-bound (index -> value -> gather chains over few rows) and the face blocks stream, so with
// PUCFEM_SKEL_SPREAD = p > 0 the skeleton blocks are dealt in units of 8 consecutive blocks evenly over
// the first p % of the grid instead of all first; units of 8 keep a face block's index congruent to its
// hardware block index mod 8 (the face kernels' XCD-grouped item order) and a skeleton unit's blocks on
// the 8 XCDs.  p = 0: the skeleton blocks first (nsk a multiple of 8 either way: Ctx::sell_blocks).
#ifndef PUCFEM_SKEL_SPREAD
#define PUCFEM_SKEL_SPREAD 0
#endif
struct BlockRole {
  bool face;
  int32_t idx;  // face item / skeleton block index
  int32_t nsk;  // skeleton blocks
};
__device__ __forceinline__ BlockRole block_role(int32_t nbf) {
  const int32_t G = (int32_t)gridDim.x, b = (int32_t)blockIdx.x, nsk = G - nbf;
  if (nbf <= 0) return BlockRole{false, b, G};
  if (nsk <= 0) return BlockRole{true, b, 0};
  if (PUCFEM_SKEL_SPREAD > 0 && (nsk & 7) == 0) {
    const int32_t s8 = nsk >> 3, u = b >> 3;
    const int32_t span = (int32_t)(((int64_t)(G >> 3) * PUCFEM_SKEL_SPREAD) / 100);
    const int32_t P = span / s8 > 1 ? span / s8 : 1;
    const int32_t k = u / P;
    if (u - k * P == 0 && k < s8) return BlockRole{false, (k << 3) | (b & 7), nsk};
    return BlockRole{true, b - 8 * (k + 1 < s8 ? k + 1 : s8), nsk};
  }
  return b >= nsk ? BlockRole{true, b - nsk, nsk} : BlockRole{false, b, nsk};
}
// row range of this block for row-wise (non-SpMV) kernels, aligned to the same slices
__device__ __forceinline__ void block_rows(int64_t nrows, int64_t& r0, int64_t& r1) {
  int64_t s0, s1;
  block_slices((nrows + 63) / 64, s0, s1);
  r0 = s0 * 64;
  r1 = s1 * 64 < nrows ? s1 * 64 : nrows;
}

// Python / numpy float modulo (npy_divmod): result has the sign of the divisor.
__device__ __forceinline__ double py_mod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}
// py_mod(a, 1.0) without fmod's loop: a - trunc(a) is fmod(a, 1) exactly (the fractional bits of a
// are representable; NaN / inf propagate as fmod's do), then the same sign fix-up
__device__ __forceinline__ double py_mod1(double a) {
  double m = a - trunc(a);
  if (m != 0.0) {
    if (m < 0) m += 1.0;
  } else {
    m = 0.0;
  }
  return m;
}

}  // namespace dev
}  // namespace pucfem
