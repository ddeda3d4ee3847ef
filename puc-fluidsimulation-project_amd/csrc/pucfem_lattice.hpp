// Macro-face lattice layout of a red-refined hierarchy (hierarchical hybrid grids, Bergen & Ruede).
//
// Red refinement splits every triangle into four similar ones (the middle child is the parent
// rotated by 180 degrees), so after l levels the nodes inside a coarse ("macro") triangle form a
// structured lattice of n = 2^l segments per macro edge, and every small triangle in it has the
// macro triangle's shape.  P1 stiffness is scale-invariant in 2D, so the operator rows of the nodes
// strictly inside a macro face are ONE constant 7-point stencil per face (and per level), the lumped
// divergence / gradient rows one constant antisymmetric stencil scaled by 2^-l.  Those rows (97.5 %
// of the rows at L7) need no stored matrix: the kernels compute the neighbour addresses from the
// lattice position and read per-face coefficients.  The remaining "skeleton" rows (nodes on macro
// edges and vertices) keep the SELL-64 format.
//
// Node layout of a face interior (lattice coordinates i, j >= 1, i + j <= n - 1, i along the macro
// edge A->B, j along A->C): 0-based rows b = j - 1 of length n - 2 - b are stored in pairs (row b
// followed by row n - 3 - b), so a face's F = (n - 1)(n - 2) / 2 interior nodes form an
// (n - 2) / 2 x (n - 1) rectangle and the offset t of a node inside its face block maps to (i, j)
// with one division.  Neighbours inside the face are at fixed offsets from t; neighbours on the
// face's three macro edges come from per-face edge descriptors (first node, stride +-1, in local
// vector indices: owned rows or ghosts).
//
// This header is shared by the host runtime (pucfem_host.cpp: ordering, tables, the host reference
// of the face stencils used by the CPU tests) and the device kernels.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define PUCFEM_HD __host__ __device__
#else
#define PUCFEM_HD
#endif

namespace pucfem {
namespace lat {

// per-face table entry (int32): local index of the first interior node, then the three edge
// descriptors (first, stride) with node(AB, i) = ab0 + abs * i, node(AC, j) = ac0 + acs * j,
// node(BC, j) = bc0 + bcs * j (lattice coordinates of the point on that edge), then the face's
// coefficient record index
struct FaceTab {
  int32_t base, ab0, abs, ac0, acs, bc0, bcs, rec;
};
static_assert(sizeof(FaceTab) == 32, "FaceTab is 32 bytes");

// per-face coefficient record (doubles) -- see pucfem_host.cpp lattice_coefs
enum Coef {
  C_KAB = 0, C_KAC, C_KBC, C_KD,   // stiffness stencil: neighbours along AB, AC, BC; diagonal
  C_G1X, C_G1Y, C_G2X, C_G2Y, C_G3X, C_G3Y,  // lumped gradient stencil (antisymmetric, zero diagonal)
  C_AS1,                            // area_sum + 1e-12 (= lumped mass + 1e-12) of an interior node
  C_VS,                             // viscous Jacobi scale s = 1 / sqrt(1 + dt nu kd)
  C_VD,                             // viscous diagonal 1 + dt nu kd
  C_DTNU,                           // dt nu
  C_DINV,                           // 1 / kd (the multigrid smoother's Jacobi factor)
  C_PAD,
  NCOEF
};

PUCFEM_HD inline int32_t interior_count(int32_t n) { return n >= 3 ? (n - 1) * (n - 2) / 2 : 0; }

// offset of 0-based interior row b (j = b + 1) inside the face block
PUCFEM_HD inline int32_t rowbase(int32_t b, int32_t n) {
  const int32_t H = (n - 2) >> 1;
  return b < H ? b * (n - 1) : (n - 3 - b) * (n - 1) + b + 1;
}

// offset t -> lattice (i, j); rinv = 1 / (n - 1) in fp32 (exact for t < 2^16: the fractional part of
// (t + 0.5) / (n - 1) stays >= 0.5 / (n - 1) away from an integer)
PUCFEM_HD inline void coords(int32_t t, int32_t n, float rinv, int32_t& i, int32_t& j) {
  const int32_t p = (int32_t)(((float)t + 0.5f) * rinv);
  const int32_t q = t - p * (n - 1);
  const int32_t len = n - 2 - p;
  if (q < len) {
    j = p + 1;
    i = q + 1;
  } else {
    j = n - 2 - p;
    i = q - len + 1;
  }
}

// the 6 neighbours of interior node (i, j) at offset t of a face, in the order
//   0 (i-1, j)   1 (i+1, j)     -- direction AB
//   2 (i, j+1)   3 (i, j-1)     -- direction AC
//   4 (i-1, j+1) 5 (i+1, j-1)   -- direction BC (C - B)
// as local vector indices; inside[k] tells whether neighbour k is a face-interior node.
PUCFEM_HD inline void neighbours(const FaceTab& f, int32_t n, int32_t t, int32_t i, int32_t j, int32_t (&nb)[6],
                                 bool (&inside)[6]) {
  const int32_t H = (n - 2) >> 1;
  const int32_t b = j - 1;
  const int32_t c = f.base + t;
  // offset to the row above (b + 1) / below (b - 1) at the same i
  const int32_t up = b + 1 < H ? (n - 1) : (b + 1 == H ? H + 1 : -(n - 2));
  const int32_t dn = b < H ? -(n - 1) : (b == H ? -(H + 1) : (n - 2));
  const bool l_in = i >= 2, r_in = i + j <= n - 2, d_in = j >= 2;
  nb[0] = l_in ? c - 1 : f.ac0 + f.acs * j;
  nb[1] = r_in ? c + 1 : f.bc0 + f.bcs * j;
  nb[2] = r_in ? c + up : f.bc0 + f.bcs * (j + 1);
  nb[3] = d_in ? c + dn : f.ab0 + f.abs * i;
  nb[4] = l_in ? c + up - 1 : f.ac0 + f.acs * (j + 1);
  nb[5] = d_in ? c + dn + 1 : f.ab0 + f.abs * (i + 1);
  inside[0] = l_in;
  inside[1] = r_in;
  inside[2] = r_in;
  inside[3] = d_in;
  inside[4] = l_in;
  inside[5] = d_in;
}

// lattice point (i, j) of a face, anywhere on its closure except the corners (which no interior
// node and no prolongation row of an interior node ever reads)
PUCFEM_HD inline int32_t point(const FaceTab& f, int32_t n, int32_t i, int32_t j) {
  if (j == 0) return f.ab0 + f.abs * i;
  if (i == 0) return f.ac0 + f.acs * j;
  if (i + j == n) return f.bc0 + f.bcs * j;
  return f.base + rowbase(j - 1, n) + i - 1;
}

// any lattice point (i, j) of a face, corners included (va, vb, vc: the nodes at A, B, C)
PUCFEM_HD inline int32_t vertex(const FaceTab& f, int32_t va, int32_t vb, int32_t vc, int32_t n, int32_t i, int32_t j) {
  if (j == 0) return i == 0 ? va : (i == n ? vb : f.ab0 + f.abs * i);
  if (i == 0) return j == n ? vc : f.ac0 + f.acs * j;
  if (i + j == n) return f.bc0 + f.bcs * j;
  return f.base + rowbase(j - 1, n) + i - 1;
}

// The small triangles of a face: cell (i, j, s) with s = 0 the "up" triangle (i, j), (i+1, j), (i, j+1)
// (the face's own orientation; i + j <= n - 1) and s = 1 the "down" one (i+1, j), (i+1, j+1), (i, j+1)
// (i + j <= n - 2), both listed counter-clockwise.  Red refinement keeps every child's orientation, so
// a fine triangle's stored vertex order is one of the three rotations of its cell's list.
PUCFEM_HD inline void cell_vertices(int32_t i, int32_t j, int32_t s, int32_t (&pi)[3], int32_t (&pj)[3]) {
  if (s == 0) {
    pi[0] = i, pj[0] = j, pi[1] = i + 1, pj[1] = j, pi[2] = i, pj[2] = j + 1;
  } else {
    pi[0] = i + 1, pj[0] = j, pi[1] = i + 1, pj[1] = j + 1, pi[2] = i, pj[2] = j + 1;
  }
}
PUCFEM_HD inline int64_t cell_index(int32_t n, int32_t i, int32_t j, int32_t s) { return ((int64_t)j * n + i) * 2 + s; }

// Per-face data of the lattice point location (semi-Lagrangian step): the frame (lattice coordinates
// (u, v) = n M (q - A), M the inverse of [B - A, C - A]), the face table in GLOBAL internal ids, the
// corner nodes and the caller id of the face's first fine triangle (children of t are 4t .. 4t+3, so
// the fine triangles of face f are f 4^L .. (f + 1) 4^L - 1)
struct SlFace {
  double ax, ay, m00, m01, m10, m11;
  FaceTab tab;
  int32_t va, vb, vc, pad;
  int64_t t0;
};

}  // namespace lat
}  // namespace pucfem
