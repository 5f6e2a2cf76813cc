// heat2d_amd — shared host/device definitions.
//
// Numerics contract: fp32 storage, the 5-point update evaluated as
//   (double)c + CX*((double)(s+n) - 2.0*(double)c) + CY*((double)(e+w) - 2.0*(double)c)
// with the neighbour pair sums as fp32 adds, left-to-right evaluation, no FMA contraction,
// rounded once to fp32.  This is exactly what the reference's C expression does:
//   grad1612_mpi_heat.c:241 (and :250-258), mpi_heat2Dn.c:225-237 (float cx promoted),
//   grad1612_cuda_heat.cu:55-62.
// Every translation unit of this library is compiled with -ffp-contract=off.
#pragma once

#include <cstdint>
#include <cstddef>

#if defined(__HIPCC__)
#define H2D_HD __host__ __device__
#else
#define H2D_HD
#endif

namespace h2d {

enum Boundary : int {
  kFixed = 0,      // Dirichlet on the NX×NY border: edge cells never change (mpi_heat2Dn.c:162-169, cuda:59)
  kGhostZero = 1,  // every owned cell updated against a zero ring outside the grid (grad1612_mpi_heat.c:238-259)
};

enum Precision : int {
  kRef = 0,   // fp64 expression, bit-exact with the reference
  kFp32 = 1,  // fp32 FMA fast path (documented tolerance, ≈1 ulp per step)
};

enum InitMode : int {
  kInitExact = 0,  // ix*(NX-ix-1)*iy*(NY-iy-1) in fp64, rounded to fp32 (the intended "center-hot" field)
  kInitInt32 = 1,  // the reference's int32 product with two's-complement wrap (mpi_heat2Dn.c:242-248, B-1)
  kInitZero = 2,   // all zeros (used by tests / resume)
};

// Coefficient presets: the original program stores cx/cy as float 0.1f promoted to double
// (mpi_heat2Dn.c:41-44); grad/CUDA use the double literal 0.1 (grad1612_mpi_heat.c:18-19).
constexpr double kCxDouble = 0.1;
constexpr double kCxFloat = (double)0.1f;

// ---------------------------------------------------------------------------------------
// Cell update.  n = u[i-1][j], s = u[i+1][j], w = u[i][j-1], e = u[i][j+1].
// ---------------------------------------------------------------------------------------
H2D_HD inline float update_ref(float c, float n, float s, float w, float e, double cx, double cy) {
  const float sn = s + n;  // fp32 add, as in C: float + float happens before the double subtraction
  const float ew = e + w;
  const double dc = (double)c;
  const double two_c = 2.0 * dc;
  double r = dc + cx * ((double)sn - two_c);
  r = r + cy * ((double)ew - two_c);
  return (float)r;
}

H2D_HD inline float update_f32(float c, float n, float s, float w, float e, float cx, float cy) {
  const float sn = s + n;
  const float ew = e + w;
  const float two_c = c + c;
  const float r = __builtin_fmaf(cx, sn - two_c, c);
  return __builtin_fmaf(cy, ew - two_c, r);
}

// ---------------------------------------------------------------------------------------
// Initial field ("center-hot", zero on the edges).
// ---------------------------------------------------------------------------------------
H2D_HD inline float init_exact(int64_t gx, int64_t gy, int64_t NX, int64_t NY) {
  const double a = (double)(gx * (NX - 1 - gx));
  const double b = (double)(gy * (NY - 1 - gy));
  return (float)(a * b);
}

H2D_HD inline float init_int32(int64_t gx, int64_t gy, int64_t NX, int64_t NY) {
  // ((ix*(nx-ix-1))*iy)*(ny-iy-1) in 32-bit two's-complement arithmetic, then int -> float.
  uint32_t p = (uint32_t)gx * (uint32_t)(NX - gx - 1);
  p = p * (uint32_t)gy;
  p = p * (uint32_t)(NY - gy - 1);
  return (float)(int32_t)p;
}

H2D_HD inline float init_value(int mode, int64_t gx, int64_t gy, int64_t NX, int64_t NY) {
  if (mode == kInitExact) return init_exact(gx, gy, NX, NY);
  if (mode == kInitInt32) return init_int32(gx, gy, NX, NY);
  return 0.0f;
}

// ---------------------------------------------------------------------------------------
// Halo-padded tile storage.  Owned cells (i, j), i in [0, xcell), j in [0, ycell), live at
// storage row i+G and column j+PL.  G rows of ghost above/below, PL >= G columns of ghost
// (padded to a multiple of 4 so every 16-byte lane load is aligned), row pitch a multiple of
// 64 floats (256 B).  Everything outside the owned block starts at zero and is only ever
// written by the halo exchange.
// ---------------------------------------------------------------------------------------
struct TileGeom {
  int64_t NX = 0, NY = 0;        // global grid
  int64_t gx0 = 0, gy0 = 0;      // global coordinate of owned (0,0)
  int64_t xcell = 0, ycell = 0;  // owned extents
  int64_t G = 0;                 // ghost depth (rows), also the max temporal block
  int64_t PL = 0;                // left column pad (>= G, multiple of 4)
  int64_t pitch = 0;             // floats per storage row
  int64_t srows = 0;             // storage rows = xcell + 2G

  H2D_HD int64_t idx(int64_t i, int64_t j) const { return (i + G) * pitch + (j + PL); }
  H2D_HD int64_t elems() const { return srows * pitch; }
};

// Streaming-kernel geometry: each wave owns a 256-column strip (4 columns per lane) and
// H output rows.  R = K rounded up to a multiple of 4 is the strip's column lead.
constexpr int kWaveCols = 256;
inline int64_t lead_cols(int K) { return (int64_t)((K + 3) & ~3); }
inline int64_t strip_out_cols(int K) { return kWaveCols - 2 * lead_cols(K); }
// Narrow strips of the persistent kernel: `cpl` columns per lane (4: 256-column strips, 2:
// 128-column strips), the lead R rounded to whole lanes.
inline int64_t wave_cols(int cpl) { return 64 * (int64_t)cpl; }
inline int64_t lead_cols(int K, int cpl) { return (int64_t)((K + cpl - 1) / cpl * cpl); }

// Directions of the 8-neighbour halo exchange (x = row index, y = column index).
enum Dir : int { kN = 0, kS, kW, kE, kNW, kNE, kSW, kSE, kNumDirs };
constexpr int kDirDx[kNumDirs] = {-1, +1, 0, 0, -1, -1, +1, +1};
constexpr int kDirDy[kNumDirs] = {0, 0, -1, +1, -1, +1, -1, +1};
constexpr int kDirOpp[kNumDirs] = {kS, kN, kE, kW, kSE, kSW, kNE, kNW};

// A rectangle of cells in owned coordinates (may extend into the ghost ring).
struct Rect {
  int64_t r0 = 0, c0 = 0, rows = 0, cols = 0;
  int64_t count() const { return rows * cols; }
};

// One strided 2-D copy, used for pack / unpack / local tile-to-tile halo copies.
struct CopyDesc {
  const float* src;
  float* dst;
  int64_t src_pitch;
  int64_t dst_pitch;
  int64_t rows;
  int64_t cols;
  int64_t tag = 0;  // integrity tag of the descriptor list (launch_copy_rects)
};

}  // namespace h2d

namespace h2d {

// Per-dimension cell mode: 0 = update, 1 = hold (fixed edge), 2 = zero (outside the grid).
// A cell's mode is the max of its row mode and its column mode.
H2D_HD inline int dim_mode(int64_t g, int64_t N, bool periodic, bool fixed) {
  if (periodic) return 0;
  if (g < 0 || g >= N) return 2;
  if (fixed && (g == 0 || g == N - 1)) return 1;
  return 0;
}

}  // namespace h2d

namespace h2d {

// Debug canary (poison mode): storage cell (i, j) in owned coordinates that no valid update
// may ever read — padding beyond the ghost ring, and (fixed mode) ghost cells outside the grid.
// Ghost cells inside the grid are also poisoned: the halo exchange must overwrite them first.
H2D_HD inline bool poisonable(const TileGeom& g, int64_t i, int64_t j, bool fixed, bool per_x, bool per_y) {
  if (i >= 0 && i < g.xcell && j >= 0 && j < g.ycell) return false;  // owned
  const bool in_ring = i >= -g.G && i < g.xcell + g.G && j >= -g.G && j < g.ycell + g.G;
  if (!in_ring) return true;
  const int64_t gx = g.gx0 + i, gy = g.gy0 + j;
  const bool outside = (!per_x && (gx < 0 || gx >= g.NX)) || (!per_y && (gy < 0 || gy >= g.NY));
  if (outside) return fixed;  // ghost-zero mode reads the zero ring
  return true;
}

}  // namespace h2d
