// heat2d_amd — domain decomposition and halo-exchange plans.
//
// Capability parity:
//   * 1-D row strips with uneven split (mpi_heat2Dn.c:87-104: averow = NX/P, the first
//     NX%P blocks get one extra row) -> gridx = P, gridy = 1.
//   * 2-D Cartesian blocks (grad1612_mpi_heat.c:46-81,113-147): rank r owns block row
//     px = r % GRIDX, block column py = r / GRIDX, non-periodic neighbours with "none" at
//     the domain edge (MPI_PROC_NULL).  Unlike the reference we also accept uneven splits
//     and compute coordinates from the topology itself (B-8), and periodic dims as an
//     extension (MPI_Cart_create's `periods`).
// The exchange plan is shared by every transport (RCCL, local multi-tile, host/gloo) so
// the message layout tested on CPU is the one RCCL moves on the GPU.
#pragma once

#include <array>
#include <string>
#include <vector>

#include "h2d_common.h"

namespace h2d {

struct Decomposition {
  int64_t NX = 0, NY = 0;
  int gridx = 1, gridy = 1;
  bool periodic_x = false, periodic_y = false;
  std::vector<int64_t> xstart, xcount;  // per block row
  std::vector<int64_t> ystart, ycount;  // per block column

  Decomposition() = default;
  Decomposition(int64_t nx, int64_t ny, int gx, int gy, bool px = false, bool py = false);

  int nranks() const { return gridx * gridy; }
  int px_of(int rank) const { return rank % gridx; }
  int py_of(int rank) const { return rank / gridx; }
  int rank_of(int px, int py) const { return py * gridx + px; }
  // Neighbour in direction d, or -1 at a non-periodic domain edge.
  int neighbor(int rank, int d) const;
  int64_t min_extent_x() const;
  int64_t min_extent_y() const;
  // Largest halo depth the decomposition supports (tiles must be at least that deep on
  // every split/periodic dimension).
  int64_t max_halo_depth() const;
  // Build the geometry of `rank`'s tile with ghost depth G.
  TileGeom tile(int rank, int64_t G) const;
};

// Per-tile exchange plan for halo depth K.
struct ExchangePlan {
  int K = 0;
  std::array<int, kNumDirs> peer;          // neighbour rank per direction (-1: none)
  std::array<Rect, kNumDirs> send_rect;    // owned cells sent in direction d
  std::array<Rect, kNumDirs> recv_rect;    // ghost cells filled from the neighbour on side d
  std::array<int64_t, kNumDirs> send_off;  // float offset of segment d in the packed send buffer
  std::array<int64_t, kNumDirs> recv_off;  // float offset of ghost side d in the packed recv buffer
  int64_t send_total = 0, recv_total = 0;
};

ExchangePlan make_plan(const Decomposition& dec, int rank, const TileGeom& g, int K);

// Builds the rectangle-copy descriptors for packing (owned -> send buffer) and unpacking
// (recv buffer -> ghost) a tile whose storage begins at `base`.
void plan_pack_descs(const ExchangePlan& p, const TileGeom& g, const float* base, float* sendbuf,
                     std::vector<CopyDesc>& out);
void plan_unpack_descs(const ExchangePlan& p, const TileGeom& g, float* base, const float* recvbuf,
                       std::vector<CopyDesc>& out);

// Geometry of a tile's storage: ghost depth G, pitch sized so every 256-column wave strip
// of the streaming kernel stays inside the allocation.
TileGeom make_tile_geom(int64_t NX, int64_t NY, int64_t gx0, int64_t gy0, int64_t xcell, int64_t ycell,
                        int64_t G);

std::string describe(const Decomposition& d);

}  // namespace h2d
