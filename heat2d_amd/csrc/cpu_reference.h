// heat2d_amd — CPU reference path.
//
// (1) `oracle_run`: the serial, bit-exact oracle on the whole NX×NY grid.  The BASELINE's
//     "serial CPU reference path (world_size=1)" does not exist in the reference (the
//     original aborts for P<4, B-7), so this implements its semantics directly:
//       fixed     — update ix in [1,NX-2], iy in [1,NY-2] (mpi_heat2Dn.c:162-169,225-237)
//       ghost-zero— update every cell against a zero ring (grad1612_mpi_heat.c:238-259)
//     with the convergence check of grad1612_mpi_heat.c:261-271 at the corrected cadence
//     (B-5): after committed step c with c % interval == 0.
// (2) `cpu_tile_advance`: K fused time steps of one halo-padded tile (the CPU twin of the
//     streaming HIP kernel), used by the CPU engine and the multi-process gloo tests.
#pragma once

#include <vector>

#include "h2d_common.h"

namespace h2d {

struct Physics {
  int boundary = kFixed;
  int precision = kRef;
  double cx = kCxDouble, cy = kCxDouble;
  bool periodic_x = false, periodic_y = false;
};

struct OracleResult {
  std::vector<float> grid;  // NX×NY, row-major
  int64_t steps_done = 0;
  bool converged = false;
  double residual = -1.0;   // last computed global residual (Σ Δ²), -1 if never checked
};

// `initial` may be null (then the field is built with `init`).
OracleResult oracle_run(int64_t NX, int64_t NY, int64_t steps, const Physics& ph, int init, bool convergence,
                        int64_t interval, double sensitivity, const float* initial = nullptr);

void init_global(std::vector<float>& u, int64_t NX, int64_t NY, int init);

// Advance a tile K levels: src storage (ghost ring valid to depth >= K) -> owned block of
// dst.  scratch0/scratch1 are two buffers of g.elems() floats.  Returns Σ (u_K - u_{K-1})²
// over the owned block when `residual` is set (else 0).
double cpu_tile_advance(const TileGeom& g, const Physics& ph, const float* src, float* dst, int K,
                        float* scratch0, float* scratch1, bool residual);

// Initialise a tile's storage: owned cells from the init formula, everything else zero.
void cpu_tile_init(const TileGeom& g, float* base, int init);

// Debug canary: NaN into every storage cell no valid update may read (see poisonable()).
void cpu_tile_poison(const TileGeom& g, float* base, bool fixed, bool per_x, bool per_y);

// Strided rectangle copies (pack / unpack / local halo copies).
void cpu_copy_rects(const std::vector<CopyDesc>& descs);

}  // namespace h2d
