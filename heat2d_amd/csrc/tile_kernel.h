// heat2d_amd — launch interface of the LDS-tiled temporally-blocked kernel (tile_kernel.hip).
#pragma once

#include "kernels.h"

namespace h2d {

// Arguments of the LDS-tiled temporally-blocked kernel (tile_kernel.hip): one NT-thread
// workgroup per TX x TY tile, K steps per launch, region RY = TY + 2K columns (32, 64 or 128).
// (the device-resident block: ArgBlocks, kernels.h)
struct TileArgs {
  ArgHead head;
  const float* src;  // owned cell (0, 0) of the single tile (whole grid)
  float* dst;
  int64_t pitch;
  int NX, NY;
  int TX, TY, RY, K;
  int NT = 256;  // threads per workgroup: 256 or 1024
  int CPL = 4;   // cells per lane and level: 1, 2 or 4 (RY / CPL <= 64: a region row in one wave)
  int tiles_y = 0, ntiles = 0;  // set by prepare_tile
  double cx, cy;
  int fixed, per_x, per_y;
  double* partials;  // [ntiles] residual partials (residual launches)
  const unsigned long long* stop = nullptr;  // converged earlier: the launch does nothing
  float* keep = nullptr;  // residual launches: level K-1 of the owned tile (rollback state)
  // residual launches: the level whose change is summed (the convergence check step inside the
  // chunk; 0 = the last level K).  With rlev < K the launch goes on to level K, and a converged
  // check is rolled back by recomputation (keep must be null).
  int rlev = 0;
  DecideArgs dec;         // residual launches: fused sum + decision (last block; seq: TileDyn::seq)
  // Deferred decision (fused check, lone tile): the PREVIOUS launch's check left `pend_n`
  // residual partials at `pend`; one extra block of this launch (blockIdx ntiles) sums them in
  // one fixed order and records the decision (pend_dec) while the tile blocks compute this
  // launch SPECULATIVELY: a converged check makes the launches after this one no-ops (they read
  // the stop word), and this one writes a buffer that is not the check's input (the engine
  // rotates three buffers in this mode), so the rollback's recompute still finds that input.
  // The check launch itself only stores its partials: no drain, ticket or decision on the
  // critical path of either launch.
  const double* pend = nullptr;
  int pend_n = 0;
  DecideArgs pend_dec;  // (seq: TileDyn::pend_seq)
};
// Per-launch part of a tiled launch.
struct TileDyn {
  unsigned long long seq = 0;       // check number of a deciding residual launch
  unsigned long long pend_seq = 0;  // check number of the pending decision
  unsigned btag = 0;                // the block's ArgHead::btag
};
size_t tile_lds_bytes(int TX, int RY, int K);
// a lane owns up to kTileMaxSweeps region rows (kept in registers across the launch's levels)
constexpr int kTileMaxSweeps = 8;
bool tile_config_ok(int TX, int RY, int K, int CPL = 4, int NT = 256);
int tile_count(int NX, int NY, int TX, int TY);
// Check a launch's configuration and fill tiles_y / ntiles (before the block is made).
void prepare_tile(TileArgs& a);
// `blk`: the device-resident copy of the prepared `host` arguments.
void launch_tile(const TileArgs* blk, const TileArgs& host, const TileDyn& d, int precision, bool residual,
                 hipStream_t s);
// No-op launches of every tiled-kernel variant of `precision`: HIP loads a translation unit's
// code object at its first launch (deferred loading, tens to hundreds of microseconds), which
// must not land inside a timed run.
void warm_tile_kernels(int precision, hipStream_t s);  // (the zero block: no tiles)

}  // namespace h2d
