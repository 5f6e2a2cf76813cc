// heat2d_amd — HIP kernel launch interface (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "h2d_common.h"

#define H2D_HIP_CHECK(call)                                                                          \
  do {                                                                                               \
    hipError_t _e = (call);                                                                          \
    if (_e != hipSuccess) {                                                                          \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + __FILE__ + \
                               ":" + std::to_string(__LINE__) + ": " #call);                        \
    }                                                                                                \
  } while (0)

namespace h2d {

// Work unit of the streaming kernel: one wave = one 256-column strip × rows [x0, x0+h).
// flags: kEdgeCols — a column of the strip's window is a global edge / outside the grid;
//        kEdgeRows — a row of the unit's K-cone is.  Computed on the host (unit_edge_flags).
//        kUnitReverse — the wave streams its rows bottom-up (a bottom halo unit of the
//        signalled pipeline: its halo-dependent rows come first);
//        kUnitSigEnd — a signalling unit that signals at its end, not after sig_rows rows.
// cb: tile column of lane 0's first element (the wave's 256-column window is [cb, cb+256));
// [olo, ohi): the strip's output columns.  Interior strips have cb = olo - R; a strip against
// a FIXED global edge column is aligned to that edge and needs no outer cone (the held edge
// column is valid at every level), so it outputs 256 - R columns (strip_layout).
struct Unit {
  int strip;
  int x0;
  int h;
  int flags;
  int cb, olo, ohi;
};
constexpr int kEdgeCols = 1, kEdgeRows = 2, kUnitReverse = 4, kUnitSigEnd = 8;

int unit_edge_flags(const TileGeom& g, int K, int64_t x0, int64_t h, int64_t cb, bool fixed, bool per_x, bool per_y);
// Column strips of a tile for depth K.  Interior strips output 256 - 2R columns; with fixed
// edges a strip at a global edge column is edge-aligned and outputs 256 - R (4096 columns at
// K=8: 248 + 15×240 + 248 = 17 strips instead of 18).
struct Strip {
  int64_t cb, lo, hi;
};
std::vector<Strip> strip_layout(const TileGeom& g, int K, bool fixed, bool per_y);
// Cut a tile into work units for depth K: ~H rows per unit, edge units shortened by
// `edge_weight` so that every wave finishes at about the same time (one wave round).
// H > 0 fixes the rows of a plain unit; H == 0 sizes units to fill `capacity` resident waves.
std::vector<Unit> build_units(const TileGeom& g, int K, int H, bool fixed, bool per_x, bool per_y,
                              double edge_weight, int64_t capacity);
// Work units of a tile split for halo overlap: `boundary` units (their K-cone reaches a ghost
// side that has a peer; hb rows each) and `interior` units (everything else, sized to fill
// `capacity` resident waves).  Without peers every unit is interior.
struct UnitPlan {
  std::vector<Unit> interior, boundary;
};
UnitPlan plan_units(const TileGeom& g, int K, int H, bool fixed, bool per_x, bool per_y, double edge_weight,
                    int64_t capacity, const bool* peer, int hb);
// Resident waves of the streaming kernel on `device` (occupancy query × CUs × 4 waves/block).
int64_t stream_wave_capacity(int K, int precision, int device);

// Arguments of the temporally-blocked streaming stencil.
struct StreamArgs {
  const float* src;
  float* dst;
  const Unit* units;
  int nunits;
  int wout;    // output columns per strip (256 - 2R)
  int R;       // column lead (round_up(K,4))
  int64_t pitch, G, PL;
  int64_t xcell, ycell;
  int64_t gx0, gy0, NX, NY;
  double cx, cy;
  int fixed;
  int per_x, per_y;
  double* partials;  // per-unit residual partial sums (only read by the RESID variant)
  float* dummy;      // >= 256 floats: store target of non-output lanes in the branch-free path
  // Residual partial of unit w goes to slot (w + prot) mod nunits (a boundary-first list keeps
  // the interior-then-boundary summation order of the split launches).
  int prot = 0;
  // Signalled halo pipeline: units [0, nsignal) release their stores at system scope and add
  // 1 to *signal when done, so the comm stream can start the exchange mid-kernel.
  int nsignal = 0;
  unsigned long long* signal = nullptr;
  // > 0: a signalling unit signals as soon as its first sig_rows output rows (in streaming
  // order) are stored, then carries on with the rest of its rows (kUnitSigEnd: at its end)
  int sig_rows = 0;
  // Device-side halo wait: units [0, nsignal) first poll *halo_ready until it reaches
  // halo_need (the exchange that fills their ghost rows has landed); after halo_polls polls
  // they give up and set bit 2 of *timed_out.
  const unsigned long long* halo_ready = nullptr;
  unsigned long long halo_need = 0;
  long long halo_polls = 0;
  unsigned int* timed_out = nullptr;
  unsigned int* timed_out_host = nullptr;  // host-mapped mirror of *timed_out (polled by the host per chunk)
};

// Largest K with a compiled streaming kernel.
constexpr int kMaxK = 16;
bool stream_k_supported(int K);

void launch_stream(const StreamArgs& a, int K, int precision, bool residual, hipStream_t s);
// No-op launches of every compiled streaming kernel with K <= kmax (both residual variants of
// `precision`), so that no code object is first loaded inside a timed run (one TU per K).
void warm_stream_kernels(int precision, int kmax, hipStream_t s);
void launch_naive_step(const TileGeom& g, const float* src, float* dst, int precision, int boundary, double cx,
                       double cy, bool per_x, bool per_y, hipStream_t s);
void launch_init(const TileGeom& g, float* base, int init, hipStream_t s);
void launch_poison(const TileGeom& g, float* base, bool fixed, bool per_x, bool per_y, hipStream_t s);
void launch_copy_rects(const CopyDesc* d_descs, int ndesc, int64_t max_elems, hipStream_t s);
void launch_reduce_sum(const double* in, int n, double* out, hipStream_t s);
// One wave polls *counter (system-scope acquire loads, s_sleep between polls) until it reaches
// `target`; after `max_polls` it gives up and sets *timed_out (the caller reports it).
void launch_wait_counter(const unsigned long long* counter, unsigned long long target, unsigned int* timed_out,
                         unsigned int* timed_out_host, long long max_polls, hipStream_t s);
// *counter = value with a system-scope release, once every earlier command on `s` is done.
void launch_set_counter(unsigned long long* counter, unsigned long long value, hipStream_t s);
// Residual of a whole tile (Σ (a-b)² over owned cells) — used by tests/ops.
void launch_tile_residual(const TileGeom& g, const float* a, const float* b, double* partials, int npartials,
                          hipStream_t s);

// Small-grid resident solver: the whole grid lives in one workgroup's LDS for all steps.
bool lds_solver_fits(int64_t NX, int64_t NY);
void launch_lds_solver(const float* in, int64_t in_pitch, float* out, int64_t out_pitch, int64_t NX, int64_t NY,
                       int64_t steps, int precision,
                       int boundary, double cx, double cy, bool per_x, bool per_y, int conv_interval,
                       double sensitivity, long long* steps_done, double* residual, hipStream_t s);

}  // namespace h2d

namespace h2d {
template <int K>
void launch_stream_k(const StreamArgs& a, bool f32, bool resid, hipStream_t s);
template <int K>
int stream_blocks_per_cu(bool f32, bool resid);
}  // namespace h2d
