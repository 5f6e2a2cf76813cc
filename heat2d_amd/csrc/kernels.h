// heat2d_amd — HIP kernel launch interface (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
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
// links (2-D direct pipeline): bits 0-5 — the unit's K-cone reads the ghost side W, E, NW, NE,
// SW, SE (kLink*), so it waits for that neighbour's pushes; bits 8-13 — its outputs are part of
// that neighbour's halo, so it pushes them there and signals at its end.  kUnitNS: the unit is
// the top (north) or, with kUnitReverse, bottom (south) halo unit of its strip.
struct Unit {
  int strip;
  int x0;
  int h;
  int flags;
  int cb, olo, ohi;
  int links;
  // integrity tag of the unit list this unit was uploaded in (StreamArgs::utag): a wave that
  // reads a unit of another list (a stale upload, a reused allocation) reports it and stops
  int tag = 0;
};
constexpr int kEdgeCols = 1, kEdgeRows = 2, kUnitReverse = 4, kUnitSigEnd = 8, kUnitNS = 16;
// side links, indexed like Dir - 2 (kW .. kSE)
constexpr int kLinkW = 1, kLinkE = 2, kLinkNW = 4, kLinkNE = 8, kLinkSW = 16, kLinkSE = 32;
constexpr int kSideLinks = 6;
// columns of one ghost-column group of the 2-D direct receive buffer (>= the deepest lead R)
constexpr int kGhostGroup = 16;

int unit_edge_flags(const TileGeom& g, int K, int64_t x0, int64_t h, int64_t cb, bool fixed, bool per_x, bool per_y,
                    int64_t wcols = kWaveCols);
// Column strips of a tile for depth K.  Interior strips output 256 - 2R columns; with fixed
// edges a strip at a global edge column is edge-aligned and outputs 256 - R (4096 columns at
// K=8: 248 + 15×240 + 248 = 17 strips instead of 18).
struct Strip {
  int64_t cb, lo, hi;
};
// cpl: columns per lane (4: 256-column strips; 2: the persistent kernel's 128-column strips).
std::vector<Strip> strip_layout(const TileGeom& g, int K, bool fixed, bool per_y, int cpl = 4);
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
// row_edge_weight: the cost weight of units whose cone reaches a global edge ROW (<= 0: edge_weight)
// side_w / side_e: strips whose outputs reach the first / last side_cols columns push them to a
// W / E neighbour (2-D direct pipeline): their units cost side_weight per row.
// halo_n / halo_s (no-peer plans whose strip-end units become the N / S halo units of the
// signalled and direct pipelines): a strip's first / last unit also costs `halo_rows` extra rows
// (its halo wait before the first row: ~3.3 µs against ~0.9 for other units, tools/timeline.py
// --units) and never gets fewer than halo_min rows.
struct HaloCost {
  bool n = false, s = false;
  double rows = 0.0;
  int min_rows = 0;
};
UnitPlan plan_units(const TileGeom& g, int K, int H, bool fixed, bool per_x, bool per_y, double edge_weight,
                    int64_t capacity, const bool* peer, int hb, double row_edge_weight = -1.0,
                    double side_weight = 1.0, int side_cols = 0, bool side_w = false, bool side_e = false,
                    const HaloCost& halo = HaloCost{});
// Resident waves of the streaming kernel on `device` (occupancy query × CUs × 4 waves/block).
int64_t stream_wave_capacity(int K, int precision, int device);

// Host-mapped record of the device-side convergence decisions.
struct ConvHost {
  unsigned long long stop_seq;  // 0: running, else the sequence number of the converged check
  double residual;              // total of the converged check
  double last;                  // total of the latest check
  unsigned long long checks;
};
// Convergence decision of check `seq` made on the device by whoever holds the total: the last
// wave of a residual launch (fused epilogue), or a reduction kernel.  ticket != nullptr: the
// launch's residual partials are summed and decided in-kernel by the wave whose ticket add
// comes last (it resets the ticket for the next check).  Inside a device-resident argument block
// `seq` is not used: the check number is a per-launch value (StreamDyn::seq, TileDyn::seq).
struct DecideArgs {
  unsigned int* ticket = nullptr;
  double* total = nullptr;
  unsigned long long* stop = nullptr;
  ConvHost* host = nullptr;
  double sens = 0.0;
  unsigned long long seq = 0;
};

// Integrity bits of the engine's device error word (StreamArgs::timed_out, shared with the
// bounded-wait timeouts 1/2/4/8): a launch that sees inconsistent inputs reports instead of
// computing on them, and the host names the cause (Engine::poll_abort).
constexpr unsigned kIntegArgs = 16u;     // kernel arguments: torn per-launch part, or a block the launch does not name
constexpr unsigned kIntegUnits = 32u;    // a unit's tag is not the tag of the list the launch names
constexpr unsigned kIntegReplay = 64u;   // a launch ran with the arguments of an earlier launch
constexpr unsigned kIntegDescs = 128u;   // a copy descriptor's tag is not the list's tag
constexpr unsigned kIntegOrder = 256u;   // a stencil launch started before its exchange copy finished
constexpr unsigned kIntegOrder2 = 512u;  // an exchange copy started before the stencil launches before it finished

// ---- kernel arguments: device-resident blocks + a small per-launch part ---------------------
// The stencil kernels take (1) a pointer to an immutable, device-resident argument block with
// everything a plan fixes — buffers, unit lists, geometry, halo wiring — and (2) a small by-value
// struct with what changes per launch (launch id, halo counts, chunk numbers, check number).
// Blocks are uploaded once per distinct content (ArgBlocks) and never rewritten while any launch
// can read them, so a launch reads only ~100 bytes of kernel arguments, once per wave — which
// makes the library's host-memory kernel arguments free (round 4's ~750-byte by-value structs
// cost +12 % per launch there: docs/ARCHITECTURE.md, "Kernel arguments").
// Every block starts with this header: ArgBlocks stamps a process-wide tag into it, the launch
// passes the same tag by value, and the kernel compares the two (kIntegArgs).
struct ArgHead {
  unsigned btag = 0;
  unsigned bytes = 0;
};

// Per-launch part of a streaming launch.
struct StreamDyn {
  // launch id (engine launches: > 0, increasing in stream order; 0: no integrity checks)
  unsigned long long lid = 0;
  // halo counts this launch's halo units wait for, per direction (Dir: N, S, W, E, NW, NE, SW, SE)
  unsigned long long need[kNumDirs] = {};
  unsigned long long copies_need = 0;  // serial pipeline: exchange copy blocks completed before this launch
  // check number of a deciding residual launch (DecideArgs::seq), or of the pending decision
  // the launch's extra block makes (StreamArgs::pend: a lone tile, whose launches never decide
  // in-launch)
  unsigned long long seq = 0;
  int nunits = 0;                      // == the block's nunits (the launcher's grid size)
  bool pend = false;                   // == (the block's pend != nullptr): one more block
  unsigned btag = 0;                   // the block's ArgHead::btag
};
// The kernel receives the per-launch scalars as separate scalar kernel arguments, read once at the
// wave's start with the block pointer (kept in SGPRs, never reloaded); the halo counts come by
// value behind them and only halo units read them.
struct StreamNeed {
  unsigned long long v[kNumDirs];
};

// Arguments of the temporally-blocked streaming stencil (the device-resident block).
struct StreamArgs {
  ArgHead head;
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
  // Halo units [0, nsignal) of the signalled / direct pipelines.  Direction d of a unit: 0 = a
  // top unit (its ghost rows are the north halo), 1 = a bottom unit (kUnitReverse, south halo).
  //   wait[d]:         before reading ghost rows, poll *wait[d] until it reaches StreamDyn::need[d]
  //                    (bounded: after halo_polls polls give up and report a timeout);
  //   hsrc[d]:         read the ghost rows from here instead of src (storage-equivalent base:
  //                    ghost row i lives at hsrc[d] + (G + i) * pitch + PL);
  //   push[d]:         also store the first sig_rows output rows here (row-0-equivalent base:
  //                    tile row i lives at push[d] + i * pitch + PL) — the neighbour's receive
  //                    buffer, mapped over xGMI by IPC;
  //   sig[d]:          once those rows are stored, release them at system scope and add 1 here.
  // sig_rows > 0: signal as soon as the first sig_rows output rows (streaming order) are stored,
  // then carry on (kUnitSigEnd: at the unit's end).
  int nsignal = 0;
  int sig_rows = 0;
  // 2-D direct pipeline, side links (index = Dir - 2: W, E, NW, NE, SW, SE):
  //   xwait[i]:          my flag for pushes from that neighbour (this chunk needs StreamDyn::need[2 + i]);
  //   xsig[i]:           that neighbour's flag for my pushes;
  //   gsrc[0/1]:         my W / E ghost-column group of this chunk's parity — ghost column j of
  //                      row i lives at gsrc[0] + (G + i) * pitch + kGhostGroup + j (j < 0) and
  //                      gsrc[1] + (G + i) * pitch + (j - ycell) (j >= ycell);
  //   xpush[i]/xpitch[i]: my cell (i, j) that belongs to that neighbour's halo is stored at
  //                      xpush[i] + i * xpitch[i] + j (the host folds every offset into xpush).
  const unsigned long long* xwait[kSideLinks] = {};
  unsigned long long* xsig[kSideLinks] = {};
  const float* gsrc[2] = {nullptr, nullptr};
  float* xpush[kSideLinks] = {};
  int64_t xpitch[kSideLinks] = {};
  unsigned long long* sig[2] = {nullptr, nullptr};
  const unsigned long long* wait[2] = {nullptr, nullptr};
  const float* hsrc[2] = {nullptr, nullptr};
  float* push[2] = {nullptr, nullptr};
  // Device-side convergence (fused check): a launch whose *stop is non-zero does nothing (its
  // halo units only signal, so gates and flags stay in step); a residual launch also stores
  // the level K-1 value of every output cell into `keep` (same layout as dst) — the state one
  // step before the check, which the run returns if the check converges (B-5 semantics).
  const unsigned long long* stop = nullptr;
  float* keep = nullptr;
  DecideArgs dec;  // residual launches of a single-tile run: fused sum + decision
  // Deferred decision of a lone tile's previous check (as TileArgs::pend): one extra block
  // (blockIdx (nunits + 3) / 4) sums the `pend_n` partials at `pend` and decides (pend_dec; its
  // seq: the launch's seq argument) while the units compute speculatively into a buffer that is
  // not the check's input.
  const double* pend = nullptr;
  int pend_n = 0;
  DecideArgs pend_dec;
  int rel = 0;  // signal release: 0 system scope, 1 agent scope, 2 drain only (payload in uncached memory)
  int acq = 0;  // halo-wait acquire: 0 system scope, 1 agent scope, 2 compiler ordering only
  // Output row stores: 0 plain (write-back L2), 1 write-through (buffer_store sc1: the line
  // leaves the XCD's L2 at once, so the launch ends with no dirty L2 to write back — the
  // dependent kernel boundary then costs the bare ~1.7 us instead of + dirty bytes / 6 TB/s).
  int wt = 0;
  long long halo_polls = 0;
  unsigned int* timed_out = nullptr;
  unsigned int* timed_out_host = nullptr;  // host-mapped mirror of *timed_out (polled by the host per chunk)
  // Observability (s_memrealtime, 100 MHz).  wait_acc (halo units of the direct / signalled
  // pipelines): [0] += ticks spent in the halo wait, [1] += 1, [2] = max ticks — the exposed
  // communication time, the analogue of the reference's MPI_Waitall share (Report.pdf p.34-37).
  // stamps (diagnostics, usually null): per wave w, stamps[4w..4w+3] = {start, halo wait done,
  // end, hardware id (XCC_ID << 16 | HW_ID[15:0])}.
  unsigned long long* wait_acc = nullptr;
  unsigned long long* stamps = nullptr;
  // integrity (StreamDyn::lid > 0): the tag every unit of `units` carries; the engine's highest
  // launch id seen (wave 0 raises it — an old value >= lid is a replayed launch); serial
  // pipeline: the exchange copy blocks completed so far must equal StreamDyn::copies_need at
  // wave 0's start
  int utag = 0;
  int dbg = 0;  // diagnostics (EngineOptions::debug_kernel): 1 every unit runs the halo bodies
  unsigned long long* lid_seen = nullptr;
  const unsigned long long* copies_done = nullptr;
  unsigned long long* waves_done = nullptr;  // serial pipeline: every wave adds 1 at its end (its stores drained)
};

// ---- persistent pipelined streaming stencil (pstream_kernel.hpp) ---------------------------
// ONE launch runs J chunks of depth K.  Every wave keeps its unit for the whole launch; units
// sit on an aligned grid (every column strip cut at the same row bands, band i streaming down
// for even i and up for odd i), and a unit starts chunk j as soon as the rows its K-cone reads
// from its eight neighbours' chunk j-1 outputs are published — no kernel boundary, no grid-wide
// drain: a unit's first rows of a chunk are what the bands above / below need first.
// Progress words: unit w publishes prog[32 w] = (chunks done) * h + (rows of the current chunk
// whose write-through stores have completed), monotonically across the plan's launches.
constexpr int kPSlots = 8;  // neighbour slots: above, below, left, right, and the four diagonals
struct PUnit {
  Unit u;  // geometry as for the streaming kernel (links unused)
  int band;
  // per slot: neighbour unit (-1: none); my stream rows [rlo, rhi) come from its outputs; its
  // output index of my stream row r is qa + qs * r (qs = +-1); its rows per chunk hv
  int nb[kPSlots], rlo[kPSlots], rhi[kPSlots], qa[kPSlots], qs[kPSlots], hv[kPSlots];
};
// Per-launch part of a persistent launch.
struct PStreamDyn {
  int nunits = 0;          // == the block's nunits (the launcher's grid size)
  int nchunks = 0;         // J (>= 1)
  unsigned cbase = 0;      // chunks this plan completed in earlier launches (progress base)
  int cur0 = 0;            // chunk j reads buf[(cur0 + j) & 1]
  int ipar0 = 0;           // receive-buffer parity of chunk 0 (direct pipeline)
  unsigned btag = 0;       // the block's ArgHead::btag
  unsigned long long need0[2] = {0, 0};  // halo flag counts chunk 0 waits for (N / S)
  unsigned long long lbase[2] = {0, 0};  // my halo units' signals before the launch (N / S, chunk order)
};
struct PStreamArgs {
  ArgHead head;
  const PUnit* units;
  int nunits;
  float* buf[2];
  unsigned* prog;       // progress words, 32 apart (one 128-B line each)
  int64_t pitch, G, PL;
  int64_t xcell, ycell;
  int64_t gx0, gy0, NX, NY;
  double cx, cy;
  int fixed;
  int per_x = 0, per_y = 0;
  int dbg = 0;  // diagnostics (EngineOptions::debug_kernel): 1 every unit runs the halo-unit bodies
  float* dummy;
  // direct (IPC) halo units, per direction (0 north / top band, 1 south / bottom band, reverse)
  // and receive-buffer parity: chunk j reads parity (PStreamDyn::ipar0 + j) & 1 and pushes to
  // the other; chunk j waits for PStreamDyn::need0[d] + j * need_inc[d] on wait[d]
  const unsigned long long* wait[2] = {nullptr, nullptr};
  unsigned long long need_inc[2] = {0, 0};
  // chunk order of the signals: a halo unit signals chunk j of the launch only once all of this
  // rank's halo units of its direction have signalled chunk j-1 (*lsig[d] counts them,
  // PStreamDyn::lbase[d] before the launch, lper[d] per chunk).  The neighbour's wait counts
  // pushes summed over ALL strips, so without it a strip running a chunk ahead could stand in
  // for a slow strip's missing push and the neighbour would read that strip's ghost rows before
  // they landed.
  unsigned long long* lsig[2] = {nullptr, nullptr};
  int lper[2] = {0, 0};
  const float* hsrc[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  float* push[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  unsigned long long* sig[2] = {nullptr, nullptr};
  int sig_rows = 0;
  int rel = 2, acq = 1;
  long long halo_polls = 0;
  unsigned int* timed_out = nullptr;
  unsigned int* timed_out_host = nullptr;
  unsigned long long* wait_acc = nullptr;
  // Fused convergence: a launch that starts with *stop != 0 (a converged check before it) does
  // nothing at all.  Every rank decides the same check identically before its next launch, so
  // all ranks skip the same launches; the flags and counters they would have bumped are reset
  // by the re-prime that a converged run needs anyway.
  const unsigned long long* stop = nullptr;
  // Diagnostics (usually null; recorded only by a build of pstream_kernel.hpp with
  // -DH2D_PSTREAM_PHASES): s_memrealtime ticks (100 MHz) summed over waves and chunks, per
  // phase of a chunk — [0] chunks, [1] chunk-start drain of the previous chunk's stores, [2]
  // chunk-start wait for the neighbours' rows, [3] halo flag wait, [4] prologue (its loads and
  // the cone rows), [5] steady rows + tail, [6] in-loop waits (the tops' vmcnt + row waits).
  unsigned long long* phase = nullptr;
};
constexpr int kPhases = 7;
// Largest K with a compiled persistent kernel (K <= 8, write-through stores).
constexpr int kMaxPK = 8;
// cpl: columns per lane of the plan (4 or 2), a template parameter of the kernel.  `blk`: the
// device-resident block (ArgBlocks).
// pingpong: the steady loop variant that loads the next rows a whole iteration ahead
void launch_pstream(const PStreamArgs* blk, const PStreamDyn& d, int K, int precision, int cpl, bool pingpong,
                    hipStream_t s);
// Resident 256-thread blocks per CU of the persistent kernel (every block must be resident).
int pstream_blocks_per_cu(int K, int precision, int cpl);
void warm_pstream_kernels(int precision, int kmax, hipStream_t s);
// The aligned unit grid of the persistent kernel (empty if the tile does not allow one):
// `bands` row bands (even when both halo directions exist), every band at least hmin rows;
// strips of 64 * cpl columns.  halo_weight: the cost weight of a band with a N / S halo (its
// units wait for the neighbour's pushes every chunk; 1: none).
std::vector<PUnit> plan_pstream(const TileGeom& g, int K, bool fixed, bool per_x, bool per_y, double row_edge_weight,
                                int64_t capacity, bool halo_n, bool halo_s, int hmin, int cpl = 4,
                                double halo_weight = 1.0);

// Largest K with a compiled streaming kernel.
constexpr int kMaxK = 16;
bool stream_k_supported(int K);

// `blk`: the device-resident block (ArgBlocks), whose host copy `host` the launcher checks
// (geometry against K, store flavour); d.nunits == 0 launches nothing.
void launch_stream(const StreamArgs* blk, const StreamArgs& host, const StreamDyn& d, int K, int precision,
                   bool residual, hipStream_t s);
// No-op launches of every compiled streaming kernel with K <= kmax (both residual variants of
// `precision`), so that no code object is first loaded inside a timed run (one TU per K).
void warm_stream_kernels(int precision, int kmax, hipStream_t s);
void launch_naive_step(const TileGeom& g, const float* src, float* dst, int precision, int boundary, double cx,
                       double cy, bool per_x, bool per_y, hipStream_t s);
void launch_init(const TileGeom& g, float* base, int init, hipStream_t s);
void launch_poison(const TileGeom& g, float* base, bool fixed, bool per_x, bool per_y, hipStream_t s);
// tag != 0: every descriptor must carry it (else kIntegDescs is reported through integ /
// integ_host and the block copies nothing); done != nullptr: each block adds 1 when its copies
// are issued and drained (the serial pipeline's ordering check, StreamArgs::copies_done).
// waves_done != nullptr: block (0, 0) checks that it equals waves_need (every stencil wave
// enqueued before the copy has finished: kIntegOrder2).
void launch_copy_rects(const CopyDesc* d_descs, int ndesc, int64_t max_elems, hipStream_t s, int64_t tag = 0,
                       unsigned long long* done = nullptr, unsigned int* integ = nullptr,
                       unsigned int* integ_host = nullptr, const unsigned long long* waves_done = nullptr,
                       unsigned long long waves_need = 0);
// blocks launch_copy_rects uses for (ndesc, max_elems): what a `done` counter advances by
int64_t copy_rects_blocks(int ndesc, int64_t max_elems);
void launch_reduce_sum(const double* in, int n, double* out, hipStream_t s);
// One wave polls *counter (system-scope acquire loads, s_sleep between polls) until it reaches
// `target`; after `max_polls` it gives up and sets *timed_out (the caller reports it).
void launch_wait_counter(const unsigned long long* counter, unsigned long long target, unsigned int* timed_out,
                         unsigned int* timed_out_host, long long max_polls, hipStream_t s);
// Direct (IPC) transport: scalar sum over ranks through every rank's mapped block (see
// Engine::ipc_allreduce_residual); bounded wait, timeout bit 4.
void launch_ipc_allreduce(const double* local, double* out, char* const* d_blocks, int me, int nranks, int parity,
                          unsigned long long target, size_t count_off, size_t slot_off, int max_ranks,
                          long long max_polls, unsigned int* timed_out, unsigned int* timed_out_host,
                          const unsigned long long* stop, const DecideArgs* decide, hipStream_t s);
void launch_decide(const double* sum, const DecideArgs& d, hipStream_t s);
// Σ in[0..n) (fixed order) and the decision in one launch.
void launch_reduce_decide(const double* in, int n, const DecideArgs& d, hipStream_t s);
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
// per-variant launch / occupancy of the streaming kernel (stream_kernel.hpp; instantiated in
// generated TUs, one per (K, precision, residual))
template <int K, bool F32, bool RESID>
void launch_stream_kv(const StreamArgs* blk, const StreamDyn& d, bool wt, hipStream_t s);  // (unpacks d)
template <int K, bool F32, bool RESID>
int stream_blocks_per_cu_v();
template <int K, bool F32, int CPL>
void launch_pstream_kv(const PStreamArgs* blk, const PStreamDyn& d, bool pingpong, hipStream_t s);
template <int K, bool F32, int CPL>
int pstream_blocks_per_cu_v();

// Immutable device-resident kernel-argument blocks, deduplicated by content.
//
// get(a, s) returns the device copy of the bytes of `a` (ArgHead excluded from the comparison):
// the first time, the bytes go to a pinned host slab and a one-wave copy kernel on stream `s`
// writes them into device memory — ordered before every later launch on `s`, no host wait, and
// written through the L2 that the kernels' scalar loads read (a DMA engine writes around it).
// A block is never rewritten and lives until the owner is destroyed (after a device sync), so
// no launch can see a block change under it.  A block first used on another stream waits for
// its upload once (host sync of the uploading stream).
class ArgBlocks {
 public:
  ArgBlocks() = default;
  ~ArgBlocks();
  ArgBlocks(const ArgBlocks&) = delete;
  ArgBlocks& operator=(const ArgBlocks&) = delete;
  template <class T>
  const T* get(T& a, hipStream_t s) {
    static_assert(offsetof(T, head) == 0, "argument blocks start with an ArgHead");
    return static_cast<const T*>(get_raw(&a, sizeof(T), &a.head, s));
  }
  size_t blocks() const { return n_blocks_; }
  size_t uploads() const { return n_uploads_; }
  size_t bytes() const { return n_bytes_; }
  // Free every block (the caller has synchronised the device).  Cap for long-lived caches
  // (bindings' op API): callers clear when blocks() exceeds their bound.
  void clear();
 private:
  // fills *head (tag, size) and returns the device block
  const void* get_raw(const void* p, size_t n, ArgHead* head, hipStream_t s);
  struct Slab {
    char* dev = nullptr;
    char* host = nullptr;  // pinned, the kernel's copy source
    size_t cap = 0, used = 0;
  };
  struct Entry {
    const void* dev;
    unsigned tag;
    hipStream_t stream;  // uploaded on
    bool ready;          // the upload is known complete (usable on any stream)
  };
  std::vector<Slab> slabs_;
  std::unordered_map<std::string, Entry> index_;  // by content (the bytes after the ArgHead)
  size_t n_blocks_ = 0, n_uploads_ = 0, n_bytes_ = 0;
};
// Process-wide block tags (never 0).
unsigned next_arg_tag();

// Argument structs are filled from all-zero bytes, padding included (ArgBlocks deduplicates
// blocks by their bytes; every member's default is zero except where the caller sets one).
template <class T>
inline void zero_args(T& a) {
  std::memset(static_cast<void*>(&a), 0, sizeof(T));
}
// A device block of kZeroArgBytes zero bytes (per device, allocated once): the argument block of
// no-op launches (warm_*_kernels: a zero unit / tile count).
constexpr size_t kZeroArgBytes = 4096;
const void* zero_arg_block();
}  // namespace h2d
