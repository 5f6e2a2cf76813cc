// heat2d_amd — the native solver engine (one per process).
//
// Replaces the reference's hand-rolled time loops (grad1612_mpi_heat.c:206-280,
// grad1612_hybrid_heat.c:241-306, grad1612_cuda_heat.cu:79-89, mpi_heat2Dn.c:175-196) with
// one MI355X-first runtime:
//   * each process owns one or more halo-padded tiles of a 2-D block decomposition;
//   * time advances in chunks of K fused steps (temporal blocking) — halos are K deep and
//     exchanged once per chunk (8-neighbour, corners included) instead of every step;
//   * per chunk: the halo exchange runs on a dedicated comm stream while the interior work
//     units (those whose K-cone does not touch the ghost ring) run on the compute stream;
//     the boundary units wait on the exchange event (the reference's grey/green/yellow
//     overlap, Report.pdf p.17-18, grad1612_mpi_heat.c:231-275);
//   * transports: in-process tile-to-tile copies (LocalMultiTile — several logical ranks on
//     one GPU or on the CPU), RCCL send/recv over xGMI (one process per GPU), or "external"
//     (the Python layer drives pack/exchange/unpack, e.g. torch.distributed gloo on CPU);
//   * convergence: Σ(Δ)² fused into the last time level of the chunk that ends on a check
//     step, deterministic per-wave partials, RCCL all-reduce across ranks (B-5 fixed cadence).
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "cpu_reference.h"
#include "decomposition.h"
#include "kernels.h"
#include "tile_kernel.h"

namespace h2d {

enum Transport : int {
  kTransportAuto = 0,      // local copies if this process owns every tile, else RCCL
  kTransportLocal = 1,     // all tiles in this process
  kTransportRccl = 2,      // one tile per process, RCCL p2p
  kTransportExternal = 3,  // caller drives pack / unpack
  kTransportIpc = 4,       // one tile per process, 1-D row strips: halo units store their rows
                           // straight into the neighbour's receive buffer (IPC-mapped over xGMI)
};

struct EngineOptions {
  int64_t nx = 10, ny = 10;
  int gridx = 1, gridy = 1;
  bool periodic_x = false, periodic_y = false;
  int boundary = kFixed;
  int precision = kRef;
  int init = kInitExact;
  double cx = kCxDouble, cy = kCxDouble;
  int tblock = 8;          // max fused steps per chunk (= halo depth)
  int rows_per_wave = 0;   // H; 0 = automatic
  // relative cost per row of a column-edge / row-edge work unit (load balance).  Measured per
  // (h + K) against a plain unit, K=7 ref (tools/timeline.py --units, profiles/unit_balance_r5.md):
  // column edge 1.16 (4096 rows) / 1.21 (2048), row edge 1.23 / 1.30; a corner unit (both)
  // is sized at max + 0.1 (plan_units)
  double edge_weight = 1.16;
  double row_edge_weight = 1.27;  // (<= 0: edge_weight)
  // signalled / direct pipelines: the extra cost of a N / S halo unit in rows of a plain unit (its
  // halo wait: 2048x4096 direct, K=7: 3.4 µs median against 0.9 for other units; 0: none).
  // 2048x4096 direct K=7, us/step, two rounds: 2 rows 5.20 / 5.23, 4 rows 5.21 / 5.24, 6 rows
  // 5.13 / 5.08 (profiles/halo_rows_r5.txt)
  double halo_rows = 6.0;
  // persistent plans: cost weight of a band with a N / S halo (its units wait for the neighbour's
  // pushes every chunk).  Strong-scaling proxy, K=8, us/step at 1.0 / 1.1 / 1.15 / 1.2, two rounds:
  // 512x4096 2.04-2.08 / 1.91-1.93 / 1.84-1.87 / 2.10-2.13; 1024x4096 3.11-3.20 / 3.11-3.12 /
  // 3.06-3.07 / 3.03-3.04 (profiles/pstream_halo_weight_r5.txt)
  double pstream_halo_weight = 1.15;
  int64_t wave_capacity = 0;  // resident waves per launch; 0 = occupancy query
  int boundary_rows = 8;      // rows per halo-dependent work unit (overlap mode; at least K)
  // Signalled pipeline: ONE launch per chunk with the halo-dependent units first; each of them
  // bumps a counter when its rows are final and the comm stream starts the exchange of the
  // next chunk as soon as the counter says so (mid-kernel).  -1 auto, 0 off,
  // 1 gate = hipStreamWaitValue64 on signal memory, 2 gate = a one-wave polling kernel.
  int signal_exchange = -1;
  // Signalled pipeline: the halo-dependent units wait for the exchange in the kernel (they
  // poll a counter the comm stream sets after the exchange), so the compute stream never
  // waits on the comm stream.  -1 auto (on), 0: the chunk launch waits on an event instead.
  int device_halo_wait = -1;
  // comm stream priority: 1 high, 0 / -1 normal (default; high was not faster on one GPU)
  int comm_priority = -1;
  // signalled pipeline unit plan for 1-D row strips: -1/1 full-size signalling units (mid-unit
  // signal, bottom units streamed bottom-up), 0 short boundary units (signal at their end)
  int signal_plan = -1;
  // Bounded device-side waits (halo wait in the stencil, exchange gate) give up after about
  // this long, report it, and the run fails instead of hanging the queue.
  double halo_timeout_s = 30.0;
  // End-of-run synchronisation (the fixed cost of a short timed run): 0 hipEvent timing pair +
  // hipEventSynchronize; 1 no timing pair, spin on one untimed completion event; 2 no events,
  // hipStreamSynchronize; 3 timing pair, spin on the end event.  device_ms is wall time in 1/2.
  int sync_mode = 0;
  // Direct (IPC) pipeline fences: release of a halo unit's push (0 system scope, 1 agent, 2
  // none: the payload went to the peer's uncached memory and is acknowledged before the flag)
  // and acquire after its halo wait (0 system, 1 agent, 2 none: ghost rows are read from
  // uncached memory).  -1: the measured default.
  // Convergence decided on the device (checks end a chunk, the check launch keeps the state one
  // step earlier, later launches see a stop word): no host round trip per check.  -1 auto (GPU,
  // native loop), 0 the host-synchronised 1-step check chunk.
  int fused_check = -1;
  int direct_release = -1;
  int direct_acquire = -1;
  // Streaming kernel output rows: 0 plain stores, 1 write-through (sc1), -1 the measured default.
  int wt_store = -1;
  // Persistent pipelined stencil (pstream_kernel.hpp): runs of >= 2 equal plain chunks in ONE
  // launch on an aligned unit grid (single tile without exchange, or the direct IPC pipeline of
  // row strips).  -1 auto, 0 off, 1 on.
  int persistent = -1;
  // Strip width of the persistent kernel: 256 (4 columns per lane), 128 (2 per lane: units twice
  // as tall for the same wave count, so a short tile's K-cone costs half as much), 0 auto.
  int pstream_cols = 0;
  // Waves of one persistent launch at most (0: one per SIMD of the device).  Ranks that share a
  // GPU (a one-GPU rehearsal of an N-GPU run) split it, so every rank's waves are resident at once.
  int pstream_waves = 0;
  // Steady loop of the persistent kernel: 1 loads the next rows a whole iteration ahead
  // (ping-pong register sets), 0 / -1 row by row as they are consumed (the measured default).
  int pstream_pingpong = -1;
  // 2-D direct pipeline: cost weight per row of the units that push to a W / E neighbour
  double side_weight = 1.35;
  // Diagnostics: per-phase timers of the persistent kernel (PStreamArgs::phase)
  bool phase_timers = false;
  double watchdog_s = 900.0;  // abort the RCCL communicator after this long without progress (0: off)
  bool trace = false;         // per-phase hipEvent timers + roctx ranges
  // Diagnostics: record the per-wave timeline (s_memrealtime stamps) of the first `timeline`
  // streaming launches of each run (0: off).  Read back with Engine::timeline().
  int timeline = 0;
  bool poison = false;        // debug canary: NaN in every cell no valid update may read
  // diagnostics: 1 every streaming unit runs the halo-unit bodies; 2 no integrity checks (launch id 0);
  // 4 persistent halo signals without their chunk order (unsafe between processes)
  int debug_kernel = 0;
  bool convergence = false;
  int64_t interval = 20;
  double sensitivity = 0.1;
  int device = 0;          // HIP device ordinal, -1 = CPU
  std::vector<int> ranks;  // tiles owned by this process (empty = all)
  int transport = kTransportAuto;
  bool overlap = true;     // overlap halo exchange with interior compute
  bool small_grid_lds = true;  // whole-grid LDS solver for small single-tile problems
  // LDS-tiled temporally-blocked kernel (tile_kernel.hip) for single-tile runs of small and
  // medium grids: -1 auto (by size), 0 off, 1 on.  tile_rows = TX, tile_width = RY (32, 64
  // or 128 region columns), tile_k = steps per launch; 0 = automatic.
  int tiled = -1;
  int tile_rows = 0, tile_width = 0, tile_k = 0;
  int tile_threads = 0;  // workgroup size of the tiled kernel: 256, 1024, 0 = automatic
  int tile_cpl = 0;      // cells per lane and level of the tiled kernel: 1, 2, 4, 0 = automatic
  bool naive = false;      // validation: one-thread-per-cell single-step kernel
  // CUs reserved for the comm stream (pack/unpack/RCCL kernels) when halos are exchanged;
  // the compute streams are masked to the other CUs so the exchange kernels never wait for
  // resident stencil waves to drain.  -1 auto, 0 off.
  int comm_cus = -1;
  int comm_cu_layout = 0;
  // Resident-wave slots the interior launch leaves free for kernels that run beside it (the
  // RCCL p2p kernel of the signalled pipeline).  The dispatcher
  // deals waves round-robin over XCDs and shader engines, so a kernel launched second only
  // finds a slot if every engine keeps some free.  -1 auto.
  int reserve_waves = -1;
  bool device_fence_events = false;  // pipeline events without the system-scope fence
  // RCCL: send/receive whole K-row halos straight from/into the tile (no pack/unpack) when
  // the decomposition has no west/east neighbours (1-D row strips).  -1 auto, 0 off.
  int contiguous_halo = -1;
};

struct RunStats {
  int64_t steps_done = 0;
  bool converged = false;
  double residual = -1.0;
  double device_ms = 0.0;  // hipEvent time of the step loop (CPU: wall time)
  double wall_ms = 0.0;
  int64_t chunks = 0;
  int64_t exchanges = 0;
  std::string path;        // "stream", "lds", "naive", "cpu"
  std::map<std::string, double> phase_ms;    // trace mode: device time per phase (boundary, interior, exchange, step)
  std::map<std::string, int64_t> phase_count;
};

class Engine {
 public:
  explicit Engine(const EngineOptions& o);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  const EngineOptions& options() const { return opt_; }
  const Decomposition& decomposition() const { return dec_; }
  int num_tiles() const { return (int)tiles_.size(); }
  int tile_rank(int t) const { return tiles_.at(t).rank; }
  TileGeom geom(int t) const { return tiles_.at(t).g; }
  int halo_depth() const { return G_; }
  bool on_gpu() const { return opt_.device >= 0; }
  bool has_exchange() const { return has_exchange_; }
  int signal_mode() const { return sig_mode_; }
  bool tiled() const { return tiled_; }
  std::vector<int> tile_config() const { return {tile_tx_, tile_ry_, tile_k_}; }
  int tile_threads() const { return tile_nt_; }
  int tile_cpl() const { return tile_cpl_; }
  // "none" (no exchange), "direct" (IPC), "external", "signal", "serial"
  std::string pipeline() const;
  int rows_per_wave(int K) const;  // largest unit height for depth K (tile 0)
  int num_units(int K) const;      // work units (waves) per chunk of depth K, all tiles
  int64_t steps_done() const { return steps_done_; }
  uintptr_t stream_handle() const { return (uintptr_t)compute_; }
  int comm_cus() const { return comm_cus_; }
  bool contiguous_halo() const { return contig_; }
  int64_t wave_capacity(int K) const;  // resident waves available to the compute streams

  // RCCL bootstrap: rank 0 creates the id, the caller broadcasts it (torch.distributed).
  static std::string rccl_unique_id();
  void init_rccl(const std::string& id, int nranks, int rank);
  bool rccl_ready() const { return rccl_comm_ != nullptr; }

  // IPC direct transport (kTransportIpc).  Bootstrap, collectively: every rank calls
  // ipc_handle(), the handles are all-gathered (index = rank), every rank calls ipc_open(all),
  // then barrier -> ipc_prime() -> barrier.  A prime is needed again after upload() or a
  // converged (rolled-back) run: ipc_primed() says so.
  std::string ipc_handle();
  void ipc_open(const std::vector<std::string>& handles);
  void ipc_prime();
  bool ipc_primed() const { return ipc_primed_; }
  bool direct() const { return direct_; }

  // Native time loop (transports local / rccl / none).
  RunStats run(int64_t steps);

  // Fine-grained API (external transports, tests).
  int next_chunk(int64_t done, int64_t total, bool* check) const;
  void advance(int k, bool residual);      // one chunk, all tiles, no exchange
  void exchange_local(int k);              // in-process halo fill for depth k
  double local_residual();                 // Σ over local tiles of the last advance(k, true)
  int64_t send_count(int t, int k) const;
  int64_t recv_count(int t, int k) const;
  std::vector<int64_t> plan_info(int t, int k) const;  // [peer, send_off, send_n, recv_off, recv_n] × 8
  void pack(int t, int k, uintptr_t sendbuf);
  void unpack(int t, int k, uintptr_t recvbuf);
  void rollback();  // undo the last chunk (convergence exit)
  void set_steps_done(int64_t s) { steps_done_ = s; }

  std::vector<float> download(int t) const;  // owned block, row-major xcell×ycell
  // diagnostics: the whole padded storage of buffer b (0/1) of tile t (srows × pitch), and which
  // buffer is current
  std::vector<float> storage(int t, int b) const;
  int current_buffer(int t) const { return tiles_.at(t).cur; }
  void upload(int t, const float* owned);
  void synchronize() const;

  // Exposed halo wait of the halo units (direct / signalled pipelines) since the last reset:
  // {total wait in us, waits, longest wait in us}.  Synchronises; not for the timed region.
  struct HaloWait {
    double total_us = 0.0, max_us = 0.0;
    int64_t waits = 0;
  };
  HaloWait halo_wait() const;
  void reset_halo_wait();
  // persistent kernel phase timers (kPhases values: chunks, then microseconds summed over waves)
  std::vector<double> pstream_phases() const;
  // Per-wave timeline of the launches recorded by the last run (EngineOptions::timeline):
  // {K, units, stamps[units][4] = start, ready (halo wait done), end, hardware id}.
  struct LaunchTimeline {
    int K = 0, units = 0;
    std::vector<unsigned long long> stamps;
  };
  std::vector<LaunchTimeline> timeline() const;
  // The work units of tile t at depth K in launch order (which: 0 all, 3 halo units first).
  std::vector<Unit> unit_list(int t, int K, int which);
  // The persistent plan's units at depth K (empty: no persistent launch at this depth).
  std::vector<PUnit> pstream_units(int K);
  int64_t pstream_launches() const { return pstream_launches_; }

 private:
  struct Tile {
    int rank = 0;
    TileGeom g;
    float* buf[2] = {nullptr, nullptr};  // device or host storage
    float* keep = nullptr;               // fused convergence: state one step before the last check
    // tiled lone tile with the fused check: the third buffer of the speculative launch after a
    // check (TileArgs::pend): that launch writes here, so the check's input survives it
    float* spare = nullptr;
    std::vector<float> host[2];          // CPU storage
    std::vector<float> scratch[2];       // CPU temporal-block scratch
    int cur = 0;
    double last_resid = 0.0;
    double* partials = nullptr;  // per-wave residual partials (device)
    int64_t pcap = 0;
  };
  struct UnitLists {
    int H = 0;
    int tag[4] = {0, 0, 0, 0};  // integrity tags of d_all, d_interior, d_boundary, d_bfirst
    Unit* d_all = nullptr;
    Unit* d_interior = nullptr;
    Unit* d_boundary = nullptr;
    Unit* d_bfirst = nullptr;  // boundary units, then interior units (signalled pipeline)
    int sig_rows = 0;          // > 0: boundary units are full-size and signal after this many rows
    int n_all = 0, n_interior = 0, n_boundary = 0;
    int n_dir[2] = {0, 0};     // halo units facing north (top) / south (bottom, kUnitReverse)
    int pushes[kNumDirs] = {};  // units pushing to the neighbour in each direction (direct pipeline)
  };

  const UnitLists& units(int t, int K);
  // which: 0 all, 1 interior, 2 boundary, 3 all boundary-first + signal; src: storage index
  // read (-1: current)
  void launch_chunk_tile(int t, int K, bool residual, int which, int src = -1, hipStream_t stream = nullptr);
  void reduce_tile_residual(int t, int K);
  void do_exchange_async(int K, hipStream_t s = nullptr);
  void h2d(void* dst, const void* src, size_t bytes) const;  // plan upload, complete on return
  void dzero(void* p, size_t bytes) const;  // zero, ordered on the compute stream  // enqueue on `s` (default: the comm stream)
  double finish_residual();       // reduce + (rccl) all-reduce, host sync
  void wait_event(hipEvent_t ev);  // blocking wait with RCCL error polling + progress watchdog
  // Progress events for the watchdog: every 16th launch records one (ring of 8); a wait resets
  // its no-progress clock whenever a newer one has completed.
  static constexpr int kProgRing = 8;
  hipEvent_t ev_prog_[kProgRing] = {};
  unsigned long long prog_seq_[kProgRing] = {};
  unsigned long long launches_ = 0, prog_seen_ = 0;
  void progress_tick(hipStream_t s);
  int chunk_len(int64_t done, int64_t total, int kmax, bool* check) const;  // convergence-aligned chunk
  RunStats run_impl(int64_t steps);
  // the time loop of each path (run_impl picks one; each advances steps_done_ to `target` or to a
  // converged check)
  void run_cpu(RunStats& st, int64_t target);
  void run_tiled(RunStats& st, int64_t target);
  void run_lds(RunStats& st, int64_t steps);
  void run_direct(RunStats& st, int64_t target);
  void run_signal(RunStats& st, int64_t target);
  void run_serial(RunStats& st, int64_t target);
  void check_tile(int t) const;
  void trace_begin(const char* phase, hipStream_t s);
  void trace_end(const char* phase, hipStream_t s);
  void trace_collect(RunStats& st);
  struct Span {
    std::string phase;
    hipEvent_t a, b;
  };
  std::vector<Span> spans_;
  std::map<std::string, hipEvent_t> open_;

  EngineOptions opt_;
  Decomposition dec_;
  int G_ = 1;
  bool has_exchange_ = false;
  int transport_ = kTransportLocal;
  std::vector<Tile> tiles_;
  int64_t steps_done_ = 0;

  // device state
  hipStream_t compute_ = nullptr, comm_ = nullptr;
  bool pooled_streams_ = false;  // borrowed from the process-wide stream pool (engine.cpp)
  int comm_prio_ = 0;
  hipEvent_t ev_ready_ = nullptr, ev_halo_ = nullptr, ev_t0_ = nullptr, ev_t1_ = nullptr, ev_done_ = nullptr;
  void end_of_run_wait(RunStats& st, std::chrono::steady_clock::time_point w0);
  std::map<std::pair<int, int>, UnitLists> units_;
  // device-resident kernel-argument blocks of this engine's launches (kernels.h); destroyed after
  // the destructor's device synchronisation
  ArgBlocks args_;
  // an uploaded copy-descriptor list: n descriptors, the largest rectangle, its integrity tag
  struct DescList {
    CopyDesc* d = nullptr;
    int n = 0;
    int64_t maxe = 0;
    int64_t tag = 0;
  };
  DescList upload_descs(std::vector<CopyDesc>& v);  // tags and uploads (GPU) or keeps (CPU) a list
  const DescList& local_descs(int K);
  const DescList& ext_descs(std::vector<CopyDesc>& v);  // pack / unpack lists, by content
  std::map<std::string, DescList> ext_descs_;
  void local_copy(const DescList& D, hipStream_t s);  // one local exchange (tagged, counted on compute_)
  std::map<std::pair<int, int>, DescList> local_descs_;  // (K, parity)
  std::map<std::pair<int, int>, DescList> pack_descs_;   // (K, parity) for rccl
  std::map<std::pair<int, int>, DescList> unpack_descs_;
  // ---- integrity checks (kInteg* bits of the device error word, named by poll_abort) ----
  unsigned long long lid_ = 0;                  // streaming launches enqueued (launch ids)
  unsigned long long* d_lid_seen_ = nullptr;    // highest launch id a launch has completed
  unsigned long long* d_copies_done_ = nullptr;  // local exchange copy blocks completed (compute stream)
  unsigned long long copies_need_ = 0;          // ... enqueued
  unsigned long long* d_waves_done_ = nullptr;  // serial pipeline: stencil waves completed
  unsigned long long waves_need_ = 0;           // ... enqueued
  static int next_tag();                        // process-wide plan tags (never 0)
  unsigned long long* d_wait_acc_ = nullptr;  // StreamArgs::wait_acc (3 words)
  unsigned long long* d_stamps_ = nullptr;    // StreamArgs::stamps ring (timeline diagnostics)
  static constexpr int kTimelineUnits = 8192; // units recorded per launch at most
  std::vector<std::pair<int, int>> tl_recs_;  // (K, units) of each launch recorded this run
  double* d_resid_ = nullptr;       // [num_tiles] + 1 total
  double* h_resid_ = nullptr;       // pinned
  long long* d_lds_steps_ = nullptr;
  float* d_dummy_ = nullptr;        // sink for the streaming kernel's non-output lanes
  float* d_send_ = nullptr;
  float* d_recv_ = nullptr;
  int64_t stage_cap_ = 0;
  int comm_cus_ = 0, device_cus_ = 0;
  bool contig_ = false;
  bool tiled_ = false;                      // resolved EngineOptions::tiled
  int tile_tx_ = 0, tile_ry_ = 0, tile_k_ = 0, tile_nt_ = 256, tile_cpl_ = 4;
  int sig_mode_ = 0;                        // resolved signal_exchange
  unsigned long long* sig_counter_ = nullptr;  // boundary units completed (cumulative)
  unsigned long long sig_target_ = 0;          // boundary units launched (cumulative, host)
  unsigned int* d_sig_timeout_ = nullptr;      // bounded waits that gave up (device word, fail-fast)
  unsigned int* h_timeout_ = nullptr;          // its host-mapped mirror, polled per chunk
  unsigned int* h_timeout_dev_ = nullptr;      // device view of h_timeout_
  bool broken_ = false;                        // a wait timed out: halos and counters are out of step
  std::string broken_why_;
  void poll_abort();                           // throw (and mark broken) if a device wait gave up
  bool dev_wait_ = false;                      // resolved device_halo_wait
  unsigned long long* halo_counter_ = nullptr;  // exchanges landed (cumulative)
  unsigned long long halo_seq_ = 0;            // exchanges enqueued (cumulative, host)
  void exchange_landed();                   // comm stream: publish halo_seq_ (or record evHalo)
  void gate_exchange();                     // comm stream: wait until sig_counter_ >= sig_target_
  // ---- IPC direct transport ----
  bool direct_ = false;
  struct IpcLayout {
    size_t flag[kNumDirs] = {};                   // pushes arrived from the neighbour in direction d
    size_t resid_count = 1024, resid_slots = 1152;  // byte offsets
    size_t lsig[2] = {2304, 2432};  // my N / S halo units' signals of persistent launches (chunk order)
    size_t recv_n[2] = {0, 0}, recv_s[2] = {0, 0};
    size_t xbuf = 0;     // W / E ghost-column groups (2-D blocks only; 0: none)
    int64_t pitch = 0;   // the tile's row pitch (floats): also the xbuf's
    size_t bytes = 0;
    // group (side 0 W / 1 E, parity p): its column 0 in xbuf row 0 (= tile row -G).  Each group
    // has a 256-byte segment of its own in every row (rows start 256-byte aligned): the parity a
    // chunk reads never shares a cache line with the parity its pushes write (measured: with the
    // groups packed 64 bytes apart, ghost columns read stale values under concurrent pushes).
    static constexpr int kGroupStride = 64;  // floats
    size_t group(int side, int p) const { return xbuf + (size_t)(2 * side + p) * kGroupStride * sizeof(float); }
  };
  static constexpr int kIpcMaxRanks = 64;
  IpcLayout ipc_layout_of(int rank) const;
  float* side_push_base(int d, int peer_rank, int parity) const;
  std::vector<IpcLayout> ipc_lays_;         // every rank's block layout (from the decomposition)
  std::vector<std::vector<int32_t>> ipc_counts_;  // per rank: units pushing per (K, direction)
  char* ipc_block_ = nullptr;               // my uncached block: flags, residual slots, receive buffers
  std::vector<char*> ipc_blocks_;           // every rank's block (mine included), mapped
  std::vector<bool> ipc_opened_;            // entries from hipIpcOpenMemHandle (closed in the dtor)
  char** d_ipc_blocks_ = nullptr;           // device copy of ipc_blocks_
  bool ipc_primed_ = false;
  unsigned long long ipc_chunk_ = 0;        // chunks since the prime (receive-buffer parity)
  unsigned long long ipc_need_[kNumDirs] = {};  // halo pushes expected from each direction (cumulative)
  unsigned long long ipc_lsig_[2] = {};         // my persistent N / S signals so far (IpcLayout::lsig)
  unsigned long long ipc_resid_epoch_ = 0;  // residual all-reduces since the prime
  // ---- persistent pipelined stencil ----
  struct PPlan {
    PUnit* d_units = nullptr;
    unsigned* d_prog = nullptr;  // progress words, 32 apart
    int n = 0;
    int cpl = 4;                 // columns per lane (strip width 64 * cpl)
    int pushes[2] = {0, 0};      // N / S halo units (direct pipeline): flag increments per chunk
    unsigned cdone = 0;          // chunks run by this plan's launches (progress base)
    std::vector<PUnit> host;
  };
  // per rank, per (K, N/S): its persistent plan's halo pushes per chunk (-1: no plan at depth K),
  // from the IPC handles; a depth runs persistent launches only if every rank has a plan
  std::vector<std::vector<int32_t>> pst_counts_;
  bool pst_everywhere(int K) const;
  std::map<int, PPlan> pplans_;  // by K (an empty plan: not eligible)
  int64_t pstream_launches_ = 0;
  unsigned long long* d_phase_ = nullptr;
  const PPlan* pplan(int K);     // build / look up; nullptr if depth K runs launch per chunk
  int plain_run(int64_t done, int64_t target, int k) const;  // equal plain chunks of depth k from `done`
  void launch_pstream_chunks(int K, int J);
  // ---- device-side convergence ----
  bool fused_ = false;
  unsigned long long* d_stop_ = nullptr;  // 0 running, else the sequence number of the converged check
  ConvHost* h_conv_ = nullptr;            // host-mapped decision record
  ConvHost* h_conv_dev_ = nullptr;
  unsigned long long chunk_seq_ = 0;
  struct CheckRec {
    unsigned long long seq;
    int64_t steps_before;
    int k;
    int src;  // the check chunk's input buffer (tile 0): unchanged by the no-op launches after it
    const float* src_ptr;  // its storage (the tiled path's three-buffer rotation moves it)
    int lvl;  // the check step's level in the chunk (== k unless the chunk runs through the check)
  };
  // A lone single-process tile keeps no rollback copy in its check launches: on convergence
  // the state one step before the check is recomputed from the check chunk's input (k-1 steps).
  bool recompute_rollback() const { return fused_ && tiles_.size() == 1 && !has_exchange_; }
  std::vector<CheckRec> checks_;
  int checks_since_sync_ = 0;
  hipEvent_t ev_check_ = nullptr;
  unsigned int* d_ticket_ = nullptr;      // per tile: last-wave tickets of fused residual launches
  bool decided_in_launch_ = false;        // the last check launch already made the decision
  const double* last_parts_ = nullptr;    // a lone tile's residual partials awaiting the decision
  int last_nparts_ = 0;
  // a lone streaming tile with a spare buffer: the last check's decision rides in the next
  // launch's extra block (StreamArgs::pend); its partials alternate between two sets
  const double* pend_parts_ = nullptr;
  int pend_nparts_ = 0;
  DecideArgs pend_dec_{};
  int pset_ = 0;
  void flush_pending_decision();
  DecideArgs decide_args(int t, bool decide) const;
  void device_decide(unsigned long long seq);
  bool check_point(int64_t steps_before, int k, int lvl = 0);
  bool finalize_convergence(RunStats& st);  // true: it enqueued recompute launches
  double ipc_allreduce_residual();
  void* rccl_comm_ = nullptr;       // ncclComm_t
  int rccl_rank_ = 0, rccl_nranks_ = 1;
};

}  // namespace h2d
