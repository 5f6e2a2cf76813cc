// heat2d_amd — native solver engine (see engine.h).
#include "engine.h"
#include "collectives.h"

#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

#define H2D_NCCL_CHECK(call)                                                                             \
  do {                                                                                                   \
    ncclResult_t _r = (call);                                                                            \
    if (_r != ncclSuccess)                                                                               \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + __FILE__ + \
                               ":" + std::to_string(__LINE__) + ": " #call);                            \
  } while (0)

namespace h2d {


namespace {
template <class T>
T* dmalloc(size_t n) {
  T* p = nullptr;
  if (n == 0) n = 1;
  H2D_HIP_CHECK(hipMalloc(&p, n * sizeof(T)));
  return p;
}
// roctx markers (optional; resolved at run time so the library is not a link dependency).
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    void* h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
    if (h) {
      push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    }
  }
};
Roctx& roctx() {
  static Roctx r;
  return r;
}

// Process-wide pool of non-blocking HIP streams, per (device, priority): an engine borrows its
// two streams and hands them back, so a process creates streams — and the HIP runtime's
// per-stream kernel-argument memory with them — once, not once per engine (round 5: a new
// engine's first launches on freshly created streams read stale kernel arguments;
// docs/ARCHITECTURE.md, "Kernel arguments").  HEAT2D_STREAM_POOL=0: create and destroy per engine.
struct StreamPool {
  std::mutex mu;
  std::map<std::pair<int, int>, std::vector<hipStream_t>> free;  // never destroyed (process lifetime)
};
StreamPool& stream_pool() {
  static StreamPool* p = new StreamPool();  // leaked: the runtime may be gone at static destruction
  return *p;
}
bool stream_pool_on() {
  static const bool on = [] {
    const char* e = std::getenv("HEAT2D_STREAM_POOL");
    return e == nullptr || std::strcmp(e, "0") != 0;
  }();
  return on;
}
hipStream_t borrow_stream(int device, int prio) {
  if (stream_pool_on()) {
    StreamPool& P = stream_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    auto& v = P.free[{device, prio}];
    if (!v.empty()) {
      hipStream_t s = v.back();
      v.pop_back();
      return s;
    }
  }
  hipStream_t s = nullptr;
  if (prio != 0) H2D_HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio));
  else H2D_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return s;
}
void return_stream(int device, int prio, hipStream_t s) {  // (the caller has synchronised it)
  if (s == nullptr) return;
  if (!stream_pool_on()) {
    hipStreamDestroy(s);
    return;
  }
  StreamPool& P = stream_pool();
  std::lock_guard<std::mutex> lk(P.mu);
  P.free[{device, prio}].push_back(s);
}
}  // namespace

void Engine::trace_begin(const char* phase, hipStream_t s) {
  if (!opt_.trace || !on_gpu()) return;
  if (roctx().push) roctx().push(phase);
  hipEvent_t a;
  H2D_HIP_CHECK(hipEventCreate(&a));
  H2D_HIP_CHECK(hipEventRecord(a, s));
  open_[phase] = a;
}

void Engine::trace_end(const char* phase, hipStream_t s) {
  if (!opt_.trace || !on_gpu()) return;
  if (roctx().pop) roctx().pop();
  hipEvent_t b;
  H2D_HIP_CHECK(hipEventCreate(&b));
  H2D_HIP_CHECK(hipEventRecord(b, s));
  spans_.push_back({phase, open_.at(phase), b});
  open_.erase(phase);
}

void Engine::trace_collect(RunStats& st) {
  if (!opt_.trace || !on_gpu()) return;
  for (auto& sp : spans_) {
    H2D_HIP_CHECK(hipEventSynchronize(sp.b));
    float ms = 0.0f;
    H2D_HIP_CHECK(hipEventElapsedTime(&ms, sp.a, sp.b));
    st.phase_ms[sp.phase] += ms;
    st.phase_count[sp.phase] += 1;
    hipEventDestroy(sp.a);
    hipEventDestroy(sp.b);
  }
  spans_.clear();
}

Engine::Engine(const EngineOptions& o) : opt_(o) {
  dec_ = Decomposition(o.nx, o.ny, o.gridx, o.gridy, o.periodic_x, o.periodic_y);
  if (o.tblock < 1) throw std::invalid_argument("tblock must be >= 1");
  if (o.convergence && o.interval < 1) throw std::invalid_argument("interval must be >= 1");
  std::vector<int> ranks = o.ranks;
  if (ranks.empty())
    for (int r = 0; r < dec_.nranks(); ++r) ranks.push_back(r);
  for (int r : ranks)
    if (r < 0 || r >= dec_.nranks()) throw std::invalid_argument("rank out of range");

  // Halo / temporal-block depth: bounded by the smallest tile on exchanged dimensions.
  int64_t G = o.tblock;
  G = std::min<int64_t>(G, dec_.max_halo_depth());
  if (on_gpu()) {
    while (G > 1 && !stream_k_supported((int)G)) --G;
  }
  G_ = (int)std::max<int64_t>(1, G);

  bool any_peer = false;
  for (int r : ranks)
    for (int d = 0; d < kNumDirs; ++d)
      if (dec_.neighbor(r, d) >= 0) any_peer = true;
  // Peers of non-local ranks also matter (a rank whose only neighbour is remote).
  has_exchange_ = any_peer;

  transport_ = o.transport;
  if (transport_ == kTransportAuto) transport_ = ((int)ranks.size() == dec_.nranks()) ? kTransportLocal : kTransportRccl;
  if (transport_ == kTransportLocal && (int)ranks.size() != dec_.nranks())
    throw std::invalid_argument("local transport needs every tile in this process");
  if (transport_ == kTransportRccl && ranks.size() != 1) throw std::invalid_argument("RCCL transport: one tile per process");
  if (transport_ == kTransportRccl && !on_gpu()) throw std::invalid_argument("RCCL transport needs a GPU");
  if (transport_ == kTransportIpc) {
    if (ranks.size() != 1 || !on_gpu()) throw std::invalid_argument("IPC transport: one tile per process, on a GPU");
    bool side = false;
    for (int d = kW; d < kNumDirs; ++d) side = side || dec_.neighbor(ranks[0], d) >= 0;
    if (side) {
      // 2-D blocks: W / E ghost columns are whole lanes of the streaming kernel (4 columns each)
      const TileGeom g0 = dec_.tile(ranks[0], G_);
      if (g0.ycell % 4 != 0 || g0.ycell < 2 * kGhostGroup)
        throw std::invalid_argument("IPC transport with west/east neighbours: the tile width (" +
                                    std::to_string(g0.ycell) + ") must be a multiple of 4 and at least " +
                                    std::to_string(2 * kGhostGroup));
    }
  }
  direct_ = transport_ == kTransportIpc && has_exchange_;

  contig_ = transport_ == kTransportRccl && o.contiguous_halo != 0 && o.gridy == 1 && !o.periodic_y;
  if (on_gpu()) {
    H2D_HIP_CHECK(hipSetDevice(o.device));
    hipDeviceProp_t prop;
    H2D_HIP_CHECK(hipGetDeviceProperties(&prop, o.device));
    device_cus_ = std::max(1, prop.multiProcessorCount);
    // auto: off (measured: masked compute queues ran the stencil ~2x slower on gfx950)
    comm_cus_ = o.comm_cus < 0 ? 0 : o.comm_cus;
    if (comm_cus_ >= device_cus_ / 2) comm_cus_ = 0;
    if (comm_cus_ > 0) {
      std::vector<uint32_t> mc((device_cus_ + 31) / 32, 0u), mx(mc.size(), 0u);
      std::vector<char> res(device_cus_, 0);
      for (int i = 0; i < comm_cus_; ++i) {
        const int c = o.comm_cu_layout == 1 ? device_cus_ - 1 - i
                      : o.comm_cu_layout == 2 ? i
                                              : (int)((int64_t)(i + 1) * device_cus_ / comm_cus_ - 1);
        res[c] = 1;
      }
      for (int c = 0; c < device_cus_; ++c) (res[c] ? mx : mc)[c / 32] |= 1u << (c % 32);
      H2D_HIP_CHECK(hipExtStreamCreateWithCUMask(&compute_, (uint32_t)mc.size(), mc.data()));
      H2D_HIP_CHECK(hipExtStreamCreateWithCUMask(&comm_, (uint32_t)mx.size(), mx.data()));
    } else {
      compute_ = borrow_stream(o.device, 0);
      // Optionally a high-priority comm stream (its waves win dispatch ties against the
      // stencil's).  Separate hardware queues for compute and comm come from
      // GPU_MAX_HW_QUEUES >= 8 (set by the bench / CLI entry points), not from the priority.
      int least = 0, greatest = 0;
      if (o.comm_priority > 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest != least)
        comm_prio_ = greatest;
      comm_ = borrow_stream(o.device, comm_prio_);
      pooled_streams_ = true;
    }
    // Pipeline events only order work on this device (RCCL fences its own cross-device
    // traffic), so they can skip the system-scope fence.
    const unsigned evf = hipEventDisableTiming | (o.device_fence_events ? hipEventDisableSystemFence : 0u);
    H2D_HIP_CHECK(hipEventCreateWithFlags(&ev_ready_, evf));
    H2D_HIP_CHECK(hipEventCreateWithFlags(&ev_halo_, evf));
    H2D_HIP_CHECK(hipEventCreate(&ev_t0_));
    H2D_HIP_CHECK(hipEventCreate(&ev_t1_));
    H2D_HIP_CHECK(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming));
    for (auto& e : ev_prog_) H2D_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    d_resid_ = dmalloc<double>(ranks.size() + 1);
    H2D_HIP_CHECK(hipHostMalloc(&h_resid_, sizeof(double) * (ranks.size() + 1)));
    d_lds_steps_ = dmalloc<long long>(1);
    d_dummy_ = dmalloc<float>(4 * kWaveCols);
    if (o.phase_timers) {
      d_phase_ = dmalloc<unsigned long long>(kPhases);
      dzero(d_phase_, kPhases * sizeof(unsigned long long));
    }
    d_wait_acc_ = dmalloc<unsigned long long>(4);
    dzero(d_wait_acc_, 4 * sizeof(unsigned long long));
    d_lid_seen_ = dmalloc<unsigned long long>(3);
    dzero(d_lid_seen_, 3 * sizeof(unsigned long long));
    d_copies_done_ = d_lid_seen_ + 1;
    d_waves_done_ = d_lid_seen_ + 2;
    if (o.timeline > 0) {
      if (o.timeline > 4096) throw std::invalid_argument("timeline: at most 4096 launches");
      d_stamps_ = dmalloc<unsigned long long>((size_t)o.timeline * kTimelineUnits * 4);
    }
    if (o.convergence && !o.naive && transport_ != kTransportExternal && o.fused_check != 0) {
      d_stop_ = dmalloc<unsigned long long>(1);
      dzero(d_stop_, sizeof(unsigned long long));
      H2D_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_conv_), sizeof(ConvHost), hipHostMallocMapped));
      std::memset(h_conv_, 0, sizeof(ConvHost));
      H2D_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_conv_dev_), h_conv_, 0));
      H2D_HIP_CHECK(hipEventCreateWithFlags(&ev_check_, hipEventDisableTiming));
      d_ticket_ = dmalloc<unsigned int>(ranks.size());
      dzero(d_ticket_, ranks.size() * sizeof(unsigned int));
    }
  }

  fused_ = on_gpu() && o.convergence && !o.naive && transport_ != kTransportExternal && o.fused_check != 0;
  for (int r : ranks) {
    Tile t;
    t.rank = r;
    t.g = dec_.tile(r, G_);
    const size_t n = (size_t)t.g.elems();
    if (on_gpu()) {
      for (int b = 0; b < 2; ++b) {
        t.buf[b] = dmalloc<float>(n);
        H2D_HIP_CHECK(hipMemsetAsync(t.buf[b], 0, n * sizeof(float), compute_));
      }
      // rollback copy for fused checks; a lone tile recomputes it instead (recompute_rollback),
      // so an HBM-filling tile with the convergence check still needs only its two buffers
      if (fused_ && !(ranks.size() == 1 && !has_exchange_)) {
        t.keep = dmalloc<float>(n);
        H2D_HIP_CHECK(hipMemsetAsync(t.keep, 0, n * sizeof(float), compute_));
        if (o.poison) launch_poison(t.g, t.keep, o.boundary == kFixed, o.periodic_x, o.periodic_y, compute_);
      }
      launch_init(t.g, t.buf[0], o.init, compute_);
      if (o.poison)
        for (int b = 0; b < 2; ++b)
          launch_poison(t.g, t.buf[b], o.boundary == kFixed, o.periodic_x, o.periodic_y, compute_);
    } else {
      for (int b = 0; b < 2; ++b) {
        t.host[b].assign(n, 0.0f);
        t.buf[b] = t.host[b].data();
        t.scratch[b].assign(n, 0.0f);
      }
      cpu_tile_init(t.g, t.buf[0], o.init);
      if (o.poison)
        for (int b = 0; b < 2; ++b) cpu_tile_poison(t.g, t.buf[b], o.boundary == kFixed, o.periodic_x, o.periodic_y);
    }
    tiles_.push_back(std::move(t));
  }
  if (on_gpu()) {
    // Build every unit list (and size the residual partials) up front: nothing is
    // allocated inside the time loop.
    for (int t = 0; t < (int)tiles_.size(); ++t) {
      tiles_[t].pcap = 256;
      tiles_[t].partials = dmalloc<double>(256);
    }
    // Bounded device waits report through these (direct and signalled pipelines).
    d_sig_timeout_ = dmalloc<unsigned int>(1);
    dzero(d_sig_timeout_, sizeof(unsigned int));
    H2D_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_timeout_), sizeof(unsigned int), hipHostMallocMapped));
    *h_timeout_ = 0u;
    H2D_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_timeout_dev_), h_timeout_, 0));
    // Signalled pipeline (default with an exchange): one launch per chunk, halo-dependent
    // units first, the exchange gated mid-kernel on their completion counter.
    sig_mode_ = 0;
    if (has_exchange_ && opt_.overlap && !opt_.naive && opt_.signal_exchange != 0 && !direct_) {
      sig_mode_ = opt_.signal_exchange < 0 ? 2 : opt_.signal_exchange;
      if (sig_mode_ == 1) {
        int ok = 0;
        hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, o.device);
        if (!ok) sig_mode_ = 2;
      }
      if (sig_mode_ == 1 &&
          hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_counter_), sizeof(unsigned long long),
                                hipMallocSignalMemory) != hipSuccess) {
        (void)hipGetLastError();
        sig_counter_ = nullptr;
        sig_mode_ = 2;  // no signal memory: polling-kernel gate
      }
      if (sig_mode_ == 2) {
        sig_counter_ = dmalloc<unsigned long long>(8);
      }
      dzero(sig_counter_, sizeof(unsigned long long));
      dev_wait_ = opt_.device_halo_wait != 0;
      if (dev_wait_) {
        halo_counter_ = dmalloc<unsigned long long>(8);
        dzero(halo_counter_, sizeof(unsigned long long));
      }
    }
    // every unit list up front (a direct plan that cannot be built fails here, before any
    // bootstrap collective)
    for (int t = 0; t < (int)tiles_.size(); ++t)
      for (int K = 1; K <= G_; ++K)
        if (stream_k_supported(K)) (void)units(t, K);
    // LDS-tiled path: one tile owning the whole grid (any periodic halo is its own wrap).
    const bool self_only = tiles_.size() == 1 && transport_ == kTransportLocal;
    if (self_only && !opt_.naive && opt_.tiled != 0) {
      const int64_t NX = dec_.NX, NY = dec_.NY;
      // Auto: the tiled path up to 640x512-class grids.  Measured on MI355X, ref precision,
      // 1000 steps (profiles/tile_sweep_r2.txt), us/step tiled / LDS solver / streaming:
      // 80x64 0.49 / 1.58 / 1.57; 160x128 0.55 / 4.08 / 1.59; 320x256 0.65 / - / 1.55;
      // 640x512 0.96 / - / 1.86; 1280x1024 2.08 / - / 2.11 (streaming kept above 600k cells).
      const int64_t cells = NX * NY;
      // (with the fused device-side check the tiled path converges without host round trips
      // too, and is faster per step: it no longer yields to the whole-grid solver)
      const bool lds_whole =
          opt_.small_grid_lds && !has_exchange_ && lds_solver_fits(NX, NY) && opt_.convergence && !fused_;
      const bool want = opt_.tiled == 1 || (cells <= 600000 && !lds_whole);
      if (want && NX < (1 << 30) && NY < (1 << 30)) {
        // Automatic shape by grid size (tools/tile_sweep.py on MI355X, ref precision, us/step,
        // profiles/tile_sweep_r2.txt): small regions of many workgroups, 1024 threads, few cells
        // per lane — the launch is latency-bound (per-level LDS round trip + barrier), not VALU-bound.
        struct AutoTile {
          int64_t max_cells;
          int ry, k, tx, nt, cpl;
        };
        static const AutoTile kAuto[] = {
            {10240, 32, 16, 8, 1024, 1},    // 80x64: 0.49
            {40960, 64, 16, 4, 1024, 2},    // 160x128: 0.55
            {163840, 64, 16, 16, 1024, 4},  // 320x256: 0.65
            {INT64_MAX, 128, 16, 16, 1024, 4},  // 640x512: 0.96
        };
        const AutoTile* at = kAuto;
        while (cells > at->max_cells) ++at;
        int RY = opt_.tile_width > 0 ? opt_.tile_width : at->ry;
        if (RY != 32 && RY != 64 && RY != 128) throw std::invalid_argument("tile_width must be 32, 64 or 128");
        int K = opt_.tile_k > 0 ? opt_.tile_k : at->k;
        K = std::max(1, std::min(K, (RY - 4) / 2));
        int TX = opt_.tile_rows > 0 ? opt_.tile_rows : at->tx;
        int CPL = opt_.tile_cpl > 0 ? opt_.tile_cpl : at->cpl;
        if (CPL != 1 && CPL != 2 && CPL != 4) throw std::invalid_argument("tile_cpl must be 1, 2 or 4");
        while (CPL < 4 && RY / CPL > 64) CPL *= 2;  // a region row must fit one wave
        const int NT = opt_.tile_threads > 0 ? opt_.tile_threads : at->nt;
        if (NT != 256 && NT != 1024) throw std::invalid_argument("tile_threads must be 256 or 1024");
        while (TX > 1 && !tile_config_ok(TX, RY, K, CPL, NT)) TX /= 2;
        if (!tile_config_ok(TX, RY, K, CPL, NT)) throw std::invalid_argument("no valid LDS tile configuration");
        tiled_ = true;
        tile_tx_ = TX;
        tile_ry_ = RY;
        tile_k_ = K;
        tile_cpl_ = CPL;
        tile_nt_ = NT;
        Tile& T = tiles_[0];
        // two partial sets: a check's partials are still read (deferred decision) by the next
        // launch while that launch may store its own check's
        const int64_t need = 2 * tile_count((int)NX, (int)NY, TX, RY - 2 * K);
        if (need > T.pcap) {
          hipFree(T.partials);
          T.pcap = need;
          T.partials = dmalloc<double>((size_t)need);
        }
        if (recompute_rollback() && T.spare == nullptr) {
          // the third buffer of the speculative launches after checks (run_tiled): a copy of
          // the second (its ghost ring / poison included; the kernel writes only in-grid cells)
          const size_t n = (size_t)T.g.elems();
          T.spare = dmalloc<float>(n);
          H2D_HIP_CHECK(hipMemcpyAsync(T.spare, T.buf[1], n * sizeof(float), hipMemcpyDeviceToDevice, compute_));
        }
      }
    }
    if (recompute_rollback() && !tiled_ && !opt_.naive && tiles_[0].spare == nullptr) {
      // a lone streaming tile's third buffer (speculative launch after a check, StreamArgs::pend)
      // where it costs at most an eighth of the free memory (not for HBM-filling tiles: those
      // keep the separate decision kernel)
      const size_t n = (size_t)tiles_[0].g.elems();
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) == hipSuccess && n * sizeof(float) <= fr / 8) {
        tiles_[0].spare = dmalloc<float>(n);
        H2D_HIP_CHECK(hipMemcpyAsync(tiles_[0].spare, tiles_[0].buf[1], n * sizeof(float), hipMemcpyDeviceToDevice,
                                     compute_));
      }
    }
    if (!opt_.naive) warm_stream_kernels(opt_.precision, G_, compute_);
    if (!opt_.naive && (opt_.persistent > 0 || (opt_.persistent < 0 && direct_)))
      warm_pstream_kernels(opt_.precision, G_, compute_);
    if (tiled_) warm_tile_kernels(opt_.precision, compute_);
    // the whole device, not only this engine's stream: nothing another stream or the null stream
    // still has in flight (copies, fills of reused allocations) may overlap the first chunk
    H2D_HIP_CHECK(hipDeviceSynchronize());
  }
}

Engine::~Engine() {
  if (rccl_comm_) ncclCommDestroy((ncclComm_t)rccl_comm_);
  if (!on_gpu()) {
    for (auto& kv : local_descs_) delete[] kv.second.d;
    return;
  }
  hipDeviceSynchronize();
  for (auto& t : tiles_) {
    for (int b = 0; b < 2; ++b) hipFree(t.buf[b]);
    if (t.keep) hipFree(t.keep);
    if (t.spare) hipFree(t.spare);
  }
  if (h_conv_) hipHostFree(h_conv_);
  if (ev_check_) hipEventDestroy(ev_check_);
  if (d_stop_) hipFree(d_stop_);
  if (d_ticket_) hipFree(d_ticket_);
  for (auto& kv : pplans_) {
    hipFree(kv.second.d_units);
    hipFree(kv.second.d_prog);
  }
  for (auto& kv : units_) {
    hipFree(kv.second.d_all);
    hipFree(kv.second.d_interior);
    hipFree(kv.second.d_boundary);
    hipFree(kv.second.d_bfirst);
  }
  for (size_t r = 0; r < ipc_blocks_.size(); ++r)
    if (ipc_opened_[r]) hipIpcCloseMemHandle(ipc_blocks_[r]);
  hipFree(ipc_block_);
  hipFree(d_ipc_blocks_);
  hipFree(sig_counter_);
  hipFree(d_sig_timeout_);
  hipFree(halo_counter_);
  for (auto* m : {&local_descs_, &pack_descs_, &unpack_descs_})
    for (auto& kv : *m) hipFree(kv.second.d);
  for (auto& kv : ext_descs_) hipFree(kv.second.d);
  hipFree(d_lid_seen_);
  hipFree(d_resid_);
  hipFree(d_lds_steps_);
  hipFree(d_dummy_);
  hipFree(d_wait_acc_);
  if (d_phase_) hipFree(d_phase_);
  if (h_timeout_) hipHostFree(h_timeout_);
  for (auto& t : tiles_) hipFree(t.partials);
  hipHostFree(h_resid_);
  if (d_stamps_) hipFree(d_stamps_);
  hipFree(d_send_);
  hipFree(d_recv_);
  hipEventDestroy(ev_ready_);
  hipEventDestroy(ev_halo_);
  hipEventDestroy(ev_t0_);
  hipEventDestroy(ev_t1_);
  hipEventDestroy(ev_done_);
  for (auto& e : ev_prog_)
    if (e) hipEventDestroy(e);
  if (pooled_streams_) {
    return_stream(opt_.device, 0, compute_);
    return_stream(opt_.device, comm_prio_, comm_);
  } else {
    hipStreamDestroy(compute_);
    hipStreamDestroy(comm_);
  }
}

void Engine::check_tile(int t) const {
  if (t < 0 || t >= (int)tiles_.size()) throw std::out_of_range("tile index");
}

int64_t Engine::wave_capacity(int K) const {
  if (opt_.wave_capacity > 0) return opt_.wave_capacity;
  const int64_t cap = stream_wave_capacity(K, opt_.precision, opt_.device);
  return comm_cus_ > 0 ? cap * (device_cus_ - comm_cus_) / device_cus_ : cap;
}

int Engine::rows_per_wave(int K) const {
  auto it = units_.find(std::make_pair(0, K));
  if (it != units_.end()) return it->second.H;
  return opt_.rows_per_wave;
}

int Engine::num_units(int K) const {
  int n = 0;
  for (int t = 0; t < (int)tiles_.size(); ++t) {
    auto it = units_.find(std::make_pair(t, K));
    if (it != units_.end()) n += it->second.n_all;
  }
  return n;
}

const Engine::UnitLists& Engine::units(int t, int K) {
  auto key = std::make_pair(t, K);
  auto it = units_.find(key);
  if (it != units_.end()) return it->second;
  const Tile& tl = tiles_[t];
  const TileGeom& g = tl.g;
  UnitLists L;
  bool peer[kNumDirs];
  for (int d = 0; d < kNumDirs; ++d) peer[d] = dec_.neighbor(tl.rank, d) >= 0;
  const int64_t cap = wave_capacity(K);
  // Halo-dependent units gate the exchange of the NEXT chunk, which may be up to G_ rows deep
  // whatever this chunk's K: they must cover (and release) at least G_ rows.
  const int hb = std::max(opt_.boundary_rows, G_);
  UnitPlan P = plan_units(g, K, opt_.rows_per_wave, opt_.boundary == kFixed, opt_.periodic_x, opt_.periodic_y,
                          opt_.edge_weight, cap, peer, hb, opt_.row_edge_weight);
  // auto headroom: 16 wave slots (4096^2 row-periodic RCCL self-exchange, round 1: 14.3 ->
  // 10.4-10.9 us/step with 16 slots kept free for the exchange kernels)
  const int64_t reserve = opt_.reserve_waves >= 0 ? opt_.reserve_waves : 16;
  if (!direct_ && has_exchange_ && sig_mode_ > 0 && !P.boundary.empty()) {
    // interior units leave room for what runs beside them: the boundary units and the exchange
    // kernels of the signalled pipeline
    const int64_t nb = (int64_t)P.boundary.size();
    const int64_t cap_in = std::max<int64_t>(cap / 2, cap - nb - reserve);
    P = plan_units(g, K, opt_.rows_per_wave, opt_.boundary == kFixed, opt_.periodic_x, opt_.periodic_y,
                   opt_.edge_weight, cap_in, peer, hb, opt_.row_edge_weight);
  }
  // Signalled pipeline with only north/south peers (1-D row strips), and the direct (IPC)
  // pipeline for any decomposition: no short boundary units.  Every strip is cut into
  // capacity-fitted units as if the tile had no peers; the top unit of a strip with a north
  // peer and the bottom unit (streamed bottom-up) of a strip with a south peer become the N/S
  // halo units (kUnitNS): they wait for the halo, signal after their first G rows (the rows the
  // exchange sends) and carry on with the rest of their rows.  So the exchange starts early and
  // no wave idles (the short-unit plan left nb waves idle for most of the launch).
  // Direct pipeline with W/E / corner peers (2-D blocks): every unit of a strip whose outputs
  // reach the first / last G columns also pushes them to the W / E neighbour (and the strip's
  // top / bottom unit its G x G corner to the diagonal one), signalling at its end; it waits for
  // the same neighbours' previous pushes first (Unit::links: waits == pushes, a superset of the
  // ghost sides its cone reads, so a push never overtakes the neighbour's reads of the buffer
  // parity it overwrites).
  L.sig_rows = 0;
  const bool ns_only = !peer[kW] && !peer[kE] && !peer[kNW] && !peer[kNE] && !peer[kSW] && !peer[kSE];
  const bool sig_plan = sig_mode_ > 0 && opt_.overlap && opt_.signal_plan != 0 && ns_only && (peer[kN] || peer[kS]);
  if (has_exchange_ && (sig_plan || direct_)) {
    // The direct pipeline keeps no wave slots in reserve: nothing runs beside its launches.
    const int64_t reserve_sig = direct_ ? 0 : opt_.reserve_waves >= 0 ? opt_.reserve_waves : 16;
    const int hmin = std::max(K, G_);  // a N/S halo unit owns every row the next exchange sends
    // Attempts: the capacity-fitted plan; the same without shortening edge-strip units (their
    // strip-end units may fall below G rows); units of at least 2*max(K, G) rows.
    for (int attempt = 0; attempt < 3 && L.sig_rows == 0; ++attempt) {
    const int Hq = attempt < 2 ? opt_.rows_per_wave : std::max(opt_.rows_per_wave, 2 * hmin);
    const double ew = attempt == 0 ? opt_.edge_weight : 1.0;
    if (attempt == 1 && ew == opt_.edge_weight) continue;
    if (attempt == 2 && Hq == opt_.rows_per_wave) break;
    // 2-D direct: strips that push to a W / E neighbour run longer (their pushes and corner
    // stores): shorter units for them (opt_.side_weight; 8192x4096 2-D periodic tile, us/step at
    // weight 1.0 / 1.15 / 1.25 / 1.35 / 1.5: 19.7 / 17.6 / 16.4 / 16.0 / 16.2, alone 14.2)
    const bool sw = direct_ && (peer[kW] || peer[kNW] || peer[kSW]), se = direct_ && (peer[kE] || peer[kNE] || peer[kSE]);
    // the strip-end units become the N / S halo units: they start with the halo wait
    HaloCost hc;
    if (attempt == 0 && Hq <= 0 && opt_.halo_rows > 0) {
      hc.n = peer[kN];
      hc.s = peer[kS];
      hc.rows = opt_.halo_rows;
      hc.min_rows = hmin;
    }
    UnitPlan Q = plan_units(g, K, Hq, opt_.boundary == kFixed, opt_.periodic_x, opt_.periodic_y,
                            ew, std::max<int64_t>(cap / 2, cap - reserve_sig), nullptr, hb,
                            attempt == 0 ? opt_.row_edge_weight : 1.0, opt_.side_weight, G_, sw, se, hc);
    std::map<int, std::pair<int, int>> ends;  // strip -> (top unit, bottom unit) indices
    for (int i = 0; i < (int)Q.interior.size(); ++i) {
      const Unit& u = Q.interior[i];
      auto e = ends.emplace(u.strip, std::make_pair(i, i)).first;
      if (u.x0 < Q.interior[e->second.first].x0) e->second.first = i;
      if (u.x0 > Q.interior[e->second.second].x0) e->second.second = i;
    }
    bool ok = true;
    std::vector<int> role(Q.interior.size(), 0);  // 1 top, 2 bottom (reverse), 3 both (signal at end)
    for (auto& kv : ends) {
      const int ti = kv.second.first, bi = kv.second.second;
      if (ti == bi) {
        if (peer[kN] || peer[kS]) role[ti] = 3;
        if (direct_ && (peer[kN] || peer[kS])) ok = false;  // one unit would need both halos and push both ways
        continue;
      }
      if (peer[kN]) role[ti] = 1;
      if (peer[kS]) role[bi] = 2;
      // the neighbouring units' K-cones must not reach the ghost rows, and a signalling unit
      // must own every row the next exchange sends (up to G_, whatever this chunk's K)
      if ((peer[kN] && Q.interior[ti].h < hmin) || (peer[kS] && Q.interior[bi].h < hmin)) ok = false;
    }
    // side links of the direct pipeline
    std::vector<int> links(Q.interior.size(), 0);
    if (direct_ && !ns_only) {
      for (int i = 0; i < (int)Q.interior.size(); ++i) {
        const Unit& u = Q.interior[i];
        const bool pw = u.olo < G_, pe = u.ohi > g.ycell - G_;  // outputs in the first / last G columns
        const auto& e = ends.at(u.strip);
        int pu = 0;
        if (pw && peer[kW]) pu |= kLinkW;
        if (pe && peer[kE]) pu |= kLinkE;
        if (i == e.first && pw && peer[kNW]) pu |= kLinkNW;
        if (i == e.first && pe && peer[kNE]) pu |= kLinkNE;
        if (i == e.second && pw && peer[kSW]) pu |= kLinkSW;
        if (i == e.second && pe && peer[kSE]) pu |= kLinkSE;
        if (pu != 0 && (u.flags & kEdgeCols) != 0)
          throw std::invalid_argument("direct transport: a " + std::to_string(g.ycell) +
                                      "-column tile is too narrow (a side-pushing strip meets a global edge column)");
        links[i] = pu | (pu << 8);
      }
    }
    if (ok) {
      std::vector<Unit> sg, rest;
      for (int i = 0; i < (int)Q.interior.size(); ++i) {
        Unit u = Q.interior[i];
        u.links = links[i];
        if (role[i] == 0 && links[i] == 0) {
          rest.push_back(u);
          continue;
        }
        if (role[i] != 0) u.flags |= kUnitNS;
        if (role[i] == 2) u.flags |= kUnitReverse;
        if (role[i] == 3) u.flags |= kUnitSigEnd;
        sg.push_back(u);
      }
      P.interior = rest;
      P.boundary = sg;
      L.sig_rows = G_;  // released rows cover the deepest exchange that can follow
    }
    }
    if (direct_ && L.sig_rows <= 0)
      throw std::invalid_argument("IPC transport: the tile is too short for full-size halo units (" +
                                  std::to_string(g.xcell) + " rows, halo depth " + std::to_string(G_) + ")");
  }
  if (!direct_ && L.sig_rows == 0)
    for (Unit& u : P.boundary) u.flags |= kUnitNS;  // short boundary units: all wait / signal
  std::vector<Unit>& in = P.interior;
  std::vector<Unit>& bd = P.boundary;
  std::vector<Unit> all = in;
  all.insert(all.end(), bd.begin(), bd.end());
  if (all.size() > (size_t)(1 << 30)) throw std::runtime_error("too many work units");
  // integrity tags: every list its own (process-wide), carried by each of its units
  for (int i = 0; i < 4; ++i) L.tag[i] = next_tag();
  for (Unit& u : all) u.tag = L.tag[0];
  for (Unit& u : in) u.tag = L.tag[1];
  for (Unit& u : bd) u.tag = L.tag[2];
  L.H = 0;
  for (const Unit& u : in) L.H = std::max(L.H, u.h);
  for (const Unit& u : bd) {
    if (u.flags & kUnitNS) {
      const int d = (u.flags & kUnitReverse) ? 1 : 0;
      ++L.n_dir[d];
      ++L.pushes[d];  // kN / kS
    }
    for (int i = 0; i < kSideLinks; ++i)
      if ((u.links >> (8 + i)) & 1) ++L.pushes[kW + i];
  }
  L.n_all = (int)all.size();
  L.n_interior = (int)in.size();
  L.n_boundary = (int)bd.size();
  if (on_gpu()) {
    L.d_all = dmalloc<Unit>(all.size());
    L.d_interior = dmalloc<Unit>(in.size());
    L.d_boundary = dmalloc<Unit>(bd.size());
    h2d(L.d_all, all.data(), all.size() * sizeof(Unit));
    if (!in.empty()) h2d(L.d_interior, in.data(), in.size() * sizeof(Unit));
    if (!bd.empty()) h2d(L.d_boundary, bd.data(), bd.size() * sizeof(Unit));
    std::vector<Unit> bfirst = bd;
    bfirst.insert(bfirst.end(), in.begin(), in.end());
    for (Unit& u : bfirst) u.tag = L.tag[3];
    L.d_bfirst = dmalloc<Unit>(bfirst.size());
    h2d(L.d_bfirst, bfirst.data(), bfirst.size() * sizeof(Unit));
    Tile& tw = tiles_[t];
    // two sets: a lone tile's check partials are read by the next launch's deciding block while
    // that launch may store its own check's
    if (2 * (int64_t)all.size() > tw.pcap) {
      H2D_HIP_CHECK(hipDeviceSynchronize());
      hipFree(tw.partials);
      tw.pcap = std::max<int64_t>(2 * (int64_t)all.size(), 256);
      tw.partials = dmalloc<double>((size_t)tw.pcap);
    }
  }
  return units_.emplace(key, L).first->second;
}

void Engine::launch_chunk_tile(int t, int K, bool residual, int which, int src, hipStream_t stream) {
  Tile& tl = tiles_[t];
  const TileGeom& g = tl.g;
  const UnitLists& L = units(t, K);
  const hipStream_t ls = stream ? stream : compute_;
  StreamArgs a;
  zero_args(a);
  StreamDyn dy;
  if (src < 0) src = tl.cur;
  a.src = tl.buf[src];
  a.dst = tl.buf[1 - src];
  a.R = (int)lead_cols(K);
  a.wout = (int)strip_out_cols(K);
  a.pitch = g.pitch;
  a.G = g.G;
  a.PL = g.PL;
  a.xcell = g.xcell;
  a.ycell = g.ycell;
  a.gx0 = g.gx0;
  a.gy0 = g.gy0;
  a.NX = g.NX;
  a.NY = g.NY;
  a.cx = opt_.cx;
  a.cy = opt_.cy;
  a.fixed = opt_.boundary == kFixed;
  a.per_x = opt_.periodic_x;
  a.per_y = opt_.periodic_y;
  a.partials = tl.partials;
  a.dummy = d_dummy_;
  // write-through stores address rows by 32-bit offsets from a unit's base: tiles whose storage
  // spans 2^31 bytes or more (HBM-filling ones) keep plain stores
  a.wt = (opt_.wt_store < 0 ? 1 : opt_.wt_store) != 0 &&
         (double)(g.xcell + 2 * g.G) * (double)g.pitch * sizeof(float) < 2147483648.0 - 1048576.0;
  const bool whole = which == 0 || which == 3;  // the launch covers every unit of the tile
  // A lone single-process tile sums its partials and decides in ONE small kernel behind the
  // launch (device_decide).  (A last-wave in-kernel reduction was measured slower here: 1024
  // waves' ticket atomics on one address serialise; the tiled kernel, with few blocks, uses it.)
  const bool lone = fused_ && tiles_.size() == 1 && !rccl_comm_ && !direct_;
  // lone tile with a spare buffer: its check partials alternate between two sets, and the launch
  // after a check decides it in an extra block while its units compute into the spare buffer
  // (the check's input must survive: a converged check is rolled back by recomputing from it)
  const bool spec = lone && which == 0 && src == tl.cur && tl.spare != nullptr && stream == nullptr;
  if (spec && residual) a.partials = tl.partials + (size_t)pset_ * (size_t)(tl.pcap / 2);
  bool to_spare = false;
  if (spec && pend_parts_ != nullptr) {
    a.pend = pend_parts_;
    a.pend_n = pend_nparts_;
    a.pend_dec = pend_dec_;
    a.pend_dec.seq = 0;  // (per launch: StreamDyn::seq)
    dy.seq = pend_dec_.seq;
    a.dst = tl.spare;
    to_spare = true;
    pend_parts_ = nullptr;
  }
  if (fused_) {
    a.stop = d_stop_;
    // the rollback copy: a lone tile recomputes it on convergence instead (no 4 B/cell write per check)
    if (residual && !recompute_rollback()) a.keep = tl.keep;
  }
  // integrity: launch id at both ends of the per-launch part, the list's tag, the device error word
  dy.lid = (opt_.debug_kernel & 2) ? 0ull : ++lid_;
  a.dbg = opt_.debug_kernel;
  a.utag = L.tag[which];
  a.lid_seen = d_lid_seen_;
  a.timed_out = d_sig_timeout_;
  a.timed_out_host = h_timeout_dev_;
  if (transport_ == kTransportLocal && has_exchange_ && sig_mode_ == 0 && (stream == nullptr || stream == compute_)) {
    // serial local pipeline: the exchange copies in front of this launch on the compute stream
    a.copies_done = d_copies_done_;
    dy.copies_need = copies_need_;
    a.waves_done = d_waves_done_;
  }
  if (which == 0) {
    a.units = L.d_all;
    a.nunits = L.n_all;
  } else if (which == 1) {
    a.units = L.d_interior;
    a.nunits = L.n_interior;
  } else if (which == 2) {
    a.units = L.d_boundary;
    a.nunits = L.n_boundary;
    a.partials = tl.partials + L.n_interior;
  } else {
    a.units = L.d_bfirst;
    a.nunits = L.n_all;
    a.prot = L.n_interior;
    a.nsignal = L.n_boundary;
    a.sig_rows = L.sig_rows;
    a.halo_polls = std::max<long long>(1000, (long long)(opt_.halo_timeout_s * 1e6));  // ~1-2 us per poll
    a.timed_out = d_sig_timeout_;
    a.timed_out_host = h_timeout_dev_;
    if (direct_) {
      // Direct pipeline: chunk c reads the ghost rows the neighbours pushed during their chunk
      // c-1 (receive buffers of parity c), and pushes its own first G rows into the
      // neighbours' buffers of parity c+1 (their chunk c+1 reads them).
      const TileGeom& g = tl.g;
      const int p = (int)(ipc_chunk_ & 1), q = p ^ 1;
      const int pn = dec_.neighbor(tl.rank, kN), ps = dec_.neighbor(tl.rank, kS);
      const int64_t rowb = g.pitch * (int64_t)sizeof(float);
      const IpcLayout& me = ipc_lays_[tl.rank];
      if (pn >= 0) {
        const IpcLayout& nl = ipc_lays_[pn];
        a.wait[0] = reinterpret_cast<const unsigned long long*>(ipc_block_ + me.flag[kN]);
        dy.need[kN] = ipc_need_[kN];
        a.hsrc[0] = reinterpret_cast<const float*>(ipc_block_ + me.recv_n[p]);  // rows -G..-1
        a.push[0] = reinterpret_cast<float*>(ipc_blocks_[pn] + nl.recv_s[q]);   // N's rows xcell.. = my 0..
        a.sig[0] = reinterpret_cast<unsigned long long*>(ipc_blocks_[pn] + nl.flag[kS]);
      }
      if (ps >= 0) {
        const IpcLayout& sl = ipc_lays_[ps];
        a.wait[1] = reinterpret_cast<const unsigned long long*>(ipc_block_ + me.flag[kS]);
        dy.need[kS] = ipc_need_[kS];
        // ghost row i (xcell <= i < xcell+G) is receive row i - xcell
        a.hsrc[1] = reinterpret_cast<const float*>(ipc_block_ + me.recv_s[p] - (g.G + g.xcell) * rowb);
        // my row i (xcell-G <= i < xcell) is S's ghost row i - xcell, its receive row i - xcell + G
        // (S has my pitch: the same block column)
        a.push[1] = reinterpret_cast<float*>(ipc_blocks_[ps] + sl.recv_n[q] - (g.xcell - g.G) * rowb);
        a.sig[1] = reinterpret_cast<unsigned long long*>(ipc_blocks_[ps] + sl.flag[kN]);
      }
      // 2-D blocks: W / E ghost-column groups (reads: mine of parity p; pushes: the neighbours'
      // of parity q) and the corners
      if (me.xbuf != 0) {
        a.gsrc[0] = reinterpret_cast<const float*>(ipc_block_ + me.group(0, p));
        a.gsrc[1] = reinterpret_cast<const float*>(ipc_block_ + me.group(1, p));
      }
      for (int i = 0; i < kSideLinks; ++i) {
        const int d = kW + i, pr = dec_.neighbor(tl.rank, d);
        if (pr < 0) continue;
        a.xwait[i] = reinterpret_cast<const unsigned long long*>(ipc_block_ + me.flag[d]);
        dy.need[d] = ipc_need_[d];
        a.xsig[i] = reinterpret_cast<unsigned long long*>(ipc_blocks_[pr] + ipc_lays_[pr].flag[kDirOpp[d]]);
        a.xpush[i] = side_push_base(d, pr, q);
        a.xpitch[i] = ipc_lays_[pr].pitch;
      }
      // Defaults (tools/direct_fence_probe.py, MI355X): the push goes to the peer's UNCACHED
      // block, so the acknowledged stores (vmcnt(0)) are complete and need no L2 write-back
      // before the flag (1024x4096 tile: 3.27 -> 3.0 us/step); the ghost rows are read from my
      // uncached block, the agent-scope acquire only drops this CU's L1 lines.
      a.rel = opt_.direct_release < 0 ? 2 : opt_.direct_release;
      a.acq = opt_.direct_acquire < 0 ? 1 : opt_.direct_acquire;
    } else {
      a.sig[0] = a.sig[1] = sig_counter_;
      sig_target_ += (unsigned long long)L.n_boundary;
      if (dev_wait_) {
        a.wait[0] = a.wait[1] = halo_counter_;
        dy.need[kN] = dy.need[kS] = halo_seq_;
      }
    }
  }
  a.wait_acc = d_wait_acc_;
  if (d_stamps_ != nullptr && (int)tl_recs_.size() < opt_.timeline && a.nunits <= kTimelineUnits) {
    a.stamps = d_stamps_ + tl_recs_.size() * (size_t)kTimelineUnits * 4;
    tl_recs_.emplace_back(K, a.nunits);
  }
  const StreamArgs* blk = args_.get(a, ls);  // the plan-constant part: device-resident, uploaded once
  dy.nunits = a.nunits;
  dy.btag = a.head.btag;
  dy.pend = a.pend != nullptr;
  launch_stream(blk, a, dy, K, opt_.precision, residual, ls);
  if (to_spare) std::swap(tl.spare, tl.buf[1 - src]);  // the check's input becomes the spare
  if (a.waves_done != nullptr) waves_need_ += (unsigned long long)a.nunits;
  progress_tick(ls);
  // the direct pipeline's one tile: its partials go straight into the check's IPC all-reduce
  // (device_decide), one kernel instead of a reduction and an all-reduce
  const bool fold = fused_ && direct_ && tiles_.size() == 1;
  if (residual && whole && !lone && !fold) reduce_tile_residual(t, K);
  if (residual && whole && fold) {
    last_parts_ = a.partials;
    last_nparts_ = L.n_all;
  }
  if (residual && whole && lone) {
    last_parts_ = a.partials;
    last_nparts_ = L.n_all;
    if (spec) pset_ ^= 1;
  }
}

void Engine::reduce_tile_residual(int t, int K) {
  // Deterministic reduction of the tile's per-wave partials (interior then boundary) into d_resid_[t].
  const UnitLists& L = units(t, K);
  launch_reduce_sum(tiles_[t].partials, L.n_all, d_resid_ + t, compute_);
}

int Engine::chunk_len(int64_t done, int64_t total, int kmax, bool* check) const {
  // A chunk never crosses a convergence check; the check step is a chunk of its own, so a
  // converged run can roll back exactly one step (B-5 semantics).
  *check = false;
  int64_t seg = total - done;  // steps up to the end of the run or the next check step
  if (seg <= 0) return 0;
  if (opt_.convergence && fused_) {
    // fused check: the check step ends its chunk (the launch keeps the state one step earlier)
    const int64_t next_check = (done / opt_.interval + 1) * opt_.interval;
    seg = std::min<int64_t>(seg, next_check - done);
    const int64_t n = (seg + kmax - 1) / kmax;
    const int64_t k = std::max<int64_t>(1, (seg + n - 1) / n);
    *check = done + k == next_check;
    return (int)k;
  }
  if (opt_.convergence) {
    const int64_t next_check = (done / opt_.interval + 1) * opt_.interval;
    if (done + 1 == next_check) {
      *check = true;
      return 1;
    }
    seg = std::min<int64_t>(seg, next_check - 1 - done);
  }
  // Balanced chunks: a segment of L steps runs as ceil(L/kmax) launches of near-equal depth
  // (20 steps at K<=8: 7+7+6, not 8+8+4 — a launch's makespan is set by its deepest units, so a
  // ragged tail costs nearly a full launch of fixed overhead for half the work).
  const int64_t n = (seg + kmax - 1) / kmax;
  return (int)std::max<int64_t>(1, (seg + n - 1) / n);
}

int Engine::next_chunk(int64_t done, int64_t total, bool* check) const {
  int64_t k = chunk_len(done, total, G_, check);
  if (k == 0) return 0;
  if (on_gpu() && !opt_.naive)
    while (k > 1 && !stream_k_supported((int)k)) --k;
  if (opt_.naive) k = 1;
  k = std::max<int64_t>(1, k);
  if (fused_ && opt_.convergence) *check = (done + k) % opt_.interval == 0;  // k may have shrunk
  return (int)k;
}

int Engine::next_tag() {
  static std::atomic<int> seq{0};
  int t = 0;
  while (t == 0) t = (int)((unsigned)seq.fetch_add(1) * 2654435761u);  // spread, never 0
  return t;
}

Engine::DescList Engine::upload_descs(std::vector<CopyDesc>& v) {
  DescList L;
  L.n = (int)v.size();
  L.tag = next_tag();
  for (CopyDesc& c : v) {
    c.tag = L.tag;
    L.maxe = std::max(L.maxe, c.rows * c.cols);
  }
  if (on_gpu()) {
    if (!v.empty()) {
      L.d = dmalloc<CopyDesc>(v.size());
      h2d(L.d, v.data(), v.size() * sizeof(CopyDesc));
    }
  } else {
    // CPU: keep the host descriptors alive in a heap block
    L.d = new CopyDesc[v.size() ? v.size() : 1];
    std::copy(v.begin(), v.end(), L.d);
  }
  return L;
}

const Engine::DescList& Engine::ext_descs(std::vector<CopyDesc>& v) {
  // the caller-driven pack / unpack lists (external transports): one upload per distinct list
  // (the descriptors name the caller's buffers), from the metadata arena
  std::string key(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(CopyDesc));
  auto it = ext_descs_.find(key);
  if (it != ext_descs_.end()) return it->second;
  return ext_descs_.emplace(std::move(key), upload_descs(v)).first->second;
}

const Engine::DescList& Engine::local_descs(int K) {
  // Tile-to-tile copies: peer's owned edge (its current buffer) -> my ghost ring.
  const int parity = tiles_[0].cur;
  auto key = std::make_pair(K, parity);
  auto it = local_descs_.find(key);
  if (it == local_descs_.end()) {
    std::vector<CopyDesc> v;
    std::map<int, int> tile_of_rank;
    for (int t = 0; t < (int)tiles_.size(); ++t) tile_of_rank[tiles_[t].rank] = t;
    for (int t = 0; t < (int)tiles_.size(); ++t) {
      Tile& T = tiles_[t];
      ExchangePlan p = make_plan(dec_, T.rank, T.g, K);
      for (int d = 0; d < kNumDirs; ++d) {
        if (p.peer[d] < 0) continue;
        const Tile& U = tiles_[tile_of_rank.at(p.peer[d])];
        ExchangePlan q = make_plan(dec_, U.rank, U.g, K);
        const Rect& s = q.send_rect[kDirOpp[d]];
        const Rect& r = p.recv_rect[d];
        if (s.rows != r.rows || s.cols != r.cols) throw std::logic_error("halo shape mismatch");
        v.push_back(CopyDesc{U.buf[U.cur] + U.g.idx(s.r0, s.c0), T.buf[T.cur] + T.g.idx(r.r0, r.c0), U.g.pitch,
                             T.g.pitch, r.rows, r.cols});
      }
    }
    it = local_descs_.emplace(key, upload_descs(v)).first;
  }
  return it->second;
}

void Engine::local_copy(const DescList& D, hipStream_t s) {
  // on the compute stream the copy blocks are counted: the serial pipeline's stencil launch
  // checks that all of them completed before it started (kIntegOrder)
  const bool counted = s == compute_;
  launch_copy_rects(D.d, D.n, D.maxe, s, D.tag, counted ? d_copies_done_ : nullptr, d_sig_timeout_, h_timeout_dev_,
                    counted ? d_waves_done_ : nullptr, waves_need_);
  if (counted) copies_need_ += (unsigned long long)copy_rects_blocks(D.n, D.maxe);
}

void Engine::exchange_local(int k) {
  if (!has_exchange_) return;
  const DescList& D = local_descs(k);
  if (D.n == 0) return;
  if (on_gpu()) {
    local_copy(D, compute_);
  } else {
    cpu_copy_rects(std::vector<CopyDesc>(D.d, D.d + D.n));
  }
}

void Engine::do_exchange_async(int K, hipStream_t s) {
  // Runs on comm_ after ev_ready_ (or, serial pipeline, in order on the compute stream).
  hipStream_t xs = s ? s : comm_;
  if (transport_ == kTransportLocal) {
    local_copy(local_descs(K), xs);
    return;
  }
  if (transport_ != kTransportRccl) throw std::logic_error("do_exchange_async: transport");
  if (!rccl_comm_) throw std::runtime_error("RCCL transport selected but init_rccl() was not called");
  Tile& T = tiles_[0];
  ncclComm_t comm = (ncclComm_t)rccl_comm_;
  if (contig_) {
    // 1-D row strips: every tile has the full row width and the same pitch, so a K-deep
    // halo is K consecutive storage rows (the west/east pad columns lie outside the global
    // grid and are never read by a valid update).  Send owned rows [0,K) north and
    // [xcell-K,xcell) south; receive straight into ghost rows [-K,0) and [xcell,xcell+K).
    // Same posting order as the general path (sends N,S; receives for ghost S,N).
    const TileGeom& g = T.g;
    float* b = T.buf[T.cur];
    const size_t cnt = (size_t)K * (size_t)g.pitch;
    const int pn = dec_.neighbor(T.rank, kN), ps = dec_.neighbor(T.rank, kS);
    auto row = [&](int64_t i) { return b + (size_t)(i + g.G) * (size_t)g.pitch; };
    H2D_NCCL_CHECK(ncclGroupStart());
    for (int d = 0; d < kNumDirs; ++d) {
      if (d == kN && pn >= 0) H2D_NCCL_CHECK(ncclSend(row(0), cnt, ncclFloat, pn, comm, xs));
      if (d == kS && ps >= 0) H2D_NCCL_CHECK(ncclSend(row(g.xcell - K), cnt, ncclFloat, ps, comm, xs));
    }
    for (int d = 0; d < kNumDirs; ++d) {
      const int gs = kDirOpp[d];
      if (gs == kN && pn >= 0) H2D_NCCL_CHECK(ncclRecv(row(-K), cnt, ncclFloat, pn, comm, xs));
      if (gs == kS && ps >= 0) H2D_NCCL_CHECK(ncclRecv(row(g.xcell), cnt, ncclFloat, ps, comm, xs));
    }
    H2D_NCCL_CHECK(ncclGroupEnd());
    return;
  }
  ExchangePlan p = make_plan(dec_, T.rank, T.g, K);
  if (p.send_total > stage_cap_ || p.recv_total > stage_cap_) {
    H2D_HIP_CHECK(hipStreamSynchronize(xs));
    hipFree(d_send_);
    hipFree(d_recv_);
    stage_cap_ = std::max(p.send_total, p.recv_total);
    d_send_ = dmalloc<float>((size_t)stage_cap_);
    d_recv_ = dmalloc<float>((size_t)stage_cap_);
    for (auto* m : {&pack_descs_, &unpack_descs_}) {
      for (auto& kv : *m) hipFree(kv.second.d);
      m->clear();
    }
  }
  auto key = std::make_pair(K, T.cur);
  auto ip = pack_descs_.find(key);
  if (ip == pack_descs_.end()) {
    std::vector<CopyDesc> pv, uv;
    plan_pack_descs(p, T.g, T.buf[T.cur], d_send_, pv);
    plan_unpack_descs(p, T.g, T.buf[T.cur], d_recv_, uv);
    DescList dp = upload_descs(pv), du = upload_descs(uv);
    ip = pack_descs_.emplace(key, dp).first;
    unpack_descs_.emplace(key, du);
  }
  auto iu = unpack_descs_.find(key);
  const DescList& P = ip->second;
  launch_copy_rects(P.d, P.n, P.maxe, xs, P.tag, nullptr, d_sig_timeout_, h_timeout_dev_);
  H2D_NCCL_CHECK(ncclGroupStart());
  // Send segment d to peer[d]; receive the peer's matching segment into ghost side opp(d)
  // from peer[opp(d)].  Posting both in direction order keeps per-peer FIFO matching
  // correct even when one peer is the neighbour on several sides (periodic, 2-wide grids).
  for (int d = 0; d < kNumDirs; ++d) {
    if (p.peer[d] < 0 || p.send_rect[d].count() == 0) continue;
    H2D_NCCL_CHECK(ncclSend(d_send_ + p.send_off[d], (size_t)p.send_rect[d].count(), ncclFloat, p.peer[d], comm, xs));
  }
  for (int d = 0; d < kNumDirs; ++d) {
    const int g = kDirOpp[d];
    if (p.peer[g] < 0 || p.recv_rect[g].count() == 0) continue;
    H2D_NCCL_CHECK(ncclRecv(d_recv_ + p.recv_off[g], (size_t)p.recv_rect[g].count(), ncclFloat, p.peer[g], comm, xs));
  }
  H2D_NCCL_CHECK(ncclGroupEnd());
  const DescList& U = iu->second;
  launch_copy_rects(U.d, U.n, U.maxe, xs, U.tag, nullptr, d_sig_timeout_, h_timeout_dev_);
}

void Engine::gate_exchange() {
  // comm stream: everything after this waits until every halo-dependent unit launched so far
  // has released its rows
  if (sig_mode_ == 1) {
    H2D_HIP_CHECK(hipStreamWaitValue64(comm_, sig_counter_, sig_target_, hipStreamWaitValueGte));
  } else {
    // ~0.5 us per poll: gives up after ~halo_timeout_s (polled by the host per chunk)
    launch_wait_counter(sig_counter_, sig_target_, d_sig_timeout_, h_timeout_dev_,
                        std::max<long long>(1000, (long long)(opt_.halo_timeout_s * 2e6)), comm_);
  }
}

void Engine::exchange_landed() {
  if (dev_wait_) {
    launch_set_counter(halo_counter_, ++halo_seq_, comm_);
  } else {
    H2D_HIP_CHECK(hipEventRecord(ev_halo_, comm_));
  }
}

std::string Engine::pipeline() const {
  if (!has_exchange_) return "none";
  if (direct_) return "direct";
  if (transport_ == kTransportExternal) return "external";
  if (sig_mode_ > 0) return "signal";
  return "serial";
}

void Engine::advance(int k, bool residual) {
  if (k < 1 || k > G_) throw std::invalid_argument("advance: chunk size must be in [1, halo depth]");
  for (int t = 0; t < (int)tiles_.size(); ++t) {
    Tile& tl = tiles_[t];
    if (on_gpu()) {
      if (opt_.naive) {
        if (k != 1) throw std::invalid_argument("naive path advances one step at a time");
        launch_naive_step(tl.g, tl.buf[tl.cur], tl.buf[1 - tl.cur], opt_.precision, opt_.boundary, opt_.cx, opt_.cy,
                          opt_.periodic_x, opt_.periodic_y, compute_);
        if (residual) {
          const int np = 256;
          launch_tile_residual(tl.g, tl.buf[1 - tl.cur], tl.buf[tl.cur], tl.partials, np, compute_);
          launch_reduce_sum(tl.partials, np, d_resid_ + t, compute_);
        }
      } else {
        launch_chunk_tile(t, k, residual, 0);
      }
    } else {
      Physics ph;
      ph.boundary = opt_.boundary;
      ph.precision = opt_.precision;
      ph.cx = opt_.cx;
      ph.cy = opt_.cy;
      ph.periodic_x = opt_.periodic_x;
      ph.periodic_y = opt_.periodic_y;
      tl.last_resid = cpu_tile_advance(tl.g, ph, tl.buf[tl.cur], tl.buf[1 - tl.cur], k, tl.scratch[0].data(),
                                       tl.scratch[1].data(), residual);
    }
    tl.cur = 1 - tl.cur;
  }
}

double Engine::local_residual() {
  double s = 0.0;
  if (on_gpu()) {
    H2D_HIP_CHECK(hipMemcpyAsync(h_resid_, d_resid_, sizeof(double) * tiles_.size(), hipMemcpyDeviceToHost, compute_));
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
    for (size_t t = 0; t < tiles_.size(); ++t) s += h_resid_[t];
  } else {
    for (const Tile& t : tiles_) s += t.last_resid;
  }
  return s;
}

void Engine::progress_tick(hipStream_t s) {
  if (!rccl_comm_ || (++launches_ % 16) != 0) return;
  const int i = (int)((launches_ / 16) % kProgRing);
  H2D_HIP_CHECK(hipEventRecord(ev_prog_[i], s));
  prog_seq_[i] = launches_;
}

void Engine::wait_event(hipEvent_t ev) {
  // Failure detection: with a communicator, poll the event and RCCL's asynchronous error
  // state instead of blocking, and abort the communicator after `watchdog_s` WITHOUT PROGRESS
  // (no newer progress event completed — a dead peer would otherwise hang the rank forever;
  // a long healthy run keeps completing launches and is never aborted).
  if (!ev) {
    H2D_HIP_CHECK(hipEventRecord(ev_done_, compute_));
    ev = ev_done_;
  }
  if (!rccl_comm_) {
    H2D_HIP_CHECK(hipEventSynchronize(ev));
    return;
  }
  auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 0;; ++spin) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) H2D_HIP_CHECK(e);
    if ((spin & 63) == 0) {
      for (int i = 0; i < kProgRing; ++i)
        if (prog_seq_[i] > prog_seen_ && hipEventQuery(ev_prog_[i]) == hipSuccess) {
          prog_seen_ = prog_seq_[i];
          t0 = std::chrono::steady_clock::now();
        }
    }
    ncclResult_t async = ncclSuccess;
    ncclCommGetAsyncError((ncclComm_t)rccl_comm_, &async);
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (async != ncclSuccess || (opt_.watchdog_s > 0 && el > opt_.watchdog_s)) {
      const std::string why = async != ncclSuccess ? std::string("RCCL async error: ") + ncclGetErrorString(async)
                                                   : "watchdog: no progress (completed launch) for " +
                                                         std::to_string(el) + " s";
      ncclCommAbort((ncclComm_t)rccl_comm_);
      rccl_comm_ = nullptr;
      throw std::runtime_error("[rank " + std::to_string(rccl_rank_) + "] " + why);
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

double Engine::finish_residual() {
  if (direct_) return ipc_allreduce_residual();
  if (on_gpu() && rccl_comm_) {
    // Local sum over tiles (one tile under RCCL) -> all-reduce across ranks on the compute stream.
    H2D_NCCL_CHECK(ncclAllReduce(d_resid_, d_resid_ + tiles_.size(), 1, ncclDouble, ncclSum, (ncclComm_t)rccl_comm_,
                                 compute_));
    H2D_HIP_CHECK(hipMemcpyAsync(h_resid_, d_resid_ + tiles_.size(), sizeof(double), hipMemcpyDeviceToHost, compute_));
    H2D_HIP_CHECK(hipEventRecord(ev_ready_, compute_));
    wait_event(ev_ready_);
    return h_resid_[0];
  }
  return local_residual();
}

void Engine::rollback() {
  for (Tile& t : tiles_) t.cur = 1 - t.cur;
  // the neighbours' receive buffers hold rows of the undone chunk: a new prime is needed
  if (direct_) ipc_primed_ = false;
}

RunStats Engine::run(int64_t steps) {
  try {
    return run_impl(steps);
  } catch (const std::exception& e) {
    const std::string m = e.what();
    if (m.rfind("[rank ", 0) == 0) throw;
    throw std::runtime_error("[rank " + std::to_string(tiles_.empty() ? 0 : tiles_[0].rank) + "] " + m);
  }
}

void Engine::poll_abort() {
  if (!h_timeout_) return;
  const unsigned int to = __atomic_load_n(h_timeout_, __ATOMIC_ACQUIRE);
  if (!to) return;
  // The device gave up on a halo: every later chunk computes on stale ghost cells and the
  // host's sig/halo sequence numbers no longer match the device counters, so this engine
  // cannot be reused.  Drain what is queued (bounded waits: it terminates).
  broken_ = true;
  hipStreamSynchronize(comm_);
  hipStreamSynchronize(compute_);
  // the host mirror holds the latest bit; the device word all of them
  unsigned int all = to;
  if (hipMemcpy(&all, d_sig_timeout_, sizeof(all), hipMemcpyDeviceToHost) != hipSuccess) all = to;
  all |= to;
  const unsigned integ = kIntegArgs | kIntegUnits | kIntegReplay | kIntegDescs | kIntegOrder | kIntegOrder2;
  if (all & integ) {
    broken_why_ = std::string("integrity check failed (bits ") + std::to_string(all) + "): " +
                  ((all & kIntegArgs) ? "torn kernel arguments (launch ids at the two ends differ) " : "") +
                  ((all & kIntegUnits) ? "a work unit of another list (stale unit-list upload) " : "") +
                  ((all & kIntegReplay) ? "a launch ran with the arguments of an earlier launch " : "") +
                  ((all & kIntegDescs) ? "a copy descriptor of another list (stale descriptor upload) " : "") +
                  ((all & kIntegOrder) ? "a stencil launch started before its exchange copy finished " : "") +
                  ((all & kIntegOrder2) ? "an exchange copy started before the stencil launches before it finished " : "");
  } else {
    broken_why_ = std::string("signalled halo pipeline timed out: ") +
                  ((all & 1) ? "the exchange gate (boundary units never completed) " : "") +
                  ((all & 2) ? "the device-side halo wait (the exchange never landed) " : "") +
                  ((all & 4) ? "the residual all-reduce (a rank never contributed) " : "") +
                  ((all & 8) ? "the persistent kernel's neighbour wait or its halo units' chunk-order wait" : "");
  }
  throw std::runtime_error(broken_why_);
}

RunStats Engine::run_impl(int64_t steps) {
  if (broken_) throw std::runtime_error("engine unusable after an earlier failure: " + broken_why_);
  if (transport_ == kTransportExternal && has_exchange_)
    throw std::runtime_error("external transport: drive the loop from the caller");
  if (transport_ == kTransportRccl && has_exchange_ && !rccl_comm_)
    throw std::runtime_error("RCCL transport selected but init_rccl() was not called");
  if (direct_ && !ipc_primed_)
    throw std::runtime_error("IPC transport: ipc_open() + ipc_prime() needed before a run (and after upload / a "
                             "converged run)");
  RunStats st;
  const auto w0 = std::chrono::steady_clock::now();
  const int64_t target = steps_done_ + steps;
  tl_recs_.clear();
  if (!on_gpu()) {
    run_cpu(st, target);
    st.steps_done = steps_done_;
    st.wall_ms = st.device_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    return st;
  }
  const bool timing = opt_.sync_mode == 0 || opt_.sync_mode == 3;
  if (timing) H2D_HIP_CHECK(hipEventRecord(ev_t0_, compute_));
  const bool single = tiles_.size() == 1 && !has_exchange_;
  if (tiled_) {
    run_tiled(st, target);
  } else if (single && opt_.small_grid_lds && !opt_.naive && lds_solver_fits(dec_.NX, dec_.NY) && steps > 0) {
    run_lds(st, steps);
  } else {
    st.path = opt_.naive ? "naive" : "stream";
    if (direct_) run_direct(st, target);
    else if (has_exchange_ && sig_mode_ > 0) run_signal(st, target);
    else run_serial(st, target);
  }
  flush_pending_decision();  // the run's last check, not followed by a launch
  end_of_run_wait(st, w0);
  poll_abort();
  if (fused_ && finalize_convergence(st)) end_of_run_wait(st, w0);  // times include the recompute launches
  trace_collect(st);
  st.steps_done = steps_done_;
  return st;
}

// CPU: the same chunk / check schedule, halos copied between the process's tiles.
void Engine::run_cpu(RunStats& st, int64_t target) {
  while (steps_done_ < target) {
    bool check = false;
    const int k = next_chunk(steps_done_, target, &check);
    if (has_exchange_) {
      exchange_local(k);
      ++st.exchanges;
    }
    advance(k, check);
    ++st.chunks;
    if (check) {
      st.residual = local_residual();
      if (st.residual < opt_.sensitivity) {
        rollback();
        st.converged = true;
        break;
      }
    }
    steps_done_ += k;
  }
  st.path = "cpu";
}

void Engine::run_tiled(RunStats& st, int64_t target) {
  // LDS-tiled path: one launch per chunk of up to tile_k_ steps, the tiling re-derived per
  // chunk length (TY = RY - 2k).
  st.path = "tiled";
  Tile& T = tiles_[0];
  // A lone fused-check tile lets a chunk run THROUGH a check step: the residual is summed at
  // that level inside the launch (TileArgs::rlev) and a converged check is rolled back by
  // recomputation, so a check costs no launch of its own (interval 20 at K 16: 1.25 launches
  // per 20 steps instead of 2).
  const bool span = fused_ && recompute_rollback();
  // span mode defers each check's decision to the next launch (TileArgs::pend): the check
  // launch only stores its partials (set `pset` of the two), the next launch's workgroups sum
  // them before their own work, and a check left pending at the end of the run is decided by
  // one small kernel
  bool pend = false;
  int pend_n = 0, pset = 0;
  DecideArgs pend_dec;
  while (steps_done_ < target) {
    bool check = false;
    int lvl = 0;
    int k;
    if (span) {
      const int64_t seg = target - steps_done_, n = (seg + tile_k_ - 1) / tile_k_;
      const int64_t next_check = (steps_done_ / opt_.interval + 1) * opt_.interval;
      int64_t kk = std::max<int64_t>(1, (seg + n - 1) / n);
      kk = std::min<int64_t>(kk, next_check + opt_.interval - 1 - steps_done_);  // one check per chunk
      k = (int)kk;
      check = opt_.convergence && steps_done_ + k >= next_check;
      lvl = check ? (int)(next_check - steps_done_) : 0;
    } else {
      k = chunk_len(steps_done_, target, tile_k_, &check);
    }
    TileArgs a;
    zero_args(a);
    TileDyn dy;
    // the launch after a check decides it in its extra block while its tiles compute: it must
    // not write the check's input (the rollback recomputes from it), so it writes the spare
    const bool to_spare = span && pend && T.spare != nullptr;
    a.src = T.buf[T.cur] + T.g.idx(0, 0);
    a.dst = (to_spare ? T.spare : T.buf[1 - T.cur]) + T.g.idx(0, 0);
    a.pitch = T.g.pitch;
    a.NX = (int)T.g.xcell;
    a.NY = (int)T.g.ycell;
    a.TX = tile_tx_;
    a.NT = tile_nt_;
    a.CPL = tile_cpl_;
    a.RY = tile_ry_;
    a.K = k;
    a.TY = tile_ry_ - 2 * k;
    a.cx = opt_.cx;
    a.cy = opt_.cy;
    a.fixed = opt_.boundary == kFixed;
    a.per_x = opt_.periodic_x;
    a.per_y = opt_.periodic_y;
    a.partials = T.partials;
    if (span && pend) {
      a.pend = T.partials + (size_t)(pset ^ 1) * (size_t)(T.pcap / 2);
      a.pend_n = pend_n;
      a.pend_dec = pend_dec;
      a.pend_dec.seq = 0;  // (per launch: TileDyn::pend_seq)
      dy.pend_seq = pend_dec.seq;
      pend = false;
    }
    if (fused_) {
      a.stop = d_stop_;
      if (check) {
        a.keep = recompute_rollback() ? nullptr : T.keep + T.g.idx(0, 0);
        a.rlev = lvl;
        if (span) {
          a.partials = T.partials + (size_t)pset * (size_t)(T.pcap / 2);
          pend = true;
          pend_n = tile_count(a.NX, a.NY, a.TX, a.TY);
          pend_dec = decide_args(0, true);
          pset ^= 1;
        } else {
          a.dec = decide_args(0, true);  // the last block sums the partials and decides
          dy.seq = a.dec.seq;
          a.dec.seq = 0;  // (per launch: TileDyn::seq)
        }
        decided_in_launch_ = true;
      }
    }
    trace_begin("step", compute_);
    prepare_tile(a);
    const TileArgs* blk = args_.get(a, compute_);  // the plan-constant part: device-resident
    dy.btag = a.head.btag;
    launch_tile(blk, a, dy, opt_.precision, check, compute_);
    trace_end("step", compute_);
    if (check && !fused_) launch_reduce_sum(a.partials, tile_count(a.NX, a.NY, a.TX, a.TY), d_resid_, compute_);
    if (to_spare) std::swap(T.spare, T.buf[1 - T.cur]);  // the check's input becomes the spare
    T.cur = 1 - T.cur;
    ++st.chunks;
    if (check) {
      if (fused_) {
        if (check_point(steps_done_, k, lvl > 0 ? lvl : k)) {
          pend = false;  // seen converged: nothing later needs deciding
          break;
        }
      } else {
        st.residual = finish_residual();
        if (st.residual < opt_.sensitivity) {
          rollback();
          st.converged = true;
          break;
        }
      }
    }
    steps_done_ += k;
  }
  // the run's last check, not followed by a launch: decide it now
  if (pend) launch_reduce_decide(T.partials + (size_t)(pset ^ 1) * (size_t)(T.pcap / 2), pend_n, pend_dec, compute_);
}

void Engine::run_lds(RunStats& st, int64_t steps) {
  // Whole run inside one workgroup's LDS.
  st.path = "lds";
  Tile& T = tiles_[0];
  const int interval = opt_.convergence ? (int)opt_.interval : 0;
  // The LDS kernel counts steps from 1; align the convergence cadence with steps_done_.
  if (interval > 0 && steps_done_ % interval != 0)
    throw std::runtime_error("LDS solver: resume point must be a multiple of the convergence interval");
  launch_lds_solver(T.buf[T.cur] + T.g.idx(0, 0), T.g.pitch, T.buf[1 - T.cur] + T.g.idx(0, 0), T.g.pitch, T.g.xcell,
                    T.g.ycell, steps, opt_.precision, opt_.boundary, opt_.cx, opt_.cy, opt_.periodic_x,
                    opt_.periodic_y, interval, opt_.sensitivity, d_lds_steps_, d_resid_, compute_);
  long long done = 0;
  H2D_HIP_CHECK(hipMemcpyAsync(&done, d_lds_steps_, sizeof(long long), hipMemcpyDeviceToHost, compute_));
  H2D_HIP_CHECK(hipMemcpyAsync(h_resid_, d_resid_, sizeof(double), hipMemcpyDeviceToHost, compute_));
  H2D_HIP_CHECK(hipStreamSynchronize(compute_));
  T.cur = 1 - T.cur;
  st.converged = done < steps;
  st.residual = h_resid_[0];
  steps_done_ += done;
  st.chunks = 1;
}

void Engine::run_direct(RunStats& st, int64_t target) {
  // Direct pipeline (IPC, 1-D row strips): ONE launch per chunk on ONE stream.  Its halo
  // units (top / bottom unit of every column strip) first wait in the kernel until the
  // neighbours' pushes for this chunk have landed (flags in my uncached block), read their
  // ghost rows from my receive buffers, and as soon as their first G output rows are
  // final they store them into the neighbours' receive buffers over xGMI, release them at
  // system scope and bump the neighbours' flags.  No comm stream, no RCCL kernel, no
  // host round trip: the exchange of chunk c+1 rides inside chunk c.
  bool check = false;
  int k = next_chunk(steps_done_, target, &check);
  while (k > 0) {
    if (!check) {
      const int J = plain_run(steps_done_, target, k);
      if (J >= 2 && pst_everywhere(k) && pplan(k) != nullptr) {
        // a run of equal plain chunks: ONE persistent launch (the same flags and receive-
        // buffer parities per chunk as the launches below; every rank's plan has a
        // persistent plan at this depth, so every rank runs this chunk run the same way)
        trace_begin("chunk", compute_);
        launch_pstream_chunks(k, J);
        trace_end("chunk", compute_);
        for (int d = kN; d <= kS; ++d) {  // 1-D row strips: N / S neighbours only
          const int pr = dec_.neighbor(tiles_[0].rank, d);
          if (pr >= 0) ipc_need_[d] += (unsigned long long)J * (unsigned long long)pst_counts_[pr].at((size_t)k * 2 + (d == kN ? 1 : 0));
        }
        ipc_chunk_ += (unsigned long long)J;
        if (J & 1) tiles_[0].cur = 1 - tiles_[0].cur;
        st.chunks += J;
        st.exchanges += J;
        poll_abort();
        steps_done_ += (int64_t)J * k;
        k = next_chunk(steps_done_, target, &check);
        continue;
      }
    }
    trace_begin("chunk", compute_);
    launch_chunk_tile(0, k, check, 3);
    trace_end("chunk", compute_);
    for (int d = 0; d < kNumDirs; ++d) {  // the neighbours' pushes this chunk, for my next one
      const int pr = dec_.neighbor(tiles_[0].rank, d);
      if (pr >= 0) ipc_need_[d] += (unsigned long long)ipc_counts_[pr].at((size_t)k * kNumDirs + kDirOpp[d]);
    }
    ++ipc_chunk_;
    tiles_[0].cur = 1 - tiles_[0].cur;
    ++st.chunks;
    ++st.exchanges;
    poll_abort();
    if (check) {
      if (fused_) {
        if (check_point(steps_done_, k)) break;  // converged (seen by the host): stop enqueueing
      } else {
        st.residual = finish_residual();
        if (st.residual < opt_.sensitivity) {
          rollback();
          st.converged = true;
          break;
        }
      }
    }
    steps_done_ += k;
    k = next_chunk(steps_done_, target, &check);
  }
}

void Engine::run_signal(RunStats& st, int64_t target) {
  // Signalled pipeline (per chunk c), two streams:
  //   compute: ONE launch of every unit of chunk c, halo-dependent units first (they are
  //            dispatched first and are short); each of them waits in the kernel until
  //            halo(c) has landed (halo_counter_), and when done releases its rows at
  //            system scope and bumps sig_counter_
  //   comm   : gate (sig_counter_ >= units launched so far) -> halo exchange of chunk c+1
  //            -> halo_counter_ = c+1
  // The exchange starts while the interior units of chunk c are still running, no unit
  // competes with a second stencil launch for wave slots, and the compute stream never
  // waits on the comm stream (a cross-queue wait costs ~6 us of dispatch latency; with
  // device_halo_wait = 0 the launch waits on an event instead).
  bool check = false;
  int k = next_chunk(steps_done_, target, &check);
  if (k > 0) {
    H2D_HIP_CHECK(hipEventRecord(ev_ready_, compute_));
    H2D_HIP_CHECK(hipStreamWaitEvent(comm_, ev_ready_, 0));
    trace_begin("exchange", comm_);
    do_exchange_async(k);
    trace_end("exchange", comm_);
    exchange_landed();
    ++st.exchanges;
  }
  while (k > 0) {
    if (!dev_wait_) H2D_HIP_CHECK(hipStreamWaitEvent(compute_, ev_halo_, 0));
    trace_begin("chunk", compute_);
    for (int t = 0; t < (int)tiles_.size(); ++t) launch_chunk_tile(t, k, check, 3);
    trace_end("chunk", compute_);
    for (Tile& tl : tiles_) tl.cur = 1 - tl.cur;
    ++st.chunks;
    poll_abort();
    bool check_next = false;
    const int k_next = next_chunk(steps_done_ + k, target, &check_next);
    if (check) {
      // nothing is in flight on the comm stream here (the exchange of chunk c completed
      // before the chunk started), so the all-reduce is the communicator's only operation
      if (fused_) {
        if (check_point(steps_done_, k)) break;  // converged (seen by the host): stop enqueueing
      } else {
        st.residual = finish_residual();
        if (st.residual < opt_.sensitivity) {
          rollback();
          st.converged = true;
          break;
        }
      }
    }
    if (k_next > 0) {
      gate_exchange();
      trace_begin("exchange", comm_);
      do_exchange_async(k_next);
      trace_end("exchange", comm_);
      exchange_landed();
      ++st.exchanges;
    }
    steps_done_ += k;
    k = k_next;
    check = check_next;
  }
  H2D_HIP_CHECK(hipEventRecord(ev_ready_, comm_));
  H2D_HIP_CHECK(hipStreamWaitEvent(compute_, ev_ready_, 0));
}

void Engine::run_serial(RunStats& st, int64_t target) {
  while (steps_done_ < target) {
    bool check = false;
    const int k = next_chunk(steps_done_, target, &check);
    if (!has_exchange_ && !check && !opt_.naive) {
      // a run of equal plain chunks: ONE persistent launch
      const int J = plain_run(steps_done_, target, k);
      if (J >= 2 && pplan(k) != nullptr) {
        flush_pending_decision();  // (a persistent launch carries no deciding block)
        trace_begin("step", compute_);
        launch_pstream_chunks(k, J);
        trace_end("step", compute_);
        if (J & 1) tiles_[0].cur = 1 - tiles_[0].cur;
        st.chunks += J;
        steps_done_ += (int64_t)J * k;
        poll_abort();
        continue;
      }
    }
    if (has_exchange_) {
      // serial: nothing overlaps the exchange, so it runs in order on the compute stream (no
      // cross-stream event pair per chunk: the GPU test suite saw this pipeline compute a wrong
      // tile now and then in a process holding many streams, never with one stream)
      trace_begin("exchange", compute_);
      do_exchange_async(k, compute_);
      trace_end("exchange", compute_);
      ++st.exchanges;
    }
    trace_begin("step", compute_);
    advance(k, check);
    trace_end("step", compute_);
    ++st.chunks;
    if (check) {
      if (fused_) {
        if (check_point(steps_done_, k)) break;  // converged (seen by the host): stop enqueueing
      } else {
        st.residual = finish_residual();
        if (st.residual < opt_.sensitivity) {
          rollback();
          st.converged = true;
          break;
        }
      }
    }
    steps_done_ += k;
  }
}

// ---- persistent pipelined stencil ----------------------------------------------------------

int Engine::plain_run(int64_t done, int64_t target, int k) const {
  // consecutive chunks of depth k without a check, starting at `done` (capped: a launch of at
  // most 256 chunks, so the host still polls for device-side failures now and then)
  int J = 0;
  while (J < 256 && done < target) {
    bool check = false;
    const int kk = next_chunk(done, target, &check);
    if (kk != k || check) break;
    done += kk;
    ++J;
  }
  return J;
}

const Engine::PPlan* Engine::pplan(int K) {
  auto it = pplans_.find(K);
  if (it != pplans_.end()) return it->second.n > 0 ? &it->second : nullptr;
  PPlan P;
  const Tile& T = tiles_[0];
  const TileGeom& g = T.g;
  // auto: only where one launch per chunk is measurably the bottleneck — the direct pipeline's
  // short per-rank strips (tools/pstream_check.py on MI355X, us/step over 840 steps, per-chunk vs
  // persistent: 512x4096 K=6 2.475 vs 2.112, 1024x4096 K=7 3.176 vs 2.873, 2048x4096 4.706 vs
  // 4.800, 4096^2 7.743 vs 8.816; a lone tile: 512x4096 2.162 vs 2.101, 1024 3.173 vs 3.328,
  // 4096^2 7.744 vs 9.207 — profiles/pstream_r3.txt).  Timeline runs stamp per-chunk launches.
  const bool want = opt_.persistent > 0 ||
                    (opt_.persistent < 0 && direct_ && has_exchange_ && g.xcell <= 1536 && opt_.timeline == 0 && K >= 2);
  // (every wave must be resident: not with CUs reserved for the comm stream)
  const bool ok_path = on_gpu() && !opt_.naive && !tiled_ && want && tiles_.size() == 1 && K <= kMaxPK && K <= G_ &&
                       stream_k_supported(K) && comm_cus_ == 0;
  bool halo_n = false, halo_s = false, ok = ok_path;
  if (ok && has_exchange_) {
    // only the direct pipeline of 1-D row strips (no west / east / corner neighbours)
    ok = direct_;
    for (int d = kW; d < kNumDirs && ok; ++d) ok = dec_.neighbor(T.rank, d) < 0;
    halo_n = dec_.neighbor(T.rank, kN) >= 0;
    halo_s = dec_.neighbor(T.rank, kS) >= 0;
  }
  // write-through stores and 32-bit row offsets (as launch_chunk_tile's a.wt)
  if (ok) ok = (opt_.wt_store < 0 ? 1 : opt_.wt_store) != 0 &&
               (double)(g.xcell + 2 * g.G) * (double)g.pitch * sizeof(float) < 2147483648.0 - 1048576.0;
  if (ok) {
    // strip width: 128 columns for short tiles (twice the unit height at the same wave count:
    // the K-cone (K-1)/h halves), else 256 (profiles/pstream_r3.txt, us/step 256 vs 128 columns,
    // K=8: 512x4096 2.077 vs 1.908; 1024 rows 2.867 vs 3.031; 2048 rows 4.789 vs 5.157)
    P.cpl = opt_.pstream_cols == 256 ? 4 : opt_.pstream_cols == 128 ? 2 : (g.xcell <= 768 ? 2 : 4);
    int64_t cap = (int64_t)device_cus_ * 4;  // one wave per SIMD, every wave resident
    if (opt_.pstream_waves > 0) cap = std::min<int64_t>(cap, opt_.pstream_waves);
    const int bpc = pstream_blocks_per_cu(K, opt_.precision, P.cpl);
    P.host = plan_pstream(g, K, opt_.boundary == kFixed, opt_.periodic_x, opt_.periodic_y,
                          opt_.row_edge_weight > 0 ? opt_.row_edge_weight : opt_.edge_weight, cap, halo_n, halo_s,
                          std::max(K, G_), P.cpl, opt_.pstream_halo_weight);
    P.n = (int)P.host.size();
    if (P.n == 0 || bpc < 1 || (P.n + 3) / 4 > (int64_t)device_cus_ * bpc) P.n = 0;
    // N / S halo units: each adds 1 to the neighbour's flag per chunk (the neighbours learn the
    // count from the IPC handle, Engine::ipc_handle)
    for (const PUnit& u : P.host)
      if (u.u.flags & kUnitNS) ++P.pushes[(u.u.flags & kUnitReverse) ? 1 : 0];
  }
  if (P.n > 0) {
    P.d_units = dmalloc<PUnit>((size_t)P.n);
    h2d(P.d_units, P.host.data(), (size_t)P.n * sizeof(PUnit));
    P.d_prog = dmalloc<unsigned>((size_t)P.n * 32);
    dzero(P.d_prog, (size_t)P.n * 32 * sizeof(unsigned));
  }
  auto& ref = pplans_.emplace(K, std::move(P)).first->second;
  return ref.n > 0 ? &ref : nullptr;
}

void Engine::launch_pstream_chunks(int K, int J) {
  PPlan& P = pplans_.at(K);
  Tile& T = tiles_[0];
  const TileGeom& g = T.g;
  PStreamArgs a;
  zero_args(a);
  a.rel = 2;
  a.acq = 1;
  PStreamDyn dy;
  a.units = P.d_units;
  a.nunits = P.n;
  dy.nunits = P.n;
  dy.nchunks = J;
  dy.cbase = P.cdone;
  a.buf[0] = T.buf[0];
  a.buf[1] = T.buf[1];
  dy.cur0 = T.cur;
  a.prog = P.d_prog;
  a.pitch = g.pitch;
  a.G = g.G;
  a.PL = g.PL;
  a.xcell = g.xcell;
  a.ycell = g.ycell;
  a.gx0 = g.gx0;
  a.gy0 = g.gy0;
  a.NX = g.NX;
  a.NY = g.NY;
  a.cx = opt_.cx;
  a.cy = opt_.cy;
  a.fixed = opt_.boundary == kFixed;
  a.per_x = opt_.periodic_x;
  a.per_y = opt_.periodic_y;
  a.dbg = opt_.debug_kernel;
  a.dummy = d_dummy_;
  a.halo_polls = std::max<long long>(1000, (long long)(opt_.halo_timeout_s * 1e6));
  a.timed_out = d_sig_timeout_;
  a.timed_out_host = h_timeout_dev_;
  a.wait_acc = d_wait_acc_;
  a.phase = d_phase_;
  if (fused_) a.stop = d_stop_;  // no-op after a converged check (the runs between checks)
  if (direct_) {
    const int64_t rowb = g.pitch * (int64_t)sizeof(float);
    const IpcLayout& me = ipc_lays_[T.rank];
    const int pn = dec_.neighbor(T.rank, kN), ps = dec_.neighbor(T.rank, kS);
    if (pn >= 0) {
      const IpcLayout& nl = ipc_lays_[pn];
      a.wait[0] = reinterpret_cast<const unsigned long long*>(ipc_block_ + me.flag[kN]);
      dy.need0[0] = ipc_need_[kN];
      a.need_inc[0] = (unsigned long long)pst_counts_[pn].at((size_t)K * 2 + 1);  // N's south pushes
      a.sig[0] = reinterpret_cast<unsigned long long*>(ipc_blocks_[pn] + nl.flag[kS]);
      for (int p = 0; p < 2; ++p) {
        a.hsrc[0][p] = reinterpret_cast<const float*>(ipc_block_ + me.recv_n[p]);
        a.push[0][p] = reinterpret_cast<float*>(ipc_blocks_[pn] + nl.recv_s[p]);
      }
    }
    if (ps >= 0) {
      const IpcLayout& sl = ipc_lays_[ps];
      a.wait[1] = reinterpret_cast<const unsigned long long*>(ipc_block_ + me.flag[kS]);
      dy.need0[1] = ipc_need_[kS];
      a.need_inc[1] = (unsigned long long)pst_counts_[ps].at((size_t)K * 2 + 0);  // S's north pushes
      a.sig[1] = reinterpret_cast<unsigned long long*>(ipc_blocks_[ps] + sl.flag[kN]);
      for (int p = 0; p < 2; ++p) {
        a.hsrc[1][p] = reinterpret_cast<const float*>(ipc_block_ + me.recv_s[p] - (g.G + g.xcell) * rowb);
        a.push[1][p] = reinterpret_cast<float*>(ipc_blocks_[ps] + sl.recv_n[p] - (g.xcell - g.G) * rowb);
      }
    }
    dy.ipar0 = (int)(ipc_chunk_ & 1);
    a.sig_rows = G_;
    for (int d = 0; d < 2; ++d) {  // chunk order of my halo units' signals (PStreamArgs::lsig)
      // (debug_kernel bit 4: without the chunk order — diagnostics only, races between processes)
      a.lsig[d] = (opt_.debug_kernel & 4) ? nullptr : reinterpret_cast<unsigned long long*>(ipc_block_ + me.lsig[d]);
      dy.lbase[d] = ipc_lsig_[d];
      a.lper[d] = P.pushes[d];
      ipc_lsig_[d] += (unsigned long long)J * (unsigned long long)P.pushes[d];
    }
    a.rel = opt_.direct_release < 0 ? 2 : opt_.direct_release;
    a.acq = opt_.direct_acquire < 0 ? 1 : opt_.direct_acquire;
  }
  const PStreamArgs* blk = args_.get(a, compute_);  // the plan-constant part: device-resident
  dy.btag = a.head.btag;
  launch_pstream(blk, dy, K, opt_.precision, P.cpl, opt_.pstream_pingpong > 0, compute_);
  P.cdone += (unsigned)J;
  ++pstream_launches_;
  progress_tick(compute_);
}

bool Engine::pst_everywhere(int K) const {
  // single process without exchange: only this engine's plan matters
  if (!direct_) return true;
  if (pst_counts_.empty()) return false;
  for (const auto& v : pst_counts_)
    if ((size_t)K * 2 >= v.size() || v[(size_t)K * 2] < 0) return false;
  return true;
}

std::vector<PUnit> Engine::pstream_units(int K) {
  const PPlan* P = pplan(K);
  return P ? P->host : std::vector<PUnit>();
}

// ---- device-side convergence (fused check) -----------------------------------------------

DecideArgs Engine::decide_args(int t, bool decide) const {
  DecideArgs d;
  d.ticket = d_ticket_ + t;
  d.total = decide ? d_resid_ + tiles_.size() : d_resid_ + t;
  d.stop = d_stop_;
  d.host = decide ? h_conv_dev_ : nullptr;
  d.sens = opt_.sensitivity;
  d.seq = chunk_seq_ + 1;  // the check this launch belongs to (check_point numbers it next)
  return d;
}

void Engine::device_decide(unsigned long long seq) {
  // Σ over this process's tiles, then over ranks, then the decision — all enqueued on the
  // compute stream; nothing waits for the host.  (A lone single-process tile decides inside
  // its residual launch: nothing to enqueue.)
  const int nt = (int)tiles_.size();
  double* total = d_resid_ + nt;
  DecideArgs d = decide_args(0, true);
  d.seq = seq;
  if (direct_) {
    ++ipc_resid_epoch_;
    const IpcLayout& me = ipc_lays_[tiles_[0].rank];
    const long long polls = std::max<long long>(1000, (long long)(opt_.halo_timeout_s * 1e6));
    const unsigned long long target = (unsigned long long)ipc_blocks_.size() * ipc_resid_epoch_;
    if (last_parts_ != nullptr) {  // the check launch's partials: summed by the all-reduce itself
      launch_ipc_allreduce_parts(last_parts_, last_nparts_, d_resid_, total, d_ipc_blocks_, tiles_[0].rank,
                                 (int)ipc_blocks_.size(), (int)(ipc_resid_epoch_ & 1), target, me.resid_count,
                                 me.resid_slots, kIpcMaxRanks, polls, d_sig_timeout_, h_timeout_dev_, d_stop_, d,
                                 compute_);
      last_parts_ = nullptr;
    } else {
      launch_ipc_allreduce(d_resid_, total, d_ipc_blocks_, tiles_[0].rank, (int)ipc_blocks_.size(),
                           (int)(ipc_resid_epoch_ & 1), target, me.resid_count, me.resid_slots, kIpcMaxRanks, polls,
                           d_sig_timeout_, h_timeout_dev_, d_stop_, &d, compute_);
    }
  } else if (rccl_comm_) {
    H2D_NCCL_CHECK(ncclAllReduce(d_resid_, total, 1, ncclDouble, ncclSum, (ncclComm_t)rccl_comm_, compute_));
    launch_decide(total, d, compute_);
  } else if (last_parts_ != nullptr) {  // a lone tile: its units' partials straight to the decision
    if (tiles_[0].spare != nullptr && !tiled_) {
      // ... made by the next launch's extra block (or flush_pending_decision at the run's end)
      flush_pending_decision();  // (an older one never consumed: decide it first)
      pend_parts_ = last_parts_;
      pend_nparts_ = last_nparts_;
      pend_dec_ = d;
    } else {
      launch_reduce_decide(last_parts_, last_nparts_, d, compute_);
    }
    last_parts_ = nullptr;
  } else {
    launch_reduce_decide(d_resid_, nt, d, compute_);
  }
}

void Engine::flush_pending_decision() {
  if (pend_parts_ == nullptr) return;
  launch_reduce_decide(pend_parts_, pend_nparts_, pend_dec_, compute_);
  pend_parts_ = nullptr;
}

bool Engine::check_point(int64_t steps_before, int k, int lvl) {
  // The chunk just enqueued ended on a check step: record it, enqueue the decision, and tell
  // the caller whether the host already sees a converged check (then it stops enqueueing;
  // launches queued after the converged one are no-ops on the device).
  const unsigned long long seq = ++chunk_seq_;
  // cur has flipped past the chunk; lvl: the check's level in the chunk (k: its last)
  checks_.push_back(CheckRec{seq, steps_before, k, 1 - tiles_[0].cur, tiles_[0].buf[1 - tiles_[0].cur],
                            lvl > 0 ? lvl : k});
  if (!decided_in_launch_) device_decide(seq);
  decided_in_launch_ = false;
  if (rccl_comm_) {
    // Ranks must enqueue the same collectives: look only at fixed points of the check sequence,
    // after the decision of that check has completed (the same answer on every rank).
    if (++checks_since_sync_ < 16) return false;
    checks_since_sync_ = 0;
    H2D_HIP_CHECK(hipEventRecord(ev_check_, compute_));
    wait_event(ev_check_);
  }
  return __atomic_load_n(&h_conv_->stop_seq, __ATOMIC_ACQUIRE) != 0ull;
}

bool Engine::finalize_convergence(RunStats& st) {
  bool launched = false;
  const unsigned long long seq = __atomic_load_n(&h_conv_->stop_seq, __ATOMIC_ACQUIRE);
  if (seq != 0ull) {
    auto it = std::find_if(checks_.begin(), checks_.end(), [&](const CheckRec& r) { return r.seq == seq; });
    if (it == checks_.end()) throw std::logic_error("converged check not found");
    // the result is the state one step before the converged check (B-5): the level K-1 rows
    // the check launch kept
    steps_done_ = it->steps_before + it->lvl - 1;
    st.converged = true;
    st.residual = h_conv_->residual;
    H2D_HIP_CHECK(hipMemsetAsync(d_stop_, 0, sizeof(unsigned long long), compute_));
    if (recompute_rollback()) {
      // the launches after the converged check were no-ops (or, tiled, wrote the spare buffer),
      // so the check chunk's input buffer still holds the state at steps_before: advance it
      // lvl-1 steps (plain launches, no check)
      Tile& T0 = tiles_[0];
      if (T0.buf[it->src] != it->src_ptr) {  // moved by the tiled path's rotation: bring it back
        float** at = T0.buf[1 - it->src] == it->src_ptr ? &T0.buf[1 - it->src] : &T0.spare;
        if (*at != it->src_ptr) throw std::logic_error("converged check's input buffer not found");
        std::swap(*at, T0.buf[it->src]);
      }
      T0.cur = it->src;
      launched = it->lvl > 1;
      for (int left = it->lvl - 1; left > 0;) {
        int kk = std::min(left, G_);
        while (kk > 1 && !stream_k_supported(kk)) --kk;
        advance(kk, false);
        left -= kk;
      }
    } else {
      for (Tile& t : tiles_) std::swap(t.keep, t.buf[t.cur]);
      // the cached exchange descriptors hold the old buffer addresses: rebuild them on next use
      H2D_HIP_CHECK(hipStreamSynchronize(compute_));
      H2D_HIP_CHECK(hipStreamSynchronize(comm_));
      for (auto* m : {&local_descs_, &pack_descs_, &unpack_descs_}) {
        for (auto& kv : *m) hipFree(kv.second.d);
        m->clear();
      }
    }
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
    __atomic_store_n(&h_conv_->stop_seq, 0ull, __ATOMIC_RELEASE);
    if (direct_) ipc_primed_ = false;  // the neighbours hold halos of later launches
  } else if (!checks_.empty()) {
    st.residual = h_conv_->last;
  }
  checks_.clear();
  checks_since_sync_ = 0;
  return launched;
}

void Engine::end_of_run_wait(RunStats& st, std::chrono::steady_clock::time_point w0) {
  // Everything of the run is on compute_ (the pipelines join the other streams into it).
  const int m = opt_.sync_mode;
  if (m == 0 || m == 3) H2D_HIP_CHECK(hipEventRecord(ev_t1_, compute_));
  if (m == 1) H2D_HIP_CHECK(hipEventRecord(ev_done_, compute_));
  if (rccl_comm_ || m == 0) {
    wait_event(m == 1 ? ev_done_ : m == 2 ? nullptr : ev_t1_);
  } else if (m == 2) {
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
  } else {
    hipEvent_t ev = m == 1 ? ev_done_ : ev_t1_;
    for (;;) {  // spin: no interrupt / yield wake-up latency on the critical path of a short run
      const hipError_t e = hipEventQuery(ev);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) H2D_HIP_CHECK(e);
    }
  }
  st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
  if (m == 0 || m == 3) {
    float ms = 0.0f;
    H2D_HIP_CHECK(hipEventElapsedTime(&ms, ev_t0_, ev_t1_));
    st.device_ms = ms;
  } else {
    st.device_ms = st.wall_ms;
  }
}

int64_t Engine::send_count(int t, int k) const {
  check_tile(t);
  return make_plan(dec_, tiles_[t].rank, tiles_[t].g, k).send_total;
}

int64_t Engine::recv_count(int t, int k) const {
  check_tile(t);
  return make_plan(dec_, tiles_[t].rank, tiles_[t].g, k).recv_total;
}

std::vector<int64_t> Engine::plan_info(int t, int k) const {
  check_tile(t);
  ExchangePlan p = make_plan(dec_, tiles_[t].rank, tiles_[t].g, k);
  std::vector<int64_t> v;
  for (int d = 0; d < kNumDirs; ++d) {
    v.push_back(p.peer[d]);
    v.push_back(p.send_off[d]);
    v.push_back(p.send_rect[d].count());
    v.push_back(p.recv_off[d]);
    v.push_back(p.recv_rect[d].count());
  }
  return v;
}

void Engine::pack(int t, int k, uintptr_t sendbuf) {
  check_tile(t);
  Tile& T = tiles_[t];
  ExchangePlan p = make_plan(dec_, T.rank, T.g, k);
  std::vector<CopyDesc> v;
  plan_pack_descs(p, T.g, T.buf[T.cur], reinterpret_cast<float*>(sendbuf), v);
  if (on_gpu()) {
    if (v.empty()) return;
    const DescList& D = ext_descs(v);
    launch_copy_rects(D.d, D.n, D.maxe, compute_, D.tag, nullptr, d_sig_timeout_, h_timeout_dev_);
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
  } else {
    cpu_copy_rects(v);
  }
}

void Engine::unpack(int t, int k, uintptr_t recvbuf) {
  check_tile(t);
  Tile& T = tiles_[t];
  ExchangePlan p = make_plan(dec_, T.rank, T.g, k);
  std::vector<CopyDesc> v;
  plan_unpack_descs(p, T.g, T.buf[T.cur], reinterpret_cast<const float*>(recvbuf), v);
  if (on_gpu()) {
    if (v.empty()) return;
    const DescList& D = ext_descs(v);
    launch_copy_rects(D.d, D.n, D.maxe, compute_, D.tag, nullptr, d_sig_timeout_, h_timeout_dev_);
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
  } else {
    cpu_copy_rects(v);
  }
}

void Engine::dzero(void* p, size_t bytes) const {
  // zeroing ordered on the compute stream (a hipMemset may complete after a kernel of the
  // non-blocking compute stream has already read the old bytes: see Engine::h2d)
  H2D_HIP_CHECK(hipMemsetAsync(p, 0, bytes, compute_));
}

void Engine::h2d(void* dst, const void* src, size_t bytes) const {
  // Host -> device copy of a plan (unit lists, copy descriptors, IPC pointers): ordered on the
  // compute stream and complete on return.  A blocking hipMemcpy from pageable memory may return
  // before its DMA has landed, and the compute stream does not wait for the null stream
  // (hipStreamNonBlocking): a kernel enqueued next could read the previous bytes of a reused
  // allocation — seen in the GPU suite as whole unit bands computed wrong, in processes that had
  // freed many engines.
  if (bytes == 0) return;
  H2D_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, compute_));
  H2D_HIP_CHECK(hipStreamSynchronize(compute_));
}

std::vector<float> Engine::download(int t) const {
  check_tile(t);
  const Tile& T = tiles_[t];
  std::vector<float> out((size_t)(T.g.xcell * T.g.ycell));
  if (on_gpu()) {
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
    H2D_HIP_CHECK(hipMemcpy2D(out.data(), T.g.ycell * sizeof(float), T.buf[T.cur] + T.g.idx(0, 0),
                              T.g.pitch * sizeof(float), T.g.ycell * sizeof(float), T.g.xcell, hipMemcpyDeviceToHost));
  } else {
    for (int64_t i = 0; i < T.g.xcell; ++i)
      std::memcpy(&out[(size_t)(i * T.g.ycell)], T.buf[T.cur] + T.g.idx(i, 0), T.g.ycell * sizeof(float));
  }
  return out;
}

std::vector<float> Engine::storage(int t, int b) const {
  check_tile(t);
  if (b != 0 && b != 1) throw std::invalid_argument("storage: buffer 0 or 1");
  const Tile& T = tiles_[t];
  std::vector<float> out((size_t)T.g.elems());
  if (on_gpu()) {
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
    H2D_HIP_CHECK(hipMemcpy(out.data(), T.buf[b], out.size() * sizeof(float), hipMemcpyDeviceToHost));
  } else {
    std::copy(T.buf[b], T.buf[b] + out.size(), out.begin());
  }
  return out;
}

void Engine::upload(int t, const float* owned) {
  check_tile(t);
  Tile& T = tiles_[t];
  if (direct_) ipc_primed_ = false;  // the neighbours must receive the new boundary rows
  if (on_gpu()) {
    // ordered on the compute stream and complete on return (see Engine::h2d)
    H2D_HIP_CHECK(hipMemcpy2DAsync(T.buf[T.cur] + T.g.idx(0, 0), T.g.pitch * sizeof(float), owned,
                                   T.g.ycell * sizeof(float), T.g.ycell * sizeof(float), T.g.xcell,
                                   hipMemcpyHostToDevice, compute_));
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
  } else {
    for (int64_t i = 0; i < T.g.xcell; ++i)
      std::memcpy(T.buf[T.cur] + T.g.idx(i, 0), owned + i * T.g.ycell, T.g.ycell * sizeof(float));
  }
}

void Engine::synchronize() const {
  if (on_gpu()) {
    H2D_HIP_CHECK(hipStreamSynchronize(comm_));
    H2D_HIP_CHECK(hipStreamSynchronize(compute_));
  }
}

Engine::HaloWait Engine::halo_wait() const {
  HaloWait h;
  if (!on_gpu()) return h;
  synchronize();
  unsigned long long v[3] = {0, 0, 0};
  H2D_HIP_CHECK(hipMemcpy(v, d_wait_acc_, sizeof(v), hipMemcpyDeviceToHost));
  h.total_us = (double)v[0] * 0.01;  // s_memrealtime: 100 MHz
  h.waits = (int64_t)v[1];
  h.max_us = (double)v[2] * 0.01;
  return h;
}

void Engine::reset_halo_wait() {
  if (!on_gpu()) return;
  synchronize();
  dzero(d_wait_acc_, 4 * sizeof(unsigned long long));
  if (d_phase_) dzero(d_phase_, kPhases * sizeof(unsigned long long));
}

std::vector<double> Engine::pstream_phases() const {
  std::vector<double> out(kPhases, 0.0);
  if (!on_gpu() || !d_phase_) return out;
  synchronize();
  unsigned long long v[kPhases];
  H2D_HIP_CHECK(hipMemcpy(v, d_phase_, sizeof(v), hipMemcpyDeviceToHost));
  out[0] = (double)v[0];
  for (int i = 1; i < kPhases; ++i) out[i] = (double)v[i] * 0.01;  // s_memrealtime: 100 MHz
  return out;
}

std::vector<Unit> Engine::unit_list(int t, int K, int which) {
  check_tile(t);
  if (!on_gpu()) throw std::runtime_error("unit_list: GPU engines only");
  if (!stream_k_supported(K) || K > G_) throw std::invalid_argument("unit_list: unsupported depth");
  const UnitLists& L = units(t, K);
  std::vector<Unit> v((size_t)L.n_all);
  if (!v.empty())
    H2D_HIP_CHECK(hipMemcpy(v.data(), which == 3 ? L.d_bfirst : L.d_all, v.size() * sizeof(Unit), hipMemcpyDeviceToHost));
  return v;
}

std::vector<Engine::LaunchTimeline> Engine::timeline() const {
  std::vector<LaunchTimeline> out;
  if (!on_gpu() || d_stamps_ == nullptr) return out;
  synchronize();
  for (size_t i = 0; i < tl_recs_.size(); ++i) {
    LaunchTimeline t;
    t.K = tl_recs_[i].first;
    t.units = tl_recs_[i].second;
    t.stamps.resize((size_t)t.units * 4);
    H2D_HIP_CHECK(hipMemcpy(t.stamps.data(), d_stamps_ + i * (size_t)kTimelineUnits * 4,
                            t.stamps.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    out.push_back(std::move(t));
  }
  return out;
}

std::string Engine::rccl_unique_id() {
  ncclUniqueId id;
  H2D_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

void Engine::init_rccl(const std::string& id, int nranks, int rank) {
  if (!on_gpu()) throw std::runtime_error("init_rccl needs a GPU engine");
  if (id.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("bad RCCL unique id");
  if (nranks != dec_.nranks()) throw std::invalid_argument("RCCL world size must equal gridx*gridy");
  if (tiles_.size() != 1 || tiles_[0].rank != rank) throw std::invalid_argument("RCCL rank must own exactly its tile");
  ncclUniqueId uid;
  std::memcpy(&uid, id.data(), sizeof(uid));
  H2D_HIP_CHECK(hipSetDevice(opt_.device));
  ncclComm_t comm;
  H2D_NCCL_CHECK(ncclCommInitRank(&comm, nranks, uid, rank));
  rccl_comm_ = comm;
  rccl_rank_ = rank;
  rccl_nranks_ = nranks;
  transport_ = kTransportRccl;
}

// ---- IPC direct transport ----------------------------------------------------------------

Engine::IpcLayout Engine::ipc_layout_of(int rank) const {
  // One uncached (MTYPE UC) device block per rank: every access goes to memory, so stores a
  // peer GPU makes over xGMI are seen by plain loads here without any cache maintenance, and
  // polls of the flags see the peers' atomics.  Flags and counters on lines of their own.
  // Computed from the decomposition alone, so every rank knows every rank's layout.
  const TileGeom g = dec_.tile(rank, G_);
  const size_t rb = (size_t)g.G * (size_t)g.pitch * sizeof(float);  // G full storage rows
  const size_t rs = (rb + 4095) & ~size_t(4095);
  IpcLayout L;
  for (int d = 0; d < kNumDirs; ++d) L.flag[d] = 128 * (size_t)d;
  size_t off = 4096;  // flags / residual slots live in the first 4 KiB
  for (int p = 0; p < 2; ++p) {
    L.recv_n[p] = off;
    off += rs;
  }
  for (int p = 0; p < 2; ++p) {
    L.recv_s[p] = off;
    off += rs;
  }
  L.pitch = g.pitch;
  bool side = false;
  for (int d = kW; d < kNumDirs; ++d) side = side || dec_.neighbor(rank, d) >= 0;
  if (side) {
    // W / E ghost-column groups (kGhostGroup columns per side and parity) in rows [-G, xcell+G),
    // with the tile's pitch (the streaming kernel's ghost lanes read them like tile rows)
    if (g.pitch < 4 * IpcLayout::kGroupStride) throw std::logic_error("IPC layout: pitch too small for the groups");
    L.xbuf = off;
    off += (((size_t)(g.xcell + 2 * g.G) * (size_t)g.pitch * sizeof(float)) + 4095) & ~size_t(4095);
  }
  L.bytes = off;
  static_assert(1152 + 2 * kIpcMaxRanks * sizeof(double) <= 2304, "IPC residual slots overflow into the signal counters");
  return L;
}

float* Engine::side_push_base(int d, int pr, int q) const {
  // My cell (i, j) that lies in neighbour pr's halo (direction d) is stored at
  // base + i * pitch(pr) + j: every offset of its ghost-column group folded in.
  const TileGeom& g = tiles_.at(0).g;
  const TileGeom n = dec_.tile(pr, G_);
  const IpcLayout& L = ipc_lays_[pr];
  const int64_t P = L.pitch;
  const bool west_of_me = d == kW || d == kNW || d == kSW;  // my first columns -> its E group
  int64_t row0 = g.G;                                       // my row i -> its row i (W, E)
  if (d == kNW || d == kNE) row0 = g.G + n.xcell;           // my row i < G -> its row xcell_n + i
  if (d == kSW || d == kSE) row0 = g.G - g.xcell;           // my row i >= xcell - G -> its row i - xcell
  const int64_t col0 = west_of_me ? 0 : kGhostGroup - g.ycell;  // my column j -> its group column
  const int64_t off = (int64_t)L.group(west_of_me ? 1 : 0, q) + (row0 * P + col0) * (int64_t)sizeof(float);
  return reinterpret_cast<float*>(ipc_blocks_[pr] + off);
}

std::string Engine::ipc_handle() {
  if (transport_ != kTransportIpc) throw std::logic_error("ipc_handle: engine transport is not IPC");
  if (!ipc_block_) {
    ipc_lays_.assign(dec_.nranks(), IpcLayout());
    for (int r = 0; r < dec_.nranks(); ++r) ipc_lays_[r] = ipc_layout_of(r);
    H2D_HIP_CHECK(hipSetDevice(opt_.device));
    const IpcLayout& L = ipc_lays_[tiles_.at(0).rank];
    H2D_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&ipc_block_), L.bytes, hipDeviceMallocUncached));
    H2D_HIP_CHECK(hipMemset(ipc_block_, 0, L.bytes));
    H2D_HIP_CHECK(hipDeviceSynchronize());
  }
  hipIpcMemHandle_t h;
  H2D_HIP_CHECK(hipIpcGetMemHandle(&h, ipc_block_));
  // the handle, then this rank's push counts per (K, direction): what its neighbours' halo
  // waits count per chunk
  std::vector<int32_t> counts((size_t)(G_ + 1) * kNumDirs, 0);
  for (int K = 1; K <= G_; ++K)
    if (stream_k_supported(K)) {
      const UnitLists& U = units(0, K);
      for (int d = 0; d < kNumDirs; ++d) counts[(size_t)K * kNumDirs + d] = U.pushes[d];
    }
  // ... and its persistent plan's N / S halo pushes per chunk at each depth (-1: no plan)
  std::vector<int32_t> pcounts((size_t)(G_ + 1) * 2, -1);
  for (int K = 1; K <= G_; ++K) {
    const PPlan* P = pplan(K);
    if (P != nullptr) {
      pcounts[(size_t)K * 2] = P->pushes[0];
      pcounts[(size_t)K * 2 + 1] = P->pushes[1];
    }
  }
  std::string blob(reinterpret_cast<const char*>(&h), sizeof(h));
  blob.append(reinterpret_cast<const char*>(counts.data()), counts.size() * sizeof(int32_t));
  blob.append(reinterpret_cast<const char*>(pcounts.data()), pcounts.size() * sizeof(int32_t));
  return blob;
}

void Engine::ipc_open(const std::vector<std::string>& handles) {
  if (!ipc_block_) throw std::logic_error("ipc_open: call ipc_handle() first");
  const int me = tiles_.at(0).rank, nr = dec_.nranks();
  if ((int)handles.size() != nr) throw std::invalid_argument("ipc_open: one handle per rank expected");
  if (nr > kIpcMaxRanks) throw std::invalid_argument("ipc_open: too many ranks");
  const size_t nc = (size_t)(G_ + 1) * kNumDirs, npc = (size_t)(G_ + 1) * 2;
  const size_t want = sizeof(hipIpcMemHandle_t) + (nc + npc) * sizeof(int32_t);
  H2D_HIP_CHECK(hipSetDevice(opt_.device));
  ipc_blocks_.assign(nr, nullptr);
  ipc_opened_.assign(nr, false);
  ipc_counts_.assign(nr, std::vector<int32_t>());
  pst_counts_.assign(nr, std::vector<int32_t>());
  for (int r = 0; r < nr; ++r) {
    if (handles[r].size() != want) throw std::invalid_argument("ipc_open: bad handle (another build or halo depth?)");
    ipc_counts_[r].resize(nc);
    std::memcpy(ipc_counts_[r].data(), handles[r].data() + sizeof(hipIpcMemHandle_t), nc * sizeof(int32_t));
    pst_counts_[r].resize(npc);
    std::memcpy(pst_counts_[r].data(), handles[r].data() + sizeof(hipIpcMemHandle_t) + nc * sizeof(int32_t),
                npc * sizeof(int32_t));
    if (r == me) {
      ipc_blocks_[r] = ipc_block_;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    H2D_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    ipc_blocks_[r] = static_cast<char*>(p);
    ipc_opened_[r] = true;
    // the mapping must work before any kernel dereferences it (a fault here is an error, not a
    // GPU memory fault inside the stencil)
    unsigned long long probe = 0;
    H2D_HIP_CHECK(hipMemcpy(&probe, ipc_blocks_[r], sizeof(probe), hipMemcpyDeviceToHost));
  }
  d_ipc_blocks_ = dmalloc<char*>((size_t)nr);
  h2d(d_ipc_blocks_, ipc_blocks_.data(), nr * sizeof(char*));
  ipc_primed_ = false;
}

void Engine::ipc_prime() {
  // Collective (the caller brackets it with barriers: no kernel of any rank is running):
  // zero my flags and counters, and write my boundary rows / columns / corners into the
  // neighbours' receive buffers of parity 0 (what their chunk 0 reads) — the initial halo.
  if (ipc_blocks_.empty()) throw std::logic_error("ipc_prime: call ipc_open() first");
  H2D_HIP_CHECK(hipSetDevice(opt_.device));
  H2D_HIP_CHECK(hipDeviceSynchronize());
  H2D_HIP_CHECK(hipMemset(ipc_block_, 0, 4096));
  const Tile& T = tiles_.at(0);
  const TileGeom& g = T.g;
  const size_t rb = (size_t)g.G * (size_t)g.pitch * sizeof(float);
  const int pn = dec_.neighbor(T.rank, kN), ps = dec_.neighbor(T.rank, kS);
  const char* cur = reinterpret_cast<const char*>(T.buf[T.cur]);
  const size_t row = (size_t)g.pitch * sizeof(float);
  if (pn >= 0)  // my rows [0, G) -> N's receive buffer for its south ghost rows
    H2D_HIP_CHECK(hipMemcpy(ipc_blocks_[pn] + ipc_lays_[pn].recv_s[0], cur + (size_t)g.G * row, rb,
                            hipMemcpyDeviceToDevice));
  if (ps >= 0)  // my rows [xcell - G, xcell) -> S's receive buffer for its north ghost rows
    H2D_HIP_CHECK(hipMemcpy(ipc_blocks_[ps] + ipc_lays_[ps].recv_n[0], cur + (size_t)g.xcell * row, rb,
                            hipMemcpyDeviceToDevice));
  for (int d = kW; d < kNumDirs; ++d) {
    const int pr = dec_.neighbor(T.rank, d);
    if (pr < 0) continue;
    // my cells of its halo: columns [0, G) or [ycell - G, ycell); rows all, [0, G) or [xcell - G, xcell)
    const bool west = d == kW || d == kNW || d == kSW;
    const int64_t c0 = west ? 0 : g.ycell - g.G;
    const int64_t r0 = (d == kSW || d == kSE) ? g.xcell - g.G : 0;
    const int64_t nrows = (d == kW || d == kE) ? g.xcell : g.G;
    float* dst = side_push_base(d, pr, 0) + r0 * ipc_lays_[pr].pitch + c0;
    H2D_HIP_CHECK(hipMemcpy2D(dst, (size_t)ipc_lays_[pr].pitch * sizeof(float), T.buf[T.cur] + g.idx(r0, c0), row,
                              (size_t)g.G * sizeof(float), (size_t)nrows, hipMemcpyDeviceToDevice));
  }
  H2D_HIP_CHECK(hipDeviceSynchronize());
  ipc_chunk_ = 0;
  for (auto& v : ipc_need_) v = 0;
  for (auto& v : ipc_lsig_) v = 0;
  ipc_resid_epoch_ = 0;
  ipc_primed_ = true;
}

double Engine::ipc_allreduce_residual() {
  // Device all-reduce of the scalar residual over the IPC blocks: every rank stores its local
  // sum into slot [parity][me] of every block and bumps each block's counter; each rank then
  // waits for all contributions and sums the slots in rank order (deterministic, identical on
  // every rank).  Parity-alternating slots: a rank reaching all-reduce e has seen everyone's
  // contribution to e-1, so nobody still reads the slots of e-2 it overwrites.
  ++ipc_resid_epoch_;
  const int nr = (int)ipc_blocks_.size();
  launch_ipc_allreduce(d_resid_, d_resid_ + tiles_.size(), d_ipc_blocks_, tiles_[0].rank, nr,
                       (int)(ipc_resid_epoch_ & 1), (unsigned long long)nr * ipc_resid_epoch_,
                       ipc_lays_[tiles_[0].rank].resid_count, ipc_lays_[tiles_[0].rank].resid_slots, kIpcMaxRanks,
                       std::max<long long>(1000, (long long)(opt_.halo_timeout_s * 1e6)), d_sig_timeout_,
                       h_timeout_dev_, nullptr, nullptr, compute_);
  H2D_HIP_CHECK(hipMemcpyAsync(h_resid_, d_resid_ + tiles_.size(), sizeof(double), hipMemcpyDeviceToHost, compute_));
  H2D_HIP_CHECK(hipStreamSynchronize(compute_));
  poll_abort();
  return h_resid_[0];
}

}  // namespace h2d
