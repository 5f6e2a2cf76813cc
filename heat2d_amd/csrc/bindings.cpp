// heat2d_amd — Python bindings (pybind11) of the native runtime: the engine, the CPU oracle,
// the decomposition/plan, I/O, device queries and raw-pointer kernel ops (for torch tensors).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime.h>

#include <functional>
#include <map>
#include <mutex>
#include <vector>

#include "cpu_reference.h"
#include "decomposition.h"
#include "engine.h"
#include "io.h"
#include "kernels.h"

namespace py = pybind11;
using namespace h2d;

namespace {

// Work-unit plans of the torch-tensor stencil op, cached per (device, geometry, K, H,
// precision, boundary): built once with the capacity-aware planner and kept in device
// memory, so a launch is asynchronous on the caller's stream (no allocation, no sync).
struct OpPlan {
  Unit* units = nullptr;
  int n = 0;
  float* dummy = nullptr;  // sink for non-output lanes (contents never read)
};

const OpPlan& op_plan(const TileGeom& g, int K, int H, int precision, bool fixed, bool per_x, bool per_y) {
  static std::mutex mu;
  static std::map<std::vector<int64_t>, OpPlan> cache;
  static std::map<int, float*> dummies;
  int dev = 0;
  H2D_HIP_CHECK(hipGetDevice(&dev));
  const std::vector<int64_t> key{dev,     g.NX,   g.NY, g.xcell, g.ycell,   g.gx0, g.gy0, g.G,  g.PL,
                                 g.pitch, K,      H,    precision, fixed, per_x, per_y};
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  if (cache.size() > 4096) throw std::runtime_error("op_stream: too many distinct tile geometries");
  const int64_t cap = stream_wave_capacity(K, precision, dev);
  std::vector<Unit> u = build_units(g, K, H, fixed, per_x, per_y, 1.2, cap);
  OpPlan P;
  P.n = (int)u.size();
  H2D_HIP_CHECK(hipMalloc(&P.units, std::max<size_t>(1, u.size()) * sizeof(Unit)));
  H2D_HIP_CHECK(hipMemcpy(P.units, u.data(), u.size() * sizeof(Unit), hipMemcpyHostToDevice));
  float*& d = dummies[dev];
  if (!d) H2D_HIP_CHECK(hipMalloc(&d, 4 * kWaveCols * sizeof(float)));
  P.dummy = d;
  return cache.emplace(key, P).first->second;
}


py::array_t<float> to_array(const std::vector<float>& v, int64_t rows, int64_t cols) {
  py::array_t<float> a({rows, cols});
  std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(float));
  return a;
}

const float* checked_grid(const py::array_t<float, py::array::c_style | py::array::forcecast>& a, int64_t rows,
                          int64_t cols) {
  if (a.ndim() != 2 || a.shape(0) != rows || a.shape(1) != cols)
    throw std::invalid_argument("expected a float32 array of shape (" + std::to_string(rows) + ", " +
                                std::to_string(cols) + ")");
  return a.data();
}

py::dict geom_dict(const TileGeom& g) {
  py::dict d;
  d["NX"] = g.NX;
  d["NY"] = g.NY;
  d["gx0"] = g.gx0;
  d["gy0"] = g.gy0;
  d["xcell"] = g.xcell;
  d["ycell"] = g.ycell;
  d["G"] = g.G;
  d["PL"] = g.PL;
  d["pitch"] = g.pitch;
  d["srows"] = g.srows;
  return d;
}

TileGeom geom_from(const py::dict& d) {
  TileGeom g;
  g.NX = d["NX"].cast<int64_t>();
  g.NY = d["NY"].cast<int64_t>();
  g.gx0 = d["gx0"].cast<int64_t>();
  g.gy0 = d["gy0"].cast<int64_t>();
  g.xcell = d["xcell"].cast<int64_t>();
  g.ycell = d["ycell"].cast<int64_t>();
  g.G = d["G"].cast<int64_t>();
  g.PL = d["PL"].cast<int64_t>();
  g.pitch = d["pitch"].cast<int64_t>();
  g.srows = d["srows"].cast<int64_t>();
  return g;
}

py::dict stats_dict(const RunStats& s) {
  py::dict d;
  d["steps_done"] = s.steps_done;
  d["converged"] = s.converged;
  d["residual"] = s.residual;
  d["device_ms"] = s.device_ms;
  d["wall_ms"] = s.wall_ms;
  d["chunks"] = s.chunks;
  d["exchanges"] = s.exchanges;
  d["path"] = s.path;
  d["phase_ms"] = s.phase_ms;
  d["phase_count"] = s.phase_count;
  return d;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

py::dict device_props(int dev) {
  hipDeviceProp_t p;
  H2D_HIP_CHECK(hipGetDeviceProperties(&p, dev));
  py::dict d;
  d["name"] = std::string(p.name);
  d["gcn_arch"] = std::string(p.gcnArchName);
  d["major"] = p.major;
  d["minor"] = p.minor;
  d["total_global_mem"] = (int64_t)p.totalGlobalMem;
  d["shared_mem_per_block"] = (int64_t)p.sharedMemPerBlock;
  d["total_const_mem"] = (int64_t)p.totalConstMem;
  d["regs_per_block"] = p.regsPerBlock;
  d["warp_size"] = p.warpSize;
  d["max_threads_per_block"] = p.maxThreadsPerBlock;
  d["max_threads_dim"] = std::vector<int>{p.maxThreadsDim[0], p.maxThreadsDim[1], p.maxThreadsDim[2]};
  d["max_grid_size"] = std::vector<int>{p.maxGridSize[0], p.maxGridSize[1], p.maxGridSize[2]};
  d["multiprocessor_count"] = p.multiProcessorCount;
  d["clock_rate_khz"] = p.clockRate;
  d["l2_cache_size"] = p.l2CacheSize;
  return d;
}

// EngineOptions fields settable by keyword from Python (Engine(nx, ny, **kw)).  One line per
// option; an unknown keyword is an error (no silently ignored typos).
using OptSetter = std::function<void(EngineOptions&, const py::handle&)>;
const std::map<std::string, OptSetter>& engine_option_table() {
#define H2D_OPT(name) {#name, [](EngineOptions& o, const py::handle& v) { o.name = v.cast<decltype(o.name)>(); }}
  static const std::map<std::string, OptSetter> t = {
      H2D_OPT(gridx), H2D_OPT(gridy), H2D_OPT(periodic_x), H2D_OPT(periodic_y), H2D_OPT(boundary),
      H2D_OPT(precision), H2D_OPT(init), H2D_OPT(cx), H2D_OPT(cy), H2D_OPT(tblock), H2D_OPT(rows_per_wave),
      H2D_OPT(edge_weight), H2D_OPT(wave_capacity), H2D_OPT(boundary_rows), H2D_OPT(concurrent),
      H2D_OPT(comm_boundary), H2D_OPT(signal_exchange), H2D_OPT(device_halo_wait), H2D_OPT(comm_priority),
      H2D_OPT(signal_plan), H2D_OPT(watchdog_s), H2D_OPT(halo_timeout_s), H2D_OPT(sync_mode), H2D_OPT(fused_check), H2D_OPT(direct_release), H2D_OPT(direct_acquire), H2D_OPT(trace), H2D_OPT(poison), H2D_OPT(convergence),
      H2D_OPT(interval), H2D_OPT(sensitivity), H2D_OPT(device), H2D_OPT(ranks), H2D_OPT(transport),
      H2D_OPT(overlap), H2D_OPT(small_grid_lds), H2D_OPT(tiled), H2D_OPT(tile_rows), H2D_OPT(tile_width),
      H2D_OPT(tile_k), H2D_OPT(naive), H2D_OPT(comm_cus), H2D_OPT(comm_cu_layout), H2D_OPT(reserve_waves),
      H2D_OPT(device_fence_events), H2D_OPT(contiguous_halo),
  };
#undef H2D_OPT
  return t;
}

void apply_engine_options(EngineOptions& o, const py::kwargs& kw) {
  const auto& t = engine_option_table();
  for (auto item : kw) {
    const std::string k = item.first.cast<std::string>();
    auto it = t.find(k);
    if (it == t.end()) throw py::type_error("Engine: unknown option '" + k + "'");
    if (item.second.is_none()) continue;
    it->second(o, item.second);
  }
}

}  // namespace

PYBIND11_MODULE(_heat2d, m) {
  m.doc() = "heat2d_amd native runtime (HIP/CDNA4 kernels, RCCL transport, CPU oracle)";

  m.attr("FIXED") = (int)kFixed;
  m.attr("GHOST_ZERO") = (int)kGhostZero;
  m.attr("REF") = (int)kRef;
  m.attr("FP32") = (int)kFp32;
  m.attr("INIT_EXACT") = (int)kInitExact;
  m.attr("INIT_INT32") = (int)kInitInt32;
  m.attr("INIT_ZERO") = (int)kInitZero;
  m.attr("CX_DOUBLE") = kCxDouble;
  m.attr("CX_FLOAT") = kCxFloat;
  m.attr("TRANSPORT_AUTO") = (int)kTransportAuto;
  m.attr("TRANSPORT_LOCAL") = (int)kTransportLocal;
  m.attr("TRANSPORT_RCCL") = (int)kTransportRccl;
  m.attr("TRANSPORT_EXTERNAL") = (int)kTransportExternal;
  m.attr("TRANSPORT_IPC") = (int)kTransportIpc;
  m.attr("TEXT_GRAD") = (int)kTextGrad;
  m.attr("TEXT_HEAT2DN") = (int)kTextHeat2dn;
  m.attr("WAVE_COLS") = kWaveCols;
  m.attr("MAX_K") = kMaxK;

  // ---- numerics -------------------------------------------------------------------------
  m.def("update_ref", &update_ref, "bit-exact reference cell update (c, n, s, w, e, cx, cy)");
  m.def("update_f32", &update_f32, "fp32 FMA cell update (c, n, s, w, e, cx, cy)");
  m.def("init_value", &init_value, py::arg("mode"), py::arg("gx"), py::arg("gy"), py::arg("NX"), py::arg("NY"));
  m.def(
      "init_global",
      [](int64_t nx, int64_t ny, int init) {
        std::vector<float> u;
        init_global(u, nx, ny, init);
        return to_array(u, nx, ny);
      },
      py::arg("nx"), py::arg("ny"), py::arg("init") = (int)kInitExact);
  m.def(
      "oracle_run",
      [](int64_t nx, int64_t ny, int64_t steps, int boundary, int precision, double cx, double cy, int init,
         bool convergence, int64_t interval, double sensitivity, bool per_x, bool per_y, py::object initial) {
        Physics ph;
        ph.boundary = boundary;
        ph.precision = precision;
        ph.cx = cx;
        ph.cy = cy;
        ph.periodic_x = per_x;
        ph.periodic_y = per_y;
        OracleResult r;
        if (initial.is_none()) {
          py::gil_scoped_release nogil;
          r = oracle_run(nx, ny, steps, ph, init, convergence, interval, sensitivity, nullptr);
        } else {
          auto a = initial.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
          const float* p = checked_grid(a, nx, ny);
          py::gil_scoped_release nogil;
          r = oracle_run(nx, ny, steps, ph, init, convergence, interval, sensitivity, p);
        }
        py::dict d;
        d["grid"] = to_array(r.grid, nx, ny);
        d["steps_done"] = r.steps_done;
        d["converged"] = r.converged;
        d["residual"] = r.residual;
        return d;
      },
      py::arg("nx"), py::arg("ny"), py::arg("steps"), py::arg("boundary") = (int)kFixed,
      py::arg("precision") = (int)kRef, py::arg("cx") = kCxDouble, py::arg("cy") = kCxDouble,
      py::arg("init") = (int)kInitExact, py::arg("convergence") = false, py::arg("interval") = 20,
      py::arg("sensitivity") = 0.1, py::arg("periodic_x") = false, py::arg("periodic_y") = false,
      py::arg("initial") = py::none());

  // ---- decomposition ----------------------------------------------------------------------
  py::class_<Decomposition>(m, "Decomposition")
      .def(py::init<int64_t, int64_t, int, int, bool, bool>(), py::arg("nx"), py::arg("ny"), py::arg("gridx"),
           py::arg("gridy"), py::arg("periodic_x") = false, py::arg("periodic_y") = false)
      .def_readonly("NX", &Decomposition::NX)
      .def_readonly("NY", &Decomposition::NY)
      .def_readonly("gridx", &Decomposition::gridx)
      .def_readonly("gridy", &Decomposition::gridy)
      .def_readonly("xstart", &Decomposition::xstart)
      .def_readonly("xcount", &Decomposition::xcount)
      .def_readonly("ystart", &Decomposition::ystart)
      .def_readonly("ycount", &Decomposition::ycount)
      .def("nranks", &Decomposition::nranks)
      .def("px_of", &Decomposition::px_of)
      .def("py_of", &Decomposition::py_of)
      .def("rank_of", &Decomposition::rank_of)
      .def("neighbor", &Decomposition::neighbor)
      .def("max_halo_depth", &Decomposition::max_halo_depth)
      .def("tile", [](const Decomposition& d, int rank, int64_t G) { return geom_dict(d.tile(rank, G)); })
      .def("plan",
           [](const Decomposition& d, int rank, int64_t G, int K) {
             ExchangePlan p = make_plan(d, rank, d.tile(rank, G), K);
             py::list out;
             for (int dir = 0; dir < kNumDirs; ++dir) {
               py::dict e;
               e["peer"] = p.peer[dir];
               e["send"] = py::make_tuple(p.send_rect[dir].r0, p.send_rect[dir].c0, p.send_rect[dir].rows,
                                          p.send_rect[dir].cols);
               e["recv"] = py::make_tuple(p.recv_rect[dir].r0, p.recv_rect[dir].c0, p.recv_rect[dir].rows,
                                          p.recv_rect[dir].cols);
               e["send_off"] = p.send_off[dir];
               e["recv_off"] = p.recv_off[dir];
               out.append(e);
             }
             return out;
           })
      .def("__repr__", [](const Decomposition& d) { return describe(d); });
  m.def("tile_geom", [](int64_t nx, int64_t ny, int64_t G) { return geom_dict(make_tile_geom(nx, ny, 0, 0, nx, ny, G)); },
        py::arg("nx"), py::arg("ny"), py::arg("G"));
  m.attr("DIR_NAMES") = std::vector<std::string>{"N", "S", "W", "E", "NW", "NE", "SW", "SE"};
  m.attr("DIR_OPP") = std::vector<int>(kDirOpp, kDirOpp + kNumDirs);

  // ---- engine -----------------------------------------------------------------------------
  py::class_<Engine>(m, "Engine")
      .def(py::init([](int64_t nx, int64_t ny, py::kwargs kw) {
             EngineOptions o;
             o.nx = nx;
             o.ny = ny;
             apply_engine_options(o, kw);
             py::gil_scoped_release nogil;
             return new Engine(o);
           }),
           py::arg("nx"), py::arg("ny"),
           "Engine(nx, ny, **options): every EngineOptions field by name (see engine.h)")
      .def_static("option_names", []() {
        std::vector<std::string> v;
        for (auto& kv : engine_option_table()) v.push_back(kv.first);
        return v;
      })
      .def("num_tiles", &Engine::num_tiles)
      .def("tile_rank", &Engine::tile_rank)
      .def("geom", [](const Engine& e, int t) { return geom_dict(e.geom(t)); })
      .def("halo_depth", &Engine::halo_depth)
      .def("has_exchange", &Engine::has_exchange)
      .def("concurrent", &Engine::concurrent)
      .def("signal_mode", &Engine::signal_mode)
      .def("pipeline", &Engine::pipeline)
      .def("tiled", &Engine::tiled)
      .def("tile_config", &Engine::tile_config)
      .def("comm_cus", &Engine::comm_cus)
      .def("contiguous_halo", &Engine::contiguous_halo)
      .def("wave_capacity", &Engine::wave_capacity)
      .def("on_gpu", &Engine::on_gpu)
      .def("rows_per_wave", &Engine::rows_per_wave)
      .def("num_units", &Engine::num_units)
      .def("steps_done", &Engine::steps_done)
      .def("set_steps_done", &Engine::set_steps_done)
      .def("stream_handle", &Engine::stream_handle)
      .def_static("rccl_unique_id", []() { return py::bytes(Engine::rccl_unique_id()); })
      .def("init_rccl", [](Engine& e, py::bytes id, int n, int r) {
        std::string s = id;
        py::gil_scoped_release nogil;
        e.init_rccl(s, n, r);
      })
      .def("rccl_ready", &Engine::rccl_ready)
      .def("ipc_handle", [](Engine& e) { return py::bytes(e.ipc_handle()); })
      .def("ipc_open",
           [](Engine& e, const std::vector<py::bytes>& hs) {
             std::vector<std::string> v;
             for (auto& h : hs) v.push_back(std::string(h));
             py::gil_scoped_release nogil;
             e.ipc_open(v);
           })
      .def("ipc_prime", &Engine::ipc_prime, py::call_guard<py::gil_scoped_release>())
      .def("ipc_primed", &Engine::ipc_primed)
      .def("direct", &Engine::direct)
      .def("run",
           [](Engine& e, int64_t steps) {
             RunStats s;
             {
               py::gil_scoped_release nogil;
               s = e.run(steps);
             }
             return stats_dict(s);
           })
      .def("next_chunk",
           [](const Engine& e, int64_t done, int64_t total) {
             bool check = false;
             const int k = e.next_chunk(done, total, &check);
             return py::make_tuple(k, check);
           })
      .def("advance", &Engine::advance, py::arg("k"), py::arg("residual") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("exchange_local", &Engine::exchange_local, py::call_guard<py::gil_scoped_release>())
      .def("local_residual", &Engine::local_residual, py::call_guard<py::gil_scoped_release>())
      .def("send_count", &Engine::send_count)
      .def("recv_count", &Engine::recv_count)
      .def("plan_info", &Engine::plan_info)
      .def("pack", &Engine::pack, py::call_guard<py::gil_scoped_release>())
      .def("unpack", &Engine::unpack, py::call_guard<py::gil_scoped_release>())
      .def("rollback", &Engine::rollback)
      .def("download",
           [](const Engine& e, int t) {
             const TileGeom g = e.geom(t);
             std::vector<float> v;
             {
               py::gil_scoped_release nogil;
               v = e.download(t);
             }
             return to_array(v, g.xcell, g.ycell);
           })
      .def("upload",
           [](Engine& e, int t, py::array_t<float, py::array::c_style | py::array::forcecast> a) {
             const TileGeom g = e.geom(t);
             e.upload(t, checked_grid(a, g.xcell, g.ycell));
           })
      .def("synchronize", &Engine::synchronize, py::call_guard<py::gil_scoped_release>());

  // ---- I/O ---------------------------------------------------------------------------------
  m.def("binary_create", &binary_create);
  m.def("binary_write_tile", [](const std::string& path, int64_t NX, int64_t NY, int64_t gx0, int64_t gy0,
                                py::array_t<float, py::array::c_style | py::array::forcecast> a) {
    if (a.ndim() != 2) throw std::invalid_argument("tile must be 2-D");
    binary_write_tile(path, NX, NY, gx0, gy0, a.shape(0), a.shape(1), a.data());
  });
  m.def("binary_read", [](const std::string& path, int64_t NX, int64_t NY) {
    return to_array(binary_read(path, NX, NY), NX, NY);
  });
  m.def("binary_to_text", &binary_to_text, py::call_guard<py::gil_scoped_release>());
  m.def("format_text", [](py::array_t<float, py::array::c_style | py::array::forcecast> a, int style) {
    if (a.ndim() != 2) throw std::invalid_argument("grid must be 2-D");
    return py::bytes(format_text(a.data(), a.shape(0), a.shape(1), style));
  });

  // ---- devices -----------------------------------------------------------------------------
  m.def("device_count", &device_count);
  m.def("device_props", &device_props);
  m.def(
      "mem_info",
      [](int dev) {
        size_t fr = 0, tot = 0;
        H2D_HIP_CHECK(hipSetDevice(dev));
        H2D_HIP_CHECK(hipMemGetInfo(&fr, &tot));
        return py::make_tuple((int64_t)fr, (int64_t)tot);
      },
      py::arg("device") = 0, "(free, total) device memory in bytes (hipMemGetInfo)");

  // ---- raw-pointer kernel ops (torch tensors laid out as TileGeom storage) ---------------
  m.def(
      "op_init",
      [](uintptr_t base, const py::dict& geom, int init, uintptr_t stream) {
        launch_init(geom_from(geom), reinterpret_cast<float*>(base), init, reinterpret_cast<hipStream_t>(stream));
      },
      py::arg("base"), py::arg("geom"), py::arg("init"), py::arg("stream") = 0);
  m.def(
      "op_stream",
      [](uintptr_t src, uintptr_t dst, const py::dict& geom, int K, int precision, int boundary, double cx, double cy,
         bool per_x, bool per_y, int H, uintptr_t partials, uintptr_t stream) {
        const TileGeom g = geom_from(geom);
        if (!stream_k_supported(K)) throw std::invalid_argument("unsupported K");
        if (K > g.G) throw std::invalid_argument("K exceeds the tile's ghost depth");
        const OpPlan& P = op_plan(g, K, H, precision, boundary == kFixed, per_x, per_y);
        StreamArgs a;
        a.src = reinterpret_cast<const float*>(src);
        a.dst = reinterpret_cast<float*>(dst);
        a.units = P.units;
        a.nunits = P.n;
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
        a.cx = cx;
        a.cy = cy;
        a.fixed = boundary == kFixed;
        a.per_x = per_x;
        a.per_y = per_y;
        a.partials = reinterpret_cast<double*>(partials);
        a.dummy = P.dummy;
        launch_stream(a, K, precision, partials != 0, reinterpret_cast<hipStream_t>(stream));
        return P.n;
      },
      py::arg("src"), py::arg("dst"), py::arg("geom"), py::arg("K"), py::arg("precision") = (int)kRef,
      py::arg("boundary") = (int)kFixed, py::arg("cx") = kCxDouble, py::arg("cy") = kCxDouble,
      py::arg("periodic_x") = false, py::arg("periodic_y") = false, py::arg("H") = 0, py::arg("partials") = 0,
      py::arg("stream") = 0);
  m.def(
      "op_num_units",
      [](const py::dict& geom, int K, int precision, int boundary, bool per_x, bool per_y, int H) {
        const TileGeom g = geom_from(geom);
        if (!stream_k_supported(K)) throw std::invalid_argument("unsupported K");
        return op_plan(g, K, H, precision, boundary == kFixed, per_x, per_y).n;
      },
      py::arg("geom"), py::arg("K"), py::arg("precision") = (int)kRef, py::arg("boundary") = (int)kFixed,
      py::arg("periodic_x") = false, py::arg("periodic_y") = false, py::arg("H") = 0);
  m.def(
      "op_naive",
      [](uintptr_t src, uintptr_t dst, const py::dict& geom, int precision, int boundary, double cx, double cy,
         bool per_x, bool per_y, uintptr_t stream) {
        launch_naive_step(geom_from(geom), reinterpret_cast<const float*>(src), reinterpret_cast<float*>(dst),
                          precision, boundary, cx, cy, per_x, per_y, reinterpret_cast<hipStream_t>(stream));
      },
      py::arg("src"), py::arg("dst"), py::arg("geom"), py::arg("precision") = (int)kRef,
      py::arg("boundary") = (int)kFixed, py::arg("cx") = kCxDouble, py::arg("cy") = kCxDouble,
      py::arg("periodic_x") = false, py::arg("periodic_y") = false, py::arg("stream") = 0);
  m.def("stream_k_supported", &stream_k_supported);
  m.def("lds_solver_fits", &lds_solver_fits);
  m.def("stream_wave_capacity", &stream_wave_capacity);
  m.def(
      "unit_plan",
      [](int64_t nx, int64_t ny, int K, int H, bool fixed, bool per_x, bool per_y, double ew, int64_t capacity) {
        const TileGeom g = make_tile_geom(nx, ny, 0, 0, nx, ny, K);
        UnitPlan p = plan_units(g, K, H, fixed, per_x, per_y, ew, capacity, nullptr, 16);
        py::list out;
        for (const Unit& u : p.interior) out.append(py::make_tuple(u.strip, u.x0, u.h, u.flags));
        return out;
      },
      "work units (strip, x0, h, flags) of a single nx×ny tile");
  m.def(
      "strip_layout",
      [](int64_t nx, int64_t ny, int K, bool fixed, bool per_y) {
        const TileGeom g = make_tile_geom(nx, ny, 0, 0, nx, ny, K);
        py::list out;
        for (const Strip& s : strip_layout(g, K, fixed, per_y)) out.append(py::make_tuple(s.cb, s.lo, s.hi));
        return out;
      },
      "column strips (cb, lo, hi) of a single nx×ny tile: lane-0 column, output columns [lo, hi)");
  m.def("lead_cols", &lead_cols);
  m.def("strip_out_cols", &strip_out_cols);
}
