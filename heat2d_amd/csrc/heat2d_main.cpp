// heat2d — the native command-line program (one process: one GPU with all GRIDX×GRIDY tiles
// as local tiles, or the CPU).  Same flags, presets, banners and output files as
// `python -m heat2d_amd` (multi-GPU runs go through torch.distributed + RCCL in Python).
//
// Replaces the compile-time #define knobs of the reference programs
// (grad1612_mpi_heat.c:5-21, mpi_heat2Dn.c:29-44, grad1612_hybrid_heat.c:6-24,
// grad1612_cuda_heat.cu:6-13) with runtime flags; banners follow C-IO-4.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <sys/stat.h>
#include <vector>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <set>

#include "bootstrap.h"
#include "cpu_reference.h"
#include "decomposition.h"
#include "engine.h"
#include "io.h"
#include "shm_barrier.h"

#include <memory>
#include <random>

using namespace h2d;

namespace {

// Node-local spin barrier for the timed region (shm_barrier.h), set up collectively: rank 0
// creates a uniquely named segment, the others open it, and every rank keeps it only if all
// succeeded (ranks on another node cannot open it: then everyone uses the TCP barrier alone).
// The name is unlinked as soon as all ranks hold the mapping.
std::unique_ptr<ShmBarrier> node_barrier(Bootstrap& boot) {
  if (boot.world() <= 1) return nullptr;
  std::string name;
  if (boot.rank() == 0) {
    std::random_device rd;
    name = "/heat2d_bar_" + std::to_string(getpid()) + "_" + std::to_string(rd());
  }
  name = boot.broadcast(name);
  std::unique_ptr<ShmBarrier> b;
  if (boot.rank() == 0) {
    try {
      b = std::make_unique<ShmBarrier>(name, 0, boot.world(), true);
    } catch (const std::exception&) {
      b.reset();
    }
  }
  boot.barrier();  // the segment exists before anyone opens it
  if (boot.rank() != 0) {
    try {
      b = std::make_unique<ShmBarrier>(name, boot.rank(), boot.world(), false);
    } catch (const std::exception&) {
      b.reset();
    }
  }
  const bool all = boot.allreduce_min(b ? 1.0 : 0.0) > 0.5;
  if (b) b->unlink();  // rank 0: every rank has opened (or given up on) the name by now
  if (!all) b.reset();
  return b;
}

struct Preset {
  int64_t nx, ny, steps;
  int gridx, gridy;
  int boundary;
  double cx;
  bool convergence;
  int64_t interval;
  double sensitivity;
  std::string report, text;
  bool binary;
  bool strips;
};

// The preset table lives in presets.def (shared with the Python package).
const std::map<std::string, Preset>& presets() {
  static const std::map<std::string, Preset> p = [] {
    const int fixed = kFixed, ghost_zero = kGhostZero;
    const double dbl = kCxDouble, flt = kCxFloat;
    (void)fixed;
    (void)ghost_zero;
    (void)dbl;
    (void)flt;
    std::map<std::string, Preset> m;
#define H2D_PRESET(name, nx, ny, steps, gx, gy, bnd, coeff, conv, interval, sens, report, text, binary, dec) \
  m[#name] = Preset{nx, ny, steps, gx, gy, bnd, std::string(#coeff) == "float" ? flt : dbl, conv != 0, interval,   \
                    sens, #report, #text, binary != 0, std::string(#dec) == "strips"};
#include "presets.def"
#undef H2D_PRESET
    return m;
  }();
  return p;
}

[[noreturn]] void usage(const char* msg) {
  if (msg) std::fprintf(stderr, "heat2d: %s\n", msg);
  std::fprintf(stderr,
               "usage: heat2d [--preset heat2d|heat2dn|grad_mpi|grad_hybrid|cuda] [--nx N] [--ny N] [--steps N]\n"
               "              [--gridx N] [--gridy N] [--convergence 0|1] [--interval N] [--sensitivity X]\n"
               "              [--cx X] [--cy X] [--boundary fixed|ghost-zero] [--init exact|ref-int32|zero]\n"
               "              [--precision ref|fp32] [--periodic none|x|y|xy] [--output auto|text|binary|both|none]\n"
               "              [--outdir DIR] [--device gpu|cpu] [--tblock K] [--rows-per-wave H] [--no-overlap]\n"
               "              [--numthreads N] [--debug 0|1] [--json] [--quiet]\n"
               "              [--np P]   run P ranks (forked here, like mpiexec -n P; or launch with\n"
               "                         torch.distributed.run --no-python: RANK/WORLD_SIZE/MASTER_ADDR)\n");
  std::exit(2);
}

void write_outputs(Engine& e, Bootstrap& boot, const std::string& outdir, const char* which, int64_t NX, int64_t NY,
                   bool binary, bool text, int style) {
  // every rank pwrites its own tile rows into the global raw file (the MPI-IO file view the
  // reference intended, B-3); rank 0 creates it first and converts it to text last
  if (!binary && !text) return;
  const std::string bin = outdir + "/" + which + "_binary.dat";
  const std::string tmp = binary ? bin : outdir + "/." + which + "_binary.tmp";
  if (boot.rank() == 0) {
    ::mkdir(outdir.c_str(), 0755);
    binary_create(tmp, NX, NY);
  }
  boot.barrier();
  for (int t = 0; t < e.num_tiles(); ++t) {
    const TileGeom g = e.geom(t);
    const std::vector<float> b = e.download(t);
    binary_write_tile(tmp, NX, NY, g.gx0, g.gy0, g.xcell, g.ycell, b.data());
  }
  boot.barrier();
  if (boot.rank() == 0) {
    if (text) binary_to_text(tmp, outdir + "/" + which + ".dat", NX, NY, style);
    if (!binary) std::remove(tmp.c_str());
  }
  boot.barrier();
}

// `heat2d --np P ...`: the mpiexec of this program.  Binds the bootstrap's listening socket
// (127.0.0.1, a free port: no collision with another job), then forks P ranks BEFORE anything
// touches a GPU.  A child returns -1 and carries on in main() as its rank (RANK / WORLD_SIZE /
// LOCAL_RANK / MASTER_ADDR set; rank 0 inherits the socket) — no exec.  The parent waits for
// all of them; on the first failure it stops the others (SIGTERM) so none is left waiting in a
// collective, and returns that failure.
int launch_ranks(int np) {
  const int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = 0;
  inet_pton(AF_INET, "127.0.0.1", &sa.sin_addr);
  socklen_t len = sizeof(sa);
  if (lfd < 0 || ::bind(lfd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(lfd, np) != 0 ||
      ::getsockname(lfd, reinterpret_cast<sockaddr*>(&sa), &len) != 0) {
    std::perror("heat2d: bootstrap socket");
    return 1;
  }
  const int port = ntohs(sa.sin_port);
  std::fflush(stdout);
  std::fflush(stderr);
  std::set<pid_t> alive;
  for (int r = 0; r < np; ++r) {
    const pid_t pid = ::fork();
    if (pid < 0) {
      std::perror("heat2d: fork");
      for (pid_t k : alive) ::kill(k, SIGTERM);
      return 1;
    }
    if (pid == 0) {
      ::setenv("RANK", std::to_string(r).c_str(), 1);
      ::setenv("LOCAL_RANK", std::to_string(r).c_str(), 1);
      ::setenv("WORLD_SIZE", std::to_string(np).c_str(), 1);
      ::setenv("MASTER_ADDR", "127.0.0.1", 1);
      ::setenv("HEAT2D_BOOT_PORT", std::to_string(port).c_str(), 1);
      ::setenv("HEAT2D_BOOT_LISTEN_FD", std::to_string(lfd).c_str(), 1);
      return -1;
    }
    alive.insert(pid);
  }
  ::close(lfd);
  int rc = 0;
  while (!alive.empty()) {
    int st = 0;
    const pid_t k = ::waitpid(-1, &st, 0);
    if (k < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (!alive.erase(k)) continue;
    const int c = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
    if (c != 0 && rc == 0) {
      rc = c;
      for (pid_t o : alive) ::kill(o, SIGTERM);
    }
  }
  return rc;
}

// The CPU multi-rank time loop: the engine's external transport, halos relayed through the
// bootstrap star (pack -> exchange -> unpack), the convergence sum over ranks in rank order.
RunStats run_external(Engine& e, Bootstrap& boot, int64_t steps, double sensitivity) {
  RunStats st;
  st.path = "cpu";
  const int me = boot.rank();
  const int64_t total = e.steps_done() + steps;
  int64_t done = e.steps_done();
  while (done < total) {
    bool check = false;
    const int k = e.next_chunk(done, total, &check);
    const std::vector<int64_t> info = e.plan_info(0, k);  // [peer, send_off, send_n, recv_off, recv_n] x 8
    std::vector<float> sb((size_t)std::max<int64_t>(1, e.send_count(0, k)));
    std::vector<float> rb((size_t)std::max<int64_t>(1, e.recv_count(0, k)));
    e.pack(0, k, reinterpret_cast<uintptr_t>(sb.data()));
    std::vector<Bootstrap::Msg> out;
    for (int d = 0; d < kNumDirs; ++d) {
      const int64_t peer = info[5 * d], so = info[5 * d + 1], sn = info[5 * d + 2];
      if (peer >= 0 && sn > 0)
        out.push_back({(int)peer, d, std::string(reinterpret_cast<const char*>(sb.data() + so), (size_t)sn * 4)});
    }
    const auto in = boot.exchange(out);
    for (int d = 0; d < kNumDirs; ++d) {
      const int g = kDirOpp[d];  // ghost side g receives the segment its peer sent in direction d
      const int64_t peer = info[5 * g], ro = info[5 * g + 3], rn = info[5 * g + 4];
      if (peer < 0 || rn <= 0) continue;
      auto it = in.find(std::make_pair((int)peer, d));
      if (it == in.end() || it->second.size() != (size_t)rn * 4)
        throw std::runtime_error("rank " + std::to_string(me) + ": halo segment missing");
      std::memcpy(rb.data() + ro, it->second.data(), (size_t)rn * 4);
    }
    e.unpack(0, k, reinterpret_cast<uintptr_t>(rb.data()));
    ++st.exchanges;
    e.advance(k, check);
    ++st.chunks;
    if (check) {
      st.residual = boot.allreduce_sum(e.local_residual());
      if (st.residual < sensitivity) {
        e.rollback();
        st.converged = true;
        break;
      }
    }
    done += k;
  }
  e.set_steps_done(done);
  st.steps_done = done;
  return st;
}

}  // namespace

int main(int argc, char** argv) {
  // kernel arguments from host memory (docs/ARCHITECTURE.md, "Kernel arguments and metadata
  // memory"); before any HIP call, and only if the user did not choose
  setenv("HIP_FORCE_DEV_KERNARG", "0", 0);
  std::map<std::string, std::string> a;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    if (k.rfind("--", 0) != 0) usage(("unexpected argument " + k).c_str());
    k = k.substr(2);
    if (k == "no-overlap" || k == "json" || k == "quiet" || k == "help") {
      a[k] = "1";
      continue;
    }
    if (i + 1 >= argc) usage(("missing value for --" + k).c_str());
    a[k] = argv[++i];
  }
  if (a.count("help")) usage(nullptr);
  if (a.count("np") && std::atoi(a["np"].c_str()) > 1) {
    const int rc = launch_ranks(std::atoi(a["np"].c_str()));
    if (rc >= 0) return rc;  // the launcher; a forked rank continues below
  }
  const RankEnv env = rank_env();
  const int world = env.world;
  const std::string pname = a.count("preset") ? a["preset"] : "heat2d";
  if (!presets().count(pname)) usage("unknown preset");
  const Preset P = presets().at(pname);
  auto geti = [&](const char* k, int64_t d) { return a.count(k) ? std::atoll(a[k].c_str()) : d; };
  auto getd = [&](const char* k, double d) { return a.count(k) ? std::atof(a[k].c_str()) : d; };

  EngineOptions o;
  o.nx = geti("nx", P.nx);
  o.ny = geti("ny", P.ny);
  const int64_t steps = geti("steps", P.steps);
  o.gridx = (int)geti("gridx", P.gridx);
  o.gridy = (int)geti("gridy", P.gridy);
  if (P.strips && !a.count("gridy")) o.gridy = 1;
  if (o.gridx == 0) o.gridx = std::max(1, world / std::max(1, o.gridy));  // automatic: strips over the ranks
  if (o.gridx < 1 || o.gridy < 1) usage("gridx/gridy must be >= 1");
  if (world > 1 && o.gridx * o.gridy != world) {
    if (env.rank == 0)
      std::printf("ERROR: the number of tasks must be equal to %d.\nQuiting...\n", o.gridx * o.gridy);
    return 1;
  }
  o.convergence = geti("convergence", P.convergence ? 1 : 0) != 0;
  o.interval = geti("interval", P.interval);
  o.sensitivity = getd("sensitivity", P.sensitivity);
  o.cx = getd("cx", P.cx);
  o.cy = getd("cy", P.cx);
  o.boundary = P.boundary;
  if (a.count("boundary")) o.boundary = a["boundary"] == "fixed" ? kFixed : kGhostZero;
  const std::string init = a.count("init") ? a["init"] : "exact";
  o.init = init == "exact" ? kInitExact : init == "ref-int32" ? kInitInt32 : kInitZero;
  o.precision = (a.count("precision") && a["precision"] == "fp32") ? kFp32 : kRef;
  const std::string per = a.count("periodic") ? a["periodic"] : "none";
  o.periodic_x = per.find('x') != std::string::npos;
  o.periodic_y = per.find('y') != std::string::npos;
  o.tblock = (int)geti("tblock", 0);
  if (o.tblock <= 0) o.tblock = o.precision == kFp32 ? 8 : 7;  // measured at 4096^2 (profiles/tblock_sweep_r2.txt)
  o.rows_per_wave = (int)geti("rows-per-wave", 0);
  o.overlap = !a.count("no-overlap");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  const std::string dev = a.count("device") ? a["device"] : (ndev > 0 ? "gpu" : "cpu");
  if (dev == "gpu" && ndev == 0) usage("--device gpu but no HIP device is visible");
  o.device = dev == "gpu" ? env.local_rank % std::max(1, ndev) : -1;
  o.transport = kTransportLocal;
  // multi-rank: one tile per process; GPUs: the direct IPC halo pipeline (rows or blocks),
  // RCCL where it cannot run; CPUs: halos relayed through the bootstrap
  const std::string tsel = a.count("transport") ? a["transport"] : "auto";
  if (world > 1) {
    o.ranks = {env.rank};
    if (dev != "gpu") o.transport = kTransportExternal;
    // direct IPC needs halo units of at least max(K, G) rows at both ends of every strip (and,
    // for 2-D blocks, tiles 4-column aligned: the engine refuses others and every rank falls
    // back to RCCL together below)
    else if (tsel == "ipc" || (tsel == "auto" && o.nx / o.gridx >= 2 * (int64_t)o.tblock))
      o.transport = kTransportIpc;
    else o.transport = kTransportRccl;
  }
  const bool quiet = a.count("quiet") > 0 || env.rank != 0;
  std::string output = a.count("output") ? a["output"] : "auto";
  if (output == "auto") {
    const bool t = P.text != "none";
    output = t && P.binary ? "both" : t ? "text" : P.binary ? "binary" : "none";
  }
  const bool wbin = output == "binary" || output == "both";
  const bool wtxt = output == "text" || output == "both";
  const std::string outdir = a.count("outdir") ? a["outdir"] : ".";
  const int tstyle = P.text == "heat2dn" ? kTextHeat2dn : kTextGrad;
  const std::string rep = P.report;

  try {
    Bootstrap boot(env.rank, world, env.addr, env.port);
    std::unique_ptr<ShmBarrier> shm = node_barrier(boot);
    if (world > 1 && o.device >= 0) {
      // ranks on one physical GPU (host + PCI bus id, whatever the visibility setup): no
      // persistent launches on any rank (each needs every one of its waves resident)
      char host[256] = {0}, bus[64] = {0};
      gethostname(host, sizeof(host) - 1);
      H2D_HIP_CHECK(hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, o.device));
      std::vector<std::string> ids = boot.allgather(std::string(host) + "|" + bus);
      std::sort(ids.begin(), ids.end());
      if (std::adjacent_find(ids.begin(), ids.end()) != ids.end()) o.persistent = 0;
    }
    std::unique_ptr<Engine> ep;
    std::string why;
    try {
      ep = std::make_unique<Engine>(o);
    } catch (const std::exception& ex) {
      why = ex.what();
    }
    // every rank agrees: an engine the automatic choice (direct IPC) cannot build on some rank
    // falls back to RCCL together; a requested transport fails as requested
    if (boot.allreduce_min(ep ? 1.0 : 0.0) < 0.5) {
      if (!(o.transport == kTransportIpc && tsel == "auto"))
        throw std::runtime_error(why.empty() ? "engine construction failed on another rank" : why);
      ep.reset();
      o.transport = kTransportRccl;
      ep = std::make_unique<Engine>(o);
    }
    Engine& e = *ep;
    if (o.transport == kTransportIpc && e.has_exchange()) {
      e.ipc_open(boot.allgather(e.ipc_handle()));
      boot.barrier();
      e.ipc_prime();
      boot.barrier();
    } else if (o.transport == kTransportRccl && e.has_exchange()) {
      e.init_rccl(boot.broadcast(env.rank == 0 ? Engine::rccl_unique_id() : std::string()), world, env.rank);
    }
    const Decomposition& d = e.decomposition();
    const int nprocs = d.nranks();
    if (!quiet) {
      if (rep == "grad" || rep == "hybrid") {
        if (rep == "grad") std::printf("Starting with %d processes\n", nprocs);
        else std::printf("Starting with %d processes and %d threads\n", nprocs, (int)geti("numthreads", 4));
        std::printf("Problem size:%lldx%lld\nEach process will take: %lldx%lld\nAmount of iterations: %lld\n",
                    (long long)o.nx, (long long)o.ny, (long long)d.xcount[0], (long long)d.ycount[0],
                    (long long)steps);
        if (o.convergence) std::printf("Check for convergence every %lld iterations\n", (long long)o.interval);
      } else if (rep == "heat2dn") {
        std::printf("Starting mpi_heat2D with %d worker tasks.\n", nprocs);
        std::printf("Grid size: X= %lld  Y= %lld  Time steps= %lld\n", (long long)o.nx, (long long)o.ny,
                    (long long)steps);
        std::printf("Initializing grid and writing initial.dat file...\n");
        for (int i = 0; i < d.gridx; ++i)
          std::printf("Sent to task %d: rows= %lld offset= %lld left= %d right= %d\n", i + 1,
                      (long long)d.xcount[i], (long long)d.xstart[i], i == 0 ? 0 : i, i == d.gridx - 1 ? 0 : i + 2);
      } else if (rep == "cuda") {
        std::printf("Problem size: %lldx%lld\nAmount of iterations: %lld\n", (long long)o.nx, (long long)o.ny,
                    (long long)steps);
      }
      if (geti("debug", 0)) {
        for (int t = 0; t < e.num_tiles(); ++t) {
          const int r = e.tile_rank(t);
          std::printf("I am %d and my neighbors are North=%d, South=%d, East=%d, West=%d (Running on %s)\n", r,
                      d.neighbor(r, kN), d.neighbor(r, kS), d.neighbor(r, kE), d.neighbor(r, kW),
                      dev == "gpu" ? "gpu0" : "cpu");
        }
      }
    }
    if (output != "none") {
      if (!quiet && (rep == "grad" || rep == "hybrid")) std::printf("Writing initial.dat ...\n");
      write_outputs(e, boot, outdir, "initial", o.nx, o.ny, wbin, wtxt, tstyle);
    }
    if (!quiet && rep == "heat2dn")
      for (int i = 0; i < d.gridx; ++i) std::printf("Task %d received work. Beginning time steps...\n", i + 1);
    std::fflush(stdout);
    e.synchronize();
    boot.barrier();
    if (shm) shm->wait();  // node-local ranks leave within ~1 us of each other (shm_barrier.h)
    const auto t0 = std::chrono::steady_clock::now();
    const RunStats st = o.transport == kTransportExternal && e.has_exchange() ? run_external(e, boot, steps, o.sensitivity)
                                                                             : e.run(steps);
    e.synchronize();
    // the loop's wall time, max over ranks (grad1612_mpi_heat.c:277-280)
    const double el = boot.allreduce_max(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    if (!quiet) {
      if (rep == "grad" || rep == "hybrid") {
        std::printf("Exiting after %lld iterations\nElapsed time: %e sec\n", (long long)st.steps_done, el);
        if (output != "none") std::printf("Writing final.dat ...\n");
      } else if (rep == "heat2dn") {
        std::printf("Elapsed time: %e sec\n", el);
        std::printf("Writing final.dat file and generating graph...\n");
        std::printf("Click on MORE button to view initial/final states.\n");
        std::printf("Click on EXIT button to quit program.\n");
      } else if (rep == "cuda") {
        std::printf("Elapsed time: %e sec\n", el);
      }
    }
    if (output != "none") write_outputs(e, boot, outdir, "final", o.nx, o.ny, wbin, wtxt, tstyle);
    if (a.count("json") && env.rank == 0) {
      const double cups = el > 0 ? (double)o.nx * (double)o.ny * (double)st.steps_done / el : 0.0;
      std::printf("{\"grid\": [%lld, %lld], \"steps\": %lld, \"elapsed_s\": %.9g, \"cell_updates_per_s\": %.9g, "
                  "\"path\": \"%s\", \"device\": \"%s\", \"tiles\": %d, \"ranks\": %d, \"pipeline\": \"%s\", "
                  "\"converged\": %s, \"chunks\": %lld}\n",
                  (long long)o.nx, (long long)o.ny, (long long)st.steps_done, el, cups, st.path.c_str(), dev.c_str(),
                  e.num_tiles(), world, e.pipeline().c_str(), st.converged ? "true" : "false", (long long)st.chunks);
    }
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "heat2d: error: %s\n", ex.what());
    return 1;
  }
  return 0;
}
