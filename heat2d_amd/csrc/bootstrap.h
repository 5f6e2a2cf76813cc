// heat2d_amd — native multi-process bootstrap for the `heat2d` executable.
//
// The reference's run model is `mpiexec -n P ./binary` (readme.md:10-19): MPI_Init, rank /
// size, MPI_Bcast of the decomposition, MPI_Barrier before timing, MPI_Reduce(MAX) of the
// elapsed time, MPI-IO output (grad1612_mpi_heat.c:42-44,146-147,206,277-280).  The native
// executable does the same without MPI: ranks find each other through a small TCP star
// rooted at rank 0 (env RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR as set by
// `torch.distributed.run --no-python` or by `heat2d --np P`, which forks the ranks itself),
// and this control plane carries:
//   * the bootstrap of the GPU data plane: the IPC block handles (direct halo pipeline) or the
//     RCCL unique id;
//   * barriers, max / sum reductions of scalars (timing, convergence on the CPU path);
//   * on the CPU, the halo exchange itself (relayed through rank 0 — a test path, not a fast one).
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace h2d {

class Bootstrap {
 public:
  // rank 0 listens on addr:port (or on the socket HEAT2D_BOOT_LISTEN_FD names, which `heat2d --np`
  // binds before forking: no port race); the others connect.  Every wait is bounded: connecting
  // and accepting by timeout_s, every later receive by io_timeout_s (a collective can legitimately
  // wait as long as a run lasts; env HEAT2D_BOOT_IO_TIMEOUT_S overrides it).
  Bootstrap(int rank, int world, const std::string& addr, int port, double timeout_s = 120.0,
            double io_timeout_s = 3600.0);
  ~Bootstrap();
  Bootstrap(const Bootstrap&) = delete;
  Bootstrap& operator=(const Bootstrap&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }

  std::vector<std::string> allgather(const std::string& mine);
  std::string broadcast(const std::string& data, int root = 0);
  void barrier();
  double allreduce_max(double x);
  double allreduce_sum(double x);
  double allreduce_min(double x);
  // personalised exchange of tagged messages: returns {(source, tag): bytes} addressed to me
  struct Msg {
    int dst, tag;
    std::string data;
  };
  std::map<std::pair<int, int>, std::string> exchange(const std::vector<Msg>& out);

 private:
  int rank_, world_;
  int listen_fd_ = -1;
  std::vector<int> fds_;  // rank 0: one socket per rank (index = rank); others: fds_[0] = to rank 0
};

// Environment of a launched rank (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT;
// the bootstrap port is HEAT2D_BOOT_PORT or MASTER_PORT + 7, next to the launcher's own store).
struct RankEnv {
  int rank = 0, world = 1, local_rank = 0;
  std::string addr = "127.0.0.1";
  int port = 29507;
};
RankEnv rank_env();

}  // namespace h2d
