// heat2d_amd — shared-memory spin barrier for the ranks of one node.
//
// The reference brackets its timed loop with MPI_Barrier and reduces the per-rank elapsed time
// with MPI_Reduce(MAX) (grad1612_mpi_heat.c:206,277-280).  The max-over-ranks time charges every
// rank for the barrier's exit skew: a rank released late starts its halo exchange late and the
// others wait for it inside their timed region.  A TCP/gloo barrier releases ranks tens of
// microseconds apart — a large share of a 20-step strong-scaling run on 8 GPUs (~50 us).  Ranks
// of one node instead meet on a generation counter in a /dev/shm page and spin (no syscall, no
// sleep): they leave within about a microsecond of each other.
//
// Protocol (sense-reversing): each arrival adds 1 to `count`; the last one resets it and bumps
// `gen`; the others spin until `gen` moves.  Every wait is bounded (throws on timeout).  The
// page is created by rank 0 and unlinked by it once every rank has mapped it (`unlink()`), so a
// crashed job leaves nothing in /dev/shm after setup.
#pragma once

#include <cstdint>
#include <string>

namespace h2d {

class ShmBarrier {
 public:
  // rank 0 creates (create=true) and the others open the segment `name` (e.g. "/heat2d_bar_<id>")
  ShmBarrier(const std::string& name, int rank, int world, bool create);
  ~ShmBarrier();
  ShmBarrier(const ShmBarrier&) = delete;
  ShmBarrier& operator=(const ShmBarrier&) = delete;

  // returns the microseconds this rank spun; throws std::runtime_error after timeout_s
  double wait(double timeout_s = 60.0);
  // remove the name (the mapping stays valid); idempotent
  void unlink();
  int world() const { return world_; }

 private:
  struct Page;
  std::string name_;
  int rank_, world_;
  Page* page_ = nullptr;
  uint64_t gen_ = 0;
  bool owner_ = false;
};

}  // namespace h2d
