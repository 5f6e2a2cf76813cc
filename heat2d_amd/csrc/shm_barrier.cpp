// heat2d_amd — shared-memory spin barrier (see shm_barrier.h).
#include "shm_barrier.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace h2d {

// count and gen on separate 128-byte lines: arrivals do not disturb the spinners' line
struct ShmBarrier::Page {
  alignas(128) std::atomic<uint64_t> count;
  alignas(128) std::atomic<uint64_t> gen;
  alignas(128) std::atomic<uint64_t> world;
  // set by a rank whose wait timed out: its arrival is still counted, so the generation count is
  // off by one for good — every later wait (any rank) fails instead of releasing ranks early
  alignas(128) std::atomic<uint64_t> broken;
};
static_assert(sizeof(std::atomic<uint64_t>) == 8 && std::atomic<uint64_t>::is_always_lock_free,
              "the barrier words must be lock-free 64-bit atomics (shared between processes)");

ShmBarrier::ShmBarrier(const std::string& name, int rank, int world, bool create)
    : name_(name), rank_(rank), world_(world), owner_(create) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("ShmBarrier: bad rank/world");
  if (name.empty() || name[0] != '/' || name.find('/', 1) != std::string::npos)
    throw std::invalid_argument("ShmBarrier: name must look like /name");
  const int fd = create ? shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600) : shm_open(name.c_str(), O_RDWR, 0);
  if (fd < 0) throw std::runtime_error("ShmBarrier: shm_open(" + name + "): " + std::strerror(errno));
  if (create && ftruncate(fd, sizeof(Page)) != 0) {
    const int e = errno;
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error(std::string("ShmBarrier: ftruncate: ") + std::strerror(e));
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < (off_t)sizeof(Page)) {
    close(fd);
    throw std::runtime_error("ShmBarrier: segment " + name + " is not initialised");
  }
  void* p = mmap(nullptr, sizeof(Page), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error(std::string("ShmBarrier: mmap: ") + std::strerror(errno));
  page_ = static_cast<Page*>(p);
  if (create) {
    // a fresh segment is zero-filled; record the world so openers can check it
    page_->world.store((uint64_t)world, std::memory_order_release);
  } else if (page_->world.load(std::memory_order_acquire) != (uint64_t)world) {
    munmap(page_, sizeof(Page));
    page_ = nullptr;
    throw std::runtime_error("ShmBarrier: world size mismatch on " + name);
  }
}

ShmBarrier::~ShmBarrier() {
  if (owner_) unlink();
  if (page_) munmap(page_, sizeof(Page));
}

void ShmBarrier::unlink() {
  if (owner_ && !name_.empty()) {
    shm_unlink(name_.c_str());
    owner_ = false;
  }
}

double ShmBarrier::wait(double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  if (page_->broken.load(std::memory_order_acquire) != 0)
    throw std::runtime_error("ShmBarrier: broken by an earlier timeout (discard it)");
  const uint64_t g = gen_;
  if (page_->count.fetch_add(1, std::memory_order_acq_rel) == (uint64_t)world_ - 1) {
    page_->count.store(0, std::memory_order_relaxed);  // nobody adds again before gen moves
    page_->gen.store(g + 1, std::memory_order_release);
  } else {
    uint64_t spins = 0;
    while (page_->gen.load(std::memory_order_acquire) == g) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
      if ((++spins & 0xffff) == 0) {
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (page_->broken.load(std::memory_order_acquire) != 0)
          throw std::runtime_error("ShmBarrier: broken by another rank's timeout");
        if (el > timeout_s) {
          page_->broken.store(1, std::memory_order_release);
          throw std::runtime_error("ShmBarrier: rank " + std::to_string(rank_) + " timed out after " +
                                   std::to_string(el) + " s (a rank did not arrive)");
        }
        // long waits (a rank still compiling / allocating): give the core back now and then
        if (el > 0.05) std::this_thread::yield();
      }
    }
  }
  gen_ = g + 1;
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace h2d
