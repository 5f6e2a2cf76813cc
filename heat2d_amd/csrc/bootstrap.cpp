// heat2d_amd — native multi-process bootstrap (see bootstrap.h).
#include "bootstrap.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace h2d {

namespace {

void send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) throw std::runtime_error("bootstrap: send failed (peer gone?)");
    c += k;
    n -= (size_t)k;
  }
}

void recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n > 0) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK))
      throw std::runtime_error("bootstrap: receive timed out (a peer stopped taking part)");
    if (k <= 0) throw std::runtime_error("bootstrap: receive failed (peer gone?)");
    c += k;
    n -= (size_t)k;
  }
}

// Bound every later receive on fd (SO_RCVTIMEO): a hung peer fails the collective instead of
// blocking this rank forever.
void recv_timeout(int fd, double s) {
  timeval tv{};
  tv.tv_sec = (time_t)s;
  tv.tv_usec = (suseconds_t)((s - (double)tv.tv_sec) * 1e6);
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

template <class TP>
double remaining(TP deadline) {
  return std::chrono::duration<double>(deadline - std::chrono::steady_clock::now()).count();
}

void send_blob(int fd, const std::string& s) {
  const uint64_t n = s.size();
  send_all(fd, &n, sizeof(n));
  if (n) send_all(fd, s.data(), n);
}

std::string recv_blob(int fd) {
  uint64_t n = 0;
  recv_all(fd, &n, sizeof(n));
  if (n > (uint64_t)1 << 34) throw std::runtime_error("bootstrap: oversized message");
  std::string s(n, '\0');
  if (n) recv_all(fd, &s[0], n);
  return s;
}

std::string pack_list(const std::vector<std::string>& v) {
  std::string out;
  for (const auto& s : v) {
    const uint64_t n = s.size();
    out.append(reinterpret_cast<const char*>(&n), sizeof(n));
    out += s;
  }
  return out;
}

std::vector<std::string> unpack_list(const std::string& b, size_t count) {
  std::vector<std::string> v;
  size_t off = 0;
  for (size_t i = 0; i < count; ++i) {
    uint64_t n = 0;
    if (off + sizeof(n) > b.size()) throw std::runtime_error("bootstrap: truncated list");
    std::memcpy(&n, b.data() + off, sizeof(n));
    off += sizeof(n);
    if (off + n > b.size()) throw std::runtime_error("bootstrap: truncated list");
    v.emplace_back(b.data() + off, n);
    off += n;
  }
  return v;
}

void nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

}  // namespace

RankEnv rank_env() {
  RankEnv e;
  auto geti = [](const char* k, int d) {
    const char* v = std::getenv(k);
    return v ? std::atoi(v) : d;
  };
  e.rank = geti("RANK", 0);
  e.world = geti("WORLD_SIZE", 1);
  e.local_rank = geti("LOCAL_RANK", e.rank);
  if (const char* a = std::getenv("MASTER_ADDR")) e.addr = a;
  e.port = geti("HEAT2D_BOOT_PORT", geti("MASTER_PORT", 29500) + 7);
  return e;
}

Bootstrap::Bootstrap(int rank, int world, const std::string& addr, int port, double timeout_s,
                     double io_timeout_s)
    : rank_(rank), world_(world) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("bootstrap: bad rank / world size");
  if (world == 1) return;
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, addr.c_str(), &sa.sin_addr) != 1) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(addr.c_str(), nullptr, &hints, &res) != 0 || !res)
      throw std::runtime_error("bootstrap: cannot resolve " + addr);
    sa.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  if (const char* v = std::getenv("HEAT2D_BOOT_IO_TIMEOUT_S")) io_timeout_s = std::atof(v);
  if (rank == 0) {
    const char* inherited = std::getenv("HEAT2D_BOOT_LISTEN_FD");
    if (inherited != nullptr) {
      listen_fd_ = std::atoi(inherited);  // bound and listening (heat2d --np)
    } else {
      // no SO_REUSEADDR: a second job on the same port fails here instead of pairing ranks
      listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
      if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0)
        throw std::runtime_error("bootstrap: rank 0 cannot bind port " + std::to_string(port) + " (in use?)");
      ::listen(listen_fd_, world);
    }
    fds_.assign(world, -1);
    for (int i = 1; i < world; ++i) {
      pollfd pf{listen_fd_, POLLIN, 0};
      const double left = remaining(deadline);
      if (left <= 0 || ::poll(&pf, 1, (int)(left * 1000.0) + 1) <= 0)
        throw std::runtime_error("bootstrap: rank 0 timed out waiting for " + std::to_string(world - i) +
                                 " rank(s) to connect");
      const int fd = ::accept(listen_fd_, nullptr, nullptr);
      if (fd < 0) throw std::runtime_error("bootstrap: accept failed");
      nodelay(fd);
      recv_timeout(fd, std::max(1.0, remaining(deadline)));
      int32_t r = -1;
      recv_all(fd, &r, sizeof(r));
      if (r <= 0 || r >= world || fds_[r] >= 0) throw std::runtime_error("bootstrap: bad peer rank");
      fds_[r] = fd;
    }
    for (int r = 1; r < world; ++r) recv_timeout(fds_[r], io_timeout_s);
  } else {
    if (const char* inherited = std::getenv("HEAT2D_BOOT_LISTEN_FD")) ::close(std::atoi(inherited));
    int fd = -1;
    for (;;) {
      fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0) break;
      ::close(fd);
      if (std::chrono::steady_clock::now() > deadline)
        throw std::runtime_error("bootstrap: rank " + std::to_string(rank) + " cannot reach rank 0 at " + addr + ":" +
                                 std::to_string(port));
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    nodelay(fd);
    recv_timeout(fd, io_timeout_s);
    const int32_t r = rank;
    send_all(fd, &r, sizeof(r));
    fds_.assign(1, fd);
  }
}

Bootstrap::~Bootstrap() {
  for (int fd : fds_)
    if (fd >= 0) ::close(fd);
  if (listen_fd_ >= 0) ::close(listen_fd_);
}

std::vector<std::string> Bootstrap::allgather(const std::string& mine) {
  if (world_ == 1) return {mine};
  if (rank_ == 0) {
    std::vector<std::string> all(world_);
    all[0] = mine;
    for (int r = 1; r < world_; ++r) all[r] = recv_blob(fds_[r]);
    const std::string packed = pack_list(all);
    for (int r = 1; r < world_; ++r) send_blob(fds_[r], packed);
    return all;
  }
  send_blob(fds_[0], mine);
  return unpack_list(recv_blob(fds_[0]), (size_t)world_);
}

std::string Bootstrap::broadcast(const std::string& data, int root) {
  return allgather(rank_ == root ? data : std::string()).at(root);
}

void Bootstrap::barrier() { (void)allgather(std::string()); }

namespace {
std::string dbl(double x) { return std::string(reinterpret_cast<const char*>(&x), sizeof(x)); }
double undbl(const std::string& s) {
  double x = 0;
  std::memcpy(&x, s.data(), sizeof(x));
  return x;
}
}  // namespace

double Bootstrap::allreduce_max(double x) {
  double m = x;
  for (auto& s : allgather(dbl(x))) m = std::max(m, undbl(s));
  return m;
}

double Bootstrap::allreduce_min(double x) {
  double m = x;
  for (auto& s : allgather(dbl(x))) m = std::min(m, undbl(s));
  return m;
}

double Bootstrap::allreduce_sum(double x) {
  double m = 0.0;  // rank order: the same bits on every rank
  for (auto& s : allgather(dbl(x))) m += undbl(s);
  return m;
}

std::map<std::pair<int, int>, std::string> Bootstrap::exchange(const std::vector<Msg>& out) {
  // every rank's outgoing messages go to everyone through rank 0's star (allgather) and each
  // keeps those addressed to it: the CPU test path of the native multi-rank program, not a
  // fast transport (GPUs use the IPC or RCCL data planes)
  std::vector<std::string> v;
  for (const Msg& m : out) {
    int hdr[2] = {m.dst, m.tag};
    v.push_back(std::string(reinterpret_cast<const char*>(hdr), sizeof(hdr)));
    v.push_back(m.data);
  }
  const std::vector<std::string> all = allgather(dbl((double)v.size()) + pack_list(v));
  std::map<std::pair<int, int>, std::string> in;
  for (int src = 0; src < world_; ++src) {
    const std::string& b = all[src];
    const size_t n = (size_t)undbl(b.substr(0, sizeof(double)));
    const std::vector<std::string> items = unpack_list(b.substr(sizeof(double)), n);
    for (size_t i = 0; i + 1 < items.size(); i += 2) {
      int hdr[2];
      std::memcpy(hdr, items[i].data(), sizeof(hdr));
      if (hdr[0] == rank_) in[std::make_pair(src, hdr[1])] = items[i + 1];
    }
  }
  return in;
}

}  // namespace h2d
