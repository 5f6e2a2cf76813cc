// heat2d_amd — output formats (see io.h).
#include "io.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace h2d {

static std::runtime_error io_error(const std::string& what, const std::string& path) {
  return std::runtime_error(what + " '" + path + "': " + std::strerror(errno));
}

void binary_create(const std::string& path, int64_t NX, int64_t NY) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw io_error("cannot create", path);
  if (::ftruncate(fd, (off_t)(NX * NY * (int64_t)sizeof(float))) != 0) {
    ::close(fd);
    throw io_error("cannot size", path);
  }
  ::close(fd);
}

void binary_write_tile(const std::string& path, int64_t NX, int64_t NY, int64_t gx0, int64_t gy0, int64_t xcell,
                       int64_t ycell, const float* data) {
  if (gx0 < 0 || gy0 < 0 || gx0 + xcell > NX || gy0 + ycell > NY) throw std::invalid_argument("tile outside grid");
  const int fd = ::open(path.c_str(), O_WRONLY);
  if (fd < 0) throw io_error("cannot open", path);
  for (int64_t i = 0; i < xcell; ++i) {
    const char* p = reinterpret_cast<const char*>(data + i * ycell);
    size_t left = (size_t)ycell * sizeof(float);
    off_t off = (off_t)(((gx0 + i) * NY + gy0) * (int64_t)sizeof(float));
    while (left > 0) {
      const ssize_t w = ::pwrite(fd, p, left, off);
      if (w < 0) {
        if (errno == EINTR) continue;
        ::close(fd);
        throw io_error("write failed", path);
      }
      p += w;
      off += w;
      left -= (size_t)w;
    }
  }
  ::close(fd);
}

std::vector<float> binary_read(const std::string& path, int64_t NX, int64_t NY) {
  std::vector<float> v((size_t)(NX * NY));
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw io_error("cannot open", path);
  const size_t n = std::fread(v.data(), sizeof(float), v.size(), f);
  std::fclose(f);
  if (n != v.size()) throw std::runtime_error("short read from '" + path + "'");
  return v;
}

std::string format_text(const float* u, int64_t NX, int64_t NY, int style) {
  std::string out;
  out.reserve((size_t)(NX * NY * 8 + NX + NY));
  char buf[64];
  if (style == kTextGrad) {
    for (int64_t i = 0; i < NX; ++i) {
      for (int64_t j = 0; j < NY; ++j) {
        const int n = std::snprintf(buf, sizeof(buf), "%6.1f ", u[i * NY + j]);
        out.append(buf, (size_t)n);
      }
      out.push_back('\n');
    }
  } else {
    for (int64_t iy = NY - 1; iy >= 0; --iy) {
      for (int64_t ix = 0; ix < NX; ++ix) {
        const int n = std::snprintf(buf, sizeof(buf), "%6.1f", u[ix * NY + iy]);
        out.append(buf, (size_t)n);
        out.push_back(ix != NX - 1 ? ' ' : '\n');
      }
    }
  }
  return out;
}

void binary_to_text(const std::string& bin, const std::string& txt, int64_t NX, int64_t NY, int style) {
  std::vector<float> u = binary_read(bin, NX, NY);
  FILE* f = std::fopen(txt.c_str(), "w");
  if (!f) throw io_error("cannot create", txt);
  // Row blocks keep memory bounded for large grids.
  if (style == kTextGrad) {
    const int64_t rows = std::max<int64_t>(1, (int64_t)(1 << 20) / std::max<int64_t>(1, NY));
    for (int64_t i0 = 0; i0 < NX; i0 += rows) {
      const int64_t n = std::min(rows, NX - i0);
      const std::string s = format_text(u.data() + i0 * NY, n, NY, kTextGrad);
      std::fwrite(s.data(), 1, s.size(), f);
    }
  } else {
    const std::string s = format_text(u.data(), NX, NY, kTextHeat2dn);
    std::fwrite(s.data(), 1, s.size(), f);
  }
  if (std::fclose(f) != 0) throw io_error("close failed", txt);
}

}  // namespace h2d
