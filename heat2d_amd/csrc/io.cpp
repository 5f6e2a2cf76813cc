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

namespace {
// Read `n` floats at element offset `e` of the raw file.
void pread_floats(int fd, float* dst, int64_t n, int64_t e, const std::string& path) {
  char* p = reinterpret_cast<char*>(dst);
  size_t left = (size_t)n * sizeof(float);
  off_t off = (off_t)(e * (int64_t)sizeof(float));
  while (left > 0) {
    const ssize_t r = ::pread(fd, p, left, off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) throw std::runtime_error("short read from '" + path + "'");
    p += r;
    off += r;
    left -= (size_t)r;
  }
}
}  // namespace

void binary_to_text(const std::string& bin, const std::string& txt, int64_t NX, int64_t NY, int style) {
  // Streamed from the file in blocks of about 1 Mi floats: memory stays bounded however large
  // the grid (a 16384^2 grid is 1 GiB raw).
  const int fd = ::open(bin.c_str(), O_RDONLY);
  if (fd < 0) throw io_error("cannot open", bin);
  FILE* f = std::fopen(txt.c_str(), "w");
  if (!f) {
    ::close(fd);
    throw io_error("cannot create", txt);
  }
  const int64_t budget = (int64_t)1 << 20;
  std::vector<float> blk;
  try {
    if (style == kTextGrad) {
      // row-major: blocks of whole rows
      const int64_t rows = std::max<int64_t>(1, budget / std::max<int64_t>(1, NY));
      blk.resize((size_t)(rows * NY));
      for (int64_t i0 = 0; i0 < NX; i0 += rows) {
        const int64_t n = std::min(rows, NX - i0);
        pread_floats(fd, blk.data(), n * NY, i0 * NY, bin);
        const std::string s = format_text(blk.data(), n, NY, kTextGrad);
        std::fwrite(s.data(), 1, s.size(), f);
      }
    } else {
      // transposed (line = one column iy, from NY-1 down): blocks of B columns, each read as
      // NX row segments; the block is kept as an NX x B grid and printed column by column
      const int64_t B = std::max<int64_t>(1, std::min<int64_t>(NY, budget / std::max<int64_t>(1, NX)));
      blk.resize((size_t)(NX * B));
      std::string line;
      char buf[64];
      for (int64_t hi = NY; hi > 0; hi -= B) {
        const int64_t lo = std::max<int64_t>(0, hi - B), w = hi - lo;
        for (int64_t ix = 0; ix < NX; ++ix) pread_floats(fd, blk.data() + ix * w, w, ix * NY + lo, bin);
        for (int64_t c = w - 1; c >= 0; --c) {
          line.clear();
          for (int64_t ix = 0; ix < NX; ++ix) {
            const int k = std::snprintf(buf, sizeof(buf), "%6.1f", blk[(size_t)(ix * w + c)]);
            line.append(buf, (size_t)k);
            line.push_back(ix != NX - 1 ? ' ' : '\n');
          }
          std::fwrite(line.data(), 1, line.size(), f);
        }
      }
    }
  } catch (...) {
    std::fclose(f);
    ::close(fd);
    throw;
  }
  ::close(fd);
  if (std::fclose(f) != 0) throw io_error("close failed", txt);
}

}  // namespace h2d
