// heat2d_amd — domain decomposition and halo-exchange plans (see decomposition.h).
#include "decomposition.h"

#include <algorithm>
#include <sstream>
#include <stdexcept>

namespace h2d {

static void split_even(int64_t n, int parts, std::vector<int64_t>& start, std::vector<int64_t>& count) {
  // Same distribution as mpi_heat2Dn.c:87-93: averow = n/parts, the first `extra` get +1.
  start.assign(parts, 0);
  count.assign(parts, 0);
  const int64_t ave = n / parts, extra = n % parts;
  int64_t off = 0;
  for (int i = 0; i < parts; ++i) {
    count[i] = ave + (i < extra ? 1 : 0);
    start[i] = off;
    off += count[i];
  }
}

Decomposition::Decomposition(int64_t nx, int64_t ny, int gx, int gy, bool px, bool py)
    : NX(nx), NY(ny), gridx(gx), gridy(gy), periodic_x(px), periodic_y(py) {
  if (nx < 1 || ny < 1) throw std::invalid_argument("grid must be at least 1x1");
  if (gx < 1 || gy < 1) throw std::invalid_argument("gridx/gridy must be >= 1");
  if (gx > nx || gy > ny) throw std::invalid_argument("more blocks than rows/columns");
  split_even(nx, gx, xstart, xcount);
  split_even(ny, gy, ystart, ycount);
}

int Decomposition::neighbor(int rank, int d) const {
  int px = px_of(rank) + kDirDx[d];
  int py = py_of(rank) + kDirDy[d];
  if (px < 0 || px >= gridx) {
    if (!periodic_x) return -1;
    px = (px + gridx) % gridx;
  }
  if (py < 0 || py >= gridy) {
    if (!periodic_y) return -1;
    py = (py + gridy) % gridy;
  }
  return rank_of(px, py);
}

int64_t Decomposition::min_extent_x() const { return *std::min_element(xcount.begin(), xcount.end()); }
int64_t Decomposition::min_extent_y() const { return *std::min_element(ycount.begin(), ycount.end()); }

int64_t Decomposition::max_halo_depth() const {
  int64_t d = INT64_MAX;
  if (gridx > 1 || periodic_x) d = std::min(d, min_extent_x());
  if (gridy > 1 || periodic_y) d = std::min(d, min_extent_y());
  return d;
}

TileGeom make_tile_geom(int64_t NX, int64_t NY, int64_t gx0, int64_t gy0, int64_t xcell, int64_t ycell,
                        int64_t G) {
  TileGeom g;
  g.NX = NX;
  g.NY = NY;
  g.gx0 = gx0;
  g.gy0 = gy0;
  g.xcell = xcell;
  g.ycell = ycell;
  g.G = G;
  // Column lead of the streaming kernel is round_up(K,4) <= round_up(G,4).
  g.PL = std::max<int64_t>(4, (G + 3) & ~int64_t(3));
  const int64_t R = g.PL;
  // Strips of the widest kernel we may launch (smallest K=1 has the widest output strip,
  // largest K the most strips): size the pitch for the worst case over K in [1, G].
  // owned + right ghost; an edge-aligned last strip's window ends at round_up(ycell, 4)
  int64_t need = g.PL + std::max(ycell + G, (ycell + 3) & ~int64_t(3));
  for (int64_t K = 1; K <= std::max<int64_t>(1, G); ++K) {
    const int64_t r = lead_cols((int)K);
    const int64_t wout = kWaveCols - 2 * r;
    const int64_t nstrips = (ycell + wout - 1) / wout;
    const int64_t last_end = g.PL + (nstrips - 1) * wout - r + kWaveCols;
    need = std::max(need, last_end);
  }
  (void)R;
  g.pitch = (need + 63) & ~int64_t(63);
  g.srows = xcell + 2 * G;
  return g;
}

TileGeom Decomposition::tile(int rank, int64_t G) const {
  const int px = px_of(rank), py = py_of(rank);
  return make_tile_geom(NX, NY, xstart[px], ystart[py], xcount[px], ycount[py], G);
}

ExchangePlan make_plan(const Decomposition& dec, int rank, const TileGeom& g, int K) {
  if (K > g.G) throw std::invalid_argument("halo depth exceeds ghost depth");
  ExchangePlan p;
  p.K = K;
  int64_t soff = 0, roff = 0;
  for (int d = 0; d < kNumDirs; ++d) {
    p.peer[d] = dec.neighbor(rank, d);
    Rect s, r;
    const int dx = kDirDx[d], dy = kDirDy[d];
    // rows
    if (dx < 0) { s.r0 = 0; s.rows = K; r.r0 = -K; r.rows = K; }
    else if (dx > 0) { s.r0 = g.xcell - K; s.rows = K; r.r0 = g.xcell; r.rows = K; }
    else { s.r0 = 0; s.rows = g.xcell; r.r0 = 0; r.rows = g.xcell; }
    // cols
    if (dy < 0) { s.c0 = 0; s.cols = K; r.c0 = -K; r.cols = K; }
    else if (dy > 0) { s.c0 = g.ycell - K; s.cols = K; r.c0 = g.ycell; r.cols = K; }
    else { s.c0 = 0; s.cols = g.ycell; r.c0 = 0; r.cols = g.ycell; }
    if (p.peer[d] < 0 || K == 0) { s.rows = s.cols = 0; r.rows = r.cols = 0; }
    p.send_rect[d] = s;
    p.recv_rect[d] = r;
    p.send_off[d] = soff;
    p.recv_off[d] = roff;
    soff += s.count();
    roff += r.count();
  }
  p.send_total = soff;
  p.recv_total = roff;
  return p;
}

void plan_pack_descs(const ExchangePlan& p, const TileGeom& g, const float* base, float* sendbuf,
                     std::vector<CopyDesc>& out) {
  for (int d = 0; d < kNumDirs; ++d) {
    const Rect& s = p.send_rect[d];
    if (s.count() == 0) continue;
    out.push_back(CopyDesc{base + g.idx(s.r0, s.c0), sendbuf + p.send_off[d], g.pitch, s.cols, s.rows, s.cols});
  }
}

void plan_unpack_descs(const ExchangePlan& p, const TileGeom& g, float* base, const float* recvbuf,
                       std::vector<CopyDesc>& out) {
  for (int d = 0; d < kNumDirs; ++d) {
    const Rect& r = p.recv_rect[d];
    if (r.count() == 0) continue;
    out.push_back(CopyDesc{recvbuf + p.recv_off[d], base + g.idx(r.r0, r.c0), r.cols, g.pitch, r.rows, r.cols});
  }
}

std::string describe(const Decomposition& d) {
  std::ostringstream os;
  os << d.NX << "x" << d.NY << " on " << d.gridx << "x" << d.gridy << " blocks";
  if (d.periodic_x || d.periodic_y) os << " (periodic " << (d.periodic_x ? "x" : "") << (d.periodic_y ? "y" : "") << ")";
  return os.str();
}

}  // namespace h2d
