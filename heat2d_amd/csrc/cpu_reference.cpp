// heat2d_amd — CPU reference path (see cpu_reference.h).  Compiled with -ffp-contract=off.
#include "cpu_reference.h"

#include <algorithm>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <thread>

namespace h2d {

void init_global(std::vector<float>& u, int64_t NX, int64_t NY, int init) {
  u.assign((size_t)(NX * NY), 0.0f);
  for (int64_t ix = 0; ix < NX; ++ix)
    for (int64_t iy = 0; iy < NY; ++iy) u[(size_t)(ix * NY + iy)] = init_value(init, ix, iy, NX, NY);
}

static inline float cell_update(const Physics& ph, float c, float n, float s, float w, float e) {
  if (ph.precision == kFp32) return update_f32(c, n, s, w, e, (float)ph.cx, (float)ph.cy);
  return update_ref(c, n, s, w, e, ph.cx, ph.cy);
}

OracleResult oracle_run(int64_t NX, int64_t NY, int64_t steps, const Physics& ph, int init, bool convergence,
                        int64_t interval, double sensitivity, const float* initial) {
  if (NX < 1 || NY < 1) throw std::invalid_argument("bad grid");
  const bool fixed = ph.boundary == kFixed;
  // Padded copy with a one-cell ring: zero outside the grid, wrapped when periodic.
  const int64_t P = NY + 2;
  std::vector<float> a((size_t)((NX + 2) * P), 0.0f), b((size_t)((NX + 2) * P), 0.0f);
  std::vector<float> g0;
  if (initial) g0.assign(initial, initial + NX * NY);
  else init_global(g0, NX, NY, init);
  for (int64_t i = 0; i < NX; ++i) std::memcpy(&a[(size_t)((i + 1) * P + 1)], &g0[(size_t)(i * NY)], NY * sizeof(float));
  b = a;

  auto fill_ring = [&](std::vector<float>& u) {
    if (ph.periodic_x) {
      std::memcpy(&u[1], &u[(size_t)(NX * P + 1)], NY * sizeof(float));
      std::memcpy(&u[(size_t)((NX + 1) * P + 1)], &u[(size_t)(P + 1)], NY * sizeof(float));
    }
    if (ph.periodic_y) {
      for (int64_t i = 0; i < NX + 2; ++i) {
        u[(size_t)(i * P)] = u[(size_t)(i * P + NY)];
        u[(size_t)(i * P + NY + 1)] = u[(size_t)(i * P + 1)];
      }
    }
  };

  OracleResult res;
  std::vector<float>* cur = &a;
  std::vector<float>* nxt = &b;
  int64_t done = 0;
  // Large grids (the bench's verification of a 4096^2 run) update row blocks on several
  // threads: every cell is independent within a step, so the result is the same bits.
  const int nthreads = NX * NY >= (int64_t)1 << 20
                           ? (int)std::max<unsigned>(1, std::min<unsigned>(16, std::thread::hardware_concurrency()))
                           : 1;
  for (int64_t k = 0; k < steps; ++k) {
    fill_ring(*cur);
    const std::vector<float>& u = *cur;
    std::vector<float>& v = *nxt;
    auto rows = [&](int64_t i0, int64_t i1) {
      for (int64_t i = i0; i < i1; ++i) {
        const int rm = dim_mode(i, NX, ph.periodic_x, fixed);
        for (int64_t j = 0; j < NY; ++j) {
          const int m = std::max(rm, dim_mode(j, NY, ph.periodic_y, fixed));
          const size_t c = (size_t)((i + 1) * P + (j + 1));
          if (m == 0) v[c] = cell_update(ph, u[c], u[c - P], u[c + P], u[c - 1], u[c + 1]);
          else v[c] = u[c];
        }
      }
    };
    if (nthreads > 1) {
      std::vector<std::thread> pool;
      for (int t = 0; t < nthreads; ++t) pool.emplace_back(rows, NX * t / nthreads, NX * (t + 1) / nthreads);
      for (auto& th : pool) th.join();
    } else {
      rows(0, NX);
    }
    const int64_t committed = k + 1;
    if (convergence && interval > 0 && committed % interval == 0) {
      double s = 0.0;
      for (int64_t i = 0; i < NX; ++i)
        for (int64_t j = 0; j < NY; ++j) {
          const size_t c = (size_t)((i + 1) * P + (j + 1));
          const double d = (double)v[c] - (double)u[c];
          s += d * d;
        }
      res.residual = s;
      if (s < sensitivity) {
        // Stop; the state after the last *committed* step is the pre-update buffer (the
        // reference breaks before its swap: grad1612_mpi_heat.c:269-273).
        res.converged = true;
        done = k;
        break;
      }
    }
    std::swap(cur, nxt);
    done = k + 1;
  }
  res.steps_done = done;
  res.grid.resize((size_t)(NX * NY));
  for (int64_t i = 0; i < NX; ++i) std::memcpy(&res.grid[(size_t)(i * NY)], &(*cur)[(size_t)((i + 1) * P + 1)], NY * sizeof(float));
  return res;
}

void cpu_tile_init(const TileGeom& g, float* base, int init) {
  std::fill(base, base + g.elems(), 0.0f);
  for (int64_t i = 0; i < g.xcell; ++i)
    for (int64_t j = 0; j < g.ycell; ++j) base[g.idx(i, j)] = init_value(init, g.gx0 + i, g.gy0 + j, g.NX, g.NY);
}

double cpu_tile_advance(const TileGeom& g, const Physics& ph, const float* src, float* dst, int K, float* scratch0,
                        float* scratch1, bool residual) {
  if (K < 1 || K > g.G) throw std::invalid_argument("cpu_tile_advance: bad K");
  const bool fixed = ph.boundary == kFixed;
  const float* in = src;
  double rsum = 0.0;
  for (int t = 1; t <= K; ++t) {
    const int64_t m = K - t;  // margin still needed around the owned block
    float* out = (t == K) ? dst : ((t & 1) ? scratch0 : scratch1);
    const int64_t r0 = (t == K) ? 0 : -m, r1 = (t == K) ? g.xcell : g.xcell + m;
    const int64_t c0 = (t == K) ? 0 : -m, c1 = (t == K) ? g.ycell : g.ycell + m;
    for (int64_t i = r0; i < r1; ++i) {
      const int rm = dim_mode(g.gx0 + i, g.NX, ph.periodic_x, fixed);
      for (int64_t j = c0; j < c1; ++j) {
        const int mode = std::max(rm, dim_mode(g.gy0 + j, g.NY, ph.periodic_y, fixed));
        const int64_t c = g.idx(i, j);
        float v;
        if (mode == 2) v = 0.0f;
        else if (mode == 1) v = in[c];
        else v = cell_update(ph, in[c], in[c - g.pitch], in[c + g.pitch], in[c - 1], in[c + 1]);
        out[c] = v;
        if (t == K && residual) {
          const double d = (double)v - (double)in[c];
          rsum += d * d;
        }
      }
    }
    in = out;
  }
  return rsum;
}

void cpu_tile_poison(const TileGeom& g, float* base, bool fixed, bool per_x, bool per_y) {
  const float nan = std::numeric_limits<float>::quiet_NaN();
  for (int64_t e = 0; e < g.elems(); ++e) {
    const int64_t i = e / g.pitch - g.G, j = e % g.pitch - g.PL;
    if (poisonable(g, i, j, fixed, per_x, per_y)) base[e] = nan;
  }
}

void cpu_copy_rects(const std::vector<CopyDesc>& descs) {
  for (const CopyDesc& d : descs)
    for (int64_t r = 0; r < d.rows; ++r)
      std::memmove(d.dst + r * d.dst_pitch, d.src + r * d.src_pitch, (size_t)d.cols * sizeof(float));
}

}  // namespace h2d
