// heat2d_amd — LDS-tiled, temporally-blocked stencil for small and medium grids (gfx950).
//
// The streaming kernel (stream_kernel.hpp) parallelises over 256-column strips and walks
// rows; on grids of 10^4..10^6 cells (the reference's whole measured table, Report.pdf p.21,
// p.26: 80x64 .. 1280x1024) that leaves most of the 1024 SIMDs idle or the waves latency
// bound.  This kernel parallelises over 2-D tiles instead:
//   * one workgroup (NT = 256 or 1024 threads) owns a TX x TY tile; it loads the tile plus a k-deep halo
//     (region (TX+2k) x RY, RY = TY+2k = 32, 64 or 128 columns) into LDS once per launch;
//   * it advances k time steps inside LDS (ping-pong buffers, one barrier per step); a level is
//     (RX - 2t) rows of RY/4 column groups, swept NT/(RY/4) rows at a time, so the 1024-thread
//     variant covers a small tile's level in one sweep (shorter serial chain per launch: the
//     small-grid latency floor) and the 256-thread one keeps 4 workgroups per CU on bigger grids;
//     recomputing the halo redundantly (overlapped tiling: no inter-workgroup exchange);
//   * each thread owns a fixed 4-column group and strides over rows: three float4 LDS reads
//     (rows r-1, r, r+1), the west / east neighbours from the adjacent lanes (DPP), one float4
//     store — the streaming kernel's row_update (packed fp32 pair sums, fp32 packed FMAs); cells outside the shrinking valid region are computed on stale data
//     but never feed a valid cell (dependency cone), so no per-cell range test is needed;
//   * global edges: fixed edges hold, the ghost-zero ring stays 0, periodic dims wrap on load;
//   * the owned tile is written back once per k steps; one launch per chunk (~1.5 us kernel
//     boundary on gfx950, cheaper than any in-kernel grid barrier).
// The tile -> workgroup map keeps neighbouring tiles on one XCD (blocks are dealt round-robin
// over the 8 XCDs) so their shared halo rows hit the same L2.
// Numerics: the same cell() as the streaming kernel (bit-exact ref path / fp32 FMA path).
// Compiled with -ffp-contract=off.
#include <type_traits>
#include "stream_kernel.hpp"
#include "tile_kernel.h"

namespace h2d {
namespace {

__device__ unsigned long long g_tile_zero_word = 0ull;  // the stop word of launches without one

__device__ __forceinline__ int wrap_idx(int i, int n) {
  i %= n;
  return i < 0 ? i + n : i;
}

// CPL consecutive cells of one LDS row <-> registers (ds_read/write_b32 / b64 / b128)
template <int CPL>
__device__ __forceinline__ void lds_get(const float* p, float (&v)[CPL]) {
  if constexpr (CPL == 4) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w;
  } else if constexpr (CPL == 2) {
    const f32x2 x = *reinterpret_cast<const f32x2*>(p);
    v[0] = x.x, v[1] = x.y;
  } else {
    v[0] = *p;
  }
}
template <int CPL>
__device__ __forceinline__ void lds_put(float* p, const float (&v)[CPL]) {
  if constexpr (CPL == 4) *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  else if constexpr (CPL == 2) *reinterpret_cast<f32x2*>(p) = f32x2{v[0], v[1]};
  else *p = v[0];
}

// One time level of a lane's CPL cells from rows r-1 (N), r (C), r+1 (S).  The west / east
// neighbours of the group are the adjacent lanes' last / first cell (DPP wave shifts: a region
// row is RY/CPL consecutive lanes of one wave); the first / last lane of a row reads another
// row's value or 0, which only reaches region columns 0 / RY-1 — outside the valid cone from
// level 1 on.  Same values as update_ref / update_f32 (fp32 adds are commutative).
template <bool F32, int CPL>
__device__ __forceinline__ void group_update(const float (&N)[CPL], const float (&C)[CPL], const float (&S)[CPL],
                                             float (&o)[CPL], const Coef& k) {
  if constexpr (CPL == 4) {
    const float4 r = row_update<F32>(make_float4(N[0], N[1], N[2], N[3]), make_float4(C[0], C[1], C[2], C[3]),
                                     make_float4(S[0], S[1], S[2], S[3]), k);
    o[0] = r.x, o[1] = r.y, o[2] = r.z, o[3] = r.w;
  } else if constexpr (CPL == 2) {
    const f32x2 sn = f32x2{N[0], N[1]} + f32x2{S[0], S[1]};
    const float ew0 = from_left(C[1]) + C[1];
    const float ew1 = C[0] + from_right(C[0]);
    if constexpr (F32) {
      const f32x2 c01 = {C[0], C[1]}, ew01 = {ew0, ew1};
      const f32x2 m2 = {-2.0f, -2.0f}, cx2 = {k.cxf, k.cxf}, cy2 = {k.cyf, k.cyf};
      f32x2 r = __builtin_elementwise_fma(cx2, __builtin_elementwise_fma(m2, c01, sn), c01);
      r = __builtin_elementwise_fma(cy2, __builtin_elementwise_fma(m2, c01, ew01), r);
      o[0] = r.x, o[1] = r.y;
    } else {
      o[0] = cell<F32>(C[0], sn.x, ew0, k);
      o[1] = cell<F32>(C[1], sn.y, ew1, k);
    }
  } else {
    o[0] = cell<F32>(C[0], N[0] + S[0], from_left(C[0]) + from_right(C[0]), k);
  }
}

template <bool F32, bool RESID, int RY, int NT, int CPL>
__global__ __launch_bounds__(NT) void tile_lds_kernel(const TileArgs* __restrict__ ap, unsigned long long seq,
                                                      unsigned long long pend_seq, unsigned btag) {
  // (per-launch values read once, up front: see stream_kernel)
  asm volatile("" : "+s"(seq), "+s"(pend_seq), "+s"(btag));
  TileDyn d;
  d.seq = seq;
  d.pend_seq = pend_seq;
  d.btag = btag;
  const TileArgs& a = *ap;  // immutable device-resident block
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  constexpr int G = RY / CPL;         // lanes per region row (a row stays inside one wave)
  static_assert(G <= 64 && NT % G == 0, "a region row must fit one wave");
  constexpr int W = RY;               // LDS row pitch: RY % 64 == 0 or RY == 32 keeps the
                                      // ds_read_b128 lane groups of rows r, r+1 conflict-free
  constexpr int RSTEP = NT / G;       // rows per sweep of the workgroup
  constexpr int MJ = kTileMaxSweeps;  // rows per lane (region rows <= MJ·RSTEP)
  const int tid = threadIdx.x;
  const int K = a.K;
  const int RX = a.TX + 2 * K;
  // XCD-aware tile order: block b runs on XCD b % 8; give each XCD a contiguous tile range.
  // Every kernel argument is read before the first branch (one batch of scalar loads, not a
  // round trip per early-exit test), and the stop word's load overlaps the region loads.
  const int nt = a.ntiles;
  int b = blockIdx.x;
  if (nt % 8 == 0) b = (b & 7) * (nt >> 3) + (b >> 3);
  const int bx = b / a.tiles_y, by = b - bx * a.tiles_y;
  const int x0 = bx * a.TX - K;  // global row of region row 0
  const int y0 = by * a.TY - K;  // global column of region column 0
  const bool live = (int)blockIdx.x < nt;  // ntiles == 0: a no-op launch (warm_tile_kernels)
  if (a.head.btag != d.btag) {  // a block the launch does not name: compute nothing (the host sees
    return;                      // the unconverged decision record; never seen in practice)
  }
  if (!live) {
    // the deciding block (grid = ntiles + 1 when `pend`): the previous check's decision, off the
    // tile blocks' critical path (they compute speculatively, see TileArgs::pend)
    if ((int)blockIdx.x == nt && nt > 0 && gp(a.pend) != nullptr && tid < 64)
      decide_pending(a.pend, a.pend_n, a.pend_dec, d.pend_seq, tid);
    return;
  }
  // unconditional load (a dummy zero word without a stop word): no branch, so no wait here
  const unsigned long long stopped =
      __hip_atomic_load(gp(a.stop) != nullptr ? gp(a.stop) : &g_tile_zero_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float* cur = lds;
  float* nxt = lds + RX * W;

  // ---- load the region (zero outside a non-periodic grid); LB loads in flight per thread
  // before the LDS stores wait on them (one global round trip per LB·NT cells, not per NT) ----
  constexpr int LB = 4;
  const int total = RX * RY;
  for (int e0 = tid; e0 < total; e0 += LB * NT) {
    float v[LB];
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int e = e0 + u * NT;
      v[u] = 0.0f;
      if (e < total) {
        const int r = e / RY, c = e - r * RY;
        int gr = x0 + r, gc = y0 + c;
        bool in = true;
        if (a.per_x) gr = wrap_idx(gr, a.NX);
        else in = gr >= 0 && gr < a.NX;
        if (a.per_y) gc = wrap_idx(gc, a.NY);
        else in = in && gc >= 0 && gc < a.NY;
        if (in) v[u] = gp(a.src)[(int64_t)gr * a.pitch + gc];
      }
    }
#pragma unroll
    for (int u = 0; u < LB; ++u)
      if (e0 + u * NT < total) cur[e0 + u * NT] = v[u];  // W == RY: region element e lives at cur[e]
  }
  // converged earlier (set by an earlier launch's deciding block, or during this launch by its
  // own: then this launch's output is discarded anyway)
  if (stopped != 0ull) return;

  // ---- per-thread column group and its edge masks (fixed: hold, ghost-zero: zero) ----
  const int q = tid % G;
  const int r_off = tid / G;
  const int gc0 = y0 + CPL * q;
  unsigned cmask = 0;
  if (!a.per_y) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int gc = gc0 + j;
      const bool m = a.fixed ? (gc == 0 || gc == a.NY - 1) : (gc < 0 || gc >= a.NY);
      cmask |= (m ? 1u : 0u) << j;
    }
  }
  // residual: owned, in-grid columns of this group
  unsigned own = 0;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = CPL * q + j;
    const bool o = c >= K && c < K + a.TY && (by * a.TY + (c - K)) < a.NY;
    own |= (o ? 1u : 0u) << j;
  }
  const Coef k{a.cx, a.cy, (float)a.cx, (float)a.cy};
  double racc = 0.0;
  __syncthreads();

  // ---- this lane's rows r_j = r_off + j·RSTEP (j < MJ) stay fixed for the whole launch: their
  // cells live in registers across levels (only rows r±1 are read from LDS), and their edge
  // masks are computed once.  Rows outside the level's valid range [t, RX-t) are skipped. ----
  const bool fixedb = a.fixed != 0;
  float Cr[MJ][CPL];
  unsigned mk[MJ];
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int r = r_off + j * RSTEP;
    mk[j] = 0u;
    if (j * RSTEP >= RX) break;  // uniform: no lane has a j-th row
    if (r < RX) {
      lds_get<CPL>(cur + r * W + CPL * q, Cr[j]);
      const int gr = x0 + r;
      bool rm = false;
      if (!a.per_x) rm = fixedb ? (gr == 0 || gr == a.NX - 1) : (gr < 0 || gr >= a.NX);
      mk[j] = rm ? ((1u << CPL) - 1u) : cmask;
    }
  }

  const int rlev = a.rlev > 0 ? a.rlev : K;
  // One level of the region; the residual's level (the check step of the chunk) is its own
  // instance, so the other levels' loop carries no residual test (a RESID launch took 11.6 us
  // against 8.3 for the plain one at 80x64, K=14, before the split).
  auto level = [&](int t, auto resid) {
    constexpr bool R = decltype(resid)::value;
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      if (j * RSTEP >= RX - t) break;  // uniform: no lane has a j-th row at this level
      const int r = r_off + j * RSTEP;
      if (r >= t && r < RX - t) {
        float N[CPL], S[CPL], o[CPL];
        lds_get<CPL>(cur + (r - 1) * W + CPL * q, N);
        lds_get<CPL>(cur + (r + 1) * W + CPL * q, S);
        group_update<F32, CPL>(N, Cr[j], S, o, k);
        if (mk[j] != 0u) {  // global edge cells: fixed -> hold, ghost-zero -> stay 0
#pragma unroll
          for (int c = 0; c < CPL; ++c)
            if (mk[j] & (1u << c)) o[c] = fixedb ? Cr[j][c] : 0.0f;
        }
        lds_put<CPL>(nxt + r * W + CPL * q, o);
        if constexpr (R) {
          if (r >= K && r < K + a.TX && bx * a.TX + (r - K) < a.NX) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) racc += (own & (1u << c)) ? sq_diff(o[c], Cr[j][c]) : 0.0;
          }
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) Cr[j][c] = o[c];
      }
    }
    __syncthreads();
    float* tmp = cur;
    cur = nxt;
    nxt = tmp;
  };
  const int plain_end = RESID ? rlev - 1 : K;
  for (int t = 1; t <= plain_end; ++t) level(t, std::false_type{});
  if constexpr (RESID) {
    level(rlev, std::true_type{});
    for (int t = rlev + 1; t <= K; ++t) level(t, std::false_type{});
  }

  // ---- the owned tile, then the residual partial (its reduction overlaps the write-back's
  // stores; with a ticket the last block also decides) ----
  const int xs = bx * a.TX, ys = by * a.TY;
  for (int e = tid; e < a.TX * a.TY; e += NT) {
    const int i = e / a.TY, j = e - i * a.TY;
    if (xs + i < a.NX && ys + j < a.NY) {
      gp(a.dst)[(int64_t)(xs + i) * a.pitch + (ys + j)] = cur[(K + i) * W + K + j];
      // after the final swap `nxt` holds level K-1
      if (RESID && gp(a.keep) != nullptr) gp(a.keep)[(int64_t)(xs + i) * a.pitch + (ys + j)] = nxt[(K + i) * W + K + j];
    }
  }
  if constexpr (RESID) {
    constexpr int NW = NT / 64;
    __shared__ double part[NW];
    racc = dpp_wave_sum(racc);
    if ((tid & 63) == 0) part[tid >> 6] = racc;
    __syncthreads();
    if (tid < 64) {
      double tot = part[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) tot += part[w];
      DecideArgs dec = a.dec;
      dec.seq = d.seq;
      publish_partial(gp(a.partials), blockIdx.x, tot, a.ntiles, dec, tid);
    }
  }
}

// host: the launch's configuration (template dispatch, grid); blk / d: the kernel's arguments
struct TileLaunch {
  const TileArgs* blk;
  const TileArgs& host;
  const TileDyn& d;
};

template <bool F32, bool RESID, int NT, int CPL>
void launch_cpl(const TileLaunch& L, size_t lds, hipStream_t s) {
  const TileArgs& a = L.host;
  // ntiles == 0: no-op launch (warm_kernels); a pending decision: one more (deciding) block
  const dim3 grid((unsigned)std::max(1, a.ntiles + (a.pend != nullptr && a.ntiles > 0 ? 1 : 0))), block(NT);
  if (a.RY == 32) hipLaunchKernelGGL((tile_lds_kernel<F32, RESID, 32, NT, CPL>), grid, block, lds, s, L.blk, L.d.seq, L.d.pend_seq, L.d.btag);
  else if (a.RY == 64) hipLaunchKernelGGL((tile_lds_kernel<F32, RESID, 64, NT, CPL>), grid, block, lds, s, L.blk, L.d.seq, L.d.pend_seq, L.d.btag);
  else if constexpr (CPL >= 2)
    hipLaunchKernelGGL((tile_lds_kernel<F32, RESID, 128, NT, CPL>), grid, block, lds, s, L.blk, L.d.seq, L.d.pend_seq, L.d.btag);
}

template <bool F32, bool RESID, int NT>
void launch_nt(const TileLaunch& L, size_t lds, hipStream_t s) {
  if (L.host.CPL == 1) launch_cpl<F32, RESID, NT, 1>(L, lds, s);
  else if (L.host.CPL == 2) launch_cpl<F32, RESID, NT, 2>(L, lds, s);
  else launch_cpl<F32, RESID, NT, 4>(L, lds, s);
}

template <bool F32, bool RESID>
void launch_ry(const TileLaunch& L, size_t lds, hipStream_t s) {
  if (L.host.NT == 1024) launch_nt<F32, RESID, 1024>(L, lds, s);
  else launch_nt<F32, RESID, 256>(L, lds, s);
}

}  // namespace

size_t tile_lds_bytes(int TX, int RY, int K) { return (size_t)2 * (size_t)(TX + 2 * K) * (size_t)RY * sizeof(float); }

bool tile_config_ok(int TX, int RY, int K, int CPL, int NT) {
  if (!(CPL == 1 || CPL == 2 || CPL == 4) || RY / CPL > 64 || !(NT == 256 || NT == 1024)) return false;
  if (TX + 2 * K > kTileMaxSweeps * (NT / (RY / CPL))) return false;  // every region row has a lane
  return (RY == 32 || RY == 64 || RY == 128) && K >= 1 && RY - 2 * K >= 4 && TX >= 1 && tile_lds_bytes(TX, RY, K) <= 65536;
}

void prepare_tile(TileArgs& a) {
  if (!tile_config_ok(a.TX, a.RY, a.K, a.CPL, a.NT)) throw std::invalid_argument("launch_tile: bad tile configuration");
  if (a.TY != a.RY - 2 * a.K) throw std::invalid_argument("launch_tile: TY must be RY - 2K");
  if (a.rlev < 0 || a.rlev > a.K || (a.rlev != 0 && a.rlev != a.K && a.keep != nullptr))
    throw std::invalid_argument("launch_tile: residual level outside the chunk (or with a rollback copy)");
  if (a.NT != 256 && a.NT != 1024) throw std::invalid_argument("launch_tile: NT must be 256 or 1024");
  a.tiles_y = (a.NY + a.TY - 1) / a.TY;
  a.ntiles = ((a.NX + a.TX - 1) / a.TX) * a.tiles_y;
}

void launch_tile(const TileArgs* blk, const TileArgs& a, const TileDyn& d, int precision, bool residual,
                 hipStream_t s) {
  if (blk == nullptr || d.btag != a.head.btag || a.ntiles != ((a.NX + a.TX - 1) / a.TX) * a.tiles_y)
    throw std::invalid_argument("launch_tile: the launch does not name its prepared argument block");
  const size_t lds = tile_lds_bytes(a.TX, a.RY, a.K);
  const bool f32 = precision == kFp32;
  const TileLaunch L{blk, a, d};
  if (f32) {
    if (residual) launch_ry<true, true>(L, lds, s);
    else launch_ry<true, false>(L, lds, s);
  } else {
    if (residual) launch_ry<false, true>(L, lds, s);
    else launch_ry<false, false>(L, lds, s);
  }
  H2D_HIP_CHECK(hipGetLastError());
}

void warm_tile_kernels(int precision, hipStream_t s) {
  static_assert(sizeof(TileArgs) <= kZeroArgBytes, "the zero block covers the tiled arguments");
  // the zero block: no tiles (every workgroup exits after its empty region load)
  const TileArgs* z = static_cast<const TileArgs*>(zero_arg_block());
  TileArgs a{};
  a.ntiles = 0;
  a.tiles_y = 1;
  const TileDyn d;
  const bool f32 = precision == kFp32;
  for (int ry : {32, 64, 128})
    for (int nt : {256, 1024})
      for (int cpl : {1, 2, 4}) {
        if (!tile_config_ok(1, ry, 1, cpl, nt)) continue;
        a.RY = ry, a.NT = nt, a.CPL = cpl;
        const TileLaunch L{z, a, d};
        if (f32) {
          launch_ry<true, true>(L, 0, s);
          launch_ry<true, false>(L, 0, s);
        } else {
          launch_ry<false, true>(L, 0, s);
          launch_ry<false, false>(L, 0, s);
        }
      }
  H2D_HIP_CHECK(hipGetLastError());
}

int tile_count(int NX, int NY, int TX, int TY) { return ((NX + TX - 1) / TX) * ((NY + TY - 1) / TY); }

}  // namespace h2d
