// heat2d_amd — hand-written CDNA4 (gfx950) HIP kernels.
//
// The hot kernel is `stream_kernel<K,...>`: a register-streaming, temporally-blocked 5-point
// Jacobi stencil.  Device equivalent of the reference's update loops
// (grad1612_cuda_heat.cu:55-62, grad1612_mpi_heat.c:238-259, mpi_heat2Dn.c:225-237), but
// designed for the CDNA4 execution model rather than translated:
//
//   * one wave64 owns a 256-column strip (4 contiguous fp32 per lane -> one 1 KiB
//     global_load_dwordx4 per row, fully coalesced) and walks DOWN the grid row by row;
//   * K time levels are kept in registers as a 2-row window per level ("2.5-D blocking"):
//     each input row is read from HBM / Infinity Cache once and each output row written
//     once per K steps, so memory traffic per cell-step is 8/K bytes;
//   * the east/west neighbours come from the adjacent lanes through DPP wave_shr/wave_shl
//     (no LDS, no barriers — waves are fully independent);
//   * the strip's column lead R = round_up(K,4) absorbs the K-deep dependency cone, so a
//     wave needs no data from any other wave; the row cone is covered by a K-row prologue;
//   * global-edge handling (fixed Dirichlet edges, zero ring, periodic wrap) is a
//     wave-uniform branch: strips away from the domain edge run the mask-free body.
//
// The kernel is fp64-VALU bound in the bit-exact `ref` precision (11 fp64-rate ops per cell:
// the reference evaluates its update in double) and Infinity-Cache/HBM bound in
// the fp32 precision.  No MFMA: a 5-point stencil has no dot-product of depth >= 16, and the
// bit-exact contract forbids the FMA contraction an MFMA formulation would impose.
//
// Included by the per-K translation units stream_k*.hip (compiled in parallel); every TU is
// compiled with -ffp-contract=off (bit-exactness of the ref path).
#pragma once
#include "kernels.h"


namespace h2d {
namespace {

// lane i <- lane i-1 (DPP wave_shr:1), lane i <- lane i+1 (DPP wave_shl:1).
__device__ __forceinline__ float from_left(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float from_right(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, false));
}

struct Coef {
  double cx, cy;
  float cxf, cyf;
};

template <bool F32>
__device__ __forceinline__ float cell(float c, float n, float s, float w, float e, const Coef& k) {
  if constexpr (F32) {
    return update_f32(c, n, s, w, e, k.cxf, k.cyf);
  } else {
    return update_ref(c, n, s, w, e, k.cx, k.cy);
  }
}

// One row of one time level: P = row i-1, C = row i, N = row i+1 of the previous level.
template <bool F32>
__device__ __forceinline__ float4 row_update(const float4& P, const float4& C, const float4& N, const Coef& k) {
  const float l = from_left(C.w);
  const float r = from_right(C.x);
  float4 o;
  o.x = cell<F32>(C.x, P.x, N.x, l, C.y, k);
  o.y = cell<F32>(C.y, P.y, N.y, C.x, C.z, k);
  o.z = cell<F32>(C.z, P.z, N.z, C.y, C.w, k);
  o.w = cell<F32>(C.w, P.w, N.w, C.z, r, k);
  return o;
}

struct LaneCtx {
  int64_t gxb;     // global row of stream input index 0
  int64_t NX;
  int fixed, per_x;
  int cm0, cm1, cm2, cm3;  // per-column modes of this lane's 4 columns
  float* out;      // dst at (output row 0 of the unit, this lane's first column)
  int64_t pitch;
  int nst;         // number of this lane's columns that are stored (0..4)
};

__device__ __forceinline__ int row_mode(int64_t gr, const LaneCtx& c) {
  if (c.per_x) return 0;
  if (gr < 0 || gr >= c.NX) return 2;
  if (c.fixed && (gr == 0 || gr == c.NX - 1)) return 1;
  return 0;
}

__device__ __forceinline__ float col_sel(int m, float o, float hold) { return m == 0 ? o : (m == 1 ? hold : 0.0f); }

template <bool EDGE>
__device__ __forceinline__ float4 apply_modes(float4 o, const float4& C, int rm, const LaneCtx& c) {
  if (rm == 2) return make_float4(0.f, 0.f, 0.f, 0.f);
  if (rm == 1) return C;
  if constexpr (EDGE) {
    o.x = col_sel(c.cm0, o.x, C.x);
    o.y = col_sel(c.cm1, o.y, C.y);
    o.z = col_sel(c.cm2, o.z, C.z);
    o.w = col_sel(c.cm3, o.w, C.w);
  }
  return o;
}

__device__ __forceinline__ void store_out(float* op, const float4& o, int nst) {
  if (nst == 4) {
    *reinterpret_cast<float4*>(op) = o;
  } else if (nst > 0) {
    op[0] = o.x;
    if (nst > 1) op[1] = o.y;
    if (nst > 2) op[2] = o.z;
  }
}

__device__ __forceinline__ double sq_diff(float a, float b) {
  const double d = (double)a - (double)b;
  return d * d;
}

// Process stream input row `ir` (level-0 value `cur`) through all K levels.
// Slot parity P = ir & 1: S[l][P] holds level-l row (ir-l-2), S[l][1-P] holds row (ir-l-1).
template <int K, bool F32, bool EDGE, bool RESID, int P, bool CHECK>
__device__ __forceinline__ void process_row(float4 (&S)[K][2], float4 cur, int ir, const LaneCtx& c, const Coef& k,
                                            double& racc) {
#pragma unroll
  for (int t = 1; t <= K; ++t) {
    if constexpr (CHECK) {
      if (ir < 2 * t) {  // level t not primed yet (wave-uniform); no early exit: keep the loop unrollable
        if (ir >= 2 * (t - 1)) S[t - 1][P] = cur;
        continue;
      }
    }
    const float4 prv = S[t - 1][P];
    const float4 mid = S[t - 1][1 - P];
    float4 o = row_update<F32>(prv, mid, cur, k);
    o = apply_modes<EDGE>(o, mid, row_mode(c.gxb + ir - t, c), c);
    S[t - 1][P] = cur;
    if (t == K) {
      float* op = c.out + (int64_t)(ir - 2 * K) * c.pitch;
      store_out(op, o, c.nst);
      if constexpr (RESID) {
        if (c.nst > 0) racc += sq_diff(o.x, mid.x);
        if (c.nst > 1) racc += sq_diff(o.y, mid.y);
        if (c.nst > 2) racc += sq_diff(o.z, mid.z);
        if (c.nst > 3) racc += sq_diff(o.w, mid.w);
      }
    }
    cur = o;
  }
}

#define H2D_SUBSTEP(D, CHECK, LIMIT)                                                      \
  {                                                                                       \
    const int ir = ir0 + (D);                                                             \
    if (ir < (LIMIT)) {                                                                   \
      const float4 nw = pf[D];                                                            \
      pf[D] = rowp[(int64_t)min(ir + 4, n - 1) * pitch4];                                 \
      process_row<K, F32, EDGE, RESID, (D)&1, CHECK>(S, nw, ir, c, k, racc);              \
    }                                                                                     \
  }

template <int K, bool F32, bool EDGE, bool RESID>
__device__ __forceinline__ void run_unit(const float4* __restrict__ rowp, int64_t pitch4, int n, const LaneCtx& c,
                                         const Coef& k, double& racc) {
  float4 S[K][2];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    S[t][0] = make_float4(0.f, 0.f, 0.f, 0.f);
    S[t][1] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 pf[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) pf[d] = rowp[(int64_t)min(d, n - 1) * pitch4];

  const int npro = min(n, (2 * K + 3) & ~3);
  int ir0 = 0;
  for (; ir0 < npro; ir0 += 4) {  // prologue: levels start one by one
    H2D_SUBSTEP(0, true, npro)
    H2D_SUBSTEP(1, true, npro)
    H2D_SUBSTEP(2, true, npro)
    H2D_SUBSTEP(3, true, npro)
  }
  for (; ir0 < n; ir0 += 4) {  // steady state: every level active, no checks
    H2D_SUBSTEP(0, false, n)
    H2D_SUBSTEP(1, false, n)
    H2D_SUBSTEP(2, false, n)
    H2D_SUBSTEP(3, false, n)
  }
}
#undef H2D_SUBSTEP

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int K, bool F32, bool RESID>
__global__ __launch_bounds__(256) void stream_kernel(StreamArgs a) {
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int w = (int)blockIdx.x * 4 + wv;
  if (w >= a.nunits) return;
  const int lane = (int)(threadIdx.x & 63);
  const Unit u = a.units[w];
  const int64_t y0 = (int64_t)u.strip * a.wout;
  const int64_t x0 = (int64_t)u.seg * a.H;
  const int h = (int)min((int64_t)a.H, a.xcell - x0);
  const int64_t cb = y0 - a.R + 4 * lane;

  LaneCtx c;
  c.gxb = a.gx0 + x0 - K;
  c.NX = a.NX;
  c.fixed = a.fixed;
  c.per_x = a.per_x;
  const int64_t gc = a.gy0 + cb;
  c.cm0 = dim_mode(gc + 0, a.NY, a.per_y != 0, a.fixed != 0);
  c.cm1 = dim_mode(gc + 1, a.NY, a.per_y != 0, a.fixed != 0);
  c.cm2 = dim_mode(gc + 2, a.NY, a.per_y != 0, a.fixed != 0);
  c.cm3 = dim_mode(gc + 3, a.NY, a.per_y != 0, a.fixed != 0);
  const bool lane_special = (c.cm0 | c.cm1 | c.cm2 | c.cm3) != 0;
  const bool in_out = (cb >= y0) && (cb + 4 <= y0 + a.wout);
  c.nst = in_out ? (int)max((int64_t)0, min((int64_t)4, a.ycell - cb)) : 0;
  c.pitch = a.pitch;
  c.out = a.dst + (a.G + x0) * a.pitch + a.PL + cb;

  const float4* rowp = reinterpret_cast<const float4*>(a.src + (a.G + x0 - K) * a.pitch + a.PL + cb);
  const int64_t pitch4 = a.pitch >> 2;
  const int n = h + 2 * K;
  Coef k{a.cx, a.cy, (float)a.cx, (float)a.cy};
  double racc = 0.0;
  if (__any(lane_special)) {
    run_unit<K, F32, true, RESID>(rowp, pitch4, n, c, k, racc);
  } else {
    run_unit<K, F32, false, RESID>(rowp, pitch4, n, c, k, racc);
  }
  if constexpr (RESID) {
    racc = wave_sum(racc);
    if (lane == 0) a.partials[w] = racc;
  }
}

}  // namespace

template <int K>
void launch_stream_k(const StreamArgs& a, bool f32, bool resid, hipStream_t s) {
  const int blocks = (a.nunits + 3) / 4;
  void (*fn)(StreamArgs);
  if (f32) fn = resid ? stream_kernel<K, true, true> : stream_kernel<K, true, false>;
  else fn = resid ? stream_kernel<K, false, true> : stream_kernel<K, false, false>;
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace h2d
