// heat2d_amd — the streaming, temporally-blocked 5-point stencil for CDNA4 (gfx950).
//
// Device equivalent of the reference's update loops (grad1612_cuda_heat.cu:55-62,
// grad1612_mpi_heat.c:238-259, mpi_heat2Dn.c:225-237), designed for the CDNA4 execution model
// rather than translated:
//
//   * one wave64 owns a 256-column strip (4 contiguous fp32 per lane -> one 1 KiB
//     global_load_dwordx4 per row, fully coalesced) and walks DOWN the grid row by row;
//   * K time levels are kept in registers as a 2-row window per level ("2.5-D blocking"):
//     each input row is read once and each output row written once per K steps, so memory
//     traffic per cell-step is 8/K bytes;
//   * east/west neighbours come from the adjacent lanes through DPP wave_shr/wave_shl (no LDS,
//     no barriers — waves are fully independent);
//   * the strip's column lead R = round_up(K,4) absorbs the K-deep dependency cone; the row
//     cone is a 2K-row prologue that is unrolled at compile time (no runtime checks);
//   * the steady state is straight-line code (4 rows × K levels, no branches), so the
//     scheduler overlaps the level chains of consecutive rows;
//   * global-edge handling (fixed Dirichlet edges, zero ring, periodic wrap, partial stores)
//     is a separate branch-free body (selects, per-element store redirection) chosen once per
//     wave; waves away from the domain edge run the mask-free body.
//
// Numerics: the ref precision evaluates the reference's double expression with its exact
// rounding sequence.  `fl(s+n - 2c)` is computed as fma(-2, c, s+n): 2c is
// exact in double, so the fused form rounds once on the same exact value — bit-identical,
// one fp64 op less (10 fp64-rate ops per cell).  No MFMA: a 5-point stencil has no
// dot-product of depth >= 16 and the contract forbids the contraction it would impose.
//
// Included by the generated per-variant translation units (build/gen/stream_k*.hip, compiled in
// parallel); every TU is
// compiled with -ffp-contract=off.
#pragma once
#include "kernels.h"

namespace h2d {
namespace {

// A pointer read from a device-resident argument block is generic (flat) to the compiler; every
// buffer the kernels touch — tiles, unit lists, peer memory mapped over xGMI, host-mapped words —
// lies in the global aperture, so say so: global_load / global_store instead of flat (in-order
// completion for the counted vmcnt waits, no lgkmcnt on every wait, and a buffer resource built
// from a uniform base instead of a readfirstlane waterfall per store).
// (Through an integer: an addrspacecast round trip generic -> global -> generic folds away.)
template <class T>
__device__ __forceinline__ T* gp(T* p) {
  return (T*)(__attribute__((address_space(1))) T*)(uintptr_t)p;
}

// lane i <- lane i-1 (DPP wave_shr:1), lane i <- lane i+1 (DPP wave_shl:1).
// bound_ctrl=1 (lanes without a source read 0, the add identity) lets the compiler fold the
// DPP move into the consuming v_add_f32 (one VALU op instead of two).
__device__ __forceinline__ float from_left(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_right(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}

struct Coef {
  double cx, cy;
  float cxf, cyf;
};

// Device cell update from the fp32 pair sums sn = s+n, ew = e+w; identical values to
// update_ref / update_f32 (h2d_common.h).
template <bool F32>
__device__ __forceinline__ float cell(float c, float sn, float ew, const Coef& k) {
  if constexpr (F32) {
    const float r = __builtin_fmaf(k.cxf, __builtin_fmaf(-2.0f, c, sn), c);
    return __builtin_fmaf(k.cyf, __builtin_fmaf(-2.0f, c, ew), r);
  } else {
    const double dc = (double)c;
    const double t1 = __builtin_fma(-2.0, dc, (double)sn);  // == fl(sn - 2c): 2c is exact
    const double t4 = __builtin_fma(-2.0, dc, (double)ew);
    double r = dc + k.cx * t1;
    r = r + k.cy * t4;
    return (float)r;
  }
}

template <bool F32>
__device__ __forceinline__ float cell(float c, float n, float s, float w, float e, const Coef& k) {
  return cell<F32>(c, s + n, e + w, k);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// One row of one time level: P = row i-1, C = row i, N = row i+1 of the previous level.
// The eight fp32 pair sums take five VALU ops: three packed adds (v_pk_add_f32, two lanes of
// fp32 per op, same IEEE rounding as v_add_f32) and two adds with the DPP neighbour fetch
// folded in (v_add_f32_dpp).
template <bool F32>
__device__ __forceinline__ float4 row_update(const float4& P, const float4& C, const float4& N, const Coef& k) {
  const f32x2 sn01 = f32x2{P.x, P.y} + f32x2{N.x, N.y};
  const f32x2 sn23 = f32x2{P.z, P.w} + f32x2{N.z, N.w};
  const f32x2 ew12 = f32x2{C.x, C.y} + f32x2{C.z, C.w};  // (C.x + C.z, C.y + C.w)
  const float ew0 = from_left(C.w) + C.y;
  const float ew3 = C.z + from_right(C.x);
  float4 o;
  if constexpr (F32) {
    // fp32 fast path: two cells per packed FMA (v_pk_fma_f32: each half is an IEEE fma, so the
    // values equal cell<true> / update_f32 bit for bit) — 4 instead of 8 FMAs per cell pair
    const f32x2 c01 = {C.x, C.y}, c23 = {C.z, C.w};
    const f32x2 ew01 = {ew0, ew12.x}, ew23 = {ew12.y, ew3};
    const f32x2 m2 = {-2.0f, -2.0f}, cx2 = {k.cxf, k.cxf}, cy2 = {k.cyf, k.cyf};
    f32x2 r01 = __builtin_elementwise_fma(cx2, __builtin_elementwise_fma(m2, c01, sn01), c01);
    f32x2 r23 = __builtin_elementwise_fma(cx2, __builtin_elementwise_fma(m2, c23, sn23), c23);
    r01 = __builtin_elementwise_fma(cy2, __builtin_elementwise_fma(m2, c01, ew01), r01);
    r23 = __builtin_elementwise_fma(cy2, __builtin_elementwise_fma(m2, c23, ew23), r23);
    o = make_float4(r01.x, r01.y, r23.x, r23.y);
  } else {
    o.x = cell<F32>(C.x, sn01.x, ew0, k);
    o.y = cell<F32>(C.y, sn01.y, ew12.x, k);
    o.z = cell<F32>(C.z, sn23.x, ew12.y, k);
    o.w = cell<F32>(C.w, sn23.y, ew3, k);
  }
  return o;
}

// The same row update for a lane that owns 2 columns (128-column strips of the persistent
// kernel): lane i holds (x, y) = columns (2i, 2i+1); west of x is the left lane's y, east of y
// is the right lane's x.
template <bool F32>
__device__ __forceinline__ float2 row_update(const float2& P, const float2& C, const float2& N, const Coef& k) {
  const f32x2 sn = f32x2{P.x, P.y} + f32x2{N.x, N.y};
  const float ew0 = from_left(C.y) + C.y;
  const float ew1 = C.x + from_right(C.x);
  float2 o;
  if constexpr (F32) {
    const f32x2 c01 = {C.x, C.y}, ew01 = {ew0, ew1};
    const f32x2 m2 = {-2.0f, -2.0f}, cx2 = {k.cxf, k.cxf}, cy2 = {k.cyf, k.cyf};
    f32x2 r = __builtin_elementwise_fma(cx2, __builtin_elementwise_fma(m2, c01, sn), c01);
    r = __builtin_elementwise_fma(cy2, __builtin_elementwise_fma(m2, c01, ew01), r);
    o = make_float2(r.x, r.y);
  } else {
    o.x = cell<F32>(C.x, sn.x, ew0, k);
    o.y = cell<F32>(C.y, sn.y, ew1, k);
  }
  return o;
}

struct LaneCtx {
  int64_t gxb;     // global row of stream input index 0
  int64_t dir;     // +1: rows stream top-down, -1: bottom-up (kUnitReverse)
  // global-edge rows: fixed -> rows rlo and rhi are held; ghost-zero -> rows < rlo or >= rhi are
  // zero (a periodic dimension: bounds no row reaches, so the masked bodies are a safe superset)
  int64_t rlo, rhi;
  bool m0, m1, m2, m3;  // per-column mask: fixed -> hold (global edge), ghost-zero -> zero (outside)
  float* sout;     // real output pointer (lanes in the output range), or a dummy slot
  int64_t spitch;  // row pitch of sout (0 for the dummy slot)
  float* pout;     // halo push: copy of output rows [0, prows) (neighbour's receive buffer) or a dummy
  int64_t ppitch;
  int prows;       // 0: this unit pushes nothing (wave-uniform)
  int rel;         // release flavour of the unit's signal (unit_signal)
  float* kout;     // RESID launches: level K-1 value of each output cell (rollback state) or a dummy
  int64_t kpitch;  // row pitch of kout (0 for the dummy slot)
  bool st0, st1, st2, st3;  // element is an owned output cell (residual accounting)
  // write-through path (StreamArgs::wt): wave-uniform base = the unit's lowest-address output
  // row, the byte offset of output row orow = obo + orow * obs (reverse units: negative step),
  // and this lane's byte offset in a row (out-of-range lanes: >= 2^31, past num_records, so the
  // buffer store drops them — no dummy slot).  The host keeps every offset below 2^31.
  float* obase;
  int obo, obs;
  unsigned voff;
  // 2-D direct pipeline side pushes (Unit::links bits 8-13), per output row orow at tile row
  // xr0 + xdir * orow: sp (W or E neighbour: every row), cn (NW / NE: rows < G), cs (SW / SE:
  // rows >= xcell - G), each with its per-orow step; em: the lane's elements that are pushed.
  bool spu;  // wave-uniform: the unit pushes to a side or corner
  unsigned em;
  float *sp, *cn, *cs;
  int64_t sps, cns, css;
  int64_t xr0, xdir, xlo, xhi;
};

// Masked element stores (a lane's float4 can straddle the G-column boundary of a side push).
__device__ __forceinline__ void store_masked(float* p, const float4& o, unsigned m) {
  if (m & 1u) p[0] = o.x;
  if (m & 2u) p[1] = o.y;
  if (m & 4u) p[2] = o.z;
  if (m & 8u) p[3] = o.w;
}

// 2-D direct pipeline: this output row's cells that lie in a W/E neighbour's halo (and, in the
// first / last G rows, a corner neighbour's) go straight into that neighbour's receive columns.
__device__ __forceinline__ void side_push(const float4& o, int64_t orow, const LaneCtx& c) {
  if (c.em == 0u) return;
  const int64_t r = c.xr0 + c.xdir * orow;
  if (c.sp != nullptr) store_masked(c.sp + orow * c.sps, o, c.em);
  if (c.cn != nullptr && r < c.xlo) store_masked(c.cn + orow * c.cns, o, c.em);
  if (c.cs != nullptr && r >= c.xhi) store_masked(c.cs + orow * c.css, o, c.em);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Wide-store data hazard (gfx950, ROCm 7.2 hipcc).  A store of more than 64 bits reads its data
// VGPRs after it issues, so a write of those VGPRs needs 2 wait states after the store.  hipcc
// does not pad a 64-bit VALU write there (v_pk_add_f32, v_mov_b64, v_cvt_f64_f32, v_add_f64 right
// after a buffer_store_dwordx4: tools/hazard_lint.py found 1 242 such pairs in the stencil
// objects).  Under memory load the store then writes the new value for some lanes — measured:
// element 1 of lanes 12-15 of every 16 in one row per unit (2-step 257x509 run), and the
// intermittent wrong tiles of round 3 (the residual launches convert each stored row to fp64 in
// place).  hipcc does pad the same store with an immediate soffset, so the write-through row
// stores carry the row offset in the vector offset (soffset 0) and need nothing more; every other wide store is followed by `s_nop 1` that reads its data
// registers, ordered after the store by its memory clobber (tools/hazard_lint.py checks every
// built code object for the pattern).
__device__ __forceinline__ void store_guard(const u32x4& d) { asm volatile("s_nop 1" ::"v"(d) : "memory"); }

__device__ __forceinline__ u32x4 as_u32x4(const float4& o) {
  return u32x4{__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z), __float_as_uint(o.w)};
}

// Plain wide store of a lane's cells (16 B guarded; 8 B needs no guard).  Global address space
// (global_store, not flat_store): it completes in issue order with the buffer loads and stores,
// so the counted `s_waitcnt vmcnt(N)` of the persistent kernel covers it (flat accesses complete
// out of order).
typedef __attribute__((address_space(1))) u32x4 gu32x4;
typedef unsigned int u32x2_ __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x2_ gu32x2;
__device__ __forceinline__ void store_cells(float* p, const float4& o) {
  const u32x4 d = as_u32x4(o);
  *(gu32x4*)p = d;
  store_guard(d);
}
__device__ __forceinline__ void store_cells(float* p, const float2& o) {
  *(gu32x2*)p = u32x2_{__float_as_uint(o.x), __float_as_uint(o.y)};
}

// Store one lane's float4 of an output row write-through (buffer_store_dwordx4 ... sc1):
// 16-B sc1 stores cost about a plain store, and leave no dirty line in the L2.  The resource is
// loop-invariant (the unit's base); the row's byte offset is added to the lane's vector offset
// (soffset 0, see the hazard note above).  A dropped lane's offset starts at 2^31 and a row
// offset stays below 2^31 (the host's limit), so it never wraps back into the record range.
__device__ __forceinline__ void store_row_wt(float* base, unsigned voff, int soff, const float4& o) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(as_u32x4(o), r, (int)(voff + (unsigned)soff), 0, 16 /* sc1 */);
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// The 2-column lane's row store (buffer_store_dwordx2 ... sc1).
__device__ __forceinline__ void store_row_wt(float* base, unsigned voff, int soff, const float2& o) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  const u32x2 d = {__float_as_uint(o.x), __float_as_uint(o.y)};
  __builtin_amdgcn_raw_buffer_store_b64(d, r, (int)voff, soff, 16 /* sc1 */);
}

__device__ __forceinline__ double sq_diff(float a, float b) {
  const double d = (double)a - (double)b;
  return d * d;
}

// Branch-free global-edge masks (EDGE bit 0: columns, bit 1: rows).  Fixed edges hold their
// previous value; in ghost-zero mode cells outside the grid stay 0.  (In fixed mode cells
// outside the grid may hold anything: the held edge row/column separates them from the
// interior.)  Row conditions are wave-uniform.
template <int EDGE, bool FIXED>
__device__ __forceinline__ float4 apply_edge(float4 o, const float4& C, int64_t gr, const LaneCtx& c) {
  if constexpr ((EDGE & 1) != 0) {
    if constexpr (FIXED) {
      o.x = c.m0 ? C.x : o.x;
      o.y = c.m1 ? C.y : o.y;
      o.z = c.m2 ? C.z : o.z;
      o.w = c.m3 ? C.w : o.w;
    } else {
      o.x = c.m0 ? 0.0f : o.x;
      o.y = c.m1 ? 0.0f : o.y;
      o.z = c.m2 ? 0.0f : o.z;
      o.w = c.m3 ? 0.0f : o.w;
    }
  }
  if constexpr ((EDGE & 2) != 0) {
    // per component: a select of a whole float4 aggregate is lowered through scratch memory
    if constexpr (FIXED) {
      const bool r = gr == c.rlo || gr == c.rhi;
      o.x = r ? C.x : o.x;
      o.y = r ? C.y : o.y;
      o.z = r ? C.z : o.z;
      o.w = r ? C.w : o.w;
    } else {
      const bool r = gr < c.rlo || gr >= c.rhi;
      o.x = r ? 0.0f : o.x;
      o.y = r ? 0.0f : o.y;
      o.z = r ? 0.0f : o.z;
      o.w = r ? 0.0f : o.w;
    }
  }
  return o;
}

template <int EDGE, bool FIXED>
__device__ __forceinline__ float2 apply_edge(float2 o, const float2& C, int64_t gr, const LaneCtx& c) {
  if constexpr ((EDGE & 1) != 0) {
    if constexpr (FIXED) {
      o.x = c.m0 ? C.x : o.x;
      o.y = c.m1 ? C.y : o.y;
    } else {
      o.x = c.m0 ? 0.0f : o.x;
      o.y = c.m1 ? 0.0f : o.y;
    }
  }
  if constexpr ((EDGE & 2) != 0) {
    if constexpr (FIXED) {
      const bool r = gr == c.rlo || gr == c.rhi;
      o.x = r ? C.x : o.x;
      o.y = r ? C.y : o.y;
    } else {
      const bool r = gr < c.rlo || gr >= c.rhi;
      o.x = r ? 0.0f : o.x;
      o.y = r ? 0.0f : o.y;
    }
  }
  return o;
}

// Process stream input row `ir` (level-0 value `cur`) through levels 1..TMAX (TMAX <= K).
// Slot parity P = ir & 1: S[l][P] holds level-l row (ir-l-2), S[l][1-P] holds row (ir-l-1).
// Level t computes row (ir - t) of level t.  Level K writes output row ir - 2K (unit-relative).
// V: the lane's cells of a row (float4: 256-column strips; float2: 128-column strips, no
// residual / side pushes).  PUSH: the unit may copy output rows into a neighbour's receive buffer
// (halo units only: the check is a branch per row, which would split the straight-line steady
// loop of every other unit into per-row blocks the scheduler cannot overlap).
template <int K, bool F32, int EDGE, bool FIXED, bool RESID, bool WT, bool SIDE, bool PUSH, int P, int TMAX, class V>
__device__ __forceinline__ void process_row(V (&S)[K][2], V cur, int ir, const LaneCtx& c, const Coef& k,
                                            double& racc) {
#pragma unroll
  for (int t = 1; t <= K; ++t) {
    if (t > TMAX) {
      if (t - 1 <= TMAX) S[t - 1][P] = cur;  // save the last active level's new row
      continue;
    }
    const V prv = S[t - 1][P];
    const V mid = S[t - 1][1 - P];
    V o = row_update<F32>(prv, mid, cur, k);
    if constexpr (EDGE != 0) o = apply_edge<EDGE, FIXED>(o, mid, c.gxb + c.dir * (ir - t), c);
    S[t - 1][P] = cur;
    if (t == K) {
      const int64_t orow = ir - 2 * K;
      if constexpr (WT) store_row_wt(c.obase, c.voff, c.obo + (int)orow * c.obs, o);
      else store_cells(c.sout + orow * c.spitch, o);
      if constexpr (PUSH)
        if (orow < c.prows) store_cells(c.pout + orow * c.ppitch, o);  // uniform branch
      if constexpr (SIDE) side_push(o, orow, c);
      if constexpr (RESID) {
        store_cells(c.kout + orow * c.kpitch, mid);
        racc += c.st0 ? sq_diff(o.x, mid.x) : 0.0;
        racc += c.st1 ? sq_diff(o.y, mid.y) : 0.0;
        racc += c.st2 ? sq_diff(o.z, mid.z) : 0.0;
        racc += c.st3 ? sq_diff(o.w, mid.w) : 0.0;
      }
    }
    cur = o;
  }
}

// Prologue row IR (compile-time): levels t <= IR/2 are primed, from rows already in registers.
template <int K, bool F32, int EDGE, bool FIXED, bool RESID, bool WT, bool SIDE, bool PUSH, int IR, class V>
__device__ __forceinline__ void prologue(V (&S)[K][2], const V (&pro)[2 * K], const LaneCtx& c, const Coef& k,
                                         double& racc) {
  if constexpr (IR < 2 * K) {
    process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, PUSH, IR & 1, IR / 2>(S, pro[IR], IR, c, k, racc);
    prologue<K, F32, EDGE, FIXED, RESID, WT, SIDE, PUSH, IR + 1>(S, pro, c, k, racc);
  }
}

// Prologue rows loaded where they are used (H2D_PRO_UPFRONT=0, the default) or all up front
// (=1).  A/B at 4096^2, depth 7, alternating processes (tools/ab_so.py, profiles/ab_prologue_r3.txt):
// us/step 1000 steps 7.67/7.84/7.79 inline vs 7.79/7.78/7.94 up front; 20 steps 8.36/8.44/8.52 vs
// 8.41/8.53/8.64.
template <int K, bool F32, int EDGE, bool FIXED, bool RESID, bool WT, bool SIDE, bool PUSH, int IR>
__device__ __forceinline__ void prologue_inline(float4 (&S)[K][2], const float4* __restrict__ rowp,
                                                const float4* __restrict__ hrowp, int64_t pitch4, const LaneCtx& c,
                                                const Coef& k, double& racc) {
  if constexpr (IR < 2 * K) {
    const float4 v = (IR < K ? hrowp : rowp)[(int64_t)IR * pitch4];
    process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, PUSH, IR & 1, IR / 2>(S, v, IR, c, k, racc);
    prologue_inline<K, F32, EDGE, FIXED, RESID, WT, SIDE, PUSH, IR + 1>(S, rowp, hrowp, pitch4, c, k, racc);
  }
}

#ifndef H2D_PRO_UPFRONT
#define H2D_PRO_UPFRONT 0
#endif

// Mid-unit signal of the signalled halo pipeline: this wave's halo rows are stored — release
// them at system scope and count the unit.  Producer recipe of the MI355X guide: the wave's
// stores drained, the release fence (L2 write-back), an explicit drain again (ROCm 7.2 can
// drop the fence's own wait), then ONE lane's atomic add.
__device__ __forceinline__ void unit_signal(unsigned long long* sig, int lane, int rel) {
  // (the pushes are flat stores: lgkmcnt too — flat accesses complete out of order)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  // rel 0: system-scope release (L2 write-back: the RCCL path's payload lives in coarse-grained
  // tile memory another agent may read); 1: agent scope; 2: none — the direct pipeline's payload
  // was stored to the peer's UNCACHED memory, so the drained (acknowledged) stores are already
  // at their destination and only the ordering of the flag after them matters.
  if (rel == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  else if (rel == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(sig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// sig_at > 0: signal (once) before processing stream row sig_at (a multiple of 4 past 2K),
// i.e. once every output row < sig_at - 2K is stored.  HALO: the unit pushes rows or signals
// (the halo units of the signalled / direct pipelines); other units' bodies have neither check.
template <int K, bool F32, int EDGE, bool FIXED, bool RESID, bool WT, bool SIDE, bool HALO>
__device__ __forceinline__ void run_unit(const float4* __restrict__ rowp, const float4* __restrict__ hrowp,
                                         int64_t pitch4, int n, const LaneCtx& c, const Coef& k, double& racc,
                                         int sig_at, unsigned long long* sig, int lane) {
  float4 S[K][2];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    S[t][0] = make_float4(0.f, 0.f, 0.f, 0.f);
    S[t][1] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // n = h + 2K >= 2K + 1: the prologue rows all exist.  Every prologue row and the first four
  // steady rows are loaded up front, all in flight at once: ONE memory round trip starts the
  // unit (left to the scheduler, each prologue load sat behind the previous row's compute and a
  // vmcnt(0) — several serialised round trips, ~3 us of every launch).  Stream rows [0, K) are
  // the unit's outer cone rows: for a halo unit, the ghost rows, read from hrowp (the halo
  // receive buffer of the direct pipeline; == rowp otherwise).
#if H2D_PRO_UPFRONT
  float4 pro[2 * K];
#pragma unroll
  for (int i = 0; i < 2 * K; ++i) pro[i] = (i < K ? hrowp : rowp)[(int64_t)i * pitch4];
  float4 pf[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) pf[d] = rowp[(int64_t)min(2 * K + d, n - 1) * pitch4];
  __builtin_amdgcn_sched_barrier(0);  // keep the loads above: each use waits only for its own row
  prologue<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 0>(S, pro, c, k, racc);
#else
  float4 pf[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) pf[d] = rowp[(int64_t)min(2 * K + d, n - 1) * pitch4];
  prologue_inline<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 0>(S, rowp, hrowp, pitch4, c, k, racc);
#endif

  int ir0 = 2 * K;  // even: slot parity of sub-step d is d & 1
  // The next four rows are loaded at the top of each 4-row half, a whole half ahead of their use,
  // into the register set the previous half consumed (ping-pong: no register copies, whose waits
  // the compiler placed as vmcnt(0) — a drain of the write-through row stores too).  Left to the
  // scheduler, the straight-line body issued the loads late and waited the same way (+3 %).
#define H2D_HALF(CUR, NXT, R0)                                                             \
  {                                                                                        \
    if constexpr (HALO)                                                                    \
      if ((R0) == sig_at) unit_signal(sig, lane, c.rel);                                   \
    _Pragma("unroll") for (int d = 0; d < 4; ++d)                                          \
        NXT[d] = rowp[(int64_t)min((R0) + d + 4, n - 1) * pitch4];                         \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 0, K>(S, CUR[0], (R0) + 0, c, k, racc); \
    process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 1, K>(S, CUR[1], (R0) + 1, c, k, racc); \
    process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 0, K>(S, CUR[2], (R0) + 2, c, k, racc); \
    process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 1, K>(S, CUR[3], (R0) + 3, c, k, racc); \
  }
  float4 nx[4];
  if constexpr (K <= 8) {  // deeper variants (off the bench's path) keep half the code: build time
    for (; ir0 + 8 <= n; ir0 += 8) {
      H2D_HALF(pf, nx, ir0)
      H2D_HALF(nx, pf, ir0 + 4)
    }
  }
  for (; ir0 + 4 <= n; ir0 += 4) {
    H2D_HALF(pf, nx, ir0)
#pragma unroll
    for (int d = 0; d < 4; ++d) pf[d] = nx[d];
  }
#undef H2D_HALF
  // tail: at most 3 rows
  if (ir0 < n) process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 0, K>(S, pf[0], ir0, c, k, racc);
  if (ir0 + 1 < n) process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 1, K>(S, pf[1], ir0 + 1, c, k, racc);
  if (ir0 + 2 < n) process_row<K, F32, EDGE, FIXED, RESID, WT, SIDE, HALO, 0, K>(S, pf[2], ir0 + 2, c, k, racc);
  // the loop visits every sig_at candidate below its exit value: a signal point at or past the
  // exit has not fired yet (unit shorter than its signal rows, or kUnitSigEnd)
  if constexpr (HALO)
    if (sig_at >= ir0) unit_signal(sig, lane, c.rel);
}

// A bounded wait gave up: set `bit` in the device word (fail-fast for later waits) and in its
// host-mapped mirror (a plain system-scope store: no PCIe atomic needed), which the host polls
// per chunk to abort the run early instead of computing on with stale halos.
__device__ __forceinline__ void report_timeout(unsigned int* dev, unsigned int* host, unsigned int bit) {
  if (dev) __hip_atomic_fetch_or(dev, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (host) __hip_atomic_store(host, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Sum over the wave, every lane gets it: DPP within each 16-lane row (quad swaps, then row
// rotations by 4 and 8: no LDS traffic, unlike the ds_bpermute butterfly above), then the four
// row sums read from lanes 0 / 16 / 32 / 48 and added in that order.  fp64 moves as two halves.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_f64(double v, int lane) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)b, lane);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double dpp_wave_sum(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x124>(v);  // row_ror:4
  v += dpp_f64<0x128>(v);  // row_ror:8
  return (lane_f64(v, 0) + lane_f64(v, 16)) + (lane_f64(v, 32) + lane_f64(v, 48));
}

template <int K, bool F32, bool RESID, bool WT, int EDGE, bool SIDE, bool HALO>
__device__ __forceinline__ void run_edge(const float4* rowp, const float4* hrowp, int64_t pitch4, int n,
                                         const LaneCtx& c, const Coef& k, double& racc, bool fixed, int sig_at,
                                         unsigned long long* sig, int lane) {
  if (fixed) run_unit<K, F32, EDGE, true, RESID, WT, SIDE, HALO>(rowp, hrowp, pitch4, n, c, k, racc, sig_at, sig, lane);
  else run_unit<K, F32, EDGE, false, RESID, WT, SIDE, HALO>(rowp, hrowp, pitch4, n, c, k, racc, sig_at, sig, lane);
}

// The bodies of the units that neither push nor signal (all but a few per launch): no per-row
// check, so the steady loop is straight-line code.
template <int K, bool F32, bool RESID, bool WT>
__device__ __forceinline__ void run_plain(const Unit& u, const float4* rowp, const float4* hrowp, int64_t pitch4,
                                          int n, const LaneCtx& c, const Coef& k, double& racc, bool fixed,
                                          int sig_at, unsigned long long* sig, int lane) {
  switch (u.flags & 3) {
    case 0: run_unit<K, F32, 0, false, RESID, WT, false, false>(rowp, hrowp, pitch4, n, c, k, racc, sig_at, sig, lane); break;
    case 1: run_edge<K, F32, RESID, WT, 1, false, false>(rowp, hrowp, pitch4, n, c, k, racc, fixed, sig_at, sig, lane); break;
    case 2: run_edge<K, F32, RESID, WT, 2, false, false>(rowp, hrowp, pitch4, n, c, k, racc, fixed, sig_at, sig, lane); break;
    default: run_edge<K, F32, RESID, WT, 3, false, false>(rowp, hrowp, pitch4, n, c, k, racc, fixed, sig_at, sig, lane); break;
  }
}

// The decision of a convergence check, by the one lane that holds the total.
__device__ __forceinline__ void decide_total(double r, const DecideArgs& d) {
  if (*gp(d.stop) != 0ull) return;  // already stopped
  __hip_atomic_store(&gp(d.host)->last, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&gp(d.host)->checks, d.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (r < d.sens) {
    *gp(d.stop) = d.seq;
    __hip_atomic_store(&gp(d.host)->residual, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&gp(d.host)->stop_seq, d.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The deferred decision of a lone tile's previous check (one wave of a launch's extra block,
// StreamArgs::pend / TileArgs::pend): the partials summed lane-strided, then over the wave.
__device__ __forceinline__ void decide_pending(const double* parts, int n, DecideArgs pd, unsigned long long seq,
                                               int lane) {
  if (__hip_atomic_load(gp(pd.stop), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull) return;  // decided earlier
  double s = 0.0;
  for (int i = lane; i < n; i += 64) s += gp(parts)[i];
  s = dpp_wave_sum(s);
  if (lane == 0) {
    pd.seq = seq;
    *gp(pd.total) = s;
    decide_total(s, pd);  // the stop word for later launches, the host record
  }
}

// Fused check epilogue (one wave): publish this wave's partial; with d.ticket, the wave whose
// ticket add is the last of `nparts` sums all partials in a fixed order and decides.  The
// partials are stored write-through (agent-scope atomic store = sc1) and drained before the
// ticket add, the last adder acquires before reading them (MI355X guide, G16 row 1).
__device__ __forceinline__ void publish_partial(double* partials, int slot, double v, int nparts,
                                                const DecideArgs& d, int lane) {
  if (lane == 0) __hip_atomic_store(partials + slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (gp(d.ticket) == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int last = 0;
  if (lane == 0) last = __hip_atomic_fetch_add(gp(d.ticket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                        (unsigned)(nparts - 1);
  last = __shfl(last, 0, 64);
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double s = 0.0;
  for (int i = lane; i < nparts; i += 64) s += __hip_atomic_load(partials + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s = wave_sum(s);
  if (lane == 0) {
    *gp(d.total) = s;
    if (gp(d.host) != nullptr) decide_total(s, d);  // else a cross-tile / cross-rank sum decides later
    __hip_atomic_store(gp(d.ticket), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int K, bool F32, bool RESID, bool WT>
__global__ __launch_bounds__(256) void stream_kernel(const StreamArgs* __restrict__ ap, unsigned long long lid_arg,
                                                     unsigned long long copies_need_arg, unsigned long long seq_arg,
                                                     unsigned btag_arg, StreamNeed need) {
  // The per-launch scalars sit in kernel-argument memory (host memory, the library's default):
  // read once, up front, in the block pointer's batch, and kept in SGPRs — the asm makes them
  // values, not loads the compiler may repeat (a host round trip each) later in the wave.
  unsigned long long lid = lid_arg, copies_need = copies_need_arg, seq = seq_arg;
  unsigned btag = btag_arg;
  asm volatile("" : "+s"(lid), "+s"(copies_need), "+s"(seq), "+s"(btag));
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int w = (int)blockIdx.x * 4 + wv;
  // the plan's arguments: an immutable device-resident block (scalar loads, L2 / K$ resident).
  // No-op launches (warm_stream_kernels) pass the zero block (zero_arg_block: nunits 0).
  const StreamArgs& a = *ap;
  // the block fields the preamble needs, loaded as ONE batch (one wait instead of a chain of
  // dependent round trips behind each early-exit test)
  // (the unit-list pointer stays a plain block load: the unit's own load must remain scalar)
  int nunits = a.nunits, nsignal = a.nsignal;
  const unsigned long long* stamps_p = gp(a.stamps);
  asm volatile("" : "+s"(nunits), "+s"(nsignal), "+s"(stamps_p));
  if (w >= nunits) {
    // the extra block of a launch carrying the previous check's decision (StreamArgs::pend)
    if (wv == 0 && (int)blockIdx.x == (nunits + 3) / 4 && gp(a.pend) != nullptr)
      decide_pending(a.pend, a.pend_n, a.pend_dec, seq, (int)(threadIdx.x & 63));
    return;
  }
  const int lane = (int)(threadIdx.x & 63);
  const bool stamping = stamps_p != nullptr;  // diagnostics: per-wave timeline
  const unsigned long long t_start = stamping ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const Unit u = gp(a.units)[w];
  const bool halo_unit = w < nsignal;
  const bool ns_unit = halo_unit && (u.flags & kUnitNS) != 0;  // top / bottom halo unit of its strip
  const int dir = (u.flags & kUnitReverse) ? 1 : 0;  // 0: north halo (top unit), 1: south (bottom unit)
  const int xreads = halo_unit ? (u.links & 0x3f) : 0;          // 2-D direct: side ghosts read
  const int xpushes = halo_unit ? ((u.links >> 8) & 0x3f) : 0;  // 2-D direct: sides pushed to
  // A wave that does no work still counts: its halo signals, so gates and flags of launches
  // already queued on other streams and ranks stay in step (and a failed launch is reported by
  // the host's poll instead of a neighbour's wait running into its timeout), and its serial-
  // pipeline wave count.
  auto skip_unit = [&]() {
    if (ns_unit && gp(a.sig[dir]) != nullptr && lane == 0)
      __hip_atomic_fetch_add(gp(a.sig[dir]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 0)
      for (int i = 0; i < kSideLinks; ++i)
        if ((xpushes >> i) & 1) __hip_atomic_fetch_add(gp(a.xsig[i]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 0 && gp(a.waves_done) != nullptr)
      __hip_atomic_fetch_add(gp(a.waves_done), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if (lid != 0ull) {
    // integrity (wave-uniform, scalar): the launch names this block, the unit comes from the
    // list the block names, and (serial pipeline) the exchange copy in front of this launch has
    // finished — else report and skip
    unsigned bad = a.head.btag != btag ? kIntegArgs : u.tag != a.utag ? kIntegUnits : 0u;
    if (bad == 0u && w == 0 && gp(a.copies_done) != nullptr &&
        __hip_atomic_load(gp(a.copies_done), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != copies_need)
      bad = kIntegOrder;
    if (bad != 0u) {
      if (lane == 0) report_timeout(gp(a.timed_out), gp(a.timed_out_host), bad);
      skip_unit();
      return;
    }
  }
  // replay check: launch ids rise in stream order, so an older or equal id seen already means this
  // launch ran with the arguments of an earlier one.  Issued here, its value is checked at the
  // wave's end (the atomic's round trip overlaps the work instead of delaying the launch's end).
  // Every other wave reads the highest id seen: engine launches all run in order on one stream,
  // so a wave whose per-launch part names an id below it ran with an older launch's arguments
  // (a wave of the same launch may have raised it to lid already; an older id never passes).
  unsigned long long lid_old = 0ull;
  const bool replay_check = lane == 0 && lid != 0ull && gp(a.lid_seen) != nullptr;
  if (replay_check) {
    if (w == 0) lid_old = __hip_atomic_fetch_max(gp(a.lid_seen), lid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else lid_old = __hip_atomic_load(gp(a.lid_seen), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (gp(a.stop) != nullptr && __hip_atomic_load(gp(a.stop), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull) {
    skip_unit();  // converged earlier in this run: no work
    return;
  }
  const bool ns_wait = ns_unit && gp(a.wait[dir]) != nullptr;
  if (ns_wait || xreads != 0) {
    // wait until the exchange that fills this unit's ghost rows has landed (a wait that already
    // timed out in this engine stops every later wait: fail fast)
    if (__hip_atomic_load(gp(a.timed_out), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      // every flag this unit needs is polled at once, one per lane (lanes 0-5: the side links,
      // lane 6: the N/S flag) — one round trip per poll, not one per flag; relaxed polls (an
      // acquire per poll is 2-3x slower per hop), ONE acquire after the match
      const unsigned long long* wp = nullptr;
      unsigned long long wneed = 0;
#pragma unroll
      for (int x = 0; x < kSideLinks; ++x)
        if (lane == x && ((xreads >> x) & 1) != 0) {
          wp = gp(a.xwait[x]);
          wneed = need.v[2 + x];
        }
      if (lane == kSideLinks && ns_wait) {
        wp = gp(a.wait[dir]);
        wneed = dir ? need.v[1] : need.v[0];
      }
      bool pending = wp != nullptr;
      for (long long i = 0;; ++i) {
        if (pending) pending = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < wneed;
        if (__ballot(pending) == 0ull) break;
        if (i >= a.halo_polls) {
          if (lane == 0) report_timeout(gp(a.timed_out), gp(a.timed_out_host), 2u);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (gp(a.wait_acc) != nullptr && lane == 0) {  // exposed halo wait of this unit (fire-and-forget atomics)
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
        __hip_atomic_fetch_add(gp(a.wait_acc), dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(gp(a.wait_acc) + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(gp(a.wait_acc) + 2, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // acq 0: system scope; 1: agent scope (this CU's L1); 2: the ghost rows are in uncached
    // memory and were polled for: only keep the compiler from hoisting their loads
    if (a.acq == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    else if (a.acq == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const unsigned long long t_ready = stamping ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const int64_t x0 = u.x0;
  const int h = u.h;
  const int64_t cb = (int64_t)u.cb + 4 * lane;

  // kUnitReverse: stream the unit's rows bottom-up (negative pitches)
  const bool rev = (u.flags & kUnitReverse) != 0;
  const int64_t xin = rev ? x0 + h - 1 + K : x0 - K;  // first stream row (tile row)
  const int64_t xout = rev ? x0 + h - 1 : x0;         // first output row
  LaneCtx c;
  c.gxb = a.gx0 + xin;
  c.dir = rev ? -1 : 1;
  const int64_t gc = a.gy0 + cb;
  const bool fixed = a.fixed != 0;
  c.rlo = a.per_x ? INT64_MIN : 0;
  c.rhi = a.per_x ? (fixed ? INT64_MIN : INT64_MAX) : (fixed ? a.NX - 1 : a.NX);
  auto colmask = [&](int64_t q) {
    return a.per_y ? false : fixed ? (q == 0 || q == a.NY - 1) : (q < 0 || q >= a.NY);
  };
  c.m0 = colmask(gc + 0);
  c.m1 = colmask(gc + 1);
  c.m2 = colmask(gc + 2);
  c.m3 = colmask(gc + 3);
  // Lanes in the output range store a full float4 (columns past ycell land in the ghost /
  // pad columns inside the pitch and hold valid cone values there); others hit a dummy slot.
  const bool in_out = (cb >= u.olo) && (cb < u.ohi);
  float* out = gp(a.dst) + (a.G + xout) * a.pitch + a.PL + cb;
  c.sout = in_out ? out : gp(a.dummy) + 4 * lane;
  c.spitch = in_out ? (rev ? -a.pitch : a.pitch) : 0;
  c.obase = gp(a.dst) + (a.G + x0) * a.pitch + a.PL + u.cb;
  c.obs = (int)((rev ? -a.pitch : a.pitch) * (int64_t)sizeof(float));
  c.obo = rev ? (h - 1) * (int)(a.pitch * (int64_t)sizeof(float)) : 0;
  c.voff = in_out ? 16u * (unsigned)lane : 0x80000000u;
  c.st0 = in_out;
  c.st1 = in_out && cb + 1 < a.ycell;
  c.st2 = in_out && cb + 2 < a.ycell;
  c.st3 = in_out && cb + 3 < a.ycell;
  const bool pushes = ns_unit && gp(a.push[dir]) != nullptr;
  c.prows = pushes ? a.sig_rows : 0;
  c.rel = a.rel;
  const bool keeps = gp(a.keep) != nullptr && in_out;
  c.kout = keeps ? gp(a.keep) + (out - gp(a.dst)) : gp(a.dummy) + 4 * lane;
  c.kpitch = keeps ? c.spitch : 0;
  c.pout = (pushes && in_out) ? gp(a.push[dir]) + xout * a.pitch + a.PL + cb : gp(a.dummy) + 4 * lane;
  c.ppitch = (pushes && in_out) ? (rev ? -a.pitch : a.pitch) : 0;

  // 2-D direct side pushes: this lane's elements in the W / E neighbour's halo columns
  c.spu = xpushes != 0;
  c.em = 0u;
  c.sp = c.cn = c.cs = nullptr;
  c.sps = c.cns = c.css = 0;
  c.xr0 = xout;
  c.xdir = rev ? -1 : 1;
  c.xlo = a.G;
  c.xhi = a.xcell - a.G;
  if (c.spu && in_out) {
    const bool wl = cb < a.G && (xpushes & (kLinkW | kLinkNW | kLinkSW)) != 0;
    const bool el = cb + 3 >= a.ycell - a.G && (xpushes & (kLinkE | kLinkNE | kLinkSE)) != 0;
    for (int e = 0; e < 4; ++e) {
      const int64_t q = cb + e;
      if ((wl && q < a.G) || (el && !wl && q >= a.ycell - a.G && q < a.ycell)) c.em |= 1u << e;
    }
    const int side = wl ? 0 : 1, cn = wl ? 2 : 3, cs = wl ? 4 : 5;  // link index W/E, NW/NE, SW/SE
    const int64_t sgn = rev ? -1 : 1;
    if (c.em != 0u) {
      if ((xpushes >> side) & 1) {
        c.sp = gp(a.xpush[side]) + xout * a.xpitch[side] + cb;
        c.sps = sgn * a.xpitch[side];
      }
      if ((xpushes >> cn) & 1) {
        c.cn = gp(a.xpush[cn]) + xout * a.xpitch[cn] + cb;
        c.cns = sgn * a.xpitch[cn];
      }
      if ((xpushes >> cs) & 1) {
        c.cs = gp(a.xpush[cs]) + xout * a.xpitch[cs] + cb;
        c.css = sgn * a.xpitch[cs];
      }
    }
  }

  const int64_t soff = (a.G + xin) * a.pitch + a.PL + cb;
  const float4* rowp = reinterpret_cast<const float4*>(gp(a.src) + soff);
  const float4* hrowp = (ns_unit && gp(a.hsrc[dir]) != nullptr) ? reinterpret_cast<const float4*>(gp(a.hsrc[dir]) + soff)
                                                            : rowp;
  // 2-D direct: lanes entirely left of column 0 / at or right of ycell are ghost columns — they
  // read every row (corners included) from my receive groups (the same pitch as the tile)
  if (xreads != 0) {
    const int64_t rb = (a.G + xin) * a.pitch;
    if (cb < 0 && (xreads & (kLinkW | kLinkNW | kLinkSW)) != 0) {
      rowp = hrowp = reinterpret_cast<const float4*>(gp(a.gsrc[0]) + rb + kGhostGroup + cb);
    } else if (cb >= a.ycell && (xreads & (kLinkE | kLinkNE | kLinkSE)) != 0) {
      rowp = hrowp = reinterpret_cast<const float4*>(gp(a.gsrc[1]) + rb + min(cb - a.ycell, (int64_t)(kGhostGroup - 4)));
    }
  }
  const int64_t pitch4 = rev ? -(a.pitch >> 2) : (a.pitch >> 2);
  const int n = h + 2 * K;
  Coef k{a.cx, a.cy, (float)a.cx, (float)a.cy};
  double racc = 0.0;
  // signalling units: mid-unit signal point (or the end); others never signal
  unsigned long long* sig = ns_unit ? gp(a.sig[dir]) : nullptr;
  const int sig_at = sig == nullptr ? -1
                     : ((u.flags & kUnitSigEnd) != 0 || a.sig_rows <= 0) ? (1 << 30)
                                                                          : 2 * K + ((a.sig_rows + 3) & ~3);
  if (c.spu) {
    // side-pushing units of the 2-D direct pipeline: their own bodies, so the push code costs the
    // common bodies no registers (the host never gives such a unit a column-edge window)
    if ((u.flags & 3) == 0) run_unit<K, F32, 0, false, RESID, WT, true, true>(rowp, hrowp, pitch4, n, c, k, racc, sig_at, sig, lane);
    else run_edge<K, F32, RESID, WT, 2, true, true>(rowp, hrowp, pitch4, n, c, k, racc, fixed, sig_at, sig, lane);
  } else if (sig != nullptr || c.prows > 0 || (a.dbg & 1) != 0) {
    // halo units (a few per launch): plain or fully masked bodies (the masks are a no-op wherever
    // the unit's flags say no edge, periodic dimensions included)
    if ((u.flags & 3) == 0) run_unit<K, F32, 0, false, RESID, WT, false, true>(rowp, hrowp, pitch4, n, c, k, racc, sig_at, sig, lane);
    else run_edge<K, F32, RESID, WT, 3, false, true>(rowp, hrowp, pitch4, n, c, k, racc, fixed, sig_at, sig, lane);
  } else {
    run_plain<K, F32, RESID, WT>(u, rowp, hrowp, pitch4, n, c, k, racc, fixed, sig_at, sig, lane);
  }
  if (xpushes != 0) {
    // side and corner pushes are complete: drain, release as the N/S signal does, then one
    // count per neighbour pushed to
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (a.rel == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    else if (a.rel == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (lane == 0)
      for (int i = 0; i < kSideLinks; ++i)
        if ((xpushes >> i) & 1) __hip_atomic_fetch_add(gp(a.xsig[i]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if constexpr (RESID) {
    racc = dpp_wave_sum(racc);
    int slot = w + a.prot;
    if (slot >= a.nunits) slot -= a.nunits;
    DecideArgs dec = a.dec;
    dec.seq = seq;
    publish_partial(gp(a.partials), slot, racc, a.nunits, dec, lane);
  }
  if (replay_check && (w == 0 ? lid_old >= lid : lid_old > lid))
    report_timeout(gp(a.timed_out), gp(a.timed_out_host), kIntegReplay);
  if (gp(a.waves_done) != nullptr) {
    // serial pipeline: this wave's stores are complete — the next exchange copy checks that every
    // wave of the launches before it got here
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(gp(a.waves_done), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (stamping) {
    // the wave's stores have drained: its work is done, not just issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    const unsigned hw = (__builtin_amdgcn_s_getreg((31 << 11) | 20) << 16) | (__builtin_amdgcn_s_getreg((31 << 11) | 4) & 0xffffu);
    if (lane == 0) {
      unsigned long long* s = gp(a.stamps) + 4 * (int64_t)w;
      s[0] = t_start;
      s[1] = t_ready;
      s[2] = t_end;
      s[3] = hw;
    }
  }
}

}  // namespace

// One (K, precision, residual) variant of the launch, both store flavours.  Each variant is
// instantiated in its own generated translation unit (heat2d_amd/_build.py writes
// build/gen/stream_k<K>_f<F32>r<RESID>.hip), so the 44 stencil objects compile in parallel.
template <int K, bool F32, bool RESID>
void launch_stream_kv(const StreamArgs* blk, const StreamDyn& d, bool wt, hipStream_t s) {
  // nunits == 0: a no-op launch (warm_kernels); a pending decision: one more (deciding) block
  const int blocks = std::max(1, (d.nunits + 3) / 4 + (d.pend ? 1 : 0));
  StreamNeed need;
  for (int i = 0; i < kNumDirs; ++i) need.v[i] = d.need[i];
  void (*fn)(const StreamArgs*, unsigned long long, unsigned long long, unsigned long long, unsigned, StreamNeed) =
      wt ? stream_kernel<K, F32, RESID, true> : stream_kernel<K, F32, RESID, false>;
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, s, blk, d.lid, d.copies_need, d.seq, d.btag, need);
}

template <int K, bool F32, bool RESID>
int stream_blocks_per_cu_v() {
  void (*fn)(const StreamArgs*, unsigned long long, unsigned long long, unsigned long long, unsigned, StreamNeed) =
      stream_kernel<K, F32, RESID, false>;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(fn), 256, 0) != hipSuccess) return 1;
  return nb > 0 ? nb : 1;
}

}  // namespace h2d
