// heat2d_amd — persistent, pipelined variant of the streaming stencil (gfx950).
//
// The launch-per-chunk streaming kernel (stream_kernel.hpp) pays, per chunk, a dependent kernel
// boundary (~1.4 us), the dispatch and unit-record load (~0.8 us), and a cold start of every
// wave: its 2K prologue rows all arrive one memory round trip after the launch, and its last
// stores drain before the grid ends (measured with the per-wave timeline: ~3.3 us of fixed
// body time per unit).  At 512 x 4096 per GPU (4096^2 over 8 GPUs) that is ~40 % of a launch.
//
// Here ONE launch runs J chunks.  Every wave keeps its work unit; units form an aligned grid
// (all column strips cut at the same row bands), band i streams DOWN for even i and UP for odd
// i, so the rows a unit's K-cone needs first from the band above / below are the rows that
// band produces FIRST.  A unit starts chunk j as soon as the rows it is about to load from its
// eight neighbours' chunk j-1 outputs are published — per row, not per grid.
//
// Hand-off (MI355X guide, Guideline 16 R1 / visibility table row 1): every output row is
// stored write-through (buffer_store sc1); a wave publishes "rows complete" in its own progress
// word with an agent-scope atomic store only after an `s_waitcnt vmcnt(2 RI)` at a steady-loop
// iteration top — every store issued before the previous top has completed, so the publication
// lags one iteration and never stalls; consumers poll progress words with relaxed agent loads
// (one vector load: lane l reads neighbour slot l) and read tile rows with sc1 buffer loads
// only (L1 bypass), so no acquire fence is needed.  The polls are issued one iteration ahead;
// a wave stalls only if a neighbour really is behind.
//
// Direct (IPC) halo units keep the launch-per-chunk protocol per chunk: wait on the flag, read
// ghost rows from the receive buffer of the chunk's parity, push the first G output rows into
// the neighbour's buffer of the other parity and signal once those stores have completed.
//
// Deadlock freedom: a unit publishes everything it has completed before every wait, and chunk
// j's outputs never depend on chunk j+1, so by induction over j every wait is eventually met.
// Every launch's waves must all be resident (the host checks occupancy); every wait is bounded
// and reports through the engine's timeout words.
#pragma once
#include "stream_kernel.hpp"

namespace h2d {
namespace {

// sc1 (L1-bypassing, coherent for write-through hand-offs) row load of one lane: 16 bytes
// (4 columns per lane, 256-column strips) or 8 bytes (2 columns, 128-column strips).
template <class V>
__device__ __forceinline__ V load_row_sc1(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff);
template <>
__device__ __forceinline__ float4 load_row_sc1<float4>(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, 16 /* sc1 */);
  return make_float4(__uint_as_float(d.x), __uint_as_float(d.y), __uint_as_float(d.z), __uint_as_float(d.w));
}
template <>
__device__ __forceinline__ float2 load_row_sc1<float2>(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  const u32x2 d = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, soff, 16 /* sc1 */);
  return make_float2(__uint_as_float(d.x), __uint_as_float(d.y));
}

template <int CPL>
struct LaneVec;
template <>
struct LaneVec<4> {
  typedef float4 T;
};
template <>
struct LaneVec<2> {
  typedef float2 T;
};

// Lane l < kPSlots holds neighbour slot l; other lanes are inert (nb < 0).
struct PSlot {
  int nb, rlo, rhi, qa, qs, hv;
  unsigned known;  // latest progress seen
};

// Progress the rows [A, B) of my stream need from this lane's neighbour (its chunk cprev).
__device__ __forceinline__ unsigned pneed(const PSlot& d, int A, int B, unsigned cprev) {
  const int lo = max(A, d.rlo), hi = min(B, d.rhi);
  if (d.nb < 0 || lo >= hi) return 0u;
  const int r = d.qs > 0 ? hi - 1 : lo;
  return cprev * (unsigned)d.hv + (unsigned)(d.qa + d.qs * r + 1);
}

// Progress words are accessed through global (address space 1) pointers: global_load / global_store
// complete in issue order with the buffer loads and stores of the rows, so the counted
// `s_waitcnt vmcnt(N)` of the publishing top stays valid, and hipcc waits for a poll's value with
// a counted vmcnt instead of the vmcnt(0) + lgkmcnt(0) a flat (generic) access forces — a drain of
// every outstanding row store at every iteration top (MI355X guide: flat_* return out of order).
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ unsigned ppoll(const PSlot& d, const unsigned* prog) {
  return d.nb >= 0 ? __hip_atomic_load((const gu32*)(prog + 32 * d.nb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : 0xffffffffu;
}

// Wait until every neighbour has published what rows [A, B) need (bounded).  false: gave up.
__device__ __forceinline__ bool pensure(PSlot& d, int A, int B, unsigned cprev, const unsigned* prog,
                                        const PStreamArgs& a, bool& dead) {
  const unsigned nd = pneed(d, A, B, cprev);
  if (dead || __ballot(nd > d.known) == 0ull) return true;
  for (long long i = 0;; ++i) {
    const unsigned v = ppoll(d, prog);
    d.known = max(d.known, v);
    if (__ballot(nd > d.known) == 0ull) return true;
    if (i > a.halo_polls ||
        ((i & 63) == 63 && __hip_atomic_load(gp(a.timed_out), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
      if (__lane_id() == 0) report_timeout(gp(a.timed_out), gp(a.timed_out_host), 8u);
      dead = true;
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ void ppublish(unsigned* p, unsigned v, int lane) {
  if (lane == 0) __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The direct pipeline's flag signal of a halo unit for chunk `jc` of the launch (its pushed rows'
// stores have completed: the pushes are global stores, in issue order with the row stores the
// publishing top's counted vmcnt covers).  First, bounded, every halo unit of this rank and
// direction must have signalled chunk jc-1 (PStreamArgs::lsig): the neighbour's flag then only
// ever counts whole chunks.
__device__ __forceinline__ void psignal(unsigned long long* sig, int rel, int lane, unsigned long long* lsig,
                                        unsigned long long lneed, const PStreamArgs& a, bool& dead) {
  if (lsig != nullptr && !dead) {
    int gave_up = 0;
    if (lane == 0) {
      long long i = 0;
      while (__hip_atomic_load(lsig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < lneed) {
        // bounded; and a wait that failed elsewhere in the engine ends this one too (fail fast:
        // one failure must not cost every later chunk's signal a full timeout)
        if (++i > a.halo_polls ||
            ((i & 63) == 0 && __hip_atomic_load(gp(a.timed_out), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
          report_timeout(gp(a.timed_out), gp(a.timed_out_host), 8u);
          gave_up = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (__builtin_amdgcn_readfirstlane(gave_up) != 0) dead = true;
  }
  if (rel == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  else if (rel == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if (rel != 2) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (lane == 0) {
    __hip_atomic_fetch_add(sig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lsig != nullptr) __hip_atomic_fetch_add(lsig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// PUSH: a direct-pipeline halo unit (copies its first rows to the neighbour GPU each chunk); the
// other units' steady loop carries no per-row push check.
template <int K, bool F32, int EDGE, bool FIXED, int CPL, bool PUSH, bool PP>
__device__ __forceinline__ void prun(const PStreamArgs& a, const PStreamDyn& d, const Unit& u, int w, int lane,
                                     PSlot& sl) {
  typedef typename LaneVec<CPL>::T V;
  // rows per steady iteration (8 for 2-column lanes was measured slower: 512x4096 K=8 2.21 vs
  // 1.91 us/step — its rows are published an iteration later, so the neighbours start later)
  constexpr int RI = 4;
  // publish (drain to the iteration before, store the progress word, poll the neighbours) at
  // every PE-th iteration top of a 2-column lane (H2D_PSTREAM_PE2).  Measured: every 2nd top is
  // slower (512x4096 K=8 2.21 vs 1.93 us/step) although it halves the drains — fresh progress
  // words matter more to the neighbours than the exposed store latency costs this wave.
#ifndef H2D_PSTREAM_PE2
#define H2D_PSTREAM_PE2 1
#endif
  constexpr int PE = CPL == 2 ? H2D_PSTREAM_PE2 : 1;
  const int h = u.h, n = h + 2 * K;
  const bool rev = (u.flags & kUnitReverse) != 0;
  const bool ns = (u.flags & kUnitNS) != 0;
  const int dir = rev ? 1 : 0;
  const int64_t x0 = u.x0;
  const int64_t cb = (int64_t)u.cb + CPL * lane;
  const int64_t xin = rev ? x0 + h - 1 + K : x0 - K;
  const int64_t xout = rev ? x0 + h - 1 : x0;
  const int pb = (int)(a.pitch * (int64_t)sizeof(float));  // row bytes (the host keeps n * pb < 2^31)
  const Coef k{a.cx, a.cy, (float)a.cx, (float)a.cy};
  unsigned* myprog = gp(a.prog) + 32 * w;

  // chunk-invariant lane context (stream_kernel's, write-through stores, no residual / sides)
  LaneCtx c;
  c.gxb = a.gx0 + xin;
  c.dir = rev ? -1 : 1;
  c.rlo = a.per_x ? INT64_MIN : 0;
  c.rhi = a.per_x ? (a.fixed ? INT64_MIN : INT64_MAX) : (a.fixed ? a.NX - 1 : a.NX);
  const int64_t gc = a.gy0 + cb;
  auto colmask = [&](int64_t q) {
    return a.per_y ? false : a.fixed ? (q == 0 || q == a.NY - 1) : (q < 0 || q >= a.NY);
  };
  c.m0 = colmask(gc + 0);
  c.m1 = colmask(gc + 1);
  c.m2 = CPL > 2 && colmask(gc + 2);
  c.m3 = CPL > 2 && colmask(gc + 3);
  const bool in_out = (cb >= u.olo) && (cb < u.ohi);
  c.sout = gp(a.dummy) + CPL * lane;  // unused: write-through path
  c.spitch = 0;
  c.obs = rev ? -pb : pb;
  c.obo = rev ? (h - 1) * pb : 0;
  c.voff = in_out ? 4u * CPL * (unsigned)lane : 0x80000000u;
  c.st0 = c.st1 = c.st2 = c.st3 = false;
  c.kout = gp(a.dummy) + CPL * lane;
  c.kpitch = 0;
  c.rel = a.rel;
  c.spu = false;
  c.em = 0u;
  c.sp = c.cn = c.cs = nullptr;
  c.sps = c.cns = c.css = 0;
  c.xr0 = xout;
  c.xdir = rev ? -1 : 1;
  c.xlo = a.G;
  c.xhi = a.xcell - a.G;
  // direction-resolved halo pointers: selects, not runtime-indexed kernel-argument arrays (a
  // runtime index into the argument block made hipcc copy the whole block to scratch and reload
  // fields from it at every iteration top)
  const unsigned long long* const waitd = rev ? gp(a.wait[1]) : gp(a.wait[0]);
  const unsigned long long need0 = rev ? d.need0[1] : d.need0[0];
  const unsigned long long needinc = rev ? a.need_inc[1] : a.need_inc[0];
  const float* const hsrc0 = rev ? gp(a.hsrc[1][0]) : gp(a.hsrc[0][0]);
  const float* const hsrc1 = rev ? gp(a.hsrc[1][1]) : gp(a.hsrc[0][1]);
  float* const push0 = rev ? gp(a.push[1][0]) : gp(a.push[0][0]);
  float* const push1 = rev ? gp(a.push[1][1]) : gp(a.push[0][1]);
  unsigned long long* const sigd = rev ? gp(a.sig[1]) : gp(a.sig[0]);
  unsigned long long* const lsigd = rev ? gp(a.lsig[1]) : gp(a.lsig[0]);
  const unsigned long long lbased = rev ? d.lbase[1] : d.lbase[0];
  const unsigned long long lperd = (unsigned long long)(rev ? a.lper[1] : a.lper[0]);
  const bool pushes = PUSH && ns && push0 != nullptr;
  c.prows = pushes ? a.sig_rows : 0;
  const int64_t in_base = (a.G + x0 - K) * a.pitch + a.PL + u.cb;  // lowest input row, lane 0
  const int64_t out_base = (a.G + x0) * a.pitch + a.PL + u.cb;     // lowest output row, lane 0
  const int64_t lane_in = (a.G + xin) * a.pitch + a.PL + cb;       // first stream row, this lane
  const int64_t pitchv = rev ? -(a.pitch / CPL) : (a.pitch / CPL);  // a row, in lane vectors
  const unsigned lvoff = 4u * CPL * (unsigned)lane;
  auto soff = [&](int r) { return rev ? (n - 1 - r) * pb : r * pb; };

  bool dead = false;         // a wait gave up: finish without waiting (the host reports it)
  bool sig_pending = false;  // a halo unit's pushes of its last chunk are not yet signalled
  int sig_chunk = 0;         // ... of that chunk
  double racc = 0.0;
  // diagnostics: per-phase time of this wave, compiled in only with -DH2D_PSTREAM_PHASES (even
  // an untaken runtime branch per iteration top cost ~30 % at 512x4096: the timers' registers
  // and the loop's scheduling)
#ifdef H2D_PSTREAM_PHASES
  const bool tm = gp(a.phase) != nullptr;
  unsigned long long ph[kPhases] = {};
  unsigned long long tq = tm ? __builtin_amdgcn_s_memrealtime() : 0ull;
  auto lap = [&](int i) {
    if (tm) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      ph[i] += t - tq;
      tq = t;
    }
  };
#else
  auto lap = [](int) {};
#endif
  for (int j = 0; j < d.nchunks; ++j) {
    const unsigned cidx = d.cbase + (unsigned)j;
    const int par = (d.cur0 + j) & 1;
    const float* src = par ? gp(a.buf[1]) : gp(a.buf[0]);
    float* dst = par ? gp(a.buf[0]) : gp(a.buf[1]);
    const int ipar = (d.ipar0 + j) & 1;
    if (j > 0) {
      // chunk start: my previous chunk's stores complete (the poll's wait drains them), publish
      // them, then the rows the up-front batch loads must be published by the neighbours
      lap(5);
      const unsigned pv = ppoll(sl, gp(a.prog));
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      ppublish(myprog, cidx * (unsigned)h, lane);
      if (sig_pending) {
        psignal(sigd, a.rel, lane, lsigd, lbased + (unsigned long long)sig_chunk * lperd, a, dead);
        sig_pending = false;
      }
      sl.known = max(sl.known, pv);
      lap(1);
      pensure(sl, 0, min(n, 2 * K + RI), cidx - 1u, gp(a.prog), a, dead);
      lap(2);
    }
    const V* hrowp = nullptr;
    if (ns && waitd != nullptr) {
      // the neighbour GPU's pushes of its chunk j-1 (this chunk's ghost rows)
      if (lane == 0 && !dead && __hip_atomic_load(gp(a.timed_out), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
        const unsigned long long need = need0 + (unsigned long long)j * needinc;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        long long i = 0;
        while (__hip_atomic_load(waitd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < need) {
          if (++i > a.halo_polls) {
            report_timeout(gp(a.timed_out), gp(a.timed_out_host), 2u);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        if (gp(a.wait_acc) != nullptr) {
          const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
          __hip_atomic_fetch_add(gp(a.wait_acc), dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(gp(a.wait_acc) + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_max(gp(a.wait_acc) + 2, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (a.acq == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      else if (a.acq == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      hrowp = reinterpret_cast<const V*>((ipar ? hsrc1 : hsrc0) + lane_in);
      lap(3);
    }
    c.obase = dst + out_base;
    c.pout = (pushes && in_out) ? (ipar ? push0 : push1) + xout * a.pitch + a.PL + cb : gp(a.dummy) + CPL * lane;
    c.ppitch = (pushes && in_out) ? (rev ? -a.pitch : a.pitch) : 0;
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src) + in_base, (short)0, n * pb, 0x00020000);

    V S[K][2];
#pragma unroll
    for (int t = 0; t < K; ++t) {
      S[t][0] = V{};
      S[t][1] = V{};
    }
    V pro[2 * K];
#pragma unroll
    for (int i = 0; i < 2 * K; ++i) pro[i] = (i < K && hrowp != nullptr) ? hrowp[(int64_t)i * pitchv]
                                                                        : load_row_sc1<V>(rin, lvoff, soff(i));
    V pf[RI];
#pragma unroll
    for (int d = 0; d < RI; ++d) pf[d] = load_row_sc1<V>(rin, lvoff, soff(min(2 * K + d, n - 1)));
    __builtin_amdgcn_sched_barrier(0);
    prologue<K, F32, EDGE, FIXED, false, true, false, PUSH, 0>(S, pro, c, k, racc);
    lap(4);

    int ir0 = 2 * K;
    int issued_prev = 0;  // output rows issued before the previous iteration top
    bool signalled = false;
    unsigned polled = 0u;
    bool have_poll = false;
    int it = 0;
    // One publishing top per RI rows: every op issued before the previous top has completed
    // (>= 8 VMEM ops since), so the progress word and the halo signal can go out, the neighbours'
    // words are polled (consumed at the next top), and the rows this iteration's loads need are
    // ensured.
#define H2D_PTOP()                                                                                \
  {                                                                                               \
    lap(5);                                                                                       \
    if (PE == 1 || (it++ % PE) == 0) {                                                            \
      if constexpr (RI == 8) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");                    \
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                                       \
      ppublish(myprog, cidx * (unsigned)h + (unsigned)issued_prev, lane);                         \
      if (pushes && !signalled && issued_prev >= a.sig_rows) { /* the pushed rows have completed */ \
        psignal(sigd, a.rel, lane, lsigd, lbased + (unsigned long long)j * lperd, a, dead);       \
        signalled = true;                                                                         \
      }                                                                                           \
      if (have_poll) sl.known = max(sl.known, polled);                                            \
      polled = ppoll(sl, gp(a.prog));                                                             \
      have_poll = true;                                                                           \
    }                                                                                             \
    issued_prev = ir0 - 2 * K;                                                                    \
    if (j > 0) pensure(sl, ir0 + RI, min(n, ir0 + 2 * RI), cidx - 1u, gp(a.prog), a, dead);       \
    lap(6);                                                                                       \
  }
    if constexpr (!PP) {
      // each row's replacement is loaded as the row is consumed (loop-carried register copies)
#define H2D_PSTEADY(D)                                                                \
  {                                                                                   \
    const V nw = pf[D];                                                               \
    pf[D] = load_row_sc1<V>(rin, lvoff, soff(min(ir0 + (D) + RI, n - 1)));            \
    process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, (D)&1, K>(S, nw, ir0 + (D), c, k, racc); \
  }
      for (; ir0 + RI <= n; ir0 += RI) {
        H2D_PTOP()
        H2D_PSTEADY(0)
        H2D_PSTEADY(1)
        H2D_PSTEADY(2)
        H2D_PSTEADY(3)
        if constexpr (RI == 8) {
          H2D_PSTEADY(4)
          H2D_PSTEADY(5)
          H2D_PSTEADY(6)
          H2D_PSTEADY(7)
        }
      }
#undef H2D_PSTEADY
    } else {
      // ping-pong: the next RI rows are loaded right after the top, a whole iteration ahead of
      // their use, into the register set the previous iteration consumed (as the streaming
      // kernel): no loop-carried register copies, whose waits drained the row stores too
#define H2D_PROW(CUR, D) \
  process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, (D)&1, K>(S, CUR[D], ir0 + (D), c, k, racc);
#define H2D_PITER(CUR, NXT)                                                         \
  {                                                                                 \
    H2D_PTOP()                                                                      \
    _Pragma("unroll") for (int d = 0; d < RI; ++d)                                  \
        NXT[d] = load_row_sc1<V>(rin, lvoff, soff(min(ir0 + d + RI, n - 1)));       \
    __builtin_amdgcn_sched_barrier(0);                                              \
    H2D_PROW(CUR, 0) H2D_PROW(CUR, 1) H2D_PROW(CUR, 2) H2D_PROW(CUR, 3)             \
    if constexpr (RI == 8) { H2D_PROW(CUR, 4) H2D_PROW(CUR, 5) H2D_PROW(CUR, 6) H2D_PROW(CUR, 7) } \
    ir0 += RI;                                                                      \
  }
      V nx[RI];
      while (ir0 + 2 * RI <= n) {
        H2D_PITER(pf, nx)
        H2D_PITER(nx, pf)
      }
      if (ir0 + RI <= n) {
        H2D_PITER(pf, nx)
#pragma unroll
        for (int d = 0; d < RI; ++d) pf[d] = nx[d];
      }
#undef H2D_PITER
#undef H2D_PROW
    }
#undef H2D_PTOP
    if (ir0 < n) process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, 0, K>(S, pf[0], ir0, c, k, racc);
    if (ir0 + 1 < n) process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, 1, K>(S, pf[1], ir0 + 1, c, k, racc);
    if (ir0 + 2 < n) process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, 0, K>(S, pf[2], ir0 + 2, c, k, racc);
    if constexpr (RI == 8) {
      if (ir0 + 3 < n) process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, 1, K>(S, pf[3], ir0 + 3, c, k, racc);
      if (ir0 + 4 < n) process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, 0, K>(S, pf[4], ir0 + 4, c, k, racc);
      if (ir0 + 5 < n) process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, 1, K>(S, pf[5], ir0 + 5, c, k, racc);
      if (ir0 + 6 < n) process_row<K, F32, EDGE, FIXED, false, true, false, PUSH, 0, K>(S, pf[6], ir0 + 6, c, k, racc);
    }
    if (have_poll) sl.known = max(sl.known, polled);
    // pushes not yet signalled at an iteration top: at the next chunk start (or launch end)
    if (pushes && !signalled) {
      sig_pending = true;
      sig_chunk = j;
    }
  }
  lap(5);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  ppublish(myprog, (d.cbase + (unsigned)d.nchunks) * (unsigned)h, lane);
  if (sig_pending) psignal(sigd, a.rel, lane, lsigd, lbased + (unsigned long long)sig_chunk * lperd, a, dead);
  lap(1);
#ifdef H2D_PSTREAM_PHASES
  if (tm && lane == 0) {
    ph[0] = (unsigned long long)d.nchunks;
#pragma unroll
    for (int i = 0; i < kPhases; ++i) __hip_atomic_fetch_add(gp(a.phase) + i, ph[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#endif
}

// The per-launch values arrive as scalar kernel arguments; prun sees them as a PStreamDyn.  PP: the
// ping-pong steady loop.
template <int K, bool F32, int CPL, bool PP>
__global__ __launch_bounds__(256) void pstream_kernel(const PStreamArgs* __restrict__ ap, unsigned long long need0n,
                                                      unsigned long long need0s, unsigned long long lbasen,
                                                      unsigned long long lbases, unsigned cbase, int nchunks,
                                                      int parities, unsigned btag) {
  // (read once, up front: see stream_kernel)
  asm volatile("" : "+s"(need0n), "+s"(need0s), "+s"(lbasen), "+s"(lbases), "+s"(cbase), "+s"(nchunks),
               "+s"(parities), "+s"(btag));
  PStreamDyn d;
  d.nchunks = nchunks;
  d.cbase = cbase;
  d.cur0 = parities & 1;
  d.ipar0 = (parities >> 1) & 1;
  d.btag = btag;
  d.need0[0] = need0n;
  d.need0[1] = need0s;
  d.lbase[0] = lbasen;
  d.lbase[1] = lbases;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int w = (int)blockIdx.x * 4 + wv;
  const PStreamArgs& a = *ap;  // the plan's immutable device-resident block (zero_arg_block: no-op)
  if (w >= a.nunits) return;
  const int lane = (int)(threadIdx.x & 63);
  if (a.head.btag != d.btag) {  // a block the launch does not name: report, compute nothing
    if (lane == 0) report_timeout(gp(a.timed_out), gp(a.timed_out_host), kIntegArgs);
    return;
  }
  if (gp(a.stop) != nullptr && __hip_atomic_load(gp(a.stop), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull)
    return;  // converged earlier in this run (PStreamArgs::stop)
  const PUnit* pu = gp(a.units) + w;
  const Unit u = pu->u;
  PSlot sl;
  if (lane < kPSlots) {
    sl.nb = pu->nb[lane];
    sl.rlo = pu->rlo[lane];
    sl.rhi = pu->rhi[lane];
    sl.qa = pu->qa[lane];
    sl.qs = pu->qs[lane];
    sl.hv = pu->hv[lane];
  } else {
    sl.nb = -1;
    sl.rlo = sl.rhi = sl.qa = sl.qs = sl.hv = 0;
  }
  sl.known = 0u;
  const bool fixed = a.fixed != 0;
  // one body family for every unit, the per-row push check included (measured: the push-free
  // straight-line body for the non-halo units was slower here — 1024x4096 direct 3.76 vs 3.42
  // us/step, 512x4096 2.21 vs 2.11: the publishing top's counted vmcnt waits on a steady loop
  // whose stores the scheduler had moved later)
  switch (u.flags & 3) {
    case 0: prun<K, F32, 0, false, CPL, true, PP>(a, d, u, w, lane, sl); break;
    case 1:
      if (fixed) prun<K, F32, 1, true, CPL, true, PP>(a, d, u, w, lane, sl);
      else prun<K, F32, 1, false, CPL, true, PP>(a, d, u, w, lane, sl);
      break;
    case 2:
      if (fixed) prun<K, F32, 2, true, CPL, true, PP>(a, d, u, w, lane, sl);
      else prun<K, F32, 2, false, CPL, true, PP>(a, d, u, w, lane, sl);
      break;
    default:
      if (fixed) prun<K, F32, 3, true, CPL, true, PP>(a, d, u, w, lane, sl);
      else prun<K, F32, 3, false, CPL, true, PP>(a, d, u, w, lane, sl);
      break;
  }
}

}  // namespace

template <int K, bool F32, int CPL>
void launch_pstream_kv(const PStreamArgs* blk, const PStreamDyn& d, bool pingpong, hipStream_t s) {
  const int blocks = std::max(1, (d.nunits + 3) / 4);  // nunits == 0: a no-op launch (warm_pstream_kernels)
  void (*fn)(const PStreamArgs*, unsigned long long, unsigned long long, unsigned long long, unsigned long long,
             unsigned, int, int, unsigned) = pingpong ? pstream_kernel<K, F32, CPL, true> : pstream_kernel<K, F32, CPL, false>;
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, s, blk, d.need0[0], d.need0[1], d.lbase[0], d.lbase[1], d.cbase,
                     d.nchunks, (d.cur0 & 1) | ((d.ipar0 & 1) << 1), d.btag);
}

template <int K, bool F32, int CPL>
int pstream_blocks_per_cu_v() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(pstream_kernel<K, F32, CPL, false>),
                                                   256, 0) != hipSuccess)
    return 0;
  return nb;
}

}  // namespace h2d
