// heat2d_amd — auxiliary HIP kernels (init, halo copies, reductions, naive step, the
// small-grid LDS-resident solver) and the streaming-kernel dispatch.  The streaming stencil
// itself lives in stream_kernel.hpp, instantiated per (K, precision, residual) in generated TUs.
// Compiled with -ffp-contract=off.
#include "stream_kernel.hpp"
#include "collectives.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace h2d {
namespace {

// ------------------------------------------------------------------------------------------
// Simple one-thread-per-cell step (validation baseline; same semantics, no temporal blocking).
// ------------------------------------------------------------------------------------------
template <bool F32>
__global__ __launch_bounds__(256) void naive_step_kernel(TileGeom g, const float* __restrict__ src,
                                                          float* __restrict__ dst, Coef k, int fixed, int per_x,
                                                          int per_y) {
  const int64_t j = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int64_t i = (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= g.xcell || j >= g.ycell) return;
  const int m = max(dim_mode(g.gx0 + i, g.NX, per_x != 0, fixed != 0), dim_mode(g.gy0 + j, g.NY, per_y != 0, fixed != 0));
  const int64_t c = g.idx(i, j);
  float v;
  if (m == 2) v = 0.0f;
  else if (m == 1) v = src[c];
  else v = cell<F32>(src[c], src[c - g.pitch], src[c + g.pitch], src[c - 1], src[c + 1], k);
  dst[c] = v;
}

__global__ void init_kernel(TileGeom g, float* __restrict__ base, int init) {
  const int64_t total = g.elems();
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / g.pitch - g.G;
    const int64_t j = e % g.pitch - g.PL;
    float v = 0.0f;
    if (i >= 0 && i < g.xcell && j >= 0 && j < g.ycell) v = init_value(init, g.gx0 + i, g.gy0 + j, g.NX, g.NY);
    base[e] = v;
  }
}

__global__ void poison_kernel(TileGeom g, float* __restrict__ base, int fixed, int per_x, int per_y) {
  const int64_t total = g.elems();
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / g.pitch - g.G, j = e % g.pitch - g.PL;
    if (poisonable(g, i, j, fixed != 0, per_x != 0, per_y != 0)) base[e] = __builtin_nanf("");
  }
}

__global__ void copy_rects_kernel(const CopyDesc* __restrict__ descs, int64_t tag, unsigned long long* done,
                                  unsigned int* integ, unsigned int* integ_host, const unsigned long long* waves_done,
                                  unsigned long long waves_need) {
  const CopyDesc d = descs[blockIdx.y];
  if (waves_done != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 &&
      __hip_atomic_load(waves_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != waves_need)
    report_timeout(integ, integ_host, kIntegOrder2);
  if (tag != 0 && d.tag != tag) {
    // a descriptor of another list (stale upload / reused allocation): copy nothing, report
    if (threadIdx.x == 0) report_timeout(integ, integ_host, kIntegDescs);
  } else {
    const int64_t total = d.rows * d.cols;
    // agent-coherent loads and write-through stores (agent-scope atomics = global_load / store
    // ... sc1), like the stencil's outputs: no dirty line of a ghost row stays in this XCD's L2,
    // and no stale line of the peer's edge rows is read from it
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
      const int64_t r = e / d.cols, cc = e - r * d.cols;
      __hip_atomic_store(d.dst + r * d.dst_pitch + cc,
                         __hip_atomic_load(d.src + r * d.src_pitch + cc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (done != nullptr) {
    // every thread's stores acknowledged, then one count for the block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Deterministic single-block sum (fixed summation order).
__global__ __launch_bounds__(256) void reduce_sum_kernel(const double* __restrict__ in, int n, double* __restrict__ out) {
  __shared__ double part[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += in[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = ((part[0] + part[1]) + part[2]) + part[3];
}

// Comm-stream gate of the signalled halo pipeline (see Engine::run_impl): one lane polls the
// boundary-unit counter with system-scope acquire loads.  Bounded: a gate that never opens
// reports a timeout instead of hanging the queue.
__global__ __launch_bounds__(64) void wait_counter_kernel(const unsigned long long* counter, unsigned long long target,
                                                          unsigned int* timed_out, unsigned int* timed_out_host,
                                                          long long max_polls) {
  if (threadIdx.x != 0) return;
  if (__hip_atomic_load(timed_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;  // fail fast
  for (long long i = 0; i < max_polls; ++i) {
    // relaxed: this wave reads no payload (the exchange kernel behind it acquires at its start)
    if (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= target) return;
    __builtin_amdgcn_s_sleep(4);
  }
  report_timeout(timed_out, timed_out_host, 1u);
}

// One wave's sum of n partials in a fixed order: 8 independent accumulators per lane, so each lane
// has 8 loads in flight (a single running sum waited for every load in turn: the check's
// all-reduce kernel took 11 µs for 1018 partials), then the wave sum.
__device__ __forceinline__ double wave_sum_partials(const double* __restrict__ p, int n, int lane) {
  double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int i = lane; i < n; i += 64 * 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i + 64 * j < n) acc[j] += p[i + 64 * j];
  }
  const double s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  return wave_sum(s);
}

// Scalar all-reduce over the IPC-mapped blocks of every rank (direct transport), one lane:
// publish my value into slot [parity][me] of every block (system-scope stores to the peers'
// uncached memory), release, bump every block's counter, wait (bounded) until mine shows all
// contributions of this epoch, then sum the slots in rank order — the same order on every
// rank, so every rank gets the same bits.
__global__ __launch_bounds__(64) void ipc_allreduce_kernel(double* local, double* out, char* const* blocks,
                                                           int me, int nr, int parity, unsigned long long target,
                                                           unsigned long long count_off, unsigned long long slot_off,
                                                           int max_ranks, long long max_polls, unsigned int* timed_out,
                                                           unsigned int* timed_out_host,
                                                           const unsigned long long* stop, DecideArgs d,
                                                           int decide, const double* parts, int nparts) {
  // after a converged check no rank contributes any more (each stops on its own schedule)
  if (stop != nullptr && __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull) return;
  // this rank's partials first, in one fixed order
  const double mine = parts != nullptr ? wave_sum_partials(parts, nparts, (int)threadIdx.x) : 0.0;
  if (threadIdx.x != 0) return;
  if (parts != nullptr) *local = mine;
  const unsigned long long v = __double_as_longlong(parts != nullptr ? mine : *local);
  for (int r = 0; r < nr; ++r) {
    unsigned long long* slot = reinterpret_cast<unsigned long long*>(blocks[r] + slot_off) + parity * max_ranks + me;
    __hip_atomic_store(slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // (system-scope release and acquire kept: dropping them, as the halo pushes to the same uncached
  // blocks do, measured no faster — the kernel's time is its chain of round trips,
  // profiles/conv_direct_r5.txt — and this path has not yet run across GPUs)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int r = 0; r < nr; ++r)
    __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(blocks[r] + count_off), 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long* cnt = reinterpret_cast<const unsigned long long*>(blocks[me] + count_off);
  long long i = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
    if (++i > max_polls) {
      report_timeout(timed_out, timed_out_host, 4u);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const unsigned long long* slots = reinterpret_cast<const unsigned long long*>(blocks[me] + slot_off) + parity * max_ranks;
  double sum = 0.0;
  for (int r = 0; r < nr; ++r)
    sum += __longlong_as_double(__hip_atomic_load(slots + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  *out = sum;
  if (decide) decide_total(sum, d);
}

__global__ __launch_bounds__(64) void decide_kernel(const double* sum, DecideArgs d) {
  if (threadIdx.x == 0) decide_total(*sum, d);
}

// Deterministic sum of n partials (one fixed order: wave_sum_partials) + the decision.
__global__ __launch_bounds__(64) void reduce_decide_kernel(const double* __restrict__ in, int n, DecideArgs d) {
  const double s = wave_sum_partials(in, n, (int)threadIdx.x);
  if (threadIdx.x == 0) {
    *d.total = s;
    decide_total(s, d);
  }
}

__global__ __launch_bounds__(64) void set_counter_kernel(unsigned long long* counter, unsigned long long value) {
  if (threadIdx.x == 0) __hip_atomic_store(counter, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void tile_residual_kernel(TileGeom g, const float* __restrict__ a,
                                                             const float* __restrict__ b, double* __restrict__ partials) {
  __shared__ double part[4];
  const int64_t total = g.xcell * g.ycell;
  double s = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / g.ycell, j = e % g.ycell;
    s += sq_diff(a[g.idx(i, j)], b[g.idx(i, j)]);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = ((part[0] + part[1]) + part[2]) + part[3];
}

// ------------------------------------------------------------------------------------------
// Small-grid resident solver: one 1024-thread workgroup keeps the whole grid in LDS and runs
// every time step (and the convergence test) without returning to the host.  Replaces
// ~2 launches/step of the reference CUDA program (grad1612_cuda_heat.cu:82-85) for grids up
// to 20480 cells, where a GPU is otherwise launch-latency bound.
// The LDS image carries a one-cell ring (zero, or the periodic wrap refreshed every step), so
// neighbour reads are fixed offsets; new values live in registers between the two barriers.
// ------------------------------------------------------------------------------------------
constexpr int kLdsCells = 20480;         // interior cells (160x128, the reference CUDA table's size)
constexpr int kLdsImage = 40960 - 256;   // ring-padded image, floats
constexpr int kLdsThreads = 1024;
constexpr int kLdsPerThread = kLdsCells / kLdsThreads;

template <bool F32>
__global__ __launch_bounds__(1024) void lds_solver_kernel(const float* __restrict__ in, int64_t in_pitch,
                                                           float* __restrict__ out, int64_t out_pitch, int NX, int NY,
                                                           long long steps, Coef k, int fixed, int per_x, int per_y,
                                                           int interval, double sens, long long* steps_done,
                                                           double* residual) {
  __shared__ float u[kLdsImage];
  __shared__ double red[16];
  __shared__ int stop_flag;
  const int tid = threadIdx.x;
  const int W = NY + 2;
  const int ncell = NX * NY;
  const int nimg = (NX + 2) * W;
  for (int e = tid; e < nimg; e += kLdsThreads) u[e] = 0.0f;
  __syncthreads();
  for (int e = tid; e < ncell; e += kLdsThreads) u[(e / NY + 1) * W + (e % NY) + 1] = in[(int64_t)(e / NY) * in_pitch + (e % NY)];
  // per-thread cells: LDS offsets and the fixed-edge hold mask
  int L[kLdsPerThread];
  unsigned hold = 0;
  {
    int i = tid / NY, j = tid % NY;
    const int di = kLdsThreads / NY, dj = kLdsThreads % NY;
#pragma unroll
    for (int q = 0; q < kLdsPerThread; ++q) {
      L[q] = (i + 1) * W + (j + 1);
      const bool h = fixed && ((!per_x && (i == 0 || i == NX - 1)) || (!per_y && (j == 0 || j == NY - 1)));
      hold |= (h ? 1u : 0u) << q;
      j += dj;
      i += di;
      if (j >= NY) {
        j -= NY;
        i += 1;
      }
    }
  }
  double last_res = -1.0;
  long long done = 0;
  __syncthreads();
  for (long long step = 1; step <= steps; ++step) {
    if (per_x || per_y) {  // refresh the periodic ring
      if (per_x)
        for (int j = tid; j < NY; j += kLdsThreads) {
          u[j + 1] = u[NX * W + j + 1];
          u[(NX + 1) * W + j + 1] = u[W + j + 1];
        }
      __syncthreads();
      if (per_y)
        for (int i = tid; i < NX + 2; i += kLdsThreads) {
          u[i * W] = u[i * W + NY];
          u[i * W + NY + 1] = u[i * W + 1];
        }
      __syncthreads();
    }
    const bool check = interval > 0 && (step % interval) == 0;
    float nv[kLdsPerThread];
    double racc = 0.0;
#pragma unroll
    for (int q = 0; q < kLdsPerThread; ++q) {
      if (tid + q * kLdsThreads < ncell) {
        const int c = L[q];
        const float cc = u[c];
        float v = cell<F32>(cc, u[c - W], u[c + W], u[c - 1], u[c + 1], k);
        v = ((hold >> q) & 1u) ? cc : v;
        nv[q] = v;
        if (check) racc += sq_diff(v, cc);
      }
    }
    if (check) {  // block-uniform
      racc = wave_sum(racc);
      if ((tid & 63) == 0) red[tid >> 6] = racc;
      __syncthreads();
      if (tid == 0) {
        double s = 0.0;
        for (int q = 0; q < kLdsThreads / 64; ++q) s += red[q];
        red[0] = s;
        stop_flag = s < sens;
      }
      __syncthreads();
      last_res = red[0];
      if (stop_flag) break;  // keep the pre-update grid: steps committed = step-1
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kLdsPerThread; ++q)
      if (tid + q * kLdsThreads < ncell) u[L[q]] = nv[q];
    __syncthreads();
    done = step;
  }
  for (int e = tid; e < ncell; e += kLdsThreads) out[(int64_t)(e / NY) * out_pitch + (e % NY)] = u[(e / NY + 1) * W + (e % NY) + 1];
  if (tid == 0) {
    *steps_done = done;
    *residual = last_res;
  }
}

}  // namespace

#define H2D_K_LIST(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(10) X(12) X(16)
// The variants live in generated translation units (heat2d_amd/_build.py: K_LIST there must
// match this list).
#define H2D_EXTERN(K)                                                                                          \
  extern template void launch_stream_kv<K, false, false>(const StreamArgs*, const StreamDyn&, bool, hipStream_t); \
  extern template void launch_stream_kv<K, false, true>(const StreamArgs*, const StreamDyn&, bool, hipStream_t);  \
  extern template void launch_stream_kv<K, true, false>(const StreamArgs*, const StreamDyn&, bool, hipStream_t);  \
  extern template void launch_stream_kv<K, true, true>(const StreamArgs*, const StreamDyn&, bool, hipStream_t);   \
  extern template int stream_blocks_per_cu_v<K, false, false>();                                \
  extern template int stream_blocks_per_cu_v<K, true, false>();
H2D_K_LIST(H2D_EXTERN)
#undef H2D_EXTERN

template <int K>
void launch_stream_k(const StreamArgs* blk, const StreamDyn& d, bool wt, bool f32, bool resid, hipStream_t s) {
  if (f32) {
    if (resid) launch_stream_kv<K, true, true>(blk, d, wt, s);
    else launch_stream_kv<K, true, false>(blk, d, wt, s);
  } else {
    if (resid) launch_stream_kv<K, false, true>(blk, d, wt, s);
    else launch_stream_kv<K, false, false>(blk, d, wt, s);
  }
}

template <int K>
int stream_blocks_per_cu(bool f32, bool /*resid*/) {
  return f32 ? stream_blocks_per_cu_v<K, true, false>() : stream_blocks_per_cu_v<K, false, false>();
}

int64_t stream_wave_capacity(int K, int precision, int device) {
  // The ref-precision stencil is VALU-bound (about 11 fp64-rate VALU ops per cell-step, one
  // wave issuing ~88 % of cycles): a second resident wave on a SIMD only splits that SIMD's
  // VALU, while halving every unit's height doubles the K-cone recompute share.  So one
  // wave per SIMD (measured on MI355X, 4096^2 K=8: 7.81 vs 8.04 us/step; 512x4096 K=6: 2.17
  // vs 3.13).  The fp32 path (3-4 VALU ops per cell) keeps the occupancy limit.
  int bpc = 1;
  const bool f32 = precision == kFp32;
  if (f32) {
    switch (K) {
#define H2D_CASE(KK) case KK: bpc = stream_blocks_per_cu<KK>(f32, false); break;
      H2D_K_LIST(H2D_CASE)
#undef H2D_CASE
      default: break;
    }
  }
  int cus = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) == hipSuccess && p.multiProcessorCount > 0) cus = p.multiProcessorCount;
  return (int64_t)bpc * cus * 4;
}

std::vector<Strip> strip_layout(const TileGeom& g, int K, bool fixed, bool per_y, int cpl) {
  const int64_t W = wave_cols(cpl), R = lead_cols(K, cpl), wout = W - 2 * R;
  const bool wide = fixed && !per_y && g.ycell >= W;
  const bool lo_edge = wide && g.gy0 == 0;
  const bool hi_edge = wide && g.gy0 + g.ycell == g.NY;
  std::vector<Strip> v;
  int64_t a = 0, b = g.ycell, rcb = 0;
  if (lo_edge) {
    v.push_back(Strip{0, 0, W - R});
    a = W - R;
  }
  if (hi_edge) {
    rcb = (g.ycell + cpl - 1) / cpl * cpl - W;  // window ends at the (lane-aligned) edge
    b = std::max(a, rcb + R);
  }
  for (int64_t p = a; p < b; p += wout) v.push_back(Strip{p - R, p, std::min(p + wout, b)});
  if (hi_edge && b < g.ycell) v.push_back(Strip{rcb, b, g.ycell});
  return v;
}

int unit_edge_flags(const TileGeom& g, int K, int64_t x0, int64_t h, int64_t cb, bool fixed, bool per_x, bool per_y,
                    int64_t wcols) {
  int f = 0;
  if (!per_y) {
    const int64_t lo = g.gy0 + cb, hi = lo + wcols - 1;  // the wave's column window
    const bool sp = fixed ? ((lo <= 0 && 0 <= hi) || (lo <= g.NY - 1 && g.NY - 1 <= hi)) : (lo < 0 || hi >= g.NY);
    if (sp) f |= kEdgeCols;
  }
  if (!per_x) {
    const int64_t lo = g.gx0 + x0 - K, hi = g.gx0 + x0 + h + K - 1;  // the unit's row cone
    const bool sp = fixed ? ((lo <= 0 && 0 <= hi) || (lo <= g.NX - 1 && g.NX - 1 <= hi)) : (lo < 0 || hi >= g.NX);
    if (sp) f |= kEdgeRows;
  }
  return f;
}

namespace {
struct RowRange {
  int64_t strip, a, b;  // rows [a, b) of strip
  bool edge;            // costs `w` per row (global-edge masks)
  bool edge_top = false, edge_bot = false;  // first / last unit is an edge unit (global edge rows)
  bool corner_top = false, corner_bot = false;  // ... of a column-edge strip: both masks (a corner unit)
  bool halo_top = false, halo_bot = false;  // first / last unit is a N / S halo unit (HaloCost)
  bool side = false;    // costs `side_weight` per row (pushes to a W / E neighbour)
};

// Cut every range into units of (nearly) equal cost, fitting `capacity` waves in one round.
// A unit of h rows costs ~ (h + K) wave-row-steps (the 2K-row prologue primes K levels); an
// edge unit costs w times more: target cost U -> h = U - K (plain) or U/w - K (edge).
std::vector<Unit> size_ranges(const TileGeom& g, int K, const std::vector<Strip>& strips,
                              const std::vector<RowRange>& ranges, int H, bool fixed, bool per_x, bool per_y,
                              double edge_weight, int64_t capacity, double row_edge_weight, double side_weight = 1.0,
                              const HaloCost& halo = HaloCost{}) {
  // edge units cost more per row: column-edge strips run the column-masked body on every row,
  // row-edge units (their K-cone reaches a global edge row) the row-masked one
  const double w = std::max(1.0, edge_weight);
  const double wr = std::max(1.0, row_edge_weight > 0 ? row_edge_weight : edge_weight);
  const double ws = std::max(1.0, side_weight);
  auto rows_for = [&](double U, bool edge) { return std::max<int64_t>(1, (int64_t)(edge ? U / w - K : U - K)); };
  auto rows_side = [&](double U) { return std::max<int64_t>(1, (int64_t)(U / ws - K)); };
  auto rows_row_edge = [&](double U) { return std::max<int64_t>(1, (int64_t)(U / wr - K)); };
  // a corner unit runs the row- AND column-masked body: measured per (h + K) at 4096^2 / 2048x4096,
  // K=7, relative to a plain unit: column edge 1.16 / 1.21, row edge 1.23 / 1.30, corner 1.29 /
  // 1.38 (tools/timeline.py --units) — sized as a column-edge unit it was the launch's last wave
  const double wc = std::max(w, wr) + 0.1;
  auto rows_corner = [&](double U) { return std::max<int64_t>(1, (int64_t)(U / wc - K)); };
  // a halo unit: its strip's weight, plus the rows its halo wait costs
  auto rows_halo = [&](double U, bool edge) {
    return std::max<int64_t>(std::max(1, halo.min_rows), (int64_t)((U - halo.rows) / (edge ? w : 1.0) - K));
  };
  auto plan = [&](double U, std::vector<Unit>* out) -> int64_t {
    int64_t count = 0;
    auto emit = [&](int64_t strip, int64_t a, int64_t b, int64_t target) {
      const int64_t len = b - a;
      if (len <= 0) return;
      const int64_t n = (len + target - 1) / target;
      count += n;
      if (out)
        for (int64_t i = 0; i < n; ++i) {
          const int64_t s0 = a + len * i / n, s1 = a + len * (i + 1) / n;
          const Strip& S = strips[(size_t)strip];
          out->push_back(Unit{(int)strip, (int)s0, (int)(s1 - s0),
                              unit_edge_flags(g, K, s0, s1 - s0, S.cb, fixed, per_x, per_y), (int)S.cb,
                              (int)S.lo, (int)S.hi});
        }
    };
    for (const RowRange& r : ranges) {
      int64_t a = r.a, b = r.b;
      const int64_t he = rows_row_edge(U), hc = rows_corner(U);
      if (r.edge_top && b > a) {
        const int64_t e = std::min(b, a + he);
        emit(r.strip, a, e, he);
        a = e;
      }
      if (r.edge_bot && b > a) {
        const int64_t e = std::max(a, b - he);
        emit(r.strip, e, b, he);
        b = e;
      }
      if (r.corner_top && b > a) {
        const int64_t e = std::min(b, a + hc);
        emit(r.strip, a, e, hc);
        a = e;
      }
      if (r.corner_bot && b > a) {
        const int64_t e = std::max(a, b - hc);
        emit(r.strip, e, b, hc);
        b = e;
      }
      if (r.halo_top && b > a) {
        const int64_t hh = rows_halo(U, r.edge), e = std::min(b, a + hh);
        emit(r.strip, a, e, hh);
        a = e;
      }
      if (r.halo_bot && b > a) {
        const int64_t hh = rows_halo(U, r.edge), e = std::max(a, b - hh);
        emit(r.strip, e, b, hh);
        b = e;
      }
      emit(r.strip, a, b, r.side ? rows_side(U) : rows_for(U, r.edge));
    }
    return count;
  };
  double U;
  if (H > 0) {
    U = (double)(H + K);
  } else {
    // Minimise the estimated makespan ceil(units / capacity) * U: one full round when the
    // tile has few strips (the usual case); several full rounds for huge tiles whose strips
    // alone outnumber the resident waves.  Units never go below 8 rows.
    const double umin = 8.0 + K, umax = (double)(g.xcell + K) * std::max(std::max(w, wr), ws) + 1.0;
    double best_u = umax, best_ms = 1e300;
    // fine steps: with ~60 units per strip a 3 % step left ~3 % of the wave slots empty
    // (4096^2: 993 of 1024 units)
    for (double u = umin; u <= umax * 1.0001; u *= 1.002) {
      const int64_t cnt = plan(u, nullptr);
      const double ms = (double)((cnt + capacity - 1) / std::max<int64_t>(1, capacity)) * u;
      if (ms < best_ms * 0.999 || (ms <= best_ms * 1.001 && u > best_u)) {
        best_ms = std::min(best_ms, ms);
        best_u = u;
      }
    }
    U = best_u;
  }
  std::vector<Unit> v;
  plan(U, &v);
  return v;
}
}  // namespace

UnitPlan plan_units(const TileGeom& g, int K, int H, bool fixed, bool per_x, bool per_y, double edge_weight,
                    int64_t capacity, const bool* peer, int hb, double row_edge_weight, double side_weight,
                    int side_cols, bool side_w, bool side_e, const HaloCost& halo) {
  UnitPlan P;
  const std::vector<Strip> strips = strip_layout(g, K, fixed, per_y);
  const int64_t nstrips = (int64_t)strips.size();
  hb = std::max(hb, K);
  const bool has_peer = peer && std::any_of(peer, peer + kNumDirs, [](bool b) { return b; });
  const bool top_bd = has_peer && (peer[kN] || peer[kNW] || peer[kNE]);
  const bool bot_bd = has_peer && (peer[kS] || peer[kSW] || peer[kSE]);
  std::vector<RowRange> in_r, bd_r;
  for (int64_t s = 0; s < nstrips; ++s) {
    const Strip& S = strips[(size_t)s];
    const int64_t y0 = S.lo, y1 = S.hi;
    const bool col_edge = unit_edge_flags(g, K, 0, 1, S.cb, fixed, true, per_y) & kEdgeCols;
    const bool row_edge_top = unit_edge_flags(g, K, 0, 1, S.cb, fixed, per_x, true) & kEdgeRows;
    const bool row_edge_bot = unit_edge_flags(g, K, g.xcell - 1, 1, S.cb, fixed, per_x, true) & kEdgeRows;
    const bool lr_bd = has_peer && ((y0 - K < 0 && (peer[kW] || peer[kNW] || peer[kSW])) ||
                                    (y1 + K > g.ycell && (peer[kE] || peer[kNE] || peer[kSE])));
    if (lr_bd) {
      bd_r.push_back(RowRange{s, 0, g.xcell, col_edge});
      continue;
    }
    int64_t top = top_bd ? std::min<int64_t>(g.xcell, hb) : 0;
    int64_t bot = bot_bd ? std::max<int64_t>(top, g.xcell - hb) : g.xcell;
    if (top > 0) bd_r.push_back(RowRange{s, 0, top, true});
    if (bot < g.xcell) bd_r.push_back(RowRange{s, bot, g.xcell, true});
    if (!has_peer) {
      // units whose K-cone reaches a global edge row are edge units (cost-balanced)
      RowRange r{s, 0, g.xcell, col_edge};
      r.side = (side_w && S.lo < side_cols) || (side_e && S.hi > g.ycell - side_cols);
      r.edge_top = !col_edge && !r.side && row_edge_top;
      r.edge_bot = !col_edge && !r.side && row_edge_bot;
      r.corner_top = col_edge && !r.side && row_edge_top;
      r.corner_bot = col_edge && !r.side && row_edge_bot;
      // (a strip end with a halo has a peer there, not a global edge row)
      r.halo_top = halo.n && !r.side && !row_edge_top;
      r.halo_bot = halo.s && !r.side && !row_edge_bot;
      in_r.push_back(r);
    } else {
      in_r.push_back(RowRange{s, top, bot, col_edge});
    }
  }
  P.interior = size_ranges(g, K, strips, in_r, H, fixed, per_x, per_y, edge_weight, capacity, row_edge_weight,
                           side_weight, halo);
  // Boundary units are short (hb rows): they run first, alone, and gate the halo exchange.
  P.boundary = size_ranges(g, K, strips, bd_r, hb, fixed, per_x, per_y, 1.0, capacity, 1.0);
  auto edge_first = [](const Unit& a, const Unit& b) { return (a.flags != 0) > (b.flags != 0); };
  std::stable_sort(P.interior.begin(), P.interior.end(), edge_first);
  return P;
}

std::vector<Unit> build_units(const TileGeom& g, int K, int H, bool fixed, bool per_x, bool per_y,
                              double edge_weight, int64_t capacity) {
  UnitPlan p = plan_units(g, K, H, fixed, per_x, per_y, edge_weight, capacity, nullptr, 16);
  return p.interior;
}

bool stream_k_supported(int K) {
  switch (K) {
#define H2D_CASE(KK) case KK: return true;
    H2D_K_LIST(H2D_CASE)
#undef H2D_CASE
    default: return false;
  }
}

void launch_stream(const StreamArgs* blk, const StreamArgs& a, const StreamDyn& d, int K, int precision,
                   bool residual, hipStream_t s) {
  if (a.nunits <= 0) return;
  if (lead_cols(K) != a.R || kWaveCols - 2 * a.R != a.wout) throw std::invalid_argument("launch_stream: R/wout mismatch");
  if (blk == nullptr || d.nunits != a.nunits || d.btag != a.head.btag || d.pend != (a.pend != nullptr))
    throw std::invalid_argument("launch_stream: the launch does not name its argument block");
  if (a.pend != nullptr && (a.dec.ticket != nullptr || a.pend_n <= 0 || a.pend_dec.stop == nullptr))
    throw std::invalid_argument("launch_stream: a pending decision needs a launch that does not decide itself");
  const bool f32 = precision == kFp32;
  switch (K) {
#define H2D_CASE(KK) case KK: launch_stream_k<KK>(blk, d, a.wt != 0, f32, residual, s); break;
    H2D_K_LIST(H2D_CASE)
#undef H2D_CASE
    default: throw std::invalid_argument("no streaming kernel compiled for K=" + std::to_string(K));
  }
  H2D_HIP_CHECK(hipGetLastError());
}

// ---- persistent pipelined variant (pstream_kernel.hpp, generated TUs pstream_k<K>_f<F>.hip) ----
#define H2D_PK_LIST(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8)
#define H2D_PEXTERN(K)                                                                                      \
  extern template void launch_pstream_kv<K, false, 4>(const PStreamArgs*, const PStreamDyn&, bool, hipStream_t); \
  extern template void launch_pstream_kv<K, true, 4>(const PStreamArgs*, const PStreamDyn&, bool, hipStream_t);  \
  extern template void launch_pstream_kv<K, false, 2>(const PStreamArgs*, const PStreamDyn&, bool, hipStream_t); \
  extern template void launch_pstream_kv<K, true, 2>(const PStreamArgs*, const PStreamDyn&, bool, hipStream_t);  \
  extern template int pstream_blocks_per_cu_v<K, false, 4>();                           \
  extern template int pstream_blocks_per_cu_v<K, true, 4>();                            \
  extern template int pstream_blocks_per_cu_v<K, false, 2>();                           \
  extern template int pstream_blocks_per_cu_v<K, true, 2>();
H2D_PK_LIST(H2D_PEXTERN)
#undef H2D_PEXTERN

void launch_pstream(const PStreamArgs* blk, const PStreamDyn& d, int K, int precision, int cpl, bool pp,
                    hipStream_t s) {
  const bool f32 = precision == kFp32;
  if (cpl != 2 && cpl != 4) throw std::invalid_argument("persistent stencil: 2 or 4 columns per lane");
  if (blk == nullptr) throw std::invalid_argument("persistent stencil: no argument block");
  switch (K) {
#define H2D_CASE(KK)                                                                                               \
  case KK:                                                                                                         \
    if (cpl == 4) f32 ? launch_pstream_kv<KK, true, 4>(blk, d, pp, s) : launch_pstream_kv<KK, false, 4>(blk, d, pp, s); \
    else f32 ? launch_pstream_kv<KK, true, 2>(blk, d, pp, s) : launch_pstream_kv<KK, false, 2>(blk, d, pp, s);          \
    break;
    H2D_PK_LIST(H2D_CASE)
#undef H2D_CASE
    default: throw std::invalid_argument("no persistent stencil compiled for K=" + std::to_string(K));
  }
  H2D_HIP_CHECK(hipGetLastError());
}

int pstream_blocks_per_cu(int K, int precision, int cpl) {
  const bool f32 = precision == kFp32;
  switch (K) {
#define H2D_CASE(KK)                                                                                 \
  case KK:                                                                                           \
    if (cpl == 2) return f32 ? pstream_blocks_per_cu_v<KK, true, 2>() : pstream_blocks_per_cu_v<KK, false, 2>(); \
    return f32 ? pstream_blocks_per_cu_v<KK, true, 4>() : pstream_blocks_per_cu_v<KK, false, 4>();
    H2D_PK_LIST(H2D_CASE)
#undef H2D_CASE
    default: return 0;
  }
}

void warm_pstream_kernels(int precision, int kmax, hipStream_t s) {
  static_assert(sizeof(PStreamArgs) <= kZeroArgBytes, "the zero block covers the persistent arguments");
  const PStreamArgs* z = static_cast<const PStreamArgs*>(zero_arg_block());  // nunits 0: every wave exits
  PStreamDyn d;
  for (int K = 1; K <= std::min(kmax, kMaxPK); ++K)
    for (int cpl : {4, 2}) launch_pstream(z, d, K, precision, cpl, false, s);
}

std::vector<PUnit> plan_pstream(const TileGeom& g, int K, bool fixed, bool per_x, bool per_y, double row_edge_weight,
                                int64_t capacity, bool halo_n, bool halo_s, int hmin, int cpl, double halo_weight) {
  std::vector<PUnit> out;
  const int64_t W = wave_cols(cpl);
  const std::vector<Strip> strips = strip_layout(g, K, fixed, per_y, cpl);
  const int S = (int)strips.size();
  if (S < 1 || capacity < S) return out;
  hmin = std::max(hmin, K);  // a K-cone spans at most the adjacent bands
  // bands: as many as one wave per SIMD allows; even when the bottom band must stream up (a
  // south halo: its ghost rows come first in its stream)
  int m = (int)std::min<int64_t>(capacity / S, g.xcell / hmin);
  if (halo_s && (m & 1)) --m;
  if (m < 1 || (halo_s && m < 2)) return out;
  // band heights: equal cost (h + K) * w, row-edge bands (their cone reaches a global edge row)
  // weighted w = row_edge_weight
  const double wr = std::max(1.0, row_edge_weight);
  std::vector<int64_t> a0, hh;
  for (;;) {
    std::vector<double> w(m, 1.0);
    auto row_edge = [&](int64_t lo, int64_t hi) {  // rows [lo, hi) of the tile, cone K
      return (unit_edge_flags(g, K, lo, hi - lo, strips[S / 2].cb, fixed, per_x, true, W) & kEdgeRows) != 0;
    };
    // first estimate with equal bands, then the weights of the bands at the tile's edge rows
    const int64_t eq = g.xcell / m;
    if (row_edge(0, eq)) w[0] = wr;
    if (row_edge(g.xcell - eq, g.xcell)) w[m - 1] = wr;
    if (halo_n) w[0] = std::max(w[0], std::max(1.0, halo_weight));
    if (halo_s) w[m - 1] = std::max(w[m - 1], std::max(1.0, halo_weight));
    double inv = 0.0;
    for (double x : w) inv += 1.0 / x;
    const double U = ((double)g.xcell + (double)m * K) / inv;
    a0.assign(m + 1, 0);
    hh.assign(m, 0);
    double acc = 0.0;
    for (int i = 0; i < m; ++i) {
      acc += U / w[i] - K;
      a0[i + 1] = (i == m - 1) ? g.xcell : std::min<int64_t>(g.xcell, (int64_t)std::llround(acc));
    }
    bool ok = true;
    for (int i = 0; i < m; ++i) {
      hh[i] = a0[i + 1] - a0[i];
      if (hh[i] < hmin) ok = false;
    }
    if (ok) break;
    m -= halo_s ? 2 : 1;
    if (m < 1 || (halo_s && m < 2)) return {};
  }
  auto uidx = [&](int band, int strip) { return band * S + strip; };
  out.resize((size_t)m * S);
  for (int i = 0; i < m; ++i) {
    for (int s = 0; s < S; ++s) {
      PUnit& p = out[(size_t)uidx(i, s)];
      const Strip& st = strips[(size_t)s];
      p.u = Unit{s, (int)a0[i], (int)hh[i], unit_edge_flags(g, K, a0[i], hh[i], st.cb, fixed, per_x, per_y, W),
                 (int)st.cb, (int)st.lo, (int)st.hi, 0};
      if (i & 1) p.u.flags |= kUnitReverse;
      if ((i == 0 && halo_n) || (i == m - 1 && halo_s)) p.u.flags |= kUnitNS;
      p.band = i;
    }
  }
  // neighbour slots: 0 above, 1 below, 2 left, 3 right, 4 above-left, 5 above-right,
  // 6 below-left, 7 below-right
  static const int kDb[kPSlots] = {-1, 1, 0, 0, -1, -1, 1, 1};
  static const int kDs[kPSlots] = {0, 0, -1, 1, -1, 1, -1, 1};
  for (int i = 0; i < m; ++i)
    for (int s = 0; s < S; ++s) {
      PUnit& p = out[(size_t)uidx(i, s)];
      const int64_t x0 = a0[i], h = hh[i];
      const bool rev = (i & 1) != 0;
      const int64_t wlo = strips[(size_t)s].cb, whi = wlo + W;  // my column window
      // a window must not reach past the adjacent strips' outputs
      for (int s2 = 0; s2 < S; ++s2)
        if (std::abs(s2 - s) > 1 && strips[(size_t)s2].lo < whi && strips[(size_t)s2].hi > wlo) return {};
      for (int l = 0; l < kPSlots; ++l) {
        p.nb[l] = -1;
        p.rlo[l] = p.rhi[l] = p.qa[l] = p.qs[l] = p.hv[l] = 0;
        const int i2 = i + kDb[l], s2 = s + kDs[l];
        if (i2 < 0 || i2 >= m || s2 < 0 || s2 >= S) continue;
        const Strip& t = strips[(size_t)s2];
        if (!(t.lo < whi && t.hi > wlo)) continue;  // no column of its outputs in my window
        const int64_t a2 = a0[i2], h2 = hh[i2];
        const bool rev2 = (i2 & 1) != 0;
        const int64_t tlo = std::max(a2, x0 - K), thi = std::min(a2 + h2, x0 + h + K);  // tile rows
        if (tlo >= thi) continue;
        int64_t rlo, rhi, qa, qs;
        if (!rev) {
          rlo = tlo - (x0 - K);
          rhi = thi - (x0 - K);
        } else {
          rlo = x0 + h + K - thi;
          rhi = x0 + h + K - tlo;
        }
        // my stream row r -> tile row T(r) -> its output index q(T)
        if (!rev && !rev2) qa = x0 - K - a2, qs = 1;
        else if (!rev && rev2) qa = a2 + h2 - 1 - x0 + K, qs = -1;
        else if (rev && !rev2) qa = x0 + h + K - 1 - a2, qs = -1;
        else qa = a2 + h2 - x0 - h - K, qs = 1;
        p.nb[l] = uidx(i2, s2);
        p.rlo[l] = (int)rlo;
        p.rhi[l] = (int)rhi;
        p.qa[l] = (int)qa;
        p.qs[l] = (int)qs;
        p.hv[l] = (int)h2;
      }
    }
  return out;
}

void warm_stream_kernels(int precision, int kmax, hipStream_t s) {
  static_assert(sizeof(StreamArgs) <= kZeroArgBytes, "the zero block covers the streaming arguments");
  const StreamArgs* z = static_cast<const StreamArgs*>(zero_arg_block());  // nunits 0: every wave exits
  StreamDyn d;
  const bool f32 = precision == kFp32;
  for (int K = 1; K <= std::min(kmax, kMaxK); ++K) {
    if (!stream_k_supported(K)) continue;
    for (bool resid : {false, true}) {
      switch (K) {
#define H2D_CASE(KK) case KK: launch_stream_k<KK>(z, d, false, f32, resid, s); break;
        H2D_K_LIST(H2D_CASE)
#undef H2D_CASE
        default: break;
      }
    }
  }
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_naive_step(const TileGeom& g, const float* src, float* dst, int precision, int boundary, double cx,
                       double cy, bool per_x, bool per_y, hipStream_t s) {
  if (g.xcell <= 0 || g.ycell <= 0) return;
  dim3 grid((unsigned)((g.ycell + 63) / 64), (unsigned)((g.xcell + 3) / 4));
  Coef k{cx, cy, (float)cx, (float)cy};
  const int fixed = boundary == kFixed;
  if (precision == kFp32)
    hipLaunchKernelGGL(naive_step_kernel<true>, grid, dim3(256), 0, s, g, src, dst, k, fixed, (int)per_x, (int)per_y);
  else
    hipLaunchKernelGGL(naive_step_kernel<false>, grid, dim3(256), 0, s, g, src, dst, k, fixed, (int)per_x, (int)per_y);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_init(const TileGeom& g, float* base, int init, hipStream_t s) {
  const int64_t total = g.elems();
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 256 * 32);
  hipLaunchKernelGGL(init_kernel, dim3(blocks), dim3(256), 0, s, g, base, init);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_poison(const TileGeom& g, float* base, bool fixed, bool per_x, bool per_y, hipStream_t s) {
  const int64_t total = g.elems();
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 256 * 32);
  hipLaunchKernelGGL(poison_kernel, dim3(blocks), dim3(256), 0, s, g, base, (int)fixed, (int)per_x, (int)per_y);
  H2D_HIP_CHECK(hipGetLastError());
}

int64_t copy_rects_blocks(int ndesc, int64_t max_elems) {
  if (ndesc <= 0 || max_elems <= 0) return 0;
  return std::min<int64_t>((max_elems + 255) / 256, 1024) * (int64_t)ndesc;
}

void launch_copy_rects(const CopyDesc* d_descs, int ndesc, int64_t max_elems, hipStream_t s, int64_t tag,
                       unsigned long long* done, unsigned int* integ, unsigned int* integ_host,
                       const unsigned long long* waves_done, unsigned long long waves_need) {
  if (ndesc <= 0 || max_elems <= 0) return;
  const unsigned bx = (unsigned)std::min<int64_t>((max_elems + 255) / 256, 1024);
  hipLaunchKernelGGL(copy_rects_kernel, dim3(bx, (unsigned)ndesc), dim3(256), 0, s, d_descs, tag, done, integ,
                     integ_host, waves_done, waves_need);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_reduce_sum(const double* in, int n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(reduce_sum_kernel, dim3(1), dim3(256), 0, s, in, n, out);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_wait_counter(const unsigned long long* counter, unsigned long long target, unsigned int* timed_out,
                         unsigned int* timed_out_host, long long max_polls, hipStream_t s) {
  hipLaunchKernelGGL(wait_counter_kernel, dim3(1), dim3(64), 0, s, counter, target, timed_out, timed_out_host,
                     max_polls);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_ipc_allreduce(const double* local, double* out, char* const* d_blocks, int me, int nranks, int parity,
                          unsigned long long target, size_t count_off, size_t slot_off, int max_ranks,
                          long long max_polls, unsigned int* timed_out, unsigned int* timed_out_host,
                          const unsigned long long* stop, const DecideArgs* decide, hipStream_t s) {
  DecideArgs d;
  if (decide) d = *decide;
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(1), dim3(64), 0, s, const_cast<double*>(local), out, d_blocks, me,
                     nranks, parity, target, (unsigned long long)count_off, (unsigned long long)slot_off, max_ranks,
                     max_polls, timed_out, timed_out_host, stop, d, decide ? 1 : 0, nullptr, 0);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_ipc_allreduce_parts(const double* parts, int nparts, double* local, double* out, char* const* d_blocks,
                                int me, int nranks, int parity, unsigned long long target, size_t count_off,
                                size_t slot_off, int max_ranks, long long max_polls, unsigned int* timed_out,
                                unsigned int* timed_out_host, const unsigned long long* stop, const DecideArgs& decide,
                                hipStream_t s) {
  if (parts == nullptr || nparts <= 0) throw std::invalid_argument("launch_ipc_allreduce_parts: no partials");
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(1), dim3(64), 0, s, local, out, d_blocks, me, nranks, parity, target,
                     (unsigned long long)count_off, (unsigned long long)slot_off, max_ranks, max_polls, timed_out,
                     timed_out_host, stop, decide, 1, parts, nparts);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_decide(const double* sum, const DecideArgs& d, hipStream_t s) {
  hipLaunchKernelGGL(decide_kernel, dim3(1), dim3(64), 0, s, sum, d);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_reduce_decide(const double* in, int n, const DecideArgs& d, hipStream_t s) {
  hipLaunchKernelGGL(reduce_decide_kernel, dim3(1), dim3(64), 0, s, in, n, d);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_set_counter(unsigned long long* counter, unsigned long long value, hipStream_t s) {
  hipLaunchKernelGGL(set_counter_kernel, dim3(1), dim3(64), 0, s, counter, value);
  H2D_HIP_CHECK(hipGetLastError());
}

void launch_tile_residual(const TileGeom& g, const float* a, const float* b, double* partials, int npartials,
                          hipStream_t s) {
  hipLaunchKernelGGL(tile_residual_kernel, dim3(npartials), dim3(256), 0, s, g, a, b, partials);
  H2D_HIP_CHECK(hipGetLastError());
}

bool lds_solver_fits(int64_t NX, int64_t NY) {
  return NX >= 1 && NY >= 1 && NX * NY <= kLdsCells && (NX + 2) * (NY + 2) <= kLdsImage;
}

void launch_lds_solver(const float* in, int64_t in_pitch, float* out, int64_t out_pitch, int64_t NX, int64_t NY,
                       int64_t steps, int precision, int boundary, double cx, double cy, bool per_x, bool per_y,
                       int conv_interval, double sensitivity, long long* steps_done, double* residual,
                       hipStream_t s) {
  if (!lds_solver_fits(NX, NY)) throw std::invalid_argument("grid too large for the LDS-resident solver");
  Coef k{cx, cy, (float)cx, (float)cy};
  const int fixed = boundary == kFixed;
  if (precision == kFp32)
    hipLaunchKernelGGL(lds_solver_kernel<true>, dim3(1), dim3(kLdsThreads), 0, s, in, in_pitch, out, out_pitch,
                       (int)NX, (int)NY, (long long)steps, k, fixed, (int)per_x, (int)per_y, conv_interval,
                       sensitivity, steps_done, residual);
  else
    hipLaunchKernelGGL(lds_solver_kernel<false>, dim3(1), dim3(kLdsThreads), 0, s, in, in_pitch, out, out_pitch,
                       (int)NX, (int)NY, (long long)steps, k, fixed, (int)per_x, (int)per_y, conv_interval,
                       sensitivity, steps_done, residual);
  H2D_HIP_CHECK(hipGetLastError());
}


// ---- device-resident kernel-argument blocks (ArgBlocks, kernels.h) ----------------------------
namespace {
// One wave copies a block from its pinned host slab into device memory: the stores go through
// the L2 that the stencil kernels' scalar loads read (kernel boundaries order them), unlike a
// DMA copy, which writes around the L2.
__global__ __launch_bounds__(64) void arg_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16) {
  for (int i = (int)threadIdx.x; i < n16; i += 64) dst[i] = src[i];
}
constexpr size_t kArgAlign = 256;       // blocks never share a cache line
constexpr size_t kArgSlab = 64 * 1024;  // bytes per slab (more for a larger block)
}  // namespace

unsigned next_arg_tag() {
  static std::atomic<unsigned> seq{0};
  unsigned t = ++seq;
  if (t == 0u) t = ++seq;
  return t;
}

const void* zero_arg_block() {
  static std::mutex mu;
  static std::map<int, void*> blocks;  // per device, never freed (process lifetime)
  int dev = 0;
  H2D_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  void*& p = blocks[dev];
  if (p == nullptr) {
    H2D_HIP_CHECK(hipMalloc(&p, kZeroArgBytes));
    H2D_HIP_CHECK(hipMemset(p, 0, kZeroArgBytes));
    H2D_HIP_CHECK(hipDeviceSynchronize());
  }
  return p;
}

ArgBlocks::~ArgBlocks() { clear(); }

void ArgBlocks::clear() {
  for (Slab& sl : slabs_) {
    if (sl.dev) hipFree(sl.dev);
    if (sl.host) hipHostFree(sl.host);
  }
  slabs_.clear();
  index_.clear();
  n_blocks_ = n_bytes_ = 0;
}

const void* ArgBlocks::get_raw(const void* p, size_t n, ArgHead* head, hipStream_t s) {
  if (n <= sizeof(ArgHead)) throw std::invalid_argument("ArgBlocks: empty argument block");
  const char* c = static_cast<const char*>(p);
  // the content after the header, and the size (blocks of different types never match)
  std::string key(c + sizeof(ArgHead), n - sizeof(ArgHead));
  key.append(reinterpret_cast<const char*>(&n), sizeof n);
  auto it = index_.find(key);
  if (it != index_.end()) {
    Entry& e = it->second;
    if (!e.ready && e.stream != s) {
      // first use on another stream: the upload (a kernel on its stream) must have completed
      H2D_HIP_CHECK(hipStreamSynchronize(e.stream));
      e.ready = true;
    }
    head->btag = e.tag;
    head->bytes = (unsigned)n;
    return e.dev;
  }
  const size_t need = (n + kArgAlign - 1) / kArgAlign * kArgAlign;
  if (slabs_.empty() || slabs_.back().used + need > slabs_.back().cap) {
    Slab sl;
    sl.cap = std::max(kArgSlab, need);
    H2D_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&sl.dev), sl.cap));
    if (hipHostMalloc(reinterpret_cast<void**>(&sl.host), sl.cap, hipHostMallocDefault) != hipSuccess) {
      hipFree(sl.dev);
      throw std::runtime_error("ArgBlocks: hipHostMalloc failed");
    }
    std::memset(sl.host, 0, sl.cap);
    slabs_.push_back(sl);
  }
  Slab& sl = slabs_.back();
  head->btag = next_arg_tag();
  head->bytes = (unsigned)n;
  char* h = sl.host + sl.used;
  char* d = sl.dev + sl.used;
  std::memcpy(h, p, n);  // (the rest of the aligned span stays zero)
  void* hd = nullptr;
  H2D_HIP_CHECK(hipHostGetDevicePointer(&hd, h, 0));
  hipLaunchKernelGGL(arg_copy_kernel, dim3(1), dim3(64), 0, s, reinterpret_cast<const uint4*>(hd),
                     reinterpret_cast<uint4*>(d), (int)(need / 16));
  H2D_HIP_CHECK(hipGetLastError());
  sl.used += need;
  ++n_blocks_;
  ++n_uploads_;
  n_bytes_ += need;
  index_.emplace(std::move(key), Entry{d, head->btag, s, false});
  return d;
}


}  // namespace h2d
