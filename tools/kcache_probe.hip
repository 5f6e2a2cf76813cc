// Standalone probe (round 5): do a kernel's SCALAR loads see what the previous kernel on the same
// stream wrote?  docs/ARCHITECTURE.md, "Kernel arguments (round 5)".
//
// Iteration i: `writer` stores i into word X with a vector store (one lane); `reader` runs one
// wave per SIMD on every CU, each reading X with a wave-uniform load that the compiler emits as
// s_load (scalar data cache), plus the same word with a vector atomic load; both values go to
// out[].  A correct stream sees i everywhere.  The HSA dispatch packet's acquire fence is what
// invalidates the scalar cache between the two kernels.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/kcache_probe.hip -o kcache_probe
// Run:   ./kcache_probe [iterations]   (once with the default kernel arguments, once with
//        HIP_FORCE_DEV_KERNARG=0; exit 1 if any stale value was seen)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(2);                                                                 \
    }                                                                               \
  } while (0)

__global__ void writer(unsigned* x, unsigned v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) x[0] = v;
}

// out[2 * wave] = scalar-load value, out[2 * wave + 1] = vector (agent-scope atomic) value
__global__ __launch_bounds__(256) void reader(const unsigned* __restrict__ x, unsigned* __restrict__ out) {
  const unsigned s = x[0];  // uniform address, read-only in the kernel: s_load
  const unsigned v = __hip_atomic_load(x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load
  const unsigned wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    out[2 * wave] = s;
    out[2 * wave + 1] = v;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount;  // 4 waves per block: one per SIMD
  const int waves = blocks * 4;
  unsigned *x = nullptr, *out = nullptr;
  CHECK(hipMalloc(&x, 4096));
  CHECK(hipMalloc(&out, sizeof(unsigned) * 2 * waves * 64));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<unsigned> h(2 * waves * 64);
  long long stale_s = 0, stale_v = 0, checks = 0;
  const int batch = 64;  // iterations between host checks (each with its own out slice)
  for (int base = 0; base < iters; base += batch) {
    for (int j = 0; j < batch; ++j) {
      hipLaunchKernelGGL(writer, dim3(1), dim3(64), 0, s, x, (unsigned)(base + j + 1));
      hipLaunchKernelGGL(reader, dim3(blocks), dim3(256), 0, s, x, out + 2 * waves * j);
    }
    CHECK(hipGetLastError());
    CHECK(hipMemcpyAsync(h.data(), out, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    CHECK(hipStreamSynchronize(s));
    for (int j = 0; j < batch; ++j)
      for (int w = 0; w < waves; ++w) {
        const unsigned want = (unsigned)(base + j + 1);
        stale_s += h[2 * waves * j + 2 * w] != want;
        stale_v += h[2 * waves * j + 2 * w + 1] != want;
        ++checks;
      }
  }
  const char* kd = std::getenv("HIP_FORCE_DEV_KERNARG");
  std::printf("kcache_probe: HIP_FORCE_DEV_KERNARG=%s, %d iterations x %d waves: stale scalar loads %lld, "
              "stale vector loads %lld (of %lld)\n", kd ? kd : "(unset)", iters, waves, stale_s, stale_v, checks);
  return (stale_s || stale_v) ? 1 : 0;
}
