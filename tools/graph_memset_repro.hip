// Pure-HIP reproducer (no torch, no libvdiff) for the stale in-graph reduction value of
// tools/graph_reduce_repro.py: the pattern of torch's multi-block reduction
// (ATen/native/hip/Reduce.cuh) -- hipMemsetAsync of a semaphore, then ONE kernel whose
// blocks write per-block partials, count themselves on the semaphore with an atomic add,
// and whose last block sums the partials into the output -- captured from a stream into a
// HIP graph and replayed with a new input each time.  Between replays the host does eager
// work on the same stream (other kernels, a device-to-host copy of the result).  If a
// replay skips or mis-orders the memset node, the semaphore does not start at 0, no block
// sees itself as the last one, and the output keeps the previous replay's value.
//   hipcc --offload-arch=gfx950 -O2 tools/graph_memset_repro.hip -o gpurun_out/graph_memset_repro
//   graph_memset_repro [replays] [host_work 0|1|2|3] [reset: 0 hipMemsetAsync | 1 a zeroing kernel
//     | 2 hipMemsetAsync and a reduction with a 1-KiB argument | 3 a 4-byte hipMemsetAsync]
// prints one JSON line: replays, mismatches, the first few (replay, got, want).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(2); } } while (0)

constexpr int kThreads = 256;

__global__ void fill_kernel(float* x, int n, float v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    x[i] = v * (1.0f + (i & 7));
}

__global__ void zero_kernel(int* p, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0;
}

__global__ void busy_kernel(float* y, int n) {  // the host's eager work between replays
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    y[i] = y[i] * 0.5f + 1.0f;
}

// per-block partial sums, the semaphore, the last block sums the partials (fixed order)
__device__ void reduce_kernel_body(const float* x, int n, float* partial, int* sem, float* out) {
  __shared__ float red[kThreads];
  __shared__ bool last;
  float s = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = kThreads / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = red[0];
    __threadfence();
    last = atomicAdd(sem, 1) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __threadfence();
    float t = 0.f;
    for (int b = 0; b < (int)gridDim.x; ++b) t += __builtin_nontemporal_load(&partial[b]);
    *out = t;
  }
}

__global__ void reduce_kernel(const float* x, int n, float* partial, int* sem, float* out) {
  reduce_kernel_body(x, n, partial, sem, out);
}

// the same reduction with its pointers inside a ~1 KiB by-value argument, like torch's
// ReduceOp (host_work 3 / reset 2): kernel arguments of graph nodes and of the eager
// launches between replays then fill the runtime's argument buffers ~4x faster
struct BigArgs {
  const float* x;
  float* partial;
  int* sem;
  float* out;
  int n;
  int pad[250];
};

__global__ void reduce_big_kernel(BigArgs a) {
  reduce_kernel_body(a.x, a.n + a.pad[249], a.partial, a.sem, a.out);
}

struct BusyArgs {
  float* y;
  int n;
  int pad[250];
};

__global__ void busy_big_kernel(BusyArgs a) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x)
    a.y[i] = a.y[i] * 0.5f + 1.0f + a.pad[i & 127];
}

int main(int argc, char** argv) {
  const int replays = argc > 1 ? std::atoi(argv[1]) : 300;
  const int host_work = argc > 2 ? std::atoi(argv[2]) : 1;
  const int reset_kernel = argc > 3 ? std::atoi(argv[3]) : 0;
  const int n = 3 * 16 * 64 * 64, nb = 192, ny = 1 << 22;
  float *x, *partial, *out, *y, *partial2, *out2;
  int *sem, *sem2;
  CK(hipMalloc(&x, n * sizeof(float)));
  CK(hipMalloc(&partial, nb * sizeof(float)));
  CK(hipMalloc(&out, sizeof(float)));
  CK(hipMalloc(&y, ny * sizeof(float)));
  CK(hipMalloc(&sem, nb * sizeof(int)));
  CK(hipMalloc(&sem2, nb * sizeof(int)));
  CK(hipMalloc(&partial2, nb * sizeof(float)));
  CK(hipMalloc(&out2, sizeof(float)));
  CK(hipMemset(y, 0, ny * sizeof(float)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipGraph_t graph;
  hipGraphExec_t exec;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  if (reset_kernel == 1)
    zero_kernel<<<1, kThreads, 0, st>>>(sem, nb);
  else if (reset_kernel == 3)  // torch's size for a one-output reduction: one int
    CK(hipMemsetAsync(sem, 0, sizeof(int), st));
  else
    CK(hipMemsetAsync(sem, 0, nb * sizeof(int), st));
  if (reset_kernel == 2) {
    BigArgs a{};
    a.x = x; a.partial = partial; a.sem = sem; a.out = out; a.n = n;
    reduce_big_kernel<<<nb, kThreads, 0, st>>>(a);
  } else {
    reduce_kernel<<<nb, kThreads, 0, st>>>(x, n, partial, sem, out);
  }
  CK(hipStreamEndCapture(st, &graph));
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  std::vector<int> bad_r;
  std::vector<float> bad_got, bad_want;
  int bad = 0;
  for (int r = 0; r < replays; ++r) {
    const float v = 1.0f + (r % 13);
    fill_kernel<<<256, kThreads, 0, st>>>(x, n, v);
    CK(hipGraphLaunch(exec, st));
    float got = 0.f;
    if (host_work) {
      busy_kernel<<<1024, kThreads, 0, st>>>(y, ny);
      busy_kernel<<<1024, kThreads, 0, st>>>(y, ny);
    }
    if (host_work >= 3) {
      BusyArgs b{};
      b.y = y; b.n = 4096;
      for (int k = 0; k < 24; ++k) busy_big_kernel<<<16, kThreads, 0, st>>>(b);
    }
    if (host_work >= 2) {  // eager memsets and an eager reduction of the same pattern
      CK(hipMemsetAsync(y, 0, 4096 * sizeof(float), st));
      CK(hipMemsetAsync(sem2, 0, nb * sizeof(int), st));
      reduce_kernel<<<nb, kThreads, 0, st>>>(y, ny, partial2, sem2, out2);
    }
    CK(hipMemcpyAsync(&got, out, sizeof(float), hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    double want = 0;
    for (int i = 0; i < n; ++i) want += v * (1.0 + (i & 7));
    if (std::abs(got - want) > 1e-4 * want) {
      if (bad < 5) { bad_r.push_back(r); bad_got.push_back(got); bad_want.push_back((float)want); }
      ++bad;
    }
  }
  const char* pc = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
  std::printf("{\"replays\": %d, \"host_work\": %d, \"reset\": \"%s\", \"mismatches\": %d, \"DEBUG_CLR_GRAPH_PACKET_CAPTURE\": \"%s\", \"first\": [",
              replays, host_work, reset_kernel == 1 ? "kernel" : reset_kernel == 2 ? "hipMemsetAsync+bigargs"
              : reset_kernel == 3 ? "hipMemsetAsync 4 B" : "hipMemsetAsync", bad,
              pc ? pc : "unset");
  for (size_t i = 0; i < bad_r.size(); ++i)
    std::printf("%s[%d, %.6g, %.6g]", i ? ", " : "", bad_r[i], bad_got[i], bad_want[i]);
  std::printf("]}\n");
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  return 0;
}
