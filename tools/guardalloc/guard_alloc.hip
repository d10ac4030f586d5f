// guard_alloc.hip -- a debugging device allocator for torch.cuda.memory.CUDAPluggableAllocator
// (TEST / DEBUG INFRASTRUCTURE; never loaded by the product path).
//
// Every allocation gets GUARD bytes of a known pattern on each side.  ga_check_all() checks the
// guards of every live allocation on the GPU (one kernel) and reports the ones that were
// overwritten: a kernel that writes past the end (or before the start) of its output or
// workspace shows up as a corrupt guard of that buffer.  ga_free() checks the block it frees.
// No caching: every torch allocation is a hipMalloc, so run one step, not a benchmark.
// Used by tools/guard_check.py ("guard bands ... asserted after one
// eager config-2 step").
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

constexpr size_t kGuard = 1 << 20;           // bytes on each side
constexpr uint32_t kPattern = 0x7FA5A5A5u;   // a NaN-free, unlikely fp32 / bf16x2 value

struct Blk {
  char* base;      // hipMalloc'd pointer (front guard starts here)
  size_t size;     // user bytes
  uint64_t id;     // allocation sequence number
};

std::mutex g_mu;
std::unordered_map<void*, Blk> g_live;
uint64_t g_next = 0;
long g_bad_total = 0;

__global__ void fill_kernel(uint32_t* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = kPattern;
}

// guards[i]: start of the checked part of one guard region (`words` words); first_bad[i] =
// first corrupt word or -1
__global__ void check_kernel(const uint32_t* const* guards, int n, size_t words,
                             long long* first_bad) {
  const int g = blockIdx.x;
  if (g >= n) return;
  const uint32_t* p = guards[g];
  __shared__ long long lo;
  if (threadIdx.x == 0) lo = -1;
  __syncthreads();
  for (size_t i = threadIdx.x; i < words; i += blockDim.x)
    if (p[i] != kPattern) {
      atomicMin(reinterpret_cast<unsigned long long*>(&lo), (unsigned long long)i);
    }
  __syncthreads();
  if (threadIdx.x == 0) first_bad[g] = lo;
}

void fill_guard(char* p) {
  fill_kernel<<<64, 256>>>(reinterpret_cast<uint32_t*>(p), kGuard / 4);
}

// check the given blocks (the `bytes` of each guard nearest the user region); returns the
// number of corrupt guards and prints them
std::mutex g_check_mu;  // check_blocks' persistent device arrays

int check_blocks(const std::vector<std::pair<void*, Blk>>& blks, const char* when,
                 size_t bytes = kGuard) {
  if (blks.empty()) return 0;
  std::lock_guard<std::mutex> lk(g_check_mu);
  if (bytes > kGuard) bytes = kGuard;
  const int n = (int)blks.size() * 2;
  std::vector<const uint32_t*> gp(n);
  for (size_t i = 0; i < blks.size(); ++i) {
    const Blk& b = blks[i].second;
    gp[2 * i] = reinterpret_cast<const uint32_t*>(b.base + kGuard - bytes);
    gp[2 * i + 1] = reinterpret_cast<const uint32_t*>(b.base + kGuard + b.size);
  }
  // persistent device arrays for the guard pointers and results (grown, never freed)
  static const uint32_t** dg = nullptr;
  static long long* dbad = nullptr;
  static int cap = 0;
  if (n > cap) {
    if (dg) (void)hipFree(dg);
    if (dbad) (void)hipFree(dbad);
    cap = n * 2 + 1024;
    if (hipMalloc(&dg, cap * sizeof(void*)) || hipMalloc(&dbad, cap * sizeof(long long))) {
      fprintf(stderr, "[guard] hipMalloc failed in check\n");
      cap = 0;
      dg = nullptr;
      dbad = nullptr;
      return -1;
    }
  }
  (void)hipMemcpy(dg, gp.data(), n * sizeof(void*), hipMemcpyHostToDevice);
  check_kernel<<<n, 256>>>(dg, n, bytes / 4, dbad);
  std::vector<long long> bad(n);
  (void)hipMemcpy(bad.data(), dbad, n * sizeof(long long), hipMemcpyDeviceToHost);
  int nbad = 0;
  for (int i = 0; i < n; ++i) {
    // atomicMin on -1 (as unsigned: max) keeps -1 when clean
    if (bad[i] == -1) continue;
    ++nbad;
    const Blk& b = blks[i / 2].second;
    const bool back = i & 1;
    fprintf(stderr,
            "[guard] %s: allocation #%llu (%zu B at %p) %s guard overwritten, first bad word %lld "
            "(%s)\n",
            when, (unsigned long long)b.id, b.size, blks[i / 2].first, back ? "BACK" : "FRONT",
            bad[i],
            back ? "words past the end" : "words from the start of the checked front band");
  }
  return nbad;
}

}  // namespace

extern "C" {

void* ga_malloc(ssize_t size, int device, hipStream_t stream) {
  (void)device;
  (void)stream;
  char* base = nullptr;
  const size_t user = (size_t)(size > 0 ? size : 0);
  const size_t pad = (user + 255) / 256 * 256;  // keep the user pointer 256-B aligned
  if (hipMalloc(&base, pad + 2 * kGuard) != hipSuccess) return nullptr;
  (void)hipDeviceSynchronize();
  fill_guard(base);
  fill_guard(base + kGuard + user);
  (void)hipDeviceSynchronize();
  void* p = base + kGuard;
  std::lock_guard<std::mutex> lk(g_mu);
  g_live[p] = Blk{base, user, g_next++};
  return p;
}

void ga_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)size;
  (void)device;
  Blk b;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_live.find(ptr);
    if (it == g_live.end()) {
      fprintf(stderr, "[guard] free of unknown pointer %p\n", ptr);
      return;
    }
    b = it->second;
    g_live.erase(it);
  }
  (void)hipStreamSynchronize(stream);
  (void)hipDeviceSynchronize();
  std::vector<std::pair<void*, Blk>> one{{ptr, b}};
  const int nb = check_blocks(one, "free");
  if (nb > 0) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_bad_total += nb;
  }
  (void)hipFree(b.base);
}

// checks every live allocation (device-synchronising): the `bytes` of each guard next to the
// user region (0 = the whole guard); returns the number of corrupt guards
int ga_check_all(const char* when, size_t bytes) {
  (void)hipDeviceSynchronize();
  std::vector<std::pair<void*, Blk>> blks;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    blks.assign(g_live.begin(), g_live.end());
  }
  const int nb = check_blocks(blks, when ? when : "check", bytes ? bytes : kGuard);
  if (nb > 0) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_bad_total += nb;
  }
  return nb;
}

// re-arms every live guard (after a reported corruption, to find the next one)
void ga_rearm_all() {
  (void)hipDeviceSynchronize();
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& kv : g_live) {
    fill_guard(kv.second.base);
    fill_guard(kv.second.base + kGuard + kv.second.size);
  }
  (void)hipDeviceSynchronize();
}

long ga_bad_total() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_bad_total;
}

long ga_live_count() {
  std::lock_guard<std::mutex> lk(g_mu);
  return (long)g_live.size();
}

size_t ga_lookup(const void* p, uint64_t* id) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_live.find(const_cast<void*>(p));
  if (it == g_live.end()) return 0;
  if (id) *id = it->second.id;
  return it->second.size;
}

}  // extern "C"
