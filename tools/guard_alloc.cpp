// guard_alloc.cpp -- test utility (not part of the product library): a torch pluggable CUDA allocator
// that puts a guard band of kGuard bytes on both sides of EVERY device allocation (torch's own outputs,
// library workspaces, ours) and checks the bands when the block is freed, on the freeing stream, so the
// check sees the bands after every kernel that used the block (stream order).  A changed band byte is
// logged (device-side, no host sync) with the block's size and the first bad offset: an out-of-bounds
// write by any kernel of the step.  Memory comes from the stream-ordered allocator (hipMallocAsync /
// hipFreeAsync), so nothing synchronises the device and two streams keep running concurrently.
//   hipcc -O2 -shared -fPIC tools/guard_alloc.cpp -o tools/libguard_alloc.so
// Driven by tools/oob_probe.py (torch.cuda.memory.CUDAPluggableAllocator).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <unordered_map>

namespace {
constexpr size_t kGuard = 256 * 1024;
constexpr uint32_t kPattern = 0xA5C3E1F7u;
constexpr int kMaxLog = 4096;

struct Log {
  unsigned count;
  unsigned pad;
  unsigned long long entry[kMaxLog][3];   // size, side (0 low / 1 high) << 32 | first bad word, block base
};
Log* g_log = nullptr;
std::mutex g_mu;
std::unordered_map<void*, size_t> g_sizes;

__global__ void fill_guard(uint32_t* p, size_t words) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x)
    p[i] = kPattern;
}

__global__ void check_guard(const uint32_t* lo, const uint32_t* hi, size_t words, unsigned long long size,
                            unsigned long long base, Log* log) {
  __shared__ unsigned first_lo, first_hi;
  if (threadIdx.x == 0) { first_lo = 0xFFFFFFFFu; first_hi = 0xFFFFFFFFu; }
  __syncthreads();
  for (size_t i = threadIdx.x; i < words; i += blockDim.x) {
    if (lo[i] != kPattern) atomicMin(&first_lo, (unsigned)i);
    if (hi[i] != kPattern) atomicMin(&first_hi, (unsigned)i);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (first_lo != 0xFFFFFFFFu) {
      const unsigned k = atomicAdd(&log->count, 1u);
      if (k < kMaxLog) { log->entry[k][0] = size; log->entry[k][1] = first_lo; log->entry[k][2] = base; }
    }
    if (first_hi != 0xFFFFFFFFu) {
      const unsigned k = atomicAdd(&log->count, 1u);
      if (k < kMaxLog) { log->entry[k][0] = size; log->entry[k][1] = (1ull << 32) | first_hi; log->entry[k][2] = base; }
    }
  }
}
}  // namespace

extern "C" {

void* guard_malloc(ssize_t size, int device, hipStream_t stream) {
  (void)device;
  if (!g_log) {
    if (hipMalloc(&g_log, sizeof(Log)) != hipSuccess) return nullptr;
    (void)hipMemset(g_log, 0, sizeof(Log));
  }
  const size_t body = ((size_t)size + 511) & ~(size_t)511;
  char* base = nullptr;
  if (hipMallocAsync((void**)&base, body + 2 * kGuard, stream) != hipSuccess) return nullptr;
  hipLaunchKernelGGL(fill_guard, dim3(64), dim3(256), 0, stream, (uint32_t*)base, kGuard / 4);
  hipLaunchKernelGGL(fill_guard, dim3(64), dim3(256), 0, stream, (uint32_t*)(base + kGuard + body), kGuard / 4);
  void* user = base + kGuard;
  std::lock_guard<std::mutex> g(g_mu);
  g_sizes[user] = body;
  return user;
}

void guard_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)device;
  (void)size;
  size_t body;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_sizes.find(ptr);
    if (it == g_sizes.end()) return;
    body = it->second;
    g_sizes.erase(it);
  }
  char* base = (char*)ptr - kGuard;
  hipLaunchKernelGGL(check_guard, dim3(1), dim3(1024), 0, stream, (const uint32_t*)base,
                     (const uint32_t*)(base + kGuard + body), kGuard / 4, (unsigned long long)body,
                     (unsigned long long)(uintptr_t)ptr, g_log);
  (void)hipFreeAsync(base, stream);
}

// host: copy the log out (call after a device synchronize); returns the violation count
int guard_report(unsigned long long* out, int max_entries) {
  if (!g_log) return 0;
  Log h;
  if (hipMemcpy(&h, g_log, sizeof(Log), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  const int n = (int)(h.count < (unsigned)kMaxLog ? h.count : kMaxLog);
  for (int i = 0; i < n && i < max_entries; ++i)
    for (int j = 0; j < 3; ++j) out[3 * i + j] = h.entry[i][j];
  return (int)h.count;
}

// host: check every block still alive (enqueued on `stream`)
void guard_check_live(hipStream_t stream) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& kv : g_sizes) {
    char* base = (char*)kv.first - kGuard;
    hipLaunchKernelGGL(check_guard, dim3(1), dim3(1024), 0, stream, (const uint32_t*)base,
                       (const uint32_t*)(base + kGuard + kv.second), kGuard / 4, (unsigned long long)kv.second,
                       (unsigned long long)(uintptr_t)kv.first, g_log);
  }
}
}
