// Host writes into device memory through the PCIe BAR vs pinned staging + DMA (measurement only,
// not part of the library). A host call that packs residues could store the packed stream
// straight into a host-visible device buffer: host DRAM then sees only the ASCII reads (no
// staging writes, no DMA reads of the staging buffer). This measures whether the host's stores
// reach the device at the link's rate.
//   build/kma_bar_bench [MiB] [threads]
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));             \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void checksum_kernel(const uint4* __restrict__ p, uint64_t n, unsigned long long* out) {
  uint64_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    s += (uint64_t)v.x + v.y + v.z + v.w;
  }
  atomicAdd(out, (unsigned long long)s);
}

using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t).count();
}

// Copy src -> dst with non-temporal 32-byte stores on `threads` threads (dst 64-byte aligned).
static double nt_copy(uint8_t* dst, const uint8_t* src, size_t bytes, int threads) {
  std::vector<std::thread> ts;
  const size_t per = (bytes / threads) & ~(size_t)63;
  const Clock::time_point t0 = Clock::now();
  for (int k = 0; k < threads; ++k)
    ts.emplace_back([=] {
      const size_t a = per * k, b = k + 1 == threads ? bytes : per * (k + 1);
      for (size_t i = a; i < b; i += 64) {
        const __m256i x0 = _mm256_loadu_si256((const __m256i*)(src + i));
        const __m256i x1 = _mm256_loadu_si256((const __m256i*)(src + i + 32));
        _mm256_stream_si256((__m256i*)(dst + i), x0);
        _mm256_stream_si256((__m256i*)(dst + i + 32), x1);
      }
      _mm_sfence();
    });
  for (auto& t : ts) t.join();
  return ms_since(t0);
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 192;
  const int threads = argc > 2 ? atoi(argv[2]) : 16;
  const size_t bytes = mib << 20;
  uint8_t* src = (uint8_t*)aligned_alloc(64, bytes);
  for (size_t i = 0; i < bytes; i += 8) *(uint64_t*)(src + i) = i * 0x9E3779B97F4A7C15ull;
  uint64_t want = 0;
  for (size_t i = 0; i < bytes; i += 4) want += *(const uint32_t*)(src + i);
  unsigned long long* d_sum;
  CK(hipMalloc(&d_sum, 8));
  std::printf("{\"bytes\": %zu, \"threads\": %d", bytes, threads);

  // Pinned staging + one DMA copy (the library's path; the staging writes timed apart).
  uint8_t *h_pin, *d_buf;
  CK(hipHostMalloc(&h_pin, bytes, 0));
  CK(hipMalloc(&d_buf, bytes));
  for (int rep = 0; rep < 2; ++rep) {
    const double st = nt_copy(h_pin, src, bytes, threads);
    const Clock::time_point t0 = Clock::now();
    CK(hipMemcpy(d_buf, h_pin, bytes, hipMemcpyHostToDevice));
    const double cp = ms_since(t0);
    if (rep) std::printf(", \"pinned_stage_ms\": %.3f, \"pinned_dma_ms\": %.3f, \"dma_GBps\": %.1f", st, cp,
                         bytes / cp / 1e6);
  }

  // Host-visible device memory: fine-grained VRAM, written by the host's stores.
  uint8_t* d_fine = nullptr;
  hipError_t e = hipExtMallocWithFlags((void**)&d_fine, bytes, hipDeviceMallocFinegrained);
  std::printf(", \"finegrained_alloc\": \"%s\"", hipGetErrorString(e));
  if (e == hipSuccess) {
    hipPointerAttribute_t at;
    CK(hipPointerGetAttributes(&at, d_fine));
    std::printf(", \"type\": %d, \"hostPointer\": %s", (int)at.type, at.hostPointer ? "true" : "false");
    uint8_t* hp = at.hostPointer ? (uint8_t*)at.hostPointer : d_fine;
    for (int rep = 0; rep < 3; ++rep) {
      const double ms = nt_copy(hp, src, bytes, threads);
      std::printf(", \"bar_write_ms_%d\": %.3f, \"bar_GBps_%d\": %.1f", rep, ms, rep, bytes / ms / 1e6);
    }
    CK(hipMemset(d_sum, 0, 8));
    hipLaunchKernelGGL(checksum_kernel, dim3(1024), dim3(256), 0, 0, (const uint4*)d_fine,
                       (uint64_t)(bytes / 16), d_sum);
    CK(hipDeviceSynchronize());
    unsigned long long got = 0;
    CK(hipMemcpy(&got, d_sum, 8, hipMemcpyDeviceToHost));
    std::printf(", \"checksum_ok\": %s", got == (unsigned long long)want ? "true" : "false");
    // the kernel's read rate of fine-grained VRAM (the probe would read the stream from there)
    const Clock::time_point t0 = Clock::now();
    hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint4*)d_fine,
                       (uint64_t)(bytes / 16), d_sum);
    CK(hipDeviceSynchronize());
    std::printf(", \"kernel_read_ms\": %.3f", ms_since(t0));
    CK(hipFree(d_fine));
  }
  std::printf("}\n");
  return 0;
}
