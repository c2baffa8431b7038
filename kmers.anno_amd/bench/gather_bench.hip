// gather_bench.hip — measured random-access roofline for the signature-table probe
// (SURVEY.md §8(d)): GUPS-style reads of 64-byte lines at uniformly random line indices of a
// buffer of a given size. Three access shapes:
//   lane  — one lane reads a whole line (4 x dwordx4),
//   quad  — four adjacent lanes read one line together (one dwordx4 each: the probe shape),
//   oct   — eight adjacent lanes read one aligned 128-byte line (one dwordx4 each): is a
//           128-byte bucket as cheap as a 64-byte one at the memory side (128-B L2 lines)?
//   quad2 — four adjacent lanes read one 128-byte line as two 64-byte halves (two dwordx4
//           each, one instruction per half),
//   hex   — sixteen adjacent lanes read one aligned 256-byte span (one dwordx4 each).
// with `inflight` independent lines per lane (lane) or per quad (quad) before any is consumed,
// plain or non-temporal loads, and `bpc` resident 256-thread blocks per CU.
//
//   kma_gather_bench <buffer_MiB> <lane|quad> <inflight> [nt=0] [bpc=8]
// Prints one JSON object: GB/s of line bytes and lines/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
  if constexpr (NT) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}

constexpr int kSteps = 64;  // lines per lane (lane shape) or per quad (quad shape)

template <int I, bool NT>
__global__ __launch_bounds__(256) void gather_lane(const uint4* __restrict__ buf, uint32_t n_lines,
                                                   uint32_t* __restrict__ sink, uint32_t salt) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int r = 0; r < kSteps; r += I) {
    uint4 v[I][4];
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const uint32_t line = (uint32_t)(((uint64_t)mix32(tid * 0x9E3779B1u + (r + j) * 0x85EBCA77u + salt) * n_lines) >> 32);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[j][q] = ld<NT>(buf + (uint64_t)line * 4 + q);
    }
#pragma unroll
    for (int j = 0; j < I; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc ^= v[j][q].x ^ v[j][q].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int I, bool NT>
__global__ __launch_bounds__(256) void gather_quad(const uint4* __restrict__ buf, uint32_t n_lines,
                                                   uint32_t* __restrict__ sink, uint32_t salt) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t quad = tid >> 2, part = tid & 3;
  uint32_t acc = 0;
  for (int r = 0; r < kSteps; r += I) {
    uint4 v[I];
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const uint32_t line = (uint32_t)(((uint64_t)mix32(quad * 0x9E3779B1u + (r + j) * 0x85EBCA77u + salt) * n_lines) >> 32);
      v[j] = ld<NT>(buf + (uint64_t)line * 4 + part);
    }
#pragma unroll
    for (int j = 0; j < I; ++j) acc ^= v[j].x ^ v[j].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int I, bool NT>
__global__ __launch_bounds__(256) void gather_oct(const uint4* __restrict__ buf, uint32_t n_lines,
                                                  uint32_t* __restrict__ sink, uint32_t salt) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t oct = tid >> 3, part = tid & 7;
  const uint32_t n128 = n_lines / 2;
  uint32_t acc = 0;
  for (int r = 0; r < kSteps; r += I) {
    uint4 v[I];
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const uint32_t line = (uint32_t)(((uint64_t)mix32(oct * 0x9E3779B1u + (r + j) * 0x85EBCA77u + salt) * n128) >> 32);
      v[j] = ld<NT>(buf + (uint64_t)line * 8 + part);
    }
#pragma unroll
    for (int j = 0; j < I; ++j) acc ^= v[j].x ^ v[j].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int I, bool NT>
__global__ __launch_bounds__(256) void gather_quad2(const uint4* __restrict__ buf, uint32_t n_lines,
                                                    uint32_t* __restrict__ sink, uint32_t salt) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t quad = tid >> 2, part = tid & 3;
  const uint32_t n128 = n_lines / 2;
  uint32_t acc = 0;
  for (int r = 0; r < kSteps; r += I) {
    uint4 v[I][2];
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const uint32_t line = (uint32_t)(((uint64_t)mix32(quad * 0x9E3779B1u + (r + j) * 0x85EBCA77u + salt) * n128) >> 32);
      v[j][0] = ld<NT>(buf + (uint64_t)line * 8 + part);
      v[j][1] = ld<NT>(buf + (uint64_t)line * 8 + 4 + part);
    }
#pragma unroll
    for (int j = 0; j < I; ++j) acc ^= v[j][0].x ^ v[j][1].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int I, bool NT>
__global__ __launch_bounds__(256) void gather_hex(const uint4* __restrict__ buf, uint32_t n_lines,
                                                  uint32_t* __restrict__ sink, uint32_t salt) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t hex = tid >> 4, part = tid & 15;
  const uint32_t n256 = n_lines / 4;
  uint32_t acc = 0;
  for (int r = 0; r < kSteps; r += I) {
    uint4 v[I];
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const uint32_t line = (uint32_t)(((uint64_t)mix32(hex * 0x9E3779B1u + (r + j) * 0x85EBCA77u + salt) * n256) >> 32);
      v[j] = ld<NT>(buf + (uint64_t)line * 16 + part);
    }
#pragma unroll
    for (int j = 0; j < I; ++j) acc ^= v[j].x ^ v[j].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// l16 / l8: each lane reads ONE random 16-byte (dwordx4) / 8-byte (dwordx2) piece: the access of
// a fingerprint-bucket probe (is an L2-resident random read capped per line or per load?).
template <int I, bool NT>
__global__ __launch_bounds__(256) void gather_l16(const uint4* __restrict__ buf, uint32_t n_lines,
                                                  uint32_t* __restrict__ sink, uint32_t salt) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n16 = n_lines * 4;
  uint32_t acc = 0;
  for (int r = 0; r < kSteps; r += I) {
    uint4 v[I];
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const uint32_t piece = (uint32_t)(((uint64_t)mix32(tid * 0x9E3779B1u + (r + j) * 0x85EBCA77u + salt) * n16) >> 32);
      v[j] = ld<NT>(buf + piece);
    }
#pragma unroll
    for (int j = 0; j < I; ++j) acc ^= v[j].x ^ v[j].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int I, bool NT>
__global__ __launch_bounds__(256) void gather_l8(const uint4* __restrict__ buf, uint32_t n_lines,
                                                 uint32_t* __restrict__ sink, uint32_t salt) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n8 = n_lines * 8;
  const uint2* b8 = reinterpret_cast<const uint2*>(buf);
  uint32_t acc = 0;
  for (int r = 0; r < kSteps; r += I) {
    uint2 v[I];
#pragma unroll
    for (int j = 0; j < I; ++j) {
      const uint32_t piece = (uint32_t)(((uint64_t)mix32(tid * 0x9E3779B1u + (r + j) * 0x85EBCA77u + salt) * n8) >> 32);
      v[j] = b8[piece];
    }
#pragma unroll
    for (int j = 0; j < I; ++j) acc ^= v[j].x ^ v[j].y;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <class F>
double time_kernel(F launch, double bytes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch(1u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int it = 0; it < 5; ++it) {
    CHECK(hipEventRecord(a));
    launch((uint32_t)it + 2);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return bytes / (best * 1e-3) / 1e9;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <buffer_MiB> <lane|quad|oct> <inflight> [nt] [bpc]\n",
                 argv[0]);
    return 1;
  }
  const uint64_t mib = std::strtoull(argv[1], nullptr, 10);
  const bool quad = !std::strcmp(argv[2], "quad"), oct = !std::strcmp(argv[2], "oct");
  const bool quad2 = !std::strcmp(argv[2], "quad2"), hex = !std::strcmp(argv[2], "hex");
  const bool l16 = !std::strcmp(argv[2], "l16"), l8 = !std::strcmp(argv[2], "l8");
  const int inflight = std::atoi(argv[3]);
  const bool nt = argc > 4 && std::atoi(argv[4]);
  const int bpc = argc > 5 ? std::atoi(argv[5]) : 8;
  const uint64_t bytes = mib << 20;
  int n_cu = 256;
  CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  uint4* buf;
  uint32_t* sink;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(buf, 1, bytes));
  const uint32_t n_lines = (uint32_t)(bytes / 64);
  const int blocks = n_cu * bpc;
  // requests (lines of the shape's size: 128 B for oct, else 64 B)
  const double lines =
      (double)blocks * 256 * kSteps / (hex ? 16 : oct ? 8 : (quad || quad2) ? 4 : 1);
  const double line_bytes = l8 ? 8 : l16 ? 16 : hex ? 256 : (oct || quad2) ? 128 : 64;
  double gbs = 0;
#define RUN(KERNEL, I, NTV)                                                                   \
  gbs = time_kernel([&](uint32_t salt) {                                                      \
    hipLaunchKernelGGL((KERNEL<I, NTV>), dim3(blocks), dim3(256), 0, 0, buf, n_lines, sink,   \
                       salt);                                                                 \
  }, lines * line_bytes)
#define CASES(KERNEL)                                           \
  if (inflight == 1) { if (nt) RUN(KERNEL, 1, true); else RUN(KERNEL, 1, false); } \
  else if (inflight == 2) { if (nt) RUN(KERNEL, 2, true); else RUN(KERNEL, 2, false); } \
  else if (inflight == 4) { if (nt) RUN(KERNEL, 4, true); else RUN(KERNEL, 4, false); } \
  else if (inflight == 8) { if (nt) RUN(KERNEL, 8, true); else RUN(KERNEL, 8, false); }
  if (l16) { CASES(gather_l16) } else if (l8) { CASES(gather_l8) }
  else if (hex) { CASES(gather_hex) } else if (quad2) { CASES(gather_quad2) }
  else if (oct) { CASES(gather_oct) } else if (quad) { CASES(gather_quad) } else { CASES(gather_lane) }
  if (gbs == 0) {
    std::fprintf(stderr, "unsupported inflight %d\n", inflight);
    return 1;
  }
  std::printf("{\"buffer_MiB\": %llu, \"shape\": \"%s\", \"inflight\": %d, \"nt\": %d, "
              "\"blocks_per_cu\": %d, \"GBps\": %.1f, \"lines_per_s\": %.4g, "
              "\"lines_per_launch\": %.0f}\n",
              (unsigned long long)mib,
              l16 ? "l16" : l8 ? "l8" : hex ? "hex" : quad2 ? "quad2" : oct ? "oct" : quad ? "quad" : "lane",
              inflight, (int)nt,
              bpc, gbs, gbs * 1e9 / line_bytes, lines);
  CHECK(hipFree(buf));
  return 0;
}
