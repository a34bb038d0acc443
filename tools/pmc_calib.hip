// pmc_calib — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// simulator's kernels use (MI355X_MICROARCH.md: only 16-B-per-lane streaming reads are calibrated,
// at x2). Each kernel touches a known number of distinct 128-B lines of a 2 GiB buffer (far past
// the 256 MiB Infinity Cache) exactly once:
//   k_stream16  16 B per lane, coalesced (the guide's calibrated case: expect FETCH x 2 = bytes)
//   k_gather4   one 4-B load per line, lines in a scrambled order (apply's entry ids, view cells)
//   k_gather1   one 1-B load per line, scrambled (select's age bounds)
//   k_gather32  32 B (two 16-B loads by one lane) per line, scrambled (infection rounds)
//   k_scatter4  one 4-B store per line, scrambled (sweep / apply cell writes)
//   k_rmw4      one 4-B load + store of the same word per line, scrambled (holdings words)
// tools/pmc_calib_summary.py divides each kernel's counter bytes by its lines x 128 B and by its
// useful bytes. Build: hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint64_t BUF = 2ull << 30;          // bytes
constexpr uint64_t LINES = BUF / 128;         // 2^24 lines
constexpr uint32_t TOUCH = 1u << 22;          // lines touched by the gather / scatter kernels

__device__ __forceinline__ uint64_t line_of(uint32_t i) {  // a bijection on [0, LINES): scrambled lines
  return ((uint64_t)i * 0x9E3779B1ull) & (LINES - 1);
}

__global__ void k_stream16(const uint4* p, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) *sink = acc;
}

__global__ void k_gather4(const uint32_t* p, uint32_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= TOUCH) return;
  const uint32_t v = p[line_of(i) * 32u];
  if (v == 0x12345678u) *sink = v;
}

__global__ void k_gather1(const uint8_t* p, uint32_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= TOUCH) return;
  const uint32_t v = p[line_of(i) * 128u + 5u];
  if (v == 0x7Bu) *sink = v;
}

__global__ void k_gather32(const uint4* p, uint32_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= TOUCH) return;
  const uint4* q = p + line_of(i) * 8u;
  const uint4 a = q[0], b = q[1];
  const uint32_t v = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
  if (v == 0x12345678u) *sink = v;
}

__global__ void k_scatter4(uint32_t* p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < TOUCH) p[line_of(i) * 32u + 3u] = i;
}

__global__ void k_rmw4(uint32_t* p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < TOUCH) {
    uint32_t* q = p + line_of(i) * 32u + 7u;
    *q = *q + 1u;
  }
}

int main() {
  void* buf = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&buf, BUF) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) {
    std::fprintf(stderr, "hipMalloc failed\n");
    return 1;
  }
  (void)hipMemset(buf, 1, BUF);
  const uint32_t g = TOUCH / 256;
  for (int rep = 0; rep < 3; ++rep) {  // the summary averages the dispatches of each kernel
    hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, (const uint4*)buf, BUF / 16, sink);
    hipLaunchKernelGGL(k_gather4, dim3(g), dim3(256), 0, 0, (const uint32_t*)buf, sink);
    hipLaunchKernelGGL(k_gather1, dim3(g), dim3(256), 0, 0, (const uint8_t*)buf, sink);
    hipLaunchKernelGGL(k_gather32, dim3(g), dim3(256), 0, 0, (const uint4*)buf, sink);
    hipLaunchKernelGGL(k_scatter4, dim3(g), dim3(256), 0, 0, (uint32_t*)buf);
    hipLaunchKernelGGL(k_rmw4, dim3(g), dim3(256), 0, 0, (uint32_t*)buf);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("{\"buffer_bytes\": %llu, \"stream16_bytes\": %llu, \"lines_touched\": %u}\n", (unsigned long long)BUF,
              (unsigned long long)BUF, TOUCH);
  (void)hipFree(buf);
  (void)hipFree(sink);
  return 0;
}
