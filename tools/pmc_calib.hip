// Calibration of the rocprofv3 FETCH_SIZE / WRITE_SIZE counters (MI355X_MICROARCH.md §HBM: "Other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern") for the access widths the scheduling
// kernels use: coalesced column reads of 4 and 8 bytes per lane (sweep, rescans, commit row loads), the guide's
// 16-byte-per-lane reference read, and 4 / 8 / 16-byte coalesced stores.  Each kernel moves a known byte count once
// (every byte read or written exactly once, 256 MiB per read kernel so that the Infinity Cache holds nothing of it
// from the previous launch); tools/pmc_calib.py divides the counters by it.
//
// The commit and select kernels do not stream: one lane of a wave loads a 4- or 8-byte field of a node row, a quota
// row or a pod column, and stores a lone word.  The gather / scatter kernels reproduce that pattern on a known set of
// 128-byte lines: every line of the buffer is touched exactly once, by one word, in a scrambled order (an odd
// multiplier modulo a power of two is a bijection), by lane 0 of each wave (gather1 / scatter1) or by all 64 lanes at
// 64 different lines (gather64).  Their factor is reported per touched line, not per algorithmic byte.
//
// build: hipcc -O3 --offload-arch=gfx950 -o build/pmc_calib tools/pmc_calib.hip
// run:   rocprofv3 --pmc FETCH_SIZE -- build/pmc_calib   (and a second run with --pmc WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

template <typename T>
__global__ void read_kernel(const T* __restrict__ src, size_t n, unsigned long long* sink) {
  T acc{};
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = src[i];
    acc ^= v;
  }
  // one store per lane only when the accumulated value is a sentinel: nothing is written in practice
  if (acc == (T)0x5a5a5a5a) sink[0] = 1;
}

template <>
__global__ void read_kernel<uint4>(const uint4* __restrict__ src, size_t n, unsigned long long* sink) {
  unsigned int acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x5a5a5a5au) sink[0] = 1;
}

template <typename T>
__global__ void write_kernel(T* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v{};
    dst[i] = v;
  }
}

// lane 0 of each wave reads one T from each of nlines 128-byte lines, lines in scrambled order
template <typename T>
__global__ void gather1_kernel(const T* __restrict__ src, size_t nlines, unsigned long long* sink) {
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  T acc{};
  if ((threadIdx.x & 63) == 0)
    for (size_t j = wave; j < nlines; j += nwaves) acc ^= src[((j * 0x9E3779B1ull) & (nlines - 1)) * (128 / sizeof(T))];
  if (acc == (T)0x5a5a5a5a) sink[0] = 1;
}

// every lane reads one T from its own scrambled 128-byte line
template <typename T>
__global__ void gather64_kernel(const T* __restrict__ src, size_t nlines, unsigned long long* sink) {
  T acc{};
  for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < nlines; j += (size_t)gridDim.x * blockDim.x)
    acc ^= src[((j * 0x9E3779B1ull) & (nlines - 1)) * (128 / sizeof(T))];
  if (acc == (T)0x5a5a5a5a) sink[0] = 1;
}

// lane 0 of each wave stores one T into each of nlines 128-byte lines, lines in scrambled order
template <typename T>
__global__ void scatter1_kernel(T* __restrict__ dst, size_t nlines) {
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  if ((threadIdx.x & 63) == 0)
    for (size_t j = wave; j < nlines; j += nwaves) dst[((j * 0x9E3779B1ull) & (nlines - 1)) * (128 / sizeof(T))] = T{};
}

int main() {
  const size_t bytes = (size_t)256 << 20;
  void* buf = nullptr;
  unsigned long long* sink = nullptr;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(buf, 1, bytes));
  CHK(hipDeviceSynchronize());
  const dim3 grid(2048), block(256);
  // read_kernel<uint32_t>: 4 B/lane, <unsigned long long>: 8 B/lane, <uint4>: 16 B/lane
  hipLaunchKernelGGL(read_kernel<uint32_t>, grid, block, 0, 0, (const uint32_t*)buf, bytes / 4, sink);
  hipLaunchKernelGGL(read_kernel<unsigned long long>, grid, block, 0, 0, (const unsigned long long*)buf, bytes / 8, sink);
  hipLaunchKernelGGL(read_kernel<uint4>, grid, block, 0, 0, (const uint4*)buf, bytes / 16, sink);
  // 32 MiB per store kernel
  const size_t wb = (size_t)32 << 20;
  hipLaunchKernelGGL(write_kernel<uint32_t>, grid, block, 0, 0, (uint32_t*)buf, wb / 4);
  hipLaunchKernelGGL(write_kernel<unsigned long long>, grid, block, 0, 0, (unsigned long long*)buf, wb / 8);
  hipLaunchKernelGGL(write_kernel<uint4>, grid, block, 0, 0, (uint4*)buf, wb / 16);
  // scattered single words: 256 MiB of lines for the reads (2 Mi lines), 32 MiB for the stores (256 Ki lines)
  const size_t rl = bytes / 128, wl = wb / 128;
  hipLaunchKernelGGL(gather1_kernel<uint32_t>, grid, block, 0, 0, (const uint32_t*)buf, rl, sink);
  hipLaunchKernelGGL(gather1_kernel<unsigned long long>, grid, block, 0, 0, (const unsigned long long*)buf, rl, sink);
  hipLaunchKernelGGL(gather64_kernel<uint32_t>, grid, block, 0, 0, (const uint32_t*)buf, rl, sink);
  hipLaunchKernelGGL(gather64_kernel<unsigned long long>, grid, block, 0, 0, (const unsigned long long*)buf, rl, sink);
  hipLaunchKernelGGL(scatter1_kernel<uint32_t>, grid, block, 0, 0, (uint32_t*)buf, wl);
  hipLaunchKernelGGL(scatter1_kernel<unsigned long long>, grid, block, 0, 0, (unsigned long long*)buf, wl);
  CHK(hipGetLastError());
  CHK(hipDeviceSynchronize());
  printf("{\"read_bytes\": %zu, \"write_bytes\": %zu, \"read_lines\": %zu, \"write_lines\": %zu}\n", bytes, wb, rl, wl);
  CHK(hipFree(buf));
  CHK(hipFree(sink));
  return 0;
}
