// Calibration of the rocprofv3 FETCH_SIZE / WRITE_SIZE counters (MI355X_MICROARCH.md §HBM: "Other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern") for the access widths the scheduling
// kernels use: coalesced column reads of 4 and 8 bytes per lane (sweep, rescans, commit row loads), the guide's
// 16-byte-per-lane reference read, and 4 / 8 / 16-byte coalesced stores.  Each kernel moves a known byte count once
// (every byte read or written exactly once, 256 MiB per read kernel so that the Infinity Cache holds nothing of it
// from the previous launch); tools/pmc_calib.py divides the counters by it.
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
  CHK(hipGetLastError());
  CHK(hipDeviceSynchronize());
  printf("{\"read_bytes\": %zu, \"write_bytes\": %zu}\n", bytes, wb);
  CHK(hipFree(buf));
  CHK(hipFree(sink));
  return 0;
}
