// FETCH_SIZE / WRITE_SIZE calibration kernels (tools/fetch_calib.py): known byte counts in the access patterns the step
// kernels use -- coalesced 4 / 8 / 16 B per lane streams (the SoA state), 16 lanes x 16 B and 16 lanes x 8 B gathers of
// one 256 / 128-byte record at a random aligned offset (a car's list heads, old / new format), one 4 / 8-byte load
// per random 128-byte line (cell map, pose records) -- over a buffer far beyond the 256 MB Infinity Cache.
// Diagnostic tooling, not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>

// sinks a value without a store unless it is (practically) never true
__device__ __forceinline__ void sink(float v, float* out) {
  if (v == 1234.5678f) out[threadIdx.x] = v;
}

__global__ void stream4(const float* __restrict__ a, size_t n, float* out) {
  float acc = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += a[i];
  sink(acc, out);
}
__global__ void stream8(const double* __restrict__ a, size_t n, float* out) {
  double acc = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += a[i];
  sink((float)acc, out);
}
__global__ void stream16(const float4* __restrict__ a, size_t n, float* out) {
  float acc = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    acc += v.x + v.y + v.z + v.w;
  }
  sink(acc, out);
}
// groups of 16 lanes: record r (random) of `rec` bytes, lane l reads bytes [l * rec / 16, (l + 1) * rec / 16)
template <typename T>
__device__ __forceinline__ void gather_rec(const T* __restrict__ a, uint32_t nrec, uint32_t records, float* out) {
  float acc = 0.0f;
  const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 4, l = threadIdx.x & 15;
  if (g < records) {
    const uint32_t r = (g * 2654435761u) & (nrec - 1);   // nrec a power of two: distinct records, scattered
    const T v = a[(size_t)r * 16 + l];
    acc = __uint_as_float(reinterpret_cast<const uint32_t*>(&v)[0]);   // (any value: the load must stay)
  }
  sink(acc, out);
}
// one T per lane at a random 128-byte line
template <typename T>
__device__ __forceinline__ void line_load(const T* __restrict__ a, uint32_t nline, uint32_t loads, float* out) {
  float acc = 0.0f;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < loads) {
    const uint32_t r = (i * 2246822519u) & (nline - 1);   // distinct lines, scattered
    const T v = a[(size_t)r * (128 / sizeof(T))];
    acc = __uint_as_float(reinterpret_cast<const uint32_t*>(&v)[0]);   // (any value: the load must stay)
  }
  sink(acc, out);
}
__global__ void gather16(const uint4* a, uint32_t nrec, uint32_t records, float* out) { gather_rec(a, nrec, records, out); }
__global__ void gather8(const uint2* a, uint32_t nrec, uint32_t records, float* out) { gather_rec(a, nrec, records, out); }
__global__ void line4(const uint32_t* a, uint32_t nline, uint32_t loads, float* out) { line_load(a, nline, loads, out); }
__global__ void line8(const uint2* a, uint32_t nline, uint32_t loads, float* out) { line_load(a, nline, loads, out); }
__global__ void wstream4(float* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (float)i;
}
__global__ void wstream8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}

extern "C" int calib_run(int which, void* buf, size_t bytes, uint32_t count, float* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int B = 256, G = 8192;
  switch (which) {
    case 0: hipLaunchKernelGGL(stream4, dim3(G), dim3(B), 0, s, (const float*)buf, bytes / 4, out); break;
    case 1: hipLaunchKernelGGL(stream8, dim3(G), dim3(B), 0, s, (const double*)buf, bytes / 8, out); break;
    case 2: hipLaunchKernelGGL(stream16, dim3(G), dim3(B), 0, s, (const float4*)buf, bytes / 16, out); break;
    case 3: hipLaunchKernelGGL(gather16, dim3((count * 16 + B - 1) / B), dim3(B), 0, s, (const uint4*)buf,
                               (uint32_t)(bytes / 256), count, out); break;
    case 4: hipLaunchKernelGGL(gather8, dim3((count * 16 + B - 1) / B), dim3(B), 0, s, (const uint2*)buf,
                               (uint32_t)(bytes / 128), count, out); break;
    case 5: hipLaunchKernelGGL(line4, dim3((count + B - 1) / B), dim3(B), 0, s, (const uint32_t*)buf,
                               (uint32_t)(bytes / 128), count, out); break;
    case 6: hipLaunchKernelGGL(line8, dim3((count + B - 1) / B), dim3(B), 0, s, (const uint2*)buf,
                               (uint32_t)(bytes / 128), count, out); break;
    case 7: hipLaunchKernelGGL(wstream4, dim3(G), dim3(B), 0, s, (float*)buf, bytes / 4); break;
    case 8: hipLaunchKernelGGL(wstream8, dim3(G), dim3(B), 0, s, (double*)buf, bytes / 8); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
