// Calibration of rocprofv3 WRITE_SIZE for the store patterns of wf_trace (development aid).
// Each kernel writes a known number of bytes; compare with WRITE_SIZE x 1024 per launch.
//   st16   16 B per lane, contiguous (the guide's calibrated case)
//   st8    8 B per lane, contiguous
//   perm8  8 B per lane, lanes of a wave scattered over a 1024-entry window (wf_trace's res
//          stores: a wave's rays come from one 1024-ray claim, finished in arbitrary order)
//   xcd8   8 B per lane, consecutive 8-B slots written by workgroups on different XCDs
//          (adjacent lines' halves from different L2s)
// Build: hipcc --offload-arch=gfx950 -O3 -o calib_write tools/calib_write.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void st16(float4* out, unsigned n) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = make_float4(i, 1, 2, 3);
}
__global__ void st8(int2* out, unsigned n) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = make_int2(i, 1);
}
__global__ void perm8(int2* out, unsigned n) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  // a 1024-entry window per 16 waves; within it a fixed odd-multiplier permutation
  const unsigned win = i & ~1023u, k = ((i & 1023u) * 389u + 17u) & 1023u;
  if (i < n) out[win + k] = make_int2(i, 1);
}
__global__ void xcd8(int2* out, unsigned n) {
  // block b writes entries j with (j / 2) % gridDim.x == b ... every 16-B pair is split over two
  // consecutive blocks (dispatched round-robin over the XCDs)
  const unsigned lane = threadIdx.x;
  const unsigned pairs = n / 2;
  for (unsigned p = blockIdx.x / 2 * blockDim.x + lane; p < pairs; p += gridDim.x / 2 * blockDim.x)
    out[2 * p + (blockIdx.x & 1)] = make_int2(p, 1);
}

int main() {
  const unsigned n = 1u << 26;  // 64 Mi entries
  void* buf;
  if (hipMalloc(&buf, (size_t)n * 16) != hipSuccess) return 1;
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(st16, dim3(n / 256), dim3(256), 0, 0, (float4*)buf, n);
    hipLaunchKernelGGL(st8, dim3(n / 256), dim3(256), 0, 0, (int2*)buf, n);
    hipLaunchKernelGGL(perm8, dim3(n / 256), dim3(256), 0, 0, (int2*)buf, n);
    hipLaunchKernelGGL(xcd8, dim3(4096), dim3(256), 0, 0, (int2*)buf, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("bytes written per launch: st16 %zu, st8/perm8/xcd8 %zu\n", (size_t)n * 16, (size_t)n * 8);
  (void)hipFree(buf);
  return 0;
}
