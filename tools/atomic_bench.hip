// Device-scope atomicAdd throughput on gfx950 (development aid): every wave's lane 0 issues `iters`
// returning atomicAdds in a dependent chain (as wf_trace's claims do) on one of `lines` counters,
// counter k at word k * stride.  Prints atomics/us for each configuration.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/atomic_bench tools/atomic_bench.hip && /tmp/atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void chain(unsigned int* c, int iters, unsigned int lines, unsigned int stride, unsigned int* sink) {
  const unsigned int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) != 0) return;
  unsigned int* p = c + (size_t)(wave % lines) * stride;
  unsigned int acc = 0;
  for (int i = 0; i < iters; i++) acc += atomicAdd(p, 1u + (acc & 1u));
  sink[wave] = acc;
}

int main() {
  unsigned int *c = nullptr, *sink = nullptr;
  hipMalloc(&c, 1 << 20);
  hipMalloc(&sink, 1 << 22);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct Cfg { unsigned int blocks, lines, stride; int iters; };
  const std::vector<Cfg> cfgs = {
      {2048, 1, 1, 64}, {2048, 8, 32, 64}, {2048, 16, 1, 64}, {2048, 64, 32, 64},
      {256, 1, 1, 64},  {64, 1, 1, 256},  {2048, 8, 1, 64},  {2048, 256, 32, 64}};
  for (const Cfg& g : cfgs) {
    hipMemset(c, 0, 1 << 20);
    hipLaunchKernelGGL(chain, dim3(g.blocks), dim3(256), 0, 0, c, 4, g.lines, g.stride, sink);  // warm
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(chain, dim3(g.blocks), dim3(256), 0, 0, c, g.iters, g.lines, g.stride, sink);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    const double n = (double)g.blocks * 4.0 * g.iters;
    printf("waves %6u  counters %3u (stride %2u words)  atomics %9.0f  %8.3f ms  %8.1f atomics/us  %6.1f per counter/us\n",
           g.blocks * 4, g.lines, g.stride, n, ms, n / (ms * 1e3), n / (ms * 1e3) / g.lines);
  }
  hipFree(c);
  hipFree(sink);
  return 0;
}
