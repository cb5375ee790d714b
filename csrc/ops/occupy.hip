// CU-occupying, time-bounded spin kernel: a stand-in for RCCL's persistent channel kernels in
// concurrency tests (tests/test_concurrency_gpu.py).
//
// Each workgroup reserves `lds_bytes` of LDS (so the host controls how many of them fit on a CU, and
// how much room is left for a GEMM workgroup beside them), then sleeps in a loop on the 100 MHz wall
// clock until `ticks` have passed, and bumps a completion counter with one vector atomic. The spin is
// bounded by time, never by another kernel's progress, so every wave exits and the grid always
// drains -- like an RCCL kernel whose peers are slow but do arrive.
#include "cs336/kernels.h"

namespace cs336 {
namespace {

__global__ __launch_bounds__(256) void occupy_kernel(uint64_t ticks, int* __restrict__ done) {
  extern __shared__ int lds_pad[];
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0) lds_pad[0] = blockIdx.x;  // touch the allocation
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(done, lds_pad[0] >= 0 ? 1 : 0);
}

}  // namespace

void occupy(int n_workgroups, int lds_bytes, double ms, int* done, hipStream_t s) {
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (khz <= 0) khz = 100000;  // MI300/MI355X wall clock: 100 MHz
  const uint64_t ticks = (uint64_t)(ms * (double)khz);
  hipLaunchKernelGGL(occupy_kernel, dim3((unsigned)n_workgroups), dim3(256), (size_t)lds_bytes, s, ticks, done);
}

}  // namespace cs336
