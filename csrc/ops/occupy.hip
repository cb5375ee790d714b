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

namespace {

// ---- co-residency probe ("cohort") ---------------------------------------------------------------
// An RCCL collective kernel only finishes once ALL of its channel blocks run (each waits for its
// ring/peer partners), so the property that matters beside a stream-K GEMM is not "an occupant ends
// by itself" (occupy_kernel above) but "an occupant that needs every one of its workgroups resident at
// the same time gets them". The cohort models exactly that: each workgroup arrives on a counter, then
// waits until all gridDim.x have arrived -- bounded by a wall-clock deadline, so a stranded cohort
// gives up instead of hanging the GPU and records the failure in state[1] (workgroups that timed
// out). Shape of one RCCL gfx950 channel block (librccl.so code-object metadata): 256 threads,
// 21,184 B static LDS, up to ~122 VGPRs -> `lds_bytes` is dynamic and the asm clobber of v127 makes
// every wave allocate 128 VGPRs. state[0] (arrivals) must be zero at launch (cohort() memsets it).
__global__ __launch_bounds__(256) void cohort_kernel(uint64_t ticks, int* __restrict__ state) {
  extern __shared__ int lds_pad[];
  asm volatile("" ::: "v127");  // hold 128 VGPRs per wave, like an RCCL channel block
  if (threadIdx.x == 0) {
    lds_pad[0] = blockIdx.x;
    const uint64_t t0 = wall_clock64();
    __hip_atomic_fetch_add(&state[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool all_in = false;
    while (wall_clock64() - t0 < ticks) {
      if (__hip_atomic_load(&state[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (int)gridDim.x) {
        all_in = true;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    if (!all_in) atomicAdd(&state[1], 1);
    // longest wait any workgroup saw for the cohort to assemble (100 MHz ticks)
    atomicMax(reinterpret_cast<unsigned*>(&state[2]), (unsigned)min<uint64_t>(wall_clock64() - t0, 0xffffffffu));
  }
  __syncthreads();
}

}  // namespace

void cohort(int n_workgroups, int lds_bytes, double deadline_ms, int* state, hipStream_t s) {
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (khz <= 0) khz = 100000;
  const uint64_t ticks = (uint64_t)(deadline_ms * (double)khz);
  (void)hipMemsetAsync(state, 0, sizeof(int), s);  // arrivals only: timeouts/max-wait accumulate
  hipLaunchKernelGGL(cohort_kernel, dim3((unsigned)n_workgroups), dim3(256), (size_t)lds_bytes, s, ticks, state);
}

}  // namespace cs336
