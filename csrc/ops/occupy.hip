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

// ---- byte-moving occupant ---------------------------------------------------------------------
// The same stand-in, but its workgroups also move the HBM bytes an RCCL ring all-reduce moves on one
// rank: each streams 16 B per lane from `src` (the bucket) to `dst` (a scratch buffer, so the
// gradients stay intact) in 16 KiB pieces, cycling over its slice, paced so that the grid moves
// `total` bytes (reads + writes) in `ticks`: a piece is issued only while the workgroup is behind its
// share of the schedule, otherwise it sleeps. It ends once the time is up AND its share is moved
// (contention can stretch it, as it stretches a real collective), and never later than 4x the time:
// every wave exits and the grid drains.
__global__ __launch_bounds__(256) void occupy_bytes_kernel(uint64_t ticks, const uint4* __restrict__ src,
                                                           uint4* __restrict__ dst, int64_t n16,
                                                           int64_t share_pieces, int* __restrict__ done) {
  extern __shared__ int lds_pad[];
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0) lds_pad[0] = blockIdx.x;
  constexpr int kPiece = 256 * 4;  // uint4 per piece: 16 KiB
  const int64_t pieces_all = n16 / kPiece;
  int64_t piece = pieces_all > 0 ? ((int64_t)blockIdx.x * pieces_all) / gridDim.x : 0;
  int64_t moved = 0;  // pieces moved by this workgroup
  while (true) {
    const uint64_t el = wall_clock64() - t0;
    if ((el >= ticks && moved >= share_pieces) || el >= 4 * ticks) break;
    // behind schedule (moved / share < elapsed / ticks): move a piece, else wait
    if (pieces_all > 0 && (double)moved * (double)ticks < (double)share_pieces * (double)el) {
      const int64_t base = piece * kPiece;
      uint4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = src[base + threadIdx.x + 256 * i];
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[base + threadIdx.x + 256 * i] = v[i];
      ++moved;
      if (++piece >= pieces_all) piece = 0;
    } else {
      __builtin_amdgcn_s_sleep(8);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(done, lds_pad[0] >= 0 ? 1 : 0);
}

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

void occupy_bytes(int n_workgroups, int lds_bytes, double ms, const void* src, void* dst, int64_t nbytes,
                  int64_t total_bytes, int* done, hipStream_t s) {
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (khz <= 0) khz = 100000;
  const uint64_t ticks = (uint64_t)(ms * (double)khz);
  // a piece = 16 KiB read + 16 KiB written
  const int64_t share = total_bytes / (2 * 16384) / (n_workgroups > 0 ? n_workgroups : 1);
  hipLaunchKernelGGL(occupy_bytes_kernel, dim3((unsigned)n_workgroups), dim3(256), (size_t)lds_bytes, s, ticks,
                     static_cast<const uint4*>(src), static_cast<uint4*>(dst), nbytes / 16, share, done);
}

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
