// Deterministic, graph-safe token-embedding backward for MI355X.
//
// Reference semantics (cs336-basics/cs336_basics/model.py:47-60, the table lookup): the weight
// gradient row v is the sum of the output gradient rows of every position whose token id is v.
// ATen's CUDA backward sorts the ids and partitions them with data-dependent sizes (a HIP graph
// captured around it faulted when replayed on batches with more distinct tokens); an index_add_
// fallback sums with float atomics, so the result changes run to run. Here the ids are sorted with
// their positions once (torch.sort, stable: fixed-size, no host sync) and one 256-thread workgroup
// per vocabulary row finds its run [lo, hi) of equal ids by binary search and adds the gradient
// rows of those positions in position order: the same bits on every run, eager or replayed, and one
// read of the output gradient plus one write of the table. Rows with no occurrence are written as
// zeros, so the output needs no memset (it can be a DDP bucket view: parallel/ddp.py).
#include "cs336/kernels.h"

namespace cs336 {
namespace {

__device__ __forceinline__ int64_t lower_bound(const int64_t* __restrict__ a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <typename TG>
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const typename Elem<TG>::storage* __restrict__ g,
                                                            const int64_t* __restrict__ sorted_ids,
                                                            const int64_t* __restrict__ perm, float* __restrict__ gw,
                                                            int64_t n_tok, int64_t D) {
  const int64_t v = blockIdx.x;
  const int64_t lo = lower_bound(sorted_ids, n_tok, v);
  const int64_t hi = lower_bound(sorted_ids, n_tok, v + 1);
  float* out = gw + v * D;
  // D % 4 == 0 (host check): float4 columns, 256 lanes stride over the row
  for (int64_t c = 4 * threadIdx.x; c < D; c += 4 * 256) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = lo; i < hi; ++i) {
      const float4 x = load4<TG>(g + perm[i] * D + c);
      acc.x += x.x;
      acc.y += x.y;
      acc.z += x.z;
      acc.w += x.w;
    }
    *reinterpret_cast<float4*>(out + c) = acc;
  }
}

}  // namespace

void embedding_bwd(const void* g, DType gt, const int64_t* sorted_ids, const int64_t* perm, float* gw, int64_t n_tok,
                   int64_t V, int64_t D, hipStream_t s) {
  if (V == 0) return;
  const dim3 grid((unsigned)V), block(256);
  switch (gt) {
    case DType::F32:
      hipLaunchKernelGGL(embedding_bwd_kernel<float>, grid, block, 0, s, static_cast<const float*>(g), sorted_ids,
                         perm, gw, n_tok, D);
      break;
    case DType::BF16:
      hipLaunchKernelGGL(embedding_bwd_kernel<BF16>, grid, block, 0, s, static_cast<const Elem<BF16>::storage*>(g),
                         sorted_ids, perm, gw, n_tok, D);
      break;
    case DType::F16:
      hipLaunchKernelGGL(embedding_bwd_kernel<F16>, grid, block, 0, s, static_cast<const Elem<F16>::storage*>(g),
                         sorted_ids, perm, gw, n_tok, D);
      break;
  }
}

}  // namespace cs336
