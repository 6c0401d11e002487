// GNN track (beyond the reference): uniform neighbour sampling on the GPU for
// mini-batch GraphSAGE.  The CSR stays resident in HBM (an ogbn-products CSR is
// ~0.5 GB of the 288 GB), so a mini-batch never leaves the device: sampling,
// relabelling (device hash map + sort in PyTorch), feature gather and training
// are one stream of kernels.
//
//   sample_neighbors_kernel   one thread per destination node v: deg <= fanout
//                             copies the whole row; otherwise Floyd's algorithm
//                             draws `fanout` distinct positions of the row
//                             (Philox keyed by (v, salt), so the sample of a node
//                             does not depend on the batch it is in or on the
//                             thread that draws it).
#include "cgnn_common.h"

using namespace cgnn;

template <int MAXF>
__global__ __launch_bounds__(256) void sample_neighbors_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ nodes, int n,
    int fanout, const int* __restrict__ out_ptr, int* __restrict__ out_col, uint32_t k0, uint32_t k1,
    uint32_t salt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int v = nodes[i];
  const int s = rowptr[v], deg = rowptr[v + 1] - s;
  int* dst = out_col + out_ptr[i];
  if (fanout < 0 || deg <= fanout) {
    for (int k = 0; k < deg; ++k) dst[k] = col[s + k];
    return;
  }
  int sel[MAXF];
  u32x4 r = {0u, 0u, 0u, 0u};
  int m = 0;
  for (int j = deg - fanout; j < deg; ++j, ++m) {
    if ((m & 3) == 0) r = philox4x32_10(u32x4{(uint32_t)v, salt, (uint32_t)(m >> 2), RNG_SAMPLE}, k0, k1);
    const uint32_t w = (m & 3) == 0 ? r.x : (m & 3) == 1 ? r.y : (m & 3) == 2 ? r.z : r.w;
    const int t = (int)(((uint64_t)w * (uint64_t)(j + 1)) >> 32);     // uniform in [0, j]
    bool dup = false;
    for (int q = 0; q < m; ++q) dup |= (sel[q] == t);
    sel[m] = dup ? j : t;
  }
  for (int k = 0; k < fanout; ++k) dst[k] = col[s + sel[k]];
}

extern "C" int gnn_launch_sample_neighbors(const int* rowptr, const int* col, const int* nodes, int n, int fanout,
                                           const int* out_ptr, int* out_col, uint32_t k0, uint32_t k1,
                                           uint32_t salt, hipStream_t st) {
  if (n <= 0) return 0;
  dim3 grid((n + 255) / 256), block(256);
  if (fanout <= 16)
    hipLaunchKernelGGL((sample_neighbors_kernel<16>), grid, block, 0, st, rowptr, col, nodes, n, fanout, out_ptr,
                       out_col, k0, k1, salt);
  else if (fanout <= 64)
    hipLaunchKernelGGL((sample_neighbors_kernel<64>), grid, block, 0, st, rowptr, col, nodes, n, fanout, out_ptr,
                       out_col, k0, k1, salt);
  else
    return -3;
  return (int)hipGetLastError();
}
