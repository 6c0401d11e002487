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
#include <algorithm>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

using namespace cgnn;

template <int MAXF>
__global__ __launch_bounds__(256) void sample_neighbors_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ nodes, int n,
    int fanout, const int* __restrict__ out_ptr, int* __restrict__ out_col, uint32_t k0, uint32_t k1,
    uint32_t salt, const int* __restrict__ n_dev, uint8_t* __restrict__ flag) {
  // n_dev (optional): the row count lives in device memory (the grid covers an upper bound);
  // flag (optional): flag[pick] = 1 for every pick (the pipeline's source marks)
  if (n_dev) n = *n_dev;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int v = nodes[i];
  const int s = rowptr[v], deg = rowptr[v + 1] - s;
  int* dst = out_col + out_ptr[i];
  if (fanout < 0 || deg <= fanout) {
    for (int k = 0; k < deg; ++k) {
      const int c = col[s + k];
      dst[k] = c;
      if (flag) flag[c] = 1;
    }
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
  for (int k = 0; k < fanout; ++k) {
    const int c = col[s + sel[k]];
    dst[k] = c;
    if (flag) flag[c] = 1;
  }
}

extern "C" int gnn_launch_sample_neighbors(const int* rowptr, const int* col, const int* nodes, int n, int fanout,
                                           const int* out_ptr, int* out_col, uint32_t k0, uint32_t k1,
                                           uint32_t salt, hipStream_t st) {
  if (n <= 0) return 0;
  dim3 grid((n + 255) / 256), block(256);
  if (fanout <= 16)
    hipLaunchKernelGGL((sample_neighbors_kernel<16>), grid, block, 0, st, rowptr, col, nodes, n, fanout, out_ptr,
                       out_col, k0, k1, salt, (const int*)nullptr, (uint8_t*)nullptr);
  else if (fanout <= 64)
    hipLaunchKernelGGL((sample_neighbors_kernel<64>), grid, block, 0, st, rowptr, col, nodes, n, fanout, out_ptr,
                       out_col, k0, k1, salt, (const int*)nullptr, (uint8_t*)nullptr);
  else
    return -3;
  return (int)hipGetLastError();
}

// ============================================================================
// Whole mini-batch sampling pipeline without host synchronisation
// (gnn_sample_blocks, driven from C++): for every level the row counts live in
// device memory and every grid covers a host-known upper bound, so the host
// enqueues all levels at once and learns the sizes with ONE copy at the end --
// on a side stream, while the previous batch trains.
//
// Level l (destinations = seeds for l = 0, else the sources of level l - 1), 7
// launches, 11 with the transposed CSR (16 before round 6):
//   count_scan    cnt = min(deg, fanout) -> per-block sums, then the exclusive scan
//                 -> rowptr, 1 / cnt, total picks: every block of the second pass sums
//                 its predecessors' block sums itself (at most a few hundred), so no
//                 single-block middle pass
//   sample        Floyd picks (sample_neighbors_kernel, device row count), marking
//                 flag[pick] = 1 as they are written
//   dst_fix       flag[dst] = 0, map[dst] = i, src[i] = dst
//   flag_scan     per 4096-id block counts (16 flags per thread), then compaction
//                 (each block sums its predecessors' counts; n_src = n_dst + new
//                 sources): the new sources in increasing id order -> src[n_dst + k],
//                 map, flag = 0
//   relabel       local[e] = map[pick[e]] (+ the transposed CSR's histogram)
//   transpose     (blocks the backward scatters through) scan of the histogram,
//                 per-destination scatter, per-bucket insertion sort: the
//                 transposed CSR in increasing destination order (deterministic)
// No state needs resetting between levels or batches: every flag set is cleared
// by dst_fix / compaction, and map entries are only read for ids set this level.
// ============================================================================
namespace {
constexpr int FLAG_BLK = 4096;

}  // namespace

// ---- multi-block exclusive scans with a device-side length (grid over an upper bound):
// A: values of a 1024-element block -> vals[], block sum -> bsum[b]
// B: one block scans the block sums -> boff[], total -> *total and out[n]
// C: block-local scan of vals + boff[b] -> out[]
constexpr int SB = 1024;          // elements per scan block (256 threads x 4)

__device__ __forceinline__ int block_excl_scan4(int v0, int v1, int v2, int v3, int* tot, int* shw) {
  // 256 threads x 4 consecutive items: returns the exclusive prefix of this thread's
  // first item within the block; *tot = block total
  const int s = v0 + v1 + v2 + v3;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) shw[w] = x;
  __syncthreads();
  int wo = 0;
  for (int q = 0; q < w; ++q) wo += shw[q];
  *tot = shw[0] + shw[1] + shw[2] + shw[3];
  return wo + x - s;
}

// count values: cnt = min(deg(node), fanout) (also 1 / cnt) or an int array (reset to 0)
__global__ __launch_bounds__(256) void sb_scanA_kernel(const int* __restrict__ rowptr, const int* __restrict__ nodes,
                                                       int fanout, float* __restrict__ inv_deg, int* __restrict__ arr,
                                                       int n_host, const int* __restrict__ n_dev,
                                                       int* __restrict__ vals, int* __restrict__ bsum) {
  __shared__ int shw[4];
  const int n = n_dev ? *n_dev : n_host;
  const int base = blockIdx.x * SB;
  if (base >= n && blockIdx.x > 0) return;
  int v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = base + 4 * threadIdx.x + q;
    int x = 0;
    if (i < n) {
      if (nodes) {
        const int nd = nodes[i];
        const int d = rowptr[nd + 1] - rowptr[nd];
        x = fanout < 0 ? d : min(d, fanout);
        inv_deg[i] = x > 0 ? 1.f / (float)x : 0.f;
      } else {
        x = arr[i];
        arr[i] = 0;                  // the histogram becomes the scatter cursor
      }
      vals[i] = x;
    }
    v[q] = x;
  }
  int tot;
  (void)block_excl_scan4(v[0], v[1], v[2], v[3], &tot, shw);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// sum of v over the block (every thread gets it); sh: 4 ints of shared memory
__device__ __forceinline__ int block_sum256(int v, int* sh) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  __syncthreads();                              // sh may still be read by a previous use
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

// second pass of the scan: block b's offset is the sum of bsum[0..b) (each block adds its
// predecessors' sums itself), then the block-local scan of vals; the last block with data
// (block 0 when n == 0) writes out[n] = total and *total
__global__ __launch_bounds__(256) void sb_scan_fin_kernel(const int* __restrict__ vals, const int* __restrict__ bsum,
                                                          int n_host, const int* __restrict__ n_dev,
                                                          int* __restrict__ out, int* __restrict__ total) {
  __shared__ int shw[4], shr[4];
  const int n = n_dev ? *n_dev : n_host;
  const int base = blockIdx.x * SB;
  if (blockIdx.x > 0 && base >= n) return;      // uniform per block
  int pre = 0;
  for (int q = threadIdx.x; q < (int)blockIdx.x; q += 256) pre += bsum[q];
  pre = block_sum256(pre, shr);
  int v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = base + 4 * threadIdx.x + q;
    v[q] = i < n ? vals[i] : 0;
  }
  int tot;
  int run = pre + block_excl_scan4(v[0], v[1], v[2], v[3], &tot, shw);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = base + 4 * threadIdx.x + q;
    if (i < n) out[i] = run;
    run += v[q];
  }
  const int last = n > 0 ? (n - 1) / SB : 0;
  if ((int)blockIdx.x == last && threadIdx.x == 0) {
    out[n] = pre + tot;
    if (total) *total = pre + tot;
  }
}

__global__ __launch_bounds__(256) void sb_dst_fix_kernel(const int* __restrict__ nodes, int n_host,
                                                         const int* __restrict__ n_dev, uint8_t* __restrict__ flag,
                                                         int* __restrict__ map, int* __restrict__ src) {
  const int n = n_dev ? *n_dev : n_host;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int v = nodes[i];
  flag[v] = 0;
  map[v] = i;
  src[i] = v;
}

// 0/1 flag bytes of a word, summed
__device__ __forceinline__ int flag_sum4(uint32_t w) { return (int)((w * 0x01010101u) >> 24); }

// per 4096-id block: the count of set flags (16 flags per thread, one 16-B load; the flag
// array is padded to whole blocks, gnn_sample_flag_bytes)
__global__ __launch_bounds__(256) void sb_flag_count_kernel(const uint8_t* __restrict__ flag,
                                                            int* __restrict__ bcount) {
  __shared__ int sh[4];
  const uint4 w = reinterpret_cast<const uint4*>(flag + (size_t)blockIdx.x * FLAG_BLK)[threadIdx.x];
  const int c = block_sum256(flag_sum4(w.x) + flag_sum4(w.y) + flag_sum4(w.z) + flag_sum4(w.w), sh);
  if (threadIdx.x == 0) bcount[blockIdx.x] = c;
}

// the new sources of each 4096-id block in increasing id order: 16 consecutive ids per
// thread, the block's offset the sum of its predecessors' counts (no single-block scan
// pass); the last block writes n_src = n_dst + new sources
__global__ __launch_bounds__(256) void sb_compact_kernel(uint8_t* __restrict__ flag, const int* __restrict__ bcount,
                                                         int n_dst_host, const int* __restrict__ n_dst_dev,
                                                         int* __restrict__ map, int* __restrict__ src,
                                                         int* __restrict__ n_src) {
  __shared__ int shw[4], shr[4];
  const int nd = n_dst_dev ? *n_dst_dev : n_dst_host;
  int pre = 0;
  for (int q = threadIdx.x; q < (int)blockIdx.x; q += 256) pre += bcount[q];
  pre = block_sum256(pre, shr);
  uint4* wp = reinterpret_cast<uint4*>(flag + (size_t)blockIdx.x * FLAG_BLK) + threadIdx.x;
  const uint4 w = *wp;
  const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
  const int c0 = flag_sum4(w.x), c1 = flag_sum4(w.y), c2 = flag_sum4(w.z), c3 = flag_sum4(w.w);
  int tot;
  int k = pre + block_excl_scan4(c0, c1, c2, c3, &tot, shw);
  if (c0 + c1 + c2 + c3) {
    const int i0 = blockIdx.x * FLAG_BLK + 16 * threadIdx.x;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if ((ww[q >> 2] >> (8 * (q & 3))) & 0xffu) {
        map[i0 + q] = nd + k;
        src[nd + k] = i0 + q;
        ++k;
      }
    }
    *wp = make_uint4(0u, 0u, 0u, 0u);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_src = nd + pre + tot;
}

// local[e] = map[pick[e]]; cnt (optional): the transposed CSR's histogram of local ids
__global__ __launch_bounds__(256) void sb_relabel_kernel(const int* __restrict__ picks, const int* __restrict__ total,
                                                         const int* __restrict__ map, int* __restrict__ local,
                                                         int* __restrict__ cnt) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < *total) {
    const int l = map[picks[e]];
    local[e] = l;
    if (cnt) atomicAdd(&cnt[l], 1);
  }
}

__global__ __launch_bounds__(256) void sb_scatter_kernel(const int* __restrict__ optr, const int* __restrict__ local,
                                                         int n_host, const int* __restrict__ n_dev,
                                                         const int* __restrict__ rp_t, int* __restrict__ cursor,
                                                         int* __restrict__ col_t) {
  const int n = n_dev ? *n_dev : n_host;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int e = optr[i]; e < optr[i + 1]; ++e) {
    const int c = local[e];
    col_t[rp_t[c] + atomicAdd(&cursor[c], 1)] = i;
  }
}

// (also clears the scatter cursors: cnt is all zero again for the slot's next batch)
__global__ __launch_bounds__(256) void sb_bucket_sort_kernel(const int* __restrict__ rp_t,
                                                             const int* __restrict__ n_dev, int* __restrict__ col_t,
                                                             int* __restrict__ cnt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= *n_dev) return;
  cnt[c] = 0;
  const int a = rp_t[c], b = rp_t[c + 1];
  for (int i = a + 1; i < b; ++i) {
    const int x = col_t[i];
    int j = i - 1;
    while (j >= a && col_t[j] > x) {
      col_t[j + 1] = col_t[j];
      --j;
    }
    col_t[j + 1] = x;
  }
}

// the level sizes to mapped host memory (read by the host after the batch's event)
__global__ void sb_publish_kernel(const int* __restrict__ counts, int* __restrict__ host, int n) {
  const int i = threadIdx.x;
  if (i < n) __hip_atomic_store(host + i, counts[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static unsigned blocks_for(long n, int t = 256) { return (unsigned)std::max(1L, (n + t - 1) / t); }

// int32 scratch the pipeline needs (bscratch argument of gnn_launch_sample_blocks)
extern "C" long gnn_sample_blocks_scratch(int n, int L, const int* fan, const int* nd_max) {
  const long nb = (n + FLAG_BLK - 1) / FLAG_BLK;
  long vmax = 1;
  for (int l = 0; l < L; ++l) vmax = std::max(vmax, std::min<long>((long)nd_max[l] * (fan[l] + 1), (long)n) + 1);
  const long sbmax = (vmax + SB - 1) / SB + 1;
  return 2 * nb + 2 + 2 * sbmax + vmax;
}

// bytes of the pipeline's flag array for n ids: whole 4096-id blocks (the flag passes
// read 16 bytes per thread without a bound check; the padding is never set)
extern "C" long gnn_sample_flag_bytes(int n) { return ((long)n + FLAG_BLK) / FLAG_BLK * FLAG_BLK; }

// One level per entry of the arrays (L levels): nd_max[l] bounds the destinations,
// fan[l] the fanout; dst of level 0 = seeds (n_seeds on the host), of level l > 0 =
// src[l - 1] with its device count counts[2 (l - 1)].  counts[2 l] = n_src of level
// l, counts[2 l + 1] = its picks.  Transposed CSR built for levels with rp_t[l] != 0.
// counts_host (optional, device address of mapped host memory): the counts published
// there by a kernel at the end (no copy call).  cnt_t[l] must be zero on entry; the
// pipeline leaves it zero.
extern "C" int gnn_launch_sample_blocks(const int* rowptr, const int* col, int n, const int* seeds, int n_seeds,
                                        int L, const int* fan, const int* nd_max, int* const* optr,
                                        float* const* inv_deg, int* const* picks, int* const* local,
                                        int* const* src, int* const* rp_t, int* const* col_t, int* const* cnt_t,
                                        int* counts, uint8_t* flag, int* map, int* bscratch, uint32_t k0,
                                        uint32_t k1, uint32_t salt, hipStream_t st, int* counts_host) {
  const int nb = (n + FLAG_BLK - 1) / FLAG_BLK;
  // scan scratch after the flag-scan counts: block sums, block offsets, values
  long vmax = 1;
  for (int l = 0; l < L; ++l) vmax = std::max(vmax, std::min<long>((long)nd_max[l] * (fan[l] + 1), (long)n) + 1);
  const long sbmax = (vmax + SB - 1) / SB + 1;
  int* sbsum = bscratch + 2 * nb + 2;
  int* svals = sbsum + 2 * sbmax;
  for (int l = 0; l < L; ++l) {
    const int fo = fan[l];
    if (fo < 1 || fo > 64) return -3;
    const int* nodes = l == 0 ? seeds : src[l - 1];
    const int* nd_dev = l == 0 ? nullptr : counts + 2 * (l - 1);
    const int ndh = l == 0 ? n_seeds : 0;
    int* total = counts + 2 * l + 1;
    int* nsrc = counts + 2 * l;
    const long pmax = (long)nd_max[l] * fo;
    // rowptr of the level: exclusive scan of min(deg, fanout) (+ 1 / cnt, total picks)
    const unsigned nbs = blocks_for(nd_max[l], SB);
    hipLaunchKernelGGL(sb_scanA_kernel, dim3(nbs), dim3(256), 0, st, rowptr, nodes, fo, inv_deg[l], (int*)nullptr,
                       ndh, nd_dev, svals, sbsum);
    hipLaunchKernelGGL(sb_scan_fin_kernel, dim3(nbs), dim3(256), 0, st, svals, sbsum, ndh, nd_dev, optr[l], total);
    const uint32_t lsalt = salt * 16u + (uint32_t)l;
    if (fo <= 16)
      hipLaunchKernelGGL((sample_neighbors_kernel<16>), dim3(blocks_for(nd_max[l])), dim3(256), 0, st, rowptr, col,
                         nodes, ndh, fo, optr[l], picks[l], k0, k1, lsalt, nd_dev, flag);
    else
      hipLaunchKernelGGL((sample_neighbors_kernel<64>), dim3(blocks_for(nd_max[l])), dim3(256), 0, st, rowptr, col,
                         nodes, ndh, fo, optr[l], picks[l], k0, k1, lsalt, nd_dev, flag);
    hipLaunchKernelGGL(sb_dst_fix_kernel, dim3(blocks_for(nd_max[l])), dim3(256), 0, st, nodes, ndh, nd_dev, flag,
                       map, src[l]);
    hipLaunchKernelGGL(sb_flag_count_kernel, dim3(nb), dim3(256), 0, st, flag, bscratch);
    hipLaunchKernelGGL(sb_compact_kernel, dim3(nb), dim3(256), 0, st, flag, bscratch, ndh, nd_dev, map, src[l],
                       nsrc);
    hipLaunchKernelGGL(sb_relabel_kernel, dim3(blocks_for(pmax)), dim3(256), 0, st, picks[l], total, map, local[l],
                       rp_t[l] ? cnt_t[l] : (int*)nullptr);
    if (rp_t[l]) {
      const long smax = std::min<long>((long)nd_max[l] * (fo + 1), (long)n);
      const unsigned nbt = blocks_for(smax, SB);
      hipLaunchKernelGGL(sb_scanA_kernel, dim3(nbt), dim3(256), 0, st, (const int*)nullptr, (const int*)nullptr, 0,
                         (float*)nullptr, cnt_t[l], 0, nsrc, svals, sbsum);
      hipLaunchKernelGGL(sb_scan_fin_kernel, dim3(nbt), dim3(256), 0, st, svals, sbsum, 0, nsrc, rp_t[l],
                         (int*)nullptr);
      hipLaunchKernelGGL(sb_scatter_kernel, dim3(blocks_for(nd_max[l])), dim3(256), 0, st, optr[l], local[l], ndh,
                         nd_dev, rp_t[l], cnt_t[l], col_t[l]);
      hipLaunchKernelGGL(sb_bucket_sort_kernel, dim3(blocks_for(smax)), dim3(256), 0, st, rp_t[l], nsrc, col_t[l],
                         cnt_t[l]);
    }
  }
  if (counts_host) hipLaunchKernelGGL(sb_publish_kernel, dim3(1), dim3(64), 0, st, counts, counts_host, 2 * L);
  return (int)hipGetLastError();
}

// ============================================================================
// Sampling worker: a native thread that owns the side stream and issues each
// batch's ~40 pipeline launches, so that the Python thread only posts a job and
// goes on enqueuing the training step (the host's launch time per batch was the
// SAGE loop's critical path: profiles/r05_sage).  Jobs run in submission order;
// each waits for the events it names (seeds ready, the slot's previous reader
// done), launches gnn_launch_sample_blocks and records the slot's done event.
// wait(seq) blocks (no GIL) until job seq was issued and its sampling finished,
// then orders the consumer stream after it.
// ============================================================================
namespace {
struct WorkerSlot {
  std::vector<int*> optr, picks, local, src, rp_t, col_t, cnt_t;
  std::vector<float*> inv;
  int* counts = nullptr;
  int* host = nullptr;
  hipEvent_t done = nullptr;
};

struct WorkerJob {
  int slot;
  const int* seeds;
  int n;
  uint32_t salt;
  std::vector<hipEvent_t> waits;
  uint64_t seq;
};

struct SampleWorker {
  int device;
  hipStream_t st;
  const int* rowptr;
  const int* col;
  int n;
  std::vector<int> fan, nd_max;
  uint8_t* flag;
  int* map;
  int* bscratch;
  uint32_t k0, k1;
  std::vector<WorkerSlot> slots;
  std::mutex m;
  std::condition_variable cv_job, cv_done;
  std::deque<WorkerJob> q;
  uint64_t submitted = 0, issued = 0;
  int err = 0;
  bool stop = false;
  std::thread th;

  void run() {
    (void)hipSetDevice(device);
    for (;;) {
      WorkerJob j;
      {
        std::unique_lock<std::mutex> lk(m);
        cv_job.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;            // stop requested and drained
        j = std::move(q.front());
        q.pop_front();
      }
      int e = 0;
      for (hipEvent_t ev : j.waits)
        if (!e) e = (int)hipStreamWaitEvent(st, ev, 0);
      WorkerSlot& s = slots[j.slot];
      if (!e)
        e = gnn_launch_sample_blocks(rowptr, col, n, j.seeds, j.n, (int)fan.size(), fan.data(), nd_max.data(),
                                     s.optr.data(), s.inv.data(), s.picks.data(), s.local.data(), s.src.data(),
                                     s.rp_t.data(), s.col_t.data(), s.cnt_t.data(), s.counts, flag, map, bscratch, k0,
                                     k1, j.salt, st, s.host);
      if (!e) e = (int)hipEventRecord(s.done, st);
      {
        std::lock_guard<std::mutex> lk(m);
        if (e && !err) err = e;
        issued = j.seq;
      }
      cv_done.notify_all();
    }
  }
};
}  // namespace

extern "C" void* gnn_sw_create(int device, hipStream_t st, const int* rowptr, const int* col, int n, int L,
                               const int* fan, const int* nd_max, uint8_t* flag, int* map, int* bscratch, uint32_t k0,
                               uint32_t k1) {
  auto* w = new SampleWorker();
  w->device = device;
  w->st = st;
  w->rowptr = rowptr;
  w->col = col;
  w->n = n;
  w->fan.assign(fan, fan + L);
  w->nd_max.assign(nd_max, nd_max + L);
  w->flag = flag;
  w->map = map;
  w->bscratch = bscratch;
  w->k0 = k0;
  w->k1 = k1;
  return w;
}

// per-level pointer arrays of one slot (L entries each); returns the slot index or < 0
extern "C" int gnn_sw_add_slot(void* h, int* const* optr, float* const* inv, int* const* picks, int* const* local,
                               int* const* src, int* const* rp_t, int* const* col_t, int* const* cnt_t, int* counts,
                               int* host) {
  auto* w = static_cast<SampleWorker*>(h);
  if (w->th.joinable()) return -1;          // slots are fixed once the thread runs
  const size_t L = w->fan.size();
  WorkerSlot s;
  s.optr.assign(optr, optr + L);
  s.inv.assign(inv, inv + L);
  s.picks.assign(picks, picks + L);
  s.local.assign(local, local + L);
  s.src.assign(src, src + L);
  s.rp_t.assign(rp_t, rp_t + L);
  s.col_t.assign(col_t, col_t + L);
  s.cnt_t.assign(cnt_t, cnt_t + L);
  s.counts = counts;
  s.host = host;
  if (hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) return -2;
  w->slots.push_back(std::move(s));
  return (int)w->slots.size() - 1;
}

// post a batch (the events are waited for on the worker's stream before the launches;
// they must stay alive until the job is issued); returns its sequence number (>= 1)
extern "C" long gnn_sw_submit(void* h, int slot, const int* seeds, int n, uint32_t salt, const hipEvent_t* waits,
                              int nw) {
  auto* w = static_cast<SampleWorker*>(h);
  if (slot < 0 || slot >= (int)w->slots.size()) return -1;
  if (n < 0 || n > w->nd_max[0]) return -2;
  WorkerJob j;
  j.slot = slot;
  j.seeds = seeds;
  j.n = n;
  j.salt = salt;
  j.waits.assign(waits, waits + nw);
  uint64_t seq;
  {
    std::lock_guard<std::mutex> lk(w->m);
    if (!w->th.joinable()) w->th = std::thread([w] { w->run(); });
    seq = j.seq = ++w->submitted;
    w->q.push_back(std::move(j));
  }
  w->cv_job.notify_one();
  return (long)seq;
}

// block until job seq is issued and the sampling of its slot finished; then order the
// consumer stream after it.  Returns 0 or the first error any job hit.
extern "C" int gnn_sw_wait(void* h, long seq, int slot, hipStream_t consumer) {
  auto* w = static_cast<SampleWorker*>(h);
  if (slot < 0 || slot >= (int)w->slots.size()) return -1;
  {
    std::unique_lock<std::mutex> lk(w->m);
    w->cv_done.wait(lk, [&] { return w->issued >= (uint64_t)seq || w->err; });
    if (w->err) return w->err;
  }
  int e = (int)hipEventSynchronize(w->slots[slot].done);
  if (!e && consumer) e = (int)hipStreamWaitEvent(consumer, w->slots[slot].done, 0);
  return e;
}

extern "C" void gnn_sw_destroy(void* h) {
  auto* w = static_cast<SampleWorker*>(h);
  {
    std::lock_guard<std::mutex> lk(w->m);
    w->stop = true;
  }
  w->cv_job.notify_all();
  if (w->th.joinable()) w->th.join();
  (void)hipStreamSynchronize(w->st);
  for (auto& s : w->slots)
    if (s.done) (void)hipEventDestroy(s.done);
  delete w;
}
