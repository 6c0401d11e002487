// Row movement of the halo exchange (parallel/halo.py) for MI355X.
//
// One kernel covers every staging step of a round: gathering the requested rows of
// several column groups into the byte-packed send buffer, unpacking received rows
// into the extended activations, and adding returned gradient rows into the
// owner's rows.  Rows are moved as 4-byte words, consecutive lanes on consecutive
// words of a row (coalesced on both sides), row pitches in bytes, optional row
// index on either side:
//
//   dst[dst_idx ? dst_idx[r] : r][w] (op)= src[src_idx ? src_idx[r] : r][w]
//
//   mode 0: copy 4-byte words              (any dtype; widths are multiples of 4 B)
//   mode 1: fp32 += fp32                   (gradient rows returned on an fp32 wire)
//   mode 2: fp32 += bf16                   (gradient rows returned on a bf16 wire)
//
// The accumulate modes need distinct dst rows within one launch: the caller
// launches once per peer slice (the rows one peer returns are distinct), in peer
// order, so the sums are deterministic without atomics -- replacing ATen's
// sort-based index_put_(accumulate=True), which dominated the emulated papers100M
// epoch (13 % for the kernel alone, plus its sorts and checks).
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(256) void halo_rows_kernel(const uint8_t* __restrict__ src, long src_pitch,
                                                        const long* __restrict__ src_idx, uint8_t* __restrict__ dst,
                                                        long dst_pitch, const long* __restrict__ dst_idx, long rows,
                                                        int words, int mode) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long r = gid / words;
  if (r >= rows) return;
  const int w = (int)(gid - r * words);
  const long sr = src_idx ? src_idx[r] : r;
  const long dr = dst_idx ? dst_idx[r] : r;
  float* __restrict__ d32 = reinterpret_cast<float*>(dst + dr * dst_pitch) + w;
  if (mode == 0) {
    *reinterpret_cast<uint32_t*>(d32) = reinterpret_cast<const uint32_t*>(src + sr * src_pitch)[w];
  } else if (mode == 1) {
    *d32 += reinterpret_cast<const float*>(src + sr * src_pitch)[w];
  } else {
    const uint16_t b = reinterpret_cast<const uint16_t*>(src + sr * src_pitch)[w];
    *d32 += __uint_as_float((uint32_t)b << 16);
  }
}

// words: 4-byte words per row (mode 2: fp32 elements of dst per row)
extern "C" int gnn_launch_halo_rows(const void* src, long src_pitch, const long* src_idx, void* dst, long dst_pitch,
                                    const long* dst_idx, long rows, int words, int mode, hipStream_t st) {
  if (rows <= 0 || words <= 0) return 0;
  if (mode < 0 || mode > 2) return -3;
  const long threads = rows * (long)words;
  hipLaunchKernelGGL(halo_rows_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                     (const uint8_t*)src, src_pitch, src_idx, (uint8_t*)dst, dst_pitch, dst_idx, rows, words, mode);
  return (int)hipGetLastError();
}
