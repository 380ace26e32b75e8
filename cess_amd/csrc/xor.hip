// Byte-stream kernels beside the codec. XOR reduction (the partial-product
// exchange of a degraded read): the decoder of a segment adds, in GF(2^8), the partial rebuilds
// other GPUs computed from the survivors they hold (cec_reconstruct_partial_batch) into its own
// partial: dst ^= src[0] ^ ... ^ src[nsrc-1].
// Addition in GF(2^8) is XOR, so this is the whole combine step; RCCL has no XOR reduction
// (rccl.h ncclRedOp_t), which is why the partials travel point to point and meet here.
//
// One lane owns 16 bytes of dst and walks the sources: read (nsrc + 1) * len, write len, all
// streaming (nontemporal). HBM-bound.
#include "dev_util.h"
#include "kernels.h"

namespace cec {

template <bool V16>
__global__ __launch_bounds__(256) void k_xor_reduce(uint8_t* __restrict__ dst,
                                                    const uint8_t* __restrict__ src, uint32_t nsrc,
                                                    uint64_t stride, uint64_t len) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if constexpr (V16) {
    if (i * 16 >= len) return;
    u32x4 acc = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(dst) + i);
    for (uint32_t j = 0; j < nsrc; ++j)
      acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + j * stride) + i);
    __builtin_nontemporal_store(acc, reinterpret_cast<u32x4*>(dst) + i);
  } else {
    if (i >= len) return;
    uint8_t acc = dst[i];
    for (uint32_t j = 0; j < nsrc; ++j) acc ^= src[j * stride + i];
    dst[i] = acc;
  }
}

void launch_xor_reduce(uint8_t* dst, const uint8_t* src, uint32_t nsrc, uint64_t stride,
                       uint64_t len, hipStream_t st) {
  if (len == 0 || nsrc == 0) return;
  const bool v16 = (((uintptr_t)dst | (uintptr_t)src | stride | len) & 15) == 0;
  const uint64_t per_block = v16 ? 256 * 16 : 256;
  const uint64_t blocks = (len + per_block - 1) / per_block;
  if (v16)
    hipLaunchKernelGGL(k_xor_reduce<true>, dim3((uint32_t)blocks), dim3(256), 0, st, dst, src,
                       nsrc, stride, len);
  else
    hipLaunchKernelGGL(k_xor_reduce<false>, dim3((uint32_t)blocks), dim3(256), 0, st, dst, src,
                       nsrc, stride, len);
}

// Per-segment equality of two [nseg][seg_bytes] device arrays (cec_verify_batch: recomputed
// parity against the stored parity): ok[seg] was set to 1 before; a lane that finds a differing
// 16-byte piece (or byte, unaligned) stores 0 there. Read-only streaming otherwise.
template <bool V16>
__global__ __launch_bounds__(256) void k_cmp_segments(const uint8_t* __restrict__ a,
                                                      const uint8_t* __restrict__ b,
                                                      uint64_t seg_bytes, uint8_t* __restrict__ ok,
                                                      uint32_t seg0) {
  const uint32_t seg = seg0 + blockIdx.y;
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint8_t* pa = a + seg * seg_bytes;
  const uint8_t* pb = b + seg * seg_bytes;
  bool diff;
  if constexpr (V16) {
    if (i * 16 >= seg_bytes) return;
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pa) + i);
    const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pb) + i);
    const u32x4 z = x ^ y;
    diff = (z.x | z.y | z.z | z.w) != 0;
  } else {
    if (i >= seg_bytes) return;
    diff = pa[i] != pb[i];
  }
  if (diff) ok[seg] = 0;
}

void launch_cmp_segments(const uint8_t* a, const uint8_t* b, uint64_t seg_bytes, uint64_t nseg,
                         uint8_t* ok, hipStream_t st) {
  if (seg_bytes == 0 || nseg == 0) return;
  const bool v16 = (((uintptr_t)a | (uintptr_t)b | seg_bytes) & 15) == 0;
  const uint64_t per_block = v16 ? 256 * 16 : 256;
  const uint64_t gx = (seg_bytes + per_block - 1) / per_block;
  for (uint64_t s0 = 0; s0 < nseg; s0 += 65535) {
    const uint32_t ny = (uint32_t)(nseg - s0 < 65535 ? nseg - s0 : 65535);
    if (v16)
      hipLaunchKernelGGL(k_cmp_segments<true>, dim3((uint32_t)gx, ny), dim3(256), 0, st, a, b,
                         seg_bytes, ok, (uint32_t)s0);
    else
      hipLaunchKernelGGL(k_cmp_segments<false>, dim3((uint32_t)gx, ny), dim3(256), 0, st, a, b,
                         seg_bytes, ok, (uint32_t)s0);
  }
}

}  // namespace cec
