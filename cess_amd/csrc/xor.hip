// XOR reduction (the partial-product exchange of a degraded read): the decoder of a
// segment adds, in GF(2^8), the partial rebuilds other GPUs computed from the survivors they hold
// (cec_reconstruct_partial_batch) into its own partial: dst ^= src[0] ^ ... ^ src[nsrc-1].
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

}  // namespace cec
