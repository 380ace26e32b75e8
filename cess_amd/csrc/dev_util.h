// Device helpers shared by the HIP translation units of libcessec (kernels.hip, sha256.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace cec {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint8_t* shard_ptr(const Layout& L, int idx, uint32_t seg) {
  return idx < L.k ? L.data + seg * L.data_seg_stride + (uint64_t)idx * L.shard_stride
                   : L.parity + seg * L.par_seg_stride + (uint64_t)(idx - L.k) * L.shard_stride;
}

// v_bitop3 with truth table 0x96: a ^ b ^ c in one VALU op.
__device__ __forceinline__ uint32_t xor3_u32(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

}  // namespace cec
