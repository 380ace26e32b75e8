// Audit chunk gather: the chunks a storage challenge names, copied out of
// every fragment of an HBM-resident batch so they can be hashed and proven.
//
// Reference: a fragment is CHUNK_COUNT = 1024 chunks (primitives/common/src/lib.rs:62), i.e.
// 8 KiB chunks of an 8 MiB fragment; a challenge names CHUNK_COUNT * 46 / 1000 = 47 distinct
// chunk indices (c-pallets/audit/src/lib.rs:955-964, NetSnapShot.random_index_list,
// types.rs:21). The PoDR2 tag arithmetic over those chunks runs in the TEE and is not in the
// reference; this is the byte-exact part: addressing and gathering.
//
// One lane moves 16 bytes; blockIdx.x walks (index, tile of the chunk), blockIdx.y the fragment.
// Pure HBM streaming: read + write nfrag * nidx * chunk_len bytes.
#include "dev_util.h"
#include "kernels.h"

namespace cec {

template <bool V16>
__global__ __launch_bounds__(256) void k_chunk_gather(Layout L, int nshards,
                                                      const uint32_t* __restrict__ idx,
                                                      uint32_t nidx, uint64_t chunk_len,
                                                      uint32_t tiles, uint32_t frag0,
                                                      uint8_t* __restrict__ out) {
  const uint32_t j = blockIdx.x / tiles, tile = blockIdx.x - j * tiles;
  const uint32_t frag = frag0 + blockIdx.y;
  const uint32_t seg = frag / nshards, sh = frag - seg * nshards;
  const uint8_t* src = shard_ptr(L, (int)sh, seg) + (uint64_t)idx[j] * chunk_len;
  uint8_t* dst = out + ((uint64_t)frag * nidx + j) * chunk_len;
  if constexpr (V16) {
    const uint64_t v = (uint64_t)tile * 256 + threadIdx.x;
    if (v * 16 < chunk_len)
      __builtin_nontemporal_store(
          __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + v),
          reinterpret_cast<u32x4*>(dst) + v);
  } else {
    const uint64_t b = (uint64_t)tile * 256 + threadIdx.x;
    if (b < chunk_len) dst[b] = src[b];
  }
}

void launch_chunk_gather(const Layout& L, int nshards, uint64_t nfrag, const uint32_t* d_idx,
                         uint32_t nidx, uint64_t chunk_len, uint8_t* out, hipStream_t st) {
  if (nfrag == 0 || nidx == 0 || chunk_len == 0) return;
  const uintptr_t bits = (uintptr_t)L.data | (uintptr_t)L.parity | L.shard_stride |
                         L.data_seg_stride | L.par_seg_stride | chunk_len | (uintptr_t)out;
  const bool v16 = (bits & 15) == 0;
  const uint64_t per_tile = v16 ? 256 * 16 : 256;
  const uint32_t tiles = (uint32_t)((chunk_len + per_tile - 1) / per_tile);
  for (uint64_t f0 = 0; f0 < nfrag; f0 += 65535) {
    const uint32_t ny = (uint32_t)(nfrag - f0 < 65535 ? nfrag - f0 : 65535);
    if (v16)
      hipLaunchKernelGGL(k_chunk_gather<true>, dim3(tiles * nidx, ny), dim3(256), 0, st, L,
                         nshards, d_idx, nidx, chunk_len, tiles, (uint32_t)f0, out);
    else
      hipLaunchKernelGGL(k_chunk_gather<false>, dim3(tiles * nidx, ny), dim3(256), 0, st, L,
                         nshards, d_idx, nidx, chunk_len, tiles, (uint32_t)f0, out);
  }
}

}  // namespace cec
