// RS(32,32) encode as an additive FFT on bit-sliced data (k_fft), for gfx950.
//
// Why: the matrix form (k_hg) spends ~2,450 VALU ops per 256 bytes moved (~9.6 per byte) on 1,024
// GF multiply-accumulates per byte column, and runs VALU-issue bound. In this code's convention
// (gf256.h: data = f(0..31), parity i = f(32 ^ i) for the unique f of degree < 32) encode is an
// interpolation over the GF(2)-subspace {0..31} and an evaluation over its coset 32 ^ {0..31}:
// the Lin-Chung-Han additive IFFT + FFT, 160 butterflies per byte column instead of 1,024
// products. Each butterfly multiplies by a compile-time skew s. On bit-sliced data (plane q =
// bit q of 32 byte columns) multiplication by s is its 8x8 GF(2) matrix: ~16 XORs per 32 bytes,
// and doubling-style arithmetic costs nothing. Total ~4.6 VALU slots per byte moved, ~2x fewer
// than k_hg, which leaves the kernel bound by HBM.
//
// Layout of the work: a lane pair owns 32 byte columns of one segment. The 32 FFT positions (shard
// indices) are split by their low bit: lane l = threadIdx & 1 holds positions t = 2j + l,
// j = 0..15, as 8 planes each (128 VGPRs). Layers with half-distance >= 2 pair positions of the
// same parity (in-lane); the half-distance-1 layers (first of the IFFT, last of the FFT) pair the
// two lanes and read the partner's planes with DPP quad_perm [1,0,3,2]. Skews depend only on the
// position bits above the layer, so both lanes of a pair use the same compile-time constant.
// Shards are bit-sliced in registers with an 8x8 bit transpose per 32 bytes (swap-moves on
// v_bitop3 selects), and transposed back before the parity stores.
//
// Memory: per shard, each load instruction of a wave's 32 even (odd) lanes reads 512 contiguous
// bytes (see ld32), so every byte moves once and fully coalesced.
//
// Bit-exactness against the matrix form and the oracles: tests/test_gpu_parity.py (golden RS(32,32)
// cases, full BASELINE config-5 geometry vs the C oracle, every kernel variant), and the
// algorithm's own restatement in tests/test_fft_model.py (CPU).
#include "fft_core.h"
#include "kernels.h"

namespace cec {

using namespace fftc;

// RS(32,32) encode, one lane pair per 32 byte columns of a segment (blockIdx.y = segment): a wave's
// 32 pairs cover 1 KiB of columns (pair p: bytes 16p..16p+15 and 512+16p..), so shard_len must be
// a multiple of 1024 with 16-byte aligned shards (checked by the launcher).
// DIAG (tuning build only): 1 = no butterflies (transposes, loads and stores only), 2 = loads and
// stores only, 3 = the same 4 shards at a time (few VGPRs, full occupancy); the outputs are then
// not parity. They measure what the memory side alone costs at
// this access pattern (with LDS > 0 at the kernel's own occupancy of 3 waves per SIMD).
// VER: compare the parity with the stored one instead of writing it (cec_verify_batch: ok[seg]
// = 0 where a byte differs).
template <bool NT, bool NTS, int DIAG, bool VER = false>
__device__ __forceinline__ void fft_cols(const Layout& L, uint32_t seg, uint64_t col,
                                         uint8_t* ok = nullptr) {
  const uint32_t l = threadIdx.x & 1;
  const uint32_t em = l ? 0u : 0xFFFFFFFFu;  // even lane (positions 2j)
  const uint32_t om = ~em;
  const uint8_t* din = L.data + seg * L.data_seg_stride + l * L.shard_stride + col;
  uint8_t* dout = L.parity + seg * L.par_seg_stride + l * L.shard_stride + col;
  const uint64_t step = 2 * L.shard_stride;  // position t -> t + 2

  if constexpr (DIAG == 3) {  // loads and stores only, 4 shards at a time (few VGPRs, 8 waves)
    sfor<4>([&](auto H) CEC_FFT_AI {
      uint32_t Y[4][8];
      sfor<4>([&](auto J) CEC_FFT_AI { ld32<NT>(din + (4 * H + J) * step, Y[J]); });
      sfor<4>([&](auto J) CEC_FFT_AI { st32<NTS>(dout + (4 * H + J) * step, Y[J]); });
    });
    return;
  }
  uint32_t X[16][8];
  sfor<16>([&](auto J) CEC_FFT_AI { ld32<NT>(din + J * step, X[J]); });
  if constexpr (DIAG == 2) {
    sfor<16>([&](auto J) CEC_FFT_AI { st32<NTS>(dout + J * step, X[J]); });
    return;
  }
  sfor<16>([&](auto J) CEC_FFT_AI { tr8(X[J]); });
  if constexpr (DIAG == 1) {
    sfor<16>([&](auto J) CEC_FFT_AI {
      tr8(X[J]);
      st32<NTS>(dout + J * step, X[J]);
    });
    return;
  }

  // encode = IFFT over the data subspace {0..31}, FFT onto the parity coset 32 ^ {0..31}
  ifft32<0>(X, em);
  fft32<32>(X, em, om);

  if constexpr (VER) {
    uint32_t diff = 0;
    sfor<16>([&](auto J) CEC_FFT_AI {
      uint32_t Y[8];
      ld32<NT>(dout + J * step, Y);
      tr8(X[J]);
      sfor<8>([&](auto Q) CEC_FFT_AI { diff |= X[J][Q] ^ Y[Q]; });
    });
    if (diff) ok[seg] = 0;
    return;
  }
  sfor<16>([&](auto J) CEC_FFT_AI {
    tr8(X[J]);
    st32<NTS>(dout + J * step, X[J]);
  });
}

// RS(32,32) verify: the encode's transform, compared with the stored parity (read-only).
__global__ __launch_bounds__(256) void k_fft3232_verify(Layout L, uint8_t* __restrict__ ok,
                                                        uint32_t seg0) {
  const uint32_t seg = seg0 + blockIdx.y;
  const uint64_t gp = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 1;  // lane pair
  const uint64_t col = (gp >> 5) * 1024 + (gp & 31) * 16;
  if (col >= L.len) return;
  fft_cols<true, true, 0, true>(L, seg, col, ok);
}

bool launch_fft_rs3232_verify(const Layout& L, uint8_t* ok, uint32_t nseg, hipStream_t st) {
  const uintptr_t bits = (uintptr_t)L.data | (uintptr_t)L.parity | L.shard_stride |
                         L.data_seg_stride | L.par_seg_stride;
  if ((bits & 15) || (L.len & 1023) || L.len == 0 || L.k != 32) return false;
  const uint64_t gx = (L.len / 32 * 2 + 255) / 256;
  for (uint32_t s0 = 0; s0 < nseg; s0 += 65535) {
    const uint32_t ny = nseg - s0 < 65535 ? nseg - s0 : 65535;
    hipLaunchKernelGGL(k_fft3232_verify, dim3((unsigned)gx, ny), dim3(256), 0, st, L, ok, s0);
  }
  return true;
}

// CPW (tuning build only, else 1): column blocks of 4 KiB per workgroup, walked in a loop, so the
// workgroups resident at once cover fewer segments.
template <bool NT, bool NTS = NT, int DIAG = 0, int CPW = 1>
__global__ __launch_bounds__(256) void k_fft3232(Layout L, const uint32_t* __restrict__ seg_list,
                                                 uint32_t seg0) {
  const uint32_t seg = seg_list ? seg_list[seg0 + blockIdx.y] : seg0 + blockIdx.y;
  if constexpr (CPW == 1) {
    const uint64_t gp = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 1;  // lane pair
    const uint64_t col = (gp >> 5) * 1024 + (gp & 31) * 16;
    if (col >= L.len) return;  // whole waves leave together
    fft_cols<NT, NTS, DIAG>(L, seg, col);
  } else {
    for (int it = 0; it < CPW; ++it) {
      const uint64_t gp = (((uint64_t)blockIdx.x * CPW + it) * 256 + threadIdx.x) >> 1;
      const uint64_t col = (gp >> 5) * 1024 + (gp & 31) * 16;
      if (col >= L.len) return;
      fft_cols<NT, NTS, DIAG>(L, seg, col);
    }
  }
}


bool launch_fft_rs3232(const Layout& L, const uint32_t* seg_list, uint32_t nseg, int nt,
                       hipStream_t st) {
  const uintptr_t bits = (uintptr_t)L.data | (uintptr_t)L.parity | L.shard_stride |
                         L.data_seg_stride | L.par_seg_stride;
  if ((bits & 15) || (L.len & 1023) || L.len == 0 || L.k != 32) return false;
  const uint64_t lanes = L.len / 32 * 2;
  const uint64_t gx = (lanes + 255) / 256;
  [[maybe_unused]] const int cpw = (nt >> 5) & 15;  // tuning build: column blocks per workgroup (0: 1)
  for (uint32_t s0 = 0; s0 < nseg; s0 += 65535) {
    const uint32_t ny = nseg - s0 < 65535 ? nseg - s0 : 65535;
    // nt: bit 0 = nontemporal loads, bit 1 = nontemporal stores; tuning build only: bits 2-3 =
    // DIAG, bit 4 = 48 KiB of LDS per workgroup (caps a CU at 3 workgroups = 3 waves per SIMD)
    switch (nt & 3) {
      case 3:
#ifdef CEC_TUNING
        if (cpw > 1) {
          const unsigned g = (unsigned)((gx + cpw - 1) / cpw);
          if (cpw == 2)
            hipLaunchKernelGGL((k_fft3232<true, true, 0, 2>), dim3(g, ny), dim3(256), 0, st, L,
                               seg_list, s0);
          else if (cpw == 4)
            hipLaunchKernelGGL((k_fft3232<true, true, 0, 4>), dim3(g, ny), dim3(256), 0, st, L,
                               seg_list, s0);
          else
            hipLaunchKernelGGL((k_fft3232<true, true, 0, 8>), dim3(g, ny), dim3(256), 0, st, L,
                               seg_list, s0);
          break;
        }
        if (nt & 12) {
          const unsigned lds = (nt & 16) ? 48 * 1024 : 0;
          if ((nt & 12) == 4)
            hipLaunchKernelGGL((k_fft3232<true, true, 1>), dim3((unsigned)gx, ny), dim3(256), lds,
                               st, L, seg_list, s0);
          else if ((nt & 12) == 12)
            hipLaunchKernelGGL((k_fft3232<true, true, 3>), dim3((unsigned)gx, ny), dim3(256), lds,
                               st, L, seg_list, s0);
          else
            hipLaunchKernelGGL((k_fft3232<true, true, 2>), dim3((unsigned)gx, ny), dim3(256), lds,
                               st, L, seg_list, s0);
          break;
        }
#endif
        hipLaunchKernelGGL((k_fft3232<true, true>), dim3((unsigned)gx, ny), dim3(256), 0, st, L,
                           seg_list, s0);
        break;
#ifdef CEC_TUNING
      case 1:
        hipLaunchKernelGGL((k_fft3232<true, false>), dim3((unsigned)gx, ny), dim3(256), 0, st, L,
                           seg_list, s0);
        break;
      case 2:
        hipLaunchKernelGGL((k_fft3232<false, true>), dim3((unsigned)gx, ny), dim3(256), 0, st, L,
                           seg_list, s0);
        break;
#endif
      default:
        hipLaunchKernelGGL((k_fft3232<false, false>), dim3((unsigned)gx, ny), dim3(256), 0, st, L,
                           seg_list, s0);
    }
  }
  return true;
}

}  // namespace cec
