// RS(32,32) erasure decode by the formal derivative (k_fftdec_d), gfx950: the rebuild whose cost
// does not grow with the number of lost fragments. A miner exit marks every fragment the miner held
// (c-pallets/file-bank/src/functions.rs:543-562), so a wide-coded segment can lose up to 32 of its
// 64 fragments at once; the syndrome decoder (fftdec.hip) pays per (output, syndrome slot) and the
// run-time matrix kernels per (output, input), while this one pays two 64-point transforms.
//
// Algorithm (plan: fftdec_plan_d in fftdec_plan.h). Points are shard indices 0..63, the GF(2)-span
// of {1, 2, .., 32}; lam(x) = prod_{e erased} (x ^ e):
//   X_t  = lam(t) c_t          (present shards; erased ones read as zeros)
//   g    = IFFT_64(X)          (Lin-Chung-Han, novel polynomial basis, coset 0)
//   g'   = D(g)                (formal derivative: D(Xhat_i) = sum_{bit j of i} c_j Xhat_{i - 2^j},
//                               c_j = W_j'(0) / W_j(2^j), compile-time)
//   c_e  = FFT_64(g')(e) / lam'(e)
//
// Layout: a quad of lanes (l = lane & 3) owns 32 byte columns of a segment; lane l holds positions
// t = 4j + l, j = 0..15, as 8 bit planes each (128 VGPRs), so each skew of layers 1..5 depends only
// on j (lane-uniform, compile-time). Layer 0's skew What_0(t & ~1) = t & ~1 has the lane's bit 1 in
// it: the uniform part 4j plus 2 on lanes 2 and 3 (one masked doubling). Layers 0 and 1 pair lanes
// through DPP quad_perm, layers 2..5 registers of one lane. A lane's 32 bytes of a shard are two
// 16-byte pieces 256 bytes apart: each load or store of a wave's 16 lanes with the same l covers 256
// contiguous bytes of one shard. The run-time multiplications by lam(t) and 1 / lam'(e) differ per
// lane (position): Horner over the coefficient bits, the lane's eight 0 / ~0 bit masks read from
// LDS (the plan carries them expanded; -DCEC_FDD_BFE makes them with v_bfe_i32 instead, 0.11 ms
// slower at 32 erasures).
#include <algorithm>
#include <utility>

#include "fft_core.h"
#include "fftdec_plan.h"
#include "kernels.h"

// Three waves per SIMD (<= 168 VGPRs, no scratch): measured 0.82 ms against 0.91 at the
// compiler's own two for 32 random erasures of 64 x 512 KiB segments (profiles/r03/fdd_libs_ab1.jsonl).
// -DCEC_FDD_WAVES=n for occupancy experiments.
#ifndef CEC_FDD_WAVES
#define CEC_FDD_WAVES 3
#endif
#define CEC_FDD_ATTR __attribute__((amdgpu_waves_per_eu(CEC_FDD_WAVES, CEC_FDD_WAVES)))

namespace cec {

using namespace fftc;

namespace {

typedef const __attribute__((address_space(4))) uint32_t* cplan_t;

// Loads and stores that a lane may skip go through a raw buffer resource: an out-of-range offset
// reads zeros / drops the write without touching memory. Offsets are 32-bit: a coset's 32 shards
// must span < 2 GiB (fftdec_layout_ok).
constexpr uint32_t kOff = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, 0x7FFFFFFF,
                                           0x00020000);
}
constexpr uint32_t kPiece = 256;  // distance of a lane's two 16-byte pieces
__device__ __forceinline__ void bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                    uint32_t (&w)[8]) {
  const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 2);  // nt
  const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, voff + kPiece, soff, 2);
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                    const uint32_t (&w)[8]) {
  const u32x4 a = {w[0], w[1], w[2], w[3]}, b = {w[4], w[5], w[6], w[7]};
  __builtin_amdgcn_raw_buffer_store_b128(a, r, voff, soff, 2);
  __builtin_amdgcn_raw_buffer_store_b128(b, r, voff + kPiece, soff, 2);
}

// every plane of a slot materialised here (an empty asm that reads and writes them): phases and
// slots start from complete registers, so the scheduler cannot interleave them into more live values
__device__ __forceinline__ void fence(uint32_t (&x)[8]) {
  asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
               "+v"(x[6]), "+v"(x[7]));
}
__device__ __forceinline__ void fence_all(uint32_t (&X)[16][8]) {
  sfor<16>([&](auto J) CEC_FFT_AI { fence(X[J]); });
}
// slot J's work starts once slot J - 1's last plane is written
template <int J>
__device__ __forceinline__ void after_prev(uint32_t (&X)[16][8]) {
  if constexpr (J > 0) asm volatile("" : "+v"(X[J][0]) : "v"(X[J - 1][7]));
}

// quad partners: lane l reads lane l ^ 1 / l ^ 2. SWZ = false: DPP quad_perm, folded by the
// compiler into the consuming v_and / v_xor where it can; every DPP form (v_mov_b32_dpp and the
// VOP2 ops with a DPP operand alike) issues at half rate on gfx950 (profiles/r04/
// valu_bench_r04.jsonl), so the 768 exchanges per block are ~1,500 issue slots. SWZ = true:
// ds_swizzle in quad-permute mode through the LDS crossbar, no VALU slot, LDS latency instead
// (tuning forms; k_fftdec_d's kFddSwz).
template <bool SWZ>
__device__ __forceinline__ uint32_t qp1(uint32_t v) {
  if constexpr (SWZ) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x80B1);
  else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);  // [1,0,3,2]
}
template <bool SWZ>
__device__ __forceinline__ uint32_t qp2(uint32_t v) {
  if constexpr (SWZ) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x804E);
  else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, true);  // [2,3,0,1]
}

struct Skews64 {
  static constexpr LchSkews<6> s = lch_skews<6>(0);
};

template <int J>
struct DConst {
  static constexpr unsigned v = lch_dconst(J);
};
static_assert(lch_dconst(0) == 1, "c_0 = 1: the b = 0 term of the derivative is a plain XOR");

// What_0 is linear: the skew of layer 0 on lanes 2, 3 is the uniform one ^ What_0(2) = ^ 2
static_assert(lch_what(0, 2) == 2, "layer-0 skew delta of the quad's upper pair");

constexpr int kXandN = 0xB4;  // a ^ (b & ~c)

// x ^= ~m & 2z (planes: 2z = z << 1 with 0x11D's taps 2, 3, 4 fed by plane 7); m = e2, so the
// doubling lands on lanes 2 and 3
__device__ __forceinline__ void xtime_acc_masked(uint32_t (&x)[8], const uint32_t (&z)[8],
                                                 uint32_t m) {
  x[0] = FFT_BOP3(x[0], z[7], m, kXandN);
  x[1] = FFT_BOP3(x[1], z[0], m, kXandN);
  x[2] = FFT_BOP3(x[2], z[1] ^ z[7], m, kXandN);
  x[3] = FFT_BOP3(x[3], z[2] ^ z[7], m, kXandN);
  x[4] = FFT_BOP3(x[4], z[3] ^ z[7], m, kXandN);
  x[5] = FFT_BOP3(x[5], z[4], m, kXandN);
  x[6] = FFT_BOP3(x[6], z[5], m, kXandN);
  x[7] = FFT_BOP3(x[7], z[6], m, kXandN);
}

// x = c * x for a per-lane constant c (bits 0..7 of cv): Horner over c's bits, each bit's mask
// (0 or ~0) from one v_bfe_i32
__device__ __forceinline__ void mul_rt(uint32_t (&x)[8], uint32_t cv) {
  uint32_t z[8], acc[8];
  sfor<8>([&](auto Q) CEC_FFT_AI { z[Q] = x[Q]; });
  {
    const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)cv, 7, 1);
    sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = z[Q] & m; });
  }
  sfor<7>([&](auto B) CEC_FFT_AI {
    constexpr int b = 6 - B;
    const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)cv, b, 1);
    const uint32_t a7 = acc[7];
    sfor<7>([&](auto Q) CEC_FFT_AI { acc[7 - Q] = acc[6 - Q]; });
    acc[0] = a7;
    acc[2] ^= a7;
    acc[3] ^= a7;
    acc[4] ^= a7;
    sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = FFT_BOP3(acc[Q], z[Q], m, kXand); });
  });
  sfor<8>([&](auto Q) CEC_FFT_AI { x[Q] = acc[Q]; });
}

// The same with the 8 masks read from LDS (the plan's expanded masks of this lane and slot:
// two 16-byte LDS reads instead of eight half-rate v_bfe_i32)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef const __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4w;
__device__ __forceinline__ void mul_rt_lds(uint32_t (&x)[8], const lds_u32* mk) {
  const u32x4 lo = *reinterpret_cast<lds_u32x4*>(mk), hi = *reinterpret_cast<lds_u32x4*>(mk + 4);
  const uint32_t m[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  uint32_t z[8], acc[8];
  sfor<8>([&](auto Q) CEC_FFT_AI { z[Q] = x[Q]; });
  sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = z[Q] & m[7]; });
  sfor<7>([&](auto B) CEC_FFT_AI {
    constexpr int b = 6 - B;
    const uint32_t a7 = acc[7];
    sfor<7>([&](auto Q) CEC_FFT_AI { acc[7 - Q] = acc[6 - Q]; });
    acc[0] = a7;
    acc[2] ^= a7;
    acc[3] ^= a7;
    acc[4] ^= a7;
    sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = FFT_BOP3(acc[Q], z[Q], m[b], kXand); });
  });
  sfor<8>([&](auto Q) CEC_FFT_AI { x[Q] = acc[Q]; });
}

// IFFT_64 (values -> coefficients), layer i: b ^= a; a ^= s*b. e1 / e2: lanes with bit 0 / bit 1
// of l clear (the lower position of a layer-0 / layer-1 pair).
template <bool SWZ>
__device__ __forceinline__ void ifft64(uint32_t (&X)[16][8], uint32_t e1, uint32_t e2) {
  using S = Skews64;
  // layer 0 (lanes l, l ^ 1). Z = a ^ b on both lanes; lower -> a ^ s*Z, upper -> Z
  sfor<16>([&](auto J) CEC_FFT_AI {
    constexpr unsigned s = S::s.s[0][2 * J];
    static_assert(S::s.s[0][2 * J + 1] == (s ^ 2u), "layer-0 skew is linear in t");
    after_prev<J>(X);
    uint32_t Z[8];
    sfor<8>([&](auto Q) CEC_FFT_AI { Z[Q] = X[J][Q] ^ qp1<SWZ>(X[J][Q]); });
    if constexpr (s == 0) {
      sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] ^= Z[Q]; });
    } else {
      mul_acc<s, true>(X[J], Z, Z);  // X ^ Z ^ s*Z
    }
    xtime_acc_masked(X[J], Z, e2);  // lanes 2, 3: the skew's extra 2
    sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] = FFT_BOP3(Z[Q], e1, X[J][Q], kXand); });
  });
  // layer 1 (lanes l, l ^ 2): skew What_1(4j), uniform
  sfor<16>([&](auto J) CEC_FFT_AI {
    constexpr unsigned s = S::s.s[1][J];
    after_prev<J>(X);
    uint32_t Z[8];
    sfor<8>([&](auto Q) CEC_FFT_AI { Z[Q] = X[J][Q] ^ qp2<SWZ>(X[J][Q]); });
    if constexpr (s == 0) {
      sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] = FFT_BOP3(e2, X[J][Q], Z[Q], kSel); });
    } else {
      mul_acc<s, true>(X[J], Z, Z);
      sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] = FFT_BOP3(Z[Q], e2, X[J][Q], kXand); });
    }
  });
  // layers 2..5 (in-lane: registers j and j + 2^(i-2)); block of position 4j: j >> (i - 1)
  sfor<4>([&](auto I2) CEC_FFT_AI {
    constexpr int i = I2 + 2, hj = 1 << (i - 2);
    sfor<16>([&](auto J) CEC_FFT_AI {
      if constexpr (!(J & hj)) {
        constexpr unsigned s = S::s.s[i][J >> (i - 1)];
        sfor<8>([&](auto Q) CEC_FFT_AI { X[J + hj][Q] = x2(X[J + hj][Q], X[J][Q]); });
        if constexpr (s != 0) mul_acc<s, false>(X[J], X[J + hj], X[J]);
      }
    });
  });
}

// FFT_64 (coefficients -> values), layer i: a ^= s*b; b ^= a (i = 5 .. 0). Layers 5..2 here;
// layers 1 and 0 pair the lanes of a quad on one register slot (fft64_tail), so the kernel runs
// them only for the slots that hold an output.
__device__ __forceinline__ void fft64_upper(uint32_t (&X)[16][8]) {
  using S = Skews64;
  sfor<4>([&](auto I2) CEC_FFT_AI {
    constexpr int i = 5 - I2, hj = 1 << (i - 2);
    sfor<16>([&](auto J) CEC_FFT_AI {
      if constexpr (!(J & hj)) {
        constexpr unsigned s = S::s.s[i][J >> (i - 1)];
        if constexpr (s != 0) mul_acc<s, false>(X[J], X[J + hj], X[J]);
        sfor<8>([&](auto Q) CEC_FFT_AI { X[J + hj][Q] = x2(X[J + hj][Q], X[J][Q]); });
      }
    });
  });
}
template <int J, bool SWZ>
__device__ __forceinline__ void fft64_tail(uint32_t (&x)[8], uint32_t e1, uint32_t e2) {
  using S = Skews64;
  {  // layer 1 (lanes l, l ^ 2). P = b on both lanes: lower -> a ^ s*P, upper -> b ^ a ^ s*P
    constexpr unsigned s = S::s.s[1][J];
    uint32_t P[8];
    sfor<8>([&](auto Q) CEC_FFT_AI {
      const uint32_t y = qp2<SWZ>(x[Q]);
      P[Q] = FFT_BOP3(e2, y, x[Q], kSel);
      x[Q] = FFT_BOP3(x[Q], y, e2, kXandN);
    });
    if constexpr (s != 0) mul_acc<s, false>(x, P, P);
  }
  {  // layer 0 (lanes l, l ^ 1), skew uniform part plus 2 on lanes 2, 3
    constexpr unsigned s = S::s.s[0][2 * J];
    uint32_t P[8];
    sfor<8>([&](auto Q) CEC_FFT_AI {
      const uint32_t y = qp1<SWZ>(x[Q]);
      P[Q] = FFT_BOP3(e1, y, x[Q], kSel);
      x[Q] = FFT_BOP3(x[Q], y, e1, kXandN);
    });
    if constexpr (s != 0) mul_acc<s, false>(x, P, P);
    xtime_acc_masked(x, P, e2);
  }
}

// g'[t] = XOR over the bits b not set in t of c_b g[t + 2^b], in place in ascending j (every
// term reads a higher register, or this register of another lane, before it is overwritten)
template <bool SWZ>
__device__ __forceinline__ void derivative(uint32_t (&X)[16][8], uint32_t e1, uint32_t e2) {
  sfor<16>([&](auto J) CEC_FFT_AI {
    after_prev<J>(X);
    uint32_t acc[8], z[8];
    sfor<8>([&](auto Q) CEC_FFT_AI {
      acc[Q] = qp1<SWZ>(X[J][Q]) & e1;  // b = 0: c_0 = 1, partner t + 1 on lanes with bit 0 clear
      z[Q] = qp2<SWZ>(X[J][Q]) & e2;    // b = 1: t + 2 on lanes with bit 1 clear
    });
    mul_acc<DConst<1>::v, false>(acc, z, z);
    sfor<4>([&](auto B) CEC_FFT_AI {  // b = B + 2: register j + 2^B
      if constexpr (!((J >> B) & 1)) mul_acc<DConst<B + 2>::v, false>(acc, X[J + (1 << B)], acc);
    });
    sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] = acc[Q]; });
  });
}

// A lane's place in its quad and its byte offsets, from an opaque lane id (asm volatile: the
// kernel derives them again after the transforms instead of keeping them live through them)
struct LaneCtx {
  uint32_t l, lcol, sh, e1, e2;
};
__device__ __forceinline__ LaneCtx lane_ctx(uint32_t wave_col, uint32_t ss) {
  uint32_t lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  LaneCtx c;
  c.l = lane & 3;
  c.lcol = wave_col + (lane >> 2) * 16 + c.l * ss;  // byte offset of position 4j + l
  c.sh = 8 * c.l;
  c.e1 = (c.l & 1) ? 0u : 0xFFFFFFFFu;
  c.e2 = (c.l & 2) ? 0u : 0xFFFFFFFFu;
  return c;
}

// SWZ: which phases exchange through the LDS crossbar (bit 0 the IFFT's layers 0, 1, bit 1 the
// derivative, bit 2 the FFT's layers 1, 0), the others through DPP. The product's: DPP everywhere
// (kFddSwz = 0). The crossbar in the IFFT and the derivative looked 4.4 % faster in an in-process
// A/B that alternates the forms launch by launch, but one form per process, as the line and a real
// rebuild run it, the two are equal within 1 % (profiles/r04/swz_standalone_runs.jsonl).
constexpr int kFddSwz = 0;
// SKIP: a slot none of whose four positions is read (all erased or unused: its loads returned
// zeros) skips its transpose and its multiplication by lam (zero in, zero out); a uniform branch
template <int SWZ, bool SKIP = true>
__global__ __launch_bounds__(256) CEC_FDD_ATTR void k_fftdec_d(Layout L, const uint32_t* __restrict__ plan1,
                                                  const uint32_t* const* __restrict__ plans,
                                                  const uint32_t* __restrict__ seg_list,
                                                  uint32_t seg0) {
  const uint32_t y = seg0 + blockIdx.y;
  const uint32_t seg = seg_list ? seg_list[y] : y;
  const uint32_t* Pg = plans ? plans[y] : plan1;
  const cplan_t P = (cplan_t)Pg;
#ifndef CEC_FDD_BFE
  // the plan's per-lane masks into LDS (4 KiB: 16 bytes per thread), before any wave leaves
  static_assert(FftDecDLayout::kMerged - FftDecDLayout::kMasks == 4 * 256 &&
                    FftDecDLayout::kMasks % 4 == 0,
                "one 16-byte piece of the mask table per thread of the 256-thread workgroup");
  __shared__ __attribute__((aligned(16))) uint32_t lmask[2 * 16 * 4 * 8];
  *reinterpret_cast<u32x4*>(lmask + 4 * threadIdx.x) =
      *reinterpret_cast<const u32x4*>(Pg + FftDecDLayout::kMasks + 4 * threadIdx.x);
  __syncthreads();
#endif
  // a wave owns 512 byte columns: 16 quads of 32 (two 16-byte pieces 256 bytes apart per lane)
  const uint32_t wave_col =
      (blockIdx.x * 4 + (__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6)) * 512;
  if (wave_col >= L.len) return;  // whole waves leave together (len % 512 == 0)
  const uint32_t ss = (uint32_t)L.shard_stride;
  const auto rD = rsrc(L.data + seg * L.data_seg_stride);
  const auto rP = rsrc(L.parity + seg * L.par_seg_stride);
  const LaneCtx c0 = lane_ctx(wave_col, ss);
  const uint32_t l = c0.l, lcol = c0.lcol, sh = c0.sh, e1 = c0.e1, e2 = c0.e2;

  uint32_t X[16][8];
  // present shards, each times lam(t) (an erased shard loads as zeros: lam(t) = 0 there)
  sfor<16>([&](auto J) CEC_FFT_AI {
    const uint32_t lw = P[FftDecDLayout::kLam + J];
    const uint32_t voff = ((lw >> sh) & 0xFF) ? lcol : kOff;
    bld(J < 8 ? rD : rP, voff, (uint32_t)(4 * (J & 7)) * ss, X[J]);
  });
  sfor<16>([&](auto J) CEC_FFT_AI {
    after_prev<J>(X);
    if (!SKIP || P[FftDecDLayout::kLam + J]) {
      tr8(X[J]);
#ifdef CEC_FDD_BFE
      mul_rt(X[J], P[FftDecDLayout::kLam + J] >> sh);
#else
      mul_rt_lds(X[J], (const lds_u32*)lmask + (J * 4 + l) * 8);
#endif
    }
  });
  fence_all(X);
  ifft64<(SWZ & 1) != 0>(X, e1, e2);
  fence_all(X);
  derivative<(SWZ & 2) != 0>(X, e1, e2);
  fence_all(X);
  fft64_upper(X);
  fence_all(X);
  const LaneCtx c1 = lane_ctx(wave_col, ss);
  // slots holding an output: the last two FFT layers, times 1 / lam'(e), back to bytes, stored
  // by the lanes whose position is an output
  sfor<16>([&](auto J) CEC_FFT_AI {
    const uint32_t dw = P[FftDecDLayout::kDinv + J];
    after_prev<J>(X);
    if (dw) {
      fft64_tail<J, (SWZ & 4) != 0>(X[J], c1.e1, c1.e2);
#ifdef CEC_FDD_BFE
      mul_rt(X[J], dw >> c1.sh);
#else
      mul_rt_lds(X[J], (const lds_u32*)lmask + ((16 + J) * 4 + c1.l) * 8);
#endif
      tr8(X[J]);
      const uint32_t voff = ((dw >> c1.sh) & 0xFF) ? c1.lcol : kOff;
      bst(J < 8 ? rD : rP, voff, (uint32_t)(4 * (J & 7)) * ss, X[J]);
    }
  });
}

#ifdef CEC_TUNING
// ---- the pipelined form (k_fftdec_dp) ----------------------------------------------------------
// Every position needs exactly one run-time multiplication: lam(t) where it is read, 1 / lam'(t)
// where it is an output. k_fftdec_d runs both per slot (a SIMD executes both sides of a lane-
// dependent choice), ~2,700 of its ~9,300 VALU per wave. Here a wave walks a run of consecutive
// 512-column blocks of one segment (one pattern): the output step of block u and the input step of
// block u + 1 share one multiplication per slot, with the merged constant of each position (the
// plan's kMerged masks: a position is never both read and an output). The operand is the next
// block's loaded input on read lanes and this block's FFT output elsewhere; the product goes back to
// the registers as the next block's input (zero on unread lanes) and to memory as this block's
// output (stored by output lanes only). The grid is the chip's resident waves (persistent), G of
// them per segment; wave i of a segment walks its blocks i, i + G, ... (one plan, no segment
// crossings).

// wave-private LDS: the merged-constant masks of the wave's current segment (2 KiB)
constexpr int kMergedWords = 16 * 4 * 8;

// The lane's 32 bytes of shard slot J (positions 4J + l) at column offset `col` of the segment
__device__ __forceinline__ void dp_load(__amdgpu_buffer_rsrc_t rD, __amdgpu_buffer_rsrc_t rP,
                                        int J, uint32_t col, uint32_t ss, bool rd,
                                        uint32_t (&w)[8]) {
  bld(J < 8 ? rD : rP, rd ? col : kOff, (uint32_t)(4 * (J & 7)) * ss, w);
}

template <int J>
__device__ __forceinline__ uint32_t dp_rdmask(cplan_t P, uint32_t sh) {
  return ((P[FftDecDLayout::kLam + J] >> sh) & 0xFF) ? 0xFFFFFFFFu : 0u;
}

__global__ __launch_bounds__(256) CEC_FDD_ATTR void k_fftdec_dp(
    Layout L, const uint32_t* __restrict__ plan1, const uint32_t* const* __restrict__ plans,
    const uint32_t* __restrict__ seg_list, uint32_t nblk, uint32_t nseg, uint32_t G,
    uint32_t prio) {
  __shared__ __attribute__((aligned(16))) uint32_t lmask_all[4][kMergedWords];
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
  // G waves per segment; wave i of a segment takes its blocks i, i + G, i + 2G, ...: the waves of
  // a workgroup (and their neighbours) read neighbouring 512-column blocks of the same shards at
  // any time, as the one-block-per-wave grid does (blocks of a run G apart, one plan)
  const uint32_t wave = blockIdx.x * 4 + wid;
  if (wave >= nseg * G) return;
  lds_u32* lmask = (lds_u32*)lmask_all[wid];
  const uint32_t ss = (uint32_t)L.shard_stride;

  uint32_t X[16][8];
  // loop state kept scalar (32-bit, wave-uniform): (segment list index, block) of the unit,
  // stepped along the run, the units left and whether the next one starts a segment afresh (no
  // division or 64-bit compare inside the loop: that is VALU work with every X register live)
  // (the divisions are VALU work: their results go back to scalars, or the plan pointer and
  // every plan word would be vector loads)
  const uint32_t y = (uint32_t)__builtin_amdgcn_readfirstlane(wave / G);
  uint32_t blk = (uint32_t)__builtin_amdgcn_readfirstlane(wave - y * G);
  uint32_t left = (uint32_t)__builtin_amdgcn_readfirstlane((nblk - blk + G - 1) / G);
  uint32_t fresh = 1;
  const uint32_t total = left;
  for (; left; --left) {
    // prio: the SIMD's arbiter favours older waves: in a long-lived (persistent) grid the oldest
    // wave of a SIMD races ahead and the youngest is left to finish alone at one wave per SIMD. A
    // wave's priority then follows the share of its run still ahead of it (lagging waves catch up).
    if (prio) {
      const uint32_t q = left * 4 / (total + 1);  // 0..3
      if (q >= 3) __builtin_amdgcn_s_setprio(3);
      else if (q == 2) __builtin_amdgcn_s_setprio(2);
      else if (q == 1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    const uint32_t seg = seg_list ? seg_list[y] : y;
    const uint32_t* Pg = plans ? plans[y] : plan1;
    {  // wave-uniform: keep the pointer (and the choice above) scalar
      const uint64_t pv = (uint64_t)Pg;
      // (readfirstlane returns int: each half goes through uint32_t, or the low half would be
      // sign-extended into the high one)
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(pv >> 32));
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)pv);
      Pg = (const uint32_t*)((uint64_t)hi << 32 | lo);
    }
    const cplan_t P = (cplan_t)Pg;
    const auto rD = rsrc(L.data + seg * L.data_seg_stride);
    const auto rP = rsrc(L.parity + seg * L.par_seg_stride);
    const uint32_t wave_col = blk * 512;
    if (fresh) {
      // this segment's merged masks (32 bytes per lane), then the block's whole input step
      {
        uint32_t lane;  // opaque: derived here, not kept live through the loop
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        // a buffer resource on the (uniform) plan: 32-bit lane offsets, no 64-bit VGPR addresses
        const auto rT = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t*>(Pg + FftDecDLayout::kMerged), (short)0, kMergedWords * 4,
            0x00020000);
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rT, 32 * lane, 0, 0);
        const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rT, 32 * lane + 16, 0, 0);
        // the previous segment's reads of the table are complete (in order within the wave)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        *reinterpret_cast<lds_u32x4w*>(lmask + 8 * lane) = a;
        *reinterpret_cast<lds_u32x4w*>(lmask + 8 * lane + 4) = b;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      const LaneCtx c0 = lane_ctx(wave_col, ss);
      sfor<16>([&](auto J) CEC_FFT_AI {
        dp_load(rD, rP, J, c0.lcol, ss, (P[FftDecDLayout::kLam + J] >> c0.sh) & 0xFF, X[J]);
      });
      sfor<16>([&](auto J) CEC_FFT_AI {
        after_prev<J>(X);
        tr8(X[J]);
        mul_rt_lds(X[J], lmask + (J * 4 + c0.l) * 8);  // unread lanes hold zeros
      });
      fresh = 0;
    }
    fence_all(X);
    ifft64<false>(X, lane_ctx(0, 0).e1, lane_ctx(0, 0).e2);
    fence_all(X);
    {
      const LaneCtx c = lane_ctx(0, 0);
      derivative<false>(X, c.e1, c.e2);
    }
    fence_all(X);
    fft64_upper(X);
    fence_all(X);
    // the next unit continues this segment: its input step rides on this block's output step.
    // Branch-free per slot (uniform branches here cost registers across the unrolled slots):
    // without a next block the loads are all out of range (no memory traffic) and rd = 0; lanes
    // that are not outputs store out of range.
    const uint32_t next = left > 1 ? 1u : 0u;
    const uint32_t nx = next ? 0xFFFFFFFFu : 0u;
    const LaneCtx c1 = lane_ctx(wave_col, ss);
    const uint32_t ncol = c1.lcol + 512 * G;  // the same lane's columns in the next block
    sfor<16>([&](auto J) CEC_FFT_AI {
      const uint32_t dw = P[FftDecDLayout::kDinv + J];
      after_prev<J>(X);
      uint32_t pre[8];
      {
        uint32_t col = ncol;  // the load is issued in its slot, not hoisted into earlier slots
        if constexpr (J > 0) asm volatile("" : "+v"(col) : "v"(X[J - 1][7]));
        dp_load(rD, rP, J, col, ss, dp_rdmask<J>(P, c1.sh) & nx, pre);
      }
      fft64_tail<J, false>(X[J], c1.e1, c1.e2);
      const uint32_t rd = dp_rdmask<J>(P, c1.sh) & nx;
      tr8(pre);
      sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] = FFT_BOP3(rd, pre[Q], X[J][Q], kSel); });
      mul_rt_lds(X[J], lmask + (J * 4 + c1.l) * 8);
      uint32_t O[8];
      sfor<8>([&](auto Q) CEC_FFT_AI {
        O[Q] = X[J][Q];
        X[J][Q] &= rd;  // next input: zero where unread
      });
      tr8(O);
      bst(J < 8 ? rD : rP, ((dw >> c1.sh) & 0xFF) ? c1.lcol : kOff, (uint32_t)(4 * (J & 7)) * ss, O);
      // the next slot starts once this slot's stored planes exist (the scheduler would otherwise
      // overlap two slots' temporaries)
      if constexpr (J + 1 < 16)
        asm volatile("" : "+v"(X[J + 1][0]), "+v"(X[J + 1][1]), "+v"(X[J + 1][2]), "+v"(X[J + 1][3])
                     : "v"(O[3]), "v"(O[7]));
    });
    fresh = next ^ 1u;
    blk += G;
  }
}

// Resident workgroups of k_fftdec_dp on the device (the persistent grid), cached per device.
uint32_t fdd_resident_wgs() {
  static uint32_t cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1024;
  if (!cache[dev]) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_fftdec_dp, 256, 0) !=
            hipSuccess ||
        cus <= 0 || per <= 0)
      return 1024;
    cache[dev] = (uint32_t)(cus * per);
  }
  return cache[dev];
}

#endif  // CEC_TUNING

}  // namespace

bool launch_fftdec_d(const Layout& L, const uint32_t* plan1, const uint32_t* const* plans,
                     const uint32_t* seg_list, uint32_t nseg, hipStream_t st, int form) {
  if (!fftdec_layout_ok(L)) return false;
  if (nseg == 0) return true;
#ifdef CEC_TUNING
  if (form == 1 || form == 3) {
    // the pipelined form: G waves per segment, the resident waves spread over the segments (at
    // least one each; more segments than resident waves: one wave per segment, in rounds)
    const uint32_t nblk = (uint32_t)(L.len / 512);
    const uint64_t waves = 4ull * fdd_resident_wgs();
    const uint32_t G = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nblk, waves / nseg));
    const uint64_t wgs = ((uint64_t)nseg * G + 3) / 4;
    if (wgs > 0x7FFFFFFFull) return false;
    hipLaunchKernelGGL(k_fftdec_dp, dim3((unsigned)wgs), dim3(256), 0, st, L, plan1, plans,
                       seg_list, nblk, nseg, G, form == 3 ? 1u : 0u);
    return true;
  }
#else
  (void)form;
#endif
  const uint64_t gx = (L.len / 512 * 64 + 255) / 256;
  auto kern = k_fftdec_d<kFddSwz>;
#ifdef CEC_TUNING
  // other exchange masks (SWZ): form 4 the crossbar in every phase, 5..9 in some, 10 DPP in every
  // phase (= the product's)
  switch (form) {
    case 4: kern = k_fftdec_d<7>; break;
    case 5: kern = k_fftdec_d<2>; break;
    case 6: kern = k_fftdec_d<3>; break;
    case 7: kern = k_fftdec_d<4>; break;
    case 8: kern = k_fftdec_d<1>; break;
    case 9: kern = k_fftdec_d<6>; break;
    case 10: kern = k_fftdec_d<0>; break;
    case 11: kern = k_fftdec_d<0, false>; break;  // no skip of unread input slots
    default: break;
  }
#endif
  for (uint32_t s0 = 0; s0 < nseg; s0 += 65535) {
    const uint32_t ny = nseg - s0 < 65535 ? nseg - s0 : 65535;
    hipLaunchKernelGGL(kern, dim3((unsigned)gx, ny), dim3(256), 0, st, L, plan1, plans,
                       seg_list, s0);
  }
  return true;
}

}  // namespace cec
