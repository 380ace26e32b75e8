// Bit-sliced additive-FFT building blocks for the RS(32,32) kernels (fft.hip: encode and verify;
// fftdec.hip: erasure decode), gfx950. Device-only, header-inlined.
//
// Data layout shared by every kernel built on this: a lane pair owns 32 byte columns of one
// segment. The 32 positions of a coset (shard indices) are split by their low bit: lane
// l = threadIdx & 1 holds positions t = 2j + l, j = 0..15, each as 8 bit planes (plane q = bit q of
// the lane's 32 bytes of that shard), X[j][q]: 128 VGPRs. A lane's 32 bytes of a shard are two
// 16-byte pieces 512 bytes apart (dwords 0-3 at p, 4-7 at p + 512), so each load / store
// instruction of a wave's 32 even (odd) lanes covers 512 contiguous bytes of one shard.
//
// Transforms (gf256.h): the Lin-Chung-Han IFFT over the coset BETA ^ {0..31} maps the values of a
// polynomial f of degree < 32 at those points to its coefficients in the novel polynomial basis;
// the FFT maps them back onto any coset. Layers with half-distance >= 2 pair registers of one lane;
// the half-distance-1 layers pair the two lanes (DPP quad_perm [1,0,3,2]). Skews depend only on
// the position bits above the layer, so both lanes of a pair multiply by the same compile-time
// constant; multiplication by a constant s is its 8x8 GF(2) matrix on the planes.
#pragma once
#include <utility>

#include "dev_util.h"
#include "gf256.h"

namespace cec {
namespace fftc {

#define CEC_FFT_AI __attribute__((always_inline))

template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) CEC_FFT_AI {
    (f(std::integral_constant<int, I>{}), ...);
  }(std::make_integer_sequence<int, N>{});
}

// skews of the 32-point transforms over the coset BETA ^ {0..31}
template <unsigned BETA>
struct Skews {
  static constexpr LchSkews<5> s = lch_skews<5>((uint8_t)BETA);
};

struct Bits8 {
  int n = 0;
  int b[8] = {};
};
constexpr Bits8 bits_of(unsigned r) {
  Bits8 o{};
  for (int p = 0; p < 8; ++p)
    if (r >> p & 1) o.b[o.n++] = p;
  return o;
}

#define FFT_BOP3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))
// truth tables (index = src0 * 4 + src1 * 2 + src2)
constexpr int kXor3 = 0x96;  // a ^ b ^ c
constexpr int kSel = 0xCA;   // a ? b : c (bitwise)
constexpr int kXand = 0x78;  // a ^ (b & c)
constexpr int kAndX = 0x28;  // (a ^ b) & c

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return FFT_BOP3(a, b, c, kXor3);
}
__device__ __forceinline__ uint32_t x2(uint32_t a, uint32_t b) { return FFT_BOP3(a, b, 0u, kXor3); }

// a + a as a full-rate v_add_u32 (LLVM would emit a half-rate left shift)
__device__ __forceinline__ uint32_t dbl(uint32_t a) {
  uint32_t r;
  asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(a));
  return r;
}

// Swap-move of an 8x8 bit transpose: bits of `a` outside M go down into b's M positions and b's M
// bits go up into a's positions outside M (shift s).
template <int S, uint32_t M>
__device__ __forceinline__ void swapmove(uint32_t& a, uint32_t& b) {
  const uint32_t bs = S == 1 ? dbl(b) : (b << S);
  const uint32_t na = FFT_BOP3(M, a, bs, kSel);
  const uint32_t nb = FFT_BOP3(M, a >> S, b, kSel);
  a = na;
  b = nb;
}

// 8 dwords (32 bytes) <-> 8 bit planes: plane p byte j bit d = bit p of byte j of dword d (an
// 8x8 bit transpose in each byte lane; the map is an involution).
__device__ __forceinline__ void tr8(uint32_t (&w)[8]) {
  sfor<4>([&](auto D) CEC_FFT_AI { swapmove<4, 0x0F0F0F0Fu>(w[D], w[D + 4]); });
  sfor<4>([&](auto D) CEC_FFT_AI {
    constexpr int d = (D & 1) + (D >> 1) * 4;  // 0, 1, 4, 5
    swapmove<2, 0x33333333u>(w[d], w[d + 2]);
  });
  sfor<4>([&](auto D) CEC_FFT_AI { swapmove<1, 0x55555555u>(w[2 * D], w[2 * D + 1]); });
}

// acc[q] ^= (C * z)[q] (+ extra[q] when EXTRA): XOR of z's planes in row q of C's bit matrix,
// folded two at a time into v_bitop3 xor3.
template <unsigned C, bool EXTRA>
__device__ __forceinline__ void mul_acc(uint32_t (&acc)[8], const uint32_t (&z)[8],
                                        const uint32_t (&extra)[8]) {
  constexpr BitMatrix M = gf_bitmatrix((uint8_t)C);
  sfor<8>([&](auto Q) CEC_FFT_AI {
    constexpr Bits8 bl = bits_of(M.row[Q]);
    constexpr int n = bl.n + (EXTRA ? 1 : 0);
    auto term = [&](auto I) CEC_FFT_AI -> uint32_t {
      if constexpr (EXTRA) {
        if constexpr (I == 0) return extra[Q];
        else return z[bl.b[I - 1]];
      } else {
        return z[bl.b[I]];
      }
    };
    sfor<(n + 1) / 2>([&](auto P) CEC_FFT_AI {
      constexpr int i = 2 * P;
      if constexpr (i + 1 < n)
        acc[Q] = x3(acc[Q], term(std::integral_constant<int, i>{}),
                    term(std::integral_constant<int, i + 1>{}));
      else
        acc[Q] = x2(acc[Q], term(std::integral_constant<int, i>{}));
    });
  });
}

__device__ __forceinline__ uint32_t partner(uint32_t v) {
  // quad_perm [1, 0, 3, 2]: lane l reads lane l ^ 1
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);
}
// the same through the LDS crossbar (ds_swizzle, quad-permute mode) when SWZ: no VALU issue slot
// (every DPP form issues at half rate on gfx950), LDS latency instead
template <bool SWZ>
__device__ __forceinline__ uint32_t partner_x(uint32_t v) {
  if constexpr (SWZ) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x80B1);
  else return partner(v);
}

template <bool NT>
__device__ __forceinline__ void ld32(const uint8_t* p, uint32_t (&w)[8]) {
  const u32x4 a = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p))
                     : *reinterpret_cast<const u32x4*>(p);
  const u32x4 b = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 512))
                     : *reinterpret_cast<const u32x4*>(p + 512);
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
template <bool NT>
__device__ __forceinline__ void st32(uint8_t* p, const uint32_t (&w)[8]) {
  const u32x4 a = {w[0], w[1], w[2], w[3]}, b = {w[4], w[5], w[6], w[7]};
  if constexpr (NT) {
    __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(p));
    __builtin_nontemporal_store(b, reinterpret_cast<u32x4*>(p + 512));
  } else {
    *reinterpret_cast<u32x4*>(p) = a;
    *reinterpret_cast<u32x4*>(p + 512) = b;
  }
}

// IFFT over the coset BETA ^ {0..31}: values -> novel-basis coefficients. em = even-lane mask.
// Layer i: b ^= a; a ^= s*b (i = 0 .. 4).
template <unsigned BETA, bool SWZ = false>
__device__ __forceinline__ void ifft32(uint32_t (&X)[16][8], uint32_t em) {
  using T = Skews<BETA>;
  // layer 0 (positions 2j, 2j + 1: across the lane pair). Z = a ^ b on both lanes; even lane ->
  // a ^ s*Z, odd lane -> Z.
  sfor<16>([&](auto J) CEC_FFT_AI {
    constexpr unsigned s = T::s.s[0][J];
    uint32_t Z[8];
    sfor<8>([&](auto Q) CEC_FFT_AI { Z[Q] = X[J][Q] ^ partner_x<SWZ>(X[J][Q]); });
    if constexpr (s == 0) {
      sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] = FFT_BOP3(em, X[J][Q], Z[Q], kSel); });
    } else {
      // W = X ^ Z ^ s*Z (= partner ^ s*Z) in place, then Z ^ (em & W)
      mul_acc<s, true>(X[J], Z, Z);
      sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] = FFT_BOP3(Z[Q], em, X[J][Q], kXand); });
    }
  });
  // layers 1..4 (in-lane: registers j and j + 2^(i-1))
  sfor<4>([&](auto I1) CEC_FFT_AI {
    constexpr int i = I1 + 1, hj = 1 << (i - 1);
    sfor<16>([&](auto J) CEC_FFT_AI {
      if constexpr (!(J & hj)) {
        constexpr unsigned s = T::s.s[i][J >> i];
        sfor<8>([&](auto Q) CEC_FFT_AI { X[J + hj][Q] = x2(X[J + hj][Q], X[J][Q]); });
        if constexpr (s != 0) mul_acc<s, false>(X[J], X[J + hj], X[J]);
      }
    });
  });
}

// FFT onto the coset BETA ^ {0..31}, layers 4..1 (in-lane) only: fft32 = this + fft32_l0 on
// every slot. Callers that need only some slots' values run fft32_l0 for those.
template <unsigned BETA>
__device__ __forceinline__ void fft32_upper(uint32_t (&X)[16][8]) {
  using T = Skews<BETA>;
  sfor<4>([&](auto I4) CEC_FFT_AI {
    constexpr int i = 4 - I4, hj = 1 << (i - 1);
    sfor<16>([&](auto J) CEC_FFT_AI {
      if constexpr (!(J & hj)) {
        constexpr unsigned s = T::s.s[i][J >> i];
        if constexpr (s != 0) mul_acc<s, false>(X[J], X[J + hj], X[J]);
        sfor<8>([&](auto Q) CEC_FFT_AI { X[J + hj][Q] = x2(X[J + hj][Q], X[J][Q]); });
      }
    });
  });
}
// layer 0 of that FFT on register slot J (positions 2J, 2J + 1: across the lane pair)
template <unsigned BETA, int J, bool SWZ = false>
__device__ __forceinline__ void fft32_l0(uint32_t (&x)[8], uint32_t em, uint32_t om) {
  constexpr unsigned s = Skews<BETA>::s.s[0][J];
  uint32_t P[8];
  sfor<8>([&](auto Q) CEC_FFT_AI {
    const uint32_t y = partner_x<SWZ>(x[Q]);
    P[Q] = FFT_BOP3(em, y, x[Q], kSel);
    x[Q] = FFT_BOP3(x[Q], om, y, kXand);
  });
  if constexpr (s != 0) mul_acc<s, false>(x, P, P);
}

// FFT onto the coset BETA ^ {0..31}: coefficients -> values. Layer i: a ^= s*b; b ^= a
// (i = 4 .. 0). em / om = even / odd-lane masks.
// SER: each slot's last-layer butterfly starts once the previous slot's is done (for callers that
// keep every output slot live after the transform: interleaved, the layer's temporaries of many
// slots add up)
template <unsigned BETA, bool SER = false>
__device__ __forceinline__ void fft32(uint32_t (&X)[16][8], uint32_t em, uint32_t om) {
  using T = Skews<BETA>;
  sfor<4>([&](auto I4) CEC_FFT_AI {
    constexpr int i = 4 - I4, hj = 1 << (i - 1);
    sfor<16>([&](auto J) CEC_FFT_AI {
      if constexpr (!(J & hj)) {
        constexpr unsigned s = T::s.s[i][J >> i];
        if constexpr (s != 0) mul_acc<s, false>(X[J], X[J + hj], X[J]);
        sfor<8>([&](auto Q) CEC_FFT_AI { X[J + hj][Q] = x2(X[J + hj][Q], X[J][Q]); });
      }
    });
  });
  // layer 0 (across the pair): a ^= s*b; b ^= a. With P = b on both lanes (even: partner,
  // odd: own): even -> a ^ s*P, odd -> b ^ a ^ s*P.
  sfor<16>([&](auto J) CEC_FFT_AI {
    constexpr unsigned s = T::s.s[0][J];
    uint32_t P[8];
    if constexpr (SER && J > 0) asm volatile("" : "+v"(X[J][0]) : "v"(X[J - 1][7]));
    sfor<8>([&](auto Q) CEC_FFT_AI {
      const uint32_t y = partner(X[J][Q]);
      P[Q] = FFT_BOP3(em, y, X[J][Q], kSel);
      X[J][Q] = FFT_BOP3(X[J][Q], om, y, kXand);
    });
    if constexpr (s != 0) mul_acc<s, false>(X[J], P, P);
  });
}

}  // namespace fftc
}  // namespace cec
