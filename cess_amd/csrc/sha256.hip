// SHA-256 kernels of libcessec (FIPS 180-4) for the fragment and segment hashes of CESS's
// SegmentList (c-pallets/file-bank/src/types.rs:13-16): one-shot batch kernels (k_sha256,
// k_sha256_2w) and the streaming hash-queue kernels (k_hashq_add, k_sha256_tick).
#include "dev_util.h"
#include "kernels.h"

namespace cec {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return xor3_u32(a, b, c);
}

#define CEC_SHA_AI __attribute__((always_inline))

// ---------------------------------------------------------------------------------------------
// SHA-256 (FIPS 180-4), one lane per buffer.
// ---------------------------------------------------------------------------------------------
// Round constants as compile-time literals: after unrolling each becomes an instruction literal,
// not 64 scalar loads hoisted into SGPRs (which spilled to VGPR lanes).
static constexpr uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

// v_bitop3 truth tables (index = a<<2 | b<<1 | c): Ch = a ? b : c, Maj = majority.
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// D >= 0: empty asm statements pin the expansion of message word t + D to round t. Without them
// (D < 0) the compiler expands all 48 schedule words up front (they do not depend on the state)
// and holds them. Pinned, the one-wave tick fits in 74 VGPRs instead of 100, leaving room for an
// RS(32,32) encode wave beside four tick waves per SIMD; measured, that co-residence slowed
// config 5's step from 1.74 to 2.03 ms, so the ticks run unpinned and only the
// prefix-digest compression (after the tick loop) is pinned.
template <int D = -1>
__device__ __forceinline__ void sha256_block(uint32_t (&h)[8], uint32_t (&w)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  auto expand = [&](int u) CEC_SHA_AI {  // W[u] into w[u & 15] (which held W[u - 16])
    const uint32_t w15 = w[(u + 1) & 15], w2 = w[(u + 14) & 15];
    const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
    const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
    w[u & 15] = w[u & 15] + s0 + w[(u + 9) & 15] + s1;
  };
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    if constexpr (D >= 0) {
      asm volatile("" : "+v"(a), "+v"(e));
      const int u = t + D;
      if (u >= 16 && u < 64) {
        asm volatile("" : "+v"(w[(u + 14) & 15]), "+v"(w[(u + 1) & 15]) : "v"(e));
        expand(u);
      }
    } else {
      if (t >= 16) expand(t);
    }
    const uint32_t wt = w[t & 15];
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t t1 = hh + S1 + ch(e, f, g) + kSha256K[t] + wt;
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t t2 = S0 + maj(a, b, c);
    hh = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

__global__ __launch_bounds__(64) void k_sha256(const uint8_t* const* __restrict__ ptrs, Layout L,
                                               int nshards, uint64_t n, uint64_t len,
                                               uint8_t* __restrict__ hex_out) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* src =
      ptrs ? ptrs[i] : shard_ptr(L, (int)(i % nshards), (uint32_t)(i / nshards));
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t w[16];
  const uint64_t nfull = len >> 6;
  const bool al16 = ((uintptr_t)src & 15) == 0;
  if (al16) {
    // The next block's 64 bytes are loaded while this block is compressed: one HBM round trip
    // per block (~1-2 us under load) would otherwise sit on every lane's serial chain.
    u32x4 nx[4];
    if (nfull) {
#pragma unroll
      for (int q = 0; q < 4; ++q) nx[q] = *reinterpret_cast<const u32x4*>(src + 16 * q);
    }
    for (uint64_t blk = 0; blk < nfull; ++blk) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[4 * q + 0] = __builtin_bswap32(nx[q].x);
        w[4 * q + 1] = __builtin_bswap32(nx[q].y);
        w[4 * q + 2] = __builtin_bswap32(nx[q].z);
        w[4 * q + 3] = __builtin_bswap32(nx[q].w);
      }
      if (blk + 1 < nfull) {
        const uint8_t* p = src + ((blk + 1) << 6);
#pragma unroll
        for (int q = 0; q < 4; ++q) nx[q] = *reinterpret_cast<const u32x4*>(p + 16 * q);
      }
      sha256_block(h, w);
    }
  } else {
    for (uint64_t blk = 0; blk < nfull; ++blk) {
      const uint8_t* p = src + (blk << 6);
#pragma unroll
      for (int q = 0; q < 16; ++q)
        w[q] = (uint32_t)p[4 * q] << 24 | (uint32_t)p[4 * q + 1] << 16 |
               (uint32_t)p[4 * q + 2] << 8 | (uint32_t)p[4 * q + 3];
      sha256_block(h, w);
    }
  }
  // Padding: remaining r bytes, 0x80, zeros, 64-bit big-endian bit length.
  const uint32_t r = (uint32_t)(len & 63);
  const uint8_t* p = src + (nfull << 6);
  const uint64_t bits = len << 3;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    uint32_t word = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t pos = 4 * q + s;
      const uint32_t byte = pos < r ? p[pos] : (pos == r ? 0x80u : 0u);
      word |= byte << (24 - 8 * s);
    }
    w[q] = word;
  }
  if (r >= 56) {
    sha256_block(h, w);
#pragma unroll
    for (int q = 0; q < 16; ++q) w[q] = 0;
  }
  w[14] = (uint32_t)(bits >> 32);
  w[15] = (uint32_t)bits;
  sha256_block(h, w);
  uint8_t* o = hex_out + i * 64;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    uint32_t word = h[q];
    uint32_t lo = 0, hi = 0;  // 8 hex chars of this word, packed little-endian for 2 stores
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t nib = (word >> (28 - 4 * s)) & 15u;
      const uint32_t ch = nib < 10 ? '0' + nib : 'a' + nib - 10;
      if (s < 4) lo |= ch << (8 * s);
      else hi |= ch << (8 * (s - 4));
    }
    *reinterpret_cast<uint32_t*>(o + 8 * q) = lo;
    *reinterpret_cast<uint32_t*>(o + 8 * q + 4) = hi;
  }
}

// Two waves per group of 64 buffers. Each buffer's hash is one serial chain, so with few
// buffers (a 1 GiB RS(32,32) batch is 4096 fragments = 64 waves on a 1024-SIMD chip) the time
// is the per-block instruction count of ONE wave. The message schedule does not depend on the
// chaining state, so wave 0 (producer) loads block i+1, byte-swaps it and expands W[0..63] + K
// into LDS while wave 1 (consumer) runs the 64 rounds of block i: the consumer's chain drops from
// ~1460 to ~900 VALU instructions per block. LDS ring: 2 buffers x 64 words x 64 lanes (32 KiB),
// [buf][word/4][lane][4] so every ds_write/read_b128 covers 1 KiB contiguous. One barrier per
// block; the padding block(s) go through the same pipeline.
__device__ __forceinline__ const uint8_t* sha_src(const uint8_t* const* ptrs, const Layout& L,
                                                  int nshards, uint64_t i) {
  return ptrs ? ptrs[i] : shard_ptr(L, (int)(i % nshards), (uint32_t)(i / nshards));
}

template <int QS = 64>
__device__ __forceinline__ void sha_expand_store(uint32_t (&w)[16], u32x4* __restrict__ dst) {
  // dst[q * QS] = {W+K}[4q .. 4q+3] for this lane
#pragma unroll
  for (int t = 0; t < 64; t += 4) {
    uint32_t o[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int u = t + s;
      uint32_t wt;
      if (u < 16) {
        wt = w[u];
      } else {
        const uint32_t w15 = w[(u + 1) & 15], w2 = w[(u + 14) & 15];
        const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
        const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
        wt = w[u & 15] + s0 + w[(u + 9) & 15] + s1;
        w[u & 15] = wt;
      }
      o[s] = wt + kSha256K[u];
    }
    dst[(t / 4) * QS] = u32x4{o[0], o[1], o[2], o[3]};
  }
}

__device__ __forceinline__ void sha_store_hex(uint8_t* __restrict__ o, const uint32_t (&h)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t word = h[q];
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t nib = (word >> (28 - 4 * s)) & 15u;
      const uint32_t chr = nib < 10 ? '0' + nib : 'a' + nib - 10;
      if (s < 4) lo |= chr << (8 * s);
      else hi |= chr << (8 * (s - 4));
    }
    *reinterpret_cast<uint32_t*>(o + 8 * q) = lo;
    *reinterpret_cast<uint32_t*>(o + 8 * q + 4) = hi;
  }
}

// Lane-pair rounds (the latency form of the two-wave kernels, k_sha256_lp and k_sha256_tick_lp):
// a chain's 64 rounds on TWO lanes of a consumer wave. The even lane carries (e, f, g, h) and
// computes T1 = h + Sigma1(e) + Ch(e, f, g) + K + W, the odd lane carries (a, b, c, d) and computes
// T2 = Sigma0(a) + Maj(a, b, c), with the same instructions: the rotate amounts sit in VGPRs
// (v_alignbit takes its shift per lane), Maj(a, b, c) = Ch(a ^ c, b, c) makes Maj a Ch of the
// lane's own history, and the odd lane reads zeros where the even lane reads K + W. One DPP
// quad_perm [1,0,3,2] exchange per round: the even lane sends T1, the odd lane d, and each adds
// what it receives (even: e = d + T1, odd: a = T2 + T1). 11 VALU instructions (16 issue slots)
// per round on the pair against 14 (22) on one lane: a lone wave's block drops from 3660 to 3204
// s_memtime ticks (tools/sha_latency.hip, profiles/r06/sha_latency_forms.jsonl). A pair spends
// two lanes per chain, so these are the kernels of the latency regime only (few chains).
__device__ __forceinline__ uint32_t sha_swap_pair(uint32_t v) {  // lane l ^ 1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}

struct ShaLp {
  uint32_t r1, r2, r3, M;
  bool even;
};

__device__ __forceinline__ ShaLp sha_lp(bool even) {
  // even: Sigma1 rotates, odd: Sigma0 rotates and the Maj operand mask (a ^ c)
  return ShaLp{even ? 6u : 2u, even ? 11u : 13u, even ? 25u : 22u, even ? 0u : ~0u, even};
}

// One block: src[q * QS] = K + W of rounds 4q .. 4q + 3 (zeros on the odd lane); the pair's
// halves (X0..X3: e, f, g, h on the even lane, a, b, c, d on the odd lane) advance in place.
template <int QS>
__device__ __forceinline__ void sha_lp_block(const u32x4* __restrict__ src, const ShaLp& L,
                                             uint32_t& X0, uint32_t& X1, uint32_t& X2,
                                             uint32_t& X3) {
  uint32_t x0 = X0, x1 = X1, x2 = X2, x3 = X3;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const u32x4 kw4 = src[q * QS];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const uint32_t kw = s4 == 0 ? kw4.x : s4 == 1 ? kw4.y : s4 == 2 ? kw4.z : kw4.w;
      const uint32_t S = xor3(__builtin_amdgcn_alignbit(x0, x0, L.r1),
                              __builtin_amdgcn_alignbit(x0, x0, L.r2),
                              __builtin_amdgcn_alignbit(x0, x0, L.r3));
      const uint32_t P = __builtin_amdgcn_bitop3_b32(x0, x2, L.M, 0x78);  // x0 ^ (x2 & M)
      const uint32_t CM = ch(P, x1, x2);          // even: Ch(e, f, g); odd: Maj(a, b, c)
      const uint32_t HK = (L.even ? x3 : 0u) + kw;  // even: h + K + W; odd: 0
      const uint32_t V = S + CM + HK;             // even: T1; odd: T2
      const uint32_t U = L.even ? V : x3;         // what the partner needs: T1 / d
      const uint32_t xn = V + sha_swap_pair(U);   // even: e = d + T1; odd: a = T2 + T1
      x3 = x2; x2 = x1; x1 = x0; x0 = xn;
    }
  }
  X0 += x0; X1 += x1; X2 += x2; X3 += x3;
}

// The whole state (a..h) from a pair's halves, on the even lane (both lanes must execute it).
__device__ __forceinline__ void sha_lp_full(uint32_t (&h)[8], uint32_t X0, uint32_t X1,
                                            uint32_t X2, uint32_t X3) {
  h[0] = sha_swap_pair(X0);
  h[1] = sha_swap_pair(X1);
  h[2] = sha_swap_pair(X2);
  h[3] = sha_swap_pair(X3);
  h[4] = X0; h[5] = X1; h[6] = X2; h[7] = X3;
}

// LP: two consumer waves on lane pairs (sha_lp_block) instead of one on single lanes; ring
// column 64 holds the odd lanes' zeros.
template <bool LP>
__global__ __launch_bounds__(LP ? 192 : 128) void k_sha256_2w(const uint8_t* const* __restrict__ ptrs,
                                                   Layout L, int nshards, uint64_t n,
                                                   uint64_t len, uint8_t* __restrict__ hex_out) {
  constexpr int QS = LP ? 65 : 64;
  __shared__ u32x4 ring[2][16][QS];
  const int lane = threadIdx.x & 63;
  // wave-uniform by construction (SGPR), so the two sides' barriers never run under one EXEC mask
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool producer = wave == 0;
  const uint64_t i = (uint64_t)blockIdx.x * 64 + lane;
  const bool live = i < n;
  const uint64_t nfull = len >> 6;
  const uint32_t r = (uint32_t)(len & 63);
  const uint64_t nb = nfull + (r >= 56 ? 2 : 1);  // blocks including padding
  if (producer) {
    const uint8_t* src = live ? sha_src(ptrs, L, nshards, i) : nullptr;
    const bool al16 = live && ((uintptr_t)src & 15) == 0;
    u32x4 nx[4] = {};
    if (al16 && nfull) {
#pragma unroll
      for (int q = 0; q < 4; ++q) nx[q] = *reinterpret_cast<const u32x4*>(src + 16 * q);
    }
    for (uint64_t blk = 0; blk < nb; ++blk) {
      uint32_t w[16];
      if (blk < nfull) {
        if (al16) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            w[4 * q + 0] = __builtin_bswap32(nx[q].x);
            w[4 * q + 1] = __builtin_bswap32(nx[q].y);
            w[4 * q + 2] = __builtin_bswap32(nx[q].z);
            w[4 * q + 3] = __builtin_bswap32(nx[q].w);
          }
          if (blk + 1 < nfull) {
            const uint8_t* p = src + ((blk + 1) << 6);
#pragma unroll
            for (int q = 0; q < 4; ++q) nx[q] = *reinterpret_cast<const u32x4*>(p + 16 * q);
          }
        } else if (live) {
          const uint8_t* p = src + (blk << 6);
#pragma unroll
          for (int q = 0; q < 16; ++q)
            w[q] = (uint32_t)p[4 * q] << 24 | (uint32_t)p[4 * q + 1] << 16 |
                   (uint32_t)p[4 * q + 2] << 8 | (uint32_t)p[4 * q + 3];
        } else {
#pragma unroll
          for (int q = 0; q < 16; ++q) w[q] = 0;
        }
      } else {
        // padding block(s): remaining r bytes, 0x80, zeros, 64-bit big-endian bit length
        const bool first_pad = blk == nfull;
        const uint8_t* p = live ? src + (nfull << 6) : nullptr;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          uint32_t word = 0;
          if (first_pad) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const uint32_t pos = 4 * q + s;
              const uint32_t byte = pos < r ? (live ? p[pos] : 0u) : (pos == r ? 0x80u : 0u);
              word |= byte << (24 - 8 * s);
            }
          }
          w[q] = word;
        }
        if (blk == nb - 1) {
          const uint64_t bits = len << 3;
          w[14] = (uint32_t)(bits >> 32);
          w[15] = (uint32_t)bits;
        }
      }
      sha_expand_store<QS>(w, &ring[blk & 1][0][lane]);
      __syncthreads();
    }
    __syncthreads();  // matches the consumer's final iteration
  } else if constexpr (LP) {
    // lane pair p = lane / 2 of consumer wave 1 or 2 hashes buffer 32 (wave - 1) + p
    const int c = 32 * (wave - 1) + (lane >> 1);
    const bool even = (lane & 1) == 0;
    if (lane < 32) ring[lane >> 4][lane & 15][64] = u32x4{0, 0, 0, 0};  // the zero column
    const uint64_t ic = (uint64_t)blockIdx.x * 64 + c;
    const ShaLp lp = sha_lp(even);
    const int col = even ? c : 64;
    uint32_t X0 = even ? 0x510e527fu : 0x6a09e667u, X1 = even ? 0x9b05688cu : 0xbb67ae85u,
             X2 = even ? 0x1f83d9abu : 0x3c6ef372u, X3 = even ? 0x5be0cd19u : 0xa54ff53au;
    __syncthreads();  // block 0 produced (and the zero column written)
    for (uint64_t blk = 0; blk < nb; ++blk) {
      sha_lp_block<QS>(&ring[blk & 1][0][col], lp, X0, X1, X2, X3);
      __syncthreads();  // this buffer consumed / next one produced
    }
    uint32_t h[8];
    sha_lp_full(h, X0, X1, X2, X3);
    if (ic < n && even) sha_store_hex(hex_out + ic * 64, h);
  } else {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                     0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    __syncthreads();  // block 0 produced
    for (uint64_t blk = 0; blk < nb; ++blk) {
      const u32x4* src = &ring[blk & 1][0][lane];
      uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const u32x4 kw4 = src[q * 64];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const uint32_t kw = s == 0 ? kw4.x : s == 1 ? kw4.y : s == 2 ? kw4.z : kw4.w;
          const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
          const uint32_t t1 = hh + S1 + ch(e, f, g) + kw;
          const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
          const uint32_t t2 = S0 + maj(a, b, c);
          hh = g; g = f; f = e; e = d + t1;
          d = c; c = b; b = a; a = t1 + t2;
        }
      }
      h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
      __syncthreads();  // this buffer consumed / next one produced
    }
    if (live) {
      uint8_t* o = hex_out + i * 64;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint32_t word = h[q];
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const uint32_t nib = (word >> (28 - 4 * s)) & 15u;
          const uint32_t chr = nib < 10 ? '0' + nib : 'a' + nib - 10;
          if (s < 4) lo |= chr << (8 * s);
          else hi |= chr << (8 * (s - 4));
        }
        *reinterpret_cast<uint32_t*>(o + 8 * q) = lo;
        *reinterpret_cast<uint32_t*>(o + 8 * q + 4) = hi;
      }
    }
  }
}

// Streaming SHA-256 over many long buffers (the hash queue, hashq.cpp). A chain's state
// (ShaChain, kernels.h) lives in HBM between launches, so one tick kernel advances every live
// chain of the queue by at most `max_blocks` 64-byte blocks and chains of different batches,
// lengths and ages share launches. With a window of several batches in flight the chip holds
// tens of thousands of chains at once, where one batch alone (4096 fragments of a 1 GiB
// RS(32,32) batch; 192 of a 1 GiB RS(2,1) batch) fills a few percent of its SIMDs. Same
// two-wave structure as k_sha256_2w; chains of one wave may be at different blocks.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// Message block `g` of a chain for the rare cases (unaligned buffer, padding block): the bytes
// go through this lane's 64-byte LDS stage (final big-endian words) one at a time, so a single load is in flight and the
// path costs a few VGPRs (64 unrolled byte loads would raise the whole kernel's VGPR count and
// cut its occupancy). Block g < nfull is message data; the first padding block holds the last
// r bytes and 0x80; the last block ends with the 64-bit big-endian bit length.
// `stage` holds the block's 16 words as 4 x u32x4 at a stride of `qstride` u32x4 (1: a lane's
// own 64 bytes; 64: this lane's column of a [4][64] u32x4 ring buffer).
__device__ __noinline__ void sha_stage_general(const uint8_t* src, uint64_t g, uint64_t nfull,
                                               uint32_t r, uint64_t nb, uint64_t len,
                                               u32x4* stage, uint32_t qstride) {
  const uint8_t* p = src + (g << 6);
  const uint32_t nbytes = g < nfull ? 64u : (g == nfull ? r : 0u);
  const uint32_t mark = g == nfull ? r : 64u;  // where the 0x80 goes (first padding block)
#pragma unroll 1
  for (uint32_t j = 0; j < 64; ++j)
    reinterpret_cast<uint8_t*>(stage + (j >> 4) * qstride)[j & 15] =
        j < nbytes ? p[j] : (j == mark ? 0x80 : 0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    u32x4 v = stage[q * qstride];
    v = u32x4{__builtin_bswap32(v.x), __builtin_bswap32(v.y), __builtin_bswap32(v.z),
              __builtin_bswap32(v.w)};
    if (q == 3 && g == nb - 1) {
      const uint64_t bits = len << 3;
      v.z = (uint32_t)(bits >> 32);
      v.w = (uint32_t)bits;
    }
    stage[q * qstride] = v;
  }
}

// The general block through the stage (the callee never sees `w`, so it stays in registers).
__device__ __forceinline__ void sha_block_general(uint32_t (&w)[16], const uint8_t* src,
                                                  uint64_t g, uint64_t nfull, uint32_t r,
                                                  uint64_t nb, uint64_t len, u32x4* stage,
                                                  uint32_t qstride) {
  sha_stage_general(src, g, nfull, r, nb, len, stage, qstride);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const u32x4 v = stage[q * qstride];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
}


// Prefix digest of a chain (ShaChain::pre_blk): finish a copy of the state after `blocks` whole
// message blocks with the one padding block of a 64-byte-multiple length, write its hex.
template <int D = -1>
__device__ __forceinline__ void sha_prefix_hex_inl(uint32_t (&h)[8], uint64_t blocks,
                                                   uint8_t* __restrict__ hex) {
  uint32_t w[16];
  const uint64_t bits = blocks << 9;
  w[0] = 0x80000000u;
#pragma unroll
  for (int q = 1; q < 14; ++q) w[q] = 0;
  w[14] = (uint32_t)(bits >> 32);
  w[15] = (uint32_t)bits;
  sha256_block<D>(h, w);
  sha_store_hex(hex, h);
}

// Out-of-line form for the two-wave tick, which reaches the prefix inside its block loop (an
// inlined second compression there would raise its VGPR count). The state goes by value (eight
// VGPR arguments): a pointer would put the caller's h in scratch.
__device__ __noinline__ void sha_prefix_hex(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3,
                                            uint32_t h4, uint32_t h5, uint32_t h6, uint32_t h7,
                                            uint64_t blocks, uint8_t* __restrict__ hex) {
  uint32_t h[8] = {h0, h1, h2, h3, h4, h5, h6, h7};
  sha_prefix_hex_inl(h, blocks, hex);
}

// The producer wave of the latency-form ticks: loads, byte-swaps and expands every block of its
// 64 chains into the LDS ring ([buf][word/4][QS columns] u32x4, column = lane), one barrier per
// block, `trips` barriers in all (the consumers' count).
template <int PF, int QS>
__device__ __forceinline__ void sha_tick_produce(u32x4* __restrict__ ring, int lane,
                                                 const ShaChain* ch_, bool live, uint64_t blk0,
                                                 uint64_t nfull, uint32_t r, uint64_t nb,
                                                 uint64_t len, uint32_t nblk, uint32_t trips) {
  const uint8_t* src = live ? ch_->src : nullptr;
  const bool al16 = live && ((uintptr_t)src & 15) == 0;
  // Fast blocks: this lane's aligned message data in this tick (the bulk of a tick), loaded with
  // the next PF blocks in flight. The count is per lane: the 64 chains of a group come from
  // adds of any size, so they may differ in length and progress (a finished chain beside a
  // running one). The wave runs the fast loop for its longest run; a lane past its own runs the
  // general path (padding blocks, unaligned buffers) or writes zeros, masked. (A wave-uniform
  // count, the minimum over the lanes, sent every chain of a group that held a finished one
  // through the byte-wise general path: 3x slower ticks, profiles/r06/gpumode_ramp/.)
  const uint64_t dat = blk0 < nfull ? nfull - blk0 : 0;
  const uint32_t mine = al16 ? (uint32_t)(dat < nblk ? dat : nblk) : 0u;
  const uint32_t nfast = __builtin_amdgcn_readfirstlane(wave_max_u32(mine));
  // nx[j] holds block b + j: PF blocks of loads in flight ahead of the one being expanded
  u32x4 nx[PF][4] = {};
#pragma unroll
  for (int j = 0; j < PF; ++j)
    if ((uint32_t)j < mine) {
      const uint8_t* p = src + ((blk0 + j) << 6);
#pragma unroll
      for (int q = 0; q < 4; ++q) nx[j][q] = *reinterpret_cast<const u32x4*>(p + 16 * q);
    }
  auto slot = [&](uint32_t blk) CEC_SHA_AI { return ring + (blk & 1) * 16 * QS + lane; };
  auto produce = [&](u32x4 (&v)[4], uint32_t blk) CEC_SHA_AI {
    uint32_t w[16];
    if (blk < mine) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[4 * q + 0] = __builtin_bswap32(v[q].x);
        w[4 * q + 1] = __builtin_bswap32(v[q].y);
        w[4 * q + 2] = __builtin_bswap32(v[q].z);
        w[4 * q + 3] = __builtin_bswap32(v[q].w);
      }
      const uint32_t nb_next = blk + PF;
      if (nb_next < mine) {
        const uint8_t* p = src + ((blk0 + nb_next) << 6);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const u32x4*>(p + 16 * q);
      }
    } else if (blk < nblk) {
      // staged in the ring buffer this block is about to be written to (consumed at blk - 2)
      sha_block_general(w, src, blk0 + blk, nfull, r, nb, len, slot(blk), QS);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = 0;
    }
    sha_expand_store<QS>(w, slot(blk));
    __syncthreads();
  };
  uint32_t b = 0;
  for (; b + PF <= nfast; b += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) produce(nx[j], b + j);
  }
#pragma unroll
  for (int j = 0; j < PF; ++j)
    if (b < nfast) {
      produce(nx[j], b);
      ++b;
    }
  for (; b < trips; ++b) {  // past every lane's fast run
    uint32_t w[16];
    if (b < nblk) {
      sha_block_general(w, src, blk0 + b, nfull, r, nb, len, slot(b), QS);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = 0;
    }
    sha_expand_store<QS>(w, slot(b));
    __syncthreads();
  }
  __syncthreads();  // matches the consumers' final iteration
}

template <int PF>
__global__ __launch_bounds__(128) void k_sha256_tick(ShaChain* __restrict__ tab, uint32_t mask,
                                                     uint64_t head, uint32_t n,
                                                     uint32_t max_blocks) {
  __shared__ u32x4 ring[2][16][64];
  const int lane = threadIdx.x & 63;
  const bool producer = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  const uint32_t i = blockIdx.x * 64 + lane;
  const bool live = i < n;
  ShaChain* ch_ = &tab[(uint32_t)(head + i) & mask];
  uint64_t len = 0, blk0 = 0;
  if (live) {
    len = ch_->len;
    blk0 = ch_->blk;
  }
  const uint64_t nfull = len >> 6;
  const uint32_t r = (uint32_t)(len & 63);
  const uint64_t nb = nfull + (r >= 56 ? 2 : 1);  // blocks including padding
  const uint64_t rem = live ? nb - blk0 : 0;
  const uint32_t nblk = rem < max_blocks ? (uint32_t)rem : max_blocks;
  // both waves see the same 64 chains, so they agree on the trip count (and barrier count)
  const uint32_t trips = wave_max_u32(nblk);
  if (trips == 0) return;
  if (producer) {
    sha_tick_produce<PF, 64>(&ring[0][0][0], lane, ch_, live, blk0, nfull, r, nb, len, nblk,
                             trips);
  } else {
    uint32_t h[8] = {};
    uint64_t pre = 0;  // block count after which the prefix digest is due (0: none)
    if (live) {
#pragma unroll
      for (int q = 0; q < 8; ++q) h[q] = ch_->h[q];
      pre = ch_->pre_blk;
    }
    __syncthreads();  // block 0 produced
    for (uint32_t b = 0; b < trips; ++b) {
      if (b < nblk) {
        const u32x4* src = &ring[b & 1][0][lane];
        uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const u32x4 kw4 = src[q * 64];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const uint32_t kw = s == 0 ? kw4.x : s == 1 ? kw4.y : s == 2 ? kw4.z : kw4.w;
            const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
            const uint32_t t1 = hh + S1 + ch(e, f, g) + kw;
            const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
            const uint32_t t2 = S0 + maj(a, bb, c);
            hh = g; g = f; f = e; e = d + t1;
            d = c; c = bb; bb = a; a = t1 + t2;
          }
        }
        h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
        if (blk0 + b + 1 == pre)
          sha_prefix_hex(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], pre, ch_->pre_hex);
      }
      __syncthreads();  // this buffer consumed / next one produced
    }
    if (live && nblk) {
#pragma unroll
      for (int q = 0; q < 8; ++q) ch_->h[q] = h[q];
      ch_->blk = blk0 + nblk;
      if (blk0 + nblk == nb && ch_->hex) sha_store_hex(ch_->hex, h);
    }
  }
}

// Lane-pair tick (the latency regime: few chains, so a chain's time is one wave's issue rate per
// block). The producer wave expands the schedules of 64 chains as in k_sha256_tick; two consumer
// waves run the rounds on lane pairs (sha_lp_block). Three waves per 64 chains: the launcher picks
// it while the live chains leave the SIMDs idle.
template <int PF>
__global__ __launch_bounds__(192) void k_sha256_tick_lp(ShaChain* __restrict__ tab, uint32_t mask,
                                                        uint64_t head, uint32_t n,
                                                        uint32_t max_blocks) {
  constexpr int QS = 65;  // column 64: zeros, the odd lanes' K + W
  __shared__ u32x4 ring[2][16][QS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // every wave computes the trip count over the group's 64 chains (lane = chain), so all three
  // agree on the number of barriers
  const uint32_t i = blockIdx.x * 64 + lane;
  const bool live = i < n;
  ShaChain* ch_ = &tab[(uint32_t)(head + i) & mask];
  uint64_t len = 0, blk0 = 0;
  if (live) {
    len = ch_->len;
    blk0 = ch_->blk;
  }
  const uint64_t nfull = len >> 6;
  const uint32_t r = (uint32_t)(len & 63);
  const uint64_t nb = nfull + (r >= 56 ? 2 : 1);
  const uint64_t rem = live ? nb - blk0 : 0;
  const uint32_t nblk = rem < max_blocks ? (uint32_t)rem : max_blocks;
  const uint32_t trips = wave_max_u32(nblk);
  if (trips == 0) return;
  if (wave == 0) {
    sha_tick_produce<PF, QS>(&ring[0][0][0], lane, ch_, live, blk0, nfull, r, nb, len, nblk,
                             trips);
    return;
  }
  // consumer wave 1 or 2: lane pair p = lane / 2 runs chain c = 32 (wave - 1) + p
  const int c = 32 * (wave - 1) + (lane >> 1);
  const bool even = (lane & 1) == 0;
  if (lane < 32) ring[lane >> 4][lane & 15][64] = u32x4{0, 0, 0, 0};  // the zero column
  const uint32_t ic = blockIdx.x * 64 + c;
  const bool livec = ic < n;
  ShaChain* cc = &tab[(uint32_t)(head + ic) & mask];
  uint64_t lenc = 0, b0 = 0, pre = 0;
  uint32_t X0 = 0, X1 = 0, X2 = 0, X3 = 0;
  if (livec) {
    lenc = cc->len;
    b0 = cc->blk;
    pre = cc->pre_blk;
    const int o = even ? 4 : 0;
    X0 = cc->h[o];
    X1 = cc->h[o + 1];
    X2 = cc->h[o + 2];
    X3 = cc->h[o + 3];
  }
  const uint64_t nbc = (lenc >> 6) + ((lenc & 63) >= 56 ? 2 : 1);
  const uint64_t remc = livec ? nbc - b0 : 0;
  const uint32_t nblkc = remc < max_blocks ? (uint32_t)remc : max_blocks;
  const ShaLp lp = sha_lp(even);
  const int col = even ? c : 64;
  auto full = [&](uint32_t (&h)[8]) CEC_SHA_AI { sha_lp_full(h, X0, X1, X2, X3); };
  __syncthreads();  // block 0 produced (and the zero column written)
  for (uint32_t b = 0; b < trips; ++b) {
    if (b < nblkc) {
      sha_lp_block<QS>(&ring[b & 1][0][col], lp, X0, X1, X2, X3);
      if (b0 + b + 1 == pre) {  // both lanes of the pair: the exchange needs the partner
        uint32_t h[8];
        full(h);
        if (even) sha_prefix_hex(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], pre, cc->pre_hex);
      }
    }
    __syncthreads();  // this buffer consumed / next one produced
  }
  if (livec && nblkc) {
    const int o = even ? 4 : 0;
    cc->h[o] = X0;
    cc->h[o + 1] = X1;
    cc->h[o + 2] = X2;
    cc->h[o + 3] = X3;
    const bool last = b0 + nblkc == nbc && cc->hex;
    uint32_t h[8];
    full(h);
    if (even) {
      cc->blk = b0 + nblkc;
      if (last) sha_store_hex(cc->hex, h);
    }
  }
}

// One-wave tick: each lane expands its own message schedule in registers (no LDS, no barrier).
// Per block it issues the whole ~1460 VALU ops on one wave instead of splitting them over a
// producer and a consumer wave, so it loses in the latency regime (few chains: one wave's issue
// rate is the bound) and can win in the throughput regime (several waves per SIMD interleave,
// and no barrier ties a consumer to its producer).
template <int D>
__global__ __launch_bounds__(64) void k_sha256_tick1(ShaChain* __restrict__ tab, uint32_t mask,
                                                     uint64_t head, uint32_t n,
                                                     uint32_t max_blocks) {
  __shared__ u32x4 stage[64][4];  // general-path byte staging
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  ShaChain* ch_ = &tab[(uint32_t)(head + i) & mask];
  const uint64_t len = ch_->len, blk0 = ch_->blk;
  const uint64_t nfull = len >> 6;
  const uint32_t r = (uint32_t)(len & 63);
  const uint64_t nb = nfull + (r >= 56 ? 2 : 1);
  const uint64_t rem = nb - blk0;
  const uint32_t nblk = rem < max_blocks ? (uint32_t)rem : max_blocks;
  if (nblk == 0) return;
  const uint8_t* src = ch_->src;
  const uint64_t pre = ch_->pre_blk;
  uint32_t h[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) h[q] = ch_->h[q];
  const bool al16 = ((uintptr_t)src & 15) == 0;
  const uint64_t dat = blk0 < nfull ? nfull - blk0 : 0;
  const uint32_t nfast = al16 ? (uint32_t)(dat < nblk ? dat : nblk) : 0u;
  // 32-bit loop state only: the prefix block relative to blk0 (0: not in this tick), a running
  // pointer for the fast path; the general path re-reads the chain record
  const uint32_t pre_rel = pre > blk0 && pre - blk0 <= nblk ? (uint32_t)(pre - blk0) : 0u;
  const uint8_t* p = src + (blk0 << 6);
  uint32_t w[16];
  u32x4 nx[4] = {};
  if (nfast) {
#pragma unroll
    for (int q = 0; q < 4; ++q) nx[q] = *reinterpret_cast<const u32x4*>(p + 16 * q);
  }
  // one compression per iteration (a second inlined copy of the rounds doubles the VGPRs)
  for (uint32_t b = 0; b < nblk; ++b) {
    if (b < nfast) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[4 * q + 0] = __builtin_bswap32(nx[q].x);
        w[4 * q + 1] = __builtin_bswap32(nx[q].y);
        w[4 * q + 2] = __builtin_bswap32(nx[q].z);
        w[4 * q + 3] = __builtin_bswap32(nx[q].w);
      }
      p += 64;
      if (b + 1 < nfast) {
#pragma unroll
        for (int q = 0; q < 4; ++q) nx[q] = *reinterpret_cast<const u32x4*>(p + 16 * q);
      }
    } else {
      const volatile ShaChain* cv = ch_;
      const uint64_t len_ = cv->len, nfull_ = len_ >> 6;
      const uint32_t r_ = (uint32_t)(len_ & 63);
      sha_block_general(w, (const uint8_t*)cv->src, cv->blk + b, nfull_, r_,
                        nfull_ + (r_ >= 56 ? 2 : 1), len_, &stage[threadIdx.x][0], 1);
    }
    sha256_block<D>(h, w);
    if (b + 1 == pre_rel) {  // parked: a call in the loop would hold the loop's live values across it
#pragma unroll
      for (int q = 0; q < 8; ++q) ch_->pre_h[q] = h[q];
    }
  }
  // the record's fields are re-read rather than held across the loop
  const volatile ShaChain* cv = ch_;
  const uint64_t blk_end = cv->blk + nblk;
  const bool done = blk_end == sha256_blocks(cv->len);
#pragma unroll
  for (int q = 0; q < 8; ++q) ch_->h[q] = h[q];
  if (pre_rel) {  // after the loop, inlined: few values are live here
    uint32_t ph[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) ph[q] = cv->pre_h[q];
    sha_prefix_hex_inl<D < 0 ? 0 : D>(ph, cv->pre_blk, cv->pre_hex);
  }
  ch_->blk = blk_end;
  if (done && cv->hex) sha_store_hex(cv->hex, h);
}

// Initialise n chains in queue slots slot0.. (mod capacity): buffer i starts at
// base + (i / per) * outer + (i % per) * inner and its hex goes to
// hex + ((i / per) * hex_outer + i % per) * 64.
__global__ __launch_bounds__(256) void k_hashq_add(ShaChain* __restrict__ tab, uint32_t mask,
                                                   uint64_t slot0, uint32_t n,
                                                   const uint8_t* base, uint32_t per,
                                                   uint64_t outer, uint64_t inner, uint64_t len,
                                                   uint8_t* hex, uint64_t hex_outer,
                                                   uint64_t pre_blk, uint8_t* pre_hex,
                                                   uint64_t pre_hex_outer,
                                                   const uint32_t* __restrict__ h0,
                                                   uint64_t blk0) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t a = i / per, b = i % per;
  ShaChain c;
  c.src = base + a * outer + b * inner;
  c.len = len;
  c.blk = h0 ? blk0 : 0;
  c.hex = hex ? hex + (a * hex_outer + b) * 64 : nullptr;
  c.pre_blk = pre_hex ? pre_blk : 0;
  c.pre_hex = pre_hex ? pre_hex + (a * pre_hex_outer + b) * 64 : nullptr;
#pragma unroll
  for (int q = 0; q < 8; ++q) c.pre_h[q] = 0;
#pragma unroll
  for (int q = 0; q < 2; ++q) c.pad_[q] = 0;
  const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                          0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  // resumed chains (h0): the state after the first blk0 blocks, computed elsewhere (the host
  // hashing fragment 0 of a segment), 8 words per chain
#pragma unroll
  for (int q = 0; q < 8; ++q) c.h[q] = h0 ? h0[8 * (size_t)i + q] : iv[q];
  tab[(uint32_t)(slot0 + i) & mask] = c;
}

void launch_sha256_hex(int sha_mode, const uint8_t* const* ptrs, const Layout* L, int nshards,
                       uint64_t n, uint64_t len, uint8_t* hex_out, hipStream_t st) {
  if (n == 0) return;
  Layout dummy{};
  const unsigned g = (unsigned)((n + 63) / 64);
  // Two waves per group while the groups leave SIMDs idle (latency regime: one serial chain
  // per buffer); one wave per group once 2 * groups would exceed the chip's 1024 SIMDs.
  // The lane-pair form (three waves per group) while those still fit one per SIMD.
  const int v = sha_mode >= 1 && sha_mode <= 3 ? sha_mode : (g <= 341 ? 3 : g <= 512 ? 2 : 1);
  if (v == 3)
    hipLaunchKernelGGL(k_sha256_2w<true>, dim3(g), dim3(192), 0, st, ptrs, L ? *L : dummy,
                       nshards, n, len, hex_out);
  else if (v == 2)
    hipLaunchKernelGGL(k_sha256_2w<false>, dim3(g), dim3(128), 0, st, ptrs, L ? *L : dummy,
                       nshards, n, len, hex_out);
  else
    hipLaunchKernelGGL(k_sha256, dim3(g), dim3(64), 0, st, ptrs, L ? *L : dummy, nshards, n, len,
                       hex_out);
}

void launch_hashq_add(ShaChain* tab, uint32_t mask, uint64_t slot0, uint32_t n,
                      const uint8_t* base, uint32_t per, uint64_t outer, uint64_t inner,
                      uint64_t len, uint8_t* hex, uint64_t hex_outer, uint64_t pre_blk,
                      uint8_t* pre_hex, uint64_t pre_hex_outer, hipStream_t st,
                      const uint32_t* h0, uint64_t blk0) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_hashq_add, dim3((n + 255) / 256), dim3(256), 0, st, tab, mask, slot0, n,
                     base, per, outer, inner, len, hex, hex_outer, pre_blk, pre_hex,
                     pre_hex_outer, h0, blk0);
}

// live chains below which the auto tick is the lane-pair form (three waves per 64 chains): at
// 32,768 chains it still hashes 823 GB/s against the two-wave tick's 693, at 65,536 783 against
// 1,366 (tools/sha_scale.py, profiles/r06/sha_scale_lp.jsonl)
constexpr uint64_t kTickLpMaxChains = 3u << 14;

void launch_sha256_tick(int tick_mode, ShaChain* tab, uint32_t mask, uint64_t head, uint32_t n,
                        uint32_t max_blocks, uint64_t live, hipStream_t st) {
  if (n == 0 || max_blocks == 0) return;
  // auto (0): the two-wave kernel while live chains are few (one wave's issue rate bounds a
  // chain), the one-wave kernel once 2^17 live chains give every SIMD several waves (measured
  // crossover, profiles/r01/sha_scale_*.jsonl)
  const int v = tick_mode >= 1 && tick_mode <= 4
                    ? tick_mode
                    : (live >= (1u << 17) ? 3 : live >= kTickLpMaxChains ? 1 : 4);
  if (v == 4)
    hipLaunchKernelGGL(k_sha256_tick_lp<1>, dim3((n + 63) / 64), dim3(192), 0, st, tab, mask,
                       head, n, max_blocks);
  else if (v == 3)
    hipLaunchKernelGGL(k_sha256_tick1<-1>, dim3((n + 63) / 64), dim3(64), 0, st, tab, mask, head,
                       n, max_blocks);
  else if (v == 2)
    hipLaunchKernelGGL(k_sha256_tick<2>, dim3((n + 63) / 64), dim3(128), 0, st, tab, mask, head,
                       n, max_blocks);
  else
    hipLaunchKernelGGL(k_sha256_tick<1>, dim3((n + 63) / 64), dim3(128), 0, st, tab, mask, head,
                       n, max_blocks);
}

}  // namespace cec
