// Host SHA-256 for SegmentList records (`Hash([u8; 64])` of
// primitives/common/src/lib.rs:16, `SegmentList` of c-pallets/file-bank/src/types.rs:13-16):
// many equal-length chains at once, on host cores.
//
// Why a host hasher beside the GPU hash queue: one SHA-256 chain is serial, and one GPU lane
// runs it ~60x slower than one SHA-NI core, so the GPU only pays with tens of
// thousands of chains in flight; an upload of a CESS file has 3 chains per 16 MiB segment. A
// host core, in turn, runs one chain latency-bound: each `sha256rnds2` waits for the previous
// one, while the unit accepts a new one every cycle or two. So a core hashes several independent
// chains at once, interleaved instruction by instruction:
//   * SHA-NI, 2 or 4 chains per core (`ni_blocks<N>`), the same two-round steps of every chain
//     issued back to back;
//   * AVX-512, 16 chains per core in the 16 dword lanes of a zmm register (`x16_blocks`): one
//     `vprord` per rotate, one `vpternlogd` per Sigma / Ch / Maj, the message words of 16 blocks
//     transposed in registers.
// Which form a core runs is measured per CPU (`cec_host_sha_probe`), not assumed. The chains of
// one call share a length (segments, fragments), so every form runs them in lock step; the tail
// (padding) blocks are built per chain on the stack.
//
// Threads: a process-wide pool of worker threads takes groups of chains from submitted jobs;
// the caller either waits for a job or polls it (the pipeline hashes a batch's chains while its
// GPU work runs). Outputs are 64 lowercase hex chars, as the GPU kernels write them.
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "host_sha.h"

namespace hsha {
namespace {

alignas(64) const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                        0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

inline uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
inline uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

// ---- portable form (CPUs without SHA-NI or AVX-512) ----------------------------------------
void scalar_blocks(uint32_t* const* st, const uint8_t* const* p, int n, size_t nblk) {
  for (int c = 0; c < n; ++c) {
    uint32_t* h = st[c];
    const uint8_t* q = p[c];
    for (size_t b = 0; b < nblk; ++b, q += 64) {
      uint32_t w[64];
      for (int t = 0; t < 16; ++t) w[t] = be32(q + 4 * t);
      for (int t = 16; t < 64; ++t) {
        const uint32_t s0 = ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3);
        const uint32_t s1 = ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
      }
      uint32_t a = h[0], bb = h[1], cc = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
      for (int t = 0; t < 64; ++t) {
        const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) +
                            K[t] + w[t];
        const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & bb) ^ (a & cc) ^ (bb & cc));
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = cc;
        cc = bb;
        bb = a;
        a = t1 + t2;
      }
      h[0] += a; h[1] += bb; h[2] += cc; h[3] += d;
      h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
  }
}

// ---- SHA-NI, N chains interleaved ------------------------------------------------------------
// State per chain in the two registers sha256rnds2 works on: ABEF and CDGH.
template <int N>
__attribute__((target("sha,sse4.1,ssse3"))) void ni_blocks(uint32_t* const* st,
                                                            const uint8_t* const* pp,
                                                            size_t nblk) {
  const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i S0[N], S1[N];
  const uint8_t* p[N];
  for (int i = 0; i < N; ++i) {
    __m128i t = _mm_loadu_si128((const __m128i*)&st[i][0]);   // A B C D (low to high)
    __m128i u = _mm_loadu_si128((const __m128i*)&st[i][4]);   // E F G H
    t = _mm_shuffle_epi32(t, 0xB1);                           // B A D C
    u = _mm_shuffle_epi32(u, 0x1B);                           // H G F E
    S0[i] = _mm_alignr_epi8(t, u, 8);                         // F E B A = ABEF
    S1[i] = _mm_blend_epi16(u, t, 0xF0);                      // H G D C = CDGH
    p[i] = pp[i];
  }
  for (size_t b = 0; b < nblk; ++b) {
    __m128i A0[N], A1[N], M[4][N];
    for (int i = 0; i < N; ++i) {
      A0[i] = S0[i];
      A1[i] = S1[i];
    }
#pragma GCC unroll 16
    for (int g = 0; g < 16; ++g) {
      const __m128i k4 = _mm_load_si128((const __m128i*)&K[4 * g]);
      for (int i = 0; i < N; ++i) {
        __m128i& w = M[g & 3][i];
        if (g < 4) {
          w = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p[i] + 16 * g)), MASK);
        } else {
          // W[t..t+3] from W[t-16..], W[t-12..], W[t-8..], W[t-4..]
          __m128i x = _mm_sha256msg1_epu32(w, M[(g + 1) & 3][i]);
          x = _mm_add_epi32(x, _mm_alignr_epi8(M[(g + 3) & 3][i], M[(g + 2) & 3][i], 4));
          w = _mm_sha256msg2_epu32(x, M[(g + 3) & 3][i]);
        }
      }
      __m128i T[N];
      for (int i = 0; i < N; ++i) T[i] = _mm_add_epi32(M[g & 3][i], k4);
      for (int i = 0; i < N; ++i) S1[i] = _mm_sha256rnds2_epu32(S1[i], S0[i], T[i]);
      for (int i = 0; i < N; ++i) T[i] = _mm_shuffle_epi32(T[i], 0x0E);
      for (int i = 0; i < N; ++i) S0[i] = _mm_sha256rnds2_epu32(S0[i], S1[i], T[i]);
    }
    for (int i = 0; i < N; ++i) {
      S0[i] = _mm_add_epi32(S0[i], A0[i]);
      S1[i] = _mm_add_epi32(S1[i], A1[i]);
      p[i] += 64;
    }
  }
  for (int i = 0; i < N; ++i) {
    __m128i t = _mm_shuffle_epi32(S0[i], 0x1B);   // A B E F -> (low to high) A B E F reversed
    __m128i u = _mm_shuffle_epi32(S1[i], 0xB1);
    const __m128i abcd = _mm_blend_epi16(t, u, 0xF0);
    const __m128i efgh = _mm_alignr_epi8(u, t, 8);
    _mm_storeu_si128((__m128i*)&st[i][0], abcd);
    _mm_storeu_si128((__m128i*)&st[i][4], efgh);
  }
}

// ---- AVX-512, 16 chains in the dword lanes ---------------------------------------------------
#define X16_TARGET __attribute__((target("avx512f,avx512bw")))

X16_TARGET inline void transpose16(__m512i r[16]) {
  __m512i t[16], u[16];
  for (int i = 0; i < 8; ++i) {
    t[2 * i] = _mm512_unpacklo_epi32(r[2 * i], r[2 * i + 1]);
    t[2 * i + 1] = _mm512_unpackhi_epi32(r[2 * i], r[2 * i + 1]);
  }
  for (int q = 0; q < 4; ++q) {  // rows 4q..4q+3
    __m512i* a = &t[4 * q];
    u[4 * q + 0] = _mm512_unpacklo_epi64(a[0], a[2]);  // column 4L+0 of the four rows
    u[4 * q + 1] = _mm512_unpackhi_epi64(a[0], a[2]);  // 4L+1
    u[4 * q + 2] = _mm512_unpacklo_epi64(a[1], a[3]);  // 4L+2
    u[4 * q + 3] = _mm512_unpackhi_epi64(a[1], a[3]);  // 4L+3
  }
  for (int c = 0; c < 4; ++c) {
    const __m512i v0 = _mm512_shuffle_i32x4(u[c], u[4 + c], 0x88);
    const __m512i v1 = _mm512_shuffle_i32x4(u[c], u[4 + c], 0xDD);
    const __m512i w0 = _mm512_shuffle_i32x4(u[8 + c], u[12 + c], 0x88);
    const __m512i w1 = _mm512_shuffle_i32x4(u[8 + c], u[12 + c], 0xDD);
    r[c] = _mm512_shuffle_i32x4(v0, w0, 0x88);
    r[c + 8] = _mm512_shuffle_i32x4(v0, w0, 0xDD);
    r[c + 4] = _mm512_shuffle_i32x4(v1, w1, 0x88);
    r[c + 12] = _mm512_shuffle_i32x4(v1, w1, 0xDD);
  }
}

X16_TARGET void x16_blocks(uint32_t* const* st, const uint8_t* const* pp, size_t nblk) {
  alignas(64) uint32_t tmp[8][16];
  for (int c = 0; c < 16; ++c)
    for (int j = 0; j < 8; ++j) tmp[j][c] = st[c][j];
  __m512i s[8];
  for (int j = 0; j < 8; ++j) s[j] = _mm512_load_si512(tmp[j]);
  const __m512i BSWAP = _mm512_set4_epi32(0x0c0d0e0f, 0x08090a0b, 0x04050607, 0x00010203);
  const uint8_t* p[16];
  for (int c = 0; c < 16; ++c) p[c] = pp[c];
  for (size_t b = 0; b < nblk; ++b) {
    __m512i w[16];
    for (int c = 0; c < 16; ++c) w[c] = _mm512_loadu_si512((const void*)p[c]);
    transpose16(w);
    for (int t = 0; t < 16; ++t) w[t] = _mm512_shuffle_epi8(w[t], BSWAP);
    __m512i a = s[0], bb = s[1], cc = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma GCC unroll 64
    for (int t = 0; t < 64; ++t) {
      if (t >= 16) {
        const __m512i x15 = w[(t - 15) & 15], x2 = w[(t - 2) & 15];
        const __m512i s0 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(x15, 7),
                                                     _mm512_ror_epi32(x15, 18),
                                                     _mm512_srli_epi32(x15, 3), 0x96);
        const __m512i s1 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(x2, 17),
                                                     _mm512_ror_epi32(x2, 19),
                                                     _mm512_srli_epi32(x2, 10), 0x96);
        w[t & 15] = _mm512_add_epi32(_mm512_add_epi32(w[t & 15], s0),
                                     _mm512_add_epi32(w[(t - 7) & 15], s1));
      }
      const __m512i S1 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(e, 6), _mm512_ror_epi32(e, 11),
                                                   _mm512_ror_epi32(e, 25), 0x96);
      const __m512i ch = _mm512_ternarylogic_epi32(e, f, g, 0xCA);
      const __m512i kw = _mm512_add_epi32(w[t & 15], _mm512_set1_epi32((int)K[t]));
      const __m512i t1 = _mm512_add_epi32(_mm512_add_epi32(h, S1), _mm512_add_epi32(ch, kw));
      const __m512i S0 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(a, 2), _mm512_ror_epi32(a, 13),
                                                   _mm512_ror_epi32(a, 22), 0x96);
      const __m512i mj = _mm512_ternarylogic_epi32(a, bb, cc, 0xE8);
      h = g;
      g = f;
      f = e;
      e = _mm512_add_epi32(d, t1);
      d = cc;
      cc = bb;
      bb = a;
      a = _mm512_add_epi32(t1, _mm512_add_epi32(S0, mj));
    }
    s[0] = _mm512_add_epi32(s[0], a);
    s[1] = _mm512_add_epi32(s[1], bb);
    s[2] = _mm512_add_epi32(s[2], cc);
    s[3] = _mm512_add_epi32(s[3], d);
    s[4] = _mm512_add_epi32(s[4], e);
    s[5] = _mm512_add_epi32(s[5], f);
    s[6] = _mm512_add_epi32(s[6], g);
    s[7] = _mm512_add_epi32(s[7], h);
    for (int c = 0; c < 16; ++c) p[c] += 64;
  }
  for (int j = 0; j < 8; ++j) _mm512_store_si512(tmp[j], s[j]);
  for (int c = 0; c < 16; ++c)
    for (int j = 0; j < 8; ++j) st[c][j] = tmp[j][c];
}

bool has_ni() {
  static const bool v = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
  return v;
}
bool has_x16() {
  static const bool v = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
  return v;
}

// Group width of a form (chains advanced together by one call of its block function).
int form_width(int form) {
  switch (form) {
    case CEC_HSHA_NI1: return 1;
    case CEC_HSHA_NI2: return 2;
    case CEC_HSHA_NI4: return 4;
    case CEC_HSHA_X16: return 16;
    default: return 1;
  }
}

// Advance n (<= the form's width) chains by nblk full blocks.
void blocks(int form, uint32_t* const* st, const uint8_t* const* p, int n, size_t nblk) {
  if (!nblk || !n) return;
  if (form == CEC_HSHA_X16 && n == 16) return x16_blocks(st, p, nblk);
  if (form == CEC_HSHA_NI4 && n == 4) return ni_blocks<4>(st, p, nblk);
  if (form != CEC_HSHA_SCALAR && has_ni()) {
    int c = 0;
    for (; c + 2 <= n && form != CEC_HSHA_NI1; c += 2) ni_blocks<2>(st + c, p + c, nblk);
    for (; c < n; ++c) ni_blocks<1>(st + c, p + c, nblk);
    return;
  }
  scalar_blocks(st, p, n, nblk);
}

std::atomic<int> g_form{-1};

int best_form() {
  int f = g_form.load(std::memory_order_relaxed);
  if (f >= 0) return f;
  // the default: 16 chains per core in AVX-512 lanes where present (5.5 GB/s per core on the
  // EPYC 9575F against 3.6 for SHA-NI x2, profiles/r06/host_sha_probe.jsonl), else SHA-NI x2
  return has_x16() ? CEC_HSHA_X16 : (has_ni() ? CEC_HSHA_NI2 : CEC_HSHA_SCALAR);
}

bool form_supported(int form) {
  switch (form) {
    case CEC_HSHA_SCALAR: return true;
    case CEC_HSHA_NI1:
    case CEC_HSHA_NI2:
    case CEC_HSHA_NI4: return has_ni();
    case CEC_HSHA_X16: return has_x16();
    default: return false;
  }
}

void to_hex(const uint32_t h[8], uint8_t* out) {
  static const char* hx = "0123456789abcdef";
  for (int j = 0; j < 8; ++j)
    for (int b = 0; b < 4; ++b) {
      const uint8_t v = (uint8_t)(h[j] >> (24 - 8 * b));
      out[8 * j + 2 * b] = (uint8_t)hx[v >> 4];
      out[8 * j + 2 * b + 1] = (uint8_t)hx[v & 15];
    }
}

// Padding blocks of a message of `len` bytes whose last len % 64 bytes are `tail`: 1 or 2 blocks.
int pad_blocks(const uint8_t* tail, size_t len, uint8_t out[128]) {
  const size_t r = len & 63;
  std::memset(out, 0, 128);
  if (r) std::memcpy(out, tail, r);
  out[r] = 0x80;
  const int nb = r >= 56 ? 2 : 1;
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) out[64 * nb - 1 - i] = (uint8_t)(bits >> (8 * i));
  return nb;
}

}  // namespace

// Hash chains [c0, c0 + n) of a job on the calling thread, in groups of the form's width.
void hash_range(const Job& j, size_t c0, size_t n, int form) {
  const int W = form_width(form);
  for (size_t g0 = c0; g0 < c0 + n; g0 += W) {
    const int gn = (int)std::min<size_t>(W, c0 + n - g0);
    uint32_t state[16][8];
    uint32_t* st[16];
    const uint8_t* p[16];
    for (int c = 0; c < gn; ++c) {
      std::memcpy(state[c], IV, sizeof IV);
      st[c] = state[c];
      p[c] = j.bufs[g0 + c];
    }
    // a narrower group (the job's last) runs the widest form that fits
    const int f = gn == W ? form : (has_ni() && form != CEC_HSHA_SCALAR ? CEC_HSHA_NI2
                                                                         : CEC_HSHA_SCALAR);
    size_t done = 0;
    if (j.prefix_len) {
      const size_t pb = j.prefix_len / 64;
      blocks(f, st, p, gn, pb);
      done = pb;
      // the prefix digest: a copy of the state finished with the prefix's padding block
      uint32_t pst[16][8];
      uint32_t* pp_[16];
      uint8_t pad[16][128];
      const uint8_t* pq[16];
      for (int c = 0; c < gn; ++c) {
        std::memcpy(pst[c], state[c], sizeof pst[c]);
        pp_[c] = pst[c];
        pad_blocks(nullptr, j.prefix_len, pad[c]);
        pq[c] = pad[c];
      }
      blocks(f, pp_, pq, gn, 1);
      for (int c = 0; c < gn; ++c) to_hex(pst[c], j.prefix_hex + ((g0 + c) / j.per * j.prefix_outer + (g0 + c) % j.per) * 64);
      for (int c = 0; c < gn; ++c) p[c] += pb * 64;
    }
    const size_t full = j.len / 64;
    blocks(f, st, p, gn, full - done);
    if (j.state_out)
      for (int c = 0; c < gn; ++c) std::memcpy(j.state_out + 8 * (g0 + c), state[c], 32);
    uint8_t pad[16][128];
    const uint8_t* pq[16];
    int nb = 1;
    for (int c = 0; c < gn; ++c) {
      nb = pad_blocks(j.bufs[g0 + c] + full * 64, j.len, pad[c]);
      pq[c] = pad[c];
    }
    blocks(f, st, pq, gn, nb);
    for (int c = 0; c < gn; ++c)
      to_hex(state[c], j.hex + ((g0 + c) / j.per * j.hex_outer + (g0 + c) % j.per) * 64);
  }
}

// ---- the worker pool ---------------------------------------------------------------------------
// Jobs queue in submission order. A job of the x16 form is handed out chain by chain: a worker
// keeps up to 16 chains in the lanes of its zmm registers and refills a lane as soon as its
// chain ends (the multi-buffer scheme), so the lanes stay full across the different lengths of
// one batch's chains (16 MiB segments, 8 MiB fragments) and across jobs. With fewer chains than
// that in its lanes a worker advances them on SHA-NI two at a time instead (x16 on n lanes does
// n/16 of its work; SHA-NI x2 beats it below ~11 lanes, by the per-thread rates of
// profiles/r06/host_sha_probe.jsonl), and chains are shared out among idle workers. Jobs of the
// other forms are handed out as tasks of whole groups.
namespace {

constexpr int kLanes = 16;
constexpr uint64_t kStepBlocks = 1024;  // lanes are refilled at least every 64 KiB per lane
constexpr int kMinX16Lanes = 11;
alignas(64) const uint8_t kZeros[kStepBlocks * 64] = {};

void one_lane_blocks(uint32_t* st, const uint8_t* p, size_t nblk) {
  uint32_t* s1[1] = {st};
  const uint8_t* p1[1] = {p};
  blocks(has_ni() ? CEC_HSHA_NI1 : CEC_HSHA_SCALAR, s1, p1, 1, nblk);
}

void chain_done(const std::shared_ptr<JobState>& js) {
  if (js->left.fetch_sub(1, std::memory_order_acq_rel) == 1) {
    std::lock_guard<std::mutex> l(js->mu);
    js->done = true;
    js->cv.notify_all();
  }
}

struct Lane {
  std::shared_ptr<JobState> js;
  size_t ci = 0;
  const uint8_t* p = nullptr;
  uint64_t done = 0, full = 0, pre = 0;  // blocks hashed, full blocks, prefix blocks (0: none)
  bool pre_done = true;
  uint32_t st[8];

  void start(std::shared_ptr<JobState> j, size_t c) {
    js = std::move(j);
    ci = c;
    p = js->job.bufs[c];
    done = 0;
    full = js->job.len / 64;
    pre = js->job.prefix_len / 64;
    pre_done = pre == 0;
    std::memcpy(st, IV, sizeof IV);
  }
  uint64_t to_event() const { return (pre_done ? full : pre) - done; }
  // the prefix digest: a copy of the state finished with the prefix's padding block
  void prefix() {
    const Job& j = js->job;
    uint32_t c[8];
    std::memcpy(c, st, sizeof c);
    uint8_t pad[128];
    pad_blocks(nullptr, j.prefix_len, pad);
    one_lane_blocks(c, pad, 1);
    to_hex(c, j.prefix_hex + (ci / j.per * j.prefix_outer + ci % j.per) * 64);
    pre_done = true;
  }
  void finish() {
    const Job& j = js->job;
    if (j.state_out) std::memcpy(j.state_out + 8 * ci, st, 32);
    uint8_t pad[128];
    const int nb = pad_blocks(j.bufs[ci] + full * 64, j.len, pad);
    one_lane_blocks(st, pad, (size_t)nb);
    to_hex(st, j.hex + (ci / j.per * j.hex_outer + ci % j.per) * 64);
    chain_done(js);
    js.reset();
  }
};

struct Counters {
  std::atomic<uint64_t> busy_ns{0}, lane_blocks{0}, x16_steps{0}, ni_steps{0}, x16_lanes{0},
      spilled{0};
} g_count;

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Advance the n active lanes by `step` blocks (step <= each lane's blocks to its next event).
void step_lanes(Lane* L, int n, uint64_t step) {
  if (!step) return;
  g_count.lane_blocks.fetch_add(step * (uint64_t)n, std::memory_order_relaxed);
  uint32_t* st[kLanes];
  const uint8_t* p[kLanes];
  if (n >= kMinX16Lanes && has_x16()) {
    uint32_t dummy[kLanes][8];
    for (int i = 0; i < kLanes; ++i) {
      st[i] = i < n ? L[i].st : dummy[i];
      p[i] = i < n ? L[i].p : kZeros;
    }
    x16_blocks(st, p, step);
    g_count.x16_steps.fetch_add(1, std::memory_order_relaxed);
    g_count.x16_lanes.fetch_add((uint64_t)n, std::memory_order_relaxed);
  } else {
    g_count.ni_steps.fetch_add(1, std::memory_order_relaxed);
    for (int i = 0; i < n; ++i) {
      st[i] = L[i].st;
      p[i] = L[i].p;
    }
    blocks(CEC_HSHA_NI2, st, p, n, step);
  }
  for (int i = 0; i < n; ++i) {
    L[i].done += step;
    L[i].p += step * 64;
  }
}

struct Pool {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::shared_ptr<JobState>> q;  // jobs with chains / tasks not yet handed out
  std::deque<Lane> spill;                   // chains in progress given back by a worker
  std::vector<std::thread> th;
  int idle = 0;
  size_t lanes_busy = 0;  // chains in the workers' lanes
  size_t avail = 0;       // x16 chains not yet in any lane (queued jobs' chains + spill)
  bool stop = false;

  ~Pool() {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  int reserved = 0;  // threads the live pipelines asked for (reserve_threads), summed
  void grow(int n) {
    std::lock_guard<std::mutex> l(mu);
    n = std::max(n, reserved);
    while ((int)th.size() < n) th.emplace_back([this] { loop(); });
  }
  // (under mu) chains of x16 jobs into free lanes. With enough chains for every worker to fill
  // kMinX16Lanes lanes, a worker fills all 16 (x16 at 5.5 GB/s per core beats SHA-NI x2's 3.6
  // once a worker holds 11 chains: 256 chains of 16 MiB on 16 threads 88.6 GB/s,
  // profiles/r06/host_sha_probe_4g.jsonl); with fewer, the chains are shared out among the idle
  // workers, who run them on SHA-NI (spreading 64 chains over 16 threads beats 4 full registers).
  // Chains a worker gave back (spill) go first.
  void take_chains(Lane* L, int& n) {
    if (!avail) return;
    size_t want = (size_t)(kLanes - n);
    const bool plenty = avail + lanes_busy >= (size_t)kMinX16Lanes * th.size();
    if (idle > 0 && !plenty)
      want = std::min(want, std::max<size_t>(1, (avail + idle) / (idle + 1)));
    want = std::min(want, avail);
    lanes_busy += want;
    avail -= want;
    while (want && !spill.empty()) {
      L[n++] = std::move(spill.front());
      spill.pop_front();
      --want;
    }
    for (auto it = q.begin(); it != q.end() && want;) {
      auto& js = *it;
      if (js->form != CEC_HSHA_X16) {
        ++it;
        continue;
      }
      while (want && js->next < js->job.n) {
        L[n++].start(js, js->next++);
        --want;
      }
      if (js->next == js->job.n)
        it = q.erase(it);
      else
        ++it;
    }
  }
  // A worker whose lanes hold more than its share of the chains in flight while other workers
  // idle and nothing is queued (a job's last chains, all taken greedily by a few workers: 32
  // chains of 16 MiB on two x16 registers take 48 ms, on 16 cores' SHA-NI 9 ms) gives the
  // surplus back; idle workers pick it up at once, the others at their next step. (under mu)
  void rebalance(Lane* L, int& n) {
    static const bool off = getenv("CEC_HOST_SHA_NO_SPILL") != nullptr;  // A/B measurements
    if (off || n <= 1 || idle == 0 || avail) return;
    const size_t fair = std::max<size_t>(1, (lanes_busy + th.size() - 1) / th.size());
    if ((size_t)n <= fair) return;
    // keep the lanes closest to their end; give back the longest
    std::sort(L, L + n, [](const Lane& a, const Lane& b) {
      return a.full - a.done < b.full - b.done;
    });
    const int give = n - (int)fair;
    for (int i = (int)fair; i < n; ++i) spill.push_back(std::move(L[i]));
    n = (int)fair;
    lanes_busy -= (size_t)give;
    avail += (size_t)give;
    g_count.spilled.fetch_add((uint64_t)give, std::memory_order_relaxed);
    cv.notify_all();
  }
  // (under mu) a task of groups from the oldest job of another form
  bool take_task(std::shared_ptr<JobState>& js, size_t& c0, size_t& cn) {
    for (auto it = q.begin(); it != q.end(); ++it) {
      if ((*it)->form == CEC_HSHA_X16) continue;
      js = *it;
      const size_t W = (size_t)form_width(js->form);
      c0 = js->next;
      cn = std::min(js->job.n - c0, js->per_task * W);
      js->next += cn;
      if (js->next == js->job.n) q.erase(it);
      return true;
    }
    return false;
  }

  void loop() {
    Lane L[kLanes];
    int n = 0;
    size_t finished = 0;  // lanes freed since this worker last held the lock
    while (true) {
      std::shared_ptr<JobState> tjs;
      size_t t0 = 0, tn = 0;
      {
        std::unique_lock<std::mutex> l(mu);
        lanes_busy -= finished;
        finished = 0;
        while (true) {
          if (n < kLanes) take_chains(L, n);
          if (n) {
            rebalance(L, n);
            break;
          }
          if (take_task(tjs, t0, tn)) break;
          if (stop) return;
          ++idle;
          cv.wait(l);
          --idle;
        }
      }
      const uint64_t b0 = now_ns();
      if (tjs) {
        hash_range(tjs->job, t0, tn, tjs->form);
        g_count.busy_ns.fetch_add(now_ns() - b0, std::memory_order_relaxed);
        // tasks count as one unit each in `left`
        chain_done(tjs);
        continue;
      }
      uint64_t step = kStepBlocks;
      for (int i = 0; i < n; ++i) step = std::min(step, L[i].to_event());
      step_lanes(L, n, step);
      g_count.busy_ns.fetch_add(now_ns() - b0, std::memory_order_relaxed);
      for (int i = 0; i < n; ++i) {
        if (!L[i].pre_done && L[i].done == L[i].pre) L[i].prefix();
        if (L[i].pre_done && L[i].done == L[i].full) {
          L[i].finish();
          if (i != n - 1) std::swap(L[i], L[n - 1]);
          --n;
          --i;
          ++finished;
        }
      }
    }
  }
};

Pool& pool() {
  static Pool* p = new Pool;  // never destroyed: workers may outlive static destruction order
  return *p;
}

}  // namespace

std::shared_ptr<JobState> submit(const Job& job, int threads) {
  auto js = std::make_shared<JobState>();
  js->job = job;
  js->form = best_form();
  if (!job.n) {
    js->done = true;
    return js;
  }
  threads = std::max(1, threads);
  if (js->form == CEC_HSHA_X16) {
    js->left.store((int)job.n);  // one unit per chain
  } else {
    // tasks of whole groups; a few per thread so a slow core does not hold the job
    const size_t W = (size_t)form_width(js->form);
    const size_t groups = (job.n + W - 1) / W;
    js->per_task = std::max<size_t>(1, groups / ((size_t)threads * 2));
    js->left.store((int)((groups + js->per_task - 1) / js->per_task));
  }
  Pool& P = pool();
  P.grow(threads);
  {
    std::lock_guard<std::mutex> l(P.mu);
    P.q.push_back(js);
    if (js->form == CEC_HSHA_X16) P.avail += job.n;
  }
  P.cv.notify_all();
  return js;
}

bool ready(const std::shared_ptr<JobState>& js) {
  return js->left.load(std::memory_order_acquire) == 0 || js->done;
}

void wait(const std::shared_ptr<JobState>& js, bool) {
  std::unique_lock<std::mutex> l(js->mu);
  js->cv.wait(l, [&] { return js->done; });
}

PoolStats stats() {
  PoolStats s;
  s.busy_s = 1e-9 * (double)g_count.busy_ns.load();
  s.lane_blocks = g_count.lane_blocks.load();
  s.x16_steps = g_count.x16_steps.load();
  s.ni_steps = g_count.ni_steps.load();
  s.x16_lane_steps = g_count.x16_lanes.load();
  s.spilled = g_count.spilled.load();
  return s;
}

// Several pipelines in one process (one per GPU, encode_file_records_multi) each bring their own
// thread count: the pool holds their sum, not the largest one. Threads are never ended; a
// released reservation leaves them idle.
void reserve_threads(int n) {
  Pool& P = pool();
  {
    std::lock_guard<std::mutex> l(P.mu);
    P.reserved += std::max(0, n);
  }
  P.grow(0);
}
void release_threads(int n) {
  Pool& P = pool();
  std::lock_guard<std::mutex> l(P.mu);
  P.reserved = std::max(0, P.reserved - std::max(0, n));
}
int pool_threads() {
  Pool& P = pool();
  std::lock_guard<std::mutex> l(P.mu);
  return (int)P.th.size();
}

void set_form(int form) { g_form.store(form); }
int get_form() { return best_form(); }
bool supported(int form) { return form_supported(form); }

}  // namespace hsha

extern "C" {

int cec_sha256_host(const uint8_t* const* bufs, size_t n, size_t len, uint8_t* hex,
                    size_t prefix_len, uint8_t* prefix_hex, int threads) {
  if (n && (!bufs || !hex)) return CEC_EINVAL;
  if (prefix_len && (!prefix_hex || prefix_len % 64 || prefix_len > len)) return CEC_EINVAL;
  hsha::Job j;
  j.bufs = bufs;
  j.n = n;
  j.len = len;
  j.hex = hex;
  j.prefix_len = prefix_hex ? prefix_len : 0;
  j.prefix_hex = prefix_hex;
  if (threads <= 1) {
    hsha::hash_range(j, 0, n, hsha::best_form());
    return 0;
  }
  auto js = hsha::submit(j, threads);
  hsha::wait(js, true);
  return 0;
}

int cec_sha256_host_state(const uint8_t* const* bufs, size_t n, size_t len, uint8_t* hex,
                          uint32_t* state_out, int threads) {
  if (n && (!bufs || !hex || !state_out)) return CEC_EINVAL;
  if (len % 64) return CEC_EINVAL;
  hsha::Job j;
  j.bufs = bufs;
  j.n = n;
  j.len = len;
  j.hex = hex;
  j.state_out = state_out;
  if (threads <= 1) {
    hsha::hash_range(j, 0, n, hsha::best_form());
    return 0;
  }
  auto js = hsha::submit(j, threads);
  hsha::wait(js, true);
  return 0;
}

int cec_host_sha_set_form(int form) {
  if (form < 0) {
    hsha::set_form(-1);
    return 0;
  }
  if (!hsha::supported(form)) return CEC_EINVAL;
  hsha::set_form(form);
  return 0;
}

int cec_host_sha_form(void) { return hsha::get_form(); }

int cec_host_sha_pool_threads(void) { return hsha::pool_threads(); }

double cec_host_sha_probe(int form, size_t bytes_per_chain, int chains) {
  if (!hsha::supported(form) || chains < 1) return -1.0;
  const size_t len = std::max<size_t>(64, bytes_per_chain & ~(size_t)63);
  std::vector<uint8_t> buf(len * (size_t)chains);
  for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 131 + 7);
  std::vector<const uint8_t*> p(chains);
  for (int c = 0; c < chains; ++c) p[c] = buf.data() + (size_t)c * len;
  std::vector<uint8_t> hex(64 * (size_t)chains);
  hsha::Job j;
  j.bufs = p.data();
  j.n = (size_t)chains;
  j.len = len;
  j.hex = hex.data();
  const auto t0 = std::chrono::steady_clock::now();
  hsha::hash_range(j, 0, j.n, form);
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return (double)len * chains / s / 1e9;
}

}  // extern "C"
