// HIP kernels for the CESS segment -> fragment Reed-Solomon codec on MI355X (gfx950, CDNA4).
//
// Everything here is HBM-streaming integer work: a GF(2^8) matrix-vector product over byte
// columns ("out[r] = XOR_j c[r][j] * in[j]") for encode and reconstruct, a per-fragment SHA-256,
// and a counter-based synthetic-data generator (SHA-256 lives in sha256.hip). There is no MFMA: GF(2^8) multiply-accumulate
// is not a float contraction.
//
// GF multiply by a constant is done without tables: 2*x on four packed bytes is one "xtime"
// (shift, mask, conditional reduction by 0x1D = 6 VALU ops per dword), and c*x is the XOR of
// the xtime powers 2^b*x selected by the set bits of c.
//  * Compile-time coefficient kernels (k_ct): the coefficient matrix is a constexpr of the
//    template, so after unrolling only the XORs for set bits are emitted (about 0.5 VALU op per
//    byte per coefficient). Small input counts use a Horner form per output row
//    (y = 2*y ^ XOR_{j: bit b of c[r][j]} x_j, b = 7..0), large ones stream the inputs and keep
//    one accumulator per output.
//  * Run-time coefficient kernel (k_rt): coefficients arrive through scalar loads and are
//    expanded to per-bit masks on the SALU; each (input, output, bit) is one v_bitop3
//    (acc ^= pow_b & mask_b).
// Each lane owns 16-byte columns (global_load_dwordx4) of every shard; blockIdx.y is the
// segment. A shard length that is not a multiple of 16 is finished byte-wise by the last block.
#include <utility>

#include "dev_util.h"
#include "gf256.h"
#include "kernels.h"

namespace cec {


// Every lambda on the compile-time path is force-inlined: an outlined body turns into a call
// with the Layout spilled to scratch.
#define CEC_AI __attribute__((always_inline))

// 2*x in GF(2^8)/0x11D on four packed bytes (5 VALU ops). The reduction mask (0xFF in every
// byte whose top bit is set) comes from one v_perm_b32: selectors 8..11 replicate the sign bit
// of bytes 1, 3, 5, 7 of {S0, S1}; with S1 = x << 8 those are x's bytes 0 and 2, with S0 = x its
// bytes 1 and 3.
__device__ __forceinline__ uint32_t xt(uint32_t x) {
  const uint32_t sign = __builtin_amdgcn_perm(x, x << 8, 0x0B090A08u);
  return __builtin_amdgcn_bitop3_b32((x & 0x7f7f7f7fu) << 1, sign, 0x1d1d1d1du, 0x78);  // a ^ (b & c)
}
__device__ __forceinline__ u32x2 xt(u32x2 x) { return u32x2{xt(x.x), xt(x.y)}; }
__device__ __forceinline__ u32x4 xt(u32x4 x) {
  return u32x4{xt(x.x), xt(x.y), xt(x.z), xt(x.w)};
}


// Shard pointer with the data/parity split known at compile time (K = data shard count).
template <int K, int IDX>
__device__ __forceinline__ uint8_t* shard_ptr_ct(const Layout& L, uint32_t seg) {
  if constexpr (IDX < K) return L.data + seg * L.data_seg_stride + (uint64_t)IDX * L.shard_stride;
  else return L.parity + seg * L.par_seg_stride + (uint64_t)(IDX - K) * L.shard_stride;
}

template <bool NT, class TV = u32x4>
__device__ __forceinline__ TV ld16(const uint8_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const TV*>(p));
  else return *reinterpret_cast<const TV*>(p);
}
template <bool NT, class TV = u32x4>
__device__ __forceinline__ void st16(uint8_t* p, TV v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<TV*>(p));
  else *reinterpret_cast<TV*>(p) = v;
}

// ---------------------------------------------------------------------------------------------
// Compile-time plans
// ---------------------------------------------------------------------------------------------
template <int NI, int NO>
struct CoefCT {
  uint8_t c[NO][NI];
  uint8_t in[NI];
  uint8_t out[NO];
  int8_t hb_col[NI];  // highest set bit over column j (-1 if the column is zero)
  int8_t hb_row[NO];  // highest set bit over row r
};

constexpr int hibit(unsigned c) {
  int h = -1;
  for (int b = 0; b < 8; ++b)
    if (c >> b & 1) h = b;
  return h;
}

template <int NI, int NO>
constexpr void finish_ct(CoefCT<NI, NO>& r) {
  for (int j = 0; j < NI; ++j) {
    int h = -1;
    for (int o = 0; o < NO; ++o) h = hibit(r.c[o][j]) > h ? hibit(r.c[o][j]) : h;
    r.hb_col[j] = (int8_t)h;
  }
  for (int o = 0; o < NO; ++o) {
    int h = -1;
    for (int j = 0; j < NI; ++j) h = hibit(r.c[o][j]) > h ? hibit(r.c[o][j]) : h;
    r.hb_row[o] = (int8_t)h;
  }
}

template <int K, int M>
constexpr CoefCT<K, M> make_encode_ct() {
  Mat<64, 64> e, top, topinv;
  Mat<64, 128> work;
  gf_encode_matrix(K, M, e, top, topinv, work);
  CoefCT<K, M> r{};
  for (int o = 0; o < M; ++o)
    for (int j = 0; j < K; ++j) r.c[o][j] = e.v[K + o][j];
  for (int j = 0; j < K; ++j) r.in[j] = (uint8_t)j;
  for (int o = 0; o < M; ++o) r.out[o] = (uint8_t)(K + o);
  finish_ct(r);
  return r;
}

// Single-erasure decode of RS(K, M): survivors are the first K present shards.
template <int K, int M, int MISSING>
constexpr CoefCT<K, 1> make_decode1_ct() {
  Mat<64, 64> e, top, topinv, sub, inv;
  Mat<64, 128> work;
  gf_encode_matrix(K, M, e, top, topinv, work);
  uint8_t present[64] = {};
  for (int i = 0; i < K + M; ++i) present[i] = i != MISSING;
  Plan<64, 64> p;
  gf_decode_plan(K, M, present, false, e, p, sub, inv, work);
  CoefCT<K, 1> r{};
  for (int j = 0; j < K; ++j) r.c[0][j] = p.coef.v[0][j];
  for (int j = 0; j < K; ++j) r.in[j] = p.in_idx[j];
  r.out[0] = p.out_idx[0];
  finish_ct(r);
  return r;
}

template <int K_, int M>
struct EncCT {
  static constexpr int K = K_;
  static constexpr int NI = K_, NO = M;
  static constexpr CoefCT<K_, M> v = make_encode_ct<K_, M>();
};
template <int K_, int M, int MISSING>
struct Dec1CT {
  static constexpr int K = K_;
  static constexpr int NI = K_, NO = 1;
  static constexpr CoefCT<K, 1> v = make_decode1_ct<K_, M, MISSING>();
};

// Horner form pays one xtime per bit of the largest row coefficient; the streaming form one per
// bit of the largest column coefficient. Horner needs every input column resident.
template <class P>
constexpr bool use_horner(int u) {
  int ch = 0, cp = 0;
  for (int o = 0; o < P::NO; ++o) ch += P::v.hb_row[o] > 0 ? P::v.hb_row[o] : 0;
  for (int j = 0; j < P::NI; ++j) cp += P::v.hb_col[j] > 0 ? P::v.hb_col[j] : 0;
  return P::NI <= 8 && P::NI * u * 4 <= 64 && ch <= cp;
}

// Compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1, fully expanded, so the
// coefficient reads below are constant expressions and only the XORs of set bits are emitted.
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) CEC_AI {
    (f(std::integral_constant<int, I>{}), ...);
  }(std::make_integer_sequence<int, N>{});
}

// XOR helpers on v_bitop3 (truth table 0x96 = a ^ b ^ c). The intrinsic is opaque to LLVM's
// reassociation, which would otherwise rebuild the per-output XOR chains as trees over every
// input power and keep them all live (hundreds of VGPRs, scratch spills on wide codes).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ u32x4 xor3(u32x4 a, u32x4 b, u32x4 c) {
  return u32x4{xor3(a.x, b.x, c.x), xor3(a.y, b.y, c.y), xor3(a.z, b.z, c.z),
               xor3(a.w, b.w, c.w)};
}
__device__ __forceinline__ u32x2 xor3(u32x2 a, u32x2 b, u32x2 c) {
  return u32x2{xor3(a.x, b.x, c.x), xor3(a.y, b.y, c.y)};
}
template <class T>
__device__ __forceinline__ T xor2(T a, T b) {
  return xor3(a, b, T(0));
}
// a ^ (b & m), m a wave-uniform mask (truth table 0x78)
__device__ __forceinline__ uint32_t bitop3_xand(uint32_t a, uint32_t b, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(a, b, m, 0x78);
}
__device__ __forceinline__ u32x2 bitop3_xand(u32x2 a, u32x2 b, uint32_t m) {
  return u32x2{bitop3_xand(a.x, b.x, m), bitop3_xand(a.y, b.y, m)};
}
__device__ __forceinline__ u32x4 bitop3_xand(u32x4 a, u32x4 b, uint32_t m) {
  return u32x4{bitop3_xand(a.x, b.x, m), bitop3_xand(a.y, b.y, m), bitop3_xand(a.z, b.z, m),
               bitop3_xand(a.w, b.w, m)};
}

struct BitList {
  int n;
  int b[8];
};
constexpr BitList set_bits(unsigned c) {
  BitList r{};
  for (int b = 0; b < 8; ++b)
    if (c >> b & 1) r.b[r.n++] = b;
  return r;
}

// acc ^= XOR of p[b] over the set bits b of constant C, two terms per v_bitop3.
template <unsigned C, class T>
__device__ __forceinline__ T mul_acc(T acc, const T (&p)[8]) {
  constexpr BitList bl = set_bits(C);
  static_for<(bl.n + 1) / 2>([&](auto Q) CEC_AI {
    constexpr int q = Q;
    if constexpr (2 * q + 1 < bl.n) acc = xor3(acc, p[bl.b[2 * q]], p[bl.b[2 * q + 1]]);
    else acc = xor2(acc, p[bl.b[2 * q]]);
  });
  return acc;
}

// out = C * x for one column element of type T (u32x4 for the vector body, uint32_t bytes for
// the tail). `ld(J)` returns input column J, `st(O, y)` stores output O (J, O integral
// constants).
template <class P, class T, class LD, class ST>
__device__ __forceinline__ void ct_column_horner(LD ld, ST st) {
  T x[P::NI];
  static_for<P::NI>([&](auto J) CEC_AI { x[J] = ld(J); });
  static_for<P::NO>([&](auto O) CEC_AI {
    constexpr int o = O;
    T y = T(0);
    static_for<8>([&](auto B) CEC_AI {
      constexpr int b = 7 - B;
      if constexpr (b < P::v.hb_row[o]) y = xt(y);
      // inputs whose coefficient has bit b set, XORed two at a time
      constexpr auto sel = [] {
        BitList r{};  // reuse as an index list (NI <= 8 here)
        int n = 0;
        int idx[P::NI] = {};
        for (int j = 0; j < P::NI; ++j)
          if ((P::v.c[o][j] >> b) & 1) idx[n++] = j;
        r.n = n;
        for (int t = 0; t < n && t < 8; ++t) r.b[t] = idx[t];
        return r;
      }();
      static_assert(sel.n <= 8, "Horner form is for narrow codes");
      static_for<(sel.n + 1) / 2>([&](auto Q) CEC_AI {
        constexpr int q = Q;
        if constexpr (2 * q + 1 < sel.n) y = xor3(y, x[sel.b[2 * q]], x[sel.b[2 * q + 1]]);
        else y = xor2(y, x[sel.b[2 * q]]);
      });
    });
    st(O, y);
  });
}

// Streaming form for wide codes: one accumulator per output, input columns consumed in order.
// PF input loads are kept in flight (a static register ring): column j+PF is issued before
// column j is multiplied in, so HBM latency hides behind the XOR work of PF columns.
template <class P, int PF, class T, class LD, class ST>
__device__ __forceinline__ void ct_column_stream(LD ld, ST st) {
  T acc[P::NO];
  T ring[PF];
  static_for<P::NO>([&](auto O) CEC_AI { acc[O] = T(0); });
  static_for<(PF < P::NI ? PF : P::NI)>([&](auto J) CEC_AI { ring[J] = ld(J); });
  static_for<P::NI>([&](auto J) CEC_AI {
    constexpr int j = J;
    T p[8];
    p[0] = ring[j % PF];
    if constexpr (j + PF < P::NI) ring[j % PF] = ld(std::integral_constant<int, j + PF>{});
    static_for<7>([&](auto B) CEC_AI {
      constexpr int b = B + 1;
      if constexpr (b <= P::v.hb_col[j]) p[b] = xt(p[b - 1]);
    });
    static_for<P::NO>([&](auto O) CEC_AI {
      constexpr int o = O;
      acc[o] = mul_acc<P::v.c[o][j]>(acc[o], p);
    });
    // Keep one column's powers live at a time (the loads above are already issued).
    if constexpr (P::NO > 8) __builtin_amdgcn_sched_barrier(0);
  });
  static_for<P::NO>([&](auto O) CEC_AI { st(O, acc[O]); });
}

// Nibble-window form (method of four Russians over the xtime basis): for input column j,
// lo[v] = (v)·x and hi[v] = (16 v)·x for v = 1..15 are built from the powers with one XOR each
// (only the entries some output uses, plus the entries they are built from), then every
// (output, input) pair costs one v_bitop3: acc ^= lo[c & 15] ^ hi[c >> 4].
template <unsigned USED>
constexpr unsigned nibble_closure() {
  unsigned need = USED & 0xFFFEu;
  for (int v = 15; v >= 1; --v)
    if ((need >> v & 1) && (v & (v - 1))) need |= 1u << (v & (v - 1));
  return need;
}

template <class P, int J, int HALF>
constexpr unsigned nibbles_used() {
  unsigned u = 0;
  for (int o = 0; o < P::NO; ++o) u |= 1u << ((P::v.c[o][J] >> (4 * HALF)) & 15);
  return u;
}

template <class P, int PF, class T, class LD, class ST>
__device__ __forceinline__ void ct_column_window(LD ld, ST st) {
  T acc[P::NO];
  T ring[PF];
  static_for<P::NO>([&](auto O) CEC_AI { acc[O] = T(0); });
  static_for<(PF < P::NI ? PF : P::NI)>([&](auto J) CEC_AI { ring[J] = ld(J); });
  static_for<P::NI>([&](auto J) CEC_AI {
    constexpr int j = J;
    T p[8];
    p[0] = ring[j % PF];
    if constexpr (j + PF < P::NI) ring[j % PF] = ld(std::integral_constant<int, j + PF>{});
    static_for<7>([&](auto B) CEC_AI {
      constexpr int b = B + 1;
      if constexpr (b <= P::v.hb_col[j]) p[b] = xt(p[b - 1]);
    });
    T lo[16], hi[16];
    constexpr unsigned need_lo = nibble_closure<nibbles_used<P, j, 0>()>();
    constexpr unsigned need_hi = nibble_closure<nibbles_used<P, j, 1>()>();
    static_for<16>([&](auto V) CEC_AI {
      constexpr int v = V;
      constexpr int low = v & -v;                 // lowest set bit of v
      constexpr int bit = low == 1 ? 0 : low == 2 ? 1 : low == 4 ? 2 : 3;
      if constexpr (v > 0 && (need_lo >> v & 1)) {
        if constexpr ((v & (v - 1)) == 0) lo[v] = p[bit];
        else lo[v] = xor2(lo[v & (v - 1)], p[bit]);
      }
      if constexpr (v > 0 && (need_hi >> v & 1)) {
        if constexpr ((v & (v - 1)) == 0) hi[v] = p[bit + 4];
        else hi[v] = xor2(hi[v & (v - 1)], p[bit + 4]);
      }
    });
    static_for<P::NO>([&](auto O) CEC_AI {
      constexpr int o = O;
      constexpr unsigned c = P::v.c[o][j];
      constexpr unsigned cl = c & 15, chh = c >> 4;
      if constexpr (cl && chh) acc[o] = xor3(acc[o], lo[cl], hi[chh]);
      else if constexpr (cl) acc[o] = xor2(acc[o], lo[cl]);
      else if constexpr (chh) acc[o] = xor2(acc[o], hi[chh]);
    });
    if constexpr (P::NO > 8) __builtin_amdgcn_sched_barrier(0);
  });
  static_for<P::NO>([&](auto O) CEC_AI { st(O, acc[O]); });
}

// ---------------------------------------------------------------------------------------------
// Horner form over input groups (wide codes)
// ---------------------------------------------------------------------------------------------
// gfx950 dual-issues only some VALU ops at the SIMD-32 rate (tools/valu_bench.hip, r01 sweep):
// v_add/v_sub/v_and/v_or/v_xor/v_bitop3/v_lshrrev_b32 run at 2 cycles per wave64 instruction,
// while v_lshlrev_b32, v_perm, v_alignbit, v_add3 and every other 3-source integer op take 4.
// xt_fast is 2*x on four packed bytes from full-rate ops only (6 ops, 6 "slots" vs 8 for xt):
// t = sign bits, v = t - (t >> 7) = 0x7F in each byte whose top bit is set, a = x without the
// sign bits, result = (a + a) ^ (v & 0x1D1D1D1D). a + a is written as v_add_u32 in asm:
// LLVM would turn it into a left shift, which is a half-rate instruction here.
__device__ __forceinline__ uint32_t add_self(uint32_t a) {
  uint32_t r;
  asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(a));
  return r;
}
__device__ __forceinline__ uint32_t xt_fast(uint32_t x) {
  const uint32_t t = x & 0x80808080u;
  const uint32_t v = t - (t >> 7);
  return __builtin_amdgcn_bitop3_b32(add_self(x ^ t), v, 0x1d1d1d1du, 0x78);  // a ^ (b & c)
}

// Same value without inline asm: the second addend is an opaque copy of a (one more full-rate
// op) so LLVM cannot fold a + a into a shift; the asm form instead costs a hazard s_nop.
__device__ __forceinline__ uint32_t xt_fast2(uint32_t x) {
  const uint32_t t = x & 0x80808080u;
  const uint32_t v = t - (t >> 7);
  const uint32_t a2 = __builtin_amdgcn_bitop3_b32(x, t, 0u, 0x3C);  // x ^ t
  return __builtin_amdgcn_bitop3_b32((x ^ t) + a2, v, 0x1d1d1d1du, 0x78);
}

// xt_fast with the sign-bit mask in an SGPR (`c80`, set once per kernel by an s_mov in asm, so
// LLVM cannot fold it back into a literal): the two 32-bit literals per xtime (0x80808080 and
// the canonicalised 0x7f7f7f7f) make 8-byte instructions; SGPR operands keep them at 4 bytes.
// The straight-line k_hg body is ~17 KB and a CU pair fetches it for 8 SIMDs, so instruction
// bytes per VALU op are a co-limiter (SQ_WAIT_INST_ANY rose with a literal-heavier xtime).
__device__ __forceinline__ uint32_t xt_fast_sc(uint32_t x, uint32_t c80, uint32_t c7f) {
  const uint32_t t = x & c80;
  const uint32_t v = t - (t >> 7);
  return __builtin_amdgcn_bitop3_b32(add_self(x & c7f), v, 0x1d1d1d1du, 0x78);  // a ^ (b & c)
}

// xtime in the bit-reversed representation (each byte's bits mirrored: v_bfrev_b32 of a dword
// mirrors its bytes and reverses their order, which the byte-wise arithmetic does not see).
// Multiplying by 2 is then a RIGHT shift, a full-rate op LLVM leaves alone, and the reduction
// constant 0x1D becomes 0xB8: r' = ((r >> 1) & 0x7F) ^ (r0 ? 0xB8 : 0). The mask comes from
// w = 0x80 - r0 (0x80 or 0x7F), and w & 0xB8 is the wanted term XOR a constant 0x80 in every
// byte. xt_rev omits that constant: xtime is GF(2)-linear, so the omission adds a data-independent
// error e = 1 ^ 2 ^ ... ^ 2^(n-1) = 2^n - 1 (original representation) after n xtimes, removed
// once per output. 5 full-rate ops, no inline asm (xt_fast: 6 ops + a hazard s_nop).
__device__ __forceinline__ uint32_t xt_rev(uint32_t r) {
  const uint32_t t = r & 0x01010101u;
  const uint32_t s = (r >> 1) & 0x7f7f7f7fu;
  const uint32_t w = 0x80808080u - t;
  return __builtin_amdgcn_bitop3_b32(s, w, 0xb8b8b8b8u, 0x78);  // s ^ (w & 0xB8)
}

// Output row o of a wide code is evaluated by Horner's rule over coefficient bits,
//   y = 2*y ^ S_b,   S_b = XOR of x_j over inputs j whose coefficient c[o][j] has bit b set,
// with S_b read from per-group tables: inputs are split into groups of G = 4 and every XOR
// combination of a group's inputs (up to 15 values, only those some (o, b) uses) is built once
// per column. Per (output, bit): one xtime (6 full-rate ops) + one v_bitop3 per two groups.
// Against the nibble-window form this moves the 7 xtimes per INPUT to 7 per OUTPUT and shrinks
// the per-input tables from 22 XORs + 7 xtimes to ~2.75 XORs (11 per group of 4).
template <class P, int G>
struct HGroup {
  static constexpr int NG = (P::NI + G - 1) / G;
  static constexpr int gsize(int g) { return g * G + G <= P::NI ? G : P::NI - g * G; }
  // combination index of group g for output o, bit b
  static constexpr unsigned idx(int o, int b, int g) {
    unsigned r = 0;
    for (int i = 0; i < gsize(g); ++i) r |= (unsigned)((P::v.c[o][g * G + i] >> b) & 1) << i;
    return r;
  }
  // combinations group g needs (used ones + the ones they are built from)
  static constexpr unsigned need(int g) {
    unsigned u = 0;
    for (int o = 0; o < P::NO; ++o)
      for (int b = 0; b < 8; ++b) u |= 1u << idx(o, b, g);
    u &= ~1u;
    for (int v = (1 << G) - 1; v >= 1; --v)
      if ((u >> v & 1) && (v & (v - 1))) u |= 1u << (v & (v - 1));
    return u;
  }
  struct Terms {
    int n;
    int g[NG];
    int v[NG];
  };
  static constexpr Terms terms(int o, int b) {
    Terms t{};
    for (int g = 0; g < NG; ++g) {
      const unsigned v = idx(o, b, g);
      if (v) { t.g[t.n] = g; t.v[t.n] = (int)v; ++t.n; }
    }
    return t;
  }
};

constexpr int ctz_c(unsigned v) {
  int b = 0;
  while (!(v >> b & 1)) ++b;
  return b;
}

// FL bit 1: xt_fast2 instead of xt_fast; bit 2: scheduling barrier between output rows; bit 3:
// bit-reversed representation (inputs v_bfrev'd on load, xt_rev, outputs reversed back and
// corrected by 2^top - 1 per byte); bit 4: xt_fast_sc (mask constant in an SGPR).
template <class P, int G, int FL, class LD, class ST>
__device__ __forceinline__ void ct_column_hgroup(LD ld_, ST st_) {
  using H = HGroup<P, G>;
  constexpr bool REV = (FL & 8) != 0;
  uint32_t c80 = 0x80808080u, c7f = 0x7f7f7f7fu;
  if constexpr ((FL & 16) != 0) {
    asm volatile("s_mov_b32 %0, 0x80808080" : "=s"(c80));
    asm volatile("s_mov_b32 %0, 0x7f7f7f7f" : "=s"(c7f));
  }
  auto ld = [&](auto J) CEC_AI -> uint32_t {
    if constexpr (REV) return __builtin_bitreverse32(ld_(J));
    else return ld_(J);
  };
  auto st = [&](auto O, uint32_t y) CEC_AI {
    if constexpr (REV) {
      constexpr int top = P::v.hb_row[(int)O];
      constexpr uint32_t corr = top > 0 ? ((1u << top) - 1u) * 0x01010101u : 0u;
      if constexpr (corr) st_(O, __builtin_bitreverse32(y) ^ corr);
      else st_(O, __builtin_bitreverse32(y));
    } else {
      st_(O, y);
    }
  };
  uint32_t comb[H::NG][1 << G];
  static_for<H::NG>([&](auto Gi) CEC_AI {
    constexpr int g = Gi;
    constexpr unsigned need = H::need(g);
    static_for<(1 << G)>([&](auto V) CEC_AI {
      constexpr int v = V;
      if constexpr (v > 0 && (need >> v & 1)) {
        constexpr int bit = ctz_c(v);
        if constexpr ((v & (v - 1)) == 0) comb[g][v] = ld(std::integral_constant<int, g * G + bit>{});
        else comb[g][v] = xor2(comb[g][v & (v - 1)], comb[g][1 << bit]);
      }
    });
  });
  static_for<P::NO>([&](auto O) CEC_AI {
    constexpr int o = O;
    constexpr int top = P::v.hb_row[o];
    uint32_t y = 0;
    static_for<8>([&](auto B) CEC_AI {
      constexpr int b = 7 - B;
      if constexpr (b <= top) {
        constexpr typename H::Terms tl = H::terms(o, b);
        if constexpr (b == top) {
          // first bit: y = XOR of the terms (the top bit of row o has at least one)
          if constexpr (tl.n >= 3)
            y = xor3(comb[tl.g[0]][tl.v[0]], comb[tl.g[1]][tl.v[1]], comb[tl.g[2]][tl.v[2]]);
          else if constexpr (tl.n == 2)
            y = xor2(comb[tl.g[0]][tl.v[0]], comb[tl.g[1]][tl.v[1]]);
          else
            y = comb[tl.g[0]][tl.v[0]];
        } else {
          if constexpr (REV) y = xt_rev(y);
          else if constexpr (FL & 16) y = xt_fast_sc(y, c80, c7f);
          else if constexpr (FL & 2) y = xt_fast2(y);
          else y = xt_fast(y);
        }
        constexpr int s0 = b == top ? (tl.n >= 3 ? 3 : tl.n) : 0;
        static_for<(tl.n - s0 + 1) / 2>([&](auto Q) CEC_AI {
          constexpr int i = s0 + 2 * Q;
          if constexpr (i + 1 < tl.n)
            y = xor3(y, comb[tl.g[i]][tl.v[i]], comb[tl.g[i + 1]][tl.v[i + 1]]);
          else
            y = xor2(y, comb[tl.g[i]][tl.v[i]]);
        });
      }
    });
    st(O, y);
  });
}

// Byte-wise finish of the last (len % 16) bytes, run by the last block of each segment.
template <class P, int VB>
__device__ __forceinline__ void ct_tail(const Layout& L, uint32_t seg) {
  const uint64_t t0 = L.len - L.len % VB;
  const uint64_t i = t0 + threadIdx.x;
  if (i >= L.len) return;
  auto ld = [&](auto J) CEC_AI -> uint32_t {
    return shard_ptr_ct<P::K, P::v.in[J]>(L, seg)[i];
  };
  auto st = [&](auto O, uint32_t y) CEC_AI {
    shard_ptr_ct<P::K, P::v.out[O]>(L, seg)[i] = (uint8_t)y;
  };
  if constexpr (use_horner<P>(1)) ct_column_horner<P, uint32_t>(ld, st);
  else ct_column_stream<P, 1, uint32_t>(ld, st);
}

// One 4-byte column of every shard per lane; shard addresses are a uniform 64-bit base plus
// a 32-bit lane offset (global_load/store with an SGPR base: no per-access VALU address math).
// The host checks len < 2^32.
// FL bit 0: nontemporal loads and stores (other bits: ct_column_hgroup).
template <class P, int G, int FL = 0, int BS = 256>
__global__ __launch_bounds__(BS) void k_hg(Layout L, const uint32_t* __restrict__ seg_list,
                                           uint32_t seg0) {
  const uint32_t seg = seg_list ? seg_list[seg0 + blockIdx.y] : seg0 + blockIdx.y;
  const uint32_t nvec = (uint32_t)(L.len / 4);
  const uint32_t v = blockIdx.x * BS + threadIdx.x;
  if (v < nvec) {
    const uint32_t off = v * 4;
    auto ld = [&](auto J) CEC_AI -> uint32_t {
      return ld16<(FL & 1) != 0, uint32_t>(shard_ptr_ct<P::K, P::v.in[J]>(L, seg) + off);
    };
    auto st = [&](auto O, uint32_t y) CEC_AI {
      st16<(FL & 1) != 0, uint32_t>(shard_ptr_ct<P::K, P::v.out[O]>(L, seg) + off, y);
    };
    ct_column_hgroup<P, G, FL>(ld, st);
  }
  if ((L.len % 4) && blockIdx.x == gridDim.x - 1) ct_tail<P, 4>(L, seg);
}

// ---------------------------------------------------------------------------------------------
// RS(2,1) single-erasure rebuilds in closed form
// ---------------------------------------------------------------------------------------------
// With p = 3*d0 ^ 2*d1 (E row [3, 2]) the matrix form multiplies by 0xF4 / 0xF5 (lost d0) or
// 0x8E / 0x8F (lost d1): seven xtimes per dword, ~60 issue slots. Solving the two equations
// directly costs 19 and 14 (left shifts are half-rate on gfx950, right shifts and v_add full):
//  * lost d0: q = p ^ 2*d1, d0 = q / 3. 3y = y ^ 2y = q gives y = P(q) ^ (P(q)_7 ? 0x0B : 0), P =
//    prefix XOR of each byte's bits from bit 0 up (0x0B = P(0x1D); P(0x1D)_7 = parity(0x1D) = 0
//    makes y_7 = P(q)_7);
//  * lost d1: q = p ^ d0 ^ 2*d0, d1 = q / 2 = (q >> 1) ^ (q_0 ? 0x8E : 0) (0x8E = 2^-1).
// Bit-exact with the oracle on the goldens (ramp patterns: every byte value) and full-size random
// segments (tests/test_gpu_parity.py); the formulas were checked for all 256 byte values.
__device__ __forceinline__ uint32_t gf_div3(uint32_t q) {
  uint32_t x = __builtin_amdgcn_bitop3_b32(q, add_self(q), 0xFEFEFEFEu, 0x78);  // a ^ (b & c)
  x = __builtin_amdgcn_bitop3_b32(x, x << 2, 0xFCFCFCFCu, 0x78);
  x = __builtin_amdgcn_bitop3_b32(x, x << 4, 0xF0F0F0F0u, 0x78);
  const uint32_t t = x & 0x80808080u;
  return __builtin_amdgcn_bitop3_b32(x, t - (t >> 7), 0x0B0B0B0Bu, 0x78);
}
__device__ __forceinline__ uint32_t gf_div2(uint32_t q) {
  const uint32_t u = q & 0x01010101u;
  const uint32_t w = u << 7;
  const uint32_t y = __builtin_amdgcn_bitop3_b32(q >> 1, w, 0x7F7F7F7Fu, 0xEC);  // (a & c) | b
  return __builtin_amdgcn_bitop3_b32(y, w - u, 0x0E0E0E0Eu, 0x78);
}
template <int MISSING>
__device__ __forceinline__ uint32_t rs21_rebuild(uint32_t x, uint32_t p) {
  // x: the surviving data fragment (d1 when MISSING = 0, d0 when MISSING = 1)
  if constexpr (MISSING == 0) return gf_div3(p ^ xt_fast(x));
  else return gf_div2(xor3(p, x, xt_fast(x)));
}
template <int MISSING, class TV, class LD, class ST>
__device__ __forceinline__ void ct_column_rs21(LD ld, ST st) {
  // Dec1CT<2, 1, MISSING> reads its survivors in index order: input 0 = the other data
  // fragment, input 1 = the parity
  const TV x = ld(std::integral_constant<int, 0>{}), p = ld(std::integral_constant<int, 1>{});
  TV y;
  if constexpr (sizeof(TV) == 16) {
    y = TV{rs21_rebuild<MISSING>(x.x, p.x), rs21_rebuild<MISSING>(x.y, p.y),
           rs21_rebuild<MISSING>(x.z, p.z), rs21_rebuild<MISSING>(x.w, p.w)};
  } else {
    y = rs21_rebuild<MISSING>(x, p);
  }
  st(std::integral_constant<int, 0>{}, y);
}
template <class P>
struct Rs21Closed {
  static constexpr int missing = -1;
};
template <int E>
struct Rs21Closed<Dec1CT<2, 1, E>> {
  static constexpr int missing = E < 2 ? E : -1;
};

// One workgroup's tile (blockIdx.x) of segment `seg`; k_ct and the mixed-pattern kernel below.
template <class P, int U, bool NT, class TV, int PF, bool WIN, int BS>
__device__ __forceinline__ void ct_tile(const Layout& L, uint32_t seg) {
  constexpr int VB = sizeof(TV);  // bytes per lane per shard per column
  const uint64_t nvec = L.len / VB;
  const uint64_t base = (uint64_t)blockIdx.x * (BS * U) + threadIdx.x;
  // Shard pointers are recomputed per use (scalar base + index * stride): holding 2 * (NI + NO)
  // SGPRs of pointers live across the body overflows the SGPR file for wide codes.
  auto column = [&](uint64_t v) CEC_AI {
    const uint64_t off = v * VB;
    auto ld = [&](auto J) CEC_AI {
      return ld16<NT, TV>(shard_ptr_ct<P::K, P::v.in[J]>(L, seg) + off);
    };
    auto st = [&](auto O, TV y) CEC_AI {
      st16<NT, TV>(shard_ptr_ct<P::K, P::v.out[O]>(L, seg) + off, y);
    };
    if constexpr (Rs21Closed<P>::missing >= 0) ct_column_rs21<Rs21Closed<P>::missing, TV>(ld, st);
    else if constexpr (use_horner<P>(U)) ct_column_horner<P, TV>(ld, st);
    else if constexpr (WIN) ct_column_window<P, PF, TV>(ld, st);
    else ct_column_stream<P, PF, TV>(ld, st);
  };
  if (base + (U - 1) * BS < nvec) {  // full tile: no per-element predicate
    static_for<U>([&](auto u) CEC_AI { column(base + u * BS); });
  } else {
    static_for<U>([&](auto u) CEC_AI {
      if (base + u * BS < nvec) column(base + u * BS);
    });
  }
  if ((L.len % VB) && blockIdx.x == gridDim.x - 1) ct_tail<P, VB>(L, seg);
}

template <class P, int U, bool NT, class TV = u32x4, int PF = 1, bool WIN = false, int BS = 256>
__global__ __launch_bounds__(BS) void k_ct(Layout L, const uint32_t* __restrict__ seg_list,
                                            uint32_t seg0) {
  const uint32_t seg = seg_list ? seg_list[seg0 + blockIdx.y] : seg0 + blockIdx.y;
  ct_tile<P, U, NT, TV, PF, WIN, BS>(L, seg);
}

// RS(2,1) degraded read with a different single erasure per segment, in one launch: entry
// seg | (erased << 30) of the tagged list picks the compile-time rebuild for the workgroup row
// (a wave-uniform branch), where one launch per erasure pattern over a third of the batch each
// paid three ramp-ups and drains per batch.
template <bool NT, int BS>
__global__ __launch_bounds__(BS) void k_ct_dec1_mixed21(Layout L,
                                                        const uint32_t* __restrict__ tagged,
                                                        uint32_t seg0) {
  const uint32_t w = tagged[seg0 + blockIdx.y];
  const uint32_t seg = w & 0x3FFFFFFFu, e = w >> 30;
  if (e == 0) ct_tile<Dec1CT<2, 1, 0>, 1, NT, u32x4, 1, false, BS>(L, seg);
  else if (e == 1) ct_tile<Dec1CT<2, 1, 1>, 1, NT, u32x4, 1, false, BS>(L, seg);
  else if (e == 2) ct_tile<EncCT<2, 1>, 1, NT, u32x4, 1, false, BS>(L, seg);
  // e == 3: a segment with nothing to rebuild in this launch, left untouched
}

// Persistent grid-stride variant: a fixed grid walks the flattened (segment, tile) space.
template <class P, bool NT, int BS>
__global__ __launch_bounds__(BS) void k_ct_persist(Layout L, const uint32_t* __restrict__ seg_list,
                                                   uint32_t nseg, uint64_t tiles_per_seg) {
  using TV = u32x4;
  const uint64_t nvec = L.len / 16;
  const uint64_t total = (uint64_t)nseg * tiles_per_seg;
  for (uint64_t t = blockIdx.x; t < total; t += gridDim.x) {
    const uint32_t y = (uint32_t)(t / tiles_per_seg);
    const uint64_t tile = t - (uint64_t)y * tiles_per_seg;
    const uint32_t seg = seg_list ? seg_list[y] : y;
    const uint64_t v = tile * BS + threadIdx.x;
    if (v < nvec) {
      const uint64_t off = v * 16;
      auto ld = [&](auto J) CEC_AI {
        return ld16<NT, TV>(shard_ptr_ct<P::K, P::v.in[J]>(L, seg) + off);
      };
      auto st = [&](auto O, TV yv) CEC_AI {
        st16<NT, TV>(shard_ptr_ct<P::K, P::v.out[O]>(L, seg) + off, yv);
      };
      ct_column_horner<P, TV>(ld, st);
    }
    if ((L.len % 16) && tile == tiles_per_seg - 1 && BS >= 16) ct_tail<P, 16>(L, seg);
  }
}

// XCD-contiguous variant (tuning build): a 1-D grid over the flattened (segment, tile) space,
// remapped so that XCD x (which receives workgroups x, x + 8, ... from the round-robin dispatch)
// walks the contiguous 1/8 of the batch starting at x * ceil(total / 8).
template <class P, bool NT, int BS>
__global__ __launch_bounds__(BS) void k_ct_xcd(Layout L, const uint32_t* __restrict__ seg_list,
                                               uint32_t nseg, uint64_t tiles_per_seg) {
  const uint64_t total = (uint64_t)nseg * tiles_per_seg;
  const uint64_t per = (total + 7) / 8;
  const uint64_t t = (uint64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= total) return;
  const uint32_t y = (uint32_t)(t / tiles_per_seg);
  const uint64_t tile = t - (uint64_t)y * tiles_per_seg;
  const uint32_t seg = seg_list ? seg_list[y] : y;
  const uint64_t v = tile * BS + threadIdx.x;
  if (v < L.len / 16) {
    const uint64_t off = v * 16;
    auto ld = [&](auto J) CEC_AI {
      return ld16<NT, u32x4>(shard_ptr_ct<P::K, P::v.in[J]>(L, seg) + off);
    };
    auto st = [&](auto O, u32x4 yv) CEC_AI {
      st16<NT, u32x4>(shard_ptr_ct<P::K, P::v.out[O]>(L, seg) + off, yv);
    };
    if constexpr (Rs21Closed<P>::missing >= 0) ct_column_rs21<Rs21Closed<P>::missing, u32x4>(ld, st);
    else ct_column_horner<P, u32x4>(ld, st);
  }
}

// Byte-granular variant for layouts whose shard starts are not 16-byte aligned.
template <class P>
__global__ __launch_bounds__(256) void k_ct_bytes(Layout L, const uint32_t* __restrict__ seg_list,
                                                  uint32_t seg0) {
  const uint32_t seg = seg_list ? seg_list[seg0 + blockIdx.y] : seg0 + blockIdx.y;
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= L.len) return;
  auto ld = [&](auto J) CEC_AI -> uint32_t {
    return shard_ptr_ct<P::K, P::v.in[J]>(L, seg)[i];
  };
  auto st = [&](auto O, uint32_t y) CEC_AI {
    shard_ptr_ct<P::K, P::v.out[O]>(L, seg)[i] = (uint8_t)y;
  };
  if constexpr (use_horner<P>(1)) ct_column_horner<P, uint32_t>(ld, st);
  else ct_column_stream<P, 1, uint32_t>(ld, st);
}

// ---------------------------------------------------------------------------------------------
// Run-time coefficients
// ---------------------------------------------------------------------------------------------
// One workgroup row (blockIdx.y) = one segment; its program chunk (indices + coefficients) is
// read with scalar loads, so segments with different erasure patterns share one launch. Per
// input column: the xtime powers up to the column's highest coefficient bit, then one
// v_bitop3 (acc ^= pow_b & mask) per (output, bit) with masks expanded on the SALU. The next
// input column's loads are issued before the current column is multiplied in.
// Program chunks are read through the constant address space: they are never written while a
// kernel runs, so uniform-address loads become s_load (SGPR results, SALU mask expansion).
typedef const uint32_t __attribute__((address_space(4))) cu32;
__device__ __forceinline__ const cu32* as_const(const uint32_t* p) {
  return (const cu32*)(uintptr_t)p;
}

template <int NOB, int U, class TV, class T, class LD>
__device__ __forceinline__ void rt_accumulate(T (&acc)[NOB][U], const cu32* __restrict__ P,
                                              LD ld) {
  const uint32_t nin = P[0];
  const cu32* __restrict__ hbs = P + 4 + 512;
  const cu32* __restrict__ masks = P + kRtHeaderWords;
  T cur[U], nxt[U];
#pragma unroll
  for (int u = 0; u < U; ++u) cur[u] = ld(P[4], u);
  for (uint32_t j = 0; j < nin; ++j) {
    if (j + 1 < nin) {
#pragma unroll
      for (int u = 0; u < U; ++u) nxt[u] = ld(P[4 + j + 1], u);
    }
    const int hb = (int)hbs[j];
    T p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) p[u] = cur[u];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      if (b > hb) break;  // wave-uniform: no higher coefficient bit in this column
      if (b > 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = xt(p[u]);
      }
      const cu32* __restrict__ mk = masks + (j * 8 + b) * NOB;
#pragma unroll
      for (int o = 0; o < NOB; ++o) {
        const uint32_t m = mk[o];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[o][u] = bitop3_xand(acc[o][u], p[u], m);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = nxt[u];
  }
}

// shard_ptr with the data/parity choice as scalar selects instead of a branch, so the run-time
// kernels' per-input index loads batch into wide scalar loads ahead of the global loads.
// (Pointer selects, not integer casts: the address stays in the global space, so the loads are
// global_load, not flat_load, whose lgkmcnt coupling would serialise them with the index reads.)
__device__ __forceinline__ uint8_t* shard_ptr_sel(const Layout& L, uint32_t idx, uint32_t seg) {
  const bool isd = idx < (uint32_t)L.k;
  uint8_t* const base = isd ? L.data : L.parity;
  const uint64_t sstr = isd ? L.data_seg_stride : L.par_seg_stride;
  const uint32_t j = isd ? idx : idx - (uint32_t)L.k;
  return base + seg * sstr + (uint64_t)j * L.shard_stride;
}

__device__ __forceinline__ const uint32_t* as_const_ptr(const uint32_t* const* a, uint32_t y) {
  typedef const uint64_t __attribute__((address_space(4))) cu64;
  return (const uint32_t*)(uintptr_t)((const cu64*)(uintptr_t)a)[y];
}

template <int NOB, int U, class TV>
__global__ __launch_bounds__(256) void k_rt(Layout L, const uint32_t* __restrict__ chunk,
                                            const uint32_t* const* __restrict__ per_seg,
                                            const uint32_t* __restrict__ seg_list, uint32_t seg0,
                                            int vec_ok) {
  const uint32_t y = seg0 + blockIdx.y;
  const uint32_t seg = seg_list ? seg_list[y] : y;
  const cu32* __restrict__ P = as_const(per_seg ? as_const_ptr(per_seg, y) : chunk);
  const uint32_t nout = P[1];
  const cu32* __restrict__ out_idx = P + 4 + 256;
  constexpr int VB = sizeof(TV);
  if (vec_ok) {
    const uint64_t nvec = L.len / VB;
    const uint64_t base = (uint64_t)blockIdx.x * (256 * U) + threadIdx.x;
    TV acc[NOB][U];
#pragma unroll
    for (int o = 0; o < NOB; ++o)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[o][u] = TV(0);
    auto ld = [&](uint32_t sh, int u) CEC_AI -> TV {
      const uint64_t v = base + u * 256;
      if (v >= nvec) return TV(0);
      return ld16<false, TV>(shard_ptr(L, (int)sh, seg) + v * VB);
    };
    rt_accumulate<NOB, U, TV>(acc, P, ld);
#pragma unroll
    for (int o = 0; o < NOB; ++o) {
      if (o < (int)nout) {
        uint8_t* dst = shard_ptr(L, (int)out_idx[o], seg);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t v = base + u * 256;
          if (v < nvec) st16<false, TV>(dst + v * VB, acc[o][u]);
        }
      }
    }
    if (!(L.len % VB) || blockIdx.x != gridDim.x - 1) return;
  }
  // byte path: whole shard (vec_ok == 0, grid covers len) or the tail (last block)
  const uint64_t i = vec_ok ? (L.len - L.len % VB) + threadIdx.x
                            : (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= L.len) return;
  uint32_t acc[NOB][1];
#pragma unroll
  for (int o = 0; o < NOB; ++o) acc[o][0] = 0;
  auto ld = [&](uint32_t sh, int) CEC_AI -> uint32_t { return shard_ptr(L, (int)sh, seg)[i]; };
  rt_accumulate<NOB, 1, uint32_t>(acc, P, ld);
#pragma unroll
  for (int o = 0; o < NOB; ++o)
    if (o < (int)nout) shard_ptr(L, (int)out_idx[o], seg)[i] = (uint8_t)acc[o][0];
}

// Bit-plane run-time matvec for few outputs (k_rtb): per output o and coefficient bit b one
// accumulator t[o][b] = XOR of the inputs whose coefficient in row o has bit b set (one v_bitop3
// per (input, output, bit) with the chunk's mask from an SGPR), then out_o by Horner over the
// bits, ((t7 * 2 ^ t6) * 2 ^ ...) ^ t0: 7 xtimes per output where k_rt spends 7 per input. Inputs
// stream through (the next column's load is issued before the current one is folded in), so the
// registers are the 8 * NOB accumulators: decode of a few lost fragments of a wide code (the
// restoral case) and partial rebuilds, where nout << nin.
template <int NOB, class TV, int PF>
__global__ __launch_bounds__(256) void k_rtb(Layout L, const uint32_t* __restrict__ chunk,
                                             const uint32_t* const* __restrict__ per_seg,
                                             const uint32_t* __restrict__ seg_list, uint32_t seg0,
                                             int vec_ok) {
  const uint32_t y = seg0 + blockIdx.y;
  const uint32_t seg = seg_list ? seg_list[y] : y;
  const cu32* __restrict__ P = as_const(per_seg ? as_const_ptr(per_seg, y) : chunk);
  const uint32_t nin = P[0], nout = P[1];
  const cu32* __restrict__ in_idx = P + 4;
  const cu32* __restrict__ out_idx = P + 4 + 256;
  const cu32* __restrict__ masks = P + kRtHeaderWords;
  // inputs stream through a ring of PF columns: column j + PF is loaded while column j folds
  auto fold = [&]<class T>(T (&t)[NOB][8], auto ld) CEC_AI {
    T ring[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q)
      if (q < (int)nin) ring[q] = ld(in_idx[q]);
    for (uint32_t j0 = 0; j0 < nin; j0 += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const uint32_t j = j0 + q;
        if (j >= nin) break;  // wave-uniform
        const T cur = ring[q];
        if (j + PF < nin) ring[q] = ld(in_idx[j + PF]);
        // all 8 bits, no branch on the column's top bit: the 8 * NOB masks of a column then
        // come in as one wide scalar load
        const cu32* __restrict__ mk = masks + j * 8 * NOB;
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
          for (int o = 0; o < NOB; ++o) t[o][b] = bitop3_xand(t[o][b], cur, mk[b * NOB + o]);
      }
    }
  };
  auto horner = [&]<class T>(const T (&t)[8]) CEC_AI -> T {
    T r = t[7];
#pragma unroll
    for (int b = 6; b >= 0; --b) r = xt(r) ^ t[b];
    return r;
  };
  constexpr int VB = sizeof(TV);
  if (vec_ok) {
    const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (v < L.len / VB) {
      TV t[NOB][8];
#pragma unroll
      for (int o = 0; o < NOB; ++o)
#pragma unroll
        for (int b = 0; b < 8; ++b) t[o][b] = TV(0);
      fold(t, [&](uint32_t sh) CEC_AI { return ld16<true, TV>(shard_ptr(L, (int)sh, seg) + v * VB); });
#pragma unroll
      for (int o = 0; o < NOB; ++o)
        if (o < (int)nout) st16<true, TV>(shard_ptr(L, (int)out_idx[o], seg) + v * VB, horner(t[o]));
    }
    if (!(L.len % VB) || blockIdx.x != gridDim.x - 1) return;
  }
  // byte path: whole shard (vec_ok == 0, grid covers len) or the tail (last block)
  const uint64_t i = vec_ok ? (L.len - L.len % VB) + threadIdx.x
                            : (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= L.len) return;
  uint32_t t[NOB][8];
#pragma unroll
  for (int o = 0; o < NOB; ++o)
#pragma unroll
    for (int b = 0; b < 8; ++b) t[o][b] = 0;
  fold(t, [&](uint32_t sh) CEC_AI -> uint32_t { return shard_ptr(L, (int)sh, seg)[i]; });
#pragma unroll
  for (int o = 0; o < NOB; ++o)
    if (o < (int)nout) shard_ptr(L, (int)out_idx[o], seg)[i] = (uint8_t)horner(t[o]);
}

// Horner over input groups with run-time coefficients (k_rth): the compile-time k_hg scheme
// with the per-(output, bit, group) combination index read from the chunk's Horner section
// through the constant address space. Each group's 16 combinations (entry 0 = 0) live in one
// 16-VGPR vector and a wave-uniform index selects one with s_set_gpr_idx (one v_mov + two SALU
// per read); per (output, bit) that is NG reads + NG XORs + one xtime, against 32 v_bitop3 masks
// (one per input) plus 7 xtimes per input column in k_rt.
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

template <int NG, class LD, class ST>
__device__ __forceinline__ void rth_column(const cu32* __restrict__ P, LD ld, ST st) {
  const uint32_t nin = P[0], nout = P[1];
  const cu32* __restrict__ in_idx = P + 4;
  const cu32* __restrict__ out_idx = P + 4 + 256;
  const cu32* __restrict__ top = P + P[3];
  const cu32* __restrict__ ix = top + 32;
  u32x16 comb[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    uint32_t x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // unconditional load (unused slots name shard 0), masked
      const uint32_t v = ld(in_idx[4 * g + i]);
      x[i] = (uint32_t)(4 * g + i) < nin ? v : 0u;
    }
    comb[g][0] = 0;
    comb[g][1] = x[0];
    comb[g][2] = x[1];
    comb[g][4] = x[2];
    comb[g][8] = x[3];
#pragma unroll
    for (int v = 3; v < 16; ++v)
      if (v & (v - 1)) comb[g][v] = xor2(comb[g][v & (v - 1)], comb[g][v & -v]);
  }
  // Every row runs all 8 bits (index 0 reads the zero entry): a branch-free body lets the
  // row's 64 indices arrive in a few s_load_dwordx16 ahead of use.
  (void)top;
  for (uint32_t o = 0; o < nout; ++o) {
    const cu32* __restrict__ q = ix + o * 64;
    uint32_t y = 0;
#pragma unroll
    for (int b = 7; b >= 0; --b) {
      if (b < 7) y = xt_fast(y);
#pragma unroll
      for (int g = 0; g < NG; ++g) y ^= comb[g][q[b * 8 + g]];
    }
    st(out_idx[o], y);
  }
}

template <int NG>
__global__ __launch_bounds__(256) void k_rth(Layout L, const uint32_t* __restrict__ chunk,
                                             const uint32_t* const* __restrict__ per_seg,
                                             const uint32_t* __restrict__ seg_list, uint32_t seg0,
                                             int vec_ok) {
  const uint32_t y = seg0 + blockIdx.y;
  const uint32_t seg = seg_list ? seg_list[y] : y;
  const cu32* __restrict__ P = as_const(per_seg ? as_const_ptr(per_seg, y) : chunk);
  if (vec_ok) {
    const uint64_t nvec = L.len / 4;
    const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (v < nvec) {
      const uint64_t off = v * 4;
      auto ld = [&](uint32_t sh) CEC_AI -> uint32_t {
        return *reinterpret_cast<const uint32_t*>(shard_ptr(L, (int)sh, seg) + off);
      };
      auto st = [&](uint32_t sh, uint32_t val) CEC_AI {
        *reinterpret_cast<uint32_t*>(shard_ptr(L, (int)sh, seg) + off) = val;
      };
      rth_column<NG>(P, ld, st);
    }
    if (!(L.len % 4) || blockIdx.x != gridDim.x - 1) return;
  }
  // byte path: whole shard (vec_ok == 0, grid covers len) or the tail (last block); one byte
  // per lane in the low byte of a dword (the arithmetic is byte-wise, upper bytes stay zero)
  const uint64_t i = vec_ok ? (L.len - L.len % 4) + threadIdx.x
                            : (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= L.len) return;
  auto ld = [&](uint32_t sh) CEC_AI -> uint32_t { return shard_ptr(L, (int)sh, seg)[i]; };
  auto st = [&](uint32_t sh, uint32_t val) CEC_AI { shard_ptr(L, (int)sh, seg)[i] = (uint8_t)val; };
  rth_column<NG>(P, ld, st);
}

// Run-time Horner over input groups with the table reads folded into the XORs (k_rthx): the
// group tables live in a fixed VGPR range above the compiler's allocation (amdgpu_num_vgpr caps
// the compiler at RTHX_R registers; the asm blocks own v[RTHX_R, RTHX_R + 16 NG)), so a read of
// entry idx of group g is the XOR's own source operand v[base_g] under s_set_gpr_idx (SRC0),
// one VALU op and one SALU op per entry (k_rth: a v_mov under on/off, then the XOR).
#define RTHX_R 24
// The tables sit above the compiler's amdgpu_num_vgpr budget, which clang calls "reserved"
// registers; the kernel descriptor's VGPR count includes them (tools/kres.py shows 24 + 16 NG).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void rthx_table0(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  asm volatile("v_mov_b32 v24, 0\n\tv_mov_b32 v25, %0\n\tv_mov_b32 v26, %1\n\tv_mov_b32 v28, %2\n\tv_mov_b32 v32, %3\n\tv_xor_b32 v27, v26, v25\n\tv_xor_b32 v29, v28, v25\n\tv_xor_b32 v30, v28, v26\n\tv_xor_b32 v31, v30, v25\n\tv_xor_b32 v33, v32, v25\n\tv_xor_b32 v34, v32, v26\n\tv_xor_b32 v35, v34, v25\n\tv_xor_b32 v36, v32, v28\n\tv_xor_b32 v37, v36, v25\n\tv_xor_b32 v38, v36, v26\n\tv_xor_b32 v39, v38, v25" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3)
               : "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
}
__device__ __forceinline__ void rthx_table1(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  asm volatile("v_mov_b32 v40, 0\n\tv_mov_b32 v41, %0\n\tv_mov_b32 v42, %1\n\tv_mov_b32 v44, %2\n\tv_mov_b32 v48, %3\n\tv_xor_b32 v43, v42, v41\n\tv_xor_b32 v45, v44, v41\n\tv_xor_b32 v46, v44, v42\n\tv_xor_b32 v47, v46, v41\n\tv_xor_b32 v49, v48, v41\n\tv_xor_b32 v50, v48, v42\n\tv_xor_b32 v51, v50, v41\n\tv_xor_b32 v52, v48, v44\n\tv_xor_b32 v53, v52, v41\n\tv_xor_b32 v54, v52, v42\n\tv_xor_b32 v55, v54, v41" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3)
               : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");
}
__device__ __forceinline__ void rthx_table2(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  asm volatile("v_mov_b32 v56, 0\n\tv_mov_b32 v57, %0\n\tv_mov_b32 v58, %1\n\tv_mov_b32 v60, %2\n\tv_mov_b32 v64, %3\n\tv_xor_b32 v59, v58, v57\n\tv_xor_b32 v61, v60, v57\n\tv_xor_b32 v62, v60, v58\n\tv_xor_b32 v63, v62, v57\n\tv_xor_b32 v65, v64, v57\n\tv_xor_b32 v66, v64, v58\n\tv_xor_b32 v67, v66, v57\n\tv_xor_b32 v68, v64, v60\n\tv_xor_b32 v69, v68, v57\n\tv_xor_b32 v70, v68, v58\n\tv_xor_b32 v71, v70, v57" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3)
               : "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71");
}
__device__ __forceinline__ void rthx_table3(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  asm volatile("v_mov_b32 v72, 0\n\tv_mov_b32 v73, %0\n\tv_mov_b32 v74, %1\n\tv_mov_b32 v76, %2\n\tv_mov_b32 v80, %3\n\tv_xor_b32 v75, v74, v73\n\tv_xor_b32 v77, v76, v73\n\tv_xor_b32 v78, v76, v74\n\tv_xor_b32 v79, v78, v73\n\tv_xor_b32 v81, v80, v73\n\tv_xor_b32 v82, v80, v74\n\tv_xor_b32 v83, v82, v73\n\tv_xor_b32 v84, v80, v76\n\tv_xor_b32 v85, v84, v73\n\tv_xor_b32 v86, v84, v74\n\tv_xor_b32 v87, v86, v73" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3)
               : "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87");
}
__device__ __forceinline__ void rthx_table4(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  asm volatile("v_mov_b32 v88, 0\n\tv_mov_b32 v89, %0\n\tv_mov_b32 v90, %1\n\tv_mov_b32 v92, %2\n\tv_mov_b32 v96, %3\n\tv_xor_b32 v91, v90, v89\n\tv_xor_b32 v93, v92, v89\n\tv_xor_b32 v94, v92, v90\n\tv_xor_b32 v95, v94, v89\n\tv_xor_b32 v97, v96, v89\n\tv_xor_b32 v98, v96, v90\n\tv_xor_b32 v99, v98, v89\n\tv_xor_b32 v100, v96, v92\n\tv_xor_b32 v101, v100, v89\n\tv_xor_b32 v102, v100, v90\n\tv_xor_b32 v103, v102, v89" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3)
               : "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103");
}
__device__ __forceinline__ void rthx_table5(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  asm volatile("v_mov_b32 v104, 0\n\tv_mov_b32 v105, %0\n\tv_mov_b32 v106, %1\n\tv_mov_b32 v108, %2\n\tv_mov_b32 v112, %3\n\tv_xor_b32 v107, v106, v105\n\tv_xor_b32 v109, v108, v105\n\tv_xor_b32 v110, v108, v106\n\tv_xor_b32 v111, v110, v105\n\tv_xor_b32 v113, v112, v105\n\tv_xor_b32 v114, v112, v106\n\tv_xor_b32 v115, v114, v105\n\tv_xor_b32 v116, v112, v108\n\tv_xor_b32 v117, v116, v105\n\tv_xor_b32 v118, v116, v106\n\tv_xor_b32 v119, v118, v105" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3)
               : "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119");
}
__device__ __forceinline__ void rthx_table6(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  asm volatile("v_mov_b32 v120, 0\n\tv_mov_b32 v121, %0\n\tv_mov_b32 v122, %1\n\tv_mov_b32 v124, %2\n\tv_mov_b32 v128, %3\n\tv_xor_b32 v123, v122, v121\n\tv_xor_b32 v125, v124, v121\n\tv_xor_b32 v126, v124, v122\n\tv_xor_b32 v127, v126, v121\n\tv_xor_b32 v129, v128, v121\n\tv_xor_b32 v130, v128, v122\n\tv_xor_b32 v131, v130, v121\n\tv_xor_b32 v132, v128, v124\n\tv_xor_b32 v133, v132, v121\n\tv_xor_b32 v134, v132, v122\n\tv_xor_b32 v135, v134, v121" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3)
               : "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135");
}
__device__ __forceinline__ void rthx_table7(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  asm volatile("v_mov_b32 v136, 0\n\tv_mov_b32 v137, %0\n\tv_mov_b32 v138, %1\n\tv_mov_b32 v140, %2\n\tv_mov_b32 v144, %3\n\tv_xor_b32 v139, v138, v137\n\tv_xor_b32 v141, v140, v137\n\tv_xor_b32 v142, v140, v138\n\tv_xor_b32 v143, v142, v137\n\tv_xor_b32 v145, v144, v137\n\tv_xor_b32 v146, v144, v138\n\tv_xor_b32 v147, v146, v137\n\tv_xor_b32 v148, v144, v140\n\tv_xor_b32 v149, v148, v137\n\tv_xor_b32 v150, v148, v138\n\tv_xor_b32 v151, v150, v137" ::"v"(x0), "v"(x1), "v"(x2), "v"(x3)
               : "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151");
}
#pragma clang diagnostic pop
// y ^= T_g[q[g]] for the NG groups, each a v_xor whose SRC0 is indexed by M0. The SALU write of
// M0 (s_set_gpr_idx_on / _idx) needs one wait state before the indexed VALU: without the s_nop
// the XOR read a stale index now and then (10 of 10 RS(32,32) 32-erasure rebuilds had 10^5 wrong
// bytes, a different set each run; with it 0 of 10, tools/stress_rthx.py). One after _off too,
// // before any VALU that names a VGPR as SRC0. Every block clobbers M0 (declared: clang warns that
// M0 is a reserved register it does not preserve; no other instruction of k_rthx uses M0, which
// tests/test_host.py checks on the shipped code object along with the wait states).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#define RTHX_ON "s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\ts_nop 0\n\tv_xor_b32 %0, v24, %0\n\t"
#define RTHX_IDX(n, reg) "s_set_gpr_idx_idx %" #n "\n\ts_nop 0\n\tv_xor_b32 %0, " reg ", %0\n\t"
#define RTHX_OFF "s_set_gpr_idx_off\n\ts_nop 0"
template <int NG>
__device__ __forceinline__ uint32_t rthx_xor(uint32_t y, const uint32_t (&q)[NG]);
template <>
__device__ __forceinline__ uint32_t rthx_xor<1>(uint32_t y, const uint32_t (&q)[1]) {
  asm volatile(RTHX_ON RTHX_OFF : "+v"(y) : "s"(q[0]) : "m0");
  return y;
}
template <>
__device__ __forceinline__ uint32_t rthx_xor<2>(uint32_t y, const uint32_t (&q)[2]) {
  asm volatile(RTHX_ON RTHX_IDX(2, "v40") RTHX_OFF : "+v"(y) : "s"(q[0]), "s"(q[1]) : "m0");
  return y;
}
template <>
__device__ __forceinline__ uint32_t rthx_xor<3>(uint32_t y, const uint32_t (&q)[3]) {
  asm volatile(RTHX_ON RTHX_IDX(2, "v40") RTHX_IDX(3, "v56") RTHX_OFF
               : "+v"(y) : "s"(q[0]), "s"(q[1]), "s"(q[2]) : "m0");
  return y;
}
template <>
__device__ __forceinline__ uint32_t rthx_xor<4>(uint32_t y, const uint32_t (&q)[4]) {
  asm volatile(RTHX_ON RTHX_IDX(2, "v40") RTHX_IDX(3, "v56") RTHX_IDX(4, "v72") RTHX_OFF
               : "+v"(y) : "s"(q[0]), "s"(q[1]), "s"(q[2]), "s"(q[3]) : "m0");
  return y;
}
template <>
__device__ __forceinline__ uint32_t rthx_xor<6>(uint32_t y, const uint32_t (&q)[6]) {
  asm volatile(RTHX_ON RTHX_IDX(2, "v40") RTHX_IDX(3, "v56") RTHX_IDX(4, "v72")
                   RTHX_IDX(5, "v88") RTHX_IDX(6, "v104") RTHX_OFF
               : "+v"(y) : "s"(q[0]), "s"(q[1]), "s"(q[2]), "s"(q[3]), "s"(q[4]), "s"(q[5]) : "m0");
  return y;
}
template <>
__device__ __forceinline__ uint32_t rthx_xor<8>(uint32_t y, const uint32_t (&q)[8]) {
  asm volatile(RTHX_ON RTHX_IDX(2, "v40") RTHX_IDX(3, "v56") RTHX_IDX(4, "v72")
                   RTHX_IDX(5, "v88") RTHX_IDX(6, "v104") RTHX_IDX(7, "v120")
                       RTHX_IDX(8, "v136") RTHX_OFF
               : "+v"(y)
               : "s"(q[0]), "s"(q[1]), "s"(q[2]), "s"(q[3]), "s"(q[4]), "s"(q[5]), "s"(q[6]),
                 "s"(q[7]) : "m0");
  return y;
}
#pragma clang diagnostic pop
#undef RTHX_ON
#undef RTHX_IDX
#undef RTHX_OFF

template <int NG, class LD, class ST>
__device__ __forceinline__ void rthx_column(const cu32* __restrict__ P, LD ld, ST st) {
  const uint32_t nin = P[0], nout = P[1];
  const cu32* __restrict__ in_idx = P + 4;
  const cu32* __restrict__ out_idx = P + 4 + 256;
  const cu32* __restrict__ ix = P + P[3] + 32;
  // unused input slots hold shard index 0 (a valid shard), so every load is unconditional and
  // the index reads batch into wide scalar loads; the value is masked afterwards. Loads run two
  // groups ahead of the table being built (the asm blocks are ordered; four live inputs per
  // group keep the compiler inside its RTHX_R registers).
  uint32_t xs[NG][4];
  auto load_group = [&](int g) CEC_AI {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t v = ld(in_idx[4 * g + i]);
      xs[g][i] = (uint32_t)(4 * g + i) < nin ? v : 0u;
    }
  };
  auto build = [&](int g) CEC_AI {
    const uint32_t* x = xs[g];
    if (g == 0) rthx_table0(x[0], x[1], x[2], x[3]);
    if (g == 1) rthx_table1(x[0], x[1], x[2], x[3]);
    if (g == 2) rthx_table2(x[0], x[1], x[2], x[3]);
    if (g == 3) rthx_table3(x[0], x[1], x[2], x[3]);
    if (g == 4) rthx_table4(x[0], x[1], x[2], x[3]);
    if (g == 5) rthx_table5(x[0], x[1], x[2], x[3]);
    if (g == 6) rthx_table6(x[0], x[1], x[2], x[3]);
    if (g == 7) rthx_table7(x[0], x[1], x[2], x[3]);
  };
  load_group(0);
  if constexpr (NG > 1) load_group(1);
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (g + 2 < NG) load_group(g + 2);
    build(g);
  }
  for (uint32_t o = 0; o < nout; ++o) {
    // the row's 8 x NG indices in SGPRs up front: one scalar-load wait per row, not per bit
    const cu32* __restrict__ q = ix + o * 64;
    uint32_t iv[8][NG];
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int g = 0; g < NG; ++g) iv[b][g] = q[b * 8 + g];
    uint32_t y = 0;
#pragma unroll
    for (int b = 7; b >= 0; --b) {
      if (b < 7) y = xt_fast(y);
      y = rthx_xor<NG>(y, iv[b]);
    }
    st(out_idx[o], y);
  }
}

template <int NG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(RTHX_R))) void k_rthx(
    Layout L, const uint32_t* __restrict__ chunk, const uint32_t* const* __restrict__ per_seg,
    const uint32_t* __restrict__ seg_list, uint32_t seg0, int vec_ok) {
  const uint32_t y = seg0 + blockIdx.y;
  const uint32_t seg = seg_list ? seg_list[y] : y;
  const cu32* __restrict__ P = as_const(per_seg ? as_const_ptr(per_seg, y) : chunk);
  if (vec_ok) {
    const uint64_t nvec = L.len / 4;
    const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (v < nvec) {
      const uint64_t off = v * 4;
      auto ld = [&](uint32_t sh) CEC_AI -> uint32_t {
        return *reinterpret_cast<const uint32_t*>(shard_ptr_sel(L, sh, seg) + off);
      };
      auto st = [&](uint32_t sh, uint32_t val) CEC_AI {
        *reinterpret_cast<uint32_t*>(shard_ptr_sel(L, sh, seg) + off) = val;
      };
      rthx_column<NG>(P, ld, st);
    }
    if (!(L.len % 4) || blockIdx.x != gridDim.x - 1) return;
  }
  const uint64_t i = vec_ok ? (L.len - L.len % 4) + threadIdx.x
                            : (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= L.len) return;
  auto ld = [&](uint32_t sh) CEC_AI -> uint32_t { return shard_ptr_sel(L, sh, seg)[i]; };
  auto st = [&](uint32_t sh, uint32_t val) CEC_AI { shard_ptr_sel(L, sh, seg)[i] = (uint8_t)val; };
  rthx_column<NG>(P, ld, st);
}

// ---------------------------------------------------------------------------------------------
// Synthetic segments
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill(uint8_t* __restrict__ out, uint64_t seg_bytes,
                                              uint64_t nseg, uint64_t seg0, uint64_t seed) {
  const uint64_t words_per_seg = seg_bytes >> 3;
  const uint64_t total = words_per_seg * nseg;
  uint64_t* o = reinterpret_cast<uint64_t*>(out);
  for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 2; i < total;
       i += (uint64_t)gridDim.x * 512) {
    const uint64_t s = i / words_per_seg, w = i - s * words_per_seg;
    const uint64_t a = splitmix64(seed ^ ((seg0 + s) << 32) ^ w);
    uint64_t b;
    if (w + 1 < words_per_seg) b = splitmix64(seed ^ ((seg0 + s) << 32) ^ (w + 1));
    else b = splitmix64(seed ^ ((seg0 + s + 1) << 32) ^ 0);
    if (i + 1 < total) {
      u32x4 v = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
      *reinterpret_cast<u32x4*>(o + i) = v;
    } else {
      o[i] = a;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------------
bool layout_vec16_ok(const Layout& L) {
  const uintptr_t bits = (uintptr_t)L.data | (uintptr_t)L.parity | L.shard_stride |
                         L.data_seg_stride | L.par_seg_stride;
  return (bits & 15) == 0;
}

namespace {

constexpr uint32_t kMaxGridY = 65535;

template <class F>
void for_seg_chunks(uint32_t nseg, F f) {
  for (uint32_t s0 = 0; s0 < nseg; s0 += kMaxGridY) f(s0, nseg - s0 < kMaxGridY ? nseg - s0 : kMaxGridY);
}

template <class P, int U, bool NT, class TV = u32x4, int PF = 1, bool WIN = false, int BS = 256>
void run_ct(const Layout& L, const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  if (layout_vec16_ok(L)) {
    const uint64_t nvec = L.len / sizeof(TV);
    uint64_t gx = (nvec + BS * U - 1) / (BS * U);
    if (gx == 0) gx = 1;  // tail-only shard
    for_seg_chunks(nseg, [&](uint32_t s0, uint32_t ny) CEC_AI {
      hipLaunchKernelGGL((k_ct<P, U, NT, TV, PF, WIN, BS>), dim3((unsigned)gx, ny), dim3(BS), 0,
                         st, L, seg_list, s0);
    });
  } else {
    const uint64_t gx = (L.len + 255) / 256;
    for_seg_chunks(nseg, [&](uint32_t s0, uint32_t ny) CEC_AI {
      hipLaunchKernelGGL((k_ct_bytes<P>), dim3((unsigned)gx, ny), dim3(256), 0, st, L, seg_list,
                         s0);
    });
  }
}

// Kernel variants for tuning sweeps (bench.py --sweep) exist only in the tuning build
// (libcessec_tune.so, -DCEC_TUNING); the product library instantiates the default of each.
template <class P>
void run_ct_variant(const KernelOpts& o, const Layout& L, const uint32_t* seg_list,
                    uint32_t nseg, hipStream_t st) {
#ifdef CEC_TUNING
  switch (o.ct_variant) {
    case 0: run_ct<P, 1, false>(L, seg_list, nseg, st); return;
    case 1: run_ct<P, 2, false>(L, seg_list, nseg, st); return;
    case 2: run_ct<P, 4, false>(L, seg_list, nseg, st); return;
    case 3: run_ct<P, 1, true>(L, seg_list, nseg, st); return;
    case 4: run_ct<P, 2, true>(L, seg_list, nseg, st); return;
    case 5: run_ct<P, 4, true>(L, seg_list, nseg, st); return;
    case 6: run_ct<P, 1, true, u32x4, 1, false, 512>(L, seg_list, nseg, st); return;
    case 7: run_ct<P, 1, true, u32x4, 1, false, 128>(L, seg_list, nseg, st); return;
    case 8: run_ct<P, 1, true, u32x4, 1, false, 1024>(L, seg_list, nseg, st); return;
    case 9: case 10: case 11: {
      if (!layout_vec16_ok(L) || (L.len & 15)) break;
      const uint64_t tiles = (L.len / 16 + 255) / 256;
      const unsigned grid = o.ct_variant == 9 ? 2048 : o.ct_variant == 10 ? 4096 : 8192;
      hipLaunchKernelGGL((k_ct_persist<P, true, 256>), dim3(grid), dim3(256), 0, st, L, seg_list,
                         nseg, tiles);
      return;
    }
    case 12: {  // XCD-contiguous tile order
      if (!layout_vec16_ok(L) || (L.len & 15) || P::NI + P::NO > 3) break;
      const uint64_t tiles = (L.len / 16 + 255) / 256;
      const uint64_t total = tiles * nseg;
      if (total >= (1ull << 31)) break;
      hipLaunchKernelGGL((k_ct_xcd<P, true, 256>), dim3((unsigned)(((total + 7) / 8) * 8)),
                         dim3(256), 0, st, L, seg_list, nseg, tiles);
      return;
    }
    default: break;
  }
#else
  (void)o;
#endif
  run_ct<P, 1, true>(L, seg_list, nseg, st);  // r01 sweep winner: one 16-B column, nontemporal
}

// Horner-over-groups kernel; needs 4-byte-aligned shards and 32-bit lane offsets (else the
// nibble-window kernel).
template <class P, int G, int FL, int BS = 256>
void run_hg(const Layout& L, const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  const uintptr_t bits = (uintptr_t)L.data | (uintptr_t)L.parity | L.shard_stride |
                         L.data_seg_stride | L.par_seg_stride;
  if ((bits & 3) || L.len >= (1ull << 32)) {
    run_ct<P, 1, false, uint32_t, 4, true>(L, seg_list, nseg, st);
    return;
  }
  uint64_t gx = (L.len / 4 + BS - 1) / BS;
  if (gx == 0) gx = 1;
  for_seg_chunks(nseg, [&](uint32_t s0, uint32_t ny) CEC_AI {
    hipLaunchKernelGGL((k_hg<P, G, FL, BS>), dim3((unsigned)gx, ny), dim3(BS), 0, st, L,
                       seg_list, s0);
  });
}

// Wide codes: Horner over input groups by default; the tuning build adds the nibble-window /
// streaming forms (per-lane width, prefetch depth) and the k_hg flag variants.
template <class P>
void run_wide_variant(const KernelOpts& o, const Layout& L, const uint32_t* seg_list,
                      uint32_t nseg, hipStream_t st) {
#ifdef CEC_TUNING
  switch (o.ct_variant) {
    case 0: run_ct<P, 1, false, u32x4, 1>(L, seg_list, nseg, st); return;
    case 1: run_ct<P, 1, false, u32x4, 2>(L, seg_list, nseg, st); return;
    case 2: run_ct<P, 1, false, u32x2, 2>(L, seg_list, nseg, st); return;
    case 3: run_ct<P, 1, false, u32x2, 4>(L, seg_list, nseg, st); return;
    case 4: run_ct<P, 1, true, u32x2, 4>(L, seg_list, nseg, st); return;
    case 5: run_ct<P, 1, false, u32x2, 8>(L, seg_list, nseg, st); return;
    case 6: run_ct<P, 1, false, u32x2, 2, true>(L, seg_list, nseg, st); return;
    case 7: run_ct<P, 1, false, uint32_t, 4, true>(L, seg_list, nseg, st); return;
    case 8: run_ct<P, 1, false, u32x2, 4, true>(L, seg_list, nseg, st); return;
    case 9: run_ct<P, 1, false, u32x4, 2, true>(L, seg_list, nseg, st); return;
    case 10: run_ct<P, 1, false, uint32_t, 4, true>(L, seg_list, nseg, st); return;
    case 11: run_hg<P, 3, 0>(L, seg_list, nseg, st); return;
    case 12: run_hg<P, 4, 1>(L, seg_list, nseg, st); return;
    case 13: run_hg<P, 4, 2>(L, seg_list, nseg, st); return;
    case 14: run_hg<P, 4, 4>(L, seg_list, nseg, st); return;
    case 15: run_hg<P, 4, 0, 128>(L, seg_list, nseg, st); return;
    case 16: run_hg<P, 4, 0, 512>(L, seg_list, nseg, st); return;
    case 17: run_hg<P, 4, 8>(L, seg_list, nseg, st); return;
    case 18: run_hg<P, 3, 8>(L, seg_list, nseg, st); return;
    case 19: run_hg<P, 4, 16>(L, seg_list, nseg, st); return;
    case 20: run_hg<P, 4, 17>(L, seg_list, nseg, st); return;
    case 21: run_hg<P, 4, 0>(L, seg_list, nseg, st); return;  // r01 default (matrix form)
    case 22: case 23: case 24:  // FFT with cached loads+stores / NT loads / NT stores
      if (P::NI == 32 && P::NO == 32 &&
          launch_fft_rs3232(L, seg_list, nseg, o.ct_variant == 22 ? 0 : o.ct_variant == 23 ? 1 : 2,
                            st))
        return;
      break;
    case 25: case 26: case 27: case 28: case 29: case 30:
      // FFT memory-side diagnostics (outputs are not parity): no butterflies / loads+stores only,
      // at the natural occupancy / capped at 3 waves per SIMD; 29/30: loads+stores 4 shards at a
      // time, uncapped / capped
      if (P::NI == 32 && P::NO == 32 &&
          launch_fft_rs3232(L, seg_list, nseg,
                            3 | (o.ct_variant >= 29 ? 12 : o.ct_variant & 1 ? 4 : 8) |
                                ((o.ct_variant == 27 || o.ct_variant == 28 || o.ct_variant == 30)
                                     ? 16 : 0),
                            st))
        return;
      break;
    case 31: case 32: case 33:  // FFT with 2 / 4 / 8 column blocks of 4 KiB per workgroup
      if (P::NI == 32 && P::NO == 32 &&
          launch_fft_rs3232(L, seg_list, nseg, 3 | ((1 << (o.ct_variant - 30)) << 5), st))
        return;
      break;
    default: break;
  }
#else
  (void)o;
#endif
  // RS(32,32): additive FFT on bit-sliced data (fft.hip) where the layout allows; else the
  // Horner-over-groups matrix form (r01 sweep: 3.11 -> 5.26 TB/s)
  if (P::NI == 32 && P::NO == 32 && launch_fft_rs3232(L, seg_list, nseg, 3, st)) return;
  run_hg<P, 4, 0>(L, seg_list, nseg, st);
}

}  // namespace

#ifdef CEC_TUNING
int max_ct_variant() { return 90; }  // 70, 72..78, 83, 85: the derivative decoder forms, 79..82, 84, 86 the syndrome-row decoder's (cess_ec.cpp fdd_form)
#else
int max_ct_variant() { return 0; }
#endif

bool launch_encode_ct(const KernelOpts& o, int k, int m, const Layout& L,
                      const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  if (k == 2 && m == 1) { run_ct_variant<EncCT<2, 1>>(o, L, seg_list, nseg, st); return true; }
  if (k == 32 && m == 32) { run_wide_variant<EncCT<32, 32>>(o, L, seg_list, nseg, st); return true; }
  return false;
}

// RS(2,1) verify fused into one pass (cec_verify_batch): the parity 2 (d0 ^ d1) ^ d0 recomputed in
// registers and compared with the stored one, (k+m) F read per segment and nothing written but
// the flag of a segment that differs.
__global__ __launch_bounds__(256) void k_verify21(Layout L, uint8_t* __restrict__ ok,
                                                  uint32_t seg0) {
  const uint32_t seg = seg0 + blockIdx.y;
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v * 16 >= L.len) return;
  const u32x4 d0 = ld16<true>(shard_ptr(L, 0, seg) + v * 16);
  const u32x4 d1 = ld16<true>(shard_ptr(L, 1, seg) + v * 16);
  const u32x4 p = ld16<true>(shard_ptr(L, 2, seg) + v * 16);
  const u32x4 z = xt(d0 ^ d1) ^ d0 ^ p;
  if (z.x | z.y | z.z | z.w) ok[seg] = 0;
}

bool launch_verify_ct(int k, int m, const Layout& L, uint8_t* ok, uint32_t nseg, hipStream_t st) {
  if (k == 32 && m == 32) return launch_fft_rs3232_verify(L, ok, nseg, st);
  if (k != 2 || m != 1 || !layout_vec16_ok(L) || (L.len & 15)) return false;
  const uint64_t gx = (L.len / 16 + 255) / 256;
  for_seg_chunks(nseg, [&](uint32_t s0, uint32_t ny) CEC_AI {
    hipLaunchKernelGGL(k_verify21, dim3((unsigned)gx, ny), dim3(256), 0, st, L, ok, s0);
  });
  return true;
}

bool launch_decode1_mixed(const KernelOpts& o, int k, int m, const Layout& L,
                          const uint32_t* tagged, uint32_t nseg, hipStream_t st) {
  // the default variant only (a variant set for a sweep keeps the per-pattern launches)
  if (k != 2 || m != 1 || o.ct_variant != -1 || !layout_vec16_ok(L)) return false;
  uint64_t gx = (L.len / 16 + 255) / 256;
  if (gx == 0) gx = 1;
  for_seg_chunks(nseg, [&](uint32_t s0, uint32_t ny) CEC_AI {
    hipLaunchKernelGGL((k_ct_dec1_mixed21<true, 256>), dim3((unsigned)gx, ny), dim3(256), 0, st,
                       L, tagged, s0);
  });
  return true;
}

#ifdef CEC_TUNING
// Tuning variant 90: the mixed-pattern RS(2,1) rebuild with the per-segment erasure passed in
// the kernel arguments (2 bits per segment row, 64 rows per launch, segments in natural order)
// instead of a tagged list each workgroup loads first.
template <bool NT, int BS>
__global__ __launch_bounds__(BS) void k_ct_dec1_mixed21_kargs(Layout L, uint32_t seg0,
                                                              uint64_t t0, uint64_t t1) {
  const uint32_t y = blockIdx.y;
  const uint64_t w = y < 32 ? t0 : t1;
  const uint32_t e = (uint32_t)(w >> (2 * (y & 31))) & 3u;
  const uint32_t seg = seg0 + y;
  if (e == 0) ct_tile<Dec1CT<2, 1, 0>, 1, NT, u32x4, 1, false, BS>(L, seg);
  else if (e == 1) ct_tile<Dec1CT<2, 1, 1>, 1, NT, u32x4, 1, false, BS>(L, seg);
  else if (e == 2) ct_tile<EncCT<2, 1>, 1, NT, u32x4, 1, false, BS>(L, seg);
  // e == 3: a segment with nothing to rebuild in this launch, left untouched
}
#endif

bool launch_decode1_mixed_kargs(int k, int m, const Layout& L, const uint8_t* erased,
                                uint32_t nseg, hipStream_t st) {
#ifdef CEC_TUNING
  if (k != 2 || m != 1 || !layout_vec16_ok(L)) return false;
  uint64_t gx = (L.len / 16 + 255) / 256;
  if (gx == 0) gx = 1;
  for (uint32_t s0 = 0; s0 < nseg; s0 += 64) {
    const uint32_t ny = nseg - s0 < 64 ? nseg - s0 : 64;
    uint64_t t[2] = {0, 0};
    for (uint32_t y = 0; y < ny; ++y) t[y >> 5] |= (uint64_t)(erased[s0 + y] & 3u) << (2 * (y & 31));
    hipLaunchKernelGGL((k_ct_dec1_mixed21_kargs<true, 256>), dim3((unsigned)gx, ny), dim3(256), 0,
                       st, L, s0, t[0], t[1]);
  }
  return true;
#else
  (void)k; (void)m; (void)L; (void)erased; (void)nseg; (void)st;
  return false;
#endif
}

bool launch_decode_ct(const KernelOpts& o, int k, int m, int missing, const Layout& L,
                      const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  if (k == 2 && m == 1) {
    switch (missing) {
      case 0: run_ct_variant<Dec1CT<2, 1, 0>>(o, L, seg_list, nseg, st); return true;
      case 1: run_ct_variant<Dec1CT<2, 1, 1>>(o, L, seg_list, nseg, st); return true;
      case 2: run_ct_variant<EncCT<2, 1>>(o, L, seg_list, nseg, st); return true;
    }
  }
  return false;
}

int rt_bucket(int nout) {
  static const int b[] = {1, 2, 3, 4, 5, 6, 7, 8, 12, 16, 24, 32};
  for (int x : b)
    if (x >= nout) return x;
  return kRtMaxOut;
}

bool has_decode_ct(int k, int m, int missing) {
  return k == 2 && m == 1 && missing >= 0 && missing < 3;
}

namespace {
template <int NOB, int U, class TV>
void run_rt(const Layout& L, const uint32_t* chunk, const uint32_t* const* per_seg,
            const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  const int vec_ok = layout_vec16_ok(L) ? 1 : 0;
  uint64_t gx = vec_ok ? (L.len / sizeof(TV) + 256 * U - 1) / (256 * U) : (L.len + 255) / 256;
  if (gx == 0) gx = 1;
  for_seg_chunks(nseg, [&](uint32_t s0, uint32_t ny) {
    hipLaunchKernelGGL((k_rt<NOB, U, TV>), dim3((unsigned)gx, ny), dim3(256), 0, st, L, chunk,
                       per_seg, seg_list, s0, vec_ok);
  });
}
}  // namespace

void launch_matvec_rt(const Layout& L, const uint32_t* chunk, const uint32_t* const* per_seg,
                      int nob, const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  switch (nob) {
    case 1: run_rt<1, 1, u32x4>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 2: run_rt<2, 1, u32x4>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 3: run_rt<3, 1, u32x4>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 4: run_rt<4, 1, u32x4>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 5: run_rt<5, 1, u32x4>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 6: run_rt<6, 1, u32x4>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 7: run_rt<7, 1, u32x2>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 8: run_rt<8, 1, u32x2>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 12: run_rt<12, 1, u32x2>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 16: run_rt<16, 1, uint32_t>(L, chunk, per_seg, seg_list, nseg, st); break;
    case 24: run_rt<24, 1, uint32_t>(L, chunk, per_seg, seg_list, nseg, st); break;
    default: run_rt<32, 1, uint32_t>(L, chunk, per_seg, seg_list, nseg, st); break;
  }
}

namespace {
template <int NOB, class TV, int PF>
void run_rtb(const Layout& L, const uint32_t* chunk, const uint32_t* const* per_seg,
             const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  const int vec_ok = layout_vec16_ok(L) ? 1 : 0;
  uint64_t gx = vec_ok ? (L.len / sizeof(TV) + 255) / 256 : (L.len + 255) / 256;
  if (gx == 0) gx = 1;
  for_seg_chunks(nseg, [&](uint32_t s0, uint32_t ny) {
    hipLaunchKernelGGL((k_rtb<NOB, TV, PF>), dim3((unsigned)gx, ny), dim3(256), 0, st, L, chunk,
                       per_seg, seg_list, s0, vec_ok);
  });
}
}  // namespace

bool launch_matvec_rtb(const Layout& L, const uint32_t* chunk, const uint32_t* const* per_seg,
                       int nob, const uint32_t* seg_list, uint32_t nseg, hipStream_t st,
                       int variant) {
#ifdef CEC_TUNING
  // tuning build (TV = column width per lane, PF = input columns in flight):
  // two outputs 40-43 = u32x4 PF1 (the first default) / u32x2 PF8 / u32x4 PF2 / u32x2 PF2;
  // one output 44-47 = u32x4 PF1 (the first default) / u32x2 PF2 / u32x2 PF1 / u32 PF4;
  // three or four outputs 48-49 = u32 PF8 / u32x2 PF4 (the first default for four)
  if (variant >= 40 && variant <= 49) {
    const int v = variant;
    if (nob == 2 && v <= 43) {
      if (v == 40) run_rtb<2, u32x4, 1>(L, chunk, per_seg, seg_list, nseg, st);
      else if (v == 41) run_rtb<2, u32x2, 8>(L, chunk, per_seg, seg_list, nseg, st);
      else if (v == 42) run_rtb<2, u32x4, 2>(L, chunk, per_seg, seg_list, nseg, st);
      else run_rtb<2, u32x2, 2>(L, chunk, per_seg, seg_list, nseg, st);
      return true;
    }
    if (nob == 1 && v >= 44 && v <= 47) {
      if (v == 44) run_rtb<1, u32x4, 1>(L, chunk, per_seg, seg_list, nseg, st);
      else if (v == 45) run_rtb<1, u32x2, 2>(L, chunk, per_seg, seg_list, nseg, st);
      else if (v == 46) run_rtb<1, u32x2, 1>(L, chunk, per_seg, seg_list, nseg, st);
      else run_rtb<1, uint32_t, 4>(L, chunk, per_seg, seg_list, nseg, st);
      return true;
    }
    if ((nob == 3 || nob == 4) && v >= 48) {
      if (nob == 3 && v == 48) run_rtb<3, uint32_t, 8>(L, chunk, per_seg, seg_list, nseg, st);
      else if (nob == 3) run_rtb<3, u32x2, 4>(L, chunk, per_seg, seg_list, nseg, st);
      else if (v == 48) run_rtb<4, uint32_t, 8>(L, chunk, per_seg, seg_list, nseg, st);
      else run_rtb<4, u32x2, 4>(L, chunk, per_seg, seg_list, nseg, st);
      return true;
    }
  }
#else
  (void)variant;
#endif
  switch (nob) {
    // 8-byte columns, several in flight (profiles/r02/rtb_sweep.txt: one output u32x4 PF1 ->
    // u32x2 PF4 0.199 -> 0.184 ms, four outputs PF4 -> PF8 0.296 -> 0.291)
    case 1: run_rtb<1, u32x2, 4>(L, chunk, per_seg, seg_list, nseg, st); return true;
    case 2: run_rtb<2, u32x2, 4>(L, chunk, per_seg, seg_list, nseg, st); return true;
    case 3: run_rtb<3, u32x2, 4>(L, chunk, per_seg, seg_list, nseg, st); return true;
    case 4: run_rtb<4, u32x2, 8>(L, chunk, per_seg, seg_list, nseg, st); return true;
  }
  return false;
}

namespace {
// rt_mode 0: Horner over input groups with index-mode XORs (k_rthx) where possible,
// 1: always k_rt (per-bit masks), 2: Horner with v_mov table reads (k_rth)
template <int NG>
void run_rth(int rt_mode, const Layout& L, const uint32_t* chunk, const uint32_t* const* per_seg,
             const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  const uintptr_t bits = (uintptr_t)L.data | (uintptr_t)L.parity | L.shard_stride |
                         L.data_seg_stride | L.par_seg_stride;
  const int vec_ok = (bits & 3) == 0;
  uint64_t gx = vec_ok ? (L.len / 4 + 255) / 256 : (L.len + 255) / 256;
  if (gx == 0) gx = 1;
  for_seg_chunks(nseg, [&](uint32_t s0, uint32_t ny) {
    if (rt_mode == 0)
      hipLaunchKernelGGL((k_rthx<NG>), dim3((unsigned)gx, ny), dim3(256), 0, st, L, chunk,
                         per_seg, seg_list, s0, vec_ok);
    else
      hipLaunchKernelGGL((k_rth<NG>), dim3((unsigned)gx, ny), dim3(256), 0, st, L, chunk,
                         per_seg, seg_list, s0, vec_ok);
  });
}
}  // namespace

bool launch_matvec_rth(const KernelOpts& o, const Layout& L, const uint32_t* chunk,
                       const uint32_t* const* per_seg, int nin_max, const uint32_t* seg_list,
                       uint32_t nseg, hipStream_t st) {
  // measured (profiles/r01/rt_modes.txt): faster than k_rt from 4 inputs up (k_rthx / k_rth /
  // k_rt: RS(10,4) encode 3.2 / 3.0 / 2.7 TB/s, RS(32,32) one-fragment repair 4.0 / 4.0 / 3.1,
  // 32-erasure rebuild 1.76 / 1.1 / 0.96); for 2-3 inputs k_rt's 16-byte columns win (RS(2,1)
  // run-time encode 6.0 vs 2.9 TB/s)
  if (o.rt_mode == 1 || nin_max > kRthMaxIn || nin_max < 4) return false;
  const int ng = (nin_max + 3) / 4;
  if (ng <= 1) run_rth<1>(o.rt_mode, L, chunk, per_seg, seg_list, nseg, st);
  else if (ng == 2) run_rth<2>(o.rt_mode, L, chunk, per_seg, seg_list, nseg, st);
  else if (ng == 3) run_rth<3>(o.rt_mode, L, chunk, per_seg, seg_list, nseg, st);
  else if (ng == 4) run_rth<4>(o.rt_mode, L, chunk, per_seg, seg_list, nseg, st);
  else if (ng <= 6) run_rth<6>(o.rt_mode, L, chunk, per_seg, seg_list, nseg, st);
  else run_rth<8>(o.rt_mode, L, chunk, per_seg, seg_list, nseg, st);
  return true;
}

void launch_fill_splitmix(uint8_t* out, uint64_t seg_bytes, uint64_t nseg, uint64_t seg0,
                          uint64_t seed, hipStream_t st) {
  const uint64_t words = (seg_bytes >> 3) * nseg;
  uint64_t blocks = (words / 2 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)blocks), dim3(256), 0, st, out, seg_bytes, nseg, seg0,
                     seed);
}

}  // namespace cec
