// Host-side plans of the RS(32,32) erasure decoder on the additive FFT (fftdec.hip). Host only,
// header-inlined so the CPU model test (tests/native/fftdec_model.cpp) builds the same plans.
//
// The code (gf256.h): data shard t = f(t), parity shard t = f(32 ^ t) for the unique f of degree
// < 32. The plan takes one coset as A (its present shards are read, its erased shards zeroed)
// and the other as B:
//   T1   q = FFT_B(IFFT_A(A values, erased zeroed)): the polynomial f_q agreeing with f on A's
//        present points and vanishing on A's erased set D, evaluated on B;
//   h    = f - f_q has degree < 32 and vanishes on A \ D, so it is fixed by its values u on D, and
//        its values on B are linear in u: h(x) = sum_{c in D} u_c l_c(x), l_c the Lagrange basis
//        of the coset A. At d = |D| present points R of B the syndromes s = p_R ^ q_R = h(R) give
//        u = inv(L[R][D]) s (any d points of B work: the code is MDS);
//   out  erased c in D: u_c; erased e in B: q_e ^ h(e) = q_e ^ L[e][D] inv(L[R][D]) s.
// Mode M (matvec) applies those rows to the syndromes in the kernel, in bit-plane form: cost
// (outputs) x (slots holding R), so the plan takes A = the coset with fewer erasures and packs R
// into as few lane-pair slots (positions 2j, 2j + 1) as the present shards allow. A row is applied
// by Horner over the coefficient bits: out = sum_b 2^b T_b, T_b = XOR of the syndromes whose
// coefficient has bit b, so a (row, slot) pair costs one mask per bit (8 words) instead of one per
// entry of its 8 x 8 bit matrix (64): the plan stays in the scalar cache at 32 outputs.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "gf256.h"

namespace cec {

// Word layout of a decode plan in HBM (uint32 words).
struct FftDecLayout {
  static constexpr int kFlags = 0;   // bit 0: side (0: A = data coset, 1: A = parity coset);
                                     // bits 8..15: mode (0 = M)
  static constexpr int kPresA = 1;   // bit t: shard t of coset A is read (present)
  static constexpr int kR = 2;       // bit t: shard t of coset B is a syndrome row (read)
  static constexpr int kEB = 3;      // bit t: shard t of coset B is not read
  static constexpr int kDA = 4;      // bit t: shard t of coset A is not read
  static constexpr int kNout = 5;    // outputs written
  static constexpr int kRslots = 6;  // bit j: slot j (positions 2j, 2j + 1 of B) holds R rows
  static constexpr int kPslots = 7;  // bit j: slot j is packed (R or an output on B)
  static constexpr int kNrs = 8;     // popcount(kRslots)
  static constexpr int kNpk = 9;
  static constexpr int kNrs1 = 10;   // 1 << nrs     // bit r: register slot r is packed after the swaps
  static constexpr int kSwap = 16;   // [16]: 1 << j_i, j_i the i-th R slot ascending (the kernel
                                     // swaps register slots i and j_i for i < nrs: R slots land
                                     // in [0, nrs))
  static constexpr int kRsl = 32;    // [16]: j_i | (R bits of slot j_i: even, odd) << 8
  static constexpr int kOuts = 48;   // [32]: output o = t | (on B) << 5 | (1 << the register slot
                                     // of its q after the swaps) << 16
  static constexpr int kMasks = 80;  // [nout][8 bits b][nrs]: bit b of the row's coefficients of
                                     // the slot's even (low nibbles) and odd (high) position
  static size_t words(int nout, int nrslots) { return kMasks + (size_t)nout * nrslots * 8; }
};

struct FftDecPlan {
  std::vector<uint32_t> w;  // the device image
  int side = 0, nout = 0, nrslots = 0;
};

namespace fdp {

inline int popc(uint32_t x) { return __builtin_popcount(x); }

// l_c(x) for the Lagrange basis of the coset {base ^ t}: prod_{a != c} (x ^ a) / (c ^ a)
inline uint8_t lagrange(unsigned base, unsigned c, unsigned x) {
  uint8_t num = 1, den = 1;
  for (unsigned t = 0; t < 32; ++t) {
    const unsigned a = base ^ t;
    if (a == c) continue;
    num = gf_mul(num, (uint8_t)(x ^ a));
    den = gf_mul(den, (uint8_t)(c ^ a));
  }
  return gf_mul(num, gf_inv(den));
}

}  // namespace fdp

// The survivors an RS(32,32) rebuild reads (the codec's survivor choice, cec_survivors): every
// present shard of the coset A with fewer lost shards (data on a tie), and d = (lost in A) present
// shards of the other coset B chosen for the syndrome-row decoder below: whole present lane-pair
// slots (positions 2j, 2j + 1) first, then a lone present position whose slot holds a lost shard
// (packed anyway), then any. Any k present shards rebuild the same bytes (MDS); this choice keeps
// the syndrome rows in as few slots as the pattern allows (first-k-present costs 1.3-1.5x the
// slots at 8-24 erasures). `read` gets 64 flags. False when more than 32 shards are lost.
inline bool fftdec_read_set(const uint8_t* present, uint8_t* read) {
  uint32_t lost_d = 0, lost_p = 0;
  for (int t = 0; t < 32; ++t) {
    if (!present[t]) lost_d |= 1u << t;
    if (!present[32 + t]) lost_p |= 1u << t;
  }
  const int nd = fdp::popc(lost_d), np = fdp::popc(lost_p);
  if (nd + np > 32) return false;
  const int side = np < nd ? 1 : 0;
  const uint32_t DA = side ? lost_p : lost_d, EB = side ? lost_d : lost_p;
  const unsigned baseA = side ? 32u : 0u, baseB = side ? 0u : 32u;
  uint32_t R = 0;
  int need = fdp::popc(DA);
  for (int j = 0; j < 16 && need >= 2; ++j)
    if (!(EB >> (2 * j) & 3)) {
      R |= 3u << (2 * j);
      need -= 2;
    }
  for (int pass = 0; pass < 2 && need > 0; ++pass)
    for (int t = 0; t < 32 && need > 0; ++t) {
      if ((EB >> t & 1) || (R >> t & 1)) continue;
      const bool packed = (EB >> (t ^ 1) & 1) || (R >> (t ^ 1) & 1);
      if (pass == 0 && !packed) continue;
      R |= 1u << t;
      --need;
    }
  for (int t = 0; t < 32; ++t) {
    read[baseA + t] = !(DA >> t & 1);
    read[baseB + t] = (R >> t & 1) ? 1 : 0;
  }
  return true;
}

// The survivors a rebuild of `present` reads (the C ABI's cec_survivors; k + m flags into
// `read`): for RS(32,32) fftdec_read_set's choice, otherwise the first k present shards
// (klauspost's). False when fewer than k shards are present.
inline bool survivor_set(int k, int m, const uint8_t* present, uint8_t* read) {
  if (k == 32 && m == 32) return fftdec_read_set(present, read);
  int got = 0;
  for (int i = 0; i < k + m; ++i) {
    read[i] = present[i] && got < k;
    got += read[i];
  }
  return got == k;
}

// Build the mode-M plan for RS(32,32) erasure pattern `present` (64 flags, shards 0..31 data,
// 32..63 parity) that reads only the shards flagged in `read` (a subset of the present ones: the
// codec's contract is that a rebuild reads the first k present shards, the survivors a caller
// stages — cess_ec.cpp's host API and the multi-GPU gathers move only those). Every shard not
// read is an erasure to the algorithm; the outputs are the shards not present (data_only: data
// shards only). Returns false when more than 32 shards are unread (the caller reports ETOOFEW) or
// there is nothing to write.
inline bool fftdec_plan_m(const uint8_t* read, const uint8_t* present, bool data_only,
                          FftDecPlan* out) {
  uint32_t erd = 0, erp = 0;  // unread data / parity
  uint32_t lost_d = 0, lost_p = 0;  // not present (the outputs)
  for (int t = 0; t < 32; ++t) {
    if (!read[t]) erd |= 1u << t;
    if (!read[32 + t]) erp |= 1u << t;
    if (!present[t]) lost_d |= 1u << t;
    if (!present[32 + t]) lost_p |= 1u << t;
  }
  if ((lost_d & ~erd) || (lost_p & ~erp)) return false;  // a read shard must be present
  const int nd = fdp::popc(erd), np = fdp::popc(erp);
  if (nd + np > 32 || nd + np == 0) return false;
  // A = the coset with fewer erasures (fewer syndrome rows); data on a tie
  const int side = np < nd ? 1 : 0;
  const unsigned baseA = side ? 32u : 0u, baseB = side ? 0u : 32u;
  const uint32_t DA = side ? erp : erd, EB = side ? erd : erp;
  // outputs on A (within DA) and on B (within EB)
  const uint32_t OA = (side ? lost_p : lost_d) & ~(data_only && side == 1 ? ~0u : 0u);
  const uint32_t OB = (side ? lost_d : lost_p) & ~(data_only && side == 0 ? ~0u : 0u);
  const int d = fdp::popc(DA);
  // R: d present points of B packed into few slots: whole present slots first, then a lone
  // read position of a slot that is packed anyway (it holds an output), then any
  uint32_t R = 0;
  int need = d;
  for (int j = 0; j < 16 && need >= 2; ++j)
    if (!(EB >> (2 * j) & 3)) {
      R |= 3u << (2 * j);
      need -= 2;
    }
  for (int pass = 0; pass < 2 && need > 0; ++pass)
    for (int t = 0; t < 32 && need > 0; ++t) {
      if ((EB >> t & 1) || (R >> t & 1)) continue;
      const bool packed = (OB >> (t ^ 1) & 1) || (R >> (t ^ 1) & 1);
      if (pass == 0 && !packed) continue;
      R |= 1u << t;
      --need;
    }
  if (need) return false;  // cannot happen with <= 32 erasures
  uint32_t rslots = 0, pslots = 0;
  for (int j = 0; j < 16; ++j) {
    if (R >> (2 * j) & 3) rslots |= 1u << j;
    if ((R | OB) >> (2 * j) & 3) pslots |= 1u << j;
  }
  // outputs: lost data always; lost parity unless data_only
  std::vector<uint32_t> outs;
  for (int t = 0; t < 32; ++t) {
    if (OA >> t & 1) outs.push_back((uint32_t)t);
    if (OB >> t & 1) outs.push_back((uint32_t)t | 32u);
  }
  if (outs.empty()) return false;
  // u = inv(L[R][D]) s;  h(e) = L[e][D] u
  std::vector<unsigned> Dl, Rl;
  for (int t = 0; t < 32; ++t) {
    if (DA >> t & 1) Dl.push_back(baseA ^ (unsigned)t);
    if (R >> t & 1) Rl.push_back(baseB ^ (unsigned)t);
  }
  using M64 = Mat<32, 32>;
  using W64 = Mat<32, 64>;
  M64 lr, linv;
  W64 work;
  for (int r = 0; r < d; ++r)
    for (int c = 0; c < d; ++c) lr.v[r][c] = fdp::lagrange(baseA, Dl[c], Rl[r]);
  if (d && !gf_invert(lr, d, linv, work)) return false;  // cannot happen (MDS)
  const int nrs = fdp::popc(rslots);
  FftDecPlan p;
  p.side = side;
  p.nout = (int)outs.size();
  p.nrslots = nrs;
  p.w.assign(FftDecLayout::words(p.nout, nrs), 0u);
  uint32_t* w = p.w.data();
  w[FftDecLayout::kFlags] = (uint32_t)side;
  w[FftDecLayout::kPresA] = ~DA;
  w[FftDecLayout::kR] = R;
  w[FftDecLayout::kEB] = EB;
  w[FftDecLayout::kDA] = DA;
  w[FftDecLayout::kNout] = (uint32_t)p.nout;
  w[FftDecLayout::kRslots] = rslots;
  w[FftDecLayout::kPslots] = pslots;
  w[FftDecLayout::kNrs] = (uint32_t)nrs;
  w[FftDecLayout::kNrs1] = 1u << nrs;
  // the kernel's slot swaps: step i exchanges register slots i and j_i (j_i >= i, and no earlier
  // step touched slot j_i), so R slot j_i ends in slot i; where every other slot ends (an erased
  // B output's q) follows from the same swaps
  int jr[16], at[16];  // jr: R slots ascending; at[j]: register slot holding original slot j
  for (int j = 0, i = 0; j < 16; ++j)
    if (rslots >> j & 1) jr[i++] = j;
  int reg[16];  // reg[r]: original slot in register slot r
  for (int j = 0; j < 16; ++j) reg[j] = j;
  for (int i = 0; i < nrs; ++i) {
    w[FftDecLayout::kSwap + i] = 1u << jr[i];
    std::swap(reg[i], reg[jr[i]]);
  }
  uint32_t npk = 0;
  for (int r = 0; r < 16; ++r) {
    at[reg[r]] = r;
    if (pslots >> reg[r] & 1) npk |= 1u << r;
  }
  w[FftDecLayout::kNpk] = npk;
  for (int i = 0; i < nrs; ++i)
    w[FftDecLayout::kRsl + i] = (uint32_t)jr[i] | (R >> (2 * jr[i]) & 3u) << 8;
  // syndrome index of each R position (column of the rows below)
  int ridx[32];
  for (int i = 0, t = 0; t < 32; ++t) ridx[t] = (R >> t & 1) ? i++ : -1;
  for (int o = 0; o < p.nout; ++o) {
    const uint32_t od = outs[o];
    const unsigned t = od & 31;
    w[FftDecLayout::kOuts + o] = od | (1u << at[t >> 1]) << 16;
    uint8_t row[32] = {};  // coefficients over the syndromes
    if (!(od & 32)) {      // an erased point of A: row of inv(L[R][D])
      const int di = (int)(std::find(Dl.begin(), Dl.end(), baseA ^ t) - Dl.begin());
      for (int r = 0; r < d; ++r) row[r] = linv.v[di][r];
    } else {  // an erased point of B: L[e][D] inv(L[R][D])
      const unsigned e = baseB ^ t;
      for (int c = 0; c < d; ++c) {
        const uint8_t le = fdp::lagrange(baseA, Dl[c], e);
        if (!le) continue;
        for (int r = 0; r < d; ++r) row[r] ^= gf_mul(le, linv.v[c][r]);
      }
    }
    uint32_t* mk = w + FftDecLayout::kMasks + (size_t)o * nrs * 8;
    for (int b = 0; b < 8; ++b)
      for (int i = 0; i < nrs; ++i) {
        const int lo = ridx[2 * jr[i]], hi = ridx[2 * jr[i] + 1];
        const bool bl = lo >= 0 && (row[lo] >> b & 1), bh = hi >= 0 && (row[hi] >> b & 1);
        mk[b * nrs + i] = (bl ? 0x0F0F0F0Fu : 0u) | (bh ? 0xF0F0F0F0u : 0u);
      }
  }
  *out = std::move(p);
  return true;
}

// ---- mode D: the formal-derivative decoder (k_fftdec_d, fftdec_d.hip) ---------------------------
// Lin-Chung-Han erasure decoding over the whole 64-point space (points = shard indices): with E the
// erased set and the error locator lam(x) = prod_{e in E} (x ^ e), g = lam * f has degree < 64 and
// its values lam(t) c_t at every point are known (zero on E). So
//   g   = IFFT_64(lam(t) c_t)               (novel-basis coefficients of g)
//   g'  = formal derivative of g            (compile-time constants, fftdec_d.hip)
//   c_e = FFT_64(g')(e) / lam'(e)           (lam(e) = 0, so g'(e) = lam'(e) f(e))
// Its cost does not depend on how many shards are lost: two 64-point transforms, the derivative,
// and per position one run-time multiplication in (lam(t)) and one out (1 / lam'(e)).
// Plan words (uint32), per register slot j of the kernel (positions 4j + l, l = 0..3 the lane of
// a quad), byte l of the word belongs to position 4j + l.
struct FftDecDLayout {
  static constexpr int kFlags = 0;  // bits 8..15: mode (1 = D)
  static constexpr int kNout = 1;
  static constexpr int kLam = 16;   // [16]: lam(t) of a read t, 0 elsewhere
  static constexpr int kDinv = 32;  // [16]: 1 / lam'(t) of an output t, 0 elsewhere
  // the same constants as bit masks, one word per (slot j, lane l, bit b): 0 or ~0 = bit b of the
  // constant of position 4j + l (the kernel's per-lane Horner masks, copied to LDS)
  static constexpr int kMasks = 48;  // [2][16][4][8]: lam, then 1 / lam'
  // the merged constant of each position, as the same masks: lam(t) where t is read, 1 / lam'(t)
  // where it is an output, 0 elsewhere (a position is never both): the pipelined kernel multiplies
  // the next column block's inputs and this block's outputs in one pass
  static constexpr int kMerged = kMasks + 2 * 16 * 4 * 8;  // [16][4][8]
  static constexpr int kWords = kMerged + 16 * 4 * 8;
};

// Build the mode-D plan for RS(32,32) pattern `present` (64 flags) reading only the shards flagged
// in `read` (present ones; see fftdec_plan_m): the locator's roots are the unread shards, the
// outputs the shards not present. False when more than 32 shards are unread or there is nothing
// to write.
inline bool fftdec_plan_d(const uint8_t* read, const uint8_t* present, bool data_only,
                          FftDecPlan* out) {
  int ne = 0, nout = 0;
  uint8_t erased[64];
  for (int t = 0; t < 64; ++t) {
    if (read[t] && !present[t]) return false;  // a read shard must be present
    if (!read[t]) erased[ne++] = (uint8_t)t;
  }
  if (ne == 0 || ne > 32) return false;
  FftDecPlan p;
  p.side = 0;
  p.w.assign(FftDecDLayout::kWords, 0u);
  uint32_t* w = p.w.data();
  w[FftDecDLayout::kFlags] = 1u << 8;
  for (int t = 0; t < 64; ++t) {
    uint8_t lam = 1;  // lam(t), or lam'(t) = prod_{e != t} (t ^ e) at an erased t
    for (int i = 0; i < ne; ++i)
      if (erased[i] != t) lam = gf_mul(lam, (uint8_t)(t ^ erased[i]));
    const int sh = 8 * (t & 3);
    if (read[t]) {
      w[FftDecDLayout::kLam + (t >> 2)] |= (uint32_t)lam << sh;
    } else if (!present[t] && !(data_only && t >= 32)) {
      w[FftDecDLayout::kDinv + (t >> 2)] |= (uint32_t)gf_inv(lam) << sh;
      ++nout;
    }
  }
  if (!nout) return false;
  w[FftDecDLayout::kNout] = (uint32_t)nout;
  for (int which = 0; which < 3; ++which)
    for (int t = 0; t < 64; ++t) {
      auto byte = [&](int base) { return (uint8_t)(w[base + (t >> 2)] >> (8 * (t & 3))); };
      const uint8_t c = which == 0 ? byte(FftDecDLayout::kLam)
                        : which == 1 ? byte(FftDecDLayout::kDinv)
                                     : (uint8_t)(byte(FftDecDLayout::kLam) | byte(FftDecDLayout::kDinv));
      for (int b = 0; b < 8; ++b)
        w[FftDecDLayout::kMasks + ((which * 16 + (t >> 2)) * 4 + (t & 3)) * 8 + b] =
            (c >> b & 1) ? 0xFFFFFFFFu : 0u;
    }
  p.nout = nout;
  *out = std::move(p);
  return true;
}

}  // namespace cec
