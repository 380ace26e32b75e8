// CPU model of the RS(32,32) FFT-domain erasure decoder (cess_amd/csrc/fftdec.hip) on the plans
// the library builds (cess_amd/csrc/fftdec_plan.h): per byte column, T1 (IFFT over coset A with
// its erased shards zeroed, FFT onto coset B), the syndromes at the plan's R rows, and every output
// from the plan's bit-plane masks exactly as the kernel applies them (low / high nibble = the
// slot's even / odd position), including the register-slot swaps that bring the R slots to the
// front and the Horner pass over each row's coefficient bits. Compared with the codeword of the product's own encode matrix for
// random erasure patterns of 1..32 shards, both sides, with and without data_only.
// The formal-derivative decoder's plans (fftdec_plan_d, kernel cess_amd/csrc/fftdec_d.hip) run
// through the same patterns: lam(t) c_t from the plan's bytes, the 64-point IFFT, the derivative
// with gf256.h's constants, the 64-point FFT, times the plan's 1 / lam'(e) at every output.
// Build: g++ -std=c++20 -O1 -fconstexpr-ops-limit=2000000000 fftdec_model.cpp
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../cess_amd/csrc/fftdec_plan.h"

using namespace cec;

static void ifft(uint8_t* v, unsigned beta) {
  const LchSkews<5> S = lch_skews<5>((uint8_t)beta);
  for (int i = 0; i < 5; ++i) {
    const int h = 1 << i;
    for (int b0 = 0; b0 < 32; b0 += 2 * h)
      for (int t = b0; t < b0 + h; ++t) {
        v[t + h] ^= v[t];
        v[t] ^= gf_mul(S.s[i][b0 >> (i + 1)], v[t + h]);
      }
  }
}
static void fft(uint8_t* v, unsigned beta) {
  const LchSkews<5> S = lch_skews<5>((uint8_t)beta);
  for (int i = 4; i >= 0; --i) {
    const int h = 1 << i;
    for (int b0 = 0; b0 < 32; b0 += 2 * h)
      for (int t = b0; t < b0 + h; ++t) {
        v[t] ^= gf_mul(S.s[i][b0 >> (i + 1)], v[t + h]);
        v[t + h] ^= v[t];
      }
  }
}
static void ifft64(uint8_t* v) {
  const LchSkews<6> S = lch_skews<6>(0);
  for (int i = 0; i < 6; ++i) {
    const int h = 1 << i;
    for (int b0 = 0; b0 < 64; b0 += 2 * h)
      for (int t = b0; t < b0 + h; ++t) {
        v[t + h] ^= v[t];
        v[t] ^= gf_mul(S.s[i][b0 >> (i + 1)], v[t + h]);
      }
  }
}
static void fft64(uint8_t* v) {
  const LchSkews<6> S = lch_skews<6>(0);
  for (int i = 5; i >= 0; --i) {
    const int h = 1 << i;
    for (int b0 = 0; b0 < 64; b0 += 2 * h)
      for (int t = b0; t < b0 + h; ++t) {
        v[t] ^= gf_mul(S.s[i][b0 >> (i + 1)], v[t + h]);
        v[t + h] ^= v[t];
      }
  }
}
// mode D on one byte column: the fails it finds
static int check_d(const uint8_t* read, const uint8_t* present, bool data_only, const uint8_t* cw,
                   int* cases) {
  FftDecPlan p;
  int want = 0, fails = 0;
  for (int i = 0; i < 64; ++i) want += !present[i] && (!data_only || i < 32);
  if (!fftdec_plan_d(read, present, data_only, &p)) return want ? 1 : 0;
  const uint32_t* w = p.w.data();
  if ((int)w[FftDecDLayout::kNout] != want || (w[FftDecDLayout::kFlags] >> 8 & 255) != 1) ++fails;
  auto byte = [&](int base, int t) { return (uint8_t)(w[base + (t >> 2)] >> (8 * (t & 3))); };
  uint8_t v[64], d[64] = {};
  for (int t = 0; t < 64; ++t) {
    const uint8_t lam = byte(FftDecDLayout::kLam, t);
    if ((lam != 0) != (read[t] != 0)) ++fails;  // only the read shards are loaded
    v[t] = gf_mul(lam, cw[t]);
  }
  // the pipelined kernel's merged constants: lam where read, 1 / lam' where an output, never both
  for (int t = 0; t < 64; ++t) {
    const uint8_t lam = byte(FftDecDLayout::kLam, t), di = byte(FftDecDLayout::kDinv, t);
    if (lam && di) ++fails;
    uint8_t merged = 0;
    for (int b = 0; b < 8; ++b) {
      const uint32_t mk = w[FftDecDLayout::kMerged + ((t >> 2) * 4 + (t & 3)) * 8 + b];
      if (mk != 0 && mk != 0xFFFFFFFFu) ++fails;
      merged |= (uint8_t)((mk & 1) << b);
    }
    if (merged != (lam | di)) ++fails;
  }
  ifft64(v);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 6; ++j)
      if (i >> j & 1) d[i - (1 << j)] ^= gf_mul(lch_dconst(j), v[i]);
  fft64(d);
  for (int t = 0; t < 64; ++t) {
    const uint8_t di = byte(FftDecDLayout::kDinv, t);
    const bool out = !present[t] && (!data_only || t < 32);
    if ((di != 0) != out) ++fails;
    if (!out) continue;
    ++*cases;
    if (gf_mul(d[t], di) != cw[t]) ++fails;
  }
  return fails;
}
// bit-sliced x -> 2x (poly 0x11D) on one byte
static uint8_t xt(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1D : 0)); }

int main() {
  using Big = Mat<64, 64>;
  using BigW = Mat<64, 128>;
  static Big E, top, topinv;
  static BigW work;
  if (!gf_encode_matrix(32, 32, E, top, topinv, work)) return 2;
  std::mt19937_64 rng(12345);
  int fails = 0, cases = 0, dfails = 0, dcases = 0;
  for (int trial = 0; trial < 600; ++trial) {
    const int e = trial < 64 ? 1 + trial % 32 : 1 + (int)(rng() % 32);
    uint8_t present[64];
    for (int i = 0; i < 64; ++i) present[i] = 1;
    int left = e;
    while (left) {
      const int i = (int)(rng() % 64);
      if (present[i]) {
        present[i] = 0;
        --left;
      }
    }
    if (trial % 7 == 3)  // a structured pattern: the first e shards of one coset
      for (int i = 0; i < 64; ++i) present[i] = !(i >= (trial & 32) && i < (trial & 32) + e);
    const bool data_only = trial % 3 == 1;
    // the shards the plans may read: the first 32 present (the codec's survivors, all a caller
    // stages), or on odd trials any 32 present ones
    uint8_t read[64] = {};
    {
      int idx[64], np = 0;
      for (int i = 0; i < 64; ++i)
        if (present[i]) idx[np++] = i;
      if (trial & 1)
        for (int i = np - 1; i > 0; --i) std::swap(idx[i], idx[(int)(rng() % (i + 1))]);
      for (int i = 0; i < 32 && i < np; ++i) read[idx[i]] = 1;
    }
    for (int col = 0; col < 4; ++col) {  // mode D
      uint8_t cw[64];
      for (int c = 0; c < 32; ++c) cw[c] = (uint8_t)rng();
      for (int r = 32; r < 64; ++r) {
        uint8_t a = 0;
        for (int c = 0; c < 32; ++c) a ^= gf_mul(E.v[r][c], cw[c]);
        cw[r] = a;
      }
      const int f = check_d(read, present, data_only, cw, &dcases);
      if (f && dfails < 10) std::printf("mode D mismatch trial %d e %d\n", trial, e);
      dfails += f;
    }
    FftDecPlan p;
    bool any_out = false;
    for (int i = 0; i < 64; ++i) any_out |= !present[i] && (!data_only || i < 32);
    if (!fftdec_plan_m(read, present, data_only, &p)) {
      if (any_out) {
        std::printf("plan refused a decodable pattern, trial %d\n", trial);
        ++fails;
      }
      continue;
    }
    const uint32_t* w = p.w.data();
    const unsigned baseA = p.side ? 32 : 0, baseB = p.side ? 0 : 32;
    const uint32_t R = w[FftDecLayout::kR], rslots = w[FftDecLayout::kRslots];
    uint32_t outB = 0;  // outputs on coset B
    for (int o = 0; o < p.nout; ++o)
      if (w[FftDecLayout::kOuts + o] & 32) outB |= 1u << (w[FftDecLayout::kOuts + o] & 31);
    for (int t = 0; t < 32; ++t)  // the kernel loads only shards the plan may read
      if (((w[FftDecLayout::kPresA] >> t & 1) && !read[baseA ^ t]) || ((R >> t & 1) && !read[baseB ^ t])) {
        std::printf("trial %d: plan reads unread shard\n", trial);
        ++fails;
      }
    for (int col = 0; col < 8; ++col) {
      uint8_t cw[64];
      for (int c = 0; c < 32; ++c) cw[c] = (uint8_t)rng();
      for (int r = 32; r < 64; ++r) {
        uint8_t a = 0;
        for (int c = 0; c < 32; ++c) a ^= gf_mul(E.v[r][c], cw[c]);
        cw[r] = a;
      }
      uint8_t v[32];
      for (int t = 0; t < 32; ++t)
        v[t] = (w[FftDecLayout::kPresA] >> t & 1) ? cw[baseA ^ t] : 0;
      ifft(v, baseA);
      fft(v, baseB);  // q on B
      uint8_t s[32] = {};
      for (int t = 0; t < 32; ++t)
        if (R >> t & 1) s[t] = (uint8_t)(cw[baseB ^ t] ^ v[t]);
      const int nrs = (int)w[FftDecLayout::kNrs];
      if (nrs != __builtin_popcount(rslots) || w[FftDecLayout::kNrs1] != 1u << nrs) ++fails;
      // register slots after the kernel's swaps: slot r holds the pair (even, odd) of positions
      // of original slot reg[r] (syndromes where R, q where an erased B output, else unused)
      uint8_t sv[16][2], qv[16][2];
      for (int j = 0; j < 16; ++j)
        for (int h = 0; h < 2; ++h) {
          sv[j][h] = s[2 * j + h];
          qv[j][h] = v[2 * j + h];
        }
      for (int i = 0; i < nrs; ++i) {
        const uint32_t jm = w[FftDecLayout::kSwap + i];
        if (__builtin_popcount(jm) != 1) ++fails;
        const int ji = __builtin_ctz(jm);
        // the syndrome loads of register slot i: shard pair j_i, its R positions
        const uint32_t rs = w[FftDecLayout::kRsl + i];
        if ((int)(rs & 15) != ji || (rs >> 8 & 3) != (R >> (2 * ji) & 3)) ++fails;
        if (ji < i || !(rslots >> ji & 1)) ++fails;
        for (int h = 0; h < 2; ++h) {
          std::swap(sv[i][h], sv[ji][h]);
          std::swap(qv[i][h], qv[ji][h]);
        }
      }
      // packed register slots after the swaps: the R slots and those holding an erased B output
      {
        int reg[16];
        for (int j = 0; j < 16; ++j) reg[j] = j;
        for (int i = 0; i < nrs; ++i) std::swap(reg[i], reg[__builtin_ctz(w[FftDecLayout::kSwap + i])]);
        uint32_t want = 0;
        for (int r = 0; r < 16; ++r)
          if ((R | outB) >> (2 * reg[r]) & 3) want |= 1u << r;
        if (want != w[FftDecLayout::kNpk]) ++fails;
      }
      for (int o = 0; o < p.nout; ++o) {
        const uint32_t od = w[FftDecLayout::kOuts + o];
        const unsigned t = od & 31, qm = od >> 16;
        if (__builtin_popcount(qm) != 1 && (od & 32)) ++fails;
        const unsigned qs = qm ? __builtin_ctz(qm) : 0;
        const uint32_t* mk = w + FftDecLayout::kMasks + (size_t)o * nrs * 8;
        uint8_t acc = 0;
        for (int b = 7; b >= 0; --b) {
          acc = xt(acc);
          for (int i = 0; i < nrs; ++i) {
            const uint32_t m = mk[b * nrs + i];
            if (m & 0x0F0F0F0Fu) acc ^= sv[i][0];
            if (m & 0xF0F0F0F0u) acc ^= sv[i][1];
          }
        }
        if (od & 32) acc ^= qv[qs][t & 1];
        const unsigned pos = ((od & 32) ? baseB : baseA) ^ t;
        ++cases;
        if (acc != cw[pos] || present[pos] || (data_only && pos >= 32)) {
          if (fails < 10)
            std::printf("mismatch trial %d e %d side %d out %u: %u != %u\n", trial, e, p.side,
                        pos, acc, cw[pos]);
          ++fails;
        }
      }
    }
    // every requested erasure is an output
    int want = 0;
    for (int i = 0; i < 64; ++i) want += !present[i] && (!data_only || i < 32);
    if (want != p.nout) {
      std::printf("trial %d: %d outputs, %d erasures requested\n", trial, p.nout, want);
      ++fails;
    }
    if (p.nrslots > (e + 1) / 2 + 0 && p.nrslots > __builtin_popcount(w[FftDecLayout::kDA])) {
      std::printf("trial %d: %d syndrome slots for %d rows\n", trial, p.nrslots,
                  __builtin_popcount(w[FftDecLayout::kDA]));
      ++fails;
    }
  }
  std::printf("fftdec model: %d outputs checked, %d failures; mode D: %d outputs, %d failures\n",
              cases, fails, dcases, dfails);
  return fails || dfails ? 1 : 0;
}
