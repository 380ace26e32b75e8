// GF(2^8) field and coding-matrix construction for the CESS segment -> fragment codec.
//
// Product code (host + compile-time). The oracle under oracle/ is an independent restatement
// and is never included from here.
//
// Convention: the systematic Vandermonde code used by the
// off-chain CESS tools (klauspost/reedsolomon `New(k, m)` default matrix, the same as
// Backblaze JavaReedSolomon):
//   * field GF(2^8), reduction polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2;
//   * V[r][c] = r^c (0^0 = 1) for r in [0, k+m), c in [0, k);
//   * E = V * inv(V[0:k, :]) so E[0:k] = I (data shards pass through) and E[k+i] is the
//     coefficient row of parity shard i;
//   * reconstruct: take the first k present rows S of E (in index order), D = inv(E[S]);
//     a missing data shard d is row d of D applied to the survivors; a missing parity shard
//     p is E[p] * D applied to the survivors (bit-identical to klauspost's two-pass
//     "data first, then re-encode parity", since GF arithmetic is exact).
//
// Geometry that fixes k and m for CESS: SEGMENT_SIZE = 16 MiB and FRAGMENT_SIZE = 8 MiB
// (reference primitives/common/src/lib.rs:60-61) give k = 2; FRAGMENT_COUNT = 3
// (reference runtime/src/lib.rs:1027) gives m = 1.
#pragma once
#include <stdint.h>

namespace cec {

constexpr unsigned kPoly = 0x11D;
constexpr int kMaxShards = 256;

struct GfTables {
  uint8_t exp[512];  // exp[i] = 2^i, doubled so exp[log a + log b] needs no modulo
  uint8_t log[256];  // log[0] unused
};

constexpr GfTables make_gf_tables() {
  GfTables t{};
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = (uint8_t)x;
    t.log[x] = (uint8_t)i;
    x <<= 1;
    if (x & 0x100) x ^= kPoly;
  }
  for (int i = 255; i < 512; ++i) t.exp[i] = t.exp[i - 255];
  return t;
}

inline constexpr GfTables kGf = make_gf_tables();

constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
  if (a == 0 || b == 0) return 0;
  return kGf.exp[kGf.log[a] + kGf.log[b]];
}

constexpr uint8_t gf_inv(uint8_t a) {  // a != 0
  return kGf.exp[255 - kGf.log[a]];
}

// a^n with 0^0 = 1 (klauspost galExp semantics).
constexpr uint8_t gf_pow(uint8_t a, int n) {
  if (n == 0) return 1;
  if (a == 0) return 0;
  return kGf.exp[(kGf.log[a] * n) % 255];
}

// Fixed-capacity row-major matrix usable both in constant evaluation (small R, C) and at run
// time (heap-allocated with R = C = kMaxShards).
template <int R, int C>
struct Mat {
  int rows = 0, cols = 0;
  uint8_t v[R][C] = {};
};

// Gauss-Jordan inverse of the n x n matrix `a` (read from a.v[0..n)[0..n)). Returns false when
// singular. `work` must have room for n x 2n.
template <int R, int C, int R2, int C2>
constexpr bool gf_invert(const Mat<R, C>& a, int n, Mat<R, C>& out, Mat<R2, C2>& work) {
  work.rows = n;
  work.cols = 2 * n;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < 2 * n; ++c)
      work.v[r][c] = c < n ? a.v[r][c] : (uint8_t)(c - n == r ? 1 : 0);
  for (int col = 0; col < n; ++col) {
    int piv = -1;
    for (int r = col; r < n; ++r)
      if (work.v[r][col] != 0) { piv = r; break; }
    if (piv < 0) return false;
    if (piv != col)
      for (int c = 0; c < 2 * n; ++c) {
        uint8_t t = work.v[col][c];
        work.v[col][c] = work.v[piv][c];
        work.v[piv][c] = t;
      }
    const uint8_t s = gf_inv(work.v[col][col]);
    for (int c = 0; c < 2 * n; ++c) work.v[col][c] = gf_mul(work.v[col][c], s);
    for (int r = 0; r < n; ++r) {
      if (r == col || work.v[r][col] == 0) continue;
      const uint8_t f = work.v[r][col];
      for (int c = 0; c < 2 * n; ++c) work.v[r][c] ^= gf_mul(f, work.v[col][c]);
    }
  }
  out.rows = out.cols = n;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) out.v[r][c] = work.v[r][n + c];
  return true;
}

// Full (k+m) x k systematic encode matrix E into `e`. `tmp*` are scratch of the same type.
template <int R, int C, int R2, int C2>
constexpr bool gf_encode_matrix(int k, int m, Mat<R, C>& e, Mat<R, C>& top, Mat<R, C>& topinv,
                                Mat<R2, C2>& work) {
  const int n = k + m;
  // V[r][c] = r^c, only its top k x k block is needed for the inverse.
  top.rows = top.cols = k;
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c) top.v[r][c] = gf_pow((uint8_t)r, c);
  if (!gf_invert(top, k, topinv, work)) return false;
  e.rows = n;
  e.cols = k;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < k; ++c) {
      uint8_t acc = 0;
      for (int t = 0; t < k; ++t) acc ^= gf_mul(gf_pow((uint8_t)r, t), topinv.v[t][c]);
      e.v[r][c] = acc;
    }
  return true;
}

// Reconstruction plan for one erasure pattern: which k survivors are read, which missing shards
// are written, and the nout x k coefficient matrix mapping survivors to outputs.
template <int R, int C>
struct Plan {
  int k = 0, nout = 0;
  uint8_t in_idx[R] = {};   // survivor shard indices (first k present, ascending)
  uint8_t out_idx[R] = {};  // shard indices written
  Mat<R, C> coef;           // nout x k
};

// Build the decode plan. `present[i]` != 0 marks shard i as available. With data_only, only
// missing data shards are produced. Returns 0 on success, -1 if fewer than k shards survive.
template <int R, int C, int R2, int C2>
constexpr int gf_decode_plan(int k, int m, const uint8_t* present, bool data_only,
                             const Mat<R, C>& e, Plan<R, C>& plan, Mat<R, C>& sub,
                             Mat<R, C>& inv, Mat<R2, C2>& work) {
  const int n = k + m;
  plan.k = k;
  int got = 0;
  for (int i = 0; i < n && got < k; ++i)
    if (present[i]) plan.in_idx[got++] = (uint8_t)i;
  if (got < k) return -1;
  sub.rows = sub.cols = k;
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c) sub.v[r][c] = e.v[plan.in_idx[r]][c];
  if (!gf_invert(sub, k, inv, work)) return -1;  // cannot happen for this code (MDS)
  plan.nout = 0;
  for (int i = 0; i < n; ++i) {
    if (present[i]) continue;
    if (data_only && i >= k) continue;
    const int o = plan.nout++;
    plan.out_idx[o] = (uint8_t)i;
    for (int c = 0; c < k; ++c) {
      if (i < k) {
        plan.coef.v[o][c] = inv.v[i][c];
      } else {
        uint8_t acc = 0;
        for (int t = 0; t < k; ++t) acc ^= gf_mul(e.v[i][t], inv.v[t][c]);
        plan.coef.v[o][c] = acc;
      }
    }
  }
  plan.coef.rows = plan.nout;
  plan.coef.cols = k;
  return 0;
}

// The same plan by the code's systematic structure (run time): the survivors (the first k present
// shards, or the k shards flagged in `read`, a subset of the present ones) are k - d data shards
// and d parity shards Ps, so only the d x d block A = E[Ps][D] over the unread data D is inverted:
// x_D = inv(A) (y_Ps ^ E[Ps][C] x_C) (any d parity rows give an invertible block: the code is
// MDS). d^3 + d^2 k products instead of the k x 2k Gauss-Jordan; the decode map from a survivor
// set is unique, so the coefficients are those of gf_decode_plan (checked on every pattern of
// small codes, tests/native/sanitize_host.cpp). Outputs are the shards not present (data_only:
// data shards only). `a`, `ainv`, `work` are scratch (d <= m). Returns 0, or -1 if fewer than k
// shards survive (or `read` does not name k present shards).
template <int R, int C, int R2, int C2>
int gf_decode_plan_sys(int k, int m, const uint8_t* present, bool data_only, const Mat<R, C>& e,
                       Plan<R, C>& plan, Mat<R, C>& a, Mat<R, C>& ainv, Mat<R2, C2>& work,
                       const uint8_t* read = nullptr) {
  const int n = k + m;
  plan.k = k;
  int got = 0;
  bool in[kMaxShards] = {};
  for (int i = 0; i < n && got < k; ++i)
    if (read ? read[i] : present[i]) {
      if (!present[i]) return -1;
      plan.in_idx[got++] = (uint8_t)i;
      in[i] = true;
    }
  if (got < k) return -1;
  int miss[kMaxShards], d = 0;  // data shards not read (the lost ones and, with `read`, others)
  for (int i = 0; i < k; ++i)
    if (!in[i]) miss[d++] = i;
  const int nc = k - d;  // survivor positions [0, nc) are data, [nc, k) parity
  a.rows = a.cols = d;
  for (int r = 0; r < d; ++r)
    for (int c = 0; c < d; ++c) a.v[r][c] = e.v[plan.in_idx[nc + r]][miss[c]];
  if (d && !gf_invert(a, d, ainv, work)) return -1;  // cannot happen for this code (MDS)
  // rows of the missing data over the k survivors, kept in a.v (a is no longer needed)
  for (int r = 0; r < d; ++r) {
    for (int p = 0; p < nc; ++p) {
      const int col = plan.in_idx[p];
      uint8_t acc = 0;
      for (int b = 0; b < d; ++b) acc ^= gf_mul(ainv.v[r][b], e.v[plan.in_idx[nc + b]][col]);
      a.v[r][p] = acc;
    }
    for (int b = 0; b < d; ++b) a.v[r][nc + b] = ainv.v[r][b];
  }
  int mrow[kMaxShards] = {};  // missing data shard -> its row in a
  for (int r = 0; r < d; ++r) mrow[miss[r]] = r;
  plan.nout = 0;
  for (int i = 0; i < n; ++i) {
    if (present[i] || (data_only && i >= k)) continue;
    const int o = plan.nout++;
    plan.out_idx[o] = (uint8_t)i;
    if (i < k) {
      for (int c = 0; c < k; ++c) plan.coef.v[o][c] = a.v[mrow[i]][c];
      continue;
    }
    // a lost parity shard: its encode row over the data, the missing data substituted
    for (int c = 0; c < k; ++c) plan.coef.v[o][c] = c < nc ? e.v[i][plan.in_idx[c]] : 0;
    for (int r = 0; r < d; ++r) {
      const uint8_t f = e.v[i][miss[r]];
      if (!f) continue;
      for (int c = 0; c < k; ++c) plan.coef.v[o][c] ^= gf_mul(f, a.v[r][c]);
    }
  }
  plan.coef.rows = plan.nout;
  plan.coef.cols = k;
  return 0;
}

// ---- additive FFT over the subspace of the first 2^K field elements -------------------------
// RS(2^K, 2^K) in this convention has data = f(0..2^K-1) and parity i = f(2^K + i) for the
// unique f of degree < 2^K (E = V * inv(V_top), V[r][c] = r^c). The points 0..2^K-1 are the
// GF(2)-span of the basis v_i = 2^i (the integers XOR-combine like field elements), and
// 2^K + i = 2^K ^ i is its coset by beta = 2^K. So encode = the Lin-Chung-Han additive IFFT
// over the subspace (data -> coefficients of f in the novel polynomial basis) followed by the
// FFT over the coset (coefficients -> parity): the same bytes as the matrix product, since f is
// unique. Skew of layer i (butterfly half-distance 2^i) for the block starting at position t0:
//   s = What_i(t0 ^ beta),  What_i(x) = W_i(x) / W_i(v_i),  W_i(x) = prod_{a in span(v_0..v_{i-1})} (x - a).
// IFFT layer i: b ^= a; a ^= s*b (i = 0 .. K-1). FFT layer i: a ^= s*b; b ^= a (i = K-1 .. 0).
constexpr uint8_t lch_w(int i, uint8_t x) {
  uint8_t r = 1;
  for (int a = 0; a < (1 << i); ++a) r = gf_mul(r, (uint8_t)(x ^ a));
  return r;
}
constexpr uint8_t lch_what(int i, uint8_t x) {
  return gf_mul(lch_w(i, x), gf_inv(lch_w(i, (uint8_t)(1 << i))));
}
// skew[i][b]: layer i, block b (positions b * 2^(i+1) .. + 2^(i+1) - 1), for shift beta
template <int K>
struct LchSkews {
  uint8_t s[K][1 << (K - 1)] = {};
};
template <int K>
constexpr LchSkews<K> lch_skews(uint8_t beta) {
  LchSkews<K> r{};
  for (int i = 0; i < K; ++i)
    for (int b = 0; b < (1 << (K - 1 - i)); ++b)
      r.s[i][b] = lch_what(i, (uint8_t)((b << (i + 1)) ^ beta));
  return r;
}
// The same transforms over the 2^K points of span(v_0..v_{K-1}) for any ordered basis v (the
// shard indices 0..63 as points, taken in another order: position p holds the point
// phi(p) = XOR of v_i over the bits i of p). What_i is GF(2)-linear, so a skew is the XOR of
// What_i(v_j) over the bits of its block above layer i.
constexpr uint8_t lchb_phi(const uint8_t* v, int K, unsigned p) {
  uint8_t x = 0;
  for (int i = 0; i < K; ++i)
    if (p >> i & 1) x ^= v[i];
  return x;
}
constexpr uint8_t lchb_w(const uint8_t* v, int i, uint8_t x) {
  uint8_t r = 1;
  for (unsigned a = 0; a < (1u << i); ++a) r = gf_mul(r, (uint8_t)(x ^ lchb_phi(v, i, a)));
  return r;
}
constexpr uint8_t lchb_what(const uint8_t* v, int i, uint8_t x) {
  return gf_mul(lchb_w(v, i, x), gf_inv(lchb_w(v, i, v[i])));
}
template <int K>
constexpr LchSkews<K> lchb_skews(const uint8_t* v) {
  LchSkews<K> r{};
  for (int i = 0; i < K; ++i)
    for (int b = 0; b < (1 << (K - 1 - i)); ++b)
      r.s[i][b] = lchb_what(v, i, lchb_phi(v, K, (unsigned)b << (i + 1)));
  return r;
}
// the formal derivative's constants in that basis: c_j = W_j'(0) / W_j(v_j), W_j'(0) the product
// of the nonzero points of span(v_0..v_{j-1})
constexpr uint8_t lchb_dconst(const uint8_t* v, int j) {
  uint8_t p = 1;
  for (unsigned a = 1; a < (1u << j); ++a) p = gf_mul(p, lchb_phi(v, j, a));
  return gf_mul(p, gf_inv(lchb_w(v, j, v[j])));
}

// Formal derivative in the novel basis: D(Xhat_i) = sum_{bit j of i} c_j Xhat_{i - 2^j} with
// c_j = What_j' = W_j'(0) / W_j(v_j). W_j is linearised, so its derivative is the constant
// prod of the nonzero points of span(v_0..v_{j-1}).
constexpr uint8_t lch_dconst(int j) {
  uint8_t p = 1;
  for (int a = 1; a < (1 << j); ++a) p = gf_mul(p, (uint8_t)a);
  return gf_mul(p, gf_inv(lch_w(j, (uint8_t)(1u << j))));
}
// GF(2) matrix of x -> c*x on bit planes: row q = mask of input bits p whose product c * 2^p has
// bit q (plane q of c*x = XOR of planes p in row q).
struct BitMatrix {
  uint8_t row[8] = {};
};
constexpr BitMatrix gf_bitmatrix(uint8_t c) {
  BitMatrix m{};
  for (int q = 0; q < 8; ++q)
    for (int p = 0; p < 8; ++p)
      if (gf_mul(c, (uint8_t)(1u << p)) >> q & 1) m.row[q] |= (uint8_t)(1u << p);
  return m;
}

}  // namespace cec
