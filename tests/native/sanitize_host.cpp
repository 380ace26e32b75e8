// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (host ASan/UBSan
// build of the CPU codec; GPU sanitizers are not available on this pool). Built and run by
// tests/test_host.py::test_host_code_under_sanitizers with g++ -fsanitize=address,undefined:
//   * libcessec's host-only code: SCALE records (records.cpp), the degraded-read plan of every
//     exchange and its RCCL group cuts at several bounds, plans of up to three rounds (dist.cpp,
//     no GPU call on that path), the GF(2^8) matrix builder and decode plans
//     (gf256.h) for every erasure pattern of small codes;
//   * the CPU codec (oracle/rs_oracle.c, the CPU baseline) in its scalar, AVX2 and GFNI forms,
//     encode + reconstruct round trips with ragged lengths.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../cess_amd/csrc/gf256.h"
#include "../../cess_amd/csrc/fftdec_plan.h"
#include "../../include/cess_ec.h"

extern "C" {
int orc_set_simd(int v);
int orc_encode(int k, int m, const uint8_t* const* data, uint8_t* const* parity, size_t len);
int orc_reconstruct(int k, int m, uint8_t* const* shards, const uint8_t* present, size_t len,
                    int data_only);
}

namespace cec {
int set_error(int code, const std::string&) { return code; }
}  // namespace cec

// dist.cpp's GPU path calls into cess_ec.cpp; the plan path exercised here never does
extern "C" {
int cec_codec_info(const cec_codec*, int*, int*, int*) { return CEC_EINVAL; }
int cec_reconstruct_batch(cec_codec*, uint8_t*, uint8_t*, size_t, size_t, const uint8_t*, int,
                          int, void*) {
  return CEC_EINVAL;
}
int cec_reconstruct_partial_batch(cec_codec*, uint8_t*, uint8_t*, size_t, size_t, const uint8_t*,
                                  const uint8_t*, int, void*) {
  return CEC_EINVAL;
}
int cec_xor_batch(uint8_t*, const uint8_t*, size_t, size_t, size_t, void*) { return CEC_EINVAL; }
const char* cec_last_error(void) { return ""; }
}

static int fails = 0;
#define CHECK(c)                                                 \
  do {                                                           \
    if (!(c)) {                                                  \
      std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                   \
    }                                                            \
  } while (0)

static std::string hex64(std::mt19937& g) {
  static const char* d = "0123456789abcdef";
  std::string s(64, '0');
  for (auto& c : s) c = d[g() % 16];
  return s;
}

static void records(std::mt19937& g) {
  uint8_t buf[8];
  size_t n = 0;
  for (uint32_t v : {0u, 63u, 64u, 16383u, 16384u, 1073741823u, 1073741824u, 0xffffffffu}) {
    CHECK(cec_scale_compact(v, nullptr, 0, &n) == CEC_OK && n >= 1 && n <= 5);
    CHECK(cec_scale_compact(v, buf, sizeof buf, &n) == CEC_OK);
  }
  for (size_t nseg : {size_t(1), size_t(7), size_t(1000), size_t(1001)}) {
    std::string seg, frag;
    for (size_t s = 0; s < nseg; ++s) {
      seg += hex64(g);
      for (int f = 0; f < 3; ++f) frag += hex64(g);
    }
    const auto* sh = reinterpret_cast<const uint8_t*>(seg.data());
    const auto* fh = reinterpret_cast<const uint8_t*>(frag.data());
    size_t need = 0;
    const int rc = cec_scale_deal_info(sh, fh, nseg, 3, nullptr, 0, &need);
    if (nseg > 1000) {
      CHECK(rc == CEC_ESEGCOUNT);
      continue;
    }
    CHECK(rc == CEC_OK && need > nseg * 4 * 64);
    std::vector<uint8_t> out(need);
    CHECK(cec_scale_deal_info(sh, fh, nseg, 3, out.data(), need, &n) == CEC_OK && n == need);
    CHECK(cec_scale_deal_info(sh, fh, nseg, 3, out.data(), need - 1, &n) != CEC_OK);
    std::string bad = seg;
    bad[5] = 'G';
    CHECK(cec_scale_deal_info(reinterpret_cast<const uint8_t*>(bad.data()), fh, nseg, 3,
                              out.data(), need, &n) == CEC_EINVAL);
    uint8_t acct[32] = {1};
    const char* name = "file.bin";
    const char* bucket = "bucket";
    size_t cn = 0;
    CHECK(cec_scale_upload_declaration(sh, sh, fh, nseg, 3, acct,
                                       reinterpret_cast<const uint8_t*>(name), std::strlen(name),
                                       reinterpret_cast<const uint8_t*>(bucket),
                                       std::strlen(bucket), nullptr, 0, &cn) == CEC_OK);
    std::vector<uint8_t> call(cn);
    CHECK(cec_scale_upload_declaration(sh, sh, fh, nseg, 3, acct,
                                       reinterpret_cast<const uint8_t*>(name), std::strlen(name),
                                       reinterpret_cast<const uint8_t*>(bucket),
                                       std::strlen(bucket), call.data(), cn, &n) == CEC_OK);
  }
  const std::string h = hex64(g);
  uint8_t id[68], back[64];
  for (uint32_t i : {0u, 1u, 999u}) {
    CHECK(cec_shard_id(reinterpret_cast<const uint8_t*>(h.data()), i, id) == CEC_OK);
    CHECK(cec_hash_from_shard_id(id, back) == CEC_OK && std::memcmp(back, h.data(), 64) == 0);
  }
  CHECK(cec_shard_id(reinterpret_cast<const uint8_t*>(h.data()), 1000, id) != CEC_OK);
}

// the RCCL group cuts of a plan (dist.cpp group_cuts via cec_dist_plan_groups): count-only and
// filled calls agree, starts ascend from 0, every round of 256 segments starts a group, a smaller
// bound never gives fewer groups, an undersized starts buffer is refused
static void group_cuts(int k, int m, int world, int ex, const std::vector<uint64_t>& seg,
                       const std::vector<uint8_t>& frag) {
  size_t nsegs = 0;
  {
    std::vector<uint64_t> u(seg);
    std::sort(u.begin(), u.end());
    nsegs = (size_t)(std::unique(u.begin(), u.end()) - u.begin());
  }
  size_t prev = 0;
  for (int bound : {4096, 1024, 64, 7, 1, 0}) {
    size_t ng = 0;
    CHECK(cec_dist_plan_groups(k, m, world, ex, bound, seg.data(), frag.data(), seg.size(),
                               nullptr, 0, &ng) == CEC_OK);
    std::vector<uint64_t> st(ng + 1, ~0ull);
    size_t ng2 = 0;
    CHECK(cec_dist_plan_groups(k, m, world, ex, bound, seg.data(), frag.data(), seg.size(),
                               st.data(), ng, &ng2) == CEC_OK && ng2 == ng);
    CHECK(st[ng] == ~0ull);  // nothing past starts_cap
    if (ng > 1)
      CHECK(cec_dist_plan_groups(k, m, world, ex, bound, seg.data(), frag.data(), seg.size(),
                                 st.data(), ng - 1, &ng2) == CEC_EINVAL);
    if (nsegs == 0) continue;
    CHECK(ng >= (nsegs + 255) / 256 && st[0] == 0);
    for (size_t i = 1; i < ng; ++i) CHECK(st[i] > st[i - 1] && st[i] < nsegs);
    for (size_t r = 256; r < nsegs; r += 256)
      CHECK(std::find(st.begin(), st.begin() + ng, (uint64_t)r) != st.begin() + ng);
    if (bound > 0) {
      CHECK(ng >= prev);
      prev = ng;
    } else {
      CHECK(ng == (nsegs + 255) / 256);
    }
  }
}

static void plans(std::mt19937& g) {
  const int codes[][2] = {{2, 1}, {4, 2}, {10, 4}, {32, 32}, {200, 56}};
  for (auto& km : codes) {
    const int k = km[0], m = km[1];
    for (int world = 1; world <= 8; ++world)
      for (int ex = 0; ex <= 2; ++ex) {
        std::vector<uint64_t> seg;
        std::vector<uint8_t> frag;
        for (int s = 0; s < 40; ++s) {
          const int e = 1 + (int)(g() % m);
          for (int q = 0; q < e; ++q) {
            seg.push_back(g() % 500);
            frag.push_back((uint8_t)(g() % (k + m)));
          }
        }
        // keep at most m distinct erasures per segment: drop the rest
        std::vector<uint64_t> s2;
        std::vector<uint8_t> f2;
        for (size_t i = 0; i < seg.size(); ++i) {
          int distinct = 0;
          bool dup = false;
          for (size_t j = 0; j < s2.size(); ++j)
            if (s2[j] == seg[i]) {
              ++distinct;
              dup |= f2[j] == frag[i];
            }
          if (dup || distinct < m) {
            s2.push_back(seg[i]);
            f2.push_back(frag[i]);
          }
        }
        size_t nm = 0;
        CHECK(cec_dist_plan_ex(k, m, world, ex, s2.data(), f2.data(), s2.size(), nullptr, 0, &nm,
                               nullptr) == CEC_OK);
        std::vector<cec_dist_move> mv(nm + 1);
        std::vector<int32_t> dec(s2.size());
        size_t nm2 = 0;
        CHECK(cec_dist_plan_ex(k, m, world, ex, s2.data(), f2.data(), s2.size(), mv.data(), nm,
                               &nm2, dec.data()) == CEC_OK && nm2 == nm);
        if (nm > 1)
          CHECK(cec_dist_plan_ex(k, m, world, ex, s2.data(), f2.data(), s2.size(), mv.data(),
                                 nm - 1, &nm2, nullptr) == CEC_EINVAL);
        for (size_t i = 0; i < nm; ++i)
          CHECK(mv[i].src >= 0 && mv[i].src < world && mv[i].dst >= 0 && mv[i].dst < world &&
                mv[i].frag >= 0 && mv[i].frag < k + m && (mv[i].kind == 0 || mv[i].kind == 1));
        group_cuts(k, m, world, ex, s2, f2);
      }
    if (k + m <= 64) {  // plans of several rounds (700 segments), ragged erasure counts
      for (int world : {2, 3, 8})
        for (int ex = 0; ex <= 2; ++ex) {
          std::vector<uint64_t> seg;
          std::vector<uint8_t> frag;
          for (uint64_t s = 0; s < 700; ++s) {
            const int e = 1 + (int)(g() % m);
            const int f0 = (int)(g() % (k + m));
            for (int q = 0; q < e; ++q) {
              seg.push_back(s * 3 + 1);
              frag.push_back((uint8_t)((f0 + q) % (k + m)));
            }
          }
          group_cuts(k, m, world, ex, seg, frag);
        }
    }
    if (k + m < 256) {  // an index past the code (uint8 holds every index of a 256-shard code)
      uint64_t s0 = 3;
      uint8_t bad = (uint8_t)(k + m);
      size_t nm = 0;
      CHECK(cec_dist_plan_ex(k, m, 2, 2, &s0, &bad, 1, nullptr, 0, &nm, nullptr) == CEC_EINVAL);
    }
  }
}

using Big = cec::Mat<cec::kMaxShards, cec::kMaxShards>;
using Work = cec::Mat<cec::kMaxShards, 2 * cec::kMaxShards>;
using BigPlan = cec::Plan<cec::kMaxShards, cec::kMaxShards>;

// the systematic plan (run time, d x d inverse) equals the Gauss-Jordan plan (k x 2k)
static void same_plans(int k, int m, const uint8_t* present, bool data_only, const Big& E) {
  auto p1 = std::make_unique<BigPlan>();
  auto p2 = std::make_unique<BigPlan>();
  auto s1 = std::make_unique<Big>();
  auto s2 = std::make_unique<Big>();
  auto i1 = std::make_unique<Big>();
  auto i2 = std::make_unique<Big>();
  auto w = std::make_unique<Work>();
  const int r1 = cec::gf_decode_plan(k, m, present, data_only, E, *p1, *s1, *i1, *w);
  const int r2 = cec::gf_decode_plan_sys(k, m, present, data_only, E, *p2, *s2, *i2, *w);
  CHECK(r1 == r2);
  if (r1) return;
  CHECK(p1->nout == p2->nout);
  for (int j = 0; j < k; ++j) CHECK(p1->in_idx[j] == p2->in_idx[j]);
  for (int o = 0; o < p1->nout; ++o) {
    CHECK(p1->out_idx[o] == p2->out_idx[o]);
    for (int c = 0; c < k; ++c) CHECK(p1->coef.v[o][c] == p2->coef.v[o][c]);
  }
}

// the systematic plan from an explicit survivor set (`read`, k present shards): every output row
// times the survivors' encode rows is the output's encode row, outputs = the shards not present
static void read_set_plan(int k, int m, const uint8_t* present, const uint8_t* read,
                          bool data_only, const Big& E) {
  auto p = std::make_unique<BigPlan>();
  auto a = std::make_unique<Big>();
  auto ai = std::make_unique<Big>();
  auto w = std::make_unique<Work>();
  CHECK(cec::gf_decode_plan_sys(k, m, present, data_only, E, *p, *a, *ai, *w, read) == 0);
  for (int j = 0, i = 0; i < k + m; ++i)
    if (read[i]) CHECK(p->in_idx[j++] == i);
  int want = 0;
  for (int i = 0; i < k + m; ++i) want += !present[i] && (!data_only || i < k);
  CHECK(p->nout == want);
  for (int o = 0; o < p->nout; ++o) {
    CHECK(!present[p->out_idx[o]]);
    for (int c = 0; c < k; ++c) {
      uint8_t acc = 0;
      for (int j = 0; j < k; ++j) acc ^= cec::gf_mul(p->coef.v[o][j], E.v[p->in_idx[j]][c]);
      CHECK(acc == E.v[p->out_idx[o]][c]);
    }
  }
}

static void matrices() {
  const int codes[][2] = {{2, 1}, {4, 2}, {5, 5}, {10, 4}, {3, 3}};
  for (auto& km : codes) {
    const int k = km[0], m = km[1], n = k + m;
    auto E = std::make_unique<Big>();
    auto top = std::make_unique<Big>();
    auto topinv = std::make_unique<Big>();
    auto work = std::make_unique<Work>();
    CHECK(cec::gf_encode_matrix(k, m, *E, *top, *topinv, *work));
    for (uint32_t mask = 0; mask < (1u << n); ++mask) {  // every erasure pattern
      uint8_t present[cec::kMaxShards] = {};
      int np = 0;
      for (int i = 0; i < n; ++i) np += present[i] = (mask >> i) & 1;
      auto plan = std::make_unique<BigPlan>();
      auto sub = std::make_unique<Big>();
      auto inv = std::make_unique<Big>();
      const int rc = cec::gf_decode_plan(k, m, present, false, *E, *plan, *sub, *inv, *work);
      CHECK((rc == 0) == (np >= k));
      if (rc) continue;
      // every output row times the survivors' encode rows is that output's encode row
      for (int o = 0; o < plan->nout; ++o)
        for (int c = 0; c < k; ++c) {
          uint8_t acc = 0;
          for (int j = 0; j < k; ++j)
            acc ^= cec::gf_mul(plan->coef.v[o][j], E->v[plan->in_idx[j]][c]);
          CHECK(acc == E->v[plan->out_idx[o]][c]);
        }
      for (int data_only = 0; data_only < 2; ++data_only) same_plans(k, m, present, data_only, *E);
    }
  }
  // the wide codes: random patterns of every erasure count
  std::mt19937 g(7);
  const int wide[][2] = {{32, 32}, {200, 56}, {17, 3}};
  for (auto& km : wide) {
    const int k = km[0], m = km[1], n = k + m;
    auto E = std::make_unique<Big>();
    auto top = std::make_unique<Big>();
    auto topinv = std::make_unique<Big>();
    auto work = std::make_unique<Work>();
    CHECK(cec::gf_encode_matrix(k, m, *E, *top, *topinv, *work));
    for (int t = 0; t < 60; ++t) {
      uint8_t present[cec::kMaxShards] = {};
      for (int i = 0; i < n; ++i) present[i] = 1;
      const int e = 1 + (int)(g() % m);
      for (int q = 0; q < e; ++q) present[g() % n] = 0;
      same_plans(k, m, present, t & 1, *E);
      // survivor sets other than the first k present: random ones, and RS(32,32)'s choice
      uint8_t read[cec::kMaxShards] = {};
      int idx[cec::kMaxShards], np = 0;
      for (int i = 0; i < n; ++i)
        if (present[i]) idx[np++] = i;
      for (int i = np - 1; i > 0; --i) std::swap(idx[i], idx[g() % (i + 1)]);
      for (int i = 0; i < k; ++i) read[idx[i]] = 1;
      read_set_plan(k, m, present, read, t & 1, *E);
      if (k == 32 && m == 32) {
        uint8_t fr[64] = {};
        CHECK(cec::fftdec_read_set(present, fr));
        int nr = 0;
        for (int i = 0; i < 64; ++i) nr += fr[i];
        CHECK(nr == 32);
        read_set_plan(k, m, present, fr, t & 1, *E);
      }
    }
  }
}

static void cpu_codec(std::mt19937& g) {
  const int codes[][2] = {{2, 1}, {4, 2}, {10, 4}, {32, 32}};
  for (int simd = 0; simd <= 2; ++simd) {
    const int got = orc_set_simd(simd);
    for (auto& km : codes)
      for (size_t len : {size_t(1), size_t(31), size_t(64), size_t(4099)}) {
        const int k = km[0], m = km[1], n = k + m;
        std::vector<std::vector<uint8_t>> sh(n, std::vector<uint8_t>(len));
        for (int i = 0; i < k; ++i)
          for (auto& b : sh[i]) b = (uint8_t)g();
        std::vector<uint8_t*> p(n);
        for (int i = 0; i < n; ++i) p[i] = sh[i].data();
        CHECK(orc_encode(k, m, p.data(), p.data() + k, len) == 0);
        auto full = sh;
        std::vector<uint8_t> present(n, 1);
        for (int e = 0; e < m; ++e) {
          const int i = (int)(g() % n);
          present[i] = 0;
          std::fill(sh[i].begin(), sh[i].end(), 0);
        }
        CHECK(orc_reconstruct(k, m, p.data(), present.data(), len, 0) == 0);
        CHECK(sh == full);
      }
    (void)got;
  }
}

int main() {
  std::mt19937 g(20261017);
  records(g);
  plans(g);
  matrices();
  cpu_codec(g);
  if (fails) {
    std::fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  std::printf("sanitize host ok\n");
  return 0;
}
