// Host-only driver over the product's cess_amd/csrc/gf256.h (no GPU): prints the encode matrix
// and decode plans so tests/test_host.py can compare them with the oracle on the CPU.
// usage: gf_plan_dump k m [present-bitstring data_only]...
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "../../cess_amd/csrc/gf256.h"

using namespace cec;
using M = Mat<kMaxShards, kMaxShards>;
using W = Mat<kMaxShards, 2 * kMaxShards>;

int main(int argc, char** argv) {
  const int k = atoi(argv[1]), m = atoi(argv[2]);
  auto e = std::make_unique<M>(), t = std::make_unique<M>(), ti = std::make_unique<M>();
  auto w = std::make_unique<W>();
  if (!gf_encode_matrix(k, m, *e, *t, *ti, *w)) return 1;
  printf("E");
  for (int r = 0; r < k + m; ++r)
    for (int c = 0; c < k; ++c) printf(" %d", e->v[r][c]);
  printf("\n");
  for (int a = 3; a + 1 < argc; a += 2) {
    uint8_t present[kMaxShards];
    for (int i = 0; i < k + m; ++i) present[i] = argv[a][i] == '1';
    auto plan = std::make_unique<Plan<kMaxShards, kMaxShards>>();
    auto sub = std::make_unique<M>(), inv = std::make_unique<M>();
    int rc = gf_decode_plan(k, m, present, atoi(argv[a + 1]) != 0, *e, *plan, *sub, *inv, *w);
    printf("P %d in", rc);
    for (int j = 0; j < (rc ? 0 : k); ++j) printf(" %d", plan->in_idx[j]);
    printf(" out");
    for (int o = 0; o < (rc ? 0 : plan->nout); ++o) printf(" %d", plan->out_idx[o]);
    printf(" coef");
    for (int o = 0; o < (rc ? 0 : plan->nout); ++o)
      for (int j = 0; j < k; ++j) printf(" %d", plan->coef.v[o][j]);
    printf("\n");
  }
  return 0;
}
