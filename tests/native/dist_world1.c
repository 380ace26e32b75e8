/* C consumer of the multi-GPU degraded read (cec_dist_*, include/cess_ec.h) at world 1: what a
 * cgo / FFI host runs on each rank, here with every fragment local. A batch of RS(k,m) segments
 * is encoded in HBM, segment s loses fragment s mod (k+m), the group rebuilds them through
 * cec_dist_degraded_read (plan, agreement all-reduce, local survivor copies, rebuild), and every
 * rebuilt fragment must equal the original; cec_dist_plan must name rank 0 for every entry, and a
 * locate callback that misses a survivor must fail with CEC_EINVAL.
 * build: gcc -O2 -D__HIP_PLATFORM_AMD__ tests/native/dist_world1.c -Iinclude -I/opt/rocm/include
 *            -Lcess_amd -lcessec -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,... -o dist_world1 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cess_ec.h"

#define CHECK(c)                                                                          \
  do {                                                                                    \
    if (!(c)) {                                                                           \
      fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, cec_last_error()); \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

typedef struct {
  int k, m;
  size_t F;
  uint8_t* d_data;
  uint8_t* d_par;
  uint64_t hole_seg;  /* locate returns NULL for (hole_seg, hole_frag) */
  int hole_frag;
} store_t;

static const uint8_t* locate(void* user, uint64_t seg, int frag) {
  const store_t* st = (const store_t*)user;
  if (seg == st->hole_seg && frag == st->hole_frag) return NULL;
  if (frag < st->k) return st->d_data + (seg * st->k + frag) * st->F;
  return st->d_par + (seg * st->m + (frag - st->k)) * st->F;
}

static int run(int k, int m, size_t nseg, size_t F) {
  const int n = k + m;
  cec_codec* c = NULL;
  CHECK(cec_create(k, m, 0, &c) == CEC_OK);
  store_t st = {k, m, F, NULL, NULL, (uint64_t)-1, -1};
  CHECK(hipMalloc((void**)&st.d_data, nseg * k * F) == hipSuccess);
  CHECK(hipMalloc((void**)&st.d_par, nseg * m * F) == hipSuccess);
  CHECK(cec_fill_synthetic(st.d_data, k * F, nseg, 0, 0xCE550004u, NULL) == CEC_OK);
  CHECK(cec_encode_batch(c, st.d_data, st.d_par, nseg, F, NULL) == CEC_OK);
  CHECK(hipDeviceSynchronize() == hipSuccess);

  uint64_t* seg = malloc(nseg * sizeof(uint64_t));
  uint8_t* frag = malloc(nseg);
  uint8_t** out = malloc(nseg * sizeof(uint8_t*));
  int32_t* dec = malloc(nseg * sizeof(int32_t));
  for (size_t s = 0; s < nseg; ++s) {
    seg[s] = s;
    frag[s] = (uint8_t)(s % n);
    CHECK(hipMalloc((void**)&out[s], F) == hipSuccess);
  }
  size_t nmoves = 0;
  CHECK(cec_dist_plan(k, m, 1, seg, frag, nseg, NULL, 0, &nmoves, dec) == CEC_OK);
  CHECK(nmoves == nseg * (size_t)k);
  for (size_t s = 0; s < nseg; ++s) CHECK(dec[s] == 0);

  uint8_t id[CEC_DIST_ID_BYTES];
  cec_dist* d = NULL;
  CHECK(cec_dist_unique_id(id) == CEC_OK);
  CHECK(cec_dist_create(c, id, 1, 0, &d) == CEC_OK);
  size_t nrebuilt = 0;
  CHECK(cec_dist_degraded_read(d, seg, frag, nseg, F, locate, &st, out, NULL, &nrebuilt) ==
        CEC_OK);
  CHECK(nrebuilt == nseg);
  uint8_t* got = malloc(F);
  uint8_t* want = malloc(F);
  for (size_t s = 0; s < nseg; ++s) {
    CHECK(hipMemcpy(got, out[s], F, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(hipMemcpy(want, locate(&st, s, frag[s]), F, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(memcmp(got, want, F) == 0);
  }
  /* a survivor the store does not hold: refused before any transfer */
  st.hole_seg = 1;
  st.hole_frag = frag[1] == 0 ? 1 : 0;
  CHECK(cec_dist_degraded_read(d, seg, frag, nseg, F, locate, &st, out, NULL, NULL) ==
        CEC_EINVAL);
  cec_dist_destroy(d);
  for (size_t s = 0; s < nseg; ++s) (void)hipFree(out[s]);
  (void)hipFree(st.d_data);
  (void)hipFree(st.d_par);
  free(seg);
  free(frag);
  free(out);
  free(dec);
  free(got);
  free(want);
  cec_destroy(c);
  return 0;
}

int main(void) {
  if (run(2, 1, 12, (size_t)1 << 20)) return 1;
  if (run(4, 2, 9, 65536 + 64)) return 1;
  printf("dist world1 ok\n");
  return 0;
}
