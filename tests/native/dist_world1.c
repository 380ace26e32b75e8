/* C consumer of the multi-GPU degraded read (cec_dist_*, include/cess_ec.h) at world 1: what a
 * cgo / FFI host runs on each rank, here with every fragment local. A batch of RS(k,m) segments
 * is encoded in HBM, segment s loses fragment s mod (k+m), the group rebuilds them through
 * cec_dist_degraded_read (plan, agreement all-reduce, local survivor copies, rebuild), and every
 * rebuilt fragment must equal the original; cec_dist_plan must name rank 0 for every entry, and a
 * locate callback that misses a survivor must fail with CEC_EINVAL. Last, a dist handle and its codec
 * are destroyed while another codec's batch runs on a side stream (destroy_under_load).
 * build: gcc -O2 -D__HIP_PLATFORM_AMD__ tests/native/dist_world1.c -Iinclude -I/opt/rocm/include
 *            -Lcess_amd -lcessec -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,... -o dist_world1 */
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
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

/* GF(2^8) (0x11D) doubling of 4 packed bytes */
static uint32_t xt4(uint32_t x) {
  const uint32_t hi = x & 0x80808080u;
  return ((x & 0x7F7F7F7Fu) << 1) ^ ((hi >> 7) * 0x1Du);
}

/* Destroying a codec, then a dist handle and its codec, each while another codec's long batch
 * (~25 ms) is still running on a side stream: the side work must complete bit-exact (RS(2,1)
 * parity p = 3 d0 ^ 2 d1 recomputed on the host), and a destruction should wait for its own
 * work only. Prints whether the side stream was still busy right after each destroy (1: not
 * drained by it; 0 after the dist destroy can come from RCCL's ncclCommDestroy, whose internal
 * synchronisation is not ours). */
static int destroy_under_load(void) {
  const size_t F = (size_t)8 << 20, nseg = 16;
  const int reps = 400;
  cec_codec *c = NULL, *side_codec = NULL;
  CHECK(cec_create(4, 2, 0, &c) == CEC_OK);
  CHECK(cec_create(2, 1, 0, &side_codec) == CEC_OK);
  hipStream_t side;
  CHECK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking) == hipSuccess);
  uint8_t *d_data, *d_par;
  CHECK(hipMalloc((void**)&d_data, nseg * 2 * F) == hipSuccess);
  CHECK(hipMalloc((void**)&d_par, nseg * F) == hipSuccess);
  CHECK(cec_fill_synthetic(d_data, 2 * F, nseg, 0, 0xCE550009u, side) == CEC_OK);
  /* the dist handle does one degraded read first (staging allocated, `done` recorded) */
  const size_t Fd = 65536, nd = 6;
  store_t st = {4, 2, Fd, NULL, NULL, (uint64_t)-1, -1};
  CHECK(hipMalloc((void**)&st.d_data, nd * 4 * Fd) == hipSuccess);
  CHECK(hipMalloc((void**)&st.d_par, nd * 2 * Fd) == hipSuccess);
  CHECK(cec_fill_synthetic(st.d_data, 4 * Fd, nd, 0, 0xCE550004u, NULL) == CEC_OK);
  CHECK(cec_encode_batch(c, st.d_data, st.d_par, nd, Fd, NULL) == CEC_OK);
  CHECK(hipDeviceSynchronize() == hipSuccess);
  uint64_t seg[6];
  uint8_t frag[6];
  uint8_t* out[6];
  for (size_t s = 0; s < nd; ++s) {
    seg[s] = s;
    frag[s] = (uint8_t)(s % 6);
    CHECK(hipMalloc((void**)&out[s], Fd) == hipSuccess);
  }
  uint8_t id[CEC_DIST_ID_BYTES];
  cec_dist* d = NULL;
  CHECK(cec_dist_unique_id(id) == CEC_OK);
  CHECK(cec_dist_create(c, id, 1, 0, &d) == CEC_OK);
  CHECK(cec_dist_degraded_read(d, seg, frag, nd, Fd, locate, &st, out, NULL, NULL) == CEC_OK);
  /* a codec that used the host API (stage) and the pool (a per-segment rebuild's plan) */
  cec_codec* lone = NULL;
  CHECK(cec_create(4, 2, 0, &lone) == CEC_OK);
  {
    uint8_t* hs[6];
    uint8_t pres[6] = {1, 0, 1, 1, 1, 1};
    for (int i = 0; i < 6; ++i) {
      hs[i] = malloc(4096);
      CHECK(hs[i] != NULL);
      memset(hs[i], i * 7 + 1, 4096);
    }
    CHECK(cec_encode(lone, hs, 4096) == CEC_OK);
    CHECK(cec_reconstruct(lone, hs, pres, 4096, 0) == CEC_OK);
    for (int i = 0; i < 6; ++i) free(hs[i]);
    uint8_t bp[6 * 6];
    for (size_t s = 0; s < nd * 6; ++s) bp[s] = (s % 6) != (s / 6) % 6;
    CHECK(cec_reconstruct_batch(lone, st.d_data, st.d_par, nd, Fd, bp, 0, 0, NULL) == CEC_OK);
    CHECK(hipDeviceSynchronize() == hipSuccess);
  }
  hipEvent_t t0, t1;
  CHECK(hipEventCreate(&t0) == hipSuccess && hipEventCreate(&t1) == hipSuccess);
  /* a long batch on the side stream, then a destroy while it runs: the lone codec first, then
   * (a second batch) the dist handle and its codec */
  int busy[4];
  float ms[3];
  for (int phase = 0; phase < 3; ++phase) {
    if (phase < 2) {
      CHECK(hipEventRecord(t0, side) == hipSuccess);
      for (int r = 0; r < reps; ++r)
        CHECK(cec_encode_batch(side_codec, d_data, d_par, nseg, F, side) == CEC_OK);
      CHECK(hipEventRecord(t1, side) == hipSuccess);
    }
    if (phase == 0) {
      cec_destroy(lone);
      busy[0] = hipStreamQuery(side) == hipErrorNotReady;
    } else if (phase == 2) {
      /* control: RCCL's own communicator teardown, no libcessec involved */
      ncclUniqueId uid;
      ncclComm_t comm;
      CHECK(ncclGetUniqueId(&uid) == ncclSuccess);
      CHECK(ncclCommInitRank(&comm, 1, uid, 0) == ncclSuccess);
      CHECK(hipEventRecord(t0, side) == hipSuccess);
      for (int r = 0; r < reps; ++r)
        CHECK(cec_encode_batch(side_codec, d_data, d_par, nseg, F, side) == CEC_OK);
      CHECK(hipEventRecord(t1, side) == hipSuccess);
      (void)ncclCommDestroy(comm);
      busy[3] = hipStreamQuery(side) == hipErrorNotReady;
    } else {
      cec_dist_destroy(d);
      busy[1] = hipStreamQuery(side) == hipErrorNotReady;
      cec_destroy(c);
      busy[2] = hipStreamQuery(side) == hipErrorNotReady;
    }
    CHECK(hipStreamSynchronize(side) == hipSuccess);
    CHECK(hipEventElapsedTime(&ms[phase], t0, t1) == hipSuccess);
  }
  printf("side stream busy after codec destroy: %d (batch %.1f ms); after dist destroy: %d, after "
         "its codec's destroy: %d (batch %.1f ms); after a bare ncclCommDestroy: %d (batch %.1f ms)\n",
         busy[0], ms[0], busy[1], busy[2], ms[1], busy[3], ms[2]);
  (void)hipEventDestroy(t0);
  (void)hipEventDestroy(t1);
  /* the side work is complete and bit-exact */
  uint32_t* h = malloc(nseg * 3 * F);
  CHECK(h != NULL);
  CHECK(hipMemcpy(h, d_data, nseg * 2 * F, hipMemcpyDeviceToHost) == hipSuccess);
  uint32_t* hp = h + nseg * 2 * F / 4;
  CHECK(hipMemcpy(hp, d_par, nseg * F, hipMemcpyDeviceToHost) == hipSuccess);
  for (size_t s = 0; s < nseg; ++s) {
    const uint32_t* d0 = h + s * 2 * F / 4;
    const uint32_t* d1 = d0 + F / 4;
    const uint32_t* p = hp + s * F / 4;
    for (size_t w = 0; w < F / 4; ++w) CHECK(p[w] == (xt4(d0[w] ^ d1[w]) ^ d0[w]));
  }
  /* and the degraded read's outputs were right */
  uint8_t* got = malloc(Fd);
  uint8_t* want = malloc(Fd);
  for (size_t s = 0; s < nd; ++s) {
    CHECK(hipMemcpy(got, out[s], Fd, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(hipMemcpy(want, locate(&st, s, frag[s]), Fd, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(memcmp(got, want, Fd) == 0);
    (void)hipFree(out[s]);
  }
  free(h);
  free(got);
  free(want);
  (void)hipFree(st.d_data);
  (void)hipFree(st.d_par);
  (void)hipFree(d_data);
  (void)hipFree(d_par);
  (void)hipStreamDestroy(side);
  cec_destroy(side_codec);
  return 0;
}

int main(void) {
  if (run(2, 1, 12, (size_t)1 << 20)) return 1;
  if (run(4, 2, 9, 65536 + 64)) return 1;
  if (destroy_under_load()) return 1;
  printf("dist world1 ok\n");
  return 0;
}
