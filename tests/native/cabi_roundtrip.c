/* C consumer of libcessec through include/cess_ec.h only (no Python, no torch): what a cgo / FFI
 * binding sees. Encodes a segment with the host-buffer API, checks the parity against the C
 * oracle (linked separately, test infrastructure), erases each fragment in turn and
 * reconstructs it, then exercises the error paths.
 * build: gcc -O2 tests/native/cabi_roundtrip.c -Iinclude -Lcess_amd -lcessec
 *            -Loracle/build -loracle -Wl,-rpath,... -o cabi_roundtrip */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cess_ec.h"

int orc_encode(int k, int m, const unsigned char* const* data, unsigned char* const* parity,
               size_t len);

#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, cec_last_error()); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

static int roundtrip(int k, int m, size_t len) {
  const int n = k + m;
  cec_codec* c = NULL;
  CHECK(cec_create(k, m, 0, &c) == CEC_OK);
  unsigned char** sh = calloc(n, sizeof(*sh));
  unsigned char** ref = calloc(n, sizeof(*ref));
  for (int i = 0; i < n; ++i) {
    sh[i] = malloc(len);
    ref[i] = malloc(len);
  }
  unsigned s = 12345u + (unsigned)(k * 131 + m);
  for (int i = 0; i < k; ++i)
    for (size_t b = 0; b < len; ++b) {
      s = s * 1103515245u + 12345u;
      sh[i][b] = ref[i][b] = (unsigned char)(s >> 16);
    }
  CHECK(cec_encode(c, sh, len) == CEC_OK);
  CHECK(orc_encode(k, m, (const unsigned char* const*)ref, ref + k, len) == 0);
  for (int i = k; i < n; ++i) CHECK(memcmp(sh[i], ref[i], len) == 0);
  int ok = 0;
  CHECK(cec_verify(c, sh, len, &ok) == CEC_OK && ok == 1);
  unsigned char* present = malloc(n);
  for (int e = 0; e < n; ++e) { /* every single erasure, incl. parity */
    memset(present, 1, n);
    present[e] = 0;
    memset(sh[e], 0xAB, len);
    CHECK(cec_reconstruct(c, sh, present, len, 0) == CEC_OK);
    CHECK(memcmp(sh[e], ref[e], len) == 0);
  }
  memset(present, 0, n); /* too few */
  for (int i = 0; i < k - 1; ++i) present[i] = 1;
  CHECK(cec_reconstruct(c, sh, present, len, 0) == CEC_ETOOFEW);
  CHECK(cec_encode(c, sh, 0) == CEC_ESHARDLEN);
  for (int i = 0; i < n; ++i) {
    free(sh[i]);
    free(ref[i]);
  }
  free(sh);
  free(ref);
  free(present);
  cec_destroy(c);
  return 0;
}

int main(void) {
  cec_codec* c = NULL;
  CHECK(cec_create(0, 1, 0, &c) == CEC_EINVAL);
  CHECK(cec_create(200, 57, 0, &c) == CEC_EINVAL);
  if (roundtrip(2, 1, 8u << 20)) return 1; /* CESS geometry: 16 MiB segment */
  if (roundtrip(4, 2, 1001)) return 1;
  if (roundtrip(32, 32, 512u << 10)) return 1;
  printf("cabi roundtrip ok (%s)\n", cec_version());
  return 0;
}
