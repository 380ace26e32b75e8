/* cec_dist_degraded_read at world > 1 on ONE GPU: the C-ABI multi-GPU degraded read (what a cgo /
 * FFI host runs per rank, include/cess_ec.h) with every rank a thread of this process on device 0,
 * over the test-only RCCL stand-in (tests/native/rccl_standin.cpp, loaded by libcessec's dlopen of
 * librccl.so.1 through LD_LIBRARY_PATH; this program does not link RCCL). It exercises the world > 1
 * protocol of cess_amd/csrc/dist.cpp that a one-GPU box cannot run over real RCCL: the agreement
 * all-reduce, send/recv pairing in plan order (survivors, then partials), rounds of 256 segments
 * enqueued back to back, the ragged-holder memset of the partial exchange, and an abort inside a
 * group. The placement is the chain's miner spread (fragment f of segment s on rank (s + f) mod
 * world, c-pallets/file-bank/src/functions.rs:187-283); the degraded read is the off-chain half of
 * restoral (c-pallets/file-bank/src/lib.rs:943-1122). Every rebuilt fragment is compared with the
 * C oracle's codeword (oracle/rs_oracle.c: the checker, test infrastructure only).
 *
 * usage: dist_world_n WORLD K M NSEG F EXCHANGE ABORT_RANK [GROUP_OPS]
 *   EXCHANGE 0 survivors, 1 partials, 2 auto; ABORT_RANK -1 = none, else that rank fails inside
 *   round 0's transfer group (CEC_DIST_OPT_TEST_ABORT), then every rank joins a fresh group;
 *   -2 = host only: print the plan's shape (and whether the stand-in was loaded), no GPU.
 *   GROUP_OPS: CEC_DIST_OPT_GROUP_OPS (transfers per rank per RCCL group; default: the library's).
 * prints one line "world_n ok ..." on success, "FAIL ..." lines otherwise (exit 1). */
#include <execinfo.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "cess_ec.h"

/* the C oracle (oracle/rs_oracle.c) */
void orc_fill_synthetic(uint8_t* out, size_t seg_bytes, size_t nseg, uint64_t seg0,
                        uint64_t seed);
double orc_encode_batch(int k, int m, const uint8_t* data, uint8_t* parity, size_t nseg,
                        size_t len, int threads, int reps);

#define SEED 0xCE550004ull
#define ROUND 256 /* dist.cpp kRound */

static int W, K, M, N, EXCH, ABORT_RANK, GROUP_OPS = -1;
static size_t NSEG, F, NLOST;
static uint8_t *h_data, *h_par;   /* the codewords: [seg][k][F], [seg][m][F] */
static uint64_t* lost_seg;
static uint8_t* lost_frag;
static int32_t* decoder;
static uint8_t* is_lost;          /* [seg][n] */
static uint8_t id1[CEC_DIST_ID_BYTES], id2[CEC_DIST_ID_BYTES];
static pthread_barrier_t bar;

static const uint8_t* host_frag(size_t s, int f) {
  return f < K ? h_data + (s * K + f) * F : h_par + (s * M + (f - K)) * F;
}

typedef struct {
  int rank;
  uint8_t* d_store;
  long long* slot;  /* [seg][n] index into d_store, -1 = not held */
  int rc_first, rc_abort_retry;
  size_t rebuilt, bad;
  uint64_t groups;
  char why[256];
} rank_t;

static const uint8_t* locate(void* user, uint64_t seg, int frag) {
  const rank_t* r = (const rank_t*)user;
  if (seg >= NSEG || frag < 0 || frag >= N) return NULL;
  const long long i = r->slot[seg * N + frag];
  return i < 0 ? NULL : r->d_store + (size_t)i * F;
}

static uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

#define RCHECK(c)                                                                        \
  do {                                                                                   \
    if (!(c)) {                                                                          \
      snprintf(r->why, sizeof r->why, "%s:%d %s (%s)", __FILE__, __LINE__, #c,           \
               cec_last_error());                                                        \
      return -1;                                                                         \
    }                                                                                    \
  } while (0)

/* one degraded read on a group; outputs checked against the oracle codewords */
static int one_read(rank_t* r, cec_codec* c, const uint8_t* id, int abort_round, hipStream_t st,
                    int* rc_out) {
  cec_dist* d = NULL;
  RCHECK(cec_dist_create(c, id, W, r->rank, &d) == CEC_OK);
  RCHECK(cec_dist_set_option(d, CEC_DIST_OPT_EXCHANGE, EXCH) == CEC_OK);
  if (abort_round >= 0) RCHECK(cec_dist_set_option(d, CEC_DIST_OPT_TEST_ABORT, abort_round) == 0);
  if (GROUP_OPS >= 0) RCHECK(cec_dist_set_option(d, CEC_DIST_OPT_GROUP_OPS, GROUP_OPS) == 0);
  uint8_t* d_out = NULL;
  size_t mine = 0;
  for (size_t i = 0; i < NLOST; ++i) mine += decoder[i] == r->rank;
  uint8_t** outs = calloc(NLOST, sizeof(uint8_t*));
  RCHECK(outs != NULL);
  if (mine) {
    RCHECK(hipMalloc((void**)&d_out, mine * F) == hipSuccess);
    RCHECK(hipMemset(d_out, 0xA5, mine * F) == hipSuccess);
  }
  for (size_t i = 0, j = 0; i < NLOST; ++i)
    if (decoder[i] == r->rank) outs[i] = d_out + (j++) * F;
  size_t nrebuilt = 0;
  /* twice on the same handle: the second call reuses the staging and waits on the first's tail */
  int rc = CEC_OK;
  for (int pass = 0; pass < 2 && rc == CEC_OK; ++pass) {
    rc = cec_dist_degraded_read(d, lost_seg, lost_frag, NLOST, F, locate, r, outs, st, &nrebuilt);
    if (rc == CEC_OK) {
      RCHECK(nrebuilt == mine);
      uint8_t* got = malloc(F);
      RCHECK(got != NULL);
      for (size_t i = 0; i < NLOST; ++i) {
        if (!outs[i]) continue;
        RCHECK(hipMemcpy(got, outs[i], F, hipMemcpyDeviceToHost) == hipSuccess);
        if (memcmp(got, host_frag(lost_seg[i], lost_frag[i]), F) != 0) {
          if (!r->bad)
            snprintf(r->why, sizeof r->why, "pass %d: fragment (%llu, %d) differs from the oracle",
                     pass, (unsigned long long)lost_seg[i], lost_frag[i]);
          ++r->bad;
        }
      }
      free(got);
      if (pass == 0) {
        r->rebuilt = nrebuilt;
        RCHECK(cec_dist_groups(d, &r->groups) == CEC_OK);
      }
      if (mine) RCHECK(hipMemsetAsync(d_out, 0x5A, mine * F, st) == hipSuccess);
    }
  }
  *rc_out = rc;
  if (rc != CEC_OK) snprintf(r->why, sizeof r->why, "degraded read: %d (%s)", rc, cec_last_error());
  if (id == id1 && ABORT_RANK >= 0) {
    /* the aborted group: every rank stops here before any handle is torn down (a peer's copy may
     * still read a buffer of this rank) */
    pthread_barrier_wait(&bar);
    RCHECK(hipDeviceSynchronize() == hipSuccess);
  }
  cec_dist_destroy(d);
  if (d_out) RCHECK(hipFree(d_out) == hipSuccess);
  free(outs);
  return 0;
}

static void* rank_main(void* arg) {
  rank_t* r = (rank_t*)arg;
  r->rc_first = r->rc_abort_retry = 1;
  if (hipSetDevice(0) != hipSuccess) {
    snprintf(r->why, sizeof r->why, "hipSetDevice");
    return (void*)1;
  }
  cec_codec* c = NULL;
  hipStream_t st = NULL;
  if (cec_create(K, M, 0, &c) != CEC_OK || hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) {
    snprintf(r->why, sizeof r->why, "create: %s", cec_last_error());
    return (void*)1;
  }
  /* this rank's store: every fragment the placement puts here that is not lost */
  r->slot = malloc(NSEG * N * sizeof(long long));
  size_t held = 0;
  for (size_t s = 0; s < NSEG; ++s)
    for (int f = 0; f < N; ++f)
      r->slot[s * N + f] = ((s + f) % W == (size_t)r->rank && !is_lost[s * N + f]) ? held++ : -1;
  if (hipMalloc((void**)&r->d_store, (held ? held : 1) * F) != hipSuccess) {
    snprintf(r->why, sizeof r->why, "hipMalloc store");
    return (void*)1;
  }
  for (size_t s = 0; s < NSEG; ++s)
    for (int f = 0; f < N; ++f)
      if (r->slot[s * N + f] >= 0 &&
          hipMemcpy(r->d_store + r->slot[s * N + f] * F, host_frag(s, f), F,
                    hipMemcpyHostToDevice) != hipSuccess) {
        snprintf(r->why, sizeof r->why, "upload");
        return (void*)1;
      }
  int ret = one_read(r, c, id1, r->rank == ABORT_RANK ? 0 : -1, st, &r->rc_first);
  if (!ret && ABORT_RANK >= 0) {
    /* after the abort: a fresh group on the same threads and codecs rebuilds bit-exact */
    const size_t bad0 = r->bad;
    ret = one_read(r, c, id2, -1, st, &r->rc_abort_retry);
    if (r->bad != bad0) ret = -1;
  }
  (void)hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  (void)hipFree(r->d_store);
  free(r->slot);
  cec_destroy(c);
  return (void*)(long)(ret != 0);
}

/* a crash names where it happened (stderr), so one failure is enough to find its cause */
static void on_fatal(int sig) {
  static const char msg[] = "dist_world_n: fatal signal, backtrace:\n";
  void* frames[64];
  const int nf = backtrace(frames, 64);
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(frames, nf, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int main(int argc, char** argv) {
  signal(SIGSEGV, on_fatal);
  signal(SIGBUS, on_fatal);
  signal(SIGABRT, on_fatal);
  if (argc != 8 && argc != 9) {
    fprintf(stderr, "usage: %s WORLD K M NSEG F EXCHANGE ABORT_RANK [GROUP_OPS]\n", argv[0]);
    return 2;
  }
  if (argc == 9) GROUP_OPS = atoi(argv[8]);
  W = atoi(argv[1]);
  K = atoi(argv[2]);
  M = atoi(argv[3]);
  NSEG = strtoull(argv[4], NULL, 10);
  F = strtoull(argv[5], NULL, 10);
  EXCH = atoi(argv[6]);
  ABORT_RANK = atoi(argv[7]);
  N = K + M;
  if (W < 1 || W > 64 || K < 1 || M < 1 || N > 256 || !NSEG || !F) return 2;

  /* codewords from the oracle (data from the same counter generator the GPU uses) */
  h_data = calloc(NSEG * K, F);
  h_par = calloc(NSEG * M, F);
  is_lost = calloc(NSEG, N);
  lost_seg = malloc(NSEG * M * sizeof(uint64_t));
  lost_frag = malloc(NSEG * M);
  decoder = malloc(NSEG * M * sizeof(int32_t));
  if (!h_data || !h_par || !is_lost || !lost_seg || !lost_frag || !decoder) return 2;
  orc_fill_synthetic(h_data, (size_t)K * F, NSEG, 0, SEED);
  orc_encode_batch(K, M, h_data, h_par, NSEG, F, 8, 1);

  /* segment s loses 1 + s mod m distinct fragments at seeded positions (listed in a scrambled
   * order: the library groups them) */
  NLOST = 0;
  for (size_t s = 0; s < NSEG; ++s) {
    const int e = 1 + (int)(s % (size_t)M);
    for (int j = 0; j < e; ++j) {
      int f = (int)(mix(SEED ^ (s << 16) ^ (uint64_t)(j * 7919 + 1)) % (uint64_t)N);
      while (is_lost[s * N + f]) f = (f + 1) % N; /* collision: the next free index */
      is_lost[s * N + f] = 1;
      lost_seg[NLOST] = s;
      lost_frag[NLOST++] = (uint8_t)f;
    }
  }
  for (size_t i = NLOST; i > 1; --i) { /* deterministic shuffle */
    const size_t j = mix(SEED + i) % i;
    uint64_t ts = lost_seg[i - 1];
    uint8_t tf = lost_frag[i - 1];
    lost_seg[i - 1] = lost_seg[j];
    lost_frag[i - 1] = lost_frag[j];
    lost_seg[j] = ts;
    lost_frag[j] = tf;
  }

  /* the plan this read runs: moves per rank per round (the size of one rank's group), whether a
   * round's partial segments have different holder counts on one decoder (the ragged memset) */
  size_t nmoves = 0;
  if (cec_dist_plan_ex(K, M, W, EXCH, lost_seg, lost_frag, NLOST, NULL, 0, &nmoves, decoder)) {
    fprintf(stderr, "FAIL plan: %s\n", cec_last_error());
    return 1;
  }
  cec_dist_move* mv = malloc((nmoves ? nmoves : 1) * sizeof(cec_dist_move));
  if (cec_dist_plan_ex(K, M, W, EXCH, lost_seg, lost_frag, NLOST, mv, nmoves, &nmoves, decoder)) {
    fprintf(stderr, "FAIL plan: %s\n", cec_last_error());
    return 1;
  }
  /* segments in plan order are ascending; a segment's round = its rank among lost segments / 256 */
  long long* seg_round = malloc(NSEG * sizeof(long long));
  size_t nlseg = 0;
  for (size_t s = 0; s < NSEG; ++s) {
    int any = 0;
    for (int f = 0; f < N; ++f) any |= is_lost[s * N + f];
    seg_round[s] = any ? (long long)(nlseg++ / ROUND) : -1;
  }
  const size_t rounds = (nlseg + ROUND - 1) / ROUND;
  size_t* ops = calloc(rounds * W, sizeof(size_t));
  size_t npartial = 0, nsurv = 0;
  /* holders per partial segment: distinct sources */
  int* hold_cnt = calloc(NSEG, sizeof(int));
  for (size_t i = 0; i < nmoves; ++i) {
    if (mv[i].src == mv[i].dst) continue;
    const long long rd = seg_round[mv[i].seg];
    ++ops[rd * W + mv[i].src];
    ++ops[rd * W + mv[i].dst];
    if (mv[i].kind == CEC_DIST_PARTIAL) {
      ++npartial;
      int seen = 0;
      for (size_t j = 0; j < i; ++j)
        seen |= mv[j].seg == mv[i].seg && mv[j].src == mv[i].src && mv[j].kind == CEC_DIST_PARTIAL;
      hold_cnt[mv[i].seg] += !seen;
    } else {
      ++nsurv;
    }
  }
  size_t max_ops = 0;
  for (size_t i = 0; i < rounds * (size_t)W; ++i) max_ops = ops[i] > max_ops ? ops[i] : max_ops;
  int ragged = 0;
  int* seg_dec = malloc(NSEG * sizeof(int));
  for (size_t i = 0; i < NLOST; ++i) seg_dec[lost_seg[i]] = decoder[i];
  for (size_t rd = 0; rd < rounds; ++rd)
    for (int dr = 0; dr < W; ++dr) {
      int lo = 1 << 30, hi = -1;
      for (size_t s = 0; s < NSEG; ++s) {
        if (seg_round[s] != (long long)rd || !hold_cnt[s] || seg_dec[s] != dr) continue;
        lo = hold_cnt[s] < lo ? hold_cnt[s] : lo;
        hi = hold_cnt[s] > hi ? hold_cnt[s] : hi;
      }
      ragged |= hi > lo;
    }

  size_t predicted = 0;
  if (cec_dist_plan_groups(K, M, W, EXCH, GROUP_OPS < 0 ? 1024 : GROUP_OPS, lost_seg, lost_frag,
                           NLOST, NULL, 0, &predicted)) {
    fprintf(stderr, "FAIL plan groups: %s\n", cec_last_error());
    return 1;
  }
  if (cec_dist_unique_id(id1) || cec_dist_unique_id(id2)) {
    fprintf(stderr, "FAIL unique id: %s\n", cec_last_error());
    return 1;
  }
  const int standin = memcmp(id1, "cess-rccl-standin", 17) == 0;
  if (ABORT_RANK == -2) { /* host only: the plan and which librccl libcessec loaded */
    printf("plan world %d RS(%d,%d) nseg %zu lost %zu rounds %zu survivor_moves %zu "
           "partial_moves %zu max_ops_per_rank_round %zu ragged %d standin %d predicted_groups %zu\n",
           W, K, M, NSEG, NLOST, rounds, nsurv, npartial, max_ops, ragged, standin, predicted);
    return 0;
  }
  pthread_barrier_init(&bar, NULL, (unsigned)W);
  rank_t* rk = calloc(W, sizeof(rank_t));
  pthread_t* th = calloc(W, sizeof(pthread_t));
  for (int i = 0; i < W; ++i) {
    rk[i].rank = i;
    pthread_create(&th[i], NULL, rank_main, &rk[i]);
  }
  int fail = 0;
  size_t rebuilt = 0;
  for (int i = 0; i < W; ++i) {
    void* ret = NULL;
    pthread_join(th[i], &ret);
    rebuilt += rk[i].rebuilt;
    const int expect_fail = ABORT_RANK >= 0;
    if (ret || rk[i].bad || (!expect_fail && rk[i].rc_first != CEC_OK) ||
        (expect_fail && (rk[i].rc_abort_retry != CEC_OK ||
                         (i == ABORT_RANK && rk[i].rc_first != CEC_ENCCL)))) {
      fprintf(stderr, "FAIL rank %d: ret %ld rc %d retry %d bad %zu: %s\n", i, (long)ret,
              rk[i].rc_first, rk[i].rc_abort_retry, rk[i].bad, rk[i].why);
      fail = 1;
    }
  }
  for (int i = 1; i < W && ABORT_RANK < 0; ++i)
    if (rk[i].groups != rk[0].groups) {
      fprintf(stderr, "FAIL rank %d issued %llu transfer groups, rank 0 %llu\n", i,
              (unsigned long long)rk[i].groups, (unsigned long long)rk[0].groups);
      fail = 1;
    }
  if (ABORT_RANK < 0 && rk[0].groups != predicted) {
    fprintf(stderr, "FAIL issued %llu transfer groups, cec_dist_plan_groups predicted %zu\n",
            (unsigned long long)rk[0].groups, predicted);
    fail = 1;
  }
  if (ABORT_RANK < 0 && rebuilt != NLOST) {
    fprintf(stderr, "FAIL rebuilt %zu of %zu lost fragments\n", rebuilt, NLOST);
    fail = 1;
  }
  if (fail) return 1;
  printf("world_n ok world %d RS(%d,%d) nseg %zu F %zu exchange %d lost %zu rebuilt %zu rounds %zu "
         "survivor_moves %zu partial_moves %zu max_ops_per_rank_round %zu ragged %d standin %d "
         "groups %llu predicted_groups %zu", W, K, M, NSEG, F, EXCH, NLOST, rebuilt, rounds, nsurv,
         npartial, max_ops, ragged, standin, (unsigned long long)rk[0].groups, predicted);
  if (ABORT_RANK >= 0) {
    printf(" abort_rank %d first_rc", ABORT_RANK);
    for (int i = 0; i < W; ++i) printf(" %d", rk[i].rc_first);
  }
  printf("\n");
  return 0;
}
