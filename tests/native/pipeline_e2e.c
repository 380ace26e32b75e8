/* C consumer of libcessec's host pipeline (cec_pipeline_*, include/cess_ec.h only): what a
 * cgo / FFI binding drives to encode a file from host memory. A synthetic source (splitmix64
 * segments, repeated every `uniq` segments) is read by an 8-thread memcpy callback; sampled
 * segments' shards and SegmentList hashes are stashed by the callbacks and checked against the
 * C oracle (linked separately, test infrastructure) after the timed run. Prints one JSON line
 * with the end-to-end rate (PCIe-inclusive: H2D of the data, D2H of the parity, hashes on the
 * GPU).
 * usage: pipeline_e2e k m F nseg batch depth hash window [uniq] [check_every] [tail]
 *                     [tail_batches]
 * hash: 0 none, 1 GPU, 2 host, 3 hybrid (CEC_PIPE_HASH_*). Hash modes 2 and 3 run through
 * cec_pipeline_run_files with the source's size (the hybrid placement of the last batches needs
 * it; tail_batches -1 = auto), the others through cec_pipeline_run.
 * build: gcc -O2 -pthread tests/native/pipeline_e2e.c -Iinclude -Lcess_amd -lcessec
 *            -Loracle/build -loracle -Wl,-rpath,... -o pipeline_e2e */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cess_ec.h"

int orc_encode(int k, int m, const unsigned char* const* data, unsigned char* const* parity,
               size_t len);
void orc_sha256_hex(const unsigned char* buf, size_t len, char out[64]);
void orc_fill_synthetic(unsigned char* out, size_t seg_bytes, size_t nseg, uint64_t seg0,
                        uint64_t seed);

typedef struct {
  uint64_t seg;
  unsigned char* shards; /* (k + m) * F */
  unsigned char hex[64 * 257];
  int have_hex;
} sample_t;

typedef struct {
  int k, m;
  size_t F, SB, nseg, uniq, check_every;
  sample_t* samples;
  size_t nsamples;
  unsigned char* src; /* uniq segments */
  size_t pos, total;  /* source bytes handed out, source size */
  uint64_t frags_seen, recs_seen, checked, bad;
  uint64_t next_frag, next_rec; /* order checks */
} ctx_t;

typedef struct {
  unsigned char* dst;
  const unsigned char* src;
  size_t n;
} cp_t;

static void* cp_worker(void* a) {
  cp_t* c = (cp_t*)a;
  memcpy(c->dst, c->src, c->n);
  return NULL;
}

/* read(): the next bytes of a file of nseg segments whose segment s is source segment s % uniq */
static long long rd(void* user, uint8_t* dst, size_t cap) {
  ctx_t* x = (ctx_t*)user;
  size_t left = x->total - x->pos;
  size_t n = cap < left ? cap : left;
  size_t done = 0;
  while (done < n) { /* split at source wrap points, copy each run with 8 threads */
    size_t off = (x->pos + done) % (x->uniq * x->SB);
    size_t run = x->uniq * x->SB - off;
    if (run > n - done) run = n - done;
    pthread_t th[8];
    cp_t jobs[8];
    size_t per = (run + 7) / 8;
    int nt = 0;
    for (size_t a = 0; a < run; a += per, ++nt) {
      jobs[nt].dst = dst + done + a;
      jobs[nt].src = x->src + off + a;
      jobs[nt].n = run - a < per ? run - a : per;
      pthread_create(&th[nt], NULL, cp_worker, &jobs[nt]);
    }
    for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
    done += run;
  }
  x->pos += n;
  return (long long)n;
}

static const unsigned char* src_shard(ctx_t* x, uint64_t seg, int j) {
  return x->src + (seg % x->uniq) * x->SB + (size_t)j * x->F;
}

static int sampled(ctx_t* x, uint64_t seg) {
  return seg % x->check_every == 0 || seg == x->nseg - 1;
}

static sample_t* sample_of(ctx_t* x, uint64_t seg) {
  for (size_t i = 0; i < x->nsamples; ++i)
    if (x->samples[i].seg == seg) return &x->samples[i];
  return NULL;
}

static int on_frags(void* user, uint64_t seg, const uint8_t* const* shards, size_t shard_len) {
  ctx_t* x = (ctx_t*)user;
  if (seg != x->next_frag++ || shard_len != x->F) {
    x->bad++;
    return 0;
  }
  x->frags_seen++;
  if (!sampled(x, seg)) return 0;
  sample_t* s = &x->samples[x->nsamples++];
  s->seg = seg;
  s->have_hex = 0;
  s->shards = malloc((size_t)(x->k + x->m) * x->F);
  for (int i = 0; i < x->k + x->m; ++i) memcpy(s->shards + (size_t)i * x->F, shards[i], x->F);
  return 0;
}

/* after the run: data shards = the source (zero-padded tail), parity = the oracle's */
static void check_frags(ctx_t* x, sample_t* sm) {
  const uint64_t seg = sm->seg;
  const size_t real = (seg + 1) * x->SB <= x->total ? x->SB : x->total - seg * x->SB;
  unsigned char* d[256];
  unsigned char* p[256];
  for (int j = 0; j < x->k; ++j) {
    d[j] = calloc(1, x->F);
    size_t off = (size_t)j * x->F;
    if (off < real) memcpy(d[j], src_shard(x, seg, j), real - off < x->F ? real - off : x->F);
    if (memcmp(d[j], sm->shards + (size_t)j * x->F, x->F)) x->bad++;
  }
  for (int j = 0; j < x->m; ++j) p[j] = malloc(x->F);
  orc_encode(x->k, x->m, (const unsigned char* const*)d, p, x->F);
  for (int j = 0; j < x->m; ++j) {
    if (memcmp(p[j], sm->shards + (size_t)(x->k + j) * x->F, x->F)) x->bad++;
    free(p[j]);
  }
  for (int j = 0; j < x->k; ++j) free(d[j]);
  x->checked++;
}

static int on_rec(void* user, uint64_t seg, const uint8_t* seg_hex, const uint8_t* frag_hex) {
  ctx_t* x = (ctx_t*)user;
  if (seg != x->next_rec++) {
    x->bad++;
    return 0;
  }
  x->recs_seen++;
  if (!sampled(x, seg)) return 0;
  sample_t* s = sample_of(x, seg);
  if (!s) {  /* on_fragments of a segment always precedes its on_record */
    x->bad++;
    return 0;
  }
  memcpy(s->hex, seg_hex, 64);
  memcpy(s->hex + 64, frag_hex, 64 * (size_t)(x->k + x->m));
  s->have_hex = 1;
  return 0;
}

/* cec_pipeline_run_files callbacks: one source, so the file index is 0 */
static int on_frags_f(void* user, size_t file, uint64_t seg, const uint8_t* const* shards,
                      size_t shard_len) {
  if (file != 0) ((ctx_t*)user)->bad++;
  return on_frags(user, seg, shards, shard_len);
}
static int on_rec_f(void* user, size_t file, uint64_t seg, const uint8_t* seg_hex,
                    const uint8_t* frag_hex) {
  if (file != 0) ((ctx_t*)user)->bad++;
  return on_rec(user, seg, seg_hex, frag_hex);
}
static int on_done_f(void* user, size_t file, const cec_pipeline_stats* st) {
  ctx_t* x = (ctx_t*)user;
  if (file != 0 || st->segments != x->nseg || st->bytes_in != x->total || x->recs_seen != x->nseg)
    x->bad++;
  return 0;
}

/* after the run: SegmentList hashes = SHA-256 hex of the oracle's segment and fragments */
static void check_rec(ctx_t* x, sample_t* sm) {
  if (!sm->have_hex) {
    x->bad++;
    return;
  }
  char h[64];
  unsigned char* segbuf = sm->shards; /* the k data shards are the zero-padded segment */
  orc_sha256_hex(segbuf, x->SB, h);
  if (memcmp(h, sm->hex, 64)) x->bad++;
  for (int i = 0; i < x->k + x->m; ++i) {
    orc_sha256_hex(segbuf + (size_t)i * x->F, x->F, h);
    if (memcmp(h, sm->hex + 64 * (i + 1), 64)) x->bad++;
  }
}

int main(int argc, char** argv) {
  if (argc < 9) {
    fprintf(stderr, "usage: %s k m F nseg batch depth hash window [uniq] [check_every] [tail]\n",
            argv[0]);
    return 2;
  }
  ctx_t x;
  memset(&x, 0, sizeof(x));
  x.k = atoi(argv[1]);
  x.m = atoi(argv[2]);
  x.F = strtoull(argv[3], 0, 10);
  x.nseg = strtoull(argv[4], 0, 10);
  cec_pipeline_opts o;
  memset(&o, 0, sizeof(o));
  o.shard_len = x.F;
  o.batch_segments = strtoull(argv[5], 0, 10);
  o.depth = atoi(argv[6]);
  o.hash = atoi(argv[7]);
  o.window = atoi(argv[8]);
  x.uniq = argc > 9 ? strtoull(argv[9], 0, 10) : 16;
  x.check_every = argc > 10 ? strtoull(argv[10], 0, 10) : 7;
  const size_t tail = argc > 11 ? strtoull(argv[11], 0, 10) : 0; /* bytes short of nseg * SB */
  o.tail_batches = argc > 12 ? atoi(argv[12]) : -1;
  if (x.uniq > x.nseg) x.uniq = x.nseg;
  x.SB = (size_t)x.k * x.F;
  x.total = x.nseg * x.SB - tail;
  x.src = malloc(x.uniq * x.SB);
  x.samples = calloc(x.nseg / x.check_every + 2, sizeof(sample_t));
  orc_fill_synthetic(x.src, x.SB, x.uniq, 0, 0xCE550004ull);

  cec_codec* c = NULL;
  cec_pipeline* p = NULL;
  if (cec_create(x.k, x.m, 0, &c) || cec_pipeline_create(c, &o, &p)) {
    fprintf(stderr, "create: %s\n", cec_last_error());
    return 1;
  }
  cec_pipeline_stats st;
  int rc;
  if (o.hash >= CEC_PIPE_HASH_HOST) {
    cec_source src = {rd, &x, x.total};
    rc = cec_pipeline_run_files(p, &src, 1, on_frags_f, on_rec_f, on_done_f, &x, &st);
  } else {
    rc = cec_pipeline_run(p, rd, on_frags, o.hash ? on_rec : NULL, &x, &st);
  }
  if (rc) {
    fprintf(stderr, "run: %d %s\n", rc, cec_last_error());
    return 1;
  }
  for (size_t i = 0; i < x.nsamples; ++i) { /* checks outside the timed run */
    check_frags(&x, &x.samples[i]);  /* parity checked first, so the hashes below use it */
    if (o.hash) check_rec(&x, &x.samples[i]);
    free(x.samples[i].shards);
  }
  const int ok = x.bad == 0 && x.frags_seen == x.nseg && (!o.hash || x.recs_seen == x.nseg) &&
                 st.segments == x.nseg && st.bytes_in == x.total;
  printf("{\"pipeline\": \"%s\", \"k\": %d, \"m\": %d, \"fragment_bytes\": %zu, "
         "\"segments\": %llu, \"batch\": %zu, \"depth\": %d, \"hash\": %d, \"window\": %d, "
         "\"tail_batches\": %d, "
         "\"bytes_in\": %llu, \"seconds\": %.4f, \"read_seconds\": %.4f, \"wait_seconds\": %.4f, "
         "\"e2e_GBps\": %.3f, \"pcie_gen5_x16_GBps_per_direction\": 63, \"checked\": %llu, "
         "\"bad\": %llu}\n",
         ok ? "ok" : "FAIL", x.k, x.m, x.F, (unsigned long long)st.segments, o.batch_segments,
         o.depth, o.hash, o.window, o.tail_batches, (unsigned long long)st.bytes_in, st.seconds, st.read_seconds,
         st.wait_seconds, st.bytes_in / st.seconds / 1e9, (unsigned long long)x.checked,
         (unsigned long long)x.bad);
  cec_pipeline_destroy(p);
  cec_destroy(c);
  free(x.src);
  return ok ? 0 : 1;
}
