/*
 * CPU oracle for the CESS segment -> fragment Reed-Solomon path, plain C restatement.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ as the checker and by bench.py's cpu_baseline leg
 * (kind "port"). The product (cess_amd/, libcessec) never links or calls this.
 *
 * Restates the same algorithm as oracle/rs_oracle.py, independently of the product code:
 *   - geometry: primitives/common/src/lib.rs:60-61 (16 MiB segment, 8 MiB fragment),
 *     runtime/src/lib.rs:1027 (3 fragments) -> RS(k=2, m=1);
 *   - arithmetic: klauspost/reedsolomon's published algorithm (galois.go, matrix.go,
 *     reedsolomon.go buildMatrix / Encode / Reconstruct), not vendored in the reference and
 *     version-unpinned: GF(2^8)/0x11D, E = V * inv(V[:k]), V[r][c] = r^c;
 *   - SHA-256: FIPS 180-4 (readable restatement in the reference at
 *     utils/ring/src/digest/sha2.rs:46-145); vectors utils/ring/third_party/NIST/SHAVS.
 * Encode uses one 256-entry product table per coefficient (scalar), the split-nibble pshufb
 * form (AVX2), or one GF(2) affine transform per coefficient (AVX-512BW + GFNI
 * vgf2p8affineqb: multiplication by a constant c is GF(2)-linear, an 8x8 bit matrix); the
 * best the host has by default, all checked against each other in tests.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#define POLY 0x11D

static uint8_t g_exp[512];
static int g_log[256];
static uint8_t g_mul[256][256];
static int g_init = 0;

static void gf_init(void) {
  if (g_init) return;
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    g_exp[i] = (uint8_t)x;
    g_log[x] = i;
    x <<= 1;
    if (x & 0x100) x ^= POLY;
  }
  for (int i = 255; i < 512; ++i) g_exp[i] = g_exp[i - 255];
  for (int a = 0; a < 256; ++a)
    for (int b = 0; b < 256; ++b)
      g_mul[a][b] = (a && b) ? g_exp[g_log[a] + g_log[b]] : 0;
  g_init = 1;
}

static uint8_t gexp(int a, int n) {
  if (n == 0) return 1;
  if (a == 0) return 0;
  return g_exp[(g_log[a] * n) % 255];
}

/* n x n inverse, row-major; returns 0 on success */
static int invert(const uint8_t* a, int n, uint8_t* out) {
  uint8_t* w = (uint8_t*)malloc((size_t)n * 2 * n);
  if (!w) return -1;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < 2 * n; ++c) w[r * 2 * n + c] = c < n ? a[r * n + c] : (c - n == r);
  for (int col = 0; col < n; ++col) {
    int p = col;
    while (p < n && !w[p * 2 * n + col]) ++p;
    if (p == n) { free(w); return -1; }
    if (p != col)
      for (int c = 0; c < 2 * n; ++c) {
        uint8_t t = w[col * 2 * n + c];
        w[col * 2 * n + c] = w[p * 2 * n + c];
        w[p * 2 * n + c] = t;
      }
    uint8_t s = g_exp[255 - g_log[w[col * 2 * n + col]]];
    for (int c = 0; c < 2 * n; ++c) w[col * 2 * n + c] = g_mul[s][w[col * 2 * n + c]];
    for (int r = 0; r < n; ++r) {
      uint8_t f = w[r * 2 * n + col];
      if (r == col || !f) continue;
      for (int c = 0; c < 2 * n; ++c) w[r * 2 * n + c] ^= g_mul[f][w[col * 2 * n + c]];
    }
  }
  for (int r = 0; r < n; ++r) memcpy(out + r * n, w + r * 2 * n + n, n);
  free(w);
  return 0;
}

/* (k+m) x k encode matrix, row-major */
int orc_matrix(int k, int m, uint8_t* out) {
  gf_init();
  if (k < 1 || m < 1 || k + m > 256) return -1;
  const int n = k + m;
  uint8_t* top = (uint8_t*)malloc((size_t)k * k);
  uint8_t* inv = (uint8_t*)malloc((size_t)k * k);
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c) top[r * k + c] = gexp(r, c);
  int rc = invert(top, k, inv);
  for (int r = 0; r < n && !rc; ++r)
    for (int c = 0; c < k; ++c) {
      uint8_t acc = 0;
      for (int t = 0; t < k; ++t) acc ^= g_mul[gexp(r, t)][inv[t * k + c]];
      out[r * k + c] = acc;
    }
  free(top);
  free(inv);
  return rc;
}

static void mul_acc_scalar(uint8_t* out, const uint8_t* in, uint8_t c, size_t len, int first) {
  const uint8_t* t = g_mul[c];
  if (first)
    for (size_t i = 0; i < len; ++i) out[i] = t[in[i]];
  else
    for (size_t i = 0; i < len; ++i) out[i] ^= t[in[i]];
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) static void mul_acc_avx2(uint8_t* out, const uint8_t* in,
                                                         uint8_t c, size_t len, int first) {
  uint8_t lo[16], hi[16];
  for (int i = 0; i < 16; ++i) {
    lo[i] = g_mul[c][i];
    hi[i] = g_mul[c][i << 4];
  }
  const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)lo));
  const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)hi));
  const __m256i mask = _mm256_set1_epi8(0x0f);
  size_t i = 0;
  for (; i + 32 <= len; i += 32) {
    __m256i x = _mm256_loadu_si256((const __m256i*)(in + i));
    __m256i l = _mm256_and_si256(x, mask);
    __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
    __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
    if (!first) p = _mm256_xor_si256(p, _mm256_loadu_si256((const __m256i*)(out + i)));
    _mm256_storeu_si256((__m256i*)(out + i), p);
  }
  if (i < len) mul_acc_scalar(out + i, in + i, c, len - i, first);
}
#endif

#if defined(__x86_64__)
/* The 8x8 GF(2) matrix of x -> c*x in vgf2p8affineqb's layout: result bit i is the parity of
 * (x AND matrix byte 7-i), so byte 7-i holds the input bits j whose product c * 2^j has bit i. */
static uint64_t affine_matrix(uint8_t c) {
  uint64_t a = 0;
  for (int i = 0; i < 8; ++i) {
    unsigned row = 0;
    for (int j = 0; j < 8; ++j)
      if (g_mul[c][1u << j] >> i & 1) row |= 1u << j;
    a |= (uint64_t)row << (8 * (7 - i));
  }
  return a;
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void mul_acc_gfni(
    uint8_t* out, const uint8_t* in, uint8_t c, size_t len, int first) {
  const __m512i A = _mm512_set1_epi64((long long)affine_matrix(c));
  size_t i = 0;
  for (; i + 64 <= len; i += 64) {
    __m512i p = _mm512_gf2p8affine_epi64_epi8(_mm512_loadu_si512((const void*)(in + i)), A, 0);
    if (!first) p = _mm512_xor_si512(p, _mm512_loadu_si512((const void*)(out + i)));
    _mm512_storeu_si512((void*)(out + i), p);
  }
  if (i < len) mul_acc_scalar(out + i, in + i, c, len - i, first);
}
#endif

static int g_simd = -1; /* -1 auto, 0 scalar, 1 avx2, 2 avx512bw + gfni */

int orc_set_simd(int v) {
  gf_init();
#if defined(__x86_64__)
  const int have_gfni = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("gfni");
  const int have_avx2 = __builtin_cpu_supports("avx2");
  if (v < 0) v = have_gfni ? 2 : have_avx2 ? 1 : 0;
  if (v == 2 && !have_gfni) v = have_avx2 ? 1 : 0;
  if (v == 1 && !have_avx2) v = 0;
#else
  v = 0;
#endif
  g_simd = v;
  return g_simd;
}

static void mul_acc(uint8_t* out, const uint8_t* in, uint8_t c, size_t len, int first) {
  if (g_simd < 0) orc_set_simd(-1);
#if defined(__x86_64__)
  if (g_simd == 2) {
    mul_acc_gfni(out, in, c, len, first);
    return;
  }
  if (g_simd == 1) {
    mul_acc_avx2(out, in, c, len, first);
    return;
  }
#endif
  mul_acc_scalar(out, in, c, len, first);
}

/* outs[o] = XOR_j rows[o*nin + j] * ins[j] */
static void code_rows(const uint8_t* rows, int nout, const uint8_t* const* ins, int nin,
                      uint8_t* const* outs, size_t len) {
  /* cache-block so every output stays hot while the inputs stream through */
  const size_t blk = 16384;
  for (size_t off = 0; off < len; off += blk) {
    const size_t n = len - off < blk ? len - off : blk;
    for (int o = 0; o < nout; ++o)
      for (int j = 0; j < nin; ++j) mul_acc(outs[o] + off, ins[j] + off, rows[o * nin + j], n, j == 0);
  }
}

int orc_encode(int k, int m, const uint8_t* const* data, uint8_t* const* parity, size_t len) {
  gf_init();
  uint8_t* e = (uint8_t*)malloc((size_t)(k + m) * k);
  if (!e || orc_matrix(k, m, e)) { free(e); return -1; }
  code_rows(e + (size_t)k * k, m, data, k, parity, len);
  free(e);
  return 0;
}

/* Two-pass klauspost Reconstruct; present[i] flags; returns -2 when too few shards. */
int orc_reconstruct(int k, int m, uint8_t* const* shards, const uint8_t* present, size_t len,
                    int data_only) {
  gf_init();
  const int n = k + m;
  int surv[256], ns = 0;
  for (int i = 0; i < n && ns < k; ++i)
    if (present[i]) surv[ns++] = i;
  if (ns < k) return -2;
  uint8_t* e = (uint8_t*)malloc((size_t)n * k);
  uint8_t* sub = (uint8_t*)malloc((size_t)k * k);
  uint8_t* inv = (uint8_t*)malloc((size_t)k * k);
  orc_matrix(k, m, e);
  for (int r = 0; r < k; ++r) memcpy(sub + r * k, e + surv[r] * k, k);
  int rc = invert(sub, k, inv);
  if (!rc) {
    const uint8_t* ins[256];
    for (int j = 0; j < k; ++j) ins[j] = shards[surv[j]];
    for (int i = 0; i < k; ++i)
      if (!present[i]) {
        uint8_t* o[1] = {shards[i]};
        code_rows(inv + i * k, 1, ins, k, o, len);
      }
    if (!data_only) {
      const uint8_t* din[256];
      for (int j = 0; j < k; ++j) din[j] = shards[j];
      for (int i = k; i < n; ++i)
        if (!present[i]) {
          uint8_t* o[1] = {shards[i]};
          code_rows(e + i * k, 1, din, k, o, len);
        }
    }
  }
  free(e);
  free(sub);
  free(inv);
  return rc;
}

/* ---- SHA-256 (FIPS 180-4) ----------------------------------------------------------------- */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha_block(uint32_t h[8], const uint8_t* p) {
  uint32_t w[64];
  for (int t = 0; t < 16; ++t)
    w[t] = (uint32_t)p[4 * t] << 24 | (uint32_t)p[4 * t + 1] << 16 | (uint32_t)p[4 * t + 2] << 8 |
           p[4 * t + 3];
  for (int t = 16; t < 64; ++t) {
    uint32_t s0 = ROR(w[t - 15], 7) ^ ROR(w[t - 15], 18) ^ (w[t - 15] >> 3);
    uint32_t s1 = ROR(w[t - 2], 17) ^ ROR(w[t - 2], 19) ^ (w[t - 2] >> 10);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 64; ++t) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[t] + w[t];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void orc_sha256(const uint8_t* buf, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha_block(h, buf + i);
  uint8_t tail[128] = {0};
  size_t r = len - i;
  memcpy(tail, buf + i, r);
  tail[r] = 0x80;
  size_t tl = r >= 56 ? 128 : 64;
  uint64_t bits = (uint64_t)len * 8;
  for (int q = 0; q < 8; ++q) tail[tl - 1 - q] = (uint8_t)(bits >> (8 * q));
  sha_block(h, tail);
  if (tl == 128) sha_block(h, tail + 64);
  for (int q = 0; q < 8; ++q) {
    out[4 * q] = (uint8_t)(h[q] >> 24);
    out[4 * q + 1] = (uint8_t)(h[q] >> 16);
    out[4 * q + 2] = (uint8_t)(h[q] >> 8);
    out[4 * q + 3] = (uint8_t)h[q];
  }
}

void orc_sha256_hex(const uint8_t* buf, size_t len, char out[64]) {
  static const char hx[] = "0123456789abcdef";
  uint8_t d[32];
  orc_sha256(buf, len, d);
  for (int i = 0; i < 32; ++i) {
    out[2 * i] = hx[d[i] >> 4];
    out[2 * i + 1] = hx[d[i] & 15];
  }
}

/* ---- synthetic segments -------------------------------------------------------------------- */
static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void orc_fill_synthetic(uint8_t* out, size_t seg_bytes, size_t nseg, uint64_t seg0,
                        uint64_t seed) {
  const size_t words = seg_bytes / 8;
  for (size_t s = 0; s < nseg; ++s)
    for (size_t w = 0; w < words; ++w) {
      uint64_t v = splitmix64(seed ^ ((seg0 + s) << 32) ^ w);
      memcpy(out + s * seg_bytes + w * 8, &v, 8); /* little-endian host */
    }
}

/* ---- multi-threaded batch encode (cpu_baseline) -------------------------------------------- */
typedef struct {
  int k, m;
  const uint8_t* e;
  const uint8_t* data;
  uint8_t* parity;
  size_t len, s0, s1;
} job_t;

static void* enc_worker(void* arg) {
  job_t* j = (job_t*)arg;
  const uint8_t* ins[256];
  uint8_t* outs[256];
  for (size_t s = j->s0; s < j->s1; ++s) {
    for (int i = 0; i < j->k; ++i) ins[i] = j->data + (s * j->k + i) * j->len;
    for (int o = 0; o < j->m; ++o) outs[o] = j->parity + (s * j->m + o) * j->len;
    code_rows(j->e + (size_t)j->k * j->k, j->m, ins, j->k, outs, j->len);
  }
  return NULL;
}

/* Encode nseg segments laid out [seg][k][len] -> [seg][m][len] with `threads` threads, `reps`
 * times. Returns wall seconds (monotonic clock). */
double orc_encode_batch(int k, int m, const uint8_t* data, uint8_t* parity, size_t nseg,
                        size_t len, int threads, int reps) {
  gf_init();
  uint8_t* e = (uint8_t*)malloc((size_t)(k + m) * k);
  orc_matrix(k, m, e);
  if (threads < 1) threads = 1;
  if ((size_t)threads > nseg) threads = (int)nseg;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  job_t* jobs = (job_t*)calloc(threads, sizeof(job_t));
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int r = 0; r < reps; ++r) {
    for (int t = 0; t < threads; ++t) {
      jobs[t] = (job_t){k, m, e, data, parity, len, nseg * t / threads, nseg * (t + 1) / threads};
      pthread_create(&th[t], NULL, enc_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  free(jobs);
  free(e);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- one segment on all threads (config 1: single-segment CPU encode + reconstruct) ------- */
typedef struct {
  int k, m, op; /* op -1: encode; e >= 0: reconstruct shard e from the others */
  uint8_t* const* shards;
  size_t len, c0, c1;
} seg_job_t;

static void* seg_worker(void* arg) {
  seg_job_t* j = (seg_job_t*)arg;
  uint8_t* sh[256];
  for (int i = 0; i < j->k + j->m; ++i) sh[i] = j->shards[i] + j->c0;
  const size_t n = j->c1 - j->c0;
  if (n == 0) return NULL;
  if (j->op < 0) {
    orc_encode(j->k, j->m, (const uint8_t* const*)sh, sh + j->k, n);
  } else {
    uint8_t present[256];
    for (int i = 0; i < j->k + j->m; ++i) present[i] = i != j->op;
    orc_reconstruct(j->k, j->m, sh, present, n, 0);
  }
  return NULL;
}

/* `reps` x (encode + every single-erasure reconstruct, shard e rebuilt in place from the
 * others) of one segment's k+m shards of `len` bytes, columns split over `threads` threads.
 * Returns wall seconds. Bytes per op = (k+m)*len (k read + 1 or m written, RS(2,1)). */
double orc_segment_ops(int k, int m, uint8_t* const* shards, size_t len, int threads, int reps) {
  gf_init();
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  seg_job_t* jobs = (seg_job_t*)calloc(threads, sizeof(seg_job_t));
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int r = 0; r < reps; ++r)
    for (int op = -1; op < k + m; ++op) {
      for (int t = 0; t < threads; ++t) {
        /* 64-byte aligned column ranges */
        size_t c0 = (len * t / threads) & ~(size_t)63, c1 = (len * (t + 1) / threads) & ~(size_t)63;
        if (t == threads - 1) c1 = len;
        jobs[t] = (seg_job_t){k, m, op, shards, len, c0, c1};
        pthread_create(&th[t], NULL, seg_worker, &jobs[t]);
      }
      for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  free(jobs);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
