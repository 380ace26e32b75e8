/*
 * cess_ec.h — C ABI of libcessec, the MI355X (gfx950) Reed-Solomon codec for CESS's
 * segment -> fragment path.
 *
 * Reference interfaces replaced (see SURVEY.md §8b and INTEGRATION.md):
 *   The reference chain (/root/reference) holds no codec: it fixes the geometry and records the
 *   codec's outputs. Its interface for this path is the on-chain record
 *     FileBank::upload_declaration(file_hash, deal_info: BoundedVec<SegmentList>, user_brief)
 *       c-pallets/file-bank/src/lib.rs:423-428
 *     SegmentList { hash: Hash, fragment_list: BoundedVec<Hash, FragmentCount> }
 *       c-pallets/file-bank/src/types.rs:13-16
 *     Hash([u8; 64])                          primitives/common/src/lib.rs:16
 *     SEGMENT_SIZE = 16 MiB, FRAGMENT_SIZE = 8 MiB   primitives/common/src/lib.rs:60-61
 *     FRAGMENT_COUNT = 3                      runtime/src/lib.rs:1027
 *   and the restoral (repair) flow whose off-chain step is a single-fragment reconstruct
 *     generate_restoral_order / restoral_order_complete   c-pallets/file-bank/src/lib.rs:943-1122
 *   The entry points below mirror the off-chain codec API those records come from
 *   (klauspost/reedsolomon Encoder: New / Encode / Reconstruct / ReconstructData / Verify /
 *   Split — not vendored in the reference), one function per operation,
 *   plus batched device-resident forms for HBM-resident segment batches.
 *
 * Conventions: GF(2^8), polynomial 0x11D, systematic Vandermonde matrix.
 * Shard i < k is data, i >= k parity. All functions return 0 or a negative CEC_E* code; no
 * exceptions cross the ABI. A codec is bound to one device and is not re-entrant; distinct
 * codecs are independent (cec_destroy waits only for the codec's own queued launches, never for
 * the device). Caller owns every shard / segment / hash buffer.
 */
#ifndef CESS_EC_H
#define CESS_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CEC_OK 0
#define CEC_EINVAL (-1)     /* bad k/m (k<1, m<1, k+m>256), null pointer, bad option */
#define CEC_ETOOFEW (-2)    /* fewer than k shards present (klauspost ErrTooFewShards) */
#define CEC_ESHARDLEN (-3)  /* zero or mismatched shard length (ErrShardSize / ErrShardNoData) */
#define CEC_EHIP (-4)       /* HIP runtime error (see cec_last_error) */
#define CEC_ENOMEM (-5)     /* device or host allocation failed */
#define CEC_ENCCL (-6)      /* RCCL error (multi-GPU paths) */
#define CEC_ESHORTDATA (-7) /* split of an empty segment (klauspost ErrShortData) */
#define CEC_ENODEV (-8)     /* no usable GPU */
#define CEC_ESEGCOUNT (-9)  /* more segments than the chain's SegmentCount bound (1000) */
#define CEC_ECALLBACK (-10) /* a pipeline callback returned an error */

typedef struct cec_codec cec_codec;

/* Library identity: "cessec <version> gfx950". */
const char* cec_version(void);
const char* cec_strerror(int code);
/* Detail text of the last error on this thread (HIP error string etc.). */
const char* cec_last_error(void);
/* Number of visible HIP devices (0 when none). */
int cec_device_count(void);

/* New(k, m): codec bound to `device`. Builds the (k+m) x k matrix; k >= 1, m >= 1, k+m <= 256. */
int cec_create(int k, int m, int device, cec_codec** out);
void cec_destroy(cec_codec* codec);
/* k, m and device of a codec (any output pointer may be NULL). */
int cec_codec_info(const cec_codec* codec, int* k, int* m, int* device);
/* Copy the (k+m) x k encode matrix, row-major, into `out`. Host only, no GPU work. */
int cec_matrix(const cec_codec* codec, uint8_t* out);

/* Host-buffer API (klauspost-shaped). `shards` holds k+m host pointers of shard_len bytes each.
 * The data is staged through HBM; calls are synchronous. */
int cec_encode(cec_codec* codec, uint8_t* const* shards, size_t shard_len);
/* present[i] != 0: shard i is valid. Missing shards are written in place; with data_only only
 * missing data shards are produced (ReconstructData). All present: no-op. Every rebuild (here and
 * in the batch calls) reads exactly the k survivors cec_survivors names, nothing else flagged
 * present: the first k present shards (klauspost's choice), or for RS(32,32) the set the
 * FFT-domain decoders rebuild from most cheaply. Any k survivors give the same bytes. */
int cec_reconstruct(cec_codec* codec, uint8_t* const* shards, const uint8_t* present,
                    size_t shard_len, int data_only);
/* Host only: the k survivors (ascending shard indices) a rebuild of the pattern `present`
 * (k + m flags) reads. A caller that moves survivors to the decoder (a multi-GPU gather, a
 * repair service fetching from peers) moves these. CEC_ETOOFEW below k present. */
int cec_survivors(int k, int m, const uint8_t* present, uint8_t* survivors);
/* *ok = 1 when every parity shard equals the encode of the data shards. */
int cec_verify(cec_codec* codec, uint8_t* const* shards, size_t shard_len, int* ok);

/* Batched device-resident API. d_data: [nseg][k][shard_len], d_parity: [nseg][m][shard_len],
 * both in HBM. Work is enqueued on `hip_stream` (NULL = the HIP null stream, as in the HIP API)
 * and the call returns without waiting.
 * HIP graph capture: the calls whose kernels take compile-time coefficients and read no
 * codec-owned memory may be captured (hipStreamBeginCapture on hip_stream) and replayed, after
 * one uncaptured call of the same shape: cec_encode_batch of RS(2,1) and RS(32,32), and
 * cec_reconstruct_batch of RS(2,1) with one pattern (per_segment = 0). Every other rebuild reads
 * a decode program from the codec's cache, which may evict it while a graph still points at it:
 * do not capture those. A single 16 MiB RS(2,1) segment's encode + three rebuilds: 29.5 us
 * eagerly, 24.8 us as one graph (profiles/r05/graph_probe.log). */
int cec_encode_batch(cec_codec* codec, const uint8_t* d_data, uint8_t* d_parity, size_t nseg,
                     size_t shard_len, void* hip_stream);
/* Rebuild missing shards in place in the same layout. `present` is a host array of k+m flags
 * (per_segment = 0: one pattern for every segment) or nseg*(k+m) flags (per_segment = 1).
 * Segments are grouped by erasure pattern; decode matrices are inverted on the host once per
 * pattern and cached. */
int cec_reconstruct_batch(cec_codec* codec, uint8_t* d_data, uint8_t* d_parity, size_t nseg,
                          size_t shard_len, const uint8_t* present, int per_segment,
                          int data_only, void* hip_stream);
/* Partial rebuild (the partial-product exchange of a multi-GPU degraded read):
 * like cec_reconstruct_batch with per-segment patterns (present: nseg*(k+m) flags; survivors =
 * cec_survivors of each segment's pattern), but every missing shard receives only the
 * contribution of the survivors flagged in `held` (nseg*(k+m) flags; flags of non-survivors are
 * ignored): out = XOR over held survivors i of D[out][i] * shard_i. Only held survivors are read
 * (a segment with no held survivor gets zeros: its program multiplies one survivor slot of the
 * batch, whatever it holds, by zero coefficients). The rebuild is linear, so XOR-ing the partials
 * of a partition of the survivors (one per GPU holding some of them, cec_xor_batch) gives the
 * missing shard. A GPU then sends one partial per lost fragment instead of its survivors. */
int cec_reconstruct_partial_batch(cec_codec* codec, uint8_t* d_data, uint8_t* d_parity,
                                  size_t nseg, size_t shard_len, const uint8_t* present,
                                  const uint8_t* held, int data_only, void* hip_stream);
/* Verify for a batch (klauspost Verify over HBM): d_ok[s] (device, nseg bytes) = 1 when the
 * parity shards of segment s equal the encode of its data shards, else 0. The parity is
 * recomputed into codec-owned scratch and compared; nothing in the batch is written. */
int cec_verify_batch(cec_codec* codec, const uint8_t* d_data, const uint8_t* d_parity,
                     size_t nseg, size_t shard_len, uint8_t* d_ok, void* hip_stream);
/* GF(2^8) addition of device buffers: d_dst[0..len) ^= d_src[j*src_stride ..][0..len) for
 * j < nsrc (src_stride >= len when nsrc > 1). Enqueued on hip_stream, which must belong to the
 * device holding the buffers (no codec: the caller's current device and stream decide). */
int cec_xor_batch(uint8_t* d_dst, const uint8_t* d_src, size_t nsrc, size_t src_stride,
                  size_t len, void* hip_stream);
/* SHA-256 of every shard of every segment in the batch layout, as 64 lowercase hex chars:
 * d_hex[(seg*(k+m) + shard)*64 ...]. d_parity may be NULL to hash the k data shards only, in
 * which case the index is seg*k + shard. */
int cec_sha256_batch(cec_codec* codec, const uint8_t* d_data, const uint8_t* d_parity,
                     size_t nseg, size_t shard_len, uint8_t* d_hex, void* hip_stream);

/* SHA-256 hex of n device buffers of `len` bytes: `d_bufs` is a host array of device pointers;
 * `hex` is host memory of n*64 bytes. Synchronous. */
int cec_sha256_hex(const uint8_t* const* d_bufs, size_t n, size_t len, uint8_t* hex,
                   void* hip_stream);

/* Host SHA-256 of n HOST buffers of `len` bytes (the records of a batch whose bytes are in host
 * memory): 64 lowercase hex chars per buffer to hex[i*64 ...]; with prefix_hex, also the hex of
 * each buffer's first prefix_len bytes (a nonzero multiple of 64, <= len; a segment's chain then
 * yields data fragment 0's hash, as cec_hashq_add_prefix does on the GPU). Runs on `threads`
 * threads of a process-wide pool (<= 1: the calling thread only); each core hashes several
 * equal-length chains at once (SHA-NI interleaved 2 or 4 ways, or AVX-512 16 lanes), because one
 * chain alone leaves most of a core's SHA throughput idle. Synchronous. Host only, no GPU. */
int cec_sha256_host(const uint8_t* const* bufs, size_t n, size_t len, uint8_t* hex,
                    size_t prefix_len, uint8_t* prefix_hex, int threads);
/* cec_sha256_host of buffers whose len is a multiple of 64 that also writes each chain's state
 * after those len bytes (8 words, before the padding) to state_out + 8 i: fragment 0's hash and
 * the state a segment chain resumes from on the GPU (cec_hashq_add_resume). */
int cec_sha256_host_state(const uint8_t* const* bufs, size_t n, size_t len, uint8_t* hex,
                          uint32_t* state_out, int threads);
/* Forms of the host hasher: which one runs is process-wide (cec_host_sha_set_form; -1 restores
 * the default: AVX-512 x16 where the CPU has it, else SHA-NI x2 where it has SHA-NI).
 * cec_host_sha_probe times one form on the calling thread over `chains` chains of
 * bytes_per_chain bytes and returns GB/s (< 0: the CPU lacks the form). */
#define CEC_HSHA_SCALAR 0
#define CEC_HSHA_NI1 1
#define CEC_HSHA_NI2 2
#define CEC_HSHA_NI4 3
#define CEC_HSHA_X16 4
int cec_host_sha_set_form(int form);
int cec_host_sha_form(void);
/* Worker threads of the process-wide host SHA-256 pool: grown to the largest `threads` a call
 * asked for, and to the sum of the host_threads of the live host / hybrid pipelines (several
 * pipelines, one per GPU, each bring their own CPU share). */
int cec_host_sha_pool_threads(void);
double cec_host_sha_probe(int form, size_t bytes_per_chain, int chains);

/* Hash queue: streaming SHA-256 of many long device buffers (fragment and segment hashes).
 * Chains keep their state in HBM between launches, so one tick advances every live chain of
 * every batch added so far; a producer that adds a batch per step and ticks once per step hashes
 * a window of batches at once (one chain per buffer is serial, so the GPU's hash rate is the
 * number of chains in flight times one wave's issue rate). All work is enqueued on the stream
 * given at creation; buffers and hex outputs must stay valid until their add is complete.
 * Completion is tracked on the host from the lengths alone (no read-back): an add is complete
 * once the ticks enqueued so far cover its blocks, i.e. when the stream reaches that tick. */
typedef struct cec_hashq cec_hashq;
/* capacity: maximum live chains, a power of two (128 B of HBM each). */
int cec_hashq_create(int device, size_t capacity, void* hip_stream, cec_hashq** out);
/* Frees the table in stream order on the queue's stream (after the launches queued there); does
 * not wait, and does not stall other streams. */
void cec_hashq_destroy(cec_hashq* q);
/* Append n chains: buffer i is d_base + (i / per) * outer_stride + (i % per) * inner_stride, len
 * bytes; its 64 lowercase hex chars go to d_hex + ((i / per) * hex_outer + i % per) * 64
 * (d_hex NULL: no output). E.g. the fragments of a batch [nseg][k][F]: per = k, outer = k*F,
 * inner = F; its segment hashes: per = 1, outer = inner = k*F, len = k*F. *ticket (optional)
 * names the add. CEC_ENOMEM when the ring would overflow (tick first). */
int cec_hashq_add(cec_hashq* q, const uint8_t* d_base, size_t n, size_t per, size_t outer_stride,
                  size_t inner_stride, size_t len, uint8_t* d_hex, size_t hex_outer,
                  uint64_t* ticket);
/* cec_hashq_add where chain i also emits the hex of its first prefix_len bytes (a nonzero
 * multiple of 64, <= len) to d_prefix_hex + ((i / per) * prefix_hex_outer + i % per) * 64.
 * The segment's chain thus yields data fragment 0's hash on the way (the split is contiguous,
 * fragment 0 = the segment's first F bytes): 32 instead of 40 MiB hashed per CESS segment.
 * Both outputs are final once the add is complete. d_prefix_hex NULL = cec_hashq_add. */
int cec_hashq_add_prefix(cec_hashq* q, const uint8_t* d_base, size_t n, size_t per,
                         size_t outer_stride, size_t inner_stride, size_t len, uint8_t* d_hex,
                         size_t hex_outer, size_t prefix_len, uint8_t* d_prefix_hex,
                         size_t prefix_hex_outer, uint64_t* ticket);
/* cec_hashq_add of chains that resume after their first start_len bytes (a multiple of 64 within
 * len's full blocks): chain i starts from the SHA-256 state d_states[8 i .. 8 i + 7] (memory
 * the device reads: device memory or pinned host memory, read by the add's kernel on the queue's
 * stream; the eight 32-bit words after start_len bytes, as cec_sha256_host_state gives them)
 * and hashes bytes start_len .. len of its buffer. A segment chain continued on the GPU after
 * the host hashed its fragment 0. */
int cec_hashq_add_resume(cec_hashq* q, const uint8_t* d_base, size_t n, size_t per,
                         size_t outer_stride, size_t inner_stride, size_t len, size_t start_len,
                         const uint32_t* d_states, uint8_t* d_hex, size_t hex_outer,
                         uint64_t* ticket);
/* Advance every live chain by at most max_blocks 64-byte blocks (0 = to completion). */
int cec_hashq_tick(cec_hashq* q, uint32_t max_blocks);
/* Tick until every chain added so far is complete (enqueued; synchronise the stream to wait). */
int cec_hashq_finish(cec_hashq* q);
/* Host-side status as of the ticks enqueued so far: *done = add `ticket` complete, *live_chains
 * = chains not yet complete, *blocks_left = most blocks any live chain still needs. Any output
 * pointer may be NULL. */
int cec_hashq_status(const cec_hashq* q, uint64_t ticket, int* done, size_t* live_chains,
                     uint64_t* blocks_left);
/* Queue options. CEC_HQOPT_TICK: tick kernel, 0 = auto by live chains, 1 or 2 = two waves
 * (schedule producer loading 1 or 2 blocks ahead + rounds consumer), 3 = one wave per 64 chains,
 * 4 = lane pairs (a producer wave + two consumer waves running each chain's rounds on two lanes:
 * the shortest chain latency, for few live chains). */
#define CEC_HQOPT_TICK 1
int cec_hashq_set_option(cec_hashq* q, int option, int value);

/* klauspost Split for one segment (host memory): shard i = seg[i*shard_len, (i+1)*shard_len),
 * zero-padded past seg_len. Requires k*shard_len >= seg_len > 0. */
int cec_split_segment(const uint8_t* seg, size_t seg_len, int k, uint8_t* const* shards,
                      size_t shard_len);

/* ---- host pipeline: files in host memory through the GPU ------------------------------------
 * The north_star's pinned hipMemcpyAsync multi-buffering behind the C ABI. A pipeline owns a
 * ring of `depth` pinned host batches and device slots for one codec; a run streams sources
 * through it batch by batch: read() fills a pinned batch (the file's next bytes; the last
 * segment is zero-padded, klauspost Split), H2D on a copy stream, cec_encode_batch on a compute
 * stream, parity D2H on a third stream, so reading batch i+1 overlaps the copies and kernels of
 * batch i and H2D overlaps D2H. The SegmentList hashes (segment hash and the k+m fragment
 * hashes, SHA-256 hex, c-pallets/file-bank/src/types.rs:13-16) are computed where `hash` says:
 *   CEC_PIPE_HASH_GPU     on the GPU by a hash queue that keeps `window` batches hashing at once
 *                         (device slots = window + 3);
 *   CEC_PIPE_HASH_HOST    on `host_threads` host threads (cec_sha256_host) from the pinned ring;
 *   CEC_PIPE_HASH_HYBRID  the segment chains (fragment 0's digest on the way) on the host, the
 *                         other fragments' chains on the GPU queue, except for the last batches
 *                         of the run's last source, which the host hashes wholly (`tail_batches`;
 *                         -1 = auto: the batches whose GPU chains would finish after the source's
 *                         remaining bytes have landed; needs the source's size). Below 12
 *                         host_threads (or with CEC_PIPELINE_RESUME=1; =0 turns it off) the host
 *                         hashes only fragment 0 and the GPU queue resumes the segment chain
 *                         from its state (cec_hashq_add_resume): half the host's bytes.
 * The pipeline is reusable: keep one for many files (its pinned ring is pinned once).
 *   read(user, dst, cap): write up to cap source bytes at dst; return the count, 0 at the end,
 *     < 0 to abort (CEC_ECALLBACK).
 *   on_fragments(user, seg, shards, shard_len): the k+m shards of segment `seg`, host memory
 *     valid during the call; in segment order, as soon as the batch's parity is back.
 *   on_record(user, seg, seg_hex, frag_hex): the segment's 64 hex chars and its k+m fragment
 *     hashes (k+m)*64 hex chars, fragment index order; in segment order.
 * Callbacks run on the calling thread and return 0 (nonzero aborts with CEC_ECALLBACK). */
#define CEC_PIPE_HASH_NONE 0
#define CEC_PIPE_HASH_GPU 1
#define CEC_PIPE_HASH_HOST 2
#define CEC_PIPE_HASH_HYBRID 3
typedef long long (*cec_read_fn)(void* user, uint8_t* dst, size_t cap);
typedef int (*cec_fragments_fn)(void* user, uint64_t seg, const uint8_t* const* shards,
                                size_t shard_len);
typedef int (*cec_record_fn)(void* user, uint64_t seg, const uint8_t* seg_hex,
                             const uint8_t* frag_hex);
typedef struct cec_pipeline_opts {
  size_t shard_len;      /* F: a segment is k * F bytes */
  size_t batch_segments; /* segments per full batch (0: 64); a run's first three batches are
                            1/8, 1/4, 1/2 of it and the last source's last ones halve down to
                            1/8 when its size is known (B >= 8; the records do not change) */
  int depth;             /* pinned host batches (0: 3, host / hybrid hashing 4; >= 2) */
  int hash;              /* CEC_PIPE_HASH_*: 0 none, 1 GPU, 2 host, 3 hybrid */
  int window;            /* batches hashing at once on the GPU queue (0: 32); the pipeline
                            holds window + 3 device batch slots (1.5 GiB each for CESS batches)
                            and shrinks the window to what free HBM holds */
  uint64_t max_segments; /* 0: no limit; else CEC_ESEGCOUNT when a source has more segments
                            (CEC_SEGMENT_COUNT: what one upload_declaration can carry) */
  int host_threads;      /* host SHA-256 threads for hash = 2 / 3 (0: 16) */
  int tail_batches;      /* hash = 3: batches at the end of the last source hashed wholly on
                            the host (-1: auto, 0: none) */
} cec_pipeline_opts;
typedef struct cec_pipeline_stats {
  uint64_t segments;   /* segments encoded */
  uint64_t bytes_in;   /* source bytes read */
  double seconds;      /* wall time of the run (per file: from its first read to its on_done) */
  double read_seconds; /* time inside read() */
  double wait_seconds; /* host time blocked on the GPU or the host hashers */
} cec_pipeline_stats;
typedef struct cec_pipeline cec_pipeline;
int cec_pipeline_create(cec_codec* codec, const cec_pipeline_opts* opts, cec_pipeline** out);
/* Waits for the pipeline's own streams and host hash jobs, then frees its pinned host ring and
 * device slots. The HIP runtime's hipHostFree / hipFree synchronise the whole device, so other
 * codecs' work on this GPU stalls until it is done: destroy a pipeline while the device is idle,
 * or keep it (a pipeline is reusable, one run per file or per list of files). */
void cec_pipeline_destroy(cec_pipeline* p);
/* The window the pipeline settled on (after fitting its slots into free HBM), its device batch
 * slots and pinned host batches. Any output may be NULL. */
int cec_pipeline_info(const cec_pipeline* p, int* window, int* device_slots, int* depth);
/* Stream one source through the pipeline (reusable: run again for the next file). */
int cec_pipeline_run(cec_pipeline* p, cec_read_fn read, cec_fragments_fn on_fragments,
                     cec_record_fn on_record, void* user, cec_pipeline_stats* stats);
/* Several sources (files) in one run, back to back: batches never mix files, segment numbers
 * count from 0 per file, each file's records come in segment order and its on_done once its
 * last record is out, in file order, while the next files already stream (the hashing of one
 * file's last batches overlaps the next file's copies). size: the source's bytes, 0 = unknown
 * (needed only for the hybrid placement of the last batches). stats: the whole run. */
typedef struct cec_source {
  cec_read_fn read;
  void* user; /* passed to read */
  uint64_t size;
} cec_source;
typedef int (*cec_file_fragments_fn)(void* user, size_t file, uint64_t seg,
                                     const uint8_t* const* shards, size_t shard_len);
typedef int (*cec_file_record_fn)(void* user, size_t file, uint64_t seg, const uint8_t* seg_hex,
                                  const uint8_t* frag_hex);
typedef int (*cec_file_done_fn)(void* user, size_t file, const cec_pipeline_stats* file_stats);
int cec_pipeline_run_files(cec_pipeline* p, const cec_source* sources, size_t nsources,
                           cec_file_fragments_fn on_fragments, cec_file_record_fn on_record,
                           cec_file_done_fn on_done, void* user, cec_pipeline_stats* stats);

/* ---- storage audit chunks ---------------------------------------------
 * A fragment is CHUNK_COUNT = 1024 chunks (primitives/common/src/lib.rs:62): 8 KiB chunks of an
 * 8 MiB fragment. A challenge names need = CHUNK_COUNT * 46 / 1000 = 47 distinct chunk indices
 * (NetSnapShot.random_index_list, c-pallets/audit/src/types.rs:21), drawn by
 * c-pallets/audit/src/lib.rs:955-964 from the chain's randomness: for seed = 1, 2, ...,
 * index = random_number(seed) % CHUNK_COUNT, repeats skipped. The PoDR2 tag arithmetic over the
 * chunks runs in the TEE and is not in the reference (unpinned, not provided). */
#define CEC_CHUNK_COUNT 1024
#define CEC_CHALLENGE_NEED (CEC_CHUNK_COUNT * 46 / 1000)
/* The selection loop over a given random stream: randoms[i] = random_number(seed i + 1) (the
 * chain's randomness, decoded as u64). Writes `need` indices; *used = randoms consumed.
 * CEC_EINVAL when the stream runs out first. Host only. */
int cec_challenge_indices(const uint64_t* randoms, size_t nrand, uint32_t chunk_count,
                          uint32_t need, uint32_t* out, size_t* used);
/* Gather chunks indices[0..nidx) of every fragment of an HBM batch ([nseg][k][shard_len] data,
 * [nseg][m][shard_len] parity; d_parity NULL: data fragments only) into d_chunks
 * [nfrag][nidx][chunk] (fragments in batch order, seg * (k+m) + shard), chunk = shard_len /
 * chunk_count, and/or the SHA-256 hex of each gathered chunk into d_hex [nfrag][nidx][64].
 * Either output may be NULL (not both). Enqueued on hip_stream. */
int cec_audit_chunks(cec_codec* codec, const uint8_t* d_data, const uint8_t* d_parity,
                     size_t nseg, size_t shard_len, uint32_t chunk_count,
                     const uint32_t* indices, uint32_t nidx, uint8_t* d_chunks, uint8_t* d_hex,
                     void* hip_stream);

/* ---- multi-GPU degraded read over RCCL ----------------------------------------
 * One process (or thread) per GPU, each with its own codec. Fragment f of segment s is stored on
 * rank (s + f) mod world, the GPU analogue of the chain's miner placement (random_assign_miner,
 * c-pallets/file-bank/src/functions.rs:187-283: a segment's fragments on distinct miners). A
 * degraded read brings the k survivors (cec_survivors) of every segment with lost fragments to
 * the rank that owns the segment's first lost fragment (repair restores a fragment where it
 * lives, restoral_order_complete, c-pallets/file-bank/src/lib.rs:1075-1122) by RCCL point-to-
 * point over xGMI, and rebuilds the lost fragments there. RCCL is loaded at run time; without it
 * these return CEC_ENCCL. This is the C form of cess_amd.distributed.degraded_read. */
#define CEC_DIST_ID_BYTES 128
typedef struct cec_dist cec_dist;
/* A fresh group id (on one rank; hand it to the others out of band, e.g. the host's control
 * plane). */
int cec_dist_unique_id(uint8_t* id /* CEC_DIST_ID_BYTES */);
/* Join the group as `rank` of `world` on the codec's device. Collective: every rank calls it
 * with the same id. The group keeps using `codec` until cec_dist_destroy. */
int cec_dist_create(cec_codec* codec, const uint8_t* id, int world, int rank, cec_dist** out);
/* Leave the group and free the handle. The handle's own teardown waits for its last degraded
 * read only, but RCCL's ncclCommDestroy, which it calls, drains the WHOLE device: every stream of
 * every codec on this GPU stalls until its queued work is done (measured: a 25 ms batch on an
 * unrelated stream finished inside the destroy, profiles/r04/destroy_report_c.log). Destroy dist
 * handles only when the device is idle (at shutdown, or between batches), never mid-traffic. */
void cec_dist_destroy(cec_dist* d);
/* One transfer of a plan. kind CEC_DIST_SURVIVOR: fragment `frag` of segment `seg` from rank src
 * to rank dst (src == dst: already local). kind CEC_DIST_PARTIAL: rank src's partial rebuild of
 * lost fragment `frag` (from the survivors src holds, cec_reconstruct_partial_batch) to the
 * decoder dst, which XORs the partials. */
#define CEC_DIST_SURVIVOR 0
#define CEC_DIST_PARTIAL 1
typedef struct cec_dist_move {
  uint64_t seg;
  int32_t frag, src, dst;
  int32_t kind;
} cec_dist_move;
/* Exchange of a degraded read (cec_dist_set_option CEC_DIST_OPT_EXCHANGE, cec_dist_plan_ex):
 * 0 = survivors (the k survivors travel to the decoder), 1 = partials (every other rank holding
 * survivors sends one partial per lost fragment), 2 = per segment whichever moves fewer
 * fragments, survivors on a tie (the default of a new group; RS(2,1) over >= 3 GPUs always ties;
 * a wide code spread over many GPUs with few erasures: RS(32,32) on 8 GPUs, one lost fragment,
 * 7 partials instead of 27-28 survivors). */
#define CEC_DIST_OPT_EXCHANGE 1
/* Test hook: value r >= 0 makes the next degraded reads fail inside round r's transfer group, as
 * an RCCL error there would (the group is ended and the communicator aborted, so peers get an
 * error instead of waiting; later calls on the handle return CEC_ENCCL). -1 = off (default). */
#define CEC_DIST_OPT_TEST_ABORT 2
/* At most `value` point-to-point transfers on any one rank per RCCL group (default 1024; 0 = one
 * group per round of 256 segments, up to ~7k transfers for RS(32,32)). A round is cut into groups
 * at the same plan positions on every rank, so every group holds both ends of its transfers; the
 * groups are enqueued back to back with no host synchronisation. */
#define CEC_DIST_OPT_GROUP_OPS 3
int cec_dist_set_option(cec_dist* d, int option, int value);
/* Transfer groups this handle has issued (diagnostic: the group split of CEC_DIST_OPT_GROUP_OPS). */
int cec_dist_groups(const cec_dist* d, uint64_t* groups);
/* Host only: the transfer groups a degraded read of the lost list issues with `group_ops`
 * (CEC_DIST_OPT_GROUP_OPS) and `exchange`: *ngroups of them, and the plan position (index of the
 * segment in ascending segment order) where each starts, written to starts (NULL: count only;
 * CEC_EINVAL if more than starts_cap). A round of 256 segments always starts a group. */
int cec_dist_plan_groups(int k, int m, int world, int exchange, int group_ops,
                         const uint64_t* lost_seg, const uint8_t* lost_frag, size_t nlost,
                         uint64_t* starts, size_t starts_cap, size_t* ngroups);
/* Host only: the plan a degraded read of the lost list runs. The list holds nlost (segment,
 * fragment) erasures, any order, duplicates allowed, at most m distinct per segment
 * (CEC_ETOOFEW otherwise; CEC_EINVAL for an index >= k+m). Writes the moves in issue order
 * (*nmoves of them; CEC_EINVAL if more than moves_cap, moves may be NULL to count) and, per lost
 * entry, the rank that rebuilds it (decoder, may be NULL). cec_dist_plan = exchange 0. */
int cec_dist_plan(int k, int m, int world, const uint64_t* lost_seg, const uint8_t* lost_frag,
                  size_t nlost, cec_dist_move* moves, size_t moves_cap, size_t* nmoves,
                  int32_t* decoder);
int cec_dist_plan_ex(int k, int m, int world, int exchange, const uint64_t* lost_seg,
                     const uint8_t* lost_frag, size_t nlost, cec_dist_move* moves,
                     size_t moves_cap, size_t* nmoves, int32_t* decoder);
/* Device address (shard_len bytes) of fragment (seg, frag) held by this rank, NULL if absent. */
typedef const uint8_t* (*cec_locate_fn)(void* user, uint64_t seg, int frag);
/* Degraded read. Collective: every rank passes the same lost list. Rank r sends the survivors
 * the placement puts on it (found through `locate`) and writes every lost fragment it rebuilds,
 * entry i, to d_out[i] (device, shard_len bytes; entries other ranks rebuild are not touched and
 * may be NULL; d_out may be NULL on a rank that rebuilds nothing). Before any byte moves the
 * ranks agree that each found its survivors: a NULL from `locate` fails the call on every rank
 * with CEC_EINVAL. Work runs on hip_stream; returns when the rebuilt fragments are in d_out.
 * *nrebuilt (optional) = fragments written on this rank. */
int cec_dist_degraded_read(cec_dist* d, const uint64_t* lost_seg, const uint8_t* lost_frag,
                           size_t nlost, size_t shard_len, cec_locate_fn locate, void* user,
                           uint8_t* const* d_out, void* hip_stream, size_t* nrebuilt);

/* ---- on-chain records (host only, no GPU) ---------------------------------------------------
 * SCALE bytes of what the codec's outputs become on chain:
 *   FileBank::upload_declaration(file_hash: Hash, deal_info: BoundedVec<SegmentList,
 *     SegmentCount>, user_brief: UserBrief)          c-pallets/file-bank/src/lib.rs:419-428
 *   SegmentList { hash: Hash, fragment_list: BoundedVec<Hash, FragmentCount> }   types.rs:13-16
 *   UserBrief { user: AccountId32, file_name, bucket_name: BoundedVec<u8, 63> }  types.rs:105-109
 *   Hash([u8; 64]) (a fixed array: 64 bytes, no length prefix)  primitives/common/src/lib.rs:16
 * Hashes are passed as 64 lowercase hex characters each. Every function writes at most out_cap
 * bytes to `out` and sets *out_len to the encoded size; out == NULL only sizes the encoding. */
#define CEC_SEGMENT_COUNT 1000 /* runtime/src/lib.rs:1026 (SegmentCount) */
#define CEC_FRAGMENT_COUNT 3   /* runtime/src/lib.rs:1027 (FragmentCount) */
#define CEC_NAME_MIN 3         /* runtime/src/lib.rs:1051 (NameMinLength) */
#define CEC_NAME_MAX 63        /* runtime/src/lib.rs:1041 (NameStrLimit) */
#define CEC_FILEBANK_PALLET 60 /* runtime/src/lib.rs:1532 */
#define CEC_CALL_UPLOAD_DECLARATION 0 /* c-pallets/file-bank/src/lib.rs:420 call_index(0) */
/* SCALE compact encoding of n. */
int cec_scale_compact(uint32_t n, uint8_t* out, size_t out_cap, size_t* out_len);
/* deal_info = compact(nseg) ++ per segment: hash ++ compact(nfrag) ++ nfrag hashes.
 * seg_hex: nseg * 64 bytes; frag_hex: nseg * nfrag * 64 (fragment index order).
 * CEC_ESEGCOUNT if nseg > CEC_SEGMENT_COUNT (the extrinsic would be rejected: split the file);
 * CEC_EINVAL if nfrag != CEC_FRAGMENT_COUNT (check_file_spec, c-pallets/file-bank/src/
 * functions.rs:4-11, rejects any other count with SpecError) or a hash is not lowercase hex. */
int cec_scale_deal_info(const uint8_t* seg_hex, const uint8_t* frag_hex, size_t nseg,
                        size_t nfrag, uint8_t* out, size_t out_cap, size_t* out_len);
/* Call data of upload_declaration: pallet index, call index, file_hash, deal_info, user_brief
 * (account: 32 bytes; names 3..63 bytes). */
int cec_scale_upload_declaration(const uint8_t* file_hash_hex, const uint8_t* seg_hex,
                                 const uint8_t* frag_hex, size_t nseg, size_t nfrag,
                                 const uint8_t* account, const uint8_t* file_name,
                                 size_t file_name_len, const uint8_t* bucket_name,
                                 size_t bucket_name_len, uint8_t* out, size_t out_cap,
                                 size_t* out_len);
/* Idle fillers: FileBank::upload_filler(tee_worker: AccountId, filler_list: Vec<FillerInfo>),
 * call_index(8) (c-pallets/file-bank/src/lib.rs:795-833); FillerInfo { block_num: u32,
 * miner_address: AccountId, filler_hash: Hash } (types.rs:82-86); at most UploadFillerLimit = 10
 * fillers per call (runtime/src/lib.rs:1033), each 8 MiB of idle space (lib.rs:821-825).
 * Call data for n fillers: block_num[n], miners n * 32 bytes, filler_hex n * 64 hex chars.
 * CEC_EINVAL past the limit (the chain's LengthExceedsLimit). */
#define CEC_CALL_UPLOAD_FILLER 8
#define CEC_UPLOAD_FILLER_LIMIT 10
#define CEC_FILLER_SIZE (8u << 20)
int cec_scale_upload_filler(const uint8_t* tee_worker, const uint32_t* block_num,
                            const uint8_t* miners, const uint8_t* filler_hex, size_t n,
                            uint8_t* out, size_t out_cap, size_t* out_len);
/* Restoral (repair) calls, c-pallets/file-bank/src/lib.rs:940-1122: a miner that lost a fragment
 * opens an order (13), another claims it (14; 15 for the fragments of an exiting miner,
 * RestoralTarget), rebuilds the fragment off chain and reports it (16). Hashes are 64 hex chars,
 * the miner an AccountId32. A repair service emits 16 only for a fragment whose rebuilt SHA-256
 * equals the recorded fragment hash. */
#define CEC_CALL_GENERATE_RESTORAL_ORDER 13
#define CEC_CALL_CLAIM_RESTORAL_ORDER 14
#define CEC_CALL_CLAIM_RESTORAL_EXIST_ORDER 15
#define CEC_CALL_RESTORAL_ORDER_COMPLETE 16
int cec_scale_generate_restoral_order(const uint8_t* file_hash_hex, const uint8_t* fragment_hex,
                                      uint8_t* out, size_t out_cap, size_t* out_len);
int cec_scale_claim_restoral_order(const uint8_t* fragment_hex, uint8_t* out, size_t out_cap,
                                   size_t* out_len);
int cec_scale_claim_restoral_exist_order(const uint8_t* miner, const uint8_t* file_hash_hex,
                                         const uint8_t* fragment_hex, uint8_t* out,
                                         size_t out_cap, size_t* out_len);
int cec_scale_restoral_order_complete(const uint8_t* fragment_hex, uint8_t* out, size_t out_cap,
                                      size_t* out_len);
/* Audit randomness inputs (c-pallets/audit/src/lib.rs:1067-1076): random_number(seed) asks the
 * chain's randomness for the subject (MyPalletId, seed).encode() = the 8 PalletId bytes ++ seed as
 * u32 LE (12 bytes; the audit pallet's id is SegbkPalletId = b"rewardpt", runtime/src/lib.rs:
 * 984,1004), and decodes the output's first 8 bytes as a little-endian u64. The randomness itself
 * (pallet_rrsc::ParentBlockRandomness) is chain state: a host holding it reproduces the inputs of
 * cec_challenge_indices with these two. */
#define CEC_AUDIT_PALLET_ID "rewardpt"
int cec_audit_random_subject(const uint8_t* pallet_id /* 8 bytes */, uint32_t seed,
                             uint8_t* out12);
int cec_audit_random_u64(const uint8_t* randomness, size_t len, uint64_t* out);
/* The challenge's random_list (NetSnapShot.random_list, c-pallets/audit/src/lib.rs:966-974): for
 * seed = now + 1, now + 2, ... (now = the block number), generate_challenge_random(seed)
 * (lib.rs:1079-1096) asks the randomness for the subject (MyPalletId, seed + 1) and keeps the first
 * 20 bytes of the H256 output; values already listed are skipped, until need = 47 values.
 * `randomness` holds nrand outputs of CEC_RANDOMNESS_BYTES each, output i being the chain's
 * randomness for cec_audit_random_subject(pallet, now + 2 + i) (a None output as 32 zero bytes,
 * the pallet's Default). Writes need * CEC_CHALLENGE_RANDOM_BYTES bytes to `out`; *used = outputs
 * consumed. CEC_EINVAL when the stream runs out first. Host only. */
#define CEC_RANDOMNESS_BYTES 32
#define CEC_CHALLENGE_RANDOM_BYTES 20
int cec_challenge_random_list(const uint8_t* randomness, size_t nrand, uint32_t need,
                              uint8_t* out, size_t* used);
/* 68-byte shard id = 64 hex chars ++ "-NNN" (index 0..999), the form Hash::from_shard_id reads
 * back (primitives/common/src/lib.rs:45-49; c-pallets/audit/src/tests.rs:267-269 builds
 * file_hash ++ "-001"). */
int cec_shard_id(const uint8_t* hash_hex, uint32_t index, uint8_t* out68);
/* Hash::from_shard_id: the first 64 bytes. */
int cec_hash_from_shard_id(const uint8_t* shard_id68, uint8_t* hash_hex_out);

/* Synthetic segments in HBM: little-endian 64-bit word w of segment s is
 * splitmix64(seed ^ ((seg0 + s) << 32) ^ w). seg_bytes must be a multiple of 8. */
int cec_fill_synthetic(uint8_t* d_out, size_t seg_bytes, size_t nseg, uint64_t seg0,
                       uint64_t seed, void* hip_stream);

/* Options, per codec (distinct codecs never affect each other). */
#define CEC_OPT_FORCE_GENERIC 1 /* 1: always use the run-time-coefficient kernel */
#define CEC_OPT_CT_VARIANT 2    /* compile-time kernel variant for tuning sweeps: -1 = default;
                                   other values need the tuning build (libcessec_tune.so) */
#define CEC_OPT_SHA_MODE 3      /* cec_sha256_batch kernel: 0 = auto, 1 = one wave per 64
                                   buffers, 2 = two waves (schedule producer + rounds consumer),
                                   3 = a producer + two consumer waves on lane pairs (the shortest
                                   chain latency; auto picks it for up to 341 x 64 buffers) */
#define CEC_OPT_RT_MODE 4       /* run-time-coefficient kernel: 0 = Horner over input groups
                                   with index-mode table XORs when 4 <= inputs <= 32, 1 = always
                                   the per-bit mask kernel, 2 = Horner with v_mov table reads */
#define CEC_OPT_DECODE_CACHE 6  /* capacity (>= 1) of the decode-program LRU cache, one entry
                                   per erasure pattern (default 4096) */
#define CEC_OPT_FFTDEC_MIN 7    /* RS(32,32): rebuilds of at least this many shards per segment
                                   may run the FFT-domain erasure decoder (0 = never; default 4) */
#define CEC_OPT_FFTDEC_MODE 8   /* RS(32,32), rebuilds past CEC_OPT_FFTDEC_MIN: 0 = the cheapest
                                   of the FFT-domain decoders (syndrome rows, formal derivative) and
                                   the run-time matrix kernel by the cost model (default), 1 = always
                                   the syndrome-row decoder, 2 = always the formal-derivative one */
int cec_set_option(cec_codec* codec, int option, int value);
/* Counters (tests / monitoring). */
#define CEC_STAT_DECODE_CACHED 1   /* erasure patterns in the decode cache */
#define CEC_STAT_RETIRED_PENDING 2 /* device blocks retired but possibly still read by queued
                                      kernels (released once those complete) */
#define CEC_STAT_POOL_BYTES 3      /* HBM held by the codec's block pool (programs, plans, small
                                      scratch); batch-sized scratch is stream-ordered and is not
                                      held after the call's launches complete */
#define CEC_STAT_FFTDEC_SEGMENTS 4 /* segments rebuilt by the RS(32,32) FFT-domain decoders so far
                                      (the rest of a rebuild ran the run-time matrix kernels) */
#define CEC_STAT_FFTDEC_D_SEGMENTS 5 /* of those, segments rebuilt by the formal-derivative decoder */
int cec_get_stat(const cec_codec* codec, int stat, uint64_t* value);

#ifdef __cplusplus
}
#endif

#endif /* CESS_EC_H */
