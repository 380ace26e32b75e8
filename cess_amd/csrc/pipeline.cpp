// libcessec host pipeline: files in host memory -> segments -> fragments (+ SegmentList hashes)
// through one GPU, with the pinned hipMemcpyAsync multi-buffering of the north_star. The records
// are `SegmentList { hash, fragment_list }` (c-pallets/file-bank/src/types.rs:13-16) for
// FileBank::upload_declaration (c-pallets/file-bank/src/lib.rs:423-499).
//
// Per batch of up to B segments of one file (segment = k * F bytes, the contiguous klauspost
// Split):
//   host:    read() fills pinned input slot hs = i % depth (zero-pads the file's last segment)
//   s_h2d:   waits until device slot ds = i % nd is free, copies the batch in
//   s_comp:  cec_encode_batch into the slot's parity
//   s_d2h:   copies parity into pinned parity slot hs
// and the hashes of the batch's records go where the pipeline's hash mode puts them:
//   GPU     every chain on the GPU hash queue (segment chain with data fragment 0 as its prefix
//           digest, the other fragments), added after the encode on s_comp and ticked once per
//           batch: `window` batches hash together and a batch's hex is final `window` ticks
//           after its add. Ticks share the compute stream with the encodes on purpose: three
//           streams fit the device's hardware queues (GPU_MAX_HW_QUEUES = 4, one taken by the
//           codec), and a fourth stream shared a queue with the parity copies, which held every
//           tick behind a 11 ms D2H (rocprof timeline, profiles/r02/).
//   HOST    every chain on host threads (sha256_host.cpp) straight from the pinned slots: the
//           segment chains (fragment 0 as prefix) and data fragments as soon as the batch is
//           read, the parity once its D2H is back.
//   HYBRID  the host takes the 16 MiB segment chains (one pass over the file's bytes, fragment
//           0's digest on the way); the GPU queue takes the 8 MiB chains of the other fragments
//           and parity, except for the last batches of the run's last source, whose chains the
//           host takes too: a GPU chain finishes ~blocks x 1.9 us after its batch lands (one
//           wave per chain), so chains added near the end would outlast the host's work.
// Reading batch i+1 on the host overlaps the copies and kernels of batch i, H2D overlaps D2H
// (PCIe is full duplex), and the hashing overlaps everything.
//
// A run takes a list of sources (files) and keeps the pipeline full across them: batches never
// mix files, the records of each file are delivered in segment order, and a file's on_done
// comes once its last record is out, while later files are already streaming.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "../../include/cess_ec.h"
#include "host_sha.h"
#include "kernels.h"

namespace cec {
int set_error(int code, const std::string& msg);
}

namespace {

#define PL_TRY(expr)                                                                        \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return cec::set_error(_e == hipErrorOutOfMemory ? CEC_ENOMEM : CEC_EHIP,              \
                            std::string(#expr) + ": " + hipGetErrorString(_e));             \
  } while (0)

#define PL_RC(expr)          \
  do {                       \
    int _rc = (expr);        \
    if (_rc) return _rc;     \
  } while (0)

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// GPU time of one 64-byte block of a lone chain (the lane-pair tick, DESIGN.md §4: 1.67-1.70 us
// measured; a little slack for the ticks' launch gaps). Used only to place a batch's chains.
constexpr double kGpuChainSecondsPerBlock = 1.8e-6;

}  // namespace

struct cec_pipeline {
  cec_codec* codec = nullptr;
  int k = 0, m = 0, device = 0;
  size_t F = 0, SB = 0, B = 0;  // shard bytes, segment bytes, segments per batch
  int depth = 0, nd = 0, window = 0;
  int mode = CEC_PIPE_HASH_NONE;
  int host_threads = 16, tail_batches = -1;
  bool threads_reserved = false;  // host_threads reserved in the host SHA pool
  uint64_t max_segments = 0;
  // pinned host ring
  std::vector<uint8_t*> h_in, h_par;
  // device slots
  std::vector<uint8_t*> d_data, d_par, d_shex, d_fhex;
  std::vector<uint8_t*> h_shex, h_fhex;  // pinned hex, per device slot
  hipStream_t s_h2d = nullptr, s_comp = nullptr, s_d2h = nullptr;
  std::vector<hipEvent_t> ev_h2d, ev_enc, ev_d2h, ev_hex;  // per device slot
  // hybrid resume (per device slot): the host hashes fragment 0 of each segment and hands its
  // chain state to the GPU queue, which continues the segment chain over fragments 1..k-1
  std::vector<uint32_t*> h_state;    // pinned, read by the add kernel in place
  std::vector<hipEvent_t> ev_state;  // after that add (h_state reusable once complete)
  std::vector<bool> state_pending;
  bool resume = false;
  cec_hashq* hq = nullptr;
  uint32_t tick_blocks = 0;
  // host hash jobs not yet known to be finished (they read the pinned ring)
  std::vector<std::shared_ptr<hsha::JobState>> host_jobs;

  bool gpu_hash() const { return mode == CEC_PIPE_HASH_GPU || mode == CEC_PIPE_HASH_HYBRID; }
  bool host_hash() const { return mode == CEC_PIPE_HASH_HOST || mode == CEC_PIPE_HASH_HYBRID; }
  // first fragment index a hybrid batch leaves to the GPU: the host's segment chain yields
  // fragment 0 as its prefix digest when F is a multiple of 64; otherwise the host hashes the
  // data fragments and the GPU only the parity
  int hybrid_gpu_first() const { return F % 64 == 0 ? 1 : k; }

  struct Batch {
    uint64_t idx = 0, seg_base = 0, ticket = 0;
    size_t file = 0, nseg = 0;
    int hs = 0, ds = 0;
    bool frags_done = false, hex_copied = false;
    bool gpu = false;         // some chains on the GPU hash queue (hex copied out of slot ds)
    bool gpu_seg = false;     // the segment chain too (GPU mode)
    bool host_frags = false;  // the host hashes every fragment chain of the batch
    bool seg_resume = false;  // hybrid: fragment 0 on the host, the segment chain resumed on the GPU
    bool resume_added = false;
    std::shared_ptr<hsha::JobState> j_seg, j_data, j_par;
    std::vector<const uint8_t*> p_seg, p_data, p_par;
    std::vector<uint8_t> shex, fhex;  // host-hashed records [nseg][64], [nseg][k+m][64]
  };

  void wait_host_jobs() {
    for (auto& j : host_jobs) hsha::wait(j, false);
    host_jobs.clear();
  }

  ~cec_pipeline() {
    (void)hipSetDevice(device);
    for (hipStream_t s : {s_h2d, s_comp, s_d2h})
      if (s) (void)hipStreamSynchronize(s);
    wait_host_jobs();
    if (threads_reserved) hsha::release_threads(host_threads);
    if (hq) cec_hashq_destroy(hq);
    for (auto* v : {&h_in, &h_par, &h_shex, &h_fhex})
      for (uint8_t* p : *v)
        if (p) (void)hipHostFree(p);
    for (uint32_t* p : h_state)
      if (p) (void)hipHostFree(p);
    for (hipEvent_t e : ev_state)
      if (e) (void)hipEventDestroy(e);
    for (auto* v : {&d_data, &d_par, &d_shex, &d_fhex})
      for (uint8_t* p : *v)
        if (p) (void)hipFree(p);
    for (auto* v : {&ev_h2d, &ev_enc, &ev_d2h, &ev_hex})
      for (hipEvent_t e : *v)
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t s : {s_h2d, s_comp, s_d2h})
      if (s) (void)hipStreamDestroy(s);
  }

  int init(const cec_pipeline_opts& o) {
    PL_RC(cec_codec_info(codec, &k, &m, &device));
    if (o.shard_len == 0) return cec::set_error(CEC_ESHARDLEN, "zero shard length");
    if (o.hash < CEC_PIPE_HASH_NONE || o.hash > CEC_PIPE_HASH_HYBRID)
      return cec::set_error(CEC_EINVAL, "hash must be 0 (none), 1 (GPU), 2 (host), 3 (hybrid)");
    F = o.shard_len;
    SB = (size_t)k * F;
    B = o.batch_segments ? o.batch_segments : 64;
    mode = o.hash;
    // host hashing holds a pinned batch until its chains are hashed (a 16 MiB chain in one of 16
    // AVX-512 lanes takes ~50 ms), so the host placements keep one batch more in the ring
    depth = o.depth ? o.depth : (host_hash() ? 4 : 3);
    if (depth < 2) return cec::set_error(CEC_EINVAL, "depth must be >= 2");
    // Ticks share the compute stream's hardware queue and, as the round-robin falls, the parity
    // copies' too (rocprof timeline, profiles/r06/): a batch then costs its D2H plus its tick
    // there, so the tick (blocks / window x ~1.7 us) must stay well under a batch's interval
    window = o.window ? o.window : 32;
    if (window < 1) return cec::set_error(CEC_EINVAL, "window must be >= 1");
    host_threads = o.host_threads > 0 ? o.host_threads : 16;
    if (host_hash()) {  // the pool holds every live pipeline's threads (one per GPU in a process)
      hsha::reserve_threads(host_threads);
      threads_reserved = true;
    }
    tail_batches = o.tail_batches;
    max_segments = o.max_segments;
    PL_TRY(hipSetDevice(device));
    // a slot is reused nd batches later; with GPU hashing its hashes are final `window` ticks
    // after its add, and two more slots keep the H2D of a reused slot from waiting on the tick
    // just enqueued. The window shrinks to what free HBM holds (one CESS slot is
    // ~1.5 GiB, so 35 slots are ~52 GiB, and several pipelines may share a GPU).
    const size_t slot_bytes = B * SB + B * (size_t)m * F + (gpu_hash() ? B * (k + m + 1) * 64 : 0);
    size_t free_b = 0, total_b = 0;
    PL_TRY(hipMemGetInfo(&free_b, &total_b));
    const size_t budget = (size_t)(0.85 * (double)free_b);
    if (gpu_hash()) {
      const size_t fit = slot_bytes ? budget / slot_bytes : 0;
      if (fit < 4)
        return cec::set_error(CEC_ENOMEM, "pipeline: free HBM holds fewer than 4 batch slots");
      window = std::min<int>(window, (int)std::min<size_t>(fit - 3, 1 << 20));
    }
    nd = gpu_hash() ? window + 3 : 3;
    // a device slot's events are re-recorded by its next batch: that batch (i + nd) must come
    // after the slot's previous batch has delivered its fragments, which the host ring guarantees
    // only for batches `depth` apart (with depth > nd the wait for an old batch's parity copy
    // became a wait for the newest one, and the ring ran one batch deep: 27-33 GB/s at depth 4
    // against 49-52 at depth 3, profiles/r05/e2e_sweep.jsonl)
    nd = std::max(nd, depth);
    if ((size_t)nd * slot_bytes > budget)
      return cec::set_error(CEC_ENOMEM, "pipeline: the device slots do not fit in free HBM");
    for (hipStream_t* s : {&s_h2d, &s_comp, &s_d2h})
      PL_TRY(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
    h_in.assign(depth, nullptr);
    h_par.assign(depth, nullptr);
    for (int i = 0; i < depth; ++i) {
      PL_TRY(hipHostMalloc(&h_in[i], B * SB, hipHostMallocDefault));
      PL_TRY(hipHostMalloc(&h_par[i], B * m * F, hipHostMallocDefault));
    }
    d_data.assign(nd, nullptr);
    d_par.assign(nd, nullptr);
    for (auto* v : {&ev_h2d, &ev_enc, &ev_d2h, &ev_hex}) v->assign(nd, nullptr);
    for (int i = 0; i < nd; ++i) {
      PL_TRY(hipMalloc(&d_data[i], B * SB));
      PL_TRY(hipMalloc(&d_par[i], B * m * F));
      for (auto* v : {&ev_h2d, &ev_enc, &ev_d2h, &ev_hex})
        PL_TRY(hipEventCreateWithFlags(&(*v)[i], hipEventDisableTiming));
    }
    if (gpu_hash()) {
      d_shex.assign(nd, nullptr);
      d_fhex.assign(nd, nullptr);
      h_shex.assign(nd, nullptr);
      h_fhex.assign(nd, nullptr);
      for (int i = 0; i < nd; ++i) {
        PL_TRY(hipMalloc(&d_shex[i], B * 64));
        PL_TRY(hipMalloc(&d_fhex[i], B * (k + m) * 64));
        PL_TRY(hipHostMalloc(&h_shex[i], B * 64, hipHostMallocDefault));
        PL_TRY(hipHostMalloc(&h_fhex[i], B * (k + m) * 64, hipHostMallocDefault));
      }
      // hybrid resume: needs fragment 0 on a block boundary. It halves the host's hashing on
      // hybrid batches (fragment 0 instead of the whole segment). With the host's 16 threads
      // (~78 GB/s of hashing, ~1x the file's bytes to hash) the stream is PCIe-bound either way
      // and resume did not pay in the bench's process; with fewer threads the host is the
      // bound and resume lifts the stream (8 threads: 38.6 vs 35.2 GB/s, 6: 36.6 vs 28.5,
      // profiles/r06/resume_threads/). So it is on below 12 threads: 12 hash ~59 GB/s at the
      // ~4.9 GB/s per thread measured, above the ~50 GB/s PCIe stream. CEC_PIPELINE_RESUME=1 / 0
      // forces it on / off.
      const char* rv = getenv("CEC_PIPELINE_RESUME");
      const bool want_resume = rv ? rv[0] != '0' : host_threads < 12;
      resume = mode == CEC_PIPE_HASH_HYBRID && F % 64 == 0 && k > 1 && want_resume;
      if (resume) {
        h_state.assign(nd, nullptr);
        ev_state.assign(nd, nullptr);
        state_pending.assign(nd, false);
        for (int i = 0; i < nd; ++i) {
          PL_TRY(hipHostMalloc(&h_state[i], B * 32, hipHostMallocDefault));
          PL_TRY(hipEventCreateWithFlags(&ev_state[i], hipEventDisableTiming));
        }
      }
      size_t chains = (size_t)(window + 1) * B * (k + m + 1), cap = 1024;
      while (cap < chains) cap <<= 1;
      PL_RC(cec_hashq_create(device, cap, s_comp, &hq));
      // GPU mode's longest chain is the segment's, hybrid's a fragment's
      const uint64_t blocks = cec::sha256_blocks(mode == CEC_PIPE_HASH_GPU ? SB : F);
      // resumed segment chains join the queue when their fragment-0 host job is done, a batch
      // or more after the batch's other chains: leave them a few ticks of slack, or the device
      // slot's reuse (window + 3 batches later) ticks synchronously until they end
      const uint64_t ticks = resume ? std::max(1, window - 4) : window;
      tick_blocks = (uint32_t)((blocks + ticks - 1) / ticks);
    }
    return CEC_OK;
  }

  // GPU chains of a batch and one tick. GPU mode: the segment chain with fragment 0 as its
  // prefix digest when F is a multiple of 64, the other data fragments, the parity. Hybrid: the
  // fragments from hybrid_gpu_first() on (the host has the segment chain).
  int add_gpu_hashes(Batch& b) {
    const int n = k + m;
    uint8_t* dd = d_data[b.ds];
    uint8_t* fh = d_fhex[b.ds];
    uint64_t t = 0;
    if (mode == CEC_PIPE_HASH_GPU) {
      if (F % 64 == 0) {
        PL_RC(cec_hashq_add_prefix(hq, dd, b.nseg, 1, SB, SB, SB, d_shex[b.ds], 1, F, fh, n, &t));
        if (k > 1)
          PL_RC(cec_hashq_add(hq, dd + F, b.nseg * (k - 1), k - 1, SB, F, F, fh + 64, n,
                              nullptr));
      } else {
        PL_RC(cec_hashq_add(hq, dd, b.nseg, 1, SB, SB, SB, d_shex[b.ds], 1, &t));
        PL_RC(cec_hashq_add(hq, dd, b.nseg * k, k, SB, F, F, fh, n, nullptr));
      }
      PL_RC(cec_hashq_add(hq, d_par[b.ds], b.nseg * m, m, (size_t)m * F, F, F, fh + 64 * k, n,
                          nullptr));
    } else {
      const int g0 = hybrid_gpu_first();
      if (g0 < k)
        PL_RC(cec_hashq_add(hq, dd + (size_t)g0 * F, b.nseg * (k - g0), k - g0, SB, F, F,
                            fh + 64 * g0, n, nullptr));
      // equal lengths: the last add completes last
      PL_RC(cec_hashq_add(hq, d_par[b.ds], b.nseg * m, m, (size_t)m * F, F, F, fh + 64 * k, n,
                          &t));
    }
    b.ticket = t;
    return cec_hashq_tick(hq, tick_blocks);
  }

  // The resumed segment chains of a hybrid batch, once its fragment-0 host job is done: the
  // states to the device, then the chains (from byte F of each segment, into the slot's segment
  // hex), on the queue's stream. Their add is the batch's last, so its ticket.
  int add_resume(Batch& b, bool block) {
    if (!b.seg_resume || b.resume_added) return CEC_OK;
    if (!hsha::ready(b.j_seg)) {
      if (!block) return CEC_OK;
      hsha::wait(b.j_seg, true);
    }
    // the add kernel reads the states straight from the pinned host slot (no copy on the
    // compute stream, where a small H2D would queue behind the batches' large copies)
    uint64_t t = 0;
    PL_RC(cec_hashq_add_resume(hq, d_data[b.ds], b.nseg, 1, SB, SB, SB, F, h_state[b.ds],
                               d_shex[b.ds], 1, &t));
    PL_TRY(hipEventRecord(ev_state[b.ds], s_comp));  // h_state[ds] reusable once read
    state_pending[b.ds] = true;
    b.ticket = t;
    b.resume_added = true;
    return CEC_OK;
  }

  bool hashed(const Batch& b) {
    if (b.seg_resume && !b.resume_added) return false;
    int done = 0;
    (void)cec_hashq_status(hq, b.ticket, &done, nullptr, nullptr);
    return done != 0;
  }

  // Tick until the batch's chains are complete, then copy its hex out (on the compute stream).
  int copy_hex(Batch& b) {
    PL_RC(add_resume(b, true));
    while (!hashed(b)) PL_RC(cec_hashq_tick(hq, tick_blocks));
    if (b.gpu_seg || b.seg_resume)
      PL_TRY(hipMemcpyAsync(h_shex[b.ds], d_shex[b.ds], b.nseg * 64, hipMemcpyDeviceToHost,
                            s_comp));
    PL_TRY(hipMemcpyAsync(h_fhex[b.ds], d_fhex[b.ds], b.nseg * (k + m) * 64,
                          hipMemcpyDeviceToHost, s_comp));
    PL_TRY(hipEventRecord(ev_hex[b.ds], s_comp));
    b.hex_copied = true;
    return CEC_OK;
  }

  std::shared_ptr<hsha::JobState> host_job(std::vector<const uint8_t*>& ptrs, size_t len,
                                           uint8_t* hex, size_t per, size_t hex_outer,
                                           size_t prefix_len, uint8_t* prefix_hex,
                                           size_t prefix_outer, uint32_t* state_out = nullptr) {
    hsha::Job j;
    j.state_out = state_out;
    j.bufs = ptrs.data();
    j.n = ptrs.size();
    j.len = len;
    j.hex = hex;
    j.per = per;
    j.hex_outer = hex_outer;
    j.prefix_len = prefix_len;
    j.prefix_hex = prefix_hex;
    j.prefix_outer = prefix_outer;
    auto js = hsha::submit(j, host_threads);
    host_jobs.push_back(js);
    return js;
  }

  // Host chains of a freshly read batch: the segment chains (fragment 0 as prefix when F is a
  // multiple of 64) and, when the host takes the batch's fragments, the data fragments.
  void submit_host_data(Batch& b) {
    const int n = k + m;
    const uint8_t* base = h_in[b.hs];
    b.shex.assign(b.nseg * 64, 0);
    b.fhex.assign(b.nseg * n * 64, 0);
    const bool prefix = F % 64 == 0;
    b.p_seg.resize(b.nseg);
    for (size_t s = 0; s < b.nseg; ++s) b.p_seg[s] = base + s * SB;
    if (b.seg_resume) {
      // fragment 0 only: its hex, and the chain state the GPU resumes the segment chain from
      // (the slot's previous states must have been copied to the device first)
      if (state_pending[b.ds]) (void)hipEventSynchronize(ev_state[b.ds]);
      state_pending[b.ds] = false;
      b.j_seg = host_job(b.p_seg, F, b.fhex.data(), 1, n, 0, nullptr, 1, h_state[b.ds]);
    } else {
      b.j_seg = host_job(b.p_seg, SB, b.shex.data(), 1, 1, prefix ? F : 0,
                         prefix ? b.fhex.data() : nullptr, n);
    }
    // data fragments the host hashes on their own chains: 1..k-1 with the prefix trick (0..k-1
    // without), for batches whose fragments are all on the host or, without the prefix trick,
    // hybrid batches too (their GPU part is the parity alone)
    const int d0 = prefix ? 1 : 0;
    if (d0 < k && (b.host_frags || (!prefix && mode == CEC_PIPE_HASH_HYBRID))) {
      b.p_data.resize(b.nseg * (k - d0));
      for (size_t s = 0; s < b.nseg; ++s)
        for (int j = d0; j < k; ++j) b.p_data[s * (k - d0) + (j - d0)] = base + s * SB + j * F;
      b.j_data = host_job(b.p_data, F, b.fhex.data() + 64 * d0, (size_t)(k - d0), n, 0,
                          nullptr, 1);
    }
  }

  // Host chains of the parity (its D2H complete).
  void submit_host_parity(Batch& b) {
    if (!b.host_frags || b.j_par) return;
    const int n = k + m;
    b.p_par.resize(b.nseg * m);
    for (size_t s = 0; s < b.nseg; ++s)
      for (int j = 0; j < m; ++j) b.p_par[s * m + j] = h_par[b.hs] + (s * m + j) * F;
    b.j_par = host_job(b.p_par, F, b.fhex.data() + 64 * k, (size_t)m, n, 0, nullptr, 1);
  }

  static bool job_ready(const std::shared_ptr<hsha::JobState>& j) { return !j || hsha::ready(j); }
  bool host_ready(const Batch& b) const {
    return job_ready(b.j_seg) && job_ready(b.j_data) && job_ready(b.j_par);
  }
  void host_wait(Batch& b) {
    for (auto* j : {&b.j_seg, &b.j_data, &b.j_par})
      if (*j) hsha::wait(*j, true);
  }
  // forget finished jobs (the list only guards the pinned ring at teardown)
  void prune_jobs() {
    host_jobs.erase(std::remove_if(host_jobs.begin(), host_jobs.end(),
                                   [](const std::shared_ptr<hsha::JobState>& j) {
                                     return hsha::ready(j);
                                   }),
                    host_jobs.end());
  }
};

namespace {

struct FileState {
  uint64_t segments = 0, bytes = 0, batches_open = 0;
  bool ended = false;
  double t0 = 0, t_read = 0;
};

}  // namespace

extern "C" {

int cec_pipeline_create(cec_codec* codec, const cec_pipeline_opts* opts, cec_pipeline** out) {
  if (!codec || !opts || !out) return cec::set_error(CEC_EINVAL, "null");
  *out = nullptr;
  auto* p = new (std::nothrow) cec_pipeline;
  if (!p) return cec::set_error(CEC_ENOMEM, "pipeline");
  p->codec = codec;
  int rc = p->init(*opts);
  if (rc) {
    delete p;
    return rc;
  }
  *out = p;
  return CEC_OK;
}

void cec_pipeline_destroy(cec_pipeline* p) { delete p; }

int cec_pipeline_info(const cec_pipeline* p, int* window, int* device_slots, int* depth) {
  if (!p) return cec::set_error(CEC_EINVAL, "null pipeline");
  if (window) *window = p->window;
  if (device_slots) *device_slots = p->nd;
  if (depth) *depth = p->depth;
  return CEC_OK;
}

int cec_pipeline_run_files(cec_pipeline* p, const cec_source* srcs, size_t nsrc,
                           cec_file_fragments_fn on_fragments, cec_file_record_fn on_record,
                           cec_file_done_fn on_done, void* user, cec_pipeline_stats* stats) {
  if (!p || (nsrc && !srcs)) return cec::set_error(CEC_EINVAL, "null pipeline or sources");
  for (size_t f = 0; f < nsrc; ++f)
    if (!srcs[f].read) return cec::set_error(CEC_EINVAL, "null read callback");
  if (on_record && p->mode == CEC_PIPE_HASH_NONE)
    return cec::set_error(CEC_EINVAL, "on_record needs hashing (hash != 0)");
  PL_TRY(hipSetDevice(p->device));
  // start clean after an aborted run: no queued copies, no live chains of the old batches, no
  // host jobs reading the ring
  if (p->hq) PL_RC(cec_hashq_finish(p->hq));
  for (hipStream_t s : {p->s_h2d, p->s_comp, p->s_d2h})
    if (s) PL_TRY(hipStreamSynchronize(s));
  p->wait_host_jobs();
  const double t0 = now_s();
  const hsha::PoolStats ps0 = hsha::stats();
  double t_read = 0, t_wait = 0;
  double w_d2h = 0, w_slot = 0, w_rec = 0;  // (CEC_PIPELINE_TRACE) where the waits went
  const int n = p->k + p->m;
  using Batch = cec_pipeline::Batch;
  std::deque<Batch> inflight;  // batch order; popped once fully delivered
  // Host jobs read the batches' pointer arrays and write their hex vectors: however the run
  // ends (an error or a callback's abort returns early), they finish before `inflight` goes.
  struct JobsGuard {
    cec_pipeline* p;
    ~JobsGuard() { p->wait_host_jobs(); }
  } jobs_guard{p};
  std::vector<FileState> files(nsrc);
  uint64_t bytes_in = 0, segs_total = 0, i = 0;
  size_t cur = 0;  // source being read
  if (nsrc) files[0].t0 = t0;
  // per-batch wall time of the source reads so far (hybrid placement of the last batches)
  double sec_per_byte = 1.0 / 45e9, last_batch_t = t0;
  // Batch sizes. A full batch is B segments; the run's first batches ramp up (B/8, B/4, B/2:
  // the first copy, encode and host hashes start after a short read instead of a whole batch),
  // and the last source's last 2B segments, when its size is known, go in halves down to B/8 (the
  // last parity copy and hashes drain after a short batch). The records do not depend on it.
  const bool ramp = p->B >= 8 && !getenv("CEC_PIPELINE_NO_RAMP");
  auto batch_bytes = [&](uint64_t idx, size_t src, uint64_t src_read) -> size_t {
    size_t segs = p->B;
    if (ramp && idx < 3) segs = p->B >> (3 - idx);
    if (ramp && src + 1 == nsrc && srcs[src].size > src_read) {
      const uint64_t left = (srcs[src].size - src_read + p->SB - 1) / p->SB;
      if (left <= 2 * p->B) {  // halves of what is left, none under B/8
        uint64_t want = std::max<uint64_t>(p->B / 8, (left + 1) / 2);
        if (left - want < p->B / 8 && left <= p->B) want = left;
        segs = std::min<size_t>(segs, (size_t)want);
      }
    }
    return segs * p->SB;
  };
  const double gpu_chain_s =
      (double)cec::sha256_blocks(p->F) * kGpuChainSecondsPerBlock;
  std::vector<uint8_t> rec(64 * (size_t)n);

  // on_done of every finished file, in file order (an empty file ends before the one in front
  // of it has delivered its records)
  size_t next_done = 0;
  auto files_done = [&]() -> int {
    while (next_done < nsrc && files[next_done].ended && !files[next_done].batches_open) {
      const FileState& fs = files[next_done];
      if (on_done) {
        cec_pipeline_stats st{fs.segments, fs.bytes, now_s() - fs.t0, fs.t_read, 0.0};
        if (on_done(user, next_done, &st))
          return cec::set_error(CEC_ECALLBACK, "on_done returned an error");
      }
      ++next_done;
    }
    return CEC_OK;
  };
  // on_fragments of batch b (its parity D2H complete); shards straight from the pinned slots
  auto deliver_frags = [&](Batch& b) -> int {
    const double w = now_s();
    PL_TRY(hipEventSynchronize(p->ev_d2h[b.ds]));  // (a later reuse of the slot only waits more)
    t_wait += now_s() - w;
    w_d2h += now_s() - w;
    p->submit_host_parity(b);
    if (on_fragments) {
      const uint8_t* sh[256];
      for (size_t s = 0; s < b.nseg; ++s) {
        for (int j = 0; j < p->k; ++j) sh[j] = p->h_in[b.hs] + s * p->SB + (size_t)j * p->F;
        for (int j = 0; j < p->m; ++j)
          sh[p->k + j] = p->h_par[b.hs] + (s * p->m + j) * p->F;
        if (on_fragments(user, b.file, b.seg_base + s, sh, p->F))
          return cec::set_error(CEC_ECALLBACK, "on_fragments returned an error");
      }
    }
    b.frags_done = true;
    return CEC_OK;
  };
  auto frags_through = [&](uint64_t idx) -> int {
    for (auto& o : inflight)
      if (o.idx <= idx && !o.frags_done) PL_RC(deliver_frags(o));
    return CEC_OK;
  };
  // host slot of batch idx + depth: every reader of the slot (fragment delivery, host chains)
  // of the batches up to idx is finished
  auto host_through = [&](uint64_t idx) -> int {
    PL_RC(frags_through(idx));
    for (auto& o : inflight)
      if (o.idx <= idx && !p->host_ready(o)) {
        const double w = now_s();
        p->host_wait(o);
        t_wait += now_s() - w;
        w_slot += now_s() - w;
      }
    return CEC_OK;
  };
  // Pop (delivering on_record) every batch up to idx; the hex copies of those are enqueued.
  std::function<int(uint64_t)> records_through;
  // Enqueue hex copies of every GPU-hashed batch up to idx. A copy lands in its device slot's
  // pinned hex buffer, so the slot's previous batch (idx - nd) must have delivered its records.
  auto hex_through = [&](uint64_t idx) -> int {
    while (true) {
      Batch* o = nullptr;
      for (auto& x : inflight)
        if (!x.hex_copied) {
          o = &x;
          break;
        }
      if (!o || o->idx > idx) return CEC_OK;
      // pops only batches before *o (deque: references to the others stay valid)
      if (o->idx >= (uint64_t)p->nd) PL_RC(records_through(o->idx - p->nd));
      PL_RC(p->copy_hex(*o));
    }
  };
  records_through = [&](uint64_t idx) -> int {
    while (!inflight.empty() && inflight.front().idx <= idx) {
      auto& b = inflight.front();
      if (!b.frags_done) PL_RC(deliver_frags(b));
      const double w = now_s();
      if (b.gpu) {
        if (!b.hex_copied) PL_RC(p->copy_hex(b));  // its slot's previous batch is popped
        PL_TRY(hipEventSynchronize(p->ev_hex[b.ds]));
      }
      p->host_wait(b);
      t_wait += now_s() - w;
      w_rec += now_s() - w;
      if (on_record && p->mode != CEC_PIPE_HASH_NONE) {
        const int g0 = b.gpu ? (b.gpu_seg ? 0 : p->hybrid_gpu_first()) : n;
        for (size_t s = 0; s < b.nseg; ++s) {
          const uint8_t* sh = b.gpu_seg || b.seg_resume ? p->h_shex[b.ds] + s * 64
                                                        : b.shex.data() + s * 64;
          for (int f = 0; f < n; ++f) {
            const uint8_t* src = f >= g0 ? p->h_fhex[b.ds] + (s * n + f) * 64
                                         : b.fhex.data() + (s * n + f) * 64;
            std::memcpy(rec.data() + 64 * f, src, 64);
          }
          if (on_record(user, b.file, b.seg_base + s, sh, rec.data()))
            return cec::set_error(CEC_ECALLBACK, "on_record returned an error");
        }
      }
      const size_t f = b.file;
      inflight.pop_front();
      files[f].batches_open--;
      PL_RC(files_done());
    }
    return CEC_OK;
  };
  auto record_ready = [&](const Batch& b) -> bool {
    if (!b.frags_done) return false;
    if (b.gpu && (!b.hex_copied || hipEventQuery(p->ev_hex[b.ds]) != hipSuccess)) return false;
    return p->host_ready(b);
  };

  while (cur < nsrc) {
    const int hs = (int)(i % p->depth);
    const int ds = (int)(i % p->nd);
    // host slot hs: the batch that used it must be done with it
    if (i >= (uint64_t)p->depth) PL_RC(host_through(i - p->depth));
    // read the next batch of the current source into pinned memory (overlaps the GPU work)
    uint8_t* dst = p->h_in[hs];
    const size_t cap = batch_bytes(i, cur, files[cur].bytes);
    size_t got = 0;
    const double r0 = now_s();
    while (got < cap) {
      const long long r = srcs[cur].read(srcs[cur].user, dst + got, cap - got);
      if (r < 0) return cec::set_error(CEC_ECALLBACK, "read returned an error");
      if (r == 0) break;
      got += (size_t)r;
    }
    const double dr = now_s() - r0;
    t_read += dr;
    files[cur].t_read += dr;
    if (got == 0) {  // source `cur` has ended: the next batch belongs to the next one
      files[cur].ended = true;
      PL_RC(files_done());
      if (++cur < nsrc) files[cur].t0 = now_s();
      continue;
    }
    FileState& fs = files[cur];
    bytes_in += got;
    const size_t nseg = (got + p->SB - 1) / p->SB;
    if (got < nseg * p->SB) std::memset(dst + got, 0, nseg * p->SB - got);  // zero-pad (Split)
    if (p->max_segments && fs.segments + nseg > p->max_segments)
      return cec::set_error(CEC_ESEGCOUNT, "source exceeds max_segments segments");
    // where this batch's fragment chains go
    bool host_frags = p->mode == CEC_PIPE_HASH_HOST;
    if (p->mode == CEC_PIPE_HASH_HYBRID && cur + 1 == nsrc && srcs[cur].size) {
      const uint64_t size = srcs[cur].size, after = fs.bytes + got;
      const uint64_t left_bytes = size > after ? size - after : 0;
      const uint64_t full = p->B * p->SB;
      if (p->tail_batches >= 0)  // full batches after this one
        host_frags = (left_bytes + full - 1) / full < (uint64_t)p->tail_batches;
      else  // auto: the GPU's chains would finish after the source's remaining bytes land
        host_frags = (double)(left_bytes + got) * sec_per_byte < gpu_chain_s;
    }
    if (i >= (uint64_t)p->nd) {
      // device slot ds: its previous batch's parity read out and (hashing) its hex copied out
      if (p->gpu_hash()) PL_RC(hex_through(i - p->nd));
      PL_TRY(hipStreamWaitEvent(p->s_h2d, p->ev_d2h[ds], 0));
      if (p->gpu_hash()) PL_TRY(hipStreamWaitEvent(p->s_h2d, p->ev_hex[ds], 0));
    }
    inflight.emplace_back();
    Batch& b = inflight.back();
    b.idx = i;
    b.file = cur;
    b.seg_base = fs.segments;
    b.nseg = nseg;
    b.hs = hs;
    b.ds = ds;
    b.host_frags = host_frags;
    b.gpu = p->mode == CEC_PIPE_HASH_GPU || (p->mode == CEC_PIPE_HASH_HYBRID && !host_frags);
    b.gpu_seg = p->mode == CEC_PIPE_HASH_GPU;
    b.seg_resume = p->resume && b.gpu && !b.gpu_seg;
    b.hex_copied = !b.gpu;
    fs.segments += nseg;
    fs.bytes += got;
    fs.batches_open++;
    segs_total += nseg;
    if (p->host_hash()) p->submit_host_data(b);
    PL_TRY(hipMemcpyAsync(p->d_data[ds], dst, nseg * p->SB, hipMemcpyHostToDevice, p->s_h2d));
    PL_TRY(hipEventRecord(p->ev_h2d[ds], p->s_h2d));
    PL_TRY(hipStreamWaitEvent(p->s_comp, p->ev_h2d[ds], 0));
    PL_RC(cec_encode_batch(p->codec, p->d_data[ds], p->d_par[ds], nseg, p->F, p->s_comp));
    PL_TRY(hipEventRecord(p->ev_enc[ds], p->s_comp));
    PL_TRY(hipStreamWaitEvent(p->s_d2h, p->ev_enc[ds], 0));
    PL_TRY(hipMemcpyAsync(p->h_par[hs], p->d_par[ds], nseg * p->m * p->F, hipMemcpyDeviceToHost,
                          p->s_d2h));
    PL_TRY(hipEventRecord(p->ev_d2h[ds], p->s_d2h));
    if (b.gpu) {
      PL_RC(p->add_gpu_hashes(b));  // on s_comp, after the encode
    } else if (p->gpu_hash()) {
      // nothing of this batch on the queue: its slot is free for reuse after the encode, and
      // the queue still ticks for the chains of earlier batches
      PL_TRY(hipEventRecord(p->ev_hex[ds], p->s_comp));
      PL_RC(cec_hashq_tick(p->hq, p->tick_blocks));
    }
    // resumed segment chains of the batches whose fragment-0 host jobs are done
    if (p->resume)
      for (auto& o : inflight) PL_RC(p->add_resume(o, false));
    const double tb = now_s();
    sec_per_byte = 0.5 * sec_per_byte + 0.5 * (tb - last_batch_t) / (double)got;
    last_batch_t = tb;
    // deliver whatever has completed, without blocking (a slot's event re-recorded by a newer
    // batch completes later on the same stream, so a query of it is conservative)
    for (auto& o : inflight) {
      if (o.frags_done) continue;
      if (hipEventQuery(p->ev_d2h[o.ds]) != hipSuccess) break;
      PL_RC(deliver_frags(o));
    }
    if (p->gpu_hash()) {
      uint64_t ready = 0;
      bool any = false;
      for (auto& o : inflight) {
        if (o.hex_copied) continue;
        if (!p->hashed(o)) break;
        ready = o.idx;
        any = true;
      }
      if (any) PL_RC(hex_through(ready));
    }
    while (!inflight.empty() && record_ready(inflight.front()))
      PL_RC(records_through(inflight.front().idx));
    p->prune_jobs();
    ++i;
  }
  // drain
  if (p->resume)
    for (auto& o : inflight) PL_RC(p->add_resume(o, true));
  if (p->hq) PL_RC(cec_hashq_finish(p->hq));
  if (i) PL_RC(records_through(i - 1));
  for (hipStream_t s : {p->s_h2d, p->s_comp, p->s_d2h})
    if (s) PL_TRY(hipStreamSynchronize(s));
  p->wait_host_jobs();
  PL_RC(files_done());
  if (getenv("CEC_PIPELINE_TRACE")) {
    const hsha::PoolStats ps = hsha::stats();
    const double wall = now_s() - t0;
    const uint64_t xs = ps.x16_steps - ps0.x16_steps;
    fprintf(stderr, "cec_pipeline: %.4f s, read %.4f, wait %.4f (d2h %.4f, host slot %.4f, "
            "records %.4f), mode %d, window %d, depth %d, resume %d; host SHA workers busy %.3f s = %.2f of "
            "%d threads, x16 steps %llu at %.1f lanes, SHA-NI steps %llu, spilled %llu\n", wall,
            t_read, t_wait, w_d2h, w_slot, w_rec, p->mode, p->window, p->depth, (int)p->resume,
            ps.busy_s - ps0.busy_s, (ps.busy_s - ps0.busy_s) / (wall * p->host_threads),
            p->host_threads, (unsigned long long)xs,
            xs ? (double)(ps.x16_lane_steps - ps0.x16_lane_steps) / (double)xs : 0.0,
            (unsigned long long)(ps.ni_steps - ps0.ni_steps),
            (unsigned long long)(ps.spilled - ps0.spilled));
  }
  if (stats) {
    stats->segments = segs_total;
    stats->bytes_in = bytes_in;
    stats->seconds = now_s() - t0;
    stats->read_seconds = t_read;
    stats->wait_seconds = t_wait;
  }
  return CEC_OK;
}

namespace {
// cec_pipeline_run's callbacks over cec_pipeline_run_files with one source
struct OneSource {
  cec_fragments_fn fr;
  cec_record_fn rc;
  void* user;
};
int one_frag(void* u, size_t, uint64_t seg, const uint8_t* const* shards, size_t len) {
  auto* o = static_cast<OneSource*>(u);
  return o->fr(o->user, seg, shards, len);
}
int one_record(void* u, size_t, uint64_t seg, const uint8_t* seg_hex, const uint8_t* frag_hex) {
  auto* o = static_cast<OneSource*>(u);
  return o->rc(o->user, seg, seg_hex, frag_hex);
}
}  // namespace

int cec_pipeline_run(cec_pipeline* p, cec_read_fn read, cec_fragments_fn on_fragments,
                     cec_record_fn on_record, void* user, cec_pipeline_stats* stats) {
  if (!p || !read) return cec::set_error(CEC_EINVAL, "null pipeline or read callback");
  OneSource o{on_fragments, on_record, user};
  cec_source s{read, user, 0};
  return cec_pipeline_run_files(p, &s, 1, on_fragments ? one_frag : nullptr,
                                on_record ? one_record : nullptr, nullptr, &o, stats);
}

}  // extern "C"
