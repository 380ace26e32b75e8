// libcessec host pipeline: a file in host memory -> segments -> fragments (+ SegmentList hashes)
// through one GPU, with the pinned hipMemcpyAsync multi-buffering of the north_star.
//
// Per batch of up to B segments (segment = k * F bytes, the contiguous klauspost Split):
//   host:    read() fills pinned input slot hs = i % depth (zero-pads the last segment)
//   s_h2d:   waits until device slot ds = i % nd is free, copies the batch in
//   s_comp:  cec_encode_batch into the slot's parity
//   s_d2h:   copies parity into pinned parity slot hs
//   s_comp:  (hash = 1) then adds the batch's segment and fragment chains to the GPU hash queue
//            and ticks it once: `window` batches hash together and a batch's hex is final
//            `window` ticks after its add (cec_hashq_*); the hex is copied to pinned memory
//            there too. Ticks share the compute stream with the encodes on purpose: three
//            streams fit the device's hardware queues (GPU_MAX_HW_QUEUES = 4, one taken by the
//            codec), and a fourth stream shared a queue with the parity copies, which held every
//            tick behind a 11 ms D2H (rocprof timeline, profiles/r02/).
// and the host delivers on_fragments (shards straight from the pinned slots) and on_record (hex)
// in segment order. Reading batch i+1 on the host overlaps the copies and kernels of batch i,
// H2D overlaps D2H (PCIe is full duplex), and the hash queue overlaps everything.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <deque>
#include <functional>
#include <string>
#include <vector>

#include "../../include/cess_ec.h"
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

}  // namespace

struct cec_pipeline {
  cec_codec* codec = nullptr;
  int k = 0, m = 0, device = 0;
  size_t F = 0, SB = 0, B = 0;  // shard bytes, segment bytes, segments per batch
  int depth = 0, nd = 0, window = 0;
  bool hash = false;
  uint64_t max_segments = 0;
  // pinned host ring
  std::vector<uint8_t*> h_in, h_par;
  // device slots
  std::vector<uint8_t*> d_data, d_par, d_shex, d_fhex;
  std::vector<uint8_t*> h_shex, h_fhex;  // pinned hex, per device slot
  hipStream_t s_h2d = nullptr, s_comp = nullptr, s_d2h = nullptr;
  std::vector<hipEvent_t> ev_h2d, ev_enc, ev_d2h, ev_hex;  // per device slot
  cec_hashq* hq = nullptr;
  uint32_t tick_blocks = 0;

  struct Batch {
    uint64_t idx, seg_base, ticket = 0;
    size_t nseg;
    int hs, ds;
    bool frags_done = false, hex_copied = false;
  };

  ~cec_pipeline() {
    (void)hipSetDevice(device);
    for (hipStream_t s : {s_h2d, s_comp, s_d2h})
      if (s) (void)hipStreamSynchronize(s);
    if (hq) cec_hashq_destroy(hq);
    for (auto* v : {&h_in, &h_par, &h_shex, &h_fhex})
      for (uint8_t* p : *v)
        if (p) (void)hipHostFree(p);
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
    F = o.shard_len;
    SB = (size_t)k * F;
    B = o.batch_segments ? o.batch_segments : 64;
    depth = o.depth ? o.depth : 3;
    if (depth < 2) return cec::set_error(CEC_EINVAL, "depth must be >= 2");
    hash = o.hash != 0;
    window = o.window ? o.window : 32;
    if (window < 1) return cec::set_error(CEC_EINVAL, "window must be >= 1");
    max_segments = o.max_segments;
    // a slot is reused nd batches later; its hashes are final `window` ticks after its add, and
    // two more slots keep the H2D of a reused slot from waiting on the tick just enqueued
    nd = hash ? window + 3 : 3;
    // a device slot's events are re-recorded by its next batch: that batch (i + nd) must come
    // after the slot's previous batch has delivered its fragments, which the host ring guarantees
    // only for batches `depth` apart (with depth > nd the wait for an old batch's parity copy
    // became a wait for the newest one, and the ring ran one batch deep: 27-33 GB/s at depth 4
    // against 49-52 at depth 3, profiles/r05/e2e_sweep.jsonl)
    nd = std::max(nd, depth);
    PL_TRY(hipSetDevice(device));
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
    if (hash) {
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
      size_t chains = (size_t)(window + 1) * B * (k + m + 1), cap = 1024;
      while (cap < chains) cap <<= 1;
      PL_RC(cec_hashq_create(device, cap, s_comp, &hq));
      const uint64_t blocks = cec::sha256_blocks(SB);
      tick_blocks = (uint32_t)((blocks + window - 1) / window);
    }
    return CEC_OK;
  }

  // Enqueue the batch's hash chains (segment chain with fragment 0 as its prefix digest when F
  // is a multiple of 64, the other data fragments, the parity fragments) and one tick.
  int add_hashes(Batch& b) {
    const int n = k + m;
    uint8_t* dd = d_data[b.ds];
    uint8_t* fh = d_fhex[b.ds];
    uint64_t t = 0;
    if (F % 64 == 0) {
      PL_RC(cec_hashq_add_prefix(hq, dd, b.nseg, 1, SB, SB, SB, d_shex[b.ds], 1, F, fh, n, &t));
      if (k > 1)
        PL_RC(cec_hashq_add(hq, dd + F, b.nseg * (k - 1), k - 1, SB, F, F, fh + 64, n, nullptr));
    } else {
      PL_RC(cec_hashq_add(hq, dd, b.nseg, 1, SB, SB, SB, d_shex[b.ds], 1, &t));
      PL_RC(cec_hashq_add(hq, dd, b.nseg * k, k, SB, F, F, fh, n, nullptr));
    }
    PL_RC(cec_hashq_add(hq, d_par[b.ds], b.nseg * m, m, (size_t)m * F, F, F, fh + 64 * k, n,
                        nullptr));
    b.ticket = t;
    return cec_hashq_tick(hq, tick_blocks);
  }

  bool hashed(const Batch& b) {
    int done = 0;
    (void)cec_hashq_status(hq, b.ticket, &done, nullptr, nullptr);
    return done != 0;
  }

  // Tick until the batch's chains are complete, then copy its hex out (on the hash stream).
  int copy_hex(Batch& b) {
    while (!hashed(b)) PL_RC(cec_hashq_tick(hq, tick_blocks));
    PL_TRY(hipMemcpyAsync(h_shex[b.ds], d_shex[b.ds], b.nseg * 64, hipMemcpyDeviceToHost,
                          s_comp));
    PL_TRY(hipMemcpyAsync(h_fhex[b.ds], d_fhex[b.ds], b.nseg * (k + m) * 64,
                          hipMemcpyDeviceToHost, s_comp));
    PL_TRY(hipEventRecord(ev_hex[b.ds], s_comp));
    b.hex_copied = true;
    return CEC_OK;
  }
};

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

int cec_pipeline_run(cec_pipeline* p, cec_read_fn read, cec_fragments_fn on_fragments,
                     cec_record_fn on_record, void* user, cec_pipeline_stats* stats) {
  if (!p || !read) return cec::set_error(CEC_EINVAL, "null pipeline or read callback");
  if (on_record && !p->hash) return cec::set_error(CEC_EINVAL, "on_record needs hash = 1");
  PL_TRY(hipSetDevice(p->device));
  // start clean after an aborted run: no queued copies, no live chains of the old batches
  if (p->hash) PL_RC(cec_hashq_finish(p->hq));
  for (hipStream_t s : {p->s_h2d, p->s_comp, p->s_d2h})
    if (s) PL_TRY(hipStreamSynchronize(s));
  const double t0 = now_s();
  double t_read = 0, t_wait = 0;
  const int n = p->k + p->m;
  std::deque<cec_pipeline::Batch> inflight;  // batch order; popped once fully delivered
  uint64_t seg_base = 0, bytes_in = 0, i = 0;

  // on_fragments of batch b (its parity D2H complete); shards straight from the pinned slots
  auto deliver_frags = [&](cec_pipeline::Batch& b) -> int {
    const double w = now_s();
    PL_TRY(hipEventSynchronize(p->ev_d2h[b.ds]));  // (a later reuse of the slot only waits more)
    t_wait += now_s() - w;
    if (on_fragments) {
      const uint8_t* sh[256];
      for (size_t s = 0; s < b.nseg; ++s) {
        for (int j = 0; j < p->k; ++j) sh[j] = p->h_in[b.hs] + s * p->SB + (size_t)j * p->F;
        for (int j = 0; j < p->m; ++j)
          sh[p->k + j] = p->h_par[b.hs] + (s * p->m + j) * p->F;
        if (on_fragments(user, b.seg_base + s, sh, p->F))
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
  // Pop (delivering on_record) every batch up to idx; the hex copies of those are enqueued.
  std::function<int(uint64_t)> records_through;
  // Enqueue hex copies of every batch up to idx. A copy lands in its device slot's pinned hex
  // buffer, so the slot's previous batch (idx - nd) must have delivered its records first.
  auto hex_through = [&](uint64_t idx) -> int {
    while (true) {
      cec_pipeline::Batch* o = nullptr;
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
      if (p->hash) {
        if (!b.hex_copied) PL_RC(p->copy_hex(b));  // its slot's previous batch is popped
        const double w = now_s();
        PL_TRY(hipEventSynchronize(p->ev_hex[b.ds]));
        t_wait += now_s() - w;
        if (on_record)
          for (size_t s = 0; s < b.nseg; ++s)
            if (on_record(user, b.seg_base + s, p->h_shex[b.ds] + s * 64,
                          p->h_fhex[b.ds] + s * n * 64))
              return cec::set_error(CEC_ECALLBACK, "on_record returned an error");
      }
      inflight.pop_front();
    }
    return CEC_OK;
  };

  while (true) {
    const int hs = (int)(i % p->depth);
    const int ds = (int)(i % p->nd);
    // host slot hs: the batch that used it must have delivered its fragments
    if (i >= (uint64_t)p->depth) PL_RC(frags_through(i - p->depth));
    // read the next batch into pinned memory (overlaps the GPU work of earlier batches)
    uint8_t* dst = p->h_in[hs];
    const size_t cap = p->B * p->SB;
    size_t got = 0;
    const double r0 = now_s();
    while (got < cap) {
      const long long r = read(user, dst + got, cap - got);
      if (r < 0) return cec::set_error(CEC_ECALLBACK, "read returned an error");
      if (r == 0) break;
      got += (size_t)r;
    }
    t_read += now_s() - r0;
    if (got == 0) break;
    bytes_in += got;
    const size_t nseg = (got + p->SB - 1) / p->SB;
    if (got < nseg * p->SB) std::memset(dst + got, 0, nseg * p->SB - got);  // zero-pad (Split)
    if (p->max_segments && seg_base + nseg > p->max_segments)
      return cec::set_error(CEC_ESEGCOUNT, "source exceeds max_segments segments");
    if (i >= (uint64_t)p->nd) {
      // device slot ds: its previous batch's parity read out and (hashing) its hex copied out
      if (p->hash) PL_RC(hex_through(i - p->nd));
      PL_TRY(hipStreamWaitEvent(p->s_h2d, p->ev_d2h[ds], 0));
      if (p->hash) PL_TRY(hipStreamWaitEvent(p->s_h2d, p->ev_hex[ds], 0));
    }
    cec_pipeline::Batch b;
    b.idx = i;
    b.seg_base = seg_base;
    b.nseg = nseg;
    b.hs = hs;
    b.ds = ds;
    PL_TRY(hipMemcpyAsync(p->d_data[ds], dst, nseg * p->SB, hipMemcpyHostToDevice, p->s_h2d));
    PL_TRY(hipEventRecord(p->ev_h2d[ds], p->s_h2d));
    PL_TRY(hipStreamWaitEvent(p->s_comp, p->ev_h2d[ds], 0));
    PL_RC(cec_encode_batch(p->codec, p->d_data[ds], p->d_par[ds], nseg, p->F, p->s_comp));
    PL_TRY(hipEventRecord(p->ev_enc[ds], p->s_comp));
    PL_TRY(hipStreamWaitEvent(p->s_d2h, p->ev_enc[ds], 0));
    PL_TRY(hipMemcpyAsync(p->h_par[hs], p->d_par[ds], nseg * p->m * p->F, hipMemcpyDeviceToHost,
                          p->s_d2h));
    PL_TRY(hipEventRecord(p->ev_d2h[ds], p->s_d2h));
    if (p->hash) PL_RC(p->add_hashes(b));  // on s_comp, after the encode
    inflight.push_back(b);
    // deliver whatever has completed, without blocking (a slot's event re-recorded by a newer
    // batch completes later on the same stream, so a query of it is conservative)
    for (auto& o : inflight) {
      if (o.frags_done) continue;
      if (hipEventQuery(p->ev_d2h[o.ds]) != hipSuccess) break;
      PL_RC(deliver_frags(o));
    }
    if (p->hash) {
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
    while (!inflight.empty()) {
      auto& f = inflight.front();
      if (!f.frags_done) break;
      if (p->hash && (!f.hex_copied || hipEventQuery(p->ev_hex[f.ds]) != hipSuccess)) break;
      PL_RC(records_through(f.idx));
    }
    seg_base += nseg;
    ++i;
  }
  // drain
  if (p->hash) PL_RC(cec_hashq_finish(p->hq));
  if (i) PL_RC(records_through(i - 1));
  for (hipStream_t s : {p->s_h2d, p->s_comp, p->s_d2h})
    if (s) PL_TRY(hipStreamSynchronize(s));
  if (stats) {
    stats->segments = seg_base;
    stats->bytes_in = bytes_in;
    stats->seconds = now_s() - t0;
    stats->read_seconds = t_read;
    stats->wait_seconds = t_wait;
  }
  return CEC_OK;
}

}  // extern "C"
