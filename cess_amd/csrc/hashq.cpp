// libcessec hash queue: streaming SHA-256 of many long device buffers (the fragment and segment
// hashes of SegmentList, c-pallets/file-bank/src/types.rs:13-16).
//
// A fragment's SHA-256 is one serial chain: on a GPU its rate is one wave's instruction issue
// (about 35 MB/s per chain), so throughput comes only from chains in flight. The queue keeps
// every chain's state in HBM (ShaChain, kernels.h) in a ring of slots; cec_hashq_add appends
// chains (one small kernel, no host->device copy), cec_hashq_tick advances every live chain by
// at most max_blocks blocks in one launch. A producer that adds a batch per step and ticks once
// per step therefore hashes a window of batches at once, and each batch's hex lands a known
// number of ticks later: completion is tracked on the host from the lengths alone, so nothing
// is read back.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <deque>
#include <string>

#include "../../include/cess_ec.h"
#include "kernels.h"

namespace cec {
int set_error(int code, const std::string& msg);
}

struct cec_hashq {
  int device = 0;
  hipStream_t stream = nullptr;
  cec::ShaChain* tab = nullptr;
  uint32_t cap = 0;
  uint64_t head = 0, tail = 0;  // absolute slot numbers; live slots are [head, tail)
  struct Add {
    uint64_t slot0, n, blocks, done, ticket;
  };
  std::deque<Add> adds;  // adds not yet complete, in slot order
  uint64_t next_ticket = 1;
  int tick_mode = 0;  // CEC_HQOPT_TICK
};

namespace {

#define HQ_TRY(expr)                                                                       \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return cec::set_error(_e == hipErrorOutOfMemory ? CEC_ENOMEM : CEC_EHIP,             \
                            std::string(#expr) + ": " + hipGetErrorString(_e));            \
  } while (0)

int launched() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return cec::set_error(CEC_EHIP, std::string("launch: ") + hipGetErrorString(e));
  return CEC_OK;
}

// Drop completed adds from the front so the tick range starts at the oldest live chain.
void retire(cec_hashq* q) {
  while (!q->adds.empty() && q->adds.front().done == q->adds.front().blocks) q->adds.pop_front();
  q->head = q->adds.empty() ? q->tail : q->adds.front().slot0;
}

}  // namespace

extern "C" {

int cec_hashq_create(int device, size_t capacity, void* hip_stream, cec_hashq** out) {
  if (!out) return cec::set_error(CEC_EINVAL, "null out");
  *out = nullptr;
  if (capacity == 0 || capacity > (1u << 31) || (capacity & (capacity - 1)))
    return cec::set_error(CEC_EINVAL, "capacity must be a power of two in [1, 2^31]");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return cec::set_error(CEC_ENODEV, "no HIP device");
  if (device < 0 || device >= ndev) return cec::set_error(CEC_EINVAL, "bad device");
  HQ_TRY(hipSetDevice(device));
  auto* q = new (std::nothrow) cec_hashq;
  if (!q) return cec::set_error(CEC_ENOMEM, "hashq");
  q->device = device;
  q->stream = reinterpret_cast<hipStream_t>(hip_stream);
  q->cap = (uint32_t)capacity;
  // stream-ordered (hipFree would synchronise the whole device at destroy): every use of the
  // table is a launch on q->stream
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&q->tab),
                                capacity * sizeof(cec::ShaChain), q->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(q->stream);
  if (e != hipSuccess) {
    delete q;
    return cec::set_error(CEC_ENOMEM, std::string("hashq table: ") + hipGetErrorString(e));
  }
  *out = q;
  return CEC_OK;
}

void cec_hashq_destroy(cec_hashq* q) {
  if (!q) return;
  (void)hipSetDevice(q->device);
  // freed in stream order, after the launches still queued on the stream that read the table
  (void)hipFreeAsync(q->tab, q->stream);
  delete q;
}

int cec_hashq_add_prefix(cec_hashq* q, const uint8_t* d_base, size_t n, size_t per,
                         size_t outer_stride, size_t inner_stride, size_t len, uint8_t* d_hex,
                         size_t hex_outer, size_t prefix_len, uint8_t* d_prefix_hex,
                         size_t prefix_hex_outer, uint64_t* ticket) {
  if (!q || (n && !d_base) || per == 0) return cec::set_error(CEC_EINVAL, "null or per == 0");
  if (n > 0xFFFFFFFFull) return cec::set_error(CEC_EINVAL, "n too large");
  if (d_prefix_hex && (prefix_len == 0 || (prefix_len & 63) || prefix_len > len))
    return cec::set_error(CEC_EINVAL, "prefix_len must be a nonzero multiple of 64 <= len");
  if (n == 0) {
    if (ticket) *ticket = 0;
    return CEC_OK;
  }
  if (q->tail + n - q->head > q->cap)
    return cec::set_error(CEC_ENOMEM, "hash queue full: tick until chains complete");
  HQ_TRY(hipSetDevice(q->device));
  cec::launch_hashq_add(q->tab, q->cap - 1, q->tail, (uint32_t)n, d_base, (uint32_t)per,
                        outer_stride, inner_stride, len, d_hex, hex_outer,
                        d_prefix_hex ? prefix_len >> 6 : 0, d_prefix_hex, prefix_hex_outer,
                        q->stream);
  int rc = launched();
  if (rc) return rc;
  // the prefix digest is written before the chain completes, so tracking the add by its full
  // length is conservative for it
  q->adds.push_back({q->tail, n, cec::sha256_blocks(len), 0, q->next_ticket});
  q->tail += n;
  if (ticket) *ticket = q->next_ticket;
  ++q->next_ticket;
  return CEC_OK;
}

int cec_hashq_add_resume(cec_hashq* q, const uint8_t* d_base, size_t n, size_t per,
                         size_t outer_stride, size_t inner_stride, size_t len, size_t start_len,
                         const uint32_t* d_states, uint8_t* d_hex, size_t hex_outer,
                         uint64_t* ticket) {
  if (!q || (n && (!d_base || !d_states)) || per == 0)
    return cec::set_error(CEC_EINVAL, "null or per == 0");
  if (n > 0xFFFFFFFFull) return cec::set_error(CEC_EINVAL, "n too large");
  if ((start_len & 63) || start_len > (len & ~(size_t)63))
    return cec::set_error(CEC_EINVAL, "start_len must be a multiple of 64 within len's full blocks");
  if (n == 0) {
    if (ticket) *ticket = 0;
    return CEC_OK;
  }
  if (q->tail + n - q->head > q->cap)
    return cec::set_error(CEC_ENOMEM, "hash queue full: tick until chains complete");
  HQ_TRY(hipSetDevice(q->device));
  cec::launch_hashq_add(q->tab, q->cap - 1, q->tail, (uint32_t)n, d_base, (uint32_t)per,
                        outer_stride, inner_stride, len, d_hex, hex_outer, 0, nullptr, 0,
                        q->stream, d_states, start_len >> 6);
  int rc = launched();
  if (rc) return rc;
  q->adds.push_back({q->tail, n, cec::sha256_blocks(len) - (start_len >> 6), 0, q->next_ticket});
  q->tail += n;
  if (ticket) *ticket = q->next_ticket;
  ++q->next_ticket;
  return CEC_OK;
}

int cec_hashq_add(cec_hashq* q, const uint8_t* d_base, size_t n, size_t per, size_t outer_stride,
                  size_t inner_stride, size_t len, uint8_t* d_hex, size_t hex_outer,
                  uint64_t* ticket) {
  return cec_hashq_add_prefix(q, d_base, n, per, outer_stride, inner_stride, len, d_hex,
                              hex_outer, 0, nullptr, 0, ticket);
}

int cec_hashq_tick(cec_hashq* q, uint32_t max_blocks) {
  if (!q) return cec::set_error(CEC_EINVAL, "null");
  if (q->adds.empty()) return CEC_OK;
  if (max_blocks == 0) {  // drain: enough blocks to complete every live chain
    uint64_t most = 0;
    for (const auto& a : q->adds) most = std::max(most, a.blocks - a.done);
    max_blocks = (uint32_t)std::min<uint64_t>(most, 0xFFFFFFFFull);
  }
  uint64_t live = 0;
  for (const auto& a : q->adds)
    if (a.done < a.blocks) live += a.n;
  HQ_TRY(hipSetDevice(q->device));
  cec::launch_sha256_tick(q->tick_mode, q->tab, q->cap - 1, q->head, (uint32_t)(q->tail - q->head), max_blocks,
                          live, q->stream);
  int rc = launched();
  if (rc) return rc;
  for (auto& a : q->adds) a.done += std::min<uint64_t>(max_blocks, a.blocks - a.done);
  retire(q);
  return CEC_OK;
}

int cec_hashq_finish(cec_hashq* q) {
  if (!q) return cec::set_error(CEC_EINVAL, "null");
  while (!q->adds.empty()) {
    int rc = cec_hashq_tick(q, 0);
    if (rc) return rc;
  }
  return CEC_OK;
}

int cec_hashq_status(const cec_hashq* q, uint64_t ticket, int* done, size_t* live_chains,
                     uint64_t* blocks_left) {
  if (!q) return cec::set_error(CEC_EINVAL, "null");
  if (done) {
    // an add is complete once it is no longer listed (tickets are increasing along the deque)
    *done = ticket < q->next_ticket ? 1 : 0;
    for (const auto& a : q->adds)
      if (a.ticket == ticket) *done = a.done == a.blocks;
  }
  uint64_t live = 0, left = 0;
  for (const auto& a : q->adds)
    if (a.done < a.blocks) {
      live += a.n;
      left = std::max(left, a.blocks - a.done);
    }
  if (live_chains) *live_chains = (size_t)live;
  if (blocks_left) *blocks_left = left;
  return CEC_OK;
}

int cec_hashq_set_option(cec_hashq* q, int option, int value) {
  if (!q) return cec::set_error(CEC_EINVAL, "null");
  if (option == CEC_HQOPT_TICK) {
    if (value < 0 || value > 4) return cec::set_error(CEC_EINVAL, "tick kernel must be 0..4");
    q->tick_mode = value;
    return CEC_OK;
  }
  return cec::set_error(CEC_EINVAL, "unknown hash queue option");
}

}  // extern "C"
