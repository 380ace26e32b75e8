// Test-only stand-in for librccl.so.1: the ten entry points libcessec's multi-GPU degraded read
// resolves at run time (cess_amd/csrc/dist.cpp, rccl()), implemented for ranks that are THREADS
// of one process, all on one GPU. It lets cec_dist_degraded_read run at world 2..8 on a one-GPU
// box, where real RCCL refuses two ranks on one device. Never shipped, never on the product path:
// tests/test_gpu_multi.py builds it into a temporary directory as librccl.so.1 and runs the C
// driver (tests/native/dist_world_n.c) with LD_LIBRARY_PATH pointing there.
//
// Semantics kept from NCCL (the ones dist.cpp relies on):
// - ncclCommInitRank is collective: it returns once every rank of the id has joined.
// - Point-to-point ops inside ncclGroupStart/End are matched per (src, dst) pair in issue order:
//   the n-th send from a to b pairs with the n-th receive on b from a; sizes must agree.
// - Stream order, no host synchronisation of the data: a send reads its buffer after everything
//   enqueued before the group on the sender's stream (an event the receiver's stream waits on),
//   the copy runs on the receiver's stream, and the sender's stream waits for the copy before
//   anything enqueued after the group (so the sender may overwrite the buffer afterwards).
// - ncclAllReduce (int32/int64/uint8/float, sum/min/max) outside a group, stream ordered (this
//   stand-in synchronises the stream on the host to read the operand).
// - ncclCommAbort: every rank still waiting in the group or a collective of that communicator
//   returns ncclRemoteError; later calls on the aborted group fail the same way.
// A group end waits on the host until every op of the group has a partner (the peers are threads
// in the same group round), bounded by CESS_STANDIN_TIMEOUT_S (default 60 s): a pairing bug in
// the caller becomes ncclSystemError with a message on stderr instead of a hang.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct SendOp {
  const void* buf = nullptr;
  size_t bytes = 0;
  hipEvent_t ready = nullptr;  // sender's stream position at the group end
  bool done = false;
  bool bad = false;            // size mismatch with the receive it paired with
  hipEvent_t copied = nullptr;  // receiver's stream after the copy
};

struct Shared {
  int world = 0;
  std::mutex mu;
  std::condition_variable cv;
  int joined = 0, refs = 0;
  bool aborted = false;
  // pending sends per (src, dst), oldest first
  std::map<std::pair<int, int>, std::deque<std::shared_ptr<SendOp>>> sends;
  // all-reduce rendezvous
  uint64_t gen = 0;
  int arrived = 0;
  std::vector<std::vector<uint8_t>> contrib;
  std::vector<uint8_t> result;
  // every event the group created (see release(): kept for the life of the process)
  std::vector<hipEvent_t> events;
};

std::mutex g_reg_mu;
std::map<std::string, std::shared_ptr<Shared>> g_reg;

double timeout_s() {
  const char* e = getenv("CESS_STANDIN_TIMEOUT_S");
  return e ? atof(e) : 60.0;
}

}  // namespace

struct ncclComm {
  std::shared_ptr<Shared> sh;
  std::string key;
  int rank = 0;
  int device = 0;
  bool released = false;
};

namespace {

struct Op {
  bool send;
  ncclComm_t comm;
  void* buf;
  size_t bytes;
  int peer;
  hipStream_t stream;
};

thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

hipEvent_t new_event(Shared& sh) {  // caller holds sh.mu
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  sh.events.push_back(e);
  return e;
}

// Wait on sh.cv until pred() or abort or the timeout; returns ncclSuccess, ncclRemoteError
// (aborted) or ncclSystemError (timed out).
template <class P>
ncclResult_t wait_for(std::unique_lock<std::mutex>& lk, Shared& sh, P pred, const char* what,
                      int rank) {
  const auto until = std::chrono::steady_clock::now() +
                     std::chrono::milliseconds((long long)(timeout_s() * 1000));
  while (!pred()) {
    if (sh.aborted) return ncclRemoteError;
    if (sh.cv.wait_until(lk, until) == std::cv_status::timeout && !pred()) {
      if (sh.aborted) return ncclRemoteError;
      fprintf(stderr, "rccl stand-in: rank %d timed out waiting in %s\n", rank, what);
      return ncclSystemError;
    }
  }
  return ncclSuccess;
}

// Run one group's point-to-point ops (all on one thread: the ops this rank issued).
ncclResult_t run_group(std::vector<Op>& ops) {
  if (ops.empty()) return ncclSuccess;
  // one communicator per group in this stand-in (dist.cpp issues a group per communicator)
  ncclComm_t comm = ops[0].comm;
  for (const Op& o : ops)
    if (o.comm != comm) return ncclInvalidUsage;
  Shared& sh = *comm->sh;
  const int me = comm->rank;
  std::vector<std::shared_ptr<SendOp>> my_sends;
  std::map<hipStream_t, hipEvent_t> ready;
  {
    std::unique_lock<std::mutex> lk(sh.mu);
    if (sh.aborted) return ncclRemoteError;
    // the sender's stream position: one event per stream the group's sends use
    for (const Op& o : ops)
      if (o.send && !ready.count(o.stream)) {
        hipEvent_t e = new_event(sh);
        if (!e || hipEventRecord(e, o.stream) != hipSuccess) return ncclUnhandledCudaError;
        ready[o.stream] = e;
      }
    for (const Op& o : ops) {
      if (!o.send) continue;
      auto s = std::make_shared<SendOp>();
      s->buf = o.buf;
      s->bytes = o.bytes;
      s->ready = ready[o.stream];
      sh.sends[{me, o.peer}].push_back(s);
      my_sends.push_back(s);
    }
    sh.cv.notify_all();
  }
  // receives in issue order: each takes the oldest unmatched send of its (peer, me) pair
  std::map<hipStream_t, std::vector<std::shared_ptr<SendOp>>> matched;
  ncclResult_t res = ncclSuccess;
  for (const Op& o : ops) {
    if (o.send) continue;
    std::shared_ptr<SendOp> s;
    {
      std::unique_lock<std::mutex> lk(sh.mu);
      auto& q = sh.sends[{o.peer, me}];
      res = wait_for(lk, sh, [&] { return !q.empty(); }, "a receive", me);
      if (res != ncclSuccess) break;
      s = q.front();
      q.pop_front();
    }
    if (s->bytes != o.bytes) {
      fprintf(stderr, "rccl stand-in: rank %d receives %zu bytes from rank %d, which sent %zu\n",
              me, o.bytes, o.peer, s->bytes);
      s->bad = true;
      res = ncclInvalidUsage;
    } else if (hipStreamWaitEvent(o.stream, s->ready, 0) != hipSuccess ||
               hipMemcpyAsync(o.buf, s->buf, o.bytes, hipMemcpyDeviceToDevice, o.stream) !=
                   hipSuccess) {
      res = ncclUnhandledCudaError;
    }
    matched[o.stream].push_back(s);
    if (res != ncclSuccess) break;
  }
  {
    std::unique_lock<std::mutex> lk(sh.mu);
    for (auto& [st, v] : matched) {
      hipEvent_t e = new_event(sh);
      const bool rec = e && hipEventRecord(e, st) == hipSuccess;
      for (auto& s : v) {
        s->copied = rec ? e : nullptr;
        s->done = true;
      }
      if (!rec && res == ncclSuccess) res = ncclUnhandledCudaError;
    }
    sh.cv.notify_all();
    if (res != ncclSuccess) return res;
    // every send of this group taken and copied; then this stream waits for the copies
    res = wait_for(lk, sh, [&] {
      for (auto& s : my_sends)
        if (!s->done) return false;
      return true;
    }, "a send", me);
    if (res != ncclSuccess) return res;
  }
  for (size_t i = 0, j = 0; i < ops.size(); ++i) {
    if (!ops[i].send) continue;
    const auto& s = my_sends[j++];
    if (s->bad) return ncclInvalidUsage;
    if (!s->copied || hipStreamWaitEvent(ops[i].stream, s->copied, 0) != hipSuccess)
      return ncclUnhandledCudaError;
  }
  return ncclSuccess;
}

ncclResult_t enqueue(bool send, const void* buf, size_t count, ncclDataType_t t, int peer,
                     ncclComm_t comm, hipStream_t st) {
  if (!comm || comm->released) return ncclInvalidArgument;
  const size_t ts = type_size(t);
  if (!ts || peer < 0 || peer >= comm->sh->world || peer == comm->rank) return ncclInvalidArgument;
  Op o{send, comm, const_cast<void*>(buf), count * ts, peer, st};
  if (t_depth > 0) {
    t_ops.push_back(o);
    return ncclSuccess;
  }
  std::vector<Op> one{o};
  return run_group(one);
}

void release(ncclComm_t comm) {
  std::shared_ptr<Shared> sh = comm->sh;
  {
    std::lock_guard<std::mutex> lk(sh->mu);
    // The group's events are not destroyed here: they were recorded on the ranks' streams, and
    // by the time the last rank leaves, the other ranks may have destroyed those streams (their
    // work complete). Synchronizing such an event can make HIP re-read its recording queue (a
    // SIGSEGV seen once in the world-8 case, profiles/r06/gpu_tests_check3.log), and a few
    // hundred events per test process are not worth the risk: they live until the process ends.
    --sh->refs;
  }
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find(comm->key);
  if (it != g_reg.end() && it->second == sh && sh->refs == 0) g_reg.erase(it);
}

}  // namespace

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (stand-in)";
    case ncclUnhandledCudaError: return "unhandled HIP error (stand-in)";
    case ncclSystemError: return "system error: a peer never paired (stand-in timeout)";
    case ncclInternalError: return "internal error (stand-in)";
    case ncclInvalidArgument: return "invalid argument (stand-in)";
    case ncclInvalidUsage: return "invalid usage (stand-in)";
    case ncclRemoteError: return "remote error: the communicator was aborted (stand-in)";
    default: return "unknown result (stand-in)";
  }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  static std::atomic<uint64_t> counter{0};
  if (!id) return ncclInvalidArgument;
  memset(id->internal, 0, sizeof id->internal);
  snprintf(id->internal, sizeof id->internal, "cess-rccl-standin:%d:%llu", (int)getpid(),
           (unsigned long long)counter.fetch_add(1));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  const std::string key(id.internal, strnlen(id.internal, sizeof id.internal));
  std::shared_ptr<Shared> sh;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto& slot = g_reg[key];
    if (!slot) {
      slot = std::make_shared<Shared>();
      slot->world = nranks;
      slot->contrib.resize(nranks);
    }
    sh = slot;
  }
  if (sh->world != nranks) return ncclInvalidUsage;
  auto* c = new ncclComm;
  c->sh = sh;
  c->key = key;
  c->rank = rank;
  (void)hipGetDevice(&c->device);
  std::unique_lock<std::mutex> lk(sh->mu);
  ++sh->joined;
  ++sh->refs;
  sh->cv.notify_all();
  ncclResult_t r = wait_for(lk, *sh, [&] { return sh->joined >= sh->world; }, "init", rank);
  if (r != ncclSuccess) {
    lk.unlock();
    release(c);
    delete c;
    return r;
  }
  *out = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  release(comm);
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  {
    std::lock_guard<std::mutex> lk(comm->sh->mu);
    comm->sh->aborted = true;
    comm->sh->cv.notify_all();
  }
  release(comm);
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  ++t_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_depth <= 0) return ncclInvalidUsage;
  if (--t_depth > 0) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(t_ops);
  return run_group(ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                      hipStream_t st) {
  return enqueue(true, buf, count, t, peer, comm, st);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                      hipStream_t st) {
  return enqueue(false, buf, count, t, peer, comm, st);
}

ncclResult_t ncclAllReduce(const void* sendbuf, void* recvbuf, size_t count, ncclDataType_t t,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t st) {
  if (!comm || comm->released) return ncclInvalidArgument;
  if (t_depth > 0) return ncclInvalidUsage;  // not needed by dist.cpp
  const size_t ts = type_size(t), bytes = count * ts;
  if (!ts || (op != ncclSum && op != ncclMin && op != ncclMax)) return ncclInvalidArgument;
  std::vector<uint8_t> mine(bytes);
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipMemcpy(mine.data(), sendbuf, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return ncclUnhandledCudaError;
  Shared& sh = *comm->sh;
  std::vector<uint8_t> out;
  {
    std::unique_lock<std::mutex> lk(sh.mu);
    if (sh.aborted) return ncclRemoteError;
    const uint64_t g = sh.gen;
    sh.contrib[comm->rank] = std::move(mine);
    if (++sh.arrived == sh.world) {
      sh.result = sh.contrib[0];
      for (int r = 1; r < sh.world; ++r) {
        if (sh.contrib[r].size() != bytes) return ncclInvalidUsage;
        for (size_t i = 0; i < count; ++i) {
          auto combine = [&](auto* a, const auto* b) {
            if (op == ncclSum) a[i] = a[i] + b[i];
            else if (op == ncclMin) a[i] = b[i] < a[i] ? b[i] : a[i];
            else a[i] = b[i] > a[i] ? b[i] : a[i];
          };
          uint8_t* a = sh.result.data();
          const uint8_t* b = sh.contrib[r].data();
          switch (t) {
            case ncclInt8: combine((int8_t*)a, (const int8_t*)b); break;
            case ncclUint8: combine(a, b); break;
            case ncclInt32: combine((int32_t*)a, (const int32_t*)b); break;
            case ncclUint32: combine((uint32_t*)a, (const uint32_t*)b); break;
            case ncclInt64: combine((int64_t*)a, (const int64_t*)b); break;
            case ncclUint64: combine((uint64_t*)a, (const uint64_t*)b); break;
            case ncclFloat32: combine((float*)a, (const float*)b); break;
            default: combine((double*)a, (const double*)b); break;
          }
        }
      }
      sh.arrived = 0;
      ++sh.gen;
      sh.cv.notify_all();
    } else {
      ncclResult_t r = wait_for(lk, sh, [&] { return sh.gen != g; }, "an all-reduce",
                                comm->rank);
      if (r != ncclSuccess) return r;
    }
    out = sh.result;  // read before this rank can arrive at the next all-reduce
  }
  if (hipMemcpyAsync(recvbuf, out.data(), bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ncclUnhandledCudaError;
  return ncclSuccess;
}

}  // extern "C"
