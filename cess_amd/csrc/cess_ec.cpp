// libcessec host side: the C ABI of include/cess_ec.h over the HIP kernels in kernels.hip.
//
// Owns, per codec: the (k+m) x k encode matrix (gf256.h), the run-time coefficient programs in
// HBM (encode + one per erasure pattern in an LRU cache), the plan of the last per-segment
// reconstruct, the kernel selection (KernelOpts), a private HIP stream for uploads and a staging
// area in HBM for the host-buffer API. Multi-GPU sharding lives above this library (one codec
// per device).
//
// Lifetime of device blocks (coefficient programs, per-segment plans): a block can still be read
// by kernels enqueued on any caller stream after the host has dropped it (an evicted pattern, a
// replaced plan). Blocks come from a per-codec DevPool and are never freed in place: dropping the
// last reference retires the block, and a retired block is reused or freed only once every
// launch enqueued before the retirement has completed. Each call that launches kernels reading
// pool blocks records a mark event on its stream; a block retired after mark n waits for marks
// 1..n (host-side event queries, no device-wide synchronisation).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <deque>
#include <list>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/cess_ec.h"
#include "fftdec_cost.h"
#include "fftdec_plan.h"
#include "gf256.h"
#include "kernels.h"

namespace {

using cec::KernelOpts;
using cec::Layout;
using BigMat = cec::Mat<cec::kMaxShards, cec::kMaxShards>;
using WorkMat = cec::Mat<cec::kMaxShards, 2 * cec::kMaxShards>;
using BigPlan = cec::Plan<cec::kMaxShards, cec::kMaxShards>;

thread_local std::string g_last_error;

int set_err(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return set_err(_e == hipErrorOutOfMemory ? CEC_ENOMEM : CEC_EHIP,                 \
                     std::string(#expr) + ": " + hipGetErrorString(_e));                \
  } while (0)

// ---- device block pool with stream-ordered retirement -------------------------------------
// Blocks come from the stream-ordered allocator on the codec's private stream and go back to it
// with hipFreeAsync: hipMalloc / hipFree would do (hipFree performs an implicit
// hipDeviceSynchronize), and destroying one codec must not wait for other codecs' work.
class DevPool {
 public:
  ~DevPool() { drain(); }
  void set_stream(hipStream_t st) { st_ = st; }

  // A block of at least `bytes` (size classes of powers of two from 4 KiB).
  int alloc(size_t bytes, void** out) {
    collect();
    const int c = cls(bytes);
    if ((size_t)c < free_.size() && !free_[c].empty()) {
      *out = free_[c].back();
      free_[c].pop_back();
      return CEC_OK;
    }
    // complete before any stream uses it (a rare host wait: freed blocks are reused)
    HIP_TRY(hipMallocAsync(out, (size_t)1 << c, st_));
    HIP_TRY(hipStreamSynchronize(st_));
    held_ += (size_t)1 << c;
    return CEC_OK;
  }
  // The last reference to a block was dropped; kernels enqueued so far may still read it.
  void retire(void* p, size_t bytes) {
    if (p) dead_.push_back({seq_, p, cls(bytes)});
  }
  // Record the completion point of the launches just enqueued on `st`.
  int mark(hipStream_t st) {
    hipEvent_t ev = nullptr;
    if (!evpool_.empty()) {
      ev = evpool_.back();
      evpool_.pop_back();
    } else {
      HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    hipError_t e = hipEventRecord(ev, st);
    if (e != hipSuccess) {
      evpool_.push_back(ev);
      return set_err(CEC_EHIP, std::string("hipEventRecord: ") + hipGetErrorString(e));
    }
    marks_.push_back({++seq_, ev});
    // bound the backlog of a producer that never synchronises
    while (marks_.size() > 1024) {
      (void)hipEventSynchronize(marks_.front().ev);
      collect();
    }
    return CEC_OK;
  }
  // Move retired blocks whose readers have completed to the free lists.
  void collect() {
    while (!marks_.empty() && hipEventQuery(marks_.front().ev) == hipSuccess) {
      done_ = marks_.front().seq;
      evpool_.push_back(marks_.front().ev);
      marks_.pop_front();
    }
    if (marks_.empty()) done_ = seq_;
    while (!dead_.empty() && dead_.front().tag <= done_) {
      const Dead& d = dead_.front();
      if ((size_t)d.c >= free_.size()) free_.resize(d.c + 1);
      free_[d.c].push_back(d.p);
      dead_.pop_front();
    }
  }
  // Wait for every mark and free every block (codec destruction).
  void drain() {
    for (auto& m : marks_) {
      (void)hipEventSynchronize(m.ev);
      evpool_.push_back(m.ev);
    }
    marks_.clear();
    done_ = seq_;
    collect();
    for (auto& fl : free_)
      for (void* p : fl) (void)hipFreeAsync(p, st_);
    if (held_) (void)hipStreamSynchronize(st_);
    free_.clear();
    held_ = 0;
    for (hipEvent_t e : evpool_) (void)hipEventDestroy(e);
    evpool_.clear();
  }
  size_t pending() const { return dead_.size(); }
  size_t held() const { return held_; }  // device bytes the pool has allocated (live + free)

 private:
  static int cls(size_t bytes) {
    int c = 12;
    while (((size_t)1 << c) < bytes) ++c;
    return c;
  }
  struct Dead {
    uint64_t tag;
    void* p;
    int c;
  };
  struct Mark {
    uint64_t seq;
    hipEvent_t ev;
  };
  std::vector<std::vector<void*>> free_;
  std::deque<Dead> dead_;  // in retirement order, so tags are non-decreasing
  std::deque<Mark> marks_;
  std::vector<hipEvent_t> evpool_;
  hipStream_t st_ = nullptr;  // the owner's private stream (allocations and frees)
  uint64_t seq_ = 0;   // marks recorded
  uint64_t done_ = 0;  // every mark <= done_ has completed
  size_t held_ = 0;
};

// Batch-sized scratch (a verify's recomputed parity, an audit's gathered chunks) is not a pool
// block: the pool rounds to powers of two and keeps blocks until the codec dies, so one verify of
// ~94 GiB would pin 128 GiB of HBM to the codec. Above this size the scratch is stream-ordered
// (hipMallocAsync / hipFreeAsync on the call's stream): exact size, returned once the stream
// passes the launches that read it, no host wait.
constexpr size_t kBigScratch = size_t(16) << 20;
struct Scratch {
  void* p = nullptr;
  size_t bytes = 0;
  bool async = false;
};

// A run-time program: chunks of up to kRtMaxOut outputs, each a device block in the layout of
// kernels.h (header, input indices, output indices, coefficients [nin][nob]).
struct RtChunk {
  uint32_t* dev = nullptr;
  size_t bytes = 0;
  int nin = 0, nout = 0, nob = 0;
};

struct Program {
  std::vector<RtChunk> chunks;
  int nout = 0;     // total outputs
  int single = -1;  // the one missing shard when exactly one output (compile-time decode)
  bool partial = false;  // rows restricted to held survivors (cec_reconstruct_partial_batch)
  // RS(32,32): the same rebuild as an FFT-domain decode plan (fftdec_plan.h), a pool block
  uint32_t* fd = nullptr;
  size_t fd_bytes = 0;
  int fd_side = 0;
  int fd_nrs = 0;  // syndrome slots of the plan (its row cost: outputs x slots)
  // and as a formal-derivative plan (fftdec_plan_d: cost independent of the erasure count)
  uint32_t* fdd = nullptr;
  size_t fdd_bytes = 0;
  uint8_t in_idx[cec::kMaxShards] = {};   // survivors read (host copy)
  uint8_t out_idx[cec::kMaxShards] = {};  // shards written (host copy)
};
using ProgPtr = std::shared_ptr<const Program>;

// Upload coefficient rows for outputs out_idx[o] (coef[o][j]) as run-time chunks. The chunk
// blocks come from `pool` and go back to it (retired) when the last ProgPtr is dropped. Uploads
// run on `upload` and are complete when this returns.
// `partial`: the rows do not rebuild a shard by themselves (cec_reconstruct_partial_batch), so
// the compile-time single-erasure kernels never stand in for the program.
// Page-locked staging for program images whose uploads stay in flight until one synchronisation
// per plan: an upload from pinned memory is a DMA enqueue, one from pageable memory is staged by
// the runtime (measured: 64 new RS(32,32) patterns per call cost ~0.9 ms of host time beyond the
// kernel with pageable images). Blocks of >= 1 MiB, kept for reuse; reset() after the sync.
// hipHostFree, like hipFree, synchronises the whole device, so destroying a codec must not free
// its arena's blocks: they go to this process-wide cache (up to kCap bytes) for the next arena.
// The cache is never destroyed (the HIP runtime may be gone by the time static destructors run).
// Blocks are reused on the device they were allocated under only.
struct PinnedCache {
  static constexpr size_t kCap = size_t(64) << 20;
  struct Block {
    uint8_t* p;
    size_t cap;
    int device;
  };
  std::mutex mu;
  std::vector<Block> blocks;
  size_t bytes = 0;
  static PinnedCache& get() {
    static PinnedCache* c = new PinnedCache;
    return *c;
  }
  // a cached block of at least `need` bytes of `device` (the smallest), or {nullptr, 0, device}
  Block take(size_t need, int device) {
    std::lock_guard<std::mutex> g(mu);
    size_t best = blocks.size();
    for (size_t i = 0; i < blocks.size(); ++i)
      if (blocks[i].device == device && blocks[i].cap >= need &&
          (best == blocks.size() || blocks[i].cap < blocks[best].cap))
        best = i;
    if (best == blocks.size()) return {nullptr, 0, device};
    const Block b = blocks[best];
    blocks.erase(blocks.begin() + best);
    bytes -= b.cap;
    return b;
  }
  void give(const Block& b) {
    {
      std::lock_guard<std::mutex> g(mu);
      if (bytes + b.cap <= kCap) {
        blocks.push_back(b);
        bytes += b.cap;
        return;
      }
    }
    (void)hipHostFree(b.p);  // past the cap: the rare device-wide synchronisation
  }
};

class PinnedArena {
 public:
  ~PinnedArena() {
    for (auto& b : blocks_) PinnedCache::get().give({b.p, b.cap, device_});
  }
  // `bytes` of zeroed page-locked memory valid until reset(), or nullptr (caller falls back)
  uint32_t* take(size_t bytes) {
    bytes = (bytes + 255) & ~size_t(255);
    for (; cur_ < blocks_.size(); ++cur_)
      if (blocks_[cur_].used + bytes <= blocks_[cur_].cap) break;
    if (cur_ == blocks_.size()) {
      Block b{nullptr, std::max(bytes, size_t(1) << 20), 0};
      if (blocks_.empty() && hipGetDevice(&device_) != hipSuccess) return nullptr;
      const PinnedCache::Block cached = PinnedCache::get().take(b.cap, device_);
      if (cached.p) {
        b.p = cached.p;
        b.cap = cached.cap;
      } else if (hipHostMalloc(reinterpret_cast<void**>(&b.p), b.cap, hipHostMallocDefault) !=
                 hipSuccess) {
        return nullptr;
      }
      blocks_.push_back(b);
    }
    Block& b = blocks_[cur_];
    uint8_t* p = b.p + b.used;
    b.used += bytes;
    std::memset(p, 0, bytes);
    return reinterpret_cast<uint32_t*>(p);
  }
  void reset() {
    for (auto& b : blocks_) b.used = 0;
    cur_ = 0;
  }
  bool busy() const { return cur_ > 0 || (!blocks_.empty() && blocks_[0].used); }

 private:
  struct Block {
    uint8_t* p;
    size_t cap, used;
  };
  std::vector<Block> blocks_;
  size_t cur_ = 0;
  int device_ = -1;  // the device current when the first block was taken (the codec's)
};

// With `keep`, the images are written into that arena and the uploads are left in flight: the
// caller synchronises `upload` once for a whole plan before launching or resetting the arena.
using HostImages = PinnedArena;
int build_program(DevPool& pool, hipStream_t upload, const uint8_t* in_idx, int nin,
                  const uint8_t* out_idx, int nout, const BigMat& coef, ProgPtr* out,
                  bool partial = false, HostImages* keep = nullptr,
                  const cec::FftDecPlan* fdp = nullptr, const cec::FftDecPlan* fddp = nullptr) {
  DevPool* pp = &pool;
  std::shared_ptr<Program> prog(new Program, [pp](Program* p) {
    for (auto& c : p->chunks) pp->retire(c.dev, c.bytes);
    pp->retire(p->fd, p->fd_bytes);
    pp->retire(p->fdd, p->fdd_bytes);
    delete p;
  });
  prog->nout = nout;
  prog->single = nout == 1 && !partial ? out_idx[0] : -1;
  prog->partial = partial;
  std::memcpy(prog->in_idx, in_idx, nin);
  std::memcpy(prog->out_idx, out_idx, nout);
  std::vector<std::vector<uint32_t>> hosts;  // images when there is no arena (or it is full)
  bool staged = keep != nullptr;
  for (int o0 = 0; o0 < nout; o0 += cec::kRtMaxOut) {
    RtChunk c;
    c.nin = nin;
    c.nout = std::min(cec::kRtMaxOut, nout - o0);
    c.nob = cec::rt_bucket(c.nout);
    const size_t words = cec::rt_chunk_bytes(nin, c.nob) / sizeof(uint32_t);
    uint32_t* h = keep ? keep->take(words * sizeof(uint32_t)) : nullptr;
    if (!h) {
      hosts.emplace_back(words, 0u);
      h = hosts.back().data();
      staged = false;  // a pageable image: synchronise before it dies
    }
    h[0] = (uint32_t)nin;
    h[1] = (uint32_t)c.nout;
    h[2] = (uint32_t)c.nob;
    for (int j = 0; j < nin; ++j) h[4 + j] = in_idx[j];
    for (int o = 0; o < c.nout; ++o) h[4 + 256 + o] = out_idx[o0 + o];
    uint32_t* hb = h + 4 + 512;
    uint32_t* mk = h + cec::kRtHeaderWords;
    for (int j = 0; j < nin; ++j) {
      int top = -1;
      for (int o = 0; o < c.nout; ++o) {
        const unsigned cf = coef.v[o0 + o][j];
        for (int b = 0; b < 8; ++b)
          if (cf >> b & 1) {
            mk[((size_t)j * 8 + b) * c.nob + o] = 0xFFFFFFFFu;
            top = std::max(top, b);
          }
      }
      hb[j] = (uint32_t)top;
    }
    if (nin <= cec::kRthMaxIn) {
      // Horner section (kernels.h): per output row, its top bit and per (bit, group) the
      // combination index of the group's inputs whose coefficient has that bit
      const size_t hoff = cec::kRtHeaderWords + (size_t)nin * 8 * c.nob;
      h[3] = (uint32_t)hoff;
      uint32_t* top = h + hoff;
      uint32_t* ix = top + 32;
      for (int o = 0; o < c.nout; ++o) {
        int t = -1;
        for (int j = 0; j < nin; ++j)
          for (int b = 0; b < 8; ++b)
            if (coef.v[o0 + o][j] >> b & 1) t = std::max(t, b);
        top[o] = (uint32_t)t;
        for (int b = 0; b < 8; ++b)
          for (int j = 0; j < nin; ++j)
            if (coef.v[o0 + o][j] >> b & 1) ix[((size_t)o * 8 + b) * 8 + j / 4] |= 1u << (j % 4);
      }
    }
    c.bytes = words * sizeof(uint32_t);
    void* d = nullptr;
    int rc = pool.alloc(c.bytes, &d);
    if (rc) return rc;  // prog's deleter retires the chunks built so far
    c.dev = static_cast<uint32_t*>(d);
    prog->chunks.push_back(c);
    HIP_TRY(hipMemcpyAsync(c.dev, h, c.bytes, hipMemcpyHostToDevice, upload));
  }
  // the FFT-domain decode plans of the same pattern
  auto upload_plan = [&](const cec::FftDecPlan& fp, uint32_t** dev, size_t* dbytes) -> int {
    const size_t bytes = fp.w.size() * sizeof(uint32_t);
    uint32_t* h = keep ? keep->take(bytes) : nullptr;
    if (!h) {
      hosts.emplace_back(fp.w);
      h = hosts.back().data();
      staged = false;
    } else {
      std::memcpy(h, fp.w.data(), bytes);
    }
    void* d = nullptr;
    int rc = pool.alloc(bytes, &d);
    if (rc) return rc;
    *dev = static_cast<uint32_t*>(d);
    *dbytes = bytes;
    HIP_TRY(hipMemcpyAsync(*dev, h, bytes, hipMemcpyHostToDevice, upload));
    return CEC_OK;
  };
  if (fdp) {
    int rc = upload_plan(*fdp, &prog->fd, &prog->fd_bytes);
    if (rc) return rc;
    prog->fd_side = fdp->side;
    prog->fd_nrs = fdp->nrslots;
  }
  if (fddp) {
    int rc = upload_plan(*fddp, &prog->fdd, &prog->fdd_bytes);
    if (rc) return rc;
  }
  // the block may be a reused one whose readers have completed; the upload must land before
  // any caller-stream launch that reads it, and pageable images die here (arena images live
  // until the caller's synchronisation)
  if (!staged) HIP_TRY(hipStreamSynchronize(upload));
  *out = std::move(prog);
  return CEC_OK;
}

// One multi-pattern run-time launch of the per-segment reconstruct path.
struct PsLaunch {
  int nob = 0, nin = 0;
  size_t off = 0, count = 0;  // into the plan's segment-list / chunk-pointer arrays
};

// Plan of one per-segment reconstruct call (cached for a repeated pattern array): either
// compile-time launches per pattern (ct: program, offset, count into list), one mixed-pattern
// RS(2,1) launch, or multi-pattern run-time launches (rt: segment list + per-segment chunk
// pointers). `progs` holds every program whose device chunks the arrays point at.
struct PsPlan {
  std::string key;
  std::vector<ProgPtr> progs;
  std::vector<std::string> keys;  // decode-cache keys of the patterns (LRU touch on reuse)
  uint32_t* list = nullptr;
  size_t list_bytes = 0;
  void* ptrs = nullptr;  // const uint32_t* [count] per run-time launch
  size_t ptrs_bytes = 0;
  std::vector<std::pair<ProgPtr, std::pair<size_t, size_t>>> ct;
  std::vector<PsLaunch> rt;
  size_t mixed_off = 0, mixed_count = 0;  // tagged list (segment | erased << 30), count 0: none
  std::vector<uint8_t> mixed_e;  // the same erasures per segment in natural order (variant 90)
  struct FdLaunch {
    int side;           // 0, 1: syndrome-row decoder of that side; 2: formal derivative
    bool big;           // cec::fftdec_big of the plans' syndrome slot count
    size_t off, count;  // segments list + per-segment FFT-domain plans (pointer array)
  };
  std::vector<FdLaunch> fd;
};

constexpr size_t kDefaultDecodeCache = 4096;

}  // namespace

struct cec_codec {
  int k = 0, m = 0, device = 0;
  std::unique_ptr<BigMat> E;
  hipStream_t stream = nullptr;  // private: uploads and the host-buffer API
  KernelOpts opts;
  bool force_generic = false;
  // RS(32,32) patterns with at least this many outputs take the FFT-domain decoder (0: never)
  int fftdec_min = 4;
  int fftdec_mode = 0;  // 0: by the cost model (fftdec_choice), 1: syndrome rows, 2: derivative
  uint64_t fd_segments = 0;  // segments rebuilt by the FFT-domain decoders (CEC_STAT_FFTDEC_SEGMENTS)
  uint64_t fdd_segments = 0;  // of those, by the formal-derivative one (CEC_STAT_FFTDEC_D_SEGMENTS)
  DevPool pool;  // declared before every holder of pool blocks: destroyed after them
  ProgPtr encode;
  // decode programs by erasure pattern (n presence flags + data_only), least recently used last
  struct Entry {
    ProgPtr prog;
    std::list<std::string>::iterator lru;
  };
  std::unordered_map<std::string, Entry> decode_cache;
  std::list<std::string> lru;
  size_t cache_cap = kDefaultDecodeCache;
  std::unique_ptr<PsPlan> ps;
  // decode-plan scratch, reused pattern after pattern (a codec is not re-entrant): allocating
  // and zeroing these ~450 KB per new pattern was most of a new plan's host time
  struct PlanScratch {
    BigPlan plan;
    BigMat a, ainv, coef;
    WorkMat work;
  };
  std::unique_ptr<PlanScratch> scratch;
  PinnedArena arena;  // program images of a plan being built (uploads in flight)
  PlanScratch& plan_scratch() {
    if (!scratch) scratch = std::make_unique<PlanScratch>();
    return *scratch;
  }
  // staging for the host-buffer API: [n][stride]
  uint8_t* stage = nullptr;
  size_t stage_bytes = 0;

  void drop_plan() {
    if (!ps) return;
    pool.retire(ps->list, ps->list_bytes);
    pool.retire(ps->ptrs, ps->ptrs_bytes);
    ps.reset();
  }
  ~cec_codec() {
    (void)hipSetDevice(device);
    // no device-wide synchronisation: every launch that reads a pool block (a run-time encode
    // or decode program, a plan's arrays, audit indices) is followed by a mark on its stream, and
    // pool.drain() waits for those marks only; other codecs' streams keep running
    drop_plan();
    decode_cache.clear();
    lru.clear();
    encode.reset();
    pool.drain();
    if (stage) {
      (void)hipFreeAsync(stage, stream);  // the host API's calls synchronise before returning
      (void)hipStreamSynchronize(stream);
    }
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

// Batched calls run on the caller's stream; NULL is the HIP null (legacy default) stream, as
// in the HIP API itself (torch's default stream has handle 0).
hipStream_t pick_stream(cec_codec*, void* s) { return reinterpret_cast<hipStream_t>(s); }

Layout batch_layout(const cec_codec* c, const uint8_t* d_data, const uint8_t* d_parity,
                    size_t shard_len) {
  Layout L{};
  L.data = const_cast<uint8_t*>(d_data);
  L.parity = const_cast<uint8_t*>(d_parity);
  L.len = shard_len;
  L.shard_stride = shard_len;
  L.data_seg_stride = (uint64_t)c->k * shard_len;
  L.par_seg_stride = (uint64_t)c->m * shard_len;
  L.k = c->k;
  return L;
}

void launch_chunk(const KernelOpts& o, const Layout& L, const uint32_t* chunk,
                  const uint32_t* const* per_seg, int nin, int nob, const uint32_t* seg_list,
                  uint32_t nseg, hipStream_t st) {
  // bit-plane accumulators for one to four outputs from a wide input set (RS(32,32) rebuilds
  // vs k_rthx: one lost fragment 5.84 vs 4.03 TB/s, two 4.89 vs 3.75, three 3.89 vs 3.55, four
  // 3.36 vs 3.33; RS(10,4) encode 3.54 vs 3.41; bench.py --config 6 --erasures e / --config 8,
  // profiles/r02/rtb_sweep.txt)
  if ((o.rt_mode == 3 || (o.rt_mode == 0 && nob <= 4 && nin >= 4)) &&
      cec::launch_matvec_rtb(L, chunk, per_seg, nob, seg_list, nseg, st, o.ct_variant))
    return;
  if (nin <= cec::kRthMaxIn &&
      cec::launch_matvec_rth(o, L, chunk, per_seg, nin, seg_list, nseg, st))
    return;
  cec::launch_matvec_rt(L, chunk, per_seg, nob, seg_list, nseg, st);
}

void run_program(const KernelOpts& o, const Program& p, const Layout& L, const uint32_t* seg_list,
                 uint32_t nseg, hipStream_t st) {
  for (const auto& c : p.chunks)
    launch_chunk(o, L, c.dev, nullptr, c.nin, c.nob, seg_list, nseg, st);
}

int check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(CEC_EHIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return CEC_OK;
}

int do_encode(cec_codec* c, const Layout& L, const uint32_t* seg_list, uint32_t nseg,
              hipStream_t st) {
  if (nseg == 0 || L.len == 0) return CEC_OK;
  if (c->force_generic || !cec::launch_encode_ct(c->opts, c->k, c->m, L, seg_list, nseg, st)) {
    // the run-time program reads pool blocks (the encode program's chunks): mark the stream so
    // the codec's destruction waits for this launch (compile-time kernels read none)
    run_program(c->opts, *c->encode, L, seg_list, nseg, st);
    int rc = check_launch();
    return rc ? rc : c->pool.mark(st);
  }
  return check_launch();
}

int scratch_alloc(cec_codec* c, size_t bytes, hipStream_t st, Scratch* s) {
  s->bytes = bytes;
  if (bytes >= kBigScratch) {
    s->async = true;
    HIP_TRY(hipMallocAsync(&s->p, bytes, st));
    return CEC_OK;
  }
  return c->pool.alloc(bytes, &s->p);
}
// after the launches reading the scratch are enqueued (and, for a pool block, marked)
void scratch_release(cec_codec* c, const Scratch& s, hipStream_t st) {
  if (!s.p) return;
  if (s.async)
    (void)hipFreeAsync(s.p, st);
  else
    c->pool.retire(s.p, s.bytes);
}

// Cache keys start with a kind tag, so keys of different kinds never compare equal whatever
// their lengths: 'F' full rebuild, 'P' partial rebuild (decode LRU); 'S' / 'Q' the per-segment
// plans of cec_reconstruct_batch / cec_reconstruct_partial_batch.
std::string pattern_key(const uint8_t* present, int n, bool data_only) {
  std::string key(n + 2, '\0');
  key[0] = 'F';
  for (int i = 0; i < n; ++i) key[1 + i] = present[i] ? 1 : 0;
  key[n + 1] = data_only ? 1 : 0;
  return key;
}

std::string partial_key(const uint8_t* present, const uint8_t* held, int n, bool data_only) {
  std::string key = pattern_key(present, n, data_only);
  key[0] = 'P';
  for (int i = 0; i < n; ++i) key.push_back(held[i] ? 1 : 0);
  return key;
}

// Decode program for one erasure pattern (LRU-cached). Nothing is evicted here: the caller
// evicts after its launches are enqueued and marked (evict_decode), so a program resolved
// earlier in the same call is never dropped under it.
int get_decode(cec_codec* c, const uint8_t* present, bool data_only, ProgPtr* out,
               HostImages* keep = nullptr) {
  const int n = c->k + c->m;
  std::string key = pattern_key(present, n, data_only);
  auto it = c->decode_cache.find(key);
  if (it != c->decode_cache.end()) {
    c->lru.splice(c->lru.begin(), c->lru, it->second.lru);
    *out = it->second.prog;
    return CEC_OK;
  }
  auto& sc = c->plan_scratch();
  auto* plan = &sc.plan;
  uint8_t flags[cec::kMaxShards], rd[cec::kMaxShards];
  for (int i = 0; i < n; ++i) flags[i] = key[1 + i];
  if (!cec::survivor_set(c->k, c->m, flags, rd) ||
      cec::gf_decode_plan_sys(c->k, c->m, flags, data_only, *c->E, *plan, sc.a, sc.ainv, sc.work,
                              rd) != 0)
    return set_err(CEC_ETOOFEW, "fewer than k shards present");
  ProgPtr prog;
  if (plan->nout > 0) {
    // RS(32,32) rebuilds of several shards: also the FFT-domain plan (picked at launch by the
    // codec's CEC_OPT_FFTDEC_MIN and the layout)
    // They read exactly the program's survivors (the first k present shards): callers stage
    // only those (the host API below, the multi-GPU gathers), so the plans must not touch any
    // other shard flagged present.
    cec::FftDecPlan fdp, fddp;
    const bool wide = c->k == 32 && c->m == 32 && plan->nout >= 2;
    uint8_t read[cec::kMaxShards] = {};
    for (int j = 0; j < c->k; ++j) read[plan->in_idx[j]] = 1;
    const bool fd = wide && cec::fftdec_plan_m(read, flags, data_only, &fdp);
    const bool fdd = wide && cec::fftdec_plan_d(read, flags, data_only, &fddp);
    int rc = build_program(c->pool, c->stream, plan->in_idx, c->k, plan->out_idx, plan->nout,
                           plan->coef, &prog, false, keep, fd ? &fdp : nullptr,
                           fdd ? &fddp : nullptr);
    if (rc) return rc;
  } else {
    prog = std::make_shared<const Program>();
  }
  c->lru.push_front(key);
  c->decode_cache.emplace(std::move(key), cec_codec::Entry{prog, c->lru.begin()});
  *out = std::move(prog);
  return CEC_OK;
}

// Partial decode program (the partial-product exchange of SURVEY.md §8e): the decode rows of
// pattern `present` (survivors = survivor_set's, cec_survivors) restricted to the survivors flagged
// in `held`. The rebuild is linear in the survivors, so the XOR of the partials over any
// partition of the survivors is the full rebuild. No held survivor: a zero program (one input
// column with zero coefficients), so the outputs are still written (as zeros). Cached in the
// decode LRU under its own key.
int get_partial(cec_codec* c, const uint8_t* present, const uint8_t* held, bool data_only,
                ProgPtr* out, HostImages* keep = nullptr) {
  const int n = c->k + c->m;
  std::string key = partial_key(present, held, n, data_only);
  auto it = c->decode_cache.find(key);
  if (it != c->decode_cache.end()) {
    c->lru.splice(c->lru.begin(), c->lru, it->second.lru);
    *out = it->second.prog;
    return CEC_OK;
  }
  auto& sc = c->plan_scratch();
  auto* plan = &sc.plan;
  uint8_t flags[cec::kMaxShards], rd[cec::kMaxShards];
  for (int i = 0; i < n; ++i) flags[i] = present[i] ? 1 : 0;
  if (!cec::survivor_set(c->k, c->m, flags, rd) ||
      cec::gf_decode_plan_sys(c->k, c->m, flags, data_only, *c->E, *plan, sc.a, sc.ainv, sc.work,
                              rd) != 0)
    return set_err(CEC_ETOOFEW, "fewer than k shards present");
  ProgPtr prog;
  if (plan->nout > 0) {
    uint8_t in_sub[cec::kMaxShards];
    int nsub = 0;
    auto* coef = &sc.coef;
    for (int o = 0; o < plan->nout; ++o) std::memset(coef->v[o], 0, sizeof coef->v[o]);
    for (int j = 0; j < c->k; ++j)
      if (held[plan->in_idx[j]]) {
        for (int o = 0; o < plan->nout; ++o) coef->v[o][nsub] = plan->coef.v[o][j];
        in_sub[nsub++] = plan->in_idx[j];
      }
    if (nsub == 0) {  // zero program: one column, zero coefficients (cleared above)
      in_sub[0] = plan->in_idx[0];
      nsub = 1;
    }
    int rc = build_program(c->pool, c->stream, in_sub, nsub, plan->out_idx, plan->nout, *coef,
                           &prog, true, keep);
    if (rc) return rc;
  } else {
    prog = std::make_shared<const Program>();
  }
  c->lru.push_front(key);
  c->decode_cache.emplace(std::move(key), cec_codec::Entry{prog, c->lru.begin()});
  *out = std::move(prog);
  return CEC_OK;
}

// Drop least recently used patterns beyond the cap. A dropped program that a cached per-segment
// plan still uses stays alive through the plan; device blocks are retired, not freed.
void evict_decode(cec_codec* c) {
  while (c->decode_cache.size() > c->cache_cap && !c->lru.empty()) {
    c->decode_cache.erase(c->lru.back());
    c->lru.pop_back();
  }
}

// "Every data shard present, every parity shard lost" is the encode itself: the compile-time
// encode kernels (RS(32,32): the additive FFT, 5.8 TB/s) rebuild it, not a run-time program of m
// outputs (k_rthx, ~2.7 TB/s at 32).
bool is_reencode(const cec_codec* c, const Program& p) {
  if (p.partial || p.nout != c->m) return false;
  for (int o = 0; o < p.nout; ++o)
    if (p.out_idx[o] != c->k + o) return false;
  for (int j = 0; j < c->k; ++j)
    if (p.in_idx[j] != j) return false;
  return true;
}

// The decoder choice per pattern and per batch: fftdec_cost.h (tested on CPU against the
// recorded warm sweep, tests/test_host.py::test_fftdec_chooser_on_recorded_costs).
using cec::kFdD;
using cec::kFdM;
using cec::kFdNone;

// tuning build: CEC_OPT_CT_VARIANT 70 runs the pipelined persistent k_fftdec_dp instead of the
// one-block-per-wave k_fftdec_d, 72 the same with wave priorities, 73 k_fftdec_d with its quad
// exchanges through the LDS crossbar, 74..78 that in some phases only: the derivative, IFFT +
// derivative, the FFT tail, the IFFT, derivative + tail; 83 DPP in every phase (= the product's);
// 85 the product's without the skip of unread input slots (A/B sweeps)
// tuning build: CEC_OPT_CT_VARIANT 79..82 run k_fftdec_m with pair exchanges through the LDS
// crossbar: the IFFT's; + the FFT's last layer; + the nibble packs; all three; 84 DPP everywhere
// (= the product's). launch_fftdec's form is 1 + that mask; 86 (form 10) the product's without
// the skip of unread input slots.
int fdm_form(const cec_codec* c) {
  switch (c->opts.ct_variant) {
    case 79: return 2;
    case 80: return 4;
    case 81: return 6;
    case 82: return 8;
    case 84: return 1;
    case 86: return 10;
    default: return 0;
  }
}

int fdd_form(const cec_codec* c) {
  switch (c->opts.ct_variant) {
    case 70: return 1;
    case 72: return 3;
    case 73: return 4;
    case 74: return 5;
    case 75: return 6;
    case 76: return 7;
    case 77: return 8;
    case 78: return 9;
    case 83: return 10;
    case 85: return 11;
    default: return 0;
  }
}

int use_fftdec(const cec_codec* c, const Program& p) {
  if (c->force_generic || (!p.fd && !p.fdd) || c->fftdec_min <= 0 || p.nout < c->fftdec_min)
    return kFdNone;
  if (c->fftdec_mode == 1) return p.fd ? kFdM : kFdNone;
  if (c->fftdec_mode == 2) return p.fdd ? kFdD : kFdNone;
  return cec::fftdec_choice(p.nout, p.fd_nrs, cec::fftdec_big(p.fd_nrs), p.fd != nullptr,
                            p.fdd != nullptr);
}

int do_decode(cec_codec* c, const Program& p, const Layout& L, const uint32_t* seg_list,
              uint32_t nseg, hipStream_t st) {
  if (p.nout == 0 || nseg == 0 || L.len == 0) return CEC_OK;
  if (!c->force_generic && p.single < 0 && is_reencode(c, p))
    return do_encode(c, L, seg_list, nseg, st);
  const int fk = use_fftdec(c, p);
  if ((fk == kFdM && cec::launch_fftdec(L, p.fd_side, cec::fftdec_big(p.fd_nrs), p.fd, nullptr,
                                        seg_list, nseg, st, fdm_form(c))) ||
      (fk == kFdD && cec::launch_fftdec_d(L, p.fdd, nullptr, seg_list, nseg, st, fdd_form(c)))) {
    c->fd_segments += nseg;
    if (fk == kFdD) c->fdd_segments += nseg;
    return check_launch();
  }
  if (c->force_generic || p.single < 0 ||
      !cec::launch_decode_ct(c->opts, c->k, c->m, p.single, L, seg_list, nseg, st))
    run_program(c->opts, p, L, seg_list, nseg, st);
  return check_launch();
}

// Grow a buffer used only on stream `st` (stream-ordered: no device-wide synchronisation).
int ensure(uint8_t** buf, size_t* have, size_t need, hipStream_t st) {
  if (*have >= need) return CEC_OK;
  if (*buf) (void)hipFreeAsync(*buf, st);
  *buf = nullptr;
  *have = 0;
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(buf), need, st));
  *have = need;
  return CEC_OK;
}

size_t pad256(size_t x) { return (x + 255) & ~size_t(255); }

// Host-buffer API staging layout: one segment, shards at stride pad256(len).
Layout stage_layout(cec_codec* c, size_t len) {
  const size_t stride = pad256(len);
  Layout L{};
  L.data = c->stage;
  L.parity = c->stage + (size_t)c->k * stride;
  L.len = len;
  L.shard_stride = stride;
  L.data_seg_stride = (uint64_t)(c->k + c->m) * stride;
  L.par_seg_stride = (uint64_t)(c->k + c->m) * stride;
  L.k = c->k;
  return L;
}

// Build the plan of a per-segment reconstruct for the pattern array `pkey` (nseg * n flags +
// data_only + force_generic) into *out; device arrays are uploaded and complete on return.
// partial: pkey holds 2n flags per segment (present, then held) and the programs are partial
// (cec_reconstruct_partial_batch).
int build_ps_plan(cec_codec* c, const std::string& pkey, size_t nseg, bool data_only,
                  std::unique_ptr<PsPlan>* out, bool partial = false, bool fdok = false,
                  size_t shard_len = 0) {
  const int n = c->k + c->m;
  const int per = partial ? 2 * n : n;
  auto plan = std::make_unique<PsPlan>();
  plan->key = pkey;
  // group segments by pattern, in first-appearance order (deterministic launch order)
  std::unordered_map<std::string, size_t> gidx;
  std::vector<std::pair<std::string, std::vector<uint32_t>>> groups;
  for (size_t s = 0; s < nseg; ++s) {
    std::string k = pkey.substr(1 + s * per, per);
    auto it = gidx.find(k);
    if (it == gidx.end()) {
      it = gidx.emplace(k, groups.size()).first;
      groups.push_back({k, {}});
    }
    groups[it->second].second.push_back((uint32_t)s);
  }
  bool all_ct = !c->force_generic;
  std::vector<std::pair<ProgPtr, const std::vector<uint32_t>*>> progs, reencode, fdg[5];
  // new patterns' program uploads stay in flight until the one synchronisation below (one per
  // plan, not per pattern: 64 new RS(32,32) patterns cost ~1 ms of waits otherwise); every return
  // path waits for them before their host images go
  struct Uploads {
    hipStream_t st;
    PinnedArena& arena;
    ~Uploads() {
      if (arena.busy()) (void)hipStreamSynchronize(st);
      arena.reset();
    }
  } up{c->stream, c->arena};
  for (auto& g : groups) {
    ProgPtr p;
    const uint8_t* flags = reinterpret_cast<const uint8_t*>(g.first.data());
    int rc = partial ? get_partial(c, flags, flags + n, data_only, &p, &up.arena)
                     : get_decode(c, flags, data_only, &p, &up.arena);
    if (rc) return rc;
    plan->keys.push_back(partial ? partial_key(flags, flags + n, n, data_only)
                                 : pattern_key(flags, n, data_only));
    if (!p->nout) continue;
    plan->progs.push_back(p);
    if (!c->force_generic && p->single < 0 && is_reencode(c, *p)) {
      reencode.push_back({p, &g.second});  // the encode kernels, whatever the other groups take
      continue;
    }
    const int fk = fdok ? use_fftdec(c, *p) : kFdNone;
    if (fk == kFdM) {  // RS(32,32) wide rebuilds: the FFT-domain decoders
      fdg[p->fd_side * 2 + (cec::fftdec_big(p->fd_nrs) ? 1 : 0)].push_back({p, &g.second});
      continue;
    }
    if (fk == kFdD) {
      fdg[4].push_back({p, &g.second});
      continue;
    }
    progs.push_back({p, &g.second});
    if (p->single < 0 || !cec::has_decode_ct(c->k, c->m, p->single)) all_ct = false;
  }
  // The cost model picks per pattern; a batch whose patterns land on both decoders runs one more
  // launch than all-derivative. Fold the syndrome-row groups into the derivative launch when the
  // whole batch is cheaper that way (costs per segment scaled from 64 x 512 KiB).
  if (!fdg[4].empty() && c->fftdec_mode == 0) {
    std::vector<cec::FdmGroup> mg;
    int mlaunches = 0;
    for (int cls = 0; cls < 4; ++cls) {
      if (fdg[cls].empty()) continue;
      ++mlaunches;
      for (auto& pr : fdg[cls]) {
        const Program& q = *pr.first;
        mg.push_back({pr.second->size(), q.nout, q.fd_nrs, cec::fftdec_big(q.fd_nrs),
                      q.fdd != nullptr});
      }
    }
    if (cec::fftdec_fold(mg, mlaunches, shard_len)) {
      for (int cls = 0; cls < 4; ++cls) {
        for (auto& pr : fdg[cls]) fdg[4].push_back(pr);
        fdg[cls].clear();
      }
    }
  }
  std::vector<uint32_t> hl;
  std::vector<const uint32_t*> hp;
  for (auto& pr : reencode) {
    plan->ct.push_back({pr.first, {hl.size(), pr.second->size()}});
    hl.insert(hl.end(), pr.second->begin(), pr.second->end());
  }
  // the run-time launches index the segment list and the chunk-pointer array with one offset:
  // keep them aligned past the re-encode lists
  hp.resize(hl.size(), nullptr);
  for (int cls = 0; cls < 5; ++cls) {  // side x size class, and the derivative: one launch each
    if (fdg[cls].empty()) continue;
    PsPlan::FdLaunch f{cls == 4 ? 2 : cls >> 1, (cls & 1) != 0, hl.size(), 0};
    for (auto& pr : fdg[cls])
      for (uint32_t sg : *pr.second) {
        hl.push_back(sg);
        hp.push_back(cls == 4 ? pr.first->fdd : pr.first->fd);
        ++f.count;
      }
    plan->fd.push_back(f);
  }
  if (all_ct) {
    std::vector<uint32_t> tagged;
    for (auto& pr : progs) {
      plan->ct.push_back({pr.first, {hl.size(), pr.second->size()}});
      hl.insert(hl.end(), pr.second->begin(), pr.second->end());
      for (uint32_t sg : *pr.second) tagged.push_back(sg | ((uint32_t)pr.first->single << 30));
    }
    if (c->k == 2 && c->m == 1 && plan->ct.size() > 1 && nseg < (1u << 30)) {
      // grouped by erasure pattern, not in segment order: the workgroups resident at once then
      // mostly share one pattern (config 3, erased = seg mod 3: 0.253 -> 0.250 ms per GiB batch;
      // a uniform pattern takes 0.244-0.248, bench.py --erase)
      plan->mixed_off = hl.size();
      plan->mixed_count = tagged.size();
      hl.insert(hl.end(), tagged.begin(), tagged.end());
      // tuning variant 90's per-row codes: the lost shard of a tagged segment, 3 = untouched (an
      // intact segment, or one another launch handles: nothing is written to it)
      plan->mixed_e.assign(nseg, 3);
      for (uint32_t w : tagged) plan->mixed_e[w & 0x3FFFFFFFu] = (uint8_t)(w >> 30);
    }
  } else {
    size_t maxchunks = 0;
    for (auto& pr : progs) maxchunks = std::max(maxchunks, pr.first->chunks.size());
    for (size_t ci = 0; ci < maxchunks; ++ci) {
      std::vector<std::pair<int, std::vector<std::pair<uint32_t, const uint32_t*>>>> byb;
      int nin_max = 0;
      for (auto& pr : progs)
        if (ci < pr.first->chunks.size()) {
          const RtChunk& ch = pr.first->chunks[ci];
          nin_max = std::max(nin_max, ch.nin);
          auto it = std::find_if(byb.begin(), byb.end(),
                                 [&](const auto& b) { return b.first == ch.nob; });
          if (it == byb.end()) it = byb.insert(byb.end(), {ch.nob, {}});
          for (uint32_t sg : *pr.second) it->second.push_back({sg, ch.dev});
        }
      for (auto& b : byb) {
        PsLaunch l;
        l.nob = b.first;
        l.nin = nin_max;
        l.off = hl.size();
        l.count = b.second.size();
        for (auto& e : b.second) {
          hl.push_back(e.first);
          hp.push_back(e.second);
        }
        plan->rt.push_back(l);
      }
    }
  }
  void* d = nullptr;
  plan->list_bytes = std::max<size_t>(hl.size(), 1) * sizeof(uint32_t);
  int rc = c->pool.alloc(plan->list_bytes, &d);
  if (rc) return rc;
  plan->list = static_cast<uint32_t*>(d);
  plan->ptrs_bytes = std::max<size_t>(hp.size(), 1) * sizeof(void*);
  rc = c->pool.alloc(plan->ptrs_bytes, &plan->ptrs);
  if (rc) {
    c->pool.retire(plan->list, plan->list_bytes);
    return rc;
  }
  hipError_t e = hipSuccess;
  if (!hl.empty())
    e = hipMemcpyAsync(plan->list, hl.data(), hl.size() * sizeof(uint32_t),
                       hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess && !hp.empty())
    e = hipMemcpyAsync(plan->ptrs, hp.data(), hp.size() * sizeof(void*), hipMemcpyHostToDevice,
                       c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // the programs' uploads too
  if (e != hipSuccess) {
    c->pool.retire(plan->list, plan->list_bytes);
    c->pool.retire(plan->ptrs, plan->ptrs_bytes);
    return set_err(CEC_EHIP, std::string("plan upload: ") + hipGetErrorString(e));
  }
  up.arena.reset();  // its uploads have landed
  *out = std::move(plan);
  return CEC_OK;
}

int launch_ps_plan(cec_codec* c, const PsPlan& p, const Layout& L, hipStream_t st) {
  if (p.mixed_count && c->opts.ct_variant == 90 &&
      cec::launch_decode1_mixed_kargs(c->k, c->m, L, p.mixed_e.data(),
                                      (uint32_t)p.mixed_e.size(), st))
    return check_launch();
  if (p.mixed_count &&
      cec::launch_decode1_mixed(c->opts, c->k, c->m, L, p.list + p.mixed_off,
                                (uint32_t)p.mixed_count, st))
    return check_launch();
  for (const auto& w : p.ct) {
    int rc = do_decode(c, *w.first, L, p.list + w.second.first, (uint32_t)w.second.second, st);
    if (rc) return rc;
  }
  const uint32_t* const* ptrs = static_cast<const uint32_t* const*>(p.ptrs);
  for (const auto& f : p.fd) {
    const bool ok = f.side == 2 ? cec::launch_fftdec_d(L, nullptr, ptrs + f.off, p.list + f.off,
                                                       (uint32_t)f.count, st, fdd_form(c))
                                : cec::launch_fftdec(L, f.side, f.big, nullptr, ptrs + f.off,
                                                     p.list + f.off, (uint32_t)f.count, st,
                                                     fdm_form(c));
    if (!ok)
      return set_err(CEC_EINVAL, "FFT-domain decode plan on a layout it does not fit");
    c->fd_segments += f.count;
    if (f.side == 2) c->fdd_segments += f.count;
    int rc = check_launch();
    if (rc) return rc;
  }
  for (const auto& l : p.rt) {
    launch_chunk(c->opts, L, nullptr, ptrs + l.off, l.nin, l.nob, p.list + l.off,
                 (uint32_t)l.count, st);
    int rc = check_launch();
    if (rc) return rc;
  }
  return CEC_OK;
}

}  // namespace

namespace cec {
// error reporting shared with hashq.cpp (same thread-local detail string)
int set_error(int code, const std::string& msg) { return set_err(code, msg); }
}  // namespace cec

extern "C" {

const char* cec_version(void) {
#ifdef CEC_TUNING
  return "cessec 0.2.0 gfx950 tuning";
#else
  return "cessec 0.2.0 gfx950";
#endif
}

const char* cec_strerror(int code) {
  switch (code) {
    case CEC_OK: return "ok";
    case CEC_EINVAL: return "invalid argument";
    case CEC_ETOOFEW: return "too few shards given";
    case CEC_ESHARDLEN: return "shard sizes do not match";
    case CEC_EHIP: return "HIP runtime error";
    case CEC_ENOMEM: return "out of memory";
    case CEC_ENCCL: return "RCCL error";
    case CEC_ESHORTDATA: return "not enough data to fill the number of requested shards";
    case CEC_ENODEV: return "no GPU device";
    case CEC_ESEGCOUNT: return "file exceeds SegmentCount segments";
    case CEC_ECALLBACK: return "callback failed";
  }
  return "unknown error";
}

const char* cec_last_error(void) { return g_last_error.c_str(); }

int cec_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int cec_create(int k, int m, int device, cec_codec** out) {
  if (!out) return set_err(CEC_EINVAL, "null out");
  *out = nullptr;
  if (k < 1 || m < 1 || k + m > cec::kMaxShards)
    return set_err(CEC_EINVAL, "need k >= 1, m >= 1, k + m <= 256");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return set_err(CEC_ENODEV, "no HIP device visible");
  if (device < 0 || device >= ndev) return set_err(CEC_EINVAL, "device index out of range");
  HIP_TRY(hipSetDevice(device));
  std::unique_ptr<cec_codec> c(new (std::nothrow) cec_codec);
  if (!c) return set_err(CEC_ENOMEM, "codec");
  c->k = k;
  c->m = m;
  c->device = device;
  c->E = std::make_unique<BigMat>();
  {
    auto top = std::make_unique<BigMat>();
    auto topinv = std::make_unique<BigMat>();
    auto work = std::make_unique<WorkMat>();
    if (!cec::gf_encode_matrix(k, m, *c->E, *top, *topinv, *work))
      return set_err(CEC_EINVAL, "singular Vandermonde top block");
  }
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  c->pool.set_stream(c->stream);
  {
    auto par = std::make_unique<BigMat>();
    uint8_t in_idx[cec::kMaxShards], out_idx[cec::kMaxShards];
    for (int j = 0; j < k; ++j) in_idx[j] = (uint8_t)j;
    for (int o = 0; o < m; ++o) {
      out_idx[o] = (uint8_t)(k + o);
      for (int j = 0; j < k; ++j) par->v[o][j] = c->E->v[k + o][j];
    }
    int rc = build_program(c->pool, c->stream, in_idx, k, out_idx, m, *par, &c->encode);
    if (rc) return rc;
  }
  *out = c.release();
  return CEC_OK;
}

void cec_destroy(cec_codec* codec) { delete codec; }

int cec_codec_info(const cec_codec* c, int* k, int* m, int* device) {
  if (!c) return set_err(CEC_EINVAL, "null codec");
  if (k) *k = c->k;
  if (m) *m = c->m;
  if (device) *device = c->device;
  return CEC_OK;
}

int cec_matrix(const cec_codec* c, uint8_t* out) {
  if (!c || !out) return set_err(CEC_EINVAL, "null");
  for (int r = 0; r < c->k + c->m; ++r)
    for (int j = 0; j < c->k; ++j) out[r * c->k + j] = c->E->v[r][j];
  return CEC_OK;
}

int cec_set_option(cec_codec* c, int option, int value) {
  if (!c) return set_err(CEC_EINVAL, "null codec");
  switch (option) {
    case CEC_OPT_FORCE_GENERIC:
      c->force_generic = value != 0;
      return CEC_OK;
    case CEC_OPT_CT_VARIANT:
      if (value < -1 || value > cec::max_ct_variant())
        return set_err(CEC_EINVAL, cec::max_ct_variant() == 0
                                       ? "kernel variants need the tuning build (libcessec_tune)"
                                       : "variant out of range");
      c->opts.ct_variant = value == 0 && cec::max_ct_variant() == 0 ? -1 : value;
      return CEC_OK;
    case CEC_OPT_SHA_MODE:
      if (value < 0 || value > 3) return set_err(CEC_EINVAL, "sha mode out of range");
      c->opts.sha_mode = value;
      return CEC_OK;
    case CEC_OPT_RT_MODE:
      if (value < 0 || value > 3) return set_err(CEC_EINVAL, "rt mode out of range");
      c->opts.rt_mode = value;
      return CEC_OK;
    case CEC_OPT_FFTDEC_MIN:
      if (value < 0 || value > 64) return set_err(CEC_EINVAL, "fftdec min outputs in 0..64");
      c->fftdec_min = value;
      return CEC_OK;
    case CEC_OPT_FFTDEC_MODE:
      if (value < 0 || value > 2)
        return set_err(CEC_EINVAL, "fftdec mode is 0 (auto), 1 (syndrome rows) or 2 (derivative)");
      c->fftdec_mode = value;
      return CEC_OK;
    case CEC_OPT_DECODE_CACHE:
      if (value < 1) return set_err(CEC_EINVAL, "decode cache capacity must be >= 1");
      c->cache_cap = (size_t)value;
      evict_decode(c);
      return CEC_OK;
  }
  return set_err(CEC_EINVAL, "unknown option");
}

int cec_get_stat(const cec_codec* c, int stat, uint64_t* value) {
  if (!c || !value) return set_err(CEC_EINVAL, "null");
  switch (stat) {
    case CEC_STAT_DECODE_CACHED: *value = c->decode_cache.size(); return CEC_OK;
    case CEC_STAT_RETIRED_PENDING: *value = c->pool.pending(); return CEC_OK;
    case CEC_STAT_POOL_BYTES: *value = c->pool.held(); return CEC_OK;
    case CEC_STAT_FFTDEC_SEGMENTS: *value = c->fd_segments; return CEC_OK;
    case CEC_STAT_FFTDEC_D_SEGMENTS: *value = c->fdd_segments; return CEC_OK;
  }
  return set_err(CEC_EINVAL, "unknown stat");
}

int cec_encode_batch(cec_codec* c, const uint8_t* d_data, uint8_t* d_parity, size_t nseg,
                     size_t shard_len, void* hip_stream) {
  if (!c || (nseg && (!d_data || !d_parity))) return set_err(CEC_EINVAL, "null");
  if (shard_len == 0) return set_err(CEC_ESHARDLEN, "zero shard length");
  if (nseg > 0xffffffffull) return set_err(CEC_EINVAL, "too many segments");
  HIP_TRY(hipSetDevice(c->device));
  Layout L = batch_layout(c, d_data, d_parity, shard_len);
  return do_encode(c, L, nullptr, (uint32_t)nseg, pick_stream(c, hip_stream));
}

int cec_reconstruct_batch(cec_codec* c, uint8_t* d_data, uint8_t* d_parity, size_t nseg,
                          size_t shard_len, const uint8_t* present, int per_segment,
                          int data_only, void* hip_stream) {
  if (!c || !present || (nseg && (!d_data || !d_parity))) return set_err(CEC_EINVAL, "null");
  if (shard_len == 0) return set_err(CEC_ESHARDLEN, "zero shard length");
  if (nseg > 0xffffffffull) return set_err(CEC_EINVAL, "too many segments");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, hip_stream);
  const int n = c->k + c->m;
  Layout L = batch_layout(c, d_data, d_parity, shard_len);
  int rc = CEC_OK;
  if (!per_segment) {
    ProgPtr p;
    rc = get_decode(c, present, data_only != 0, &p);
    if (rc) return rc;
    rc = do_decode(c, *p, L, nullptr, (uint32_t)nseg, st);
  } else {
    // Per-segment patterns. Segments are grouped by pattern once and the plan is cached for a
    // repeated pattern array (degraded-read bench and repair loops pass the same map each
    // call):
    //  * every pattern has a compile-time single-erasure kernel (RS(2,1)): one mixed-pattern
    //    launch (or one launch per pattern over its segment list);
    //  * otherwise: one multi-pattern run-time launch per (chunk index, bucket), each segment's
    //    workgroup row reading its own pattern's chunk, so a batch where every segment has a
    //    different erasure map is still one full-grid launch.
    std::string pkey(1, 'S');
    pkey.reserve(nseg * n + 6);
    for (size_t i = 0; i < nseg * n; ++i) pkey.push_back(present[i] ? 1 : 0);
    pkey.push_back(data_only ? 1 : 0);
    pkey.push_back(c->force_generic ? 1 : 0);
    const bool fdok = cec::fftdec_layout_ok(L);
    pkey.push_back(fdok ? 1 : 0);
    pkey.push_back((char)c->fftdec_min);
    pkey.push_back((char)c->fftdec_mode);
    for (int b = 0; b < 8; ++b) pkey.push_back((char)(shard_len >> (8 * b)));  // the split rule
    if (!c->ps || c->ps->key != pkey) {
      std::unique_ptr<PsPlan> plan;
      rc = build_ps_plan(c, pkey, nseg, data_only != 0, &plan, false, fdok, shard_len);
      if (rc) return rc;
      c->drop_plan();  // the old plan's arrays are retired: launches already enqueued keep them
      c->ps = std::move(plan);
    } else {
      for (const auto& key : c->ps->keys) {  // the reused plan's patterns stay recently used
        auto it = c->decode_cache.find(key);
        if (it != c->decode_cache.end()) c->lru.splice(c->lru.begin(), c->lru, it->second.lru);
      }
    }
    rc = launch_ps_plan(c, *c->ps, L, st);
  }
  // completion point of these launches; only then may evicted programs be retired
  int mrc = c->pool.mark(st);
  evict_decode(c);
  return rc ? rc : mrc;
}

int cec_reconstruct_partial_batch(cec_codec* c, uint8_t* d_data, uint8_t* d_parity, size_t nseg,
                                  size_t shard_len, const uint8_t* present, const uint8_t* held,
                                  int data_only, void* hip_stream) {
  if (!c || !present || !held || (nseg && (!d_data || !d_parity)))
    return set_err(CEC_EINVAL, "null");
  if (shard_len == 0) return set_err(CEC_ESHARDLEN, "zero shard length");
  if (nseg > 0xffffffffull) return set_err(CEC_EINVAL, "too many segments");
  if (nseg == 0) return CEC_OK;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, hip_stream);
  const int n = c->k + c->m;
  Layout L = batch_layout(c, d_data, d_parity, shard_len);
  // per segment: n presence flags then n held flags; the same plan cache as the full rebuild
  // (the leading kind tag keeps the keys apart)
  std::string pkey(1, 'Q');
  pkey.reserve(nseg * 2 * n + 3);
  for (size_t s = 0; s < nseg; ++s) {
    for (int i = 0; i < n; ++i) pkey.push_back(present[s * n + i] ? 1 : 0);
    for (int i = 0; i < n; ++i) pkey.push_back(held[s * n + i] ? 1 : 0);
  }
  pkey.push_back(data_only ? 1 : 0);
  pkey.push_back(c->force_generic ? 1 : 0);
  int rc = CEC_OK;
  if (!c->ps || c->ps->key != pkey) {
    std::unique_ptr<PsPlan> plan;
    rc = build_ps_plan(c, pkey, nseg, data_only != 0, &plan, true);
    if (rc) return rc;
    c->drop_plan();
    c->ps = std::move(plan);
  } else {
    for (const auto& key : c->ps->keys) {
      auto it = c->decode_cache.find(key);
      if (it != c->decode_cache.end()) c->lru.splice(c->lru.begin(), c->lru, it->second.lru);
    }
  }
  rc = launch_ps_plan(c, *c->ps, L, st);
  int mrc = c->pool.mark(st);
  evict_decode(c);
  return rc ? rc : mrc;
}

int cec_verify_batch(cec_codec* c, const uint8_t* d_data, const uint8_t* d_parity, size_t nseg,
                     size_t shard_len, uint8_t* d_ok, void* hip_stream) {
  if (!c || !d_ok || (nseg && (!d_data || !d_parity))) return set_err(CEC_EINVAL, "null");
  if (shard_len == 0) return set_err(CEC_ESHARDLEN, "zero shard length");
  if (nseg > 0xffffffffull) return set_err(CEC_EINVAL, "too many segments");
  if (nseg == 0) return CEC_OK;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, hip_stream);
  if (!c->force_generic) {  // RS(2,1): recompute and compare in one read-only pass
    Layout L = batch_layout(c, d_data, const_cast<uint8_t*>(d_parity), shard_len);
    HIP_TRY(hipMemsetAsync(d_ok, 1, nseg, st));
    if (cec::launch_verify_ct(c->k, c->m, L, d_ok, (uint32_t)nseg, st)) return check_launch();
  }
  // the parity recomputed into a scratch batch (the encode kernels: FFT for RS(32,32)), then
  // compared segment by segment with the stored parity
  const size_t pbytes = nseg * (size_t)c->m * shard_len;
  Scratch sc;
  int rc = scratch_alloc(c, pbytes, st, &sc);
  if (rc) return rc;
  void* scratch = sc.p;
  Layout L = batch_layout(c, d_data, static_cast<uint8_t*>(scratch), shard_len);
  hipError_t e = hipMemsetAsync(d_ok, 1, nseg, st);
  if (e == hipSuccess) {
    rc = do_encode(c, L, nullptr, (uint32_t)nseg, st);
    if (!rc) {
      cec::launch_cmp_segments(static_cast<const uint8_t*>(scratch), d_parity,
                               (uint64_t)c->m * shard_len, nseg, d_ok, st);
      rc = check_launch();
    }
  } else {
    rc = set_err(CEC_EHIP, std::string("verify: ") + hipGetErrorString(e));
  }
  const int mrc = c->pool.mark(st);  // the scratch stays until these launches complete
  scratch_release(c, sc, st);
  return rc ? rc : mrc;
}

int cec_xor_batch(uint8_t* d_dst, const uint8_t* d_src, size_t nsrc, size_t src_stride,
                  size_t len, void* hip_stream) {
  if ((len && nsrc && (!d_dst || !d_src)) || nsrc > 0xffffffffull)
    return set_err(CEC_EINVAL, "null buffer or too many sources");
  if (nsrc > 1 && src_stride < len)
    return set_err(CEC_EINVAL, "src_stride < len: sources overlap");
  if ((len + 255) / 256 > 0x7fffffffull) return set_err(CEC_EINVAL, "len too large (> 512 GiB)");
  if (len == 0 || nsrc == 0) return CEC_OK;
  cec::launch_xor_reduce(d_dst, d_src, (uint32_t)nsrc, src_stride, len,
                         reinterpret_cast<hipStream_t>(hip_stream));
  return check_launch();
}

int cec_sha256_batch(cec_codec* c, const uint8_t* d_data, const uint8_t* d_parity, size_t nseg,
                     size_t shard_len, uint8_t* d_hex, void* hip_stream) {
  if (!c || !d_hex || (nseg && !d_data)) return set_err(CEC_EINVAL, "null");
  HIP_TRY(hipSetDevice(c->device));
  Layout L = batch_layout(c, d_data, d_parity, shard_len);
  int nsh = c->k + c->m;
  if (!d_parity) {
    nsh = c->k;
    L.parity = nullptr;
  }
  cec::launch_sha256_hex(c->opts.sha_mode, nullptr, &L, nsh, (uint64_t)nseg * nsh, shard_len,
                         d_hex, pick_stream(c, hip_stream));
  return check_launch();
}

int cec_sha256_hex(const uint8_t* const* d_bufs, size_t n, size_t len, uint8_t* hex,
                   void* hip_stream) {
  if (!hex || (n && !d_bufs)) return set_err(CEC_EINVAL, "null");
  if (n == 0) return CEC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
  const uint8_t** dptrs = nullptr;
  uint8_t* dhex = nullptr;
  // stream-ordered (hipFree would synchronise the whole device)
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&dptrs), n * sizeof(void*), st));
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&dhex), n * 64, st);
  if (e != hipSuccess) {
    (void)hipFreeAsync(dptrs, st);
    return set_err(CEC_ENOMEM, "hex buffer");
  }
  int rc = CEC_OK;
  do {
    if ((e = hipMemcpyAsync(dptrs, d_bufs, n * sizeof(void*), hipMemcpyHostToDevice, st))) break;
    cec::launch_sha256_hex(0, dptrs, nullptr, 1, n, len, dhex, st);
    if ((e = hipGetLastError())) break;
    if ((e = hipMemcpyAsync(hex, dhex, n * 64, hipMemcpyDeviceToHost, st))) break;
    e = hipStreamSynchronize(st);
  } while (0);
  if (e != hipSuccess) rc = set_err(CEC_EHIP, std::string("sha256: ") + hipGetErrorString(e));
  (void)hipFreeAsync(dptrs, st);
  (void)hipFreeAsync(dhex, st);
  return rc;
}

int cec_split_segment(const uint8_t* seg, size_t seg_len, int k, uint8_t* const* shards,
                      size_t shard_len) {
  if (!shards || k < 1) return set_err(CEC_EINVAL, "null shards or k < 1");
  if (seg_len == 0 || !seg) return set_err(CEC_ESHORTDATA, "empty segment");
  if (shard_len == 0 || (size_t)k * shard_len < seg_len)
    return set_err(CEC_ESHARDLEN, "k * shard_len < seg_len");
  for (int i = 0; i < k; ++i) {
    if (!shards[i]) return set_err(CEC_EINVAL, "null shard");
    const size_t off = (size_t)i * shard_len;
    const size_t take = off >= seg_len ? 0 : std::min(shard_len, seg_len - off);
    if (take) std::memcpy(shards[i], seg + off, take);
    if (take < shard_len) std::memset(shards[i] + take, 0, shard_len - take);
  }
  return CEC_OK;
}

int cec_fill_synthetic(uint8_t* d_out, size_t seg_bytes, size_t nseg, uint64_t seg0,
                       uint64_t seed, void* hip_stream) {
  if (!d_out && nseg) return set_err(CEC_EINVAL, "null");
  if (seg_bytes % 8) return set_err(CEC_EINVAL, "seg_bytes must be a multiple of 8");
  if (nseg == 0 || seg_bytes == 0) return CEC_OK;
  cec::launch_fill_splitmix(d_out, seg_bytes, nseg, seg0, seed,
                            reinterpret_cast<hipStream_t>(hip_stream));
  return check_launch();
}

// ---- storage audit chunks -----------------------------------------------------------------

int cec_challenge_indices(const uint64_t* randoms, size_t nrand, uint32_t chunk_count,
                          uint32_t need, uint32_t* out, size_t* used) {
  if ((nrand && !randoms) || (need && !out)) return set_err(CEC_EINVAL, "null");
  if (chunk_count == 0 || need > chunk_count)
    return set_err(CEC_EINVAL, "need must be <= chunk_count, chunk_count > 0");
  // c-pallets/audit/src/lib.rs:955-964
  uint32_t got = 0;
  size_t i = 0;
  for (; i < nrand && got < need; ++i) {
    const uint32_t idx = (uint32_t)(randoms[i] % chunk_count);
    bool seen = false;
    for (uint32_t q = 0; q < got && !seen; ++q) seen = out[q] == idx;
    if (!seen) out[got++] = idx;
  }
  if (used) *used = i;
  if (got < need) return set_err(CEC_EINVAL, "random stream exhausted before `need` indices");
  return CEC_OK;
}

int cec_audit_chunks(cec_codec* c, const uint8_t* d_data, const uint8_t* d_parity, size_t nseg,
                     size_t shard_len, uint32_t chunk_count, const uint32_t* indices,
                     uint32_t nidx, uint8_t* d_chunks, uint8_t* d_hex, void* hip_stream) {
  if (!c || !indices || (nseg && !d_data) || (!d_chunks && !d_hex))
    return set_err(CEC_EINVAL, "null");
  if (chunk_count == 0 || shard_len == 0 || shard_len % chunk_count)
    return set_err(CEC_ESHARDLEN, "shard_len must be a nonzero multiple of chunk_count");
  for (uint32_t j = 0; j < nidx; ++j)
    if (indices[j] >= chunk_count) return set_err(CEC_EINVAL, "chunk index out of range");
  if (nseg == 0 || nidx == 0) return CEC_OK;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, hip_stream);
  const int nsh = d_parity ? c->k + c->m : c->k;
  const uint64_t nfrag = (uint64_t)nseg * nsh;
  const uint64_t chunk = shard_len / chunk_count;
  Layout L = batch_layout(c, d_data, d_parity, shard_len);
  void* d_idx = nullptr;
  int rc = c->pool.alloc(nidx * sizeof(uint32_t), &d_idx);
  if (rc) return rc;
  const size_t idx_bytes = nidx * sizeof(uint32_t);
  hipError_t e = hipMemcpyAsync(d_idx, indices, idx_bytes, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    c->pool.retire(d_idx, idx_bytes);
    return set_err(CEC_EHIP, std::string("index upload: ") + hipGetErrorString(e));
  }
  Scratch sc;
  const size_t gbytes = nfrag * nidx * chunk;
  if (!d_chunks) {
    rc = scratch_alloc(c, gbytes, st, &sc);
    if (rc) {
      c->pool.retire(d_idx, idx_bytes);
      return rc;
    }
    d_chunks = static_cast<uint8_t*>(sc.p);
  }
  cec::launch_chunk_gather(L, nsh, nfrag, static_cast<const uint32_t*>(d_idx), nidx, chunk,
                           d_chunks, st);
  rc = check_launch();
  if (!rc && d_hex) {
    Layout G{};  // the gathered chunks as nfrag * nidx one-shard "segments"
    G.data = d_chunks;
    G.len = chunk;
    G.shard_stride = chunk;
    G.data_seg_stride = chunk;
    G.k = 1;
    cec::launch_sha256_hex(c->opts.sha_mode, nullptr, &G, 1, nfrag * nidx, chunk, d_hex, st);
    rc = check_launch();
  }
  const int mrc = c->pool.mark(st);  // the index array and scratch stay until these complete
  c->pool.retire(d_idx, idx_bytes);
  scratch_release(c, sc, st);
  return rc ? rc : mrc;
}

// ---- host-buffer API -------------------------------------------------------------------

int cec_encode(cec_codec* c, uint8_t* const* shards, size_t shard_len) {
  if (!c || !shards) return set_err(CEC_EINVAL, "null");
  if (shard_len == 0) return set_err(CEC_ESHARDLEN, "zero shard length");
  const int n = c->k + c->m;
  for (int i = 0; i < n; ++i)
    if (!shards[i]) return set_err(CEC_EINVAL, "null shard");
  HIP_TRY(hipSetDevice(c->device));
  const size_t stride = pad256(shard_len);
  int rc = ensure(&c->stage, &c->stage_bytes, stride * n, c->stream);
  if (rc) return rc;
  Layout L = stage_layout(c, shard_len);
  for (int i = 0; i < c->k; ++i)
    HIP_TRY(hipMemcpyAsync(c->stage + i * stride, shards[i], shard_len, hipMemcpyHostToDevice,
                           c->stream));
  rc = do_encode(c, L, nullptr, 1, c->stream);
  if (rc) return rc;
  for (int o = 0; o < c->m; ++o)
    HIP_TRY(hipMemcpyAsync(shards[c->k + o], c->stage + (c->k + o) * stride, shard_len,
                           hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return CEC_OK;
}

int cec_reconstruct(cec_codec* c, uint8_t* const* shards, const uint8_t* present,
                    size_t shard_len, int data_only) {
  if (!c || !shards || !present) return set_err(CEC_EINVAL, "null");
  if (shard_len == 0) return set_err(CEC_ESHARDLEN, "zero shard length");
  const int n = c->k + c->m;
  HIP_TRY(hipSetDevice(c->device));
  ProgPtr p;
  int rc = get_decode(c, present, data_only != 0, &p);
  if (rc) return rc;
  if (p->nout == 0) return CEC_OK;
  for (int i = 0; i < n; ++i)
    if (!shards[i]) return set_err(CEC_EINVAL, "null shard");
  const size_t stride = pad256(shard_len);
  rc = ensure(&c->stage, &c->stage_bytes, stride * n, c->stream);
  if (rc) return rc;
  Layout L = stage_layout(c, shard_len);
  // Upload only the survivors the plan reads.
  for (int j = 0; j < c->k; ++j) {
    const int i = p->in_idx[j];
    HIP_TRY(hipMemcpyAsync(c->stage + i * stride, shards[i], shard_len, hipMemcpyHostToDevice,
                           c->stream));
  }
  rc = do_decode(c, *p, L, nullptr, 1, c->stream);
  if (rc) return rc;
  for (int o = 0; o < p->nout; ++o) {
    const int i = p->out_idx[o];
    HIP_TRY(hipMemcpyAsync(shards[i], c->stage + i * stride, shard_len, hipMemcpyDeviceToHost,
                           c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  evict_decode(c);  // the launch above has completed
  return CEC_OK;
}

int cec_verify(cec_codec* c, uint8_t* const* shards, size_t shard_len, int* ok) {
  if (!c || !shards || !ok) return set_err(CEC_EINVAL, "null");
  if (shard_len == 0) return set_err(CEC_ESHARDLEN, "zero shard length");
  const int n = c->k + c->m;
  for (int i = 0; i < n; ++i)
    if (!shards[i]) return set_err(CEC_EINVAL, "null shard");
  HIP_TRY(hipSetDevice(c->device));
  const size_t stride = pad256(shard_len);
  int rc = ensure(&c->stage, &c->stage_bytes, stride * n, c->stream);
  if (rc) return rc;
  Layout L = stage_layout(c, shard_len);
  for (int i = 0; i < c->k; ++i)
    HIP_TRY(hipMemcpyAsync(c->stage + i * stride, shards[i], shard_len, hipMemcpyHostToDevice,
                           c->stream));
  rc = do_encode(c, L, nullptr, 1, c->stream);
  if (rc) return rc;
  std::vector<uint8_t> par(shard_len);
  *ok = 1;
  for (int o = 0; o < c->m && *ok; ++o) {
    HIP_TRY(hipMemcpyAsync(par.data(), c->stage + (c->k + o) * stride, shard_len,
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (std::memcmp(par.data(), shards[c->k + o], shard_len) != 0) *ok = 0;
  }
  return CEC_OK;
}

}  // extern "C"
