// libcessec multi-GPU degraded read: one process (or thread) per GPU, RCCL over
// xGMI for the one exchange step of the path.
//
// Placement: fragment f of segment s lives on rank (s + f) mod world, the GPU analogue of the
// chain's miner assignment (random_assign_miner, c-pallets/file-bank/src/functions.rs:187-283,
// which puts a segment's fragments on distinct miners). A degraded read gathers, for every
// segment with lost fragments, the k survivors the codec reads (cec_survivors) on
// the rank that owns the segment's first lost fragment (repair restores a fragment where it
// lives, c-pallets/file-bank/src/lib.rs:943-1122), straight into a [seg][shard][F] staging batch,
// and rebuilds the lost fragments there with one cec_reconstruct_batch (per-segment patterns).
// RCCL has no XOR reduction (rccl.h ncclRedOp_t), so survivors move by grouped point-to-point
// send/recv; every rank issues the moves in the same (segment, fragment) order, which is what
// pairs each send with its receive. Before any byte moves, the ranks agree (one 4-byte min
// all-reduce) that every rank found its local survivors and holds staging for the largest
// round, so a caller error fails on all ranks instead of leaving the others waiting in a receive.
// After that no rank leaves early: a local failure (a copy or rebuild that could not be enqueued)
// skips that rank's remaining local work but it still takes part in every round's transfers (its
// sources and staging are valid), and reports the error once all are enqueued. So the rounds are
// enqueued back to back with no host synchronisation between them: a round's transfers overlap
// the previous round's rebuild on the stream.
//
// RCCL is loaded at run time (dlopen): the rest of libcessec does not depend on it, and without
// it the cec_dist_* entry points return CEC_ENCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cess_ec.h"
#include "fftdec_plan.h"

namespace cec {
int set_error(int code, const std::string& msg);
}

namespace {

#define DI_TRY(expr)                                                                        \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return cec::set_error(_e == hipErrorOutOfMemory ? CEC_ENOMEM : CEC_EHIP,              \
                            std::string(#expr) + ": " + hipGetErrorString(_e));             \
  } while (0)

struct Rccl {
  bool ok = false;
  std::string why;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;  // optional
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      r.why = std::string("librccl not loadable: ") + dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      all &= fn != nullptr;
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.send, "ncclSend");
    sym(r.recv, "ncclRecv");
    sym(r.all_reduce, "ncclAllReduce");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.error_string, "ncclGetErrorString");
    r.ok = all;
    r.comm_abort = reinterpret_cast<decltype(&ncclCommAbort)>(dlsym(h, "ncclCommAbort"));
    if (!all) r.why = "librccl lacks an expected symbol";
  });
  return r;
}

int nccl_err(ncclResult_t res, const char* what) {
  return cec::set_error(CEC_ENCCL, std::string(what) + ": " + rccl().error_string(res));
}

#define NC_TRY(expr)                                 \
  do {                                               \
    ncclResult_t _r = (expr);                        \
    if (_r != ncclSuccess) return nccl_err(_r, #expr); \
  } while (0)

constexpr size_t kRound = 256;  // segments per round of a degraded read (staging bound)

int owner(uint64_t s, int f, int world) { return (int)((s + (uint64_t)f) % (uint64_t)world); }

struct Seg {
  uint64_t seg;
  std::vector<int> lost;  // sorted, distinct
  int decoder;
  std::vector<int> surv;  // the k survivors the rebuild reads (cec_survivors)
  bool partial = false;   // partial-product exchange: `holders` send one partial per lost
  std::vector<int> holders;  // ranks other than the decoder holding survivors, ascending
};

// Group the lost list by segment and apply the placement rule (shared by cec_dist_plan_ex and
// the degraded read, so the plan a caller inspects is the one that runs). exchange: 0 survivors,
// 1 partials, 2 per segment whichever moves fewer fragments (survivors on a tie).
int make_plan(int k, int m, int world, int exchange, const uint64_t* lost_seg,
              const uint8_t* lost_frag, size_t nlost, std::vector<Seg>* out) {
  if (k < 1 || m < 1 || k + m > 256 || world < 1 || (nlost && (!lost_seg || !lost_frag)))
    return cec::set_error(CEC_EINVAL, "dist plan: bad k, m, world or null lost list");
  if (exchange < 0 || exchange > 2) return cec::set_error(CEC_EINVAL, "dist plan: bad exchange");
  std::map<uint64_t, std::vector<int>> by;
  for (size_t i = 0; i < nlost; ++i) {
    if (lost_frag[i] >= k + m)
      return cec::set_error(CEC_EINVAL, "dist plan: lost fragment index " +
                                            std::to_string(lost_frag[i]) + " outside 0..k+m-1");
    by[lost_seg[i]].push_back(lost_frag[i]);
  }
  out->clear();
  for (auto& [s, v] : by) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    if ((int)v.size() > m)
      return cec::set_error(CEC_ETOOFEW, "dist plan: segment " + std::to_string(s) + " lost " +
                                             std::to_string(v.size()) + " > m fragments");
    Seg g{s, v, owner(s, v[0], world), {}};
    {
      uint8_t pres[256], sv[256];
      for (int f = 0; f < k + m; ++f) pres[f] = !std::binary_search(v.begin(), v.end(), f);
      int rc = cec_survivors(k, m, pres, sv);
      if (rc) return rc;
      g.surv.assign(sv, sv + k);
    }
    size_t n_surv = 0;
    for (int f : g.surv) {
      const int o = owner(s, f, world);
      if (o == g.decoder) continue;
      ++n_surv;
      if (!std::binary_search(g.holders.begin(), g.holders.end(), o))
        g.holders.insert(std::upper_bound(g.holders.begin(), g.holders.end(), o), o);
    }
    const size_t n_part = g.lost.size() * g.holders.size();
    g.partial = exchange == 1 || (exchange == 2 && n_part < n_surv);
    if (!g.partial) g.holders.clear();
    out->push_back(std::move(g));
  }
  return CEC_OK;
}

// Where the transfer groups of plan segments [r0, r1) start (plan positions, ascending, r0 first;
// r1 appended last): a new group begins before a segment whose transfers would take some rank past
// `group_ops` transfers in the current group (0: no bound). A segment's transfers never split.
// Every rank computes every rank's counts from the shared plan, so all cut alike.
void group_cuts(const std::vector<Seg>& plan, size_t r0, size_t r1, int world, int group_ops,
                std::vector<size_t>* cuts) {
  cuts->assign(1, r0);
  if (group_ops > 0) {
    std::vector<size_t> cnt(world, 0), one(world, 0);
    for (size_t i = r0; i < r1; ++i) {
      const Seg& g = plan[i];
      std::fill(one.begin(), one.end(), 0);
      if (g.partial) {
        for (int h : g.holders) {
          one[h] += g.lost.size();
          one[g.decoder] += g.lost.size();
        }
      } else {
        for (int f : g.surv) {
          const int o = owner(g.seg, f, world);
          if (o != g.decoder) {
            ++one[o];
            ++one[g.decoder];
          }
        }
      }
      bool over = false;
      for (int w = 0; w < world; ++w) over |= cnt[w] + one[w] > (size_t)group_ops;
      if (over && i > cuts->back()) {
        cuts->push_back(i);
        std::fill(cnt.begin(), cnt.end(), 0);
      }
      for (int w = 0; w < world; ++w) cnt[w] += one[w];
    }
  }
  cuts->push_back(r1);
}

}  // namespace

struct cec_dist {
  cec_codec* codec = nullptr;
  int k = 0, m = 0, device = 0, world = 0, rank = 0;
  int exchange = 2;  // CEC_DIST_OPT_EXCHANGE (auto: the cheaper exchange per segment)
  ncclComm_t comm = nullptr;
  uint8_t* stage = nullptr;  // staging batch: data [nseg_d][k][F], then parity [nseg_d][m][F]
  size_t stage_bytes = 0;
  // partial-product segments: their batch (same layout) and the decoder's partial rows
  // [holders + 1][pairs][F]
  uint8_t* pstage = nullptr;
  size_t pstage_bytes = 0;
  int* d_flag = nullptr;
  bool broken = false;  // the communicator was aborted after a failure inside a transfer group
  int test_abort_round = -1;  // CEC_DIST_OPT_TEST_ABORT: fail inside this round's transfer group
  int group_ops = 1024;       // CEC_DIST_OPT_GROUP_OPS: point-to-point ops per rank per group
  uint64_t groups = 0;        // transfer groups issued (cec_dist_groups)
  // Device memory is stream-ordered (hipMallocAsync / hipFreeAsync): hipFree performs an implicit
  // hipDeviceSynchronize, which would stall every other codec on the device. `done` is recorded on
  // the caller's stream at the end of every degraded read (its last enqueued work); destruction
  // waits for it alone and frees on the handle's own stream.
  hipStream_t own = nullptr;
  hipEvent_t done = nullptr;
  bool used = false;
};

namespace {
// Grow a device buffer on `st` (the caller's stream, ordered after the previous call's `done`).
int grow(uint8_t** buf, size_t* have, size_t need, hipStream_t st) {
  if (need <= *have) return CEC_OK;
  if (*buf) DI_TRY(hipFreeAsync(*buf, st));
  *buf = nullptr;
  *have = 0;
  DI_TRY(hipMallocAsync(reinterpret_cast<void**>(buf), need, st));
  *have = need;
  return CEC_OK;
}
}  // namespace

extern "C" {

int cec_survivors(int k, int m, const uint8_t* present, uint8_t* survivors) {
  if (!present || !survivors) return cec::set_error(CEC_EINVAL, "null");
  if (k < 1 || m < 1 || k + m > cec::kMaxShards)
    return cec::set_error(CEC_EINVAL, "need k >= 1, m >= 1, k + m <= 256");
  uint8_t flags[cec::kMaxShards], rd[cec::kMaxShards];
  for (int i = 0; i < k + m; ++i) flags[i] = present[i] ? 1 : 0;
  if (!cec::survivor_set(k, m, flags, rd))
    return cec::set_error(CEC_ETOOFEW, "fewer than k shards present");
  for (int i = 0, o = 0; i < k + m; ++i)
    if (rd[i]) survivors[o++] = (uint8_t)i;
  return CEC_OK;
}

int cec_dist_unique_id(uint8_t* id) {
  if (!id) return cec::set_error(CEC_EINVAL, "null id");
  const Rccl& r = rccl();
  if (!r.ok) return cec::set_error(CEC_ENCCL, r.why);
  ncclUniqueId u;
  NC_TRY(r.get_unique_id(&u));
  std::copy(u.internal, u.internal + NCCL_UNIQUE_ID_BYTES, reinterpret_cast<char*>(id));
  return CEC_OK;
}

int cec_dist_create(cec_codec* codec, const uint8_t* id, int world, int rank, cec_dist** out) {
  if (!codec || !id || !out || world < 1 || rank < 0 || rank >= world)
    return cec::set_error(CEC_EINVAL, "dist create: null argument or rank outside 0..world-1");
  static_assert(CEC_DIST_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
  const Rccl& r = rccl();
  if (!r.ok) return cec::set_error(CEC_ENCCL, r.why);
  auto* d = new cec_dist;
  d->codec = codec;
  d->world = world;
  d->rank = rank;
  cec_codec_info(codec, &d->k, &d->m, &d->device);
  ncclUniqueId u;
  std::copy(id, id + NCCL_UNIQUE_ID_BYTES, reinterpret_cast<uint8_t*>(u.internal));
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipError_t he = hipSetDevice(d->device);
  ncclResult_t res = he == hipSuccess ? r.comm_init_rank(&d->comm, world, u, rank) : ncclSuccess;
  if (he == hipSuccess && res == ncclSuccess)
    he = hipStreamCreateWithFlags(&d->own, hipStreamNonBlocking);
  if (he == hipSuccess && res == ncclSuccess)
    he = hipEventCreateWithFlags(&d->done, hipEventDisableTiming);
  if (he == hipSuccess && res == ncclSuccess)
    he = hipMallocAsync(reinterpret_cast<void**>(&d->d_flag), sizeof(int), d->own);
  if (he == hipSuccess && res == ncclSuccess) he = hipStreamSynchronize(d->own);
  if (he != hipSuccess || res != ncclSuccess) {
    int rc = he != hipSuccess ? cec::set_error(CEC_EHIP, std::string("dist create: ") +
                                                             hipGetErrorString(he))
                              : nccl_err(res, "ncclCommInitRank");
    if (d->comm) r.comm_destroy(d->comm);
    if (d->d_flag) (void)hipFreeAsync(d->d_flag, d->own);
    if (d->own) {
      (void)hipStreamSynchronize(d->own);
      (void)hipStreamDestroy(d->own);
    }
    if (d->done) (void)hipEventDestroy(d->done);
    (void)hipSetDevice(prev);
    delete d;
    return rc;
  }
  (void)hipSetDevice(prev);
  *out = d;
  return CEC_OK;
}

void cec_dist_destroy(cec_dist* d) {
  if (!d) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(d->device);
  // only this handle's work: the last degraded read's tail on its caller's stream (a failed call
  // may have left copies or transfers queued there); other streams of the device keep running
  if (d->used) (void)hipEventSynchronize(d->done);
  if (d->comm) rccl().comm_destroy(d->comm);
  if (d->stage) (void)hipFreeAsync(d->stage, d->own);
  if (d->pstage) (void)hipFreeAsync(d->pstage, d->own);
  if (d->d_flag) (void)hipFreeAsync(d->d_flag, d->own);
  (void)hipStreamSynchronize(d->own);
  (void)hipStreamDestroy(d->own);
  (void)hipEventDestroy(d->done);
  (void)hipSetDevice(prev);
  delete d;
}

int cec_dist_set_option(cec_dist* d, int option, int value) {
  if (!d) return cec::set_error(CEC_EINVAL, "null dist");
  if (option == CEC_DIST_OPT_EXCHANGE) {
    if (value < 0 || value > 2) return cec::set_error(CEC_EINVAL, "exchange must be 0, 1 or 2");
    d->exchange = value;
    return CEC_OK;
  }
  if (option == CEC_DIST_OPT_TEST_ABORT) {
    d->test_abort_round = value < 0 ? -1 : value;
    return CEC_OK;
  }
  if (option == CEC_DIST_OPT_GROUP_OPS) {
    if (value < 0) return cec::set_error(CEC_EINVAL, "group ops must be >= 0");
    d->group_ops = value;
    return CEC_OK;
  }
  return cec::set_error(CEC_EINVAL, "unknown dist option");
}

int cec_dist_groups(const cec_dist* d, uint64_t* groups) {
  if (!d || !groups) return cec::set_error(CEC_EINVAL, "null dist or output");
  *groups = d->groups;
  return CEC_OK;
}

int cec_dist_plan(int k, int m, int world, const uint64_t* lost_seg, const uint8_t* lost_frag,
                  size_t nlost, cec_dist_move* moves, size_t moves_cap, size_t* nmoves,
                  int32_t* decoder) {
  return cec_dist_plan_ex(k, m, world, 0, lost_seg, lost_frag, nlost, moves, moves_cap, nmoves,
                          decoder);
}

int cec_dist_plan_ex(int k, int m, int world, int exchange, const uint64_t* lost_seg,
                     const uint8_t* lost_frag, size_t nlost, cec_dist_move* moves,
                     size_t moves_cap, size_t* nmoves, int32_t* decoder) {
  std::vector<Seg> plan;
  int rc = make_plan(k, m, world, exchange, lost_seg, lost_frag, nlost, &plan);
  if (rc) return rc;
  size_t n = 0;
  for (const Seg& g : plan) {
    if (g.partial) {
      for (int h : g.holders)
        for (int f : g.lost) {
          if (moves && n < moves_cap)
            moves[n] = cec_dist_move{g.seg, f, h, g.decoder, CEC_DIST_PARTIAL};
          ++n;
        }
      continue;
    }
    for (int f : g.surv) {
      if (moves && n < moves_cap)
        moves[n] = cec_dist_move{g.seg, f, owner(g.seg, f, world), g.decoder, CEC_DIST_SURVIVOR};
      ++n;
    }
  }
  if (nmoves) *nmoves = n;
  if (decoder)
    for (size_t i = 0; i < nlost; ++i)
      decoder[i] = std::lower_bound(plan.begin(), plan.end(), lost_seg[i],
                                    [](const Seg& g, uint64_t s) { return g.seg < s; })
                       ->decoder;
  if (moves && n > moves_cap) return cec::set_error(CEC_EINVAL, "dist plan: moves_cap too small");
  return CEC_OK;
}

int cec_dist_plan_groups(int k, int m, int world, int exchange, int group_ops,
                         const uint64_t* lost_seg, const uint8_t* lost_frag, size_t nlost,
                         uint64_t* starts, size_t starts_cap, size_t* ngroups) {
  if (group_ops < 0) return cec::set_error(CEC_EINVAL, "group ops must be >= 0");
  std::vector<Seg> plan;
  int rc = make_plan(k, m, world, exchange, lost_seg, lost_frag, nlost, &plan);
  if (rc) return rc;
  size_t n = 0;
  std::vector<size_t> cuts;
  for (size_t r0 = 0; r0 < plan.size(); r0 += kRound) {
    group_cuts(plan, r0, std::min(plan.size(), r0 + kRound), world, group_ops, &cuts);
    for (size_t c = 0; c + 1 < cuts.size(); ++c) {
      if (starts && n < starts_cap) starts[n] = cuts[c];
      ++n;
    }
  }
  if (ngroups) *ngroups = n;
  if (starts && n > starts_cap) return cec::set_error(CEC_EINVAL, "plan groups: starts_cap too small");
  return CEC_OK;
}

int cec_dist_degraded_read(cec_dist* d, const uint64_t* lost_seg, const uint8_t* lost_frag,
                           size_t nlost, size_t shard_len, cec_locate_fn locate, void* user,
                           uint8_t* const* d_out, void* hip_stream, size_t* nrebuilt) {
  if (!d || !locate || shard_len == 0)
    return cec::set_error(CEC_EINVAL, "dist degraded read: null argument or zero shard_len");
  const Rccl& r = rccl();
  const int k = d->k, m = d->m, n = k + m, world = d->world, rank = d->rank;
  const size_t F = shard_len;
  std::vector<Seg> plan;
  int rc = make_plan(k, m, world, d->exchange, lost_seg, lost_frag, nlost, &plan);
  if (rc) return rc;  // every rank sees the same list, so every rank fails here alike

  // lost entries per segment, and this rank's checks: its survivors found, its outputs given
  std::map<uint64_t, std::vector<size_t>> entries;
  for (size_t i = 0; i < nlost; ++i) entries[lost_seg[i]].push_back(i);
  int ok = 1;
  std::string why;
  std::vector<const uint8_t*> src_ptr;  // survivors this rank holds, in plan order
  for (const Seg& g : plan) {
    for (int f : g.surv)
      if (owner(g.seg, f, world) == rank) {
        const uint8_t* p = locate(user, g.seg, f);
        if (!p && ok) {
          ok = 0;
          why = "locate returned NULL for fragment (" + std::to_string(g.seg) + ", " +
                std::to_string(f) + ") the placement assigns to rank " + std::to_string(rank);
        }
        src_ptr.push_back(p);
      }
    if (g.decoder == rank)
      for (size_t i : entries[g.seg])
        if ((!d_out || !d_out[i]) && ok) {
          ok = 0;
          why = "no output buffer for lost entry " + std::to_string(i) + ", rebuilt on this rank";
        }
  }

  int prev = 0;
  (void)hipGetDevice(&prev);
  DI_TRY(hipSetDevice(d->device));
  struct Restore {
    int dev;
    ~Restore() { (void)hipSetDevice(dev); }
  } restore{prev};
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  if (d->broken) return cec::set_error(CEC_ENCCL, "dist degraded read: group aborted earlier");
  // after the previous call's tail (it may have run on another stream), and `done` recorded after
  // whatever this call enqueues, on every return path
  if (d->used) DI_TRY(hipStreamWaitEvent(st, d->done, 0));
  struct Tail {
    cec_dist* d;
    hipStream_t st;
    ~Tail() { d->used = hipEventRecord(d->done, st) == hipSuccess || d->used; }
  } tail{d, st};

  // Rounds of at most kRound segments of the plan (the same split on every rank) bound the
  // staging; rounds follow each other on the stream, so a round's receives land after the
  // previous round's rebuild has read the staging.
  struct Round {
    // survivor segments this rank rebuilds; partial segments it decodes or holds survivors of
    std::vector<const Seg*> mine, pmine;
    std::map<uint64_t, size_t> row, prow;
    size_t npairs = 0, H = 0;
    std::map<std::pair<uint64_t, int>, size_t> pair;  // (segment, lost fragment) -> acc row
  };
  auto classify = [&](size_t r0, size_t r1) {
    Round R;
    for (size_t i = r0; i < r1; ++i) {
      const Seg& g = plan[i];
      if (!g.partial) {
        if (g.decoder == rank) {
          R.row[g.seg] = R.mine.size();
          R.mine.push_back(&g);
        }
        continue;
      }
      const bool holder = std::binary_search(g.holders.begin(), g.holders.end(), rank);
      if (g.decoder != rank && !holder) continue;
      R.prow[g.seg] = R.pmine.size();
      R.pmine.push_back(&g);
      if (g.decoder == rank) {
        R.H = std::max(R.H, g.holders.size());
        for (int f : g.lost) R.pair[{g.seg, f}] = R.npairs++;
      }
    }
    return R;
  };
  // Staging for the largest round, allocated before the ranks agree: an allocation failure is
  // then one rank's `ok = 0`, not a return while its peers wait in a receive.
  if (ok) {
    size_t need = 0, pneed = 0;
    for (size_t r0 = 0; r0 < plan.size(); r0 += kRound) {
      const Round R = classify(r0, std::min(plan.size(), r0 + kRound));
      need = std::max(need, R.mine.size() * (size_t)n * F);
      pneed = std::max(pneed, R.pmine.size() * (size_t)n * F + (R.H + 1) * R.npairs * F);
    }
    int grc = grow(&d->stage, &d->stage_bytes, need, st);
    if (!grc) grc = grow(&d->pstage, &d->pstage_bytes, pneed, st);
    if (grc) {
      ok = 0;
      why = std::string("staging allocation: ") + cec_last_error();
    }
  }

  // min over ranks of a success flag; every rank calls it at the same points
  auto agree = [&](int mine_ok, int* all_ok) -> int {
    DI_TRY(hipMemcpyAsync(d->d_flag, &mine_ok, sizeof(int), hipMemcpyHostToDevice, st));
    NC_TRY(r.all_reduce(d->d_flag, d->d_flag, 1, ncclInt32, ncclMin, d->comm, st));
    DI_TRY(hipMemcpyAsync(all_ok, d->d_flag, sizeof(int), hipMemcpyDeviceToHost, st));
    DI_TRY(hipStreamSynchronize(st));
    return CEC_OK;
  };
  // agree before any byte moves
  int all_ok = 0;
  rc = agree(ok, &all_ok);
  if (rc) return rc;
  if (!ok) return cec::set_error(CEC_EINVAL, "dist degraded read: " + why);
  if (!all_ok)
    return cec::set_error(CEC_EINVAL, "dist degraded read: another rank failed its checks");

  // A local failure after the agreement (a copy, the partial rebuild, the rebuild after a round)
  // is held in `lrc`: the rank skips its remaining local work but keeps issuing every round's
  // transfers, so no peer waits for it, and returns the error at the end. An error inside a
  // transfer group aborts the communicator (peers get an RCCL error instead of waiting for this
  // rank).
  int lrc = CEC_OK;
  std::string lwhy;
  auto local = [&](int code) {
    if (code && !lrc) {
      lrc = code;
      lwhy = cec_last_error();
    }
    return code == CEC_OK;
  };
  auto hip_ok = [&](hipError_t e, const char* what) {
    return local(e == hipSuccess ? CEC_OK
                                 : cec::set_error(e == hipErrorOutOfMemory ? CEC_ENOMEM : CEC_EHIP,
                                                  std::string(what) + ": " +
                                                      hipGetErrorString(e)));
  };
  size_t rebuilt = 0, si = 0;
  for (size_t r0 = 0; r0 < plan.size(); r0 += kRound) {
    const size_t r1 = std::min(plan.size(), r0 + kRound);
    Round R = classify(r0, r1);
    auto& mine = R.mine;
    auto& pmine = R.pmine;
    const size_t npairs = R.npairs, H = R.H;
    const size_t pbatch = pmine.size() * (size_t)n * F, acc_row = npairs * F;
    uint8_t* const st_data = d->stage;
    uint8_t* const st_par = d->stage + mine.size() * (size_t)k * F;
    uint8_t* const p_data = d->pstage;
    uint8_t* const p_par = d->pstage + pmine.size() * (size_t)k * F;
    uint8_t* const acc = d->pstage + pbatch;
    auto slot = [&](uint64_t s, int f) {
      return f < k ? st_data + (R.row.at(s) * (size_t)k + f) * F
                   : st_par + (R.row.at(s) * (size_t)m + (f - k)) * F;
    };
    auto pslot = [&](uint64_t s, int f) {
      return f < k ? p_data + (R.prow.at(s) * (size_t)k + f) * F
                   : p_par + (R.prow.at(s) * (size_t)m + (f - k)) * F;
    };
    // local survivors into the survivor staging (decoder) or the partial batch (held), and
    // this rank's survivors of the round in plan order for the sends
    std::vector<uint8_t> ppres(pmine.size() * n, 0), pheld(pmine.size() * n, 0);
    std::vector<const uint8_t*> round_src;
    for (size_t i = r0; i < r1; ++i) {
      const Seg& g = plan[i];
      const bool pm = g.partial && R.prow.count(g.seg);
      if (pm)  // every fragment not lost: the rebuild writes the lost ones only
        for (int f = 0; f < n; ++f)
          ppres[R.prow[g.seg] * n + f] = !std::binary_search(g.lost.begin(), g.lost.end(), f);
      for (int f : g.surv) {
        if (owner(g.seg, f, world) != rank) continue;
        const uint8_t* p = src_ptr[si++];
        round_src.push_back(p);
        if (lrc) continue;
        if (pm) {
          pheld[R.prow[g.seg] * n + f] = 1;
          hip_ok(hipMemcpyAsync(pslot(g.seg, f), p, F, hipMemcpyDeviceToDevice, st), "copy");
        } else if (!g.partial && g.decoder == rank) {
          hip_ok(hipMemcpyAsync(slot(g.seg, f), p, F, hipMemcpyDeviceToDevice, st), "copy");
        }
      }
    }
    if (!pmine.empty() && !lrc &&
        local(cec_reconstruct_partial_batch(d->codec, p_data, p_par, pmine.size(), F,
                                            ppres.data(), pheld.data(), 0, st))) {
      for (const auto& [key, i] : R.pair)
        if (!hip_ok(hipMemcpyAsync(acc + i * F, pslot(key.first, key.second), F,
                                   hipMemcpyDeviceToDevice, st), "copy"))
          break;
      bool ragged = false;
      for (const Seg* g : pmine) ragged |= g->decoder == rank && g->holders.size() < H;
      if (ragged && !lrc) hip_ok(hipMemsetAsync(acc + acc_row, 0, H * acc_row, st), "memset");
    }
    // Transfer groups of at most d->group_ops point-to-point ops on any one rank
    // (CEC_DIST_OPT_GROUP_OPS; a wide code's round is up to ~7k ops otherwise): the round's
    // segments are cut at the same plan positions on every rank (each computes every rank's counts
    // from the shared plan), so a group holds both ends of each of its transfers and no group
    // waits on another rank's later group. Within a group: survivor moves, then partials, each in
    // plan order (which pairs every send with its receive on the peer). The groups follow each
    // other on the stream with no host synchronisation.
    std::vector<size_t> cuts;
    group_cuts(plan, r0, r1, world, d->group_ops, &cuts);
    size_t rj = 0;
    auto fail = [&](ncclResult_t res, const char* what) {
      // end the half-built group (this thread's group state is then clean; what was enqueued is
      // launched), then abort the communicator so those transfers and the peers' pending ones
      // fail instead of waiting for the ones this rank never issued
      const int code = nccl_err(res, what);
      (void)r.group_end();
      if (r.comm_abort) r.comm_abort(d->comm);
      d->comm = nullptr;
      d->broken = true;
      return code;
    };
    auto pit = pmine.begin();
    for (size_t c = 0; c + 1 < cuts.size(); ++c) {
      const size_t c0 = cuts[c], c1 = cuts[c + 1];
      NC_TRY(r.group_start());
      if (c == 0 && d->test_abort_round == (int)(r0 / kRound))
        return fail(ncclInternalError, "test abort (CEC_DIST_OPT_TEST_ABORT)");
      for (size_t i = c0; i < c1; ++i) {
        const Seg& g = plan[i];
        for (int f : g.surv) {
          const int src = owner(g.seg, f, world);
          if (src == rank) {
            const uint8_t* p = round_src[rj++];
            if (!g.partial && g.decoder != rank) {
              ncclResult_t res = r.send(p, F, ncclUint8, g.decoder, d->comm, st);
              if (res != ncclSuccess) return fail(res, "ncclSend");
            }
          } else if (!g.partial && g.decoder == rank) {
            ncclResult_t res = r.recv(slot(g.seg, f), F, ncclUint8, src, d->comm, st);
            if (res != ncclSuccess) return fail(res, "ncclRecv");
          }
        }
      }
      for (; pit != pmine.end() && (size_t)(*pit - plan.data()) < c1; ++pit) {
        const Seg* g = *pit;
        if (g->decoder == rank) {
          for (size_t h = 0; h < g->holders.size(); ++h)
            for (int f : g->lost) {
              ncclResult_t res = r.recv(acc + (h + 1) * acc_row + R.pair.at({g->seg, f}) * F, F,
                                        ncclUint8, g->holders[h], d->comm, st);
              if (res != ncclSuccess) return fail(res, "ncclRecv");
            }
        } else {
          for (int f : g->lost) {
            ncclResult_t res = r.send(pslot(g->seg, f), F, ncclUint8, g->decoder, d->comm, st);
            if (res != ncclSuccess) return fail(res, "ncclSend");
          }
        }
      }
      ncclResult_t res = r.group_end();
      if (res != ncclSuccess) return fail(res, "ncclGroupEnd");
      ++d->groups;
    }
    if (!mine.empty()) {
      // every fragment not lost is flagged present (the codec reads its k survivors, the gathered
      // survivors): the rebuild writes only the lost fragments, not the unused survivors
      std::vector<uint8_t> present(mine.size() * n, 0);
      for (size_t i = 0; i < mine.size(); ++i)
        for (int f = 0; f < n; ++f)
          present[i * n + f] = !std::binary_search(mine[i]->lost.begin(), mine[i]->lost.end(), f);
      if (local(cec_reconstruct_batch(d->codec, st_data, st_par, mine.size(), F, present.data(),
                                      1, 0, st)))
        for (const Seg* g : mine)
          for (size_t i : entries[g->seg]) {
            if (!hip_ok(hipMemcpyAsync(d_out[i], slot(g->seg, lost_frag[i]), F,
                                       hipMemcpyDeviceToDevice, st), "copy"))
              break;
            ++rebuilt;
          }
    }
    if (npairs && !lrc) {
      if (!H || local(cec_xor_batch(acc, acc + acc_row, H, acc_row, acc_row, st)))
        for (const Seg* g : pmine)
          if (g->decoder == rank)
            for (size_t i : entries[g->seg]) {
              if (!hip_ok(hipMemcpyAsync(d_out[i], acc + R.pair.at({g->seg, (int)lost_frag[i]}) * F,
                                         F, hipMemcpyDeviceToDevice, st), "copy"))
                break;
              ++rebuilt;
            }
    }
  }
  // a failure after the last round's transfers leaves no peer waiting
  if (lrc) return cec::set_error(lrc, "dist degraded read: " + lwhy);
  DI_TRY(hipStreamSynchronize(st));
  if (nrebuilt) *nrebuilt = rebuilt;
  return CEC_OK;
}

}  // extern "C"
