// libcessec host side: the C ABI of include/cess_ec.h over the HIP kernels in kernels.hip.
//
// Owns, per codec: the (k+m) x k encode matrix (gf256.h), the run-time coefficient programs in
// HBM (encode + one per erasure pattern, cached), a HIP stream and a staging area in HBM for the
// host-buffer API. Multi-GPU sharding lives above this library (one codec per device).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/cess_ec.h"
#include "gf256.h"
#include "kernels.h"

namespace cec {
void set_ct_variant(int v);
void set_sha_mode(int v);
void set_rt_mode(int v);
void set_tick_prefetch(int v);
}

namespace {

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

// A run-time program: chunks of up to kRtMaxOut outputs, each a device block in the layout of
// kernels.h (header, input indices, output indices, coefficients [nin][nob]).
struct RtChunk {
  uint32_t* dev = nullptr;
  int nin = 0, nout = 0, nob = 0;
};

struct Program {
  std::vector<RtChunk> chunks;
  int nout = 0;     // total outputs
  int single = -1;  // the one missing shard when exactly one output (compile-time decode)
  uint8_t in_idx[cec::kMaxShards] = {};   // survivors read (host copy)
  uint8_t out_idx[cec::kMaxShards] = {};  // shards written (host copy)
};

void free_program(Program& p) {
  for (auto& c : p.chunks)
    if (c.dev) (void)hipFree(c.dev);
  p.chunks.clear();
}

// Upload coefficient rows for outputs out_idx[o] (coef[o][j]) as run-time chunks.
int build_program(const uint8_t* in_idx, int nin, const uint8_t* out_idx, int nout,
                  const BigMat& coef, Program& prog) {
  prog.nout = nout;
  prog.single = nout == 1 ? out_idx[0] : -1;
  std::memcpy(prog.in_idx, in_idx, nin);
  std::memcpy(prog.out_idx, out_idx, nout);
  for (int o0 = 0; o0 < nout; o0 += cec::kRtMaxOut) {
    RtChunk c;
    c.nin = nin;
    c.nout = std::min(cec::kRtMaxOut, nout - o0);
    c.nob = cec::rt_bucket(c.nout);
    std::vector<uint32_t> h(cec::rt_chunk_bytes(nin, c.nob) / sizeof(uint32_t), 0u);
    h[0] = (uint32_t)nin;
    h[1] = (uint32_t)c.nout;
    h[2] = (uint32_t)c.nob;
    for (int j = 0; j < nin; ++j) h[4 + j] = in_idx[j];
    for (int o = 0; o < c.nout; ++o) h[4 + 256 + o] = out_idx[o0 + o];
    uint32_t* hb = h.data() + 4 + 512;
    uint32_t* mk = h.data() + cec::kRtHeaderWords;
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
      uint32_t* top = h.data() + hoff;
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
    HIP_TRY(hipMalloc(&c.dev, h.size() * sizeof(uint32_t)));
    prog.chunks.push_back(c);
    HIP_TRY(hipMemcpy(c.dev, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  }
  return CEC_OK;
}

// One multi-pattern run-time launch of the per-segment reconstruct path.
struct PsLaunch {
  int nob = 0, nin = 0;
  size_t off = 0, count = 0;  // into the cached segment-list / chunk-pointer arrays
};

}  // namespace

struct cec_codec {
  int k = 0, m = 0, device = 0;
  std::unique_ptr<BigMat> E;
  hipStream_t stream = nullptr;
  Program encode;
  std::unordered_map<std::string, Program> decode_cache;
  bool force_generic = false;
  // staging for the host-buffer API: [n][stride]
  uint8_t* stage = nullptr;
  size_t stage_bytes = 0;
  // cached plan of the last per-segment reconstruct call: either compile-time launches per
  // pattern (ps_ct: pattern key, offset, count into ps_list) or multi-pattern run-time
  // launches (ps_rt: segment list + per-segment chunk pointers)
  std::string ps_key;
  bool ps_valid = false;
  uint32_t* ps_list = nullptr;
  size_t ps_list_bytes = 0;
  uint8_t* ps_ptrs = nullptr;  // const uint32_t* [count] per launch
  size_t ps_ptrs_bytes = 0;
  std::vector<std::pair<std::string, std::pair<size_t, size_t>>> ps_ct;
  std::vector<PsLaunch> ps_rt;
  // RS(2,1), every segment a single erasure: offset/count of the tagged list (segment |
  // erased << 30) in ps_list for one mixed-pattern launch (count 0: none)
  size_t ps_mixed_off = 0, ps_mixed_count = 0;

  ~cec_codec() {
    (void)hipSetDevice(device);
    free_program(encode);
    for (auto& kv : decode_cache) free_program(kv.second);
    if (stage) (void)hipFree(stage);
    if (ps_list) (void)hipFree(ps_list);
    if (ps_ptrs) (void)hipFree(ps_ptrs);
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

void launch_chunk(const Layout& L, const uint32_t* chunk, const uint32_t* const* per_seg,
                  int nin, int nob, const uint32_t* seg_list, uint32_t nseg, hipStream_t st) {
  if (nin <= cec::kRthMaxIn && cec::launch_matvec_rth(L, chunk, per_seg, nin, seg_list, nseg, st))
    return;
  cec::launch_matvec_rt(L, chunk, per_seg, nob, seg_list, nseg, st);
}

void run_program(const Program& p, const Layout& L, const uint32_t* seg_list, uint32_t nseg,
                 hipStream_t st) {
  for (const auto& c : p.chunks) launch_chunk(L, c.dev, nullptr, c.nin, c.nob, seg_list, nseg, st);
}

int check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(CEC_EHIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return CEC_OK;
}

int do_encode(cec_codec* c, const Layout& L, const uint32_t* seg_list, uint32_t nseg,
              hipStream_t st) {
  if (nseg == 0 || L.len == 0) return CEC_OK;
  if (c->force_generic || !cec::launch_encode_ct(c->k, c->m, L, seg_list, nseg, st))
    run_program(c->encode, L, seg_list, nseg, st);
  return check_launch();
}

// Decode program for one erasure pattern (cached).
int get_decode(cec_codec* c, const uint8_t* present, bool data_only, const Program** out) {
  const int n = c->k + c->m;
  std::string key(n + 1, '\0');
  for (int i = 0; i < n; ++i) key[i] = present[i] ? 1 : 0;
  key[n] = data_only ? 1 : 0;
  auto it = c->decode_cache.find(key);
  if (it != c->decode_cache.end()) {
    *out = &it->second;
    return CEC_OK;
  }
  auto plan = std::make_unique<BigPlan>();
  auto sub = std::make_unique<BigMat>();
  auto inv = std::make_unique<BigMat>();
  auto work = std::make_unique<WorkMat>();
  uint8_t flags[cec::kMaxShards];
  for (int i = 0; i < n; ++i) flags[i] = key[i];
  if (cec::gf_decode_plan(c->k, c->m, flags, data_only, *c->E, *plan, *sub, *inv, *work) != 0)
    return set_err(CEC_ETOOFEW, "fewer than k shards present");
  if (c->decode_cache.size() >= 4096) {
    // Drain users of the cached device coefficients before freeing them.
    (void)hipDeviceSynchronize();
    for (auto& kv : c->decode_cache) free_program(kv.second);
    c->decode_cache.clear();
    c->ps_valid = false;  // its chunk pointers referred to the freed programs
  }
  Program prog;
  if (plan->nout > 0) {
    int rc = build_program(plan->in_idx, c->k, plan->out_idx, plan->nout, plan->coef, prog);
    if (rc) {
      free_program(prog);
      return rc;
    }
  }
  auto res = c->decode_cache.emplace(key, std::move(prog));
  *out = &res.first->second;
  return CEC_OK;
}

int do_decode(cec_codec* c, const Program& p, const Layout& L, const uint32_t* seg_list,
              uint32_t nseg, hipStream_t st) {
  if (p.nout == 0 || nseg == 0 || L.len == 0) return CEC_OK;
  if (c->force_generic || p.single < 0 ||
      !cec::launch_decode_ct(c->k, c->m, p.single, L, seg_list, nseg, st))
    run_program(p, L, seg_list, nseg, st);
  return check_launch();
}

int ensure(uint8_t** buf, size_t* have, size_t need) {
  if (*have >= need) return CEC_OK;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *have = 0;
  HIP_TRY(hipMalloc(buf, need));
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

}  // namespace

namespace cec {
// error reporting shared with hashq.cpp (same thread-local detail string)
int set_error(int code, const std::string& msg) { return set_err(code, msg); }
}  // namespace cec

extern "C" {

const char* cec_version(void) { return "cessec 0.1.0 gfx950"; }

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
  {
    auto par = std::make_unique<BigMat>();
    uint8_t in_idx[cec::kMaxShards], out_idx[cec::kMaxShards];
    for (int j = 0; j < k; ++j) in_idx[j] = (uint8_t)j;
    for (int o = 0; o < m; ++o) {
      out_idx[o] = (uint8_t)(k + o);
      for (int j = 0; j < k; ++j) par->v[o][j] = c->E->v[k + o][j];
    }
    int rc = build_program(in_idx, k, out_idx, m, *par, c->encode);
    if (rc) return rc;
  }
  *out = c.release();
  return CEC_OK;
}

void cec_destroy(cec_codec* codec) { delete codec; }

int cec_matrix(const cec_codec* c, uint8_t* out) {
  if (!c || !out) return set_err(CEC_EINVAL, "null");
  for (int r = 0; r < c->k + c->m; ++r)
    for (int j = 0; j < c->k; ++j) out[r * c->k + j] = c->E->v[r][j];
  return CEC_OK;
}

int cec_set_option(cec_codec* c, int option, int value) {
  switch (option) {
    case CEC_OPT_FORCE_GENERIC:
      if (!c) return set_err(CEC_EINVAL, "null codec");
      c->force_generic = value != 0;
      return CEC_OK;
    case CEC_OPT_CT_VARIANT:
      if (value < -1 || value > 31) return set_err(CEC_EINVAL, "variant out of range");
      cec::set_ct_variant(value);
      return CEC_OK;
    case CEC_OPT_SHA_MODE:
      if (value < 0 || value > 2) return set_err(CEC_EINVAL, "sha mode out of range");
      cec::set_sha_mode(value);
      return CEC_OK;
    case CEC_OPT_RT_MODE:
      if (value < 0 || value > 2) return set_err(CEC_EINVAL, "rt mode out of range");
      cec::set_rt_mode(value);
      return CEC_OK;
    case CEC_OPT_TICK_PREFETCH:
      if (value < 0 || value > 3) return set_err(CEC_EINVAL, "tick variant must be 0..3");
      cec::set_tick_prefetch(value);
      return CEC_OK;
  }
  return set_err(CEC_EINVAL, "unknown option");
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
  if (!per_segment) {
    const Program* p = nullptr;
    int rc = get_decode(c, present, data_only != 0, &p);
    if (rc) return rc;
    return do_decode(c, *p, L, nullptr, (uint32_t)nseg, st);
  }
  // Per-segment patterns. Segments are grouped by pattern once and the grouping is cached for a
  // repeated pattern array (degraded-read bench and repair loops pass the same map each call).
  //  * every pattern has a compile-time single-erasure kernel (RS(2,1)): one launch per
  //    pattern over its segment list;
  //  * otherwise: one multi-pattern run-time launch per (chunk index, bucket), each segment's
  //    workgroup row reading its own pattern's chunk, so a batch where every segment has a
  //    different erasure map is still one full-grid launch.
  std::string pkey(reinterpret_cast<const char*>(present), nseg * n);
  for (auto& ch : pkey) ch = ch ? 1 : 0;
  pkey.push_back(data_only ? 1 : 0);
  pkey.push_back(c->force_generic ? 1 : 0);
  if (c->ps_key != pkey || !c->ps_valid) {
    c->ps_valid = false;
    c->ps_ct.clear();
    c->ps_rt.clear();
    c->ps_mixed_count = 0;
    std::unordered_map<std::string, std::vector<uint32_t>> groups;
    for (size_t s = 0; s < nseg; ++s) groups[pkey.substr(s * n, n)].push_back((uint32_t)s);
    bool all_ct = !c->force_generic;
    std::vector<std::pair<const Program*, const std::vector<uint32_t>*>> progs;
    for (auto& g : groups) {
      const Program* p = nullptr;
      int rc = get_decode(c, reinterpret_cast<const uint8_t*>(g.first.data()), data_only != 0, &p);
      if (rc) return rc;
      if (!p->nout) continue;
      progs.push_back({p, &g.second});
      if (p->single < 0 || !cec::has_decode_ct(c->k, c->m, p->single)) all_ct = false;
    }
    std::vector<uint32_t> hl;
    std::vector<const uint32_t*> hp;
    if (all_ct) {
      std::vector<uint32_t> tagged;
      for (auto& g : groups) {
        const Program* p = nullptr;
        get_decode(c, reinterpret_cast<const uint8_t*>(g.first.data()), data_only != 0, &p);
        if (!p->nout) continue;
        c->ps_ct.push_back({g.first, {hl.size(), g.second.size()}});
        hl.insert(hl.end(), g.second.begin(), g.second.end());
        for (uint32_t sg : g.second) tagged.push_back(sg | ((uint32_t)p->single << 30));
      }
      if (c->k == 2 && c->m == 1 && c->ps_ct.size() > 1 && nseg < (1u << 30)) {
        std::sort(tagged.begin(), tagged.end(),
                  [](uint32_t a, uint32_t b) { return (a & 0x3FFFFFFFu) < (b & 0x3FFFFFFFu); });
        c->ps_mixed_off = hl.size();
        c->ps_mixed_count = tagged.size();
        hl.insert(hl.end(), tagged.begin(), tagged.end());
      }
    } else {
      size_t maxchunks = 0;
      for (auto& pr : progs) maxchunks = std::max(maxchunks, pr.first->chunks.size());
      for (size_t ci = 0; ci < maxchunks; ++ci) {
        std::unordered_map<int, std::vector<std::pair<uint32_t, const uint32_t*>>> byb;
        int nin_max = 0;
        for (auto& pr : progs)
          if (ci < pr.first->chunks.size()) {
            nin_max = std::max(nin_max, pr.first->chunks[ci].nin);
            for (uint32_t sg : *pr.second)
              byb[pr.first->chunks[ci].nob].push_back({sg, pr.first->chunks[ci].dev});
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
          c->ps_rt.push_back(l);
        }
      }
    }
    int rc = ensure(reinterpret_cast<uint8_t**>(&c->ps_list), &c->ps_list_bytes,
                    std::max<size_t>(hl.size(), 1) * sizeof(uint32_t));
    if (rc) return rc;
    rc = ensure(&c->ps_ptrs, &c->ps_ptrs_bytes, std::max<size_t>(hp.size(), 1) * sizeof(void*));
    if (rc) return rc;
    if (!hl.empty())
      HIP_TRY(hipMemcpy(c->ps_list, hl.data(), hl.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    if (!hp.empty())
      HIP_TRY(hipMemcpy(c->ps_ptrs, hp.data(), hp.size() * sizeof(void*), hipMemcpyHostToDevice));
    c->ps_key = std::move(pkey);
    c->ps_valid = true;
  }
  if (c->ps_mixed_count &&
      cec::launch_decode1_mixed(c->k, c->m, L, c->ps_list + c->ps_mixed_off,
                                (uint32_t)c->ps_mixed_count, st))
    return check_launch();
  for (const auto& w : c->ps_ct) {
    const Program* p = nullptr;
    int rc = get_decode(c, reinterpret_cast<const uint8_t*>(w.first.data()), data_only != 0, &p);
    if (rc) return rc;
    rc = do_decode(c, *p, L, c->ps_list + w.second.first, (uint32_t)w.second.second, st);
    if (rc) return rc;
  }
  const uint32_t* const* ptrs = reinterpret_cast<const uint32_t* const*>(c->ps_ptrs);
  for (const auto& l : c->ps_rt) {
    launch_chunk(L, nullptr, ptrs + l.off, l.nin, l.nob, c->ps_list + l.off, (uint32_t)l.count,
                 st);
    int rc = check_launch();
    if (rc) return rc;
  }
  return CEC_OK;
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
  cec::launch_sha256_hex(nullptr, &L, nsh, (uint64_t)nseg * nsh, shard_len, d_hex,
                         pick_stream(c, hip_stream));
  return check_launch();
}

int cec_sha256_hex(const uint8_t* const* d_bufs, size_t n, size_t len, uint8_t* hex,
                   void* hip_stream) {
  if (!hex || (n && !d_bufs)) return set_err(CEC_EINVAL, "null");
  if (n == 0) return CEC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
  const uint8_t** dptrs = nullptr;
  uint8_t* dhex = nullptr;
  HIP_TRY(hipMalloc(&dptrs, n * sizeof(void*)));
  hipError_t e = hipMalloc(&dhex, n * 64);
  if (e != hipSuccess) {
    (void)hipFree(dptrs);
    return set_err(CEC_ENOMEM, "hex buffer");
  }
  int rc = CEC_OK;
  do {
    if ((e = hipMemcpyAsync(dptrs, d_bufs, n * sizeof(void*), hipMemcpyHostToDevice, st))) break;
    cec::launch_sha256_hex(dptrs, nullptr, 1, n, len, dhex, st);
    if ((e = hipGetLastError())) break;
    if ((e = hipMemcpyAsync(hex, dhex, n * 64, hipMemcpyDeviceToHost, st))) break;
    e = hipStreamSynchronize(st);
  } while (0);
  if (e != hipSuccess) rc = set_err(CEC_EHIP, std::string("sha256: ") + hipGetErrorString(e));
  (void)hipFree(dptrs);
  (void)hipFree(dhex);
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

// ---- host-buffer API -------------------------------------------------------------------

int cec_encode(cec_codec* c, uint8_t* const* shards, size_t shard_len) {
  if (!c || !shards) return set_err(CEC_EINVAL, "null");
  if (shard_len == 0) return set_err(CEC_ESHARDLEN, "zero shard length");
  const int n = c->k + c->m;
  for (int i = 0; i < n; ++i)
    if (!shards[i]) return set_err(CEC_EINVAL, "null shard");
  HIP_TRY(hipSetDevice(c->device));
  const size_t stride = pad256(shard_len);
  int rc = ensure(&c->stage, &c->stage_bytes, stride * n);
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
  const Program* p = nullptr;
  int rc = get_decode(c, present, data_only != 0, &p);
  if (rc) return rc;
  if (p->nout == 0) return CEC_OK;
  for (int i = 0; i < n; ++i)
    if (!shards[i]) return set_err(CEC_EINVAL, "null shard");
  const size_t stride = pad256(shard_len);
  rc = ensure(&c->stage, &c->stage_bytes, stride * n);
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
  int rc = ensure(&c->stage, &c->stage_bytes, stride * n);
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
