// Host-side launch interface of the HIP kernels in kernels.hip (internal to libcessec).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cec {

// Where shard `i` of segment `s` lives in HBM. The batched device layout of the C ABI is
// [seg][shard][len] for data and for parity, i.e. for i < k:
//   data   + s * data_seg_stride + i * shard_stride
// and for i >= k:
//   parity + s * par_seg_stride + (i - k) * shard_stride.
struct Layout {
  uint8_t* data;
  uint8_t* parity;
  uint64_t len;              // bytes per shard
  uint64_t shard_stride;     // bytes between consecutive shards of one segment
  uint64_t data_seg_stride;  // bytes between consecutive segments in `data`
  uint64_t par_seg_stride;   // bytes between consecutive segments in `parity`
  int k;
};

// One run-time-coefficient program chunk in HBM: up to kRtMaxOut outputs from `nin` inputs.
// Layout (all uint32): header {nin, nout, nob, 0}, in[256], out[256], hb[256] (highest set
// coefficient bit of input column j, -1 for a zero column), then masks[nin][8][nob]:
// masks[j][b][o] = 0xFFFFFFFF when bit b of coef[o][j] is set (zero padded to the bucket nob).
// When nin <= kRthMaxIn, header[3] is the word offset of a Horner section used by the
// Horner-over-input-groups kernel (k_rth): top[32] (highest set coefficient bit of output row
// o, 0xFFFFFFFF for a zero row), then idx[32][8][8]: idx[o][b][g] = the 4-bit combination of
// input group g (inputs 4g..4g+3) whose coefficients in row o have bit b set.
constexpr int kRtMaxOut = 32;
constexpr int kRthMaxIn = 32;
constexpr size_t kRtHeaderWords = 4 + 256 + 256 + 256;
constexpr size_t kRthWords = 32 + 32 * 8 * 8;
inline size_t rt_chunk_bytes(int nin, int nob) {
  return (kRtHeaderWords + (size_t)nin * 8 * nob + (nin <= kRthMaxIn ? kRthWords : 0)) *
         sizeof(uint32_t);
}

// True when every shard start and the shard length allow 16-byte vector access.
bool layout_vec16_ok(const Layout& L);

// Kernel selection of one codec (cec_set_option). Held per codec, passed to every launcher: no
// process-wide state, so distinct codecs on distinct threads stay independent.
struct KernelOpts {
  int ct_variant = -1;  // compile-time kernel variant: -1 = default; others only in tuning
                        // builds (libcessec_tune.so, -DCEC_TUNING)
  int rt_mode = 0;      // run-time kernel: 0 Horner + index-mode XORs (4..32 inputs), 1 per-bit
                        // masks, 2 Horner + v_mov table reads, 3 bit-plane accumulators for
                        // chunks of <= 4 outputs (k_rtb)
  int sha_mode = 0;     // one-shot SHA-256: 0 auto, 1 one wave, 2 two waves per 64 buffers
};
// Highest ct_variant this build instantiates (0 in the product library: default only).
int max_ct_variant();

// Compile-time-coefficient kernels. Return false if no specialised kernel exists for the
// request (caller then uses the run-time kernel).
bool launch_encode_ct(const KernelOpts& o, int k, int m, const Layout& L,
                      const uint32_t* seg_list, uint32_t nseg, hipStream_t st);
// Decode for a single erasure of RS(k, m) codes that have a specialised plan; `missing` is the
// erased shard index and `data_only` drops a parity output.
bool launch_decode_ct(const KernelOpts& o, int k, int m, int missing, const Layout& L,
                      const uint32_t* seg_list, uint32_t nseg, hipStream_t st);
// RS(2,1) single erasures, a different one per segment, in one launch: tagged[i] = segment |
// (erased index << 30) for the nseg segments of the launch. False if not applicable.
// tuning variant 90 (libcessec_tune.so only; false elsewhere): erasures in the kernel arguments
bool launch_decode1_mixed_kargs(int k, int m, const Layout& L, const uint8_t* erased,
                                uint32_t nseg, hipStream_t st);
bool launch_decode1_mixed(const KernelOpts& o, int k, int m, const Layout& L,
                          const uint32_t* tagged, uint32_t nseg, hipStream_t st);

// Verify fused with the recompute (RS(2,1), RS(32,32)): ok[s] = 0 where the stored parity differs
// (ok preset by the caller). False (nothing launched) for other codes or layouts.
bool launch_verify_ct(int k, int m, const Layout& L, uint8_t* ok, uint32_t nseg, hipStream_t st);

// RS(32,32) encode as an additive FFT on bit-sliced data (fft.hip). False (nothing launched)
// when the layout does not fit (shard_len % 1024, 16-byte alignment).
bool launch_fft_rs3232(const Layout& L, const uint32_t* seg_list, uint32_t nseg, int nt,
                       hipStream_t st);

// RS(32,32) verify by the same transform, compared with the stored parity (ok preset by the
// caller; ok[s] = 0 where segment s differs). False (nothing launched) where the layout does not fit.
bool launch_fft_rs3232_verify(const Layout& L, uint8_t* ok, uint32_t nseg, hipStream_t st);

// RS(32,32) erasure decode on the additive FFT (fftdec.hip) with plans of fftdec_plan.h: every
// segment uses `plan1`, or listed segment y uses plans[y] (all of the launch's plans take the same
// side and the same size class, fftdec_big of their syndrome slot count). False (nothing launched)
// when the layout does not fit (fftdec_layout_ok).
bool fftdec_layout_ok(const Layout& L);
bool fftdec_big(int nrs);
// form 0: the product's (every pair exchange through DPP); tuning build only: 1 + a mask of the
// exchanges through the LDS crossbar (bit 0 the IFFT's, 1 the FFT's last layer, 2 the nibble packs),
// 10 the product's without the skip of unread input slots.
bool launch_fftdec(const Layout& L, int side, bool big, const uint32_t* plan1,
                   const uint32_t* const* plans, const uint32_t* seg_list, uint32_t nseg,
                   hipStream_t st, int form = 0);
// The formal-derivative decoder (fftdec_d.hip, plans of fftdec_plan_d): same arguments, any side.
// form 0: one 512-column block per wave (k_fftdec_d, the product's). Tuning build only: 1 the
// persistent kernel that merges a block's output multiplication with the next block's input
// multiplication (k_fftdec_dp), 3 the same with wave priorities by remaining work (DESIGN.md §4:
// 9 % fewer VALU per block, slower overall), 4..10 k_fftdec_d with other masks of the phases whose
// quad exchanges go through the LDS crossbar (ds_swizzle) instead of DPP (fftdec_d.hip kFddSwz),
// 11 the product's without the skip of unread input slots.
bool launch_fftdec_d(const Layout& L, const uint32_t* plan1, const uint32_t* const* plans,
                     const uint32_t* seg_list, uint32_t nseg, hipStream_t st, int form = 0);

// Whether a compile-time single-erasure decode kernel exists for (k, m, missing).
bool has_decode_ct(int k, int m, int missing);

// Bucketed output count the run-time kernel is instantiated for (>= nout).
int rt_bucket(int nout);
// Run-time coefficient GF matvec: out[r] = XOR_j coef[j][r] * in[j]. Either every segment uses
// the chunk `chunk`, or listed segment y uses per_seg[y] (all chunks of one launch share the
// bucket `nob`). Chunks are device memory laid out as described at RtChunk above.
void launch_matvec_rt(const Layout& L, const uint32_t* chunk, const uint32_t* const* per_seg,
                      int nob, const uint32_t* seg_list, uint32_t nseg, hipStream_t st);
// Same product by bit-plane accumulators (k_rtb) for chunks of nob <= 4 outputs; false (nothing
// launched) for a wider bucket.
bool launch_matvec_rtb(const Layout& L, const uint32_t* chunk, const uint32_t* const* per_seg,
                       int nob, const uint32_t* seg_list, uint32_t nseg, hipStream_t st,
                       int variant = -1);
// Same product from the chunks' Horner sections (every chunk of the launch has nin <= nin_max
// <= kRthMaxIn). Returns false (nothing launched) if the form is disabled by the variant knob.
bool launch_matvec_rth(const KernelOpts& o, const Layout& L, const uint32_t* chunk,
                       const uint32_t* const* per_seg, int nin_max, const uint32_t* seg_list,
                       uint32_t nseg, hipStream_t st);

// SHA-256 of `n` equal-length buffers, written as 64 lowercase hex characters each into
// `hex_out` (device, n * 64 bytes). If `ptrs` is null, buffer i is shard (i % nshards) of
// segment (i / nshards) in layout L.
void launch_sha256_hex(int sha_mode, const uint8_t* const* ptrs, const Layout* L, int nshards,
                       uint64_t n, uint64_t len, uint8_t* hex_out, hipStream_t st);

// One chain of the streaming SHA-256 queue (hashq.cpp), 128 bytes in HBM. `blk` counts the
// 64-byte blocks already compressed into `h`, padding blocks included; the chain is complete
// when blk == (len >> 6) + ((len & 63) >= 56 ? 2 : 1), and its hex (if `hex` is set) is written
// by the launch that completes it. Prefix digest: when `pre_blk` > 0 the chain also writes the
// SHA-256 hex of its first pre_blk * 64 bytes to `pre_hex`, from a copy of `h` taken right after
// block pre_blk - 1 and one padding block (a segment's chain gives its first fragment's hash).
struct ShaChain {
  const uint8_t* src;
  uint64_t len;
  uint64_t blk;
  uint8_t* hex;
  uint32_t h[8];
  uint8_t* pre_hex;
  uint64_t pre_blk;
  uint32_t pre_h[8];  // state after pre_blk blocks, parked by the one-wave tick until its loop ends
  uint64_t pad_[2];
};
static_assert(sizeof(ShaChain) == 128, "ShaChain is one 128-byte record");

__host__ __device__ inline uint64_t sha256_blocks(uint64_t len) { return (len >> 6) + ((len & 63) >= 56 ? 2 : 1); }

// Initialise n chains in slots slot0.. of the ring `tab` (capacity mask + 1, a power of two).
// pre_blk > 0: chain i also writes the hex of its first pre_blk blocks to
// pre_hex + ((i / per) * pre_hex_outer + i % per) * 64.
void launch_hashq_add(ShaChain* tab, uint32_t mask, uint64_t slot0, uint32_t n,
                      const uint8_t* base, uint32_t per, uint64_t outer, uint64_t inner,
                      uint64_t len, uint8_t* hex, uint64_t hex_outer, uint64_t pre_blk,
                      uint8_t* pre_hex, uint64_t pre_hex_outer, hipStream_t st,
                      const uint32_t* h0 = nullptr, uint64_t blk0 = 0);
// Advance the n chains in slots head.. by at most max_blocks blocks each; tick_mode 0 lets `live`
// (chains not yet complete among them) pick the kernel form, 1 or 2 = two waves with that many
// blocks prefetched, 3 = one wave per 64 chains.
void launch_sha256_tick(int tick_mode, ShaChain* tab, uint32_t mask, uint64_t head, uint32_t n,
                        uint32_t max_blocks, uint64_t live, hipStream_t st);

// Audit chunk gather (audit.hip): chunk idx[j] (chunk_len bytes) of fragment f, fragments in
// batch order (f = seg * nshards + shard, shards of layout L), to out[(f * nidx + j) * chunk_len].
void launch_chunk_gather(const Layout& L, int nshards, uint64_t nfrag, const uint32_t* d_idx,
                         uint32_t nidx, uint64_t chunk_len, uint8_t* out, hipStream_t st);

// XOR reduction (xor.hip): dst[0..len) ^= src[j * stride ..][0..len) for j < nsrc.
void launch_xor_reduce(uint8_t* dst, const uint8_t* src, uint32_t nsrc, uint64_t stride,
                       uint64_t len, hipStream_t st);

// ok[s] = 0 for every segment s whose seg_bytes of a and b differ (ok preset by the caller).
void launch_cmp_segments(const uint8_t* a, const uint8_t* b, uint64_t seg_bytes, uint64_t nseg,
                         uint8_t* ok, hipStream_t st);

// Synthetic segment bytes: 64-bit word w of segment s = splitmix64(seed ^ (s << 32) ^ w),
// little-endian; segments are seg_bytes long and contiguous from `out`.
void launch_fill_splitmix(uint8_t* out, uint64_t seg_bytes, uint64_t nseg, uint64_t seg0,
                          uint64_t seed, hipStream_t st);

}  // namespace cec
