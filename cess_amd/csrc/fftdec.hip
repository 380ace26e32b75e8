// RS(32,32) erasure decode on the additive FFT (k_fftdec_m), for gfx950: rebuilds of many lost
// fragments of a wide-coded segment (a miner exit marks every fragment it held,
// c-pallets/file-bank/src/functions.rs:543-562), where the run-time matrix kernels (k_rthx) are
// scalar-issue bound.
//
// Algorithm (plans: fftdec_plan.h). Coset A's present shards are read with its erased set D
// zeroed; T1 = IFFT_A then FFT_B (the encode transform of fft.hip, 160 butterflies per byte
// column) gives q = f_q on coset B. At the plan's |D| present rows R of B the syndromes
// s = p ^ q are the values there of h = f - f_q, a polynomial vanishing on A \ D; every output is
// a GF(2^8)-linear function of s (erased B outputs add their own q). Those run-time rows are
// applied in bit-plane form with per-segment masks from HBM (scalar loads): the two positions of a
// lane-pair slot are first packed into the nibble halves of each plane (lane 0 keeps its
// columns 0-15, lane 1 its columns 16-31, of both positions), so a mask word carries the
// coefficient bits of both positions and every lane applies the same SGPR mask. A row is applied by
// Horner over its coefficient bits (out = 2 out ^ T_b, T_b = XOR of the syndromes whose coefficient
// has bit b): one v_bitop3 per (plane, bit) and slot, 8 scalar masks per (row, slot), 2 VALU per
// byte per (output, syndrome pair) plus 3 per output and bit for the doubling. The R slots are
// first swapped to the front of the register array (uniform branches, once per column block), so
// the row loop is compiled per slot count with no branch inside. Cost: T1 + the transposes (~4 VALU
// per byte of 64 shards) + 64 x outputs x syndrome slots per lane pair.
//
// Layout of the work as k_fft3232 (fft_core.h): one lane pair per 32 byte columns of a segment,
// blockIdx.y = a segment of the launch's list with its own plan, shard_len % 1024 == 0.
#include <utility>

#include "fft_core.h"
#include "fftdec_plan.h"
#include "kernels.h"

// occupancy experiments: -DCEC_FD_WAVES=n asks the compiler for n waves per SIMD
#ifdef CEC_FD_WAVES
#define CEC_FD_ATTR __attribute__((amdgpu_waves_per_eu(CEC_FD_WAVES, CEC_FD_WAVES)))
#else
#define CEC_FD_ATTR
#endif

namespace cec {

using namespace fftc;

namespace {

// The plan lives in HBM and is read through the scalar cache (constant address space: uniform
// s_load, the masks go straight into SGPRs as v_bitop3 operands instead of VGPRs).
typedef const __attribute__((address_space(4))) uint32_t* cplan_t;

// Loads that may be switched off per lane go through a raw buffer resource: an out-of-range
// offset returns zeros without touching memory, so an erased shard is "loaded" as zeros with no
// divergent branch (and no HBM traffic). Offsets are 32-bit: 32 shards of one coset must span
// < 2 GiB (checked by the launcher).
constexpr uint32_t kOff = 0x80000000u;  // out of range: reads zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, 0x7FFFFFFF,
                                           0x00020000);
}
// voffset: the lane's part (or kOff), soffset: the uniform part (an SGPR)
__device__ __forceinline__ void bld32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                      uint32_t (&w)[8]) {
  const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 2);  // nt
  const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, voff + 512, soff, 2);
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// every plane of a slot materialised here (an empty asm that reads and writes them)
__device__ __forceinline__ void fence(uint32_t (&x)[8]) {
  asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
               "+v"(x[6]), "+v"(x[7]));
}

// Lane pair slot J (positions 2J, 2J + 1) -> nibble-packed: both lanes hold both positions for
// their half of the columns (lane 0: columns of dwords 0-3 = the low nibble of every plane byte,
// lane 1: dwords 4-7 = the high nibble), the even position in the low nibble, the odd in the high.
// Each lane reads its partner's plane (DPP straight from the register, no wait states) and rotates
// it (rot: 28 on lane 0, the partner's low nibbles go up; 4 on lane 1, its high nibbles go down)
// into the half it does not keep.
template <bool SWZ>
__device__ __forceinline__ void pack_slot(uint32_t (&x)[8], uint32_t keep, uint32_t rot) {
  sfor<8>([&](auto Q) CEC_FFT_AI {
    const uint32_t p = partner_x<SWZ>(x[Q]);
    const uint32_t y = __builtin_amdgcn_alignbit(p, p, rot);
    x[Q] = FFT_BOP3(keep, x[Q], y, kSel);
  });
}

// The first LR syndrome slots' rows are fetched at the start into LDS (buffer loads to LDS, 2 x
// 1 KiB per slot and wave), so they land while the transform runs instead of being waited for after
// it. Two kernels by syndrome slot count (the plan's nrs): up to kSmallNr slots in at most 168
// VGPRs with LR = 4 (32 KiB per workgroup: three waves per SIMD), more slots at two waves per SIMD
// with LR = 8 (64 KiB).
constexpr int kSmallNr = 4;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef const __attribute__((address_space(3))) u32x4 lds_u32x4;

// SWZ: which pair exchanges go through the LDS crossbar (bit 0 the IFFT's layer 0, bit 1 the FFT's
// layer 0 on the slots read, bit 2 the nibble packs), the others through DPP
// SKIP: a lane-pair slot of coset A with neither position read (both erased: zeros loaded) skips
// its transpose (zero in, zero out)
template <unsigned SIDE, int NLO, int NHI, int LR, int SWZ, bool SKIP>
__device__ __forceinline__ void dec_m_cols(const Layout& L, uint32_t seg, uint64_t col,
                                           cplan_t P, lds_u32* lw) {
  constexpr unsigned BA = SIDE ? 32u : 0u, BB = SIDE ? 0u : 32u;
  const uint32_t l = threadIdx.x & 1;
  const uint32_t em = l ? 0u : 0xFFFFFFFFu, om = ~em;
  uint8_t* const dat = L.data + seg * L.data_seg_stride;
  uint8_t* const par = L.parity + seg * L.par_seg_stride;
  uint8_t* const baseA = SIDE ? par : dat;
  uint8_t* const baseB = SIDE ? dat : par;
  const auto rA = rsrc(baseA), rB = rsrc(baseB);
  const uint32_t ss = (uint32_t)L.shard_stride;
  const uint32_t lcol = (uint32_t)col + l * ss;  // this lane's byte offset of position 0 / 1
  const uint32_t vst = (uint32_t)col + l * 512;   // its 16 bytes of an output row (packed form)
  const uint32_t presA = P[FftDecLayout::kPresA];
  const uint32_t nout = P[FftDecLayout::kNout];

  uint32_t X[16][8];
  // coset A, erased shards zeroed (out-of-range loads: no memory traffic), then bit-sliced
  sfor<16>([&](auto J) CEC_FFT_AI {
    bld32(rA, (presA >> (2 * J + l)) & 1 ? lcol : kOff, 2 * J * ss, X[J]);
  });
  // the syndrome rows of the first LR R slots into this wave's LDS area (lane k's 16 bytes of a
  // piece land at 16 k: each lane reads back only what it loaded)
  const uint32_t nrs = P[FftDecLayout::kNrs];
  const uint32_t npre = nrs < (uint32_t)LR ? nrs : (uint32_t)LR;
  for (uint32_t i = 0; i < npre; ++i) {
    const uint32_t rs = P[FftDecLayout::kRsl + i];
    const uint32_t voff = (rs >> (8 + l)) & 1 ? lcol : kOff;
    const uint32_t soff = 2 * (rs & 15) * ss;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_u32*)(lw + i * 512), 16, voff, soff, 0, 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_u32*)(lw + i * 512 + 256), 16, voff + 512,
                                             soff, 0, 2);
  }
  sfor<16>([&](auto J) CEC_FFT_AI {
    if (!SKIP || ((presA >> (2 * J)) & 3)) tr8(X[J]);
  });
  ifft32<BA, (SWZ & 1) != 0>(X, em);
  // q on coset B; its last layer only on the slots whose q is read (syndrome rows R, erased
  // outputs of B: the plan's kPslots, numbered before the swaps below)
  fft32_upper<BB>(X);
  sfor<16>([&](auto J) CEC_FFT_AI { fence(X[J]); });
  const uint32_t pslots = P[FftDecLayout::kPslots];
  sfor<16>([&](auto J) CEC_FFT_AI {
    if constexpr (J > 0) asm volatile("" : "+v"(X[J][0]) : "v"(X[J - 1][7]));
    if ((pslots >> J) & 1) fft32_l0<BB, J, (SWZ & 2) != 0>(X[J], em, om);
  });
  // X is complete here: the phases below start from it (keeps the compiler from interleaving the
  // transform's tail with them, which costs registers)
  sfor<16>([&](auto J) CEC_FFT_AI { fence(X[J]); });
  // R slots to the front: step i swaps register slots i and j_i (the plan's swap list)
  sfor<15>([&](auto I) CEC_FFT_AI {
    if (I < nrs) {
      const uint32_t jm = P[FftDecLayout::kSwap + I];  // 1 << j_i
      sfor<15 - I>([&](auto D) CEC_FFT_AI {
        constexpr int J = I + 1 + D;
        // bit tests, not ji == J: an equality chain becomes a switch whose cases LLVM merges into
        // one swap with X indexed at run time (X then lives in scratch)
        if ((jm >> J) & 1) {
          asm volatile("");
          sfor<8>([&](auto Q) CEC_FFT_AI { std::swap(X[I][Q], X[J][Q]); });
        }
      });
    }
  });
  const uint32_t keep = l ? 0xF0F0F0F0u : 0x0F0F0F0Fu;
  const uint32_t rot = l ? 4u : 28u;  // pack_slot rotates the partner's plane: by the partner's amount
  const uint32_t npk = P[FftDecLayout::kNpk];
  auto outputs = [&](auto N) CEC_FFT_AI {
    constexpr int NR = decltype(N)::value;
    // syndromes s = p ^ q in register slots [0, NR): the R rows of B (an erased or unused position
    // of a slot loads zeros), from LDS for the first LR slots; past them slot i's load address
    // waits on slot i - 3 (three slots of loads in flight beyond X).
    if constexpr (NR > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS rows
    const uint32_t lane = threadIdx.x & 63;
    sfor<NR>([&](auto I) CEC_FFT_AI {
      uint32_t Y[8];
      if constexpr (I < LR) {
        // a lane whose position is not an R row loaded out of range: the LDS DMA then writes
        // nothing, so its bytes there are stale and are masked to zero here
        const uint32_t rs = P[FftDecLayout::kRsl + I];
        const uint32_t keepm = 0u - ((rs >> (8 + l)) & 1);
        const u32x4 a = *reinterpret_cast<lds_u32x4*>(lw + I * 512 + lane * 4);
        const u32x4 b = *reinterpret_cast<lds_u32x4*>(lw + I * 512 + 256 + lane * 4);
        Y[0] = a.x & keepm; Y[1] = a.y & keepm; Y[2] = a.z & keepm; Y[3] = a.w & keepm;
        Y[4] = b.x & keepm; Y[5] = b.y & keepm; Y[6] = b.z & keepm; Y[7] = b.w & keepm;
      } else {
        const uint32_t rs = P[FftDecLayout::kRsl + I];  // j_i | R bits of the slot << 8
        uint32_t voff = (rs >> (8 + l)) & 1 ? lcol : kOff;
        asm volatile("" : "+v"(voff) : "v"(X[I - 3][7]));
        bld32(rB, voff, 2 * (rs & 15) * ss, Y);
      }
      tr8(Y);
      sfor<8>([&](auto Q) CEC_FFT_AI { X[I][Q] ^= Y[Q]; });
    });
    // nibble-pack the R slots and the slots holding an erased B output's q, one slot after the
    // other (interleaved, the packs of 16 slots hold twice the registers)
    sfor<NR>([&](auto I) CEC_FFT_AI {
      if constexpr (I > 0)
        asm volatile("" : "+v"(X[I][0]), "+v"(X[I][1]), "+v"(X[I][2]), "+v"(X[I][3]),
                     "+v"(X[I][4]), "+v"(X[I][5]), "+v"(X[I][6]), "+v"(X[I][7])
                     : "v"(X[I - 1][7]));
      pack_slot<(SWZ & 4) != 0>(X[I], keep, rot);
    });
    sfor<16 - NR>([&](auto D) CEC_FFT_AI {
      constexpr int J = NR + D;
      if ((npk >> J) & 1) {
        asm volatile("");  // a branch, not a select over every slot
        pack_slot<(SWZ & 4) != 0>(X[J], keep, rot);
      }
    });
    for (uint32_t o = 0; o < nout; ++o) {
      const uint32_t od = P[FftDecLayout::kOuts + o];
      const uint32_t t = od & 31, qm = od >> 16;  // qm = 1 << (slot of q)
      const cplan_t mk = P + FftDecLayout::kMasks + o * (8 * NR);
      uint32_t acc[8] = {};
      // a step's masks are loaded once the step two before it is done (one step of prefetch): at
      // 16 slots all 128 masks of a row up front would not fit the SGPRs
      uint32_t dep1 = 0, dep2 = 0;
      if constexpr (NR > 0) sfor<8>([&](auto B) CEC_FFT_AI {
        constexpr int b = 7 - B;
        cplan_t mb = mk + b * NR;
        if constexpr (B >= 2) asm volatile("" : "+s"(mb) : "v"(dep2));
        if constexpr (b == 7) {
          sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = X[0][Q] & mb[0]; });
        } else {  // acc = 2 acc (planes: 0 <- 7, q <- q - 1, 2..4 also ^= 7; poly 0x11D)
          const uint32_t a7 = acc[7];
          sfor<7>([&](auto Q) CEC_FFT_AI { acc[7 - Q] = acc[6 - Q]; });
          acc[0] = a7;
          acc[2] ^= a7;
          acc[3] ^= a7;
          acc[4] ^= a7;
          sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = FFT_BOP3(acc[Q], X[0][Q], mb[0], kXand); });
        }
        sfor<NR - 1>([&](auto I) CEC_FFT_AI {
          sfor<8>([&](auto Q) CEC_FFT_AI {
            acc[Q] = FFT_BOP3(acc[Q], X[I + 1][Q], mb[I + 1], kXand);
          });
        });
        dep2 = dep1;
        dep1 = acc[7];
      });
      if (od & 32) {  // an erased shard of B: add its q
        const uint32_t nib = (t & 1) ? 0xF0F0F0F0u : 0x0F0F0F0Fu;
        sfor<16>([&](auto J) CEC_FFT_AI {
          if ((qm >> J) & 1) sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = FFT_BOP3(acc[Q], X[J][Q], nib, kXand); });
        });
      }
      // both positions' contributions to the lane's 16 columns, in the low nibbles; back to bytes
      uint32_t w[8];
      sfor<8>([&](auto Q) CEC_FFT_AI { w[Q] = FFT_BOP3(acc[Q], acc[Q] >> 4, 0x0F0F0F0Fu, kAndX); });
      tr8(w);
      // a buffer store: the shard offset is scalar, the lane's column offset the same every row
      const u32x4 v = {w[0], w[1], w[2], w[3]};
      if (od & 32)
        __builtin_amdgcn_raw_buffer_store_b128(v, rB, vst, t * ss, 2);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, rA, vst, t * ss, 2);
    }
  };
  // one row loop per slot count (NLO..NHI), selected by a bit test of the one-hot count (an equality
  // chain becomes a switch, and LLVM then sinks the variants' common tails into one block whose
  // registers are the union of all of them)
  const uint32_t nrs1 = P[FftDecLayout::kNrs1];
  sfor<NHI + 1 - NLO>([&](auto N0) CEC_FFT_AI {
    constexpr int N = NLO + N0;
    if ((nrs1 >> N) & 1) outputs(std::integral_constant<int, N>{});
  });
}

// plans: per listed segment (y) its plan, or `plan1` for every segment. BIG: plans with more than
// kSmallNr syndrome slots (the host sorts them, fftdec_big). SWZ: the exchanges through the LDS
// crossbar (dec_m_cols). The product's: DPP everywhere (kFdmSwz = 0); the IFFT's exchange through
// the crossbar is no faster one form per process (profiles/r04/swz_standalone_runs.jsonl), the
// nibble packs through it take the small class past 168 VGPRs.
constexpr int kFdmSwz = 0;
template <unsigned SIDE, bool BIG, int SWZ, bool SKIP = true>
__global__ __launch_bounds__(256) CEC_FD_ATTR void k_fftdec_m(Layout L, const uint32_t* __restrict__ plan1,
                                                  const uint32_t* const* __restrict__ plans,
                                                  const uint32_t* __restrict__ seg_list,
                                                  uint32_t seg0) {
  constexpr int NLO = BIG ? kSmallNr + 1 : 0, NHI = BIG ? 16 : kSmallNr, LR = BIG ? 8 : kSmallNr;
  const uint32_t y = seg0 + blockIdx.y;
  const uint32_t seg = seg_list ? seg_list[y] : y;
  const uint32_t* P = plans ? plans[y] : plan1;
  const uint64_t gp = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 1;  // lane pair
  const uint64_t col = (gp >> 5) * 1024 + (gp & 31) * 16;
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * LR * 512];
  if (col >= L.len) return;  // whole waves leave together
  dec_m_cols<SIDE, NLO, NHI, LR, SWZ, SKIP>(L, seg, col, (cplan_t)P,
                                 (lds_u32*)(lds + (threadIdx.x >> 6) * (LR * 512)));
}

}  // namespace

bool fftdec_big(int nrs) { return nrs > kSmallNr; }

bool fftdec_layout_ok(const Layout& L) {
  const uintptr_t bits = (uintptr_t)L.data | (uintptr_t)L.parity | L.shard_stride |
                         L.data_seg_stride | L.par_seg_stride;
  return !(bits & 15) && !(L.len & 1023) && L.len != 0 && L.k == 32 &&
         L.shard_stride < (uint64_t(1) << 26);  // 32-bit buffer offsets over a coset
}

bool launch_fftdec(const Layout& L, int side, bool big, const uint32_t* plan1,
                   const uint32_t* const* plans, const uint32_t* seg_list, uint32_t nseg,
                   hipStream_t st, int form) {
  if (!fftdec_layout_ok(L) || (side != 0 && side != 1)) return false;
  const uint64_t gx = (L.len / 32 * 2 + 255) / 256;
  auto kern = side ? (big ? k_fftdec_m<1, true, kFdmSwz> : k_fftdec_m<1, false, kFdmSwz>)
                   : (big ? k_fftdec_m<0, true, kFdmSwz> : k_fftdec_m<0, false, kFdmSwz>);
#ifdef CEC_TUNING
  auto pick = [&](auto S) {
    constexpr int M = decltype(S)::value;
    kern = side ? (big ? k_fftdec_m<1, true, M> : k_fftdec_m<1, false, M>)
                : (big ? k_fftdec_m<0, true, M> : k_fftdec_m<0, false, M>);
  };
  switch (form) {  // form = 1 + the SWZ mask
    case 1: pick(std::integral_constant<int, 0>{}); break;
    case 2: pick(std::integral_constant<int, 1>{}); break;
    case 4: pick(std::integral_constant<int, 3>{}); break;
    case 6: pick(std::integral_constant<int, 5>{}); break;
    case 8: pick(std::integral_constant<int, 7>{}); break;
    case 10:  // the product's without the skip of unread slots
      kern = side ? (big ? k_fftdec_m<1, true, 0, false> : k_fftdec_m<1, false, 0, false>)
                  : (big ? k_fftdec_m<0, true, 0, false> : k_fftdec_m<0, false, 0, false>);
      break;
    default: break;
  }
#else
  (void)form;
#endif
  for (uint32_t s0 = 0; s0 < nseg; s0 += 65535) {
    const uint32_t ny = nseg - s0 < 65535 ? nseg - s0 : 65535;
    hipLaunchKernelGGL(kern, dim3((unsigned)gx, ny), dim3(256), 0, st, L, plan1, plans, seg_list,
                       s0);
  }
  return true;
}

}  // namespace cec
