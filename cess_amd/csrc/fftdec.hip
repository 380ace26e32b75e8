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
// coefficient bits of both positions and every lane applies the same SGPR mask: one v_bitop3 per
// (plane, plane) pair and slot, 2 VALU per byte per (output, syndrome pair). Cost: T1 + the
// transposes (~4 VALU per byte of 64 shards) + 64 x outputs x syndrome slots per lane pair.
//
// Layout of the work as k_fft3232 (fft_core.h): one lane pair per 32 byte columns of a segment,
// blockIdx.y = a segment of the launch's list with its own plan, shard_len % 1024 == 0.
#include "fft_core.h"
#include "fftdec_plan.h"
#include "kernels.h"

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
// Lane 0 sends its high nibbles down, lane 1 its low nibbles up: a rotate by 4 / 28 (the wrapped
// bits land in the half the receiver keeps from its own register).
__device__ __forceinline__ void pack_slot(uint32_t (&x)[8], uint32_t keep, uint32_t rot) {
  sfor<8>([&](auto Q) CEC_FFT_AI {
    const uint32_t send = __builtin_amdgcn_alignbit(x[Q], x[Q], rot);
    x[Q] = FFT_BOP3(keep, x[Q], partner(send), kSel);
  });
}

template <unsigned SIDE>
__device__ __forceinline__ void dec_m_cols(const Layout& L, uint32_t seg, uint64_t col,
                                           cplan_t P) {
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
  const uint32_t presA = P[FftDecLayout::kPresA], R = P[FftDecLayout::kR];
  const uint32_t nout = P[FftDecLayout::kNout], rslots = P[FftDecLayout::kRslots];
  const uint32_t pslots = P[FftDecLayout::kPslots];

  uint32_t X[16][8];
  // coset A, erased shards zeroed (out-of-range loads: no memory traffic), then bit-sliced
  sfor<16>([&](auto J) CEC_FFT_AI {
    bld32(rA, (presA >> (2 * J + l)) & 1 ? lcol : kOff, 2 * J * ss, X[J]);
  });
  sfor<16>([&](auto J) CEC_FFT_AI { tr8(X[J]); });
  ifft32<BA>(X, em);
  fft32<BB>(X, em, om);  // q on coset B
  // X is complete here: the phases below start from it (keeps the compiler from interleaving the
  // transform's tail with them, which costs registers)
  sfor<16>([&](auto J) CEC_FFT_AI { fence(X[J]); });
  // syndromes s = p ^ q at the R rows. A slot's load address waits on the slot four before it
  // (four slots of loads in flight beyond X) and the first ones on the transform's end, so no
  // load is hoisted above the transform or speculated out of its slot's branch.
  sfor<16>([&](auto J) CEC_FFT_AI {
    if ((R >> (2 * J)) & 3) {
      uint32_t voff = (R >> (2 * J + l)) & 1 ? lcol : kOff;
      if constexpr (J < 4)
        asm volatile("" : "+v"(voff) : "v"(X[15][7]), "v"(X[14][7]));
      else
        asm volatile("" : "+v"(voff) : "v"(X[J - 4][7]));
      uint32_t Y[8];
      bld32(rB, voff, 2 * J * ss, Y);
      tr8(Y);
      sfor<8>([&](auto Q) CEC_FFT_AI { X[J][Q] ^= Y[Q]; });
    }
  });
  const uint32_t keep = l ? 0xF0F0F0F0u : 0x0F0F0F0Fu;
  const uint32_t rot = l ? 28u : 4u;
  sfor<16>([&](auto J) CEC_FFT_AI {
    if ((pslots >> J) & 1) {
      asm volatile("");  // a branch, not a select over every slot
      pack_slot(X[J], keep, rot);
    }
  });
  cplan_t mp = P + FftDecLayout::kMasks;
  for (uint32_t o = 0; o < nout; ++o) {
    const uint32_t od = P[FftDecLayout::kOuts + o];
    const uint32_t t = od & 31;
    uint32_t acc[8];
    sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = 0; });
    if (od & 32) {  // an erased shard of B: its q, then the syndrome rows
      const uint32_t nib = (t & 1) ? 0xF0F0F0F0u : 0x0F0F0F0Fu;
      sfor<16>([&](auto J) CEC_FFT_AI {
        if ((t >> 1) == J) sfor<8>([&](auto Q) CEC_FFT_AI { acc[Q] = X[J][Q] & nib; });
      });
    }
    sfor<16>([&](auto J) CEC_FFT_AI {
      if ((rslots >> J) & 1) {
        sfor<8>([&](auto Q) CEC_FFT_AI {
          sfor<8>([&](auto Pp) CEC_FFT_AI {
            acc[Q] = FFT_BOP3(acc[Q], X[J][Pp], mp[Q * 8 + Pp], kXand);
          });
        });
        mp += 64;
      }
    });
    // both positions' contributions to the lane's 16 columns, in the low nibbles; back to bytes
    uint32_t w[8];
    sfor<8>([&](auto Q) CEC_FFT_AI { w[Q] = FFT_BOP3(acc[Q], acc[Q] >> 4, 0x0F0F0F0Fu, kAndX); });
    tr8(w);
    uint8_t* dst = ((od & 32) ? baseB : baseA) + col + (uint64_t)t * ss + l * 512;
    __builtin_nontemporal_store(u32x4{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4*>(dst));
  }
}

// plans: per listed segment (y) its plan, or `plan1` for every segment
template <unsigned SIDE>
__global__ __launch_bounds__(256) void k_fftdec_m(Layout L, const uint32_t* __restrict__ plan1,
                                                  const uint32_t* const* __restrict__ plans,
                                                  const uint32_t* __restrict__ seg_list,
                                                  uint32_t seg0) {
  const uint32_t y = seg0 + blockIdx.y;
  const uint32_t seg = seg_list ? seg_list[y] : y;
  const uint32_t* P = plans ? plans[y] : plan1;
  const uint64_t gp = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 1;  // lane pair
  const uint64_t col = (gp >> 5) * 1024 + (gp & 31) * 16;
  if (col >= L.len) return;  // whole waves leave together
  dec_m_cols<SIDE>(L, seg, col, (cplan_t)P);
}

}  // namespace

bool fftdec_layout_ok(const Layout& L) {
  const uintptr_t bits = (uintptr_t)L.data | (uintptr_t)L.parity | L.shard_stride |
                         L.data_seg_stride | L.par_seg_stride;
  return !(bits & 15) && !(L.len & 1023) && L.len != 0 && L.k == 32 &&
         L.shard_stride < (uint64_t(1) << 26);  // 32-bit buffer offsets over a coset
}

bool launch_fftdec(const Layout& L, int side, const uint32_t* plan1,
                   const uint32_t* const* plans, const uint32_t* seg_list, uint32_t nseg,
                   hipStream_t st) {
  if (!fftdec_layout_ok(L) || (side != 0 && side != 1)) return false;
  const uint64_t gx = (L.len / 32 * 2 + 255) / 256;
  for (uint32_t s0 = 0; s0 < nseg; s0 += 65535) {
    const uint32_t ny = nseg - s0 < 65535 ? nseg - s0 : 65535;
    if (side)
      hipLaunchKernelGGL(k_fftdec_m<1>, dim3((unsigned)gx, ny), dim3(256), 0, st, L, plan1, plans,
                         seg_list, s0);
    else
      hipLaunchKernelGGL(k_fftdec_m<0>, dim3((unsigned)gx, ny), dim3(256), 0, st, L, plan1, plans,
                         seg_list, s0);
  }
  return true;
}

}  // namespace cec
