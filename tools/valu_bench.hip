// VALU issue-rate microbenchmark for the instructions the codec's kernels are made of
// (v_bitop3_b32, v_perm_b32, v_lshlrev_b32, v_alignbit_b32, v_add3_u32, v_add_u32, v_xor_b32,
// v_lshl_or_b32, v_and_b32)
// next to v_fma_f32. Each wave runs 8 independent chains of one instruction (inline asm, so the
// compiler cannot fold or reorder them), timed in-kernel with s_memtime.
// Reports cycles per wave-instruction per SIMD at 1 wave/SIMD (issue cost of a lone wave) and
// at 8 waves/SIMD (SIMD throughput).
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_bench.hip -o tools/valu_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <utility>

#define REP8(X) X X X X X X X X
#define CHAINS(OP)                                                                        \
  asm volatile(OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)                            \
               : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), \
                 "+v"(r7)                                                                 \
               : "v"(k1), "v"(k2));

#define O_0(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x96\n\t"
#define O_1(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n\t"
#define O_2(i) "v_lshlrev_b32 %" #i ", 1, %" #i "\n\t"
#define O_3(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 7\n\t"
#define O_4(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n\t"
#define O_5(i) "v_add_u32 %" #i ", %" #i ", %8\n\t"
#define O_6(i) "v_xor_b32 %" #i ", %" #i ", %8\n\t"
#define O_7(i) "v_lshl_or_b32 %" #i ", %" #i ", 1, %8\n\t"
#define O_8(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n\t"
#define O_9(i) "v_and_b32 %" #i ", %" #i ", %8\n\t"
#define O_10(i) "v_mul_u32_u24 %" #i ", %" #i ", %8\n\t"
#define O_11(i) "v_mad_u32_u24 %" #i ", %" #i ", %8, %9\n\t"
#define O_12(i) "v_pk_add_u16 %" #i ", %" #i ", %8\n\t"
#define O_13(i) "v_pk_lshlrev_b16 %" #i ", 1, %" #i "\n\t"
#define O_14(i) "v_cndmask_b32 %" #i ", %" #i ", %8, vcc\n\t"
#define O_15(i) "v_bfi_b32 %" #i ", %" #i ", %8, %9\n\t"
#define O_16(i) "v_sub_u32 %" #i ", %" #i ", %8\n\t"
#define O_17(i) "v_or3_b32 %" #i ", %" #i ", %8, %9\n\t"
#define O_18(i) "v_and_or_b32 %" #i ", %" #i ", %8, %9\n\t"
#define O_19(i) "v_xad_u32 %" #i ", %" #i ", %8, %9\n\t"
#define O_20(i) "v_lshl_add_u32 %" #i ", %" #i ", 1, %8\n\t"
#define O_21(i) "v_bfe_u32 %" #i ", %" #i ", 3, 8\n\t"
#define O_22(i) "v_lshrrev_b32 %" #i ", 7, %" #i "\n\t"
#define O_23(i) "v_mul_lo_u32 %" #i ", %" #i ", %8\n\t"
#define O_24(i) "v_mov_b32_dpp %" #i ", %" #i " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define O_25(i) "v_add_u32_sdwa %" #i ", %" #i ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n\t"
#define O_26(i) "v_lshlrev_b16 %" #i ", 1, %" #i "\n\t"

#define O_27(i) "v_lshlrev_b32 %" #i ", 7, %" #i "\n\t"
#define O_28(i) "v_lshrrev_b32 %" #i ", 1, %" #i "\n\t"
#define O_29(i) "v_lshlrev_b32 %" #i ", %8, %" #i "\n\t"
#define O_30(i) "v_or_b32 %" #i ", %" #i ", %8\n\t"
#define O_31(i) "v_not_b32 %" #i ", %" #i "\n\t"
#define O_32(i) "v_mov_b32 %" #i ", %8\n\t"
#define O_33(i) "v_add_co_u32 %" #i ", vcc, %" #i ", %8\n\t"
#define O_34(i) "v_ashrrev_i32 %" #i ", 7, %" #i "\n\t"
#define O_35(i) "v_bitop3_b16 %" #i ", %" #i ", %8, %9 bitop3:0x96\n\t"
#define O_36(i) "v_add_u16 %" #i ", %" #i ", %8\n\t"
#define O_37(i) "v_xor_b32 %" #i ", 0x1d1d1d1d, %" #i "\n\t"
#define O_38(i) "v_and_b32 %" #i ", 0x7f7f7f7f, %" #i "\n\t"
#define O_39(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x78\n\t"
#define O_40(i) "v_max_u32 %" #i ", %" #i ", %8\n\t"
#define O_41(i) "v_lshlrev_b16_e64 %" #i ", 1, %" #i "\n\t"
#define O_44(i) "v_xor_b32_dpp %" #i ", %" #i ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define O_45(i) "v_and_b32_dpp %" #i ", %" #i ", %8 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
// lane-half swaps write both operands: eight per asm over the eight chains (a ring of pairs)
#define SWAPS(INS)                                                                          \
  asm volatile(INS " %0, %1\n\t" INS " %2, %3\n\t" INS " %4, %5\n\t" INS " %6, %7\n\t" INS   \
               " %1, %2\n\t" INS " %3, %4\n\t" INS " %5, %6\n\t" INS " %7, %0\n\t"               \
               : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));

// 64-bit operand chains (rotates as one 64-bit shift of a doubled word, and their helpers)
#define CHAINS64(OP)                                                                      \
  asm volatile(OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)                            \
               : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), \
                 "+v"(q7)                                                                 \
               : "v"(kq));
#define Q_46(i) "v_lshrrev_b64 %" #i ", 7, %" #i "\n\t"
#define Q_47(i) "v_lshlrev_b64 %" #i ", 7, %" #i "\n\t"
#define Q_48(i) "v_pk_mov_b32 %" #i ", %" #i ", %" #i " op_sel:[1,0]\n\t"
#define Q_49(i) "v_mov_b64 %" #i ", %8\n\t"
#define Q_50(i) "v_lshl_add_u64 %" #i ", %" #i ", 3, %8\n\t"
#define Q_51(i) "v_pk_add_f32 %" #i ", %" #i ", %8\n\t"
#define Q_52(i) "v_pk_fma_f32 %" #i ", %" #i ", %8, %8\n\t"

template <int OPI>
__global__ void k_valu(uint32_t* out, uint64_t* cyc, int iters, uint32_t a, uint32_t b) {
  uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
           r6 = r0 + 6, r7 = r0 + 7;
  uint32_t k1 = a + threadIdx.x, k2 = b;
  uint64_t q0 = r0 * 0x100000001ull, q1 = q0 + 1, q2 = q0 + 2, q3 = q0 + 3, q4 = q0 + 4,
           q5 = q0 + 5, q6 = q0 + 6, q7 = q0 + 7, kq = k1 * 0x100000001ull + b;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    // 8 x 8 = 64 instructions per iteration
    if constexpr (OPI == 0) { REP8(CHAINS(O_0)) }
    if constexpr (OPI == 1) { REP8(CHAINS(O_1)) }
    if constexpr (OPI == 2) { REP8(CHAINS(O_2)) }
    if constexpr (OPI == 3) { REP8(CHAINS(O_3)) }
    if constexpr (OPI == 4) { REP8(CHAINS(O_4)) }
    if constexpr (OPI == 5) { REP8(CHAINS(O_5)) }
    if constexpr (OPI == 6) { REP8(CHAINS(O_6)) }
    if constexpr (OPI == 7) { REP8(CHAINS(O_7)) }
    if constexpr (OPI == 8) { REP8(CHAINS(O_8)) }
    if constexpr (OPI == 9) { REP8(CHAINS(O_9)) }
    if constexpr (OPI == 10) { REP8(CHAINS(O_10)) }
    if constexpr (OPI == 11) { REP8(CHAINS(O_11)) }
    if constexpr (OPI == 12) { REP8(CHAINS(O_12)) }
    if constexpr (OPI == 13) { REP8(CHAINS(O_13)) }
    if constexpr (OPI == 14) { REP8(CHAINS(O_14)) }
    if constexpr (OPI == 15) { REP8(CHAINS(O_15)) }
    if constexpr (OPI == 16) { REP8(CHAINS(O_16)) }
    if constexpr (OPI == 17) { REP8(CHAINS(O_17)) }
    if constexpr (OPI == 18) { REP8(CHAINS(O_18)) }
    if constexpr (OPI == 19) { REP8(CHAINS(O_19)) }
    if constexpr (OPI == 20) { REP8(CHAINS(O_20)) }
    if constexpr (OPI == 21) { REP8(CHAINS(O_21)) }
    if constexpr (OPI == 22) { REP8(CHAINS(O_22)) }
    if constexpr (OPI == 23) { REP8(CHAINS(O_23)) }
    if constexpr (OPI == 24) { REP8(CHAINS(O_24)) }
    if constexpr (OPI == 25) { REP8(CHAINS(O_25)) }
    if constexpr (OPI == 26) { REP8(CHAINS(O_26)) }
    if constexpr (OPI == 27) { REP8(CHAINS(O_27)) }
    if constexpr (OPI == 28) { REP8(CHAINS(O_28)) }
    if constexpr (OPI == 29) { REP8(CHAINS(O_29)) }
    if constexpr (OPI == 30) { REP8(CHAINS(O_30)) }
    if constexpr (OPI == 31) { REP8(CHAINS(O_31)) }
    if constexpr (OPI == 32) { REP8(CHAINS(O_32)) }
    if constexpr (OPI == 33) { REP8(CHAINS(O_33)) }
    if constexpr (OPI == 34) { REP8(CHAINS(O_34)) }
    if constexpr (OPI == 35) { REP8(CHAINS(O_35)) }
    if constexpr (OPI == 36) { REP8(CHAINS(O_36)) }
    if constexpr (OPI == 37) { REP8(CHAINS(O_37)) }
    if constexpr (OPI == 38) { REP8(CHAINS(O_38)) }
    if constexpr (OPI == 39) { REP8(CHAINS(O_39)) }
    if constexpr (OPI == 40) { REP8(CHAINS(O_40)) }
    if constexpr (OPI == 41) { REP8(CHAINS(O_41)) }
    if constexpr (OPI == 42) { REP8(SWAPS("v_permlane32_swap_b32")) }
    if constexpr (OPI == 43) { REP8(SWAPS("v_permlane16_swap_b32")) }
    if constexpr (OPI == 44) { REP8(CHAINS(O_44)) }
    if constexpr (OPI == 45) { REP8(CHAINS(O_45)) }
    if constexpr (OPI == 46) { REP8(CHAINS64(Q_46)) }
    if constexpr (OPI == 47) { REP8(CHAINS64(Q_47)) }
    if constexpr (OPI == 48) { REP8(CHAINS64(Q_48)) }
    if constexpr (OPI == 49) { REP8(CHAINS64(Q_49)) }
    if constexpr (OPI == 50) { REP8(CHAINS64(Q_50)) }
    if constexpr (OPI == 51) { REP8(CHAINS64(Q_51)) }
    if constexpr (OPI == 52) { REP8(CHAINS64(Q_52)) }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] =
      r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ (uint32_t)(q0 ^ q1 ^ q2 ^ q3 ^ q4 ^ q5 ^ q6 ^ q7);
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static const char* kNames[] = {"v_bitop3_b32", "v_perm_b32", "v_lshlrev_b32", "v_alignbit_b32", "v_add3_u32", "v_add_u32", "v_xor_b32", "v_lshl_or_b32", "v_fma_f32", "v_and_b32", "v_mul_u32_u24", "v_mad_u32_u24", "v_pk_add_u16", "v_pk_lshlrev_b16", "v_cndmask_b32", "v_bfi_b32", "v_sub_u32", "v_or3_b32", "v_and_or_b32", "v_xad_u32", "v_lshl_add_u32", "v_bfe_u32", "v_lshrrev_b32", "v_mul_lo_u32", "v_mov_b32_dpp", "v_add_u32_sdwa", "v_lshlrev_b16", "v_lshlrev_b32_by7", "v_lshrrev_b32_by1", "v_lshlrev_b32_vreg", "v_or_b32", "v_not_b32", "v_mov_b32", "v_add_co_u32", "v_ashrrev_i32", "v_bitop3_b16", "v_add_u16", "v_xor_b32_e64_lit", "v_and_b32_lit", "v_bitop3_lit", "v_max_u32", "v_lshlrev_b16_by1_e64", "v_permlane32_swap_b32", "v_permlane16_swap_b32", "v_xor_b32_dpp", "v_and_b32_dpp", "v_lshrrev_b64", "v_lshlrev_b64", "v_pk_mov_b32_swap", "v_mov_b64", "v_lshl_add_u64", "v_pk_add_f32", "v_pk_fma_f32"};

template <int OPI>
void run(int waves_per_simd, int cus) {
  const int threads = 256 * waves_per_simd > 1024 ? 1024 : 256 * waves_per_simd;
  const int blocks_per_cu = (256 * waves_per_simd) / threads;
  const int blocks = cus * blocks_per_cu;
  const int iters = 2000;
  uint32_t* out;
  uint64_t* cyc;
  const int nw = blocks * threads / 64;
  hipMalloc(&out, (size_t)blocks * threads * 4);
  hipMalloc(&cyc, (size_t)nw * 8);
  hipLaunchKernelGGL(k_valu<OPI>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 10, 3u, 5u);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_valu<OPI>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 3u, 5u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint64_t> h(nw);
  hipMemcpy(h.data(), cyc, nw * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double instr = 64.0 * iters;
  const double med = (double)h[nw / 2];
  const double total_lane_ops = instr * 64.0 * nw;
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cus\": %d, \"cyc_per_instr_per_wave\": %.3f, "
         "\"cyc_per_instr_per_simd\": %.3f, \"ms\": %.4f, \"Tlane_ops_per_s\": %.2f}\n",
         kNames[OPI], waves_per_simd, cus, med / instr, med / instr / waves_per_simd, ms,
         total_lane_ops / (ms * 1e-3) / 1e12);
  hipFree(out);
  hipFree(cyc);
}

template <int OPI>
void run_all() {
  run<OPI>(1, 256);
  run<OPI>(2, 256);
  run<OPI>(4, 256);
  run<OPI>(8, 256);
}

template <int... I>
void run_list(std::integer_sequence<int, I...>, int from) { ((I >= from ? run_all<I>() : void()), ...); }

int main(int argc, char** argv) {
  run_list(std::make_integer_sequence<int, 53>{}, argc > 1 ? atoi(argv[1]) : 27);
  return 0;
}
