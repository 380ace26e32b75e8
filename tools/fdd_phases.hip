// Probe kernels for the per-phase instruction count of k_fftdec_d (tools/fdd_phase_count.py):
// each runs one phase of the decoder (cess_amd/csrc/fftdec_d.hip, included as is) on the 16 x 8
// register slots of a lane, between fences, so the difference of its VALU count against p_none is
// that phase's instructions on the shipped code path (same helpers and exchange forms, kFddSwz;
// same occupancy attribute).
#include "../cess_amd/csrc/fftdec_d.hip"

namespace cec {
#define CEC_PROBE(NAME, BODY)                                                                  \
  __global__ __launch_bounds__(256) CEC_FDD_ATTR void NAME(uint32_t* o, uint32_t e1, uint32_t e2) { \
    uint32_t X[16][8];                                                                         \
    for (int j = 0; j < 16; ++j)                                                               \
      for (int q = 0; q < 8; ++q) X[j][q] = o[(j * 8 + q) * 256 + threadIdx.x];                \
    fence_all(X);                                                                              \
    BODY;                                                                                      \
    fence_all(X);                                                                              \
    for (int j = 0; j < 16; ++j)                                                               \
      for (int q = 0; q < 8; ++q) o[(j * 8 + q) * 256 + threadIdx.x] = X[j][q];                \
  }
__shared__ uint32_t probe_masks[4096];
CEC_PROBE(p_none, {})
CEC_PROBE(p_tr8, { sfor<16>([&](auto J) CEC_FFT_AI { after_prev<J>(X); tr8(X[J]); }); })
CEC_PROBE(p_mul, {
  sfor<16>([&](auto J) CEC_FFT_AI {
    after_prev<J>(X);
    mul_rt_lds(X[J], (const lds_u32*)probe_masks + (J * 4 + (threadIdx.x & 3)) * 8);
  });
})
CEC_PROBE(p_ifft64, { ifft64<(kFddSwz & 1) != 0>(X, e1, e2); })
CEC_PROBE(p_derivative, { derivative<(kFddSwz & 2) != 0>(X, e1, e2); })
CEC_PROBE(p_fft64_upper, { fft64_upper(X); })
CEC_PROBE(p_fft64_tail, {
  sfor<16>([&](auto J) CEC_FFT_AI { after_prev<J>(X); fft64_tail<J, (kFddSwz & 4) != 0>(X[J], e1, e2); });
})
}  // namespace cec
