// Host-only cost model that picks the RS(32,32) rebuild decoder per erasure pattern and per
// batch (cess_ec.cpp build_ps_plan / do_decode). Header-only so tests/native/fftdec_chooser.cpp
// runs the same rule on CPU against the recorded warm sweep (tests/golden/fftdec_sweep_r04.json).
//
// Costs are microseconds for one launch over 64 segments of 512 KiB shards (bench.py --config 6
// --erasures e, 30 warm-up launches, 20 timed; profiles/r04/c6_sweep_warm30.jsonl), per pattern:
//  - k_fftdec_m (syndrome rows, fftdec.hip): T1 plus (outputs x syndrome slots) Horner rows;
//    three waves per SIMD up to four slots, two past four (the "big" class);
//  - k_fftdec_d (formal derivative, fftdec_d.hip): nearly flat, the last FFT layers, the division
//    and the stores only for slots holding an output;
//  - k_rthx (the matrix decoder): about the same per output at every pattern; up to four outputs
//    the alternative is k_rtb.
#pragma once

#include <cstddef>
#include <vector>

namespace cec {

enum FdKind { kFdNone = 0, kFdM = 1, kFdD = 2 };

inline double fdd_cost(int nout) { return 565.0 + 7.0 * nout; }
inline double fdm_cost(int nout, int nrs, bool big) {
  return big ? 424.0 + 3.63 * nout * nrs : 265.0 + 3.82 * nout * nrs;
}
inline double rt_cost(int nout) { return nout <= 4 ? 130.0 + 57.0 * nout : 235.0 + 33.9 * nout; }

// A batch split between the two decoders runs one launch more per syndrome-row class; its ramp
// and tail cost about this much beyond the per-segment costs.
constexpr double kSplitLaunchUs = 20.0;

// Per pattern: the syndrome-row decoder only with a 15 % margin over the derivative (a split
// batch runs two smaller launches), the matrix decoder when neither FFT decoder is cheaper.
inline int fftdec_choice(int nout, int nrs, bool big, bool has_m, bool has_d) {
  const double alt = rt_cost(nout);
  const double m = has_m ? fdm_cost(nout, nrs, big) : 1e30;
  const double d = has_d ? fdd_cost(nout) : 1e30;
  if (m < alt && m < 0.85 * d) return kFdM;
  if (d < alt) return kFdD;
  return kFdNone;
}

// One pattern group the per-pattern rule sent to the syndrome-row decoder.
struct FdmGroup {
  size_t nseg;
  int nout, nrs;
  bool big, has_d;
};

// Per batch: fold the syndrome-row groups (mlaunches launches, one per side x size class) into the
// derivative launch the batch already runs when that is cheaper as a whole. Per-segment costs are
// scaled from the 64 x 512 KiB fit by shard_len.
inline bool fftdec_fold(const std::vector<FdmGroup>& groups, int mlaunches, size_t shard_len) {
  if (!mlaunches) return false;
  const double scale = (double)shard_len / (512.0 * 1024.0) / 64.0;
  double delta = 0;  // all-derivative minus split
  for (const FdmGroup& g : groups) {
    if (!g.has_d) return false;
    delta += g.nseg * scale * (fdd_cost(g.nout) - fdm_cost(g.nout, g.nrs, g.big));
  }
  return delta < kSplitLaunchUs * mlaunches;
}

}  // namespace cec
