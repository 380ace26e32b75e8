// The RS(32,32) rebuild decoder chooser (cess_amd/csrc/fftdec_cost.h) run on CPU over batches of
// erasure patterns, with the plans the library builds for them (fftdec_plan.h: the survivor read
// set, the syndrome-row plan's slot count, whether each FFT plan exists) and the same grouping as
// cess_ec.cpp build_ps_plan: per pattern fftdec_choice, then the batch fold.
// stdin: per batch a line "nseg shard_len" followed by nseg lines of 64 '0'/'1' present flags.
// stdout: per batch "m <segments> d <segments> rt <segments> mlaunches <n> cost_m <us> cost_d <us>
// cost_rt <us> rows_small <x> rows_big <x> frac_big <f> cost_chosen <us>": the model's
// all-on-one-decoder predictions for the batch (per-segment means of the 64-segment costs; a
// pattern without that plan costs nan), the syndrome-row decoder's fit features (per-segment
// means of outputs x slots by size class), and the model's cost of the assignment chosen (plus
// the split's extra launches).
// Build: g++ -std=c++20 -O1 -fconstexpr-ops-limit=2000000000 fftdec_chooser.cpp
#include <cmath>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "../../cess_amd/csrc/fftdec_cost.h"
#include "../../cess_amd/csrc/fftdec_plan.h"

using namespace cec;

// fftdec.hip kSmallNr: the syndrome-row kernel's three-waves-per-SIMD class holds four slots
static bool big_class(int nrs) { return nrs > 4; }

int main() {
  size_t nseg, shard_len;
  const int kMin = 4;  // cess_ec.cpp fftdec_min default: fewer outputs stay on the matrix decoders
  while (std::scanf("%zu %zu", &nseg, &shard_len) == 2) {
    struct Group {
      size_t nseg = 0;
      int nout = 0, nrs = 0, side = 0;
      bool has_m = false, has_d = false;
    };
    std::map<std::string, Group> groups;
    double cm = 0, cd = 0, crt = 0, xs = 0, xb = 0, nb = 0;
    for (size_t s = 0; s < nseg; ++s) {
      char buf[80];
      if (std::scanf("%79s", buf) != 1) return 2;
      std::string key(buf);
      if (key.size() != 64) return 2;
      Group& g = groups[key];
      if (g.nseg++ == 0) {
        uint8_t present[64], read[64] = {};
        for (int i = 0; i < 64; ++i) present[i] = key[i] == '1';
        for (int i = 0; i < 64; ++i) g.nout += !present[i];
        if (!survivor_set(32, 32, present, read)) return 3;
        FftDecPlan pm, pd;
        g.has_m = g.nout >= 2 && fftdec_plan_m(read, present, false, &pm);
        g.has_d = g.nout >= 2 && fftdec_plan_d(read, present, false, &pd);
        g.nrs = g.has_m ? pm.nrslots : 0;
        g.side = g.has_m ? pm.side : 0;
      }
      cm += g.has_m ? fdm_cost(g.nout, g.nrs, big_class(g.nrs)) : NAN;
      cd += g.has_d ? fdd_cost(g.nout) : NAN;
      crt += rt_cost(g.nout);
      if (g.has_m) (big_class(g.nrs) ? xb : xs) += g.nout * g.nrs, nb += big_class(g.nrs);
    }
    size_t on_m = 0, on_d = 0, on_rt = 0;
    double c_m = 0, c_d = 0, c_rt = 0, c_md = 0;  // chosen costs by decoder; c_md: m groups on d
    std::vector<FdmGroup> mg;
    bool mcls[4] = {};
    for (auto& [key, g] : groups) {
      int fk = kFdNone;
      if ((g.has_m || g.has_d) && g.nout >= kMin)
        fk = fftdec_choice(g.nout, g.nrs, big_class(g.nrs), g.has_m, g.has_d);
      if (fk == kFdM) {
        mg.push_back({g.nseg, g.nout, g.nrs, big_class(g.nrs), g.has_d});
        mcls[g.side * 2 + (big_class(g.nrs) ? 1 : 0)] = true;
        on_m += g.nseg;
        c_m += g.nseg * fdm_cost(g.nout, g.nrs, big_class(g.nrs));
        c_md += g.has_d ? g.nseg * fdd_cost(g.nout) : NAN;
      } else if (fk == kFdD) {
        on_d += g.nseg;
        c_d += g.nseg * fdd_cost(g.nout);
      } else {
        on_rt += g.nseg;
        c_rt += g.nseg * rt_cost(g.nout);
      }
    }
    const int mlaunches = mcls[0] + mcls[1] + mcls[2] + mcls[3];
    double chosen = c_rt + c_d;
    if (on_d && fftdec_fold(mg, mlaunches, shard_len)) {
      on_d += on_m;
      on_m = 0;
      chosen += c_md;
    } else {
      chosen += c_m + (on_m && on_d ? kSplitLaunchUs * mlaunches : 0.0);
    }
    std::printf("m %zu d %zu rt %zu mlaunches %d cost_m %.1f cost_d %.1f cost_rt %.1f "
                "rows_small %.2f rows_big %.2f frac_big %.3f cost_chosen %.1f\n",
                on_m, on_d, on_rt, on_m ? mlaunches : 0, cm / nseg, cd / nseg, crt / nseg,
                xs / nseg, xb / nseg, nb / nseg, chosen / nseg);
  }
  return 0;
}
