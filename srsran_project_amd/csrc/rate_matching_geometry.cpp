// rate_matching_geometry.cpp -- see rate_matching_common.h.
#include "ldpc_common.h"
#include "rate_matching_common.h"
#include <cmath>

namespace srs_amd {

const char* make_rm_geometry(rm_geometry& g, uint32_t bg, uint32_t Z, uint32_t rv, uint32_t Qm, uint32_t Nref,
                             uint32_t F)
{
  // ldpc_rate_matcher_impl.cpp:33 / ldpc_rate_dematcher_impl.cpp:33
  static const double shift_factor_bg1[4] = {0, 17, 33, 56};
  static const double shift_factor_bg2[4] = {0, 13, 25, 43};
  if (bg != 1 && bg != 2) {
    return "invalid base graph";
  }
  if (lifting_index(static_cast<int>(Z)) < 0) {
    return "invalid lifting size";
  }
  if (rv > 3) {
    return "RV should an integer between 0 and 3.";
  }
  if (Qm != 1 && Qm != 2 && Qm != 4 && Qm != 6 && Qm != 8) {
    return "invalid modulation order";
  }
  const uint32_t N_short = bg == 1 ? 66 : 50;
  const uint32_t K_bg    = bg == 1 ? 22 : 10;
  g.N                    = N_short * Z;
  if (Nref > 66u * MAX_LIFTING_SIZE) { // MAX_CODEBLOCK_SIZE (ldpc.h:113)
    return "N_ref must be smaller or equal to MAX_CODEBLOCK_SIZE.";
  }
  g.Ncb     = (Nref > 0 && Nref < g.N) ? Nref : g.N;
  g.nof_sys = (K_bg - 2) * Z;
  if (F >= g.nof_sys) {
    return "invalid number of filler bits.";
  }
  if (g.Ncb < g.nof_sys) {
    // The reference's circular read is undefined (unsigned wrap) there.
    return "limited buffer shorter than the systematic part";
  }
  g.F        = F;
  g.nof_info = g.nof_sys - F;
  g.L        = g.Ncb - F;
  g.Qm       = Qm;
  const double sf = (bg == 1 ? shift_factor_bg1 : shift_factor_bg2)[rv];
  g.k0            = static_cast<uint32_t>(std::floor(sf * g.Ncb / g.N)) * Z;
  uint32_t k0eff  = (g.k0 >= g.nof_info && g.k0 < g.nof_sys) ? g.nof_sys : g.k0;
  g.rank0         = k0eff < g.nof_info ? k0eff : k0eff - F;
  return nullptr;
}

} // namespace srs_amd
