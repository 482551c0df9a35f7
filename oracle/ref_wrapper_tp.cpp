// ref_wrapper_tp.cpp -- extern "C" glue around the REFERENCE's own transform_precoder_dft_impl
// (lib/phy/generic_functions/transform_precoding/transform_precoder_dft_impl.cpp) with generic inverse DFTs
// for every valid M_rb (ref_builders.h make_transform_precoder) -- TEST INFRASTRUCTURE ONLY.
#include "ref_builders.h"

using namespace srsran;
using srs_ref::make_transform_precoder;

namespace {

transform_precoder& precoder()
{
  static std::unique_ptr<transform_precoder> tp = make_transform_precoder(MAX_NOF_PRBS);
  return *tp;
}

} // namespace

extern "C" {

// deprecode_ofdm_symbol: out / in interleaved (re, im) floats of M = 12 M_rb subcarriers.
int srs_ref_transform_deprecode(float* out, const float* in, unsigned M)
{
  if (M == 0 || M % NRE != 0 || !transform_precoding::is_nof_prbs_valid(M / NRE)) {
    return -1;
  }
  precoder().deprecode_ofdm_symbol(span<cf_t>(reinterpret_cast<cf_t*>(out), M),
                                   span<const cf_t>(reinterpret_cast<const cf_t*>(in), M));
  return 0;
}

int srs_ref_transform_deprecode_noise(float* out, const float* in, unsigned M)
{
  precoder().deprecode_ofdm_symbol_noise(span<float>(out, M), span<const float>(in, M));
  return 0;
}

int srs_ref_transform_nof_prbs_valid(unsigned nof_prb)
{
  return transform_precoding::is_nof_prbs_valid(nof_prb) ? 1 : 0;
}

} // extern "C"
