// channel_equalizer_hip.cpp -- srsran::channel_equalizer over srs_amd_channel_equalize (see the header).
#include "channel_equalizer_hip.h"

#include "srsran_amd/equalizer.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <vector>

using namespace srsran;

namespace {

class channel_equalizer_hip : public channel_equalizer
{
public:
  explicit channel_equalizer_hip(srs_amd_channel_equalizer* e) : eq(e) {}
  ~channel_equalizer_hip() override { srs_amd_channel_equalizer_destroy(eq); }

  bool is_supported(unsigned nof_ports, unsigned nof_layers) override
  {
    return srs_amd_channel_equalizer_is_supported(eq, nof_ports, nof_layers) != 0;
  }

  // channel_equalizer.h:89.  Gathers the receive symbols ([port][re], re_buffer_reader slices) and the channel
  // estimates ([layer][port][re], ch_est_list::get_channel) into the C-ABI's dense cbf16 layouts.
  void equalize(span<cf_t>                       eq_symbols,
                span<float>                      eq_noise_vars,
                const re_buffer_reader<cbf16_t>& ch_symbols,
                const ch_est_list&               ch_estimates,
                span<const float>                noise_var_estimates,
                float                            tx_scaling) override
  {
    const unsigned nof_re = ch_symbols.get_nof_re();
    const unsigned P      = ch_symbols.get_nof_slices();
    const unsigned L      = ch_estimates.get_nof_tx_layers();
    sym.resize(static_cast<size_t>(P) * nof_re);
    est.resize(static_cast<size_t>(L) * P * nof_re);
    for (unsigned p = 0; p != P; ++p) {
      std::memcpy(sym.data() + static_cast<size_t>(p) * nof_re, ch_symbols.get_slice(p).data(),
                  sizeof(cbf16_t) * nof_re);
      for (unsigned l = 0; l != L; ++l) {
        std::memcpy(est.data() + (static_cast<size_t>(l) * P + p) * nof_re, ch_estimates.get_channel(p, l).data(),
                    sizeof(cbf16_t) * nof_re);
      }
    }
    if (srs_amd_channel_equalize(eq, reinterpret_cast<float*>(eq_symbols.data()), eq_noise_vars.data(),
                                 reinterpret_cast<const uint16_t*>(sym.data()),
                                 reinterpret_cast<const uint16_t*>(est.data()), noise_var_estimates.data(), nof_re, P,
                                 L, tx_scaling) != SRS_AMD_OK) {
      // the interface has no error path: report, and mark every symbol unusable (zero symbol, infinite variance --
      // what the reference writes for a RE it cannot equalize)
      std::fprintf(stderr, "channel_equalizer_hip: %s\n", srs_amd_last_error());
      std::fill(eq_symbols.begin(), eq_symbols.end(), cf_t());
      std::fill(eq_noise_vars.begin(), eq_noise_vars.end(), std::numeric_limits<float>::infinity());
    }
  }

private:
  srs_amd_channel_equalizer* eq;
  std::vector<cbf16_t>       sym, est;
};

class channel_equalizer_factory_hip : public channel_equalizer_factory
{
public:
  channel_equalizer_factory_hip(channel_equalizer_algorithm_type t, int d) : type(t), device(d) {}
  std::unique_ptr<channel_equalizer> create() override
  {
    int dev = device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
      return nullptr;
    }
    srs_amd_channel_equalizer* e = nullptr;
    if (srs_amd_channel_equalizer_create(
            &e, type == channel_equalizer_algorithm_type::zf ? SRS_AMD_EQ_ZF : SRS_AMD_EQ_MMSE, dev) != SRS_AMD_OK) {
      return nullptr;
    }
    return std::make_unique<channel_equalizer_hip>(e);
  }

private:
  channel_equalizer_algorithm_type type;
  int                              device;
};

} // namespace

std::shared_ptr<channel_equalizer_factory>
srsran::hip::create_channel_equalizer_factory_hip(channel_equalizer_algorithm_type type, int device)
{
  return std::make_shared<channel_equalizer_factory_hip>(type, device);
}
