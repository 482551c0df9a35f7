// equalizer_args.h -- argument block of the equalizer kernels (equalizer.hip),
// shared with their C-ABI (equalizer_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

struct equalizer_args {
  const void* symbols;        // cbf16 [port][nof_re]
  const void* estimates;      // cbf16 [layer][port][nof_re]
  float*      eq_symbols;     // cf [nof_re][layer]
  float*      eq_noise_vars;  // [nof_re][layer]
  uint32_t    nof_re;
  float       tx_scaling;
  // 1 layer: per-port noise variances and the ports with a valid one
  // (isnormal and > 0, channel_equalizer_generic_impl.cpp:131 / equalize_zf_1xn.h:145)
  float       port_noise_var[4];
  uint32_t    valid_ports;
  // 2 layers: the largest per-port variance (channel_equalizer_generic_impl.cpp:304)
  float       noise_var;
  int32_t     noise_ok;       // isnormal(noise_var) && noise_var >= 0 (equalize_zf_2xn.h:57)
  int32_t     mmse;           // SRS_AMD_EQ_MMSE (L >= 2: the unbiased MMSE solve of equalizer_device.h)
};

hipError_t launch_equalizer(const equalizer_args& a, uint32_t nof_ports, uint32_t nof_layers, hipStream_t stream);

} // namespace srs_amd
