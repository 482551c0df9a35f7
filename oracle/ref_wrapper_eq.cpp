// ref_wrapper_eq.cpp -- extern "C" glue around the REFERENCE's channel equalizer
// (lib/phy/upper/equalization/channel_equalizer_generic_impl.cpp, compiled from
// /root/reference by oracle/Makefile).  TEST INFRASTRUCTURE ONLY: pins
// oracle/equalizer.py and times the reference for the equalizer bench leg.
// Inputs use the reference's own containers: dynamic_re_buffer<cbf16_t>
// [port][re] and dynamic_ch_est_list [layer][port][re].
#include "phy/upper/equalization/channel_equalizer_generic_impl.h"
#include "srsran/phy/support/re_buffer.h"
#include "srsran/phy/upper/equalization/dynamic_ch_est_list.h"
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

using namespace srsran;

extern "C" {

int srs_ref_equalizer_is_supported(int mmse, unsigned nof_ports, unsigned nof_layers)
{
  channel_equalizer_generic_impl eq(mmse ? channel_equalizer_algorithm_type::mmse : channel_equalizer_algorithm_type::zf);
  return eq.is_supported(nof_ports, nof_layers) ? 1 : 0;
}

// symbols: cbf16 [ports][nof_re]; est: cbf16 [layers][ports][nof_re]; nvars [ports];
// eq_out: cf [nof_re][layers]; nv_out: float [nof_re][layers].
int srs_ref_equalize(int             mmse,
                     unsigned        nof_re,
                     unsigned        nof_ports,
                     unsigned        nof_layers,
                     const uint16_t* symbols,
                     const uint16_t* est,
                     const float*    nvars,
                     float           tx_scaling,
                     float*          eq_out,
                     float*          nv_out)
{
  channel_equalizer_generic_impl eq(mmse ? channel_equalizer_algorithm_type::mmse : channel_equalizer_algorithm_type::zf);
  if (!eq.is_supported(nof_ports, nof_layers)) {
    return -1;
  }
  dynamic_re_buffer<cbf16_t> rx(nof_ports, nof_re);
  rx.resize(nof_ports, nof_re);
  for (unsigned p = 0; p != nof_ports; ++p) {
    std::memcpy(rx.get_slice(p).data(), symbols + 2 * static_cast<size_t>(p) * nof_re, nof_re * sizeof(cbf16_t));
  }
  dynamic_ch_est_list ch(nof_re, nof_ports, nof_layers);
  for (unsigned l = 0; l != nof_layers; ++l) {
    for (unsigned p = 0; p != nof_ports; ++p) {
      std::memcpy(ch.get_channel(p, l).data(),
                  est + 2 * (static_cast<size_t>(l) * nof_ports + p) * nof_re,
                  nof_re * sizeof(cbf16_t));
    }
  }
  eq.equalize(span<cf_t>(reinterpret_cast<cf_t*>(eq_out), nof_re * nof_layers),
              span<float>(nv_out, nof_re * nof_layers),
              rx,
              ch,
              span<const float>(nvars, nof_ports),
              tx_scaling);
  return 0;
}

// CPU baseline: `reps` equalizations of the same allocation per thread; returns seconds.
double srs_ref_equalize_many(unsigned        nof_re,
                             unsigned        nof_ports,
                             unsigned        nof_layers,
                             const uint16_t* symbols,
                             const uint16_t* est,
                             const float*    nvars,
                             unsigned        reps,
                             unsigned        threads)
{
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < threads; ++t) {
    pool.emplace_back([=]() {
      std::vector<float> eq(2 * static_cast<size_t>(nof_re) * nof_layers), nv(static_cast<size_t>(nof_re) * nof_layers);
      for (unsigned r = t; r < reps; r += threads) {
        srs_ref_equalize(0, nof_re, nof_ports, nof_layers, symbols, est, nvars, 1.0F, eq.data(), nv.data());
      }
    });
  }
  for (auto& th : pool) {
    th.join();
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

} // extern "C"
