// ref_wrapper_chest.cpp -- extern "C" glue around the REFERENCE's own PUSCH
// DM-RS channel estimator (dmrs_pusch_estimator_impl + port_channel_estimator_average_impl,
// linear interpolator, DFT time-alignment estimator), compiled from
// /root/reference by oracle/Makefile into oracle/_ref/libsrsran_ref.so.
//
// TEST INFRASTRUCTURE ONLY: pins oracle/chest.py (tests/test_oracle_vs_ref.py)
// and is timed as the CPU baseline of the channel-estimation row.
//
// Glue (interfaces implemented here, nothing of the reference replaced):
//   inline_executor            task_executor that refuses deferral, so the estimator
//                              runs each port inline (dmrs_pusch_estimator_impl.cpp:62-66);
//   counting_notifier          dmrs_pusch_estimator_notifier.
// The grid is the reference's own resource_grid_reader_impl over its tensor.
#include "phy/generic_functions/dft_processor_generic_impl.h"
#include "phy/support/interpolator/interpolator_linear_impl.h"
#include "phy/support/resource_grid_reader_impl.h"
#include "phy/support/time_alignment_estimator/time_alignment_estimator_dft_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "phy/upper/signal_processors/channel_estimator/port_channel_estimator_average_impl.h"
#include "phy/upper/sequence_generators/low_papr_sequence_generator_impl.h"
#include "phy/upper/signal_processors/pusch/dmrs_pusch_estimator_impl.h"
#include "srsran/adt/tensor.h"
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>

using namespace srsran;

namespace {

class inline_executor : public task_executor
{
public:
  bool execute(unique_task task) override
  {
    task();
    return true;
  }
  bool defer(unique_task) override { return false; }
};


class counting_notifier : public dmrs_pusch_estimator_notifier
{
public:
  void     on_estimation_complete() override { ++count; }
  unsigned count = 0;
};

using grid_tensor =
    dynamic_tensor<static_cast<unsigned>(resource_grid_dimensions::all), cbf16_t, resource_grid_dimensions>;

std::unique_ptr<port_channel_estimator> make_port_estimator(int fd, int td, int cfo)
{
  time_alignment_estimator_dft_impl::collection_dft_processors dfts;
  for (unsigned n = time_alignment_estimator_dft_impl::min_dft_size; n <= time_alignment_estimator_dft_impl::max_dft_size;
       n *= 2) {
    dfts.emplace(n,
                 std::make_unique<dft_processor_generic_impl>(
                     dft_processor::configuration{n, dft_processor::direction::INVERSE}));
  }
  auto ta = std::make_unique<time_alignment_estimator_dft_impl>(std::move(dfts));
  return std::make_unique<port_channel_estimator_average_impl>(
      std::make_unique<interpolator_linear_impl>(),
      std::move(ta),
      static_cast<port_channel_estimator_fd_smoothing_strategy>(fd),
      static_cast<port_channel_estimator_td_interpolation_strategy>(td),
      cfo != 0);
}

struct chest_ctx {
  inline_executor                           exec;
  std::unique_ptr<dmrs_pusch_estimator_impl> est;
  chest_ctx(int fd, int td, int cfo)
  {
    est = std::make_unique<dmrs_pusch_estimator_impl>(std::make_unique<pseudo_random_generator_impl>(),
                                                      std::make_unique<low_papr_sequence_generator_impl>(),
                                                      make_port_estimator(fd, td, cfo),
                                                      exec);
  }
};

dmrs_pusch_estimator::configuration make_config(unsigned       numerology,
                                                unsigned       slot_index,
                                                int            type2,
                                                unsigned       nof_layers,
                                                unsigned       scrambling_id,
                                                int            n_scid,
                                                float          scaling,
                                                unsigned       symbols_mask,
                                                const uint8_t* crbs,
                                                unsigned       nof_prb,
                                                unsigned       first_symbol,
                                                unsigned       nof_symbols,
                                                unsigned       nof_rx_ports)
{
  dmrs_pusch_estimator::configuration cfg;
  cfg.slot = slot_point(numerology, slot_index);
  if (type2 == 2) {
    // transform precoding: low-PAPR sequence of identifier n_rs_id (passed as scrambling_id)
    cfg.sequence_config = dmrs_pusch_estimator::low_papr_sequence_configuration{scrambling_id};
  } else {
    dmrs_pusch_estimator::pseudo_random_sequence_configuration seq;
    seq.type            = type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
    seq.nof_tx_layers   = nof_layers;
    seq.scrambling_id   = scrambling_id;
    seq.n_scid          = n_scid != 0;
    cfg.sequence_config = seq;
  }
  cfg.scaling         = scaling;
  cfg.c_prefix        = cyclic_prefix::NORMAL;
  cfg.symbols_mask    = bounded_bitset<MAX_NSYMB_PER_SLOT>(MAX_NSYMB_PER_SLOT);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    if ((symbols_mask >> l) & 1u) {
      cfg.symbols_mask.set(l);
    }
  }
  cfg.rb_mask.resize(nof_prb);
  for (unsigned i = 0; i != nof_prb; ++i) {
    if (crbs[i]) {
      cfg.rb_mask.set(i);
    }
  }
  cfg.first_symbol = first_symbol;
  cfg.nof_symbols  = nof_symbols;
  for (unsigned p = 0; p != nof_rx_ports; ++p) {
    cfg.rx_ports.push_back(static_cast<uint8_t>(p));
  }
  return cfg;
}

void load_grid(grid_tensor& data, const uint32_t* grid, unsigned nports, unsigned nsubc)
{
  for (unsigned p = 0; p != nports; ++p) {
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
      std::memcpy(row.data(), grid + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * sizeof(cbf16_t));
    }
  }
}

} // namespace

extern "C" {

// dmrs_pusch_estimator::estimate (dmrs_pusch_estimator_impl.cpp:28-70) for all
// nof_rx_ports ports of a grid [nof_rx_ports][14][nsubc] (cbf16 as uint32).
// type2: 0 DM-RS type 1, 1 type 2, 2 the low-PAPR sequence of transform precoding with n_rs_id = scrambling_id.
// fd: 0 none, 1 mean, 2 filter; td: 0 interpolate, 1 average (the reference enums).
// Outputs: estimates uint32 [port][layer][14][nsubc] (only the REs the
// reference writes are changed), per port noise_var, epre, snr, per
// (port, layer) rsrp, ta_s, cfo_hz (NaN when the reference has none).
int srs_ref_pusch_chest(const uint32_t* grid,
                        unsigned        nof_rx_ports,
                        unsigned        nsubc,
                        unsigned        numerology,
                        unsigned        slot_index,
                        int             type2,
                        unsigned        nof_layers,
                        unsigned        scrambling_id,
                        int             n_scid,
                        float           scaling,
                        unsigned        symbols_mask,
                        const uint8_t*  crbs,
                        unsigned        first_symbol,
                        unsigned        nof_symbols,
                        int             fd,
                        int             td,
                        int             compensate_cfo,
                        uint32_t*       estimates,
                        float*          noise_var,
                        float*          epre,
                        float*          snr,
                        float*          rsrp,
                        double*         ta_s,
                        float*          cfo_hz)
{
  const unsigned nof_prb = nsubc / NRE;
  chest_ctx      ctx(fd, td, compensate_cfo);
  auto           cfg = make_config(numerology, slot_index, type2, nof_layers, scrambling_id, n_scid, scaling,
                         symbols_mask, crbs, nof_prb, first_symbol, nof_symbols, nof_rx_ports);

  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_rx_ports});
  load_grid(data, grid, nof_rx_ports, nsubc);
  std::atomic<unsigned>    empty{0};
  resource_grid_reader_impl reader(data, empty);

  channel_estimate  est;
  counting_notifier notifier;
  // Pre-fill the estimate with the caller's buffer so untouched REs compare equal.
  est.resize({nof_prb, MAX_NSYMB_PER_SLOT, nof_rx_ports, nof_layers});
  for (unsigned p = 0; p != nof_rx_ports; ++p) {
    for (unsigned v = 0; v != nof_layers; ++v) {
      for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
        span<cbf16_t> s = est.get_symbol_ch_estimate(l, p, v);
        std::memcpy(s.data(), estimates + ((p * nof_layers + v) * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * 4);
      }
    }
  }
  ctx.est->estimate(est, notifier, reader, cfg);
  if (notifier.count != 1) {
    return -1;
  }
  const unsigned nsym_est = first_symbol + nof_symbols;
  for (unsigned p = 0; p != nof_rx_ports; ++p) {
    noise_var[p] = est.get_noise_variance(p);
    epre[p]      = est.get_epre(p);
    snr[p]       = est.get_snr(p);
    for (unsigned v = 0; v != nof_layers; ++v) {
      rsrp[p * nof_layers + v]         = est.get_rsrp(p, v);
      ta_s[p * nof_layers + v]         = est.get_time_alignment(p, v).to_seconds();
      std::optional<float> c           = est.get_cfo_Hz(p, v);
      cfo_hz[p * nof_layers + v]       = c.has_value() ? *c : NAN;
      for (unsigned l = 0; l != nsym_est; ++l) {
        span<const cbf16_t> s = est.get_symbol_ch_estimate(l, p, v);
        std::memcpy(estimates + ((p * nof_layers + v) * MAX_NSYMB_PER_SLOT + l) * nsubc, s.data(), nsubc * 4);
      }
    }
  }
  return 0;
}

// low_papr_sequence_generator_impl::generate(sequence, u, v, 0, 1): M interleaved (re, im) floats.
void srs_ref_low_papr(float* out, unsigned M, unsigned u, unsigned v)
{
  low_papr_sequence_generator_impl gen;
  gen.generate(span<cf_t>(reinterpret_cast<cf_t*>(out), M), u, v, 0, 1);
}

// CPU baseline: `iterations` estimations of the same grid on `threads` threads
// (one estimator each); returns wall seconds.
double srs_ref_pusch_chest_many(const uint32_t* grid,
                                unsigned        nof_rx_ports,
                                unsigned        nsubc,
                                int             type2,
                                unsigned        nof_layers,
                                unsigned        symbols_mask,
                                const uint8_t*  crbs,
                                unsigned        first_symbol,
                                unsigned        nof_symbols,
                                unsigned        iterations,
                                unsigned        threads);

} // extern "C"

#include <thread>
#include <vector>

double srs_ref_pusch_chest_many(const uint32_t* grid,
                                unsigned        nof_rx_ports,
                                unsigned        nsubc,
                                int             type2,
                                unsigned        nof_layers,
                                unsigned        symbols_mask,
                                const uint8_t*  crbs,
                                unsigned        first_symbol,
                                unsigned        nof_symbols,
                                unsigned        iterations,
                                unsigned        threads)
{
  const unsigned nof_prb = nsubc / NRE;
  auto           t0      = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (unsigned t = 0; t != threads; ++t) {
    pool.emplace_back([&, t]() {
      chest_ctx   ctx(2, 1, 1);
      auto        cfg = make_config(1, 0, type2, nof_layers, 1, 0, 1.0F, symbols_mask, crbs, nof_prb, first_symbol,
                             nof_symbols, nof_rx_ports);
      grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_rx_ports});
      load_grid(data, grid, nof_rx_ports, nsubc);
      std::atomic<unsigned>     empty{0};
      resource_grid_reader_impl reader(data, empty);
      channel_estimate          est;
      counting_notifier         notifier;
      for (unsigned i = t; i < iterations; i += threads) {
        ctx.est->estimate(est, notifier, reader, cfg);
      }
    });
  }
  for (auto& th : pool) {
    th.join();
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
