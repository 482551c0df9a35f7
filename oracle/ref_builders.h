// ref_builders.h -- builds the REFERENCE's own PUSCH receive chain objects
// (compiled from /root/reference by oracle/Makefile), shared by
// ref_wrapper_pusch.cpp (parity pins) and ref_chain.cpp (the CPU baseline).
//
// TEST INFRASTRUCTURE ONLY.
//
// Implementation choice: `impl::automatic` reproduces the run-time selection of
// the reference's "auto" software factories on this host
// (lib/phy/upper/channel_coding/channel_coding_factories.cpp:64-80 CRC: CLMUL
// when pclmul + sse4.1, else LUT; :111-121 LDPC decoder: AVX512 > AVX2 > generic;
// :184-188 rate dematcher: AVX512 (with VBMI) > AVX2 > generic). `generic` and
// `avx2` force those classes.
//
// Glue (interfaces implemented here; nothing of the reference is replaced):
//   inline_executor       task_executor that runs tasks inline
//                         (the benchmark's inline_task_executor);
//   ref_rx_buffer         unique_rx_buffer::callback over host vectors (the role
//                         of lib/phy/upper/rx_buffer_impl.h), one HARQ process.
#pragma once

#include "phy/generic_functions/dft_processor_generic_impl.h"
#include "srsran/phy/lower/modulation/ofdm_demodulator.h"
#include "srsran/phy/lower/modulation/ofdm_modulator.h"
#include "phy/generic_functions/transform_precoding/transform_precoder_dft_impl.h"
#include "phy/support/interpolator/interpolator_linear_impl.h"
#include "phy/support/time_alignment_estimator/time_alignment_estimator_dft_impl.h"
#include "phy/upper/channel_coding/crc_calculator_clmul_impl.h"
#include "phy/upper/channel_coding/crc_calculator_generic_impl.h"
#include "phy/upper/channel_coding/crc_calculator_lut_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_decoder_avx2.h"
#include "phy/upper/channel_coding/ldpc/ldpc_decoder_avx512.h"
#include "phy/upper/channel_coding/ldpc/ldpc_decoder_generic.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_avx2_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_avx512_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_segmenter_rx_impl.h"
#include "phy/upper/channel_modulation/demodulation_mapper_impl.h"
#include "phy/upper/channel_processors/pusch/pusch_decoder_impl.h"
#include "phy/upper/channel_processors/pusch/pusch_demodulator_impl.h"
#include "phy/upper/channel_processors/pusch/pusch_processor_impl.h"
#include "phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.h"
#include "phy/upper/equalization/channel_equalizer_generic_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "phy/upper/signal_processors/channel_estimator/port_channel_estimator_average_impl.h"
#include "phy/upper/sequence_generators/low_papr_sequence_generator_impl.h"
#include "phy/upper/channel_coding/polar/polar_code_impl.h"
#include "phy/upper/channel_coding/polar/polar_deallocator_impl.h"
#include "phy/upper/channel_coding/polar/polar_decoder_impl.h"
#include "phy/upper/channel_coding/polar/polar_encoder_impl.h"
#include "phy/upper/channel_coding/polar/polar_rate_dematcher_impl.h"
#include "phy/upper/channel_coding/short/short_block_detector_impl.h"
#include "phy/upper/channel_processors/uci/uci_decoder_impl.h"
#include "phy/upper/signal_processors/pusch/dmrs_pusch_estimator_impl.h"
#include "srsran/phy/upper/unique_rx_buffer.h"
#include "srsran/support/cpu_features.h"
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

namespace srs_ref {

using namespace srsran;

enum class impl { generic = 0, avx2 = 1, automatic = 2 };

inline bool host_has_clmul()
{
  return cpu_supports_feature(cpu_feature::pclmul) && cpu_supports_feature(cpu_feature::sse4_1);
}
inline bool host_has_avx512_ldpc()
{
  return cpu_supports_feature(cpu_feature::avx512f) && cpu_supports_feature(cpu_feature::avx512bw);
}
inline bool host_has_avx512_dematcher()
{
  return host_has_avx512_ldpc() && cpu_supports_feature(cpu_feature::avx512vbmi);
}

class inline_executor : public task_executor
{
public:
  bool execute(unique_task task) override
  {
    task();
    return true;
  }
  bool defer(unique_task task) override
  {
    task();
    return true;
  }
};


// uci_decoder_impl as create_uci_decoder_factory_generic builds it (uci/factories.cpp:44-55) from the short block
// detector, the polar chain (nMax = 10) and the CRC6 / CRC11 calculators (the CRC factory takes the generic
// calculator for CRC6, channel_coding_factories.cpp:70-72).
inline std::unique_ptr<uci_decoder> make_uci_decoder()
{
  return std::make_unique<uci_decoder_impl>(std::make_unique<short_block_detector_impl>(),
                                            std::make_unique<polar_code_impl>(),
                                            std::make_unique<polar_rate_dematcher_impl>(),
                                            std::make_unique<polar_decoder_impl>(std::make_unique<polar_encoder_impl>(),
                                                                                 polar_code::NMAX_LOG),
                                            std::make_unique<polar_deallocator_impl>(),
                                            std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC6),
                                            std::make_unique<crc_calculator_lut_impl>(crc_generator_poly::CRC11));
}

class ref_rx_buffer : public unique_rx_buffer::callback
{
public:
  explicit ref_rx_buffer(unsigned nof_cbs) : soft(nof_cbs), data(nof_cbs), crcs(nof_cbs, 0)
  {
    for (unsigned i = 0; i != nof_cbs; ++i) {
      soft[i].assign(3 * 8448 + 64, log_likelihood_ratio(0));
      data[i].resize(8448 + 64);
    }
  }
  unsigned   get_nof_codeblocks() const override { return soft.size(); }
  void       reset_codeblocks_crc() override { std::fill(crcs.begin(), crcs.end(), 0); }
  span<bool> get_codeblocks_crc() override { return span<bool>(reinterpret_cast<bool*>(crcs.data()), crcs.size()); }
  unsigned   get_absolute_codeblock_id(unsigned codeblock_id) const override { return codeblock_id; }
  span<log_likelihood_ratio> get_codeblock_soft_bits(unsigned id, unsigned size) override
  {
    return span<log_likelihood_ratio>(soft[id]).first(size);
  }
  bit_buffer get_codeblock_data_bits(unsigned id, unsigned size) override { return data[id].first(size); }
  bool       try_lock() override { return true; }
  void       unlock() override {}
  void       release() override {}

private:
  std::vector<std::vector<log_likelihood_ratio>> soft;
  std::vector<dynamic_bit_buffer>                data;
  std::vector<char>                              crcs;
};

inline std::unique_ptr<crc_calculator> make_crc(crc_generator_poly poly, impl choice)
{
  if (poly == crc_generator_poly::CRC6 || choice == impl::generic) {
    return std::make_unique<crc_calculator_generic_impl>(poly);
  }
  if (host_has_clmul()) {
    return std::make_unique<crc_calculator_clmul_impl>(poly);
  }
  return std::make_unique<crc_calculator_lut_impl>(poly);
}

inline std::unique_ptr<ldpc_decoder> make_ldpc_decoder(impl choice)
{
  if (choice == impl::automatic && host_has_avx512_ldpc()) {
    return std::make_unique<ldpc_decoder_avx512>(false);
  }
  if (choice != impl::generic) {
    return std::make_unique<ldpc_decoder_avx2>(false);
  }
  return std::make_unique<ldpc_decoder_generic>(false);
}

inline std::unique_ptr<ldpc_rate_dematcher> make_dematcher(impl choice)
{
  if (choice == impl::automatic && host_has_avx512_dematcher()) {
    return std::make_unique<ldpc_rate_dematcher_avx512_impl>();
  }
  if (choice != impl::generic) {
    return std::make_unique<ldpc_rate_dematcher_avx2_impl>();
  }
  return std::make_unique<ldpc_rate_dematcher_impl>();
}

inline const char* describe(impl choice)
{
  static std::string s;
  s = std::string("CRC ") + (choice == impl::generic ? "generic" : (host_has_clmul() ? "clmul" : "lut")) +
      ", LDPC decoder " +
      (choice == impl::generic ? "generic" : (choice == impl::automatic && host_has_avx512_ldpc() ? "avx512" : "avx2")) +
      ", rate dematcher " +
      (choice == impl::generic ? "generic"
                               : (choice == impl::automatic && host_has_avx512_dematcher() ? "avx512" : "avx2"));
  return s.c_str();
}

// pusch_decoder_impl with one codeblock decoder and no executor (codeblocks decoded inline, as the
// reference benchmark with nof_pusch_decoder_threads = 0).
inline std::unique_ptr<pusch_decoder_impl> make_pusch_decoder(impl choice)
{
  std::vector<std::unique_ptr<pusch_codeblock_decoder>> cbdec;
  pusch_codeblock_decoder::sch_crc                      c;
  c.crc16  = make_crc(crc_generator_poly::CRC16, choice);
  c.crc24A = make_crc(crc_generator_poly::CRC24A, choice);
  c.crc24B = make_crc(crc_generator_poly::CRC24B, choice);
  cbdec.emplace_back(std::make_unique<pusch_codeblock_decoder>(make_dematcher(choice), make_ldpc_decoder(choice), c));
  auto                        pool = std::make_shared<pusch_decoder_impl::codeblock_decoder_pool>(cbdec);
  pusch_decoder_impl::sch_crc crcs;
  crcs.crc16  = make_crc(crc_generator_poly::CRC16, choice);
  crcs.crc24A = make_crc(crc_generator_poly::CRC24A, choice);
  crcs.crc24B = make_crc(crc_generator_poly::CRC24B, choice);
  return std::make_unique<pusch_decoder_impl>(
      std::make_unique<ldpc_segmenter_rx_impl>(), pool, std::move(crcs), nullptr, MAX_RB, 4);
}

// fd: 0 none, 1 mean, 2 filter; td: 0 interpolate, 1 average (the reference enums).
inline std::unique_ptr<port_channel_estimator> make_port_estimator(int fd, int td, bool cfo)
{
  time_alignment_estimator_dft_impl::collection_dft_processors dfts;
  for (unsigned n = time_alignment_estimator_dft_impl::min_dft_size; n <= time_alignment_estimator_dft_impl::max_dft_size;
       n *= 2) {
    dfts.emplace(n,
                 std::make_unique<dft_processor_generic_impl>(
                     dft_processor::configuration{n, dft_processor::direction::INVERSE}));
  }
  return std::make_unique<port_channel_estimator_average_impl>(
      std::make_unique<interpolator_linear_impl>(),
      std::make_unique<time_alignment_estimator_dft_impl>(std::move(dfts)),
      static_cast<port_channel_estimator_fd_smoothing_strategy>(fd),
      static_cast<port_channel_estimator_td_interpolation_strategy>(td),
      cfo);
}

// Transform precoder with inverse DFTs for every valid M_rb up to max_nof_rb
// (create_dft_transform_precoder_factory).
inline std::unique_ptr<transform_precoder> make_transform_precoder(unsigned max_nof_rb)
{
  transform_precoder_dft_impl::collection_dft_processors dfts;
  for (unsigned m = 1; m <= max_nof_rb; ++m) {
    if (transform_precoding::is_nof_prbs_valid(m)) {
      dfts.emplace(m,
                   std::make_unique<dft_processor_generic_impl>(
                       dft_processor::configuration{m * NRE, dft_processor::direction::INVERSE}));
    }
  }
  return std::make_unique<transform_precoder_dft_impl>(std::move(dfts));
}

// eq: 0 ZF, 1 MMSE (channel_equalizer_algorithm_type).
// custom: an equalizer to use instead of channel_equalizer_generic_impl (the harness's MI355X adapter).
inline std::unique_ptr<pusch_demodulator_impl> make_pusch_demodulator(int                                eq,
                                                                      unsigned                           max_nof_rb,
                                                                      bool                               compute_post_eq_sinr,
                                                                      bool                               with_transform_precoder,
                                                                      std::unique_ptr<channel_equalizer> custom = nullptr)
{
  return std::make_unique<pusch_demodulator_impl>(
      custom ? std::move(custom)
             : std::make_unique<channel_equalizer_generic_impl>(eq == 0 ? channel_equalizer_algorithm_type::zf
                                                                        : channel_equalizer_algorithm_type::mmse),
      with_transform_precoder ? make_transform_precoder(max_nof_rb) : nullptr,
      std::make_unique<demodulation_mapper_impl>(),
      nullptr,
      std::make_unique<pseudo_random_generator_impl>(),
      max_nof_rb,
      compute_post_eq_sinr);
}

// pusch_processor_impl as pusch_processor_factory_generic builds it (factories.cpp:207-251) with the
// components of the reference PUSCH processor benchmark (pusch_processor_benchmark.cpp:133-140,
// 560-640): ZF equalizer, filter FD smoothing, interpolate TD strategy, CFO compensation, no EVM,
// no post-equalization SINR, the given decoder iterations with early stop.
struct pusch_processor_bundle {
  inline_executor                       exec;
  std::unique_ptr<pusch_processor_impl> proc;
};

inline std::unique_ptr<pusch_processor_bundle>
make_pusch_processor(impl choice, unsigned max_nof_rb, unsigned nof_rx_ports, unsigned max_layers, unsigned iterations,
                     int eq, int fd, int td, bool cfo)
{
  auto b = std::make_unique<pusch_processor_bundle>();
  channel_estimate::channel_estimate_dimensions dims;
  dims.nof_prb       = max_nof_rb;
  dims.nof_symbols   = MAX_NSYMB_PER_SLOT;
  dims.nof_rx_ports  = nof_rx_ports;
  dims.nof_tx_layers = max_layers;
  std::vector<std::unique_ptr<pusch_processor_impl::concurrent_dependencies>> deps;
  deps.emplace_back(std::make_unique<pusch_processor_impl::concurrent_dependencies>(
      std::make_unique<dmrs_pusch_estimator_impl>(std::make_unique<pseudo_random_generator_impl>(),
                                                  std::make_unique<low_papr_sequence_generator_impl>(),
                                                  make_port_estimator(fd, td, cfo),
                                                  b->exec),
      make_pusch_demodulator(eq, max_nof_rb, false, true),
      std::make_unique<ulsch_demultiplex_impl>(),
      make_uci_decoder(),
      dims));
  pusch_processor_impl::configuration cfg;
  cfg.dependencies_pool     = std::make_shared<pusch_processor_impl::concurrent_dependencies_pool_type>(deps);
  cfg.decoder               = make_pusch_decoder(choice);
  cfg.dec_nof_iterations    = iterations;
  cfg.dec_enable_early_stop = true;
  cfg.dec_force_decoding    = false;
  cfg.csi_sinr_calc_method  = channel_state_information::sinr_type::channel_estimator;
  b->proc                   = std::make_unique<pusch_processor_impl>(cfg);
  return b;
}

// ---- defined in the wrappers (libsrsran_ref.so); the adapter harness (adapter_harness.cpp) runs the reference's
// own classes with the MI355X adapters of integration/ injected through them.
std::unique_ptr<pusch_decoder_impl> make_pusch_decoder_with(std::unique_ptr<ldpc_decoder> dec, bool generic);
int pusch_decode_on(pusch_decoder_impl& dec, void* rx_buffer, const int8_t* llrs, unsigned nof_llrs, uint8_t* tb,
                    unsigned tb_bytes, unsigned bg, unsigned rv, unsigned qm, unsigned Nref, unsigned nof_layers,
                    unsigned nof_iterations, int force_decoding, int use_early_stop, int new_data, double* result);
int ofdm_modulate_slot_with(std::unique_ptr<dft_processor> dft, unsigned numerology, unsigned bw_rb, unsigned dft_size,
                            int extended_cp, float scale, double fc, unsigned slot, const uint16_t* grid, float* out);
int ofdm_demodulate_slot_with(std::unique_ptr<dft_processor> dft, unsigned numerology, unsigned bw_rb,
                              unsigned dft_size, int extended_cp, unsigned window_offset, float scale, double fc,
                              unsigned slot, const float* in, uint16_t* grid);
// One port of one slot through a given slot / symbol (de)modulator over a dense [symbol][subcarrier] cbf16 grid
// (the plug-in factories of integration/ofdm_modulator_hip.h, or the reference's own classes).
void ofdm_run_slot_modulator(ofdm_slot_modulator& mod, unsigned nsymb, unsigned nsubc, unsigned slot,
                             const uint16_t* grid, float* out);
void ofdm_run_symbol_modulator(ofdm_symbol_modulator& mod, unsigned nsymb, unsigned nsubc, unsigned slot,
                               const uint16_t* grid, float* out);
void ofdm_run_slot_demodulator(ofdm_slot_demodulator& dem, unsigned nsymb, unsigned nsubc, unsigned slot,
                               const float* in, uint16_t* grid);
void ofdm_run_symbol_demodulator(ofdm_symbol_demodulator& dem, unsigned nsymb, unsigned nsubc, unsigned slot,
                                 const float* in, uint16_t* grid);
// The reference's ofdm_slot_(de)modulator_impl over the generic DFT (the CPU baseline of the plug-in).
std::unique_ptr<ofdm_slot_modulator>   make_ref_ofdm_slot_modulator(const ofdm_modulator_configuration& cfg);
std::unique_ptr<ofdm_slot_demodulator> make_ref_ofdm_slot_demodulator(const ofdm_demodulator_configuration& cfg);
// The reference's ofdm_symbol_demodulator_impl over the generic DFT (what puxch_processor_impl calls per port and
// symbol, puxch_processor_impl.cpp:73-82).
std::unique_ptr<ofdm_symbol_demodulator> make_ref_ofdm_symbol_demodulator(const ofdm_demodulator_configuration& cfg);
// The reference's ofdm_symbol_modulator_impl over the generic DFT (pdxch_processor_impl's modulator).
std::unique_ptr<ofdm_symbol_modulator> make_ref_ofdm_symbol_modulator(const ofdm_modulator_configuration& cfg);
int pusch_demodulate_with(std::unique_ptr<channel_equalizer> eq_impl, const uint32_t* grid, unsigned nof_rx_ports,
                          unsigned nsubc, const uint32_t* estimates, unsigned nof_layers, const float* noise_vars,
                          unsigned rnti, unsigned n_id, int qm, const uint8_t* crbs, unsigned start_symbol,
                          unsigned nof_symbols, unsigned dmrs_symb_mask, int dmrs_type2,
                          unsigned nof_cdm_groups_without_data, int eq, int transform_precoding, int post_eq_sinr,
                          int8_t* llrs, unsigned nof_llrs, float* sinr_out);

} // namespace srs_ref
