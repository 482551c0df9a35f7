// ref_wrapper_pusch.cpp -- extern "C" glue around the REFERENCE's own PUSCH
// demodulator (pusch_demodulator_impl) and PUSCH processor
// (pusch_processor_impl: DM-RS estimator -> demodulator -> UL-SCH
// demultiplexer -> decoder), compiled from /root/reference by oracle/Makefile
// into oracle/_ref/libsrsran_ref.so.
//
// TEST INFRASTRUCTURE ONLY: pins the GPU PUSCH demodulator and PUSCH processor
// (tests/test_pusch_demod_gpu.py, tests/test_pusch_processor_gpu.py) and the
// configs[0] plumbing run.  Never loaded by the product.
//
// Glue (interfaces implemented here, nothing of the reference replaced; see
// ref_builders.h): an in-memory pusch_codeword_buffer that hands out views
// exactly as pusch_decoder_impl::get_next_block_view does (the requested block,
// pusch_decoder_impl.cpp:140-157) so the demodulator splits its demapper calls
// per OFDM symbol as in the real chain; notifiers that record the results.
#include "ref_builders.h"
#include "srsran/ran/pusch/ulsch_info.h"
#include "phy/support/resource_grid_reader_impl.h"
#include "srsran/adt/tensor.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_codeword_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_demodulator_notifier.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_processor_result_notifier.h"
#include "srsran/ran/sch/sch_constants.h"
#include <atomic>
#include <vector>
#include <cmath>
#include <cstring>

using namespace srsran;
using namespace srs_ref;

namespace {

using grid_tensor =
    dynamic_tensor<static_cast<unsigned>(resource_grid_dimensions::all), cbf16_t, resource_grid_dimensions>;

modulation_scheme scheme_of(int qm)
{
  switch (qm) {
    case 0:
      return modulation_scheme::PI_2_BPSK;
    case 1:
      return modulation_scheme::BPSK;
    case 2:
      return modulation_scheme::QPSK;
    case 4:
      return modulation_scheme::QAM16;
    case 6:
      return modulation_scheme::QAM64;
    default:
      return modulation_scheme::QAM256;
  }
}

symbol_slot_mask to_symbols(unsigned mask)
{
  symbol_slot_mask s(MAX_NSYMB_PER_SLOT);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    if ((mask >> l) & 1u) {
      s.set(l);
    }
  }
  return s;
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

class vector_codeword_buffer : public pusch_codeword_buffer
{
public:
  explicit vector_codeword_buffer(span<log_likelihood_ratio> out_) : out(out_) {}
  span<log_likelihood_ratio> get_next_block_view(unsigned block_size) override
  {
    if (count + block_size > out.size()) {
      std::abort();
    }
    return out.subspan(count, block_size);
  }
  void on_new_block(span<const log_likelihood_ratio> data, const bit_buffer&) override
  {
    if (data.data() != out.data() + count) {
      std::memcpy(out.data() + count, data.data(), data.size());
    }
    count += data.size();
    ++nof_blocks;
  }
  void                       on_end_codeword() override { ended = true; }
  span<log_likelihood_ratio> out;
  unsigned                   count      = 0;
  unsigned                   nof_blocks = 0;
  bool                       ended      = false;
};

class stats_notifier : public pusch_demodulator_notifier
{
public:
  void on_provisional_stats(unsigned i_symbol, const demodulation_stats& stats) override
  {
    if (i_symbol < MAX_NSYMB_PER_SLOT) {
      sinr[i_symbol] = stats.sinr_dB.value_or(NAN);
    }
  }
  void  on_end_stats(const demodulation_stats& stats) override { end_sinr = stats.sinr_dB.value_or(NAN); }
  float sinr[MAX_NSYMB_PER_SLOT] = {NAN, NAN, NAN, NAN, NAN, NAN, NAN, NAN, NAN, NAN, NAN, NAN, NAN, NAN};
  float end_sinr                 = NAN;
};

class result_notifier : public pusch_processor_result_notifier
{
public:
  void on_uci(const pusch_processor_result_control& uci) override
  {
    ++nof_uci;
    uci_csi         = uci.csi;
    harq_ack_status = static_cast<int>(uci.harq_ack.status);
    csi1_status     = static_cast<int>(uci.csi_part1.status);
    csi2_status     = static_cast<int>(uci.csi_part2.status);
    csi2.resize(uci.csi_part2.payload.size());
    for (size_t i = 0; i != csi2.size(); ++i) {
      csi2[i] = uci.csi_part2.payload.test(i) ? 1 : 0;
    }
    harq_ack.resize(uci.harq_ack.payload.size());
    for (size_t i = 0; i != harq_ack.size(); ++i) {
      harq_ack[i] = uci.harq_ack.payload.test(i) ? 1 : 0;
    }
    csi1.resize(uci.csi_part1.payload.size());
    for (size_t i = 0; i != csi1.size(); ++i) {
      csi1[i] = uci.csi_part1.payload.test(i) ? 1 : 0;
    }
  }
  void on_sch(const pusch_processor_result_data& sch) override
  {
    result = sch;
    done   = true;
  }
  pusch_processor_result_data result;
  channel_state_information   uci_csi;
  bool                        done    = false;
  unsigned                    nof_uci = 0;
  int                         harq_ack_status = 0, csi1_status = 0, csi2_status = 0;
  std::vector<uint8_t>        harq_ack, csi1, csi2;
};

} // namespace

// pusch_demodulator_impl with a given channel equalizer (nullptr: channel_equalizer_generic_impl); the harness runs
// it with the MI355X channel_equalizer adapter. Arguments as srs_ref_pusch_demodulate.
int srs_ref::pusch_demodulate_with(std::unique_ptr<channel_equalizer> eq_impl,
                                   const uint32_t*                    grid,
                                   unsigned                           nof_rx_ports,
                                   unsigned                           nsubc,
                                   const uint32_t*                    estimates,
                                   unsigned                           nof_layers,
                                   const float*                       noise_vars,
                                   unsigned                           rnti,
                                   unsigned                           n_id,
                                   int                                qm,
                                   const uint8_t*                     crbs,
                                   unsigned                           start_symbol,
                                   unsigned                           nof_symbols,
                                   unsigned                           dmrs_symb_mask,
                                   int                                dmrs_type2,
                                   unsigned                           nof_cdm_groups_without_data,
                                   int                                eq,
                                   int                                transform_precoding,
                                   int                                post_eq_sinr,
                                   int8_t*                            llrs,
                                   unsigned                           nof_llrs,
                                   float*                             sinr_out)
{
  const unsigned nof_prb = nsubc / NRE;
  auto           demod   = make_pusch_demodulator(eq, nof_prb, post_eq_sinr != 0, transform_precoding != 0,
                                                  std::move(eq_impl));

  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_rx_ports});
  load_grid(data, grid, nof_rx_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);

  channel_estimate::channel_estimate_dimensions dims;
  dims.nof_prb       = nof_prb;
  dims.nof_symbols   = MAX_NSYMB_PER_SLOT;
  dims.nof_rx_ports  = nof_rx_ports;
  dims.nof_tx_layers = nof_layers;
  channel_estimate est(dims);
  for (unsigned p = 0; p != nof_rx_ports; ++p) {
    est.set_noise_variance(noise_vars[p], p);
    for (unsigned v = 0; v != nof_layers; ++v) {
      for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
        span<cbf16_t> s = est.get_symbol_ch_estimate(l, p, v);
        std::memcpy(s.data(), estimates + ((p * nof_layers + v) * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * 4);
      }
    }
  }

  pusch_demodulator::configuration cfg;
  cfg.rnti = static_cast<uint16_t>(rnti);
  cfg.rb_mask.resize(nof_prb);
  for (unsigned i = 0; i != nof_prb; ++i) {
    if (crbs[i]) {
      cfg.rb_mask.set(i);
    }
  }
  cfg.modulation                  = scheme_of(qm);
  cfg.start_symbol_index          = start_symbol;
  cfg.nof_symbols                 = nof_symbols;
  cfg.dmrs_symb_pos               = to_symbols(dmrs_symb_mask);
  cfg.dmrs_config_type            = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  cfg.n_id                        = n_id;
  cfg.nof_tx_layers               = nof_layers;
  cfg.enable_transform_precoding  = transform_precoding != 0;
  for (unsigned p = 0; p != nof_rx_ports; ++p) {
    cfg.rx_ports.push_back(static_cast<uint8_t>(p));
  }

  vector_codeword_buffer buf(span<log_likelihood_ratio>(reinterpret_cast<log_likelihood_ratio*>(llrs), nof_llrs));
  stats_notifier         notifier;
  demod->demodulate(buf, notifier, reader, est, cfg);
  if (buf.count != nof_llrs || !buf.ended) {
    return -1;
  }
  if (sinr_out != nullptr) {
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      sinr_out[l] = notifier.sinr[l];
    }
    sinr_out[MAX_NSYMB_PER_SLOT] = notifier.end_sinr;
  }
  return static_cast<int>(buf.nof_blocks);
}

// CSI part 2 of the next srs_ref_pusch_process call (test glue: the call's argument list stays as it is): the
// uci_part2_size_description as flat uint16 words [nof_entries, then per entry nof_parameters, offset0, width0,
// offset1, width1, map_size, map[16]] and its beta offset; the decoded payload and status of that call.
std::vector<uint16_t> g_part2_descr;
float                 g_part2_beta = 5.0F;
std::vector<uint8_t>  g_part2_out;
int                   g_part2_status = 0;
// pdu_t::dc_position (-1: unset) and a PDU without codeword (UCI only) for the next srs_ref_pusch_process call
int g_dc_position = -1;
int g_no_codeword = 0;

extern "C" {

void srs_ref_pusch_set_options(int dc_position, int no_codeword)
{
  g_dc_position = dc_position;
  g_no_codeword = no_codeword;
}

void srs_ref_pusch_set_csi_part2(const uint16_t* descr, unsigned nof_words, float beta)
{
  g_part2_descr.assign(descr, descr + nof_words);
  g_part2_beta = beta;
}

// the last call's CSI part 2 payload (one bit per byte) into out[max_bits]; returns its size, status in *status
int srs_ref_pusch_get_csi_part2(uint8_t* out, unsigned max_bits, int* status)
{
  *status = g_part2_status;
  for (size_t i = 0; i != g_part2_out.size() && i < max_bits; ++i) {
    out[i] = g_part2_out[i];
  }
  return static_cast<int>(g_part2_out.size());
}

// pusch_demodulator::demodulate (pusch_demodulator_impl.cpp:203-445) of one grid [P][14][nsubc]
// with channel estimates [P][L][14][nsubc] (cbf16 as uint32) and per-port noise variances.
// crbs: 0/1 bytes [nsubc / 12]. eq: 0 ZF, 1 MMSE. llrs: nof_llrs (= data REs x L x Qm) int8.
// sinr_out[15]: per-OFDM-symbol provisional SINR (dB, NaN when not notified) then the final one
// (computed only when post_eq_sinr != 0). Returns the number of codeword blocks the demodulator
// produced, or -1 on a size mismatch.
int srs_ref_pusch_demodulate(const uint32_t* grid,
                             unsigned        nof_rx_ports,
                             unsigned        nsubc,
                             const uint32_t* estimates,
                             unsigned        nof_layers,
                             const float*    noise_vars,
                             unsigned        rnti,
                             unsigned        n_id,
                             int             qm,
                             const uint8_t*  crbs,
                             unsigned        start_symbol,
                             unsigned        nof_symbols,
                             unsigned        dmrs_symb_mask,
                             int             dmrs_type2,
                             unsigned        nof_cdm_groups_without_data,
                             int             eq,
                             int             transform_precoding,
                             int             post_eq_sinr,
                             int8_t*         llrs,
                             unsigned        nof_llrs,
                             float*          sinr_out)
{
  return srs_ref::pusch_demodulate_with(nullptr, grid, nof_rx_ports, nsubc, estimates, nof_layers, noise_vars, rnti,
                                        n_id, qm, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2,
                                        nof_cdm_groups_without_data, eq, transform_precoding, post_eq_sinr, llrs,
                                        nof_llrs, sinr_out);
}

// pusch_processor::process (pusch_processor_impl.cpp:134-386) of one PDU on a received grid
// [P][14][nsubc] (cbf16 as uint32), configured as the reference PUSCH processor benchmark.
// Type-1 contiguous allocation [rb_start, rb_start + rb_count) of a BWP [bwp_start, +bwp_size).
// dmrs_type2: 0 type 1, 1 type 2, 2 transform precoding (low-PAPR DM-RS, n_rs_id = scrambling_id).
// choice: 0 generic, 1 AVX2, 2 the "auto" factory choice (ref_builders.h).
// rx_buffer: srs_ref_rx_buffer_create handle (HARQ process). tb: tb_bytes output bytes.
// UCI: nof_harq_ack / nof_csi_part1 payload bits with their alpha / beta offsets; the decoded payloads (one bit per
// byte) and uci_status values (0 unknown, 1 valid, 2 invalid) come back in harq_ack_out / csi_part1_out /
// uci_status_out[2].
// result[0..5] = tb_crc_ok, nof_codeblocks_total, LDPC observations, sum, min, max;
// csi[0..3] = SINR (channel estimator, dB), EPRE dB, RSRP dB, time alignment (s).
int srs_ref_pusch_process(const uint32_t* grid,
                          unsigned        nof_rx_ports,
                          unsigned        nsubc,
                          unsigned        numerology,
                          unsigned        slot_index,
                          unsigned        rnti,
                          unsigned        bwp_start,
                          unsigned        bwp_size,
                          int             qm,
                          float           target_code_rate,
                          unsigned        rv,
                          unsigned        base_graph,
                          int             new_data,
                          unsigned        n_id,
                          unsigned        nof_layers,
                          unsigned        dmrs_symb_mask,
                          int             dmrs_type2,
                          unsigned        scrambling_id,
                          int             n_scid,
                          unsigned        nof_cdm_groups_without_data,
                          unsigned        rb_start,
                          unsigned        rb_count,
                          unsigned        start_symbol,
                          unsigned        nof_symbols,
                          unsigned        tbs_lbrm_bytes,
                          unsigned        iterations,
                          int             choice,
                          void*           rx_buffer,
                          uint8_t*        tb,
                          unsigned        tb_bytes,
                          double*         result,
                          double*         csi,
                          unsigned        nof_harq_ack,
                          unsigned        nof_csi_part1,
                          float           alpha_scaling,
                          float           beta_harq_ack,
                          float           beta_csi_part1,
                          uint8_t*        harq_ack_out,
                          uint8_t*        csi_part1_out,
                          int*            uci_status_out)
{
  const unsigned nof_prb = nsubc / NRE;
  auto           bundle  = make_pusch_processor(
      static_cast<impl>(choice), nof_prb, nof_rx_ports, nof_layers, iterations, 0, 2, 0, true);

  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_rx_ports});
  load_grid(data, grid, nof_rx_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);

  pusch_processor::pdu_t pdu = {};
  pdu.slot                   = slot_point(numerology, slot_index);
  pdu.rnti                   = static_cast<uint16_t>(rnti);
  pdu.bwp_size_rb            = bwp_size;
  pdu.bwp_start_rb           = bwp_start;
  pdu.cp                     = cyclic_prefix::NORMAL;
  pdu.mcs_descr              = sch_mcs_description{scheme_of(qm), target_code_rate};
  pdu.codeword.emplace(pusch_processor::codeword_description{
      rv, base_graph == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2, new_data != 0});
  pdu.uci.alpha_scaling         = alpha_scaling;
  pdu.uci.beta_offset_harq_ack  = beta_harq_ack;
  pdu.uci.beta_offset_csi_part1 = beta_csi_part1;
  pdu.uci.beta_offset_csi_part2 = g_part2_beta;
  if (!g_part2_descr.empty()) {
    const uint16_t* w = g_part2_descr.data();
    for (unsigned e = 0; e != w[0]; ++e) {
      const uint16_t*                    x  = w + 1 + e * 22;
      uci_part2_size_description::entry& en = pdu.uci.csi_part2_size.entries.emplace_back();
      for (unsigned q = 0; q != x[0]; ++q) {
        en.parameters.push_back(uci_part2_size_description::parameter{x[1 + 2 * q], static_cast<uint8_t>(x[2 + 2 * q])});
      }
      for (unsigned m = 0; m != x[5]; ++m) {
        en.map.push_back(x[6 + m]);
      }
    }
  }
  pdu.uci.nof_harq_ack          = nof_harq_ack;
  pdu.uci.nof_csi_part1         = nof_csi_part1;
  pdu.n_id                      = n_id;
  pdu.nof_tx_layers             = nof_layers;
  for (unsigned p = 0; p != nof_rx_ports; ++p) {
    pdu.rx_ports.push_back(static_cast<uint8_t>(p));
  }
  pdu.dmrs_symbol_mask   = to_symbols(dmrs_symb_mask);
  if (dmrs_type2 == 2) {
    // transform precoding (DFT-s-OFDM): low-PAPR DM-RS of identifier n_rs_id, passed as scrambling_id
    pdu.dmrs = pusch_processor::dmrs_transform_precoding_configuration{.n_rs_id = scrambling_id};
  } else {
    pdu.dmrs = pusch_processor::dmrs_configuration{.dmrs          = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1,
                                                   .scrambling_id = scrambling_id,
                                                   .n_scid        = n_scid != 0,
                                                   .nof_cdm_groups_without_data = nof_cdm_groups_without_data};
  }
  pdu.freq_alloc         = rb_allocation::make_type1(rb_start, rb_count);
  pdu.start_symbol_index = start_symbol;
  pdu.nof_symbols        = nof_symbols;
  pdu.tbs_lbrm           = tbs_lbrm_bytes ? units::bytes(tbs_lbrm_bytes) : tbs_lbrm_default;
  if (g_dc_position >= 0) {
    pdu.dc_position = static_cast<unsigned>(g_dc_position);
  }
  const bool uci_only = g_no_codeword != 0;
  if (uci_only) {
    pdu.codeword.reset();
  }
  g_dc_position = -1;
  g_no_codeword = 0;

  result_notifier  notifier;
  unique_rx_buffer buf = uci_only ? unique_rx_buffer() : unique_rx_buffer(*static_cast<ref_rx_buffer*>(rx_buffer));
  bundle->proc->process(span<uint8_t>(tb, uci_only ? 0 : tb_bytes), std::move(buf), notifier, reader, pdu);
  g_part2_descr.clear();
  g_part2_beta   = 5.0F;
  g_part2_out    = notifier.csi2;
  g_part2_status = notifier.csi2_status;
  if (!(uci_only ? notifier.nof_uci != 0 : notifier.done)) {
    return -1;
  }
  if (uci_status_out != nullptr) {
    uci_status_out[0] = notifier.harq_ack_status;
    uci_status_out[1] = notifier.csi1_status;
    for (size_t i = 0; i != notifier.harq_ack.size() && harq_ack_out != nullptr; ++i) {
      harq_ack_out[i] = notifier.harq_ack[i];
    }
    for (size_t i = 0; i != notifier.csi1.size() && csi_part1_out != nullptr; ++i) {
      csi_part1_out[i] = notifier.csi1[i];
    }
  }
  const pusch_decoder_result& r  = notifier.result.data;
  const auto&                 st = r.ldpc_decoder_stats;
  result[0]                      = r.tb_crc_ok ? 1 : 0;
  result[1]                      = r.nof_codeblocks_total;
  result[2]                      = st.get_nof_observations();
  result[3]                      = st.get_mean() * st.get_nof_observations();
  result[4]                      = st.get_min();
  result[5]                      = st.get_max();
  if (csi != nullptr) {
    const channel_state_information& c = uci_only ? notifier.uci_csi : notifier.result.csi;
    csi[0]                             = c.get_sinr_dB().value_or(NAN);
    csi[1]                             = c.get_epre_dB().value_or(NAN);
    csi[2]                             = c.get_rsrp_dB().value_or(NAN);
    csi[3]                             = c.get_time_alignment().has_value() ? c.get_time_alignment()->to_seconds() : NAN;
  }
  return 0;
}

// get_ulsch_information (lib/ran/pusch/ulsch_info.cpp:158-358). out[15] = nof_ul_sch_bits, nof_harq_ack_bits,
// nof_harq_ack_rvd, nof_csi_part1_bits, nof_csi_part2_bits, nof_harq_ack_re, nof_csi_part1_re, nof_csi_part2_re,
// nof_dc_overlap_bits, then the UL-SCH segmentation: tb_crc_size, base graph, nof_cb, lifting_size,
// nof_bits_per_cb, nof_filler_bits_per_cb (0 without UL-SCH).
void srs_ref_ulsch_information(unsigned tbs, int qm, float target_code_rate, unsigned nof_harq_ack_bits,
                               unsigned nof_csi_part1_bits, unsigned nof_csi_part2_bits, float alpha_scaling,
                               float beta_ack, float beta_csi1, float beta_csi2, unsigned nof_rb,
                               unsigned start_symbol, unsigned nof_symbols, int dmrs_type2, unsigned dmrs_symbol_mask,
                               unsigned nof_cdm_groups_without_data, unsigned nof_layers, int contains_dc,
                               unsigned* out)
{
  ulsch_configuration c;
  c.tbs                         = units::bits(tbs);
  c.mcs_descr                   = sch_mcs_description{scheme_of(qm), target_code_rate};
  c.nof_harq_ack_bits           = units::bits(nof_harq_ack_bits);
  c.nof_csi_part1_bits          = units::bits(nof_csi_part1_bits);
  c.nof_csi_part2_bits          = units::bits(nof_csi_part2_bits);
  c.alpha_scaling               = alpha_scaling;
  c.beta_offset_harq_ack        = beta_ack;
  c.beta_offset_csi_part1       = beta_csi1;
  c.beta_offset_csi_part2       = beta_csi2;
  c.nof_rb                      = nof_rb;
  c.start_symbol_index          = start_symbol;
  c.nof_symbols                 = nof_symbols;
  c.dmrs_type                   = dmrs_type2 ? dmrs_config_type::type2 : dmrs_config_type::type1;
  c.dmrs_symbol_mask            = to_symbols(dmrs_symbol_mask);
  c.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  c.nof_layers                  = nof_layers;
  c.contains_dc                 = contains_dc != 0;
  const ulsch_information r     = get_ulsch_information(c);
  out[0]                        = r.nof_ul_sch_bits.value();
  out[1]                        = r.nof_harq_ack_bits.value();
  out[2]                        = r.nof_harq_ack_rvd.value();
  out[3]                        = r.nof_csi_part1_bits.value();
  out[4]                        = r.nof_csi_part2_bits.value();
  out[5]                        = r.nof_harq_ack_re;
  out[6]                        = r.nof_csi_part1_re;
  out[7]                        = r.nof_csi_part2_re;
  out[8]                        = r.nof_dc_overlap_bits.value();
  for (unsigned i = 9; i != 15; ++i) {
    out[i] = 0;
  }
  if (r.sch.has_value()) {
    out[9]  = r.sch->tb_crc_size.value();
    out[10] = r.sch->base_graph == ldpc_base_graph_type::BG1 ? 1 : 2;
    out[11] = r.sch->nof_cb;
    out[12] = r.sch->lifting_size;
    out[13] = r.sch->nof_bits_per_cb.value();
    out[14] = r.sch->nof_filler_bits_per_cb.value();
  }
}

// Describes what choice 2 ("auto") selects on this host.
const char* srs_ref_describe_choice(int choice)
{
  return describe(static_cast<impl>(choice));
}

} // extern "C"
