// ref_chain.cpp -- the REFERENCE's full PDSCH + PUSCH slot chain for one cell,
// built from the reference's own classes compiled from /root/reference
// (oracle/Makefile) with the implementations its "auto" software factories pick
// on this host, run one chain per worker thread.
//
// TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg (the reference CPU PHY
// timed on the GPU box's host cores) and tests/test_pipeline_gpu.py (the
// end-to-end pipeline parity reference).  Never loaded by the product.
//
// Per cell-slot, as the reference upper/lower PHY runs it:
//   PDSCH  pdsch_encoder_impl (ldpc_segmenter_tx_impl with the factory CRC, LDPC
//          encoder AVX2 -- channel_coding_factories.cpp:137-141 --, rate matcher)
//          -> pdsch_modulator_impl (resource_grid_mapper_impl with the factory's
//          AVX512 / AVX2 precoder, precoding_factories.cpp:47-66)
//          -> dmrs_pdsch_processor_impl -> ofdm_slot_modulator_impl per port
//          (generic DFT: FFTW is not in this image, generic_functions_factories.cpp).
//   PUSCH  ofdm_slot_demodulator_impl per port -> pusch_processor_impl (estimator,
//          demodulator, UL-SCH demultiplexer, decoder with the factory's CLMUL CRC,
//          AVX512 LDPC decoder and rate dematcher; ref_builders.h).
#include "ref_builders.h"
#include "phy/generic_functions/precoding/channel_precoder_avx2.h"
#include "phy/generic_functions/precoding/channel_precoder_avx512.h"
#include "phy/lower/modulation/ofdm_demodulator_impl.h"
#include "phy/lower/modulation/ofdm_modulator_impl.h"
#include "phy/support/resource_grid_mapper_impl.h"
#include "phy/support/resource_grid_reader_impl.h"
#include "phy/support/resource_grid_writer_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_encoder_avx2.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.h"
#include "phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "phy/upper/channel_processors/pdsch/pdsch_encoder_impl.h"
#include "phy/upper/channel_processors/pdsch/pdsch_modulator_impl.h"
#include "phy/upper/signal_processors/pdsch/dmrs_pdsch_processor_impl.h"
#include "srsran/adt/tensor.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_processor_result_notifier.h"
#include "srsran/ran/sch/sch_constants.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc.h"
#include "srsran/srsvec/bit.h"
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

using namespace srsran;
using namespace srs_ref;

extern "C" {

// Slot configuration of the pipeline (bench_pipeline.py builds it; same layout as RefChainConfig there).
struct srs_ref_chain_config {
  uint32_t numerology, slot, nof_prb, dft_size;
  uint32_t rnti, n_id, qm, dmrs_symbol_mask, nof_cdm_groups_without_data;
  // PDSCH
  uint32_t dl_layers, dl_ports, dl_start, dl_nsym, dl_tbs, dl_bg;
  float    dl_weights[4 * 4 * 2]; // [layer][port] complex
  float    dl_dmrs_amplitude;
  // PUSCH
  uint32_t ul_layers, ul_ports, ul_start, ul_nsym, ul_tbs, ul_bg, ul_iterations;
  float    ul_target_code_rate;
  int32_t  choice; // 0 generic, 1 avx2, 2 auto
  int32_t  ul_td;  // estimator time-domain strategy: 0 interpolate, 1 average (the reference app's default)
};

} // extern "C"

namespace {

using grid_tensor =
    dynamic_tensor<static_cast<unsigned>(resource_grid_dimensions::all), cbf16_t, resource_grid_dimensions>;

modulation_scheme scheme_of(unsigned qm)
{
  return qm == 2 ? modulation_scheme::QPSK
                 : qm == 4 ? modulation_scheme::QAM16 : qm == 6 ? modulation_scheme::QAM64 : modulation_scheme::QAM256;
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

std::unique_ptr<channel_precoder> make_precoder(impl choice)
{
  if (choice == impl::automatic && host_has_avx512_ldpc()) {
    return std::make_unique<channel_precoder_avx512>();
  }
  return std::make_unique<channel_precoder_avx2>();
}

class result_notifier : public pusch_processor_result_notifier
{
public:
  void on_uci(const pusch_processor_result_control&) override {}
  void on_sch(const pusch_processor_result_data& sch) override
  {
    crc_ok = sch.data.tb_crc_ok;
    iters  = static_cast<unsigned>(sch.data.ldpc_decoder_stats.get_mean() *
                                  sch.data.ldpc_decoder_stats.get_nof_observations() + 0.5F);
    done   = true;
  }
  bool     crc_ok = false, done = false;
  unsigned iters  = 0;
};

struct chain {
  const srs_ref_chain_config&            c;
  impl                                   choice;
  std::unique_ptr<pdsch_encoder_impl>    enc;
  std::unique_ptr<pdsch_modulator_impl>  mod;
  std::unique_ptr<dmrs_pdsch_processor_impl> dmrs;
  std::unique_ptr<ofdm_slot_modulator>   ofdm_mod;
  std::unique_ptr<ofdm_slot_demodulator> ofdm_dem;
  std::unique_ptr<pusch_processor_bundle> pusch;
  ref_rx_buffer                          rx_buf;
  grid_tensor                            dl_grid, ul_grid;
  std::atomic<unsigned>                  dl_empty{0}, ul_empty{0};
  std::vector<uint8_t>                   cw_bits;
  dynamic_bit_buffer                     cw;
  std::vector<cf_t>                      dl_samples;
  std::vector<uint8_t>                   tb_out;
  pdsch_encoder::configuration           enc_cfg = {};
  pdsch_modulator::config_t              mod_cfg = {};
  dmrs_pdsch_processor::config_t         dmrs_cfg = {};
  pusch_processor::pdu_t                 pdu = {};
  double                                 stage[5] = {0, 0, 0, 0, 0};
  unsigned                               ok = 0, iters = 0, slots = 0;

  static ofdm_modulator_configuration mod_config(const srs_ref_chain_config& c)
  {
    ofdm_modulator_configuration m;
    m.numerology     = c.numerology;
    m.bw_rb          = c.nof_prb;
    m.dft_size       = c.dft_size;
    m.cp             = cyclic_prefix::NORMAL;
    m.scale          = 1.0F;
    m.center_freq_Hz = 3.5e9;
    return m;
  }

  chain(const srs_ref_chain_config& c_, impl choice_) :
    c(c_),
    choice(choice_),
    rx_buf(ldpc::compute_nof_codeblocks(units::bits(c_.ul_tbs),
                                        c_.ul_bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2)),
    dl_grid({c_.nof_prb * NRE, MAX_NSYMB_PER_SLOT, c_.dl_ports}),
    ul_grid({c_.nof_prb * NRE, MAX_NSYMB_PER_SLOT, c_.ul_ports})
  {
    ldpc_segmenter_tx_impl::sch_crc crcs;
    crcs.crc16  = make_crc(crc_generator_poly::CRC16, choice);
    crcs.crc24A = make_crc(crc_generator_poly::CRC24A, choice);
    crcs.crc24B = make_crc(crc_generator_poly::CRC24B, choice);
    enc         = std::make_unique<pdsch_encoder_impl>(std::make_unique<ldpc_segmenter_tx_impl>(crcs),
                                                       std::make_unique<ldpc_encoder_avx2>(),
                                                       std::make_unique<ldpc_rate_matcher_impl>());
    mod         = std::make_unique<pdsch_modulator_impl>(std::make_unique<modulation_mapper_lut_impl>(),
                                                         std::make_unique<pseudo_random_generator_impl>(),
                                                         std::make_unique<resource_grid_mapper_impl>(make_precoder(choice)));
    dmrs        = std::make_unique<dmrs_pdsch_processor_impl>(std::make_unique<pseudo_random_generator_impl>(),
                                                              std::make_unique<resource_grid_mapper_impl>(make_precoder(choice)));
    {
      ofdm_modulator_common_configuration common;
      common.dft = std::make_unique<dft_processor_generic_impl>(
          dft_processor::configuration{c.dft_size, dft_processor::direction::INVERSE});
      auto cfg = mod_config(c);
      ofdm_mod = std::make_unique<ofdm_slot_modulator_impl>(cfg, std::make_unique<ofdm_symbol_modulator_impl>(common, cfg));
    }
    {
      ofdm_demodulator_configuration cfg;
      cfg.numerology                = c.numerology;
      cfg.bw_rb                     = c.nof_prb;
      cfg.dft_size                  = c.dft_size;
      cfg.cp                        = cyclic_prefix::NORMAL;
      cfg.nof_samples_window_offset = 0;
      cfg.scale                     = 1.0F;
      cfg.center_freq_Hz            = 3.5e9;
      ofdm_demodulator_common_configuration common;
      common.dft = std::make_unique<dft_processor_generic_impl>(
          dft_processor::configuration{c.dft_size, dft_processor::direction::DIRECT});
      ofdm_dem = std::make_unique<ofdm_slot_demodulator_impl>(cfg, std::make_unique<ofdm_symbol_demodulator_impl>(common, cfg));
    }
    pusch = make_pusch_processor(choice, c.nof_prb, c.ul_ports, c.ul_layers, c.ul_iterations, 0, 2, c.ul_td, true);
    dl_samples.resize(ofdm_mod->get_slot_size(c.slot));
    tb_out.resize(c.ul_tbs / 8);
    // PDSCH encoder configuration (bench_pipeline.py: 273 PRB, the DL data REs)
    const unsigned nre_dl = c.nof_prb * NRE * (c.dl_nsym - __builtin_popcount(c.dmrs_symbol_mask & (((1u << c.dl_nsym) - 1) << c.dl_start)));
    enc_cfg.base_graph     = c.dl_bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
    enc_cfg.rv             = 0;
    enc_cfg.mod            = scheme_of(c.qm);
    enc_cfg.Nref           = 0;
    enc_cfg.nof_layers     = c.dl_layers;
    enc_cfg.nof_ch_symbols = nre_dl * c.dl_layers;
    cw_bits.resize(enc_cfg.nof_ch_symbols * c.qm);
    cw.resize(cw_bits.size());
    // PDSCH modulator
    mod_cfg.rnti        = static_cast<uint16_t>(c.rnti);
    mod_cfg.bwp         = crb_interval{0, c.nof_prb};
    mod_cfg.modulation1 = scheme_of(c.qm);
    mod_cfg.modulation2 = scheme_of(c.qm);
    vrb_bitmap vrbs(c.nof_prb);
    vrbs.fill(0, c.nof_prb);
    mod_cfg.freq_allocation             = rb_allocation::make_type0(vrbs);
    mod_cfg.time_alloc                  = ofdm_symbol_range(c.dl_start, c.dl_start + c.dl_nsym);
    mod_cfg.dmrs_symb_pos               = to_symbols(c.dmrs_symbol_mask);
    mod_cfg.dmrs_config_type            = dmrs_type::TYPE1;
    mod_cfg.nof_cdm_groups_without_data = c.nof_cdm_groups_without_data;
    mod_cfg.n_id                        = c.n_id;
    mod_cfg.scaling                     = 1.0F;
    mod_cfg.precoding                   = precoding_configuration(c.dl_layers, c.dl_ports, 1, MAX_RB);
    for (unsigned l = 0; l != c.dl_layers; ++l) {
      for (unsigned p = 0; p != c.dl_ports; ++p) {
        const float* w = c.dl_weights + 2 * (l * c.dl_ports + p);
        mod_cfg.precoding.set_coefficient(cf_t(w[0], w[1]), l, p, 0);
      }
    }
    dmrs_cfg.slot                 = slot_point(c.numerology, c.slot);
    dmrs_cfg.reference_point_k_rb = 0;
    dmrs_cfg.type                 = dmrs_type::TYPE1;
    dmrs_cfg.scrambling_id        = c.n_id;
    dmrs_cfg.n_scid               = false;
    dmrs_cfg.amplitude            = c.dl_dmrs_amplitude;
    dmrs_cfg.symbols_mask         = to_symbols(c.dmrs_symbol_mask);
    dmrs_cfg.rb_mask.resize(MAX_RB);
    dmrs_cfg.rb_mask.fill(0, c.nof_prb);
    dmrs_cfg.precoding = mod_cfg.precoding;
    // PUSCH PDU (pusch_processor_benchmark.cpp:396-431 shape, the pipeline's allocation)
    pdu.slot         = slot_point(c.numerology, c.slot);
    pdu.rnti         = static_cast<uint16_t>(c.rnti);
    pdu.bwp_size_rb  = c.nof_prb;
    pdu.bwp_start_rb = 0;
    pdu.cp           = cyclic_prefix::NORMAL;
    pdu.mcs_descr    = sch_mcs_description{scheme_of(c.qm), c.ul_target_code_rate};
    pdu.codeword.emplace(pusch_processor::codeword_description{
        0, c.ul_bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2, true});
    pdu.uci.alpha_scaling         = 1.0;
    pdu.uci.beta_offset_harq_ack  = 5.0;
    pdu.uci.beta_offset_csi_part1 = 5.0;
    pdu.uci.beta_offset_csi_part2 = 5.0;
    pdu.uci.nof_harq_ack          = 0;
    pdu.uci.nof_csi_part1         = 0;
    pdu.n_id                      = c.n_id;
    pdu.nof_tx_layers             = c.ul_layers;
    for (unsigned p = 0; p != c.ul_ports; ++p) {
      pdu.rx_ports.push_back(static_cast<uint8_t>(p));
    }
    pdu.dmrs_symbol_mask = to_symbols(c.dmrs_symbol_mask);
    pdu.dmrs             = pusch_processor::dmrs_configuration{.dmrs                        = dmrs_type::TYPE1,
                                                               .scrambling_id               = c.n_id,
                                                               .n_scid                      = false,
                                                               .nof_cdm_groups_without_data = c.nof_cdm_groups_without_data};
    pdu.freq_alloc         = rb_allocation::make_type1(0, c.nof_prb);
    pdu.start_symbol_index = c.ul_start;
    pdu.nof_symbols        = c.ul_nsym;
    pdu.tbs_lbrm           = tbs_lbrm_default;
  }

  // One cell-slot: tb_dl -> DL baseband (per port, into dl_samples sequentially); ul_samples [port][slot size]
  // -> decoded UL TB. Outputs optional: dl_grid_out cbf16 [port][14][nsubc], dl_out cf [port][slot size],
  // ul_tb_out.
  void run(const uint8_t* tb_dl, const cf_t* ul_samples, cbf16_t* dl_grid_out, cf_t* dl_out, uint8_t* ul_tb_out)
  {
    using clk = std::chrono::steady_clock;
    auto t0   = clk::now();
    enc->encode(span<uint8_t>(cw_bits), span<const uint8_t>(tb_dl, c.dl_tbs / 8), enc_cfg);
    srsvec::bit_pack(cw, span<const uint8_t>(cw_bits));
    auto t1 = clk::now();
    {
      resource_grid_writer_impl writer(dl_grid, dl_empty);
      bit_buffer                cws[1] = {cw};
      mod->modulate(writer, cws, mod_cfg);
      dmrs->map(writer, dmrs_cfg);
    }
    auto t2 = clk::now();
    {
      resource_grid_reader_impl reader(dl_grid, dl_empty);
      const unsigned            n = ofdm_mod->get_slot_size(c.slot);
      for (unsigned p = 0; p != c.dl_ports; ++p) {
        cf_t* out = dl_out ? dl_out + static_cast<size_t>(p) * n : dl_samples.data();
        ofdm_mod->modulate(span<cf_t>(out, n), reader, p, c.slot);
      }
    }
    auto t3 = clk::now();
    {
      resource_grid_writer_impl writer(ul_grid, ul_empty);
      const unsigned            n = ofdm_dem->get_slot_size(c.slot);
      for (unsigned p = 0; p != c.ul_ports; ++p) {
        ofdm_dem->demodulate(writer, span<const cf_t>(ul_samples + static_cast<size_t>(p) * n, n), p, c.slot);
      }
    }
    auto t4 = clk::now();
    {
      resource_grid_reader_impl reader(ul_grid, ul_empty);
      result_notifier           notifier;
      unique_rx_buffer          buf(rx_buf);
      uint8_t*                  tb = ul_tb_out ? ul_tb_out : tb_out.data();
      pusch->proc->process(span<uint8_t>(tb, c.ul_tbs / 8), std::move(buf), notifier, reader, pdu);
      ok += notifier.done && notifier.crc_ok;
      iters += notifier.iters;
    }
    auto t5 = clk::now();
    stage[0] += std::chrono::duration<double>(t1 - t0).count();
    stage[1] += std::chrono::duration<double>(t2 - t1).count();
    stage[2] += std::chrono::duration<double>(t3 - t2).count();
    stage[3] += std::chrono::duration<double>(t4 - t3).count();
    stage[4] += std::chrono::duration<double>(t5 - t4).count();
    ++slots;
    if (dl_grid_out) {
      for (unsigned p = 0; p != c.dl_ports; ++p) {
        for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
          span<const cbf16_t> row = dl_grid.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
          std::memcpy(dl_grid_out + (static_cast<size_t>(p) * MAX_NSYMB_PER_SLOT + l) * row.size(), row.data(),
                      row.size() * sizeof(cbf16_t));
        }
      }
    }
  }
};

} // namespace

extern "C" {

// Samples per port of one slot (ofdm_slot_modulator::get_slot_size).
unsigned srs_ref_chain_slot_size(const srs_ref_chain_config* c)
{
  chain ch(*c, static_cast<impl>(c->choice));
  return ch.ofdm_mod->get_slot_size(c->slot);
}

// One cell-slot through the reference chain: tb_dl (dl_tbs/8 bytes) -> dl_grid_out cbf16
// [dl_ports][14][nsubc] and dl_samples_out cf [dl_ports][slot size]; ul_samples cf [ul_ports][slot size]
// -> ul_tb_out (ul_tbs/8 bytes). result[0] = PUSCH TB CRC ok, result[1] = LDPC iterations (sum).
int srs_ref_chain_run(const srs_ref_chain_config* c,
                      const uint8_t*              tb_dl,
                      const float*                ul_samples,
                      uint16_t*                   dl_grid_out,
                      float*                      dl_samples_out,
                      uint8_t*                    ul_tb_out,
                      double*                     result)
{
  chain ch(*c, static_cast<impl>(c->choice));
  ch.run(tb_dl,
         reinterpret_cast<const cf_t*>(ul_samples),
         reinterpret_cast<cbf16_t*>(dl_grid_out),
         reinterpret_cast<cf_t*>(dl_samples_out),
         ul_tb_out);
  result[0] = ch.ok;
  result[1] = ch.iters;
  return 0;
}

// CPU baseline: nof_slots cell-slots (all with the same inputs) on `threads` worker threads, one
// reference chain per thread (the chains are built before the clock starts). Returns wall seconds;
// stage_s[5] = summed per-stage seconds over all slots (PDSCH encode, PDSCH modulate + DM-RS, OFDM
// modulate, OFDM demodulate, PUSCH processor); counts[0] = slots with PUSCH TB CRC ok, counts[1] = LDPC
// iterations summed.
double srs_ref_chain_many(const srs_ref_chain_config* c,
                          const uint8_t*              tb_dl,
                          const float*                ul_samples,
                          unsigned                    nof_slots,
                          unsigned                    threads,
                          double*                     stage_s,
                          unsigned*                   counts)
{
  std::vector<std::unique_ptr<chain>> chains;
  for (unsigned t = 0; t != threads; ++t) {
    chains.emplace_back(std::make_unique<chain>(*c, static_cast<impl>(c->choice)));
  }
  std::atomic<unsigned> next{0};
  auto                  t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (unsigned t = 0; t != threads; ++t) {
    pool.emplace_back([&, t]() {
      while (next.fetch_add(1) < nof_slots) {
        chains[t]->run(tb_dl, reinterpret_cast<const cf_t*>(ul_samples), nullptr, nullptr, nullptr);
      }
    });
  }
  for (auto& th : pool) {
    th.join();
  }
  const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (unsigned k = 0; k != 5; ++k) {
    stage_s[k] = 0;
  }
  counts[0] = counts[1] = 0;
  for (auto& ch : chains) {
    for (unsigned k = 0; k != 5; ++k) {
      stage_s[k] += ch->stage[k];
    }
    counts[0] += ch->ok;
    counts[1] += ch->iters;
  }
  return wall;
}

} // extern "C"
