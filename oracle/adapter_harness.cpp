// adapter_harness.cpp -- TEST INFRASTRUCTURE: runs the REFERENCE's own classes (compiled from /root/reference into
// oracle/_ref/libsrsran_ref.so) with the MI355X adapters of integration/ injected where the reference's factories
// would plug them, so tests/test_integration_gpu.py checks each adapter THROUGH reference code:
//   pdsch_encoder_hw_impl  (pdsch_encoder_hw_impl.cpp)  + hip_accelerator_pdsch_enc   vs pdsch_encoder_impl
//   ofdm_slot_(de)modulator_impl (ofdm_(de)modulator_impl.cpp) + dft_processor_hip     vs the generic DFT
//   pusch_demodulator_impl (pusch_demodulator_impl.cpp) + channel_equalizer_hip        vs channel_equalizer_generic
//   ofdm_modulator_factory / ofdm_demodulator_factory plug-ins (ofdm_modulator_hip)      vs ofdm_slot_*_impl
//   pusch_decoder_impl / pusch_codeblock_decoder (pusch_codeblock_decoder.cpp) + ldpc_decoder_hip
//                                                                                        vs the AVX2 / generic decoders
// Built by oracle/Makefile into oracle/_ref/libsrsran_ref_hw.so with hw_harness.cpp.  Never loaded by the product.
#include "ref_builders.h"

#include "../integration/channel_equalizer_hip.h"
#include "../integration/dft_processor_hip.h"
#include "../integration/hip_accelerator_pdsch_enc.h"
#include "../integration/ldpc_decoder_hip.h"
#include "../integration/ofdm_modulator_hip.h"
#include "phy/upper/channel_coding/crc_calculator_generic_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.h"
#include "phy/upper/channel_processors/pdsch/pdsch_encoder_hw_impl.h"
#include <chrono>
#include <map>
#include <memory>

using namespace srsran;

namespace {

modulation_scheme scheme(unsigned qm)
{
  switch (qm) {
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

// pdsch_encoder_hw_impl as pdsch_encoder_factory_hw builds it (factories.cpp), with the MI355X accelerator.
std::unique_ptr<pdsch_encoder_hw_impl> make_pdsch_encoder_hw(int device, bool cb_mode)
{
  ldpc_segmenter_tx_impl::sch_crc seg_crc;
  seg_crc.crc16  = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC16);
  seg_crc.crc24A = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24A);
  seg_crc.crc24B = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24B);
  pdsch_encoder_hw_impl::sch_crc crcs;
  crcs.crc16  = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC16);
  crcs.crc24A = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24A);
  crcs.crc24B = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24B);
  hip::pdsch_enc_accelerator_config acc;
  acc.device  = device;
  acc.cb_mode = cb_mode;
  auto factory = hip::create_hip_pdsch_enc_acc_factory(acc);
  return std::make_unique<pdsch_encoder_hw_impl>(crcs, std::make_unique<ldpc_segmenter_tx_impl>(seg_crc),
                                                 factory->create());
}

} // namespace

extern "C" {

/* pdsch_encoder::encode through the reference's pdsch_encoder_hw_impl and the MI355X accelerator (TB mode, or CB
 * mode when cb_mode != 0): codeword nof_ch_symbols * qm entries, one bit per byte (as srs_ref_pdsch_encode). */
int srs_ref_hw_pdsch_encode(int            device,
                            int            cb_mode,
                            const uint8_t* tb,
                            unsigned       tb_bytes,
                            unsigned       bg,
                            unsigned       rv,
                            unsigned       qm,
                            unsigned       Nref,
                            unsigned       nof_layers,
                            unsigned       nof_ch_symbols,
                            uint8_t*       codeword)
{
  static std::map<int, std::unique_ptr<pdsch_encoder_hw_impl>> encs;
  auto&                                                         enc = encs[cb_mode != 0];
  if (!enc) {
    enc = make_pdsch_encoder_hw(device, cb_mode != 0);
  }
  pdsch_encoder::configuration cfg;
  cfg.base_graph     = bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  cfg.rv             = rv;
  cfg.mod            = scheme(qm);
  cfg.Nref           = Nref;
  cfg.nof_layers     = nof_layers;
  cfg.nof_ch_symbols = nof_ch_symbols;
  enc->encode(span<uint8_t>(codeword, nof_ch_symbols * qm), span<const uint8_t>(tb, tb_bytes), cfg);
  return 0;
}

/* A failed PDSCH encoding operation must not stall the reference's driver, which calls dequeue_operation until it
 * returns true (pdsch_encoder_hw_impl.cpp:150-160): the plug-in is handed a transport block whose size differs from
 * its configuration (TB mode) and a codeblock shorter than K - F bits (CB mode).  Returns 0 when both dequeues
 * return true on the first call with the configured length of zeros, a negative step number otherwise. */
int srs_ref_hw_pdsch_enc_forced_failure(int device)
{
  for (int cb_mode = 0; cb_mode != 2; ++cb_mode) {
    hip::pdsch_enc_accelerator_config acc;
    acc.device   = device;
    acc.cb_mode  = cb_mode != 0;
    auto factory = hip::create_hip_pdsch_enc_acc_factory(acc);
    auto enc     = factory->create();
    hal::hw_pdsch_encoder_configuration c{};
    c.nof_tb_bits        = 8 * 1000;
    c.nof_tb_crc_bits    = 24;
    c.base_graph_index   = ldpc_base_graph_type::BG1;
    c.modulation         = modulation_scheme::QPSK;
    c.nof_segments       = 1;
    c.nof_short_segments = 0;
    c.rv                 = 0;
    c.cw_length_a        = 0;
    c.cw_length_b        = 17000;
    c.lifting_size       = 384;
    c.Ncb                = 66 * 384;
    c.Nref               = 66 * 384;
    c.nof_segment_bits   = 8024;
    c.nof_filler_bits    = 22 * 384 - 8024;
    c.rm_length          = 17000;
    c.cb_mode            = cb_mode != 0;
    enc->reserve_queue();
    enc->configure_operation(c, 0);
    std::vector<uint8_t> tb(cb_mode ? 10 : 999, 0x5a); // TB one byte short / CB far shorter than K - F
    if (!enc->enqueue_operation(tb, {}, 0)) {
      return -1 - 10 * cb_mode;
    }
    std::vector<uint8_t> cw(17000, 1), packed((17000 + 7) / 8, 0xff);
    if (!enc->dequeue_operation(cw, packed, 0)) {
      return -2 - 10 * cb_mode;
    }
    for (uint8_t b : cw) {
      if (b != 0) {
        return -3 - 10 * cb_mode;
      }
    }
    for (uint8_t b : packed) {
      if (b != 0) {
        return -4 - 10 * cb_mode;
      }
    }
    enc->free_queue();
  }
  return 0;
}

/* ofdm_slot_modulator_impl / ofdm_slot_demodulator_impl of one port with the MI355X dft_processor (layouts as
 * srs_ref_ofdm_modulate_slot / srs_ref_ofdm_demodulate_slot); -1 when the adapter refuses the DFT size. */
int srs_ref_hip_ofdm_modulate_slot(int             device,
                                   unsigned        numerology,
                                   unsigned        bw_rb,
                                   unsigned        dft_size,
                                   int             extended_cp,
                                   float           scale,
                                   double          fc,
                                   unsigned        slot,
                                   const uint16_t* grid,
                                   float*          out)
{
  auto dft = hip::create_dft_processor_factory_hip(device)->create({dft_size, dft_processor::direction::INVERSE});
  return srs_ref::ofdm_modulate_slot_with(std::move(dft), numerology, bw_rb, dft_size, extended_cp, scale, fc, slot,
                                          grid, out);
}

int srs_ref_hip_ofdm_demodulate_slot(int          device,
                                     unsigned     numerology,
                                     unsigned     bw_rb,
                                     unsigned     dft_size,
                                     int          extended_cp,
                                     unsigned     window_offset,
                                     float        scale,
                                     double       fc,
                                     unsigned     slot,
                                     const float* in,
                                     uint16_t*    grid)
{
  auto dft = hip::create_dft_processor_factory_hip(device)->create({dft_size, dft_processor::direction::DIRECT});
  return srs_ref::ofdm_demodulate_slot_with(std::move(dft), numerology, bw_rb, dft_size, extended_cp, window_offset,
                                            scale, fc, slot, in, grid);
}

/* pusch_demodulator_impl with the MI355X channel_equalizer (arguments as srs_ref_pusch_demodulate). */
int srs_ref_hip_pusch_demodulate(int             device,
                                 const uint32_t* grid,
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
  auto eq_impl = hip::create_channel_equalizer_factory_hip(
                     eq == 0 ? channel_equalizer_algorithm_type::zf : channel_equalizer_algorithm_type::mmse, device)
                     ->create();
  if (!eq_impl) {
    return -2;
  }
  return srs_ref::pusch_demodulate_with(std::move(eq_impl), grid, nof_rx_ports, nsubc, estimates, nof_layers,
                                        noise_vars, rnti, n_id, qm, crbs, start_symbol, nof_symbols, dmrs_symb_mask,
                                        dmrs_type2, nof_cdm_groups_without_data, eq, transform_precoding,
                                        post_eq_sinr, llrs, nof_llrs, sinr_out);
}

/* pusch_decoder_impl (the reference's rate dematcher, segmenter, CRCs and pusch_codeblock_decoder) whose LDPC
 * decoder is the MI355X ldpc_decoder adapter ("hip" = the AVX2/AVX512 arithmetic with the AVX2 dematcher,
 * generic != 0: "hip-generic" with the generic dematcher). Arguments / result as srs_ref_pusch_decode. */
int srs_ref_hip_ldpc_pusch_decode(int           device,
                                  void*         rx_buffer,
                                  const int8_t* llrs,
                                  unsigned      nof_llrs,
                                  uint8_t*      tb,
                                  unsigned      tb_bytes,
                                  unsigned      bg,
                                  unsigned      rv,
                                  unsigned      qm,
                                  unsigned      Nref,
                                  unsigned      nof_layers,
                                  unsigned      nof_iterations,
                                  int           force_decoding,
                                  int           use_early_stop,
                                  int           new_data,
                                  int           generic,
                                  double*       result)
{
  static std::map<std::pair<int, int>, std::unique_ptr<pusch_decoder_impl>> decs;
  auto& dec = decs[{generic != 0, force_decoding != 0}];
  if (!dec) {
    auto f = hip::create_ldpc_decoder_factory_hip(generic ? "hip-generic" : "hip", force_decoding != 0, device);
    dec    = srs_ref::make_pusch_decoder_with(f->create(), generic != 0);
  }
  return srs_ref::pusch_decode_on(*dec, rx_buffer, llrs, nof_llrs, tb, tb_bytes, bg, rv, qm, Nref, nof_layers,
                                  nof_iterations, force_decoding, use_early_stop, new_data, result);
}

} // extern "C"

namespace {

ofdm_modulator_configuration ofdm_mod_cfg(unsigned mu, unsigned bw_rb, unsigned dft_size, int ext, float scale,
                                          double fc)
{
  ofdm_modulator_configuration c;
  c.numerology     = mu;
  c.bw_rb          = bw_rb;
  c.dft_size       = dft_size;
  c.cp             = ext ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  c.scale          = scale;
  c.center_freq_Hz = fc;
  return c;
}

ofdm_demodulator_configuration ofdm_dem_cfg(unsigned mu, unsigned bw_rb, unsigned dft_size, int ext, unsigned offset,
                                            float scale, double fc)
{
  ofdm_demodulator_configuration c;
  c.numerology                = mu;
  c.bw_rb                     = bw_rb;
  c.dft_size                  = dft_size;
  c.cp                        = ext ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  c.nof_samples_window_offset = offset;
  c.scale                     = scale;
  c.center_freq_Hz            = fc;
  return c;
}

} // namespace

extern "C" {

/* One port of one slot through the OFDM plug-ins of integration/ofdm_modulator_hip.h, created by their factories:
 * mode 0 ofdm_slot_modulator, 1 ofdm_symbol_modulator (the slot's symbols one by one; fc2 != fc: after
 * set_center_frequency(fc2)), 2 ofdm_slot_demodulator, 3 ofdm_symbol_demodulator.  Modulators read `grid` and
 * write `samples`, demodulators the reverse.  -1 when a factory refuses the configuration. */
int srs_ref_hw_ofdm_plugin(int             device,
                           int             mode,
                           unsigned        mu,
                           unsigned        bw_rb,
                           unsigned        dft_size,
                           int             ext,
                           unsigned        window_offset,
                           float           scale,
                           double          fc,
                           double          fc2,
                           unsigned        slot,
                           uint16_t*       grid,
                           float*          samples)
{
  const unsigned nsymb = ext ? 12 : 14;
  const unsigned nsubc = bw_rb * NRE;
  if (mode < 2) {
    auto f = hip::create_ofdm_modulator_factory_hip(device);
    auto c = ofdm_mod_cfg(mu, bw_rb, dft_size, ext, scale, fc);
    if (mode == 0) {
      auto m = f->create_ofdm_slot_modulator(c);
      if (!m) {
        return -1;
      }
      srs_ref::ofdm_run_slot_modulator(*m, nsymb, nsubc, slot, grid, samples);
      return 0;
    }
    auto m = f->create_ofdm_symbol_modulator(c);
    if (!m) {
      return -1;
    }
    if (fc2 != fc) {
      m->set_center_frequency(fc2);
    }
    srs_ref::ofdm_run_symbol_modulator(*m, nsymb, nsubc, slot, grid, samples);
    return 0;
  }
  auto f = hip::create_ofdm_demodulator_factory_hip(device);
  auto c = ofdm_dem_cfg(mu, bw_rb, dft_size, ext, window_offset, scale, fc);
  if (mode == 2) {
    auto d = f->create_ofdm_slot_demodulator(c);
    if (!d) {
      return -1;
    }
    srs_ref::ofdm_run_slot_demodulator(*d, nsymb, nsubc, slot, samples, grid);
    return 0;
  }
  auto d = f->create_ofdm_symbol_demodulator(c);
  if (!d) {
    return -1;
  }
  if (fc2 != fc) {
    d->set_center_frequency(fc2);
  }
  srs_ref::ofdm_run_symbol_demodulator(*d, nsymb, nsubc, slot, samples, grid);
  return 0;
}

/* Throughput of slot (de)modulation of one port: `calls` slots through the plug-in (plugin = 1) or the reference's
 * ofdm_slot_(de)modulator_impl over the generic DFT (plugin = 0, this thread), cycling over the slots of a
 * subframe; returns the seconds taken (-1 on a refused configuration). */
double srs_ref_hw_ofdm_bench(int device, int plugin, int demod, unsigned mu, unsigned bw_rb, unsigned dft_size,
                             unsigned calls, const uint16_t* grid, float* samples, uint16_t* grid_out)
{
  const unsigned nsymb = 14, nsubc = bw_rb * NRE, nslots = 1u << mu;
  std::unique_ptr<ofdm_slot_modulator>   mod;
  std::unique_ptr<ofdm_slot_demodulator> dem;
  if (demod) {
    auto c = ofdm_dem_cfg(mu, bw_rb, dft_size, 0, 0, 1.0f, 3.5e9);
    dem    = plugin ? hip::create_ofdm_demodulator_factory_hip(device)->create_ofdm_slot_demodulator(c)
                    : srs_ref::make_ref_ofdm_slot_demodulator(c);
  } else {
    auto c = ofdm_mod_cfg(mu, bw_rb, dft_size, 0, 1.0f, 3.5e9);
    mod    = plugin ? hip::create_ofdm_modulator_factory_hip(device)->create_ofdm_slot_modulator(c)
                    : srs_ref::make_ref_ofdm_slot_modulator(c);
  }
  if (!mod && !dem) {
    return -1;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned k = 0; k != calls; ++k) {
    if (demod) {
      srs_ref::ofdm_run_slot_demodulator(*dem, nsymb, nsubc, k % nslots, samples, grid_out);
    } else {
      srs_ref::ofdm_run_slot_modulator(*mod, nsymb, nsubc, k % nslots, grid, samples);
    }
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

} // extern "C"
