// ref_wrapper_sch.cpp -- extern "C" glue around the REFERENCE's PDSCH encoder and
// PUSCH decoder, compiled from the sources under /root/reference by
// oracle/Makefile into oracle/_ref/libsrsran_ref.so (git-ignored).
//
// TEST INFRASTRUCTURE ONLY: pins oracle/sch.py and the GPU transport-block
// chain in tests/; bench.py's pipeline cpu_baseline times it.  Never loaded by
// the product.
//
// Wrapped reference classes:
//   lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.cpp   (+ ldpc_segmenter_tx_impl, AVX2 LDPC encoder,
//                                                                     ldpc_rate_matcher_impl)
//   lib/phy/upper/channel_processors/pusch/pusch_decoder_impl.cpp   (+ ldpc_segmenter_rx_impl, pusch_codeblock_decoder
//                                                                     with the AVX2 dematcher / decoder)
// The rx_buffer the PUSCH decoder needs is an in-memory implementation of the
// reference's unique_rx_buffer::callback interface (the role of
// lib/phy/upper/rx_buffer_impl.h), kept per HARQ process by the caller.
#include "ref_builders.h"
#include "phy/upper/channel_coding/crc_calculator_generic_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_decoder_avx2.h"
#include "phy/upper/channel_coding/ldpc/ldpc_decoder_generic.h"
#include "phy/upper/channel_coding/ldpc/ldpc_encoder_avx2.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_avx2_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_segmenter_rx_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.h"
#include "phy/upper/channel_processors/pdsch/pdsch_encoder_impl.h"
#include "phy/upper/channel_processors/pusch/pusch_decoder_impl.h"
#include "srsran/adt/bit_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_notifier.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_result.h"
#include "srsran/phy/upper/unique_rx_buffer.h"
#include <chrono>
#include <cstring>
#include <memory>
#include <vector>

using namespace srsran;

namespace {

modulation_scheme scheme_of(unsigned qm)
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

ldpc_segmenter_tx_impl::sch_crc tx_crcs()
{
  ldpc_segmenter_tx_impl::sch_crc c;
  c.crc16  = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC16);
  c.crc24A = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24A);
  c.crc24B = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24B);
  return c;
}

std::unique_ptr<pdsch_encoder_impl> make_pdsch_encoder()
{
  auto crcs = tx_crcs();
  return std::make_unique<pdsch_encoder_impl>(std::make_unique<ldpc_segmenter_tx_impl>(crcs),
                                              std::make_unique<ldpc_encoder_avx2>(),
                                              std::make_unique<ldpc_rate_matcher_impl>());
}

using srs_ref::ref_rx_buffer; // in-memory rx_buffer (one HARQ process), ref_builders.h

class result_catcher : public pusch_decoder_notifier
{
public:
  void on_sch_data(const pusch_decoder_result& r) override
  {
    result = r;
    done   = true;
  }
  pusch_decoder_result result;
  bool                 done = false;
};

std::unique_ptr<pusch_decoder_impl> make_pusch_decoder(bool generic, std::unique_ptr<ldpc_decoder> custom = nullptr)
{
  std::vector<std::unique_ptr<pusch_codeblock_decoder>> cbdec;
  pusch_codeblock_decoder::sch_crc                      c;
  c.crc16  = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC16);
  c.crc24A = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24A);
  c.crc24B = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24B);
  std::unique_ptr<ldpc_decoder>        dec;
  std::unique_ptr<ldpc_rate_dematcher> dm;
  if (generic) {
    dec = std::make_unique<ldpc_decoder_generic>(false);
    dm  = std::make_unique<ldpc_rate_dematcher_impl>();
  } else {
    dec = std::make_unique<ldpc_decoder_avx2>(false);
    dm  = std::make_unique<ldpc_rate_dematcher_avx2_impl>();
  }
  if (custom) {
    dec = std::move(custom); // the decoder under test (srs_ref::make_pusch_decoder_with)
  }
  cbdec.emplace_back(std::make_unique<pusch_codeblock_decoder>(std::move(dm), std::move(dec), c));
  auto pool = std::make_shared<pusch_decoder_impl::codeblock_decoder_pool>(cbdec);
  pusch_decoder_impl::sch_crc crcs;
  crcs.crc16  = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC16);
  crcs.crc24A = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24A);
  crcs.crc24B = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24B);
  return std::make_unique<pusch_decoder_impl>(
      std::make_unique<ldpc_segmenter_rx_impl>(), pool, std::move(crcs), nullptr, MAX_RB, 4);
}

} // namespace

// pusch_decoder_impl (pusch_codeblock_decoder with the generic or AVX2 rate dematcher) around a given LDPC decoder:
// the harness runs the reference decoder chain with the MI355X ldpc_decoder adapter (integration/ldpc_decoder_hip).
std::unique_ptr<pusch_decoder_impl> srs_ref::make_pusch_decoder_with(std::unique_ptr<ldpc_decoder> dec, bool generic)
{
  return ::make_pusch_decoder(generic, std::move(dec));
}

// new_data + on_new_softbits + on_end_softbits on `dec`; result as srs_ref_pusch_decode.
int srs_ref::pusch_decode_on(pusch_decoder_impl& dec,
                             void*               rx_buffer,
                             const int8_t*       llrs,
                             unsigned            nof_llrs,
                             uint8_t*            tb,
                             unsigned            tb_bytes,
                             unsigned            bg,
                             unsigned            rv,
                             unsigned            qm,
                             unsigned            Nref,
                             unsigned            nof_layers,
                             unsigned            nof_iterations,
                             int                 force_decoding,
                             int                 use_early_stop,
                             int                 new_data,
                             double*             result)
{
  pusch_decoder::configuration cfg;
  cfg.base_graph          = bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  cfg.rv                  = rv;
  cfg.mod                 = scheme_of(qm);
  cfg.Nref                = Nref;
  cfg.nof_layers          = nof_layers;
  cfg.nof_ldpc_iterations = nof_iterations;
  cfg.force_decoding      = force_decoding != 0;
  cfg.use_early_stop      = use_early_stop != 0;
  cfg.new_data            = new_data != 0;
  result_catcher   notifier;
  unique_rx_buffer buf(*static_cast<ref_rx_buffer*>(rx_buffer));
  pusch_decoder_buffer& in = dec.new_data(span<uint8_t>(tb, tb_bytes), std::move(buf), notifier, cfg);
  in.on_new_softbits(span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llrs), nof_llrs));
  in.on_end_softbits();
  if (!notifier.done) {
    return -1;
  }
  const auto& st = notifier.result.ldpc_decoder_stats;
  result[0]      = notifier.result.tb_crc_ok ? 1 : 0;
  result[1]      = notifier.result.nof_codeblocks_total;
  result[2]      = st.get_nof_observations();
  result[3]      = st.get_mean() * st.get_nof_observations();
  result[4]      = st.get_min();
  result[5]      = st.get_max();
  return 0;
}

extern "C" {

/* pdsch_encoder::encode: codeword (nof_ch_symbols * qm entries, one bit per byte). */
int srs_ref_pdsch_encode(const uint8_t* tb,
                         unsigned       tb_bytes,
                         unsigned       bg,
                         unsigned       rv,
                         unsigned       qm,
                         unsigned       Nref,
                         unsigned       nof_layers,
                         unsigned       nof_ch_symbols,
                         uint8_t*       codeword)
{
  static thread_local std::unique_ptr<pdsch_encoder_impl> enc = make_pdsch_encoder();
  pdsch_encoder::configuration                            cfg;
  cfg.base_graph     = bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  cfg.rv             = rv;
  cfg.mod            = scheme_of(qm);
  cfg.Nref           = Nref;
  cfg.nof_layers     = nof_layers;
  cfg.nof_ch_symbols = nof_ch_symbols;
  enc->encode(span<uint8_t>(codeword, nof_ch_symbols * qm), span<const uint8_t>(tb, tb_bytes), cfg);
  return 0;
}

/* HARQ process state of the reference PUSCH decoder. */
void* srs_ref_rx_buffer_create(unsigned nof_cbs)
{
  return new ref_rx_buffer(nof_cbs);
}

void srs_ref_rx_buffer_destroy(void* b)
{
  delete static_cast<ref_rx_buffer*>(b);
}

/* pusch_decoder::new_data + on_new_softbits + on_end_softbits.
 * result[0..5] = tb_crc_ok, nof_codeblocks_total, nof observations, sum, min, max of the LDPC statistics. */
int srs_ref_pusch_decode(void*         rx_buffer,
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
  static thread_local std::unique_ptr<pusch_decoder_impl> dec_simd    = make_pusch_decoder(false);
  static thread_local std::unique_ptr<pusch_decoder_impl> dec_generic = make_pusch_decoder(true);
  pusch_decoder_impl&                                     dec         = generic ? *dec_generic : *dec_simd;
  return srs_ref::pusch_decode_on(dec, rx_buffer, llrs, nof_llrs, tb, tb_bytes, bg, rv, qm, Nref, nof_layers,
                                  nof_iterations, force_decoding, use_early_stop, new_data, result);
}

} // extern "C"
