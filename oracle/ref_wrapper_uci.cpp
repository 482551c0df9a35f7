// ref_wrapper_uci.cpp -- extern "C" glue around the REFERENCE's own UL-SCH demultiplexer
// (lib/phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.cpp) for the UCI-on-PUSCH tests.  Test
// infrastructure only.
//
// Glue (interfaces implemented here, nothing of the reference replaced):
//   recording_buffer   pusch_decoder_buffer that appends every soft bit it is given.
#include "ref_builders.h"
#include "phy/upper/channel_coding/short/short_block_encoder_impl.h"
#include "phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "srsran/adt/bit_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_buffer.h"
#include "srsran/ran/uci/uci_part2_size_calculator.h"
#include <functional>
#include <memory>
#include <vector>

using namespace srsran;

namespace {

class recording_buffer : public pusch_decoder_buffer
{
public:
  span<log_likelihood_ratio> get_next_block_view(unsigned block_size) override
  {
    view.resize(block_size);
    return view;
  }
  void on_new_softbits(span<const log_likelihood_ratio> softbits) override
  {
    data.insert(data.end(), softbits.begin(), softbits.end());
  }
  void on_end_softbits() override
  {
    ended = true;
    if (on_end) {
      on_end();
    }
  }

  std::vector<log_likelihood_ratio> view, data;
  bool                              ended = false;
  std::function<void()>             on_end; // the CSI part 1 buffer configures CSI part 2 here, as the processor does
};

modulation_scheme scheme_uci(int qm)
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

} // namespace

extern "C" {

// ulsch_demultiplex::demultiplex (ulsch_demultiplex_impl.cpp:196-590) of one codeword of nof_llrs descrambled LLRs
// fed as one block with its scrambling sequence (c_init); outputs the UL-SCH, HARQ-ACK and CSI part 1 streams and
// their lengths (counts[3]); returns -1 when a stream did not end.
int srs_ref_ulsch_demultiplex(int qm, unsigned nof_layers, unsigned nof_prb, unsigned start_symbol,
                              unsigned nof_symbols, unsigned nof_harq_ack_rvd, int dmrs_type2, unsigned dmrs_mask,
                              unsigned nof_cdm_groups_without_data, unsigned nof_harq_ack_bits,
                              unsigned nof_enc_harq_ack_bits, unsigned nof_csi_part1_bits,
                              unsigned nof_enc_csi_part1_bits, unsigned c_init, const int8_t* llrs, unsigned nof_llrs,
                              int8_t* sch, int8_t* ack, int8_t* csi1, unsigned* counts)
{
  ulsch_demultiplex::configuration cfg;
  cfg.modulation         = scheme_uci(qm);
  cfg.nof_layers         = nof_layers;
  cfg.nof_prb            = nof_prb;
  cfg.start_symbol_index = start_symbol;
  cfg.nof_symbols        = nof_symbols;
  cfg.nof_harq_ack_rvd   = nof_harq_ack_rvd;
  cfg.dmrs               = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.dmrs_symbol_mask   = symbol_slot_mask(MAX_NSYMB_PER_SLOT);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    if ((dmrs_mask >> l) & 1u) {
      cfg.dmrs_symbol_mask.set(l);
    }
  }
  cfg.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  cfg.nof_harq_ack_bits           = nof_harq_ack_bits;
  cfg.nof_enc_harq_ack_bits       = nof_enc_harq_ack_bits;
  cfg.nof_csi_part1_bits          = nof_csi_part1_bits;
  cfg.nof_enc_csi_part1_bits      = nof_enc_csi_part1_bits;

  pseudo_random_generator_impl prg;
  dynamic_bit_buffer           seq(nof_llrs);
  prg.init(c_init);
  prg.generate(seq);

  // on the heap: the demultiplexer holds a 100 KiB per-OFDM-symbol buffer
  auto                   demux = std::make_unique<ulsch_demultiplex_impl>();
  recording_buffer       b_sch, b_ack, b_csi1;
  pusch_codeword_buffer& cw = demux->demultiplex(b_sch, b_ack, b_csi1, cfg);
  cw.on_new_block(span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llrs), nof_llrs),
                  seq);
  cw.on_end_codeword();
  counts[0] = static_cast<unsigned>(b_sch.data.size());
  counts[1] = static_cast<unsigned>(b_ack.data.size());
  counts[2] = static_cast<unsigned>(b_csi1.data.size());
  for (size_t i = 0; i != b_sch.data.size(); ++i) {
    sch[i] = b_sch.data[i].to_value_type();
  }
  for (size_t i = 0; i != b_ack.data.size(); ++i) {
    ack[i] = b_ack.data[i].to_value_type();
  }
  for (size_t i = 0; i != b_csi1.data.size(); ++i) {
    csi1[i] = b_csi1.data[i].to_value_type();
  }
  const bool ok = b_sch.ended && (nof_harq_ack_bits == 0 || b_ack.ended) && (nof_csi_part1_bits == 0 || b_csi1.ended);
  return ok ? 0 : -1;
}

// As srs_ref_ulsch_demultiplex, with CSI part 2: nof_csi_part2_bits / nof_enc_csi_part2_bits are handed to the
// demultiplexer's set_csi_part2 when the CSI part 1 stream ends, the moment the reference's PUSCH processor does it
// (pusch_processor_impl.cpp:73-103, on_csi_part1 from the CSI part 1 decoder the demultiplexer feeds);
// counts[3] = CSI part 2 LLRs.
int srs_ref_ulsch_demultiplex2(int qm, unsigned nof_layers, unsigned nof_prb, unsigned start_symbol,
                               unsigned nof_symbols, unsigned nof_harq_ack_rvd, int dmrs_type2, unsigned dmrs_mask,
                               unsigned nof_cdm_groups_without_data, unsigned nof_harq_ack_bits,
                               unsigned nof_enc_harq_ack_bits, unsigned nof_csi_part1_bits,
                               unsigned nof_enc_csi_part1_bits, unsigned nof_csi_part2_bits,
                               unsigned nof_enc_csi_part2_bits, unsigned c_init, const int8_t* llrs, unsigned nof_llrs,
                               int8_t* sch, int8_t* ack, int8_t* csi1, int8_t* csi2, unsigned* counts)
{
  ulsch_demultiplex::configuration cfg;
  cfg.modulation         = scheme_uci(qm);
  cfg.nof_layers         = nof_layers;
  cfg.nof_prb            = nof_prb;
  cfg.start_symbol_index = start_symbol;
  cfg.nof_symbols        = nof_symbols;
  cfg.nof_harq_ack_rvd   = nof_harq_ack_rvd;
  cfg.dmrs               = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.dmrs_symbol_mask   = symbol_slot_mask(MAX_NSYMB_PER_SLOT);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    if ((dmrs_mask >> l) & 1u) {
      cfg.dmrs_symbol_mask.set(l);
    }
  }
  cfg.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  cfg.nof_harq_ack_bits           = nof_harq_ack_bits;
  cfg.nof_enc_harq_ack_bits       = nof_enc_harq_ack_bits;
  cfg.nof_csi_part1_bits          = nof_csi_part1_bits;
  cfg.nof_enc_csi_part1_bits      = nof_enc_csi_part1_bits;

  pseudo_random_generator_impl prg;
  dynamic_bit_buffer           seq(nof_llrs);
  prg.init(c_init);
  prg.generate(seq);

  auto             demux = std::make_unique<ulsch_demultiplex_impl>();
  recording_buffer b_sch, b_ack, b_csi1, b_csi2;
  if (nof_csi_part2_bits != 0) {
    b_csi1.on_end = [&]() { demux->set_csi_part2(b_csi2, nof_csi_part2_bits, nof_enc_csi_part2_bits); };
  }
  pusch_codeword_buffer& cw = demux->demultiplex(b_sch, b_ack, b_csi1, cfg);
  cw.on_new_block(span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llrs), nof_llrs),
                  seq);
  cw.on_end_codeword();
  counts[0] = static_cast<unsigned>(b_sch.data.size());
  counts[1] = static_cast<unsigned>(b_ack.data.size());
  counts[2] = static_cast<unsigned>(b_csi1.data.size());
  counts[3] = static_cast<unsigned>(b_csi2.data.size());
  for (size_t i = 0; i != b_sch.data.size(); ++i) {
    sch[i] = b_sch.data[i].to_value_type();
  }
  for (size_t i = 0; i != b_ack.data.size(); ++i) {
    ack[i] = b_ack.data[i].to_value_type();
  }
  for (size_t i = 0; i != b_csi1.data.size(); ++i) {
    csi1[i] = b_csi1.data[i].to_value_type();
  }
  for (size_t i = 0; i != b_csi2.data.size(); ++i) {
    csi2[i] = b_csi2.data[i].to_value_type();
  }
  const bool ok = b_sch.ended && (nof_harq_ack_bits == 0 || b_ack.ended) && (nof_csi_part1_bits == 0 || b_csi1.ended) &&
                  (nof_csi_part2_bits == 0 || b_csi2.ended);
  return ok ? 0 : -1;
}

// uci_part2_get_size (lib/ran/uci/uci_part2_size_calculator.cpp:53-89) of a CSI part 1 payload (one bit per byte) and a
// description given as flat words [nof_entries, then per entry nof_parameters, offset0, width0, offset1, width1,
// map_size, map[16]].
unsigned srs_ref_uci_part2_get_size(const uint8_t* part1, unsigned nof_bits, const uint16_t* w)
{
  uci_payload_type payload(nof_bits);
  for (unsigned i = 0; i != nof_bits; ++i) {
    payload.set(i, part1[i] != 0);
  }
  uci_part2_size_description d;
  for (unsigned e = 0; e != w[0]; ++e) {
    const uint16_t*                    x  = w + 1 + e * 22;
    uci_part2_size_description::entry& en = d.entries.emplace_back();
    for (unsigned q = 0; q != x[0]; ++q) {
      en.parameters.push_back(uci_part2_size_description::parameter{x[1 + 2 * q], static_cast<uint8_t>(x[2 + 2 * q])});
    }
    for (unsigned m = 0; m != x[5]; ++m) {
      en.map.push_back(x[6 + m]);
    }
  }
  return uci_part2_get_size(payload, d);
}

// uci_decoder_impl::decode (uci_decoder_impl.cpp:117-129) of E LLRs into K message bits; returns the uci_status.
int srs_ref_uci_decode(const int8_t* llrs, unsigned E, unsigned K, int qm, uint8_t* message)
{
  auto                        dec = srs_ref::make_uci_decoder();
  uci_decoder::configuration  cfg;
  cfg.modulation = scheme_uci(qm);
  return static_cast<int>(dec->decode(span<uint8_t>(message, K),
                                      span<const log_likelihood_ratio>(
                                          reinterpret_cast<const log_likelihood_ratio*>(llrs), E),
                                      cfg));
}

// short_block_encoder_impl::encode (short_block_encoder_impl.cpp): K <= 11 message bits into E coded bits
// (placeholders as the encoder writes them: 255 = x "one", 254 = y "repeat").
void srs_ref_short_block_encode(const uint8_t* message, unsigned K, unsigned E, int qm, uint8_t* out)
{
  short_block_encoder_impl enc;
  enc.encode(span<uint8_t>(out, E), span<const uint8_t>(message, K), scheme_uci(qm));
}

} // extern "C"
