// ref_wrapper_pucch.cpp -- extern "C" glue around the REFERENCE's own PUCCH Format 0 / 1 detectors, compiled from
// /root/reference by oracle/Makefile into oracle/_ref/libsrsran_ref.so.
//
// TEST INFRASTRUCTURE ONLY: the oracle of tests/test_pucch_gpu.py.
//
// Wrapped reference classes:
//   lib/phy/upper/channel_processors/pucch/pucch_detector_format0.cpp            pucch_detector_format0
//   lib/phy/upper/channel_processors/pucch/pucch_detector_format1.cpp            pucch_detector_format1
//     (12-point DFT / IDFT: lib/phy/generic_functions/dft_processor_generic_impl.cpp)
//   lib/phy/upper/sequence_generators/low_papr_sequence_collection_impl.cpp      low_papr_sequence_collection_impl
//     (alphas of the PUCCH factory: the 12 cyclic shifts 2 pi n / 12)
// The PDU crosses the boundary as the MI355X C-ABI's srs_amd_pucch_f0_pdu / srs_amd_pucch_f1_batch
// (include/srsran_amd/pucch.h), the result as its srs_amd_pucch_result; the grid as a dense complex-bf16 array
// [port][14][subcarrier].
#include "phy/support/resource_grid_reader_impl.h"
#include "ref_builders.h"
#include "phy/generic_functions/dft_processor_generic_impl.h"
#include "phy/upper/channel_processors/pucch/pucch_demodulator_format2.h"
#include "phy/upper/channel_processors/pucch/pucch_demodulator_format3.h"
#include "phy/upper/channel_processors/pucch/pucch_demodulator_format4.h"
#include "phy/upper/channel_processors/pucch/pucch_demodulator_impl.h"
#include "phy/upper/channel_processors/pucch/pucch_detector_impl.h"
#include "phy/upper/channel_processors/pucch/pucch_processor_impl.h"
#include "phy/upper/signal_processors/pucch/dmrs_pucch_estimator_format2.h"
#include "phy/upper/signal_processors/pucch/dmrs_pucch_estimator_formats3_4.h"
#include "phy/upper/signal_processors/pucch/dmrs_pucch_estimator_impl.h"
#include "phy/upper/channel_processors/pucch/pucch_detector_format0.h"
#include "phy/upper/channel_processors/pucch/pucch_detector_format1.h"
#include "phy/upper/sequence_generators/low_papr_sequence_collection_impl.h"
#include "phy/upper/sequence_generators/low_papr_sequence_generator_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "srsran/adt/tensor.h"
#include "srsran/ran/cyclic_prefix.h"
#include "srsran_amd/pucch.h"
#include <atomic>
#include <chrono>
#include <vector>
#include <cmath>
#include <cstring>
#include <memory>

using namespace srsran;

namespace {

using grid_tensor = dynamic_tensor<static_cast<unsigned>(resource_grid_dimensions::all), cbf16_t, resource_grid_dimensions>;

std::unique_ptr<low_papr_sequence_collection> make_low_papr()
{
  // the cyclic shifts of the PUCCH detector factory: alpha_i = 2 pi i / 12
  std::array<float, NRE> alphas;
  for (unsigned i = 0; i != NRE; ++i) {
    alphas[i] = TWOPI * static_cast<float>(i) / static_cast<float>(NRE);
  }
  low_papr_sequence_generator_impl gen;
  return std::make_unique<low_papr_sequence_collection_impl>(gen, 1, 0, alphas);
}

std::unique_ptr<pucch_detector_format0> make_detector()
{
  return std::make_unique<pucch_detector_format0>(std::make_unique<pseudo_random_generator_impl>(), make_low_papr());
}

std::unique_ptr<pucch_detector_format1> make_detector_f1()
{
  return std::make_unique<pucch_detector_format1>(
      make_low_papr(),
      std::make_unique<pseudo_random_generator_impl>(),
      std::make_unique<dft_processor_generic_impl>(dft_processor::configuration{NRE, dft_processor::direction::DIRECT}),
      std::make_unique<dft_processor_generic_impl>(
          dft_processor::configuration{NRE, dft_processor::direction::INVERSE}));
}

// pucch_processor_impl as the reference's PUCCH factories assemble it: DM-RS estimators with the FD filter, TD
// averaging and CFO compensation (Format 2) / none (Formats 3, 4) (signal_processors/pucch/factories.cpp:52-64),
// ZF equalizers (upper_phy_factories.cpp:676-677), the UCI decoder.
std::unique_ptr<pucch_processor> make_processor(unsigned nof_prb, unsigned nof_ports)
{
  using namespace srs_ref;
  auto est = std::make_unique<dmrs_pucch_estimator_impl>(
      std::make_unique<dmrs_pucch_estimator_format2>(std::make_unique<pseudo_random_generator_impl>(),
                                                     make_port_estimator(2, 1, true)),
      std::make_unique<dmrs_pucch_estimator_formats3_4>(std::make_unique<pseudo_random_generator_impl>(),
                                                        std::make_unique<low_papr_sequence_generator_impl>(),
                                                        make_port_estimator(2, 1, false)));
  auto det   = std::make_unique<pucch_detector_impl>(make_detector(), make_detector_f1());
  auto eq    = [] { return std::make_unique<channel_equalizer_generic_impl>(channel_equalizer_algorithm_type::zf); };
  auto demod = std::make_unique<pucch_demodulator_impl>(
      std::make_unique<pucch_demodulator_format2>(
          eq(), std::make_unique<demodulation_mapper_impl>(), std::make_unique<pseudo_random_generator_impl>()),
      std::make_unique<pucch_demodulator_format3>(eq(),
                                                  std::make_unique<demodulation_mapper_impl>(),
                                                  std::make_unique<pseudo_random_generator_impl>(),
                                                  make_transform_precoder(16)),
      std::make_unique<pucch_demodulator_format4>(eq(),
                                                  std::make_unique<demodulation_mapper_impl>(),
                                                  std::make_unique<pseudo_random_generator_impl>(),
                                                  make_transform_precoder(16)));
  channel_estimate::channel_estimate_dimensions dims;
  dims.nof_prb       = nof_prb;
  dims.nof_symbols   = MAX_NSYMB_PER_SLOT;
  dims.nof_rx_ports  = nof_ports;
  dims.nof_tx_layers = 1;
  return std::make_unique<pucch_processor_impl>(std::make_unique<pucch_pdu_validator_impl>(dims),
                                                std::move(est),
                                                std::move(det),
                                                std::move(demod),
                                                make_uci_decoder(),
                                                dims);
}

void fill_uci_result(const pucch_processor_result& r, srs_amd_pucch_uci_result* out, uint8_t* payload)
{
  std::memset(out, 0, sizeof(*out));
  out->status        = static_cast<uint32_t>(r.message.get_status());
  out->nof_harq_ack  = r.message.get_harq_ack_bits().size();
  out->nof_sr        = r.message.get_sr_bits().size();
  out->nof_csi_part1 = r.message.get_csi_part1_bits().size();
  out->nof_csi_part2 = r.message.get_csi_part2_bits().size();
  const auto full    = r.message.get_full_payload();
  std::memcpy(payload, full.data(), full.size());
  out->sinr_dB          = r.csi.get_sinr_dB().value_or(NAN);
  out->rsrp_dB          = r.csi.get_rsrp_dB().value_or(NAN);
  out->epre_dB          = r.csi.get_epre_dB().value_or(NAN);
  out->time_alignment_s = r.csi.get_time_alignment().has_value() ? r.csi.get_time_alignment()->to_seconds() : NAN;
  out->cfo_Hz           = r.csi.get_cfo_Hz().value_or(NAN);
}

void fill_grid(grid_tensor& data, const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc)
{
  for (unsigned port = 0; port != nof_grid_ports; ++port) {
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, port});
      std::memcpy(row.data(), grid + (port * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * sizeof(cbf16_t));
    }
  }
}

} // namespace

extern "C" {

// pucch_detector_format0::detect of one PDU on grid [nof_grid_ports][14][nsubc].
void srs_ref_pucch_f0_detect(const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc,
                             const srs_amd_pucch_f0_pdu* p, srs_amd_pucch_f0_result* out)
{
  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  fill_grid(data, grid, nof_grid_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);

  pucch_detector::format0_configuration cfg;
  cfg.slot                 = slot_point(p->numerology, p->slot_index);
  cfg.cp                   = cyclic_prefix::NORMAL;
  cfg.starting_prb         = p->starting_prb;
  if (p->second_hop_prb >= 0) {
    cfg.second_hop_prb = static_cast<unsigned>(p->second_hop_prb);
  }
  cfg.start_symbol_index   = p->start_symbol_index;
  cfg.nof_symbols          = p->nof_symbols;
  cfg.initial_cyclic_shift = p->initial_cyclic_shift;
  cfg.n_id                 = p->n_id;
  cfg.nof_harq_ack         = p->nof_harq_ack;
  cfg.sr_opportunity       = p->sr_opportunity != 0;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    cfg.ports.push_back(p->ports[i]);
  }
  auto det = make_detector();
  auto res = det->detect(reader, cfg);

  std::memset(out, 0, sizeof(*out));
  out->status       = static_cast<uint32_t>(res.first.get_status());
  out->nof_sr       = static_cast<uint32_t>(res.first.get_sr_bits().size());
  out->nof_harq_ack = static_cast<uint32_t>(res.first.get_harq_ack_bits().size());
  if (!res.first.get_sr_bits().empty()) {
    out->sr = res.first.get_sr_bits()[0];
  }
  for (unsigned i = 0; i != res.first.get_harq_ack_bits().size() && i != 2; ++i) {
    out->harq_ack[i] = res.first.get_harq_ack_bits()[i];
  }
  out->sinr_dB          = res.second.get_sinr_dB().value_or(NAN);
  out->rsrp_dB          = res.second.get_rsrp_dB().value_or(NAN);
  out->epre_dB          = res.second.get_epre_dB().value_or(NAN);
  out->detection_metric = std::pow(10.0F, out->sinr_dB / 10.0F);
}

// pucch_detector_format1::detect of one batch on grid [nof_grid_ports][14][nsubc]; the detector reads grid ports
// 0 .. nof_grid_ports - 1 (the batch's ports[] are passed as the configuration's port list, which it does not read).
// out[e] receives the result of batch->entries[e].
void srs_ref_pucch_f1_detect(const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc,
                             const srs_amd_pucch_f1_batch* b, srs_amd_pucch_result* out)
{
  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  fill_grid(data, grid, nof_grid_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);

  pucch_detector::format1_configuration cfg;
  cfg.slot         = slot_point(b->numerology, b->slot_index);
  cfg.cp           = cyclic_prefix::NORMAL;
  cfg.starting_prb = b->starting_prb;
  if (b->second_hop_prb >= 0) {
    cfg.second_hop_prb = static_cast<unsigned>(b->second_hop_prb);
  }
  cfg.start_symbol_index = b->start_symbol_index;
  cfg.nof_symbols        = b->nof_symbols;
  cfg.group_hopping      = pucch_group_hopping::NEITHER;
  for (unsigned i = 0; i != b->nof_ports; ++i) {
    cfg.ports.push_back(b->ports[i]);
  }
  cfg.beta_pucch = 1.0F;
  cfg.n_id       = b->n_id;
  pucch_format1_map<unsigned> mux;
  for (unsigned e = 0; e != b->nof_entries; ++e) {
    mux.insert(b->entries[e].initial_cyclic_shift, b->entries[e].time_domain_occ, b->entries[e].nof_harq_ack);
  }
  auto        det = make_detector_f1();
  const auto& res = det->detect(reader, cfg, mux);
  for (unsigned e = 0; e != b->nof_entries; ++e) {
    const auto& r = res.get(b->entries[e].initial_cyclic_shift, b->entries[e].time_domain_occ);
    std::memset(&out[e], 0, sizeof(out[e]));
    const pucch_uci_message& msg = r.detection_result.uci_message;
    out[e].status                = static_cast<uint32_t>(msg.get_status());
    out[e].nof_sr                = static_cast<uint32_t>(msg.get_sr_bits().size());
    out[e].nof_harq_ack          = static_cast<uint32_t>(msg.get_harq_ack_bits().size());
    for (unsigned i = 0; i != msg.get_harq_ack_bits().size() && i != 2; ++i) {
      out[e].harq_ack[i] = msg.get_harq_ack_bits()[i];
    }
    out[e].detection_metric = r.detection_result.detection_metric;
    out[e].sinr_dB          = r.csi.get_sinr_dB().value_or(NAN);
    out[e].rsrp_dB          = r.csi.get_rsrp_dB().value_or(NAN);
    out[e].epre_dB          = r.csi.get_epre_dB().value_or(NAN);
  }
}

// dmrs_pucch_estimator::estimate + pucch_demodulator::demodulate of one Format 2 PDU (as pucch_processor_impl.cpp:
// 158-201 calls them): llrs[16 nof_prb nof_symbols].
void srs_ref_pucch_f2_demodulate(const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc,
                                 const srs_amd_pucch_f2_pdu* p, int8_t* llrs)
{
  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  fill_grid(data, grid, nof_grid_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);
  using namespace srs_ref;
  dmrs_pucch_estimator_format2 est(std::make_unique<pseudo_random_generator_impl>(), make_port_estimator(2, 1, true));
  pucch_demodulator_format2    dem(std::make_unique<channel_equalizer_generic_impl>(channel_equalizer_algorithm_type::zf),
                                std::make_unique<demodulation_mapper_impl>(),
                                std::make_unique<pseudo_random_generator_impl>());
  const unsigned prb0 = p->bwp_start_rb + p->starting_prb;
  std::optional<unsigned> hop;
  if (p->second_hop_prb >= 0) {
    hop = p->bwp_start_rb + static_cast<unsigned>(p->second_hop_prb);
  }
  dmrs_pucch_estimator::format2_configuration ec;
  ec.slot               = slot_point(p->numerology, p->slot_index);
  ec.cp                 = cyclic_prefix::NORMAL;
  ec.group_hopping      = pucch_group_hopping::NEITHER;
  ec.start_symbol_index = p->start_symbol_index;
  ec.nof_symbols        = p->nof_symbols;
  ec.starting_prb       = prb0;
  ec.second_hop_prb     = hop;
  ec.nof_prb            = p->nof_prb;
  ec.n_id_0             = p->n_id_0;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    ec.ports.push_back(p->ports[i]);
  }
  channel_estimate::channel_estimate_dimensions dims;
  dims.nof_prb       = nsubc / NRE;
  dims.nof_symbols   = MAX_NSYMB_PER_SLOT;
  dims.nof_rx_ports  = p->nof_ports;
  dims.nof_tx_layers = 1;
  channel_estimate ce(dims);
  est.estimate(ce, reader, ec);
  pucch_demodulator::format2_configuration dc;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    dc.rx_ports.push_back(p->ports[i]);
  }
  dc.first_prb          = prb0;
  dc.second_hop_prb     = hop;
  dc.nof_prb            = p->nof_prb;
  dc.start_symbol_index = p->start_symbol_index;
  dc.nof_symbols        = p->nof_symbols;
  dc.rnti               = static_cast<uint16_t>(p->rnti);
  dc.n_id               = p->n_id;
  dem.demodulate(span<log_likelihood_ratio>(reinterpret_cast<log_likelihood_ratio*>(llrs),
                                            16 * p->nof_prb * p->nof_symbols),
                 reader,
                 ce,
                 dc);
}

static void fill_f34(const srs_amd_pucch_f34_pdu* p, pucch_processor::format3_configuration& c)
{
  c.slot         = slot_point(p->numerology, p->slot_index);
  c.cp           = cyclic_prefix::NORMAL;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    c.ports.push_back(p->ports[i]);
  }
  c.bwp_size_rb  = p->bwp_size_rb;
  c.bwp_start_rb = p->bwp_start_rb;
  c.starting_prb = p->starting_prb;
  if (p->second_hop_prb >= 0) {
    c.second_hop_prb = static_cast<unsigned>(p->second_hop_prb);
  }
  c.nof_prb            = p->nof_prb;
  c.start_symbol_index = p->start_symbol_index;
  c.nof_symbols        = p->nof_symbols;
  c.rnti               = static_cast<uint16_t>(p->rnti);
  c.n_id_hopping       = p->n_id_hopping;
  c.n_id_scrambling    = p->n_id_scrambling;
  c.nof_harq_ack       = p->nof_harq_ack;
  c.nof_sr             = p->nof_sr;
  c.nof_csi_part1      = p->nof_csi_part1;
  c.nof_csi_part2      = p->nof_csi_part2;
  c.additional_dmrs    = p->additional_dmrs != 0;
  c.pi2_bpsk           = p->pi2_bpsk != 0;
}

static pucch_processor::format4_configuration to_f4(const srs_amd_pucch_f34_pdu* p)
{
  pucch_processor::format3_configuration c3;
  fill_f34(p, c3);
  pucch_processor::format4_configuration c;
  c.slot               = c3.slot;
  c.cp                 = c3.cp;
  c.ports              = c3.ports;
  c.bwp_size_rb        = c3.bwp_size_rb;
  c.bwp_start_rb       = c3.bwp_start_rb;
  c.starting_prb       = c3.starting_prb;
  c.second_hop_prb     = c3.second_hop_prb;
  c.start_symbol_index = c3.start_symbol_index;
  c.nof_symbols        = c3.nof_symbols;
  c.rnti               = c3.rnti;
  c.n_id_hopping       = c3.n_id_hopping;
  c.n_id_scrambling    = c3.n_id_scrambling;
  c.nof_harq_ack       = c3.nof_harq_ack;
  c.nof_sr             = c3.nof_sr;
  c.nof_csi_part1      = c3.nof_csi_part1;
  c.nof_csi_part2      = c3.nof_csi_part2;
  c.additional_dmrs    = c3.additional_dmrs;
  c.pi2_bpsk           = c3.pi2_bpsk;
  c.occ_index          = p->occ_index;
  c.occ_length         = p->occ_length;
  return c;
}

// pucch_processor_impl::process of one Format 3 / 4 PDU on grid [nof_grid_ports][14][nsubc].
void srs_ref_pucch_f34_process(const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc,
                               const srs_amd_pucch_f34_pdu* p, srs_amd_pucch_uci_result* out, uint8_t* payload)
{
  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  fill_grid(data, grid, nof_grid_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);
  auto                      proc = make_processor(nsubc / NRE, nof_grid_ports);
  if (p->format == 4) {
    fill_uci_result(proc->process(reader, to_f4(p)), out, payload);
  } else {
    pucch_processor::format3_configuration c;
    fill_f34(p, c);
    fill_uci_result(proc->process(reader, c), out, payload);
  }
}

// dmrs_pucch_estimator::estimate + pucch_demodulator::demodulate of one Format 3 / 4 PDU (as
// pucch_processor_impl.cpp:240-289 / 328-378 call them): the descrambled LLRs.
void srs_ref_pucch_f34_demodulate(const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc,
                                  const srs_amd_pucch_f34_pdu* p, int8_t* llrs, unsigned nof_llrs)
{
  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  fill_grid(data, grid, nof_grid_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);
  using namespace srs_ref;
  dmrs_pucch_estimator_formats3_4 est(std::make_unique<pseudo_random_generator_impl>(),
                                      std::make_unique<low_papr_sequence_generator_impl>(),
                                      make_port_estimator(2, 1, false));
  auto eq = [] { return std::make_unique<channel_equalizer_generic_impl>(channel_equalizer_algorithm_type::zf); };
  channel_estimate::channel_estimate_dimensions dims;
  dims.nof_prb       = nsubc / NRE;
  dims.nof_symbols   = MAX_NSYMB_PER_SLOT;
  dims.nof_rx_ports  = p->nof_ports;
  dims.nof_tx_layers = 1;
  channel_estimate ce(dims);
  const unsigned   prb0 = p->bwp_start_rb + p->starting_prb;
  std::optional<unsigned> hop;
  if (p->second_hop_prb >= 0) {
    hop = p->bwp_start_rb + static_cast<unsigned>(p->second_hop_prb);
  }
  static_vector<uint8_t, MAX_PORTS> ports;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    ports.push_back(p->ports[i]);
  }
  span<log_likelihood_ratio> out(reinterpret_cast<log_likelihood_ratio*>(llrs), nof_llrs);
  if (p->format == 4) {
    dmrs_pucch_estimator::format4_configuration ec;
    ec.slot               = slot_point(p->numerology, p->slot_index);
    ec.cp                 = cyclic_prefix::NORMAL;
    ec.group_hopping      = pucch_group_hopping::NEITHER;
    ec.start_symbol_index = p->start_symbol_index;
    ec.nof_symbols        = p->nof_symbols;
    ec.starting_prb       = prb0;
    ec.second_hop_prb     = hop;
    ec.n_id               = p->n_id_hopping;
    ec.ports.assign(ports.begin(), ports.end());
    ec.additional_dmrs = p->additional_dmrs != 0;
    ec.occ_index       = p->occ_index;
    est.estimate(ce, reader, ec);
    pucch_demodulator_format4 dem(
        eq(), std::make_unique<demodulation_mapper_impl>(), std::make_unique<pseudo_random_generator_impl>(),
        make_transform_precoder(16));
    pucch_demodulator::format4_configuration dc;
    dc.rx_ports           = ports;
    dc.first_prb          = prb0;
    dc.second_hop_prb     = hop;
    dc.start_symbol_index = p->start_symbol_index;
    dc.nof_symbols        = p->nof_symbols;
    dc.rnti               = static_cast<uint16_t>(p->rnti);
    dc.n_id               = p->n_id_scrambling;
    dc.additional_dmrs    = p->additional_dmrs != 0;
    dc.pi2_bpsk           = p->pi2_bpsk != 0;
    dc.occ_index          = p->occ_index;
    dc.occ_length         = p->occ_length;
    dem.demodulate(out, reader, ce, dc);
    return;
  }
  dmrs_pucch_estimator::format3_configuration ec;
  ec.slot               = slot_point(p->numerology, p->slot_index);
  ec.cp                 = cyclic_prefix::NORMAL;
  ec.group_hopping      = pucch_group_hopping::NEITHER;
  ec.start_symbol_index = p->start_symbol_index;
  ec.nof_symbols        = p->nof_symbols;
  ec.starting_prb       = prb0;
  ec.second_hop_prb     = hop;
  ec.nof_prb            = p->nof_prb;
  ec.n_id               = p->n_id_hopping;
  ec.ports.assign(ports.begin(), ports.end());
  ec.additional_dmrs = p->additional_dmrs != 0;
  est.estimate(ce, reader, ec);
  pucch_demodulator_format3 dem(
      eq(), std::make_unique<demodulation_mapper_impl>(), std::make_unique<pseudo_random_generator_impl>(),
      make_transform_precoder(16));
  pucch_demodulator::format3_configuration dc;
  dc.rx_ports           = ports;
  dc.first_prb          = prb0;
  dc.second_hop_prb     = hop;
  dc.nof_prb            = p->nof_prb;
  dc.start_symbol_index = p->start_symbol_index;
  dc.nof_symbols        = p->nof_symbols;
  dc.rnti               = static_cast<uint16_t>(p->rnti);
  dc.n_id               = p->n_id_scrambling;
  dc.additional_dmrs    = p->additional_dmrs != 0;
  dc.pi2_bpsk           = p->pi2_bpsk != 0;
  dem.demodulate(out, reader, ce, dc);
}

// CPU baseline of bench.py --workload pucch: one pucch_processor_impl (built once) processes every PDU of the lists
// on grid [nof_grid_ports][14][nsubc], reps times, on the calling thread; returns the seconds taken.  Format 0 / 1
// PDUs carry absolute PRBs (BWP from PRB 0).
double srs_ref_pucch_time(const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc,
                          const srs_amd_pucch_f0_pdu* f0, unsigned n0, const srs_amd_pucch_f1_batch* f1, unsigned n1,
                          const srs_amd_pucch_f2_pdu* f2, unsigned n2, const srs_amd_pucch_f34_pdu* f34, unsigned n34,
                          unsigned reps)
{
  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  fill_grid(data, grid, nof_grid_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);
  auto                      proc = make_processor(nsubc / NRE, nof_grid_ports);
  std::vector<pucch_processor::format0_configuration>       c0(n0);
  std::vector<pucch_processor::format1_batch_configuration> c1(n1);
  std::vector<pucch_processor::format2_configuration>       c2(n2);
  std::vector<pucch_processor::format3_configuration>       c3;
  std::vector<pucch_processor::format4_configuration>       c4;
  for (unsigned i = 0; i != n0; ++i) {
    const srs_amd_pucch_f0_pdu& p = f0[i];
    auto&                       c = c0[i];
    c.slot                        = slot_point(p.numerology, p.slot_index);
    c.cp                          = cyclic_prefix::NORMAL;
    c.bwp_size_rb                 = nsubc / NRE;
    c.bwp_start_rb                = 0;
    c.starting_prb                = p.starting_prb;
    if (p.second_hop_prb >= 0) {
      c.second_hop_prb = static_cast<unsigned>(p.second_hop_prb);
    }
    c.start_symbol_index   = p.start_symbol_index;
    c.nof_symbols          = p.nof_symbols;
    c.initial_cyclic_shift = p.initial_cyclic_shift;
    c.n_id                 = p.n_id;
    c.nof_harq_ack         = p.nof_harq_ack;
    c.sr_opportunity       = p.sr_opportunity != 0;
    for (unsigned k = 0; k != p.nof_ports; ++k) {
      c.ports.push_back(p.ports[k]);
    }
  }
  for (unsigned i = 0; i != n1; ++i) {
    const srs_amd_pucch_f1_batch& b = f1[i];
    auto&                         c = c1[i].common_config;
    c.slot                          = slot_point(b.numerology, b.slot_index);
    c.bwp_size_rb                   = nsubc / NRE;
    c.bwp_start_rb                  = 0;
    c.cp                            = cyclic_prefix::NORMAL;
    c.starting_prb                  = b.starting_prb;
    if (b.second_hop_prb >= 0) {
      c.second_hop_prb = static_cast<unsigned>(b.second_hop_prb);
    }
    c.n_id = b.n_id;
    for (unsigned k = 0; k != b.nof_ports; ++k) {
      c.ports.push_back(b.ports[k]);
    }
    c.nof_symbols        = b.nof_symbols;
    c.start_symbol_index = b.start_symbol_index;
    for (unsigned e = 0; e != b.nof_entries; ++e) {
      c1[i].entries.insert(b.entries[e].initial_cyclic_shift, b.entries[e].time_domain_occ,
                           {.context = std::nullopt, .nof_harq_ack = b.entries[e].nof_harq_ack});
    }
  }
  for (unsigned i = 0; i != n2; ++i) {
    const srs_amd_pucch_f2_pdu& p = f2[i];
    auto&                       c = c2[i];
    c.slot                        = slot_point(p.numerology, p.slot_index);
    c.bwp_size_rb                 = p.bwp_size_rb;
    c.bwp_start_rb                = p.bwp_start_rb;
    c.cp                          = cyclic_prefix::NORMAL;
    c.starting_prb                = p.starting_prb;
    if (p.second_hop_prb >= 0) {
      c.second_hop_prb = static_cast<unsigned>(p.second_hop_prb);
    }
    c.nof_prb            = p.nof_prb;
    c.start_symbol_index = p.start_symbol_index;
    c.nof_symbols        = p.nof_symbols;
    c.rnti               = static_cast<uint16_t>(p.rnti);
    c.n_id               = p.n_id;
    c.n_id_0             = p.n_id_0;
    c.nof_harq_ack       = p.nof_harq_ack;
    c.nof_sr             = p.nof_sr;
    c.nof_csi_part1      = p.nof_csi_part1;
    c.nof_csi_part2      = p.nof_csi_part2;
    for (unsigned k = 0; k != p.nof_ports; ++k) {
      c.ports.push_back(p.ports[k]);
    }
  }
  for (unsigned i = 0; i != n34; ++i) {
    if (f34[i].format == 4) {
      c4.push_back(to_f4(&f34[i]));
    } else {
      c3.emplace_back();
      fill_f34(&f34[i], c3.back());
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned r = 0; r != reps; ++r) {
    for (const auto& c : c0) {
      (void)proc->process(reader, c);
    }
    for (const auto& c : c1) {
      (void)proc->process(reader, c);
    }
    for (const auto& c : c2) {
      (void)proc->process(reader, c);
    }
    for (const auto& c : c3) {
      (void)proc->process(reader, c);
    }
    for (const auto& c : c4) {
      (void)proc->process(reader, c);
    }
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// pucch_processor_impl::process of one Format 2 PDU on grid [nof_grid_ports][14][nsubc].
void srs_ref_pucch_f2_process(const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc,
                              const srs_amd_pucch_f2_pdu* p, srs_amd_pucch_uci_result* out, uint8_t* payload)
{
  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  fill_grid(data, grid, nof_grid_ports, nsubc);
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader(data, empty);

  pucch_processor::format2_configuration cfg;
  cfg.slot         = slot_point(p->numerology, p->slot_index);
  cfg.bwp_size_rb  = p->bwp_size_rb;
  cfg.bwp_start_rb = p->bwp_start_rb;
  cfg.cp           = cyclic_prefix::NORMAL;
  cfg.starting_prb = p->starting_prb;
  if (p->second_hop_prb >= 0) {
    cfg.second_hop_prb = static_cast<unsigned>(p->second_hop_prb);
  }
  cfg.nof_prb            = p->nof_prb;
  cfg.start_symbol_index = p->start_symbol_index;
  cfg.nof_symbols        = p->nof_symbols;
  cfg.rnti               = static_cast<uint16_t>(p->rnti);
  cfg.n_id               = p->n_id;
  cfg.n_id_0             = p->n_id_0;
  cfg.nof_harq_ack       = p->nof_harq_ack;
  cfg.nof_sr             = p->nof_sr;
  cfg.nof_csi_part1      = p->nof_csi_part1;
  cfg.nof_csi_part2      = p->nof_csi_part2;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    cfg.ports.push_back(p->ports[i]);
  }
  auto proc = make_processor(nsubc / NRE, nof_grid_ports);
  fill_uci_result(proc->process(reader, cfg), out, payload);
}

} // extern "C"
