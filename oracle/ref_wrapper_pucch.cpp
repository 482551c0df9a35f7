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
#include "phy/generic_functions/dft_processor_generic_impl.h"
#include "phy/upper/channel_processors/pucch/pucch_detector_format0.h"
#include "phy/upper/channel_processors/pucch/pucch_detector_format1.h"
#include "phy/upper/sequence_generators/low_papr_sequence_collection_impl.h"
#include "phy/upper/sequence_generators/low_papr_sequence_generator_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "srsran/adt/tensor.h"
#include "srsran/ran/cyclic_prefix.h"
#include "srsran_amd/pucch.h"
#include <atomic>
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

} // extern "C"
