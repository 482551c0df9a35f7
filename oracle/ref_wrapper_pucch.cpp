// ref_wrapper_pucch.cpp -- extern "C" glue around the REFERENCE's own PUCCH Format 0 detector, compiled from
// /root/reference by oracle/Makefile into oracle/_ref/libsrsran_ref.so.
//
// TEST INFRASTRUCTURE ONLY: the oracle of tests/test_pucch_gpu.py.
//
// Wrapped reference classes:
//   lib/phy/upper/channel_processors/pucch/pucch_detector_format0.cpp            pucch_detector_format0
//   lib/phy/upper/sequence_generators/low_papr_sequence_collection_impl.cpp      low_papr_sequence_collection_impl
//     (alphas of the PUCCH factory: the 12 cyclic shifts 2 pi n / 12)
// The PDU crosses the boundary as the MI355X C-ABI's srs_amd_pucch_f0_pdu (include/srsran_amd/pucch.h), the result
// as its srs_amd_pucch_f0_result; the grid as a dense complex-bf16 array [port][14][subcarrier].
#include "phy/support/resource_grid_reader_impl.h"
#include "phy/upper/channel_processors/pucch/pucch_detector_format0.h"
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

std::unique_ptr<pucch_detector_format0> make_detector()
{
  // the cyclic shifts of the PUCCH detector factory: alpha_i = 2 pi i / 12
  std::array<float, NRE> alphas;
  for (unsigned i = 0; i != NRE; ++i) {
    alphas[i] = TWOPI * static_cast<float>(i) / static_cast<float>(NRE);
  }
  low_papr_sequence_generator_impl gen;
  return std::make_unique<pucch_detector_format0>(
      std::make_unique<pseudo_random_generator_impl>(),
      std::make_unique<low_papr_sequence_collection_impl>(gen, 1, 0, alphas));
}

} // namespace

extern "C" {

// pucch_detector_format0::detect of one PDU on grid [nof_grid_ports][14][nsubc].
void srs_ref_pucch_f0_detect(const uint32_t* grid, unsigned nof_grid_ports, unsigned nsubc,
                             const srs_amd_pucch_f0_pdu* p, srs_amd_pucch_f0_result* out)
{
  grid_tensor data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  for (unsigned port = 0; port != nof_grid_ports; ++port) {
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, port});
      std::memcpy(row.data(), grid + (port * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * sizeof(cbf16_t));
    }
  }
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

} // extern "C"
