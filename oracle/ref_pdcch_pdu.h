// ref_pdcch_pdu.h -- TEST INFRASTRUCTURE: srs_amd_pdcch_pdu (include/srsran_amd/pdcch.h) -> the reference's
// pdcch_processor::pdu_t (pdcch_processor.h:55-121), shared by ref_wrapper_pdcch.cpp (the reference processor) and
// phy_harness.cpp (the plug-in driven through the reference interface), so both see the same PDU.
#pragma once

#include "srsran/phy/upper/channel_processors/pdcch/pdcch_processor.h"
#include "srsran_amd/pdcch.h"

namespace srs_ref {

inline srsran::pdcch_processor::pdu_t pdcch_pdu_from_amd(const srs_amd_pdcch_pdu& p)
{
  using namespace srsran;
  pdcch_processor::pdu_t pdu;
  pdu.slot                       = slot_point(p.numerology, p.slot_index);
  pdu.cp                         = cyclic_prefix::NORMAL;
  pdu.coreset.bwp_size_rb        = p.coreset.bwp_size_rb;
  pdu.coreset.bwp_start_rb       = p.coreset.bwp_start_rb;
  pdu.coreset.start_symbol_index = p.coreset.start_symbol_index;
  pdu.coreset.duration           = p.coreset.duration;
  pdu.coreset.frequency_resources.resize(pdcch_constants::MAX_NOF_FREQ_RESOURCES);
  for (unsigned i = 0; i != pdu.coreset.frequency_resources.size(); ++i) {
    pdu.coreset.frequency_resources.set(i, (p.coreset.frequency_resources[i / 8] >> (i % 8)) & 1u);
  }
  pdu.coreset.cce_to_reg_mapping = static_cast<pdcch_processor::cce_to_reg_mapping_type>(p.coreset.cce_to_reg_mapping);
  pdu.coreset.reg_bundle_size    = p.coreset.reg_bundle_size;
  pdu.coreset.interleaver_size   = p.coreset.interleaver_size;
  pdu.coreset.shift_index        = p.coreset.shift_index;
  pdu.dci.rnti                   = p.dci.rnti;
  pdu.dci.n_id_pdcch_dmrs        = p.dci.n_id_pdcch_dmrs;
  pdu.dci.n_id_pdcch_data        = p.dci.n_id_pdcch_data;
  pdu.dci.n_rnti                 = p.dci.n_rnti;
  pdu.dci.cce_index              = p.dci.cce_index;
  pdu.dci.aggregation_level      = p.dci.aggregation_level;
  pdu.dci.dmrs_power_offset_dB   = p.dci.dmrs_power_offset_dB;
  pdu.dci.data_power_offset_dB   = p.dci.data_power_offset_dB;
  pdu.dci.payload.assign(p.dci.payload, p.dci.payload + p.dci.payload_size);
  pdu.dci.precoding = precoding_configuration(1, p.dci.nof_ports, 1, MAX_RB);
  for (unsigned a = 0; a != p.dci.nof_ports; ++a) {
    pdu.dci.precoding.set_coefficient(cf_t(p.dci.weights[a][0], p.dci.weights[a][1]), 0, a, 0);
  }
  return pdu;
}

} // namespace srs_ref
