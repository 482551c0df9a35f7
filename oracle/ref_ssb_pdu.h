// ref_ssb_pdu.h -- TEST INFRASTRUCTURE: srs_amd_ssb_pdu (include/srsran_amd/ssb.h) -> the reference's
// ssb_processor::pdu_t (ssb_processor.h:33-62), shared by ref_wrapper_ssb.cpp (the reference processor) and
// phy_harness.cpp (the plug-in driven through the reference interface), so both see the same PDU.
#pragma once

#include "srsran/phy/upper/channel_processors/ssb/ssb_processor.h"
#include "srsran_amd/ssb.h"

namespace srs_ref {

inline srsran::ssb_processor::pdu_t ssb_pdu_from_amd(const srs_amd_ssb_pdu& p)
{
  using namespace srsran;
  ssb_processor::pdu_t pdu;
  pdu.slot              = slot_point(p.numerology, p.sfn, p.slot_index);
  pdu.phys_cell_id      = static_cast<pci_t>(p.phys_cell_id);
  pdu.beta_pss          = p.beta_pss_dB;
  pdu.ssb_idx           = p.ssb_idx;
  pdu.L_max             = p.L_max;
  pdu.common_scs        = static_cast<subcarrier_spacing>(p.common_scs);
  pdu.subcarrier_offset = ssb_subcarrier_offset(p.subcarrier_offset);
  pdu.offset_to_pointA  = ssb_offset_to_pointA(p.offset_to_pointA);
  pdu.pattern_case      = static_cast<ssb_pattern_case>(p.pattern_case);
  for (unsigned i = 0; i != ssb_processor::MIB_PAYLOAD_SIZE; ++i) {
    pdu.mib_payload[i] = p.mib_payload[i];
  }
  for (unsigned i = 0; i != p.nof_ports; ++i) {
    pdu.ports.push_back(p.ports[i]);
  }
  return pdu;
}

} // namespace srs_ref
