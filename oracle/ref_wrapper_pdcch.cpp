// ref_wrapper_pdcch.cpp -- extern "C" glue around the REFERENCE's own PDCCH processor (DCI encoding, modulation,
// mapping and DM-RS), compiled from /root/reference by oracle/Makefile into oracle/_ref/libsrsran_ref.so.
//
// TEST INFRASTRUCTURE ONLY: the oracle of tests/test_pdcch_gpu.py.
//
// Wrapped reference classes:
//   lib/phy/upper/channel_processors/pdcch/pdcch_processor_impl.cpp       pdcch_processor_impl
//   lib/phy/upper/channel_processors/pdcch/pdcch_encoder_impl.cpp         pdcch_encoder_impl (CRC24C, polar chain)
//   lib/phy/upper/channel_processors/pdcch/pdcch_modulator_impl.cpp       pdcch_modulator_impl
//   lib/phy/upper/signal_processors/pdcch/dmrs_pdcch_processor_impl.cpp   dmrs_pdcch_processor_impl
//   lib/phy/upper/channel_processors/pdcch/pdcch_processor_validator_impl.cpp
//   lib/ran/pdcch/cce_to_prb_mapping.cpp
// The PDU crosses the boundary as the MI355X C-ABI's srs_amd_pdcch_pdu (include/srsran_amd/pdcch.h, converted by
// ref_pdcch_pdu.h), so one ctypes structure drives both; the grid as a dense complex-bf16 array [port][14][subcarrier].
#include "phy/support/resource_grid_mapper_impl.h"
#include "phy/support/resource_grid_writer_impl.h"
#include "phy/generic_functions/precoding/channel_precoder_avx2.h"
#include "phy/upper/channel_coding/crc_calculator_generic_impl.h"
#include "phy/upper/channel_coding/polar/polar_allocator_impl.h"
#include "phy/upper/channel_coding/polar/polar_code_impl.h"
#include "phy/upper/channel_coding/polar/polar_encoder_impl.h"
#include "phy/upper/channel_coding/polar/polar_interleaver_impl.h"
#include "phy/upper/channel_coding/polar/polar_rate_matcher_impl.h"
#include "phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "phy/upper/channel_processors/pdcch/pdcch_encoder_impl.h"
#include "phy/upper/channel_processors/pdcch/pdcch_modulator_impl.h"
#include "phy/upper/channel_processors/pdcch/pdcch_processor_impl.h"
#include "phy/upper/channel_processors/pdcch/pdcch_processor_validator_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "phy/upper/signal_processors/pdcch/dmrs_pdcch_processor_impl.h"
#include "srsran/adt/tensor.h"
#include "srsran/ran/pdcch/cce_to_prb_mapping.h"
#include "ref_pdcch_pdu.h"
#include <atomic>
#include <cstring>
#include <memory>

using namespace srsran;

namespace {

using grid_tensor = dynamic_tensor<static_cast<unsigned>(resource_grid_dimensions::all), cbf16_t, resource_grid_dimensions>;

pdcch_processor::pdu_t to_pdu(const srs_amd_pdcch_pdu& p)
{
  return srs_ref::pdcch_pdu_from_amd(p);
}

std::unique_ptr<pdcch_processor> make_processor()
{
  auto encoder = std::make_unique<pdcch_encoder_impl>(
      std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24C), std::make_unique<polar_interleaver_impl>(),
      std::make_unique<polar_allocator_impl>(), std::make_unique<polar_code_impl>(),
      std::make_unique<polar_encoder_impl>(), std::make_unique<polar_rate_matcher_impl>());
  auto modulator = std::make_unique<pdcch_modulator_impl>(
      std::make_unique<modulation_mapper_lut_impl>(), std::make_unique<pseudo_random_generator_impl>(),
      std::make_unique<resource_grid_mapper_impl>(std::make_unique<channel_precoder_avx2>()));
  auto dmrs = std::make_unique<dmrs_pdcch_processor_impl>(
      std::make_unique<pseudo_random_generator_impl>(),
      std::make_unique<resource_grid_mapper_impl>(std::make_unique<channel_precoder_avx2>()));
  return std::make_unique<pdcch_processor_impl>(std::move(encoder), std::move(modulator), std::move(dmrs));
}

} // namespace

extern "C" {

// pdcch_processor_impl::process (pdcch_processor_impl.cpp:79-130) of nof_pdus PDUs in order onto one grid
// [nof_grid_ports][14][nsubc] (modified in place).  Returns 0, or -1 (msg filled) when the reference validator
// rejects a PDU (nothing processed).
int srs_ref_pdcch_process(uint16_t* grid, unsigned nof_grid_ports, unsigned nsubc, const srs_amd_pdcch_pdu* pdus,
                          unsigned nof_pdus, char* msg, unsigned msg_size)
{
  std::vector<pdcch_processor::pdu_t> list;
  for (unsigned i = 0; i != nof_pdus; ++i) {
    list.push_back(to_pdu(pdus[i]));
    error_type<std::string> ok = pdcch_processor_validator_impl().is_valid(list.back());
    if (!ok.has_value()) {
      std::snprintf(msg, msg_size, "%s", ok.error().c_str());
      return -1;
    }
  }
  std::unique_ptr<pdcch_processor> proc = make_processor();
  grid_tensor                      data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  auto*                            flat = reinterpret_cast<cbf16_t*>(grid);
  for (unsigned p = 0; p != nof_grid_ports; ++p) {
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
      std::memcpy(row.data(), flat + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * sizeof(cbf16_t));
    }
  }
  std::atomic<unsigned>     empty{0};
  resource_grid_writer_impl writer(data, empty);
  for (const auto& pdu : list) {
    proc->process(writer, pdu);
  }
  for (unsigned p = 0; p != nof_grid_ports; ++p) {
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      span<const cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
      std::memcpy(flat + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, row.data(), nsubc * sizeof(cbf16_t));
    }
  }
  return 0;
}

// The reference's CRB list of one DCI (cce_to_prb_mapping_*), in the order the mapping functions return it.
int srs_ref_pdcch_prbs(const srs_amd_pdcch_pdu* p, uint16_t* prbs)
{
  pdcch_processor::pdu_t pdu = to_pdu(*p);
  prb_index_list         l;
  switch (pdu.coreset.cce_to_reg_mapping) {
    case pdcch_processor::cce_to_reg_mapping_type::CORESET0:
      l = cce_to_prb_mapping_coreset0(pdu.coreset.bwp_start_rb, pdu.coreset.bwp_size_rb, pdu.coreset.duration,
                                      pdu.coreset.shift_index, pdu.dci.aggregation_level, pdu.dci.cce_index);
      break;
    case pdcch_processor::cce_to_reg_mapping_type::NON_INTERLEAVED:
      l = cce_to_prb_mapping_non_interleaved(pdu.coreset.bwp_start_rb, pdu.coreset.frequency_resources,
                                             pdu.coreset.duration, pdu.dci.aggregation_level, pdu.dci.cce_index);
      break;
    default:
      l = cce_to_prb_mapping_interleaved(pdu.coreset.bwp_start_rb, pdu.coreset.frequency_resources,
                                         pdu.coreset.duration, pdu.coreset.reg_bundle_size,
                                         pdu.coreset.interleaver_size, pdu.coreset.shift_index,
                                         pdu.dci.aggregation_level, pdu.dci.cce_index);
  }
  for (unsigned i = 0; i != l.size(); ++i) {
    prbs[i] = l[i];
  }
  return static_cast<int>(l.size());
}

} // extern "C"
