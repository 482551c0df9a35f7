// ref_wrapper_ssb.cpp -- extern "C" glue around the REFERENCE's own SS/PBCH block processor (PBCH encoding,
// modulation, DM-RS, PSS and SSS), compiled from /root/reference by oracle/Makefile into oracle/_ref/libsrsran_ref.so.
//
// TEST INFRASTRUCTURE ONLY: the oracle of tests/test_ssb_gpu.py.
//
// Wrapped reference classes:
//   lib/phy/upper/channel_processors/ssb/ssb_processor_impl.cpp       ssb_processor_impl
//   lib/phy/upper/channel_processors/ssb/pbch_encoder_impl.cpp        pbch_encoder_impl (payload, CRC24C, polar chain)
//   lib/phy/upper/channel_processors/ssb/pbch_modulator_impl.cpp      pbch_modulator_impl
//   lib/phy/upper/signal_processors/ssb/dmrs_pbch_processor_impl.cpp  dmrs_pbch_processor_impl
//   lib/phy/upper/signal_processors/ssb/pss_processor_impl.cpp        pss_processor_impl
//   lib/phy/upper/signal_processors/ssb/sss_processor_impl.cpp        sss_processor_impl
// The PDU crosses the boundary as the MI355X C-ABI's srs_amd_ssb_pdu (include/srsran_amd/ssb.h, converted by
// ref_ssb_pdu.h); the grid as a dense complex-bf16 array [port][14][subcarrier].  The reference asserts (aborts) on
// an invalid PDU, so the tests pass only valid ones here.
#include "phy/support/resource_grid_writer_impl.h"
#include "phy/upper/channel_coding/crc_calculator_generic_impl.h"
#include "phy/upper/channel_coding/polar/polar_allocator_impl.h"
#include "phy/upper/channel_coding/polar/polar_code_impl.h"
#include "phy/upper/channel_coding/polar/polar_encoder_impl.h"
#include "phy/upper/channel_coding/polar/polar_interleaver_impl.h"
#include "phy/upper/channel_coding/polar/polar_rate_matcher_impl.h"
#include "phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "phy/upper/channel_processors/ssb/pbch_encoder_impl.h"
#include "phy/upper/channel_processors/ssb/pbch_modulator_impl.h"
#include "phy/upper/channel_processors/ssb/ssb_processor_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "phy/upper/signal_processors/ssb/dmrs_pbch_processor_impl.h"
#include "phy/upper/signal_processors/ssb/pss_processor_impl.h"
#include "phy/upper/signal_processors/ssb/sss_processor_impl.h"
#include "srsran/adt/tensor.h"
#include "srsran/phy/constants.h"
#include "srsran/ran/cyclic_prefix.h"
#include "srsran/ran/ssb/ssb_mapping.h"
#include "ref_ssb_pdu.h"
#include <atomic>
#include <cstring>
#include <memory>

using namespace srsran;

namespace {

using grid_tensor = dynamic_tensor<static_cast<unsigned>(resource_grid_dimensions::all), cbf16_t, resource_grid_dimensions>;

std::unique_ptr<ssb_processor> make_processor()
{
  ssb_processor_config cfg;
  cfg.encoder = std::make_unique<pbch_encoder_impl>(
      std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24C),
      std::make_unique<pseudo_random_generator_impl>(), std::make_unique<polar_interleaver_impl>(),
      std::make_unique<polar_allocator_impl>(), std::make_unique<polar_code_impl>(),
      std::make_unique<polar_encoder_impl>(), std::make_unique<polar_rate_matcher_impl>());
  cfg.modulator = std::make_unique<pbch_modulator_impl>(std::make_unique<modulation_mapper_lut_impl>(),
                                                        std::make_unique<pseudo_random_generator_impl>());
  cfg.dmrs      = std::make_unique<dmrs_pbch_processor_impl>(std::make_unique<pseudo_random_generator_impl>());
  cfg.pss       = std::make_unique<pss_processor_impl>();
  cfg.sss       = std::make_unique<sss_processor_impl>();
  return std::make_unique<ssb_processor_impl>(std::move(cfg));
}

} // namespace

extern "C" {

// ssb_processor_impl::process (ssb_processor_impl.cpp:29-109) of nof_pdus PDUs in order onto one grid
// [nof_grid_ports][14][nsubc] (modified in place).
int srs_ref_ssb_process(uint16_t* grid, unsigned nof_grid_ports, unsigned nsubc, const srs_amd_ssb_pdu* pdus,
                        unsigned nof_pdus)
{
  std::unique_ptr<ssb_processor> proc = make_processor();
  grid_tensor                    data({nsubc, MAX_NSYMB_PER_SLOT, nof_grid_ports});
  auto*                          flat = reinterpret_cast<cbf16_t*>(grid);
  for (unsigned p = 0; p != nof_grid_ports; ++p) {
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
      std::memcpy(row.data(), flat + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * sizeof(cbf16_t));
    }
  }
  std::atomic<unsigned>     empty{0};
  resource_grid_writer_impl writer(data, empty);
  for (unsigned i = 0; i != nof_pdus; ++i) {
    proc->process(writer, srs_ref::ssb_pdu_from_amd(pdus[i]));
  }
  for (unsigned p = 0; p != nof_grid_ports; ++p) {
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      span<const cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
      std::memcpy(flat + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, row.data(), nsubc * sizeof(cbf16_t));
    }
  }
  return 0;
}

// ssb_get_l_first / ssb_get_k_first of a valid PDU (the block's symbol in its slot and first subcarrier).
void srs_ref_ssb_position(const srs_amd_ssb_pdu* p, unsigned* l0, unsigned* k0)
{
  ssb_processor::pdu_t pdu = srs_ref::ssb_pdu_from_amd(*p);
  *l0 = ssb_get_l_first(pdu.pattern_case, pdu.ssb_idx) % MAX_NSYMB_PER_SLOT;
  *k0 = ssb_get_k_first(to_frequency_range(pdu.pattern_case), to_subcarrier_spacing(pdu.pattern_case),
                        pdu.common_scs, pdu.offset_to_pointA, pdu.subcarrier_offset);
}

} // extern "C"
