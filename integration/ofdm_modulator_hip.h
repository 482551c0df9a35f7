// ofdm_modulator_hip.h -- srsran::ofdm_modulator_factory / ofdm_demodulator_factory
// (include/srsran/phy/lower/modulation/modulation_factories.h:34-72) over the srsran_amd OFDM C-ABI
// (include/srsran_amd/ofdm.h): the "hip" branch next to create_ofdm_modulator_factory_generic.
//
//   ofdm_slot_modulator::modulate(output, grid, port, slot)     (ofdm_modulator.h:89-110): the whole slot of one
//       port in one launch (srs_amd_ofdm_modulate_slot: one workgroup per OFDM symbol, DFT + CP + phase
//       compensation + scaling fused), where the reference's ofdm_slot_modulator_impl runs its symbol modulator
//       (and a dft_processor) symbol by symbol;
//   ofdm_symbol_modulator::modulate(output, grid, port, symbol) (ofdm_modulator.h:47-76): one symbol per launch
//       (srs_amd_ofdm_modulate_symbol), set_center_frequency taking effect on the next call;
//   the demodulator twins (ofdm_demodulator.h:44-100): srs_amd_ofdm_demodulate_slot / _symbol, every subcarrier of
//       the demodulated symbols stored through resource_grid_writer::get_view (the reference's symbol demodulator
//       writes the whole symbol with resource_grid_writer::put).
// Grid rows are read with resource_grid_reader::get_view into pinned staging (an empty port gives zeros, as
// ofdm_symbol_modulator_impl::modulate); every call is synchronous, as the interface is.  Errors are logged and give
// zeros; nothing aborts.  create_* returns nullptr for a configuration the MI355X kernels do not take (DFT sizes of
// include/srsran_amd/ofdm.h).  Compiled against the reference's headers by integration/Makefile.
#pragma once

#include "srsran/phy/lower/modulation/modulation_factories.h"
#include <memory>

namespace srsran {
namespace hip {

std::shared_ptr<ofdm_modulator_factory>   create_ofdm_modulator_factory_hip(int device = -1);
std::shared_ptr<ofdm_demodulator_factory> create_ofdm_demodulator_factory_hip(int device = -1);

} // namespace hip
} // namespace srsran
