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
// On a reference grid, rows are read with resource_grid_reader::get_view into pinned staging (an empty port gives
// zeros, as ofdm_symbol_modulator_impl::modulate) and written back through resource_grid_writer::get_view; every call
// is synchronous.
//
// On a device-resident grid (hip_resource_grid.h) the grid never crosses PCIe (r06):
//   demodulators: each call copies its samples into pinned staging with the symbol index and grid row, and registers
//       with the grid as a deferred writer; the staged symbols are demodulated into the device copy in ONE launch
//       (srs_amd_ofdm_demodulate_symbols_async) when the grid is next accessed -- the PUSCH plug-in's read -- or when
//       64 are staged.  A call makes no HIP call and never waits for the device (1.2-1.7 us per 4096-point symbol on
//       one host thread, profiles/r06_ofdm_symbol_plugin_rate_*.json); the kernel reads the pinned samples over the
//       bus (SRS_AMD_OFDM_STAGING=dma / copy-kernel: DMA or a copy kernel into HBM first, measured slower).
//   modulators: the first call for a slot modulates every port of that slot in place in one launch
//       (srs_amd_ofdm_modulate_batch on the device copy, samples DMA-copied to pinned memory); the later calls of the
//       slot copy their share while the grid is unchanged (hip_resource_grid::unchanged_since): the lower PHY calls
//       per port and symbol on a finished grid.  The samples leave the device because the interface returns them.
// Errors are logged and give zeros; nothing aborts.  create_* returns nullptr for a configuration the MI355X kernels
// do not take (DFT sizes of include/srsran_amd/ofdm.h).  Compiled against the reference's headers by
// integration/Makefile, into libsrsran_amd_phy.so with hip_resource_grid.
#pragma once

#include "srsran/phy/lower/modulation/modulation_factories.h"
#include <memory>

namespace srsran {
namespace hip {

std::shared_ptr<ofdm_modulator_factory>   create_ofdm_modulator_factory_hip(int device = -1);
std::shared_ptr<ofdm_demodulator_factory> create_ofdm_demodulator_factory_hip(int device = -1);

} // namespace hip
} // namespace srsran
