// pdcch_processor_hip.h -- srsran::pdcch_processor (include/srsran/phy/upper/channel_processors/pdcch/
// pdcch_processor.h:129) and srsran::pdcch_processor_factory (pdcch/factories.h:60-67) over the srsran_amd PDCCH
// C-ABI (include/srsran_amd/pdcch.h): the DCI's CRC, interleaving, polar coding, scrambling, QPSK, precoding,
// mapping and DM-RS on the GPU, bit-exact with pdcch_processor_impl.
//
// The reference's downlink processor calls pdcch_processor::process once per DCI with the slot's
// resource_grid_writer (downlink_processor_multi_executor_impl.cpp process_pdcch); the grid must hold the DCI when
// process returns.
//  - A hip_resource_grid writer (hip_resource_grid.h): the launches go onto the processor's stream against the
//    grid's device copy and process returns without waiting; the grid's ready event orders every later reader (the
//    OFDM modulator plug-in on the device, or a host access, which downloads the grid once).
//  - Any other writer: the DCI's REs are computed on the GPU into a scratch grid, the CORESET symbols' rows come
//    back in one copy, and exactly the REs the reference writes (its CRBs' 12 subcarriers on the CORESET symbols, on
//    the precoding's ports) are stored through resource_grid_writer::get_view; process returns when they are.
// Not supported (logged, the grid left untouched): extended cyclic prefix, precoding that differs between PRGs, more
// than four ports.  Compiled against the reference's headers by integration/Makefile.
#pragma once

#include "srsran/phy/upper/channel_processors/pdcch/factories.h"
#include "srsran/phy/upper/channel_processors/pdcch/pdcch_processor.h"
#include <cstdint>
#include <memory>

namespace srsran {
namespace hip {

struct pdcch_processor_hip_config {
  /// HIP device (-1: the current one).
  int device = -1;
};

class pdcch_processor_factory_hip : public pdcch_processor_factory
{
public:
  struct statistics {
    uint64_t nof_pdus = 0, nof_errors = 0;
    /// PDUs written in place into a device-resident grid (hip_resource_grid).
    uint64_t nof_device_grids = 0;
  };
  virtual statistics get_statistics() const = 0;
};

/// nullptr when the device or the MI355X PDCCH processor cannot be created (logged).
std::shared_ptr<pdcch_processor_factory_hip> create_pdcch_processor_factory_hip(const pdcch_processor_hip_config& cfg);

} // namespace hip
} // namespace srsran
