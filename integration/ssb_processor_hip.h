// ssb_processor_hip.h -- srsran::ssb_processor (include/srsran/phy/upper/channel_processors/ssb/ssb_processor.h:77)
// and srsran::ssb_processor_factory (ssb/factories.h:59-66) over the srsran_amd SS/PBCH block C-ABI
// (include/srsran_amd/ssb.h): PBCH encoding, scrambling, QPSK, DM-RS, PSS and SSS on the GPU, bit-exact with
// ssb_processor_impl.
//
// The reference's downlink processor calls ssb_processor::process once per block with the slot's
// resource_grid_writer; the grid must hold the block when process returns.
//  - A hip_resource_grid writer (hip_resource_grid.h): the launches go onto the processor's stream against the
//    grid's device copy and process returns without waiting; the grid's ready event orders every later reader.
//  - Any other writer: the block is computed on the GPU into a scratch grid, its four OFDM symbols come back in one
//    copy, and exactly the REs the reference writes (PSS, SSS, PBCH and its DM-RS on the PDU's ports) are stored
//    through resource_grid_writer::get_view; process returns when they are.
// A PDU the reference would assert on (slot without the block, offsets that give no integer subcarrier, SSB index
// beyond the pattern) is logged and not written.  Compiled against the reference's headers by integration/Makefile.
#pragma once

#include "srsran/phy/upper/channel_processors/ssb/factories.h"
#include "srsran/phy/upper/channel_processors/ssb/ssb_processor.h"
#include <cstdint>
#include <memory>

namespace srsran {
namespace hip {

struct ssb_processor_hip_config {
  /// HIP device (-1: the current one).
  int device = -1;
};

class ssb_processor_factory_hip : public ssb_processor_factory
{
public:
  struct statistics {
    uint64_t nof_pdus = 0, nof_errors = 0;
    /// PDUs written in place into a device-resident grid (hip_resource_grid).
    uint64_t nof_device_grids = 0;
  };
  virtual statistics get_statistics() const = 0;
};

/// nullptr when the device or the MI355X SSB processor cannot be created (logged).
std::shared_ptr<ssb_processor_factory_hip> create_ssb_processor_factory_hip(const ssb_processor_hip_config& cfg);

} // namespace hip
} // namespace srsran
