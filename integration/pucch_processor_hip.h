// pucch_processor_hip.h -- srsran::pucch_processor (include/srsran/phy/upper/channel_processors/pucch/
// pucch_processor.h:396-432) and srsran::pucch_processor_factory (pucch/factories.h:64-70) over the srsran_amd PUCCH
// C-ABI (include/srsran_amd/pucch.h): Format 0 detection, Format 1 batches of multiplexed PUCCHs, Format 2
// estimation / equalization / demodulation / UCI decoding, Formats 3 / 4 (below) on the GPU.
//
// The reference's uplink processor calls process() once per PUCCH (or Format 1 batch) with the slot's
// resource_grid_reader and takes the result synchronously:
//  - a hip_resource_grid reader (hip_resource_grid.h): the kernels read the grid's device copy in place;
//  - any other reader: the PDU's OFDM symbols of the ports it reads are copied into a device scratch grid first.
// Formats 3 and 4 (DFT-s-OFDM PUCCH): low-PAPR DM-RS estimation, ZF, transform deprecoding, Format 4 despreading,
// QPSK / pi/2-BPSK demapping and UCI decoding on the GPU.  Compiled against the reference's headers by
// integration/Makefile.
#pragma once

#include "srsran/phy/upper/channel_processors/pucch/factories.h"
#include "srsran/phy/upper/channel_processors/pucch/pucch_processor.h"
#include <cstdint>
#include <memory>

namespace srsran {
namespace hip {

struct pucch_processor_hip_config {
  /// HIP device (-1: the current one).
  int device = -1;
  /// Channel-estimate dimensions of the reference's PUCCH processor (pucch_pdu_validator_impl checks against them).
  unsigned max_nof_prb   = 275;
  unsigned max_nof_ports = 4;
};

class pucch_processor_factory_hip : public pucch_processor_factory
{
public:
  struct statistics {
    uint64_t nof_pdus = 0, nof_errors = 0;
    /// PDUs read in place from a device-resident grid (hip_resource_grid).
    uint64_t nof_device_grids = 0;
  };
  virtual statistics get_statistics() const = 0;
};

/// nullptr when the device or the MI355X PUCCH processor cannot be created (logged).
std::shared_ptr<pucch_processor_factory_hip> create_pucch_processor_factory_hip(const pucch_processor_hip_config& cfg);

} // namespace hip
} // namespace srsran
