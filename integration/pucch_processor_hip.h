// pucch_processor_hip.h -- srsran::pucch_processor (include/srsran/phy/upper/channel_processors/pucch/
// pucch_processor.h:396-432) and srsran::pucch_processor_factory (pucch/factories.h:64-70) over the srsran_amd PUCCH
// C-ABI (include/srsran_amd/pucch.h): Format 0 detection, Format 1 batches of multiplexed PUCCHs, Format 2
// estimation / equalization / demodulation / UCI decoding, Formats 3 / 4 (below) on the GPU.
//
// The reference's uplink processor calls process() once per PUCCH (or Format 1 batch) with the slot's
// resource_grid_reader and takes the result synchronously (uplink_processor_impl.cpp:199-229 posts every PUCCH of the
// slot's end symbol to the PUCCH executor at once, one task per PDU):
//  - a hip_resource_grid reader (hip_resource_grid.h): the call joins the factory's rendezvous -- the calls of all
//    processors waiting together share one slot-form launch per format, one result download and one
//    synchronisation, the first of them leading the batch (r06) -- and the kernels read the grids in place;
//  - any other reader: the PDU's OFDM symbols of the ports it reads are copied into a device scratch grid first, one
//    launch per call.
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
  /// Device-resident grids: how long the first caller of a rendezvous batch waits for more calls before launching
  /// (0: no wait -- calls that arrive while a batch is on the GPU form the next one).
  unsigned rendezvous_window_us = 0;
};

class pucch_processor_factory_hip : public pucch_processor_factory
{
public:
  struct statistics {
    uint64_t nof_pdus = 0, nof_errors = 0;
    /// PDUs read in place from a device-resident grid (hip_resource_grid).
    uint64_t nof_device_grids = 0;
    /// Rendezvous batches (one slot-form launch per format each) the device-grid calls went in, and the leaders' time
    /// in them: grid reads + descriptor builds + launches (host), then the wait for the results.
    uint64_t nof_batches = 0, batch_host_us = 0, batch_wait_us = 0;
  };
  virtual statistics get_statistics() const = 0;
};

/// nullptr when the device or the MI355X PUCCH processor cannot be created (logged).
std::shared_ptr<pucch_processor_factory_hip> create_pucch_processor_factory_hip(const pucch_processor_hip_config& cfg);

} // namespace hip
} // namespace srsran
