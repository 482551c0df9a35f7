// hip_accelerator_pdsch_enc.h -- the MI355X as a srsRAN hardware-accelerator plug-in for the PDSCH encoder:
// implements hal::hw_accelerator_pdsch_enc
//   (include/srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc.h:85-104)
// and hal::hw_accelerator_pdsch_enc_factory (hw_accelerator_pdsch_enc_factory.h:31), so the reference's own
// pdsch_encoder_hw_impl (lib/phy/upper/channel_processors/pdsch/pdsch_encoder_hw_impl.cpp) encodes through the
// C-ABI of include/srsran_amd.  Compiled against the reference's headers by integration/Makefile.
//
// TB mode (default, is_cb_mode_supported() == false): pdsch_encoder_hw_impl hands over the whole transport
// block and the segmentation geometry; the enqueue runs TB CRC, segmentation, CB CRC, LDPC encoding and rate
// matching of every codeblock as ONE srs_amd_pdsch_encode call (one launch sequence on the GPU), the dequeue
// returns the codeword (one bit per byte, as the reference writes it).
// CB mode (cb_mode = true): the reference segments and attaches the CRCs on the host; every codeblock is LDPC
// encoded and rate matched on the GPU (srs_amd_ldpc_encode + srs_amd_ldpc_rate_match).
// Errors never abort: they are logged and the dequeue reports failure once the operation cannot complete.
#pragma once

#include "srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc.h"
#include "srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc_factory.h"
#include <memory>

namespace srsran {
namespace hip {

struct pdsch_enc_accelerator_config {
  int      device          = -1;      // HIP device (-1: current)
  bool     cb_mode         = false;   // true: the reference segments, the GPU encodes codeblock by codeblock
  unsigned max_buffer_size = 1u << 22; // TB mode: the largest transport block / packed codeword in bytes
};

/// Creates the plug-in factory (the role of hal::create_bbdev_pdsch_enc_acc_factory for the MI355X).
std::shared_ptr<hal::hw_accelerator_pdsch_enc_factory>
create_hip_pdsch_enc_acc_factory(const pdsch_enc_accelerator_config& cfg = {});

} // namespace hip
} // namespace srsran
