// hip_accelerator_pusch_dec.h -- the MI355X as a srsRAN hardware-accelerator plug-in for the PUSCH
// decoder: implements hal::hw_accelerator_pusch_dec
//   (include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h:83)
// and hal::hw_accelerator_pusch_dec_factory (hw_accelerator_pusch_dec_factory.h), so the reference's own
// pusch_decoder_hw_impl (lib/phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.cpp) decodes through
// the C-ABI of include/srsran_amd (rate dematching + HARQ combining + LDPC decoding with CB CRC early stop
// on the GPU).  Compiled against the reference's headers by integration/Makefile.
//
// External HARQ (is_harq_external() == true): the HARQ soft buffers live in HBM, keyed by the reference's
// absolute codeblock id; pusch_decoder_hw_impl then enqueues every codeblock of a transport block before
// dequeuing any (pusch_decoder_hw_impl.cpp:230-300), and the first dequeue runs the whole transport block
// as ONE batch: one H2D copy of the codeblocks' LLRs, srs_amd_ldpc_rate_dematch_batch into the transport
// block's contiguous HARQ rows, srs_amd_ldpc_decode_batch, one D2H copy of messages and iteration counts.
#pragma once

#include "srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h"
#include "srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec_factory.h"
#include <memory>

namespace srsran {
namespace hip {

struct pusch_dec_accelerator_config {
  int      device        = -1;   // HIP device (-1: current)
  int      arith         = 0;    // SRS_AMD_ARITH_SIMD ("avx2"/"avx512"/"auto") or SRS_AMD_ARITH_GENERIC
  unsigned max_harq_rows = 4096; // HARQ codeblock soft buffers held in HBM (66 x 384 LLRs each)
};

/// Creates the plug-in factory (the role of hal::create_bbdev_pusch_dec_acc_factory for the MI355X).
std::shared_ptr<hal::hw_accelerator_pusch_dec_factory>
create_hip_pusch_dec_acc_factory(const pusch_dec_accelerator_config& cfg = {});

} // namespace hip
} // namespace srsran
