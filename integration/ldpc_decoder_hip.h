// ldpc_decoder_hip.h -- srsran::ldpc_decoder (include/srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h:37)
// and srsran::ldpc_decoder_factory (channel_coding_factories.h:53) over the srsran_amd C-ABI
// (include/srsran_amd/ldpc.h, srs_amd_ldpc_decode): the "hip" / "hip-generic" branches a maintainer adds to
// ldpc_decoder_factory_sw::create() (lib/phy/upper/channel_coding/channel_coding_factories.cpp:102).
// One codeblock per call (host buffers); the batched form is the PUSCH accelerator plug-in
// (hip_accelerator_pusch_dec.h).  Compiled against the reference's headers by integration/Makefile.
#pragma once

#include "srsran/phy/upper/channel_coding/channel_coding_factories.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h"
#include <memory>

namespace srsran {
namespace hip {

/// dec_type "hip" reproduces the reference's "avx2" / "avx512" / "auto" arithmetic bit-exactly, "hip-generic"
/// its "generic" decoder.
std::shared_ptr<ldpc_decoder_factory> create_ldpc_decoder_factory_hip(const std::string& dec_type,
                                                                      bool               force_decoding = false,
                                                                      int                device         = -1);

} // namespace hip
} // namespace srsran
