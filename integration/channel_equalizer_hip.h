// channel_equalizer_hip.h -- srsran::channel_equalizer (include/srsran/phy/upper/equalization/channel_equalizer.h:
// 62-89) and srsran::channel_equalizer_factory (equalization_factories.h:35-44) over the srsran_amd C-ABI
// (include/srsran_amd/equalizer.h, srs_amd_channel_equalize): the "hip" branch a maintainer adds next to
// create_channel_equalizer_generic_factory, so the reference's pusch_demodulator_impl equalizes on the MI355X.
// is_supported() answers for the topologies of include/srsran_amd/equalizer.h: the reference's own (ZF 1 x {1, 2,
// 4}, ZF 2 x {2, 4}, MMSE 1 layer) and the L-layer solves the open reference asserts for.  Host buffers, one
// equalize() per call (the fused device path is srs_amd_pusch_demodulate_batch).  Compiled against the reference's
// headers by integration/Makefile.
#pragma once

#include "srsran/phy/upper/equalization/channel_equalizer.h"
#include "srsran/phy/upper/equalization/equalization_factories.h"
#include <memory>

namespace srsran {
namespace hip {

std::shared_ptr<channel_equalizer_factory> create_channel_equalizer_factory_hip(channel_equalizer_algorithm_type type,
                                                                                int device = -1);

} // namespace hip
} // namespace srsran
