// dft_processor_hip.h -- srsran::dft_processor (include/srsran/phy/generic_functions/dft_processor.h:34-72) and
// srsran::dft_processor_factory (generic_functions_factories.h:31-41) over the srsran_amd C-ABI
// (include/srsran_amd/ofdm.h, srs_amd_dft_create / srs_amd_dft_run): the "hip" branch a maintainer adds next to
// create_dft_processor_factory_generic / _fftw, so the reference's OFDM modulator / demodulator (and every other
// dft_processor user) runs its transforms on the MI355X.  One transform per run() on host buffers (the batched
// slot forms are the OFDM C-ABI, srs_amd_ofdm_modulate_batch).  Compiled against the reference's headers by
// integration/Makefile.
#pragma once

#include "srsran/phy/generic_functions/dft_processor.h"
#include "srsran/phy/generic_functions/generic_functions_factories.h"
#include <memory>

namespace srsran {
namespace hip {

/// Sizes the MI355X DFT kernels support (radix 2/3/4/8/16 Stockham stages); create() returns nullptr otherwise,
/// as the factory contract asks.
std::shared_ptr<dft_processor_factory> create_dft_processor_factory_hip(int device = -1);

} // namespace hip
} // namespace srsran
