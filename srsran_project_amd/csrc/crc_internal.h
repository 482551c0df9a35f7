// crc_internal.h -- library-internal access to a CRC calculator's device table.
#pragma once

#include <cstdint>

#include "srsran_amd/crc.h"

namespace srs_amd {

// x^(k+L) mod g for k < max_bits + 32, resident on the calculator's device.
const uint32_t* crc_device_table(const srs_amd_crc_calculator* crc);

// Generator polynomial (including the x^L term) and its order L.
uint32_t crc_polynom(const srs_amd_crc_calculator* crc);
uint32_t crc_order(const srs_amd_crc_calculator* crc);

} // namespace srs_amd
