// crc_args.h -- argument block of the CRC kernel (crc.hip), shared with its
// C-ABI (crc_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

struct crc_args {
  uint8_t*        bits;      // rows of stride bytes, packed MSB-first
  uint32_t*       checksums; // per row (may be null when attaching)
  uint32_t*       acc;       // per-row accumulator for rows longer than one chunk (may be null)
  const uint32_t* table;     // x^(k+L) mod g, k < nof_bits + L
  uint32_t        stride;
  uint32_t        nof_bits;
  uint32_t        polynom;   // including the x^L term
  uint32_t        order;     // L
  int32_t         attach;
};

hipError_t launch_crc(const crc_args& a, uint32_t nof_rows, hipStream_t stream);

// True when a row of nof_bits is split over several workgroups (launch_crc then needs acc).
bool crc_needs_accumulator(uint32_t nof_bits);

} // namespace srs_amd
