// uci_args.h -- argument blocks of the UCI decoder kernels (uci_decoder.hip), shared with their C-ABI
// (uci_decoder_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

struct uci_short_args {
  const int8_t* llrs;
  uint64_t      llr_stride;
  uint8_t*      msgs;
  uint64_t      msg_stride;
  int32_t*      status;
  uint64_t      status_stride; // bytes
  uint32_t      E;
  uint32_t      K;             // 1 .. 11
  uint32_t      qm;            // bits per modulation symbol
};

// Polar codeblocks already decoded (deallocated message bits, one per byte, rows of cb_stride): CRC check,
// filler removal, status.
struct uci_polar_args {
  const uint8_t* cbs;      // [message][C][cb_stride]
  uint64_t       cb_stride;
  uint8_t*       msgs;
  uint64_t       msg_stride;
  int32_t*       status;
  uint64_t       status_stride;
  uint32_t       C;        // codeblocks (1 or 2)
  uint32_t       A0, F0;   // payload bits / filler bits of codeblock 0
  uint32_t       A1;       // payload bits of codeblock 1
  uint32_t       L;        // CRC bits (6 or 11)
};

hipError_t launch_uci_short(const uci_short_args& a, uint32_t nof, hipStream_t stream);
hipError_t launch_uci_polar_finish(const uci_polar_args& a, uint32_t nof, hipStream_t stream);

} // namespace srs_amd
