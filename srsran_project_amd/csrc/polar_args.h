// polar_args.h -- argument block of the polar kernels (polar.hip), shared with
// their C-ABI (polar_api.cpp).  Tables are device copies of polar_code_desc.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "polar_code.h"

struct srs_amd_polar_code;

namespace srs_amd {

struct polar_args {
  // codewords
  const uint8_t*  msgs;   // encode input / decode output: [nof][msg_stride], one bit per byte
  uint8_t*        cws;    // encode output: [nof][cw_stride], one bit per byte
  const int8_t*   llrs;   // decode input: [nof][llr_stride]
  uint8_t*        msgs_out;
  uint32_t        msg_stride, cw_stride, llr_stride, nof;
  // code
  uint32_t        K, E, N, nPC, mode, prog_len;
  uint32_t        pc_set[4];
  const uint8_t*  kset;    // [N]
  const uint16_t* msg_pos; // [K]
  const uint16_t* tx_map;  // [E]
  const uint16_t* rx_e2f;  // [E]
  const uint16_t* blk;     // [N]
  const uint32_t* program; // [prog_len]
  // slot form (launch_polar_decode_items): decoded only when *pred == pred_val (pred null: always)
  const int32_t*  pred     = nullptr;
  int32_t         pred_val = 0;
};

hipError_t launch_polar_encode(const polar_args& a, hipStream_t stream);
hipError_t launch_polar_decode(const polar_args& a, hipStream_t stream);
// The code's argument block (tables, sizes) to which a launch adds its buffers.
const polar_args& polar_code_base(const ::srs_amd_polar_code* code);
// Slot form: one argument block per codeword (device array, nof = 1 each), each with its own code.
hipError_t launch_polar_decode_items(const polar_args* items, uint32_t n, hipStream_t stream);

} // namespace srs_amd
