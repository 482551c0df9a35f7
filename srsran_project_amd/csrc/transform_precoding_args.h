// transform_precoding_args.h -- argument block of the transform deprecoder kernel (transform_precoding.hip),
// shared with its C-ABI (transform_precoding_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

struct tp_args {
  float2*  symbols;    // rows of M complex values
  uint64_t sym_stride; // complex values between rows
  float*   noise;      // optional noise-variance rows
  uint64_t nv_stride;
  uint32_t M, M1, M2;  // M = M1 M2
  uint32_t nof_rows;
  float    scale;      // 1 / sqrt(M)
};

hipError_t launch_transform_deprecode(const tp_args& a, hipStream_t stream);
// Slot form: one argument block per PDU (device array); lds_bytes: the largest (2 M + M1 + M2) x 8 of the items.
hipError_t launch_transform_deprecode_items(const tp_args* items, uint32_t n, uint32_t max_rows, size_t lds_bytes,
                                            hipStream_t stream);
// The argument block of rows of nof_subc symbols (srs_amd_transform_deprecode_batch's); lds: its LDS bytes.
int make_tp_args(float2* symbols, uint64_t sym_stride, float* noise, uint64_t nv_stride, uint32_t nof_subc,
                 uint32_t nof_rows, tp_args& out, size_t& lds);

} // namespace srs_amd
