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

} // namespace srs_amd
