// bf16_device.h -- complex float -> complex bf16 (cbf16: real part in the low half) on gfx950.
//
// The reference rounds to bf16 half-to-even on the 16 discarded bits (srsran/adt/bf16.h to_bf16); gfx950's
// v_cvt_pk_bf16_f32 is the same round-to-nearest-even conversion for every non-NaN value, two floats per
// instruction (the bit-pattern formulation costs five to six VALU instructions per complex value).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

typedef float  bf16_f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16_b2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cbf16_pack(float re, float im)
{
  const bf16_f2v f = {re, im};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16_b2v));
}

} // namespace srs_amd
