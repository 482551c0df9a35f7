// modulation_args.h -- argument blocks of the modulation / demodulation /
// scrambling kernels (modulation.hip), shared with their C-ABI (modulation_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gold_sequence.h"

namespace srs_amd {

// Soft-demapper piecewise-linear LLR table of one PAM axis bit.
struct demod_interval_table {
  int32_t n;      // intervals
  float   width;
  float   slope[16];
  float   icpt[16];
};

struct modulate_args {
  const uint8_t* bits;    // packed MSB-first
  float*         symbols; // interleaved re/im
  const float*   table;   // [2^Qm][2] re/im (Qm >= 2)
  uint32_t       nof_symbols;
  int32_t        qm;      // 0 pi/2-BPSK, 1 BPSK, 2, 4, 6, 8
};

struct demodulate_args {
  const float*         symbols;
  const float*         noise_vars;
  int8_t*              llrs;
  uint32_t             nof_symbols;
  uint32_t             block_end; // symbols [0, block_end) follow the reference's AVX2 kernel, the rest its scalar code
  int32_t              qm;
  float                qam16_scale; // 1/sqrt(10) as the reference computes it (host float sqrt)
  demod_interval_table tab[4];
};

struct prbs_args {
  const uint8_t* in_bits;  // scramble: packed input (may be null: generate c)
  uint8_t*       out_bits;
  const int8_t*  in_llrs;  // descramble LLRs
  int8_t*        out_llrs;
  const uint32_t* jump;    // [2][NJUMP][31] GF(2) jump matrices (columns), x1 then x2
  uint32_t       c_init;
  uint32_t       length;   // bits / LLRs
};


hipError_t launch_modulate(const modulate_args& a, hipStream_t stream);
hipError_t launch_demodulate(const demodulate_args& a, hipStream_t stream);
hipError_t launch_scramble_bits(const prbs_args& a, hipStream_t stream);
hipError_t launch_descramble_llrs(const prbs_args& a, hipStream_t stream);

} // namespace srs_amd
