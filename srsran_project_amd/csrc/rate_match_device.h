// rate_match_device.h -- device helpers of the LDPC rate matcher shared by ldpc_rate_matching.hip and the fused
// PDSCH codeblock kernel (pdsch_encoder.hip): division by a run-time constant, the 8 x 8 bit transpose of the
// symbol interleaver and the walk over the circular buffer (rate_matching_common.h).
#pragma once

#include <hip/hip_runtime.h>

#include "rate_matching_common.h"
#include <cstdint>

namespace srs_amd {

// q = n / d, r = n % d for n < 2^24 via a float reciprocal and one correction
// (the float estimate is off by at most one).
struct fast_div {
  uint32_t d;
  float    rcp;
  __device__ explicit fast_div(uint32_t d_) : d(d_), rcp(1.0f / static_cast<float>(d_ ? d_ : 1)) {}
  __device__ __forceinline__ uint32_t div(uint32_t n, uint32_t& r) const
  {
    uint32_t q = static_cast<uint32_t>(static_cast<float>(n) * rcp);
    int32_t  x = static_cast<int32_t>(n - q * d);
    if (x < 0) {
      q -= 1;
      x += static_cast<int32_t>(d);
    } else if (x >= static_cast<int32_t>(d)) {
      q += 1;
      x -= static_cast<int32_t>(d);
    }
    r = static_cast<uint32_t>(x);
    return q;
  }
};

// 8 x 8 bit transpose: byte j (from the most significant) = row j, bit 7 - k = column k  ->  byte k = column k,
// its bit 7 - j = row j.
__device__ __forceinline__ uint64_t transpose8x8(uint64_t x)
{
  uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x          = x ^ t ^ (t << 7);
  t          = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x          = x ^ t ^ (t << 14);
  t          = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  return x ^ t ^ (t << 28);
}

// Bits e[w], e[w + 1], .. e[w + 7] of the walk (w < L), MSB first, from the staged circular buffer: one
// two-byte read when the run neither wraps nor crosses the filler gap, else bit by bit.
__device__ __forceinline__ uint32_t rm_walk_byte(const uint8_t* s_cw, const rm_geometry& g, uint32_t w)
{
  if (w + 7 < g.L && (w + 7 < g.nof_info || w >= g.nof_info)) {
    const uint32_t p = w < g.nof_info ? w : w + g.F;
    const uint32_t v = (static_cast<uint32_t>(s_cw[p >> 3]) << 8) | s_cw[(p >> 3) + 1];
    return (v >> (8 - (p & 7))) & 0xffu;
  }
  uint32_t row = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    uint32_t ww = w + k;
    ww          = ww >= g.L ? ww - g.L : ww;
    const uint32_t p = ww < g.nof_info ? ww : ww + g.F;
    row |= ((s_cw[p >> 3] >> (7 - (p & 7))) & 1u) << (7 - k);
  }
  return row;
}

} // namespace srs_amd
