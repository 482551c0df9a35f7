// crc_device.h -- block-wide CRC of one row of packed bits (device code shared
// by crc.hip and sch.hip).
//
// Linear CRC split into one contiguous byte chunk per thread: thread t divides
// its chunk (R_t = chunk_t(x) mod g, shift register as
// crc_calculator_generic_impl.cpp:98-127), moves it to the row's end with
// table[k] = x^(k+L) mod g (R_t(x) * x^(n - e_t + L) mod g = XOR of
// table[j + n - e_t] over the set bits j of R_t) and the block XOR-reduces.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

__device__ __forceinline__ uint32_t crc_wave_xor(uint32_t v)
{
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    v ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), o, 64));
  }
  return v;
}

// Every thread of the block must call it; returns the CRC of the n-bit
// message whose byte j is fetch(j) (MSB first) to all threads.
// `partial` is __shared__ storage of THREADS / 64 words.
template <int THREADS, typename Fetch>
__device__ uint32_t block_crc_bytes(const Fetch&    fetch,
                                    uint32_t        n,
                                    uint32_t        order,
                                    uint32_t        polynom,
                                    const uint32_t* table,
                                    uint32_t*       partial)
{
  const uint32_t highbit = 1u << order;
  const uint32_t nbytes  = (n + 7) / 8;
  const uint32_t per     = (nbytes + THREADS - 1) / THREADS;
  const uint32_t b0      = threadIdx.x * per;
  const uint32_t b1      = min(nbytes, b0 + per);
  uint32_t       contrib = 0;
  if (b0 < b1) {
    uint32_t r = 0;
    for (uint32_t b = b0; b < b1; ++b) {
      const uint32_t byte = fetch(b);
      const int      nb   = (b * 8 + 8 <= n) ? 8 : static_cast<int>(n - b * 8);
      for (int i = 0; i < nb; ++i) {
        r = (r << 1) | ((byte >> (7 - i)) & 1u);
        if (r & highbit) {
          r ^= polynom;
        }
      }
    }
    const uint32_t e = min(n, b1 * 8);
    for (uint32_t j = 0; j < order; ++j) {
      if ((r >> j) & 1u) {
        contrib ^= table[j + n - e];
      }
    }
  }
  contrib = crc_wave_xor(contrib);
  __syncthreads(); // `partial` may still be read by a previous call
  if ((threadIdx.x & 63) == 0) {
    partial[threadIdx.x >> 6] = contrib;
  }
  __syncthreads();
  uint32_t crc = 0;
#pragma unroll
  for (int w = 0; w < THREADS / 64; ++w) {
    crc ^= partial[w];
  }
  return crc;
}

struct row_fetch {
  const uint8_t* row;
  __device__ uint32_t operator()(uint32_t j) const { return row[j]; }
};

template <int THREADS>
__device__ uint32_t block_row_crc(const uint8_t*  row,
                                  uint32_t        n,
                                  uint32_t        order,
                                  uint32_t        polynom,
                                  const uint32_t* table,
                                  uint32_t*       partial)
{
  return block_crc_bytes<THREADS>(row_fetch{row}, n, order, polynom, table, partial);
}

} // namespace srs_amd
