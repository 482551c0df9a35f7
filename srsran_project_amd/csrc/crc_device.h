// crc_device.h -- linear CRC of rows of packed bits (device code shared by
// crc.hip and sch.hip).
//
// The CRC is linear, so a row is split into contiguous byte chunks, one per
// thread (and, for long rows, several workgroups per row): a thread divides
// its chunk, R_t = chunk_t(x) mod g, byte by byte with a 256-entry table in
// LDS (T[t] = t(x) x^L mod g; bitwise for the partial last byte and for
// L < 8, the shift register of crc_calculator_generic_impl.cpp:98-127), moves
// it to the row's end with table[k] = x^(k+L) mod g (R_t(x) x^(n - e_t + L)
// mod g = XOR of table[j + n - e_t] over the set bits j of R_t) and the
// contributions are XOR-reduced (wave shuffles, LDS, atomics across
// workgroups).
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

// T[t] = t(x) x^L mod g for t < 256 (L >= 8). All threads of the block call it.
template <int THREADS>
__device__ __forceinline__ void crc_table8_init(uint32_t* T, uint32_t order, uint32_t polynom)
{
  if (order < 8) {
    return;
  }
  const uint32_t highbit = 1u << order;
  for (uint32_t t = threadIdx.x; t < 256; t += THREADS) {
    uint32_t r = t << (order - 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      r <<= 1;
      if (r & highbit) {
        r ^= polynom;
      }
    }
    T[t] = r;
  }
}

// This thread's contribution to the CRC of the n-bit message (byte j = fetch(j), MSB first) from
// its bytes [b0, b1).
template <typename Fetch>
__device__ __forceinline__ uint32_t crc_chunk_contrib(const Fetch&    fetch,
                                                      uint32_t        b0,
                                                      uint32_t        b1,
                                                      uint32_t        n,
                                                      uint32_t        order,
                                                      uint32_t        polynom,
                                                      const uint32_t* table,
                                                      const uint32_t* T)
{
  if (b0 >= b1) {
    return 0;
  }
  const uint32_t highbit = 1u << order;
  const uint32_t mask    = highbit - 1u;
  const uint32_t full    = min(b1, n / 8); // whole bytes
  uint32_t       r       = 0;
  uint32_t       b       = b0;
  if (order >= 8) {
    for (; b < full; ++b) {
      r = T[r >> (order - 8)] ^ ((r << 8) & mask) ^ fetch(b);
    }
  }
  for (; b < b1; ++b) {
    const uint32_t byte = fetch(b);
    const int      nb   = (b * 8 + 8 <= n) ? 8 : static_cast<int>(n - b * 8);
    for (int i = 0; i < nb; ++i) {
      r = (r << 1) | ((byte >> (7 - i)) & 1u);
      if (r & highbit) {
        r ^= polynom;
      }
    }
  }
  const uint32_t e       = min(n, b1 * 8);
  uint32_t       contrib = 0;
  for (uint32_t j = 0; j < order; ++j) {
    if ((r >> j) & 1u) {
      contrib ^= table[j + n - e];
    }
  }
  return contrib;
}

// XOR of v over the block (result to all threads). `partial`: __shared__, THREADS / 64 words.
template <int THREADS>
__device__ __forceinline__ uint32_t crc_block_xor(uint32_t v, uint32_t* partial)
{
  v = crc_wave_xor(v);
  __syncthreads(); // `partial` may still be read by a previous call
  if ((threadIdx.x & 63) == 0) {
    partial[threadIdx.x >> 6] = v;
  }
  __syncthreads();
  uint32_t crc = 0;
#pragma unroll
  for (int w = 0; w < THREADS / 64; ++w) {
    crc ^= partial[w];
  }
  return crc;
}

// Every thread of the block must call it; returns the CRC of the whole n-bit message to all
// threads. T: the crc_table8_init table (LDS). `partial` is __shared__ storage of THREADS / 64 words.
template <int THREADS, typename Fetch>
__device__ uint32_t block_crc_bytes(const Fetch&    fetch,
                                    uint32_t        n,
                                    uint32_t        order,
                                    uint32_t        polynom,
                                    const uint32_t* table,
                                    const uint32_t* T,
                                    uint32_t*       partial)
{
  const uint32_t nbytes = (n + 7) / 8;
  const uint32_t per    = (nbytes + THREADS - 1) / THREADS;
  const uint32_t b0     = threadIdx.x * per;
  const uint32_t b1     = min(nbytes, b0 + per);
  return crc_block_xor<THREADS>(crc_chunk_contrib(fetch, b0, b1, n, order, polynom, table, T), partial);
}

struct row_fetch {
  const uint8_t* row;
  __device__ uint32_t operator()(uint32_t j) const { return row[j]; }
};

} // namespace srs_amd
