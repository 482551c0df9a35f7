// crc.hip -- CRC calculation / attachment over rows of packed bits (MI355X).
//
// The reference computes crc_calculator::calculate (crc_calculator.h:81) by
// bitwise or byte-table long division of the whole message, one bit after the
// other (crc_calculator_generic_impl.cpp:98-127).  The CRC is linear, so the
// GPU splits each row into one contiguous chunk per thread:
//   1. thread t divides its own chunk:   R_t = chunk_t(x) mod g  (shift register)
//   2. and moves it to the row's end:     R_t(x) * x^(n - e_t + L) mod g
//      = XOR over set bits j of R_t of table[j + n - e_t]   (table[k] = x^(k+L) mod g)
//   3. the block XOR-reduces the contributions (wave shuffles + LDS).
// One workgroup per row; the chunk loop reads whole bytes, so a row costs one
// pass over its ceil(n/8) bytes plus <= L table reads per thread.
#include <hip/hip_runtime.h>

#include "crc_args.h"
#include "crc_device.h"

namespace srs_amd {

namespace {

constexpr int CRC_THREADS = 256;

__global__ void __launch_bounds__(CRC_THREADS) crc_kernel(crc_args a)
{
  __shared__ uint32_t partial[CRC_THREADS / 64];
  uint8_t*            row = a.bits + static_cast<size_t>(blockIdx.x) * a.stride;
  const uint32_t      crc = block_row_crc<CRC_THREADS>(row, a.nof_bits, a.order, a.polynom, a.table, partial);
  if (threadIdx.x != 0) {
    return;
  }
  if (a.checksums != nullptr) {
    a.checksums[blockIdx.x] = crc;
  }
  if (a.attach) {
    // CRC bits MSB-first into bits [n, n + L); other bits of the touched bytes kept.
    for (uint32_t k = 0; k < a.order; ++k) {
      const uint32_t pos  = a.nof_bits + k;
      const uint32_t bit  = (crc >> (a.order - 1 - k)) & 1u;
      const uint8_t  mask = static_cast<uint8_t>(0x80u >> (pos & 7));
      row[pos >> 3]       = static_cast<uint8_t>((row[pos >> 3] & ~mask) | (bit ? mask : 0));
    }
  }
}

} // namespace

hipError_t launch_crc(const crc_args& a, uint32_t nof_rows, hipStream_t stream)
{
  hipLaunchKernelGGL(crc_kernel, dim3(nof_rows), dim3(CRC_THREADS), 0, stream, a);
  return hipGetLastError();
}

} // namespace srs_amd
