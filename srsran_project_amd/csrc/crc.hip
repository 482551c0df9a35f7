// crc.hip -- CRC calculation / attachment over rows of packed bits (MI355X).
//
// The reference computes crc_calculator::calculate (crc_calculator.h:81) by
// bitwise or byte-table long division of the whole message, one bit after the
// other (crc_calculator_generic_impl.cpp:98-127).  The CRC is linear
// (crc_device.h): every thread divides a contiguous chunk of the row with a
// byte table in LDS and moves its remainder to the row's end.
//   rows <= 8 KiB   crc_kernel: one workgroup per row.
//   longer rows     crc_chunk_kernel: one workgroup per 8 KiB of a row, partial
//                   CRCs XOR-ed into a per-row accumulator (atomicXor), then
//                   crc_finalize_kernel writes / attaches the checksums; a 1 Mbit
//                   transport block spreads over ~17 workgroups instead of one.
#include <hip/hip_runtime.h>

#include "crc_args.h"
#include "crc_device.h"

namespace srs_amd {

namespace {

constexpr int      CRC_THREADS = 256;
constexpr uint32_t CRC_PER     = 32;                      // bytes per thread
constexpr uint32_t CRC_CHUNK   = CRC_THREADS * CRC_PER;   // bytes per workgroup

__device__ void write_crc(const crc_args& a, uint32_t row_index, uint32_t crc)
{
  if (a.checksums != nullptr) {
    a.checksums[row_index] = crc;
  }
  if (a.attach) {
    // CRC bits MSB-first into bits [n, n + L); other bits of the touched bytes kept.
    // each touched byte read and written once (at most 4 bytes for a 24-bit CRC)
    uint8_t* row = a.bits + static_cast<size_t>(row_index) * a.stride;
    attach_crc_bits(row, a.nof_bits, a.order, crc);
  }
}

// One wave per row: ~17 bytes per lane for a 1056-byte codeblock, so few remainder moves per byte.
constexpr int CRC_ROW_THREADS = 64;

__global__ void __launch_bounds__(CRC_ROW_THREADS) crc_kernel(crc_args a)
{
  __shared__ uint32_t partial[1];
  __shared__ uint32_t T[256];
  crc_table8_init<CRC_ROW_THREADS>(T, a.order, a.polynom);
  __syncthreads();
  const uint8_t* row = a.bits + static_cast<size_t>(blockIdx.x) * a.stride;
  const uint32_t crc = block_crc_bytes<CRC_ROW_THREADS>(row_fetch{row}, a.nof_bits, a.order, a.polynom, a.table, T,
                                                        partial);
  if (threadIdx.x == 0) {
    write_crc(a, blockIdx.x, crc);
  }
}

__global__ void __launch_bounds__(CRC_THREADS) crc_chunk_kernel(crc_args a)
{
  __shared__ uint32_t partial[CRC_THREADS / 64];
  __shared__ uint32_t T[256];
  __shared__ __attribute__((aligned(16))) uint8_t s_chunk[CRC_CHUNK];
  crc_table8_init<CRC_THREADS>(T, a.order, a.polynom);
  const uint8_t* row    = a.bits + static_cast<size_t>(blockIdx.y) * a.stride;
  const uint32_t nbytes = (a.nof_bits + 7) / 8;
  const uint32_t c0     = blockIdx.x * CRC_CHUNK;
  // the chunk staged in LDS with coalesced loads (each thread then divides 32 contiguous bytes)
  crc_stage_bytes<CRC_THREADS>(s_chunk, row, c0, min(CRC_CHUNK, nbytes - c0));
  __syncthreads();
  const uint32_t b0     = c0 + threadIdx.x * CRC_PER;
  const uint32_t b1     = min(nbytes, b0 + CRC_PER);
  // contributions summed at the end of the workgroup's chunk, then moved to the message end once
  const uint32_t to     = min(a.nof_bits, (blockIdx.x + 1) * CRC_CHUNK * 8);
  const uint32_t v      = crc_block_xor<CRC_THREADS>(
      crc_chunk_contrib(lds_chunk_fetch{s_chunk, c0}, b0, b1, a.nof_bits, a.order, a.polynom, a.table, T, to),
      partial);
  if (threadIdx.x == 0 && v != 0) {
    atomicXor(a.acc + blockIdx.y, crc_move(v, a.nof_bits - to, a.order, a.table));
  }
}

__global__ void __launch_bounds__(64) crc_finalize_kernel(crc_args a, uint32_t nof_rows)
{
  const uint32_t r = blockIdx.x * 64 + threadIdx.x;
  if (r < nof_rows) {
    write_crc(a, r, a.acc[r]);
  }
}

} // namespace

bool crc_needs_accumulator(uint32_t nof_bits)
{
  return (nof_bits + 7) / 8 > CRC_CHUNK;
}

hipError_t launch_crc(const crc_args& a, uint32_t nof_rows, hipStream_t stream)
{
  if (nof_rows == 0) {
    return hipSuccess;
  }
  const uint32_t nbytes = (a.nof_bits + 7) / 8;
  if (nbytes <= CRC_CHUNK || a.acc == nullptr) {
    hipLaunchKernelGGL(crc_kernel, dim3(nof_rows), dim3(CRC_ROW_THREADS), 0, stream, a);
    return hipGetLastError();
  }
  hipError_t e = hipMemsetAsync(a.acc, 0, sizeof(uint32_t) * nof_rows, stream);
  if (e != hipSuccess) {
    return e;
  }
  hipLaunchKernelGGL(crc_chunk_kernel, dim3((nbytes + CRC_CHUNK - 1) / CRC_CHUNK, nof_rows), dim3(CRC_THREADS), 0,
                     stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) {
    return e;
  }
  hipLaunchKernelGGL(crc_finalize_kernel, dim3((nof_rows + 63) / 64), dim3(64), 0, stream, a, nof_rows);
  return hipGetLastError();
}

} // namespace srs_amd
