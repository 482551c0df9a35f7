// pdcch.hip -- MI355X PDCCH kernels (include/srsran_amd/pdcch.h).
//
// pdcch_crc_kernel: one thread per DCI: c' = 24 ones | payload, its CRC24C (crc_calculator::calculate_bit, MSB
// first), the last 16 parity bits XOR-ed with the RNTI (pdcch_encoder_impl.cpp:33-58), then the DCI input bit
// interleaver (polar_interleaver, tx direction) into the polar encoder's message row.
//
// pdcch_map_kernel: one thread per (DCI, CORESET symbol, RE of its RBs): data REs (k mod 4 != 1) get the QPSK symbol
// of codeword bits 2 j, 2 j + 1 (j = the RE's index in the mapper's symbol / CRB / RE order), scrambled with the Gold
// sequence of c_init_data (pdcch_modulator_impl.cpp:32-58), scaled (when the amplitude is a normal number) and
// precoded onto every port; DM-RS REs (k = 4 n + 1) the sequence of dmrs_sequence_generate (dmrs_helper.cpp:64-95,
// three per RB from the reference point) at M_SQRT1_2 x amplitude, precoded likewise (dmrs_pdcch_processor_impl.cpp).
// The arithmetic follows the PDSCH kernels (pdsch_modulator.hip): the same QPSK values, float scaling, the precoder's
// fmaddsub complex product and round-half-even cbf16 packing, so the grid is bit-exact with the reference.
#include <hip/hip_runtime.h>

#include "bf16_device.h"
#include "gold_sequence.h"
#include "pdcch_args.h"

#pragma clang fp contract(off)

namespace srs_amd {
namespace {

constexpr uint32_t CRC24C_POLY = 0x1b2b117u;
constexpr uint32_t MAP_THREADS = 256;

__global__ __launch_bounds__(64) void pdcch_crc_kernel(const pdcch_desc* desc, uint32_t nof, const uint8_t* payloads,
                                                       uint8_t* msgs)
{
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= nof) {
    return;
  }
  const pdcch_desc& d = desc[i];
  const uint8_t*    a = payloads + d.payload_offset;
  uint8_t           c[PDCCH_MAX_K];
  uint32_t          reg = 0;
  auto              feed = [&](uint32_t bit) {
    const uint32_t fb = ((reg >> 23) & 1u) ^ bit;
    reg               = (reg << 1) & 0xffffffu;
    reg ^= fb ? (CRC24C_POLY & 0xffffffu) : 0u;
  };
  for (uint32_t k = 0; k < 24; ++k) {
    feed(1u);
  }
  for (uint32_t k = 0; k < d.payload_size; ++k) {
    c[k] = a[k] & 1u;
    feed(c[k]);
  }
  for (uint32_t k = 0; k < 24; ++k) {
    uint32_t p = (reg >> (23 - k)) & 1u;
    if (k >= 8) {
      p ^= (d.rnti >> (15 - (k - 8))) & 1u; // RNTI bits MSB first over the last 16 parity bits
    }
    c[d.payload_size + k] = static_cast<uint8_t>(p);
  }
  uint8_t* m = msgs + d.msg_offset;
  for (uint32_t k = 0; k < d.K; ++k) {
    m[k] = c[d.perm[k]];
  }
}

// x * w as _mm256_fmaddsub_ps(x, w.re, swap(x) * w.im) (the reference precoder)
__device__ __forceinline__ float2 cmul_simd(float2 x, float wr, float wi)
{
  return make_float2(__builtin_fmaf(x.x, wr, -(x.y * wi)), __builtin_fmaf(x.y, wr, x.x * wi));
}

__global__ __launch_bounds__(MAP_THREADS) void pdcch_map_kernel(const pdcch_desc* desc, const uint8_t* cws,
                                                                 const uint32_t* jump)
{
  const pdcch_desc& d  = desc[blockIdx.z];
  const uint32_t    li = blockIdx.y; // CORESET symbol
  const uint32_t    e  = blockIdx.x * MAP_THREADS + threadIdx.x;
  if (li >= d.duration || e >= d.nof_rb * 12) {
    return;
  }
  const uint32_t i   = e / 12; // RB index within the DCI
  const uint32_t r   = e % 12;
  const uint32_t crb = d.crbs[i];
  const uint32_t l   = d.start_symbol + li;
  float2         x;
  if ((r & 3u) == 1u) {
    // DM-RS: sequence index m = 3 (crb - ref) + r / 4, bits 2 m and 2 m + 1 of the symbol's sequence
    const uint32_t m    = PDCCH_DMRS_PER_RB * (crb - d.ref_k_rb) + r / 4;
    const uint32_t b    = 2 * m;
    const uint32_t word = gold_word(jump, d.c_init_dmrs[li], 32 * (b / 32));
    const uint32_t bits = word >> (b % 32);
    const float    amp  = d.dmrs_amp;
    x                   = make_float2((bits & 1u) ? -amp : amp, (bits & 2u) ? -amp : amp);
  } else {
    // data: index j in the mapper's order (symbol, CRB, RE), codeword bits 2 j and 2 j + 1 scrambled
    const uint32_t j    = (li * d.nof_rb + i) * PDCCH_DATA_PER_RB + (r - (r + 3) / 4);
    const uint32_t b    = 2 * j;
    const uint32_t word = gold_word(jump, d.c_init_data, 32 * (b / 32));
    const uint8_t* cw   = cws + d.cw_offset;
    const uint32_t b0   = cw[b] ^ ((word >> (b % 32)) & 1u);
    const uint32_t b1   = cw[b + 1] ^ ((word >> ((b + 1) % 32)) & 1u);
    const float    s    = static_cast<float>(M_SQRT1_2); // modulation_mapper QPSK: (1 - 2 b) / sqrt(2)
    x                   = make_float2(b0 ? -s : s, b1 ? -s : s);
    if (d.data_scaled) {
      x = make_float2(x.x * d.data_amp, x.y * d.data_amp);
    }
  }
  uint32_t* row = d.grid + static_cast<uint64_t>(l) * d.nof_subc + 12 * crb + r;
  for (uint32_t p = 0; p < d.nof_ports; ++p) {
    const float2 v                               = cmul_simd(x, d.w[p][0], d.w[p][1]);
    row[static_cast<uint64_t>(p) * d.port_stride] = cbf16_pack(v.x, v.y);
  }
}

} // namespace

hipError_t launch_pdcch_crc(const pdcch_desc* d_desc, uint32_t nof, const uint8_t* d_payloads, uint8_t* d_msgs,
                            hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pdcch_crc_kernel, dim3((nof + 63) / 64), dim3(64), 0, stream, d_desc, nof, d_payloads, d_msgs);
  return hipGetLastError();
}

hipError_t launch_pdcch_map(const pdcch_desc* d_desc, uint32_t nof, uint32_t max_rb, uint32_t max_symbols,
                            const uint8_t* d_cws, const uint32_t* jump, hipStream_t stream)
{
  if (nof == 0 || max_rb == 0 || max_symbols == 0) {
    return hipSuccess;
  }
  const dim3 grid((max_rb * 12 + MAP_THREADS - 1) / MAP_THREADS, max_symbols, nof);
  hipLaunchKernelGGL(pdcch_map_kernel, grid, dim3(MAP_THREADS), 0, stream, d_desc, d_cws, jump);
  return hipGetLastError();
}

} // namespace srs_amd
