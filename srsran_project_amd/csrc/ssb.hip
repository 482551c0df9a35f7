// ssb.hip -- MI355X SS/PBCH block kernels (include/srsran_amd/ssb.h).
//
// ssb_encode_kernel: one thread per block: the PBCH payload a (pbch_encoder_impl.cpp:37-74: MIB bits through the
// interleaver pattern G of TS 38.212 Table 7.1.1-1, the 4 LSBs of the SFN, the half-frame bit and the SSB index or
// k_SSB bits), the first scrambling (:76-110: Gold sequence of N_ID from M v, no sequence bit consumed by the SSB
// index / half-frame / SFN 2nd and 3rd LSB positions), CRC24C (:112-126) and the input bit interleaver, into the
// polar encoder's message row (K = 56).
//
// ssb_map_kernel: one thread per (block, OFDM symbol of the block, subcarrier of its 240): symbol 0 the PSS
// (pss_processor_impl.cpp, subcarriers 56..182), symbol 2 the SSS (sss_processor_impl.cpp) between the PBCH edges,
// and the PBCH (pbch_modulator_impl.cpp: second scrambling from (ssb_idx mod 8) x 864, QPSK, symbols 1 and 3 and the
// edges of symbol 2 without the DM-RS subcarriers v + 4 i) and its DM-RS (dmrs_pbch_processor_impl.cpp: Gold sequence
// of c_init, QPSK at M_SQRT1_2) on every port; each value rounded to cbf16 half to even as the reference's grid
// writer.
#include <hip/hip_runtime.h>

#include "bf16_device.h"
#include "gold_sequence.h"
#include "ssb_args.h"

#pragma clang fp contract(off)

namespace srs_amd {
namespace {

constexpr uint32_t CRC24C_POLY = 0x1b2b117u;

// TS 38.212 Table 7.1.1-1: PBCH payload interleaver pattern G(j).
__constant__ uint8_t PBCH_G[SSB_A] = {16, 23, 18, 17, 8,  30, 10, 6,  24, 7,  0,  5,  3,  2,  1,  4,
                                      9,  11, 12, 13, 14, 15, 19, 20, 21, 22, 25, 26, 27, 28, 29, 31};

__global__ __launch_bounds__(64) void ssb_encode_kernel(const ssb_desc* desc, uint32_t nof, uint8_t* msgs,
                                                        const uint32_t* jump)
{
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= nof) {
    return;
  }
  const ssb_desc& d = desc[i];
  uint8_t         a[SSB_A];
  // payload generation: MIB bit 1..6 (the SFN's 6 MSBs) go to G[0..5], the others to G[14..31]
  uint32_t j_sfn = 0, j_other = 14;
  for (uint32_t k = 0; k != 24; ++k) {
    if (k >= 1 && k < 7) {
      a[PBCH_G[j_sfn++]] = d.mib[k] & 1u;
    } else {
      a[PBCH_G[j_other++]] = d.mib[k] & 1u;
    }
  }
  for (uint32_t k = 0; k != 4; ++k) { // 4th, 3rd, 2nd, 1st LSB of the SFN
    a[PBCH_G[j_sfn++]] = static_cast<uint8_t>((d.sfn >> (3 - k)) & 1u);
  }
  a[PBCH_G[10]] = static_cast<uint8_t>(d.hrf & 1u);
  if (d.L_max == 64) {
    a[PBCH_G[11]] = static_cast<uint8_t>((d.ssb_idx >> 5) & 1u);
    a[PBCH_G[12]] = static_cast<uint8_t>((d.ssb_idx >> 4) & 1u);
    a[PBCH_G[13]] = static_cast<uint8_t>((d.ssb_idx >> 3) & 1u);
  } else {
    a[PBCH_G[11]] = static_cast<uint8_t>((d.k_ssb >> 4) & 1u);
    a[PBCH_G[12]] = 0;
    a[PBCH_G[13]] = 0;
  }
  // first scrambling: the sequence from bit M v on, one bit per position that is not exempt
  const uint32_t w0   = d.enc_offset / 32;
  const uint32_t c_lo = gold_word(jump, d.pci, 32 * w0);
  const uint32_t c_hi = gold_word(jump, d.pci, 32 * (w0 + 1));
  const uint64_t c    = (static_cast<uint64_t>(c_hi) << 32 | c_lo) >> (d.enc_offset % 32);
  uint32_t       j    = 0;
  uint32_t       reg  = 0;
  uint8_t        b[SSB_K];
  for (uint32_t k = 0; k != SSB_A; ++k) {
    const bool ssb_bit = d.L_max == 64 && (k == PBCH_G[11] || k == PBCH_G[12] || k == PBCH_G[13]);
    uint32_t   s       = 0;
    if (!(ssb_bit || k == PBCH_G[10] || k == PBCH_G[8] || k == PBCH_G[7])) {
      s = static_cast<uint32_t>(c >> j) & 1u;
      ++j;
    }
    b[k] = static_cast<uint8_t>(a[k] ^ s);
    // CRC24C, MSB first (crc_calculator::calculate_bit)
    const uint32_t fb = ((reg >> 23) & 1u) ^ b[k];
    reg               = (reg << 1) & 0xffffffu;
    reg ^= fb ? (CRC24C_POLY & 0xffffffu) : 0u;
  }
  for (uint32_t k = 0; k != 24; ++k) {
    b[SSB_A + k] = static_cast<uint8_t>((reg >> (23 - k)) & 1u);
  }
  uint8_t* m = msgs + d.msg_offset;
  for (uint32_t k = 0; k != SSB_K; ++k) {
    m[k] = b[d.perm[k]];
  }
}

// Gold-sequence bit n of c_init
__device__ __forceinline__ uint32_t gold_bit(const uint32_t* jump, uint32_t c_init, uint32_t n)
{
  return (gold_word(jump, c_init, 32 * (n / 32)) >> (n % 32)) & 1u;
}

__global__ __launch_bounds__(256) void ssb_map_kernel(const ssb_desc* desc, const uint8_t* cws, const uint8_t* seq,
                                                      const uint32_t* jump)
{
  const ssb_desc& d   = desc[blockIdx.z];
  const uint32_t  sym = blockIdx.y; // OFDM symbol of the block
  const uint32_t  r   = threadIdx.x;
  if (r >= SSB_SC) {
    return;
  }
  const float    S = static_cast<float>(M_SQRT1_2);
  const uint32_t v = d.pci % 4;
  float2         x;
  if (sym == 0 || (sym == 2 && r >= 48 && r < 192)) {
    if (r < 56 || r >= 56 + SSB_SEQLEN) {
      return; // outside the PSS / SSS and the PBCH edges: untouched
    }
    const uint32_t i = r - 56;
    if (sym == 0) {
      // PSS: x[(i + m) mod 127] mapped to 1 - 2 x, times the amplitude (sc_prod: the imaginary part 0 x amp)
      const float s = 1.0f - 2.0f * static_cast<float>(seq[(i + d.pss_m) % SSB_SEQLEN]);
      x             = make_float2(s * d.pss_amp, 0.0f * d.pss_amp);
    } else {
      // SSS: d0 (amplitude 1) times d1 as the reference's complex product (out x d1)
      const float a0 = 1.0f - 2.0f * static_cast<float>(seq[SSB_SEQLEN + (i + d.sss_m0) % SSB_SEQLEN]);
      const float d1 = 1.0f - 2.0f * static_cast<float>(seq[2 * SSB_SEQLEN + (i + d.sss_m1) % SSB_SEQLEN]);
      const float xr = a0 * 1.0f, xi = 0.0f * 1.0f;
      x              = make_float2(xr * d1 - xi * 0.0f, xr * 0.0f + xi * d1);
    }
  } else {
    const bool     lower = r < 48;
    const uint32_t rr    = (sym == 2 && !lower) ? r - 192 : r; // position within the segment (starts at 0 mod 4)
    if (r % 4 == v) {
      // DM-RS: symbol 1 (60), symbol 2 lower (12) and upper (12), symbol 3 (60)
      const uint32_t n = sym == 1 ? r / 4 : (sym == 3 ? 84 + r / 4 : (lower ? 60 + rr / 4 : 72 + rr / 4));
      x = make_float2(gold_bit(jump, d.c_init_dmrs, 2 * n) ? -S : S, gold_bit(jump, d.c_init_dmrs, 2 * n + 1) ? -S : S);
    } else {
      // PBCH symbol j: symbol 1 (180), symbol 2 lower (36) and upper (36), symbol 3 (180)
      const uint32_t below = rr - (rr + 3 - v) / 4; // PBCH REs before rr in the segment
      const uint32_t j     = sym == 1 ? below : (sym == 3 ? 252 + below : (lower ? 180 + below : 216 + below));
      const uint8_t* cw    = cws + d.cw_offset;
      const uint32_t b0    = cw[2 * j] ^ gold_bit(jump, d.pci, d.mod_offset + 2 * j);
      const uint32_t b1    = cw[2 * j + 1] ^ gold_bit(jump, d.pci, d.mod_offset + 2 * j + 1);
      x                    = make_float2(b0 ? -S : S, b1 ? -S : S);
    }
  }
  const uint32_t  val = cbf16_pack(x.x, x.y);
  const uint64_t  off = static_cast<uint64_t>(d.l0 + sym) * d.nof_subc + d.k0 + r;
  for (uint32_t p = 0; p != d.nof_ports; ++p) {
    d.grid[static_cast<uint64_t>(d.ports[p]) * d.port_stride + off] = val;
  }
}

} // namespace

hipError_t launch_ssb_encode(const ssb_desc* d_desc, uint32_t nof, uint8_t* d_msgs, const uint32_t* jump,
                             hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ssb_encode_kernel, dim3((nof + 63) / 64), dim3(64), 0, stream, d_desc, nof, d_msgs, jump);
  return hipGetLastError();
}

hipError_t launch_ssb_map(const ssb_desc* d_desc, uint32_t nof, const uint8_t* d_cws, const uint8_t* seq,
                          const uint32_t* jump, hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ssb_map_kernel, dim3(1, 4, nof), dim3(256), 0, stream, d_desc, d_cws, seq, jump);
  return hipGetLastError();
}

} // namespace srs_amd
