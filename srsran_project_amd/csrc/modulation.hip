// modulation.hip -- MI355X modulation mapper, soft demodulation mapper and
// Gold-sequence scrambling (PDSCH / PUSCH data path).
//
// Reference: lib/phy/upper/channel_modulation/modulation_mapper_lut_impl.cpp
// (table modulator, bit order MSB-first), demodulation_mapper_*.cpp (soft
// demapping; the kernel reproduces an x86-64-v3 build of the reference: the
// AVX2 arithmetic -- reciprocal of the noise, mul / add without contraction,
// interval index from a multiply by 1/width, quantisation by a scale, clip and
// round-half-even -- for symbols [0, block_end) and the scalar code -- IEEE
// division, FMA interval lines, round-half-away -- for the remainder), and
// lib/phy/upper/sequence_generators/pseudo_random_generator_impl.cpp (TS 38.211
// 5.2.1 Gold sequence, Nc = 1600).
// All three are one-thread-per-element, HBM-bound gathers; the Gold sequence
// is produced 32 bits per thread from the LFSR states jumped ahead with
// precomputed GF(2) matrices (A^(2^k)), so a whole codeword is scrambled in
// one launch without any sequential pass.
#include <hip/hip_runtime.h>

#include "demap_device.h"
#include "gold_sequence.h"
#include "modulation_args.h"

#pragma clang fp contract(off)

namespace srs_amd {
using namespace demap;
namespace {

__device__ __forceinline__ unsigned get_bit(const uint8_t* b, unsigned p)
{
  return (b[p >> 3] >> (7 - (p & 7))) & 1u;
}

} // namespace

__global__ __launch_bounds__(256) void modulate_kernel(modulate_args a)
{
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.nof_symbols) {
    return;
  }
  constexpr float R2 = 0.70710678118654752440f;
  float2          v;
  if (a.qm <= 1) {
    const unsigned b = get_bit(a.bits, i);
    v                = b ? float2{-R2, -R2} : float2{R2, R2};
    if (a.qm == 0 && (i & 1)) {
      v = b ? float2{R2, -R2} : float2{-R2, R2};
    }
  } else {
    unsigned idx = 0;
    for (int k = 0; k < a.qm; ++k) {
      idx = (idx << 1) | get_bit(a.bits, i * a.qm + k);
    }
    v = reinterpret_cast<const float2*>(a.table)[idx];
  }
  reinterpret_cast<float2*>(a.symbols)[i] = v;
}

__global__ __launch_bounds__(256) void demodulate_kernel(demodulate_args a)
{
  __shared__ float lt[4 * 2 * 16];
  stage_interval_tables(a, lt);
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.nof_symbols) {
    return;
  }
  demap_symbol(a, lt, reinterpret_cast<const float2*>(a.symbols)[i], a.noise_vars[i], i, i < a.block_end,
               a.llrs + static_cast<size_t>(i) * (a.qm < 1 ? 1 : a.qm));
}

// Soft demapping + descrambling of nof_grids codewords (PUSCH, pusch_demodulator_impl.cpp:203-400,
// one demapper call per OFDM symbol as the reference makes them):
// symbols [grid][grid_symbols], LLRs [grid][llr_stride]. A workgroup demaps DD_SYMS symbols of one
// grid into LDS (4 per thread), builds the Gold words of its LLR range (one per lane, each wave's base
// state jumped once on the scalar unit) and writes the descrambled LLRs 8 bytes at a time.
constexpr uint32_t DD_SYMS = 1024;

// MULTI: one argument pair per PDU (items[blockIdx.y], grid 0), the PUSCH processor's slot form
template <bool MULTI>
__global__ __launch_bounds__(256) void demap_descramble_kernel(demodulate_args own_a, demap_descramble_args own_d,
                                                               const demap_item* items)
{
  const demodulate_args&       a = MULTI ? items[blockIdx.y].a : own_a;
  const demap_descramble_args& d = MULTI ? items[blockIdx.y].d : own_d;
  if (MULTI && blockIdx.x * DD_SYMS >= d.grid_symbols) {
    return;
  }
  __shared__ int8_t   s_llr[DD_SYMS * 8];
  __shared__ uint32_t words[DD_SYMS * 8 / 32];
  __shared__ float    lt[4 * 2 * 16];
  stage_interval_tables(a, lt);
  const uint32_t      g   = MULTI ? 0u : blockIdx.y;
  const uint32_t      bpp = a.qm < 1 ? 1u : static_cast<uint32_t>(a.qm); // LLRs per symbol
  const uint32_t      s0  = blockIdx.x * DD_SYMS;                        // first symbol (within the grid)
  const uint32_t      n0  = s0 * bpp;                                    // first LLR of the workgroup
  if (threadIdx.x < DD_SYMS * bpp / 32) {
    uint32_t x1, x2;
    gold_state_wave(d.jump, d.c_init, n0 + 32 * (threadIdx.x & ~63u), 32 * (threadIdx.x & 63u), x1, x2);
    words[threadIdx.x] = gold_next32(x1, x2);
  }
#pragma unroll
  for (uint32_t r = 0; r < DD_SYMS / 256; ++r) {
    const uint32_t t = r * 256 + threadIdx.x, i = s0 + t;
    if (i < d.grid_symbols) {
      const size_t gs = static_cast<size_t>(g) * d.grid_symbols + i;
      bool simd = false;
#pragma unroll
      for (int l = 0; l < 14; ++l) { // uniform bounds (SGPRs): the OFDM symbol's SIMD block range
        simd |= (i >= d.sym_lo[l]) & (i < d.simd_hi[l]);
      }
      demap_symbol(a, lt, reinterpret_cast<const float2*>(a.symbols)[gs], a.noise_vars[gs], i, simd,
                   s_llr + t * bpp);
    }
  }
  __syncthreads();
  const uint32_t nb  = min(DD_SYMS, d.grid_symbols - s0) * bpp;
  int8_t*        row = d.llrs + static_cast<uint64_t>(g) * d.llr_stride + n0;
  for (uint32_t b0 = 8 * threadIdx.x; b0 < nb; b0 += 8 * 256) {
    const uint32_t c = words[b0 / 32] >> (b0 % 32);
    union {
      uint2  v;
      int8_t b[8];
    } x;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int v = s_llr[b0 + k];
      x.b[k]      = static_cast<int8_t>(((c >> k) & 1u) ? -v : v);
    }
    if (b0 + 8 <= nb && (reinterpret_cast<uintptr_t>(row + b0) & 7u) == 0) {
      *reinterpret_cast<uint2*>(row + b0) = x.v;
    } else {
      for (uint32_t k = 0; k < 8 && b0 + k < nb; ++k) {
        row[b0 + k] = x.b[k];
      }
    }
  }
}

__global__ __launch_bounds__(256) void scramble_bits_kernel(prbs_args a)
{
  const uint32_t w = blockIdx.x * 256 + threadIdx.x; // 32-bit word of the sequence
  if (w * 32 >= a.length) {
    return;
  }
  uint32_t x1, x2; // the wave's first word is the scalar jump, lanes advance by 32 x lane bits
  gold_state_wave(a.jump, a.c_init, (w - (threadIdx.x & 63u)) * 32, (threadIdx.x & 63u) * 32, x1, x2);
  const uint32_t c = gold_next32(x1, x2);
#pragma unroll
  for (int byte = 0; byte < 4; ++byte) {
    const uint32_t p = w * 4 + byte;
    if (p * 8 >= a.length) {
      break;
    }
    // sequence bits 8p .. 8p+7 -> MSB-first byte
    const uint32_t cb  = (c >> (8 * byte)) & 0xffu;
    const uint32_t rev = __builtin_bitreverse32(cb) >> 24;
    uint32_t       v   = (a.in_bits ? a.in_bits[p] : 0u) ^ rev;
    const uint32_t rem = a.length - p * 8;
    if (rem < 8) {
      v &= 0xffu << (8 - rem); // bits past the end stay zero
    }
    a.out_bits[p] = static_cast<uint8_t>(v);
  }
}

__global__ __launch_bounds__(256) void descramble_llrs_kernel(prbs_args a)
{
  const uint32_t w = blockIdx.x * 256 + threadIdx.x;
  if (w * 32 >= a.length) {
    return;
  }
  uint32_t x1, x2; // the wave's first word is the scalar jump, lanes advance by 32 x lane bits
  gold_state_wave(a.jump, a.c_init, (w - (threadIdx.x & 63u)) * 32, (threadIdx.x & 63u) * 32, x1, x2);
  const uint32_t c = gold_next32(x1, x2);
  for (int b = 0; b < 32; ++b) {
    const uint32_t i = w * 32 + b;
    if (i >= a.length) {
      break;
    }
    const int v   = a.in_llrs[i];
    a.out_llrs[i] = static_cast<int8_t>(((c >> b) & 1u) ? -v : v);
  }
}

// Words 0 .. nof_words of the Gold sequence of c_init (c(32 w + b) at bit b of word w): the PUSCH
// equalizer's descrambling table (pusch_demod.hip), generated once per demodulator plan.
__global__ __launch_bounds__(256) void gold_words_kernel(const uint32_t* jump, uint32_t c_init, uint32_t* out,
                                                         uint32_t nof_words)
{
  const uint32_t w = blockIdx.x * 256 + threadIdx.x;
  uint32_t       x1, x2;
  gold_state_wave(jump, c_init, (w - (threadIdx.x & 63u)) * 32, (threadIdx.x & 63u) * 32, x1, x2);
  const uint32_t c = gold_next32(x1, x2);
  if (w < nof_words) {
    out[w] = c;
  }
}

hipError_t launch_gold_words(const uint32_t* jump, uint32_t c_init, uint32_t* out, uint32_t nof_words,
                             hipStream_t stream)
{
  if (nof_words == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(gold_words_kernel, dim3((nof_words + 255) / 256), dim3(256), 0, stream, jump, c_init, out,
                     nof_words);
  return hipGetLastError();
}

hipError_t launch_modulate(const modulate_args& a, hipStream_t stream)
{
  if (a.nof_symbols == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(modulate_kernel, dim3((a.nof_symbols + 255) / 256), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_demodulate(const demodulate_args& a, hipStream_t stream)
{
  if (a.nof_symbols == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(demodulate_kernel, dim3((a.nof_symbols + 255) / 256), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_demap_descramble(const demodulate_args& a, const demap_descramble_args& d, uint32_t nof_grids,
                                  hipStream_t stream)
{
  if (d.grid_symbols == 0 || nof_grids == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(demap_descramble_kernel<false>, dim3((d.grid_symbols + DD_SYMS - 1) / DD_SYMS, nof_grids),
                     dim3(256), 0, stream, a, d, nullptr);
  return hipGetLastError();
}

hipError_t launch_demap_descramble_items(const demap_item* items, uint32_t n, uint32_t max_symbols, hipStream_t stream)
{
  if (n == 0 || max_symbols == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(demap_descramble_kernel<true>, dim3((max_symbols + DD_SYMS - 1) / DD_SYMS, n), dim3(256), 0,
                     stream, demodulate_args{}, demap_descramble_args{}, items);
  return hipGetLastError();
}

hipError_t launch_scramble_bits(const prbs_args& a, hipStream_t stream)
{
  if (a.length == 0) {
    return hipSuccess;
  }
  const uint32_t words = (a.length + 31) / 32;
  hipLaunchKernelGGL(scramble_bits_kernel, dim3((words + 255) / 256), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_descramble_llrs(const prbs_args& a, hipStream_t stream)
{
  if (a.length == 0) {
    return hipSuccess;
  }
  const uint32_t words = (a.length + 31) / 32;
  hipLaunchKernelGGL(descramble_llrs_kernel, dim3((words + 255) / 256), dim3(256), 0, stream, a);
  return hipGetLastError();
}

} // namespace srs_amd
