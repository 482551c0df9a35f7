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

#include "gold_sequence.h"
#include "modulation_args.h"

#pragma clang fp contract(off)

namespace srs_amd {
namespace {

constexpr float NEAR_ZERO = 1e-9f;

__device__ __forceinline__ unsigned get_bit(const uint8_t* b, unsigned p)
{
  return (b[p >> 3] >> (7 - (p & 7))) & 1u;
}

__device__ __forceinline__ float safe_rcp(float nv)
{
  return nv > 0.0f ? 1.0f / nv : 0.0f;
}

// quantize_ps (avx2_helpers.h:121): scale, clip to +-120, round half to even.
__device__ __forceinline__ int q_simd(float v, float range)
{
  float x = v * (120.0f / range);
  x       = x > 120.0f ? 120.0f : x;
  x       = x < -120.0f ? -120.0f : x;
  x       = __builtin_rintf(x);
  return x != x ? 0 : static_cast<int>(x);
}

// log_likelihood_ratio::quantize: clip to the range, round half away from zero.
__device__ __forceinline__ int q_scalar(float v, float range)
{
  const float c = fabsf(v) > range ? copysignf(range, v) : v;
  return static_cast<int>(roundf(c / range * 120.0f));
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
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.nof_symbols) {
    return;
  }
  const float2 s    = reinterpret_cast<const float2*>(a.symbols)[i];
  const float  nv   = a.noise_vars[i];
  const bool   simd = i < a.block_end;
  const float  xs[2] = {s.x, s.y};
  constexpr float SQRT2 = 1.41421356237309504880f;
  if (a.qm <= 1) { // BPSK / pi/2-BPSK: scalar code only
    float re = s.x, im = s.y;
    if (a.qm == 0 && (i & 1)) {
      const float t = re;
      re            = im;
      im            = -t;
    }
    a.llrs[i] = static_cast<int8_t>(nv > 0.0f ? q_scalar(2.0f * SQRT2 * (re + im) / nv, 24.0f) : 0);
    return;
  }
  int8_t* o = a.llrs + static_cast<size_t>(i) * a.qm;
  if (a.qm == 2) {
    const float GAIN = 2.0f * SQRT2;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      o[c] = static_cast<int8_t>(simd ? q_simd((GAIN * xs[c]) * safe_rcp(nv), 24.0f)
                                      : (nv > 0.0f ? q_scalar(GAIN * xs[c] / nv, 24.0f) : 0));
    }
    return;
  }
  if (a.qm == 4) {
    const float S = a.qam16_scale;
    const float G = 4.0f * S, TH = 2.0f * S;
    if (simd) {
      const float rcp = safe_rcp(nv);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float x   = xs[c];
        const float f   = G * x;
        float       l01 = fabsf(x) > TH ? (2.0f * f - copysignf(0.8f, x)) : f;
        float       l23 = 0.8f - fabsf(f);
        l01 *= rcp;
        l23 *= rcp;
        if (fabsf(x) <= NEAR_ZERO) {
          l01 = 0.0f;
          l23 = 0.0f;
        }
        o[c]     = static_cast<int8_t>(q_simd(l01, 20.0f));
        o[2 + c] = static_cast<int8_t>(q_simd(l23, 20.0f));
      }
    } else {
      const bool zero = (s.x * s.x + s.y * s.y) < NEAR_ZERO;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float x = xs[c];
        if (zero || !(nv > 0.0f)) {
          o[c]     = 0;
          o[2 + c] = 0;
          continue;
        }
        float l = G * x;
        if (fabsf(x) > TH) {
          l = __builtin_fmaf(2.0f, l, -copysignf(0.8f, x));
        }
        o[c]           = static_cast<int8_t>(q_scalar(l / nv, 20.0f));
        const float l2 = __builtin_fmaf(-G, fabsf(x), 0.8f);
        o[2 + c]       = static_cast<int8_t>(q_scalar(l2 / nv, 20.0f));
      }
    }
    return;
  }
  // 64QAM / 256QAM: interval functions.
  const int  m    = a.qm / 2;
  const bool zero = !simd && (s.x * s.x + s.y * s.y) < NEAR_ZERO;
  const float rcp = safe_rcp(nv);
  for (int k = 0; k < m; ++k) {
    const demod_interval_table& t = a.tab[k];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float x = xs[c];
      int         q;
      if (zero) {
        q = 0;
      } else if (simd) {
        int idx = static_cast<int>(floorf(x * (1.0f / t.width))) + t.n / 2;
        idx     = idx < 0 ? 0 : (idx > t.n - 1 ? t.n - 1 : idx);
        float l = (t.slope[idx] * x + t.icpt[idx]) * rcp;
        if (fabsf(x) <= NEAR_ZERO) {
          l = 0.0f;
        }
        q = q_simd(l, 20.0f);
      } else {
        int idx = static_cast<int>(floorf(x / t.width)) + t.n / 2;
        idx     = idx < 0 ? 0 : (idx > t.n - 1 ? t.n - 1 : idx);
        float l = __builtin_fmaf(t.slope[idx], x, t.icpt[idx]);
        l *= rcp;
        q = q_scalar(l, 20.0f);
      }
      o[2 * k + c] = static_cast<int8_t>(q);
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
