// demap_device.h -- the soft demodulation mapper of one symbol (demodulation_mapper_*.cpp, see
// modulation.hip), shared by the demapper kernels (modulation.hip) and the PUSCH equalizer that demaps and
// descrambles its own output (pusch_demod.hip), so both produce the same LLR bits from the same symbol.
// The reference's AVX2 arithmetic is reproduced without floating-point contraction (the pragma inside
// each function keeps that independent of the including file).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "modulation_args.h"

namespace srs_amd {
namespace demap {

constexpr float NEAR_ZERO = 1e-9f;

__device__ __forceinline__ float safe_rcp(float nv)
{
#pragma clang fp contract(off)
  return nv > 0.0f ? 1.0f / nv : 0.0f;
}

// median(x, lo, hi) as one v_med3_i32 (lo <= hi)
__device__ __forceinline__ int med3_int(int x, int lo, int hi)
{
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
  return r;
}

// v_cvt_i32_f32: round toward zero, out-of-range values saturate, NaN converts to 0 (the instruction's defined
// behaviour, which a C++ conversion does not promise)
__device__ __forceinline__ int cvt_i32(float x)
{
  int r;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

#ifndef DEMAP_Q_CVT
#define DEMAP_Q_CVT 1
#endif
// quantize_ps (avx2_helpers.h:121): scale, clip to +-120, round half to even.
__device__ __forceinline__ int q_simd(float v, float range)
{
#pragma clang fp contract(off)
  const float x = v * (120.0f / range);
#if DEMAP_Q_CVT
  // round, convert (NaN -> 0, infinities saturate), then clip as one v_med3_i32: the same integer as clipping the
  // float first for every x (the bounds are integers), without a per-value NaN compare and select (r06)
  return med3_int(cvt_i32(__builtin_rintf(x)), -120, 120);
#else
  // clip as one v_med3_f32 (equal to the two compares for every non-NaN x; a NaN x gives 0 below)
  const float c = __builtin_rintf(__builtin_amdgcn_fmed3f(x, -120.0f, 120.0f));
  return x != x ? 0 : static_cast<int>(c);
#endif
}

// log_likelihood_ratio::quantize: clip to the range, round half away from zero.
__device__ __forceinline__ int q_scalar(float v, float range)
{
#pragma clang fp contract(off)
  const float c = fabsf(v) > range ? copysignf(range, v) : v;
  return static_cast<int>(roundf(c / range * 120.0f));
}

// LLRs of one symbol into o[0 .. max(qm, 1)); i: the symbol's index in its demodulation call (the
// pi/2-BPSK rotation parity), simd: the symbol lies in the reference's AVX2 blocks.
__device__ __forceinline__ void demap_symbol(const demodulate_args& a, const float* lt, float2 s, float nv, uint32_t i,
                                             bool simd, int8_t* o)
{
#pragma clang fp contract(off)
  const float  xs[2] = {s.x, s.y};
  constexpr float SQRT2 = 1.41421356237309504880f;
  if (a.qm <= 1) { // BPSK / pi/2-BPSK: scalar code only
    float re = s.x, im = s.y;
    if (a.qm == 0 && (i & 1)) {
      const float t = re;
      re            = im;
      im            = -t;
    }
    o[0] = static_cast<int8_t>(nv > 0.0f ? q_scalar(2.0f * SQRT2 * (re + im) / nv, 24.0f) : 0);
    return;
  }
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
  // 64QAM / 256QAM: interval functions.  One branch per symbol around the whole loop (the SIMD-block
  // arithmetic or the scalar tail's): a branch per LLR costs its exec-mask bookkeeping 2 qm times.
  const int   m   = a.qm / 2;
  const float rcp = safe_rcp(nv);
  if (simd) {
#if DEMAP_Q_CVT
    // |x| <= NEAR_ZERO gives LLR 0: a zero reciprocal for that component (the quantizer maps the 0 * (finite) and
    // 0 * inf = NaN products alike to 0), one select per component instead of one per LLR
    const float rc[2] = {fabsf(xs[0]) <= NEAR_ZERO ? 0.0f : rcp, fabsf(xs[1]) <= NEAR_ZERO ? 0.0f : rcp};
#endif
#pragma unroll
    for (int k = 0; k < 4; ++k) { // compile-time k: the table fields are scalar loads
      if (k >= m) {
        break;
      }
      const demod_interval_table& t = a.tab[k];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float x   = xs[c];
        const int   idx = med3_int(static_cast<int>(floorf(x * t.inv_width)) + t.n / 2, 0, t.n - 1);
#if DEMAP_Q_CVT
        const float l = (lt[(2 * k) * 16 + idx] * x + lt[(2 * k + 1) * 16 + idx]) * rc[c];
#else
        float l = (lt[(2 * k) * 16 + idx] * x + lt[(2 * k + 1) * 16 + idx]) * rcp;
        if (fabsf(x) <= NEAR_ZERO) {
          l = 0.0f;
        }
#endif
        o[2 * k + c] = static_cast<int8_t>(q_simd(l, 20.0f));
      }
    }
    return;
  }
  const bool zero = (s.x * s.x + s.y * s.y) < NEAR_ZERO;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k >= m) {
      break;
    }
    const demod_interval_table& t = a.tab[k];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float x = xs[c];
      int         q = 0;
      if (!zero) {
        int idx = static_cast<int>(floorf(x / t.width)) + t.n / 2;
        idx     = idx < 0 ? 0 : (idx > t.n - 1 ? t.n - 1 : idx);
        float l = __builtin_fmaf(lt[(2 * k) * 16 + idx], x, lt[(2 * k + 1) * 16 + idx]);
        l *= rcp;
        q = q_scalar(l, 20.0f);
      }
      o[2 * k + c] = static_cast<int8_t>(q);
    }
  }
}

// The interval tables' slopes and intercepts ([k][slope, icpt][16]) into LDS: per-lane lookups at a
// data-dependent interval would otherwise be loads from the kernel-argument segment.
__device__ __forceinline__ void stage_interval_tables(const demodulate_args& a, float* lt)
{
  for (uint32_t x = threadIdx.x; x < 4 * 2 * 16; x += blockDim.x) {
    const uint32_t k = x / 32, w = (x / 16) % 2, j = x % 16;
    lt[x]            = w == 0 ? a.tab[k].slope[j] : a.tab[k].icpt[j];
  }
  __syncthreads();
}

} // namespace demap
} // namespace srs_amd
