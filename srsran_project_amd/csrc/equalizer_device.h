// equalizer_device.h -- per-RE ZF / MMSE equalizer math shared by the
// stand-alone equalizer (equalizer.hip) and the fused PUSCH demodulator
// (pusch_demod.hip).
//
// Reference: lib/phy/upper/equalization/equalize_zf_1xn.h:131-170 and
// equalize_zf_2xn.h:185-250 (scalar path: the same float operations in the same
// order, IEEE division); port validity / reduction of
// channel_equalizer_generic_impl.cpp:122-170, 290-378.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {
namespace eq {

struct cplx {
  float x, y;
};

__device__ __forceinline__ cplx from_cbf16(uint32_t u)
{
  return {__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}

__device__ __forceinline__ float norm(cplx a)
{
  return a.x * a.x + a.y * a.y;
}

// a * conj(b)
__device__ __forceinline__ cplx mul_conj(cplx a, cplx b)
{
  return {a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y};
}

__device__ __forceinline__ cplx cmul(cplx a, cplx b)
{
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}

// One layer over P ports: y[p], h[p]; port_nv / valid_ports as channel_equalizer_generic_impl.cpp:131.
template <int P>
__device__ __forceinline__ void
equalize_1xn(const cplx* y, const cplx* h, const float* port_nv, uint32_t valid_ports, float tx_scaling, cplx& out,
             float& nv)
{
  float ch_mod_sq = 0.0f, nvar_acc = 0.0f;
  cplx  re_out    = {0.0f, 0.0f};
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const float hn = norm(h[p]);
    if (__builtin_isnormal(hn) && ((valid_ports >> p) & 1u)) {
      ch_mod_sq += hn;
      nvar_acc += hn * port_nv[p];
      const cplx t = mul_conj(y[p], h[p]);
      re_out.x += t.x;
      re_out.y += t.y;
    }
  }
  out           = {0.0f, 0.0f};
  nv            = __builtin_inff();
  const float d = tx_scaling * ch_mod_sq;
  if (__builtin_isnormal(d) && __builtin_isnormal(nvar_acc)) {
    const float rcp = 1.0f / d;
    out             = {re_out.x * rcp, re_out.y * rcp};
    nv              = nvar_acc * rcp * rcp;
  }
}

// Two layers over P ports: h0[p], h1[p]; noise_var = the largest port variance, noise_ok its validity.
template <int P>
__device__ __forceinline__ void equalize_2xn(const cplx* y,
                                             const cplx* h0,
                                             const cplx* h1,
                                             float       noise_var,
                                             bool        noise_ok,
                                             float       tx_scaling,
                                             float4&     out,
                                             float2&     nv)
{
  float n0 = 0.0f, n1 = 0.0f;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    n0 += norm(h0[p]);
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    n1 += norm(h1[p]);
  }
  cplx xi = {0.0f, 0.0f}, m0 = {0.0f, 0.0f}, m1 = {0.0f, 0.0f};
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const cplx t = mul_conj(h1[p], h0[p]); // conj(h0) * h1
    xi.x += t.x;
    xi.y += t.y;
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const cplx t0 = mul_conj(y[p], h0[p]);
    const cplx t1 = mul_conj(y[p], h1[p]);
    m0.x += t0.x;
    m0.y += t0.y;
    m1.x += t1.x;
    m1.y += t1.y;
  }
  const float xi_mod_sq = norm(xi);
  const float d_pinv    = tx_scaling * ((n0 * n1) - xi_mod_sq);
  const float d_nvars   = tx_scaling * d_pinv;
  out                   = {0.0f, 0.0f, 0.0f, 0.0f};
  nv                    = {__builtin_inff(), __builtin_inff()};
  if (noise_ok && __builtin_isnormal(d_pinv)) {
    const float rcp  = 1.0f / d_pinv;
    const float nrcp = 1.0f / d_nvars;
    const cplx  xm1  = cmul(xi, m1);
    const cplx  xm0  = cmul({xi.x, -xi.y}, m0);
    out.x            = ((n1 * m0.x) - xm1.x) * rcp;
    out.y            = ((n1 * m0.y) - xm1.y) * rcp;
    out.z            = ((n0 * m1.x) - xm0.x) * rcp;
    out.w            = ((n0 * m1.y) - xm0.y) * rcp;
    nv.x             = noise_var * n1 * nrcp;
    nv.y             = noise_var * n0 * nrcp;
  }
}

} // namespace eq
} // namespace srs_amd
