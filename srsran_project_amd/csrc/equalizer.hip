// equalizer.hip -- MI355X channel equalizer (ZF 1xN, ZF 2xN, MMSE 1xN).
//
// Reference: lib/phy/upper/equalization/equalize_zf_1xn.h:131-170 and
// equalize_zf_2xn.h:185-250 (scalar path: the same float operations in the same
// order, IEEE division), dispatch and port reduction in
// channel_equalizer_generic_impl.cpp:122-170, 290-378.
// One thread per resource element; per RE the kernel reads the P received
// samples and the L*P channel coefficients (cbf16, 4 B each) and writes L
// complex symbols and L variances: purely HBM-bound, no reuse to exploit.
// Algorithmic bytes per RE: 4*P*(1 + L) + 12*L.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "equalizer_args.h"

namespace srs_amd {
namespace {

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

template <int P>
__global__ __launch_bounds__(256) void equalize_1xn_kernel(equalizer_args a)
{
  const uint32_t* sym = static_cast<const uint32_t*>(a.symbols);
  const uint32_t* est = static_cast<const uint32_t*>(a.estimates);
  for (uint32_t re = blockIdx.x * 256 + threadIdx.x; re < a.nof_re; re += gridDim.x * 256) {
    float ch_mod_sq = 0.0f, nvar_acc = 0.0f;
    cplx  re_out    = {0.0f, 0.0f};
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const cplx  y  = from_cbf16(sym[p * a.nof_re + re]);
      const cplx  h  = from_cbf16(est[p * a.nof_re + re]);
      const float hn = norm(h);
      if (__builtin_isnormal(hn) && ((a.valid_ports >> p) & 1u)) {
        ch_mod_sq += hn;
        nvar_acc += hn * a.port_noise_var[p];
        const cplx t = mul_conj(y, h);
        re_out.x += t.x;
        re_out.y += t.y;
      }
    }
    cplx  out = {0.0f, 0.0f};
    float nv  = __builtin_inff();
    const float d = a.tx_scaling * ch_mod_sq;
    if (__builtin_isnormal(d) && __builtin_isnormal(nvar_acc)) {
      const float rcp = 1.0f / d;
      out             = {re_out.x * rcp, re_out.y * rcp};
      nv              = nvar_acc * rcp * rcp;
    }
    reinterpret_cast<cplx*>(a.eq_symbols)[re] = out;
    a.eq_noise_vars[re]                       = nv;
  }
}

template <int P>
__global__ __launch_bounds__(256) void equalize_2xn_kernel(equalizer_args a)
{
  const uint32_t* sym = static_cast<const uint32_t*>(a.symbols);
  const uint32_t* est = static_cast<const uint32_t*>(a.estimates);
  for (uint32_t re = blockIdx.x * 256 + threadIdx.x; re < a.nof_re; re += gridDim.x * 256) {
    cplx y[P], h0[P], h1[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      y[p]  = from_cbf16(sym[p * a.nof_re + re]);
      h0[p] = from_cbf16(est[p * a.nof_re + re]);
      h1[p] = from_cbf16(est[(P + p) * a.nof_re + re]);
    }
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
    const float d_pinv    = a.tx_scaling * ((n0 * n1) - xi_mod_sq);
    const float d_nvars   = a.tx_scaling * d_pinv;
    float4      out       = {0.0f, 0.0f, 0.0f, 0.0f};
    float2      nv        = {__builtin_inff(), __builtin_inff()};
    if (a.noise_ok && __builtin_isnormal(d_pinv)) {
      const float rcp  = 1.0f / d_pinv;
      const float nrcp = 1.0f / d_nvars;
      const cplx  xm1  = cmul(xi, m1);
      const cplx  xm0  = cmul({xi.x, -xi.y}, m0);
      out.x            = ((n1 * m0.x) - xm1.x) * rcp;
      out.y            = ((n1 * m0.y) - xm1.y) * rcp;
      out.z            = ((n0 * m1.x) - xm0.x) * rcp;
      out.w            = ((n0 * m1.y) - xm0.y) * rcp;
      nv.x             = a.noise_var * n1 * nrcp;
      nv.y             = a.noise_var * n0 * nrcp;
    }
    reinterpret_cast<float4*>(a.eq_symbols)[re]    = out;
    reinterpret_cast<float2*>(a.eq_noise_vars)[re] = nv;
  }
}

} // namespace

hipError_t launch_equalizer(const equalizer_args& a, uint32_t nof_ports, uint32_t nof_layers, hipStream_t stream)
{
  if (a.nof_re == 0) {
    return hipSuccess;
  }
  uint32_t blocks = (a.nof_re + 255) / 256;
  blocks          = blocks > 65536u ? 65536u : blocks;
  if (nof_layers == 1) {
    switch (nof_ports) {
      case 1:
        hipLaunchKernelGGL(equalize_1xn_kernel<1>, dim3(blocks), dim3(256), 0, stream, a);
        break;
      case 2:
        hipLaunchKernelGGL(equalize_1xn_kernel<2>, dim3(blocks), dim3(256), 0, stream, a);
        break;
      case 4:
        hipLaunchKernelGGL(equalize_1xn_kernel<4>, dim3(blocks), dim3(256), 0, stream, a);
        break;
      default:
        return hipErrorInvalidValue;
    }
  } else if (nof_layers == 2) {
    switch (nof_ports) {
      case 2:
        hipLaunchKernelGGL(equalize_2xn_kernel<2>, dim3(blocks), dim3(256), 0, stream, a);
        break;
      case 4:
        hipLaunchKernelGGL(equalize_2xn_kernel<4>, dim3(blocks), dim3(256), 0, stream, a);
        break;
      default:
        return hipErrorInvalidValue;
    }
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

} // namespace srs_amd
