// equalizer.hip -- MI355X channel equalizer (ZF 1xN, ZF 2xN, MMSE 1xN).
//
// Reference math in equalizer_device.h (equalize_zf_1xn.h:131-170,
// equalize_zf_2xn.h:185-250, channel_equalizer_generic_impl.cpp:122-170, 290-378).
// One thread per resource element; per RE the kernel reads the P received
// samples and the L*P channel coefficients (cbf16, 4 B each) and writes L
// complex symbols and L variances: purely HBM-bound, no reuse to exploit.
// Algorithmic bytes per RE: 4*P*(1 + L) + 12*L.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "equalizer_args.h"
#include "equalizer_device.h"

namespace srs_amd {
namespace {

using eq::cplx;
using eq::from_cbf16;

template <int P>
__global__ __launch_bounds__(256) void equalize_1xn_kernel(equalizer_args a)
{
  const uint32_t* sym = static_cast<const uint32_t*>(a.symbols);
  const uint32_t* est = static_cast<const uint32_t*>(a.estimates);
  for (uint32_t re = blockIdx.x * 256 + threadIdx.x; re < a.nof_re; re += gridDim.x * 256) {
    cplx y[P], h[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      y[p] = from_cbf16(sym[p * a.nof_re + re]);
      h[p] = from_cbf16(est[p * a.nof_re + re]);
    }
    cplx  out;
    float nv;
    eq::equalize_1xn<P>(y, h, a.port_noise_var, a.valid_ports, a.tx_scaling, out, nv);
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
    float4 out;
    float2 nv;
    eq::equalize_2xn<P>(y, h0, h1, a.noise_var, a.noise_ok != 0, a.tx_scaling, out, nv);
    reinterpret_cast<float4*>(a.eq_symbols)[re]    = out;
    reinterpret_cast<float2*>(a.eq_noise_vars)[re] = nv;
  }
}

// L-layer ZF / MMSE (equalize_mimo): estimates [layer][port][re], outputs [re][layer].
template <int P, int L, bool MMSE>
__global__ __launch_bounds__(256) void equalize_mimo_kernel(equalizer_args a)
{
  const uint32_t* sym = static_cast<const uint32_t*>(a.symbols);
  const uint32_t* est = static_cast<const uint32_t*>(a.estimates);
  for (uint32_t re = blockIdx.x * 256 + threadIdx.x; re < a.nof_re; re += gridDim.x * 256) {
    cplx y[P], h[P * L];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      y[p] = from_cbf16(sym[p * a.nof_re + re]);
#pragma unroll
      for (int l = 0; l < L; ++l) {
        h[p * L + l] = from_cbf16(est[(l * P + p) * a.nof_re + re]);
      }
    }
    cplx  out[L];
    float nv[L];
    eq::equalize_mimo<P, L, MMSE>(y, h, a.noise_var, a.noise_ok != 0, a.tx_scaling, out, nv);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      reinterpret_cast<float2*>(a.eq_symbols)[static_cast<uint64_t>(re) * L + l] = make_float2(out[l].x, out[l].y);
      a.eq_noise_vars[static_cast<uint64_t>(re) * L + l]                         = nv[l];
    }
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
  } else if (nof_layers == 2 && !a.mmse) {
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
#define SRS_MIMO_CASE(PP, LL, MM)                                                                                     \
  if (nof_ports == PP && nof_layers == LL && (a.mmse != 0) == MM) {                                                   \
    hipLaunchKernelGGL((equalize_mimo_kernel<PP, LL, MM>), dim3(blocks), dim3(256), 0, stream, a);                   \
    return hipGetLastError();                                                                                         \
  }
    SRS_MIMO_CASE(2, 2, true)
    SRS_MIMO_CASE(4, 2, true)
    SRS_MIMO_CASE(4, 3, false)
    SRS_MIMO_CASE(4, 3, true)
    SRS_MIMO_CASE(4, 4, false)
    SRS_MIMO_CASE(4, 4, true)
#undef SRS_MIMO_CASE
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

} // namespace srs_amd
