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
