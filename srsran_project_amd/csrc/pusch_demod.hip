// pusch_demod.hip -- MI355X PUSCH demodulator kernels.
//
// pusch_equalize_kernel<P, L>: one thread per (grid, OFDM symbol, subcarrier) of
// the allocation. Its data-RE index j (codeword order: symbol-major,
// subcarrier ascending, DM-RS CDM groups without data excluded on DM-RS
// symbols, pusch_demodulator_impl.cpp:218-262) comes from the per-(symbol, PRB)
// table; it gathers the P received samples and the L x P channel
// coefficients straight from the grid and the estimate tensor (the reference
// copies both into temporary buffers first, get_ch_data_re /
// get_ch_data_estimates) and equalizes with the shared ZF math
// (equalizer_device.h: the reference's ZF 1 x N / 2 x N, or the L-layer Cholesky solve for the
// ZF 3 x 4 / 4 x 4 and MMSE 2 x N / 3 x 4 / 4 x 4 cases the open reference does not implement),
// writing [j][layer] symbols and variances.
// The per-port noise variances come from the DM-RS estimator's measurements
// on the device, so the chain needs no host round trip.
// The soft demapper and revert_scrambling (pusch_demodulator_impl.cpp:36-190) run fused in
// demap_descramble_kernel (modulation.hip).
#include <hip/hip_runtime.h>

#include "equalizer_device.h"
#include "pusch_demod_args.h"

namespace srs_amd {
namespace {

template <int P, int L, bool MMSE>
__global__ __launch_bounds__(256) void pusch_equalize_kernel(pusch_eq_args a)
{
  const uint32_t  l   = a.first_symbol + blockIdx.y;
  const uint32_t  sc  = a.first_subc + blockIdx.x * 256 + threadIdx.x;
  const uint32_t  gi  = blockIdx.z;
  if (sc >= a.nof_subc) {
    return;
  }
  const uint32_t e   = a.re_table[l * a.nof_prb + sc / 12];
  const uint32_t bit = sc % 12;
  if (((e >> bit) & 1u) == 0) {
    return;
  }
  const uint32_t j = (e >> 12) + __builtin_popcount(e & ((1u << bit) - 1u));

  const uint32_t* grid = a.grids + gi * a.grid_stride + l * a.nof_subc + sc;
  const uint32_t* est  = a.estimates + gi * a.est_stride + l * a.nof_subc + sc;
  const srs_amd_chest_port_stats* st = a.stats + gi * P;
  const uint32_t  plane = 14 * a.nof_subc;

  eq::cplx y[P], h[P * L];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    y[p] = eq::from_cbf16(grid[static_cast<uint64_t>(p) * plane]);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      h[p * L + l] = eq::from_cbf16(est[static_cast<uint64_t>(p * L + l) * plane]);
    }
  }
  const uint64_t out = static_cast<uint64_t>(gi) * a.nof_re * L + static_cast<uint64_t>(j) * L;
  if (L == 1) {
    eq::cplx h0[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      h0[p] = h[p];
    }
    float    nvp[P];
    uint32_t valid = 0;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      nvp[p] = st[p].noise_var;
      valid |= (__builtin_isnormal(nvp[p]) && nvp[p] > 0.0f) ? (1u << p) : 0u;
    }
    eq::cplx s;
    float    nv;
    eq::equalize_1xn<P>(y, h0, nvp, valid, 1.0f, s, nv);
    a.eq_symbols[out]    = make_float2(s.x, s.y);
    a.eq_noise_vars[out] = nv;
  } else {
    // channel_equalizer_generic_impl.cpp:304: the largest port variance (std::max_element order).
    float nmax = st[0].noise_var;
#pragma unroll
    for (int p = 1; p < P; ++p) {
      nmax = (nmax < st[p].noise_var) ? st[p].noise_var : nmax;
    }
    const bool ok = __builtin_isnormal(nmax) && nmax >= 0.0f;
    if constexpr (L == 2 && !MMSE) {
      eq::cplx h0[P], h1[P];
#pragma unroll
      for (int p = 0; p < P; ++p) {
        h0[p] = h[p * 2];
        h1[p] = h[p * 2 + 1];
      }
      float4 s;
      float2 nv;
      eq::equalize_2xn<P>(y, h0, h1, nmax, ok, 1.0f, s, nv);
      a.eq_symbols[out]        = make_float2(s.x, s.y);
      a.eq_symbols[out + 1]    = make_float2(s.z, s.w);
      a.eq_noise_vars[out]     = nv.x;
      a.eq_noise_vars[out + 1] = nv.y;
    } else {
      eq::cplx s[L];
      float    nv[L];
      eq::equalize_mimo<P, L, MMSE>(y, h, nmax, ok, 1.0f, s, nv);
#pragma unroll
      for (int l = 0; l < L; ++l) {
        a.eq_symbols[out + l]    = make_float2(s[l].x, s[l].y);
        a.eq_noise_vars[out + l] = nv[l];
      }
    }
  }
}

} // namespace

hipError_t launch_pusch_equalize(const pusch_eq_args& a, uint32_t nof_ports, uint32_t nof_layers, bool mmse,
                                 uint32_t nof_symbols, uint32_t span_subc, uint32_t nof_grids, hipStream_t stream)
{
  if (nof_symbols == 0 || span_subc == 0 || nof_grids == 0) {
    return hipSuccess;
  }
  const dim3 grid((span_subc + 255) / 256, nof_symbols, nof_grids);
#define SRS_EQ_CASE(PP, LL, MM)                                                                                       \
  if (nof_ports == PP && nof_layers == LL && mmse == MM) {                                                            \
    hipLaunchKernelGGL((pusch_equalize_kernel<PP, LL, MM>), grid, dim3(256), 0, stream, a);                          \
    return hipGetLastError();                                                                                         \
  }
  // one layer: MMSE is the ZF equalizer (channel_equalizer_generic_impl.cpp:343)
  SRS_EQ_CASE(1, 1, false)
  SRS_EQ_CASE(2, 1, false)
  SRS_EQ_CASE(4, 1, false)
  SRS_EQ_CASE(2, 2, false)
  SRS_EQ_CASE(4, 2, false)
  SRS_EQ_CASE(4, 3, false)
  SRS_EQ_CASE(4, 4, false)
  SRS_EQ_CASE(2, 2, true)
  SRS_EQ_CASE(4, 2, true)
  SRS_EQ_CASE(4, 3, true)
  SRS_EQ_CASE(4, 4, true)
#undef SRS_EQ_CASE
  return hipErrorInvalidValue;
}


} // namespace srs_amd
