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

#include "chest_device.h"
#include "demap_device.h"
#include "equalizer_device.h"
#include "pusch_demod_args.h"
#include "kernel_probe.h"
#include "srsran_amd/profiling.h"

namespace srs_amd {
namespace {

// Soft demapping and descrambling of the L x QM LLRs of data RE j (codeword symbols i = j L + layer) into
// the grid's LLR row: demap_device.h's demapper (the SIMD or scalar arithmetic by the symbol's place in its
// OFDM symbol, as the reference's per-OFDM-symbol demapper calls), the sign flipped where the Gold sequence
// bit is one (the RE's L QM <= 32 sequence bits from two table words).
template <int L, int QM>
__device__ __forceinline__ void emit_re_llrs(const pusch_eq_args& a, const float* lt, int8_t* row, uint32_t j,
                                             uint32_t simd_hi, const float2 (&s)[L], const float (&nv)[L])
{
  const uint32_t b0 = j * L * QM;
  const uint64_t cc = static_cast<uint64_t>(a.scr[b0 / 32]) | (static_cast<uint64_t>(a.scr[b0 / 32 + 1]) << 32);
  const uint32_t cw = static_cast<uint32_t>(cc >> (b0 % 32));
#pragma unroll
  for (int v = 0; v < L; ++v) {
    const uint32_t i = j * L + v;
    int8_t         o[8];
    demap::demap_symbol(a.dm, lt, s[v], nv[v], i, i < simd_hi, o);
    const uint32_t c = cw >> (v * QM);
    uint64_t       x = 0;
#pragma unroll
    for (int k = 0; k < QM; ++k) {
      const int q = ((c >> k) & 1u) ? -o[k] : o[k];
      x |= static_cast<uint64_t>(static_cast<uint8_t>(q)) << (8 * k);
    }
    int8_t* dst = row + i * QM;
    if constexpr (QM == 8) {
      *reinterpret_cast<uint2*>(dst) = make_uint2(static_cast<uint32_t>(x), static_cast<uint32_t>(x >> 32));
    } else if constexpr (QM == 6) {
      uint16_t* d16 = reinterpret_cast<uint16_t*>(dst); // i * 6 is even
      d16[0]        = static_cast<uint16_t>(x);
      d16[1]        = static_cast<uint16_t>(x >> 16);
      d16[2]        = static_cast<uint16_t>(x >> 32);
    } else if constexpr (QM == 4) {
      *reinterpret_cast<uint32_t*>(dst) = static_cast<uint32_t>(x);
    } else if constexpr (QM == 2) {
      *reinterpret_cast<uint16_t*>(dst) = static_cast<uint16_t>(x);
    } else {
      *dst = static_cast<int8_t>(x);
    }
  }
}

// The L equalized symbols of data RE j (OFDM symbol l) of grid gi straight to LLRs.
template <int L>
__device__ __forceinline__ void emit_llrs(const pusch_eq_args& a, const float* lt, uint32_t gi, uint32_t j, uint32_t l,
                                          const float2 (&s)[L], const float (&nv)[L])
{
  if (a.eq_out != nullptr) {
#pragma unroll
    for (int v = 0; v < L; ++v) {
      a.eq_out[gi * a.eq_stride + j * L + v] = s[v];
      a.nv_out[gi * a.eq_stride + j * L + v] = nv[v];
    }
    return;
  }
  int8_t*        row     = a.llrs + static_cast<uint64_t>(gi) * a.llr_stride;
  const uint32_t simd_hi = a.simd_hi[l];
  switch (a.dm.qm) {
    case 8:
      emit_re_llrs<L, 8>(a, lt, row, j, simd_hi, s, nv);
      break;
    case 6:
      emit_re_llrs<L, 6>(a, lt, row, j, simd_hi, s, nv);
      break;
    case 4:
      emit_re_llrs<L, 4>(a, lt, row, j, simd_hi, s, nv);
      break;
    case 2:
      emit_re_llrs<L, 2>(a, lt, row, j, simd_hi, s, nv);
      break;
    default:
      emit_re_llrs<L, 1>(a, lt, row, j, simd_hi, s, nv);
      break;
  }
}

// channel_equalizer_generic_impl.cpp:304: the largest port variance (std::max_element order) of grid gi.
template <int P>
__device__ __forceinline__ void port_noise_max(const pusch_eq_args& a, uint32_t gi, float& nmax, bool& ok)
{
  const srs_amd_chest_port_stats* st = a.stats + gi * P;
  nmax                               = st[0].noise_var;
#pragma unroll
  for (int p = 1; p < P; ++p) {
    nmax = (nmax < st[p].noise_var) ? st[p].noise_var : nmax;
  }
  ok = __builtin_isnormal(nmax) && nmax >= 0.0f;
}

// Equalizes data RE j (OFDM symbol l) of grid gi from its received samples y[P] and channel coefficients
// h[P][L], then demaps and descrambles the L symbols into the grid's LLR row (no symbol round trip via HBM).
template <int P, int L, bool MMSE>
__device__ __forceinline__ void equalize_write(const pusch_eq_args& a, const float* lt, uint32_t gi, uint32_t j,
                                               uint32_t l, const eq::cplx* y, const eq::cplx* h)
{
  const srs_amd_chest_port_stats* st = a.stats + gi * P;
  float2                          so[L];
  float                           nvo[L];
  if constexpr (L == 1) {
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
    so[0]  = make_float2(s.x, s.y);
    nvo[0] = nv;
  } else {
    float nmax;
    bool  ok;
    port_noise_max<P>(a, gi, nmax, ok);
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
      so[0]  = make_float2(s.x, s.y);
      so[1]  = make_float2(s.z, s.w);
      nvo[0] = nv.x;
      nvo[1] = nv.y;
    } else {
      eq::cplx s[L];
      float    nv[L];
      eq::equalize_mimo<P, L, MMSE>(y, h, nmax, ok, 1.0f, s, nv);
#pragma unroll
      for (int v = 0; v < L; ++v) {
        so[v]  = make_float2(s[v].x, s[v].y);
        nvo[v] = nv[v];
      }
    }
  }
  emit_llrs<L>(a, lt, gi, j, l, so, nvo);
}

template <int P, int L, bool MMSE>
__global__ __launch_bounds__(256) void pusch_equalize_kernel(pusch_eq_args a)
{
  __shared__ float lt[4 * 2 * 16];
  demap::stage_interval_tables(a.dm, lt);
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

  const uint32_t* grid  = a.grids + gi * a.grid_stride + l * a.nof_subc + sc;
  const uint32_t* est   = a.estimates + gi * a.est_stride + l * a.nof_subc + sc;
  const uint32_t  plane = 14 * a.nof_subc;
  const bool      dc    = sc == a.dc_subc; // the processor's zeroed DC estimate

  eq::cplx y[P], h[P * L];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    y[p] = eq::from_cbf16(grid[static_cast<uint64_t>(p) * plane]);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      h[p * L + l] = eq::from_cbf16(dc ? 0u : est[static_cast<uint64_t>(p * L + l) * plane]);
    }
  }
  equalize_write<P, L, MMSE>(a, lt, gi, j, l, y, h);
}

// Estimator-fused form: one thread per (grid, OFDM symbol, subcarrier) rebuilds the channel coefficients of
// its data RE from the estimator's per-subcarrier values (c.freq: the one or two LSE slices the symbol
// reads) and per-port CFO phases with the expansion kernel's own operations (chest_device.h expand_pair:
// identical cbf16 estimates), so the P x L x 14 x subcarrier estimate tensor is neither written nor read.
constexpr uint32_t EQ_XCDS = 8;

template <bool MULTI>
__device__ __forceinline__ const eq_item& eq_item_of(const eq_item& own, const eq_items& m)
{
  if constexpr (MULTI) {
    const uint32_t z = m.ids != nullptr ? m.ids[blockIdx.y] : blockIdx.y;
    return m.items[z];
  } else {
    return own;
  }
}

template <int P, int L, bool MMSE, bool MULTI>
// six waves per SIMD (<= 80 VGPRs, no spills for the 4 x 4 solve) to hide the per-RE memory latency
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void pusch_equalize_fused_kernel(eq_item own, eq_items items)
{
  // batch form: the launch's argument pair; slot form: the pair of PDU ids[blockIdx.y] (one grid per PDU)
  const eq_item&       it = eq_item_of<MULTI>(own, items);
  const pusch_eq_args& a  = it.a;
  const chest_args&    c  = it.c;
  __shared__ float2 s_ph[P];
  __shared__ int    s_rot[P];
  __shared__ float  lt[4 * 2 * 16];
  // XCD-aware order: workgroups are dispatched to the 8 XCDs round-robin, so the symbols of one (grid,
  // subcarrier tile) are placed on one XCD -- its L2 then serves their common LSE slices.
  const uint32_t xcd  = blockIdx.x % EQ_XCDS, r = blockIdx.x / EQ_XCDS;
  const uint32_t tile = xcd + EQ_XCDS * (r / c.nof_symbols);
  if (tile >= a.nof_tiles) {
    return;
  }
  const uint32_t gi = tile / a.tiles_x;
  const uint32_t tx = tile % a.tiles_x;
  const uint32_t l  = c.first_symbol + r % c.nof_symbols;
  if (threadIdx.x < P) {
    const float* acc    = c.acc + (static_cast<uint64_t>(gi) * P + threadIdx.x) * CH_ACC;
    s_ph[threadIdx.x]  = chdev::cfo_phase(c, acc, l);
    s_rot[threadIdx.x] = chdev::cfo_rotates(c, acc) ? 1 : 0;
  }
  demap::stage_interval_tables(a.dm, lt); // (synchronizes)
  const uint32_t sc = a.first_subc + tx * 256 + threadIdx.x;
  const uint32_t kk = sc - 12 * c.prb_lo; // estimator allocation index (wraps below it)
  if (sc >= a.nof_subc || kk >= c.nof_re) {
    return;
  }
  const uint32_t e   = a.re_table[l * a.nof_prb + sc / 12];
  const uint32_t bit = sc % 12;
  if (((e >> bit) & 1u) == 0) {
    return;
  }
  const uint32_t  j     = (e >> 12) + __builtin_popcount(e & ((1u << bit) - 1u));
  const uint32_t* grid  = a.grids + gi * a.grid_stride + l * a.nof_subc + sc;
  const uint32_t  plane = 14 * a.nof_subc;
  const int       i0    = chdev::lse_index(c, l);
  const bool      two   = c.td != SRS_AMD_CHEST_TD_AVERAGE && c.td_interp[l];
  const bool      dc    = sc == a.dc_subc; // the processor's zeroed DC estimate (pusch_processor_impl.cpp:235-249)
  // channel coefficient of port p, layer v
  auto coef = [&](int p, int v) {
    const float2*  fr = c.freq + (((static_cast<uint64_t>(gi) * P + p) * L + v) * c.nof_lse + i0) * c.nof_re + kk;
    const float2   x0 = fr[0];
    const float2   x1 = two ? fr[c.nof_re] : x0;
    const uint32_t u  = chdev::expand_pair(c, x0, x1, l, s_rot[p] != 0, s_ph[p]);
    return eq::from_cbf16(dc ? 0u : u);
  };
  if constexpr (L >= 3 || (L == 2 && MMSE)) {
    // the normal equations built port by port as the coefficients are rebuilt (few live registers)
    eq::mimo_system<L> sys;
    eq::mimo_init(sys);
#pragma unroll
    for (int p = 0; p < P; ++p) {
      eq::cplx hp[L];
#pragma unroll
      for (int v = 0; v < L; ++v) {
        hp[v] = coef(p, v);
      }
      eq::mimo_add_port(sys, hp, eq::from_cbf16(grid[static_cast<uint64_t>(p) * plane]));
    }
    float nmax;
    bool  ok;
    port_noise_max<P>(a, gi, nmax, ok);
    eq::cplx s[L];
    float    nv[L];
    eq::mimo_solve<L, MMSE>(sys, nmax, ok, 1.0f, s, nv);
    float2 so[L];
#pragma unroll
    for (int v = 0; v < L; ++v) {
      so[v] = make_float2(s[v].x, s[v].y);
    }
    emit_llrs<L>(a, lt, gi, j, l, so, nv);
  } else {
    eq::cplx y[P], h[P * L];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      y[p] = eq::from_cbf16(grid[static_cast<uint64_t>(p) * plane]);
#pragma unroll
      for (int v = 0; v < L; ++v) {
        h[p * L + v] = coef(p, v);
      }
    }
    equalize_write<P, L, MMSE>(a, lt, gi, j, l, y, h);
  }
}

// One thread per (grid, estimate plane, OFDM symbol of the allocation): the DC subcarrier's estimate set to zero.
__global__ __launch_bounds__(256) void pusch_dc_zero_kernel(uint32_t* est, uint64_t est_stride, uint32_t nof_planes,
                                                            uint32_t nof_subc, uint32_t first_symbol,
                                                            uint32_t nof_symbols, uint32_t dc, uint32_t total)
{
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total) {
    return;
  }
  const uint32_t l  = first_symbol + t % nof_symbols;
  const uint32_t pl = (t / nof_symbols) % nof_planes;
  const uint32_t g  = t / (nof_symbols * nof_planes);
  est[g * est_stride + (static_cast<uint64_t>(pl) * 14 + l) * nof_subc + dc] = 0u;
}

} // namespace

hipError_t launch_pusch_dc_zero(uint32_t* estimates, uint64_t est_stride, uint32_t nof_planes, uint32_t nof_subc,
                                uint32_t first_symbol, uint32_t nof_symbols, uint32_t dc_subc, uint32_t nof_grids,
                                hipStream_t stream)
{
  const uint32_t total = nof_grids * nof_planes * nof_symbols;
  if (total == 0 || dc_subc >= nof_subc || first_symbol + nof_symbols > 14) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pusch_dc_zero_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, estimates, est_stride,
                     nof_planes, nof_subc, first_symbol, nof_symbols, dc_subc, total);
  return hipGetLastError();
}

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

bool pusch_equalize_fusable(uint32_t nof_ports, uint32_t nof_layers, bool mmse, uint32_t nof_lse)
{
  (void)mmse;
  return nof_lse >= 1 && nof_lse <= CH_MAXDMRS && nof_layers >= 1 && nof_layers <= 4 && nof_layers <= nof_ports &&
         (nof_ports == 1 || nof_ports == 2 || nof_ports == 4) && !(nof_layers == 3 && nof_ports != 4);
}

uint32_t pusch_equalize_fused_blocks(uint32_t nof_symbols, uint32_t nof_tiles)
{
  return EQ_XCDS * nof_symbols * ((nof_tiles + EQ_XCDS - 1) / EQ_XCDS);
}

hipError_t launch_pusch_equalize_fused(const pusch_eq_args& a, const chest_args& c, uint32_t nof_ports,
                                       uint32_t nof_layers, bool mmse, uint32_t span_subc, uint32_t nof_grids,
                                       hipStream_t stream)
{
  if (span_subc == 0 || nof_grids == 0 || c.nof_symbols == 0) {
    return hipSuccess;
  }
  pusch_eq_args ax = a;
  ax.tiles_x       = (span_subc + 255) / 256;
  ax.nof_tiles     = ax.tiles_x * nof_grids;
  const dim3 grid(pusch_equalize_fused_blocks(c.nof_symbols, ax.nof_tiles));
#define SRS_EQF_CASE(PP, LL, MM)                                                                                      \
  if (nof_ports == PP && nof_layers == LL && mmse == MM) {                                                            \
    SRS_PROBED_LAUNCH(SRS_AMD_PROBE_EQUALIZER, (pusch_equalize_fused_kernel<PP, LL, MM, false>), grid, dim3(256), 0, \
                      stream, eq_item{ax, c}, eq_items{});                                                            \
    return hipGetLastError();                                                                                         \
  }
  SRS_EQF_CASE(1, 1, false)
  SRS_EQF_CASE(2, 1, false)
  SRS_EQF_CASE(4, 1, false)
  SRS_EQF_CASE(2, 2, false)
  SRS_EQF_CASE(4, 2, false)
  SRS_EQF_CASE(4, 3, false)
  SRS_EQF_CASE(4, 4, false)
  SRS_EQF_CASE(2, 2, true)
  SRS_EQF_CASE(4, 2, true)
  SRS_EQF_CASE(4, 3, true)
  SRS_EQF_CASE(4, 4, true)
#undef SRS_EQF_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_pusch_equalize_fused_items(const eq_items& items, uint32_t count, uint32_t nof_ports,
                                             uint32_t nof_layers, bool mmse, uint32_t max_blocks, hipStream_t stream)
{
  if (count == 0 || max_blocks == 0) {
    return hipSuccess;
  }
  const dim3    grid(max_blocks, count);
  const eq_item none{};
#define SRS_EQF_CASE(PP, LL, MM)                                                                                      \
  if (nof_ports == PP && nof_layers == LL && mmse == MM) {                                                            \
    SRS_PROBED_LAUNCH(SRS_AMD_PROBE_EQUALIZER, (pusch_equalize_fused_kernel<PP, LL, MM, true>), grid, dim3(256), 0,  \
                      stream, none, items);                                                                           \
    return hipGetLastError();                                                                                         \
  }
  SRS_EQF_CASE(1, 1, false)
  SRS_EQF_CASE(2, 1, false)
  SRS_EQF_CASE(4, 1, false)
  SRS_EQF_CASE(2, 2, false)
  SRS_EQF_CASE(4, 2, false)
  SRS_EQF_CASE(4, 3, false)
  SRS_EQF_CASE(4, 4, false)
  SRS_EQF_CASE(2, 2, true)
  SRS_EQF_CASE(4, 2, true)
  SRS_EQF_CASE(4, 3, true)
  SRS_EQF_CASE(4, 4, true)
#undef SRS_EQF_CASE
  return hipErrorInvalidValue;
}

} // namespace srs_amd
