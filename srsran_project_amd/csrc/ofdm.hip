// ofdm.hip -- MI355X OFDM modulator / demodulator and batched DFT processor.
//
// Reference behaviour (per OFDM symbol):
//   lib/phy/lower/modulation/ofdm_modulator_impl.cpp:56-106
//     DFT input = [grid[rg/2 .. rg) | zeros | grid[0 .. rg/2)], inverse DFT (no
//     normalisation), times phase_compensation * scale, then the last cp_len
//     samples are copied in front (cyclic prefix).
//   lib/phy/lower/modulation/ofdm_demodulator_impl.cpp:95-145
//     DFT of the N samples after cp_len - window_offset, times
//     phase_compensation * scale, times exp(i*omega*k) when window_offset != 0,
//     grid[0 .. rg/2) = Y[N - rg/2 ..), grid[rg/2 .. rg) = Y[0 .. rg/2);
//     the grid stores complex bfloat16 (round half to even, bf16.h:39).
// One workgroup per (slot, port, symbol); the whole symbol is one Stockham
// FFT in registers + LDS (dft_engine.h) with the mapping, scaling, CP and bf16
// conversion fused into its first and last passes: every byte crosses HBM
// once.  Algorithmic traffic per symbol: modulation 4*rg (cbf16 grid) +
// 8*(N + cp) (samples) bytes, demodulation 8*N + 4*rg bytes.
#include <hip/hip_runtime.h>

#include "bf16_device.h"

#include "dft_engine.h"
#include "ofdm_args.h"
#include "kernel_probe.h"
#include "srsran_amd/profiling.h"

namespace srs_amd {

using dft::cf;

#ifndef OFDM_NONTEMPORAL_DEFAULT
#define OFDM_NONTEMPORAL_DEFAULT 1
#endif
constexpr bool OFDM_NONTEMPORAL = OFDM_NONTEMPORAL_DEFAULT;

namespace {

__device__ __forceinline__ cf from_cbf16(uint32_t u)
{
  return {__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}

// to_bf16 (bf16.h:39): round half to even on the 16 discarded bits.
__device__ __forceinline__ uint32_t bf16_bits(float f)
{
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

// Streaming (non-temporal) stores for the outputs and loads for the
// demodulator's baseband input: every sample is touched exactly once, so
// keeping it out of the caches measured +40 % (modulator) / +5 % (demodulator);
// non-temporal grid loads in the modulator measured slower and are not used.
template <class T>
__device__ __forceinline__ void stream_store(T* p, T v)
{
  if constexpr (OFDM_NONTEMPORAL) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// a complex sample as ONE 8-byte access (global_store_dwordx2 / global_load_dwordx2): two 4-byte accesses per
// sample issue twice the memory instructions, each with every other dword of its lanes' span
__device__ __forceinline__ void stream_store(cf* p, cf v)
{
  stream_store(reinterpret_cast<uint64_t*>(p), __builtin_bit_cast(uint64_t, v));
}

#ifndef OFDM_NT_LOADS
#define OFDM_NT_LOADS 1
#endif
template <class T>
__device__ __forceinline__ T stream_load(const T* p)
{
  if constexpr (OFDM_NT_LOADS) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

__device__ __forceinline__ cf stream_load(const cf* p)
{
  return __builtin_bit_cast(cf, stream_load(reinterpret_cast<const uint64_t*>(p)));
}

__device__ __forceinline__ uint32_t to_cbf16(cf v)
{
  return cbf16_pack(v.x, v.y); // == bf16_bits(v.x) | bf16_bits(v.y) << 16 (bf16_device.h)
}

template <int N>
__global__ __launch_bounds__(dft::plan<N>::T) void ofdm_modulate_kernel(ofdm_args a)
{
  __shared__ cf lds[dft::lds_complex<N>()];
  const uint32_t sym  = blockIdx.x % a.nsymb;
  const uint32_t item = blockIdx.x / a.nsymb;
  const uint32_t slot = (a.first_slot + item / a.nof_ports) % a.slots_per_subframe;
  const ofdm_symbol_info si = a.symbols[slot * a.nsymb + sym];
  const uint32_t* grid = static_cast<const uint32_t*>(a.in) + (static_cast<size_t>(item) * a.nsymb + sym) * a.rg_size;
  cf*             out  = static_cast<cf*>(a.out) + static_cast<size_t>(item) * a.sample_stride + si.offset;
  const int       half = static_cast<int>(a.rg_size / 2);
  const int       cp   = static_cast<int>(si.cp_len);
  const cf        coef = {si.coef_re, si.coef_im};

  auto load = [&](int i) -> cf {
    if (i < half) {
      return from_cbf16(grid[half + i]);
    }
    if (i >= N - half) {
      return from_cbf16(grid[i - (N - half)]);
    }
    return cf{0.0f, 0.0f};
  };
  auto store = [&](int n, cf v) {
    v          = dft::cmul(v, coef);
    stream_store(out + cp + n, v);
    if (n >= N - cp) {
      stream_store(out + n - (N - cp), v);
    }
  };
  dft::plan<N>::template engine<+1>::run(lds, reinterpret_cast<const cf*>(a.twiddles), load, store);
}

template <int N>
__global__ __launch_bounds__(dft::plan<N>::T) void ofdm_demodulate_kernel(ofdm_args a)
{
  __shared__ cf lds[dft::lds_complex<N>()];
  const cf*        in;
  uint32_t*        grid;
  ofdm_symbol_info si;
  if (a.items != nullptr) {
    // a staged symbol: its own symbol index and grid row (workgroup-uniform)
    const uint32_t s   = a.items[2 * blockIdx.x];
    const uint32_t row = a.items[2 * blockIdx.x + 1];
    if (s >= a.nof_symbol_infos) {
      return;
    }
    si   = a.symbols[s];
    in   = static_cast<const cf*>(a.in) + static_cast<size_t>(blockIdx.x) * a.sample_stride + si.cp_len -
           a.window_offset;
    grid = static_cast<uint32_t*>(a.out) + row;
  } else {
    const uint32_t sym  = blockIdx.x % a.nsymb;
    const uint32_t item = blockIdx.x / a.nsymb;
    const uint32_t slot = (a.first_slot + item / a.nof_ports) % a.slots_per_subframe;
    si   = a.symbols[slot * a.nsymb + sym];
    in   = static_cast<const cf*>(a.in) + static_cast<size_t>(item) * a.sample_stride + si.offset + si.cp_len -
           a.window_offset;
    grid = static_cast<uint32_t*>(a.out) + (static_cast<size_t>(item) * a.nsymb + sym) * a.rg_size;
  }
  const int       half = static_cast<int>(a.rg_size / 2);
  const cf        coef = {si.coef_re, si.coef_im};
  const cf*       win  = reinterpret_cast<const cf*>(a.window);

  auto load  = [&](int i) -> cf { return stream_load(in + i); };
  auto store = [&](int k, cf v) {
    if (k >= half && k < N - half) {
      return; // guard band
    }
    v = dft::cmul(v, coef);
    if (win != nullptr) {
      v = dft::cmul(v, win[k]);
    }
    stream_store(grid + (k < half ? k + half : k - (N - half)), to_cbf16(v));
  };
  dft::plan<N>::template engine<-1>::run(lds, reinterpret_cast<const cf*>(a.twiddles), load, store);
}

template <int N, int S>
__global__ __launch_bounds__(dft::plan<N>::T) void dft_kernel(dft_args a)
{
  __shared__ cf lds[dft::lds_complex<N>()];
  const cf* in  = reinterpret_cast<const cf*>(a.in) + static_cast<size_t>(blockIdx.x) * N;
  cf*       out = reinterpret_cast<cf*>(a.out) + static_cast<size_t>(blockIdx.x) * N;
  auto      load  = [&](int i) -> cf { return in[i]; };
  auto      store = [&](int k, cf v) { out[k] = v; };
  dft::plan<N>::template engine<S>::run(lds, reinterpret_cast<const cf*>(a.twiddles), load, store);
}

constexpr uint32_t MAX_GRID_X = 0x7fffffffu;

} // namespace

bool ofdm_size_supported(uint32_t N)
{
#define SRS_CASE(NN)                                                                                                   \
  if (N == NN)                                                                                                         \
    return true;
  SRS_DFT_FOR_EACH_SIZE(SRS_CASE)
#undef SRS_CASE
  return false;
}

hipError_t launch_ofdm_modulate(const ofdm_args& a, uint32_t N, hipStream_t stream)
{
  const uint64_t blocks = static_cast<uint64_t>(a.nof_items) * a.nsymb;
  if (blocks == 0) {
    return hipSuccess;
  }
  if (blocks > MAX_GRID_X) {
    return hipErrorInvalidValue;
  }
#define SRS_CASE(NN)                                                                                                   \
  if (N == NN) {                                                                                                       \
    SRS_PROBED_LAUNCH(SRS_AMD_PROBE_OFDM_MOD, ofdm_modulate_kernel<NN>, dim3(blocks), dim3(dft::plan<NN>::T), 0,     \
                      stream, a);                                                                                     \
    return hipGetLastError();                                                                                          \
  }
  SRS_DFT_FOR_EACH_SIZE(SRS_CASE)
#undef SRS_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_ofdm_demodulate(const ofdm_args& a, uint32_t N, hipStream_t stream)
{
  const uint64_t blocks = static_cast<uint64_t>(a.nof_items) * a.nsymb;
  if (blocks == 0) {
    return hipSuccess;
  }
  if (blocks > MAX_GRID_X) {
    return hipErrorInvalidValue;
  }
#define SRS_CASE(NN)                                                                                                   \
  if (N == NN) {                                                                                                       \
    SRS_PROBED_LAUNCH(SRS_AMD_PROBE_OFDM_DEMOD, ofdm_demodulate_kernel<NN>, dim3(blocks), dim3(dft::plan<NN>::T), 0, \
                      stream, a);                                                                                     \
    return hipGetLastError();                                                                                          \
  }
  SRS_DFT_FOR_EACH_SIZE(SRS_CASE)
#undef SRS_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_dft(const dft_args& a, uint32_t N, int inverse, hipStream_t stream)
{
  if (a.nof == 0) {
    return hipSuccess;
  }
#define SRS_CASE(NN)                                                                                                   \
  if (N == NN) {                                                                                                       \
    if (inverse) {                                                                                                     \
      hipLaunchKernelGGL((dft_kernel<NN, +1>), dim3(a.nof), dim3(dft::plan<NN>::T), 0, stream, a);                   \
    } else {                                                                                                           \
      hipLaunchKernelGGL((dft_kernel<NN, -1>), dim3(a.nof), dim3(dft::plan<NN>::T), 0, stream, a);                   \
    }                                                                                                                  \
    return hipGetLastError();                                                                                          \
  }
  SRS_DFT_FOR_EACH_SIZE(SRS_CASE)
#undef SRS_CASE
  return hipErrorInvalidValue;
}

} // namespace srs_amd
