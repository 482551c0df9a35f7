// uci_decoder.hip -- MI355X UCI decoder kernels (include/srsran_amd/uci_decoder.h).
//
// uci_short_kernel: one wavefront per message of 1-11 bits (short_block_detector_impl.cpp:160-223): the
// non-zero LLR count check, rate dematching to T = Qm / 3 Qm / 32 soft bits by saturated sums (the AVX2
// log_likelihood_ratio::sum: clamp to +-120, log_likelihood_ratio.cpp:432-445), then ML detection -- 1 bit by
// sign, 2 bits over the four (c0, c1, c0 ^ c1) codewords, 3-11 bits over the 2^(K-1) even-message (32, K)
// Reed-Muller codewords (the odd ones are their complements: negative correlation), each lane correlating a
// stride of codewords and the wave reducing (largest |metric|, lowest index as the reference's sequential scan)
// -- and the GLRT metric against the reference's thresholds, in double as the reference.
// uci_polar_finish_kernel: one thread per message: the CRC6 / CRC11 remainder of each decoded polar codeblock
// (bit-serial, the generator of TS 38.212 5.1), status, filler removal (uci_decoder_impl.cpp:47-111).
#include <hip/hip_runtime.h>

#include "uci_args.h"

namespace srs_amd {
namespace {

// TS 38.212 Table 5.3.3.3-1: basis sequence M_{i,n} of the (32, K) code, bit i of word n.
__constant__ uint32_t RM_BASIS[11] = {0xffffffffu, 0x4ba5a933u, 0x7d910e5au, 0x6d26339cu, 0x71c7c3e0u, 0x7e0ffc00u,
                                      0x731d8e64u, 0x6b44f5b0u, 0x7dc218ecu, 0x4da1b746u, 0x42f0ffffu};
// short_block_detector_impl.cpp: min_small_block_rm_size (uci_info.h:85) and the GLRT thresholds (:219)
__constant__ uint32_t MIN_RM_BITS[11] = {2, 3, 9, 10, 11, 12, 13, 14, 14, 15, 17};
__constant__ double   THRESHOLDS[11]  = {0, 0, 12, 14, 16, 18, 20, 22, 24, 26, 29};

constexpr int LLR_MAX = 120;

__device__ __forceinline__ int wave_sum(int v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v += __shfl_xor(v, o, 64);
  }
  return v;
}

// MULTI: one argument block per message (items[blockIdx.x], row 0), the slot form of the PUSCH processor
template <bool MULTI>
__global__ __launch_bounds__(64) void uci_short_kernel(uci_short_args own, const uci_short_args* items)
{
  const uci_short_args& a = MULTI ? items[blockIdx.x] : own;
  __shared__ int tmp[32];
  if (MULTI && a.pred != nullptr && *a.pred != a.pred_val) {
    return;
  }
  const uint32_t row  = MULTI ? 0u : blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const int8_t*  in   = a.llrs + row * a.llr_stride;
  uint8_t*       msg  = a.msgs + row * a.msg_stride;
  int32_t*       st   = reinterpret_cast<int32_t*>(reinterpret_cast<uint8_t*>(a.status) + row * a.status_stride);
  const uint32_t K    = a.K;

  // validate_spans: enough non-zero soft bits
  int nz = 0;
  for (uint32_t i = lane; i < a.E; i += 64) {
    nz += in[i] != 0 ? 1 : 0;
  }
  nz = wave_sum(nz);
  if (static_cast<uint32_t>(nz) < MIN_RM_BITS[K - 1] || (K <= 2 && a.E < a.qm)) {
    if (lane < K) {
      msg[lane] = 1;
    }
    if (lane == 0) {
      *st = 2; // invalid
    }
    return;
  }
  // rate dematching to T soft bits
  const uint32_t T = K == 1 ? a.qm : (K == 2 ? 3 * a.qm : 32u);
  if (lane < T) {
    int acc = lane < a.E ? in[lane] : 0;
    for (uint32_t j = lane + T; j < a.E; j += T) {
      acc = min(max(acc + in[j], -LLR_MAX), LLR_MAX);
    }
    tmp[lane] = acc;
  }
  __syncthreads();
  if (K == 1) {
    if (lane == 0) {
      msg[0] = tmp[0] > 0 ? 0 : 1;
      *st    = 1; // metric 1 > threshold 0
    }
    return;
  }
  if (K == 2) {
    if (lane != 0) {
      return;
    }
    int l[3];
    if (T == 3) {
      l[0] = tmp[0], l[1] = tmp[1], l[2] = tmp[2];
    } else {
      const uint32_t step = T / 3 - 2;
      l[0]                = tmp[0] + tmp[step + 3];
      l[1]                = tmp[1] + tmp[2 * step + 4];
      l[2]                = tmp[step + 2] + tmp[2 * step + 5];
    }
    const int tab[4][3] = {{1, 1, 1}, {-1, 1, -1}, {1, -1, -1}, {-1, -1, 1}};
    uint32_t  best      = 0;
    double    best_m    = 2.2250738585072014e-308; // std::numeric_limits<double>::min()
    for (uint32_t c = 0; c < 4; ++c) {
      const int m = l[0] * tab[c][0] + l[1] * tab[c][1] + l[2] * tab[c][2];
      if (m > best_m) {
        best_m = m;
        best   = c;
      }
    }
    msg[0]           = best & 1u;
    msg[1]           = (best >> 1) & 1u;
    best_m           = best_m * best_m;
    const int norm   = l[0] * l[0] + l[1] * l[1] + l[2] * l[2];
    const double glr = 2.0 * best_m / (3.0 * norm - best_m);
    *st              = glr > THRESHOLDS[1] ? 1 : 2;
    return;
  }
  // 3 .. 11 bits: correlate the 2^(K-1) even-message codewords
  const uint32_t ncw = 1u << (K - 1);
  int            x[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    x[i] = tmp[i];
  }
  int      best_abs = 0, best_m = 0;
  uint32_t best     = 0xffffffffu;
  for (uint32_t c = lane; c < ncw; c += 64) {
    uint32_t cw = 0;
    for (uint32_t b = 0; b + 1 < K; ++b) {
      cw ^= ((c >> b) & 1u) ? RM_BASIS[b + 1] : 0u;
    }
    int m = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      m += ((cw >> i) & 1u) ? -x[i] : x[i];
    }
    const int am = m < 0 ? -m : m;
    if (am > best_abs) { // strictly larger: the lowest index wins ties, as the sequential scan
      best_abs = am;
      best_m   = m;
      best     = c;
    }
  }
  // wave argmax: larger |metric|, then lower index
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int      oa = __shfl_xor(best_abs, o, 64);
    const int      om = __shfl_xor(best_m, o, 64);
    const uint32_t oi = __shfl_xor(best, o, 64);
    if (oa > best_abs || (oa == best_abs && oi < best)) {
      best_abs = oa;
      best_m   = om;
      best     = oi;
    }
  }
  if (best == 0xffffffffu || best_abs == 0) { // no positive correlation: the reference keeps index 0, bit0 0
    best   = 0;
    best_m = 0;
  }
  const uint32_t value = 2 * best + (best_m < 0 ? 1u : 0u);
  if (lane < K) {
    msg[lane] = (value >> lane) & 1u;
  }
  if (lane == 0) {
    int norm = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      norm += x[i] * x[i];
    }
    double m = best_abs > 0 ? static_cast<double>(best_abs) : 2.2250738585072014e-308;
    m        = m * m;
    // (MAX_BLOCK_LENGTH - 1) * m / (MAX_BLOCK_LENGTH * norm - m), the product 32 * norm in unsigned arithmetic
    const double glr = 31.0 * m / (static_cast<double>(32u * static_cast<uint32_t>(norm)) - m);
    *st              = glr > THRESHOLDS[K - 1] ? 1 : 2;
  }
}

__device__ bool crc_ok(const uint8_t* bits, uint32_t n, uint32_t L)
{
  const uint32_t poly = L == 6 ? 0x21u : 0x621u; // CRC6: D^6 + D^5 + 1, CRC11: D^11 + D^10 + D^9 + D^5 + 1
  const uint32_t top  = 1u << (L - 1);
  const uint32_t mask = (1u << L) - 1u;
  uint32_t       crc  = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t fb = ((crc & top) != 0) ^ (bits[i] & 1u);
    crc               = (crc << 1) & mask;
    crc ^= fb ? poly : 0u;
  }
  return crc == 0;
}

template <bool MULTI>
__global__ __launch_bounds__(64) void uci_polar_finish_kernel(uci_polar_args own, const uci_polar_args* items,
                                                              uint32_t nof)
{
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= nof) {
    return;
  }
  const uci_polar_args& a   = MULTI ? items[i] : own;
  const uint32_t        row = MULTI ? 0u : i;
  if (MULTI && a.pred != nullptr && *a.pred != a.pred_val) {
    return;
  }
  const uint8_t* cb0 = a.cbs + static_cast<uint64_t>(row) * a.C * a.cb_stride;
  uint8_t*       msg = a.msgs + row * a.msg_stride;
  int32_t* st = reinterpret_cast<int32_t*>(reinterpret_cast<uint8_t*>(a.status) + row * a.status_stride);
  const uint32_t K0 = a.A0 + a.F0 + a.L;
  bool           ok = crc_ok(cb0, K0, a.L);
  for (uint32_t i = 0; i < a.A0; ++i) {
    msg[i] = cb0[a.F0 + i];
  }
  if (a.C > 1) {
    // uci_decoder_impl.cpp:64-76: the second codeblock is decoded only after a valid first one; otherwise its
    // payload bits are left as the caller's (zero-initialised) buffer holds them -- zero here
    const uint8_t* cb1 = cb0 + a.cb_stride;
    const bool     use = ok;
    ok                 = ok && crc_ok(cb1, a.A1 + a.L, a.L);
    for (uint32_t i = 0; i < a.A1; ++i) {
      msg[a.A0 + i] = use ? cb1[i] : uint8_t(0);
    }
  }
  *st = ok ? 1 : 2;
}

} // namespace

hipError_t launch_uci_short(const uci_short_args& a, uint32_t nof, hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(uci_short_kernel<false>, dim3(nof), dim3(64), 0, stream, a, nullptr);
  return hipGetLastError();
}

hipError_t launch_uci_polar_finish(const uci_polar_args& a, uint32_t nof, hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(uci_polar_finish_kernel<false>, dim3((nof + 63) / 64), dim3(64), 0, stream, a, nullptr, nof);
  return hipGetLastError();
}

hipError_t launch_uci_short_items(const uci_short_args* items, uint32_t n, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(uci_short_kernel<true>, dim3(n), dim3(64), 0, stream, uci_short_args{}, items);
  return hipGetLastError();
}

hipError_t launch_uci_polar_finish_items(const uci_polar_args* items, uint32_t n, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(uci_polar_finish_kernel<true>, dim3((n + 63) / 64), dim3(64), 0, stream, uci_polar_args{},
                     items, n);
  return hipGetLastError();
}

} // namespace srs_amd
