// transform_precoding.hip -- MI355X transform deprecoder (DFT-s-OFDM PUSCH): the inverse M-point DFT of
// every data OFDM symbol, M = 12 M_rb with M_rb = 2^a 3^b 5^c (transform_precoder_dft_impl.cpp:31-56), and
// the per-symbol noise-variance mean (:58-84).
//
// One workgroup per OFDM symbol.  M is not a power of two, so instead of a radix pipeline the DFT is the
// two-factor (four-step) decomposition M = M1 M2 with M1 ~ sqrt(M), both passes direct sums in LDS:
//   A[n2][k1] = W_M^(n2 k1) sum_n1 x[M2 n1 + n2] W_M1^(n1 k1)
//   X[k1 + M1 k2] = sum_n2 A[n2][k1] W_M2^(n2 k2)
// with W_N = exp(+j 2 pi / N) (inverse DFT), every twiddle read from one table of the M roots of unity.
// M (M1 + M2) complex MACs per symbol -- 0.37 M for the largest symbol, M = 3240 -- against M^2 for the
// direct sum; the symbol and the intermediate (2 x 26 KiB) stay in LDS with the M1- and M2-point roots of
// unity, and the M-point twiddle of each intermediate is computed once (sincospi).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "transform_precoding_args.h"

namespace srs_amd {

constexpr int TP_THREADS = 256;

namespace {

__device__ __forceinline__ float2 cmac(float2 acc, float2 a, float2 w)
{
  acc.x = fmaf(a.x, w.x, fmaf(-a.y, w.y, acc.x));
  acc.y = fmaf(a.x, w.y, fmaf(a.y, w.x, acc.y));
  return acc;
}

__device__ __forceinline__ bool valid_nv(float v)
{
  return v > 0.0f && !isnan(v) && !isinf(v);
}

} // namespace

// MULTI: one argument block per PDU (items[blockIdx.y], its own M), the PUSCH processor's slot form
template <bool MULTI>
__global__ __launch_bounds__(TP_THREADS) void transform_deprecode_kernel(tp_args own, const tp_args* items)
{
  const tp_args& a = MULTI ? items[blockIdx.y] : own;
  extern __shared__ float2 lds[];
  const uint32_t M = a.M, M1 = a.M1, M2 = a.M2;
  float2*        x  = lds;     // [M] input symbol
  float2*        A  = x + M;   // [M2][M1] first pass
  float2*        t1 = A + M;   // [M1] exp(+j 2 pi i / M1)
  float2*        t2 = t1 + M1; // [M2] exp(+j 2 pi i / M2)
  for (uint32_t i = threadIdx.x; i < M1 + M2; i += TP_THREADS) {
    const uint32_t n = i < M1 ? M1 : M2, k = i < M1 ? i : i - M1;
    float          s, c;
    sincospif(2.0f * static_cast<float>(k) / static_cast<float>(n), &s, &c);
    t1[i] = make_float2(c, s);
  }
  for (uint32_t row = blockIdx.x; row < a.nof_rows; row += gridDim.x) {
    float2* sym = a.symbols + row * a.sym_stride;
    for (uint32_t i = threadIdx.x; i < M; i += TP_THREADS) {
      x[i] = sym[i];
    }
    __syncthreads();
    // first pass: one (n2, k1) pair per thread iteration
    for (uint32_t i = threadIdx.x; i < M; i += TP_THREADS) {
      const uint32_t n2 = i / M1, k1 = i - n2 * M1;
      float2         acc = make_float2(0.0f, 0.0f);
      uint32_t       t   = 0; // n1 k1 mod M1
      for (uint32_t n1 = 0; n1 < M1; ++n1) {
        acc = cmac(acc, x[M2 * n1 + n2], t1[t]);
        t += k1;
        t = t >= M1 ? t - M1 : t;
      }
      float s, c;
      sincospif(2.0f * static_cast<float>((n2 * k1) % M) / static_cast<float>(M), &s, &c);
      A[i] = make_float2(acc.x * c - acc.y * s, acc.x * s + acc.y * c);
    }
    __syncthreads();
    // second pass: output X[k1 + M1 k2]
    for (uint32_t i = threadIdx.x; i < M; i += TP_THREADS) {
      const uint32_t k2 = i / M1, k1 = i - k2 * M1;
      float2         acc = make_float2(0.0f, 0.0f);
      uint32_t       t   = 0; // n2 k2 mod M2
      for (uint32_t n2 = 0; n2 < M2; ++n2) {
        acc = cmac(acc, A[n2 * M1 + k1], t2[t]);
        t += k2;
        t = t >= M2 ? t - M2 : t;
      }
      sym[i] = make_float2(acc.x * a.scale, acc.y * a.scale);
    }
    if (a.noise != nullptr) {
      // mean of the valid noise variances of the symbol; the valid ones replaced by it
      __shared__ float    s_sum[TP_THREADS / 64];
      __shared__ uint32_t s_cnt[TP_THREADS / 64];
      float*              nv  = a.noise + row * a.nv_stride;
      float               sum = 0.0f;
      uint32_t            cnt = 0;
      for (uint32_t i = threadIdx.x; i < M; i += TP_THREADS) {
        const float v = nv[i];
        if (valid_nv(v)) {
          sum += v;
          ++cnt;
        }
      }
      for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        cnt += __shfl_xor(cnt, o);
      }
      if ((threadIdx.x & 63) == 0) {
        s_sum[threadIdx.x / 64] = sum;
        s_cnt[threadIdx.x / 64] = cnt;
      }
      __syncthreads();
      float    tot = 0.0f;
      uint32_t n   = 0;
      for (int w = 0; w < TP_THREADS / 64; ++w) {
        tot += s_sum[w];
        n += s_cnt[w];
      }
      const float mean = n != 0 ? tot / static_cast<float>(n) : 0.0f;
      for (uint32_t i = threadIdx.x; i < M; i += TP_THREADS) {
        const float v = nv[i];
        nv[i]         = valid_nv(v) ? mean : v;
      }
    }
    __syncthreads(); // LDS reused by the next row
  }
}

hipError_t launch_transform_deprecode(const tp_args& a, hipStream_t stream)
{
  if (a.nof_rows == 0) {
    return hipSuccess;
  }
  const uint32_t grid = a.nof_rows < 65535u ? a.nof_rows : 65535u;
  const size_t   lds  = (2 * a.M + a.M1 + a.M2) * sizeof(float2); // <= 53 KiB (M <= 3300)
  hipLaunchKernelGGL(transform_deprecode_kernel<false>, dim3(grid), dim3(TP_THREADS), lds, stream, a, nullptr);
  return hipGetLastError();
}

hipError_t launch_transform_deprecode_items(const tp_args* items, uint32_t n, uint32_t max_rows, size_t lds_bytes,
                                            hipStream_t stream)
{
  if (n == 0 || max_rows == 0) {
    return hipSuccess;
  }
  const uint32_t grid = max_rows < 65535u ? max_rows : 65535u;
  hipLaunchKernelGGL(transform_deprecode_kernel<true>, dim3(grid, n), dim3(TP_THREADS), lds_bytes, stream, tp_args{},
                     items);
  return hipGetLastError();
}

} // namespace srs_amd
