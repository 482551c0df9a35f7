// pucch.hip -- MI355X PUCCH Format 0 detector (include/srsran_amd/pucch.h), after pucch_detector_format0.cpp:124-246.
//
// One 64-thread workgroup per PDU: the received REs of every symbol and port into LDS (12 per symbol and port, the
// second hop's PRB for symbol 1), the EPRE, then one thread per candidate cyclic shift: per symbol and port the
// average power, the correlation with the shift's low-PAPR sequence (sum of rx conj(seq)), |corr|^2 / 12 into the
// correlation sum and 12 power - |corr|^2 / 12 into the noise sum, the metric corr / max(noise, 1e-6); thread 0
// keeps the first largest metric in table order, compares it with the threshold and writes the message and the
// SINR / RSRP / EPRE in dB.
#include <hip/hip_runtime.h>

#include "pucch_args.h"

namespace srs_amd {
namespace {

__device__ __forceinline__ float2 from_cbf16(uint32_t u)
{
  return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
}

__device__ __forceinline__ float to_dB(float x) // convert_power_to_dB (math_utils.h)
{
  return 10.0f * log10f(x);
}

__global__ __launch_bounds__(64) void pucch_f0_kernel(const pucch_f0_desc* desc, srs_amd_pucch_f0_result* results)
{
  const pucch_f0_desc& d = desc[blockIdx.x];
  __shared__ float2    re[2][4][12];
  __shared__ float     s_metric[PUCCH_F0_MAX_CAND], s_corr[PUCCH_F0_MAX_CAND];
  const uint32_t       t = threadIdx.x;
  for (uint32_t i = t; i < d.nsym * d.nof_ports * 12; i += 64) {
    const uint32_t l = i / (d.nof_ports * 12), p = (i / 12) % d.nof_ports, k = i % 12;
    re[l][p][k] = from_cbf16(d.grid[static_cast<uint64_t>(d.ports[p]) * d.port_stride +
                                    static_cast<uint64_t>(d.l0 + l) * d.nof_subc + d.subc0[l] + k]);
  }
  __syncthreads();
  // average_power of each (symbol, port) row
  auto power = [&](uint32_t l, uint32_t p) {
    float s = 0.0f;
    for (uint32_t k = 0; k != 12; ++k) {
      s += re[l][p][k].x * re[l][p][k].x + re[l][p][k].y * re[l][p][k].y;
    }
    return s / 12.0f;
  };
  if (t < d.nof_cand) {
    float sum_corr = 0.0f, sum_noise = 0.0f;
    for (uint32_t l = 0; l != d.nsym; ++l) {
      for (uint32_t p = 0; p != d.nof_ports; ++p) {
        float2 c = make_float2(0.0f, 0.0f);
        for (uint32_t k = 0; k != 12; ++k) { // rx conj(seq)
          const float2 x = re[l][p][k], y = d.seq[t][l][k];
          c.x += x.x * y.x + x.y * y.y;
          c.y += x.y * y.x - x.x * y.y;
        }
        const float contrib = (c.x * c.x + c.y * c.y) / 12.0f;
        sum_corr += contrib;
        sum_noise += power(l, p) * 12.0f - contrib;
      }
    }
    float metric = 0.0f;
    if (!isnan(sum_noise) && !isinf(sum_noise)) {
      metric = sum_corr / fmaxf(sum_noise, 1e-6f);
    }
    s_metric[t] = metric;
    s_corr[t]   = sum_corr;
  }
  __syncthreads();
  if (t == 0) {
    float epre = 0.0f;
    for (uint32_t l = 0; l != d.nsym; ++l) {
      for (uint32_t p = 0; p != d.nof_ports; ++p) {
        epre += power(l, p);
      }
    }
    epre /= static_cast<float>(d.nsym * d.nof_ports);
    int   best        = -1;
    float best_metric = 0.0f, best_rsrp = 0.0f;
    for (uint32_t c = 0; c != d.nof_cand; ++c) {
      if (s_metric[c] > best_metric) {
        best_metric = s_metric[c];
        best_rsrp   = s_corr[c];
        best        = static_cast<int>(c);
      }
    }
    srs_amd_pucch_f0_result r{};
    r.nof_sr       = best >= 0 ? d.nof_sr : d.nof_sr_default;
    r.nof_harq_ack = d.nof_harq;
    if (best >= 0) { // otherwise the default message: zero bits
      r.sr          = d.msg[best][0];
      r.harq_ack[0] = d.msg[best][1];
      r.harq_ack[1] = d.msg[best][2];
    }
    r.status           = best_metric > d.threshold ? SRS_AMD_UCI_STATUS_VALID : SRS_AMD_UCI_STATUS_INVALID;
    r.detection_metric = best_metric;
    r.sinr_dB          = to_dB(best_metric);
    r.rsrp_dB          = to_dB(best_rsrp);
    r.epre_dB          = to_dB(epre);
    results[blockIdx.x] = r;
  }
}

} // namespace

hipError_t launch_pucch_f0(const pucch_f0_desc* d_desc, uint32_t nof, srs_amd_pucch_f0_result* d_results,
                           hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pucch_f0_kernel, dim3(nof), dim3(64), 0, stream, d_desc, d_results);
  return hipGetLastError();
}

} // namespace srs_amd
