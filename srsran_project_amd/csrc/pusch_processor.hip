// pusch_processor.hip -- the PUSCH processor's result kernel: per transport block, the
// decoder result plus the channel state information of channel_estimate::
// get_channel_state_information (channel_estimation.h:244-286) from the estimator's port stats.
#include <hip/hip_runtime.h>

#include "pusch_processor_args.h"

namespace srs_amd {

__global__ __launch_bounds__(64) void pusch_result_kernel(pusch_result_args a)
{
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= a.nof_grids) {
    return;
  }
  const uint32_t                  P  = a.port_counts != nullptr ? a.port_counts[g] : a.nof_ports;
  const uint32_t                  sg = (a.stats_by_id && a.result_ids != nullptr) ? a.result_ids[g] : g;
  const srs_amd_chest_port_stats* st = a.stats + static_cast<size_t>(sg) * (a.stats_stride ? a.stats_stride : P);
  float    noise = 0.0f, rsrp = 0.0f, epre = 0.0f, best_snr = 0.0f;
  uint32_t best  = 0;
  for (uint32_t p = 0; p < P; ++p) {
    noise += st[p].noise_var;
    rsrp += st[p].rsrp;
    epre += st[p].epre;
    if (st[p].snr > best_snr) {
      best_snr = st[p].snr;
      best     = p;
    }
  }
  srs_amd_pusch_processor_result r;
  r.data             = a.dec_results[g];
  const bool normal  = isfinite(noise) && fabsf(noise) >= 1.17549435e-38f;
  r.sinr_db          = 10.0f * log10f(normal ? rsrp / noise : 0.0f);
  r.epre_db          = 10.0f * log10f(epre / static_cast<float>(P));
  r.rsrp_db          = 10.0f * log10f(rsrp / static_cast<float>(P));
  r.time_alignment_s = st[best].time_alignment_s;
  r.cfo_hz           = st[best].cfo_hz;
  const uint32_t mask = a.uci_masks != nullptr ? a.uci_masks[g] : a.uci_mask;
  r.harq_ack_status  = (mask & 1u) ? a.uci_status[4 * g] : 0;
  r.csi_part1_status = (mask & 2u) ? a.uci_status[4 * g + 1] : 0;
  r.csi_part2_status = (mask & 4u) ? a.uci_status[4 * g + 2] : 0;
  r.nof_csi_part2    = (mask & 4u) ? static_cast<uint32_t>(a.uci_status[4 * g + 3]) : 0u;
  a.results[a.result_ids != nullptr ? a.result_ids[g] : g] = r;
}

__global__ __launch_bounds__(64) void csi2_select_kernel(const csi2_select_args* items, uint32_t n)
{
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) {
    return;
  }
  const csi2_select_args& a  = items[i];
  int32_t                 n2 = 0;
  if (*a.status1 == SRS_AMD_UCI_VALID) { // on_csi_part1 is notified with a valid CSI part 1 only
    for (uint32_t e = 0; e < a.descr.nof_entries && e < 2; ++e) {
      const srs_amd_uci_part2_entry& en    = a.descr.entries[e];
      uint32_t                       index = 0;
      for (uint32_t q = 0; q < en.nof_parameters && q < 2; ++q) {
        // the field's first bit is its most significant (uci_part2_size_calculator.cpp extract_parameter)
        uint32_t value = 0;
        for (uint32_t b = 0; b < en.parameters[q].width; ++b) {
          value = (value << 1) | (a.part1[en.parameters[q].offset + b] & 1u);
        }
        index = (index << en.parameters[q].width) | value;
      }
      n2 += index < en.map_size && index < 16 ? en.map[index] : 0;
    }
  }
  int32_t s = -1;
  for (uint32_t c = 0; c < a.nof_cand && n2 != 0; ++c) {
    s = a.cand[c] == n2 ? static_cast<int32_t>(c) : s;
  }
  *a.nof_part2 = s >= 0 ? n2 : 0;
  *a.sel       = s;
}

hipError_t launch_csi2_select(const csi2_select_args* items, uint32_t n, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(csi2_select_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, items, n);
  return hipGetLastError();
}

hipError_t launch_pusch_result(const pusch_result_args& a, hipStream_t stream)
{
  if (a.nof_grids == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pusch_result_kernel, dim3((a.nof_grids + 63) / 64), dim3(64), 0, stream, a);
  return hipGetLastError();
}

} // namespace srs_amd
