// pusch_processor_args.h -- argument block of the PUSCH processor's result kernel
// (pusch_processor.hip), shared with its C-ABI (pusch_processor_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "srsran_amd/pusch_processor.h"

namespace srs_amd {

struct pusch_result_args {
  const srs_amd_pusch_decoder_result* dec_results; // [grid]
  const srs_amd_chest_port_stats*     stats;       // [grid][port]
  srs_amd_pusch_processor_result*     results;     // [grid]
  uint32_t                            nof_grids;
  uint32_t                            nof_ports;
  // slot form: PDU g has port_counts[g] ports, its stats at stats + g * stats_stride
  const uint32_t*                     port_counts  = nullptr;
  uint32_t                            stats_stride = 0;
  // UCI on PUSCH: [grid][4] = HARQ-ACK, CSI part 1, CSI part 2 statuses of the fields set in uci_mask (bits 0-2),
  // CSI part 2 payload bits
  const int32_t*                      uci_status   = nullptr;
  uint32_t                            uci_mask     = 0;
  // slot form: result g's own field mask (overrides uci_mask)
  const uint32_t*                     uci_masks    = nullptr;
  // slot form with PDUs outside the fused group: result g goes to results[result_ids[g]]
  const uint32_t*                     result_ids   = nullptr;
  // the port measurements of result g are those of PDU result_ids[g] (caller's per-PDU buffer)
  bool                                stats_by_id  = false;
};

hipError_t launch_pusch_result(const pusch_result_args& a, hipStream_t stream);

// A UE of the slot decoder with HARQ state: its transport block's soft buffer (srs_amd_pusch_soft_buffer_layout rows)
// and whether this is a new transmission; soft NULL: a new transmission with internal buffers.
struct slot_harq {
  int8_t* soft;
  int     new_data;
};

// srs_amd_pusch_decode_slot (pusch_api.cpp) with per-codeblock iteration counts: UE u's C values at
// d_cb_iterations + cb_offsets[u] (host array; both NULL: not returned), and optionally HARQ state per UE (harq[u],
// host array; NULL: every UE a new transmission with internal buffers; cfg->new_data is then ignored and
// cfg->use_early_stop must be set).
int pusch_decode_slot_ex(srs_amd_pusch_decoder*              dec,
                         const srs_amd_pusch_decoder_config* cfg,
                         const srs_amd_pusch_ue*             ues,
                         uint32_t                            nof_ues,
                         const int8_t*                       d_llrs,
                         uint8_t*                            d_tbs,
                         srs_amd_pusch_decoder_result*       d_results,
                         const uint32_t*                     cb_offsets,
                         int32_t*                            d_cb_iterations,
                         hipStream_t                         stream,
                         const slot_harq*                    harq = nullptr);

} // namespace srs_amd
