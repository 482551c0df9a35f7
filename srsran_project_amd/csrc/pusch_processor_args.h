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

// CSI part 2 size of a fused-group PDU from its decoded CSI part 1, on the device (pusch_processor_impl.cpp:73-103:
// on_csi_part1 -> uci_part2_get_size, uci_part2_size_calculator.cpp:53-89): a valid CSI part 1 gives the size of
// its description, an invalid one none; the size goes to nof_part2 (the result's fourth status column) and its index
// among the plan's candidate sizes (every size the description can produce) to sel, -1 for none (the geometry
// without CSI part 2 stays).  The demultiplexer, UCI decoder and UL-SCH row patches of the candidates run only for
// the selected one.
struct csi2_select_args {
  const uint8_t*                     part1;     // CSI part 1 payload, one bit per byte
  const int32_t*                     status1;   // CSI part 1 status
  int32_t*                           nof_part2; // out
  int32_t*                           sel;       // out
  const int32_t*                     cand;      // [nof_cand] candidate sizes (device, the plan's)
  uint32_t                           nof_cand;
  uint32_t                           nof_part1;
  srs_amd_uci_part2_size_description descr;
};
hipError_t launch_csi2_select(const csi2_select_args* items, uint32_t n, hipStream_t stream);

// A UE of the slot decoder with HARQ state: its transport block's soft buffer (srs_amd_pusch_soft_buffer_layout rows)
// and whether this is a new transmission; soft NULL: a new transmission with internal buffers.
struct slot_harq {
  int8_t* soft;
  int     new_data;
  int     lazy = 0; // new data: soft LLRs kept only when the decoding leaves the TB failed (harq_row_desc::lazy)
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
                         const slot_harq*                    harq         = nullptr,
                         const struct slot_ue_patch*         patches      = nullptr,
                         uint32_t                            nof_patches  = 0);

// A UE of the slot decoder whose UL-SCH geometry is chosen on the device (CSI part 2): before rate dematching, its
// rows take the rate-matching lengths / LLR offsets of candidate *sel ([nof_cand][C] device tables; offsets relative
// to the UE's LLR row); *sel < 0 keeps the geometry of its plan.
struct slot_ue_patch {
  uint32_t        ue;
  const int32_t*  sel;
  const uint32_t* cand_E;
  const uint32_t* cand_off;
};

} // namespace srs_amd
