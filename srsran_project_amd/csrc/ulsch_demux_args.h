// ulsch_demux_args.h -- argument block of the UL-SCH demultiplexer kernel (ulsch_demux.hip), shared with its
// C-ABI (ulsch_demux_api.cpp) and the PUSCH processor.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "srsran_amd/ulsch_demux.h"

namespace srs_amd {

constexpr uint32_t DMX_NONE = 0xffffffffu;
constexpr uint32_t DMX_ZERO = 1u << 30;         // sch entry: the UL-SCH copy of a 1/2-bit HARQ-ACK RE is zero
constexpr uint32_t DMX_KIND_SHIFT = 28;         // uci entry: kind << 28 | RE index of the stream
constexpr uint32_t DMX_INDEX_MASK = (1u << 28) - 1;
constexpr uint32_t DMX_ACK  = 1;
constexpr uint32_t DMX_CSI1 = 2;

struct demux_args {
  const int8_t*   cws;
  int8_t*         sch;
  int8_t*         ack;
  int8_t*         csi1;
  const uint32_t* sch_map; // [nof_re]: UL-SCH RE index | DMX_ZERO, or DMX_NONE
  const uint32_t* uci_map; // [nof_re]: kind << 28 | stream RE index, or DMX_NONE
  const uint32_t* csi2_map; // [nof_re]: CSI part 2 RE index | DMX_ZERO, or DMX_NONE (null: no CSI part 2)
  int8_t*         csi2;
  const uint32_t* scr;     // Gold words of c_init over the codeword
  uint64_t        cw_stride;
  uint64_t        sch_stride;
  uint64_t        ack_stride;
  uint64_t        csi1_stride;
  uint64_t        csi2_stride;
  uint32_t        nof_re;
  uint32_t        qm;
  uint32_t        bpre;    // bits per RE: Qm x layers
  uint32_t        ack_ph;  // HARQ-ACK payload bits when 1 or 2 (placeholders), else 0
  uint32_t        csi1_ph; // CSI part 1 payload bits when 1 or 2, else 0
  uint32_t        csi2_ph; // CSI part 2 payload bits when 1 or 2, else 0
  // slot form: the block runs only when *sel == sel_val (one block per CSI part 2 size candidate of a PDU, the size
  // selected on the device from the decoded CSI part 1); sel null: always
  const int32_t*  sel     = nullptr;
  int32_t         sel_val = 0;
};

// Host placement (ulsch_demultiplex_impl.cpp:285-444) of every data RE of the codeword, in demodulator order.
struct demux_placement {
  std::vector<uint32_t> sch_map, uci_map, csi2_map;
  uint32_t              nof_re = 0, nof_sch_re = 0, nof_ack_re = 0, nof_csi1_re = 0, nof_csi2_re = 0;
};
int build_demux_placement(const srs_amd_ulsch_demux_config& cfg, demux_placement& out);

hipError_t launch_ulsch_demux(const demux_args& a, uint32_t nof_cws, hipStream_t stream);
// Slot form: one argument block per codeword (device array), each with its own plan; max_re: the largest nof_re.
hipError_t launch_ulsch_demux_items(const demux_args* items, uint32_t n, uint32_t max_re, hipStream_t stream);
// The argument block of one codeword of `plan` (no CSI part 2): codeword LLRs cws, outputs sch / ack / csi1.
demux_args make_demux_args(const srs_amd_ulsch_demux_plan* plan, const int8_t* cws, int8_t* sch, int8_t* ack,
                           int8_t* csi1);
// The same with the plan's CSI part 2 placement (a plan created with nof_csi_part2_bits != 0) into csi2.
demux_args make_demux_args_csi2(const srs_amd_ulsch_demux_plan* plan, const int8_t* cws, int8_t* sch, int8_t* ack,
                                int8_t* csi1, int8_t* csi2);

} // namespace srs_amd
