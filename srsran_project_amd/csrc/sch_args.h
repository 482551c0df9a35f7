// sch_args.h -- argument blocks of the transport-block kernels (sch.hip),
// shared with their C-ABI (pdsch_api.cpp, pusch_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "srsran_amd/sch.h"

namespace srs_amd {

struct rm_geometry;
struct enc_row_desc;

// ldpc_segmenter_tx_impl::read_codeblock (ldpc_segmenter_tx_impl.cpp:137-207) for
// every (TB, segment) pair: data bits, TB CRC + zero pad in the last segment,
// zeros where the CB CRC (attached afterwards) and the filler bits go.
struct segment_args {
  const uint8_t*  tbs;        // nof_tbs rows of tb_stride bytes
  const uint32_t* tb_crcs;    // TB checksum per TB
  uint8_t*        msgs;       // nof_tbs * C rows of msg_stride bytes
  uint32_t        tb_stride;
  uint32_t        msg_stride;
  uint32_t        msg_bytes;  // ceil(K / 8)
  uint32_t        nof_segments;
  uint32_t        cb_info_bits;
  uint32_t        last_data_bits; // TB bits in the last segment
  uint32_t        tb_crc_bits;
  uint32_t        nof_rows;   // nof_tbs * C
  // CRC24B attachment in the same pass (C > 1): the codeblock CRC over bits [0, cb_info_bits) written at
  // bit cb_info_bits (ldpc_segmenter_tx_impl.cpp:196); null table: segmentation only
  const uint32_t* cb_crc_table; // x^(k+24) mod g (crc_linear_table)
  uint32_t        cb_crc_poly;
};

// Per-CB soft-buffer row (HARQ rx_buffer): [soft LLRs | saved message | CRC flag].
struct soft_row_layout {
  uint32_t soft_bytes; // N_short * Z
  uint32_t msg_offset;
  uint32_t flag_offset;
  uint32_t row_bytes;
};

// One transport block of a heterogeneous batch (srs_amd_pusch_decode_slot / srs_amd_pdsch_encode_slot): its
// codeblock rows are [row0, row0 + nof_segments) of the scratch, its bytes at tbs + tb_offset.
struct tb_desc {
  uint64_t tb_offset;
  uint32_t row0;
  uint32_t nof_segments;
  uint32_t cb_info_bits;
  uint32_t tbs_bits;
  uint32_t tb_crc_bits; // 16 / 24
  uint32_t zero_pad;
  uint32_t msg_bytes;   // ceil(K / 8)
  uint32_t pad;         // decode: index of the TB's first codeblock in assemble_args::cb_iterations
};

// PDSCH encoder of a heterogeneous batch: TB CRCs (CRC16 or CRC24A per TB, linear CRC over chunks XOR-ed
// into acc[t]), segmentation, and the CRC24B of the codeblocks of segmented TBs (per-row lengths).
struct tx_slot_args {
  const uint8_t*  tbs;        // TB bytes (tds[t].tb_offset)
  const tb_desc*  tds;
  const uint32_t* row_tb;     // TB of each message row
  uint32_t*       acc;        // per-TB CRC accumulators (zeroed before tx_tb_crc_kernel)
  uint8_t*        msgs;       // message rows of msg_stride bytes
  const uint32_t* crc16_table;
  const uint32_t* crc24a_table;
  const uint32_t* crc24b_table;
  uint32_t        crc16_poly, crc24a_poly, crc24b_poly;
  uint32_t        msg_stride;
  uint32_t        nof_tbs;
  uint32_t        nof_rows;
  uint32_t        max_tb_bytes;
  uint32_t        max_msg_bytes;
};
hipError_t launch_tx_slot_segment(const tx_slot_args& a, hipStream_t stream);

// Fused PDSCH encoder (pdsch_encoder.hip): TB CRC partials, then one workgroup per codeblock that builds,
// CRC-attaches, LDPC-encodes and rate-matches its codeblock in LDS.
struct pdsch_fused_args {
  const uint8_t*                 tbs;      // TB bytes (tds[t].tb_offset)
  const tb_desc*                 tds;      // per TB
  const uint32_t*                row_tb;   // per codeblock: TB index
  const uint32_t*                row_E;    // per codeblock: rate-matched length
  const uint32_t*                row_out;  // per codeblock: first codeword bit (absolute)
  const uint32_t*                row_geo;  // per codeblock: index into geos
  const struct rm_geometry*      geos;
  const struct enc_row_desc*     enc_rows; // per codeblock: lifted graph, encoded window
  const uint32_t*                edges;    // every lifted graph (enc_row_desc::edge_off)
  uint32_t*                      tb_parts; // [nof_tbs][part_stride] TB CRC partials (pdsch_tb_crc_kernel)
  uint32_t                       part_stride;
  uint32_t                       max_tb_bytes;
  const uint32_t*                crc16_table;
  const uint32_t*                crc24a_table;
  const uint32_t*                crc24b_table;
  uint32_t                       crc16_poly, crc24a_poly, crc24b_poly;
  uint8_t*                       cw;       // codewords
  uint32_t                       nof_tbs;
  uint32_t                       nof_cbs;
  const uint32_t*                last_rows; // [nof_tbs]: the row of each TB's last codeblock
  uint32_t                       last_only; // set by launch_pdsch_fused
  int32_t                        row_start[2][47]; // check-row edge offsets of BG1 / BG2
};
constexpr uint32_t PE_TB_CHUNK = 8192; // TB bytes per partial of the TB CRC
// phase 0: TB CRC partials on crc_stream, every codeblock but the TBs' last ones on cb_stream; phase 1 (after both):
// the TBs' last codeblocks on stream; phase 2: the TB CRC partials, then every codeblock, on stream.
hipError_t launch_pdsch_fused(const pdsch_fused_args& a, hipStream_t crc_stream, hipStream_t cb_stream,
                              hipStream_t stream, int phase);

// pusch_decoder_impl.cpp:309-500 after the decoder: per-CB CRC status (kept in the
// soft buffer across HARQ transmissions), statistics, codeblock concatenation
// and the TB CRC check.
struct assemble_args {
  const uint8_t*                msgs;         // decoder output rows (msg_stride)
  const int32_t*                iters;        // decoder iterations per CB (-1: CRC failed)
  const uint32_t*               crc_checks;   // non-null when decoding without early stop: CRC of each message
  uint8_t*                      soft;         // soft-buffer rows, or null
  uint8_t*                      tbs;          // output TB rows
  srs_amd_pusch_decoder_result* results;
  int32_t*                      cb_iterations; // optional per-CB report
  const uint32_t*               crc24a_table; // x^(k+24) mod g(CRC24A)
  uint32_t*                     acc;          // per-TB CRC accumulators (nof_tbs words of scratch)
  soft_row_layout               lay;
  uint32_t                      msg_stride;
  uint32_t                      tb_stride;
  uint32_t                      nof_segments;
  uint32_t                      cb_info_bits;
  uint32_t                      tbs_bits;
  uint32_t                      max_iterations;
  int32_t                       new_data;
  // optional per-TB descriptors (replace nof_segments / cb_info_bits / tbs_bits / tb_stride, rows of TB t
  // start at tds[t].row0); soft must be null.  max_tb_bits: the largest tbs_bits (grid of asm_tb_kernel).
  const tb_desc*                tds;
  uint32_t                      max_tb_bits;
};

// HARQ state of the PUSCH slot decoder (pusch_api.cpp decode_slot_locked): the codeblocks of transport blocks with a
// caller soft buffer are decoded in the slot's internal rows; their soft bits are gathered from the caller's rows
// before the rate dematcher combines into them and scattered back after decoding, with the message / CRC-flag
// bookkeeping of pusch_decoder_impl.cpp:320-375 and 416-437 (what the assemble kernels do for a uniform batch).
struct harq_row_desc {
  uint8_t* soft_row;    // the caller's soft-buffer row: soft LLRs | message bytes | int32 flag (soft_row_layout)
  uint32_t row;         // the decoder row
  uint32_t soft_bytes;  // soft LLR bytes
  uint32_t msg_offset;
  uint32_t msg_bytes;
  uint32_t flag_offset;
  uint32_t new_data;
  // lazy (new data only): the soft LLRs are copied back only when some codeblock of the TB (decoder rows
  // tb_row0 .. tb_row0 + tb_C - 1) failed its CRC -- the state a retransmission combines with; the message and flag
  // are written always
  uint32_t lazy;
  uint32_t tb_row0;
  uint32_t tb_C;
};
struct harq_tb_desc {
  uint8_t* soft;        // the caller's soft buffer (C rows)
  uint32_t result;      // index of the TB's decoder result
  uint32_t C;
  uint32_t row_bytes;
  uint32_t flag_offset;
  uint32_t lazy;        // as harq_row_desc::lazy: a TB whose codeblocks all passed but whose TB CRC failed then copies
  uint32_t row0;        // its soft LLRs back here (decoder rows row0 .., soft_bytes each)
  uint32_t soft_bytes;
};
struct harq_args {
  const harq_row_desc*          rows;
  uint32_t                      nof_rows;
  const harq_tb_desc*           tbs;
  uint32_t                      nof_tbs;
  int8_t*                       internal; // decoder soft rows, stride S
  uint32_t                      S;
  uint8_t*                      msgs;     // decoder message rows, stride M
  uint32_t                      M;
  int32_t*                      iters;    // decoder iterations per row (-1: CRC failed)
  int32_t*                      prev;     // [nof_rows]: the codeblock's flag before this transmission
  srs_amd_pusch_decoder_result* results;
};
// Before the rate dematcher: soft bits of the retransmitted rows into the decoder rows, the previous flags.
hipError_t launch_harq_gather(const harq_args& a, uint32_t max_soft_bytes, hipStream_t stream);
// After the LDPC decoder, before the assembly: soft bits back, messages / iterations of codeblocks OK from an
// earlier transmission into the decoder rows, the fresh messages and flags into the caller's rows.
hipError_t launch_harq_scatter(const harq_args& a, uint32_t max_soft_bytes, hipStream_t stream);
// After the assembly: a TB whose codeblocks all passed but whose TB CRC failed clears its CRC flags.
hipError_t launch_harq_final(const harq_args& a, hipStream_t stream);

// Slot decoder rows of a UE whose UL-SCH geometry is selected on the device (pusch_processor_args.h slot_ue_patch):
// rows row_E[0 .. C) / row_in[0 .. C) of the uploaded descriptors take candidate *sel's lengths and offsets.
struct slot_row_patch {
  uint32_t*       row_E;
  uint32_t*       row_in;
  const int32_t*  sel;
  const uint32_t* cand_E;   // [nof_cand][C]
  const uint32_t* cand_off; // [nof_cand][C], relative to the UE's LLR row
  uint32_t        llr_offset;
  uint32_t        C;
};
hipError_t launch_slot_row_patch(const slot_row_patch* items, uint32_t n, hipStream_t stream);

hipError_t launch_segment(const segment_args& a, hipStream_t stream);
// true when launch_segment also attaches the codeblock CRCs (segment_crc_kernel)
bool       segment_attaches_crc(const segment_args& a);
// Per-codeblock rate-matching lengths and codeword offsets of nof_tbs transport blocks of one plan
// (srs_amd_sch_plan_segments per TB), written on the device: arrays[row] = E_r, arrays[rows + row] =
// tb * tb_units + offset_r, row = tb * C + r.  No host upload, so a plan change never blocks the host.
hipError_t launch_rm_arrays(uint32_t* arrays, uint32_t nof_tbs, uint32_t C, uint32_t nof_short, uint32_t e_short,
                            uint32_t e_long, uint32_t tb_units, hipStream_t stream);
hipError_t launch_assemble(const assemble_args& a, uint32_t nof_tbs, hipStream_t stream);

} // namespace srs_amd
