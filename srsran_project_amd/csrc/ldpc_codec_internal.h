// ldpc_codec_internal.h -- library-internal entry points of the LDPC rate matching objects.
#pragma once

#include "srsran_amd/ldpc.h"
#include "srsran_amd/ldpc_encoder.h"
#include "srsran_amd/ldpc_rate_matching.h"

namespace srs_amd {

// srs_amd_ldpc_rate_dematch_batch with `fresh`: with new_data set, the soft
// buffers' previous contents are taken as zero and not read (internal,
// freshly owned buffers; saves one N-byte read per codeblock).  The C-ABI
// entry point keeps the reference's semantics, where positions outside the
// rate-matched window keep what the buffer held.  write_end (0: the whole codeblock): soft-buffer
// bytes from write_end on are not written -- an internal buffer whose consumer reads only a prefix.
int rate_dematch_batch_ex(srs_amd_ldpc_rate_dematcher*      dm,
                          const srs_amd_codeblock_metadata* cfg,
                          int                               new_data,
                          const int8_t*                     d_input,
                          const uint32_t*                   d_in_offsets,
                          const uint32_t*                   d_rm_lengths,
                          int8_t*                           d_soft,
                          uint32_t                          soft_stride,
                          uint32_t                          nof_cbs,
                          void*                             stream,
                          bool                              fresh,
                          uint32_t                          write_end = 0);

// srs_amd_ldpc_encode_batch producing only the first max_bits of each shortened
// codeword (the rows of the extension region beyond them are not computed and
// the codeblock rows are written up to ceil(max_bits / 8) bytes): what a rate
// matcher reading the circular buffer window [0, max_bits) needs.
int ldpc_encode_batch_ex(srs_amd_ldpc_encoder*              enc,
                         const srs_amd_ldpc_encoder_config* cfg,
                         const uint8_t*                     d_messages,
                         uint32_t                           msg_stride,
                         uint8_t*                           d_codeblocks,
                         uint32_t                           cb_stride,
                         uint32_t                           nof_cbs,
                         void*                              stream,
                         uint32_t                           max_bits);

// srs_amd_ldpc_decode_batch with an optional per-codeblock skip flag (int32 at d_skip_flags + cb *
// skip_stride, non-zero: not decoded, nof_iters[cb] = -2): the PUSCH decoder's retransmissions of
// codeblocks whose CRC passed in an earlier transmission (pusch_decoder_impl.cpp:330-345).
// Codeblock rows built from the received codeword (decode_args::cw_llrs): the rate dematcher's new-data,
// fresh-buffer, k0 = 0, no-wrap case fused into the high-rate decoder's load; d_llrs is then unused.
struct ldpc_cw_rows {
  const int8_t*   llrs;     // codeword LLRs
  const uint32_t* offsets;  // [nof_cbs] byte offset of each codeblock's E LLRs
  const uint32_t* lengths;  // [nof_cbs] E
  uint32_t        qm, nof_info, filler;
};

int ldpc_decode_batch_ex(srs_amd_ldpc_decoder*              d,
                         const srs_amd_ldpc_decoder_config* cfg,
                         int                                crc_poly,
                         const int8_t*                      d_llrs,
                         uint32_t                           llr_stride,
                         const uint32_t*                    d_llr_lens,
                         uint32_t                           llr_len,
                         uint8_t*                           d_output,
                         uint32_t                           out_stride,
                         int32_t*                           d_nof_iters,
                         int8_t*                            d_soft_out,
                         uint32_t                           nof_cbs,
                         void*                              stream,
                         const uint8_t*                     d_skip_flags,
                         uint32_t                           skip_stride,
                         const int32_t*                     d_fillers = nullptr,
                         const ldpc_cw_rows*                cw        = nullptr);

// LDPC decoding of codeblocks of one base graph with per-codeblock lifting sizes (srs_amd_pusch_decode_slot):
// row cb has lifting size row_z[cb] <= max_z < 384, input length llr_lens[cb], filler bits fillers[cb] and
// CRC polynomial row_crc[cb] (SRS_AMD_NO_CRC: none), its soft row at d_llrs + cb * llr_stride.
int ldpc_decode_mixed(srs_amd_ldpc_decoder* d,
                      uint32_t              bg,
                      uint32_t              max_z,
                      uint32_t              max_iterations,
                      const int8_t*         d_llrs,
                      uint32_t              llr_stride,
                      const uint32_t*       d_llr_lens,
                      uint8_t*              d_output,
                      uint32_t              out_stride,
                      int32_t*              d_nof_iters,
                      uint32_t              nof_cbs,
                      void*                 stream,
                      const int32_t*        d_fillers,
                      const void*           d_rows);

// Device row descriptor of ldpc_decode_mixed (16 bytes) for a codeblock of lifting size Z and CRC poly.
void ldpc_mixed_row(void* row, uint32_t bg, uint32_t Z, int crc_poly);

// LDPC encoding of codeblocks of one base graph with per-codeblock lifting sizes (all >= 32) in one launch
// (srs_amd_pdsch_encode_slot): d_rows holds ldpc_encode_mixed_row descriptors; max_z / max_rows_eff size the
// launch (the largest Z and extension row count of the batch).
int ldpc_encode_mixed(srs_amd_ldpc_encoder* enc,
                      uint32_t              bg,
                      uint32_t              max_z,
                      uint32_t              max_rows_eff,
                      const uint8_t*        d_messages,
                      uint32_t              msg_stride,
                      uint8_t*              d_codeblocks,
                      uint32_t              cb_stride,
                      uint32_t              nof_cbs,
                      void*                 stream,
                      const void*           d_rows);

// Row descriptor (32 bytes) of ldpc_encode_mixed for a codeblock of lifting size Z whose rate matcher reads
// the first max_bits of the shortened codeword; returns the extension rows it computes (M_eff).
uint32_t ldpc_encode_mixed_row(void* row, uint32_t bg, uint32_t Z, uint32_t max_bits);
constexpr size_t LDPC_ENCODE_ROW_BYTES = 32;

// Device table of every lifted graph's edges (ldpc_encode_mixed_row's edge_off indexes it).
const uint32_t* ldpc_encoder_edges(const srs_amd_ldpc_encoder* enc);

// Rate matching of codeblocks with per-codeblock geometry (srs_amd_pdsch_encode_slot): codeblock cb uses
// geos[row_geo[cb]]; d_out_offsets are bit offsets into d_output.
int rate_match_ragged(srs_amd_ldpc_rate_matcher* rm,
                      const uint8_t*             d_codeblocks,
                      uint32_t                   cb_stride,
                      const uint32_t*            d_rm_lengths,
                      const uint32_t*            d_out_offsets,
                      const uint32_t*            d_row_geo,
                      const void*                d_geos,
                      uint8_t*                   d_output,
                      uint32_t                   nof_cbs,
                      void*                      stream);

// Rate dematching of codeblocks with per-codeblock geometry (srs_amd_pusch_decode_slot): codeblock cb
// uses geos[row_geo[cb]] and writes soft-buffer bytes [0, geo_write_end[row_geo[cb]]) of its row
// (new data into fresh internal buffers, whose old contents are taken as zero; with d_row_flags, codeblock cb's
// new-data / fresh flags: bit 0 / bit 1 of d_row_flags[cb]).
int rate_dematch_ragged(srs_amd_ldpc_rate_dematcher* dm,
                        const int8_t*                d_input,
                        const uint32_t*              d_in_offsets,
                        const uint32_t*              d_rm_lengths,
                        const uint32_t*              d_row_geo,
                        const void*                  d_geos,
                        const uint32_t*              d_geo_write_end,
                        int8_t*                      d_soft,
                        uint32_t                     soft_stride,
                        uint32_t                     nof_cbs,
                        void*                        stream,
                        const uint8_t*               d_row_flags = nullptr);

} // namespace srs_amd
