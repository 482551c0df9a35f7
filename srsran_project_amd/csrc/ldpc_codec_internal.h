// ldpc_codec_internal.h -- library-internal entry points of the LDPC rate matching objects.
#pragma once

#include "srsran_amd/ldpc_encoder.h"
#include "srsran_amd/ldpc_rate_matching.h"

namespace srs_amd {

// srs_amd_ldpc_rate_dematch_batch with `fresh`: with new_data set, the soft
// buffers' previous contents are taken as zero and not read (internal,
// freshly owned buffers; saves one N-byte read per codeblock).  The C-ABI
// entry point keeps the reference's semantics, where positions outside the
// rate-matched window keep what the buffer held.
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
                          bool                              fresh);

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

} // namespace srs_amd
