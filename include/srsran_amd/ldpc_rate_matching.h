/*
 * srsran_amd/ldpc_rate_matching.h -- C-ABI of the MI355X LDPC rate matcher
 * (PDSCH) and rate dematcher (PUSCH), TS 38.212 Section 5.4.2.
 *
 * Replaces (include/srsran/phy/upper/channel_coding/ldpc/):
 *   srs_amd_ldpc_rate_matcher_create / srs_amd_ldpc_rate_dematcher_create
 *       create_ldpc_rate_matcher_factory_sw()->create(),
 *       create_ldpc_rate_dematcher_factory_sw(type)->create()
 *       (lib/phy/upper/channel_coding/channel_coding_factories.cpp:172-215,297-305)
 *   srs_amd_ldpc_rate_match
 *       ldpc_rate_matcher::rate_match(bit_buffer& output, const ldpc_encoder_buffer& input,
 *                                     const codeblock_metadata& cfg)            ldpc_rate_matcher.h:47
 *   srs_amd_ldpc_rate_dematch
 *       ldpc_rate_dematcher::rate_dematch(span<log_likelihood_ratio> output,
 *                                         span<const log_likelihood_ratio> input, bool new_data,
 *                                         const codeblock_metadata& cfg)        ldpc_rate_dematcher.h:54
 *   *_batch
 *       the same for all codeblocks of a transport block, device-resident and
 *       asynchronous: the codeblocks' rate-matched segments are concatenated in
 *       one codeword (pdsch_encoder_impl.cpp / pusch_decoder_impl.cpp layout).
 *
 * Bit-exactness: the rate matcher is exact for every input.  The dematcher
 * reproduces ldpc_rate_dematcher_impl ("generic") for every int8 input,
 * including its zeroing rules when new_data is set and the LLR sum's
 * infinity rules when combining; the AVX2/AVX512 dematchers combine with a
 * clamped byte add and agree with it on finite LLRs (all a PUSCH soft buffer
 * ever combines).
 */
#ifndef SRSRAN_AMD_LDPC_RATE_MATCHING_H
#define SRSRAN_AMD_LDPC_RATE_MATCHING_H

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srs_amd_ldpc_rate_matcher   srs_amd_ldpc_rate_matcher;
typedef struct srs_amd_ldpc_rate_dematcher srs_amd_ldpc_rate_dematcher;

int  srs_amd_ldpc_rate_matcher_create(srs_amd_ldpc_rate_matcher** rm, int device);
void srs_amd_ldpc_rate_matcher_destroy(srs_amd_ldpc_rate_matcher* rm);
int  srs_amd_ldpc_rate_dematcher_create(srs_amd_ldpc_rate_dematcher** dm, int device);
void srs_amd_ldpc_rate_dematcher_destroy(srs_amd_ldpc_rate_dematcher* dm);

/* Single codeblock, HOST buffers, synchronous.
 *   output_packed : ceil(output_len/8) bytes; output_len = E (multiple of Qm)
 *   codeblock     : the encoded codeblock, N_short*Z bytes, one bit per byte
 *                   (what ldpc_encoder_buffer::write_codeblock produces)       */
int srs_amd_ldpc_rate_match(srs_amd_ldpc_rate_matcher*        rm,
                            uint8_t*                          output_packed,
                            uint32_t                          output_len,
                            const uint8_t*                    codeblock,
                            uint32_t                          codeblock_len,
                            const srs_amd_codeblock_metadata* cfg);

/* Batch, DEVICE buffers, asynchronous.
 *   d_codeblocks  : packed codeblocks as written by srs_amd_ldpc_encode_batch
 *   d_rm_lengths  : E_r per codeblock (multiples of Qm, <= max_rm_length)
 *   d_out_offsets : bit offset of codeblock r's segment in d_output
 *                   (segments are consecutive: offset[r+1] = offset[r] + E_r)
 *   d_output      : the concatenated codeword, packed MSB-first; every byte
 *                   that holds a bit of a segment is written whole (bits after
 *                   the last segment are 0).                                  */
int srs_amd_ldpc_rate_match_batch(srs_amd_ldpc_rate_matcher*        rm,
                                  const srs_amd_codeblock_metadata* cfg,
                                  const uint8_t*                    d_codeblocks,
                                  uint32_t                          cb_stride,
                                  const uint32_t*                   d_rm_lengths,
                                  const uint32_t*                   d_out_offsets,
                                  uint32_t                          max_rm_length,
                                  uint8_t*                          d_output,
                                  uint32_t                          nof_cbs,
                                  void*                             stream);

/* Single codeblock, HOST buffers, synchronous.  As the reference, the base
 * graph and lifting size follow from output_len (N_short*Z), Nref/rv/Qm/filler
 * from cfg; `output` is the codeblock soft buffer, read and written in place. */
int srs_amd_ldpc_rate_dematch(srs_amd_ldpc_rate_dematcher*      dm,
                              int8_t*                           output,
                              uint32_t                          output_len,
                              const int8_t*                     input,
                              uint32_t                          input_len,
                              int                               new_data,
                              const srs_amd_codeblock_metadata* cfg);

/* Batch, DEVICE buffers, asynchronous.
 *   d_input       : the received codeword LLRs (int8)
 *   d_in_offsets  : start of codeblock r's E_r LLRs in d_input
 *   d_rm_lengths  : E_r per codeblock (multiples of Qm)
 *   d_soft        : nof_cbs soft buffers of soft_stride bytes, N_short*Z LLRs
 *                   used (BG and Z from cfg), updated in place (HARQ).        */
int srs_amd_ldpc_rate_dematch_batch(srs_amd_ldpc_rate_dematcher*      dm,
                                    const srs_amd_codeblock_metadata* cfg,
                                    int                               new_data,
                                    const int8_t*                     d_input,
                                    const uint32_t*                   d_in_offsets,
                                    const uint32_t*                   d_rm_lengths,
                                    int8_t*                           d_soft,
                                    uint32_t                          soft_stride,
                                    uint32_t                          nof_cbs,
                                    void*                             stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_LDPC_RATE_MATCHING_H */
