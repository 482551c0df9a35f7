/*
 * srsran_amd/ldpc_encoder.h -- C-ABI of the MI355X LDPC encoder.
 *
 * Replaces (include/srsran/phy/upper/channel_coding/ldpc/):
 *   srs_amd_ldpc_encoder_create
 *       create_ldpc_encoder_factory_sw(enc_type)->create()
 *       (lib/phy/upper/channel_coding/channel_coding_factories.cpp:141-170,291)
 *   srs_amd_ldpc_encode
 *       ldpc_encoder::encode(const bit_buffer& input, const configuration& cfg)   ldpc_encoder.h:59
 *       followed by ldpc_encoder_buffer::write_codeblock(data, 0)              ldpc_encoder_buffer.h:49
 *       for the whole N_short*Z-bit codeblock (one bit per byte, as write_codeblock).
 *   srs_amd_ldpc_encode_batch
 *       the same for many codeblocks of one transport block, device-resident and
 *       asynchronous; the codeblocks stay packed (bit_buffer layout) so that
 *       srs_amd_ldpc_rate_match_batch can read them (the ldpc_encoder_buffer role).
 *
 * Message: K*Z bits packed MSB-first (bit_buffer layout), filler bits set to 0
 * (ldpc_encoder.h:55).  Codeblock: the shortened codeword (the first 2Z
 * systematic bits removed), N_short*Z bits.  All reference encoders (generic,
 * AVX2, AVX512, NEON) produce the same codeword.
 */
#ifndef SRSRAN_AMD_LDPC_ENCODER_H
#define SRSRAN_AMD_LDPC_ENCODER_H

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srs_amd_ldpc_encoder srs_amd_ldpc_encoder;

/* ldpc_encoder::configuration (ldpc_encoder.h:43). Nref does not change the
 * codeword (only the rate matcher reads it) and is accepted for parity. */
typedef struct srs_amd_ldpc_encoder_config {
  uint32_t base_graph;   /* 1 = BG1, 2 = BG2 */
  uint32_t lifting_size; /* ldpc::lifting_size_t */
  uint32_t Nref;
} srs_amd_ldpc_encoder_config;

int  srs_amd_ldpc_encoder_create(srs_amd_ldpc_encoder** encoder, int device);
void srs_amd_ldpc_encoder_destroy(srs_amd_ldpc_encoder* encoder);

/* Single codeblock, HOST buffers, synchronous.
 *   message_packed : ceil(K*Z/8) bytes, message_len must equal K*Z bits
 *   codeblock      : N_short*Z bytes, one bit (0/1) per byte            */
int srs_amd_ldpc_encode(srs_amd_ldpc_encoder*              encoder,
                        uint8_t*                           codeblock,
                        uint32_t                           codeblock_len,
                        const uint8_t*                     message_packed,
                        uint32_t                           message_len,
                        const srs_amd_ldpc_encoder_config* cfg);

/* Batch, DEVICE buffers, asynchronous on `stream` (hipStream_t, NULL = default).
 *   d_messages   : nof_cbs rows of msg_stride bytes (>= ceil(K*Z/8)), packed
 *   d_codeblocks : nof_cbs rows of cb_stride bytes (>= ceil(N_short*Z/8)), packed
 *                  MSB-first; trailing bits of the last byte are 0.        */
int srs_amd_ldpc_encode_batch(srs_amd_ldpc_encoder*              encoder,
                              const srs_amd_ldpc_encoder_config* cfg,
                              const uint8_t*                     d_messages,
                              uint32_t                           msg_stride,
                              uint8_t*                           d_codeblocks,
                              uint32_t                           cb_stride,
                              uint32_t                           nof_cbs,
                              void*                              stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_LDPC_ENCODER_H */
