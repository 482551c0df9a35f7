/*
 * srsran_amd/ldpc.h -- C-ABI of the MI355X LDPC / CRC channel-coding path.
 *
 * This is the drop-in boundary.  Every entry point takes plain pointers and
 * sizes (no torch, no C++ types) and replaces one reference interface:
 *
 *   srs_amd_ldpc_decoder_create
 *       create_ldpc_decoder_factory_sw(dec_type, {force_decoding})->create()
 *       include/srsran/phy/upper/channel_coding/channel_coding_factories.h
 *       (implementation selection: lib/phy/upper/channel_coding/channel_coding_factories.cpp:102-139,285;
 *        `arith` selects which reference implementation's rounding is reproduced
 *        bit-exactly: SRS_AMD_ARITH_SIMD = "avx2"/"avx512"/"auto" on x86,
 *        SRS_AMD_ARITH_GENERIC = "generic")
 *   srs_amd_ldpc_decode
 *       ldpc_decoder::decode(bit_buffer&, span<const log_likelihood_ratio>, crc_calculator*, const configuration&)
 *       include/srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h:72
 *   srs_amd_ldpc_decode_batch
 *       the same operation for many codeblocks of one transport block / slot,
 *       device-resident: the enqueue/dequeue pair of
 *       hal::hw_accelerator_pusch_dec (include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h:84)
 *       collapsed into one asynchronous launch on a caller-given HIP stream.
 *
 * Conventions (as the reference):
 *   - LLRs are int8 log_likelihood_ratio values in [-120, 120] or +-127 (infinity).
 *   - Decoded messages are packed MSB-first, K*Z bits (bit_buffer layout,
 *     include/srsran/adt/bit_buffer.h:239), trailing bits of the last byte 0.
 *   - crc_poly is a crc_generator_poly value (CRC24A=0, CRC24B=1, CRC24C=2,
 *     CRC16=3, CRC11=4, CRC6=5) or SRS_AMD_NO_CRC for `crc == nullptr`.
 *   - nof_iterations: number of iterations when the CRC passed, -1 when the
 *     reference returns an empty std::optional.
 *   - Invalid configurations (reference: srsran_assert abort) return
 *     SRS_AMD_EINVAL and set srs_amd_last_error().
 */
#ifndef SRSRAN_AMD_LDPC_H
#define SRSRAN_AMD_LDPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRS_AMD_OK 0
#define SRS_AMD_EINVAL (-1)
#define SRS_AMD_EHIP (-2)
#define SRS_AMD_ENOMEM (-3)

#define SRS_AMD_NO_CRC (-1)

#define SRS_AMD_ARITH_SIMD 0
#define SRS_AMD_ARITH_GENERIC 1

/* ldpc_decoder::configuration (ldpc_decoder.h:44). */
typedef struct srs_amd_ldpc_decoder_config {
  uint32_t base_graph;      /* 1 = BG1, 2 = BG2 (ldpc_base_graph_type) */
  uint32_t lifting_size;    /* ldpc::lifting_size_t */
  uint32_t nof_filler_bits; /* filler bits in the full codeblock */
  uint32_t nof_crc_bits;    /* 16 or 24 */
  uint32_t max_iterations;  /* > 0 */
} srs_amd_ldpc_decoder_config;

typedef struct srs_amd_ldpc_decoder srs_amd_ldpc_decoder;

/* The codeblock_metadata fields the rate matcher / dematcher use
 * (include/srsran/phy/upper/codeblock_metadata.h:44 tb_common, :63 cb_specific). */
typedef struct srs_amd_codeblock_metadata {
  uint32_t base_graph;       /* tb_common.base_graph: 1 = BG1, 2 = BG2 */
  uint32_t lifting_size;     /* tb_common.lifting_size */
  uint32_t rv;               /* tb_common.rv, 0..3 */
  uint32_t modulation_order; /* get_bits_per_symbol(tb_common.mod): 1, 2, 4, 6 or 8 */
  uint32_t Nref;             /* tb_common.Nref: limited-buffer length, 0 = unlimited */
  uint32_t nof_filler_bits;  /* cb_specific.nof_filler_bits */
} srs_amd_codeblock_metadata;

/* Last error message of the calling thread ("" if none). */
const char* srs_amd_last_error(void);

/* Library version string. */
const char* srs_amd_version(void);

/* Creates a decoder bound to HIP device `device` (current device if < 0). */
int srs_amd_ldpc_decoder_create(srs_amd_ldpc_decoder** decoder, int arith, int force_decoding, int device);
void srs_amd_ldpc_decoder_destroy(srs_amd_ldpc_decoder* decoder);

/* Caps the launch grid (workgroups); larger batches are walked grid-stride.
 * Default 2^20 (one workgroup per codeblock). */
int srs_amd_ldpc_decoder_set_max_slots(srs_amd_ldpc_decoder* decoder, uint32_t max_slots);

/* Single codeblock, HOST buffers, synchronous: ldpc_decoder::decode. */
int srs_amd_ldpc_decode(srs_amd_ldpc_decoder*              decoder,
                        uint8_t*                           output_packed,
                        const int8_t*                      input,
                        uint32_t                           input_len,
                        int                                crc_poly,
                        const srs_amd_ldpc_decoder_config* cfg,
                        int32_t*                           nof_iterations);

/* Batch of codeblocks sharing one configuration, DEVICE buffers, asynchronous
 * on `stream` (a hipStream_t, NULL = default stream).
 *   d_llrs        : nof_cbs rows of llr_stride bytes
 *   d_llr_lens    : per-row input lengths, or NULL to use llr_len for all
 *   d_output      : nof_cbs rows of out_stride bytes (>= ceil(K*Z/8))
 *   d_nof_iters   : nof_cbs int32 results
 *   d_soft_out    : optional, nof_cbs rows of N_full*Z final soft bits (debug / parity)
 */
int srs_amd_ldpc_decode_batch(srs_amd_ldpc_decoder*              decoder,
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
                              void*                              stream);

/* Message / codeword lengths for a (base graph, lifting size) pair, 0 if invalid:
 * K*Z (message bits) and N_short*Z (encoded codeblock bits after shortening). */
uint32_t srs_amd_ldpc_message_length(uint32_t base_graph, uint32_t lifting_size);
uint32_t srs_amd_ldpc_codeblock_length(uint32_t base_graph, uint32_t lifting_size);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_LDPC_H */
