/*
 * srsran_amd/polar.h -- C-ABI of the MI355X polar channel coding (PDCCH DCI,
 * PUCCH / PUSCH UCI), TS 38.212 Sections 5.3.1 and 5.4.1.
 *
 * Replaces (include/srsran/phy/upper/channel_coding/polar/, factory
 * create_polar_factory_sw(), lib/phy/upper/channel_coding/channel_coding_factories.cpp:245-275,323):
 *   srs_amd_polar_code_create        polar_code::set(K, E, nMax, ibil)            polar_code.h:110
 *   srs_amd_polar_code_get_*         polar_code::get_N / get_n / get_nPC / get_K_set / get_PC_set
 *   srs_amd_polar_encode(_batch)     polar_allocator::allocate -> polar_encoder::encode ->
 *                                    polar_rate_matcher::rate_match (the pdcch_encoder_impl chain)
 *   srs_amd_polar_decode(_batch)     polar_rate_dematcher::rate_dematch -> polar_decoder::decode ->
 *                                    polar_deallocator::deallocate (the UCI polar decoding chain)
 *   srs_amd_polar_interleave         polar_interleaver::interleave (DCI input bit interleaver)
 *
 * Bits are one per byte (0/1), LLRs int8 (log_likelihood_ratio), exactly the
 * reference's span types.  Bit-exact with the reference (tests/test_polar_gpu.py).
 */
#ifndef SRSRAN_AMD_POLAR_H
#define SRSRAN_AMD_POLAR_H

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srs_amd_polar_code srs_amd_polar_code;

/* nMax 9 (downlink) or 10 (uplink); ibil: channel interleaver present (uplink). */
int      srs_amd_polar_code_create(srs_amd_polar_code** code, uint32_t K, uint32_t E, uint32_t nMax, int ibil,
                                   int device);
void     srs_amd_polar_code_destroy(srs_amd_polar_code* code);
uint32_t srs_amd_polar_code_get_N(const srs_amd_polar_code* code);
uint32_t srs_amd_polar_code_get_n(const srs_amd_polar_code* code);
uint32_t srs_amd_polar_code_get_nPC(const srs_amd_polar_code* code);
/* K_set mask (N bytes, 1 = information or parity-check position) and PC set (nPC entries). */
int srs_amd_polar_code_get_K_set(const srs_amd_polar_code* code, uint8_t* mask);
int srs_amd_polar_code_get_PC_set(const srs_amd_polar_code* code, uint16_t* pc_set);

/* Host-only construction (no device): returns N, or 0 for an invalid code
 * (srs_amd_last_error says why); fills the K_set mask (N bytes) and PC set. */
uint32_t srs_amd_polar_code_construct(uint32_t K, uint32_t E, uint32_t nMax, uint8_t* mask, uint16_t* pc_set,
                                      uint32_t* nPC);

/* One codeword, HOST buffers, synchronous: message K bits -> E coded bits. */
int srs_amd_polar_encode(srs_amd_polar_code* code, uint8_t* output, const uint8_t* message);
/* One codeword, HOST buffers, synchronous: E LLRs -> message K bits. */
int srs_amd_polar_decode(srs_amd_polar_code* code, uint8_t* message, const int8_t* llrs);

/* Batches of codewords of one code, DEVICE buffers, asynchronous on `stream`. */
int srs_amd_polar_encode_batch(srs_amd_polar_code* code,
                               const uint8_t*      d_messages,
                               uint32_t            msg_stride,
                               uint8_t*            d_output,
                               uint32_t            out_stride,
                               uint32_t            nof,
                               void*               stream);
int srs_amd_polar_decode_batch(srs_amd_polar_code* code,
                               const int8_t*       d_llrs,
                               uint32_t            llr_stride,
                               uint8_t*            d_messages,
                               uint32_t            msg_stride,
                               uint32_t            nof,
                               void*               stream);

/* DCI input bit interleaver, K <= 164, direction 0 = tx, 1 = rx (host). */
int srs_amd_polar_interleave(uint8_t* output, const uint8_t* input, uint32_t K, int direction);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_POLAR_H */
