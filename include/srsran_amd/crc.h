/*
 * srsran_amd/crc.h -- C-ABI of the MI355X CRC calculator (TB and codeblock CRCs).
 *
 * Replaces:
 *   srs_amd_crc_calculator_create   create_crc_calculator_factory_sw(type)->create(poly)
 *                                   (lib/phy/upper/channel_coding/channel_coding_factories.cpp)
 *   srs_amd_crc_calculate(_batch)   crc_calculator::calculate(const bit_buffer&)
 *                                   include/srsran/phy/upper/channel_coding/crc_calculator.h:81
 *   srs_amd_crc_attach_batch        the CRC attachment of ldpc_segmenter_tx (TS 38.212 5.1/5.2.2):
 *                                   the L CRC bits written right after the payload bits.
 * Linear CRC: every set payload bit contributes x^(position + L) mod g from a
 * table; bit-exact with crc_calculator_generic_impl.
 */
#ifndef SRSRAN_AMD_CRC_H
#define SRSRAN_AMD_CRC_H

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srs_amd_crc_calculator srs_amd_crc_calculator;

/* poly: crc_generator_poly value (CRC24A=0, CRC24B=1, CRC24C=2, CRC16=3, CRC11=4, CRC6=5);
 * max_bits: longest payload (bits) this calculator will see. */
int      srs_amd_crc_calculator_create(srs_amd_crc_calculator** crc, int poly, uint32_t max_bits, int device);
void     srs_amd_crc_calculator_destroy(srs_amd_crc_calculator* crc);
uint32_t srs_amd_crc_order(const srs_amd_crc_calculator* crc);

/* HOST: CRC of nof_bits bits packed MSB-first. */
int srs_amd_crc_calculate(srs_amd_crc_calculator* crc, uint32_t* checksum, const uint8_t* bits, uint32_t nof_bits);

/* DEVICE, asynchronous: CRCs of nof_rows rows of stride bytes (the first nof_bits bits of each). */
int srs_amd_crc_calculate_batch(srs_amd_crc_calculator* crc,
                                uint32_t*               d_checksums,
                                const uint8_t*          d_bits,
                                uint32_t                stride,
                                uint32_t                nof_bits,
                                uint32_t                nof_rows,
                                void*                   stream);
/* DEVICE, asynchronous: as above, and the order() CRC bits are written MSB-first
 * into bits [nof_bits, nof_bits + order) of each row. */
int srs_amd_crc_attach_batch(srs_amd_crc_calculator* crc,
                             uint8_t*                d_bits,
                             uint32_t                stride,
                             uint32_t                nof_bits,
                             uint32_t                nof_rows,
                             void*                   stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_CRC_H */
