/*
 * srsran_amd/uci_decoder.h -- C-ABI of the MI355X UCI decoder: HARQ-ACK / CSI payloads multiplexed on PUSCH.
 *
 * Replaces (reference interface):
 *   uci_decoder::decode(span<uint8_t> message, span<const log_likelihood_ratio> llr, const configuration&)
 *       include/srsran/phy/upper/channel_processors/uci/uci_decoder.h:59
 *       (impl lib/phy/upper/channel_processors/uci/uci_decoder_impl.cpp:30-129:
 *        1-11 bits: short_block_detector_impl::detect (lib/phy/upper/channel_coding/short/
 *          short_block_detector_impl.cpp:160-223: rate dematching by saturated LLR sums, ML detection over the
 *          (32, K) Reed-Muller codewords of TS 38.212 5.3.3.3 / the 1- and 2-bit repetition codes, GLRT threshold);
 *        12-1706 bits: one or two polar codeblocks (TS 38.212 6.3.1.2-6.3.1.4: CRC6 / CRC11, nMax = 10, input
 *          interleaver) through the polar chain of polar.h, CRC check, filler removal)
 * Payload bits one per byte; status SRS_AMD_UCI_VALID / SRS_AMD_UCI_INVALID (uci_status).  Bit-exact.
 */
#ifndef SRSRAN_AMD_UCI_DECODER_H
#define SRSRAN_AMD_UCI_DECODER_H

#include <stdint.h>

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRS_AMD_UCI_UNKNOWN 0
#define SRS_AMD_UCI_VALID 1
#define SRS_AMD_UCI_INVALID 2

typedef struct srs_amd_uci_decoder srs_amd_uci_decoder;

int  srs_amd_uci_decoder_create(srs_amd_uci_decoder** dec, int device);
void srs_amd_uci_decoder_destroy(srs_amd_uci_decoder* dec);

/* DEVICE, asynchronous: nof messages of K payload bits, each from E LLRs (rows of llr_stride bytes), modulation Qm
 * (uci_decoder::configuration::modulation: 0 / 1 BPSK, 2, 4, 6, 8).  Payload bits to d_messages (rows of
 * msg_stride bytes); the status of message i as int32 at (uint8_t*) d_status + i * status_stride. */
int srs_amd_uci_decode_batch(srs_amd_uci_decoder* dec,
                             const int8_t*        d_llrs,
                             uint64_t             llr_stride,
                             uint32_t             E,
                             uint32_t             K,
                             int32_t              modulation,
                             uint8_t*             d_messages,
                             uint64_t             msg_stride,
                             int32_t*             d_status,
                             uint64_t             status_stride,
                             uint32_t             nof,
                             void*                stream);

/* HOST, synchronous: one message; returns the status (>= 0) or an error code (< 0). */
int srs_amd_uci_decode(srs_amd_uci_decoder* dec, uint8_t* message, uint32_t K, const int8_t* llrs, uint32_t E,
                       int32_t modulation);

/* uci_part2_size_description (include/srsran/ran/uci/uci_part2_size_description.h:30-95): at most two entries, each
 * combining at most two CSI part 1 fields (bit offset, width; at most four bits in all) into an index of its map of
 * CSI part 2 sizes. */
typedef struct srs_amd_uci_part2_parameter {
  uint16_t offset; /* bit offset in CSI part 1 */
  uint16_t width;
} srs_amd_uci_part2_parameter;
typedef struct srs_amd_uci_part2_entry {
  uint32_t                    nof_parameters;
  srs_amd_uci_part2_parameter parameters[2];
  uint32_t                    map_size; /* 1 << (sum of the widths) */
  uint16_t                    map[16];
} srs_amd_uci_part2_entry;
typedef struct srs_amd_uci_part2_size_description {
  uint32_t                nof_entries; /* 0: no CSI part 2 */
  srs_amd_uci_part2_entry entries[2];
} srs_amd_uci_part2_size_description;

/* HOST: uci_part2_get_size (lib/ran/uci/uci_part2_size_calculator.cpp:53-89): the CSI part 2 payload size of a decoded
 * CSI part 1 (one bit per byte), each field read MSB first.  Returns the size, or -1 for a field past the payload or
 * a map of the wrong size (the reference asserts). */
int32_t srs_amd_uci_part2_get_size(const uint8_t*                            part1,
                                   uint32_t                                  nof_part1_bits,
                                   const srs_amd_uci_part2_size_description* descr);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_UCI_DECODER_H */
