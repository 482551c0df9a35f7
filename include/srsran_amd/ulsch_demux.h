/*
 * srsran_amd/ulsch_demux.h -- C-ABI of the MI355X UL-SCH demultiplexer: splits the descrambled codeword LLRs of a
 * PUSCH transmission into the UL-SCH, HARQ-ACK and CSI part 1 streams (TS 38.212 6.2.7), reverting the
 * scrambling of the repetition placeholders of 1- and 2-bit UCI payloads.
 *
 * Replaces (reference interface):
 *   ulsch_demultiplex::demultiplex(pusch_decoder_buffer& sch_data, pusch_decoder_buffer& harq_ack,
 *                                  pusch_decoder_buffer& csi_part1, const configuration&)
 *       include/srsran/phy/upper/channel_processors/pusch/ulsch_demultiplex.h:97
 *       (impl lib/phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.cpp:196-590: per OFDM symbol the
 *        reserved HARQ-ACK REs, the HARQ-ACK REs (> 2 bits), the CSI part 1 REs, the UL-SCH REs and the 1/2-bit
 *        HARQ-ACK REs in the reserved set, each chosen every d-th RE; placeholders x / y un-scrambled;
 *        the UL-SCH copy of a 1/2-bit HARQ-ACK RE zeroed)
 * The placement is resolved once per plan on the host into a per-RE table; the device pass reads every
 * codeword LLR once and writes each stream once.  Bit-exact.
 * CSI part 2 (ulsch_demultiplex::set_csi_part2, ulsch_demultiplex_impl.cpp:241-251, 450-472): its size comes from the
 * decoded CSI part 1, and the reference sets it while demultiplexing the OFDM symbol in which CSI part 1 ends, so
 * its REs start in that symbol (every d-th remaining UCI RE, reserved HARQ-ACK REs included; where a 1/2-bit
 * HARQ-ACK shares the RE the CSI part 2 LLRs are zero).  A plan with nof_csi_part2_bits != 0 places it the same way.
 */
#ifndef SRSRAN_AMD_ULSCH_DEMUX_H
#define SRSRAN_AMD_ULSCH_DEMUX_H

#include <stdint.h>

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ulsch_demultiplex::configuration (ulsch_demultiplex.h:48-75) plus the codeword's scrambling c_init
 * (rnti << 15 + n_id, the descrambler's sequence the placeholders revert). */
typedef struct srs_amd_ulsch_demux_config {
  int32_t  modulation;                  /* Qm: 1, 2, 4, 6, 8 */
  uint32_t nof_layers;
  uint32_t nof_prb;
  uint32_t start_symbol_index;
  uint32_t nof_symbols;
  uint32_t nof_harq_ack_rvd;            /* bits (ulsch_information::nof_harq_ack_rvd) */
  uint32_t dmrs_type;                   /* 1 or 2 */
  uint32_t dmrs_symbol_mask;
  uint32_t nof_cdm_groups_without_data;
  uint32_t nof_harq_ack_bits;           /* payload */
  uint32_t nof_enc_harq_ack_bits;       /* rate matched (ulsch_information::nof_harq_ack_bits) */
  uint32_t nof_csi_part1_bits;
  uint32_t nof_enc_csi_part1_bits;
  uint32_t c_init;
  uint32_t nof_csi_part2_bits;          /* payload (0: no CSI part 2) */
  uint32_t nof_enc_csi_part2_bits;      /* rate matched (ulsch_information::nof_csi_part2_bits) */
} srs_amd_ulsch_demux_config;

typedef struct srs_amd_ulsch_demux      srs_amd_ulsch_demux;
typedef struct srs_amd_ulsch_demux_plan srs_amd_ulsch_demux_plan;

int  srs_amd_ulsch_demux_create(srs_amd_ulsch_demux** demux, int device);
void srs_amd_ulsch_demux_destroy(srs_amd_ulsch_demux* demux);

/* Resolves the placement; outputs (optional): codeword bits (all data REs x layers x Qm) and UL-SCH bits. */
int  srs_amd_ulsch_demux_plan_create(srs_amd_ulsch_demux*              demux,
                                     const srs_amd_ulsch_demux_config* cfg,
                                     srs_amd_ulsch_demux_plan**        plan,
                                     uint32_t*                         nof_codeword_bits,
                                     uint32_t*                         nof_sch_bits);
void srs_amd_ulsch_demux_plan_destroy(srs_amd_ulsch_demux_plan* plan);

/* DEVICE, asynchronous: nof_cws codewords (int8 rows of cw_stride bytes) into the UL-SCH rows (sch_stride), the
 * HARQ-ACK rows (ack_stride, nof_enc_harq_ack_bits each) and the CSI part 1 rows (csi1_stride); a stream whose
 * size is zero may be NULL. */
int srs_amd_ulsch_demultiplex_batch(srs_amd_ulsch_demux*            demux,
                                    const srs_amd_ulsch_demux_plan* plan,
                                    const int8_t*                   d_cws,
                                    uint64_t                        cw_stride,
                                    int8_t*                         d_sch,
                                    uint64_t                        sch_stride,
                                    int8_t*                         d_ack,
                                    uint64_t                        ack_stride,
                                    int8_t*                         d_csi1,
                                    uint64_t                        csi1_stride,
                                    uint32_t                        nof_cws,
                                    void*                           stream);

/* HOST, synchronous: one codeword. */
int srs_amd_ulsch_demultiplex(srs_amd_ulsch_demux*            demux,
                              const srs_amd_ulsch_demux_plan* plan,
                              const int8_t*                   codeword,
                              int8_t*                         sch,
                              int8_t*                         ack,
                              int8_t*                         csi1);

/* As srs_amd_ulsch_demultiplex_batch / srs_amd_ulsch_demultiplex, plus the CSI part 2 rows (csi2_stride apart,
 * nof_enc_csi_part2_bits each).  The forms above require a plan without CSI part 2. */
int srs_amd_ulsch_demultiplex_csi2_batch(srs_amd_ulsch_demux*            demux,
                                         const srs_amd_ulsch_demux_plan* plan,
                                         const int8_t*                   d_cws,
                                         uint64_t                        cw_stride,
                                         int8_t*                         d_sch,
                                         uint64_t                        sch_stride,
                                         int8_t*                         d_ack,
                                         uint64_t                        ack_stride,
                                         int8_t*                         d_csi1,
                                         uint64_t                        csi1_stride,
                                         int8_t*                         d_csi2,
                                         uint64_t                        csi2_stride,
                                         uint32_t                        nof_cws,
                                         void*                           stream);
int srs_amd_ulsch_demultiplex_csi2(srs_amd_ulsch_demux*            demux,
                                   const srs_amd_ulsch_demux_plan* plan,
                                   const int8_t*                   codeword,
                                   int8_t*                         sch,
                                   int8_t*                         ack,
                                   int8_t*                         csi1,
                                   int8_t*                         csi2);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_ULSCH_DEMUX_H */
