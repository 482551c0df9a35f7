/*
 * srsran_amd/ulsch_info.h -- UL-SCH / UCI multiplexing geometry of one PUSCH transmission (TS 38.212 6.3.2.4
 * and 6.2.7), the quantities the PUSCH processor, demultiplexer and decoders size themselves by.
 *
 * Replaces (reference interface):
 *   get_ulsch_information(const ulsch_configuration&)   include/srsran/ran/pusch/ulsch_info.h:163
 *       (impl lib/ran/pusch/ulsch_info.cpp:158-358: the HARQ-ACK / CSI part 1 / CSI part 2 RE counts
 *        Q'_ACK, Q'_CSI1, Q'_CSI2 of 6.3.2.4.1.1-3 with and without UL-SCH, the reserved HARQ-ACK REs of
 *        payloads of <= 2 bits, the UL-SCH bits G_SCH and the DC-overlap bits; float arithmetic as the
 *        reference evaluates it)
 * Host only.  Integer results identical to the reference's.
 */
#ifndef SRSRAN_AMD_ULSCH_INFO_H
#define SRSRAN_AMD_ULSCH_INFO_H

#include <stdint.h>

#include "srsran_amd/ldpc.h" /* SRS_AMD_OK / SRS_AMD_EINVAL */

#ifdef __cplusplus
extern "C" {
#endif

/* ulsch_configuration (ulsch_info.h:39-76). */
typedef struct srs_amd_ulsch_config {
  uint32_t tbs;                         /* bits; 0: no UL-SCH */
  int32_t  modulation;                  /* Qm: 1 (BPSK / pi/2-BPSK), 2, 4, 6, 8 */
  float    target_code_rate;            /* R x 1024 (sch_mcs_description) */
  uint32_t nof_harq_ack_bits;
  uint32_t nof_csi_part1_bits;
  uint32_t nof_csi_part2_bits;
  float    alpha_scaling;
  float    beta_offset_harq_ack;
  float    beta_offset_csi_part1;
  float    beta_offset_csi_part2;
  uint32_t nof_rb;
  uint32_t start_symbol_index;
  uint32_t nof_symbols;
  uint32_t dmrs_type;                   /* 1 or 2 */
  uint32_t dmrs_symbol_mask;            /* bit l: OFDM symbol l carries DM-RS */
  uint32_t nof_cdm_groups_without_data;
  uint32_t nof_layers;
  int32_t  contains_dc;
} srs_amd_ulsch_config;

/* ulsch_information (ulsch_info.h:81-103); sch_* = sch_information of the UL-SCH (0 without UL-SCH). */
typedef struct srs_amd_ulsch_info {
  uint32_t nof_ul_sch_bits;
  uint32_t nof_harq_ack_bits;   /* encoded (rate-matched) HARQ-ACK bits */
  uint32_t nof_harq_ack_rvd;    /* bits reserved for HARQ-ACK payloads of <= 2 bits */
  uint32_t nof_csi_part1_bits;  /* encoded */
  uint32_t nof_csi_part2_bits;  /* encoded */
  uint32_t nof_harq_ack_re;
  uint32_t nof_csi_part1_re;
  uint32_t nof_csi_part2_re;
  uint32_t nof_dc_overlap_bits;
  uint32_t sch_tb_crc_size;
  uint32_t sch_base_graph;
  uint32_t sch_nof_cb;
  uint32_t sch_lifting_size;
  uint32_t sch_nof_bits_per_cb;
  uint32_t sch_nof_filler_bits_per_cb;
} srs_amd_ulsch_info;

/* SRS_AMD_EINVAL where the reference asserts (CDM groups, DM-RS symbols outside the allocation, rate). */
int srs_amd_ulsch_information(const srs_amd_ulsch_config* cfg, srs_amd_ulsch_info* info);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_ULSCH_INFO_H */
