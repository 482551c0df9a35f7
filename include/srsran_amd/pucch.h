/*
 * srsran_amd/pucch.h -- C-ABI of the MI355X PUCCH Format 0 detector: for every PDU of a slot, the 12 received REs of
 * each OFDM symbol and receive port correlated with the low-PAPR sequence of every cyclic shift the UCI payload allows
 * (TS 38.213 9.2.3 / 9.2.5 tables), the detection metric (correlation over the residual energy), the best shift's
 * HARQ-ACK / SR bits, validity against the reference's threshold table, and the SINR / RSRP / EPRE measurements.
 *
 * Replaces (reference interface):
 *   pucch_detector::detect(const resource_grid_reader&, const format0_configuration&)
 *       include/srsran/phy/upper/channel_processors/pucch/pucch_detector.h:44-77 (format0_configuration)
 *       (impl lib/phy/upper/channel_processors/pucch/pucch_detector_format0.cpp:124-246: cyclic shift alpha from
 *        include/srsran/phy/upper/pucch_helper.h get_alpha_index, group sequence u = n_id mod 30 without hopping,
 *        low-PAPR sequences of low_papr_sequence_collection_impl.cpp)
 *   the Format 0 branch of pucch_processor::process (pucch_processor_impl.cpp).
 * The slot form detects every PDU of many cells' grids in one launch.  Grids are cbf16 [port][14][nof_subc].
 * Message bits and status equal the reference's; the CSI values are float measurements (tests/test_pucch_gpu.py
 * states the tolerance).
 */
#ifndef SRSRAN_AMD_PUCCH_H
#define SRSRAN_AMD_PUCCH_H

#include <stdint.h>

#include "srsran_amd/ldpc.h" /* SRS_AMD_OK, SRS_AMD_EINVAL, srs_amd_last_error */

#ifdef __cplusplus
extern "C" {
#endif

/* pucch_detector::format0_configuration and the grid it reads. */
typedef struct srs_amd_pucch_f0_pdu {
  uint32_t  numerology;
  uint32_t  slot_index;           /* slot within the frame */
  uint32_t  starting_prb;
  int32_t   second_hop_prb;       /* -1: no frequency hopping */
  uint32_t  start_symbol_index;
  uint32_t  nof_symbols;          /* 1 or 2 */
  uint32_t  initial_cyclic_shift; /* m0, 0 .. 11 */
  uint32_t  n_id;                 /* hopping identity */
  uint32_t  nof_harq_ack;         /* 0 .. 2 */
  uint32_t  sr_opportunity;       /* 0 / 1 */
  uint32_t  nof_ports;            /* 1 .. 4 */
  uint8_t   ports[4];
  uint32_t  grid;                 /* index of the grid in d_grids */
  const uint32_t* d_grid;         /* non-NULL: this PDU's own DEVICE grid instead of d_grids[grid] */
} srs_amd_pucch_f0_pdu;

#define SRS_AMD_UCI_STATUS_VALID 1 /* uci_status (uci_status.h): unknown 0, valid 1, invalid 2 */
#define SRS_AMD_UCI_STATUS_INVALID 2

/* The detector's pucch_uci_message and channel_state_information. */
typedef struct srs_amd_pucch_f0_result {
  uint32_t status;           /* SRS_AMD_UCI_STATUS_* */
  uint32_t nof_sr;           /* 0 / 1 */
  uint32_t nof_harq_ack;
  uint8_t  sr;               /* SR bit */
  uint8_t  harq_ack[2];
  uint8_t  reserved;
  float    detection_metric; /* the best shift's metric (linear) */
  float    sinr_dB;          /* convert_power_to_dB(metric) */
  float    rsrp_dB;
  float    epre_dB;
} srs_amd_pucch_f0_result;

typedef struct srs_amd_pucch_processor srs_amd_pucch_processor;

int  srs_amd_pucch_processor_create(srs_amd_pucch_processor** proc, int device);
void srs_amd_pucch_processor_destroy(srs_amd_pucch_processor* proc);

/* DEVICE, asynchronous: every Format 0 PDU of a slot (several grids) detected into d_results[nof_pdus]. */
int srs_amd_pucch_f0_detect_slot(srs_amd_pucch_processor*    proc,
                                 const srs_amd_pucch_f0_pdu* pdus,
                                 uint32_t                    nof_pdus,
                                 const uint32_t*             d_grids,
                                 uint64_t                    grid_stride,
                                 uint32_t                    nof_grids,
                                 uint32_t                    nof_grid_ports,
                                 uint32_t                    nof_subc,
                                 srs_amd_pucch_f0_result*    d_results,
                                 void*                       stream);

/* HOST, synchronous: one PDU on a host grid [nof_ports][14][nof_subc]. */
int srs_amd_pucch_f0_detect(srs_amd_pucch_processor*    proc,
                            const srs_amd_pucch_f0_pdu* pdu,
                            const uint32_t*             grid,
                            uint32_t                    nof_ports,
                            uint32_t                    nof_subc,
                            srs_amd_pucch_f0_result*    result);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_PUCCH_H */
