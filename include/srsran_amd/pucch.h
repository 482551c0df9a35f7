/*
 * srsran_amd/pucch.h -- C-ABI of the MI355X PUCCH Format 0 and Format 1 detectors.
 *
 * Format 0: for every PDU of a slot, the 12 received REs of each OFDM symbol and receive port correlated with the
 * low-PAPR sequence of every cyclic shift the UCI payload allows (TS 38.213 9.2.3 / 9.2.5 tables), the detection
 * metric (correlation over the residual energy), the best shift's HARQ-ACK / SR bits, validity against the
 * reference's threshold table, and the SINR / RSRP / EPRE measurements.
 *
 * Format 1: for every batch of a slot (the PUCCHs multiplexed on one PRB / symbol allocation by initial cyclic shift
 * and time-domain OCC), per hop the received REs matched to the base sequence and despread by a 12-point DFT, per OCC
 * in use the OCC combination of data and DM-RS symbols, the per-shift channel estimates (shifts 10 dB below the
 * strongest dropped), the noise from the DM-RS minus its reconstruction, and per multiplexed PUCCH the BPSK / QPSK
 * symbol, the detection metric against the reference's threshold and the CSI.
 *
 * Format 2: for every PDU of a slot, the DM-RS channel estimate of every receive port (port_channel_estimator_average
 * with the frequency-domain filter, time-domain averaging and CFO compensation, per hop), ZF equalization of the data
 * REs over the ports, QPSK soft demapping, descrambling, and the UCI decoder (short block or polar) -- payload bits,
 * status and the CSI (SINR, RSRP, EPRE, time alignment, CFO).
 *
 * Formats 3 and 4 (DFT-s-OFDM): per port the estimate from the low-PAPR DM-RS symbols (filter, averaging, CFO
 * measured but not compensated), per data symbol ZF equalization and transform deprecoding (IDFT of 12 nof_prb points,
 * mean noise), Format 4's inverse block-wise spreading (OCC of length 2 / 4), QPSK or pi/2-BPSK demapping,
 * descrambling, and the UCI decoder.
 *
 * Replaces (reference interface):
 *   pucch_detector::detect(const resource_grid_reader&, const format0_configuration&)
 *       include/srsran/phy/upper/channel_processors/pucch/pucch_detector.h:44-77 (format0_configuration)
 *       (impl lib/phy/upper/channel_processors/pucch/pucch_detector_format0.cpp:124-246: cyclic shift alpha from
 *        include/srsran/phy/upper/pucch_helper.h get_alpha_index, group sequence u = n_id mod 30 without hopping,
 *        low-PAPR sequences of low_papr_sequence_collection_impl.cpp)
 *   the Format 0 branch of pucch_processor::process (pucch_processor_impl.cpp).
 *   pucch_detector::detect(const resource_grid_reader&, const format1_configuration&, const pucch_format1_map<unsigned>&)
 *       pucch_detector.h:86-118, 155-160 (impl pucch_detector_format1.cpp:156-663, OCCs of
 *       include/srsran/phy/upper/pucch_orthogonal_sequence.h), and
 *   pucch_processor::process(const resource_grid_reader&, const format1_batch_configuration&)
 *       pucch_processor_impl.cpp:74-138.
 *   pucch_processor::process(const resource_grid_reader&, const format2_configuration&)
 *       pucch_processor_impl.cpp:140-220 (dmrs_pucch_estimator_format2.cpp, port_channel_estimator_average_impl.cpp
 *       with filter / average / CFO compensation as signal_processors/pucch/factories.cpp:52-56 builds it,
 *       pucch_demodulator_format2.cpp with the ZF equalizer of upper_phy_factories.cpp:676-677,
 *       uci_decoder_impl.cpp).  The reference's demodulator reads grid ports 0 .. n-1 while its estimator reads
 *       ports[]; here both read ports[] (identical when ports[] = 0 .. n-1).
 * The slot forms detect every PDU / batch of many cells' grids in one launch.  Grids are cbf16 [port][14][nof_subc].
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

/* The detector's pucch_uci_message and channel_state_information (both formats). */
typedef struct srs_amd_pucch_result {
  uint32_t status;           /* SRS_AMD_UCI_STATUS_* */
  uint32_t nof_sr;           /* 0 / 1 */
  uint32_t nof_harq_ack;
  uint8_t  sr;               /* SR bit */
  uint8_t  harq_ack[2];
  uint8_t  reserved;
  float    detection_metric; /* F0: the best shift's metric (linear); F1: the metric over the threshold */
  float    sinr_dB;          /* F0: convert_power_to_dB(metric); F1: RSRP over the noise variance */
  float    rsrp_dB;
  float    epre_dB;
} srs_amd_pucch_result;
typedef srs_amd_pucch_result srs_amd_pucch_f0_result;

/* One multiplexed Format 1 PUCCH of a batch (an entry of format1_batch_configuration / pucch_format1_map<unsigned>). */
typedef struct srs_amd_pucch_f1_entry {
  uint8_t initial_cyclic_shift; /* 0 .. 11 */
  uint8_t time_domain_occ;      /* 0 .. 6, below nof_symbols / 2 (/ 4 with frequency hopping) */
  uint8_t nof_harq_ack;         /* 0 (SR only) .. 2 */
  uint8_t reserved;
} srs_amd_pucch_f1_entry;

/* pucch_detector::format1_configuration with the batch's entries.  The reference detector reads grid ports 0 ..
 * nof_ports - 1 of the reader it is given (pucch_detector_format1.cpp:568-583); here the PDU's ports[] name them. */
typedef struct srs_amd_pucch_f1_batch {
  uint32_t numerology;
  uint32_t slot_index;
  uint32_t starting_prb;
  int32_t  second_hop_prb;        /* -1: no frequency hopping */
  uint32_t start_symbol_index;    /* 0 .. 10 */
  uint32_t nof_symbols;           /* 4 .. 14 */
  uint32_t n_id;
  uint32_t nof_ports;             /* 1, 2 or 4 */
  uint8_t  ports[4];
  uint32_t nof_entries;           /* 1 .. 84, no two with the same (shift, OCC) */
  const srs_amd_pucch_f1_entry* entries;
  uint32_t grid;                  /* index of the grid in d_grids */
  const uint32_t* d_grid;         /* non-NULL: this batch's own DEVICE grid instead of d_grids[grid] */
} srs_amd_pucch_f1_batch;

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

/* pucch_processor::format2_configuration (pucch_processor.h:223-275). */
typedef struct srs_amd_pucch_f2_pdu {
  uint32_t numerology;
  uint32_t slot_index;
  uint32_t bwp_start_rb;
  uint32_t bwp_size_rb;
  uint32_t starting_prb;        /* within the BWP */
  int32_t  second_hop_prb;      /* within the BWP; -1: no frequency hopping */
  uint32_t nof_prb;             /* 1 .. 16 */
  uint32_t start_symbol_index;
  uint32_t nof_symbols;         /* 1 or 2 */
  uint32_t rnti;
  uint32_t n_id;                /* data scrambling identity */
  uint32_t n_id_0;              /* DM-RS scrambling identity */
  uint32_t nof_harq_ack;
  uint32_t nof_sr;
  uint32_t nof_csi_part1;
  uint32_t nof_csi_part2;       /* must be 0, as the reference's validator requires */
  uint32_t nof_ports;           /* 1 .. 4 */
  uint8_t  ports[4];
  uint32_t grid;                /* index of the grid in d_grids */
  const uint32_t* d_grid;       /* non-NULL: this PDU's own DEVICE grid instead of d_grids[grid] */
} srs_amd_pucch_f2_pdu;

/* pucch_processor_result of Formats 2 / 3 / 4: the UCI status and the CSI; the payload bits (HARQ-ACK, SR, CSI part 1,
 * CSI part 2, one per byte) go to a separate row. */
typedef struct srs_amd_pucch_uci_result {
  uint32_t status;              /* SRS_AMD_UCI_STATUS_* */
  uint32_t nof_harq_ack;
  uint32_t nof_sr;
  uint32_t nof_csi_part1;
  uint32_t nof_csi_part2;
  float    sinr_dB;
  float    rsrp_dB;
  float    epre_dB;
  float    time_alignment_s;    /* phy_time_unit of the best-SNR port, in seconds */
  float    cfo_Hz;              /* NaN: not measured */
} srs_amd_pucch_uci_result;

/* DEVICE, asynchronous: every Format 2 PDU of a slot; result i to d_results[i], its payload bits to
 * d_payloads + i * payload_stride. */
int srs_amd_pucch_f2_process_slot(srs_amd_pucch_processor*    proc,
                                  const srs_amd_pucch_f2_pdu* pdus,
                                  uint32_t                    nof_pdus,
                                  const uint32_t*             d_grids,
                                  uint64_t                    grid_stride,
                                  uint32_t                    nof_grids,
                                  uint32_t                    nof_grid_ports,
                                  uint32_t                    nof_subc,
                                  srs_amd_pucch_uci_result*   d_results,
                                  uint8_t*                    d_payloads,
                                  uint64_t                    payload_stride,
                                  void*                       stream);

/* HOST, synchronous: one PDU on a host grid [nof_ports][14][nof_subc]; payload[nof bits]. */
int srs_amd_pucch_f2_process(srs_amd_pucch_processor*    proc,
                             const srs_amd_pucch_f2_pdu* pdu,
                             const uint32_t*             grid,
                             uint32_t                    nof_ports,
                             uint32_t                    nof_subc,
                             srs_amd_pucch_uci_result*   result,
                             uint8_t*                    payload);

/* pucch_processor::format3_configuration / format4_configuration (pucch_processor.h:277-394). */
typedef struct srs_amd_pucch_f34_pdu {
  uint32_t format;              /* 3 or 4 */
  uint32_t numerology;
  uint32_t slot_index;
  uint32_t bwp_start_rb;
  uint32_t bwp_size_rb;
  uint32_t starting_prb;        /* within the BWP */
  int32_t  second_hop_prb;      /* within the BWP; -1: no frequency hopping */
  uint32_t nof_prb;             /* Format 3: 1 .. 16 with 2^a 3^b 5^c PRBs; Format 4: 1 */
  uint32_t start_symbol_index;
  uint32_t nof_symbols;         /* 4 .. 14 */
  uint32_t rnti;
  uint32_t n_id_hopping;        /* DM-RS sequence group / cyclic-shift hopping identity */
  uint32_t n_id_scrambling;     /* data scrambling identity */
  uint32_t nof_harq_ack;
  uint32_t nof_sr;
  uint32_t nof_csi_part1;
  uint32_t nof_csi_part2;       /* must be 0 */
  uint32_t additional_dmrs;     /* 0 / 1 */
  uint32_t pi2_bpsk;            /* 0: QPSK, 1: pi/2-BPSK */
  uint32_t occ_index;           /* Format 4 */
  uint32_t occ_length;          /* Format 4: 2 or 4 */
  uint32_t nof_ports;           /* 1 .. 4 */
  uint8_t  ports[4];
  uint32_t grid;
  const uint32_t* d_grid;
} srs_amd_pucch_f34_pdu;

/* DEVICE, asynchronous: every Format 3 / 4 PDU of a slot; result i to d_results[i], its payload bits to
 * d_payloads + i * payload_stride. */
int srs_amd_pucch_f34_process_slot(srs_amd_pucch_processor*     proc,
                                   const srs_amd_pucch_f34_pdu* pdus,
                                   uint32_t                     nof_pdus,
                                   const uint32_t*              d_grids,
                                   uint64_t                     grid_stride,
                                   uint32_t                     nof_grids,
                                   uint32_t                     nof_grid_ports,
                                   uint32_t                     nof_subc,
                                   srs_amd_pucch_uci_result*    d_results,
                                   uint8_t*                     d_payloads,
                                   uint64_t                     payload_stride,
                                   void*                        stream);

/* HOST, synchronous: one Format 3 / 4 PDU; payload[nof bits]. */
int srs_amd_pucch_f34_process(srs_amd_pucch_processor*     proc,
                              const srs_amd_pucch_f34_pdu* pdu,
                              const uint32_t*              grid,
                              uint32_t                     nof_ports,
                              uint32_t                     nof_subc,
                              srs_amd_pucch_uci_result*    result,
                              uint8_t*                     payload);

/* HOST, synchronous: estimator + pucch_demodulator (format3 / format4, pucch_demodulator_format3.cpp /
 * pucch_demodulator_format4.cpp) of one PDU -- the descrambled LLRs. */
int srs_amd_pucch_f34_demodulate(srs_amd_pucch_processor*     proc,
                                 const srs_amd_pucch_f34_pdu* pdu,
                                 const uint32_t*              grid,
                                 uint32_t                     nof_ports,
                                 uint32_t                     nof_subc,
                                 int8_t*                      llrs);

/* HOST, synchronous: the estimator and demodulator of one Format 2 PDU -- pucch_demodulator::demodulate
 * (pucch_demodulator.h, impl pucch_demodulator_format2.cpp:92-160) after dmrs_pucch_estimator::estimate --
 * llrs[16 nof_prb nof_symbols], descrambled. */
int srs_amd_pucch_f2_demodulate(srs_amd_pucch_processor*    proc,
                                const srs_amd_pucch_f2_pdu* pdu,
                                const uint32_t*             grid,
                                uint32_t                    nof_ports,
                                uint32_t                    nof_subc,
                                int8_t*                     llrs);

/* DEVICE, asynchronous: every Format 1 batch of a slot detected; the result of entry e of batch b goes to
 * d_results[nof_entries(0) + ... + nof_entries(b - 1) + e]. */
int srs_amd_pucch_f1_detect_slot(srs_amd_pucch_processor*      proc,
                                 const srs_amd_pucch_f1_batch* batches,
                                 uint32_t                      nof_batches,
                                 const uint32_t*               d_grids,
                                 uint64_t                      grid_stride,
                                 uint32_t                      nof_grids,
                                 uint32_t                      nof_grid_ports,
                                 uint32_t                      nof_subc,
                                 srs_amd_pucch_result*         d_results,
                                 void*                         stream);

/* HOST, synchronous: one batch on a host grid [nof_ports][14][nof_subc], results[batch->nof_entries]. */
int srs_amd_pucch_f1_detect(srs_amd_pucch_processor*      proc,
                            const srs_amd_pucch_f1_batch* batch,
                            const uint32_t*               grid,
                            uint32_t                      nof_ports,
                            uint32_t                      nof_subc,
                            srs_amd_pucch_result*         results);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_PUCCH_H */
