/*
 * srsran_amd/pusch_processor.h -- C-ABI of the MI355X PUSCH processor: DM-RS
 * channel estimation -> demodulation (equalizer, soft demapper, descrambler)
 * -> UL-SCH decoding (rate dematching, LDPC, CB/TB CRC) of a batch of received
 * slot grids, one transport block per grid.
 *
 * Replaces (reference interface):
 *   pusch_processor::process(span<uint8_t> data, unique_rx_buffer rm_buffer,
 *                            pusch_processor_result_notifier& notifier,
 *                            const resource_grid_reader& grid, const pdu_t& pdu)
 *       include/srsran/phy/upper/channel_processors/pusch/pusch_processor.h:181
 *       (impl lib/phy/upper/channel_processors/pusch/pusch_processor_impl.cpp:134-386)
 *   created as pusch_processor_factory_sw_configuration describes
 *       (include/srsran/phy/upper/channel_processors/pusch/factories.h:107-130).
 *
 * Composition: srs_amd_pusch_chest (pusch_chest.h) -> srs_amd_pusch_demodulator
 * (pusch_demodulator.h) -> srs_amd_pusch_decoder (sch.h), three asynchronous
 * stages on the caller's stream; the processor owns the intermediate channel
 * estimates, port measurements and codeword LLRs in HBM.
 * Derived exactly as pusch_processor_impl does it: DM-RS scaling
 * convert_dB_to_amplitude(-get_sch_to_dmrs_ratio_dB(cdm groups)) (:193),
 * Nref = compute_N_ref(tbs_lbrm, C) (ldpc.h:225), nof_ch_symbols from
 * get_ulsch_information without UCI (all data REs x layers), rb_mask of the
 * type-1 allocation relative to the BWP (:166).
 * Scope: PUSCH with a codeword and, optionally, HARQ-ACK, CSI part 1 and CSI part 2 multiplexed on it
 * (ulsch_demux.h, uci_decoder.h: ulsch_demultiplex_impl + uci_decoder_impl as pusch_processor_impl.cpp:252-334
 * wires them), or UCI only (no codeword, tbs = 0: pusch_processor_impl.cpp:305-324 -- estimator, demodulator,
 * demultiplexer and UCI decoders, no UL-SCH decoding), DM-RS type 1 with the pseudo-random sequence, or transform
 * precoding with the low-PAPR DM-RS (pusch_processor_impl.cpp:172-196, validator :148-174).  The DC subcarrier
 * (pdu.dc_position) of a CP-OFDM PDU has its channel estimate zeroed on every receive port, layer and OFDM symbol of
 * the allocation (pusch_processor_impl.cpp:235-249), so its REs equalize to zero symbols of infinite variance (zero
 * LLRs); transform precoding leaves it untouched, as the reference.  DM-RS type 2 is rejected as the reference's own
 * validator rejects it (pusch_processor_validator_impl.cpp:151-154); the reference PUSCH has no intra-slot frequency
 * hopping.
 */
#ifndef SRSRAN_AMD_PUSCH_PROCESSOR_H
#define SRSRAN_AMD_PUSCH_PROCESSOR_H

#include <stdint.h>

#include "srsran_amd/pusch_chest.h"
#include "srsran_amd/pusch_demodulator.h"
#include "srsran_amd/sch.h"
#include "srsran_amd/uci_decoder.h"

#ifdef __cplusplus
extern "C" {
#endif

/* pusch_processor_factory_sw_configuration (factories.h:107-130) / the components it
 * builds (pusch_processor_benchmark.cpp:133-140, 560-640). */
typedef struct srs_amd_pusch_processor_config {
  uint32_t dec_nof_iterations;    /* LDPC iterations (factory default 10; the benchmark uses 2) */
  int32_t  dec_enable_early_stop; /* CRC early stop */
  int32_t  dec_force_decoding;
  int32_t  equalizer;             /* SRS_AMD_EQ_ZF / SRS_AMD_EQ_MMSE */
  int32_t  fd_smoothing;          /* SRS_AMD_CHEST_FD_* */
  int32_t  td_interpolation;      /* SRS_AMD_CHEST_TD_* */
  int32_t  compensate_cfo;
  int32_t  ldpc_arith;            /* SRS_AMD_ARITH_SIMD ("auto" on x86) or SRS_AMD_ARITH_GENERIC */
} srs_amd_pusch_processor_config;

/* pusch_processor::pdu_t (pusch_processor.h:117-167), data-only subset. */
typedef struct srs_amd_pusch_pdu {
  uint32_t numerology;        /* slot */
  uint32_t slot_index;
  uint32_t rnti;
  uint32_t bwp_start_rb;
  uint32_t bwp_size_rb;
  int32_t  modulation;        /* mcs_descr.modulation as Qm (2, 4, 6, 8) */
  float    target_code_rate;  /* mcs_descr.target_code_rate (R x 1024) */
  uint32_t rv;                /* codeword */
  uint32_t base_graph;        /* 1 or 2 */
  int32_t  new_data;
  uint32_t n_id;
  uint32_t nof_tx_layers;
  uint32_t nof_rx_ports;      /* rx_ports = 0 .. nof_rx_ports - 1 */
  uint32_t dmrs_symbol_mask;
  uint32_t dmrs_type;         /* 1 */
  uint32_t scrambling_id;     /* dmrs_configuration */
  uint32_t n_scid;
  uint32_t nof_cdm_groups_without_data;
  uint32_t rb_start;          /* freq_alloc: type-1 VRBs [rb_start, rb_start + rb_count) of the BWP */
  uint32_t rb_count;
  uint32_t start_symbol_index;
  uint32_t nof_symbols;
  uint32_t tbs_lbrm_bytes;    /* 0: tbs_lbrm_default (159749) */
  uint32_t tbs;               /* transport block size in bits (data.size() * 8) */
  uint32_t transform_precoding; /* dmrs = dmrs_transform_precoding_configuration (DFT-s-OFDM): one layer, valid
                                   PRB count, low-PAPR DM-RS of n_rs_id; dmrs_type / scrambling_id / n_scid /
                                   nof_cdm_groups_without_data are then unused (two CDM groups, as the reference) */
  uint32_t n_rs_id;           /* {0 .. 1007} */
  /* uci_description (pusch_processor.h:64-90): HARQ-ACK and CSI part 1 payloads multiplexed with the UL-SCH
     (0: none), the scaling and beta offsets of TS 38.213 9.3 */
  uint32_t nof_harq_ack;
  uint32_t nof_csi_part1;
  float    alpha_scaling;
  float    beta_offset_harq_ack;
  float    beta_offset_csi_part1;
  /* CSI part 2 (uci_description::csi_part2_size, beta_offset_csi_part2): its size comes from the decoded CSI part 1
     (uci_part2_get_size, pusch_processor_impl.cpp:73-103); no entries: none.  The processor decodes CSI part 1
     first, selects each grid's CSI part 2 size on the device (among every size the description can produce; no host
     synchronisation) and demultiplexes and decodes CSI part 2 and the UL-SCH of each grid with the geometry of that
     size.  (A UCI-only PDU with CSI part 2 has no consistent geometry in the reference -- its CSI part 1 is sized for
     "no CSI part 2", ulsch_info.cpp:96-123 -- and keeps a host readback that fails if a part 2 size is selected.) */
  float                              beta_offset_csi_part2;
  srs_amd_uci_part2_size_description csi_part2_size;
  /* pdu_t::dc_position (pusch_processor.h:161): subcarrier index of the DC within the resource grid (the FAPI PDU's
     tx_direct_current_location, lib/fapi_adaptor/phy/messages/pusch.cpp:150-152); has_dc_position = 0: unset.  A
     position outside the grid changes nothing. */
  uint32_t                           has_dc_position;
  uint32_t                           dc_position;
} srs_amd_pusch_pdu;

/* Per-transport-block results: pusch_decoder_result (sch.h), the UCI statuses and the channel
 * state information channel_estimate::get_channel_state_information derives
 * (channel_estimation.h:244-286): SINR from the channel estimator
 * (layer-0 RSRP summed over ports / noise variances summed over ports), EPRE
 * and RSRP averaged linearly over ports, time alignment of the best-SNR port. */
typedef struct srs_amd_pusch_processor_result {
  srs_amd_pusch_decoder_result data;
  float                        sinr_db;
  float                        epre_db;
  float                        rsrp_db;
  float                        time_alignment_s;
  int32_t                      harq_ack_status;  /* SRS_AMD_UCI_* (uci_decoder.h); 0 without HARQ-ACK */
  int32_t                      csi_part1_status; /* SRS_AMD_UCI_*; 0 without CSI part 1 */
  int32_t                      csi_part2_status; /* SRS_AMD_UCI_*; 0 without CSI part 2 */
  uint32_t                     nof_csi_part2;    /* CSI part 2 payload bits (from the decoded CSI part 1) */
  float                        cfo_hz;           /* CFO of the best-SNR port (channel_estimation.h:273-276); NaN:
                                                    none estimated (one DM-RS symbol or CFO compensation off) */
} srs_amd_pusch_processor_result;

typedef struct srs_amd_pusch_processor      srs_amd_pusch_processor;
typedef struct srs_amd_pusch_processor_plan srs_amd_pusch_processor_plan;

int  srs_amd_pusch_processor_create(srs_amd_pusch_processor**             proc,
                                    const srs_amd_pusch_processor_config* cfg,
                                    int                                   device);
void srs_amd_pusch_processor_destroy(srs_amd_pusch_processor* proc);

/* Resolves a PDU for grids of nof_subc subcarriers (host, once per configuration):
 * estimator configuration, demodulator data-RE table, segmentation plan.
 * Outputs (optional): the UL-SCH plan and the HARQ soft-buffer bytes per TB. */
int  srs_amd_pusch_processor_plan_create(srs_amd_pusch_processor*       proc,
                                         const srs_amd_pusch_pdu*       pdu,
                                         uint32_t                       nof_subc,
                                         srs_amd_pusch_processor_plan** plan,
                                         srs_amd_sch_plan*              sch_plan,
                                         uint64_t*                      soft_buffer_bytes);
void srs_amd_pusch_processor_plan_destroy(srs_amd_pusch_processor_plan* plan);

/* Optional caller-owned DEVICE buffers for the processor's intermediate results
 * (any member NULL: the processor uses its own scratch for that one):
 * channel estimates cbf16 [grid][rx port][layer][14][nof_subc] (est_stride uint32
 * apart), estimator measurements [grid][rx port], codeword LLRs int8 [grid][G]
 * (llr_stride bytes apart). Lets a caller inspect or reuse every stage's output. */
typedef struct srs_amd_pusch_intermediates {
  uint32_t*                 d_estimates;
  uint64_t                  est_stride;
  srs_amd_chest_port_stats* d_port_stats;
  int8_t*                   d_llrs;
  uint32_t                  llr_stride;
  /* UCI payloads (one bit per byte, pusch_processor_result_control::harq_ack / csi_part1): rows of nof_harq_ack /
     nof_csi_part1 bytes, *_stride apart; NULL: not returned (the statuses are in the results either way) */
  uint8_t*                  d_harq_ack;
  uint32_t                  harq_ack_stride;
  uint8_t*                  d_csi_part1;
  uint32_t                  csi_part1_stride;
  /* CSI part 2 payloads: rows of csi_part2_stride bytes (at least the largest size the description allows) */
  uint8_t*                  d_csi_part2;
  uint32_t                  csi_part2_stride;
  /* per-codeblock LDPC iteration counts [grid][C] (C = the plan's codeblocks, contiguous), in codeblock order as
     pusch_decoder_impl fills cb_stats (pusch_decoder_impl.cpp:370-375, 414): the count of the decoding that passed
     the codeblock CRC, or -1 when it failed (the reference's statistic is then nof_ldpc_iterations); codeblocks OK
     from an earlier transmission report their soft-buffer flag value.  NULL: not returned. */
  int32_t*                  d_cb_iterations;
} srs_amd_pusch_intermediates;

/* DEVICE, asynchronous: nof_grids received grids cbf16 [grid][port][14][nof_subc]
 * (grid_stride uint32 apart) -> transport blocks (rows of tb_stride bytes) and
 * d_results[nof_grids]. d_soft: nof_grids HARQ soft buffers (soft_buffer_bytes
 * each, kept between transmissions by the caller) or NULL for new-data-only
 * decoding. io: optional caller buffers for the intermediates (or NULL). */
int srs_amd_pusch_process_batch(srs_amd_pusch_processor*            proc,
                                const srs_amd_pusch_processor_plan* plan,
                                const uint32_t*                     d_grids,
                                uint64_t                            grid_stride,
                                uint32_t                            nof_grids,
                                uint8_t*                            d_tbs,
                                uint32_t                            tb_stride,
                                srs_amd_pusch_processor_result*     d_results,
                                int8_t*                             d_soft,
                                const srs_amd_pusch_intermediates*  io,
                                void*                               stream);

/* One PUSCH PDU of a slot (srs_amd_pusch_process_slot). */
typedef struct srs_amd_pusch_slot_pdu {
  const srs_amd_pusch_processor_plan* plan;       /* a plan of this processor */
  uint32_t                            grid;       /* index of the received grid the PDU occupies in d_grids */
  uint32_t                            cb_offset;  /* index of its first codeblock in io->d_cb_iterations */
  uint64_t                            tb_offset;  /* byte offset of its tbs / 8 transport-block bytes in d_tbs */
  int8_t*                             d_soft;     /* DEVICE HARQ soft buffer (the plan's soft_buffer_bytes), kept by
                                                     the caller between transmissions; NULL: new data, not kept */
  uint64_t                            uci_offset; /* byte offset of its UCI payload row in io->d_uci: HARQ-ACK
                                                     (nof_harq_ack) | CSI part 1 (nof_csi_part1) | CSI part 2 (the
                                                     largest size its description allows), one bit per byte */
  uint32_t                            has_slot;   /* 1: this PDU's slot is (numerology, slot_index) below, whatever
                                                     slot the shared plan was created or last moved to (PDUs of
                                                     different slots may share one plan within a call); 0: the plan's */
  uint32_t                            numerology;
  uint32_t                            slot_index;
  const uint32_t*                     d_grid;     /* non-NULL: this PDU's own DEVICE grid cbf16 [port][14][nof_subc]
                                                     (a device-resident resource grid, receive ports 0 .. P - 1),
                                                     instead of d_grids[grid] */
  uint32_t                            soft_on_failure; /* new data with d_soft: 1 = its soft LLRs are written to
                                                     d_soft only when the decoding leaves the transport block failed
                                                     (the state a retransmission combines with, as an rx_buffer the
                                                     reference would unlock rather than release); messages and CRC
                                                     flags always.  0: every soft LLR written */
} srs_amd_pusch_slot_pdu;

/* Optional outputs of srs_amd_pusch_process_slot_ex (any member NULL: not returned). */
typedef struct srs_amd_pusch_slot_io {
  int32_t* d_cb_iterations; /* per-codeblock iteration counts (as srs_amd_pusch_intermediates), PDU i's C values from
                               pdus[i].cb_offset */
  uint8_t* d_uci;           /* UCI payload rows, PDU i's at pdus[i].uci_offset */
  srs_amd_chest_port_stats* d_port_stats; /* estimator measurements [pdu][4], PDU i's receive ports from 4 * i (the
                                             per-port inputs of channel_estimate::get_channel_state_information) */
} srs_amd_pusch_slot_io;

/* DEVICE, asynchronous: every PUSCH PDU of a slot -- several UEs on disjoint PRBs of one received grid (or of
 * several grids), each with its own PRB range, layers, modulation, DM-RS symbols and scrambling, rnti / n_id
 * and code rate -- as ONE launch sequence.  What uplink_processor_impl::process_pusch
 * (uplink_processor_impl.cpp:270-326) does by calling pusch_processor_impl::process once per PDU.  Result of
 * pdus[i] in d_results[i], transport block at d_tbs + pdus[i].tb_offset; per PDU identical to
 * srs_amd_pusch_process_batch on that PDU's grid.
 * Every PDU whose equalizer kind the fused estimator-equalizer covers runs fused -- data, HARQ processes with a
 * soft buffer (d_soft; early-stop decoding), UCI on PUSCH (HARQ-ACK, CSI part 1, CSI part 2 sized on the device from
 * the decoded CSI part 1), UCI-only PDUs (tbs = 0), transform precoding: one channel-estimator sequence over all of
 * them (per-PDU argument blocks), one fused equalizer-demapper launch per (ports, layers, equalizer) kind, one
 * demultiplexer launch and one UCI decoder set over the UCI PDUs, one slot decoder sequence
 * (srs_amd_pusch_decode_slot) and one result launch.  Other PDUs run in the same call on the same stream through the
 * batch chain of their plan (srs_amd_pusch_process_batch with one grid), before the fused group.  Plans created for
 * the same nof_subc.  No host synchronisation. */
int srs_amd_pusch_process_slot_ex(srs_amd_pusch_processor*        proc,
                                  const srs_amd_pusch_slot_pdu*   pdus,
                                  uint32_t                        nof_pdus,
                                  const uint32_t*                 d_grids,
                                  uint64_t                        grid_stride,
                                  uint32_t                        nof_grids,
                                  uint8_t*                        d_tbs,
                                  srs_amd_pusch_processor_result* d_results,
                                  const srs_amd_pusch_slot_io*    io,
                                  void*                           stream);

/* srs_amd_pusch_process_slot_ex without the optional outputs. */
int srs_amd_pusch_process_slot(srs_amd_pusch_processor*        proc,
                               const srs_amd_pusch_slot_pdu*   pdus,
                               uint32_t                        nof_pdus,
                               const uint32_t*                 d_grids,
                               uint64_t                        grid_stride,
                               uint32_t                        nof_grids,
                               uint8_t*                        d_tbs,
                               srs_amd_pusch_processor_result* d_results,
                               void*                           stream);

/* Moves a plan to another slot (pdu_t::slot): the DM-RS sequences are the only per-slot quantity of a PDU
 * configuration, so a caller keeps one plan per configuration across slots (plan creation uploads tables and
 * synchronises; this does not).  Not while a call that uses the plan is being issued on another thread. */
int srs_amd_pusch_processor_plan_set_slot(srs_amd_pusch_processor_plan* plan, uint32_t numerology,
                                          uint32_t slot_index);

/* The plan's transport block and segmentation: codeblocks C and the CSI part 2 payload row length
 * (srs_amd_pusch_slot_pdu::uci_offset rows: nof_harq_ack + nof_csi_part1 + max_csi_part2 bytes). */
int srs_amd_pusch_processor_plan_info(const srs_amd_pusch_processor_plan* plan, uint32_t* nof_codeblocks,
                                      uint32_t* max_csi_part2, uint64_t* soft_buffer_bytes);

/* HOST, synchronous: one grid [port][14][nof_subc]; tb gets tbs/8 bytes;
 * soft_buffer: HOST HARQ buffer of soft_buffer_bytes (or NULL for new data only). */
int srs_amd_pusch_process(srs_amd_pusch_processor*            proc,
                          const srs_amd_pusch_processor_plan* plan,
                          const uint32_t*                     grid,
                          uint8_t*                            tb,
                          srs_amd_pusch_processor_result*     result,
                          int8_t*                             soft_buffer);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_PUSCH_PROCESSOR_H */
