/*
 * srsran_amd/sch.h -- C-ABI of the MI355X shared-channel (PDSCH / PUSCH) transport
 * block processing: segmentation geometry, the PDSCH encoder and the PUSCH decoder.
 *
 * Replaces:
 *   srs_amd_sch_plan_compute      ldpc_segmenter_tx_impl::new_transmission / ldpc_segmenter_rx_impl::segment
 *                                 (lib/phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.cpp:53-123,
 *                                  ldpc_segmenter_rx_impl.cpp:51-104; TS 38.212 5.2.2 + 5.4.2.1), host only
 *   srs_amd_pdsch_encode(_batch)  pdsch_encoder::encode(span<uint8_t> codeword, span<const uint8_t> transport_block,
 *                                                       const configuration&)
 *                                 include/srsran/phy/upper/channel_processors/pdsch/pdsch_encoder.h:61
 *                                 (pdsch_encoder_impl.cpp: TB CRC, segmentation + CB CRC, LDPC encoding, rate
 *                                  matching, concatenation)
 *   srs_amd_pusch_decode(_batch)  pusch_decoder::new_data + pusch_decoder_buffer softbits + on_end_softbits
 *                                 include/srsran/phy/upper/channel_processors/pusch/pusch_decoder.h:77
 *                                 (pusch_decoder_impl.cpp: segmentation, rate dematching + HARQ combining, LDPC
 *                                  decoding with CB CRC early stop, concatenation, TB CRC check; result as
 *                                  pusch_decoder_result.h)
 * Batches hold nof_tbs transport blocks that share one plan (e.g. the slots of
 * a frame or the cells of a sector group), all device-resident and
 * asynchronous on the caller's HIP stream.
 */
#ifndef SRSRAN_AMD_SCH_H
#define SRSRAN_AMD_SCH_H

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Segmentation geometry of one transport block (segment_parameters, ldpc_segmenter_helpers.h:33). */
typedef struct srs_amd_sch_plan {
  uint32_t tbs;                /* transport block size, bits (multiple of 8) */
  uint32_t base_graph;         /* 1 = BG1, 2 = BG2 */
  uint32_t rv;                 /* redundancy version 0..3 */
  uint32_t modulation_order;   /* Qm: 1, 2, 4, 6, 8 */
  uint32_t Nref;               /* limited-buffer rate matching length, 0 = unlimited */
  uint32_t nof_layers;         /* 1..4 */
  uint32_t nof_ch_symbols;     /* channel symbols (REs x layers) of the codeword */
  /* derived */
  uint32_t lifting_size;       /* Z */
  uint32_t segment_length;     /* K = 22Z (BG1) / 10Z (BG2) */
  uint32_t nof_segments;       /* C */
  uint32_t nof_tb_crc_bits;    /* 16 (TBS <= 3824) or 24 */
  uint32_t nof_crc_bits;       /* codeblock CRC bits: 24 if C > 1, else 0 */
  uint32_t cb_info_bits;       /* segment bits before the CB CRC (the last one includes TB CRC + zero pad) */
  uint32_t zero_pad;           /* zero-padding bits of the last segment */
  uint32_t nof_filler_bits;    /* F */
  uint32_t nof_short_segments; /* segments rate matched to rm_length_short */
  uint32_t rm_length_short;    /* E_r, r < nof_short_segments */
  uint32_t rm_length_long;     /* E_r, r >= nof_short_segments */
  uint32_t cw_length;          /* G = nof_ch_symbols * Qm */
} srs_amd_sch_plan;

/* Fills the derived fields; SRS_AMD_EINVAL where the reference asserts. */
int srs_amd_sch_plan_compute(srs_amd_sch_plan* plan,
                             uint32_t          tbs,
                             uint32_t          base_graph,
                             uint32_t          rv,
                             uint32_t          modulation_order,
                             uint32_t          Nref,
                             uint32_t          nof_layers,
                             uint32_t          nof_ch_symbols);

/* Per-segment rate-matched lengths and codeword offsets (nof_segments entries each, HOST). */
int srs_amd_sch_plan_segments(const srs_amd_sch_plan* plan, uint32_t* rm_lengths, uint32_t* cw_offsets);

/* TS 38.214 5.1.3.2 transport block size: tbs_calculator_calculate
 * (include/srsran/ran/sch/tbs_calculator.h, lib/ran/sch/tbs_calculator.cpp).
 * target_code_rate: R x 1024 (sch_mcs_description::target_code_rate).  0 on invalid input. */
uint32_t srs_amd_tbs_calculate(uint32_t nof_symb_sh,
                               uint32_t nof_dmrs_prb,
                               uint32_t nof_oh_prb,
                               uint32_t modulation_order,
                               float    target_code_rate,
                               uint32_t nof_layers,
                               uint32_t tb_scaling_field,
                               uint32_t n_prb);

/* ---- PDSCH encoder -------------------------------------------------------- */
typedef struct srs_amd_pdsch_encoder srs_amd_pdsch_encoder;

int  srs_amd_pdsch_encoder_create(srs_amd_pdsch_encoder** enc, int device);
void srs_amd_pdsch_encoder_destroy(srs_amd_pdsch_encoder* enc);

/* HOST, synchronous: codeword gets plan->cw_length bits, ONE BIT PER BYTE as the
 * reference's pdsch_encoder::encode; transport_block holds tbs/8 bytes. */
int srs_amd_pdsch_encode(srs_amd_pdsch_encoder* enc, uint8_t* codeword, const uint8_t* transport_block,
                         const srs_amd_sch_plan* plan);

/* DEVICE, asynchronous: nof_tbs transport blocks (rows of tb_stride bytes) into
 * nof_tbs packed codewords (rows of cw_stride >= ceil(G/8) bytes, MSB first). */
int srs_amd_pdsch_encode_batch(srs_amd_pdsch_encoder*  enc,
                               const srs_amd_sch_plan* plan,
                               uint8_t*                d_codewords,
                               uint32_t                cw_stride,
                               const uint8_t*          d_tbs,
                               uint32_t                tb_stride,
                               uint32_t                nof_tbs,
                               void*                   stream);

/* One UE's transport block of a heterogeneous slot batch (srs_amd_pdsch_encode_slot). */
typedef struct srs_amd_pdsch_ue {
  srs_amd_sch_plan plan;      /* computed with srs_amd_sch_plan_compute; any BG / Z / Qm / rv / Nref / TBS */
  uint64_t         tb_offset; /* byte offset of this UE's plan.tbs / 8 transport-block bytes in d_tbs */
  uint64_t         cw_offset; /* byte offset of its packed codeword (ceil(G / 8) bytes, MSB first) in d_codewords */
} srs_amd_pdsch_ue;

/* DEVICE, asynchronous: the transport blocks of nof_ues UEs with DIFFERENT plans (the PDSCH PDUs of one
 * slot, pdsch_processor_impl calling pdsch_encoder::encode once per codeword,
 * pdsch_encoder.h:61) encoded as one launch sequence: TB CRCs, segmentation and codeblock CRCs with
 * per-TB descriptors, one LDPC encoding launch per (base graph, lifting size), one rate-matching launch
 * (per-codeblock geometry).  Each codeword is bit-exact with srs_amd_pdsch_encode_batch of its plan.
 * ues: HOST array.  The codeword bit span of the batch must stay below 2^32 bits. */
int srs_amd_pdsch_encode_slot(srs_amd_pdsch_encoder*  enc,
                              const srs_amd_pdsch_ue* ues,
                              uint32_t                nof_ues,
                              const uint8_t*          d_tbs,
                              uint8_t*                d_codewords,
                              void*                   stream);

/* ---- PUSCH decoder -------------------------------------------------------- */
typedef struct srs_amd_pusch_decoder srs_amd_pusch_decoder;

/* pusch_decoder::configuration fields beyond the plan (pusch_decoder.h:49). */
typedef struct srs_amd_pusch_decoder_config {
  uint32_t nof_ldpc_iterations; /* default 6 */
  int32_t  force_decoding;
  int32_t  use_early_stop;      /* default 1 */
  int32_t  new_data;            /* 1 = first transmission (soft buffers reset) */
} srs_amd_pusch_decoder_config;

/* pusch_decoder_result (pusch_decoder_result.h:31), ldpc statistics flattened. */
typedef struct srs_amd_pusch_decoder_result {
  int32_t  tb_crc_ok;
  uint32_t nof_codeblocks_total;
  uint32_t ldpc_iterations_sum;  /* over all codeblocks; failed ones count nof_ldpc_iterations */
  uint32_t ldpc_iterations_min;
  uint32_t ldpc_iterations_max;
  uint32_t nof_codeblocks_crc_ok;
} srs_amd_pusch_decoder_result;

/* arith: SRS_AMD_ARITH_SIMD / SRS_AMD_ARITH_GENERIC (LDPC decoder rounding, as srs_amd_ldpc_decoder_create). */
int  srs_amd_pusch_decoder_create(srs_amd_pusch_decoder** dec, int arith, int device);
void srs_amd_pusch_decoder_destroy(srs_amd_pusch_decoder* dec);

/* Bytes of device soft buffer one transport block of this plan needs (HARQ rx_buffer). */
uint64_t srs_amd_pusch_soft_buffer_size(const srs_amd_sch_plan* plan);

/* Layout of the soft buffer: C rows of row_bytes, codeblock c at c * row_bytes holding its N = 66 Z (BG1) / 50 Z
 * (BG2) rate-dematched LLRs (rx_buffer::get_codeblock_soft_bits, int8 log_likelihood_ratio) at 0, its decoded
 * message (rx_buffer::get_codeblock_data_bits: K bits packed MSB first, as bit_buffer) at msg_offset and an int32
 * flag at flag_offset: the LDPC iteration count of the decoding that passed the codeblock CRC, 0 while it has not
 * (rx_buffer::get_codeblocks_crc).  A caller mirroring the reference's rx_buffer copies these three fields. */
int srs_amd_pusch_soft_buffer_layout(const srs_amd_sch_plan* plan, uint32_t* row_bytes, uint32_t* nof_llrs,
                                     uint32_t* msg_offset, uint32_t* flag_offset);

/* LLRs per soft-buffer row the LDPC decoder scans after rate dematching this plan's codeblocks
 * (the rest of the row is provably zero): the whole row unless new data with k0 = 0 and no
 * circular wrap lands in a fresh buffer (fresh != 0) or covers the information bits of a
 * full-length buffer; then max(E + F, (K_bg - 2) Z) rounded up to whole Z nodes.  The reference
 * decoder trims its input at the last non-zero LLR the same way (ldpc_decoder_impl.cpp:86). */
uint32_t srs_amd_pusch_decoder_llr_prefix(const srs_amd_sch_plan* plan, int new_data, int fresh);

/* HOST, synchronous: one codeword of plan->cw_length LLRs -> transport block
 * (tbs/8 bytes, written only where the reference writes it) + result.
 * soft_buffer: HOST HARQ buffer of srs_amd_pusch_soft_buffer_size() bytes, kept
 * between transmissions by the caller. */
int srs_amd_pusch_decode(srs_amd_pusch_decoder*              dec,
                         uint8_t*                            transport_block,
                         srs_amd_pusch_decoder_result*       result,
                         const int8_t*                       llrs,
                         int8_t*                             soft_buffer,
                         const srs_amd_sch_plan*             plan,
                         const srs_amd_pusch_decoder_config* cfg);

/* DEVICE, asynchronous: nof_tbs codewords (LLR rows of llr_stride bytes) ->
 * transport blocks (rows of tb_stride bytes) + d_results[nof_tbs].
 * d_soft: nof_tbs soft buffers of srs_amd_pusch_soft_buffer_size() bytes each
 * (device), or NULL for new_data-only decoding with internal buffers.
 * d_cb_iterations: optional nof_tbs * C int32 (iterations, -1 = CRC failed). */
int srs_amd_pusch_decode_batch(srs_amd_pusch_decoder*              dec,
                               const srs_amd_sch_plan*             plan,
                               const srs_amd_pusch_decoder_config* cfg,
                               uint8_t*                            d_tbs,
                               uint32_t                            tb_stride,
                               srs_amd_pusch_decoder_result*       d_results,
                               const int8_t*                       d_llrs,
                               uint32_t                            llr_stride,
                               int8_t*                             d_soft,
                               int32_t*                            d_cb_iterations,
                               uint32_t                            nof_tbs,
                               void*                               stream);

/* One UE's transport block of a heterogeneous slot batch (srs_amd_pusch_decode_slot). */
typedef struct srs_amd_pusch_ue {
  srs_amd_sch_plan plan;       /* computed with srs_amd_sch_plan_compute; any BG / Z / Qm / rv / Nref / TBS */
  uint64_t         llr_offset; /* byte offset of this UE's plan.cw_length LLRs in d_llrs */
  uint64_t         tb_offset;  /* byte offset of this UE's plan.tbs / 8 transport-block bytes in d_tbs */
} srs_amd_pusch_ue;

/* DEVICE, asynchronous: the new transmissions of nof_ues UEs with DIFFERENT plans (the PUSCH
 * allocations of one slot: PRBs, MCS, layers, rv differ per UE), decoded as one launch sequence
 * rather than one per UE -- what pusch_decoder_impl::new_data does once per PUSCH PDU of the slot
 * (pusch_decoder_impl.cpp:89, called per PDU at pusch_processor_impl.cpp:343).  ues: HOST array; the codeword
 * LLRs of UE u start at d_llrs + ues[u].llr_offset, its transport block is written at
 * d_tbs + ues[u].tb_offset and its result to d_results[u].  Semantics per UE identical to
 * srs_amd_pusch_decode_batch with new_data = 1 and internal soft buffers: cfg->new_data must be 1
 * (HARQ retransmissions keep their caller soft buffers through srs_amd_pusch_decode_batch).
 * One rate-dematching launch over every codeblock of the slot (per-codeblock geometry), one
 * LDPC decoding launch per (base graph, lifting size, CRC, bounded LLR prefix) bucket, one assembly sequence
 * (per-TB descriptors).  The LLR span of the batch must stay below 2^32 bytes. */
int srs_amd_pusch_decode_slot(srs_amd_pusch_decoder*              dec,
                              const srs_amd_pusch_decoder_config* cfg,
                              const srs_amd_pusch_ue*             ues,
                              uint32_t                            nof_ues,
                              const int8_t*                       d_llrs,
                              uint8_t*                            d_tbs,
                              srs_amd_pusch_decoder_result*       d_results,
                              void*                               stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_SCH_H */
