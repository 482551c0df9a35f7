/*
 * srsran_amd/pusch_demodulator.h -- C-ABI of the MI355X PUSCH demodulator:
 * data-RE extraction around the DM-RS, channel equalization, soft demapping
 * and descrambling of a batch of slot grids into codeword LLRs.
 *
 * Replaces (reference interface):
 *   pusch_demodulator::demodulate(pusch_codeword_buffer&, pusch_demodulator_notifier&,
 *                                 const resource_grid_reader&, const channel_estimate&,
 *                                 const configuration&)
 *       include/srsran/phy/upper/channel_processors/pusch/pusch_demodulator.h:95
 *       (impl lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.cpp:203-330)
 *
 * Scope: transform precoding (DFT-s-OFDM, pusch_demodulator_impl.cpp:344-351: equalized symbols ->
 * transform_precoding.h deprecoder -> demapper), no UCI multiplexing (the codeword is all
 * UL-SCH), the equalizers of equalizer.h: the open-source reference's (ZF 1 layer x
 * {1,2,4} ports, ZF 2 layers x {2,4} ports, MMSE 1 layer) and the L-layer ZF 3x4 / 4x4 and
 * MMSE 2x2 / 2x4 / 3x4 / 4x4 solves (parity unpinned). The post-equalization SINR / EVM
 * statistics are not produced.
 * Inputs per grid: the received grid cbf16 [port][14][subc], the channel
 * estimates cbf16 [port][layer][14][subc] and per-port measurements
 * (srs_amd_chest_port_stats, the noise variances) from the DM-RS estimator
 * (pusch_chest.h). Output: int8 LLRs in codeword order (RE-major, layer,
 * bit), descrambled (c_init = rnti * 2^15 + n_id).
 * Numerics: equalizer as equalizer.h (float tolerance); soft demapper as
 * modulation.h; LLRs agree with the reference within one quantisation step.
 */
#ifndef SRSRAN_AMD_PUSCH_DEMODULATOR_H
#define SRSRAN_AMD_PUSCH_DEMODULATOR_H

#include <stdint.h>

#include "srsran_amd/equalizer.h"
#include "srsran_amd/pdsch_modulator.h"
#include "srsran_amd/pusch_chest.h"

#ifdef __cplusplus
extern "C" {
#endif

/* pusch_demodulator::configuration (pusch_demodulator.h:51-80). */
typedef struct srs_amd_pusch_demod_config {
  uint32_t rnti;
  uint32_t n_id;
  int32_t  modulation;                 /* Qm code (modulation.h) */
  uint8_t  crb_mask[SRS_AMD_CRB_MASK_BYTES]; /* rb_mask */
  uint8_t  reserved0;
  uint32_t start_symbol;
  uint32_t nof_symbols;
  uint32_t dmrs_symbol_mask;           /* dmrs_symb_pos */
  uint32_t dmrs_type;                  /* 1 or 2 */
  uint32_t nof_cdm_groups_without_data;
  uint32_t nof_tx_layers;              /* 1 to 4 (no more than nof_rx_ports) */
  uint32_t nof_rx_ports;               /* 1, 2 or 4 */
  int32_t  equalizer;                  /* SRS_AMD_EQ_ZF or SRS_AMD_EQ_MMSE */
  uint32_t transform_precoding;        /* enable_transform_precoding: DFT-s-OFDM, one layer, every data OFDM
                                          symbol 12 x M_rb REs with M_rb valid (transform_precoding.h) */
} srs_amd_pusch_demod_config;

typedef struct srs_amd_pusch_demodulator srs_amd_pusch_demodulator;
typedef struct srs_amd_pusch_demod_plan  srs_amd_pusch_demod_plan;

int  srs_amd_pusch_demodulator_create(srs_amd_pusch_demodulator** dem, int device);
void srs_amd_pusch_demodulator_destroy(srs_amd_pusch_demodulator* dem);

/* Resolves the data REs of a configuration for grids of nof_subc subcarriers;
 * *nof_re = data REs per layer, the codeword holds nof_re * layers * Qm LLRs. */
int  srs_amd_pusch_demod_plan_create(srs_amd_pusch_demodulator*        dem,
                                     const srs_amd_pusch_demod_config* cfg,
                                     uint32_t                          nof_subc,
                                     srs_amd_pusch_demod_plan**        plan,
                                     uint32_t*                         nof_re);
void srs_amd_pusch_demod_plan_destroy(srs_amd_pusch_demod_plan* plan);

/* HOST, synchronous: one grid. llrs gets nof_re * layers * Qm values. */
int srs_amd_pusch_demodulate(srs_amd_pusch_demodulator*      dem,
                             const srs_amd_pusch_demod_plan* plan,
                             const uint32_t*                 grid,
                             const uint32_t*                 estimates,
                             const srs_amd_chest_port_stats* stats,
                             int8_t*                         llrs);

/* DEVICE, asynchronous: nof_grids grids; stats [nof_grids][nof_rx_ports]. */
int srs_amd_pusch_demodulate_batch(srs_amd_pusch_demodulator*      dem,
                                   const srs_amd_pusch_demod_plan* plan,
                                   const uint32_t*                 d_grids,
                                   uint64_t                        grid_stride,
                                   const uint32_t*                 d_estimates,
                                   uint64_t                        est_stride,
                                   const srs_amd_chest_port_stats* d_stats,
                                   int8_t*                         d_llrs,
                                   uint64_t                        llr_stride,
                                   uint32_t                        nof_grids,
                                   void*                           stream);

/* DEVICE, asynchronous: the demodulator's last two steps alone -- soft demapping
 * (one demapper call per OFDM symbol, pusch_demodulator_impl.cpp:363-400) and
 * revert_scrambling (:36-190) -- of equalized symbols produced elsewhere (a custom
 * MIMO detector, or the reference's own equalizer). d_eq_symbols complex float
 * [grid][nof_re][layer] (interleaved re/im), d_eq_noise_vars float
 * [grid][nof_re][layer], both with a per-grid stride of nof_re * layers entries;
 * LLRs as srs_amd_pusch_demodulate_batch. */
int srs_amd_pusch_demap_descramble_batch(srs_amd_pusch_demodulator*      dem,
                                         const srs_amd_pusch_demod_plan* plan,
                                         const float*                    d_eq_symbols,
                                         const float*                    d_eq_noise_vars,
                                         int8_t*                         d_llrs,
                                         uint64_t                        llr_stride,
                                         uint32_t                        nof_grids,
                                         void*                           stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_PUSCH_DEMODULATOR_H */
