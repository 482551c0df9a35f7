/*
 * srsran_amd/pusch_chest.h -- C-ABI of the MI355X PUSCH DM-RS channel estimator.
 *
 * Replaces (reference interface):
 *   dmrs_pusch_estimator::estimate(channel_estimate&, dmrs_pusch_estimator_notifier&,
 *                                  const resource_grid_reader&, const configuration&)
 *       include/srsran/phy/upper/signal_processors/pusch/dmrs_pusch_estimator.h:135
 *       (impl lib/phy/upper/signal_processors/pusch/dmrs_pusch_estimator_impl.cpp:28-184 with
 *        port_channel_estimator_average_impl.cpp, the channel estimator the PUSCH processor uses)
 *
 * Scope: pseudo-random DM-RS sequence or, with transform precoding, the low-PAPR
 * sequence (low_papr = 1: one layer, include/srsran_amd/low_papr.h), DM-RS type 1,
 * 1..4 layers, 1..4 DM-RS symbols, one hop (the reference's PUSCH estimator has no
 * hopping: dmrs_pusch_estimator::configuration carries one rb_mask and
 * dmrs_pusch_estimator_impl.cpp:177-180 never sets a hopping symbol),
 * contiguous PRB allocation, all smoothing / interpolation / CFO options of
 * port_channel_estimator_average_impl. Type 2 is rejected: the reference's
 * linear interpolator reads past its pilot buffer for that pattern
 * (interpolator_linear_impl.cpp:103-113). Non-contiguous allocations are
 * rejected: the reference maps every PRB of one at the allocation start
 * (port_channel_estimator_average_impl.cpp:330-343).
 *
 * Grids: complex bf16 [port][symbol (14)][subcarrier] (uint32, real in the low
 * half). Estimates: complex bf16 [port][layer][symbol (14)][subcarrier]; the
 * REs of the allocation (symbols first_symbol .. first_symbol + nof_symbols - 1,
 * the allocated PRBs) are written; with CFO compensation the reference also
 * rotates the rest of those OFDM symbols in place (it multiplies whole symbol
 * spans, port_channel_estimator_average_impl.cpp:184-193), and so does this.
 */
#ifndef SRSRAN_AMD_PUSCH_CHEST_H
#define SRSRAN_AMD_PUSCH_CHEST_H

#include <stdint.h>

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* port_channel_estimator_fd_smoothing_strategy / _td_interpolation_strategy
 * (port_channel_estimator_parameters.h:28-43), same values. */
#define SRS_AMD_CHEST_FD_NONE 0
#define SRS_AMD_CHEST_FD_MEAN 1
#define SRS_AMD_CHEST_FD_FILTER 2
#define SRS_AMD_CHEST_TD_INTERPOLATE 0
#define SRS_AMD_CHEST_TD_AVERAGE 1

/* dmrs_pusch_estimator::configuration (dmrs_pusch_estimator.h:73-112) with the
 * estimator-construction options (port_channel_estimator_average_impl.h:59-63). */
typedef struct srs_amd_pusch_chest_config {
  uint32_t numerology;       /* slot.numerology() */
  uint32_t slot_index;       /* slot.slot_index() */
  uint32_t scrambling_id;
  uint32_t n_scid;
  uint32_t nof_tx_layers;    /* 1..4 */
  float    scaling;          /* DM-RS-to-data amplitude gain, > 0 */
  uint32_t symbols_mask;     /* OFDM symbols carrying DM-RS */
  uint32_t rb_start;         /* contiguous rb_mask */
  uint32_t rb_count;
  uint32_t first_symbol;
  uint32_t nof_symbols;
  int32_t  fd_smoothing;     /* SRS_AMD_CHEST_FD_* (PUSCH default: filter) */
  int32_t  td_interpolation; /* SRS_AMD_CHEST_TD_* (PUSCH default: average) */
  int32_t  compensate_cfo;   /* default 1 */
  int32_t  low_papr;         /* transform precoding: low_papr_sequence_configuration (dmrs_pusch_estimator.h:67-77),
                                one layer, sequence group n_rs_id mod 30, no scrambling_id / n_scid */
  uint32_t n_rs_id;          /* {0 .. 1007} */
} srs_amd_pusch_chest_config;

/* channel_estimate per-port measurements (channel_estimation.h:125-190); rsrp,
 * time alignment and CFO are the same for every layer of a port. */
typedef struct srs_amd_chest_port_stats {
  float noise_var;
  float epre;
  float rsrp;
  float snr;
  float time_alignment_s; /* phy_time_unit resolution (Tc) as the reference */
  float cfo_hz;           /* NaN when the reference has no CFO (one DM-RS symbol) */
} srs_amd_chest_port_stats;

typedef struct srs_amd_pusch_chest srs_amd_pusch_chest;

int  srs_amd_pusch_chest_create(srs_amd_pusch_chest** chest, int device);
void srs_amd_pusch_chest_destroy(srs_amd_pusch_chest* chest);

/* HOST, synchronous: grid [nof_ports][14][nof_subc]; estimates [nof_ports][layers][14][nof_subc]
 * (in/out); stats [nof_ports]. */
int srs_amd_pusch_chest_estimate(srs_amd_pusch_chest*              chest,
                                 const srs_amd_pusch_chest_config* cfg,
                                 const uint32_t*                   grid,
                                 uint32_t                          nof_ports,
                                 uint32_t                          nof_subc,
                                 uint32_t*                         estimates,
                                 srs_amd_chest_port_stats*         stats);

/* DEVICE, asynchronous: nof_grids grids (grid_stride REs apart), estimates
 * est_stride REs apart, stats [nof_grids][nof_ports]. */
int srs_amd_pusch_chest_estimate_batch(srs_amd_pusch_chest*              chest,
                                       const srs_amd_pusch_chest_config* cfg,
                                       const uint32_t*                   d_grids,
                                       uint64_t                          grid_stride,
                                       uint32_t                          nof_ports,
                                       uint32_t                          nof_subc,
                                       uint32_t                          nof_grids,
                                       uint32_t*                         d_estimates,
                                       uint64_t                          est_stride,
                                       srs_amd_chest_port_stats*         d_stats,
                                       void*                             stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_PUSCH_CHEST_H */
