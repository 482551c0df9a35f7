/*
 * srsran_amd/equalizer.h -- C-ABI of the MI355X channel equalizer (PUSCH/PDSCH
 * receive path, TS 38.211 layer demapping after channel estimation).
 *
 * Replaces:
 *   srs_amd_channel_equalizer_create
 *       create_channel_equalizer_generic_factory(type)->create()
 *       (lib/phy/upper/equalization/equalization_factories.cpp:47)
 *   srs_amd_channel_equalizer_is_supported
 *       channel_equalizer::is_supported(nof_ports, nof_layers)
 *       include/srsran/phy/upper/equalization/channel_equalizer.h:65
 *   srs_amd_channel_equalize
 *       channel_equalizer::equalize(eq_symbols, eq_noise_vars, ch_symbols, ch_estimates,
 *                                   noise_var_estimates, tx_scaling)   channel_equalizer.h:89
 *   srs_amd_channel_equalize_batch: the same on device buffers, asynchronous.
 *
 * Supported: the open-source reference's topologies (channel_equalizer_generic_impl.cpp:240-270,
 * pinned): ZF 1 layer x {1, 2, 4} ports, ZF 2 layers x {2, 4} ports, MMSE 1 layer (equal to ZF
 * there); and the ones the open reference declares but asserts for (:197-247, the enterprise
 * build's equalize_zf_3x4 / 4x4, equalize_mmse_2x2 / 2x4 / 3x4 / 4x4), PARITY UNPINNED: an L x L
 * Cholesky solve per RE of ZF or the unbiased MMSE estimate (equalizer_device.h equalize_mimo),
 * checked against an fp64 solve (tests/test_equalizer_mimo_gpu.py, tolerance stated there).
 * Layouts (the reference containers):
 *   ch_symbols   : cbf16 [port][nof_re]            (re_buffer_reader<cbf16_t> slices)
 *   ch_estimates : cbf16 [layer][port][nof_re]     (dynamic_ch_est_list.h dims {re, port, layer})
 *   eq_symbols   : complex float [nof_re][layer];  eq_noise_vars: float [nof_re][layer]
 * Numerics: float32 with IEEE division, the semantics of the reference's
 * scalar path (zero symbol / infinite variance where the reference's
 * isnormal() checks fail); the reference's AVX2 path uses an approximate
 * reciprocal, so results agree within the relative tolerance stated in
 * tests/test_equalizer_gpu.py (1e-3 on symbols, 2e-3 on variances).
 */
#ifndef SRSRAN_AMD_EQUALIZER_H
#define SRSRAN_AMD_EQUALIZER_H

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRS_AMD_EQ_ZF 0   /* channel_equalizer_algorithm_type::zf */
#define SRS_AMD_EQ_MMSE 1 /* channel_equalizer_algorithm_type::mmse */

typedef struct srs_amd_channel_equalizer srs_amd_channel_equalizer;

int  srs_amd_channel_equalizer_create(srs_amd_channel_equalizer** eq, int algorithm, int device);
void srs_amd_channel_equalizer_destroy(srs_amd_channel_equalizer* eq);
int  srs_amd_channel_equalizer_is_supported(const srs_amd_channel_equalizer* eq, uint32_t nof_ports,
                                            uint32_t nof_layers);

/* HOST buffers, synchronous.  noise_var_estimates: nof_ports floats. */
int srs_amd_channel_equalize(srs_amd_channel_equalizer* eq,
                             float*                     eq_symbols,
                             float*                     eq_noise_vars,
                             const uint16_t*            ch_symbols,
                             const uint16_t*            ch_estimates,
                             const float*               noise_var_estimates,
                             uint32_t                   nof_re,
                             uint32_t                   nof_ports,
                             uint32_t                   nof_layers,
                             float                      tx_scaling);

/* DEVICE buffers (noise_var_estimates stays a HOST array of nof_ports floats),
 * asynchronous on `stream`. */
int srs_amd_channel_equalize_batch(srs_amd_channel_equalizer* eq,
                                   float*                     d_eq_symbols,
                                   float*                     d_eq_noise_vars,
                                   const uint16_t*            d_ch_symbols,
                                   const uint16_t*            d_ch_estimates,
                                   const float*               noise_var_estimates,
                                   uint32_t                   nof_re,
                                   uint32_t                   nof_ports,
                                   uint32_t                   nof_layers,
                                   float                      tx_scaling,
                                   void*                      stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_EQUALIZER_H */
