/*
 * srsran_amd/transform_precoding.h -- C-ABI of the MI355X transform deprecoder (DFT-s-OFDM PUSCH).
 *
 * Replaces (reference interface):
 *   transform_precoder::deprecode_ofdm_symbol(span<cf_t> out, span<const cf_t> in)
 *       include/srsran/phy/generic_functions/transform_precoding/transform_precoder.h:55
 *   transform_precoder::deprecode_ofdm_symbol_noise(span<float> out, span<const float> in)
 *       transform_precoder.h:63
 *   (impl lib/phy/generic_functions/transform_precoding/transform_precoder_dft_impl.cpp:31-84: an inverse
 *    M-point DFT scaled by 1/sqrt(M), M = 12 M_rb; the noise variances of the symbol replaced by their mean
 *    over the valid (positive, finite) values)
 *   transform_precoding::is_nof_prbs_valid (include/srsran/ran/transform_precoding/transform_precoding_helpers.h:64)
 * Numerics: float DFT as a two-factor (M = M1 M2) decomposition in LDS; outputs within float rounding of the
 * exact transform (the reference's generic DFT is itself float).
 */
#ifndef SRSRAN_AMD_TRANSFORM_PRECODING_H
#define SRSRAN_AMD_TRANSFORM_PRECODING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srs_amd_transform_precoder srs_amd_transform_precoder;

int  srs_amd_transform_precoder_create(srs_amd_transform_precoder** tp, int device);
void srs_amd_transform_precoder_destroy(srs_amd_transform_precoder* tp);

/* 1 when M_rb = 2^a 3^b 5^c and 1 <= M_rb <= 275 (MAX_NOF_PRBS), else 0. */
int srs_amd_transform_precoding_nof_prbs_valid(uint32_t nof_prb);

/* HOST, synchronous: out[k] = 1/sqrt(M) sum_n in[n] exp(+j 2 pi n k / M), M = nof_subc (interleaved re, im
 * floats); in and out may alias.  SRS_AMD_EINVAL when nof_subc is not 12 x a valid number of PRBs. */
int srs_amd_transform_deprecode(srs_amd_transform_precoder* tp, float* out, const float* in, uint32_t nof_subc);

/* HOST: noise variances of one OFDM symbol (transform_precoder_dft_impl.cpp:58-84). */
int srs_amd_transform_deprecode_noise(srs_amd_transform_precoder* tp, float* out, const float* in, uint32_t nof_subc);

/* DEVICE, asynchronous, in place: nof_rows OFDM symbols of nof_subc complex floats (rows sym_stride complex
 * values apart) and, when d_noise_vars is not NULL, their noise variances (rows nv_stride floats apart). */
int srs_amd_transform_deprecode_batch(srs_amd_transform_precoder* tp,
                                      float*                      d_symbols,
                                      uint64_t                    sym_stride,
                                      float*                      d_noise_vars,
                                      uint64_t                    nv_stride,
                                      uint32_t                    nof_subc,
                                      uint32_t                    nof_rows,
                                      void*                       stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_TRANSFORM_PRECODING_H */
