/*
 * srsran_amd/low_papr.h -- low-PAPR base sequences of TS 38.211 Section 5.2.2 (the DM-RS of transform-precoded
 * PUSCH), generated on the host once per configuration and uploaded by the estimator (pusch_chest.h).
 *
 * Replaces (reference interface):
 *   low_papr_sequence_generator::generate(span<cf_t> sequence, unsigned u, unsigned v, unsigned alpha_num,
 *                                         unsigned alpha_den)
 *       include/srsran/phy/upper/sequence_generators/low_papr_sequence_generator.h:46
 *       (impl lib/phy/upper/sequence_generators/low_papr_sequence_generator_impl.cpp: phase tables for
 *        M = 6, 12, 18, 24, the 31-point form for M = 30, Zadoff-Chu of the largest prime below M otherwise,
 *        each value read from a float complex-exponential table of 2 N_ZC entries)
 * Values identical to the reference's (same float table, same indices).  Scope: no cyclic shift
 * (alpha_num = 0), as the PUSCH DM-RS uses it (dmrs_pusch_estimator_impl.cpp:88-92).
 */
#ifndef SRSRAN_AMD_LOW_PAPR_H
#define SRSRAN_AMD_LOW_PAPR_H

#include <stdint.h>

#include "srsran_amd/ldpc.h" /* SRS_AMD_OK / SRS_AMD_EINVAL */

#ifdef __cplusplus
extern "C" {
#endif

/* 1 when M is a length the reference generates (6 x a valid transform-precoding PRB count, <= 1632). */
int srs_amd_low_papr_length_valid(uint32_t M);

/* HOST: r_{u,v}(n), n = 0 .. M-1, as interleaved (re, im) floats; u in [0, 30), v in {0, 1} (v = 0 for M < 72).
 * SRS_AMD_EINVAL for an invalid length or group / number. */
int srs_amd_low_papr_sequence(float* out, uint32_t M, uint32_t u, uint32_t v);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_LOW_PAPR_H */
