/*
 * srsran_amd/modulation.h -- C-ABI of the MI355X modulation mapper, soft
 * demodulation mapper and Gold-sequence scrambling (PDSCH / PUSCH data path).
 *
 * Replaces:
 *   srs_amd_modulate(_batch)
 *       modulation_mapper::modulate(span<cf_t> symbols, const bit_buffer& input, modulation_scheme)
 *       include/srsran/phy/upper/channel_modulation/modulation_mapper.h:52
 *   srs_amd_demodulate_soft(_batch)
 *       demodulation_mapper::demodulate_soft(span<log_likelihood_ratio>, span<const cf_t>,
 *                                            span<const float> noise_vars, modulation_scheme)
 *       include/srsran/phy/upper/channel_modulation/demodulation_mapper.h:66
 *   srs_amd_scramble_bits(_batch) / srs_amd_descramble_llrs(_batch)
 *       pseudo_random_generator::init(c_init) + apply_xor(bit_buffer&, const bit_buffer&) /
 *       apply_xor(span<log_likelihood_ratio>, span<const log_likelihood_ratio>)
 *       include/srsran/phy/upper/sequence_generators/pseudo_random_generator.h:54,79,102
 *   (factories: create_modulation_mapper_factory / create_demodulation_mapper_factory /
 *    create_pseudo_random_generator_sw_factory)
 *
 * Modulation codes (bits per symbol; modulation_scheme): 0 = pi/2-BPSK, 1 = BPSK,
 * 2 = QPSK, 4 = 16QAM, 6 = 64QAM, 8 = 256QAM.  Bits are packed MSB-first
 * (bit_buffer), symbols interleaved complex float, LLRs int8.
 * Bit-exact with an x86-64-v3 (AVX2) build of the reference, soft demapping
 * included (tests/test_modulation_gpu.py).
 */
#ifndef SRSRAN_AMD_MODULATION_H
#define SRSRAN_AMD_MODULATION_H

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srs_amd_modulator srs_amd_modulator;

/* One object serves all three roles (tables + device state + stream). */
int  srs_amd_modulator_create(srs_amd_modulator** mod, int device);
void srs_amd_modulator_destroy(srs_amd_modulator* mod);

/* HOST buffers, synchronous. */
int srs_amd_modulate(srs_amd_modulator* mod, float* symbols, const uint8_t* bits, uint32_t nof_symbols, int qm);
int srs_amd_demodulate_soft(srs_amd_modulator* mod,
                            int8_t*            llrs,
                            const float*       symbols,
                            const float*       noise_vars,
                            uint32_t           nof_symbols,
                            int                qm);
int srs_amd_scramble_bits(srs_amd_modulator* mod, uint8_t* out, const uint8_t* in, uint32_t nof_bits, uint32_t c_init);
int srs_amd_descramble_llrs(srs_amd_modulator* mod, int8_t* out, const int8_t* in, uint32_t nof_llrs, uint32_t c_init);

/* DEVICE buffers, asynchronous on `stream`. */
int srs_amd_modulate_batch(srs_amd_modulator* mod, float* d_symbols, const uint8_t* d_bits, uint32_t nof_symbols,
                           int qm, void* stream);
int srs_amd_demodulate_soft_batch(srs_amd_modulator* mod,
                                  int8_t*            d_llrs,
                                  const float*       d_symbols,
                                  const float*       d_noise_vars,
                                  uint32_t           nof_symbols,
                                  int                qm,
                                  void*              stream);
int srs_amd_scramble_bits_batch(srs_amd_modulator* mod, uint8_t* d_out, const uint8_t* d_in, uint32_t nof_bits,
                                uint32_t c_init, void* stream);
int srs_amd_descramble_llrs_batch(srs_amd_modulator* mod, int8_t* d_out, const int8_t* d_in, uint32_t nof_llrs,
                                  uint32_t c_init, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_MODULATION_H */
