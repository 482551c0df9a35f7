/*
 * srsran_amd/ofdm.h -- C-ABI of the MI355X OFDM modulator / demodulator and DFT
 * processor (lower PHY, TS 38.211 Sections 5.3-5.4).
 *
 * Replaces:
 *   srs_amd_ofdm_modulator_create
 *       create_ofdm_modulator_factory_generic({dft_factory})->create_ofdm_slot_modulator(config)
 *       include/srsran/phy/lower/modulation/modulation_factories.h,
 *       lib/phy/lower/modulation/modulation_factories.cpp:34-57,214
 *   srs_amd_ofdm_modulator_get_slot_size / srs_amd_ofdm_modulate_slot
 *       ofdm_slot_modulator::get_slot_size / ::modulate(output, grid, port, slot_index)
 *       include/srsran/phy/lower/modulation/ofdm_modulator.h:98,108
 *   srs_amd_ofdm_modulator_get_symbol_size / _set_center_frequency / srs_amd_ofdm_modulate_symbol
 *       ofdm_symbol_modulator::get_symbol_size / ::set_center_frequency / ::modulate(output, grid, port, symbol)
 *       include/srsran/phy/lower/modulation/ofdm_modulator.h:47-76
 *   srs_amd_ofdm_demodulator_* (same for ofdm_demodulator.h, nof_samples_window_offset honoured)
 *   srs_amd_dft_create / srs_amd_dft_run
 *       create_dft_processor_factory_generic()->create({size, dir}) / dft_processor::run()
 *       include/srsran/phy/generic_functions/dft_processor.h:48,68,72
 *   *_batch: many (slot, port) pairs, device-resident, one launch.
 *
 * Data layout (as the reference):
 *   resource grid: complex bfloat16 (cbf16_t: real, imag as uint16 bf16),
 *     [symbol][subcarrier] per port (lib/phy/support/resource_grid_impl.h:50);
 *   baseband samples: complex float (cf_t), the slot's symbols back to back,
 *     each cyclic prefix + DFT size samples.
 *   Batches: grid [nof_slots][nof_ports][nsymb][bw_rb*12] cbf16,
 *            samples [nof_slots][nof_ports][sample_stride] cf_t; slot s of the
 *            batch is slot (first_slot + s) mod slots_per_subframe of a subframe.
 *
 * Numerics: float32 with exactly rounded twiddles; outputs match the reference
 * within the float tolerance stated in tests/test_ofdm_gpu.py (samples:
 * max error <= 2e-5 x RMS; grids: bf16 values equal to the exactly computed
 * value rounded half-to-even, up to one bf16 ulp at rounding ties).
 * Supported DFT sizes: 128, 256, 384, 512, 768, 1024, 1536, 2048, 3072, 4096,
 * 6144, 8192 (every srsRAN sampling rate from 1.92 to 245.76 MHz that is
 * 2^a or 3*2^a times the SCS).
 */
#ifndef SRSRAN_AMD_OFDM_H
#define SRSRAN_AMD_OFDM_H

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ofdm_modulator_configuration / ofdm_demodulator_configuration
 * (ofdm_modulator.h:33, ofdm_demodulator.h:34). */
typedef struct srs_amd_ofdm_config {
  uint32_t numerology;                /* subcarrier spacing index mu */
  uint32_t bw_rb;                     /* resource grid bandwidth in RB */
  uint32_t dft_size;                  /* > bw_rb * 12 */
  uint32_t cp_extended;               /* 0 = normal CP, 1 = extended */
  uint32_t nof_samples_window_offset; /* demodulator only (< 144*dft_size/2048) */
  float    scale;                     /* normal (non-zero, finite) */
  double   center_freq_hz;
} srs_amd_ofdm_config;

typedef struct srs_amd_ofdm_modulator   srs_amd_ofdm_modulator;
typedef struct srs_amd_ofdm_demodulator srs_amd_ofdm_demodulator;
typedef struct srs_amd_dft              srs_amd_dft;

int      srs_amd_ofdm_modulator_create(srs_amd_ofdm_modulator** mod, const srs_amd_ofdm_config* cfg, int device);
void     srs_amd_ofdm_modulator_destroy(srs_amd_ofdm_modulator* mod);
uint32_t srs_amd_ofdm_modulator_get_slot_size(const srs_amd_ofdm_modulator* mod, uint32_t slot_index);
/* One port of one slot, HOST buffers, synchronous.
 *   output : get_slot_size(slot_index) complex float samples (2 floats each)
 *   grid   : nsymb * bw_rb * 12 cbf16 (2 uint16 each)                      */
int srs_amd_ofdm_modulate_slot(srs_amd_ofdm_modulator* mod, float* output, const uint16_t* grid, uint32_t slot_index);
int srs_amd_ofdm_modulate_batch(srs_amd_ofdm_modulator* mod,
                                const uint16_t*         d_grid,
                                uint32_t                nof_ports,
                                uint32_t                first_slot,
                                uint32_t                nof_slots,
                                float*                  d_samples,
                                uint32_t                sample_stride,
                                void*                   stream);

/* Symbol granularity (ofdm_symbol_modulator, ofdm_modulator.h:47-76): symbol_index within the subframe,
 * HOST buffers, synchronous.
 *   get_symbol_size : cyclic prefix + DFT size samples (ofdm_symbol_modulator::get_symbol_size)
 *   set_center_frequency : phase compensation of the following calls (ofdm_symbol_modulator::set_center_frequency;
 *                          the slot forms use it too)
 *   modulate_symbol : output get_symbol_size(symbol_index) complex floats; grid_symbol bw_rb * 12 cbf16 */
uint32_t srs_amd_ofdm_modulator_get_symbol_size(const srs_amd_ofdm_modulator* mod, uint32_t symbol_index);
int      srs_amd_ofdm_modulator_set_center_frequency(srs_amd_ofdm_modulator* mod, double center_freq_hz);
int      srs_amd_ofdm_modulate_symbol(srs_amd_ofdm_modulator* mod,
                                      float*                  output,
                                      const uint16_t*         grid_symbol,
                                      uint32_t                symbol_index);

int      srs_amd_ofdm_demodulator_create(srs_amd_ofdm_demodulator** dem, const srs_amd_ofdm_config* cfg, int device);
void     srs_amd_ofdm_demodulator_destroy(srs_amd_ofdm_demodulator* dem);
uint32_t srs_amd_ofdm_demodulator_get_slot_size(const srs_amd_ofdm_demodulator* dem, uint32_t slot_index);
int      srs_amd_ofdm_demodulate_slot(srs_amd_ofdm_demodulator* dem,
                                      uint16_t*                 grid,
                                      const float*              input,
                                      uint32_t                  slot_index);
int      srs_amd_ofdm_demodulate_batch(srs_amd_ofdm_demodulator* dem,
                                       const float*              d_samples,
                                       uint32_t                  sample_stride,
                                       uint32_t                  nof_ports,
                                       uint32_t                  first_slot,
                                       uint32_t                  nof_slots,
                                       uint16_t*                 d_grid,
                                       void*                     stream);

/* ofdm_symbol_demodulator (ofdm_demodulator.h:44-73): as the modulator's symbol forms; grid_symbol receives the
 * bw_rb * 12 cbf16 subcarriers of the symbol. */
uint32_t srs_amd_ofdm_demodulator_get_symbol_size(const srs_amd_ofdm_demodulator* dem, uint32_t symbol_index);
int      srs_amd_ofdm_demodulator_set_center_frequency(srs_amd_ofdm_demodulator* dem, double center_freq_hz);
int      srs_amd_ofdm_demodulate_symbol(srs_amd_ofdm_demodulator* dem,
                                        uint16_t*                 grid_symbol,
                                        const float*              input,
                                        uint32_t                  symbol_index);

/* Symbol granularity, ASYNCHRONOUS on `stream`: the same transforms with both buffers device-accessible (device
 * memory, or pinned host memory the kernel reads / writes over the bus): no copy, no synchronisation.  What the
 * reference-side OFDM plug-ins run per ofdm_symbol_(de)modulator call on a device-resident resource grid
 * (integration/ofdm_modulator_hip.cpp), the grid row being (port, symbol % nsymb) of the device copy. */
int srs_amd_ofdm_modulate_symbol_async(srs_amd_ofdm_modulator* mod,
                                       float*                  output,
                                       const uint16_t*         grid_symbol,
                                       uint32_t                symbol_index,
                                       void*                   stream);
int srs_amd_ofdm_demodulate_symbol_async(srs_amd_ofdm_demodulator* dem,
                                         uint16_t*                 grid_symbol,
                                         const float*              input,
                                         uint32_t                  symbol_index,
                                         void*                     stream);
/* Many staged symbols in one launch, ASYNCHRONOUS on `stream` (the deferred form of the symbol demodulator plug-in:
 * each ofdm_symbol_demodulator::demodulate call copies its samples into pinned staging, the symbols of a slot go in
 * one launch).  items [count][2] = {symbol index within the subframe, offset of the symbol's grid row in cbf16
 * pairs from `grid`}; samples [count][sample_stride] complex floats, symbol i's get_symbol_size(items[2i]) samples
 * (cyclic prefix first) at the start of its row; sample_stride >= the longest symbol.  items and samples
 * device-accessible (pinned host memory is).  An item with an out-of-range symbol index is skipped.
 * d_scratch: NULL -- the kernel reads items and samples where they are (over the bus when pinned); else items and
 * samples are pinned host memory, first copied into d_scratch (device memory of count * (8 * sample_stride + 8)
 * bytes) by a copy kernel (wide reads, many in flight), and the transform reads HBM. */
int srs_amd_ofdm_demodulate_symbols_async(srs_amd_ofdm_demodulator* dem,
                                          uint16_t*                 grid,
                                          const uint32_t*           items,
                                          const float*              samples,
                                          uint32_t                  sample_stride,
                                          uint32_t                  count,
                                          void*                     d_scratch,
                                          void*                     stream);

/* dft_processor: direction 0 = DIRECT (exp(-2*pi*i*n*k/N)), 1 = INVERSE; no normalisation. */
int  srs_amd_dft_create(srs_amd_dft** dft, uint32_t size, int direction, int device);
void srs_amd_dft_destroy(srs_amd_dft* dft);
/* One transform, HOST buffers (size complex floats each), synchronous. */
int srs_amd_dft_run(srs_amd_dft* dft, float* output, const float* input);
/* nof transforms of consecutive size-point vectors, DEVICE buffers, asynchronous. */
int srs_amd_dft_run_batch(srs_amd_dft* dft, const float* d_input, float* d_output, uint32_t nof, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_OFDM_H */
