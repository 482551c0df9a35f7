// modulation_args.h -- argument blocks of the modulation / demodulation /
// scrambling kernels (modulation.hip), shared with their C-ABI (modulation_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gold_sequence.h"

namespace srs_amd {

// Soft-demapper piecewise-linear LLR table of one PAM axis bit.
struct demod_interval_table {
  int32_t n;         // intervals
  float   width;
  float   inv_width; // 1.0f / width (the reference's SIMD path multiplies by it)
  float   slope[16];
  float   icpt[16];
};

struct modulate_args {
  const uint8_t* bits;    // packed MSB-first
  float*         symbols; // interleaved re/im
  const float*   table;   // [2^Qm][2] re/im (Qm >= 2)
  uint32_t       nof_symbols;
  int32_t        qm;      // 0 pi/2-BPSK, 1 BPSK, 2, 4, 6, 8
};

struct demodulate_args {
  const float*         symbols;
  const float*         noise_vars;
  int8_t*              llrs;
  uint32_t             nof_symbols;
  uint32_t             block_end; // symbols [0, block_end) follow the reference's AVX2 kernel, the rest its scalar code
  int32_t              qm;
  float                qam16_scale; // 1/sqrt(10) as the reference computes it (host float sqrt)
  demod_interval_table tab[4];
};

struct prbs_args {
  const uint8_t* in_bits;  // scramble: packed input (may be null: generate c)
  uint8_t*       out_bits;
  const int8_t*  in_llrs;  // descramble LLRs
  int8_t*        out_llrs;
  const uint32_t* jump;    // [2][NJUMP][31] GF(2) jump matrices (columns), x1 then x2
  uint32_t       c_init;
  uint32_t       length;   // bits / LLRs
};


hipError_t launch_modulate(const modulate_args& a, hipStream_t stream);
hipError_t launch_demodulate(const demodulate_args& a, hipStream_t stream);

struct demap_descramble_args {
  int8_t*         llrs;         // [grid][llr_stride]
  const uint32_t* jump;         // gold_jump_tables()
  uint64_t        llr_stride;
  uint32_t        grid_symbols; // symbols per grid
  uint32_t        c_init;
  // The reference demaps each OFDM symbol in its own call (pusch_demodulator_impl.cpp:363-400), so the
  // SIMD blocks end at every symbol's end: symbols [sym_lo[l], simd_hi[l]) of the grid take the SIMD
  // arithmetic, the rest of [sym_lo[l], sym_lo[l + 1]) the scalar tail (sym_lo = simd_hi when empty).
  uint32_t        sym_lo[14];
  uint32_t        simd_hi[14];
};
hipError_t launch_demap_descramble(const demodulate_args& a, const demap_descramble_args& d, uint32_t nof_grids,
                                   hipStream_t stream);
// Slot form: one argument pair per PDU (device array, one grid each), max_symbols: the largest grid_symbols.
struct demap_item {
  demodulate_args       a;
  demap_descramble_args d;
};
hipError_t launch_demap_descramble_items(const demap_item* items, uint32_t n, uint32_t max_symbols,
                                         hipStream_t stream);
// Gold-sequence words 0 .. nof_words of c_init into out (c(32 w + b) at bit b of word w).
hipError_t launch_gold_words(const uint32_t* jump, uint32_t c_init, uint32_t* out, uint32_t nof_words,
                             hipStream_t stream);

} // namespace srs_amd

struct srs_amd_modulator;

namespace srs_amd {

// Demapper arguments (tables, AVX2 block end) for calls of nof_symbols symbols (modulation_api.cpp).
demodulate_args demodulate_args_for(const srs_amd_modulator* mod, int qm, uint32_t nof_symbols);
// The reference demaps each OFDM symbol in its own call: per OFDM symbol l (sym_counts[l] demapper symbols),
// its first symbol sym_lo[l] and the end of its SIMD blocks simd_hi[l]; returns the total.
uint32_t demap_symbol_bounds(int qm, const uint32_t* sym_counts, uint32_t* sym_lo, uint32_t* simd_hi);

// Soft demapping of nof_grids x grid_symbols symbols and descrambling of each grid's LLRs with the
// Gold sequence of c_init, one launch (the PUSCH demodulator's last two steps).
// sym_counts[l]: demapper symbols (REs x layers) of OFDM symbol l, in grid order (sum = grid_symbols).
int demap_descramble_batch(srs_amd_modulator* mod, int qm, int8_t* d_llrs, uint64_t llr_stride, const float* d_symbols,
                           const float* d_noise_vars, uint32_t grid_symbols, const uint32_t* sym_counts,
                           uint32_t nof_grids, const uint32_t* d_jump, uint32_t c_init, void* stream);
// The argument pair demap_descramble_batch launches for one grid (the slot form's item).
int make_demap_item(srs_amd_modulator* mod, int qm, int8_t* d_llrs, const float* d_symbols, const float* d_noise_vars,
                    uint32_t grid_symbols, const uint32_t* sym_counts, const uint32_t* d_jump, uint32_t c_init,
                    demap_item& out);
hipError_t launch_scramble_bits(const prbs_args& a, hipStream_t stream);
hipError_t launch_descramble_llrs(const prbs_args& a, hipStream_t stream);

} // namespace srs_amd
