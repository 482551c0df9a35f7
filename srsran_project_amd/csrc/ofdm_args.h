// ofdm_args.h -- kernel argument blocks of the OFDM modulator / demodulator and
// DFT processor kernels (ofdm.hip), shared with their C-ABI (ofdm_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

// Per OFDM symbol of a subframe (slots_per_subframe * nsymb entries).
struct ofdm_symbol_info {
  uint32_t cp_len;      // cyclic prefix samples
  uint32_t offset;      // first sample of the symbol (CP included) within its slot
  float    coef_re;     // phase compensation * scale (phase_compensation_lut.h, cf_t * float)
  float    coef_im;
};

struct ofdm_args {
  const void*             in;        // mod: cbf16 grid; demod: cf samples
  void*                   out;       // mod: cf samples; demod: cbf16 grid
  const ofdm_symbol_info* symbols;   // [slots_per_subframe][nsymb]
  const float*            twiddles;  // W_N^m, m in [0, N), interleaved re/im
  const float*            window;    // demod: window-offset compensation per bin (re/im), or null
  uint32_t                rg_size;   // subcarriers (bw_rb * 12)
  uint32_t                nsymb;
  uint32_t                nof_ports;
  uint32_t                first_slot;
  uint32_t                slots_per_subframe;
  uint32_t                nof_items; // slots * ports
  uint32_t                sample_stride; // complex samples per (slot, port) row
  uint32_t                window_offset; // demod: nof_samples_window_offset
  // demod, staged symbols (nsymb = 1, one workgroup per item): item i = {symbol index within the subframe (into
  // `symbols`, entries with offset 0), first cbf16 of its grid row in `out`}, its samples (CP first) at
  // in + i * sample_stride; items with a symbol index >= nof_symbol_infos are skipped.  nullptr: the regular layout.
  const uint32_t*         items;
  uint32_t                nof_symbol_infos;
};

struct dft_args {
  const float* in;        // [nof][N] complex
  float*       out;       // [nof][N] complex
  const float* twiddles;
  uint32_t     nof;
};

bool       ofdm_size_supported(uint32_t N);
hipError_t launch_ofdm_modulate(const ofdm_args& a, uint32_t N, hipStream_t stream);
hipError_t launch_ofdm_demodulate(const ofdm_args& a, uint32_t N, hipStream_t stream);
hipError_t launch_dft(const dft_args& a, uint32_t N, int inverse, hipStream_t stream);

} // namespace srs_amd
