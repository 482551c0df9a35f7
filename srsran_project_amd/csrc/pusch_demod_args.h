// pusch_demod_args.h -- argument blocks of the PUSCH demodulator kernels
// (pusch_demod.hip), shared with their C-ABI (pusch_demod_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "srsran_amd/pusch_chest.h"
#include "srsran_amd/pusch_demodulator.h"
#include "modulation_args.h"
#include "pusch_chest_args.h"

namespace srs_amd {

struct pusch_eq_args {
  const uint32_t*                 grids;     // cbf16 [grid][port][14][subc]
  const uint32_t*                 estimates; // cbf16 [grid][port][layer][14][subc]
  const srs_amd_chest_port_stats* stats;     // [grid][port]
  const uint32_t*                 re_table;  // [14][nof_prb]: data RE index << 12 | 12-bit mask
  uint64_t                        grid_stride;
  uint64_t                        est_stride;
  uint32_t                        nof_subc;
  uint32_t                        nof_prb;
  uint32_t                        nof_re;
  uint32_t                        first_symbol;
  uint32_t                        first_subc;
  // demapping + descrambling in the equalizer: LLR n of a grid at llrs[grid * llr_stride + n], codeword
  // symbol i = j L + layer of data RE j; scr: Gold words of the plan's c_init (c(n) at bit n % 32 of word
  // n / 32, one word past the codeword); symbols i < simd_hi[l] of OFDM symbol l take the SIMD demapper
  int8_t*                         llrs;
  const uint32_t*                 scr;
  uint64_t                        llr_stride;
  uint32_t                        simd_hi[14];
  demodulate_args                 dm;
  // transform precoding: the equalizer writes its symbols / noise variances (grid rows of eq_stride
  // codeword symbols) instead of LLRs; the deprecoder and the demapper follow
  float2*                         eq_out;
  float*                          nv_out;
  uint64_t                        eq_stride;
  uint32_t                        tiles_x;   // fused equalizer: 256-subcarrier tiles per grid
  uint32_t                        nof_tiles; // tiles_x x grids
  // DC subcarrier whose channel coefficients are taken as zero (pusch_processor_impl.cpp:235-249); ~0u: none
  uint32_t                        dc_subc;
};

// The processor's DC zeroing (pusch_processor_impl.cpp:235-249) for a demodulator plan: every equalizer form then
// reads zero channel coefficients at grid subcarrier dc_subc (~0u: none).  Plans with transform precoding ignore it.
void pusch_demod_plan_set_dc(::srs_amd_pusch_demod_plan* plan, uint32_t dc_subc);

// Zeroes subcarrier dc_subc of the expanded estimates [grid][P x L][14][nof_subc] (est_stride uint32 per grid) in
// OFDM symbols [first_symbol, first_symbol + nof_symbols): the reference's ch_estimate after the DC step.
hipError_t launch_pusch_dc_zero(uint32_t* estimates, uint64_t est_stride, uint32_t nof_planes, uint32_t nof_subc,
                                uint32_t first_symbol, uint32_t nof_symbols, uint32_t dc_subc, uint32_t nof_grids,
                                hipStream_t stream);


hipError_t launch_pusch_equalize(const pusch_eq_args& a, uint32_t nof_ports, uint32_t nof_layers, bool mmse,
                                 uint32_t nof_symbols, uint32_t span_subc, uint32_t nof_grids, hipStream_t stream);

// Estimator-fused equalizer (pusch_demod.hip pusch_equalize_fused_kernel): the channel coefficients of each data
// RE rebuilt from the estimator's unexpanded output c (chest_estimate_batch_unexpanded); a.estimates unused.
bool       pusch_equalize_fusable(uint32_t nof_ports, uint32_t nof_layers, bool mmse, uint32_t nof_lse);
hipError_t launch_pusch_equalize_fused(const pusch_eq_args& a, const chest_args& c, uint32_t nof_ports,
                                       uint32_t nof_layers, bool mmse, uint32_t span_subc, uint32_t nof_grids,
                                       hipStream_t stream);

// Slot form of the fused equalizer (srs_amd_pusch_process_slot): one (equalizer, estimator) argument pair per
// PDU, each on one grid (a.nof_tiles = a.tiles_x); a launch covers the PDUs ids[blockIdx.y] (ids == nullptr:
// PDU blockIdx.y) of one (ports, layers, MMSE) kernel; max_blocks = the largest PDU's blockIdx.x extent.
struct eq_item {
  pusch_eq_args a;
  chest_args    c;
};
struct eq_items {
  const eq_item*  items = nullptr;
  const uint32_t* ids   = nullptr;
};
hipError_t launch_pusch_equalize_fused_items(const eq_items& items, uint32_t count, uint32_t nof_ports,
                                             uint32_t nof_layers, bool mmse, uint32_t max_blocks, hipStream_t stream);
uint32_t   pusch_equalize_fused_blocks(uint32_t nof_symbols, uint32_t nof_tiles);

// One PDU of a slot for pusch_demodulate_slot_fused: its plan, the estimator view of its unexpanded
// estimates (chest_estimate_slot_unexpanded), its grid, port measurements and codeword LLR row.
struct demod_slot_item {
  const ::srs_amd_pusch_demod_plan* plan;
  const chest_args*                 chest_view;
  const uint32_t*                   d_grid;
  const srs_amd_chest_port_stats*   d_stats;
  int8_t*                           d_llrs;
};
int pusch_demodulate_slot_fused(::srs_amd_pusch_demodulator* dem,
                                const demod_slot_item*       items,
                                uint32_t                     nof_items,
                                void*                        stream);

// srs_amd_pusch_demodulate_batch with the estimator-fused equalizer (no estimate tensor).
int pusch_demodulate_batch_fused(::srs_amd_pusch_demodulator*      dem,
                                 const ::srs_amd_pusch_demod_plan* plan,
                                 const uint32_t*                   d_grids,
                                 uint64_t                          grid_stride,
                                 const chest_args&                 chest_view,
                                 const srs_amd_chest_port_stats*   d_stats,
                                 int8_t*                           d_llrs,
                                 uint64_t                          llr_stride,
                                 uint32_t                          nof_grids,
                                 void*                             stream);

} // namespace srs_amd
