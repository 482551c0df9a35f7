// pdsch_modulator_args.h -- argument blocks of the PDSCH modulator and PDSCH
// DM-RS kernels (pdsch_modulator.hip), shared with their C-ABI (pdsch_modulator_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

constexpr int PDSCH_NSYMB   = 14;
constexpr int PDSCH_NRE     = 12;
constexpr int PDSCH_MAX_RB  = 275;
constexpr int PDSCH_THREADS = 256;

struct pdsch_map_args {
  const uint8_t*  codewords;  // packed MSB first, rows of cw_stride bytes
  uint32_t*       grids;      // cbf16 REs
  const uint32_t* re_table;   // [14][nof_prb]: (data RE index of the PRB's first RE) << 12 | 12-bit data RE mask
  const uint32_t* jump;       // Gold-sequence jump matrices
  const uint32_t* scr;        // Gold words of c_init (c(32 w + b) at bit b of word w), one past the codeword
  uint64_t        grid_stride;
  uint32_t        port_stride; // 14 * nof_subc
  uint32_t        nof_subc;
  uint32_t        nof_prb;     // ceil(nof_subc / 12)
  uint32_t        cw_stride;
  uint32_t        nof_bits;
  uint32_t        c_init;
  uint32_t        first_symbol;
  int32_t         qm;
  int32_t         nof_layers;
  int32_t         nof_ports;
  uint32_t        first_subc;  // first allocated subcarrier (grid.x offset)
  uint32_t        nof_symbols; // slot form: blockIdx.y extent of this PDU
  uint32_t        nof_tiles;   // slot form: blockIdx.x extent of this PDU
  float           w[4][4][2];  // [layer][port] weights x modulation scaling x config scaling
};

struct dmrs_pdsch_args {
  uint32_t*       grids;
  const uint32_t* jump;
  uint64_t        grid_stride;
  uint32_t        port_stride;
  uint32_t        nof_crb;
  uint32_t        reference_point_k_rb;
  int32_t         type2;
  int32_t         nof_layers;
  int32_t         nof_ports;
  float           amplitude;    // M_SQRT1_2 * config amplitude (double product rounded to float)
  uint32_t        nof_dmrs_symbols;
  uint8_t         symbol[PDSCH_NSYMB];
  uint8_t         lprime[PDSCH_NSYMB];
  uint32_t        c_init[PDSCH_NSYMB];
  float           w[4][4][2];   // [layer][port]
  uint16_t        crbs[PDSCH_MAX_RB];
};

// PT-RS of one PDU (ptrs_pdsch_generator_impl.cpp:30-130): PT-RS PRB i (CRB rb_begin + i rb_stride) carries, on
// every symbol of symbol_mask, sequence bits bit0 + i bit_step and the next one, at M_SQRT1_2 x amplitude, precoded
// with the layer-0 weights of the CRB's PRG.
struct ptrs_pdsch_args {
  uint32_t*       grid;        // cbf16 [port][14][nof_subc]
  const uint32_t* jump;        // Gold-sequence jump matrices
  const float*    w;           // [nof_prg][nof_ports] (re, im), device
  uint32_t        port_stride; // 14 x nof_subc
  uint32_t        nof_subc;
  uint32_t        c_init;
  uint32_t        bit0;
  uint32_t        bit_step;
  uint32_t        rb_begin;
  uint32_t        rb_stride;
  uint32_t        nof_prb;     // PT-RS PRBs
  uint32_t        k;           // subcarrier within the RB
  uint32_t        symbol_mask;
  float           amplitude;
  uint32_t        nof_ports;
  uint32_t        prg_size;
};

hipError_t launch_ptrs_pdsch_items(const ptrs_pdsch_args* items, uint32_t count, uint32_t max_prb, hipStream_t stream);

hipError_t launch_pdsch_map(const pdsch_map_args& a, uint32_t nof_symbols, uint32_t span_subc, uint32_t nof_cws,
                            hipStream_t stream);
hipError_t launch_dmrs_pdsch(const dmrs_pdsch_args& a, uint32_t nof_grids, hipStream_t stream);

// Slot form (srs_amd_pdsch_modulate_slot): one argument block per PDU in device memory (each on one grid and
// codeword, strides 0), PDU blockIdx.z; the launch covers the largest PDU (max_tiles x max_symbols
// workgroups, max_crb_blocks x max_symbols for the DM-RS) and each PDU's workgroups past its own extent exit.
hipError_t launch_pdsch_map_items(const pdsch_map_args* items, uint32_t count, uint32_t max_tiles,
                                  uint32_t max_symbols, hipStream_t stream);
hipError_t launch_dmrs_pdsch_items(const dmrs_pdsch_args* items, uint32_t count, uint32_t max_crb_blocks,
                                   uint32_t max_symbols, hipStream_t stream);

} // namespace srs_amd
