// pdcch_args.h -- per-DCI descriptor of the PDCCH kernels (pdcch.hip), built by the C-ABI (pdcch_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

constexpr uint32_t PDCCH_MAX_RB      = 96;  // aggregation level 16 x 6 REGs, one RB per REG bundle row
constexpr uint32_t PDCCH_MAX_K       = 164; // payload + CRC24 (DCI input bit interleaver K_IL^max)
constexpr uint32_t PDCCH_DATA_PER_RB = 9;   // data REs per RB and symbol (k mod 4 != 1)
constexpr uint32_t PDCCH_DMRS_PER_RB = 3;   // DM-RS REs per RB and symbol (k = 4 n + 1)

struct pdcch_desc {
  // encoding (pdcch_encoder_impl.cpp:43-98)
  uint32_t payload_offset; // its A payload bits (one per byte) in the payload buffer
  uint32_t payload_size;   // A
  uint32_t K;              // A + 24
  uint32_t rnti;           // scrambles the last 16 CRC bits
  uint32_t msg_offset;     // its K interleaved bits in the message buffer (the polar encoder's input)
  uint32_t cw_offset;      // its E coded bits (one per byte) in the codeword buffer
  uint32_t E;              // 108 x aggregation level
  uint8_t  perm[PDCCH_MAX_K]; // DCI input bit interleaver: c'[k] = c[perm[k]] (TS 38.212 5.3.1.1)
  // mapping (pdcch_modulator_impl.cpp, dmrs_pdcch_processor_impl.cpp)
  uint32_t* grid;          // cbf16 [port][14][nof_subc]
  uint32_t  port_stride;   // 14 x nof_subc
  uint32_t  nof_subc;
  uint32_t  nof_rb;        // CRBs of the DCI (ascending in crbs)
  uint32_t  start_symbol, duration;
  uint32_t  ref_k_rb;      // DM-RS reference point (CORESET0: the BWP start, else 0)
  uint32_t  c_init_data;   // (n_rnti 2^16 + n_id) mod 2^31
  uint32_t  c_init_dmrs[3];
  float     data_amp;      // convert_dB_to_amplitude(data power offset)
  int32_t   data_scaled;   // std::isnormal(data_amp): the symbols are multiplied by it
  float     dmrs_amp;      // M_SQRT1_2 x convert_dB_to_amplitude(DM-RS power offset), double product rounded
  uint32_t  nof_ports;
  float     w[4][2];       // port weights of the layer
  uint16_t  crbs[PDCCH_MAX_RB];
};

// CRC attachment, RNTI scrambling and interleaving of every DCI (one thread per DCI).
hipError_t launch_pdcch_crc(const pdcch_desc* d_desc, uint32_t nof, const uint8_t* d_payloads, uint8_t* d_msgs,
                            hipStream_t stream);
// Scrambling, QPSK, scaling, precoding and mapping of every DCI's data REs and its DM-RS (one workgroup per (DCI,
// symbol, 256 REs of its RBs)); jump: gold_jump_tables().
hipError_t launch_pdcch_map(const pdcch_desc* d_desc, uint32_t nof, uint32_t max_rb, uint32_t max_symbols,
                            const uint8_t* d_cws, const uint32_t* jump, hipStream_t stream);

} // namespace srs_amd
