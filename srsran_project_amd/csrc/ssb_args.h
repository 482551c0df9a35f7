// ssb_args.h -- per-block descriptor of the SS/PBCH block kernels (ssb.hip), built by the C-ABI (ssb_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

constexpr uint32_t SSB_A      = 32;  // PBCH payload bits (pbch_encoder::A)
constexpr uint32_t SSB_K      = 56;  // A + 24 CRC bits
constexpr uint32_t SSB_E      = 864; // rate-matched bits (pbch_encoder::E = pbch_modulator::M_bit)
constexpr uint32_t SSB_SC     = 240; // subcarriers of the block (20 RBs)
constexpr uint32_t SSB_SEQLEN = 127; // PSS / SSS length

struct ssb_desc {
  // encoding (pbch_encoder_impl.cpp:30-170)
  uint8_t  mib[24];        // MIB payload bits
  uint32_t sfn;
  uint32_t hrf;            // half-frame bit
  uint32_t ssb_idx;
  uint32_t L_max;
  uint32_t k_ssb;          // subcarrier offset (its bit 4 enters the payload when L_max != 64)
  uint32_t pci;            // scrambling c_init of the encoder and the modulator
  uint32_t enc_offset;     // first scrambling bit of the encoder: M v (M = A - 3 or A - 6, v = 2 sfn[2] + sfn[1])
  uint32_t msg_offset;     // its K interleaved bits in the message buffer (the polar encoder's input)
  uint32_t cw_offset;      // its E coded bits in the codeword buffer
  uint8_t  perm[SSB_K];    // PBCH input bit interleaver: c'[k] = c[perm[k]]
  // mapping (pbch_modulator_impl.cpp, dmrs_pbch_processor_impl.cpp, pss/sss_processor_impl.cpp)
  uint32_t* grid;          // cbf16 [port][14][nof_subc]
  uint32_t  port_stride;   // 14 x nof_subc
  uint32_t  nof_subc;
  uint32_t  k0, l0;        // first subcarrier and OFDM symbol of the block
  uint32_t  nof_ports;
  uint32_t  ports[4];
  uint32_t  mod_offset;    // first scrambling bit of the modulator: (ssb_idx & 7) x 864
  uint32_t  c_init_dmrs;
  float     pss_amp;       // convert_dB_to_amplitude(beta_pss)
  uint32_t  pss_m;         // 43 N_ID2 mod 127
  uint32_t  sss_m0, sss_m1;
};

// Payload generation, first scrambling, CRC24C attachment and interleaving of every block (one thread per block).
hipError_t launch_ssb_encode(const ssb_desc* d_desc, uint32_t nof, uint8_t* d_msgs, const uint32_t* jump,
                             hipStream_t stream);
// PBCH scrambling and QPSK, DM-RS, PSS and SSS of every block into its grid (one workgroup per (block, symbol));
// seq: the m-sequences x (PSS), x0, x1 (SSS), SSB_SEQLEN bytes each.
hipError_t launch_ssb_map(const ssb_desc* d_desc, uint32_t nof, const uint8_t* d_cws, const uint8_t* seq,
                          const uint32_t* jump, hipStream_t stream);

} // namespace srs_amd
