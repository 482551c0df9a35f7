// pucch_args.h -- per-PDU / per-batch descriptors of the PUCCH Format 0 and Format 1 detector kernels (pucch.hip),
// built by the C-ABI (pucch_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "srsran_amd/pucch.h"

namespace srs_amd {

constexpr uint32_t PUCCH_F0_MAX_CAND = 8; // cyclic shifts of two HARQ-ACK bits with an SR opportunity

struct pucch_f0_desc {
  const uint32_t* grid;        // cbf16 [port][14][nof_subc]
  uint32_t        port_stride; // 14 x nof_subc
  uint32_t        nof_subc;
  uint32_t        l0, nsym;    // first OFDM symbol, 1 or 2 symbols
  uint32_t        subc0[2];    // first subcarrier of each symbol (second hop)
  uint32_t        nof_ports;
  uint32_t        ports[4];
  uint32_t        nof_cand;    // cyclic shifts to evaluate (1, 2, 4 or 8)
  uint32_t        nof_sr, nof_harq; // of the table's messages
  uint32_t        nof_sr_default;   // of the default (invalid) message: the SR opportunity
  float           threshold;   // pick_threshold(ports, symbols, candidates)
  uint8_t         msg[PUCCH_F0_MAX_CAND][3]; // SR, HARQ-ACK 0, HARQ-ACK 1 of each candidate (table order)
  uint8_t         alpha[PUCCH_F0_MAX_CAND][2]; // cyclic shift (m0 + m_cs + n_cs) mod 12 of each candidate and symbol
  float2          base[12];    // low-PAPR base sequence of group n_id mod 30
};

// Detection of every PDU (one 64-thread workgroup per PDU), results into d_results.
hipError_t launch_pucch_f0(const pucch_f0_desc* d_desc, uint32_t nof, srs_amd_pucch_f0_result* d_results,
                           hipStream_t stream);

constexpr uint32_t PUCCH_F1_MAX_ENTRIES = 84; // 12 initial cyclic shifts x 7 time-domain OCCs

struct pucch_f1_desc {
  const uint32_t* grid;        // cbf16 [port][14][nof_subc]
  uint32_t        port_stride; // 14 x nof_subc
  uint32_t        nof_subc;
  uint32_t        l0, nsym;    // allocation: first symbol and 4 .. 14 symbols
  uint32_t        nof_hops;    // 1, or 2 with frequency hopping
  uint32_t        subc0[2];    // first subcarrier of each hop
  uint32_t        nof_ports;
  uint32_t        ports[4];
  uint32_t        occ_mask;    // time-domain OCC indices in use
  uint32_t        nof_entries;
  uint32_t        entry0;      // first entry / result of the batch
  float           threshold;   // by ports x hops (pucch_detector_format1.cpp:194-212)
  uint8_t         alpha[14];   // base cyclic shift n_cs of each allocated symbol (m0 = m_cs = 0)
  float2          base[12];    // low-PAPR base sequence of group n_id mod 30
};

// Detection of every batch (one 64-thread workgroup per batch); entries[] of all batches, results alike.
hipError_t launch_pucch_f1(const pucch_f1_desc* d_desc, uint32_t nof, const srs_amd_pucch_f1_entry* d_entries,
                           srs_amd_pucch_result* d_results, hipStream_t stream);

constexpr uint32_t PUCCH_F2_MAX_PRB = 16;
constexpr uint32_t PUCCH_F2_MAX_RE  = 8 * PUCCH_F2_MAX_PRB * 2; // data REs of 16 PRBs over 2 symbols
constexpr uint32_t PUCCH_F2_MAX_E   = 2 * PUCCH_F2_MAX_RE;      // QPSK LLRs
constexpr uint32_t PUCCH_MAX_TA_N   = 256;                      // largest time-alignment IDFT of a PUCCH estimate

struct pucch_f2_desc {
  const uint32_t*           grid;        // cbf16 [port][14][nof_subc]
  uint32_t                  port_stride; // 14 x nof_subc
  uint32_t                  nof_subc;
  uint32_t                  l0, nsym;    // allocation: first symbol, 1 or 2 symbols
  uint32_t                  hop;         // frequency hopping (two hops of one symbol)
  uint32_t                  nof_prb;
  uint32_t                  prb[2];      // first PRB of allocated symbols 0 / 1 (absolute)
  uint32_t                  nof_ports;
  uint32_t                  ports[4];
  float                     epoch[2];    // start epochs of allocated symbols 0 / 1 (symbol units)
  float                     scs_hz;
  int32_t                   nof_taps;    // FD filter (filter_type(min(nof_prb, 3), 3))
  int32_t                   nof_v;       // virtual pilots per side
  float                     rc[11];
  uint32_t                  ta_n;        // time-alignment IDFT size
  int32_t                   ta_max_taps;
  int32_t                   ta_frac;     // fractional-delay refinement (ta_n below the largest IDFT)
  double                    ta_fs;       // sampling rate of the IDFT (x stride 3)
  uint32_t                  pil[2][4];   // DM-RS QPSK bits of allocated symbols 0 / 1 (2 per pilot)
  uint32_t                  scr[PUCCH_F2_MAX_E / 32]; // data scrambling sequence c(0 .. E - 1)
  uint32_t                  n_re;        // data REs, 8 nof_prb nsym
  uint32_t                  counts[4];   // HARQ-ACK, SR, CSI part 1, CSI part 2 bits
  int8_t*                   llr;         // the PDU's LLR row
  srs_amd_pucch_uci_result* result;      // its result record (CSI fields)
};

// Estimation, equalization, demapping and descrambling of every Format 2 PDU (one 256-thread workgroup each).
hipError_t launch_pucch_f2(const pucch_f2_desc* d_desc, uint32_t nof, hipStream_t stream);

// Status and payload bits of row j (decoder order) to result / payload row perm[j] (user order).
hipError_t launch_pucch_uci_finish(const int32_t* status, const uint8_t* messages, uint32_t msg_stride,
                                   const uint32_t* perm, const uint32_t* nbits, uint32_t nof,
                                   srs_amd_pucch_uci_result* results, uint8_t* payloads, uint64_t payload_stride,
                                   hipStream_t stream);

constexpr uint32_t PUCCH_F3_MAX_M    = 12 * 16;                   // subcarriers of a Format 3 allocation
constexpr uint32_t PUCCH_F3_MAX_DATA = 12;                        // data symbols (14 minus two DM-RS symbols)
constexpr uint32_t PUCCH_F3_MAX_E    = 2 * PUCCH_F3_MAX_M * PUCCH_F3_MAX_DATA;

struct pucch_f34_desc {
  const uint32_t*           grid;        // cbf16 [port][14][nof_subc]
  uint32_t                  port_stride;
  uint32_t                  nof_subc;
  uint32_t                  l0, nsym;
  uint32_t                  M;           // subcarriers (12 nof_prb)
  uint32_t                  dmrs_mask;   // allocated symbols carrying DM-RS
  uint32_t                  hop_sym;     // first allocated symbol of the second hop (nsym: no hopping)
  uint32_t                  subc0[2];    // first subcarrier of each hop
  uint32_t                  nof_ports;
  uint32_t                  ports[4];
  float                     epoch[14];   // start epochs of the allocated symbols
  float                     scs_hz;
  int32_t                   nof_taps, nof_v;
  float                     rc[31];
  uint32_t                  ta_n;
  int32_t                   ta_max_taps;
  int32_t                   ta_frac;
  double                    ta_fs;
  uint32_t                  qm;          // 0: pi/2-BPSK, 2: QPSK
  uint32_t                  occ_len;     // Format 4 spreading factor (1: Format 3)
  float2                    occ_w[12];   // Format 4 OCC w_n(k)
  uint32_t                  n_sym;       // modulation symbols after deprecoding / despreading
  uint32_t                  counts[4];
  const float2*             pil;         // DM-RS of each DM-RS symbol [nof DM-RS][M] (device)
  const uint32_t*           scr;         // scrambling sequence words (device)
  int8_t*                   llr;
  srs_amd_pucch_uci_result* result;
};

// Estimation, equalization, deprecoding, despreading, demapping and descrambling of every Format 3 / 4 PDU.
hipError_t launch_pucch_f34(const pucch_f34_desc* d_desc, uint32_t nof, hipStream_t stream);

} // namespace srs_amd
