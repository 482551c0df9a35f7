// pucch_args.h -- per-PDU descriptor of the PUCCH Format 0 detector kernel (pucch.hip), built by the C-ABI
// (pucch_api.cpp).
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
  float2          seq[PUCCH_F0_MAX_CAND][2][12]; // the low-PAPR sequence of each candidate and symbol
};

// Detection of every PDU (one 64-thread workgroup per PDU), results into d_results.
hipError_t launch_pucch_f0(const pucch_f0_desc* d_desc, uint32_t nof, srs_amd_pucch_f0_result* d_results,
                           hipStream_t stream);

} // namespace srs_amd
