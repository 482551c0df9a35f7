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
  float2          seq[PUCCH_F0_MAX_CAND][2][12]; // the low-PAPR sequence of each candidate and symbol
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

} // namespace srs_amd
