// uci_args.h -- argument blocks of the UCI decoder kernels (uci_decoder.hip), shared with their C-ABI
// (uci_decoder_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "polar_args.h"

struct srs_amd_uci_decoder;

namespace srs_amd {

struct uci_short_args {
  const int8_t* llrs;
  uint64_t      llr_stride;
  uint8_t*      msgs;
  uint64_t      msg_stride;
  int32_t*      status;
  uint64_t      status_stride; // bytes
  uint32_t      E;
  uint32_t      K;             // 1 .. 11
  uint32_t      qm;            // bits per modulation symbol
  // slot form: decoded only when *pred == pred_val (pred null: always), see uci_slot_message
  const int32_t* pred     = nullptr;
  int32_t        pred_val = 0;
};

// Polar codeblocks already decoded (deallocated message bits, one per byte, rows of cb_stride): CRC check,
// filler removal, status.
struct uci_polar_args {
  const uint8_t* cbs;      // [message][C][cb_stride]
  uint64_t       cb_stride;
  uint8_t*       msgs;
  uint64_t       msg_stride;
  int32_t*       status;
  uint64_t       status_stride;
  uint32_t       C;        // codeblocks (1 or 2)
  uint32_t       A0, F0;   // payload bits / filler bits of codeblock 0
  uint32_t       A1;       // payload bits of codeblock 1
  uint32_t       L;        // CRC bits (6 or 11)
  const int32_t* pred     = nullptr; // slot form: as uci_short_args
  int32_t        pred_val = 0;
};

hipError_t launch_uci_short(const uci_short_args& a, uint32_t nof, hipStream_t stream);
hipError_t launch_uci_polar_finish(const uci_polar_args& a, uint32_t nof, hipStream_t stream);
// One UCI message of a slot (HARQ-ACK, CSI part 1 ... of one PUSCH PDU): its E LLRs, K payload bits and status.
struct uci_slot_message {
  const int8_t* llrs;
  uint32_t      E, K;
  int32_t       modulation;
  uint8_t*      msg;
  int32_t*      status;
  // decoded only when *pred == pred_val on the device (pred null: always): the CSI part 2 messages of a PDU, one per
  // size its CSI part 1 may select, share the PDU's LLR row, payload and status and run only for the selected size
  const int32_t* pred     = nullptr;
  int32_t        pred_val = 0;
};
// The descriptors of a slot's UCI decoding (uci_decoder_impl.cpp:47-111 per message): the 1-11 bit messages for the
// short-block kernel, every polar codeblock (its own code) for the polar decoder, the polar messages' CRC / filler
// step; cb_bytes: the decoded-codeblock scratch the polar rows take at d_cbs.
struct uci_slot_plan {
  std::vector<uci_short_args> shorts;
  std::vector<polar_args>     polars;
  std::vector<uci_polar_args> finishes;
  size_t                      cb_bytes = 0;
};
// Builds the plan (d_cbs may be null to size the scratch first).  Codes are created and cached by the decoder.
int uci_slot_build(::srs_amd_uci_decoder* dec, const uci_slot_message* msgs, uint32_t n, uint8_t* d_cbs,
                   uci_slot_plan& out);

// Slot forms: one argument block per message (device arrays), each with its own E / K / Qm.
hipError_t launch_uci_short_items(const uci_short_args* items, uint32_t n, hipStream_t stream);
hipError_t launch_uci_polar_finish_items(const uci_polar_args* items, uint32_t n, hipStream_t stream);

} // namespace srs_amd
