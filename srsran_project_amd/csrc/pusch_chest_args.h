// pusch_chest_args.h -- argument block of the PUSCH DM-RS channel-estimator
// kernels (pusch_chest.hip), shared with their C-ABI (pusch_chest_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "srsran_amd/pusch_chest.h"

namespace srs_amd {

constexpr int CH_MAXPIL   = 2048;           // pilots per DM-RS symbol (type 1: 6 x 275 = 1650)
constexpr int CS_THREADS  = 256;            // slice and stats kernel workgroups
constexpr int CS_PPT      = CH_MAXPIL / CS_THREADS;
constexpr int CH_TA_MAXN  = 4096;           // largest time-alignment IDFT
constexpr int CH_MAXV     = 12;             // MAX_V_PILOTS
constexpr int CH_MAXDMRS  = 4;              // DM-RS symbols per slot
constexpr int CH_MAXL     = 4;              // layers
constexpr int CH_SEQWORDS = 2 * CH_MAXPIL / 32 + 2;
constexpr int CH_NSYMB    = 14;
// per (grid, port) accumulators: [0] EPRE, [3] CFO valid, [4] CFO (normalised), [CH_ACC_RSRP + slice] the
// slices' RSRP shares
constexpr int CH_ACC_RSRP = 8;
constexpr int CH_ACC      = CH_ACC_RSRP + CH_MAXL * CH_MAXDMRS;

struct chest_args {
  // inputs / outputs
  const uint32_t*           grids;
  uint64_t                  grid_stride;
  uint32_t*                 estimates;
  uint64_t                  est_stride;
  srs_amd_chest_port_stats* stats;
  // scratch (per grid and port)
  float2* filt; // [L][nof_lse][npil]
  float2* freq; // [L][nof_lse][nof_re]
  float*  acc;  // [CH_ACC]: epre, -, -, cfo valid, cfo, -, -, -, rsrp per slice
  float*  corr; // [L][nof_lse][ta_n]: time-alignment correlation per slice
  uint32_t* dmrs_seq; // [CH_MAXDMRS][CH_SEQWORDS]: DM-RS Gold words of the batch
  const float2* lp_seq; // transform precoding: the low-PAPR pilot sequence [npil] (nullptr: Gold sequence)
  // constants
  const uint32_t* jump;    // Gold-sequence jump matrices
  const uint32_t* gold_basis; // Gold-sequence word basis [32][GOLD_BASIS_WORDS] (gold_sequence.h)
  const float2*   ta_tw;   // W_N^m table of the time-alignment IDFT size
  uint32_t nof_ports;
  uint32_t nsubc;
  uint32_t L;
  uint32_t ncdm;
  uint32_t nds;            // DM-RS symbols
  uint32_t nof_lse;        // 1 (average) or nds
  uint32_t npil;           // pilots per DM-RS symbol
  uint32_t nof_re;         // 12 x rb_count
  uint32_t prb_lo;
  uint32_t first_symbol;
  uint32_t nof_symbols;
  uint32_t dmrs_sym[CH_MAXDMRS];
  uint32_t c_init[CH_MAXDMRS];
  float    epoch[CH_NSYMB];
  float    beta;
  int32_t  fd;
  int32_t  td;
  int32_t  compensate_cfo;
  int32_t  nof_taps;
  int32_t  nof_v;          // virtual pilots per side (filter)
  float    rc[CH_MAXV + 4]; // filter coefficients (<= 15)
  // time-domain strategy per symbol of the allocation: lse slice i0, weight, interpolate flag
  int32_t  td_i0[CH_NSYMB];
  float    td_w[CH_NSYMB];
  int32_t  td_interp[CH_NSYMB];
  // time alignment
  uint32_t ta_n;
  int32_t  ta_max_taps;
  int32_t  ta_frac;
  double   ta_fs;
  float    scs_hz;
};

// Slot form (several PDUs of one grid, srs_amd_pusch_process_slot): one argument block per work item (one PDU on
// one grid, nof_ports of its own, grids / scratch / stats pointers of its own) in device memory; the kernels of a
// launch take item ids[blockIdx.z] (ids == nullptr: item blockIdx.z).
struct chest_items {
  const chest_args* items = nullptr;
  const uint32_t*   ids   = nullptr;
};

// The argument block of this workgroup: the launch's own (batch forms) or its item's (slot form); uniform
// addresses of memory no kernel of the launch writes, so the fields are scalar loads.
template <bool MULTI>
__device__ __forceinline__ const chest_args& item_args(const chest_args& a, const chest_items& m)
{
  if constexpr (MULTI) {
    const uint32_t z = m.ids != nullptr ? m.ids[blockIdx.z] : blockIdx.z;
    return m.items[z];
  } else {
    return a;
  }
}

// The slot form's pilot and statistics kernels over nof_items items (no expansion: the fused equalizer consumes
// freq / acc).  max_ports / max_slices: the largest nof_ports / L x nof_lse of the items.
hipError_t launch_chest_items(const chest_items& items, uint32_t nof_items, uint32_t max_ports, uint32_t max_slices,
                              uint32_t nof_small, hipStream_t stream);
// nof_small: items of at most 412 pilots per DM-RS symbol (the narrow workgroups, pusch_chest.hip chest_small).

// expand = false: pilot and time-alignment kernels only -- the per-subcarrier estimates (freq) and the
// per-port accumulators (acc) stay in the estimator's scratch for a consumer that rebuilds each RE's
// estimate itself (the PUSCH demodulator's fused equalizer, chest_device.h).
hipError_t launch_chest(const chest_args& a, uint32_t nof_grids, hipStream_t stream, bool expand = true);

// srs_amd_pusch_chest_estimate_batch without the expansion to per-RE estimates (nothing is written to an
// estimate tensor): *view receives the argument block whose freq / acc scratch the fused consumer reads,
// valid until the next call on this estimator.  Same validation and errors as the C-ABI call.
int chest_estimate_batch_unexpanded(::srs_amd_pusch_chest*            chest,
                                    const srs_amd_pusch_chest_config* cfg,
                                    const uint32_t*                   d_grids,
                                    uint64_t                          grid_stride,
                                    uint32_t                          nof_ports,
                                    uint32_t                          nof_subc,
                                    uint32_t                          nof_grids,
                                    srs_amd_chest_port_stats*         d_stats,
                                    void*                             stream,
                                    chest_args*                       view);

// One PDU of a slot (srs_amd_pusch_process_slot): its estimator configuration, the grid it occupies
// (cbf16 [port][14][nof_subc], shared with the slot's other PDUs) and its nof_ports port measurements.
struct chest_slot_item {
  const srs_amd_pusch_chest_config* cfg;
  const uint32_t*                   d_grid;
  uint32_t                          nof_ports;
  srs_amd_chest_port_stats*         d_stats;
};

// The unexpanded estimate of every PDU of a slot in one launch sequence (chest_items): per-PDU scratch and
// argument blocks, TA launches grouped by IDFT size.  views[i] receives PDU i's argument block (host copy)
// for the fused equalizer, valid until the next call on this estimator.
int chest_estimate_slot_unexpanded(::srs_amd_pusch_chest*  chest,
                                   const chest_slot_item*  items,
                                   uint32_t                nof_items,
                                   uint32_t                nof_subc,
                                   void*                   stream,
                                   chest_args*             views);

} // namespace srs_amd
