// rate_matching_common.h -- circular-buffer geometry of LDPC rate matching
// (TS 38.212 Section 5.4.2.1), shared by the host and the kernels.
//
// Reference: lib/phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.cpp:36-91 (init)
// and ldpc_rate_dematcher_impl.cpp:45-118 (rate_dematch): Ncb = min(Nref, N) (N
// when Nref = 0), k0 = floor(shift_factor[rv] * Ncb / N) * Z, filler bits are
// the F positions [nof_sys - F, nof_sys) with nof_sys = (K_bg - 2) * Z, and the
// circular read skips them.
//
// "Walk" coordinates: the non-filler positions of [0, Ncb) numbered in order
// (position p < nof_info has walk index p, p >= nof_sys has p - F); the rate
// matcher reads walk indices rank0, rank0 + 1, ... modulo L = Ncb - F.
#pragma once

#include <cstdint>

namespace srs_amd {

struct rm_geometry {
  uint32_t N;        // N_short * Z: codeblock / soft-buffer length
  uint32_t Ncb;      // circular buffer length
  uint32_t nof_info; // nof_sys - F
  uint32_t nof_sys;  // (K_bg - 2) * Z
  uint32_t F;        // filler bits
  uint32_t k0;       // reference shift_k0
  uint32_t rank0;    // walk index of the first bit read
  uint32_t L;        // Ncb - F
  uint32_t Qm;       // modulation order
};

// Returns nullptr on success, else the reference's assertion message.
const char* make_rm_geometry(rm_geometry& g, uint32_t bg, uint32_t Z, uint32_t rv, uint32_t Qm, uint32_t Nref,
                             uint32_t F);

} // namespace srs_amd
