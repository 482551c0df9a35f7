// ldpc_codec_args.h -- kernel argument blocks and launchers of the LDPC
// encoder (ldpc_encoder.hip) and rate (de)matcher (ldpc_rate_matching.hip),
// shared with their C-ABI (ldpc_codec_api.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include "ldpc_common.h"
#include "rate_matching_common.h"

namespace srs_amd {

struct encode_args {
  const uint8_t*  msgs;      // [nof_cbs][msg_stride] packed messages
  uint8_t*        cws;       // [nof_cbs][cw_stride] packed shortened codewords
  const uint32_t* edges;     // lifted edge descriptors (var*Z | shift << 16), row-major
  uint32_t        msg_stride;
  uint32_t        cw_stride;
  uint32_t        nof_cbs;
  int32_t         bg;
  int32_t         Z;
  int32_t         K;         // K_bg
  int32_t         M;         // check rows
  int32_t         M_eff;     // rows computed: 4 + the extension rows whose parity columns are read
  int32_t         pack_bits; // leading bits of the shortened codeword written (multiple of 8 or N_short * Z)
  int32_t         N_short;
  int32_t         p0_shift;  // s: p0 = P^-s (sum of lambdas)
  int32_t         core_a[4]; // shift of column K_bg in rows 0..3 (0 where absent)
  int32_t         row_start[MAX_BG_M + 1];
  // optional per-codeblock lifting size (bit-sliced kernel, every Z >= 32 of one base graph): codeblock cb
  // uses rows[cb] and its edges at edges + rows[cb].edge_off; Z / M_eff above are then the launch maxima
  const struct enc_row_desc* rows;
};

// Per-codeblock graph of a mixed-lifting-size encoder launch (srs_amd_pdsch_encode_slot).
struct enc_row_desc {
  uint32_t Z;
  uint32_t edge_off;
  uint32_t M_eff;
  uint32_t pack_bits;
  uint32_t p0_shift;
  uint32_t core_a[3];
};

struct dematch_args {
  const int8_t*   in;
  const uint32_t* in_offsets;
  const uint32_t* rm_lengths;
  int8_t*         soft;
  uint32_t        soft_stride;
  uint32_t        nof_cbs;
  int32_t         new_data;
  int32_t         fresh;     // previous soft-buffer contents are known to be zero (not read)
  uint32_t        write_end; // soft-buffer bytes [write_end, N) are not written (nobody reads them); N: all
  rm_geometry     g;
  // optional per-codeblock geometry (replaces g / write_end): codeblock cb uses geos[row_geo[cb]]
  const uint32_t*    row_geo;
  const rm_geometry* geos;
  const uint32_t*    geo_write_end;
  // optional per-codeblock flags (replace new_data / fresh): bit 0 new data, bit 1 fresh (PUSCH slot form with HARQ)
  const uint8_t*     row_flags;
};

struct rate_match_args {
  const uint8_t*  cw;
  uint32_t        cw_stride;
  const uint32_t* rm_lengths;
  const uint32_t* out_offsets;
  uint8_t*        out;
  uint32_t        nof_cbs;
  rm_geometry     g;
  // optional per-codeblock geometry (replaces g): codeblock cb uses geos[row_geo[cb]]; the codeblocks
  // of one codeword share a geometry and the codewords of different geometries share no byte
  const uint32_t*    row_geo;
  const rm_geometry* geos;
};

hipError_t launch_ldpc_encode(const encode_args& a, int grid, hipStream_t stream);
size_t     ldpc_encode_lds_bytes(int K, int M_eff, int Z);
hipError_t launch_rate_dematch(const dematch_args& a, hipStream_t stream);
hipError_t launch_rate_match(const rate_match_args& a, uint32_t max_rm_length, hipStream_t stream);

} // namespace srs_amd
