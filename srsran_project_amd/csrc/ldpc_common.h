// ldpc_common.h -- host/device shared definitions for the MI355X LDPC path.
//
// Mirrors the constants of the reference:
//   include/srsran/phy/upper/channel_coding/ldpc/ldpc.h        (lifting sizes, lengths)
//   lib/phy/upper/channel_coding/ldpc/ldpc_graph_impl.h:36-60   (BG dimensions)
//   include/srsran/phy/upper/log_likelihood_ratio.h:300-311      (LLR_MAX=120, LLR_INFTY=127)
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace srs_amd {

constexpr int LLR_MAX      = 120;
constexpr int LLR_INFINITY = 127;
// ldpc_decoder_impl.h:233 soft_bits_clamp_low/high.
constexpr int SOFT_CLAMP = 64;

constexpr int MAX_LIFTING_SIZE = 384;
constexpr int MAX_BG_M         = 46;
constexpr int MAX_BG_N_FULL    = 68;
constexpr int MAX_EDGES        = 316;
constexpr int BG1_MAX_DEGREE   = 19;
constexpr int BG2_MAX_DEGREE   = 10;

enum arith_flavour : int {
  // avx2_support.h:65 scale_epi8: floor(x * 52428 / 65536) -- AVX2/AVX512 decoders.
  ARITH_SIMD = 0,
  // ldpc_decoder_generic.cpp:66 scale_llr: round(x * 0.8f).
  ARITH_GENERIC = 1,
};

// Lifted Tanner graph of one (base graph, lifting size) pair, passed to the
// kernels by value (kernarg segment -> scalar loads).
struct lifted_graph {
  int32_t  bg;
  int32_t  Z;
  int32_t  K;       // information nodes (22 / 10)
  int32_t  N_full;  // 68 / 52
  int32_t  N_short; // 66 / 50
  int32_t  M;       // check nodes (46 / 42)
  int32_t  nedges;
  int32_t  row_start[MAX_BG_M + 1];
  // edge e: (var * Z) | (shift << 16), edges of check row m in [row_start[m], row_start[m+1]).
  uint32_t edge[MAX_EDGES];
};

// Arguments of the batched decoder kernel (ldpc_decoder.hip).
struct decode_args {
  const int8_t*   llrs;         // [nof_cbs][llr_stride]
  const uint32_t* llr_lens;     // optional per-codeblock input length
  uint8_t*        out;          // [nof_cbs][out_stride] packed MSB-first hard bits
  int32_t*        nof_iters;    // [nof_cbs]: iterations on CRC pass, -1 = no value
  int8_t*         soft_out;     // optional [nof_cbs][N_full*Z] final soft bits
  const uint32_t* crc_table;    // x^(k+L) mod g, k = 0..K*Z-1 (null = no CRC)
  const uint32_t* edges;        // device copy of lifted_graph::edge for this (BG, Z)
  uint32_t        llr_stride;
  uint32_t        llr_len;
  uint32_t        out_stride;
  uint32_t        nof_cbs;
  int32_t         nof_filler_bits;
  int32_t         max_iterations;
  int32_t         force_decoding;
  int32_t         aligned4;     // llrs and llr_stride are multiples of 4 bytes (vector loads)
  // optional: codeblock cb is not decoded (nof_iters[cb] = -2, output untouched) when the int32 at
  // skip_flags + cb * skip_stride is non-zero -- a PUSCH HARQ retransmission of a codeblock whose CRC
  // passed earlier is only rate dematched (pusch_decoder_impl.cpp:330-345)
  const uint8_t*  skip_flags;
  uint32_t        skip_stride;
  // optional per-codeblock filler-bit count (replaces nof_filler_bits): a launch over the codeblocks of
  // several transport blocks with different segmentations (srs_amd_pusch_decode_slot)
  const int32_t*  fillers;
  // optional per-codeblock graph (runtime-Z kernel only): codeblock cb has lifting size rows[cb].Z, its
  // edges at edges + rows[cb].edge_off and its CRC table at crc_table + rows[cb].crc_off (NO_CRC_ROW: none)
  const struct ldpc_row_desc* rows;
  // optional (high-rate kernel only): the soft row of codeblock cb is built in LDS from its received codeword LLRs
  // (cw_lengths[cb] = E of them at cw_llrs + cw_offsets[cb]) instead of read from llrs -- the PUSCH rate
  // dematcher's new-data, fresh-buffer, k0 = 0, no-wrap case (ldpc_rate_dematch_kernel) fused into the load:
  // position p < cw_nof_info takes deinterleaved LLR p, [cw_nof_info, + cw_filler) +infinity, then LLR p - filler
  // up to E + filler, zeros after
  const int8_t*   cw_llrs;
  const uint32_t* cw_offsets;
  const uint32_t* cw_lengths;
  uint32_t        cw_qm;
  uint32_t        cw_nof_info;
  uint32_t        cw_filler;
};

// Per-codeblock graph of a mixed-lifting-size launch (srs_amd_pusch_decode_slot).
struct ldpc_row_desc {
  uint32_t Z;
  uint32_t edge_off;
  uint32_t crc_off;
  uint32_t zmagic; // ldpc_z_magic(Z): i / Z = umulhi(i, zmagic) for i < 2^16
};

// ceil-ish 2^32 / Z with umulhi(i, m) == i / Z for every i < 2^16 and valid lifting size Z.
uint32_t ldpc_z_magic(uint32_t Z);

// The high-rate kernel takes (bg, Z) rows of llr_len LLRs (the launch conditions of ldpc_decode_hr_eligible that do
// not depend on buffers): the PUSCH decoder then fuses its rate dematching into the decoder's load.
bool ldpc_hr_takes(int bg, int Z, uint32_t llr_len);

// Waves per codeblock of the packed runtime-Z decoder kernel for (bg, Z) (Z a multiple of 4), 0 when that
// kernel does not take it (SRSRAN_AMD_LDPC_PK=0 disables it).
int ldpc_pk_waves(int bg, int Z);
constexpr uint32_t NO_CRC_ROW = 0xffffffffu;
constexpr int32_t LDPC_ITERS_SKIPPED = -2;

// Position of a lifting size in the 51-entry list (ldpc.h all_lifting_sizes), -1 if invalid.
int lifting_size_position(int Z);
constexpr int NOF_LIFTING_SIZES = 51;

// Fills g for (bg, Z); returns false for an invalid pair.
bool build_lifted_graph(lifted_graph& g, int bg, int Z);

// Edge descriptors of every lifted graph, [2 base graphs][51 lifting sizes][MAX_EDGES],
// in the order of build_lifted_graph (device tables of the decoder and encoder).
std::vector<uint32_t> all_lifted_edges();

// Offset of the (bg, Z) graph in all_lifted_edges().
inline size_t lifted_edges_offset(int bg, int Z)
{
  return (static_cast<size_t>(bg - 1) * NOF_LIFTING_SIZES + lifting_size_position(Z)) * MAX_EDGES;
}

// TS 38.212 Table 5.3.2-1 lifting-size set index, -1 if Z is not a valid lifting size.
int lifting_index(int Z);

// CRC polynomials of crc_calculator_generic_impl.cpp:27-52, by crc_generator_poly value.
bool crc_params(int poly, uint32_t& polynom, int& order);

// x^(k+L) mod g for k = 0..nbits-1: the CRC of a single 1 bit followed by k
// zeros (crc_calculator_generic_impl.cpp:116 long division), so the CRC of an
// n-bit message is the XOR of table[n-1-i] over its set bits i.
std::vector<uint32_t> crc_linear_table(int poly, int nbits);

} // namespace srs_amd
