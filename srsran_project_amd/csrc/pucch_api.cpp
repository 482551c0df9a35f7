// pucch_api.cpp -- C-ABI of the MI355X PUCCH Format 0 detector (include/srsran_amd/pucch.h):
// pucch_detector_format0::detect (pucch_detector_format0.cpp:124-246) for every PDU of a slot.  Host side, per PDU:
// the cyclic-shift table of the payload (TS 38.213 Tables 9.2.3-3 / 9.2.3-4 / 9.2.5-1 / 9.2.5-2 as the reference
// lists them, :48-71), the detection threshold (pick_threshold, :73-122), the group sequence u = n_id mod 30
// (pucch_helper::compute_group_sequence without hopping) and for every candidate and symbol the cyclic shift
// alpha = (m0 + m_cs + n_cs) mod 12, n_cs = sum_m 2^m c(8 (14 n_slot + l) + m) of the Gold sequence of n_id
// (pucch_helper::get_alpha_index), and its low-PAPR sequence (srs_amd_low_papr_sequence x e^(j 2 pi alpha n / 12));
// device side: pucch_f0_kernel.
//
// Format 1 (pucch_detector_format1.cpp:156-663 behind pucch_processor_impl.cpp:74-138): per batch, the checks of
// validate_config (:57-98) and of the processor's PDU validator, the threshold by ports x hops (:194-212), the base
// cyclic shift n_cs of every allocated symbol (get_alpha_index with m0 = m_cs = 0, :562), the base sequence of group
// n_id mod 30 and the set of OCC indices in use; device side: pucch_f1_kernel.
#include "srsran_amd/pucch.h"
#include "srsran_amd/low_papr.h"
#include "srsran_amd/uci_decoder.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "gold_sequence.h"
#include "pucch_args.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <numeric>
#include <vector>

using namespace srs_amd;

struct srs_amd_pucch_processor {
  int                   device = 0;
  std::vector<uint32_t> jump; // host copy of gold_jump_tables()
  device_buffer         buf, host_grid, host_res, work, host_payload;
  srs_amd_uci_decoder*  uci = nullptr;     // Formats 2 / 3 / 4
  pinned_stage          stage;
  stream_order          order;
  hipStream_t           stream = nullptr; // host calls
  std::mutex            mtx;
  std::mutex            host_mtx;
  ~srs_amd_pucch_processor()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    if (uci != nullptr) {
      srs_amd_uci_decoder_destroy(uci);
    }
  }
};

namespace {

constexpr uint32_t NSYMB = 14;

struct f0_entry {
  uint32_t m_cs;
  uint8_t  sr, h0, h1;
};
// pucch_detector_format0.cpp:48-71 (table order)
const f0_entry T_SR[1]       = {{0, 1, 0, 0}};
const f0_entry T_1H[2]       = {{0, 0, 0, 0}, {6, 0, 1, 0}};
const f0_entry T_2H[4]       = {{0, 0, 0, 0}, {3, 0, 0, 1}, {6, 0, 1, 1}, {9, 0, 1, 0}};
const f0_entry T_1H_SR[4]    = {{0, 0, 0, 0}, {6, 0, 1, 0}, {3, 1, 0, 0}, {9, 1, 1, 0}};
const f0_entry T_2H_SR[8]    = {{0, 0, 0, 0}, {3, 0, 0, 1}, {6, 0, 1, 1}, {9, 0, 1, 0},
                                {1, 1, 0, 0}, {4, 1, 0, 1}, {7, 1, 1, 1}, {10, 1, 1, 0}};

// pick_threshold (:73-122): the first entry (degrees of freedom, sequences) >= the request; < 0 when none.
float threshold(uint32_t nof_ports, uint32_t nof_symbols, uint32_t nof_seq)
{
  struct entry {
    uint32_t dof, nseq;
    float    th;
  };
  static const entry t[16] = {{1, 1, 0.5373f}, {1, 2, 0.6460f}, {1, 4, 0.7556f}, {1, 8, 1.6818f},
                              {2, 1, 0.5273f}, {2, 2, 0.4038f}, {2, 4, 0.7273f}, {2, 8, 0.8364f},
                              {4, 1, 0.3455f}, {4, 2, 0.2800f}, {4, 4, 0.4455f}, {4, 8, 0.5000f},
                              {8, 1, 0.2545f}, {8, 2, 0.2083f}, {8, 4, 0.3000f}, {8, 8, 0.3273f}};
  const uint32_t dof = nof_ports * nof_symbols;
  for (const entry& e : t) {
    if (e.dof > dof || (e.dof == dof && e.nseq >= nof_seq)) {
      return e.th;
    }
  }
  return -1.0f;
}

// e^(j 2 pi m / 12), m = 0 .. 11 (cos / sin in double, rounded to float), for the cyclic shifts.
const float2* twelfth_roots()
{
  static const std::vector<float2> t = [] {
    std::vector<float2> v(12);
    for (uint32_t m = 0; m != 12; ++m) {
      const double ph = 2.0 * M_PI * static_cast<double>(m) / 12.0;
      v[m]            = make_float2(static_cast<float>(std::cos(ph)), static_cast<float>(std::sin(ph)));
    }
    return v;
  }();
  return t.data();
}

uint32_t gf2_apply_h(const uint32_t* cols, uint32_t s)
{
  uint32_t r = 0;
  for (int j = 0; j < 31; ++j) {
    if ((s >> j) & 1u) {
      r ^= cols[j];
    }
  }
  return r;
}

// Gold-sequence bits c(n0 .. n0 + 7) of c_init (bit m of the result = c(n0 + m)), with the host jump tables.
uint32_t gold_byte(const std::vector<uint32_t>& jump, uint32_t c_init, uint32_t n0)
{
  uint32_t       x1 = 1u, x2 = c_init & 0x7fffffffu;
  const uint32_t steps = n0 + 1600u;
  for (int k = 0; k < PRBS_NJUMP; ++k) {
    if ((steps >> k) & 1u) {
      x1 = gf2_apply_h(jump.data() + (0 * PRBS_NJUMP + k) * 31, x1);
      x2 = gf2_apply_h(jump.data() + (1 * PRBS_NJUMP + k) * 31, x2);
    }
  }
  uint32_t out = 0;
  for (uint32_t m = 0; m != 8; ++m) {
    out |= ((x1 ^ x2) & 1u) << m;
    const uint32_t n1 = ((x1 >> 3) ^ x1) & 1u;
    const uint32_t n2 = ((x2 >> 3) ^ (x2 >> 2) ^ (x2 >> 1) ^ x2) & 1u;
    x1                = (x1 >> 1) | (n1 << 30);
    x2                = (x2 >> 1) | (n2 << 30);
  }
  return out;
}

// Gold-sequence bits c(n0 .. n0 + nbits - 1) of c_init into out (bit i of word i / 32).
void gold_bits(const std::vector<uint32_t>& jump, uint32_t c_init, uint32_t n0, uint32_t nbits, uint32_t* out)
{
  uint32_t       x1 = 1u, x2 = c_init & 0x7fffffffu;
  const uint32_t steps = n0 + 1600u;
  for (int k = 0; k < PRBS_NJUMP; ++k) {
    if ((steps >> k) & 1u) {
      x1 = gf2_apply_h(jump.data() + (0 * PRBS_NJUMP + k) * 31, x1);
      x2 = gf2_apply_h(jump.data() + (1 * PRBS_NJUMP + k) * 31, x2);
    }
  }
  // 32 outputs per step, word-parallel (the host twin of gold_sequence.h gold_next32): bit b of word w = c(n0 + 32 w + b)
  const uint32_t nwords = (nbits + 31) / 32;
  for (uint32_t w = 0; w != nwords; ++w) {
    uint64_t a = x1;
    a |= static_cast<uint64_t>(((a >> 3) ^ a) & 0x0fffffffu) << 31;
    a |= static_cast<uint64_t>(((a >> 31) ^ (a >> 28)) & 0xfu) << 59;
    uint64_t b = x2;
    b |= static_cast<uint64_t>(((b >> 3) ^ (b >> 2) ^ (b >> 1) ^ b) & 0x0fffffffu) << 31;
    b |= static_cast<uint64_t>(((b >> 31) ^ (b >> 30) ^ (b >> 29) ^ (b >> 28)) & 0xfu) << 59;
    x1     = static_cast<uint32_t>(a >> 32) & 0x7fffffffu;
    x2     = static_cast<uint32_t>(b >> 32) & 0x7fffffffu;
    out[w] = static_cast<uint32_t>(a ^ b);
  }
  if (nbits % 32 != 0) {
    out[nwords - 1] &= (1u << (nbits % 32)) - 1u;
  }
}

constexpr double T_C = 1.0 / (480000.0 * 4096.0);

// initialize_symbol_start_epochs (port_channel_estimator_average_impl.cpp:543-554), normal cyclic prefix.
void symbol_epochs(uint32_t mu, float* epoch)
{
  const unsigned scs_k = 15u << mu;
  auto           cp_s  = [mu](unsigned i) {
    unsigned k = 144u >> mu;
    if (i == 0 || i == 7u * (1u << mu)) {
      k += 16;
    }
    return static_cast<double>(k * 64) * T_C;
  };
  epoch[0] = static_cast<float>(cp_s(0) * scs_k * 1000);
  for (unsigned i = 1; i < NSYMB; ++i) {
    epoch[i] = static_cast<float>(epoch[i - 1] + cp_s(i) * scs_k * 1000 + 1.0F);
  }
}

const float RC_FILTER[31] = {-0.0641253, -0.0660711, -0.0611526, -0.0485918, -0.0281126, 0.0000000, 0.0348830,
                             0.0751249,  0.1188406,  0.1637874,  0.2075139,  0.2475302,  0.2814857, 0.3073415,
                             0.3235207,  0.3290274,  0.3235207,  0.3073415,  0.2814857,  0.2475302, 0.2075139,
                             0.1637874,  0.1188406,  0.0751249,  0.0348830,  0.0000000,  -0.0281126, -0.0485918,
                             -0.0611526, -0.0660711, -0.0641253};

// filter_type(nof_rb, stride) (port_channel_estimator_helpers.cpp:84-111) and the virtual pilots per side.
void fd_filter(uint32_t nof_rb, uint32_t stride, uint32_t npil, float* rc, int32_t& nof_taps, int32_t& nof_v)
{
  const unsigned nrb       = std::min(nof_rb, 3u);
  const unsigned nof_coefs = nrb * 10 + 1;
  unsigned       n_out     = nof_coefs / 2 / stride;
  const unsigned n_first   = 31 / 2 - n_out * stride;
  n_out                    = 2 * n_out + 1;
  float total              = 0;
  for (unsigned i = 0; i < n_out; ++i) {
    rc[i] = RC_FILTER[n_first + stride * i];
    total += rc[i];
  }
  const float inv = 1 / total;
  for (unsigned i = 0; i < n_out; ++i) {
    rc[i] *= inv;
  }
  nof_taps = static_cast<int32_t>(n_out);
  nof_v    = nof_rb == 1 ? static_cast<int32_t>(npil) : std::min<int32_t>(12, nof_taps / 2);
}

// time_alignment_estimator_dft_impl::get_idft / estimate_ta_correlation constants for npil pilots of a stride.
void ta_setup(uint32_t npil, uint32_t stride, uint32_t mu, uint32_t& n, int32_t& max_taps, int32_t& frac, double& fs)
{
  constexpr uint32_t MAX_N = 4096, MIN_N = 128;
  const uint32_t     req   = npil * MAX_N / (275 * 12);
  uint32_t           N     = 1;
  while (N < req) {
    N <<= 1;
  }
  N                     = std::max(MIN_N, N);
  n                     = N;
  fs                    = static_cast<double>(N) * (15u << mu) * 1000 * stride;
  const double half_cp  = static_cast<double>((144u * 64u) >> (mu + 1)) * T_C;
  max_taps              = static_cast<int32_t>(std::floor(half_cp * fs));
  frac                  = N != MAX_N ? 1 : 0;
}

// UCI CRC bits (uci_info.h:40-77).
uint32_t uci_crc_bits(uint32_t A, uint32_t E)
{
  const uint32_t C = ((A >= 360 && E >= 1088) || A >= 1013) ? 2u : 1u;
  const uint32_t L = A <= 11 ? 0u : (A <= 19 ? 6u : 11u);
  return C * L;
}

int make_f2_desc(const srs_amd_pucch_processor* proc, const srs_amd_pucch_f2_pdu& p, const uint32_t* d_grids,
                 uint64_t grid_stride, uint32_t nof_grids, uint32_t nof_grid_ports, uint32_t nof_subc,
                 pucch_f2_desc& d)
{
  const uint32_t grid_prb = nof_subc / 12;
  if (p.bwp_start_rb + p.bwp_size_rb > grid_prb) {
    return fail(SRS_AMD_EINVAL, "BWP allocation goes up to PRB %u, exceeding the configured maximum grid RB size, i.e., %u.",
                p.bwp_start_rb + p.bwp_size_rb, grid_prb);
  }
  if (p.nof_prb == 0 || p.nof_prb > PUCCH_F2_MAX_PRB || p.starting_prb + p.nof_prb > p.bwp_size_rb) {
    return fail(SRS_AMD_EINVAL, "PRB allocation within the BWP goes up to PRB %u, exceeding BWP size, i.e., %u.",
                p.starting_prb + p.nof_prb, p.bwp_size_rb);
  }
  if (p.nof_symbols == 0 || p.nof_symbols > 2 || p.start_symbol_index + p.nof_symbols > NSYMB) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 2 symbols (start %u, %u symbols).", p.start_symbol_index,
                p.nof_symbols);
  }
  if (p.second_hop_prb >= 0 && (p.nof_symbols != 2 ||
                                (p.bwp_start_rb + static_cast<uint32_t>(p.second_hop_prb) + p.nof_prb) > grid_prb)) {
    return fail(SRS_AMD_EINVAL, "Frequency hopping requires 2 OFDM symbols inside the grid.");
  }
  if (p.nof_ports == 0 || p.nof_ports > 4) {
    return fail(SRS_AMD_EINVAL, "The number of receive ports, i.e. %u, is not 1 to 4.", p.nof_ports);
  }
  if (p.nof_csi_part2 != 0) {
    return fail(SRS_AMD_EINVAL, "CSI Part 2 is not currently supported.");
  }
  if (p.numerology > 4 || p.slot_index >= (10u << p.numerology) || p.n_id > 1023 || p.rnti > 65535 ||
      p.n_id_0 > 65535) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 2 PDU (slot %u, numerology %u, RNTI %u, n_id %u, n_id_0 %u).",
                p.slot_index, p.numerology, p.rnti, p.n_id, p.n_id_0);
  }
  const uint32_t K = p.nof_harq_ack + p.nof_sr + p.nof_csi_part1 + p.nof_csi_part2;
  const uint32_t E = 16 * p.nof_prb * p.nof_symbols;
  if (K < 3 || K > 1706) {
    return fail(SRS_AMD_EINVAL, "UCI Payload length, i.e., %u is not supported. Payload length must be 3 to 1706 bits.",
                K);
  }
  if (static_cast<float>(K + uci_crc_bits(K, E)) / static_cast<float>(E) > 0.80F) {
    return fail(SRS_AMD_EINVAL, "The effective code rate exceeds the maximum allowed 0.8.");
  }
  if (p.d_grid == nullptr && (d_grids == nullptr || p.grid >= nof_grids)) {
    return fail(SRS_AMD_EINVAL, "grid index %u out of range (or no grid).", p.grid);
  }
  d             = pucch_f2_desc{};
  d.grid        = p.d_grid != nullptr ? p.d_grid : d_grids + p.grid * grid_stride;
  d.port_stride = NSYMB * nof_subc;
  d.nof_subc    = nof_subc;
  d.l0          = p.start_symbol_index;
  d.nsym        = p.nof_symbols;
  d.hop         = p.second_hop_prb >= 0 ? 1u : 0u;
  d.nof_prb     = p.nof_prb;
  d.prb[0]      = p.bwp_start_rb + p.starting_prb;
  d.prb[1]      = d.hop ? p.bwp_start_rb + static_cast<uint32_t>(p.second_hop_prb) : d.prb[0];
  d.nof_ports   = p.nof_ports;
  for (uint32_t i = 0; i != p.nof_ports; ++i) {
    if (p.ports[i] >= nof_grid_ports) {
      return fail(SRS_AMD_EINVAL, "port %u outside the grid's %u ports.", p.ports[i], nof_grid_ports);
    }
    d.ports[i] = p.ports[i];
  }
  float epoch[NSYMB];
  symbol_epochs(p.numerology, epoch);
  const uint32_t np = 4 * p.nof_prb;
  for (uint32_t s = 0; s != p.nof_symbols; ++s) {
    const uint32_t l      = p.start_symbol_index + s;
    d.epoch[s]            = epoch[l];
    const uint64_t c_init = ((static_cast<uint64_t>(NSYMB) * p.slot_index + l + 1) * (2ull * p.n_id_0 + 1) *
                                 (1ull << 17) + 2ull * p.n_id_0) % (1ull << 31);
    gold_bits(proc->jump, static_cast<uint32_t>(c_init), d.prb[s] * 4 * 2, 2 * np, d.pil[s]);
  }
  d.scs_hz = static_cast<float>((15u << p.numerology) * 1000);
  fd_filter(p.nof_prb, 3, np, d.rc, d.nof_taps, d.nof_v);
  ta_setup(np, 3, p.numerology, d.ta_n, d.ta_max_taps, d.ta_frac, d.ta_fs);
  gold_bits(proc->jump, p.rnti * (1u << 15) + p.n_id, 0, E, d.scr);
  d.n_re   = 8 * p.nof_prb * p.nof_symbols;
  d.counts[0] = p.nof_harq_ack;
  d.counts[1] = p.nof_sr;
  d.counts[2] = p.nof_csi_part1;
  d.counts[3] = p.nof_csi_part2;
  return SRS_AMD_OK;
}

// get_pucch_formats3_4_dmrs_symbol_mask (pucch_formats3_4_helpers.h): DM-RS symbols of a Format 3 / 4 allocation.
uint32_t f34_dmrs_mask(uint32_t nsym, bool hop, bool add)
{
  switch (nsym) {
    case 4:
      return hop ? 0b101u : 0b10u;
    case 5:
      return 0b1001u;
    case 6:
    case 7:
      return 0b10010u;
    case 8:
      return 0b100010u;
    case 9:
      return 0b1000010u;
    case 10:
      return add ? ((1u << 1) | (1u << 3) | (1u << 6) | (1u << 8)) : ((1u << 2) | (1u << 7));
    case 11:
      return add ? ((1u << 1) | (1u << 3) | (1u << 6) | (1u << 9)) : ((1u << 2) | (1u << 7));
    case 12:
      return add ? ((1u << 1) | (1u << 4) | (1u << 7) | (1u << 10)) : ((1u << 2) | (1u << 8));
    case 13:
      return add ? ((1u << 1) | (1u << 4) | (1u << 7) | (1u << 11)) : ((1u << 2) | (1u << 9));
    case 14:
      return add ? ((1u << 1) | (1u << 5) | (1u << 8) | (1u << 12)) : ((1u << 3) | (1u << 10));
    default:
      return 0;
  }
}

bool tp_prb_valid(uint32_t n) // transform_precoding::is_nof_prbs_valid: 2^a 3^b 5^c
{
  if (n == 0) {
    return false;
  }
  for (uint32_t f : {2u, 3u, 5u}) {
    while (n % f == 0) {
      n /= f;
    }
  }
  return n == 1;
}

// Formats 3 / 4: the descriptor plus the PDU's DM-RS (pil: nof DM-RS x M values) and scrambling words (scr).
int make_f34_desc(const srs_amd_pucch_processor* proc, const srs_amd_pucch_f34_pdu& p, const uint32_t* d_grids,
                  uint64_t grid_stride, uint32_t nof_grids, uint32_t nof_grid_ports, uint32_t nof_subc,
                  pucch_f34_desc& d, std::vector<float2>& pil, std::vector<uint32_t>& scr, uint32_t& E, uint32_t& K)
{
  const bool     f4       = p.format == 4;
  const uint32_t grid_prb = nof_subc / 12;
  if (p.format != 3 && p.format != 4) {
    return fail(SRS_AMD_EINVAL, "PUCCH format %u is not 3 or 4.", p.format);
  }
  const uint32_t nprb = f4 ? 1u : p.nof_prb;
  if (p.bwp_start_rb + p.bwp_size_rb > grid_prb) {
    return fail(SRS_AMD_EINVAL, "BWP allocation goes up to PRB %u, exceeding the configured maximum grid RB size, i.e., %u.",
                p.bwp_start_rb + p.bwp_size_rb, grid_prb);
  }
  if (nprb == 0 || nprb > 16 || !tp_prb_valid(nprb) || p.starting_prb + nprb > p.bwp_size_rb) {
    return fail(SRS_AMD_EINVAL, "Invalid PUCCH Format %u PRB allocation (%u PRBs from PRB %u of a %u-PRB BWP).",
                p.format, nprb, p.starting_prb, p.bwp_size_rb);
  }
  if (p.nof_symbols < 4 || p.nof_symbols > 14 || p.start_symbol_index + p.nof_symbols > NSYMB) {
    return fail(SRS_AMD_EINVAL, "Invalid Format %u symbols (start %u, %u symbols).", p.format, p.start_symbol_index,
                p.nof_symbols);
  }
  const bool hop = p.second_hop_prb >= 0;
  if (hop && p.bwp_start_rb + static_cast<uint32_t>(p.second_hop_prb) + nprb > grid_prb) {
    return fail(SRS_AMD_EINVAL, "Second hop PRB allocation outside the grid.");
  }
  if (p.nof_ports == 0 || p.nof_ports > 4) {
    return fail(SRS_AMD_EINVAL, "The number of receive ports, i.e. %u, is not 1 to 4.", p.nof_ports);
  }
  if (p.nof_csi_part2 != 0) {
    return fail(SRS_AMD_EINVAL, "CSI Part 2 is not currently supported.");
  }
  if (f4 && ((p.occ_length != 2 && p.occ_length != 4) || p.occ_index >= p.occ_length)) {
    return fail(SRS_AMD_EINVAL, "Invalid OCC length value (i.e., %u) or index (i.e., %u).", p.occ_length,
                p.occ_index);
  }
  if (p.numerology > 4 || p.slot_index >= (10u << p.numerology) || p.n_id_hopping > 1023 ||
      p.n_id_scrambling > 1023 || p.rnti > 65535) {
    return fail(SRS_AMD_EINVAL, "Invalid Format %u PDU (slot %u, numerology %u, RNTI %u, n_id %u / %u).", p.format,
                p.slot_index, p.numerology, p.rnti, p.n_id_hopping, p.n_id_scrambling);
  }
  const uint32_t mask = f34_dmrs_mask(p.nof_symbols, hop, p.additional_dmrs != 0);
  const uint32_t nd   = static_cast<uint32_t>(__builtin_popcount(mask));
  const uint32_t nds  = p.nof_symbols - nd;
  const uint32_t qb   = p.pi2_bpsk ? 1u : 2u;
  const uint32_t M    = 12 * nprb;
  const uint32_t occ  = f4 ? p.occ_length : 1u;
  K                   = p.nof_harq_ack + p.nof_sr + p.nof_csi_part1 + p.nof_csi_part2;
  E                   = nds * M * qb / occ;
  // pucch_format3_code_rate / pucch_format4_code_rate (pucch_info.h:80-120)
  const uint32_t e_tot = f4 ? 12 * nds * qb / occ : M * nds * qb;
  const uint32_t chan  = f4 ? 12 * nds * qb : M * nds * qb;
  if (K < 3 || K > 1706) {
    return fail(SRS_AMD_EINVAL, "UCI Payload length (i.e., %u) is outside the supported range (i.e., [3, 1706]).", K);
  }
  if (static_cast<float>(K + uci_crc_bits(K, e_tot)) / static_cast<float>(chan) > 0.80F) {
    return fail(SRS_AMD_EINVAL, "The effective code rate exceeds the maximum allowed 0.8.");
  }
  if (p.d_grid == nullptr && (d_grids == nullptr || p.grid >= nof_grids)) {
    return fail(SRS_AMD_EINVAL, "grid index %u out of range (or no grid).", p.grid);
  }
  d             = pucch_f34_desc{};
  d.grid        = p.d_grid != nullptr ? p.d_grid : d_grids + p.grid * grid_stride;
  d.port_stride = NSYMB * nof_subc;
  d.nof_subc    = nof_subc;
  d.l0          = p.start_symbol_index;
  d.nsym        = p.nof_symbols;
  d.M           = M;
  d.dmrs_mask   = mask;
  d.hop_sym     = hop ? p.nof_symbols / 2 : p.nof_symbols;
  d.subc0[0]    = 12 * (p.bwp_start_rb + p.starting_prb);
  d.subc0[1]    = hop ? 12 * (p.bwp_start_rb + static_cast<uint32_t>(p.second_hop_prb)) : d.subc0[0];
  d.nof_ports   = p.nof_ports;
  for (uint32_t i = 0; i != p.nof_ports; ++i) {
    if (p.ports[i] >= nof_grid_ports) {
      return fail(SRS_AMD_EINVAL, "port %u outside the grid's %u ports.", p.ports[i], nof_grid_ports);
    }
    d.ports[i] = p.ports[i];
  }
  float epoch[NSYMB];
  symbol_epochs(p.numerology, epoch);
  for (uint32_t r = 0; r != p.nof_symbols; ++r) {
    d.epoch[r] = epoch[p.start_symbol_index + r];
  }
  d.scs_hz = static_cast<float>((15u << p.numerology) * 1000);
  fd_filter(nprb, 1, M, d.rc, d.nof_taps, d.nof_v);
  ta_setup(M, 1, p.numerology, d.ta_n, d.ta_max_taps, d.ta_frac, d.ta_fs);
  // DM-RS: the low-PAPR sequence of group n_id mod 30 (v = 0), cyclic shift (m0 + n_cs) mod 12 per DM-RS symbol with
  // m0 = 0, 6, 3, 9 for OCC index 0 .. 3 (dmrs_pucch_estimator_formats3_4.cpp:30-55)
  std::vector<float> base(2 * M);
  if (srs_amd_low_papr_sequence(base.data(), M, p.n_id_hopping % 30, 0) != SRS_AMD_OK) {
    return SRS_AMD_EINVAL;
  }
  static const uint32_t m0_of[4] = {0, 6, 3, 9};
  const uint32_t        m0       = f4 ? m0_of[p.occ_index & 3] : 0u;
  for (uint32_t r = 0; r != p.nof_symbols; ++r) {
    if (!((mask >> r) & 1u)) {
      continue;
    }
    const uint32_t n_cs  = gold_byte(proc->jump, p.n_id_hopping, 8 * (NSYMB * p.slot_index + p.start_symbol_index + r));
    const uint32_t alpha = (m0 + n_cs) % 12;
    const float2* ph = twelfth_roots();
    for (uint32_t k = 0; k != M; ++k) {
      const float2 e = ph[(alpha * k) % 12];
      const float  br = base[2 * k], bi = base[2 * k + 1];
      pil.push_back(make_float2(br * e.x - bi * e.y, br * e.y + bi * e.x));
    }
  }
  d.qm      = p.pi2_bpsk ? 0u : 2u;
  d.occ_len = occ;
  if (f4) {
    // pucch_orthogonal_sequence_format4 (pucch_orthogonal_sequence.h:162-172)
    static const float2 W2[2][12] = {{{1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0},
                                      {1, 0}, {1, 0}},
                                     {{1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {-1, 0}, {-1, 0}, {-1, 0},
                                      {-1, 0}, {-1, 0}, {-1, 0}}};
    static const float2 W4[4][12] = {
        {{1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}, {1, 0}},
        {{1, 0}, {1, 0}, {1, 0}, {0, -1}, {0, -1}, {0, -1}, {-1, 0}, {-1, 0}, {-1, 0}, {0, 1}, {0, 1}, {0, 1}},
        {{1, 0}, {1, 0}, {1, 0}, {-1, 0}, {-1, 0}, {-1, 0}, {1, 0}, {1, 0}, {1, 0}, {-1, 0}, {-1, 0}, {-1, 0}},
        {{1, 0}, {1, 0}, {1, 0}, {0, 1}, {0, 1}, {0, 1}, {-1, 0}, {-1, 0}, {-1, 0}, {0, -1}, {0, -1}, {0, -1}}};
    for (uint32_t k = 0; k != 12; ++k) {
      d.occ_w[k] = occ == 2 ? W2[p.occ_index][k] : W4[p.occ_index][k];
    }
  }
  d.n_sym = nds * M / occ;
  scr.assign((E + 31) / 32, 0u);
  gold_bits(proc->jump, p.rnti * (1u << 15) + p.n_id_scrambling, 0, E, scr.data());
  d.counts[0] = p.nof_harq_ack;
  d.counts[1] = p.nof_sr;
  d.counts[2] = p.nof_csi_part1;
  d.counts[3] = p.nof_csi_part2;
  return SRS_AMD_OK;
}

// The Format 3 / 4 slot form; decode = false stops after the LLRs (rows of PUCCH_F3_MAX_E in proc->work).
int f34_slot(srs_amd_pucch_processor*     proc,
             const srs_amd_pucch_f34_pdu* pdus,
             uint32_t                     nof_pdus,
             const uint32_t*              d_grids,
             uint64_t                     grid_stride,
             uint32_t                     nof_grids,
             uint32_t                     nof_grid_ports,
             uint32_t                     nof_subc,
             srs_amd_pucch_uci_result*    d_results,
             uint8_t*                     d_payloads,
             uint64_t                     payload_stride,
             void*                        stream,
             bool                         decode)
{
  if (proc == nullptr || (nof_pdus != 0 && (pdus == nullptr || d_results == nullptr || d_payloads == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_pdus == 0) {
    return SRS_AMD_OK;
  }
  if (nof_subc == 0 || nof_subc % 12 != 0) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  std::lock_guard<std::mutex>        lock(proc->mtx);
  std::vector<pucch_f34_desc>        desc(nof_pdus);
  std::vector<std::vector<float2>>   pil(nof_pdus);
  std::vector<std::vector<uint32_t>> scr(nof_pdus);
  std::vector<uint32_t>              K(nof_pdus), E(nof_pdus), Q(nof_pdus);
  uint32_t                           max_k = 0;
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const int rc = make_f34_desc(proc, pdus[i], d_grids, grid_stride, nof_grids, nof_grid_ports, nof_subc, desc[i],
                                 pil[i], scr[i], E[i], K[i]);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    if (K[i] > payload_stride) {
      return fail(SRS_AMD_EINVAL, "payload_stride %llu below the PDU's %u payload bits.",
                  static_cast<unsigned long long>(payload_stride), K[i]);
    }
    Q[i]  = pdus[i].pi2_bpsk ? 0u : 2u;
    max_k = std::max(max_k, K[i]);
  }
  std::vector<uint32_t> perm(nof_pdus);
  std::iota(perm.begin(), perm.end(), 0u);
  std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) {
    return K[a] != K[b] ? K[a] < K[b] : (E[a] != E[b] ? E[a] < E[b] : Q[a] < Q[b]);
  });
  const uint32_t msg_stride = (std::max(max_k, 1u) + 63) / 64 * 64;
  const size_t   llr_bytes  = static_cast<size_t>(nof_pdus) * PUCCH_F3_MAX_E;
  const size_t   msg_bytes  = static_cast<size_t>(nof_pdus) * msg_stride;
  const size_t   st_bytes   = static_cast<size_t>(nof_pdus) * sizeof(int32_t);
  auto           s          = static_cast<hipStream_t>(stream);
  hipError_t     e          = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->work.ensure(llr_bytes + msg_bytes + st_bytes);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH processor scratch");
  }
  int8_t*  d_llr = proc->work.as<int8_t>();
  uint8_t* d_msg = proc->work.as<uint8_t>() + llr_bytes;
  int32_t* d_st  = reinterpret_cast<int32_t*>(proc->work.as<uint8_t>() + llr_bytes + msg_bytes);
  // stage layout: descriptors (decoder order), perm, nbits, then every PDU's DM-RS and scrambling words
  const size_t dbytes = sizeof(pucch_f34_desc) * nof_pdus;
  const size_t ioff   = (dbytes + 255) & ~size_t(255);
  const size_t ibytes = sizeof(uint32_t) * nof_pdus;
  size_t       off    = (ioff + 2 * ibytes + 255) & ~size_t(255);
  std::vector<size_t> pil_off(nof_pdus), scr_off(nof_pdus);
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    pil_off[i] = off;
    off        = (off + pil[i].size() * sizeof(float2) + 15) & ~size_t(15);
    scr_off[i] = off;
    off        = (off + scr[i].size() * sizeof(uint32_t) + 15) & ~size_t(15);
  }
  const size_t bytes = off;
  if (e == hipSuccess) {
    e = proc->buf.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->stage.acquire(bytes);
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH processor scratch");
  }
  std::vector<pucch_f34_desc> ordered(nof_pdus);
  std::vector<uint32_t>       nbits(nof_pdus);
  for (uint32_t j = 0; j != nof_pdus; ++j) {
    const uint32_t i = perm[j];
    ordered[j]       = desc[i];
    ordered[j].pil    = reinterpret_cast<const float2*>(proc->buf.as<uint8_t>() + pil_off[i]);
    ordered[j].scr    = reinterpret_cast<const uint32_t*>(proc->buf.as<uint8_t>() + scr_off[i]);
    ordered[j].llr    = d_llr + static_cast<size_t>(j) * PUCCH_F3_MAX_E;
    ordered[j].result = d_results + i;
    nbits[j]          = K[i];
  }
  call_scope scope(proc->order, nullptr, s);
  std::memcpy(proc->stage.at<uint8_t>(0), ordered.data(), dbytes);
  std::memcpy(proc->stage.at<uint8_t>(ioff), perm.data(), ibytes);
  std::memcpy(proc->stage.at<uint8_t>(ioff + ibytes), nbits.data(), ibytes);
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    std::memcpy(proc->stage.at<uint8_t>(pil_off[i]), pil[i].data(), pil[i].size() * sizeof(float2));
    std::memcpy(proc->stage.at<uint8_t>(scr_off[i]), scr[i].data(), scr[i].size() * sizeof(uint32_t));
  }
  e = proc->stage.upload(proc->buf.ptr, bytes, s);
  if (e == hipSuccess) {
    e = launch_pucch_f34(proc->buf.as<pucch_f34_desc>(), nof_pdus, s);
  }
  int rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pucch_f34_kernel launch");
  for (uint32_t j0 = 0; decode && rc == SRS_AMD_OK && j0 != nof_pdus;) {
    const uint32_t i0 = perm[j0];
    uint32_t       j1 = j0 + 1;
    while (j1 != nof_pdus && K[perm[j1]] == K[i0] && E[perm[j1]] == E[i0] && Q[perm[j1]] == Q[i0]) {
      ++j1;
    }
    rc = srs_amd_uci_decode_batch(proc->uci, d_llr + static_cast<size_t>(j0) * PUCCH_F3_MAX_E, PUCCH_F3_MAX_E, E[i0],
                                  K[i0], static_cast<int32_t>(Q[i0]), d_msg + static_cast<size_t>(j0) * msg_stride,
                                  msg_stride, d_st + j0, sizeof(int32_t), j1 - j0, s);
    j0 = j1;
  }
  if (decode && rc == SRS_AMD_OK) {
    const uint32_t* d_perm = reinterpret_cast<const uint32_t*>(proc->buf.as<uint8_t>() + ioff);
    e  = launch_pucch_uci_finish(d_st, d_msg, msg_stride, d_perm, d_perm + nof_pdus, nof_pdus, d_results, d_payloads,
                                 payload_stride, s);
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pucch_uci_finish_kernel launch");
  }
  const hipError_t done = scope.close();
  return rc != SRS_AMD_OK ? rc : (done == hipSuccess ? SRS_AMD_OK : hip_fail(done, "PUCCH completion event"));
}

int make_desc(const srs_amd_pucch_processor* proc, const srs_amd_pucch_f0_pdu& p, const uint32_t* d_grids,
              uint64_t grid_stride, uint32_t nof_grids, uint32_t nof_grid_ports, uint32_t nof_subc, pucch_f0_desc& d)
{
  if (p.nof_symbols < 1 || p.nof_symbols > 2 || p.start_symbol_index + p.nof_symbols > NSYMB) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 0 symbols (start %u, %u symbols).", p.start_symbol_index,
                p.nof_symbols);
  }
  if (p.second_hop_prb >= 0 && p.nof_symbols != 2) {
    return fail(SRS_AMD_EINVAL, "Frequency hopping needs 2 OFDM symbols.");
  }
  if (p.initial_cyclic_shift > 11 || p.nof_harq_ack > 2 || p.nof_ports == 0 || p.nof_ports > 4 ||
      p.numerology > 4 || p.slot_index >= (10u << p.numerology) || p.n_id > 1023) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 0 PDU (m0 %u, %u HARQ-ACK bits, %u ports, slot %u, n_id %u).",
                p.initial_cyclic_shift, p.nof_harq_ack, p.nof_ports, p.slot_index, p.n_id);
  }
  if (p.nof_harq_ack == 0 && !p.sr_opportunity) {
    return fail(SRS_AMD_EINVAL, "Invalid payload combination.");
  }
  if (p.d_grid == nullptr && (d_grids == nullptr || p.grid >= nof_grids)) {
    return fail(SRS_AMD_EINVAL, "grid index %u out of range (or no grid).", p.grid);
  }
  d      = pucch_f0_desc{};
  d.grid = p.d_grid != nullptr ? p.d_grid : d_grids + p.grid * grid_stride;
  d.port_stride = NSYMB * nof_subc;
  d.nof_subc    = nof_subc;
  d.l0          = p.start_symbol_index;
  d.nsym        = p.nof_symbols;
  for (uint32_t l = 0; l != p.nof_symbols; ++l) {
    const uint32_t prb = (l != 0 && p.second_hop_prb >= 0) ? static_cast<uint32_t>(p.second_hop_prb) : p.starting_prb;
    if (12 * (prb + 1) > nof_subc) {
      return fail(SRS_AMD_EINVAL, "PRB %u outside the grid.", prb);
    }
    d.subc0[l] = 12 * prb;
  }
  d.nof_ports = p.nof_ports;
  for (uint32_t i = 0; i != p.nof_ports; ++i) {
    if (p.ports[i] >= nof_grid_ports) {
      return fail(SRS_AMD_EINVAL, "port %u outside the grid's %u ports.", p.ports[i], nof_grid_ports);
    }
    d.ports[i] = p.ports[i];
  }
  const f0_entry* tab = T_SR;
  uint32_t        n   = 1;
  if (p.nof_harq_ack == 1) {
    tab = p.sr_opportunity ? T_1H_SR : T_1H;
    n   = p.sr_opportunity ? 4 : 2;
  } else if (p.nof_harq_ack == 2) {
    tab = p.sr_opportunity ? T_2H_SR : T_2H;
    n   = p.sr_opportunity ? 8 : 4;
  }
  d.nof_cand       = n;
  d.nof_sr         = p.nof_harq_ack == 0 ? 1u : (p.sr_opportunity ? 1u : 0u);
  d.nof_harq       = p.nof_harq_ack;
  d.nof_sr_default = p.sr_opportunity ? 1u : 0u;
  d.threshold      = threshold(p.nof_ports, p.nof_symbols, n);
  if (d.threshold < 0) {
    return fail(SRS_AMD_EINVAL, "Requested configuration (%u antenna ports, %u OFDM symbols, %u sequences) not supported.",
                p.nof_ports, p.nof_symbols, n);
  }
  // base sequence of group u = n_id mod 30 (v = 0), then the cyclic shift of each candidate and symbol
  float base[24];
  if (srs_amd_low_papr_sequence(base, 12, p.n_id % 30, 0) != SRS_AMD_OK) {
    return SRS_AMD_EINVAL;
  }
  uint32_t n_cs[2] = {0, 0}; // the Gold-sequence shift of each symbol, common to every candidate
  for (uint32_t l = 0; l != p.nof_symbols; ++l) {
    n_cs[l] = gold_byte(proc->jump, p.n_id, 8 * (NSYMB * p.slot_index + p.start_symbol_index + l));
  }
  for (uint32_t k = 0; k != 12; ++k) {
    d.base[k] = make_float2(base[2 * k], base[2 * k + 1]);
  }
  for (uint32_t c = 0; c != n; ++c) {
    d.msg[c][0] = tab[c].sr;
    d.msg[c][1] = tab[c].h0;
    d.msg[c][2] = tab[c].h1;
    for (uint32_t l = 0; l != p.nof_symbols; ++l) {
      d.alpha[c][l] = static_cast<uint8_t>((p.initial_cyclic_shift + tab[c].m_cs + n_cs[l]) % 12);
    }
  }
  return SRS_AMD_OK;
}

int make_f1_desc(const srs_amd_pucch_processor* proc, const srs_amd_pucch_f1_batch& b, const uint32_t* d_grids,
                 uint64_t grid_stride, uint32_t nof_grids, uint32_t nof_grid_ports, uint32_t nof_subc, uint32_t entry0,
                 pucch_f1_desc& d)
{
  if (b.start_symbol_index > 10 || b.nof_symbols < 4 || b.nof_symbols > 14 ||
      b.start_symbol_index + b.nof_symbols > NSYMB) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 1 symbols (start %u, %u symbols).", b.start_symbol_index,
                b.nof_symbols);
  }
  if (b.numerology > 4 || b.slot_index >= (10u << b.numerology) || b.n_id > 1023) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 1 batch (slot %u, numerology %u, n_id %u).", b.slot_index,
                b.numerology, b.n_id);
  }
  const uint32_t hops = b.second_hop_prb >= 0 ? 2u : 1u;
  const uint32_t contributions = b.nof_ports * hops;
  if (b.nof_ports == 0 || b.nof_ports > 4 ||
      (contributions != 1 && contributions != 2 && contributions != 4 && contributions != 8)) {
    return fail(SRS_AMD_EINVAL, "The PUCCH detector does not support %u ports.", b.nof_ports);
  }
  if (b.nof_entries == 0 || b.nof_entries > PUCCH_F1_MAX_ENTRIES || b.entries == nullptr) {
    return fail(SRS_AMD_EINVAL, "Invalid number of multiplexed PUCCH (i.e., %u).", b.nof_entries);
  }
  if (b.d_grid == nullptr && (d_grids == nullptr || b.grid >= nof_grids)) {
    return fail(SRS_AMD_EINVAL, "grid index %u out of range (or no grid).", b.grid);
  }
  d             = pucch_f1_desc{};
  d.grid        = b.d_grid != nullptr ? b.d_grid : d_grids + b.grid * grid_stride;
  d.port_stride = NSYMB * nof_subc;
  d.nof_subc    = nof_subc;
  d.l0          = b.start_symbol_index;
  d.nsym        = b.nof_symbols;
  d.nof_hops    = hops;
  for (uint32_t h = 0; h != hops; ++h) {
    const uint32_t prb = h == 0 ? b.starting_prb : static_cast<uint32_t>(b.second_hop_prb);
    if (prb > 274 || 12 * (prb + 1) > nof_subc) {
      return fail(SRS_AMD_EINVAL, "PRB %u outside the grid.", prb);
    }
    d.subc0[h] = 12 * prb;
  }
  d.nof_ports = b.nof_ports;
  for (uint32_t i = 0; i != b.nof_ports; ++i) {
    if (b.ports[i] >= nof_grid_ports) {
      return fail(SRS_AMD_EINVAL, "port %u outside the grid's %u ports.", b.ports[i], nof_grid_ports);
    }
    d.ports[i] = b.ports[i];
  }
  const uint32_t occ_ratio = hops == 2 ? 4u : 2u;
  uint32_t       used[7]   = {};
  for (uint32_t e = 0; e != b.nof_entries; ++e) {
    const srs_amd_pucch_f1_entry& en = b.entries[e];
    if (en.initial_cyclic_shift > 11 || en.time_domain_occ > 6 || en.time_domain_occ >= b.nof_symbols / occ_ratio ||
        en.nof_harq_ack > 2) {
      return fail(SRS_AMD_EINVAL, "Invalid multiplexed PUCCH (shift %u, OCC %u, %u HARQ-ACK bits, %u symbols).",
                  en.initial_cyclic_shift, en.time_domain_occ, en.nof_harq_ack, b.nof_symbols);
    }
    if ((used[en.time_domain_occ] >> en.initial_cyclic_shift) & 1u) {
      return fail(SRS_AMD_EINVAL, "Two PUCCH with shift %u and OCC %u.", en.initial_cyclic_shift, en.time_domain_occ);
    }
    used[en.time_domain_occ] |= 1u << en.initial_cyclic_shift;
    d.occ_mask |= 1u << en.time_domain_occ;
  }
  d.nof_entries = b.nof_entries;
  d.entry0      = entry0;
  d.threshold   = contributions == 1 ? 0.9f : contributions == 2 ? 3.0f : contributions == 4 ? 4.45f : 6.95f;
  for (uint32_t r = 0; r != b.nof_symbols; ++r) {
    d.alpha[r] = static_cast<uint8_t>(
        gold_byte(proc->jump, b.n_id, 8 * (NSYMB * b.slot_index + b.start_symbol_index + r)) % 12);
  }
  float base[24];
  if (srs_amd_low_papr_sequence(base, 12, b.n_id % 30, 0) != SRS_AMD_OK) {
    return SRS_AMD_EINVAL;
  }
  for (uint32_t k = 0; k != 12; ++k) {
    d.base[k] = make_float2(base[2 * k], base[2 * k + 1]);
  }
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_pucch_processor_create(srs_amd_pucch_processor** proc, int device)
{
  if (proc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *proc  = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* p   = new srs_amd_pucch_processor();
  p->device = device;
  p->jump   = gold_jump_tables();
  if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
    delete p;
    return hip_fail(hipErrorUnknown, "PUCCH processor stream");
  }
  rc = srs_amd_uci_decoder_create(&p->uci, device);
  if (rc != SRS_AMD_OK) {
    delete p;
    return rc;
  }
  *proc = p;
  return SRS_AMD_OK;
}

void srs_amd_pucch_processor_destroy(srs_amd_pucch_processor* proc)
{
  delete proc;
}

int srs_amd_pucch_f0_detect_slot(srs_amd_pucch_processor*    proc,
                                 const srs_amd_pucch_f0_pdu* pdus,
                                 uint32_t                    nof_pdus,
                                 const uint32_t*             d_grids,
                                 uint64_t                    grid_stride,
                                 uint32_t                    nof_grids,
                                 uint32_t                    nof_grid_ports,
                                 uint32_t                    nof_subc,
                                 srs_amd_pucch_f0_result*    d_results,
                                 void*                       stream)
{
  if (proc == nullptr || (nof_pdus != 0 && (pdus == nullptr || d_results == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_pdus == 0) {
    return SRS_AMD_OK;
  }
  if (nof_subc == 0 || nof_subc % 12 != 0) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  std::lock_guard<std::mutex> lock(proc->mtx);
  std::vector<pucch_f0_desc>  desc(nof_pdus);
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const int rc = make_desc(proc, pdus[i], d_grids, grid_stride, nof_grids, nof_grid_ports, nof_subc, desc[i]);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  const size_t bytes = sizeof(pucch_f0_desc) * nof_pdus;
  auto         s     = static_cast<hipStream_t>(stream);
  hipError_t   e     = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->buf.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->stage.acquire(bytes);
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH processor scratch");
  }
  call_scope scope(proc->order, nullptr, s);
  std::memcpy(proc->stage.at<uint8_t>(0), desc.data(), bytes);
  e = proc->stage.upload(proc->buf.ptr, bytes, s);
  if (e == hipSuccess) {
    e = launch_pucch_f0(proc->buf.as<pucch_f0_desc>(), nof_pdus, d_results, s);
  }
  const int        rc   = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pucch_f0_kernel launch");
  const hipError_t done = scope.close();
  return rc != SRS_AMD_OK ? rc : (done == hipSuccess ? SRS_AMD_OK : hip_fail(done, "PUCCH completion event"));
}

int srs_amd_pucch_f0_detect(srs_amd_pucch_processor*    proc,
                            const srs_amd_pucch_f0_pdu* pdu,
                            const uint32_t*             grid,
                            uint32_t                    nof_ports,
                            uint32_t                    nof_subc,
                            srs_amd_pucch_f0_result*    result)
{
  if (proc == nullptr || pdu == nullptr || grid == nullptr || result == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->host_res.ensure(sizeof(srs_amd_pucch_f0_result));
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH grid upload");
  }
  srs_amd_pucch_f0_pdu p = *pdu;
  p.grid                 = 0;
  p.d_grid               = nullptr;
  int rc = srs_amd_pucch_f0_detect_slot(proc, &p, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_ports, nof_subc,
                                        proc->host_res.as<srs_amd_pucch_f0_result>(), proc->stream);
  if (rc == SRS_AMD_OK) {
    e  = hipMemcpyAsync(result, proc->host_res.ptr, sizeof(*result), hipMemcpyDeviceToHost, proc->stream);
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUCCH result download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

} // extern "C"

namespace {

// The Format 2 slot form; decode = false stops after the LLRs (rows of PUCCH_F2_MAX_E in proc->work, decoder order).
int f2_slot(srs_amd_pucch_processor*    proc,
            const srs_amd_pucch_f2_pdu* pdus,
            uint32_t                    nof_pdus,
            const uint32_t*             d_grids,
            uint64_t                    grid_stride,
            uint32_t                    nof_grids,
            uint32_t                    nof_grid_ports,
            uint32_t                    nof_subc,
            srs_amd_pucch_uci_result*   d_results,
            uint8_t*                    d_payloads,
            uint64_t                    payload_stride,
            void*                       stream,
            bool                        decode)
{
  if (proc == nullptr || (nof_pdus != 0 && (pdus == nullptr || d_results == nullptr || d_payloads == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_pdus == 0) {
    return SRS_AMD_OK;
  }
  if (nof_subc == 0 || nof_subc % 12 != 0) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  std::lock_guard<std::mutex> lock(proc->mtx);
  std::vector<pucch_f2_desc>  desc(nof_pdus);
  std::vector<uint32_t>       K(nof_pdus), E(nof_pdus);
  uint32_t                    max_k = 0;
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const srs_amd_pucch_f2_pdu& p = pdus[i];
    if (p.nof_harq_ack + p.nof_sr + p.nof_csi_part1 + p.nof_csi_part2 > payload_stride) {
      return fail(SRS_AMD_EINVAL, "payload_stride %llu below the PDU's %u payload bits.",
                  static_cast<unsigned long long>(payload_stride),
                  p.nof_harq_ack + p.nof_sr + p.nof_csi_part1 + p.nof_csi_part2);
    }
  }
  // decoder order: PDUs grouped by (payload, codeword) size, one UCI decoder launch per group
  std::vector<uint32_t> perm(nof_pdus);
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const srs_amd_pucch_f2_pdu& p = pdus[i];
    K[i]  = p.nof_harq_ack + p.nof_sr + p.nof_csi_part1 + p.nof_csi_part2;
    E[i]  = 16 * p.nof_prb * p.nof_symbols;
    max_k = std::max(max_k, K[i]);
  }
  std::iota(perm.begin(), perm.end(), 0u);
  std::stable_sort(perm.begin(), perm.end(),
                   [&](uint32_t a, uint32_t b) { return K[a] != K[b] ? K[a] < K[b] : E[a] < E[b]; });
  const uint32_t msg_stride = (std::max(max_k, 1u) + 63) / 64 * 64;
  const size_t   llr_bytes  = static_cast<size_t>(nof_pdus) * PUCCH_F2_MAX_E;
  const size_t   msg_bytes  = static_cast<size_t>(nof_pdus) * msg_stride;
  const size_t   st_bytes   = static_cast<size_t>(nof_pdus) * sizeof(int32_t);
  auto           s          = static_cast<hipStream_t>(stream);
  hipError_t     e          = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->work.ensure(llr_bytes + msg_bytes + st_bytes);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH processor scratch");
  }
  int8_t*  d_llr = proc->work.as<int8_t>();
  uint8_t* d_msg = proc->work.as<uint8_t>() + llr_bytes;
  int32_t* d_st  = reinterpret_cast<int32_t*>(proc->work.as<uint8_t>() + llr_bytes + msg_bytes);
  std::vector<uint32_t> nbits(nof_pdus);
  for (uint32_t j = 0; j != nof_pdus; ++j) {
    const uint32_t i = perm[j];
    const int rc = make_f2_desc(proc, pdus[i], d_grids, grid_stride, nof_grids, nof_grid_ports, nof_subc, desc[j]);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    desc[j].llr    = d_llr + static_cast<size_t>(j) * PUCCH_F2_MAX_E;
    desc[j].result = d_results + i;
    nbits[j]       = K[i];
  }
  const size_t dbytes = sizeof(pucch_f2_desc) * nof_pdus;
  const size_t ioff   = (dbytes + 255) & ~size_t(255);
  const size_t ibytes = sizeof(uint32_t) * nof_pdus;
  const size_t bytes  = ioff + 2 * ibytes;
  if (e == hipSuccess) {
    e = proc->buf.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->stage.acquire(bytes);
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH processor scratch");
  }
  call_scope scope(proc->order, nullptr, s);
  std::memcpy(proc->stage.at<uint8_t>(0), desc.data(), dbytes);
  std::memcpy(proc->stage.at<uint8_t>(ioff), perm.data(), ibytes);
  std::memcpy(proc->stage.at<uint8_t>(ioff + ibytes), nbits.data(), ibytes);
  e = proc->stage.upload(proc->buf.ptr, bytes, s);
  if (e == hipSuccess) {
    e = launch_pucch_f2(proc->buf.as<pucch_f2_desc>(), nof_pdus, s);
  }
  int rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pucch_f2_kernel launch");
  for (uint32_t j0 = 0; decode && rc == SRS_AMD_OK && j0 != nof_pdus;) {
    uint32_t j1 = j0 + 1;
    while (j1 != nof_pdus && K[perm[j1]] == K[perm[j0]] && E[perm[j1]] == E[perm[j0]]) {
      ++j1;
    }
    rc = srs_amd_uci_decode_batch(proc->uci, d_llr + static_cast<size_t>(j0) * PUCCH_F2_MAX_E, PUCCH_F2_MAX_E,
                                  E[perm[j0]], K[perm[j0]], 2, d_msg + static_cast<size_t>(j0) * msg_stride,
                                  msg_stride, d_st + j0, sizeof(int32_t), j1 - j0, s);
    j0 = j1;
  }
  if (decode && rc == SRS_AMD_OK) {
    const uint32_t* d_perm = reinterpret_cast<const uint32_t*>(proc->buf.as<uint8_t>() + ioff);
    e  = launch_pucch_uci_finish(d_st, d_msg, msg_stride, d_perm, d_perm + nof_pdus, nof_pdus, d_results, d_payloads,
                                 payload_stride, s);
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pucch_uci_finish_kernel launch");
  }
  const hipError_t done = scope.close();
  return rc != SRS_AMD_OK ? rc : (done == hipSuccess ? SRS_AMD_OK : hip_fail(done, "PUCCH completion event"));
}

} // namespace

extern "C" {

int srs_amd_pucch_f2_process_slot(srs_amd_pucch_processor*    proc,
                                  const srs_amd_pucch_f2_pdu* pdus,
                                  uint32_t                    nof_pdus,
                                  const uint32_t*             d_grids,
                                  uint64_t                    grid_stride,
                                  uint32_t                    nof_grids,
                                  uint32_t                    nof_grid_ports,
                                  uint32_t                    nof_subc,
                                  srs_amd_pucch_uci_result*   d_results,
                                  uint8_t*                    d_payloads,
                                  uint64_t                    payload_stride,
                                  void*                       stream)
{
  return f2_slot(proc, pdus, nof_pdus, d_grids, grid_stride, nof_grids, nof_grid_ports, nof_subc, d_results,
                 d_payloads, payload_stride, stream, true);
}

int srs_amd_pucch_f2_demodulate(srs_amd_pucch_processor*    proc,
                                const srs_amd_pucch_f2_pdu* pdu,
                                const uint32_t*             grid,
                                uint32_t                    nof_ports,
                                uint32_t                    nof_subc,
                                int8_t*                     llrs)
{
  if (proc == nullptr || pdu == nullptr || grid == nullptr || llrs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const uint32_t              E     = 16 * pdu->nof_prb * pdu->nof_symbols;
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->host_res.ensure(sizeof(srs_amd_pucch_uci_result));
  }
  if (e == hipSuccess) {
    e = proc->host_payload.ensure(1706);
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH grid upload");
  }
  srs_amd_pucch_f2_pdu p = *pdu;
  p.grid                 = 0;
  p.d_grid               = nullptr;
  int rc = f2_slot(proc, &p, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_ports, nof_subc,
                   proc->host_res.as<srs_amd_pucch_uci_result>(), proc->host_payload.as<uint8_t>(), 1706,
                   proc->stream, false);
  if (rc == SRS_AMD_OK) {
    e  = hipMemcpyAsync(llrs, proc->work.ptr, E, hipMemcpyDeviceToHost, proc->stream);
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUCCH LLR download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

int srs_amd_pucch_f2_process(srs_amd_pucch_processor*    proc,
                             const srs_amd_pucch_f2_pdu* pdu,
                             const uint32_t*             grid,
                             uint32_t                    nof_ports,
                             uint32_t                    nof_subc,
                             srs_amd_pucch_uci_result*   result,
                             uint8_t*                    payload)
{
  if (proc == nullptr || pdu == nullptr || grid == nullptr || result == nullptr || payload == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const uint32_t              K     = pdu->nof_harq_ack + pdu->nof_sr + pdu->nof_csi_part1 + pdu->nof_csi_part2;
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->host_res.ensure(sizeof(srs_amd_pucch_uci_result));
  }
  if (e == hipSuccess) {
    e = proc->host_payload.ensure(std::max(K, 1u));
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH grid upload");
  }
  srs_amd_pucch_f2_pdu p = *pdu;
  p.grid                 = 0;
  p.d_grid               = nullptr;
  int rc = srs_amd_pucch_f2_process_slot(proc, &p, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_ports, nof_subc,
                                         proc->host_res.as<srs_amd_pucch_uci_result>(),
                                         proc->host_payload.as<uint8_t>(), std::max(K, 1u), proc->stream);
  if (rc == SRS_AMD_OK) {
    e = hipMemcpyAsync(result, proc->host_res.ptr, sizeof(*result), hipMemcpyDeviceToHost, proc->stream);
    if (e == hipSuccess && K != 0) {
      e = hipMemcpyAsync(payload, proc->host_payload.ptr, K, hipMemcpyDeviceToHost, proc->stream);
    }
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUCCH result download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

int srs_amd_pucch_f34_process_slot(srs_amd_pucch_processor*     proc,
                                   const srs_amd_pucch_f34_pdu* pdus,
                                   uint32_t                     nof_pdus,
                                   const uint32_t*              d_grids,
                                   uint64_t                     grid_stride,
                                   uint32_t                     nof_grids,
                                   uint32_t                     nof_grid_ports,
                                   uint32_t                     nof_subc,
                                   srs_amd_pucch_uci_result*    d_results,
                                   uint8_t*                     d_payloads,
                                   uint64_t                     payload_stride,
                                   void*                        stream)
{
  return f34_slot(proc, pdus, nof_pdus, d_grids, grid_stride, nof_grids, nof_grid_ports, nof_subc, d_results,
                  d_payloads, payload_stride, stream, true);
}

namespace {

// Host forms of Formats 3 / 4: the grid up, one PDU, the result and payload (or the LLRs) down.
int f34_host(srs_amd_pucch_processor* proc, const srs_amd_pucch_f34_pdu* pdu, const uint32_t* grid,
             uint32_t nof_ports, uint32_t nof_subc, srs_amd_pucch_uci_result* result, uint8_t* payload, int8_t* llrs)
{
  if (proc == nullptr || pdu == nullptr || grid == nullptr || (llrs == nullptr && (result == nullptr || payload == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const uint32_t              K     = pdu->nof_harq_ack + pdu->nof_sr + pdu->nof_csi_part1 + pdu->nof_csi_part2;
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->host_res.ensure(sizeof(srs_amd_pucch_uci_result));
  }
  if (e == hipSuccess) {
    e = proc->host_payload.ensure(1706);
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH grid upload");
  }
  srs_amd_pucch_f34_pdu p = *pdu;
  p.grid                  = 0;
  p.d_grid                = nullptr;
  int rc = f34_slot(proc, &p, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_ports, nof_subc,
                    proc->host_res.as<srs_amd_pucch_uci_result>(), proc->host_payload.as<uint8_t>(), 1706,
                    proc->stream, llrs == nullptr);
  if (rc == SRS_AMD_OK) {
    if (llrs != nullptr) {
      const bool     f4  = p.format == 4;
      const uint32_t nd  = static_cast<uint32_t>(__builtin_popcount(f34_dmrs_mask(p.nof_symbols, p.second_hop_prb >= 0,
                                                                                  p.additional_dmrs != 0)));
      const uint32_t E   = (p.nof_symbols - nd) * 12 * (f4 ? 1u : p.nof_prb) * (p.pi2_bpsk ? 1u : 2u) /
                         (f4 ? p.occ_length : 1u);
      e = hipMemcpyAsync(llrs, proc->work.ptr, E, hipMemcpyDeviceToHost, proc->stream);
    } else {
      e = hipMemcpyAsync(result, proc->host_res.ptr, sizeof(*result), hipMemcpyDeviceToHost, proc->stream);
      if (e == hipSuccess && K != 0) {
        e = hipMemcpyAsync(payload, proc->host_payload.ptr, K, hipMemcpyDeviceToHost, proc->stream);
      }
    }
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUCCH result download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

} // namespace

int srs_amd_pucch_f34_process(srs_amd_pucch_processor*     proc,
                              const srs_amd_pucch_f34_pdu* pdu,
                              const uint32_t*              grid,
                              uint32_t                     nof_ports,
                              uint32_t                     nof_subc,
                              srs_amd_pucch_uci_result*    result,
                              uint8_t*                     payload)
{
  if (result == nullptr || payload == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  return f34_host(proc, pdu, grid, nof_ports, nof_subc, result, payload, nullptr);
}

int srs_amd_pucch_f34_demodulate(srs_amd_pucch_processor*     proc,
                                 const srs_amd_pucch_f34_pdu* pdu,
                                 const uint32_t*              grid,
                                 uint32_t                     nof_ports,
                                 uint32_t                     nof_subc,
                                 int8_t*                      llrs)
{
  if (llrs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  return f34_host(proc, pdu, grid, nof_ports, nof_subc, nullptr, nullptr, llrs);
}

int srs_amd_pucch_f1_detect_slot(srs_amd_pucch_processor*      proc,
                                 const srs_amd_pucch_f1_batch* batches,
                                 uint32_t                      nof_batches,
                                 const uint32_t*               d_grids,
                                 uint64_t                      grid_stride,
                                 uint32_t                      nof_grids,
                                 uint32_t                      nof_grid_ports,
                                 uint32_t                      nof_subc,
                                 srs_amd_pucch_result*         d_results,
                                 void*                         stream)
{
  if (proc == nullptr || (nof_batches != 0 && (batches == nullptr || d_results == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_batches == 0) {
    return SRS_AMD_OK;
  }
  if (nof_subc == 0 || nof_subc % 12 != 0) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  std::lock_guard<std::mutex>         lock(proc->mtx);
  std::vector<pucch_f1_desc>          desc(nof_batches);
  std::vector<srs_amd_pucch_f1_entry> ent;
  for (uint32_t i = 0; i != nof_batches; ++i) {
    const int rc = make_f1_desc(proc, batches[i], d_grids, grid_stride, nof_grids, nof_grid_ports, nof_subc,
                                static_cast<uint32_t>(ent.size()), desc[i]);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    ent.insert(ent.end(), batches[i].entries, batches[i].entries + batches[i].nof_entries);
  }
  const size_t dbytes = sizeof(pucch_f1_desc) * nof_batches;
  const size_t ebytes = sizeof(srs_amd_pucch_f1_entry) * ent.size();
  const size_t eoff   = (dbytes + 255) & ~size_t(255);
  const size_t bytes  = eoff + ebytes;
  auto         s      = static_cast<hipStream_t>(stream);
  hipError_t   e      = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->buf.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->stage.acquire(bytes);
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH processor scratch");
  }
  call_scope scope(proc->order, nullptr, s);
  std::memcpy(proc->stage.at<uint8_t>(0), desc.data(), dbytes);
  std::memcpy(proc->stage.at<uint8_t>(eoff), ent.data(), ebytes);
  e = proc->stage.upload(proc->buf.ptr, bytes, s);
  if (e == hipSuccess) {
    e = launch_pucch_f1(proc->buf.as<pucch_f1_desc>(),
                        nof_batches,
                        reinterpret_cast<const srs_amd_pucch_f1_entry*>(proc->buf.as<uint8_t>() + eoff),
                        d_results,
                        s);
  }
  const int        rc   = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pucch_f1_kernel launch");
  const hipError_t done = scope.close();
  return rc != SRS_AMD_OK ? rc : (done == hipSuccess ? SRS_AMD_OK : hip_fail(done, "PUCCH completion event"));
}

int srs_amd_pucch_f1_detect(srs_amd_pucch_processor*      proc,
                            const srs_amd_pucch_f1_batch* batch,
                            const uint32_t*               grid,
                            uint32_t                      nof_ports,
                            uint32_t                      nof_subc,
                            srs_amd_pucch_result*         results)
{
  if (proc == nullptr || batch == nullptr || grid == nullptr || results == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (batch->nof_entries == 0 || batch->nof_entries > PUCCH_F1_MAX_ENTRIES) {
    return fail(SRS_AMD_EINVAL, "Invalid number of multiplexed PUCCH (i.e., %u).", batch->nof_entries);
  }
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  const size_t                rbytes = sizeof(srs_amd_pucch_result) * batch->nof_entries;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->host_res.ensure(rbytes);
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH grid upload");
  }
  srs_amd_pucch_f1_batch b = *batch;
  b.grid                   = 0;
  b.d_grid                 = nullptr;
  int rc = srs_amd_pucch_f1_detect_slot(proc, &b, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_ports, nof_subc,
                                        proc->host_res.as<srs_amd_pucch_result>(), proc->stream);
  if (rc == SRS_AMD_OK) {
    e  = hipMemcpyAsync(results, proc->host_res.ptr, rbytes, hipMemcpyDeviceToHost, proc->stream);
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUCCH result download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

} // extern "C"
