// sch_plan.cpp -- transport-block segmentation geometry (host only), the
// computations of ldpc_segmenter_tx_impl::new_transmission
// (ldpc_segmenter_tx_impl.cpp:53-123) and ldpc_segmenter_rx_impl::segment,
// with the helpers of include/srsran/phy/upper/channel_coding/ldpc/ldpc.h:128-207
// (compute_tb_crc_size, compute_nof_codeblocks, compute_lifting_size) and
// ldpc_segmenter_helpers.h:82-94 (compute_rm_length).
#include "srsran_amd/sch.h"

#include "api_common.h"
#include <algorithm>
#include <cmath>

using namespace srs_amd;

namespace {

constexpr uint32_t MAX_TBS          = 1277992; // ldpc_segmenter_tx_impl.cpp:37, including the TB CRC
constexpr uint32_t MAX_BITS_CRC16   = 3824;
constexpr uint32_t SEG_CRC_LENGTH   = 24;
// sch_constants.h:38: 156 REs x 275 PRB x 4 layers x 8 bits / 8448.
constexpr uint32_t MAX_NOF_SEGMENTS = (156 * 275 * 4 * 8) / (22 * 384);
constexpr uint32_t LIFTING_SIZES[]  = {2,  3,  4,   5,   6,   7,   8,   9,   10,  11,  12,  13,  14,
                                       15, 16, 18,  20,  22,  24,  26,  28,  30,  32,  36,  40,  44,
                                       48, 52, 56,  60,  64,  72,  80,  88,  96,  104, 112, 120, 128,
                                       144, 160, 176, 192, 208, 224, 240, 256, 288, 320, 352, 384};

uint32_t divide_ceil(uint32_t a, uint32_t b)
{
  return (a + b - 1) / b;
}

uint32_t tb_crc_size(uint32_t tbs)
{
  return tbs <= MAX_BITS_CRC16 ? 16 : 24;
}

uint32_t nof_codeblocks(uint32_t tbs, uint32_t bg)
{
  const uint32_t b   = tbs + tb_crc_size(tbs);
  const uint32_t max = bg == 1 ? 8448 : 3840;
  return b <= max ? 1 : divide_ceil(b, max - SEG_CRC_LENGTH);
}

uint32_t lifting_size(uint32_t tbs, uint32_t bg, uint32_t C)
{
  const uint32_t b   = tbs + tb_crc_size(tbs);
  uint32_t       ref = 22;
  if (bg == 2) {
    ref = b > 640 ? 10 : b > 560 ? 9 : b > 192 ? 8 : 6;
  }
  const uint32_t total = C * ref;
  const uint32_t out   = b + (C > 1 ? 24 * C : 0);
  for (uint32_t ls : LIFTING_SIZES) {
    if (ls * total >= out) {
      return ls;
    }
  }
  return 0;
}

} // namespace

extern "C" {

int srs_amd_sch_plan_compute(srs_amd_sch_plan* p,
                             uint32_t          tbs,
                             uint32_t          base_graph,
                             uint32_t          rv,
                             uint32_t          qm,
                             uint32_t          Nref,
                             uint32_t          nof_layers,
                             uint32_t          nof_ch_symbols)
{
  if (p == nullptr) {
    return fail(SRS_AMD_EINVAL, "null plan");
  }
  *p = srs_amd_sch_plan{};
  if (tbs == 0 || tbs % 8 != 0) {
    return fail(SRS_AMD_EINVAL, "Argument transport_block should not be empty (TBS %u must be a positive multiple of 8).",
                tbs);
  }
  if (tbs + 24 > MAX_TBS) {
    return fail(SRS_AMD_EINVAL, "Transport block too long. The admissible size, including CRC, is %u.", MAX_TBS / 8);
  }
  if (base_graph != 1 && base_graph != 2) {
    return fail(SRS_AMD_EINVAL, "Invalid base graph %u.", base_graph);
  }
  if (rv > 3) {
    return fail(SRS_AMD_EINVAL, "Invalid redundancy version.");
  }
  if (nof_layers < 1 || nof_layers > 4) {
    return fail(SRS_AMD_EINVAL, "Invalid number of layers.");
  }
  if (qm != 1 && qm != 2 && qm != 4 && qm != 6 && qm != 8) {
    return fail(SRS_AMD_EINVAL, "Invalid modulation order %u.", qm);
  }
  if (nof_ch_symbols == 0 || nof_ch_symbols % nof_layers != 0) {
    return fail(SRS_AMD_EINVAL,
                "The number of channel symbols should be a multiple of the product between the number of layers.");
  }
  p->tbs              = tbs;
  p->base_graph       = base_graph;
  p->rv               = rv;
  p->modulation_order = qm;
  p->Nref             = Nref;
  p->nof_layers       = nof_layers;
  p->nof_ch_symbols   = nof_ch_symbols;

  p->nof_tb_crc_bits     = tb_crc_size(tbs);
  const uint32_t tb_in   = tbs + p->nof_tb_crc_bits;
  p->nof_segments        = nof_codeblocks(tbs, base_graph);
  const uint32_t tb_out  = tb_in + (p->nof_segments > 1 ? p->nof_segments * SEG_CRC_LENGTH : 0);
  p->lifting_size        = lifting_size(tbs, base_graph, p->nof_segments);
  if (p->lifting_size == 0) {
    return fail(SRS_AMD_EINVAL, "Lifting size cannot be 0");
  }
  if (p->nof_segments > MAX_NOF_SEGMENTS) {
    return fail(SRS_AMD_EINVAL, "%u segments exceed the maximum of %u.", p->nof_segments, MAX_NOF_SEGMENTS);
  }
  p->segment_length = (base_graph == 1 ? 22 : 10) * p->lifting_size;
  p->nof_crc_bits   = p->nof_segments > 1 ? SEG_CRC_LENGTH : 0;
  p->cb_info_bits   = divide_ceil(tb_out, p->nof_segments) - p->nof_crc_bits;
  p->zero_pad       = (p->cb_info_bits + p->nof_crc_bits) * p->nof_segments - tb_out;
  p->nof_filler_bits = p->segment_length - p->cb_info_bits - p->nof_crc_bits;

  const uint32_t per_layer = nof_ch_symbols / nof_layers;
  p->nof_short_segments    = p->nof_segments - per_layer % p->nof_segments;
  p->rm_length_short       = per_layer / p->nof_segments * nof_layers * qm;
  p->rm_length_long        = divide_ceil(per_layer, p->nof_segments) * nof_layers * qm;
  p->cw_length             = nof_ch_symbols * qm;
  if (p->rm_length_short == 0 && p->nof_short_segments > 0) {
    return fail(SRS_AMD_EINVAL, "%u channel symbols cannot carry %u codeblocks.", nof_ch_symbols, p->nof_segments);
  }
  return SRS_AMD_OK;
}

int srs_amd_sch_plan_segments(const srs_amd_sch_plan* p, uint32_t* rm_lengths, uint32_t* cw_offsets)
{
  if (p == nullptr || p->nof_segments == 0) {
    return fail(SRS_AMD_EINVAL, "invalid plan");
  }
  uint32_t off = 0;
  for (uint32_t r = 0; r < p->nof_segments; ++r) {
    const uint32_t E = r < p->nof_short_segments ? p->rm_length_short : p->rm_length_long;
    if (rm_lengths) {
      rm_lengths[r] = E;
    }
    if (cw_offsets) {
      cw_offsets[r] = off;
    }
    off += E;
  }
  return SRS_AMD_OK;
}

} // extern "C"

// ---- TS 38.214 5.1.3.2 transport block size (host only) -------------------
// Restates lib/ran/sch/tbs_calculator.cpp:30-148 (float arithmetic kept as the
// reference computes it); Table 5.1.3.2-1 TBS values for N_info <= 3824.
namespace {

constexpr uint32_t TBS_TABLE[] = {
    24,   32,   40,   48,   56,   64,   72,   80,   88,   96,   104,  112,  120,  128,  136,  144,  152,  160,  168,
    176,  184,  192,  208,  224,  240,  256,  272,  288,  304,  320,  336,  352,  368,  384,  408,  432,  456,  480,
    504,  528,  552,  576,  608,  640,  672,  704,  736,  768,  808,  848,  888,  928,  984,  1032, 1064, 1128, 1160,
    1192, 1224, 1256, 1288, 1320, 1352, 1416, 1480, 1544, 1608, 1672, 1736, 1800, 1864, 1928, 2024, 2088, 2152, 2216,
    2280, 2408, 2472, 2536, 2600, 2664, 2728, 2792, 2856, 2976, 3104, 3240, 3368, 3496, 3624, 3752, 3824};

uint32_t tbs_step3(float nof_info)
{
  uint32_t n = 3;
  if (nof_info > 512.0F) {
    n = static_cast<uint32_t>(std::floor(std::log2(nof_info))) - 6U;
  }
  const uint32_t prime =
      std::max(24U, (1U << n) * static_cast<uint32_t>(std::floor(nof_info / static_cast<float>(1U << n))));
  for (uint32_t v : TBS_TABLE) {
    if (v >= prime) {
      return v;
    }
  }
  return 0;
}

uint32_t tbs_step4(float nof_info, float tcr)
{
  const uint32_t n     = static_cast<uint32_t>(std::floor(std::log2(nof_info - 24)) - 5.0F);
  const uint32_t prime = std::max(
      3840U, (1U << n) * static_cast<uint32_t>(std::round((nof_info - 24) / static_cast<float>(1U << n))));
  uint32_t C = 1;
  if (tcr <= 0.25F) {
    C = divide_ceil(prime + 24, 3816);
  } else if (prime > 8424) {
    C = divide_ceil(prime + 24, 8424);
  }
  return 8 * C * divide_ceil(prime + 24, 8 * C) - 24;
}

} // namespace

extern "C" uint32_t srs_amd_tbs_calculate(uint32_t nof_symb_sh,
                                          uint32_t nof_dmrs_prb,
                                          uint32_t nof_oh_prb,
                                          uint32_t modulation_order,
                                          float    target_code_rate,
                                          uint32_t nof_layers,
                                          uint32_t tb_scaling_field,
                                          uint32_t n_prb)
{
  if (modulation_order < 2 || tb_scaling_field > 2 || 12 * nof_symb_sh < nof_dmrs_prb + nof_oh_prb) {
    fail(SRS_AMD_EINVAL, "invalid TBS calculator configuration");
    return 0;
  }
  const uint32_t nof_re_prime = 12 * nof_symb_sh - nof_dmrs_prb - nof_oh_prb;
  const uint32_t nof_re       = std::min(nof_re_prime, 156U) * n_prb;
  const float    scaling      = 1.0F / static_cast<float>(1U << tb_scaling_field);
  const float    tcr          = target_code_rate * (1.F / 1024);
  const float    nof_info     = scaling * static_cast<float>(nof_re) * tcr * static_cast<float>(modulation_order) *
                         static_cast<float>(nof_layers);
  return nof_info <= 3824 ? tbs_step3(nof_info) : tbs_step4(nof_info, tcr);
}

// ---- get_ulsch_information (lib/ran/pusch/ulsch_info.cpp) -------------------------------------------------------
#include "srsran_amd/ulsch_info.h"

#include <algorithm>
#include <cmath>

#pragma clang fp contract(off)

namespace {

// get_uci_crc_size (include/srsran/ran/uci/uci_info.h:54-65)
uint32_t uci_crc_size(uint32_t a)
{
  return a < 12 ? 0u : (a < 20 ? 6u : 11u);
}

// calculate_nof_re_harq_ack (ulsch_info.cpp:30-48), float as the reference
uint32_t re_harq_ack(uint32_t o, float beta, uint32_t nre_uci, uint32_t sum_cb, float alpha, uint32_t nre_l0)
{
  if (o == 0) {
    return 0;
  }
  const uint32_t left  = static_cast<uint32_t>(std::ceil(static_cast<float>(o + uci_crc_size(o)) * beta *
                                                        static_cast<float>(nre_uci) / static_cast<float>(sum_cb)));
  const uint32_t right = static_cast<uint32_t>(std::ceil(alpha * static_cast<float>(nre_l0)));
  return std::min(left, right);
}

// calculate_nof_re_harq_ack_without_sch (:50-68)
uint32_t re_harq_ack_no_sch(uint32_t o, float beta, float rate, uint32_t qm, float alpha, uint32_t nre_l0)
{
  if (o == 0) {
    return 0;
  }
  const uint32_t left  = static_cast<uint32_t>(
      std::ceil(static_cast<float>(o + uci_crc_size(o)) * beta / (rate * static_cast<float>(qm))));
  const uint32_t right = static_cast<uint32_t>(std::ceil(alpha * static_cast<float>(nre_l0)));
  return std::min(left, right);
}

// calculate_nof_re_csi_part1 (:70-89)
uint32_t re_csi1(uint32_t o, float beta, uint32_t nre_uci, uint32_t nre_ack, uint32_t sum_cb, float alpha)
{
  if (o == 0) {
    return 0;
  }
  const uint32_t left  = static_cast<uint32_t>(std::ceil(static_cast<float>(o + uci_crc_size(o)) * beta *
                                                        static_cast<float>(nre_uci) / static_cast<float>(sum_cb)));
  const uint32_t right = static_cast<uint32_t>(std::ceil(alpha * static_cast<float>(nre_uci))) - nre_ack;
  return std::min(left, right);
}

// calculate_nof_re_csi_part1_without_sch (:91-118)
uint32_t re_csi1_no_sch(uint32_t o, uint32_t o2, uint32_t nre_uci, uint32_t nre_ack, float beta, float rate, uint32_t qm)
{
  if (o == 0) {
    return 0;
  }
  if (o2 == 0) {
    return nre_uci - nre_ack;
  }
  const uint32_t left = static_cast<uint32_t>(
      std::ceil(static_cast<float>(o + uci_crc_size(o)) * beta / (rate * static_cast<float>(qm))));
  return std::min(left, nre_uci - nre_ack);
}

// calculate_nof_re_csi_part2 (:120-141)
uint32_t re_csi2(uint32_t o, float beta, uint32_t nre_uci, uint32_t nre_ack, uint32_t nre_csi1, uint32_t sum_cb,
                 float alpha)
{
  if (o == 0) {
    return 0;
  }
  const uint32_t left  = static_cast<uint32_t>(std::ceil(static_cast<float>(o + uci_crc_size(o)) * beta *
                                                        static_cast<float>(nre_uci) / static_cast<float>(sum_cb)));
  const uint32_t right =
      static_cast<uint32_t>(std::ceil(alpha * static_cast<float>(nre_uci))) - nre_ack - nre_csi1;
  return std::min(left, right);
}

} // namespace

extern "C" int srs_amd_ulsch_information(const srs_amd_ulsch_config* c, srs_amd_ulsch_info* r)
{
  if (c == nullptr || r == nullptr) {
    return srs_amd::fail(SRS_AMD_EINVAL, "null argument");
  }
  *r                  = srs_amd_ulsch_info{};
  const float    rate = c->target_code_rate * (1.F / 1024);
  const uint32_t qm   = c->modulation < 2 ? 1u : static_cast<uint32_t>(c->modulation);
  const uint32_t max_cdm = c->dmrs_type == 1 ? 2u : 3u;
  if (c->dmrs_type < 1 || c->dmrs_type > 2 || c->nof_cdm_groups_without_data < 1 ||
      c->nof_cdm_groups_without_data > max_cdm) {
    return srs_amd::fail(SRS_AMD_EINVAL, "Invalid DM-RS type / CDM groups without data.");
  }
  const uint32_t end  = c->start_symbol_index + c->nof_symbols;
  const uint32_t mask = c->dmrs_symbol_mask & 0x3fffu;
  if (mask == 0 || end > 14 || static_cast<uint32_t>(__builtin_ctz(mask)) < c->start_symbol_index ||
      static_cast<uint32_t>(31 - __builtin_clz(mask)) >= end) {
    return srs_amd::fail(SRS_AMD_EINVAL, "DM-RS symbols outside the time allocation.");
  }
  uint32_t sum_cb = 0;
  if (c->tbs > 0) {
    if (!(rate > 0.F && rate < 1.F)) {
      return srs_amd::fail(SRS_AMD_EINVAL, "Invalid target code rate.");
    }
    // get_sch_segmentation_info (lib/ran/sch/sch_segmentation.cpp:30-63), get_ldpc_base_graph (ldpc_base_graph.h:38)
    const uint32_t bg = (c->tbs <= 292 || rate <= 0.25F || (c->tbs <= 3824 && rate <= 0.67F)) ? 2u : 1u;
    const uint32_t C  = nof_codeblocks(c->tbs, bg);
    const uint32_t Z  = lifting_size(c->tbs, bg, C);
    const uint32_t K  = (bg == 1 ? 22u : 10u) * Z;
    uint32_t       per_cb = (c->tbs + tb_crc_size(c->tbs)) / C;
    if (C > 1) {
      per_cb += SEG_CRC_LENGTH;
    }
    r->sch_tb_crc_size            = tb_crc_size(c->tbs);
    r->sch_base_graph             = bg;
    r->sch_nof_cb                 = C;
    r->sch_lifting_size           = Z;
    r->sch_nof_bits_per_cb        = K;
    r->sch_nof_filler_bits_per_cb = K - per_cb;
    sum_cb                        = C * K;
  }
  const uint32_t nds        = static_cast<uint32_t>(__builtin_popcount(mask));
  const uint32_t dmrs_re_rb = nds * c->nof_cdm_groups_without_data * (c->dmrs_type == 1 ? 6u : 4u);
  const uint32_t re_total   = c->nof_rb * (c->nof_symbols * 12 - dmrs_re_rb);
  const uint32_t re_uci     = (c->nof_symbols - nds) * c->nof_rb * 12;
  uint32_t       re_uci_l0  = 0;
  for (uint32_t l = static_cast<uint32_t>(__builtin_ctz(mask)); l < end; ++l) {
    re_uci_l0 += ((mask >> l) & 1u) ? 0u : c->nof_rb * 12;
  }
  const bool sch = c->tbs > 0;
  r->nof_harq_ack_re = sch ? re_harq_ack(c->nof_harq_ack_bits, c->beta_offset_harq_ack, re_uci, sum_cb,
                                         c->alpha_scaling, re_uci_l0)
                           : re_harq_ack_no_sch(c->nof_harq_ack_bits, c->beta_offset_harq_ack, rate, qm,
                                                c->alpha_scaling, re_uci_l0);
  uint32_t rvd_re = 0;
  if (c->nof_harq_ack_bits < 2) {
    rvd_re = sch ? re_harq_ack(2, c->beta_offset_harq_ack, re_uci, sum_cb, c->alpha_scaling, re_uci_l0)
                 : re_harq_ack_no_sch(2, c->beta_offset_harq_ack, rate, qm, c->alpha_scaling, re_uci_l0);
  } else if (c->nof_harq_ack_bits == 2) {
    rvd_re = r->nof_harq_ack_re;
  }
  const uint32_t ack_for_csi1 = c->nof_harq_ack_bits <= 2 ? rvd_re : r->nof_harq_ack_re;
  r->nof_csi_part1_re = sch ? re_csi1(c->nof_csi_part1_bits, c->beta_offset_csi_part1, re_uci, ack_for_csi1, sum_cb,
                                      c->alpha_scaling)
                            : re_csi1_no_sch(c->nof_csi_part1_bits, c->nof_csi_part2_bits, re_uci, ack_for_csi1,
                                             c->beta_offset_csi_part1, rate, qm);
  const uint32_t ack_for_csi2 = c->nof_harq_ack_bits <= 2 ? 0u : r->nof_harq_ack_re;
  r->nof_csi_part2_re = sch ? re_csi2(c->nof_csi_part2_bits, c->beta_offset_csi_part2, re_uci, ack_for_csi2,
                                      r->nof_csi_part1_re, sum_cb, c->alpha_scaling)
                            : (c->nof_csi_part2_bits == 0 ? 0u : re_uci - ack_for_csi2 - r->nof_csi_part1_re);
  const uint32_t ack_re = c->nof_harq_ack_bits > 2 ? r->nof_harq_ack_re : 0u;
  const uint32_t sch_re = sch ? re_total - ack_re - r->nof_csi_part1_re - r->nof_csi_part2_re : 0u;
  const uint32_t bpre   = c->nof_layers * qm;
  r->nof_ul_sch_bits     = sch_re * bpre;
  r->nof_harq_ack_bits   = r->nof_harq_ack_re * bpre;
  r->nof_harq_ack_rvd    = rvd_re * bpre;
  r->nof_csi_part1_bits  = r->nof_csi_part1_re * bpre;
  r->nof_csi_part2_bits  = r->nof_csi_part2_re * bpre;
  r->nof_dc_overlap_bits = c->contains_dc ? c->nof_symbols * qm : 0u;
  return SRS_AMD_OK;
}
