// pusch_processor_api.cpp -- C-ABI of the MI355X PUSCH processor
// (include/srsran_amd/pusch_processor.h): pusch_processor_impl::process
// (pusch_processor_impl.cpp:134-386) as three asynchronous device stages --
// DM-RS channel estimation, demodulation, UL-SCH decoding -- over a batch of
// grids, with the processor's own HBM scratch between them.
#include "srsran_amd/pusch_processor.h"
#include "srsran_amd/transform_precoding.h"
#include "srsran_amd/uci_decoder.h"
#include "srsran_amd/ulsch_demux.h"
#include "srsran_amd/ulsch_info.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "uci_args.h"
#include "ulsch_demux_args.h"
#include "pusch_chest_args.h"
#include "pusch_demod_args.h"
#include "pusch_processor_args.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_pusch_processor {
  int                            device = 0;
  srs_amd_pusch_processor_config cfg{};
  srs_amd_pusch_chest*           chest  = nullptr;
  srs_amd_pusch_demodulator*     demod  = nullptr;
  srs_amd_pusch_decoder*         dec    = nullptr;
  srs_amd_ulsch_demux*           demux  = nullptr; // UCI on PUSCH: demultiplexer and decoder
  srs_amd_uci_decoder*           uci    = nullptr;
  device_buffer                  cw_llrs, uci_llrs, uci_payload, uci_status;
  hipStream_t                    stream = nullptr; // host-call stream
  device_buffer                  estimates, stats, llrs, dec_results, host_io, slot_ports;
  stream_order                   order;
  pinned_stage                   stage;  // slot form: per-PDU port counts and result indices
  pinned_stage                   stage2; // CSI part 2 sizes of a batch
  pinned_stage                   stage3; // slot form: UCI descriptors (demultiplexer, decoders, field masks)
  device_buffer                  uci_items, uci_cbs;
  device_buffer                  csi2_sel; // slot form: CSI part 2 size candidate selected per fused PDU
  stream_fan                     fan; // slot form: the UCI decoders beside the UL-SCH decoder
  size_t                         uci_masks_offset = 0; // of the fused group's per-PDU UCI field masks in uci_items
  std::mutex                     mtx;
  bool                           fuse = true; // SRSRAN_AMD_PUSCH_FUSED=0: always expand the estimates
  ~srs_amd_pusch_processor()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    srs_amd_pusch_chest_destroy(chest);
    srs_amd_pusch_demodulator_destroy(demod);
    srs_amd_pusch_decoder_destroy(dec);
    srs_amd_ulsch_demux_destroy(demux);
    srs_amd_uci_decoder_destroy(uci);
  }
};

struct srs_amd_pusch_processor_plan {
  srs_amd_pusch_pdu            pdu{};
  uint32_t                     nof_subc = 0;
  srs_amd_pusch_chest_config   chest_cfg{};
  srs_amd_pusch_demod_plan*    demod_plan = nullptr;
  uint32_t                     nof_re     = 0;
  srs_amd_sch_plan             sch{};
  srs_amd_pusch_decoder_config dec_cfg{};
  uint64_t                     soft_bytes = 0;
  bool                         fusable    = false; // the fused estimator-equalizer path covers this PDU
  bool                         has_sch    = true;  // a codeword (tbs != 0); UCI-only PUSCH otherwise
  uint32_t                     dc_subc    = ~0u;   // DC subcarrier zeroed in the estimates (CP-OFDM only)
  uint32_t                     dummy_sch_bits = 0; // UCI only: the demultiplexer's discarded UL-SCH stream length
  // UCI on PUSCH: multiplexing geometry (get_ulsch_information), demultiplexer plan, codeword bits
  bool                         uci        = false;
  srs_amd_ulsch_info           info{};
  srs_amd_ulsch_demux_plan*    demux_plan = nullptr;
  uint32_t                     cw_bits    = 0;
  // CSI part 2 (its size known only once CSI part 1 is decoded): the multiplexing / demultiplexing / UL-SCH
  // configurations to recompute, and their results per CSI part 2 size (filled on first use)
  bool                         csi2       = false;
  uint32_t                     max_csi2   = 0; // largest size the description allows
  srs_amd_ulsch_config         ucfg{};
  srs_amd_ulsch_demux_config   dxcfg{};
  uint32_t                     nref       = 0;
  struct part2_geometry {
    srs_amd_ulsch_info        info{};
    srs_amd_ulsch_demux_plan* demux = nullptr;
    srs_amd_sch_plan          sch{};
  };
  mutable std::map<uint32_t, part2_geometry> part2;
  mutable std::mutex                         part2_mtx;
  // every CSI part 2 size the description can produce (the fused slot group selects among them on the device),
  // built on first use: sizes, geometries, the largest encoded length, and the device table
  // [NC] int32 sizes | [NC][C] rate-matching lengths | [NC][C] LLR offsets (srs_amd_sch_plan_segments)
  struct csi2_candidates {
    std::vector<uint32_t>              n2;
    std::vector<const part2_geometry*> geo;
    uint32_t                           max_e2 = 0;
    device_buffer                      d;
    bool                               ready = false;
    int                                rc    = SRS_AMD_OK; // a size without a geometry (cached)
  };
  mutable csi2_candidates cand;
  mutable std::mutex      cand_mtx;
  ~srs_amd_pusch_processor_plan()
  {
    srs_amd_pusch_demod_plan_destroy(demod_plan);
    srs_amd_ulsch_demux_plan_destroy(demux_plan);
    for (auto& kv : part2) {
      srs_amd_ulsch_demux_plan_destroy(kv.second.demux);
    }
  }
};

namespace {

// ldpc::compute_nof_codeblocks (ldpc.h:140-151).
uint32_t nof_codeblocks(uint32_t tbs, uint32_t bg)
{
  const uint32_t tb_and_crc = tbs + (tbs > 3824 ? 24u : 16u);
  const uint32_t max_seg    = bg == 1 ? 8448u : 3840u;
  return tb_and_crc <= max_seg ? 1u : (tb_and_crc + (max_seg - 24) - 1) / (max_seg - 24);
}

// ldpc::compute_N_ref (ldpc.h:225-228); MAX_CODEBLOCK_SIZE = 384 x 66.
uint32_t compute_N_ref(uint32_t tbs_lbrm_bytes, uint32_t C)
{
  const uint64_t n = static_cast<uint64_t>(tbs_lbrm_bytes) * 8 * 3 / (2 * C);
  return static_cast<uint32_t>(std::min<uint64_t>(n, 384 * 66));
}

// convert_dB_to_amplitude(-get_sch_to_dmrs_ratio_dB(n)) (sch_dmrs_power.h, math_utils.h:118), in float as
// the reference evaluates it.
float dmrs_scaling(uint32_t nof_cdm_groups_without_data)
{
  static const float beta_dmrs_db[4] = {NAN, 0.0F, -3.0F, -4.77F};
  const float        v               = -beta_dmrs_db[nof_cdm_groups_without_data];
  return std::pow(10.0F, v / 20.0F);
}

// The multiplexing geometry, demultiplexer plan and UL-SCH plan of `pl` with n2 CSI part 2 bits
// (pusch_processor_impl.cpp:73-103: get_ulsch_information again, set_csi_part2, set_nof_softbits), cached per size.
int plan_part2(srs_amd_pusch_processor*                                    proc,
               const srs_amd_pusch_processor_plan*                         pl,
               uint32_t                                                    n2,
               const srs_amd_pusch_processor_plan::part2_geometry**        out)
{
  std::lock_guard<std::mutex> lock(pl->part2_mtx);
  auto                        it = pl->part2.find(n2);
  if (it != pl->part2.end()) {
    *out = &it->second;
    return SRS_AMD_OK;
  }
  srs_amd_pusch_processor_plan::part2_geometry g;
  srs_amd_ulsch_config                         uc = pl->ucfg;
  uc.nof_csi_part2_bits                           = n2;
  int rc                                          = srs_amd_ulsch_information(&uc, &g.info);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  srs_amd_ulsch_demux_config dx = pl->dxcfg;
  dx.nof_csi_part2_bits         = n2;
  dx.nof_enc_csi_part2_bits     = g.info.nof_csi_part2_bits;
  uint32_t total = 0, sch_bits = 0;
  rc             = srs_amd_ulsch_demux_plan_create(proc->demux, &dx, &g.demux, &total, &sch_bits);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const uint32_t qm_bits = pl->pdu.modulation < 2 ? 1u : static_cast<uint32_t>(pl->pdu.modulation);
  if (total != pl->cw_bits || (pl->has_sch && sch_bits != g.info.nof_ul_sch_bits)) {
    srs_amd_ulsch_demux_plan_destroy(g.demux);
    return fail(SRS_AMD_EINVAL, "CSI part 2 multiplexing geometry mismatch (%u / %u UL-SCH bits).", sch_bits,
                g.info.nof_ul_sch_bits);
  }
  rc = !pl->has_sch ? SRS_AMD_OK
                    : srs_amd_sch_plan_compute(&g.sch, pl->pdu.tbs, pl->pdu.base_graph, pl->pdu.rv,
                                               static_cast<uint32_t>(pl->pdu.modulation), pl->nref,
                                               pl->pdu.nof_tx_layers, sch_bits / qm_bits);
  if (rc != SRS_AMD_OK) {
    srs_amd_ulsch_demux_plan_destroy(g.demux);
    return rc;
  }
  *out = &pl->part2.emplace(n2, g).first->second;
  return SRS_AMD_OK;
}

// The CSI part 2 candidates of `pl` (every size its description maps some CSI part 1 value to), with their
// geometries and device table; built once per plan (one synchronous upload).
int plan_csi2_candidates(srs_amd_pusch_processor* proc, const srs_amd_pusch_processor_plan* pl,
                         const srs_amd_pusch_processor_plan::csi2_candidates** out)
{
  std::lock_guard<std::mutex> lock(pl->cand_mtx);
  auto&                       c = pl->cand;
  if (c.ready && c.rc != SRS_AMD_OK) {
    return c.rc;
  }
  if (!c.ready) {
    const srs_amd_uci_part2_size_description& d  = pl->pdu.csi_part2_size;
    const uint32_t                            m0 = d.nof_entries > 0 ? d.entries[0].map_size : 1u;
    const uint32_t                            m1 = d.nof_entries > 1 ? d.entries[1].map_size : 1u;
    std::vector<uint32_t>                     sizes;
    for (uint32_t i0 = 0; i0 < m0 && i0 < 16; ++i0) {
      for (uint32_t i1 = 0; i1 < m1 && i1 < 16; ++i1) {
        const uint32_t n = (d.nof_entries > 0 ? d.entries[0].map[i0] : 0u) + (d.nof_entries > 1 ? d.entries[1].map[i1] : 0u);
        if (n != 0 && std::find(sizes.begin(), sizes.end(), n) == sizes.end()) {
          sizes.push_back(n);
        }
      }
    }
    std::sort(sizes.begin(), sizes.end());
    c.n2.clear();
    c.geo.clear();
    c.max_e2 = 0;
    for (uint32_t n : sizes) {
      const srs_amd_pusch_processor_plan::part2_geometry* g = nullptr;
      int rc = plan_part2(proc, pl, n, &g);
      if (rc != SRS_AMD_OK) {
        c.ready = true;
        c.rc    = rc;
        return rc;
      }
      c.n2.push_back(n);
      c.geo.push_back(g);
      c.max_e2 = std::max(c.max_e2, g->info.nof_csi_part2_bits);
    }
    const size_t          NC = c.n2.size();
    const uint32_t        C  = pl->has_sch ? pl->sch.nof_segments : 0u;
    std::vector<uint32_t> tab(NC + 2 * NC * C);
    for (size_t k = 0; k < NC; ++k) {
      tab[k] = c.n2[k];
      if (C != 0) {
        (void)srs_amd_sch_plan_segments(&c.geo[k]->sch, tab.data() + NC + k * C, tab.data() + NC + NC * C + k * C);
      }
    }
    hipError_t e = c.d.ensure(std::max<size_t>(tab.size(), 1) * sizeof(uint32_t));
    if (e == hipSuccess && !tab.empty()) {
      e = hipMemcpy(c.d.ptr, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "CSI part 2 candidate table");
    }
    c.ready = true;
  }
  *out = &c;
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_pusch_processor_create(srs_amd_pusch_processor**             proc,
                                   const srs_amd_pusch_processor_config* cfg,
                                   int                                   device)
{
  if (proc == nullptr || cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  *proc = nullptr;
  if (cfg->dec_nof_iterations == 0) {
    return fail(SRS_AMD_EINVAL, "The decoder number of iterations must be non-zero.");
  }
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* p   = new srs_amd_pusch_processor();
  p->device = device;
  p->cfg    = *cfg;
  if (const char* v = std::getenv("SRSRAN_AMD_PUSCH_FUSED")) {
    p->fuse = std::strcmp(v, "0") != 0;
  }
  rc = srs_amd_pusch_chest_create(&p->chest, device);
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_pusch_demodulator_create(&p->demod, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_pusch_decoder_create(&p->dec, cfg->ldpc_arith, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_ulsch_demux_create(&p->demux, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_uci_decoder_create(&p->uci, device);
  }
  if (rc == SRS_AMD_OK) {
    hipError_t e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      rc = hip_fail(e, "PUSCH processor stream");
    }
  }
  if (rc != SRS_AMD_OK) {
    delete p;
    return rc;
  }
  *proc = p;
  return SRS_AMD_OK;
}

void srs_amd_pusch_processor_destroy(srs_amd_pusch_processor* proc)
{
  delete proc;
}

int srs_amd_pusch_processor_plan_create(srs_amd_pusch_processor*       proc,
                                        const srs_amd_pusch_pdu*       pdu,
                                        uint32_t                       nof_subc,
                                        srs_amd_pusch_processor_plan** plan,
                                        srs_amd_sch_plan*              sch_plan,
                                        uint64_t*                      soft_buffer_bytes)
{
  if (proc == nullptr || pdu == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  *plan = nullptr;
  // pusch_processor_validator_impl.cpp checks, where the C-ABI subset narrows them
  const bool tp = pdu->transform_precoding != 0;
  if (tp) {
    if (pdu->nof_tx_layers != 1) {
      return fail(SRS_AMD_EINVAL, "Transform precoding is only possible with one layer.");
    }
    if (!srs_amd_transform_precoding_nof_prbs_valid(pdu->rb_count)) {
      return fail(SRS_AMD_EINVAL, "Transform precoding is only possible with a valid number of PRB.");
    }
    if (pdu->n_rs_id > 1007) {
      return fail(SRS_AMD_EINVAL, "Invalid n_rs_id %u.", pdu->n_rs_id);
    }
  } else {
    if (pdu->dmrs_type != 1) {
      return fail(SRS_AMD_EINVAL, "Only DM-RS type 1 is supported.");
    }
    if (pdu->nof_cdm_groups_without_data < 1 || pdu->nof_cdm_groups_without_data > 2) {
      return fail(SRS_AMD_EINVAL, "Invalid number of CDM groups without data (i.e., %u).",
                  pdu->nof_cdm_groups_without_data);
    }
  }
  // transform precoding keeps the default of two CDM groups without data (pusch_processor_impl.cpp:176)
  const uint32_t ncdm = tp ? 2u : pdu->nof_cdm_groups_without_data;
  if (pdu->rb_count == 0 || pdu->rb_start + pdu->rb_count > pdu->bwp_size_rb) {
    return fail(SRS_AMD_EINVAL, "Invalid frequency allocation.");
  }
  if (pdu->bwp_start_rb + pdu->bwp_size_rb > nof_subc / 12) {
    return fail(SRS_AMD_EINVAL, "The BWP exceeds the resource grid.");
  }
  // no codeword (tbs = 0): UCI only (pusch_processor_impl.cpp:305-324), which needs some UCI to carry
  const bool has_sch = pdu->tbs != 0;
  if (pdu->tbs % 8 != 0 || (!has_sch && pdu->nof_harq_ack == 0 && pdu->nof_csi_part1 == 0)) {
    return fail(SRS_AMD_EINVAL, "Invalid transport block size (i.e., %u).", pdu->tbs);
  }
  if (has_sch && pdu->base_graph != 1 && pdu->base_graph != 2) {
    return fail(SRS_AMD_EINVAL, "Invalid base graph.");
  }
  auto* pl     = new srs_amd_pusch_processor_plan();
  pl->pdu      = *pdu;
  pl->nof_subc = nof_subc;
  pl->has_sch  = has_sch;
  // DC subcarrier (pusch_processor_impl.cpp:235-249): zeroed in the estimates of CP-OFDM PDUs inside the grid
  if (!tp && pdu->has_dc_position && pdu->dc_position < nof_subc) {
    pl->dc_subc = pdu->dc_position;
  }
  // DM-RS estimator configuration (pusch_processor_impl.cpp:184-200)
  const uint32_t crb0       = pdu->bwp_start_rb + pdu->rb_start;
  srs_amd_pusch_chest_config& c = pl->chest_cfg;
  c.numerology              = pdu->numerology;
  c.slot_index              = pdu->slot_index;
  c.scrambling_id           = pdu->scrambling_id;
  c.n_scid                  = pdu->n_scid;
  c.nof_tx_layers           = pdu->nof_tx_layers;
  c.scaling                 = dmrs_scaling(ncdm);
  c.symbols_mask            = pdu->dmrs_symbol_mask;
  c.rb_start                = crb0;
  c.rb_count                = pdu->rb_count;
  c.first_symbol            = pdu->start_symbol_index;
  c.nof_symbols             = pdu->nof_symbols;
  c.fd_smoothing            = proc->cfg.fd_smoothing;
  c.td_interpolation        = proc->cfg.td_interpolation;
  c.compensate_cfo          = proc->cfg.compensate_cfo;
  c.low_papr                = tp ? 1 : 0;
  c.n_rs_id                 = pdu->n_rs_id;
  // demodulator configuration (pusch_processor_impl.cpp:368-383)
  srs_amd_pusch_demod_config dc{};
  dc.rnti = pdu->rnti;
  dc.n_id = pdu->n_id;
  dc.modulation = pdu->modulation;
  for (uint32_t r = crb0; r < crb0 + pdu->rb_count; ++r) {
    dc.crb_mask[r / 8] |= static_cast<uint8_t>(1u << (r % 8));
  }
  dc.start_symbol                = pdu->start_symbol_index;
  dc.nof_symbols                 = pdu->nof_symbols;
  dc.dmrs_symbol_mask            = pdu->dmrs_symbol_mask;
  dc.dmrs_type                   = tp ? 1u : pdu->dmrs_type;
  dc.nof_cdm_groups_without_data = ncdm;
  dc.transform_precoding         = tp ? 1u : 0u;
  dc.nof_tx_layers               = pdu->nof_tx_layers;
  dc.nof_rx_ports                = pdu->nof_rx_ports;
  dc.equalizer                   = proc->cfg.equalizer;
  {
    // the fused equalizer reads the one or two LSE slices of each symbol (any number of DM-RS symbols)
    const uint32_t nof_lse = c.td_interpolation == SRS_AMD_CHEST_TD_AVERAGE
                                 ? 1u
                                 : static_cast<uint32_t>(__builtin_popcount(c.symbols_mask & 0x3fffu));
    const bool mmse = proc->cfg.equalizer == SRS_AMD_EQ_MMSE && pdu->nof_tx_layers > 1;
    pl->fusable     = pusch_equalize_fusable(pdu->nof_rx_ports, pdu->nof_tx_layers, mmse, nof_lse);
  }
  int rc = srs_amd_pusch_demod_plan_create(proc->demod, &dc, nof_subc, &pl->demod_plan, &pl->nof_re);
  if (rc != SRS_AMD_OK) {
    delete pl;
    return rc;
  }
  pusch_demod_plan_set_dc(pl->demod_plan, pl->dc_subc);
  // UCI multiplexing (pusch_processor_impl.cpp:252-299): the geometry of get_ulsch_information, the
  // demultiplexer's placement; the UL-SCH then gets nof_ul_sch_bits of the codeword's bits
  const uint32_t qm_bits  = pdu->modulation < 2 ? 1u : static_cast<uint32_t>(pdu->modulation);
  pl->cw_bits             = pl->nof_re * pdu->nof_tx_layers * qm_bits;
  uint32_t       sch_bits = pl->cw_bits;
  pl->uci                 = pdu->nof_harq_ack != 0 || pdu->nof_csi_part1 != 0;
  // the allocation overlaps the DC (pusch_processor_impl.cpp:262-286 contains_dc: nof_dc_overlap_bits of the
  // multiplexing geometry, informational)
  const uint32_t dc_prb   = pdu->has_dc_position ? pdu->dc_position / 12 : ~0u;
  const int32_t  with_dc  = dc_prb >= crb0 && dc_prb < crb0 + pdu->rb_count ? 1 : 0;
  pl->csi2                = pdu->nof_csi_part1 != 0 && pdu->csi_part2_size.nof_entries != 0;
  if (pdu->csi_part2_size.nof_entries > 2) {
    delete pl;
    return fail(SRS_AMD_EINVAL, "At most two CSI part 2 size entries.");
  }
  for (uint32_t e = 0; e < pdu->csi_part2_size.nof_entries && pl->csi2; ++e) {
    const srs_amd_uci_part2_entry& en = pdu->csi_part2_size.entries[e];
    uint32_t                       w  = 0, mx = 0;
    for (uint32_t q = 0; q < en.nof_parameters && q < 2; ++q) {
      w += en.parameters[q].width;
      if (static_cast<uint32_t>(en.parameters[q].offset) + en.parameters[q].width > pdu->nof_csi_part1) {
        delete pl;
        return fail(SRS_AMD_EINVAL, "CSI part 2 size parameter beyond the CSI part 1 payload.");
      }
    }
    if (en.nof_parameters > 2 || w > 4 || en.map_size != (1u << w)) {
      delete pl;
      return fail(SRS_AMD_EINVAL, "Invalid CSI part 2 size entry (parameters, widths or map size).");
    }
    for (uint32_t m = 0; m < en.map_size; ++m) {
      mx = std::max<uint32_t>(mx, en.map[m]);
    }
    pl->max_csi2 += mx;
  }
  if (pl->uci) {
    srs_amd_ulsch_config uc{};
    uc.tbs                         = pdu->tbs;
    uc.modulation                  = pdu->modulation;
    uc.target_code_rate            = pdu->target_code_rate;
    uc.nof_harq_ack_bits           = pdu->nof_harq_ack;
    uc.nof_csi_part1_bits          = pdu->nof_csi_part1;
    uc.alpha_scaling               = pdu->alpha_scaling;
    uc.beta_offset_harq_ack        = pdu->beta_offset_harq_ack;
    uc.beta_offset_csi_part1       = pdu->beta_offset_csi_part1;
    uc.nof_rb                      = pdu->rb_count;
    uc.start_symbol_index          = pdu->start_symbol_index;
    uc.nof_symbols                 = pdu->nof_symbols;
    uc.dmrs_type                   = 1;
    uc.dmrs_symbol_mask            = pdu->dmrs_symbol_mask;
    uc.nof_cdm_groups_without_data = ncdm;
    uc.nof_layers                  = pdu->nof_tx_layers;
    uc.beta_offset_csi_part2       = pdu->beta_offset_csi_part2;
    uc.contains_dc                 = with_dc;
    rc                             = srs_amd_ulsch_information(&uc, &pl->info);
    pl->ucfg                       = uc;
    srs_amd_ulsch_demux_config dx{};
    dx.modulation                  = pdu->modulation;
    dx.nof_layers                  = pdu->nof_tx_layers;
    dx.nof_prb                     = pdu->rb_count;
    dx.start_symbol_index          = pdu->start_symbol_index;
    dx.nof_symbols                 = pdu->nof_symbols;
    dx.nof_harq_ack_rvd            = pl->info.nof_harq_ack_rvd;
    dx.dmrs_type                   = 1;
    dx.dmrs_symbol_mask            = pdu->dmrs_symbol_mask;
    dx.nof_cdm_groups_without_data = ncdm;
    dx.nof_harq_ack_bits           = pdu->nof_harq_ack;
    dx.nof_enc_harq_ack_bits       = pl->info.nof_harq_ack_bits;
    dx.nof_csi_part1_bits          = pdu->nof_csi_part1;
    dx.nof_enc_csi_part1_bits      = pl->info.nof_csi_part1_bits;
    dx.c_init                      = (pdu->rnti << 15) + pdu->n_id;
    pl->dxcfg                      = dx;
    uint32_t total                 = 0;
    if (rc == SRS_AMD_OK) {
      rc = srs_amd_ulsch_demux_plan_create(proc->demux, &dx, &pl->demux_plan, &total, &sch_bits);
    }
    if (rc == SRS_AMD_OK && (total != pl->cw_bits || (has_sch && sch_bits != pl->info.nof_ul_sch_bits))) {
      rc = fail(SRS_AMD_EINVAL, "UCI multiplexing geometry mismatch (%u / %u codeword bits, %u / %u UL-SCH bits).",
                total, pl->cw_bits, sch_bits, pl->info.nof_ul_sch_bits);
    }
    if (rc != SRS_AMD_OK) {
      delete pl;
      return rc;
    }
  }
  // decoder configuration (pusch_processor_impl.cpp:322-347): the UL-SCH's share of the codeword
  if (has_sch) {
    const uint32_t C        = nof_codeblocks(pdu->tbs, pdu->base_graph);
    const uint32_t tbs_lbrm = pdu->tbs_lbrm_bytes ? pdu->tbs_lbrm_bytes : 159749u; // tbs_lbrm_default
    pl->nref                = compute_N_ref(tbs_lbrm, C);
    rc = srs_amd_sch_plan_compute(&pl->sch, pdu->tbs, pdu->base_graph, pdu->rv,
                                  static_cast<uint32_t>(pdu->modulation), pl->nref, pdu->nof_tx_layers,
                                  sch_bits / qm_bits);
  } else {
    // UCI only: REs the UCI leaves free go to the demultiplexer's UL-SCH stream, which nothing decodes (the
    // reference's decoder_buffer_dummy, pusch_processor_impl.cpp:300-305): a discarded row of that length
    pl->dummy_sch_bits = sch_bits;
  }
  if (rc != SRS_AMD_OK) {
    delete pl;
    return rc;
  }
  pl->dec_cfg.nof_ldpc_iterations = proc->cfg.dec_nof_iterations;
  pl->dec_cfg.force_decoding      = proc->cfg.dec_force_decoding;
  pl->dec_cfg.use_early_stop      = proc->cfg.dec_enable_early_stop;
  pl->dec_cfg.new_data            = pdu->new_data;
  pl->soft_bytes                  = srs_amd_pusch_soft_buffer_size(&pl->sch);
  if (sch_plan != nullptr) {
    *sch_plan = pl->sch;
  }
  if (soft_buffer_bytes != nullptr) {
    *soft_buffer_bytes = pl->soft_bytes;
  }
  *plan = pl;
  return SRS_AMD_OK;
}

void srs_amd_pusch_processor_plan_destroy(srs_amd_pusch_processor_plan* plan)
{
  delete plan;
}

} // extern "C"

namespace {

// The UCI PDUs (index ucis[j] of the fused group) of a slot call: one demultiplexer launch over every codeword, the
// HARQ-ACK / CSI part 1 messages through the slot-form UCI decoder (uci_slot_build), statuses into uci_status[k][4]
// (zeroed first) and payloads into the caller's UCI rows (d_uci + uci_offset) or scratch; the per-PDU field masks
// of the result kernel (every fused PDU k) after the descriptors in uci_items.
// CSI part 2 PDUs (cands[k] non-null): after their CSI part 1 is decoded, csi2_select_kernel picks the size on the
// device (sel[k], the fourth status column); a second demultiplexer launch with one block per (PDU, candidate size)
// and one UCI decoder set per (PDU, candidate size) run only for the selected candidate (device predicates), so the
// UL-SCH rows and the CSI part 2 message take that size's geometry with no host round trip
// (pusch_processor_impl.cpp:56-103 does the same from on_csi_part1).  Without CSI part 2 the UCI decoders run on a
// helper stream beside the UL-SCH decoder; with it they run on the call's stream, before the decoder.
int fused_uci(srs_amd_pusch_processor* proc, const srs_amd_pusch_slot_pdu* pdus, const std::vector<uint32_t>& fused,
              const std::vector<uint32_t>& ucis, const std::vector<size_t>& cw_off, const std::vector<size_t>& uci_off,
              const std::vector<size_t>& c2_off, const std::vector<size_t>& pay_off,
              const std::vector<const srs_amd_pusch_processor_plan::csi2_candidates*>& cands, int8_t* llrs,
              const std::vector<size_t>& llr_off, uint8_t* d_uci, hipStream_t s)
{
  const uint32_t n  = static_cast<uint32_t>(fused.size());
  int8_t*        cw = proc->cw_llrs.as<int8_t>();
  int8_t*        ur = proc->uci_llrs.as<int8_t>();
  int32_t*       st = proc->uci_status.as<int32_t>();
  int32_t*       sel = proc->csi2_sel.as<int32_t>();
  std::vector<demux_args>       dx, dx2;
  std::vector<uci_slot_message> msgs, msgs2;
  std::vector<csi2_select_args> sels;
  std::vector<uint32_t>         masks(n, 0);
  uint32_t                      max_re = 0, max_re2 = 0;
  for (uint32_t k : ucis) {
    const srs_amd_pusch_slot_pdu&       u    = pdus[fused[k]];
    const srs_amd_pusch_processor_plan* pl   = u.plan;
    const uint32_t                      ka   = pl->pdu.nof_harq_ack, kc = pl->pdu.nof_csi_part1;
    const uint32_t                      ea   = pl->info.nof_harq_ack_bits, ec = pl->info.nof_csi_part1_bits;
    int8_t*                             rows = ur + uci_off[k];
    uint8_t* pay = d_uci != nullptr ? d_uci + u.uci_offset : proc->uci_payload.as<uint8_t>() + pay_off[k];
    dx.push_back(make_demux_args(pl->demux_plan, cw + cw_off[k], llrs + llr_off[k], rows, rows + ea));
    max_re = std::max(max_re, dx.back().nof_re);
    if (ka != 0) {
      msgs.push_back(uci_slot_message{rows, ea, ka, pl->pdu.modulation, pay, st + 4 * k});
    }
    if (kc != 0) {
      msgs.push_back(uci_slot_message{rows + ea, ec, kc, pl->pdu.modulation, pay + ka, st + 4 * k + 1});
    }
    masks[k] = (ka != 0 ? 1u : 0u) | (kc != 0 ? 2u : 0u);
    const auto* c = cands[k];
    if (c == nullptr) {
      continue;
    }
    masks[k] |= 4u;
    csi2_select_args sa{};
    sa.part1     = pay + ka;
    sa.status1   = st + 4 * k + 1;
    sa.nof_part2 = st + 4 * k + 3;
    sa.sel       = sel + k;
    sa.cand      = c->d.as<int32_t>();
    sa.nof_cand  = static_cast<uint32_t>(c->n2.size());
    sa.nof_part1 = kc;
    sa.descr     = pl->pdu.csi_part2_size;
    sels.push_back(sa);
    int8_t* c2 = ur + c2_off[k];
    for (size_t q = 0; q < c->n2.size(); ++q) {
      const auto* g = c->geo[q];
      demux_args  d = make_demux_args_csi2(g->demux, cw + cw_off[k], llrs + llr_off[k], rows, rows + ea, c2);
      d.sel         = sel + k;
      d.sel_val     = static_cast<int32_t>(q);
      dx2.push_back(d);
      max_re2 = std::max(max_re2, d.nof_re);
      uci_slot_message m{c2, g->info.nof_csi_part2_bits, c->n2[q], pl->pdu.modulation, pay + ka + kc, st + 4 * k + 2};
      m.pred     = sel + k;
      m.pred_val = static_cast<int32_t>(q);
      msgs2.push_back(m);
    }
  }
  uci_slot_plan up, up2;
  int           rc = uci_slot_build(proc->uci, msgs.data(), static_cast<uint32_t>(msgs.size()), nullptr, up);
  if (rc == SRS_AMD_OK) {
    rc = uci_slot_build(proc->uci, msgs2.data(), static_cast<uint32_t>(msgs2.size()), nullptr, up2);
  }
  hipError_t e = hipSuccess;
  if (rc == SRS_AMD_OK && up.cb_bytes + up2.cb_bytes != 0) {
    e = proc->uci_cbs.ensure(up.cb_bytes + up2.cb_bytes);
  }
  if (rc == SRS_AMD_OK && e == hipSuccess) {
    rc = uci_slot_build(proc->uci, msgs.data(), static_cast<uint32_t>(msgs.size()), proc->uci_cbs.as<uint8_t>(), up);
  }
  if (rc == SRS_AMD_OK && e == hipSuccess) {
    rc = uci_slot_build(proc->uci, msgs2.data(), static_cast<uint32_t>(msgs2.size()),
                        proc->uci_cbs.as<uint8_t>() + up.cb_bytes, up2);
  }
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // staging layout: pass-1 demux | shorts | polars | finishes | field masks | CSI part 2 selections | pass-2 demux |
  // CSI part 2 shorts | polars | finishes
  size_t     off = 0;
  const auto put = [&](size_t bytes) {
    const size_t o = off;
    off            = align_up(off + bytes, 64);
    return o;
  };
  const size_t o_dx  = put(sizeof(demux_args) * dx.size());
  const size_t o_sh  = put(sizeof(uci_short_args) * up.shorts.size());
  const size_t o_po  = put(sizeof(polar_args) * up.polars.size());
  const size_t o_fi  = put(sizeof(uci_polar_args) * up.finishes.size());
  const size_t o_mk  = put(sizeof(uint32_t) * n);
  const size_t o_se  = put(sizeof(csi2_select_args) * sels.size());
  const size_t o_dx2 = put(sizeof(demux_args) * dx2.size());
  const size_t o_sh2 = put(sizeof(uci_short_args) * up2.shorts.size());
  const size_t o_po2 = put(sizeof(polar_args) * up2.polars.size());
  const size_t o_fi2 = put(sizeof(uci_polar_args) * up2.finishes.size());
  const size_t total = off;
  if (e == hipSuccess) {
    e = proc->uci_items.ensure(total);
  }
  if (e == hipSuccess) {
    e = proc->stage3.acquire(total);
  }
  if (e == hipSuccess) {
    e = hipMemsetAsync(st, 0, sizeof(int32_t) * 4 * n, s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH slot UCI scratch");
  }
  auto copy = [&](size_t o, const void* src, size_t bytes) {
    if (bytes != 0) {
      std::memcpy(proc->stage3.at<uint8_t>(o), src, bytes);
    }
  };
  copy(o_dx, dx.data(), sizeof(demux_args) * dx.size());
  copy(o_sh, up.shorts.data(), sizeof(uci_short_args) * up.shorts.size());
  copy(o_po, up.polars.data(), sizeof(polar_args) * up.polars.size());
  copy(o_fi, up.finishes.data(), sizeof(uci_polar_args) * up.finishes.size());
  copy(o_mk, masks.data(), sizeof(uint32_t) * n);
  copy(o_se, sels.data(), sizeof(csi2_select_args) * sels.size());
  copy(o_dx2, dx2.data(), sizeof(demux_args) * dx2.size());
  copy(o_sh2, up2.shorts.data(), sizeof(uci_short_args) * up2.shorts.size());
  copy(o_po2, up2.polars.data(), sizeof(polar_args) * up2.polars.size());
  copy(o_fi2, up2.finishes.data(), sizeof(uci_polar_args) * up2.finishes.size());
  proc->uci_masks_offset = o_mk;
  auto* d = proc->uci_items.as<uint8_t>();
  e       = proc->stage3.upload(d, total, s);
  if (e == hipSuccess) {
    e = launch_ulsch_demux_items(reinterpret_cast<const demux_args*>(d + o_dx), static_cast<uint32_t>(dx.size()),
                                 max_re, s);
  }
  // the UCI decoders depend only on the demultiplexer: on a helper stream beside the UL-SCH decoder (joined by the
  // caller before the result kernel) -- unless CSI part 2 sizes the UL-SCH geometry, then on this stream
  const bool serial = !sels.empty();
  if (e == hipSuccess && !serial) {
    e = proc->fan.begin(s, 2);
  }
  const hipStream_t hs = serial ? s : proc->fan.stream(s, 0);
  if (e == hipSuccess) {
    e = launch_uci_short_items(reinterpret_cast<const uci_short_args*>(d + o_sh),
                               static_cast<uint32_t>(up.shorts.size()), hs);
  }
  if (e == hipSuccess) {
    e = launch_polar_decode_items(reinterpret_cast<const polar_args*>(d + o_po),
                                  static_cast<uint32_t>(up.polars.size()), hs);
  }
  if (e == hipSuccess) {
    e = launch_uci_polar_finish_items(reinterpret_cast<const uci_polar_args*>(d + o_fi),
                                      static_cast<uint32_t>(up.finishes.size()), hs);
  }
  if (serial) {
    if (e == hipSuccess) {
      e = launch_csi2_select(reinterpret_cast<const csi2_select_args*>(d + o_se), static_cast<uint32_t>(sels.size()), s);
    }
    if (e == hipSuccess) {
      e = launch_ulsch_demux_items(reinterpret_cast<const demux_args*>(d + o_dx2), static_cast<uint32_t>(dx2.size()),
                                   max_re2, s);
    }
    if (e == hipSuccess) {
      e = launch_uci_short_items(reinterpret_cast<const uci_short_args*>(d + o_sh2),
                                 static_cast<uint32_t>(up2.shorts.size()), s);
    }
    if (e == hipSuccess) {
      e = launch_polar_decode_items(reinterpret_cast<const polar_args*>(d + o_po2),
                                    static_cast<uint32_t>(up2.polars.size()), s);
    }
    if (e == hipSuccess) {
      e = launch_uci_polar_finish_items(reinterpret_cast<const uci_polar_args*>(d + o_fi2),
                                        static_cast<uint32_t>(up2.finishes.size()), s);
    }
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUSCH slot UCI launches");
}

// CSI part 2 of a batch of grids of one plan on the device, after its CSI part 1 decoding (statuses [g][4] in
// uci_status): the size selection per grid, the second demultiplexer pass and the CSI part 2 decoders per (grid,
// candidate size) under device predicates, and the UL-SCH of every grid through the slot decoder with per-grid row
// patches to the selected size's geometry (pusch_processor_impl.cpp:56-103, as the fused slot group does).
int csi2_batch_device(srs_amd_pusch_processor* proc, const srs_amd_pusch_processor_plan* plan,
                      const srs_amd_pusch_processor_plan::csi2_candidates* cand, uint32_t nof_grids,
                      const int8_t* dem_rows, uint64_t cw_stride, int8_t* llrs, uint64_t llr_stride, int8_t* uci_rows,
                      uint64_t uci_stride, uint64_t ack_e, uint64_t csi2_stride, const uint8_t* part1,
                      uint64_t part1_stride, uint8_t* part2, uint64_t part2_stride, uint8_t* d_tbs, uint32_t tb_stride,
                      int8_t* d_soft, int32_t* cb_iters, hipStream_t s)
{
  int32_t*       st  = proc->uci_status.as<int32_t>();
  hipError_t     e   = proc->csi2_sel.ensure(sizeof(int32_t) * nof_grids);
  if (e != hipSuccess) {
    return hip_fail(e, "CSI part 2 selection scratch");
  }
  int32_t*                      sel = proc->csi2_sel.as<int32_t>();
  const size_t                  NC  = cand->n2.size();
  std::vector<csi2_select_args> sels(nof_grids);
  std::vector<demux_args>       dx;
  std::vector<uci_slot_message> msgs;
  uint32_t                      max_re = 0;
  int8_t* const                 c2_base = uci_rows + static_cast<uint64_t>(nof_grids) * uci_stride;
  for (uint32_t g = 0; g < nof_grids; ++g) {
    csi2_select_args& a = sels[g];
    a.part1     = part1 + g * part1_stride;
    a.status1   = st + 4 * g + 1;
    a.nof_part2 = st + 4 * g + 3;
    a.sel       = sel + g;
    a.cand      = cand->d.as<int32_t>();
    a.nof_cand  = static_cast<uint32_t>(NC);
    a.nof_part1 = plan->pdu.nof_csi_part1;
    a.descr     = plan->pdu.csi_part2_size;
    int8_t* u1  = uci_rows + g * uci_stride;
    int8_t* c2  = c2_base + g * csi2_stride;
    for (size_t q = 0; q < NC; ++q) {
      const auto* geo = cand->geo[q];
      demux_args  d   = make_demux_args_csi2(geo->demux, dem_rows + g * cw_stride, llrs + g * llr_stride, u1,
                                             u1 + ack_e, c2);
      d.sel           = sel + g;
      d.sel_val       = static_cast<int32_t>(q);
      dx.push_back(d);
      max_re = std::max(max_re, d.nof_re);
      uci_slot_message m{c2, geo->info.nof_csi_part2_bits, cand->n2[q], plan->pdu.modulation, part2 + g * part2_stride,
                         st + 4 * g + 2};
      m.pred     = sel + g;
      m.pred_val = static_cast<int32_t>(q);
      msgs.push_back(m);
    }
  }
  uci_slot_plan up;
  int           rc = uci_slot_build(proc->uci, msgs.data(), static_cast<uint32_t>(msgs.size()), nullptr, up);
  if (rc == SRS_AMD_OK && up.cb_bytes != 0) {
    e = proc->uci_cbs.ensure(up.cb_bytes);
  }
  if (rc == SRS_AMD_OK && e == hipSuccess) {
    rc = uci_slot_build(proc->uci, msgs.data(), static_cast<uint32_t>(msgs.size()), proc->uci_cbs.as<uint8_t>(), up);
  }
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const size_t o_se  = 0;
  const size_t o_dx  = align_up(sizeof(csi2_select_args) * sels.size(), 64);
  const size_t o_sh  = o_dx + align_up(sizeof(demux_args) * dx.size(), 64);
  const size_t o_po  = o_sh + align_up(sizeof(uci_short_args) * up.shorts.size(), 64);
  const size_t o_fi  = o_po + align_up(sizeof(polar_args) * up.polars.size(), 64);
  const size_t total = o_fi + sizeof(uci_polar_args) * up.finishes.size();
  if (e == hipSuccess) {
    e = proc->uci_items.ensure(total);
  }
  if (e == hipSuccess) {
    e = proc->stage3.acquire(total);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "CSI part 2 descriptors");
  }
  std::memcpy(proc->stage3.at<uint8_t>(o_se), sels.data(), sizeof(csi2_select_args) * sels.size());
  std::memcpy(proc->stage3.at<uint8_t>(o_dx), dx.data(), sizeof(demux_args) * dx.size());
  std::memcpy(proc->stage3.at<uint8_t>(o_sh), up.shorts.data(), sizeof(uci_short_args) * up.shorts.size());
  std::memcpy(proc->stage3.at<uint8_t>(o_po), up.polars.data(), sizeof(polar_args) * up.polars.size());
  std::memcpy(proc->stage3.at<uint8_t>(o_fi), up.finishes.data(), sizeof(uci_polar_args) * up.finishes.size());
  auto* d = proc->uci_items.as<uint8_t>();
  e       = proc->stage3.upload(d, total, s);
  if (e == hipSuccess) {
    e = launch_csi2_select(reinterpret_cast<const csi2_select_args*>(d + o_se), nof_grids, s);
  }
  if (e == hipSuccess) {
    e = launch_ulsch_demux_items(reinterpret_cast<const demux_args*>(d + o_dx), static_cast<uint32_t>(dx.size()),
                                 max_re, s);
  }
  if (e == hipSuccess) {
    e = launch_uci_short_items(reinterpret_cast<const uci_short_args*>(d + o_sh),
                               static_cast<uint32_t>(up.shorts.size()), s);
  }
  if (e == hipSuccess) {
    e = launch_polar_decode_items(reinterpret_cast<const polar_args*>(d + o_po), static_cast<uint32_t>(up.polars.size()),
                                  s);
  }
  if (e == hipSuccess) {
    e = launch_uci_polar_finish_items(reinterpret_cast<const uci_polar_args*>(d + o_fi),
                                      static_cast<uint32_t>(up.finishes.size()), s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "CSI part 2 launches");
  }
  auto* dres = proc->dec_results.as<srs_amd_pusch_decoder_result>();
  if (!plan->has_sch) {
    e = hipMemsetAsync(dres, 0, sizeof(srs_amd_pusch_decoder_result) * nof_grids, s);
    return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUSCH processor UCI-only result");
  }
  // the UL-SCH of every grid: one slot-decoder UE per grid, rows patched to the selected size's geometry
  const uint32_t                NCu = static_cast<uint32_t>(NC), C = plan->sch.nof_segments;
  const auto*                   t   = cand->d.as<uint32_t>();
  std::vector<srs_amd_pusch_ue> ues(nof_grids);
  std::vector<uint32_t>         cb_off(nof_grids);
  std::vector<slot_harq>        harq(nof_grids);
  std::vector<slot_ue_patch>    patches(nof_grids);
  for (uint32_t g = 0; g < nof_grids; ++g) {
    ues[g]     = srs_amd_pusch_ue{plan->sch, g * llr_stride, static_cast<uint64_t>(g) * tb_stride};
    cb_off[g]  = g * C;
    harq[g]    = slot_harq{d_soft != nullptr ? d_soft + g * plan->soft_bytes : nullptr, plan->dec_cfg.new_data};
    patches[g] = slot_ue_patch{g, sel + g, t + NCu, t + NCu + NCu * C};
  }
  return pusch_decode_slot_ex(proc->dec, &plan->dec_cfg, ues.data(), nof_grids, llrs, d_tbs, dres,
                              cb_iters != nullptr ? cb_off.data() : nullptr, cb_iters, s,
                              d_soft != nullptr ? harq.data() : nullptr, patches.data(), nof_grids);
}

// chest: the estimator configuration to run (the plan's, or a copy in another slot); nullptr: the plan's.
int process_batch_locked(srs_amd_pusch_processor*            proc,
                         const srs_amd_pusch_processor_plan* plan,
                         const uint32_t*                     d_grids,
                         uint64_t                            grid_stride,
                         uint32_t                            nof_grids,
                         uint8_t*                            d_tbs,
                         uint32_t                            tb_stride,
                         srs_amd_pusch_processor_result*     d_results,
                         int8_t*                             d_soft,
                         const srs_amd_pusch_intermediates*  io,
                         void*                               stream,
                         const srs_amd_pusch_chest_config*   chest = nullptr)
{
  if (proc == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_grids == 0) {
    return SRS_AMD_OK;
  }
  if (d_grids == nullptr || (d_tbs == nullptr && plan->has_sch) || d_results == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  const uint32_t P     = plan->pdu.nof_rx_ports;
  const uint32_t L     = plan->pdu.nof_tx_layers;
  const uint64_t plane = 14ull * plan->nof_subc;
  if (nof_grids > 1 && (grid_stride < P * plane || tb_stride < plan->pdu.tbs / 8)) {
    return fail(SRS_AMD_EINVAL, "grid or transport block stride too small");
  }
  const srs_amd_pusch_chest_config* cc = chest != nullptr ? chest : &plan->chest_cfg;
  const uint32_t G            = plan->has_sch ? plan->sch.cw_length : plan->dummy_sch_bits;
  const bool     uci          = plan->uci;
  const bool     own_est      = io == nullptr || io->d_estimates == nullptr;
  // Without a caller estimate buffer the equalizer rebuilds each RE's estimate from the estimator's
  // per-subcarrier output (pusch_demod.hip pusch_equalize_fused_kernel): no estimate tensor in HBM.
  const bool     fused        = own_est && plan->fusable && proc->fuse;
  const bool     own_llrs     = io == nullptr || io->d_llrs == nullptr;
  const uint64_t est_stride   = own_est ? P * L * plane : io->est_stride;
  const uint32_t llr_stride   = own_llrs ? static_cast<uint32_t>(align_up(G, 64)) : io->llr_stride;
  if ((!own_est && nof_grids > 1 && est_stride < P * L * plane) || (!own_llrs && llr_stride < G)) {
    return fail(SRS_AMD_EINVAL, "intermediate estimate or LLR stride too small");
  }
  auto           s          = static_cast<hipStream_t>(stream);
  hipError_t     e          = hipSetDevice(proc->device);
  if (e == hipSuccess && own_est && !fused) {
    e = proc->estimates.ensure(nof_grids * est_stride * 4);
  }
  if (e == hipSuccess) {
    e = proc->stats.ensure(static_cast<size_t>(nof_grids) * P * sizeof(srs_amd_chest_port_stats));
  }
  if (e == hipSuccess && own_llrs) {
    e = proc->llrs.ensure(static_cast<size_t>(nof_grids) * llr_stride);
  }
  if (e == hipSuccess) {
    e = proc->dec_results.ensure(static_cast<size_t>(nof_grids) * sizeof(srs_amd_pusch_decoder_result));
  }
  // UCI: the whole codeword's LLRs before the demultiplexer, the UCI streams, payloads and statuses
  const uint64_t cw_stride  = align_up(plan->cw_bits, 64);
  const uint64_t ack_e      = plan->info.nof_harq_ack_bits, csi1_e = plan->info.nof_csi_part1_bits;
  const uint64_t uci_stride = align_up(ack_e + csi1_e, 64);
  const uint32_t K_ack = plan->pdu.nof_harq_ack, K_csi1 = plan->pdu.nof_csi_part1;
  // payload rows: HARQ-ACK | CSI part 1 | CSI part 2 (largest size); statuses [grid][4] (pusch_result_args)
  const uint64_t pay_stride = align_up(K_ack + K_csi1 + plan->max_csi2, 64);
  // CSI part 2 LLR rows: the largest encoded size any CSI part 2 size can take is below the codeword length
  const uint64_t csi2_stride = plan->csi2 ? cw_stride : 0;
  if (e == hipSuccess && uci) {
    e = proc->cw_llrs.ensure(nof_grids * cw_stride);
  }
  if (e == hipSuccess && uci) {
    e = proc->uci_llrs.ensure(nof_grids * (uci_stride + csi2_stride));
  }
  if (e == hipSuccess && uci) {
    e = proc->uci_payload.ensure(nof_grids * pay_stride);
  }
  if (e == hipSuccess && uci) {
    e = proc->uci_status.ensure(static_cast<size_t>(nof_grids) * 4 * sizeof(int32_t));
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH processor scratch");
  }
  // every return from here records the completion event the next call on another stream waits for
  call_scope scope(proc->order, nullptr, s);
  if (uci) { // after begin: a previous call on another stream may still read the statuses
    e = hipMemsetAsync(proc->uci_status.ptr, 0, static_cast<size_t>(nof_grids) * 4 * sizeof(int32_t), s);
    if (e != hipSuccess) {
      return hip_fail(e, "PUSCH processor UCI status reset");
    }
  }
  int32_t* const cb_iters = io != nullptr ? io->d_cb_iterations : nullptr;
  const uint32_t C        = plan->sch.nof_segments;
  srs_amd_chest_port_stats* st   = (io && io->d_port_stats) ? io->d_port_stats : proc->stats.as<srs_amd_chest_port_stats>();
  uint32_t*                 est  = own_est ? proc->estimates.as<uint32_t>() : io->d_estimates;
  int8_t*                   llrs = own_llrs ? proc->llrs.as<int8_t>() : io->d_llrs;
  // the demodulator's rows: the UL-SCH LLRs directly, or with UCI the whole codeword for the demultiplexer
  int8_t*        dem_rows   = uci ? proc->cw_llrs.as<int8_t>() : llrs;
  const uint64_t dem_stride = uci ? cw_stride : llr_stride;
  int rc;
  if (fused) {
    chest_args view;
    rc = chest_estimate_batch_unexpanded(proc->chest, cc, d_grids, grid_stride, P, plan->nof_subc, nof_grids, st,
                                         stream, &view);
    if (rc == SRS_AMD_OK) {
      rc = pusch_demodulate_batch_fused(proc->demod, plan->demod_plan, d_grids, grid_stride, view, st, dem_rows,
                                        dem_stride, nof_grids, stream);
    }
  } else {
    rc = srs_amd_pusch_chest_estimate_batch(proc->chest, cc, d_grids, grid_stride, P, plan->nof_subc, nof_grids, est,
                                            est_stride, st, stream);
    // the DC step of pusch_processor_impl.cpp:235-249 on the caller's estimates (the equalizer reads the DC
    // subcarrier as zero in any case)
    if (rc == SRS_AMD_OK && !own_est && plan->dc_subc != ~0u) {
      e  = launch_pusch_dc_zero(est, est_stride, P * L, plan->nof_subc, plan->pdu.start_symbol_index,
                                plan->pdu.nof_symbols, plan->dc_subc, nof_grids, s);
      rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pusch_dc_zero_kernel launch");
    }
    if (rc == SRS_AMD_OK) {
      rc = srs_amd_pusch_demodulate_batch(proc->demod, plan->demod_plan, d_grids, grid_stride, est, est_stride, st,
                                          dem_rows, dem_stride, nof_grids, stream);
    }
  }
  // UL-SCH / HARQ-ACK / CSI part 1 (ulsch_demultiplex_impl), then the UCI decoders (uci_decoder_impl)
  int8_t* uci_rows = proc->uci_llrs.as<int8_t>();
  if (rc == SRS_AMD_OK && uci) {
    rc = srs_amd_ulsch_demultiplex_batch(proc->demux, plan->demux_plan, dem_rows, cw_stride, llrs, llr_stride,
                                         uci_rows, uci_stride, uci_rows + ack_e, uci_stride, nof_grids, stream);
  }
  if (rc == SRS_AMD_OK && uci && K_ack != 0) {
    const bool out = io != nullptr && io->d_harq_ack != nullptr;
    rc = srs_amd_uci_decode_batch(proc->uci, uci_rows, uci_stride, static_cast<uint32_t>(ack_e), K_ack,
                                  plan->pdu.modulation, out ? io->d_harq_ack : proc->uci_payload.as<uint8_t>(),
                                  out ? io->harq_ack_stride : pay_stride, proc->uci_status.as<int32_t>(),
                                  4 * sizeof(int32_t), nof_grids, stream);
  }
  if (rc == SRS_AMD_OK && uci && K_csi1 != 0) {
    const bool out = io != nullptr && io->d_csi_part1 != nullptr;
    rc = srs_amd_uci_decode_batch(proc->uci, uci_rows + ack_e, uci_stride, static_cast<uint32_t>(csi1_e), K_csi1,
                                  plan->pdu.modulation,
                                  out ? io->d_csi_part1 : proc->uci_payload.as<uint8_t>() + K_ack,
                                  out ? io->csi_part1_stride : pay_stride, proc->uci_status.as<int32_t>() + 1,
                                  4 * sizeof(int32_t), nof_grids, stream);
  }
  // CSI part 2 sized on the device (csi2_batch_device: no host round trip) whenever the plan's candidate sizes all
  // have a geometry and the UL-SCH can go through the slot decoder; otherwise the sizes come from one readback of the
  // decoded CSI part 1 below.  Grids without CSI part 2 keep the plan's geometry.
  if (rc == SRS_AMD_OK && plan->csi2) {
    const srs_amd_pusch_processor_plan::csi2_candidates* cand = nullptr;
    const bool dev2 = (!plan->has_sch || d_soft == nullptr || plan->dec_cfg.use_early_stop) &&
                      (plan->has_sch || d_soft == nullptr) && plan_csi2_candidates(proc, plan, &cand) == SRS_AMD_OK &&
                      !cand->n2.empty() && (plan->dec_cfg.new_data || d_soft != nullptr);
    if (dev2) {
      const bool     out1 = io != nullptr && io->d_csi_part1 != nullptr;
      const uint8_t* p1   = out1 ? io->d_csi_part1 : proc->uci_payload.as<uint8_t>() + K_ack;
      const uint64_t p1s  = out1 ? io->csi_part1_stride : pay_stride;
      const bool     out2 = io != nullptr && io->d_csi_part2 != nullptr;
      if (out2 && io->csi_part2_stride < plan->max_csi2) {
        return fail(SRS_AMD_EINVAL, "CSI part 2 payload stride too small (%u bits)", plan->max_csi2);
      }
      rc = csi2_batch_device(proc, plan, cand, nof_grids, dem_rows, cw_stride, llrs, llr_stride, uci_rows, uci_stride,
                             ack_e, csi2_stride, p1, p1s,
                             out2 ? io->d_csi_part2 : proc->uci_payload.as<uint8_t>() + K_ack + K_csi1,
                             out2 ? io->csi_part2_stride : pay_stride, d_tbs, tb_stride, d_soft, cb_iters, s);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
      pusch_result_args a{};
      a.dec_results = proc->dec_results.as<srs_amd_pusch_decoder_result>();
      a.stats       = st;
      a.results     = d_results;
      a.nof_grids   = nof_grids;
      a.nof_ports   = P;
      a.uci_status  = proc->uci_status.as<int32_t>();
      a.uci_mask    = (K_ack != 0 ? 1 : 0) | (K_csi1 != 0 ? 2 : 0) | 4;
      e                     = launch_pusch_result(a, s);
      const hipError_t done = scope.close();
      e                     = e != hipSuccess ? e : done;
      return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pusch_result_kernel launch");
    }
  }
  std::vector<uint32_t> n2(nof_grids, 0);
  std::vector<int32_t>  st1; // statuses [grid][4] read back with CSI part 1
  if (rc == SRS_AMD_OK && plan->csi2) {
    const bool     out1 = io != nullptr && io->d_csi_part1 != nullptr;
    const uint8_t* p1   = out1 ? io->d_csi_part1 : proc->uci_payload.as<uint8_t>() + K_ack;
    const uint64_t p1s  = out1 ? io->csi_part1_stride : pay_stride;
    st1.assign(static_cast<size_t>(nof_grids) * 4, 0);
    std::vector<uint8_t> part1(static_cast<size_t>(nof_grids) * K_csi1);
    e = hipMemcpyAsync(st1.data(), proc->uci_status.ptr, st1.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) {
      e = hipMemcpy2DAsync(part1.data(), K_csi1, p1, p1s, K_csi1, nof_grids, hipMemcpyDeviceToHost, s);
    }
    if (e == hipSuccess) {
      e = hipStreamSynchronize(s);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "CSI part 1 readback");
    }
    for (uint32_t g = 0; g < nof_grids && rc == SRS_AMD_OK; ++g) {
      if (st1[4 * g + 1] == SRS_AMD_UCI_VALID) { // on_csi_part1 feeds back only a valid CSI part 1
        const int32_t v = srs_amd_uci_part2_get_size(part1.data() + static_cast<size_t>(g) * K_csi1, K_csi1,
                                                      &plan->pdu.csi_part2_size);
        rc              = v < 0 ? fail(SRS_AMD_EINVAL, "CSI part 2 size description does not fit CSI part 1") : rc;
        n2[g]           = v < 0 ? 0u : static_cast<uint32_t>(v);
      }
    }
  }
  const bool any2 = std::any_of(n2.begin(), n2.end(), [](uint32_t v) { return v != 0; });
  // UCI only: no UL-SCH decoding (pusch_processor_impl.cpp:305: has_sch_data), an empty decoder result
  if (rc == SRS_AMD_OK && !plan->has_sch) {
    e  = hipMemsetAsync(proc->dec_results.ptr, 0, sizeof(srs_amd_pusch_decoder_result) * nof_grids, s);
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUSCH processor UCI-only result");
  }
  if (rc == SRS_AMD_OK && !any2 && plan->has_sch) {
    rc = srs_amd_pusch_decode_batch(proc->dec, &plan->sch, &plan->dec_cfg, d_tbs, tb_stride,
                                    proc->dec_results.as<srs_amd_pusch_decoder_result>(), llrs, llr_stride, d_soft,
                                    cb_iters, nof_grids, stream);
  }
  // grid by grid when some CSI part 2 is present: each size has its own UL-SCH geometry; the sizes go into the
  // statuses' fourth column: the statuses read back above (HARQ-ACK, CSI part 1) with the sizes, uploaded whole
  // by the copy kernel (upload_pinned: no small SDMA transfer)
  if (rc == SRS_AMD_OK && any2) {
    e = proc->stage2.acquire(4 * sizeof(int32_t) * nof_grids);
    if (e == hipSuccess) {
      for (uint32_t g = 0; g < nof_grids; ++g) {
        int32_t* row = proc->stage2.at<int32_t>(4 * sizeof(int32_t) * g);
        for (uint32_t k = 0; k < 4; ++k) {
          row[k] = st1[4 * g + k];
        }
        row[3] = static_cast<int32_t>(n2[g]);
      }
      e = proc->stage2.upload(proc->uci_status.ptr, 4 * sizeof(int32_t) * nof_grids, s);
    }
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "CSI part 2 size upload");
  }
  for (uint32_t g = 0; g < nof_grids && rc == SRS_AMD_OK && any2; ++g) {
    const srs_amd_sch_plan* sch = &plan->sch;
    int8_t*                 row = llrs + static_cast<uint64_t>(g) * llr_stride;
    if (n2[g] != 0) {
      const srs_amd_pusch_processor_plan::part2_geometry* geo = nullptr;
      rc = plan_part2(proc, plan, n2[g], &geo);
      if (rc != SRS_AMD_OK) {
        break;
      }
      sch                = &geo->sch;
      int8_t*        c2  = uci_rows + static_cast<uint64_t>(nof_grids) * uci_stride + g * csi2_stride;
      const uint64_t e2  = geo->info.nof_csi_part2_bits;
      int8_t*        u1  = uci_rows + static_cast<uint64_t>(g) * uci_stride;
      rc = srs_amd_ulsch_demultiplex_csi2_batch(proc->demux, geo->demux, dem_rows + g * cw_stride, cw_stride, row,
                                                llr_stride, u1, uci_stride, u1 + ack_e, uci_stride, c2, csi2_stride, 1,
                                                stream);
      const bool out2 = io != nullptr && io->d_csi_part2 != nullptr;
      if (rc == SRS_AMD_OK && out2 && io->csi_part2_stride < n2[g]) {
        rc = fail(SRS_AMD_EINVAL, "CSI part 2 payload stride too small (%u bits)", n2[g]);
      }
      if (rc == SRS_AMD_OK) {
        rc = srs_amd_uci_decode_batch(proc->uci, c2, csi2_stride, static_cast<uint32_t>(e2), n2[g],
                                      plan->pdu.modulation,
                                      out2 ? io->d_csi_part2 + static_cast<uint64_t>(g) * io->csi_part2_stride
                                           : proc->uci_payload.as<uint8_t>() + g * pay_stride + K_ack + K_csi1,
                                      pay_stride, proc->uci_status.as<int32_t>() + 4 * g + 2, 4 * sizeof(int32_t), 1,
                                      stream);
      }
    }
    if (rc == SRS_AMD_OK && plan->has_sch) {
      rc = srs_amd_pusch_decode_batch(proc->dec, sch, &plan->dec_cfg, d_tbs + static_cast<uint64_t>(g) * tb_stride,
                                      tb_stride, proc->dec_results.as<srs_amd_pusch_decoder_result>() + g, row,
                                      llr_stride, d_soft ? d_soft + g * plan->soft_bytes : nullptr,
                                      cb_iters != nullptr ? cb_iters + static_cast<size_t>(g) * C : nullptr, 1,
                                      stream);
    }
  }
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  pusch_result_args a{};
  a.dec_results = proc->dec_results.as<srs_amd_pusch_decoder_result>();
  a.stats       = st;
  a.results     = d_results;
  a.nof_grids   = nof_grids;
  a.nof_ports   = P;
  if (uci) {
    a.uci_status = proc->uci_status.as<int32_t>();
    a.uci_mask   = (K_ack != 0 ? 1 : 0) | (K_csi1 != 0 ? 2 : 0) | (plan->csi2 ? 4 : 0);
  }
  e                     = launch_pusch_result(a, s);
  const hipError_t done = scope.close();
  e                     = e != hipSuccess ? e : done;
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pusch_result_kernel launch");
}

} // namespace

extern "C" {

int srs_amd_pusch_process_batch(srs_amd_pusch_processor*            proc,
                                const srs_amd_pusch_processor_plan* plan,
                                const uint32_t*                     d_grids,
                                uint64_t                            grid_stride,
                                uint32_t                            nof_grids,
                                uint8_t*                            d_tbs,
                                uint32_t                            tb_stride,
                                srs_amd_pusch_processor_result*     d_results,
                                int8_t*                             d_soft,
                                const srs_amd_pusch_intermediates*  io,
                                void*                               stream)
{
  if (proc == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  std::lock_guard<std::mutex> lock(proc->mtx);
  return process_batch_locked(proc, plan, d_grids, grid_stride, nof_grids, d_tbs, tb_stride, d_results, d_soft, io,
                              stream);
}


int srs_amd_pusch_process_slot_ex(srs_amd_pusch_processor*        proc,
                                  const srs_amd_pusch_slot_pdu*   pdus,
                                  uint32_t                        nof_pdus,
                                  const uint32_t*                 d_grids,
                                  uint64_t                        grid_stride,
                                  uint32_t                        nof_grids,
                                  uint8_t*                        d_tbs,
                                  srs_amd_pusch_processor_result* d_results,
                                  const srs_amd_pusch_slot_io*    io,
                                  void*                           stream)
{
  if (proc == nullptr || (nof_pdus != 0 && pdus == nullptr)) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_pdus == 0) {
    return SRS_AMD_OK;
  }
  if (d_tbs == nullptr || d_results == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  constexpr uint32_t STATS_STRIDE = 4; // port measurements per PDU (at most four receive ports)
  const uint32_t     nof_subc     = pdus[0].plan != nullptr ? pdus[0].plan->nof_subc : 0;
  int32_t* const     cb_iters     = io != nullptr ? io->d_cb_iterations : nullptr;
  uint8_t* const     d_uci        = io != nullptr ? io->d_uci : nullptr;
  srs_amd_chest_port_stats* const out_stats = io != nullptr ? io->d_port_stats : nullptr;
  // the fused group (new data, no UCI, CP-OFDM, no soft buffer to keep) and the PDUs of the batch chain
  std::vector<uint32_t> fused, others;
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const srs_amd_pusch_processor_plan* pl = pdus[i].plan;
    if (pl == nullptr) {
      return fail(SRS_AMD_EINVAL, "null plan");
    }
    const uint32_t P = pl->pdu.nof_rx_ports;
    if (pl->nof_subc != nof_subc) {
      return fail(SRS_AMD_EINVAL, "PDU %u: plans of different grid sizes", i);
    }
    if (pdus[i].d_grid == nullptr &&
        (d_grids == nullptr || pdus[i].grid >= nof_grids || (nof_grids > 1 && grid_stride < 14ull * nof_subc * P))) {
      return fail(SRS_AMD_EINVAL, "PDU %u: grid index or grid stride out of range", i);
    }
    if (pl->has_sch && !pl->dec_cfg.new_data && pdus[i].d_soft == nullptr) {
      return fail(SRS_AMD_EINVAL, "PDU %u: a HARQ retransmission needs its soft buffer (d_soft)", i);
    }
    if (pdus[i].has_slot && (pdus[i].numerology > 4 || pdus[i].slot_index >= (10u << pdus[i].numerology))) {
      return fail(SRS_AMD_EINVAL, "PDU %u: invalid slot %u of numerology %u", i, pdus[i].slot_index,
                  pdus[i].numerology);
    }
    // HARQ-ACK / CSI part 1 / CSI part 2 on the UL-SCH, UCI-only and DFT-s-OFDM PDUs join the group (slot-form
    // demultiplexer and UCI decoders, CSI part 2 sized on the device; the equalizer's symbols through the transform
    // deprecoder); HARQ processes with a soft buffer (new data or retransmission) join it too (the slot decoder's
    // HARQ rows, early-stop decoding)
    bool f = proc->fuse && pl->fusable && P <= STATS_STRIDE &&
             (!pl->has_sch || (pdus[i].d_soft == nullptr ? pl->dec_cfg.new_data != 0 : pl->dec_cfg.use_early_stop != 0));
    if (f && pl->csi2) {
      // every CSI part 2 size of the description must have a geometry (a UCI-only PDU with CSI part 2 has none: its
      // CSI part 1 takes every RE, ulsch_info.cpp:96-123); otherwise the PDU keeps the batch chain, which fails
      // only when a decoded CSI part 1 selects such a size
      const srs_amd_pusch_processor_plan::csi2_candidates* c = nullptr;
      f = plan_csi2_candidates(proc, pl, &c) == SRS_AMD_OK;
    }
    (f ? fused : others).push_back(i);
  }
  // PDUs with a codeword first: the slot decoder's UEs are then the first nsch PDUs of the group (results are
  // scattered back to the PDU indices by the result kernel)
  std::stable_partition(fused.begin(), fused.end(), [&](uint32_t i) { return pdus[i].plan->has_sch; });
  uint32_t nsch = 0;
  for (uint32_t i : fused) {
    nsch += pdus[i].plan->has_sch ? 1u : 0u;
  }
  // each PDU's estimator configuration: its plan's, moved to the PDU's own slot when it carries one (the DM-RS
  // sequences are the only per-slot quantity; PDUs of several slots may share a plan within one call)
  std::vector<srs_amd_pusch_chest_config> ccfg(nof_pdus);
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    ccfg[i] = pdus[i].plan->chest_cfg;
    if (pdus[i].has_slot) {
      ccfg[i].numerology = pdus[i].numerology;
      ccfg[i].slot_index = pdus[i].slot_index;
    }
  }
  // each PDU's received grid: its own device grid, or its slot of d_grids
  auto grid_of = [&](const srs_amd_pusch_slot_pdu& u) {
    return u.d_grid != nullptr ? u.d_grid : d_grids + u.grid * grid_stride;
  };
  auto                        s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(proc->mtx);
  // 1. PDUs outside the fused group: each through its plan's batch chain on this stream
  for (uint32_t i : others) {
    const srs_amd_pusch_processor_plan* pl = pdus[i].plan;
    srs_amd_pusch_intermediates         x{};
    x.d_cb_iterations = cb_iters != nullptr ? cb_iters + pdus[i].cb_offset : nullptr;
    x.d_port_stats    = out_stats != nullptr ? out_stats + static_cast<size_t>(STATS_STRIDE) * i : nullptr;
    if (d_uci != nullptr && pl->uci) {
      uint8_t* row       = d_uci + pdus[i].uci_offset;
      x.d_harq_ack       = pl->pdu.nof_harq_ack != 0 ? row : nullptr;
      x.harq_ack_stride  = std::max<uint32_t>(pl->pdu.nof_harq_ack, 1);
      x.d_csi_part1      = pl->pdu.nof_csi_part1 != 0 ? row + pl->pdu.nof_harq_ack : nullptr;
      x.csi_part1_stride = std::max<uint32_t>(pl->pdu.nof_csi_part1, 1);
      x.d_csi_part2      = pl->csi2 ? row + pl->pdu.nof_harq_ack + pl->pdu.nof_csi_part1 : nullptr;
      x.csi_part2_stride = std::max<uint32_t>(pl->max_csi2, 1);
    }
    const int rc = process_batch_locked(proc, pl, grid_of(pdus[i]), grid_stride, 1,
                                        d_tbs + pdus[i].tb_offset, std::max<uint32_t>(pl->pdu.tbs / 8, 1),
                                        d_results + i, pdus[i].d_soft, &x, stream, &ccfg[i]);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  const uint32_t n = static_cast<uint32_t>(fused.size());
  if (n == 0) {
    return SRS_AMD_OK;
  }
  // 2. the fused group
  // UL-SCH LLR rows (a UCI-only PDU's row takes the demultiplexer's discarded UL-SCH stream)
  std::vector<size_t> llr_off(n);
  size_t              llr_bytes = 0;
  for (uint32_t k = 0; k != n; ++k) {
    const srs_amd_pusch_processor_plan* pl = pdus[fused[k]].plan;
    llr_off[k]                             = llr_bytes;
    llr_bytes += align_up(std::max<uint32_t>(pl->has_sch ? pl->sch.cw_length : pl->dummy_sch_bits, 1), 64);
  }
  const size_t     o_ids  = align_up(sizeof(uint32_t) * n, 16);
  // UCI PDUs of the group: the demodulator's codeword rows, the demultiplexed HARQ-ACK / CSI part 1 (/ CSI part 2)
  // rows, payload rows (the caller's d_uci, or scratch) and statuses [k][4]
  std::vector<uint32_t> ucis;
  std::vector<size_t>   cw_off(n), uci_off(n), c2_off(n), pay_off(n);
  std::vector<const srs_amd_pusch_processor_plan::csi2_candidates*> cands(n, nullptr);
  size_t                cw_bytes = 0, uci_bytes = 0, pay_bytes = 0;
  for (uint32_t k = 0; k != n; ++k) {
    const srs_amd_pusch_processor_plan* pl = pdus[fused[k]].plan;
    if (!pl->uci) {
      continue;
    }
    if (pl->csi2) {
      const int rc = plan_csi2_candidates(proc, pl, &cands[k]);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
      cands[k] = cands[k]->n2.empty() ? nullptr : cands[k];
    }
    ucis.push_back(k);
    cw_off[k]  = cw_bytes;
    uci_off[k] = uci_bytes;
    pay_off[k] = pay_bytes;
    cw_bytes += align_up(pl->cw_bits, 64);
    uci_bytes += align_up(pl->info.nof_harq_ack_bits + pl->info.nof_csi_part1_bits, 64);
    if (cands[k] != nullptr) {
      c2_off[k] = uci_bytes;
      uci_bytes += align_up(cands[k]->max_e2, 64);
    }
    pay_bytes += align_up(pl->pdu.nof_harq_ack + pl->pdu.nof_csi_part1 + pl->max_csi2, 64);
  }
  const uint32_t nu = static_cast<uint32_t>(ucis.size());
  hipError_t       e      = hipSetDevice(proc->device);
  if (e == hipSuccess && nu != 0) {
    e = proc->csi2_sel.ensure(sizeof(int32_t) * n);
  }
  if (e == hipSuccess && nu != 0) {
    e = proc->cw_llrs.ensure(cw_bytes);
  }
  if (e == hipSuccess && nu != 0) {
    e = proc->uci_llrs.ensure(uci_bytes);
  }
  if (e == hipSuccess && nu != 0) {
    e = proc->uci_payload.ensure(pay_bytes);
  }
  if (e == hipSuccess && nu != 0) {
    e = proc->uci_status.ensure(static_cast<size_t>(n) * 4 * sizeof(int32_t));
  }
  if (e == hipSuccess) {
    e = proc->stats.ensure(static_cast<size_t>(n) * STATS_STRIDE * sizeof(srs_amd_chest_port_stats));
  }
  if (e == hipSuccess) {
    e = proc->llrs.ensure(std::max<size_t>(llr_bytes, 64));
  }
  if (e == hipSuccess) {
    e = proc->dec_results.ensure(static_cast<size_t>(n) * sizeof(srs_amd_pusch_decoder_result));
  }
  if (e == hipSuccess) {
    e = proc->slot_ports.ensure(o_ids + sizeof(uint32_t) * n);
  }
  if (e == hipSuccess) {
    e = proc->stage.acquire(o_ids + sizeof(uint32_t) * n);
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH processor slot scratch");
  }
  call_scope scope(proc->order, &proc->fan, s);
  // port measurements of fused PDU k at st + k * STATS_STRIDE, or straight in the caller's buffer at its PDU index
  auto*      st   = out_stats != nullptr ? out_stats : proc->stats.as<srs_amd_chest_port_stats>();
  auto*      llrs = proc->llrs.as<int8_t>();
  auto       stats_of = [&](uint32_t k) { return st + static_cast<size_t>(out_stats ? fused[k] : k) * STATS_STRIDE; };
  // 2a. channel estimation of every fused PDU (one launch sequence)
  std::vector<chest_slot_item> citems(n);
  for (uint32_t k = 0; k != n; ++k) {
    const srs_amd_pusch_slot_pdu& u = pdus[fused[k]];
    citems[k] = chest_slot_item{&ccfg[fused[k]], grid_of(u), u.plan->pdu.nof_rx_ports,
                                stats_of(k)};
  }
  std::vector<chest_args> views(n);
  int rc = chest_estimate_slot_unexpanded(proc->chest, citems.data(), n, nof_subc, stream, views.data());
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // 2b. equalization, demapping and descrambling into each PDU's codeword LLR row (one launch per kernel kind)
  // (a UCI PDU's whole codeword goes to its codeword row, for the demultiplexer)
  std::vector<demod_slot_item> ditems(n);
  int8_t* const                cw_rows = proc->cw_llrs.as<int8_t>();
  for (uint32_t k = 0; k != n; ++k) {
    const srs_amd_pusch_processor_plan* pl = pdus[fused[k]].plan;
    ditems[k] = demod_slot_item{pl->demod_plan, &views[k], citems[k].d_grid, citems[k].d_stats,
                                pl->uci ? cw_rows + cw_off[k] : llrs + llr_off[k]};
  }
  rc = pusch_demodulate_slot_fused(proc->demod, ditems.data(), n, stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // 2b'. UCI PDUs: the demultiplexer of every codeword (UL-SCH LLRs into the PDU's decoder row) in one launch, then
  //      the HARQ-ACK and CSI part 1 decoders of every PDU (one short-block, one polar and one CRC launch)
  if (nu != 0) {
    rc = fused_uci(proc, pdus, fused, ucis, cw_off, uci_off, c2_off, pay_off, cands, llrs, llr_off, d_uci, s);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  // 2c. UL-SCH decoding of every transport block of the group (srs_amd_pusch_decode_slot): the first nsch PDUs; a
  //     UCI-only PDU's decoder result is empty (pusch_processor_impl.cpp:305); a CSI part 2 PDU's rows take the
  //     geometry of the size selected in 2b' (row patches)
  std::vector<srs_amd_pusch_ue> ues(nsch);
  std::vector<uint32_t>         cb_off(nsch);
  std::vector<slot_harq>        harq(nsch);
  std::vector<slot_ue_patch>    patches;
  bool                          any_harq = false;
  for (uint32_t k = 0; k != nsch; ++k) {
    const srs_amd_pusch_slot_pdu& u = pdus[fused[k]];
    ues[k]    = srs_amd_pusch_ue{u.plan->sch, llr_off[k], u.tb_offset};
    cb_off[k] = u.cb_offset;
    harq[k]   = slot_harq{u.d_soft, u.plan->dec_cfg.new_data, u.soft_on_failure != 0 ? 1 : 0};
    any_harq |= u.d_soft != nullptr;
    if (cands[k] != nullptr) {
      const uint32_t NC = static_cast<uint32_t>(cands[k]->n2.size()), C = u.plan->sch.nof_segments;
      const auto*    t  = cands[k]->d.as<uint32_t>();
      patches.push_back(slot_ue_patch{k, proc->csi2_sel.as<int32_t>() + k, t + NC, t + NC + NC * C});
    }
  }
  if (nsch < n) {
    e = hipMemsetAsync(proc->dec_results.as<srs_amd_pusch_decoder_result>() + nsch, 0,
                       sizeof(srs_amd_pusch_decoder_result) * (n - nsch), s);
    if (e != hipSuccess) {
      return hip_fail(e, "PUSCH slot UCI-only results");
    }
  }
  if (nsch != 0) {
    rc = pusch_decode_slot_ex(proc->dec, &pdus[fused[0]].plan->dec_cfg, ues.data(), nsch, llrs, d_tbs,
                              proc->dec_results.as<srs_amd_pusch_decoder_result>(),
                              cb_iters != nullptr ? cb_off.data() : nullptr, cb_iters, s,
                              any_harq ? harq.data() : nullptr, patches.data(), static_cast<uint32_t>(patches.size()));
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  // the UCI decoders' helper stream rejoins (statuses read by the result kernel)
  e = proc->fan.end(s);
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH slot UCI stream join");
  }
  // 2d. per-PDU results (decoder result + CSI from the PDU's own port measurements)
  for (uint32_t k = 0; k != n; ++k) {
    *proc->stage.at<uint32_t>(sizeof(uint32_t) * k)         = pdus[fused[k]].plan->pdu.nof_rx_ports;
    *proc->stage.at<uint32_t>(o_ids + sizeof(uint32_t) * k) = fused[k];
  }
  e = proc->stage.upload(proc->slot_ports.ptr, o_ids + sizeof(uint32_t) * n, s);
  if (e == hipSuccess) {
    pusch_result_args a{};
    a.dec_results  = proc->dec_results.as<srs_amd_pusch_decoder_result>();
    a.stats        = st;
    a.results      = d_results;
    a.nof_grids    = n;
    a.nof_ports    = 0;
    a.port_counts  = proc->slot_ports.as<uint32_t>();
    a.stats_stride = STATS_STRIDE;
    a.stats_by_id  = out_stats != nullptr;
    a.result_ids   = reinterpret_cast<const uint32_t*>(proc->slot_ports.as<uint8_t>() + o_ids);
    if (nu != 0) { // the field masks follow the UCI descriptors (fused_uci)
      a.uci_status = proc->uci_status.as<int32_t>();
      a.uci_masks  = reinterpret_cast<const uint32_t*>(proc->uci_items.as<uint8_t>() + proc->uci_masks_offset);
    }
    e              = launch_pusch_result(a, s);
  }
  const hipError_t done = scope.close();
  e                     = e != hipSuccess ? e : done;
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pusch_result_kernel slot launch");
}

int srs_amd_pusch_process_slot(srs_amd_pusch_processor*        proc,
                               const srs_amd_pusch_slot_pdu*   pdus,
                               uint32_t                        nof_pdus,
                               const uint32_t*                 d_grids,
                               uint64_t                        grid_stride,
                               uint32_t                        nof_grids,
                               uint8_t*                        d_tbs,
                               srs_amd_pusch_processor_result* d_results,
                               void*                           stream)
{
  return srs_amd_pusch_process_slot_ex(proc, pdus, nof_pdus, d_grids, grid_stride, nof_grids, d_tbs, d_results,
                                       nullptr, stream);
}

int srs_amd_pusch_processor_plan_set_slot(srs_amd_pusch_processor_plan* plan, uint32_t numerology,
                                          uint32_t slot_index)
{
  if (plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null plan");
  }
  if (numerology > 4 || slot_index >= (10u << numerology)) {
    return fail(SRS_AMD_EINVAL, "invalid slot %u of numerology %u", slot_index, numerology);
  }
  plan->pdu.numerology       = numerology;
  plan->pdu.slot_index       = slot_index;
  plan->chest_cfg.numerology = numerology;
  plan->chest_cfg.slot_index = slot_index;
  return SRS_AMD_OK;
}

int srs_amd_pusch_processor_plan_info(const srs_amd_pusch_processor_plan* plan, uint32_t* nof_codeblocks,
                                      uint32_t* max_csi_part2, uint64_t* soft_buffer_bytes)
{
  if (plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null plan");
  }
  if (nof_codeblocks != nullptr) {
    *nof_codeblocks = plan->sch.nof_segments;
  }
  if (max_csi_part2 != nullptr) {
    *max_csi_part2 = plan->csi2 ? plan->max_csi2 : 0;
  }
  if (soft_buffer_bytes != nullptr) {
    *soft_buffer_bytes = plan->soft_bytes;
  }
  return SRS_AMD_OK;
}

int srs_amd_pusch_process(srs_amd_pusch_processor*            proc,
                          const srs_amd_pusch_processor_plan* plan,
                          const uint32_t*                     grid,
                          uint8_t*                            tb,
                          srs_amd_pusch_processor_result*     result,
                          int8_t*                             soft_buffer)
{
  if (proc == nullptr || plan == nullptr || grid == nullptr || tb == nullptr || result == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t grid_bytes = plan->pdu.nof_rx_ports * 14ull * plan->nof_subc * 4;
  const size_t tb_bytes   = plan->pdu.tbs / 8;
  const size_t soft_bytes = soft_buffer ? plan->soft_bytes : 0;
  const size_t off_tb     = align_up(grid_bytes, 256);
  const size_t off_res    = off_tb + align_up(tb_bytes, 256);
  const size_t off_soft   = off_res + align_up(sizeof(srs_amd_pusch_processor_result), 256);
  hipError_t   e;
  {
    std::lock_guard<std::mutex> lock(proc->mtx);
    e = hipSetDevice(proc->device);
    if (e == hipSuccess) {
      e = proc->host_io.ensure(off_soft + soft_bytes);
    }
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH processor buffers");
  }
  auto* b = proc->host_io.as<uint8_t>();
  e       = hipMemcpyAsync(b, grid, grid_bytes, hipMemcpyHostToDevice, proc->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(b + off_tb, tb, tb_bytes, hipMemcpyHostToDevice, proc->stream); // untouched bytes keep
  }
  if (e == hipSuccess && soft_buffer) {
    e = hipMemcpyAsync(b + off_soft, soft_buffer, soft_bytes, hipMemcpyHostToDevice, proc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH processor upload");
  }
  int rc = srs_amd_pusch_process_batch(proc, plan, reinterpret_cast<const uint32_t*>(b), grid_bytes / 4, 1, b + off_tb,
                                       static_cast<uint32_t>(tb_bytes),
                                       reinterpret_cast<srs_amd_pusch_processor_result*>(b + off_res),
                                       soft_buffer ? reinterpret_cast<int8_t*>(b + off_soft) : nullptr, nullptr,
                                       proc->stream);
  if (rc != SRS_AMD_OK) {
    (void)hipStreamSynchronize(proc->stream);
    return rc;
  }
  e = hipMemcpyAsync(tb, b + off_tb, tb_bytes, hipMemcpyDeviceToHost, proc->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(result, b + off_res, sizeof(*result), hipMemcpyDeviceToHost, proc->stream);
  }
  if (e == hipSuccess && soft_buffer) {
    e = hipMemcpyAsync(soft_buffer, b + off_soft, soft_bytes, hipMemcpyDeviceToHost, proc->stream);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(proc->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUSCH processor download");
}

} // extern "C"
