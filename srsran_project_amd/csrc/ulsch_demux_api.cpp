// ulsch_demux_api.cpp -- C-ABI of the MI355X UL-SCH demultiplexer (include/srsran_amd/ulsch_demux.h): the host
// resolves the placement of ulsch_demultiplex_impl (ulsch_demultiplex_impl.cpp:285-472, one OFDM symbol at a
// time: reserved HARQ-ACK REs, HARQ-ACK > 2 bits, CSI part 1, CSI part 2, UL-SCH, HARQ-ACK <= 2 bits in the
// reserved REs, each taken every d-th RE of its candidate set) into per-RE tables once per plan; the device pass
// (ulsch_demux.hip) moves the LLRs.
#include "srsran_amd/ulsch_demux.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "gold_sequence.h"
#include "modulation_args.h"
#include "ulsch_demux_args.h"
#include <algorithm>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_ulsch_demux {
  int           device = 0;
  hipStream_t   stream = nullptr;
  uint32_t*     d_jump = nullptr;
  device_buffer host_io;
  std::mutex    mtx;
  ~srs_amd_ulsch_demux()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(d_jump);
  }
};

struct srs_amd_ulsch_demux_plan {
  int                        device = 0;
  srs_amd_ulsch_demux_config cfg{};
  demux_placement            pl;
  uint32_t*                  d_maps = nullptr; // sch_map then uci_map
  uint32_t*                  d_scr  = nullptr;
  ~srs_amd_ulsch_demux_plan()
  {
    (void)hipSetDevice(device);
    (void)hipFree(d_maps);
    (void)hipFree(d_scr);
  }
};

namespace {

using re_set = std::vector<char>;

uint32_t count(const re_set& s)
{
  return static_cast<uint32_t>(std::count(s.begin(), s.end(), 1));
}

// re_set_select (ulsch_demultiplex_impl.cpp:78-99): the first m elements of `set` taken every d-th.
re_set select(const re_set& set, uint32_t d, uint32_t m)
{
  re_set out(set.size(), 0);
  for (uint32_t i = 0, taken = 0, seen = 0; i < set.size() && taken != m; ++i) {
    if (!set[i]) {
      continue;
    }
    if (seen % d == 0) {
      out[i] = 1;
      ++taken;
    }
    ++seen;
  }
  return out;
}

uint32_t bits_per_symbol(int32_t qm)
{
  return qm < 2 ? 1u : static_cast<uint32_t>(qm);
}

} // namespace

int srs_amd::build_demux_placement(const srs_amd_ulsch_demux_config& c, demux_placement& out)
{
  const uint32_t mask = c.dmrs_symbol_mask & 0x3fffu;
  const uint32_t end  = c.start_symbol_index + c.nof_symbols;
  if (mask == 0 || end > 14 || c.nof_layers < 1 || c.nof_layers > 4 || c.nof_prb == 0 || c.nof_prb > 275 ||
      !(c.modulation == 0 || c.modulation == 1 || c.modulation == 2 || c.modulation == 4 || c.modulation == 6 ||
        c.modulation == 8) ||
      (c.dmrs_type != 1 && c.dmrs_type != 2) || c.nof_cdm_groups_without_data < 1 ||
      c.nof_cdm_groups_without_data > (c.dmrs_type == 1 ? 2u : 3u)) {
    return fail(SRS_AMD_EINVAL, "Invalid UL-SCH demultiplexer configuration.");
  }
  const uint32_t bpre = bits_per_symbol(c.modulation) * c.nof_layers;
  // l1: first OFDM symbol without DM-RS after the first DM-RS symbol; l1_csi: first symbol without DM-RS
  const uint32_t first_dmrs = static_cast<uint32_t>(__builtin_ctz(mask));
  uint32_t       l1 = first_dmrs, l1_csi = 0;
  while (l1 < 14 && ((mask >> l1) & 1u)) {
    ++l1;
  }
  while (l1_csi < 14 && ((mask >> l1_csi) & 1u)) {
    ++l1_csi;
  }
  const uint32_t nof_re_dmrs =
      (12 - c.nof_cdm_groups_without_data * (c.dmrs_type == 1 ? 6u : 4u)) * c.nof_prb; // get_..._nof_re_prb_dmrs
  out = demux_placement{};
  uint32_t m_rvd = 0, m_ack = 0, m_csi1 = 0, m_csi2 = 0;
  // CSI part 2 is configured (set_csi_part2) once CSI part 1 has been decoded, i.e. while demultiplexing the
  // OFDM symbol in which the CSI part 1 REs end (ulsch_demultiplex_impl.cpp:241-251): it starts in that symbol
  const bool     has_csi2  = c.nof_csi_part2_bits != 0 && c.nof_csi_part1_bits != 0;
  bool           csi2_live = false;
  for (uint32_t l = c.start_symbol_index; l < end; ++l) {
    const bool     dmrs = (mask >> l) & 1u;
    const uint32_t M    = dmrs ? nof_re_dmrs : c.nof_prb * 12;
    if (M == 0) {
      continue;
    }
    re_set   ulsch(M, 1), uci(M, dmrs ? 0 : 1), rvd(M, 0), ack(M, 0), csi1(M, 0);
    uint32_t M_uci = count(uci);
    // step 1: reserved HARQ-ACK REs
    const uint32_t rem_rvd = (c.nof_harq_ack_rvd - m_rvd) / bpre;
    if (l >= l1 && M_uci > 0 && rem_rvd > 0) {
      const uint32_t d = rem_rvd < M_uci ? M_uci / rem_rvd : 1;
      const uint32_t m = rem_rvd < M_uci ? rem_rvd : M_uci;
      rvd              = select(ulsch, d, m);
      m_rvd += m * bpre;
    }
    // step 2: HARQ-ACK of more than two bits
    const uint32_t rem_ack = (c.nof_enc_harq_ack_bits - m_ack) / bpre;
    if (l >= l1 && M_uci > 0 && c.nof_harq_ack_bits > 2 && rem_ack > 0) {
      const uint32_t d = rem_ack < M_uci ? M_uci / rem_ack : 1;
      const uint32_t m = rem_ack < M_uci ? rem_ack : M_uci;
      ack              = select(uci, d, m);
      for (uint32_t i = 0; i < M; ++i) {
        ulsch[i] &= !ack[i];
        uci[i] &= !ack[i];
      }
      M_uci = count(uci);
      m_ack += m * bpre;
    }
    // step 3: CSI part 1 outside the reserved REs
    const uint32_t rem_csi1 = (c.nof_enc_csi_part1_bits - m_csi1) / bpre;
    const uint32_t M_rvd    = count(rvd);
    if (l >= l1_csi && (M_uci - M_rvd) > 0 && rem_csi1 > 0) {
      const uint32_t avail = M_uci - M_rvd;
      const uint32_t d     = rem_csi1 < avail ? avail / rem_csi1 : 1;
      const uint32_t m     = rem_csi1 < avail ? rem_csi1 : avail;
      re_set         cand(M, 0);
      for (uint32_t i = 0; i < M; ++i) {
        cand[i] = !rvd[i] && uci[i];
      }
      csi1 = select(cand, d, m);
      for (uint32_t i = 0; i < M; ++i) {
        ulsch[i] &= !csi1[i];
        uci[i] &= !csi1[i];
      }
      m_csi1 += m * bpre;
    }
    // step 3bis: CSI part 2 (configure_csi_part2_current_ofdm_symbol, :450-472), from the symbol where CSI part 1
    // completes, every d-th of the remaining UCI REs (reserved REs included)
    csi2_live          = csi2_live || (has_csi2 && m_csi1 == c.nof_enc_csi_part1_bits);
    re_set         csi2(M, 0);
    const uint32_t M_uci2   = count(uci);
    const uint32_t rem_csi2 = csi2_live ? (c.nof_enc_csi_part2_bits - m_csi2) / bpre : 0u;
    if (l >= l1_csi && M_uci2 > 0 && rem_csi2 > 0) {
      const uint32_t d = rem_csi2 < M_uci2 ? M_uci2 / rem_csi2 : 1;
      const uint32_t m = rem_csi2 < M_uci2 ? rem_csi2 : M_uci2;
      csi2             = select(uci, d, m);
      for (uint32_t i = 0; i < M; ++i) {
        ulsch[i] &= !csi2[i];
        uci[i] &= !csi2[i];
      }
      m_csi2 += m * bpre;
    }
    // step 5: HARQ-ACK of one or two bits in the reserved REs (they stay UL-SCH REs, zeroed there)
    if (M_rvd > 0 && c.nof_harq_ack_bits <= 2 && rem_ack > 0) {
      const uint32_t d = rem_ack < M_rvd ? M_rvd / rem_ack : 1;
      const uint32_t m = rem_ack < M_rvd ? rem_ack : M_rvd;
      ack              = select(rvd, d, m);
      m_ack += m * bpre;
    }
    for (uint32_t i = 0; i < M; ++i) {
      uint32_t s = DMX_NONE, u = DMX_NONE;
      if (ack[i]) {
        u = (DMX_ACK << DMX_KIND_SHIFT) | out.nof_ack_re++;
      } else if (csi1[i]) {
        u = (DMX_CSI1 << DMX_KIND_SHIFT) | out.nof_csi1_re++;
      }
      if (ulsch[i]) {
        s = out.nof_sch_re++ | ((ack[i] && c.nof_harq_ack_bits <= 2) ? DMX_ZERO : 0u);
      }
      uint32_t v2 = DMX_NONE;
      if (csi2[i]) {
        v2 = out.nof_csi2_re++ | ((ack[i] && c.nof_harq_ack_bits <= 2) ? DMX_ZERO : 0u);
      }
      out.sch_map.push_back(s);
      out.uci_map.push_back(u);
      out.csi2_map.push_back(v2);
    }
  }
  out.nof_re = static_cast<uint32_t>(out.sch_map.size());
  if (out.nof_ack_re * bpre != (c.nof_harq_ack_bits ? c.nof_enc_harq_ack_bits : 0u) ||
      out.nof_csi1_re * bpre != (c.nof_csi_part1_bits ? c.nof_enc_csi_part1_bits : 0u) ||
      out.nof_csi2_re * bpre != (has_csi2 ? c.nof_enc_csi_part2_bits : 0u)) {
    return fail(SRS_AMD_EINVAL,
                "The UCI does not fit the allocation (HARQ-ACK %u of %u bits, CSI part 1 %u of %u, CSI part 2 %u of %u).",
                out.nof_ack_re * bpre, c.nof_enc_harq_ack_bits, out.nof_csi1_re * bpre, c.nof_enc_csi_part1_bits,
                out.nof_csi2_re * bpre, c.nof_enc_csi_part2_bits);
  }
  return SRS_AMD_OK;
}

extern "C" {

int srs_amd_ulsch_demux_create(srs_amd_ulsch_demux** demux, int device)
{
  if (demux == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *demux = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* d                 = new srs_amd_ulsch_demux();
  d->device               = device;
  std::vector<uint32_t> j = gold_jump_tables();
  hipError_t            e = hipMalloc(&d->d_jump, j.size() * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = hipMemcpy(d->d_jump, j.data(), j.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete d;
    return hip_fail(e, "UL-SCH demultiplexer tables");
  }
  *demux = d;
  return SRS_AMD_OK;
}

void srs_amd_ulsch_demux_destroy(srs_amd_ulsch_demux* demux)
{
  delete demux;
}

int srs_amd_ulsch_demux_plan_create(srs_amd_ulsch_demux*              demux,
                                    const srs_amd_ulsch_demux_config* cfg,
                                    srs_amd_ulsch_demux_plan**        plan,
                                    uint32_t*                         nof_codeword_bits,
                                    uint32_t*                         nof_sch_bits)
{
  if (demux == nullptr || cfg == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  *plan   = nullptr;
  auto* p = new srs_amd_ulsch_demux_plan();
  p->cfg  = *cfg;
  int rc  = build_demux_placement(*cfg, p->pl);
  if (rc != SRS_AMD_OK) {
    delete p;
    return rc;
  }
  p->device               = demux->device;
  const uint32_t bpre     = bits_per_symbol(cfg->modulation) * cfg->nof_layers;
  const uint32_t cw_bits  = p->pl.nof_re * bpre;
  const uint32_t nwords   = cw_bits / 32 + 2;
  hipError_t     e        = hipSetDevice(demux->device);
  if (e == hipSuccess) {
    e = hipMalloc(&p->d_maps, sizeof(uint32_t) * 3 * std::max(p->pl.nof_re, 1u));
  }
  if (e == hipSuccess && p->pl.nof_re != 0) {
    e = hipMemcpy(p->d_maps, p->pl.sch_map.data(), sizeof(uint32_t) * p->pl.nof_re, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess && p->pl.nof_re != 0) {
    e = hipMemcpy(p->d_maps + p->pl.nof_re, p->pl.uci_map.data(), sizeof(uint32_t) * p->pl.nof_re,
                  hipMemcpyHostToDevice);
  }
  if (e == hipSuccess && p->pl.nof_re != 0) {
    e = hipMemcpy(p->d_maps + 2 * p->pl.nof_re, p->pl.csi2_map.data(), sizeof(uint32_t) * p->pl.nof_re,
                  hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipMalloc(&p->d_scr, sizeof(uint32_t) * nwords);
  }
  if (e == hipSuccess) {
    e = launch_gold_words(demux->d_jump, cfg->c_init, p->d_scr, nwords, nullptr);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(nullptr);
  }
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "UL-SCH demultiplexer plan");
  }
  if (nof_codeword_bits != nullptr) {
    *nof_codeword_bits = cw_bits;
  }
  if (nof_sch_bits != nullptr) {
    *nof_sch_bits = p->pl.nof_sch_re * bpre;
  }
  *plan = p;
  return SRS_AMD_OK;
}

void srs_amd_ulsch_demux_plan_destroy(srs_amd_ulsch_demux_plan* plan)
{
  delete plan;
}

int srs_amd_ulsch_demultiplex_batch(srs_amd_ulsch_demux*            demux,
                                    const srs_amd_ulsch_demux_plan* plan,
                                    const int8_t*                   d_cws,
                                    uint64_t                        cw_stride,
                                    int8_t*                         d_sch,
                                    uint64_t                        sch_stride,
                                    int8_t*                         d_ack,
                                    uint64_t                        ack_stride,
                                    int8_t*                         d_csi1,
                                    uint64_t                        csi1_stride,
                                    uint32_t                        nof_cws,
                                    void*                           stream)
{
  return srs_amd_ulsch_demultiplex_csi2_batch(demux, plan, d_cws, cw_stride, d_sch, sch_stride, d_ack, ack_stride,
                                              d_csi1, csi1_stride, nullptr, 0, nof_cws, stream);
}

int srs_amd_ulsch_demultiplex_csi2_batch(srs_amd_ulsch_demux*            demux,
                                         const srs_amd_ulsch_demux_plan* plan,
                                         const int8_t*                   d_cws,
                                         uint64_t                        cw_stride,
                                         int8_t*                         d_sch,
                                         uint64_t                        sch_stride,
                                         int8_t*                         d_ack,
                                         uint64_t                        ack_stride,
                                         int8_t*                         d_csi1,
                                         uint64_t                        csi1_stride,
                                         int8_t*                         d_csi2,
                                         uint64_t                        csi2_stride,
                                         uint32_t                        nof_cws,
                                         void*                           stream)
{
  if (demux == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_cws == 0 || plan->pl.nof_re == 0) {
    return SRS_AMD_OK;
  }
  const uint32_t bpre = bits_per_symbol(plan->cfg.modulation) * plan->cfg.nof_layers;
  if (d_cws == nullptr || (plan->pl.nof_sch_re && d_sch == nullptr) || (plan->pl.nof_ack_re && d_ack == nullptr) ||
      (plan->pl.nof_csi1_re && d_csi1 == nullptr) || (plan->pl.nof_csi2_re && d_csi2 == nullptr)) {
    return fail(SRS_AMD_EINVAL, "null device buffer (a plan with CSI part 2 needs its rows)");
  }
  if (nof_cws > 1 && (cw_stride < uint64_t(plan->pl.nof_re) * bpre || sch_stride < uint64_t(plan->pl.nof_sch_re) * bpre ||
                      ack_stride < uint64_t(plan->pl.nof_ack_re) * bpre ||
                      csi1_stride < uint64_t(plan->pl.nof_csi1_re) * bpre ||
                      csi2_stride < uint64_t(plan->pl.nof_csi2_re) * bpre)) {
    return fail(SRS_AMD_EINVAL, "stride too small");
  }
  demux_args a{};
  a.cws         = d_cws;
  a.sch         = d_sch;
  a.ack         = d_ack;
  a.csi1        = d_csi1;
  a.sch_map     = plan->d_maps;
  a.uci_map     = plan->d_maps + plan->pl.nof_re;
  a.scr         = plan->d_scr;
  a.cw_stride   = cw_stride;
  a.sch_stride  = sch_stride;
  a.ack_stride  = ack_stride;
  a.csi1_stride = csi1_stride;
  a.nof_re      = plan->pl.nof_re;
  a.qm          = bits_per_symbol(plan->cfg.modulation);
  a.bpre        = bpre;
  a.ack_ph      = plan->cfg.nof_harq_ack_bits <= 2 ? plan->cfg.nof_harq_ack_bits : 0u;
  a.csi1_ph     = plan->cfg.nof_csi_part1_bits <= 2 ? plan->cfg.nof_csi_part1_bits : 0u;
  a.csi2_map    = plan->pl.nof_csi2_re != 0 ? plan->d_maps + 2 * plan->pl.nof_re : nullptr;
  a.csi2        = d_csi2;
  a.csi2_stride = csi2_stride;
  a.csi2_ph     = plan->cfg.nof_csi_part2_bits <= 2 ? plan->cfg.nof_csi_part2_bits : 0u;
  hipError_t e  = hipSetDevice(demux->device);
  if (e == hipSuccess) {
    e = launch_ulsch_demux(a, nof_cws, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ulsch_demux_kernel launch");
}

int srs_amd_ulsch_demultiplex(srs_amd_ulsch_demux*            demux,
                              const srs_amd_ulsch_demux_plan* plan,
                              const int8_t*                   codeword,
                              int8_t*                         sch,
                              int8_t*                         ack,
                              int8_t*                         csi1)
{
  return srs_amd_ulsch_demultiplex_csi2(demux, plan, codeword, sch, ack, csi1, nullptr);
}

int srs_amd_ulsch_demultiplex_csi2(srs_amd_ulsch_demux*            demux,
                                   const srs_amd_ulsch_demux_plan* plan,
                                   const int8_t*                   codeword,
                                   int8_t*                         sch,
                                   int8_t*                         ack,
                                   int8_t*                         csi1,
                                   int8_t*                         csi2)
{
  if (demux == nullptr || plan == nullptr || codeword == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const uint32_t bpre   = bits_per_symbol(plan->cfg.modulation) * plan->cfg.nof_layers;
  const size_t   n_cw   = size_t(plan->pl.nof_re) * bpre;
  const size_t   n_sch  = size_t(plan->pl.nof_sch_re) * bpre;
  const size_t   n_ack  = size_t(plan->pl.nof_ack_re) * bpre;
  const size_t   n_csi1 = size_t(plan->pl.nof_csi1_re) * bpre;
  const size_t   n_csi2 = size_t(plan->pl.nof_csi2_re) * bpre;
  if ((n_sch && sch == nullptr) || (n_ack && ack == nullptr) || (n_csi1 && csi1 == nullptr) ||
      (n_csi2 && csi2 == nullptr)) {
    return fail(SRS_AMD_EINVAL, "null output");
  }
  std::lock_guard<std::mutex> lock(demux->mtx);
  const size_t                o_sch = align_up(n_cw, 256), o_ack = o_sch + align_up(n_sch, 256),
                o_csi1 = o_ack + align_up(n_ack, 256), o_csi2 = o_csi1 + align_up(n_csi1, 256);
  hipError_t e         = hipSetDevice(demux->device);
  if (e == hipSuccess) {
    e = demux->host_io.ensure(o_csi2 + n_csi2 + 256);
  }
  auto* b = demux->host_io.as<int8_t>();
  if (e == hipSuccess && n_cw) {
    e = hipMemcpyAsync(b, codeword, n_cw, hipMemcpyHostToDevice, demux->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "UL-SCH demultiplexer upload");
  }
  int rc = srs_amd_ulsch_demultiplex_csi2_batch(demux, plan, b, n_cw, b + o_sch, n_sch, b + o_ack, n_ack, b + o_csi1,
                                                n_csi1, b + o_csi2, n_csi2, 1, demux->stream);
  if (rc != SRS_AMD_OK) {
    (void)hipStreamSynchronize(demux->stream);
    return rc;
  }
  if (n_sch) {
    e = hipMemcpyAsync(sch, b + o_sch, n_sch, hipMemcpyDeviceToHost, demux->stream);
  }
  if (e == hipSuccess && n_ack) {
    e = hipMemcpyAsync(ack, b + o_ack, n_ack, hipMemcpyDeviceToHost, demux->stream);
  }
  if (e == hipSuccess && n_csi1) {
    e = hipMemcpyAsync(csi1, b + o_csi1, n_csi1, hipMemcpyDeviceToHost, demux->stream);
  }
  if (e == hipSuccess && n_csi2) {
    e = hipMemcpyAsync(csi2, b + o_csi2, n_csi2, hipMemcpyDeviceToHost, demux->stream);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(demux->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "UL-SCH demultiplexer download");
}

} // extern "C"

demux_args srs_amd::make_demux_args(const srs_amd_ulsch_demux_plan* plan, const int8_t* cws, int8_t* sch, int8_t* ack,
                                    int8_t* csi1)
{
  demux_args a{};
  a.cws     = cws;
  a.sch     = sch;
  a.ack     = ack;
  a.csi1    = csi1;
  a.sch_map = plan->d_maps;
  a.uci_map = plan->d_maps + plan->pl.nof_re;
  a.scr     = plan->d_scr;
  a.nof_re  = plan->pl.nof_re;
  a.qm      = bits_per_symbol(plan->cfg.modulation);
  a.bpre    = a.qm * plan->cfg.nof_layers;
  a.ack_ph  = plan->cfg.nof_harq_ack_bits <= 2 ? plan->cfg.nof_harq_ack_bits : 0u;
  a.csi1_ph = plan->cfg.nof_csi_part1_bits <= 2 ? plan->cfg.nof_csi_part1_bits : 0u;
  return a;
}

demux_args srs_amd::make_demux_args_csi2(const srs_amd_ulsch_demux_plan* plan, const int8_t* cws, int8_t* sch,
                                         int8_t* ack, int8_t* csi1, int8_t* csi2)
{
  demux_args a = make_demux_args(plan, cws, sch, ack, csi1);
  a.csi2_map   = plan->pl.nof_csi2_re != 0 ? plan->d_maps + 2 * plan->pl.nof_re : nullptr;
  a.csi2       = csi2;
  a.csi2_ph    = plan->cfg.nof_csi_part2_bits <= 2 ? plan->cfg.nof_csi_part2_bits : 0u;
  return a;
}
