// pusch_demod_api.cpp -- C-ABI of the MI355X PUSCH demodulator
// (include/srsran_amd/pusch_demodulator.h).
//
// Host-side logic, once per plan: the data-RE table of pusch_demodulator_impl.cpp:218-262
// (rb_mask x all 12 REs, or x the REs outside the DM-RS CDM groups without data
// on DM-RS symbols, dmrs_mapping.h:76-91), the equalizer support check
// (channel_equalizer_generic_impl.cpp:240-270). Per batch: equalize (fused
// gather), soft demapping (the modulator object's kernel, modulation.h) and
// descrambling, three launches on the caller's stream.
#include "srsran_amd/pusch_demodulator.h"
#include "srsran_amd/transform_precoding.h"
#include "transform_precoding_args.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "gold_sequence.h"
#include "modulation_args.h"
#include "pusch_demod_args.h"
#include "srsran_amd/modulation.h"
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_pusch_demodulator {
  int                 device = 0;
  hipStream_t         stream = nullptr;
  uint32_t*           d_jump = nullptr;
  srs_amd_modulator*  demapper = nullptr;
  device_buffer       scratch;
  stream_order        order; // scratch reuse across the callers' streams
  srs_amd_transform_precoder* tp = nullptr; // transform precoding plans, created on first use
  device_buffer       host_io;
  device_buffer       slot_items; // slot form: per-PDU argument pairs
  pinned_stage        stage;
  std::mutex          mtx;
  ~srs_amd_pusch_demodulator()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    srs_amd_modulator_destroy(demapper);
    srs_amd_transform_precoder_destroy(tp);
    (void)hipFree(d_jump);
  }
};

struct srs_amd_pusch_demod_plan {
  int           device = 0;
  pusch_eq_args args{};
  uint32_t      nof_ports   = 0;
  uint32_t      nof_layers  = 0;
  bool          mmse        = false;
  uint32_t      nof_symbols = 0;
  uint32_t      span_subc   = 0;
  int32_t       qm          = 0;
  uint32_t      c_init      = 0;
  uint32_t      sym_counts[14] = {}; // demapper symbols (data REs x layers) per OFDM symbol
  uint32_t      tp_subc     = 0;     // transform precoding: subcarriers per data OFDM symbol (0: off)
  uint32_t*     d_table     = nullptr;
  uint32_t*     d_scr       = nullptr; // Gold words of c_init over the codeword (+1)
  ~srs_amd_pusch_demod_plan()
  {
    (void)hipSetDevice(device);
    (void)hipFree(d_table);
    (void)hipFree(d_scr);
  }
  uint32_t nof_llrs() const { return args.nof_re * nof_layers * (qm < 2 ? 1u : static_cast<uint32_t>(qm)); }
};

namespace {

bool crb_bit(const uint8_t* mask, uint32_t i)
{
  return i < SRS_AMD_MAX_RB && ((mask[i / 8] >> (i % 8)) & 1u);
}

uint32_t dmrs_prb_mask(uint32_t type, uint32_t nof_cdm_groups_without_data)
{
  uint32_t m = 0;
  for (uint32_t k = 0; k < 12; ++k) {
    const bool in = type == 1 ? (k % 2) < nof_cdm_groups_without_data : (k % 6) < 2 * nof_cdm_groups_without_data;
    m |= in ? (1u << k) : 0u;
  }
  return m;
}

// channel_equalizer_generic_impl.cpp:240-270 (one, two or four ports, no more layers than ports), extended
// by the L-layer solves of equalizer_device.h: ZF and MMSE for 1 to 4 layers (3 and 4 layers on four ports).
bool equalizer_supported(int algorithm, uint32_t ports, uint32_t layers)
{
  if ((ports != 1 && ports != 2 && ports != 4) || ports < layers || layers < 1 || layers > 4) {
    return false;
  }
  return algorithm == SRS_AMD_EQ_ZF || algorithm == SRS_AMD_EQ_MMSE;
}

} // namespace

// The equalizer + demapper pass of a batch; the channel coefficients come from an expanded estimate tensor
// (d_estimates) or, when fused != nullptr, are rebuilt per RE from the estimator's unexpanded output.
static int demodulate_impl(srs_amd_pusch_demodulator*      dem,
                           const srs_amd_pusch_demod_plan* plan,
                           const uint32_t*                 d_grids,
                           uint64_t                        grid_stride,
                           const uint32_t*                 d_estimates,
                           uint64_t                        est_stride,
                           const chest_args*               fused,
                           const srs_amd_chest_port_stats* d_stats,
                           int8_t*                         d_llrs,
                           uint64_t                        llr_stride,
                           uint32_t                        nof_grids,
                           void*                           stream)
{
  if (dem == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_grids == 0 || plan->args.nof_re == 0) {
    return SRS_AMD_OK;
  }
  if (d_grids == nullptr || (fused == nullptr && d_estimates == nullptr) || d_stats == nullptr || d_llrs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  const uint32_t nllr  = plan->nof_llrs();
  const uint64_t plane = 14ull * plan->args.nof_subc;
  if (nof_grids > 1 && (grid_stride < plan->nof_ports * plane ||
                        (fused == nullptr && est_stride < plan->nof_ports * plan->nof_layers * plane) ||
                        llr_stride < nllr)) {
    return fail(SRS_AMD_EINVAL, "grid, estimate or LLR stride too small");
  }
  if (fused != nullptr) {
    // the estimator's allocation must cover every data RE and describe the same ports, layers and symbols
    const chest_args& c = *fused;
    if (c.nof_ports != plan->nof_ports || c.L != plan->nof_layers || c.nsubc != plan->args.nof_subc ||
        c.first_symbol != plan->args.first_symbol || c.nof_symbols != plan->nof_symbols ||
        plan->args.first_subc < 12 * c.prb_lo || plan->args.first_subc + plan->span_subc > 12 * c.prb_lo + c.nof_re ||
        !pusch_equalize_fusable(plan->nof_ports, plan->nof_layers, plan->mmse, c.nof_lse)) {
      return fail(SRS_AMD_EINVAL, "channel estimator output does not match the demodulator plan");
    }
  }
  // the equalizer demaps and descrambles its own symbols: LLRs straight into the caller's rows, no scratch;
  // with transform precoding it writes equalized symbols to scratch for the deprecoder and the demapper
  hipError_t    e = hipSetDevice(dem->device);
  pusch_eq_args a = plan->args;
  auto          s = static_cast<hipStream_t>(stream);
  const bool    tp = plan->tp_subc != 0;
  if (tp) {
    const uint64_t n = static_cast<uint64_t>(nof_grids) * plan->args.nof_re; // one layer
    if (e == hipSuccess && dem->tp == nullptr) {
      int rc = srs_amd_transform_precoder_create(&dem->tp, dem->device);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
    }
    if (e == hipSuccess) {
      e = dem->scratch.ensure(n * (sizeof(float2) + sizeof(float)));
    }
    if (e == hipSuccess) {
      e = dem->order.begin(s);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "PUSCH demodulator transform-precoding scratch");
    }
    a.eq_out    = dem->scratch.as<float2>();
    a.nv_out    = reinterpret_cast<float*>(dem->scratch.as<float2>() + n);
    a.eq_stride = plan->args.nof_re;
  }
  a.grids         = d_grids;
  a.grid_stride   = grid_stride;
  a.estimates     = d_estimates;
  a.est_stride    = est_stride;
  a.stats         = d_stats;
  a.llrs          = d_llrs;
  a.llr_stride    = llr_stride;
  if (e == hipSuccess) {
    e = fused != nullptr ? launch_pusch_equalize_fused(a, *fused, plan->nof_ports, plan->nof_layers, plan->mmse,
                                                       plan->span_subc, nof_grids, s)
                         : launch_pusch_equalize(a, plan->nof_ports, plan->nof_layers, plan->mmse, plan->nof_symbols,
                                                 plan->span_subc, nof_grids, s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "pusch_equalize_kernel launch");
  }
  if (!tp) {
    return SRS_AMD_OK;
  }
  // transform deprecoding of every data OFDM symbol (rows of tp_subc symbols, pusch_demodulator_impl.cpp:344-351),
  // then demapping + descrambling per OFDM symbol
  const uint32_t rows = nof_grids * (plan->args.nof_re / plan->tp_subc);
  int rc = srs_amd_transform_deprecode_batch(dem->tp, reinterpret_cast<float*>(a.eq_out), plan->tp_subc, a.nv_out,
                                             plan->tp_subc, plan->tp_subc, rows, stream);
  if (rc == SRS_AMD_OK) {
    rc = demap_descramble_batch(dem->demapper, plan->qm, d_llrs, llr_stride, reinterpret_cast<const float*>(a.eq_out),
                                a.nv_out, plan->args.nof_re, plan->sym_counts, nof_grids, dem->d_jump, plan->c_init,
                                stream);
  }
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  e = dem->order.end(s);
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUSCH demodulator completion event");
}

void srs_amd::pusch_demod_plan_set_dc(::srs_amd_pusch_demod_plan* plan, uint32_t dc_subc)
{
  if (plan != nullptr) {
    plan->args.dc_subc = (plan->tp_subc == 0 && dc_subc < plan->args.nof_subc) ? dc_subc : ~0u;
  }
}

int srs_amd::pusch_demodulate_batch_fused(::srs_amd_pusch_demodulator*      dem,
                                          const ::srs_amd_pusch_demod_plan* plan,
                                          const uint32_t*                   d_grids,
                                          uint64_t                          grid_stride,
                                          const chest_args&                 chest_view,
                                          const srs_amd_chest_port_stats*   d_stats,
                                          int8_t*                           d_llrs,
                                          uint64_t                          llr_stride,
                                          uint32_t                          nof_grids,
                                          void*                             stream)
{
  return demodulate_impl(dem, plan, d_grids, grid_stride, nullptr, 0, &chest_view, d_stats, d_llrs, llr_stride,
                         nof_grids, stream);
}

int srs_amd::pusch_demodulate_slot_fused(::srs_amd_pusch_demodulator* dem,
                                         const demod_slot_item*       items,
                                         uint32_t                     nof_items,
                                         void*                        stream)
{
  if (dem == nullptr || (nof_items != 0 && items == nullptr)) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  // kernel groups (ports, layers, MMSE): item ids of each group, back to back
  struct group {
    uint32_t P, L;
    bool     mmse;
    uint32_t first, count, max_blocks;
  };
  std::vector<group>    groups;
  std::vector<uint32_t> order;
  std::vector<eq_item>  pairs(nof_items);
  for (uint32_t i = 0; i != nof_items; ++i) {
    const demod_slot_item& it = items[i];
    const auto*            pl = it.plan;
    if (pl == nullptr || it.chest_view == nullptr) {
      return fail(SRS_AMD_EINVAL, "null argument");
    }
    if (it.d_grid == nullptr || it.d_stats == nullptr || (pl->args.nof_re != 0 && it.d_llrs == nullptr)) {
      return fail(SRS_AMD_EINVAL, "null device buffer");
    }
    const chest_args& c = *it.chest_view;
    if (c.nof_ports != pl->nof_ports || c.L != pl->nof_layers || c.nsubc != pl->args.nof_subc ||
        c.first_symbol != pl->args.first_symbol || c.nof_symbols != pl->nof_symbols ||
        pl->args.first_subc < 12 * c.prb_lo || pl->args.first_subc + pl->span_subc > 12 * c.prb_lo + c.nof_re ||
        !pusch_equalize_fusable(pl->nof_ports, pl->nof_layers, pl->mmse, c.nof_lse)) {
      return fail(SRS_AMD_EINVAL, "channel estimator output does not match the demodulator plan");
    }
    pusch_eq_args a = pl->args;
    a.grids         = it.d_grid;
    a.grid_stride   = 0;
    a.estimates     = nullptr;
    a.est_stride    = 0;
    a.stats         = it.d_stats;
    a.llrs          = it.d_llrs;
    a.llr_stride    = 0;
    a.tiles_x       = (pl->span_subc + 255) / 256;
    a.nof_tiles     = a.tiles_x;
    pairs[i]        = eq_item{a, c};
  }
  // transform precoding (one layer): the equalizer writes its symbols and noise variances to scratch, then per PDU
  // the deprecoder and the demapper (pusch_demodulator_impl.cpp:344-351, as demodulate_impl)
  std::vector<size_t> tp_off(nof_items, 0);
  size_t              tp_res = 0;
  for (uint32_t i = 0; i != nof_items; ++i) {
    if (items[i].plan->tp_subc != 0) {
      tp_off[i] = tp_res;
      tp_res += items[i].plan->args.nof_re;
    }
  }
  for (uint32_t i = 0; i != nof_items; ++i) {
    const auto* pl = items[i].plan;
    if (pl->args.nof_re == 0 || pl->span_subc == 0) {
      continue; // nothing to equalize
    }
    bool seen = false;
    for (const group& g : groups) {
      seen |= g.P == pl->nof_ports && g.L == pl->nof_layers && g.mmse == pl->mmse;
    }
    if (seen) {
      continue;
    }
    group g{pl->nof_ports, pl->nof_layers, pl->mmse, static_cast<uint32_t>(order.size()), 0, 0};
    for (uint32_t k = i; k != nof_items; ++k) {
      const auto* q = items[k].plan;
      if (q->args.nof_re != 0 && q->span_subc != 0 && q->nof_ports == g.P && q->nof_layers == g.L &&
          q->mmse == g.mmse) {
        order.push_back(k);
        ++g.count;
        g.max_blocks = std::max(g.max_blocks, pusch_equalize_fused_blocks(pairs[k].c.nof_symbols, pairs[k].a.nof_tiles));
      }
    }
    groups.push_back(g);
  }
  if (groups.empty()) {
    return SRS_AMD_OK;
  }
  const size_t o_ids = align_up(sizeof(eq_item) * nof_items, 256);
  const size_t n_tp  = std::count_if(items, items + nof_items, [](const demod_slot_item& it) {
    return it.plan->tp_subc != 0 && it.plan->args.nof_re != 0;
  });
  const size_t o_tp  = align_up(o_ids + sizeof(uint32_t) * order.size(), 256);
  const size_t o_dm  = align_up(o_tp + sizeof(tp_args) * n_tp, 256);
  const size_t total = n_tp == 0 ? o_ids + sizeof(uint32_t) * order.size() : o_dm + sizeof(demap_item) * n_tp;
  auto         s     = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(dem->mtx);
  hipError_t                  e = hipSetDevice(dem->device);
  if (e == hipSuccess) {
    e = dem->slot_items.ensure(total);
  }
  if (e == hipSuccess && tp_res != 0) {
    e = dem->scratch.ensure(tp_res * (sizeof(float2) + sizeof(float)));
  }
  float2* const eq_out = dem->scratch.as<float2>();
  float* const  nv_out = reinterpret_cast<float*>(eq_out + tp_res);
  for (uint32_t i = 0; i != nof_items && e == hipSuccess; ++i) {
    if (items[i].plan->tp_subc != 0) {
      pairs[i].a.eq_out    = eq_out + tp_off[i];
      pairs[i].a.nv_out    = nv_out + tp_off[i];
      pairs[i].a.eq_stride = items[i].plan->args.nof_re;
    }
  }
  if (e == hipSuccess) {
    e = dem->stage.acquire(total);
  }
  if (e == hipSuccess) {
    e = dem->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH demodulator slot descriptors");
  }
  call_scope scope(dem->order, nullptr, s);
  std::memcpy(dem->stage.at<eq_item>(0), pairs.data(), sizeof(eq_item) * nof_items);
  std::memcpy(dem->stage.at<uint32_t>(o_ids), order.data(), sizeof(uint32_t) * order.size());
  // transform-precoded PDUs: deprecoder rows and demapper of each (one launch each for all of them)
  uint32_t tp_rows = 0, tp_syms = 0;
  size_t   tp_lds  = 0;
  for (uint32_t i = 0, k = 0; i != nof_items; ++i) {
    const auto* pl = items[i].plan;
    if (pl->tp_subc == 0 || pl->args.nof_re == 0) {
      continue;
    }
    float2*  y   = eq_out + tp_off[i];
    float*   v   = nv_out + tp_off[i];
    size_t   lds = 0;
    tp_args  ta;
    int      rc  = make_tp_args(y, pl->tp_subc, v, pl->tp_subc, pl->tp_subc, pl->args.nof_re / pl->tp_subc, ta, lds);
    demap_item di;
    if (rc == SRS_AMD_OK) {
      rc = make_demap_item(dem->demapper, pl->qm, items[i].d_llrs, reinterpret_cast<const float*>(y), v,
                           pl->args.nof_re, pl->sym_counts, dem->d_jump, pl->c_init, di);
    }
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    std::memcpy(dem->stage.at<tp_args>(o_tp + sizeof(tp_args) * k), &ta, sizeof(ta));
    std::memcpy(dem->stage.at<demap_item>(o_dm + sizeof(demap_item) * k), &di, sizeof(di));
    tp_rows = std::max(tp_rows, ta.nof_rows);
    tp_syms = std::max(tp_syms, pl->args.nof_re);
    tp_lds  = std::max(tp_lds, lds);
    ++k;
  }
  auto* d = dem->slot_items.as<uint8_t>();
  e       = dem->stage.upload(d, total, s);
  for (const group& g : groups) {
    if (e != hipSuccess) {
      break;
    }
    const eq_items m{reinterpret_cast<const eq_item*>(d), reinterpret_cast<const uint32_t*>(d + o_ids) + g.first};
    e = launch_pusch_equalize_fused_items(m, g.count, g.P, g.L, g.mmse, g.max_blocks, s);
  }
  if (e == hipSuccess && n_tp != 0) {
    e = launch_transform_deprecode_items(reinterpret_cast<const tp_args*>(d + o_tp), static_cast<uint32_t>(n_tp),
                                         tp_rows, tp_lds, s);
  }
  if (e == hipSuccess && n_tp != 0) {
    e = launch_demap_descramble_items(reinterpret_cast<const demap_item*>(d + o_dm), static_cast<uint32_t>(n_tp),
                                      tp_syms, s);
  }
  const hipError_t done = scope.close();
  e                     = e != hipSuccess ? e : done;
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pusch_equalize_fused_kernel slot launch");
}

extern "C" {

int srs_amd_pusch_demodulator_create(srs_amd_pusch_demodulator** dem, int device)
{
  if (dem == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *dem   = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* d   = new srs_amd_pusch_demodulator();
  d->device = device;
  rc        = srs_amd_modulator_create(&d->demapper, device);
  if (rc != SRS_AMD_OK) {
    delete d;
    return rc;
  }
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
    return hip_fail(e, "PUSCH demodulator tables");
  }
  *dem = d;
  return SRS_AMD_OK;
}

void srs_amd_pusch_demodulator_destroy(srs_amd_pusch_demodulator* dem)
{
  delete dem;
}

int srs_amd_pusch_demod_plan_create(srs_amd_pusch_demodulator*        dem,
                                    const srs_amd_pusch_demod_config* cfg,
                                    uint32_t                          nof_subc,
                                    srs_amd_pusch_demod_plan**        plan,
                                    uint32_t*                         nof_re)
{
  if (dem == nullptr || cfg == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  *plan = nullptr;
  if (nof_subc == 0 || nof_subc % 12 != 0 || nof_subc > 12 * SRS_AMD_MAX_RB) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  const int qm = cfg->modulation;
  if (!(qm == 0 || qm == 1 || qm == 2 || qm == 4 || qm == 6 || qm == 8)) {
    return fail(SRS_AMD_EINVAL, "Invalid modulation scheme %d.", qm);
  }
  if (!equalizer_supported(cfg->equalizer, cfg->nof_rx_ports, cfg->nof_tx_layers)) {
    return fail(SRS_AMD_EINVAL,
                "Invalid combination of channel spatial topology (i.e., %u Rx ports, %u Tx layers) and algorithm.",
                cfg->nof_rx_ports, cfg->nof_tx_layers);
  }
  if (cfg->nof_symbols == 0 || cfg->start_symbol + cfg->nof_symbols > 14) {
    return fail(SRS_AMD_EINVAL, "Invalid time allocation.");
  }
  if ((cfg->dmrs_type != 1 && cfg->dmrs_type != 2) || cfg->nof_cdm_groups_without_data < 1 ||
      cfg->nof_cdm_groups_without_data > (cfg->dmrs_type == 1 ? 2u : 3u)) {
    return fail(SRS_AMD_EINVAL, "Invalid DM-RS configuration.");
  }
  const uint32_t nof_prb = nof_subc / 12;
  uint32_t       lo = nof_prb, hi = 0;
  for (uint32_t c = 0; c < SRS_AMD_MAX_RB; ++c) {
    if (crb_bit(cfg->crb_mask, c)) {
      if (c >= nof_prb) {
        return fail(SRS_AMD_EINVAL, "Allocated RB %u exceeds the grid bandwidth.", c);
      }
      lo = std::min(lo, c);
      hi = c + 1;
    }
  }
  if (hi == 0) {
    return fail(SRS_AMD_EINVAL, "Empty frequency allocation.");
  }
  const uint32_t        dmrs_excl = dmrs_prb_mask(cfg->dmrs_type, cfg->nof_cdm_groups_without_data);
  std::vector<uint32_t> table(14 * nof_prb, 0);
  uint32_t              count = 0;
  uint32_t              sym_counts[14];
  for (uint32_t l = 0; l < 14; ++l) {
    const uint32_t sym_start = count;
    const bool in_time = l >= cfg->start_symbol && l < cfg->start_symbol + cfg->nof_symbols;
    const bool dmrs    = (cfg->dmrs_symbol_mask >> l) & 1u;
    for (uint32_t c = 0; c < nof_prb; ++c) {
      uint32_t m = (in_time && crb_bit(cfg->crb_mask, c)) ? 0xfffu : 0u;
      if (dmrs) {
        m &= ~dmrs_excl;
      }
      table[l * nof_prb + c] = (count << 12) | m;
      count += static_cast<uint32_t>(__builtin_popcount(m));
    }
    sym_counts[l] = count - sym_start;
  }
  uint32_t tp_subc = 0;
  if (cfg->transform_precoding) {
    // pusch_demodulator_impl.cpp:345-349 and transform_precoder_dft_impl.cpp:35-41
    if (cfg->nof_tx_layers != 1) {
      return fail(SRS_AMD_EINVAL, "Transform precoding is only possible with one layer (i.e. %u).", cfg->nof_tx_layers);
    }
    for (uint32_t l = 0; l < 14; ++l) {
      if (sym_counts[l] == 0) {
        continue;
      }
      if (tp_subc != 0 && sym_counts[l] != tp_subc) {
        return fail(SRS_AMD_EINVAL, "transform precoding: OFDM symbols with %u and %u data REs", tp_subc, sym_counts[l]);
      }
      tp_subc = sym_counts[l];
    }
    if (tp_subc % 12 != 0 || !srs_amd_transform_precoding_nof_prbs_valid(tp_subc / 12)) {
      return fail(SRS_AMD_EINVAL, "The number of PRB (i.e., %u) is not valid.", tp_subc / 12);
    }
  }
  auto* p         = new srs_amd_pusch_demod_plan();
  p->tp_subc      = tp_subc;
  p->device       = dem->device;
  p->nof_ports    = cfg->nof_rx_ports;
  p->nof_layers   = cfg->nof_tx_layers;
  p->mmse         = cfg->equalizer == SRS_AMD_EQ_MMSE && cfg->nof_tx_layers > 1; // one layer: ZF (generic_impl:343)
  p->nof_symbols  = cfg->nof_symbols;
  p->span_subc    = (hi - lo) * 12;
  p->qm           = qm;
  p->c_init       = cfg->rnti * (1u << 15) + cfg->n_id; // pusch_demodulator_impl.cpp:209
  for (uint32_t l = 0; l < 14; ++l) {
    p->sym_counts[l] = sym_counts[l] * cfg->nof_tx_layers;
  }
  pusch_eq_args& a = p->args;
  a.nof_subc       = nof_subc;
  a.nof_prb        = nof_prb;
  a.nof_re         = count;
  a.first_symbol   = cfg->start_symbol;
  a.first_subc     = lo * 12;
  a.dc_subc        = ~0u;
  hipError_t e     = hipSetDevice(dem->device);
  if (e == hipSuccess) {
    e = hipMalloc(&p->d_table, table.size() * sizeof(uint32_t));
  }
  if (e == hipSuccess) {
    e = hipMemcpy(p->d_table, table.data(), table.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "PUSCH demodulator plan");
  }
  a.re_table = p->d_table;
  // demapper tables, per-OFDM-symbol SIMD bounds and the descrambling words of the equalizer's LLR output
  const uint32_t grid_symbols = count * cfg->nof_tx_layers;
  a.dm                        = demodulate_args_for(dem->demapper, qm, grid_symbols);
  uint32_t sym_lo[14];
  (void)demap_symbol_bounds(qm, p->sym_counts, sym_lo, a.simd_hi);
  const uint32_t nof_words = (p->nof_llrs() + 31) / 32 + 1;
  e                        = hipMalloc(&p->d_scr, nof_words * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = launch_gold_words(dem->d_jump, p->c_init, p->d_scr, nof_words, nullptr);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(nullptr);
  }
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "PUSCH demodulator plan scrambling words");
  }
  a.scr = p->d_scr;
  *plan = p;
  if (nof_re != nullptr) {
    *nof_re = count;
  }
  return SRS_AMD_OK;
}

void srs_amd_pusch_demod_plan_destroy(srs_amd_pusch_demod_plan* plan)
{
  delete plan;
}

int srs_amd_pusch_demodulate_batch(srs_amd_pusch_demodulator*      dem,
                                   const srs_amd_pusch_demod_plan* plan,
                                   const uint32_t*                 d_grids,
                                   uint64_t                        grid_stride,
                                   const uint32_t*                 d_estimates,
                                   uint64_t                        est_stride,
                                   const srs_amd_chest_port_stats* d_stats,
                                   int8_t*                         d_llrs,
                                   uint64_t                        llr_stride,
                                   uint32_t                        nof_grids,
                                   void*                           stream)
{
  return demodulate_impl(dem, plan, d_grids, grid_stride, d_estimates, est_stride, nullptr, d_stats, d_llrs,
                         llr_stride, nof_grids, stream);
}

int srs_amd_pusch_demap_descramble_batch(srs_amd_pusch_demodulator*      dem,
                                         const srs_amd_pusch_demod_plan* plan,
                                         const float*                    d_eq_symbols,
                                         const float*                    d_eq_noise_vars,
                                         int8_t*                         d_llrs,
                                         uint64_t                        llr_stride,
                                         uint32_t                        nof_grids,
                                         void*                           stream)
{
  if (dem == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_grids == 0 || plan->args.nof_re == 0) {
    return SRS_AMD_OK;
  }
  if (d_eq_symbols == nullptr || d_eq_noise_vars == nullptr || d_llrs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (nof_grids > 1 && llr_stride < plan->nof_llrs()) {
    return fail(SRS_AMD_EINVAL, "LLR stride too small");
  }
  hipError_t e = hipSetDevice(dem->device);
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH demodulator device");
  }
  return demap_descramble_batch(dem->demapper, plan->qm, d_llrs, llr_stride, d_eq_symbols, d_eq_noise_vars,
                                static_cast<uint32_t>(plan->args.nof_re * plan->nof_layers), plan->sym_counts,
                                nof_grids, dem->d_jump, plan->c_init, stream);
}

int srs_amd_pusch_demodulate(srs_amd_pusch_demodulator*      dem,
                             const srs_amd_pusch_demod_plan* plan,
                             const uint32_t*                 grid,
                             const uint32_t*                 estimates,
                             const srs_amd_chest_port_stats* stats,
                             int8_t*                         llrs)
{
  if (dem == nullptr || plan == nullptr || grid == nullptr || estimates == nullptr || stats == nullptr ||
      llrs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t grid_bytes = plan->nof_ports * 14ull * plan->args.nof_subc * 4;
  const size_t est_bytes  = grid_bytes * plan->nof_layers;
  const size_t st_bytes   = plan->nof_ports * sizeof(srs_amd_chest_port_stats);
  const size_t nllr       = plan->nof_llrs();
  hipError_t   e;
  {
    std::lock_guard<std::mutex> lock(dem->mtx);
    e = hipSetDevice(dem->device);
    if (e == hipSuccess) {
      e = dem->host_io.ensure(align_up(grid_bytes, 256) + align_up(est_bytes, 256) + align_up(st_bytes, 256) + nllr);
    }
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH demodulator buffers");
  }
  auto* b      = dem->host_io.as<uint8_t>();
  auto* d_grid = reinterpret_cast<uint32_t*>(b);
  auto* d_est  = reinterpret_cast<uint32_t*>(b + align_up(grid_bytes, 256));
  auto* d_st   = reinterpret_cast<srs_amd_chest_port_stats*>(b + align_up(grid_bytes, 256) + align_up(est_bytes, 256));
  auto* d_llr  = reinterpret_cast<int8_t*>(b + align_up(grid_bytes, 256) + align_up(est_bytes, 256) +
                                          align_up(st_bytes, 256));
  e            = hipMemcpyAsync(d_grid, grid, grid_bytes, hipMemcpyHostToDevice, dem->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(d_est, estimates, est_bytes, hipMemcpyHostToDevice, dem->stream);
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(d_st, stats, st_bytes, hipMemcpyHostToDevice, dem->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH demodulator upload");
  }
  int rc = srs_amd_pusch_demodulate_batch(dem, plan, d_grid, 0, d_est, 0, d_st, d_llr, 0, 1, dem->stream);
  if (rc != SRS_AMD_OK) {
    (void)hipStreamSynchronize(dem->stream);
    return rc;
  }
  e = hipMemcpyAsync(llrs, d_llr, nllr, hipMemcpyDeviceToHost, dem->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(dem->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUSCH demodulator download");
}

} // extern "C"
