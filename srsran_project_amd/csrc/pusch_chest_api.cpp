// pusch_chest_api.cpp -- C-ABI of the MI355X PUSCH DM-RS channel estimator
// (include/srsran_amd/pusch_chest.h).
//
// Host-side logic, once per call (a few hundred bytes of kernel arguments):
//   DM-RS c_init per symbol (dmrs_pusch_estimator_impl.cpp:95-108);
//   symbol start epochs (port_channel_estimator_average_impl.cpp:542-553);
//   raised-cosine filter taps and virtual-pilot count
//     (port_channel_estimator_helpers.cpp:58-100, 230-240);
//   the time-domain interpolation table (apply_td_domain_strategy, :555-620);
//   the time-alignment IDFT size, sampling rate and search window
//     (time_alignment_estimator_dft_impl.cpp:230-275).
#include "srsran_amd/pusch_chest.h"
#include "srsran_amd/low_papr.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "gold_sequence.h"
#include "pusch_chest_args.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

using namespace srs_amd;

namespace {

constexpr double T_C      = 1.0 / (480000.0 * 4096.0);
constexpr int    TA_MIN_N = 128;  // pow2(log2_ceil(1 / (15 kHz x TA unit)))
constexpr int    TA_MAX_N = 4096; // pow2(log2_ceil(275 x 12))

const float RC_FILTER[31] = {-0.0641253, -0.0660711, -0.0611526, -0.0485918, -0.0281126, 0.0000000, 0.0348830,
                             0.0751249,  0.1188406,  0.1637874,  0.2075139,  0.2475302,  0.2814857, 0.3073415,
                             0.3235207,  0.3290274,  0.3235207,  0.3073415,  0.2814857,  0.2475302, 0.2075139,
                             0.1637874,  0.1188406,  0.0751249,  0.0348830,  0.0000000,  -0.0281126, -0.0485918,
                             -0.0611526, -0.0660711, -0.0641253};

std::vector<float> twiddles(uint32_t N)
{
  std::vector<float> t(2 * N);
  for (uint32_t m = 0; m < N; ++m) {
    const double a = -2.0 * M_PI * static_cast<double>(m) / static_cast<double>(N);
    t[2 * m]       = static_cast<float>(std::cos(a));
    t[2 * m + 1]   = static_cast<float>(std::sin(a));
  }
  return t;
}

int log2_ceil(uint32_t x)
{
  int r = 0;
  while ((1u << r) < x) {
    ++r;
  }
  return r;
}

} // namespace

struct srs_amd_pusch_chest {
  int           device = 0;
  hipStream_t   stream = nullptr;
  uint32_t*     d_jump = nullptr;
  uint32_t*     d_gold_basis = nullptr;
  float*        d_tw   = nullptr; // twiddle tables of N = 128 .. 4096, back to back
  device_buffer scratch;
  device_buffer host_io;
  stream_order  order; // scratch reuse across the callers' streams
  pinned_stage  stage; // slot form: per-PDU argument blocks
  std::mutex    mtx;
  // transform precoding: low-PAPR pilot sequences by (length, group), generated on first use and kept
  std::map<uint64_t, float2*> lp_tables;
  ~srs_amd_pusch_chest()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(d_jump);
    (void)hipFree(d_gold_basis);
    (void)hipFree(d_tw);
    for (auto& t : lp_tables) {
      (void)hipFree(t.second);
    }
  }
  // The device copy of r_{u,0}(n), n < M (caller holds mtx); nullptr on failure (the error is recorded).
  const float2* low_papr(uint32_t M, uint32_t u)
  {
    const uint64_t key = (static_cast<uint64_t>(M) << 8) | u;
    auto           it  = lp_tables.find(key);
    if (it != lp_tables.end()) {
      return it->second;
    }
    std::vector<float> h(2 * M);
    if (srs_amd_low_papr_sequence(h.data(), M, u, 0) != SRS_AMD_OK) {
      return nullptr;
    }
    float2*    d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(float2) * M);
    if (e == hipSuccess) {
      e = hipMemcpy(d, h.data(), sizeof(float2) * M, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
      (void)hipFree(d);
      hip_fail(e, "low-PAPR sequence upload");
      return nullptr;
    }
    lp_tables.emplace(key, d);
    return d;
  }
  const float2* tw(uint32_t N) const
  {
    size_t off = 0;
    for (uint32_t n = TA_MIN_N; n < N; n *= 2) {
      off += 2 * n;
    }
    return reinterpret_cast<const float2*>(d_tw + off);
  }
};

namespace {

int make_args(chest_args& a, const srs_amd_pusch_chest_config* cfg, uint32_t nof_ports, uint32_t nof_subc)
{
  if (cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null configuration");
  }
  if (cfg->nof_tx_layers < 1 || cfg->nof_tx_layers > CH_MAXL) {
    return fail(SRS_AMD_EINVAL, "The number of Tx layers is %u, max %d supported.", cfg->nof_tx_layers, CH_MAXL);
  }
  if (cfg->low_papr && (cfg->nof_tx_layers != 1 || cfg->n_rs_id > 1007)) {
    return fail(SRS_AMD_EINVAL, "Transform precoding is only possible with one layer and n_rs_id <= 1007.");
  }
  if (cfg->low_papr && !srs_amd_low_papr_length_valid(6 * cfg->rb_count)) {
    return fail(SRS_AMD_EINVAL, "No low-PAPR sequence of length %u (transform precoding with %u PRB).",
                6 * cfg->rb_count, cfg->rb_count);
  }
  if (!(cfg->scaling > 0)) {
    return fail(SRS_AMD_EINVAL, "The DM-RS to data scaling factor should be a positive number.");
  }
  if (nof_ports == 0 || nof_subc == 0 || nof_subc % 12 != 0 || nof_subc > 12 * 275) {
    return fail(SRS_AMD_EINVAL, "Invalid grid (%u ports, %u subcarriers).", nof_ports, nof_subc);
  }
  if (cfg->rb_count == 0 || cfg->rb_start + cfg->rb_count > nof_subc / 12) {
    return fail(SRS_AMD_EINVAL, "PRB allocation [%u, %u) outside the grid.", cfg->rb_start,
                cfg->rb_start + cfg->rb_count);
  }
  if (cfg->nof_symbols == 0 || cfg->first_symbol + cfg->nof_symbols > CH_NSYMB) {
    return fail(SRS_AMD_EINVAL, "Invalid time allocation.");
  }
  if (cfg->fd_smoothing < 0 || cfg->fd_smoothing > 2 || cfg->td_interpolation < 0 || cfg->td_interpolation > 1) {
    return fail(SRS_AMD_EINVAL, "Invalid estimator strategy.");
  }
  if (cfg->numerology > 4) {
    return fail(SRS_AMD_EINVAL, "Invalid numerology %u.", cfg->numerology);
  }
  a                = chest_args{};
  a.nof_ports      = nof_ports;
  a.nsubc          = nof_subc;
  a.L              = cfg->nof_tx_layers;
  a.ncdm           = (cfg->nof_tx_layers + 1) / 2;
  a.npil           = 6 * cfg->rb_count;
  a.nof_re         = 12 * cfg->rb_count;
  a.prb_lo         = cfg->rb_start;
  a.first_symbol   = cfg->first_symbol;
  a.nof_symbols    = cfg->nof_symbols;
  a.beta           = cfg->scaling;
  a.fd             = cfg->fd_smoothing;
  a.td             = cfg->td_interpolation;
  a.compensate_cfo = cfg->compensate_cfo ? 1 : 0;

  const uint32_t last = cfg->first_symbol + cfg->nof_symbols;
  for (uint32_t l = 0; l < CH_NSYMB; ++l) {
    if (((cfg->symbols_mask >> l) & 1u) == 0) {
      continue;
    }
    if (l < cfg->first_symbol || l >= last) {
      return fail(SRS_AMD_EINVAL, "DM-RS symbol %u outside the allocation.", l);
    }
    if (a.nds == CH_MAXDMRS) {
      return fail(SRS_AMD_EINVAL, "More than %d DM-RS symbols.", CH_MAXDMRS);
    }
    const unsigned nid = cfg->scrambling_id, nscid = cfg->n_scid ? 1 : 0;
    a.dmrs_sym[a.nds] = l;
    a.c_init[a.nds]   = ((CH_NSYMB * cfg->slot_index + l + 1) * (2 * nid + 1) * (1u << 17) + (2 * nid + nscid)) %
                      (1u << 31);
    ++a.nds;
  }
  if (a.nds == 0) {
    return fail(SRS_AMD_EINVAL, "No DM-RS symbols were found.");
  }
  a.nof_lse = a.td == SRS_AMD_CHEST_TD_AVERAGE ? 1 : a.nds;

  // Symbol start epochs in units of the symbol duration (float, as the reference accumulates them).
  const unsigned mu     = cfg->numerology;
  const unsigned scs_k  = 15u << mu;
  a.scs_hz              = static_cast<float>(scs_k * 1000);
  auto cp_s = [mu](unsigned i) {
    unsigned k = 144u >> mu;
    if (i == 0 || i == 7u * (1u << mu)) {
      k += 16;
    }
    return static_cast<double>(k * 64) * T_C;
  };
  a.epoch[0] = static_cast<float>(cp_s(0) * scs_k * 1000);
  for (unsigned i = 1; i < CH_NSYMB; ++i) {
    a.epoch[i] = static_cast<float>(a.epoch[i - 1] + cp_s(i) * scs_k * 1000 + 1.0F);
  }

  // filter_type(nof_rb, stride = 2).
  {
    const unsigned nrb       = std::min(cfg->rb_count, 3u);
    const unsigned nof_coefs = nrb * 10 + 1;
    unsigned       n_out     = nof_coefs / 2 / 2;
    const unsigned n_first   = 31 / 2 - n_out * 2;
    n_out                    = 2 * n_out + 1;
    float total              = 0;
    for (unsigned i = 0; i < n_out; ++i) {
      a.rc[i] = RC_FILTER[n_first + 2 * i];
      total += a.rc[i];
    }
    const float inv = 1 / total;
    for (unsigned i = 0; i < n_out; ++i) {
      a.rc[i] *= inv;
    }
    a.nof_taps = static_cast<int32_t>(n_out);
    a.nof_v    = cfg->rb_count == 1 ? static_cast<int32_t>(a.npil) : std::min<int32_t>(CH_MAXV, a.nof_taps / 2);
  }

  // Time-domain interpolation table (apply_td_domain_strategy).
  for (int l = static_cast<int>(cfg->first_symbol); l < static_cast<int>(last); ++l) {
    auto is_dmrs = [&](int s) { return (cfg->symbols_mask >> s) & 1u; };
    int  before  = -1;
    for (int s = static_cast<int>(cfg->first_symbol); s < l; ++s) {
      before = is_dmrs(s) ? s : before;
    }
    int after = -1;
    for (int s = l; s < static_cast<int>(last) && after < 0; ++s) {
      after = is_dmrs(s) ? s : -1;
    }
    a.td_interp[l] = 1;
    if (before == -1) {
      int second = -1;
      for (int s = after + 1; s < static_cast<int>(last) && second < 0; ++s) {
        second = is_dmrs(s) ? s : -1;
      }
      if (second == -1) {
        a.td_i0[l]     = 0;
        a.td_interp[l] = 0;
        continue;
      }
      before = after;
      after  = second;
    }
    if (after == -1) {
      int second_last = -1;
      for (int s = static_cast<int>(cfg->first_symbol); s < before; ++s) {
        second_last = is_dmrs(s) ? s : second_last;
      }
      if (second_last == -1) {
        a.td_i0[l]     = static_cast<int32_t>(a.nds) - 1;
        a.td_interp[l] = 0;
        continue;
      }
      after  = before;
      before = second_last;
    }
    int i0 = 0;
    for (int s = static_cast<int>(cfg->first_symbol); s < before; ++s) {
      i0 += is_dmrs(s) ? 1 : 0;
    }
    a.td_i0[l] = i0;
    a.td_w[l]  = static_cast<float>(l - before) / static_cast<float>(after - before);
  }

  // Time alignment: IDFT size, sampling rate, half-CP search window (stride 2 for the PUSCH pattern).
  uint32_t req = a.npil * TA_MAX_N / (275 * 12);
  uint32_t N   = 1u << log2_ceil(std::max(req, 1u));
  N            = std::max<uint32_t>(TA_MIN_N, N);
  if (N > 2048) { // the fused pilot kernel's largest IDFT (npil <= 6 x 275)
    return fail(SRS_AMD_EINVAL, "Time-alignment IDFT of %u points exceeds 2048.", N);
  }
  a.ta_n       = N;
  a.ta_fs      = static_cast<double>(N) * scs_k * 1000 * 2;
  const double half_cp_s = static_cast<double>((144u * 64u) >> (mu + 1)) * T_C;
  a.ta_max_taps          = static_cast<int32_t>(std::floor(half_cp_s * a.ta_fs));
  a.ta_frac              = N != TA_MAX_N ? 1 : 0;
  return SRS_AMD_OK;
}

size_t scratch_bytes(const chest_args& a, uint32_t nof_grids)
{
  const size_t gp = static_cast<size_t>(nof_grids) * a.nof_ports;
  return align_up(gp * a.L * a.nof_lse * a.npil * 8, 256) + align_up(gp * a.L * a.nof_lse * a.nof_re * 8, 256) +
         align_up(gp * CH_ACC * 4, 256) + align_up(gp * a.L * a.nof_lse * a.ta_n * 4, 256) +
         CH_MAXDMRS * CH_SEQWORDS * 4;
}

} // namespace

extern "C" {

int srs_amd_pusch_chest_create(srs_amd_pusch_chest** chest, int device)
{
  if (chest == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *chest = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* c                 = new srs_amd_pusch_chest();
  c->device               = device;
  std::vector<uint32_t> j = gold_jump_tables();
  std::vector<float>    tw;
  for (uint32_t n = TA_MIN_N; n <= TA_MAX_N; n *= 2) {
    std::vector<float> t = twiddles(n);
    tw.insert(tw.end(), t.begin(), t.end());
  }
  hipError_t e = hipMalloc(&c->d_jump, j.size() * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = hipMemcpy(c->d_jump, j.data(), j.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  const std::vector<uint32_t> gb = gold_word_basis();
  if (e == hipSuccess) {
    e = hipMalloc(&c->d_gold_basis, gb.size() * sizeof(uint32_t));
  }
  if (e == hipSuccess) {
    e = hipMemcpy(c->d_gold_basis, gb.data(), gb.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipMalloc(&c->d_tw, tw.size() * sizeof(float));
  }
  if (e == hipSuccess) {
    e = hipMemcpy(c->d_tw, tw.data(), tw.size() * sizeof(float), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "PUSCH channel estimator tables");
  }
  *chest = c;
  return SRS_AMD_OK;
}

void srs_amd_pusch_chest_destroy(srs_amd_pusch_chest* chest)
{
  delete chest;
}

} // extern "C"

static int estimate_batch_impl(srs_amd_pusch_chest*              chest,
                                       const srs_amd_pusch_chest_config* cfg,
                                       const uint32_t*                   d_grids,
                                       uint64_t                          grid_stride,
                                       uint32_t                          nof_ports,
                                       uint32_t                          nof_subc,
                                       uint32_t                          nof_grids,
                                       uint32_t*                         d_estimates,
                                       uint64_t                          est_stride,
                                       srs_amd_chest_port_stats*         d_stats,
                                       void*                             stream,
                                       bool                              expand,
                                       chest_args*                       view)
{
  if (chest == nullptr) {
    return fail(SRS_AMD_EINVAL, "null estimator");
  }
  chest_args a;
  int        rc = make_args(a, cfg, nof_ports, nof_subc);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_grids == 0) {
    return SRS_AMD_OK;
  }
  if (d_grids == nullptr || (expand && d_estimates == nullptr) || d_stats == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (nof_grids > 1 && (grid_stride < static_cast<uint64_t>(nof_ports) * CH_NSYMB * nof_subc ||
                        (expand && est_stride < static_cast<uint64_t>(nof_ports) * a.L * CH_NSYMB * nof_subc))) {
    return fail(SRS_AMD_EINVAL, "grid or estimate stride too small");
  }
  std::lock_guard<std::mutex> lock(chest->mtx);
  hipError_t                  e = hipSetDevice(chest->device);
  if (e == hipSuccess) {
    // One scratch per object: a batch on another stream than the previous one waits for it
    // (stream_order); a growing reallocation frees the old block only after the device is idle (hipFree).
    e = chest->scratch.ensure(scratch_bytes(a, nof_grids));
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH channel estimator scratch");
  }
  const size_t gp = static_cast<size_t>(nof_grids) * nof_ports;
  auto*        base = chest->scratch.as<uint8_t>();
  a.filt            = reinterpret_cast<float2*>(base);
  base += align_up(gp * a.L * a.nof_lse * a.npil * 8, 256);
  a.freq = reinterpret_cast<float2*>(base);
  base += align_up(gp * a.L * a.nof_lse * a.nof_re * 8, 256);
  a.acc         = reinterpret_cast<float*>(base);
  base += align_up(gp * CH_ACC * 4, 256);
  a.corr        = reinterpret_cast<float*>(base);
  base += align_up(gp * a.L * a.nof_lse * a.ta_n * 4, 256);
  a.dmrs_seq    = reinterpret_cast<uint32_t*>(base);
  a.grids       = d_grids;
  a.grid_stride = grid_stride;
  a.estimates   = d_estimates;
  a.est_stride  = est_stride;
  a.stats       = d_stats;
  a.jump        = chest->d_jump;
  a.gold_basis  = chest->d_gold_basis;
  a.ta_tw       = chest->tw(a.ta_n);
  a.lp_seq      = nullptr;
  if (cfg->low_papr) {
    a.lp_seq = chest->low_papr(a.npil, cfg->n_rs_id % 30);
    if (a.lp_seq == nullptr) {
      return SRS_AMD_EHIP;
    }
  }
  e             = chest->order.begin(static_cast<hipStream_t>(stream));
  if (e == hipSuccess) {
    e = launch_chest(a, nof_grids, static_cast<hipStream_t>(stream), expand);
  }
  if (e == hipSuccess) {
    e = chest->order.end(static_cast<hipStream_t>(stream));
  }
  if (view != nullptr) {
    *view = a;
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "channel estimator launch");
}

int srs_amd::chest_estimate_batch_unexpanded(::srs_amd_pusch_chest*            chest,
                                             const srs_amd_pusch_chest_config* cfg,
                                             const uint32_t*                   d_grids,
                                             uint64_t                          grid_stride,
                                             uint32_t                          nof_ports,
                                             uint32_t                          nof_subc,
                                             uint32_t                          nof_grids,
                                             srs_amd_chest_port_stats*         d_stats,
                                             void*                             stream,
                                             chest_args*                       view)
{
  return estimate_batch_impl(chest, cfg, d_grids, grid_stride, nof_ports, nof_subc, nof_grids, nullptr, 0, d_stats,
                             stream, false, view);
}

int srs_amd::chest_estimate_slot_unexpanded(::srs_amd_pusch_chest* chest,
                                            const chest_slot_item* items,
                                            uint32_t               nof_items,
                                            uint32_t               nof_subc,
                                            void*                  stream,
                                            chest_args*            views)
{
  if (chest == nullptr || (nof_items != 0 && (items == nullptr || views == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_items == 0) {
    return SRS_AMD_OK;
  }
  // host argument blocks; per-PDU scratch laid out back to back (offsets first, pointers once allocated)
  std::vector<size_t> offset(nof_items);
  size_t              total      = 0;
  uint32_t            max_ports  = 0;
  uint32_t            max_slices = 0;
  for (uint32_t i = 0; i != nof_items; ++i) {
    int rc = make_args(views[i], items[i].cfg, items[i].nof_ports, nof_subc);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    if (items[i].d_grid == nullptr || items[i].d_stats == nullptr) {
      return fail(SRS_AMD_EINVAL, "null device buffer");
    }
    offset[i] = total;
    total += align_up(scratch_bytes(views[i], 1), 256);
    max_ports  = std::max(max_ports, views[i].nof_ports);
    max_slices = std::max(max_slices, views[i].L * views[i].nof_lse);
  }
  const size_t o_args = total;
  const size_t stage  = sizeof(chest_args) * nof_items;
  std::lock_guard<std::mutex> lock(chest->mtx);
  hipError_t                  e = hipSetDevice(chest->device);
  if (e == hipSuccess) {
    e = chest->scratch.ensure(o_args + stage);
  }
  if (e == hipSuccess) {
    e = chest->stage.acquire(stage);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH channel estimator slot scratch");
  }
  auto* base = chest->scratch.as<uint8_t>();
  for (uint32_t i = 0; i != nof_items; ++i) {
    chest_args& a = views[i];
    uint8_t*    b = base + offset[i];
    a.filt        = reinterpret_cast<float2*>(b);
    b += align_up(static_cast<size_t>(a.nof_ports) * a.L * a.nof_lse * a.npil * 8, 256);
    a.freq = reinterpret_cast<float2*>(b);
    b += align_up(static_cast<size_t>(a.nof_ports) * a.L * a.nof_lse * a.nof_re * 8, 256);
    a.acc = reinterpret_cast<float*>(b);
    b += align_up(static_cast<size_t>(a.nof_ports) * CH_ACC * 4, 256);
    a.corr = reinterpret_cast<float*>(b);
    b += align_up(static_cast<size_t>(a.nof_ports) * a.L * a.nof_lse * a.ta_n * 4, 256);
    a.dmrs_seq    = reinterpret_cast<uint32_t*>(b);
    a.grids       = items[i].d_grid;
    a.grid_stride = 0;
    a.estimates   = nullptr;
    a.est_stride  = 0;
    a.stats       = items[i].d_stats;
    a.jump        = chest->d_jump;
    a.gold_basis  = chest->d_gold_basis;
    a.ta_tw       = chest->tw(a.ta_n);
    a.lp_seq      = nullptr;
    if (items[i].cfg->low_papr) {
      a.lp_seq = chest->low_papr(a.npil, items[i].cfg->n_rs_id % 30);
      if (a.lp_seq == nullptr) {
        return SRS_AMD_EHIP;
      }
    }
  }
  std::memcpy(chest->stage.at<chest_args>(0), views, sizeof(chest_args) * nof_items);
  auto s = static_cast<hipStream_t>(stream);
  e      = chest->order.begin(s);
  if (e != hipSuccess) {
    return hip_fail(e, "channel estimator slot launch");
  }
  call_scope scope(chest->order, nullptr, s);
  e = chest->stage.upload(base + o_args, stage, s);
  if (e == hipSuccess) {
    const chest_items all{reinterpret_cast<const chest_args*>(base + o_args), nullptr};
    uint32_t nof_small = 0;
    for (uint32_t i = 0; i != nof_items; ++i) {
      nof_small += views[i].npil <= 412 ? 1u : 0u;
    }
    e = launch_chest_items(all, nof_items, max_ports, max_slices, nof_small, s);
  }
  const hipError_t done = scope.close();
  e                     = e != hipSuccess ? e : done;
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "channel estimator slot launch");
}

extern "C" {

int srs_amd_pusch_chest_estimate_batch(srs_amd_pusch_chest*              chest,
                                       const srs_amd_pusch_chest_config* cfg,
                                       const uint32_t*                   d_grids,
                                       uint64_t                          grid_stride,
                                       uint32_t                          nof_ports,
                                       uint32_t                          nof_subc,
                                       uint32_t                          nof_grids,
                                       uint32_t*                         d_estimates,
                                       uint64_t                          est_stride,
                                       srs_amd_chest_port_stats*         d_stats,
                                       void*                             stream)
{
  return estimate_batch_impl(chest, cfg, d_grids, grid_stride, nof_ports, nof_subc, nof_grids, d_estimates,
                             est_stride, d_stats, stream, true, nullptr);
}

int srs_amd_pusch_chest_estimate(srs_amd_pusch_chest*              chest,
                                 const srs_amd_pusch_chest_config* cfg,
                                 const uint32_t*                   grid,
                                 uint32_t                          nof_ports,
                                 uint32_t                          nof_subc,
                                 uint32_t*                         estimates,
                                 srs_amd_chest_port_stats*         stats)
{
  if (chest == nullptr || cfg == nullptr || grid == nullptr || estimates == nullptr || stats == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  chest_args a;
  int        rc = make_args(a, cfg, nof_ports, nof_subc);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const size_t grid_bytes  = static_cast<size_t>(nof_ports) * CH_NSYMB * nof_subc * 4;
  const size_t est_bytes   = grid_bytes * a.L;
  const size_t stats_bytes = nof_ports * sizeof(srs_amd_chest_port_stats);
  hipError_t   e;
  {
    std::lock_guard<std::mutex> lock(chest->mtx);
    e = hipSetDevice(chest->device);
    if (e == hipSuccess) {
      e = chest->host_io.ensure(align_up(grid_bytes, 256) + align_up(est_bytes, 256) + stats_bytes);
    }
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH channel estimator buffers");
  }
  auto* d_grid  = chest->host_io.as<uint32_t>();
  auto* d_est   = reinterpret_cast<uint32_t*>(chest->host_io.as<uint8_t>() + align_up(grid_bytes, 256));
  auto* d_stats = reinterpret_cast<srs_amd_chest_port_stats*>(chest->host_io.as<uint8_t>() +
                                                              align_up(grid_bytes, 256) + align_up(est_bytes, 256));
  e             = hipMemcpyAsync(d_grid, grid, grid_bytes, hipMemcpyHostToDevice, chest->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(d_est, estimates, est_bytes, hipMemcpyHostToDevice, chest->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUSCH channel estimator upload");
  }
  rc = srs_amd_pusch_chest_estimate_batch(chest, cfg, d_grid, 0, nof_ports, nof_subc, 1, d_est, 0, d_stats,
                                          chest->stream);
  if (rc != SRS_AMD_OK) {
    (void)hipStreamSynchronize(chest->stream);
    return rc;
  }
  e = hipMemcpyAsync(estimates, d_est, est_bytes, hipMemcpyDeviceToHost, chest->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(stats, d_stats, stats_bytes, hipMemcpyDeviceToHost, chest->stream);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(chest->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUSCH channel estimator download");
}

} // extern "C"
