// pdsch_modulator_api.cpp -- C-ABI of the MI355X PDSCH modulator and PDSCH
// DM-RS processor (include/srsran_amd/pdsch_modulator.h).
//
// Host-side logic:
//   plan: the RE allocation of pdsch_modulator_impl::map (pdsch_modulator_impl.cpp:53-86):
//     allocated CRBs minus the reserved patterns and the DM-RS pattern
//     (dmrs_type::get_dmrs_pattern, dmrs_mapping.h:76-123) in every symbol of the
//     time allocation, flattened to a per-(symbol, PRB) table;
//   scaling: modulation scaling (sqrt(1 / average power), modulation_mapper_lut_impl.cpp:60-66)
//     times config.scaling when normal, folded into the precoding weights (:74-79);
//   scrambling: c_init = rnti << 15 + q << 14 + n_id, q = 0 (pdsch_modulator_impl.cpp:33);
//   DM-RS: c_init per symbol (dmrs_pdsch_processor_impl.cpp:66), amplitude
//     M_SQRT1_2 * amplitude (:60), CRB list of the rb_mask.
#include "srsran_amd/pdsch_modulator.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "gold_sequence.h"
#include "modulation_args.h"
#include "pdsch_modulator_args.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_pdsch_modulator {
  int           device = 0;
  hipStream_t   stream = nullptr;
  uint32_t*     d_jump = nullptr;
  device_buffer scratch;
  device_buffer slot_items; // slot form: per-PDU argument blocks
  pinned_stage  stage;
  stream_order  order;
  std::mutex    mtx;
  ~srs_amd_pdsch_modulator()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(d_jump);
  }
};

struct srs_amd_pdsch_mod_plan {
  int            device = 0;
  pdsch_map_args args{};
  uint32_t       nof_symbols = 0;
  uint32_t       span_subc   = 0;
  uint32_t       nof_re      = 0;
  uint32_t*      d_table     = nullptr;
  uint32_t*      d_scr       = nullptr; // Gold words of c_init over the codeword (+1)
  ~srs_amd_pdsch_mod_plan()
  {
    (void)hipSetDevice(device);
    (void)hipFree(d_table);
    (void)hipFree(d_scr);
  }
};

namespace {

bool crb_bit(const uint8_t* mask, uint32_t i)
{
  return i < SRS_AMD_MAX_RB && ((mask[i / 8] >> (i % 8)) & 1u);
}

bool valid_qm(int qm)
{
  return qm == 0 || qm == 1 || qm == 2 || qm == 4 || qm == 6 || qm == 8;
}

// modulation_mapper_lut_impl.cpp:40-67 (QAM) and :176 / :205 (BPSK, pi/2-BPSK).
float modulation_scaling(int qm)
{
  if (qm < 2) {
    return static_cast<float>(M_SQRT1_2);
  }
  const int L   = 1 << qm;
  float     sum = 0;
  for (int i = 0; i < L; ++i) {
    float off = -1, re = 0, im = 0;
    for (int j = 0; j < qm / 2; ++j) {
      re += off;
      im += off;
      off *= 2;
      re *= ((i & (1 << (2 * j + 1))) != 0) ? +1 : -1;
      im *= ((i & (1 << (2 * j + 0))) != 0) ? +1 : -1;
    }
    sum += re * re + im * im; // integers: exact
  }
  return std::sqrt(1 / (sum / static_cast<float>(L)));
}

// get_dmrs_prb_mask (dmrs_mapping.h:76-91).
uint32_t dmrs_prb_mask(uint32_t type, uint32_t nof_cdm_groups_without_data)
{
  uint32_t m = 0;
  for (uint32_t k = 0; k < 12; ++k) {
    const bool in = type == 1 ? (k % 2) < nof_cdm_groups_without_data : (k % 6) < 2 * nof_cdm_groups_without_data;
    m |= in ? (1u << k) : 0u;
  }
  return m;
}

int check_weights(uint32_t nof_layers, uint32_t nof_ports)
{
  if (nof_layers < 1 || nof_layers > SRS_AMD_MAX_LAYERS) {
    return fail(SRS_AMD_EINVAL, "The number of layers (i.e., %u) must be in range [1, %d].", nof_layers,
                SRS_AMD_MAX_LAYERS);
  }
  if (nof_ports < nof_layers || nof_ports > SRS_AMD_MAX_TX_PORTS) {
    return fail(SRS_AMD_EINVAL, "The number of antennas (i.e., %u) must be in range [%u, %d].", nof_ports,
                nof_layers, SRS_AMD_MAX_TX_PORTS);
  }
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_pdsch_modulator_create(srs_amd_pdsch_modulator** mod, int device)
{
  if (mod == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *mod   = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* m                 = new srs_amd_pdsch_modulator();
  m->device               = device;
  std::vector<uint32_t> j = gold_jump_tables();
  hipError_t            e = hipMalloc(&m->d_jump, j.size() * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = hipMemcpy(m->d_jump, j.data(), j.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete m;
    return hip_fail(e, "PDSCH modulator tables");
  }
  *mod = m;
  return SRS_AMD_OK;
}

void srs_amd_pdsch_modulator_destroy(srs_amd_pdsch_modulator* mod)
{
  delete mod;
}

int srs_amd_pdsch_mod_plan_create(srs_amd_pdsch_modulator*        mod,
                                  const srs_amd_pdsch_mod_config* cfg,
                                  uint32_t                        nof_subc,
                                  srs_amd_pdsch_mod_plan**        plan,
                                  uint32_t*                       nof_re)
{
  if (mod == nullptr || cfg == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  *plan = nullptr;
  if (nof_subc == 0 || nof_subc % 12 != 0 || nof_subc > 12 * SRS_AMD_MAX_RB) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  if (!valid_qm(cfg->modulation)) {
    return fail(SRS_AMD_EINVAL, "Invalid modulation scheme %d.", cfg->modulation);
  }
  int rc = check_weights(cfg->nof_layers, cfg->nof_ports);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (cfg->nof_symbols == 0 || cfg->start_symbol + cfg->nof_symbols > PDSCH_NSYMB) {
    return fail(SRS_AMD_EINVAL, "The time allocation of the transmission [%u, %u) exceeds the slot boundary.",
                cfg->start_symbol, cfg->start_symbol + cfg->nof_symbols);
  }
  if (cfg->dmrs_type != 1 && cfg->dmrs_type != 2) {
    return fail(SRS_AMD_EINVAL, "Invalid DM-RS type %u.", cfg->dmrs_type);
  }
  if (cfg->nof_cdm_groups_without_data < 1 || cfg->nof_cdm_groups_without_data > (cfg->dmrs_type == 1 ? 2u : 3u)) {
    return fail(SRS_AMD_EINVAL, "Invalid number of CDM groups without data (i.e., %u).",
                cfg->nof_cdm_groups_without_data);
  }
  if (cfg->nof_reserved > SRS_AMD_MAX_RE_PATTERNS) {
    return fail(SRS_AMD_EINVAL, "Too many reserved RE patterns (i.e., %u).", cfg->nof_reserved);
  }
  const uint32_t nof_prb = nof_subc / 12;
  uint32_t       lo = nof_prb, hi = 0;
  for (uint32_t c = 0; c < nof_prb; ++c) {
    if (crb_bit(cfg->crb_mask, c)) {
      lo = std::min(lo, c);
      hi = c + 1;
    }
  }
  for (uint32_t c = nof_prb; c < SRS_AMD_MAX_RB; ++c) {
    if (crb_bit(cfg->crb_mask, c)) {
      return fail(SRS_AMD_EINVAL, "Allocated CRB %u exceeds the grid bandwidth (%u RB).", c, nof_prb);
    }
  }
  if (hi == 0) {
    return fail(SRS_AMD_EINVAL, "Empty frequency allocation.");
  }

  // re_pattern_list::get_exclusion_mask per symbol (re_pattern.cpp:62-100), DM-RS pattern merged.
  const uint32_t        dmrs_re = dmrs_prb_mask(cfg->dmrs_type, cfg->nof_cdm_groups_without_data);
  std::vector<uint32_t> table(PDSCH_NSYMB * nof_prb, 0);
  uint32_t              count = 0;
  for (uint32_t l = 0; l < PDSCH_NSYMB; ++l) {
    const bool in_time = l >= cfg->start_symbol && l < cfg->start_symbol + cfg->nof_symbols;
    for (uint32_t c = 0; c < nof_prb; ++c) {
      uint32_t m = (in_time && crb_bit(cfg->crb_mask, c)) ? 0xfffu : 0u;
      if (m != 0) {
        for (uint32_t r = 0; r < cfg->nof_reserved; ++r) {
          const srs_amd_re_pattern& p = cfg->reserved[r];
          if (((p.symbols >> l) & 1u) && crb_bit(p.crb_mask, c)) {
            m &= ~static_cast<uint32_t>(p.re_mask);
          }
        }
        if (((cfg->dmrs_symbol_mask >> l) & 1u) && c >= cfg->bwp_start && c < cfg->bwp_start + cfg->bwp_size) {
          m &= ~dmrs_re;
        }
      }
      table[l * nof_prb + c] = (count << 12) | m;
      count += static_cast<uint32_t>(__builtin_popcount(m));
    }
  }

  auto* p                 = new srs_amd_pdsch_mod_plan();
  p->device               = mod->device;
  p->nof_re               = count;
  p->nof_symbols          = cfg->nof_symbols;
  p->span_subc            = (hi - lo) * 12;
  pdsch_map_args& a       = p->args;
  a.jump                  = mod->d_jump;
  a.port_stride           = PDSCH_NSYMB * nof_subc;
  a.nof_subc              = nof_subc;
  a.nof_prb               = nof_prb;
  a.c_init                = (cfg->rnti << 15) + cfg->n_id;
  a.first_symbol          = cfg->start_symbol;
  a.qm                    = cfg->modulation;
  a.nof_layers            = static_cast<int32_t>(cfg->nof_layers);
  a.nof_ports             = static_cast<int32_t>(cfg->nof_ports);
  a.first_subc            = lo * 12;
  a.nof_symbols           = cfg->nof_symbols;
  a.nof_tiles             = (p->span_subc + PDSCH_THREADS - 1) / PDSCH_THREADS;
  float scaling           = modulation_scaling(cfg->modulation);
  if (std::isnormal(cfg->scaling)) {
    scaling *= cfg->scaling;
  }
  for (uint32_t v = 0; v < cfg->nof_layers; ++v) {
    for (uint32_t q = 0; q < cfg->nof_ports; ++q) {
      a.w[v][q][0] = cfg->weights[v][q][0] * scaling;
      a.w[v][q][1] = cfg->weights[v][q][1] * scaling;
    }
  }
  hipError_t e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = hipMalloc(&p->d_table, table.size() * sizeof(uint32_t));
  }
  if (e == hipSuccess) {
    e = hipMemcpy(p->d_table, table.data(), table.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  // the scrambling sequence of the plan's c_init, generated once (the map kernel XORs table words)
  const uint32_t bps       = cfg->modulation < 2 ? 1u : static_cast<uint32_t>(cfg->modulation);
  const uint32_t nof_words = (count * cfg->nof_layers * bps + 31) / 32 + 1;
  if (e == hipSuccess) {
    e = hipMalloc(&p->d_scr, nof_words * sizeof(uint32_t));
  }
  if (e == hipSuccess) {
    e = launch_gold_words(mod->d_jump, a.c_init, p->d_scr, nof_words, nullptr);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(nullptr);
  }
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "PDSCH modulator plan");
  }
  a.scr      = p->d_scr;
  a.re_table = p->d_table;
  *plan      = p;
  if (nof_re != nullptr) {
    *nof_re = count;
  }
  return SRS_AMD_OK;
}

void srs_amd_pdsch_mod_plan_destroy(srs_amd_pdsch_mod_plan* plan)
{
  delete plan;
}

int srs_amd_pdsch_modulate_batch(srs_amd_pdsch_modulator*      mod,
                                 const srs_amd_pdsch_mod_plan* plan,
                                 uint32_t*                     d_grids,
                                 uint64_t                      grid_stride,
                                 const uint8_t*                d_codewords,
                                 uint32_t                      cw_stride,
                                 uint32_t                      nof_bits,
                                 uint32_t                      nof_cws,
                                 void*                         stream)
{
  if (mod == nullptr || plan == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const pdsch_map_args& pa  = plan->args;
  const uint32_t        bps = pa.qm < 2 ? 1u : static_cast<uint32_t>(pa.qm);
  if (nof_bits == 0 || nof_bits % (pa.nof_layers * bps) != 0) {
    return fail(SRS_AMD_EINVAL, "The codeword length (i.e., %u bits) is not a whole number of REs (%d layers x %u bits).",
                nof_bits, pa.nof_layers, bps);
  }
  if (nof_cws == 0) {
    return SRS_AMD_OK;
  }
  if (d_grids == nullptr || d_codewords == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (nof_cws > 1 && (cw_stride < (nof_bits + 7) / 8 || grid_stride < static_cast<uint64_t>(pa.nof_ports) *
                                                                           pa.port_stride)) {
    return fail(SRS_AMD_EINVAL, "codeword or grid stride too small");
  }
  pdsch_map_args a = pa;
  a.codewords      = d_codewords;
  a.grids          = d_grids;
  a.grid_stride    = grid_stride;
  a.cw_stride      = cw_stride;
  a.nof_bits       = nof_bits;
  hipError_t e     = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = launch_pdsch_map(a, plan->nof_symbols, plan->span_subc, nof_cws, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pdsch_map_kernel launch");
}

int srs_amd_pdsch_modulate(srs_amd_pdsch_modulator*      mod,
                           const srs_amd_pdsch_mod_plan* plan,
                           uint32_t*                     grid,
                           uint32_t                      grid_ports,
                           const uint8_t*                codeword,
                           uint32_t                      nof_bits)
{
  if (mod == nullptr || plan == nullptr || grid == nullptr || codeword == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (grid_ports < static_cast<uint32_t>(plan->args.nof_ports)) {
    return fail(SRS_AMD_EINVAL, "The precoding number of ports (i.e., %d) exceeds the grid number of ports (i.e., %u).",
                plan->args.nof_ports, grid_ports);
  }
  std::lock_guard<std::mutex> lock(mod->mtx);
  const size_t                grid_bytes = static_cast<size_t>(grid_ports) * plan->args.port_stride * 4;
  const size_t                cw_bytes   = (nof_bits + 7) / 8;
  hipError_t                  e          = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = mod->scratch.ensure(grid_bytes + align_up(cw_bytes, 256) + 256);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PDSCH modulator scratch");
  }
  auto* d_grid = mod->scratch.as<uint32_t>();
  auto* d_cw   = mod->scratch.as<uint8_t>() + align_up(grid_bytes, 256);
  e            = hipMemcpyAsync(d_grid, grid, grid_bytes, hipMemcpyHostToDevice, mod->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(d_cw, codeword, cw_bytes, hipMemcpyHostToDevice, mod->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PDSCH modulator upload");
  }
  int rc = srs_amd_pdsch_modulate_batch(mod, plan, d_grid, 0, d_cw, static_cast<uint32_t>(cw_bytes), nof_bits, 1,
                                        mod->stream);
  if (rc != SRS_AMD_OK) {
    (void)hipStreamSynchronize(mod->stream);
    return rc;
  }
  e = hipMemcpyAsync(grid, d_grid, grid_bytes, hipMemcpyDeviceToHost, mod->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(mod->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PDSCH modulator download");
}

} // extern "C"

// get_ptrs_pattern (lib/ran/ptrs/ptrs_pattern.cpp:54-110) for the PT-RS of cfg: PRBs rb_begin, rb_begin + stride, ..
// < rb_end, subcarrier k of the RB (the first port's k_re_ref, TS 38.211 Table 7.4.1.2.2-1), symbols of symbol_mask.
struct ptrs_layout {
  uint32_t rb_begin = 0, rb_end = 0, stride = 1, k = 0, symbol_mask = 0, mask_begin = 0;
};

static int ptrs_pattern(const srs_amd_ptrs_pdsch_config* c, ptrs_layout& o)
{
  if (c->dmrs_type != 1 && c->dmrs_type != 2) {
    return fail(SRS_AMD_EINVAL, "Invalid DM-RS type %u.", c->dmrs_type);
  }
  if (c->freq_density != 2 && c->freq_density != 4) {
    return fail(SRS_AMD_EINVAL, "Invalid PT-RS frequency density %u.", c->freq_density);
  }
  if (c->time_density != 1 && c->time_density != 2 && c->time_density != 4) {
    return fail(SRS_AMD_EINVAL, "Invalid PT-RS time density %u.", c->time_density);
  }
  if (c->re_offset > 3 || c->start_symbol + c->nof_symbols > PDSCH_NSYMB || c->nof_symbols == 0) {
    return fail(SRS_AMD_EINVAL, "Invalid PT-RS RE offset or time allocation.");
  }
  int lo = -1, hi = -1, n = 0;
  for (uint32_t r = 0; r != SRS_AMD_MAX_RB; ++r) {
    if (crb_bit(c->crb_mask, r)) {
      lo = lo < 0 ? static_cast<int>(r) : lo;
      hi = static_cast<int>(r);
      ++n;
    }
  }
  if (lo < 0 || hi - lo + 1 != n) {
    return fail(SRS_AMD_EINVAL, "Only contiguous allocations are supported.");
  }
  static const uint8_t k_type1[4] = {0, 2, 6, 8};
  static const uint8_t k_type2[4] = {0, 1, 6, 7};
  const uint32_t       K          = c->freq_density;
  const uint32_t       L          = c->time_density;
  uint32_t             k_rb_ref   = (c->rnti & 0xffffu) % K;
  if (n % K != 0) {
    k_rb_ref = (c->rnti & 0xffffu) % (n % K);
  }
  o.mask_begin  = static_cast<uint32_t>(lo);
  o.rb_begin    = k_rb_ref + static_cast<uint32_t>(lo);
  o.rb_end      = static_cast<uint32_t>(lo + n);
  o.stride      = K;
  o.k           = c->dmrs_type == 1 ? k_type1[c->re_offset] : k_type2[c->re_offset];
  o.symbol_mask = 0;
  const int stop = static_cast<int>(c->start_symbol + c->nof_symbols);
  int       i = 0, l_ref = static_cast<int>(c->start_symbol);
  while (l_ref + i * static_cast<int>(L) < stop) {
    const int startpos = std::max(l_ref + (i - 1) * static_cast<int>(L) + 1, l_ref);
    const int endpos   = l_ref + i * static_cast<int>(L);
    int       dmrs_pos = -1;
    for (int l = endpos; l >= startpos; --l) {
      if ((c->dmrs_symbols_mask >> l) & 1u) {
        dmrs_pos = l;
        break;
      }
    }
    if (dmrs_pos >= 0) {
      i     = 1;
      l_ref = dmrs_pos;
      continue;
    }
    o.symbol_mask |= 1u << (l_ref + i * static_cast<int>(L));
    ++i;
  }
  return SRS_AMD_OK;
}

// The PT-RS argument block of cfg (ptrs_pdsch_generator_impl.cpp:30-130); weights_offset: where cfg's weights will
// be in the device weight array (floats).
static int make_ptrs_args(const srs_amd_pdsch_modulator* mod, const srs_amd_ptrs_pdsch_config* c, uint32_t nof_subc,
                          ptrs_pdsch_args& a)
{
  ptrs_layout o;
  int         rc = ptrs_pattern(c, o);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (c->nof_ports == 0 || c->nof_ports > SRS_AMD_MAX_TX_PORTS || c->nof_prg == 0 || c->prg_size == 0 ||
      c->weights == nullptr) {
    return fail(SRS_AMD_EINVAL, "Invalid PT-RS precoding (%u ports, %u PRGs of %u PRBs).", c->nof_ports, c->nof_prg,
                c->prg_size);
  }
  if (o.rb_end > nof_subc / 12 || o.mask_begin < c->reference_point_k_rb) {
    return fail(SRS_AMD_EINVAL, "PT-RS CRBs outside the grid or below the reference point.");
  }
  const uint32_t nd = c->dmrs_type == 1 ? 6 : 4;
  a                 = ptrs_pdsch_args{};
  a.jump            = mod->d_jump;
  a.port_stride     = PDSCH_NSYMB * nof_subc;
  a.nof_subc        = nof_subc;
  a.rb_begin        = o.rb_begin;
  a.rb_stride       = o.stride;
  a.nof_prb         = o.rb_end > o.rb_begin ? (o.rb_end - o.rb_begin + o.stride - 1) / o.stride : 0;
  if (a.nof_prb != 0 && (o.rb_begin + (a.nof_prb - 1) * o.stride) / c->prg_size >= c->nof_prg) {
    return fail(SRS_AMD_EINVAL, "PT-RS CRBs beyond the precoding PRGs.");
  }
  a.k           = o.k;
  a.symbol_mask = o.symbol_mask;
  // ptrs_pdsch_generator_impl.cpp: l_0 = the first DM-RS symbol; unsigned arithmetic modulo 2^32 then % 2^31
  const uint32_t l0    = c->dmrs_symbols_mask != 0 ? static_cast<uint32_t>(__builtin_ctz(c->dmrs_symbols_mask)) : 0u;
  const uint32_t nid   = c->scrambling_id;
  const uint32_t nscid = c->n_scid ? 1u : 0u;
  a.c_init   = ((PDSCH_NSYMB * c->slot_index + l0 + 1) * (2 * nid + 1) * (1u << 17) + (2 * nid + nscid)) % (1u << 31);
  a.bit0     = 2 * ((o.rb_begin - c->reference_point_k_rb) * nd + o.k / 2);
  a.bit_step = 2 * nd * o.stride;
  a.amplitude = static_cast<float>(M_SQRT1_2 * c->amplitude);
  a.nof_ports = c->nof_ports;
  a.prg_size  = c->prg_size;
  return SRS_AMD_OK;
}

// The DM-RS argument block of cfg (dmrs_pdsch_processor_impl.cpp:40-90) for grids of nof_subc subcarriers.
static int make_dmrs_args(const srs_amd_pdsch_modulator* mod, const srs_amd_dmrs_pdsch_config* cfg, uint32_t nof_subc,
                          dmrs_pdsch_args& a)
{
  int rc = check_weights(cfg->nof_layers, cfg->nof_ports);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (cfg->type != 1 && cfg->type != 2) {
    return fail(SRS_AMD_EINVAL, "Invalid DM-RS type %u.", cfg->type);
  }
  if (nof_subc == 0 || nof_subc % 12 != 0 || nof_subc > 12 * SRS_AMD_MAX_RB) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  a = dmrs_pdsch_args{};
  a.jump                 = mod->d_jump;
  a.port_stride          = PDSCH_NSYMB * nof_subc;
  a.reference_point_k_rb = cfg->reference_point_k_rb;
  a.type2                = cfg->type == 2 ? 1 : 0;
  a.nof_layers           = static_cast<int32_t>(cfg->nof_layers);
  a.nof_ports            = static_cast<int32_t>(cfg->nof_ports);
  a.amplitude            = static_cast<float>(M_SQRT1_2 * cfg->amplitude);
  for (uint32_t c = 0; c < SRS_AMD_MAX_RB; ++c) {
    if (crb_bit(cfg->crb_mask, c)) {
      if (c >= nof_subc / 12) {
        return fail(SRS_AMD_EINVAL, "DM-RS CRB %u exceeds the grid bandwidth.", c);
      }
      if (c < cfg->reference_point_k_rb) {
        return fail(SRS_AMD_EINVAL, "DM-RS CRB %u below the reference point %u.", c, cfg->reference_point_k_rb);
      }
      a.crbs[a.nof_crb++] = static_cast<uint16_t>(c);
    }
  }
  const unsigned nslot = cfg->slot_index;
  const unsigned nid   = cfg->scrambling_id;
  const unsigned nscid = cfg->n_scid ? 1 : 0;
  for (uint32_t l = 0; l < PDSCH_NSYMB; ++l) {
    if ((cfg->symbols_mask >> l) & 1u) {
      const uint32_t i = a.nof_dmrs_symbols++;
      a.symbol[i]      = static_cast<uint8_t>(l);
      a.lprime[i]      = (l > 0 && ((cfg->symbols_mask >> (l - 1)) & 1u)) ? 1 : 0;
      // dmrs_pdsch_processor_impl.cpp:66, unsigned arithmetic modulo 2^32 then % 2^31.
      a.c_init[i] = ((PDSCH_NSYMB * nslot + l + 1) * (2 * nid + 1) * (1u << 17) + (2 * nid + nscid)) % (1u << 31);
    }
  }
  for (uint32_t v = 0; v < cfg->nof_layers; ++v) {
    for (uint32_t q = 0; q < cfg->nof_ports; ++q) {
      a.w[v][q][0] = cfg->weights[v][q][0];
      a.w[v][q][1] = cfg->weights[v][q][1];
    }
  }
  return SRS_AMD_OK;
}

extern "C" {

int srs_amd_dmrs_pdsch_map_batch(srs_amd_pdsch_modulator*         mod,
                                 const srs_amd_dmrs_pdsch_config* cfg,
                                 uint32_t*                        d_grids,
                                 uint64_t                         grid_stride,
                                 uint32_t                         nof_subc,
                                 uint32_t                         nof_grids,
                                 void*                            stream)
{
  if (mod == nullptr || cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  dmrs_pdsch_args a;
  int             rc = make_dmrs_args(mod, cfg, nof_subc, a);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  a.grids       = d_grids;
  a.grid_stride = grid_stride;
  if (nof_grids == 0 || a.nof_crb == 0 || a.nof_dmrs_symbols == 0) {
    return SRS_AMD_OK;
  }
  if (d_grids == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (nof_grids > 1 && grid_stride < static_cast<uint64_t>(cfg->nof_ports) * a.port_stride) {
    return fail(SRS_AMD_EINVAL, "grid stride too small");
  }
  hipError_t e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = launch_dmrs_pdsch(a, nof_grids, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "dmrs_pdsch_kernel launch");
}

int srs_amd_dmrs_pdsch_map(srs_amd_pdsch_modulator*         mod,
                           const srs_amd_dmrs_pdsch_config* cfg,
                           uint32_t*                        grid,
                           uint32_t                         grid_ports,
                           uint32_t                         nof_subc)
{
  if (mod == nullptr || cfg == nullptr || grid == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (grid_ports < cfg->nof_ports) {
    return fail(SRS_AMD_EINVAL, "The precoding number of ports (i.e., %u) exceeds the grid number of ports (i.e., %u).",
                cfg->nof_ports, grid_ports);
  }
  std::lock_guard<std::mutex> lock(mod->mtx);
  const size_t                grid_bytes = static_cast<size_t>(grid_ports) * PDSCH_NSYMB * nof_subc * 4;
  hipError_t                  e          = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = mod->scratch.ensure(grid_bytes);
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(mod->scratch.ptr, grid, grid_bytes, hipMemcpyHostToDevice, mod->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "DM-RS upload");
  }
  int rc = srs_amd_dmrs_pdsch_map_batch(mod, cfg, mod->scratch.as<uint32_t>(), 0, nof_subc, 1, mod->stream);
  if (rc != SRS_AMD_OK) {
    (void)hipStreamSynchronize(mod->stream);
    return rc;
  }
  e = hipMemcpyAsync(grid, mod->scratch.ptr, grid_bytes, hipMemcpyDeviceToHost, mod->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(mod->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "DM-RS download");
}

int srs_amd_pdsch_modulate_slot(srs_amd_pdsch_modulator*      mod,
                                const srs_amd_pdsch_slot_pdu* pdus,
                                uint32_t                      nof_pdus,
                                uint32_t*                     d_grids,
                                uint64_t                      grid_stride,
                                uint32_t                      nof_grids,
                                uint32_t                      nof_subc,
                                const uint8_t*                d_codewords,
                                void*                         stream)
{
  if (mod == nullptr || (nof_pdus != 0 && pdus == nullptr)) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_pdus == 0) {
    return SRS_AMD_OK;
  }
  std::vector<pdsch_map_args>  maps;
  std::vector<dmrs_pdsch_args> dmrs;
  std::vector<ptrs_pdsch_args> ptrs;
  std::vector<float>           ptrs_w;    // every PT-RS PDU's [prg][port] weights
  std::vector<size_t>          ptrs_woff; // offset of each PT-RS PDU's weights in ptrs_w
  uint32_t                     max_tiles = 0, max_symbols = 0, max_blocks = 0, max_dmrs_symbols = 0, max_ptrs = 0;
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const srs_amd_pdsch_slot_pdu& u = pdus[i];
    if (u.d_grid == nullptr && (d_grids == nullptr || u.grid >= nof_grids)) {
      return fail(SRS_AMD_EINVAL, "PDU %u: grid index %u out of range (or no grid).", i, u.grid);
    }
    // a PDU with its own grid (device-resident resource grid) is checked as a single-grid call
    const bool      own  = u.d_grid != nullptr;
    uint32_t* const grid = own ? u.d_grid : d_grids + u.grid * grid_stride;
    const uint32_t  ng   = own ? 1u : nof_grids;
    if (u.plan != nullptr) {
      const pdsch_map_args& pa  = u.plan->args;
      const uint32_t        bps = pa.qm < 2 ? 1u : static_cast<uint32_t>(pa.qm);
      if (pa.nof_subc != nof_subc) {
        return fail(SRS_AMD_EINVAL, "PDU %u: plan for %u subcarriers, grid of %u.", i, pa.nof_subc, nof_subc);
      }
      // a codeword longer than the allocation maps its first nof_re x layers symbols, a shorter one its first
      // nof_bits / (layers x Qm) REs (as the reference's mapper, see pdsch_modulator.h)
      if (u.nof_bits == 0 || u.nof_bits % (pa.nof_layers * bps) != 0) {
        return fail(SRS_AMD_EINVAL, "PDU %u: the codeword length (i.e., %u bits) is not a whole number of REs.", i,
                    u.nof_bits);
      }
      if (ng > 1 && grid_stride < static_cast<uint64_t>(pa.nof_ports) * pa.port_stride) {
        return fail(SRS_AMD_EINVAL, "grid stride too small");
      }
      if (d_codewords == nullptr) {
        return fail(SRS_AMD_EINVAL, "null device buffer");
      }
      pdsch_map_args a = pa;
      a.codewords      = d_codewords + u.cw_offset;
      a.grids          = grid;
      a.grid_stride    = 0;
      a.cw_stride      = 0;
      a.nof_bits       = u.nof_bits;
      maps.push_back(a);
      max_tiles   = std::max(max_tiles, a.nof_tiles);
      max_symbols = std::max(max_symbols, a.nof_symbols);
    }
    if (u.dmrs != nullptr) {
      dmrs_pdsch_args a;
      int             rc = make_dmrs_args(mod, u.dmrs, nof_subc, a);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
      if (ng > 1 && grid_stride < static_cast<uint64_t>(a.nof_ports) * a.port_stride) {
        return fail(SRS_AMD_EINVAL, "grid stride too small");
      }
      a.grids       = grid;
      a.grid_stride = 0;
      if (a.nof_crb != 0 && a.nof_dmrs_symbols != 0) {
        dmrs.push_back(a);
        max_blocks       = std::max(max_blocks, (a.nof_crb * PDSCH_NRE + 255) / 256); // dmrs_pdsch_kernel REs per WG
        max_dmrs_symbols = std::max(max_dmrs_symbols, a.nof_dmrs_symbols);
      }
    }
    if (u.ptrs != nullptr) {
      ptrs_pdsch_args a;
      int             rc = make_ptrs_args(mod, u.ptrs, nof_subc, a);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
      if (ng > 1 && grid_stride < static_cast<uint64_t>(a.nof_ports) * a.port_stride) {
        return fail(SRS_AMD_EINVAL, "grid stride too small");
      }
      a.grid = grid;
      if (a.nof_prb != 0 && a.symbol_mask != 0) {
        ptrs_woff.push_back(ptrs_w.size());
        ptrs_w.insert(ptrs_w.end(), u.ptrs->weights, u.ptrs->weights + 2 * u.ptrs->nof_prg * u.ptrs->nof_ports);
        ptrs.push_back(a);
        max_ptrs = std::max(max_ptrs, a.nof_prb);
      }
    }
  }
  const size_t o_dmrs = align_up(sizeof(pdsch_map_args) * maps.size(), 256);
  const size_t o_ptrs = align_up(o_dmrs + sizeof(dmrs_pdsch_args) * dmrs.size(), 256);
  const size_t o_w    = align_up(o_ptrs + sizeof(ptrs_pdsch_args) * ptrs.size(), 256);
  const size_t total  = ptrs.empty() ? o_dmrs + sizeof(dmrs_pdsch_args) * dmrs.size() : o_w + sizeof(float) * ptrs_w.size();
  if (total == 0) {
    return SRS_AMD_OK;
  }
  auto                        s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(mod->mtx);
  hipError_t                  e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = mod->slot_items.ensure(total);
  }
  if (e == hipSuccess) {
    e = mod->stage.acquire(total);
  }
  if (e == hipSuccess) {
    e = mod->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PDSCH modulator slot descriptors");
  }
  call_scope scope(mod->order, nullptr, s);
  std::memcpy(mod->stage.at<pdsch_map_args>(0), maps.data(), sizeof(pdsch_map_args) * maps.size());
  std::memcpy(mod->stage.at<dmrs_pdsch_args>(o_dmrs), dmrs.data(), sizeof(dmrs_pdsch_args) * dmrs.size());
  auto* d = mod->slot_items.as<uint8_t>();
  for (size_t q = 0; q != ptrs.size(); ++q) {
    ptrs[q].w = reinterpret_cast<const float*>(d + o_w) + ptrs_woff[q];
  }
  if (!ptrs.empty()) {
    std::memcpy(mod->stage.at<ptrs_pdsch_args>(o_ptrs), ptrs.data(), sizeof(ptrs_pdsch_args) * ptrs.size());
    std::memcpy(mod->stage.at<float>(o_w), ptrs_w.data(), sizeof(float) * ptrs_w.size());
  }
  e       = mod->stage.upload(d, total, s);
  if (e == hipSuccess) {
    e = launch_pdsch_map_items(reinterpret_cast<const pdsch_map_args*>(d), static_cast<uint32_t>(maps.size()),
                               max_tiles, max_symbols, s);
  }
  if (e == hipSuccess) {
    // pdsch_processor_impl.cpp:80-88: the PT-RS after the data (over the data mapped at its REs), then the DM-RS
    e = launch_ptrs_pdsch_items(reinterpret_cast<const ptrs_pdsch_args*>(d + o_ptrs),
                                static_cast<uint32_t>(ptrs.size()), max_ptrs, s);
  }
  if (e == hipSuccess) {
    e = launch_dmrs_pdsch_items(reinterpret_cast<const dmrs_pdsch_args*>(d + o_dmrs),
                                static_cast<uint32_t>(dmrs.size()), max_blocks, max_dmrs_symbols, s);
  }
  const hipError_t done = scope.close();
  e                     = e != hipSuccess ? e : done;
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PDSCH modulator slot launch");
}

int srs_amd_ptrs_pdsch_reserved(const srs_amd_ptrs_pdsch_config* cfg, srs_amd_re_pattern* pattern)
{
  if (cfg == nullptr || pattern == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  ptrs_layout o;
  int         rc = ptrs_pattern(cfg, o);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  *pattern = srs_amd_re_pattern{};
  for (uint32_t r = o.rb_begin; r < o.rb_end; r += o.stride) {
    pattern->crb_mask[r / 8] |= static_cast<uint8_t>(1u << (r % 8));
  }
  pattern->re_mask = static_cast<uint16_t>(1u << o.k);
  pattern->symbols = static_cast<uint16_t>(o.symbol_mask);
  return SRS_AMD_OK;
}

} // extern "C"
