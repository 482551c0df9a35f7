// pdsch_processor_hip.cpp -- srsran::pdsch_processor over the srsran_amd PDSCH slot C-ABI (see the header).
#include "pdsch_processor_hip.h"
#include "hip_resource_grid.h"
#include "slot_collector.h"

#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran/support/math/math_utils.h"
#include "srsran_amd/pdsch_modulator.h"
#include "srsran_amd/sch.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <list>
#include <optional>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

using namespace srsran;
using namespace srsran::hip;

namespace {

constexpr unsigned NSYMB     = 14;          // OFDM symbols of a normal-CP slot
constexpr unsigned MAX_PORTS = 4;           // transmit ports of one grid
constexpr uint32_t SENTINEL  = 0xffffffffu; // bf16 NaN pair: never a PDSCH / DM-RS RE value

void log_error(const char* what, const std::string& detail)
{
  std::fprintf(stderr, "pdsch_processor_hip: %s: %s\n", what, detail.c_str());
}

int32_t qm_code(modulation_scheme m)
{
  switch (m) {
    case modulation_scheme::PI_2_BPSK:
      return 0;
    case modulation_scheme::BPSK:
      return 1;
    default:
      return static_cast<int32_t>(get_bits_per_symbol(m));
  }
}

// ldpc::compute_nof_codeblocks / compute_N_ref (ldpc.h:140-151, 225-228).
uint32_t nof_codeblocks(uint32_t tbs, uint32_t bg)
{
  const uint32_t b = tbs + (tbs > 3824 ? 24u : 16u);
  const uint32_t m = bg == 1 ? 8448u : 3840u;
  return b <= m ? 1u : (b + (m - 24) - 1) / (m - 24);
}

uint32_t compute_N_ref(uint32_t tbs_lbrm_bytes, uint32_t C)
{
  const uint64_t n = static_cast<uint64_t>(tbs_lbrm_bytes) * 8 * 3 / (2 * C);
  return static_cast<uint32_t>(std::min<uint64_t>(n, 384 * 66));
}

/// One queued process() call.
struct pending_pdu {
  resource_grid_writer*     grid     = nullptr;
  pdsch_processor_notifier* notifier = nullptr;
  std::optional<shared_transport_block> tb;
  pdsch_processor::pdu_t    pdu;
  srs_amd_pdsch_mod_config  mod{};
  srs_amd_dmrs_pdsch_config dmrs{};
  uint32_t                  numerology = 0;
  std::string               error;
  // PT-RS (pdsch_process_ptrs, pdsch_processor_helpers.h:78-118): its configuration and layer-0 weights per PRG
  bool                      has_ptrs = false;
  srs_amd_ptrs_pdsch_config ptrs{};
  std::vector<float>        ptrs_w;
};

template <typename Mask>
void set_mask_bytes(uint8_t* bytes, const Mask& m, unsigned n)
{
  for (unsigned i = 0; i != n && i < m.size(); ++i) {
    if (m.test(i)) {
      bytes[i / 8] |= static_cast<uint8_t>(1u << (i % 8));
    }
  }
}

// pdu_t -> the modulator / DM-RS configurations pdsch_processor_impl::modulate and pdsch_process_dmrs build
// (pdsch_processor_impl.cpp:185-200, pdsch_processor_helpers.h:36-62); an empty string when supported.
std::string convert(pending_pdu& p, unsigned nof_prb)
{
  const pdsch_processor::pdu_t& pdu = p.pdu;
  if (pdu.cp != cyclic_prefix::NORMAL) {
    return "extended cyclic prefix";
  }
  if (pdu.codewords.size() != 1) {
    return "two codewords";
  }
  const precoding_configuration& pc = pdu.precoding;
  const unsigned                 L  = pc.get_nof_layers();
  const unsigned                 P  = pc.get_nof_ports();
  if (L == 0 || L > SRS_AMD_MAX_LAYERS || P == 0 || P > MAX_PORTS || P < L) {
    return "layers / ports outside 1..4";
  }
  // precoding that differs between PRGs: the reference's data mapper would take the first PRG's weights for every
  // PRB (resource_grid_mapper_impl.cpp:322-323), but its DM-RS processor writes PRG >= 1 weights into a one-PRG
  // configuration (dmrs_pdsch_processor_impl.cpp:150-160: an assertion, or an out-of-bounds write without asserts),
  // so there is no reference output to reproduce
  for (unsigned g = 1; g < pc.get_nof_prg(); ++g) {
    if (!(pc.get_prg_coefficients(g) == pc.get_prg_coefficients(0))) {
      return "precoding that differs between PRGs";
    }
  }
  if (pdu.reserved.get_nof_entries() > SRS_AMD_MAX_RE_PATTERNS) {
    return "more than eight reserved RE patterns";
  }
  if (pdu.start_symbol_index + pdu.nof_symbols > NSYMB || pdu.bwp_start_rb + pdu.bwp_size_rb > nof_prb) {
    return "allocation outside the slot / grid";
  }
  const crb_bitmap crbs = pdu.freq_alloc.get_crb_mask(pdu.bwp_start_rb, pdu.bwp_size_rb);
  if (crbs.none()) {
    return "empty frequency allocation";
  }
  srs_amd_pdsch_mod_config& m = p.mod;
  m                           = srs_amd_pdsch_mod_config{};
  m.rnti                      = pdu.rnti;
  m.n_id                      = pdu.n_id;
  m.modulation                = qm_code(pdu.codewords[0].modulation);
  m.bwp_start                 = pdu.bwp_start_rb;
  m.bwp_size                  = pdu.bwp_size_rb;
  set_mask_bytes(m.crb_mask, crbs, SRS_AMD_MAX_RB);
  m.start_symbol = pdu.start_symbol_index;
  m.nof_symbols  = pdu.nof_symbols;
  for (unsigned l = 0; l != NSYMB && l < pdu.dmrs_symbol_mask.size(); ++l) {
    m.dmrs_symbol_mask |= pdu.dmrs_symbol_mask.test(l) ? (1u << l) : 0u;
  }
  // pdsch_processor_impl::modulate (pdsch_processor_impl.cpp:185-200) leaves pdsch_modulator::config_t::
  // dmrs_config_type at its default, TYPE1: the data REs avoid the type-1 DM-RS pattern of the PDU's CDM groups
  // whatever its DM-RS type (the DM-RS itself is mapped with the PDU's type afterwards)
  m.dmrs_type                   = 1;
  m.nof_cdm_groups_without_data = pdu.nof_cdm_groups_without_data;
  m.scaling                     = convert_dB_to_amplitude(-pdu.ratio_pdsch_data_to_sss_dB);
  m.nof_layers                  = L;
  m.nof_ports                   = P;
  for (unsigned l = 0; l != L; ++l) {
    for (unsigned q = 0; q != P; ++q) {
      const cf_t w       = pc.get_coefficient(l, q, 0);
      m.weights[l][q][0] = w.real();
      m.weights[l][q][1] = w.imag();
    }
  }
  span<const re_pattern> res = pdu.reserved.get_re_patterns();
  m.nof_reserved             = static_cast<uint32_t>(res.size());
  for (size_t r = 0; r != res.size(); ++r) {
    set_mask_bytes(m.reserved[r].crb_mask, res[r].crb_mask, SRS_AMD_MAX_RB);
    for (unsigned k = 0; k != 12; ++k) {
      m.reserved[r].re_mask |= res[r].re_mask.test(k) ? static_cast<uint16_t>(1u << k) : 0;
    }
    for (unsigned l = 0; l != NSYMB; ++l) {
      m.reserved[r].symbols |= res[r].symbols.test(l) ? static_cast<uint16_t>(1u << l) : 0;
    }
  }
  srs_amd_dmrs_pdsch_config& d = p.dmrs;
  d                            = srs_amd_dmrs_pdsch_config{};
  d.slot_index                 = pdu.slot.slot_index();
  d.reference_point_k_rb       = pdu.ref_point == pdsch_processor::pdu_t::PRB0 ? pdu.bwp_start_rb : 0;
  d.type                       = pdu.dmrs == dmrs_type::TYPE1 ? 1u : 2u;
  d.scrambling_id              = pdu.scrambling_id;
  d.n_scid                     = pdu.n_scid ? 1 : 0;
  d.amplitude                  = convert_dB_to_amplitude(-pdu.ratio_pdsch_dmrs_to_sss_dB);
  d.symbols_mask               = m.dmrs_symbol_mask;
  std::memcpy(d.crb_mask, m.crb_mask, sizeof(d.crb_mask));
  d.nof_layers = L;
  d.nof_ports  = P;
  std::memcpy(d.weights, m.weights, sizeof(d.weights));
  p.numerology = to_numerology_value(pdu.slot.scs());
  p.has_ptrs   = pdu.ptrs.has_value();
  if (p.has_ptrs) {
    const pdsch_processor::ptrs_configuration& t = *pdu.ptrs;
    srs_amd_ptrs_pdsch_config&                 c = p.ptrs;
    c                                            = srs_amd_ptrs_pdsch_config{};
    c.slot_index                                 = d.slot_index;
    c.rnti                                       = pdu.rnti;
    c.dmrs_type                                  = d.type;
    c.reference_point_k_rb                       = d.reference_point_k_rb;
    c.scrambling_id                              = pdu.scrambling_id;
    c.n_scid                                     = d.n_scid;
    c.amplitude         = convert_dB_to_amplitude(t.ratio_ptrs_to_pdsch_data_dB - pdu.ratio_pdsch_data_to_sss_dB);
    c.dmrs_symbols_mask = m.dmrs_symbol_mask;
    std::memcpy(c.crb_mask, m.crb_mask, sizeof(c.crb_mask));
    c.start_symbol = pdu.start_symbol_index;
    c.nof_symbols  = pdu.nof_symbols;
    c.freq_density = to_value(t.freq_density);
    c.time_density = to_value(t.time_density);
    c.re_offset    = to_value(t.re_offset);
    c.nof_ports    = P;
    c.nof_prg      = pc.get_nof_prg();
    c.prg_size     = pc.get_prg_size();
    p.ptrs_w.resize(2 * c.nof_prg * P);
    for (unsigned g = 0; g != c.nof_prg; ++g) {
      for (unsigned q = 0; q != P; ++q) {
        const cf_t w                   = pc.get_coefficient(0, q, g);
        p.ptrs_w[2 * (g * P + q)]     = w.real();
        p.ptrs_w[2 * (g * P + q) + 1] = w.imag();
      }
    }
    c.weights = p.ptrs_w.data();
    srs_amd_re_pattern pattern; // validates the PT-RS configuration (the pattern itself reserves nothing, see .h)
    if (srs_amd_ptrs_pdsch_reserved(&c, &pattern) != SRS_AMD_OK) {
      return srs_amd_last_error();
    }
  }
  return {};
}

// pdsch_compute_nof_data_re (pdsch_processor_helpers.h:97-140): the codeword's REs per layer -- the allocation minus
// the reserved REs (counted without overlap) minus the DM-RS pattern of the PDU's own DM-RS type.
uint32_t nof_data_re(const pending_pdu& p)
{
  const srs_amd_pdsch_mod_config& m    = p.mod;
  const bool                      t2   = p.pdu.dmrs != dmrs_type::TYPE1;
  const uint32_t                  ncdm = m.nof_cdm_groups_without_data;
  uint32_t                        dmrs_re = 0;
  for (uint32_t k = 0; k != 12; ++k) {
    dmrs_re += (t2 ? (k % 6) < 2 * ncdm : (k % 2) < ncdm) ? 1 : 0;
  }
  uint32_t nof_prb = 0, reserved = 0;
  for (uint32_t r = 0; r != SRS_AMD_MAX_RB; ++r) {
    if (!((m.crb_mask[r / 8] >> (r % 8)) & 1u)) {
      continue;
    }
    ++nof_prb;
    for (uint32_t l = m.start_symbol; l != m.start_symbol + m.nof_symbols; ++l) {
      uint16_t res = 0;
      for (uint32_t q = 0; q != m.nof_reserved; ++q) {
        const srs_amd_re_pattern& pat = m.reserved[q];
        if (((pat.crb_mask[r / 8] >> (r % 8)) & 1u) && ((pat.symbols >> l) & 1u)) {
          res |= pat.re_mask;
        }
      }
      reserved += static_cast<uint32_t>(__builtin_popcount(res & 0xfffu));
    }
  }
  const uint32_t nof_dmrs_symbols = static_cast<uint32_t>(__builtin_popcount(m.dmrs_symbol_mask & 0x3fffu));
  const uint32_t grid_re          = nof_prb * 12 * m.nof_symbols;
  const uint32_t grid_dmrs        = nof_prb * dmrs_re * nof_dmrs_symbols;
  return grid_re > reserved + grid_dmrs ? grid_re - reserved - grid_dmrs : 0;
}

/// The slot collector and the MI355X encoder / modulator shared by every pdsch_processor of one factory.  As the
/// PUSCH engine, a batch runs in two halves: the collector thread uploads the transport blocks and issues the slot
/// encoder, the slot modulator (into the device copy of each hip_resource_grid writer, or into staging grids for
/// host writers) and the staging downloads; the completion thread waits for the batch, merges the written REs of
/// the staging grids into the host writers (a pool of worker threads, one row each) and calls the notifiers.  Two
/// buffer sets alternate between batches.
class pdsch_engine
{
public:
  explicit pdsch_engine(const pdsch_processor_hip_config& c) : cfg(c), nsubc(12 * c.nof_prb), pool(c.nof_copy_threads)
  {
    device = cfg.device;
    if (device < 0 && hipGetDevice(&device) != hipSuccess) {
      throw std::runtime_error("pdsch_processor_hip: hipGetDevice");
    }
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
      throw std::runtime_error("pdsch_processor_hip: device / stream");
    }
    for (auto& bs : sets) {
      if (hipEventCreateWithFlags(&bs.done, hipEventDisableTiming) != hipSuccess) {
        throw std::runtime_error("pdsch_processor_hip: event");
      }
    }
    if (srs_amd_pdsch_encoder_create(&enc, device) != SRS_AMD_OK ||
        srs_amd_pdsch_modulator_create(&mod, device) != SRS_AMD_OK) {
      const std::string e = srs_amd_last_error();
      srs_amd_pdsch_encoder_destroy(enc);
      (void)hipStreamDestroy(stream);
      throw std::runtime_error("pdsch_processor_hip: encoder / modulator: " + e);
    }
    completer = std::thread([this] { complete_loop(); });
    collector = std::make_unique<slot_collector<pending_pdu>>(
        cfg.max_pdus_per_batch, cfg.max_wait_us, [this](std::vector<pending_pdu>& b) { return process(b); });
  }

  ~pdsch_engine()
  {
    collector.reset();
    {
      std::lock_guard<std::mutex> lock(jmtx);
      stop = true;
    }
    jcv.notify_all();
    completer.join();
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    for (auto& kv : plans) {
      srs_amd_pdsch_mod_plan_destroy(kv.second.plan);
    }
    srs_amd_pdsch_modulator_destroy(mod);
    srs_amd_pdsch_encoder_destroy(enc);
    for (auto& bs : sets) {
      (void)hipEventDestroy(bs.done);
    }
    (void)hipStreamDestroy(stream);
  }

  void enqueue(pending_pdu&& p)
  {
    const uint64_t key = (static_cast<uint64_t>(p.numerology) << 32) | p.pdu.slot.slot_index();
    collector->enqueue(std::move(p), key);
  }
  void flush() { collector->flush(); }
  void wait_idle()
  {
    collector->wait_idle();
    std::unique_lock<std::mutex> lock(jmtx);
    jcv.wait(lock, [this] { return jobs.empty() && !completing; });
  }
  pdsch_processor_factory_hip::statistics get_statistics() const
  {
    const auto                              c = collector->get_counters();
    pdsch_processor_factory_hip::statistics s;
    s.nof_pdus         = c.nof_pdus;
    s.nof_batches      = c.nof_batches;
    s.nof_errors       = c.nof_errors + stats_late_errors;
    s.nof_device_grids = stats_device_grids;
    return s;
  }

private:
  struct plan_entry {
    srs_amd_pdsch_mod_plan*          plan   = nullptr;
    uint32_t                         nof_re = 0; // data REs per layer (pdsch_compute_nof_data_re)
    std::list<std::string>::iterator lru;
    uint64_t                         last_seq = 0; // the last batch that used the plan (eviction: completed_seq)
  };

  struct buffer_set {
    hip_mirrored_buffer grids, tbs, cws;
    hipEvent_t          done = nullptr;
    bool                busy = false;
  };

  /// A host writer's staging grid and the region its PDUs wrote.
  struct host_grid {
    resource_grid_writer* writer;
    unsigned              ports = 0, l0 = NSYMB, l1 = 0, k0 = 0, k1 = 0;
  };

  struct job {
    uint64_t                 seq = 0; // dispatch sequence number (plan eviction)
    std::vector<pending_pdu> pdus;
    std::vector<host_grid>   hosts;
    buffer_set*              bs     = nullptr;
    bool                     failed = false;
  };

  plan_entry* plan_of(const srs_amd_pdsch_mod_config& m, std::string& error)
  {
    std::string key(reinterpret_cast<const char*>(&m), sizeof(m));
    auto        it = plans.find(key);
    if (it != plans.end()) {
      lru.splice(lru.begin(), lru, it->second.lru);
      it->second.last_seq = cur_seq;
      return &it->second;
    }
    plan_entry e;
    if (srs_amd_pdsch_mod_plan_create(mod, &m, nsubc, &e.plan, &e.nof_re) != SRS_AMD_OK) {
      error = srs_amd_last_error();
      return nullptr;
    }
    lru.push_front(key);
    e.lru      = lru.begin();
    e.last_seq = cur_seq;
    return &plans.emplace(key, e).first->second;
  }

  // Least recently used plans beyond the cache size, once no dispatched batch can still use them: a plan last used
  // by batch n is free when batch n has completed (batches complete in dispatch order).  (the r05 form
  // evicted only when nothing was in flight, which never happens under back-to-back slots.)
  void evict_plans()
  {
    const uint64_t done = completed_seq.load();
    while (plans.size() > cfg.max_cached_plans && !lru.empty()) {
      auto it = plans.find(lru.back());
      if (it->second.last_seq > done) {
        break; // the least recently used plan may still be in flight, and so may every more recent one
      }
      srs_amd_pdsch_mod_plan_destroy(it->second.plan);
      plans.erase(it);
      lru.pop_back();
    }
  }


  buffer_set* acquire_set()
  {
    std::unique_lock<std::mutex> lock(jmtx);
    for (;;) {
      for (auto& bs : sets) {
        if (!bs.busy) {
          bs.busy = true;
          return &bs;
        }
      }
      jcv.wait(lock);
    }
  }

  unsigned process(std::vector<pending_pdu>& batch)
  {
    const unsigned n      = static_cast<unsigned>(batch.size());
    unsigned       errors = 0;
    auto           done   = [](pending_pdu& p) { p.notifier->on_finish_processing(); };
    if (hipSetDevice(device) != hipSuccess) {
      for (auto& p : batch) {
        done(p);
      }
      return n;
    }
    evict_plans();
    cur_seq = ++dispatch_seq;
    // plans, segmentation, the writers' device grids
    auto                                j = std::make_unique<job>();
    j->seq                                = cur_seq;
    std::vector<plan_entry*>            pl;
    std::vector<srs_amd_pdsch_ue>       ues;
    std::vector<srs_amd_pdsch_slot_pdu> sp;
    std::vector<hip_resource_grid*>     dev_grids; // device-resident writers of the batch
    std::vector<unsigned>               grid_of;
    uint64_t                            tb_total = 0, cw_total = 0;
    for (unsigned i = 0; i != n; ++i) {
      pending_pdu& p = batch[i];
      if (p.error.empty() && (p.grid->get_nof_subc() != nsubc || p.grid->get_nof_ports() < p.mod.nof_ports)) {
        p.error = "resource grid dimensions differ from the processor's";
      }
      plan_entry* pe = nullptr;
      if (p.error.empty()) {
        pe = plan_of(p.mod, p.error);
      }
      srs_amd_pdsch_ue u{};
      if (p.error.empty()) {
        const uint32_t tbs = static_cast<uint32_t>(p.tb->get_buffer().size() * 8);
        const uint32_t bg  = p.pdu.ldpc_base_graph == ldpc_base_graph_type::BG1 ? 1 : 2;
        const uint32_t C   = nof_codeblocks(tbs, bg);
        // pdsch_processor_impl::encode (pdsch_processor_impl.cpp:146-180)
        const uint32_t nre = nof_data_re(p);
        if (nre < pe->nof_re) {
          p.error = "codeword shorter than the REs the modulator maps (the reference's mapper would overrun it)";
        } else if (srs_amd_sch_plan_compute(&u.plan, tbs, bg, p.pdu.codewords[0].rv,
                                            get_bits_per_symbol(p.pdu.codewords[0].modulation),
                                            compute_N_ref(static_cast<uint32_t>(p.pdu.tbs_lbrm.value()), C),
                                            p.mod.nof_layers, nre * p.mod.nof_layers) != SRS_AMD_OK) {
          p.error = srs_amd_last_error();
        }
      }
      if (!p.error.empty()) {
        log_error("PDU not processed", p.error);
        done(p);
        ++errors;
        continue;
      }
      u.tb_offset = tb_total;
      u.cw_offset = cw_total;
      tb_total += (p.tb->get_buffer().size() + 63) / 64 * 64;
      cw_total += (u.plan.cw_length + 511) / 512 * 64;
      hip_resource_grid* hg = hip_grid_of(*p.grid);
      if (hg != nullptr && (hg->device() != device || hg->nof_subc() != nsubc || hg->nof_symbols() != NSYMB)) {
        hg = nullptr; // not usable in place: through the host path
      }
      unsigned g = 0;
      if (hg != nullptr) {
        while (g != dev_grids.size() && dev_grids[g] != hg) {
          ++g;
        }
        if (g == dev_grids.size()) {
          dev_grids.push_back(hg);
        }
        g |= 0x80000000u; // a device grid
      } else {
        while (g != j->hosts.size() && j->hosts[g].writer != p.grid) {
          ++g;
        }
        if (g == j->hosts.size()) {
          j->hosts.push_back(host_grid{p.grid, 0, NSYMB, 0, nsubc, 0});
        }
        // the region of the host writer the PDUs write (rows and subcarriers merged back)
        host_grid&                      h = j->hosts[g];
        const srs_amd_pdsch_mod_config& m = p.mod;
        h.ports                           = std::max(h.ports, m.nof_ports);
        h.l0                              = std::min(h.l0, m.start_symbol);
        h.l1                              = std::max(h.l1, m.start_symbol + m.nof_symbols);
        for (unsigned r = 0; r != SRS_AMD_MAX_RB; ++r) {
          if ((m.crb_mask[r / 8] >> (r % 8)) & 1u) {
            h.k0 = std::min(h.k0, 12 * r);
            h.k1 = std::max(h.k1, 12 * r + 12);
          }
        }
      }
      grid_of.push_back(g);
      ues.push_back(u);
      pl.push_back(pe);
      j->pdus.push_back(std::move(p));
    }
    const size_t m = j->pdus.size();
    if (m == 0) {
      return errors;
    }
    buffer_set*  bs         = acquire_set();
    j->bs                   = bs;
    const size_t grid_words = static_cast<size_t>(MAX_PORTS) * NSYMB * nsubc;
    const size_t nh         = j->hosts.size();
    if (!bs->grids.ensure(std::max<size_t>(nh, 1) * grid_words * 4) || !bs->tbs.ensure(std::max<uint64_t>(tb_total, 64)) ||
        !bs->cws.ensure(std::max<uint64_t>(cw_total, 64))) {
      log_error("batch", "device / pinned buffer allocation");
      for (auto& p : j->pdus) {
        done(p);
      }
      std::lock_guard<std::mutex> lock(jmtx);
      bs->busy = false;
      return n;
    }
    // device grids: made current on this stream (the host's own writes, e.g. PDCCH, uploaded first)
    std::vector<uint32_t*> dptr(dev_grids.size());
    for (size_t g = 0; g != dev_grids.size(); ++g) {
      dptr[g] = dev_grids[g]->device_write(stream);
    }
    stats_device_grids += dev_grids.size();
    for (size_t k = 0; k != m; ++k) {
      const pending_pdu& p = j->pdus[k];
      std::memcpy(bs->tbs.h + ues[k].tb_offset, p.tb->get_buffer().data(), p.tb->get_buffer().size());
      srs_amd_pdsch_slot_pdu s{};
      s.plan      = pl[k]->plan;
      s.dmrs      = &p.dmrs;
      if (p.has_ptrs) {
        pending_pdu& q    = j->pdus[k];
        q.ptrs.weights    = q.ptrs_w.data();
        s.ptrs            = &q.ptrs;
      }
      s.nof_bits  = ues[k].plan.cw_length;
      s.cw_offset = ues[k].cw_offset;
      if (grid_of[k] & 0x80000000u) {
        s.d_grid = dptr[grid_of[k] & 0x7fffffffu];
      } else {
        s.grid = grid_of[k];
      }
      sp.push_back(s);
    }
    hipError_t e = hipMemcpyAsync(bs->tbs.d, bs->tbs.h, tb_total, hipMemcpyHostToDevice, stream);
    e = (e == hipSuccess && nh != 0) ? hipMemsetAsync(bs->grids.d, 0xff, nh * grid_words * 4, stream) : e;
    int rc = e == hipSuccess ? srs_amd_pdsch_encode_slot(enc, ues.data(), static_cast<uint32_t>(ues.size()),
                                                         bs->tbs.d, bs->cws.d, stream)
                             : SRS_AMD_EHIP;
    if (rc == SRS_AMD_OK) {
      rc = srs_amd_pdsch_modulate_slot(mod, sp.data(), static_cast<uint32_t>(sp.size()),
                                       reinterpret_cast<uint32_t*>(bs->grids.d), grid_words,
                                       static_cast<uint32_t>(std::max<size_t>(nh, 1)), nsubc, bs->cws.d, stream);
    }
    for (hip_resource_grid* g : dev_grids) {
      g->device_written(stream); // host accesses and the OFDM modulator wait for the slot call
    }
    e = (rc == SRS_AMD_OK && nh != 0)
            ? hipMemcpyAsync(bs->grids.h, bs->grids.d, nh * grid_words * 4, hipMemcpyDeviceToHost, stream)
            : e;
    e = (rc == SRS_AMD_OK && e == hipSuccess) ? hipEventRecord(bs->done, stream) : e;
    if (rc != SRS_AMD_OK || e != hipSuccess) {
      log_error("slot call", rc != SRS_AMD_OK ? std::string(srs_amd_last_error()) : hipGetErrorString(e));
      (void)hipStreamSynchronize(stream);
      j->failed = true;
    }
    {
      std::lock_guard<std::mutex> lock(jmtx);
      jobs.push_back(std::move(j));
    }
    jcv.notify_all();
    return errors;
  }

  void complete_loop()
  {
    for (;;) {
      std::unique_ptr<job> j;
      {
        std::unique_lock<std::mutex> lock(jmtx);
        jcv.wait(lock, [this] { return stop || !jobs.empty(); });
        if (jobs.empty()) {
          return;
        }
        j = std::move(jobs.front());
        jobs.pop_front();
        completing = true;
      }
      (void)hipSetDevice(device);
      complete(*j);
      completed_seq.store(j->seq); // batches complete in dispatch order
      buffer_set* bs = j->bs;
      j.reset();
      {
        std::lock_guard<std::mutex> lock(jmtx);
        bs->busy   = false;
        completing = false;
      }
      jcv.notify_all();
    }
  }

  void complete(job& j)
  {
    buffer_set* bs = j.bs;
    if (!j.failed) {
      hipError_t e;
      while ((e = hipEventQuery(bs->done)) == hipErrorNotReady) {
        std::this_thread::yield();
      }
      if (e != hipSuccess) {
        log_error("batch", hipGetErrorString(e));
        j.failed = true;
      }
    }
    if (j.failed) {
      stats_late_errors += j.pdus.size();
    } else {
      // the written REs into each host writer (its other REs untouched): one (grid, port, symbol) row per task
      size_t rows = 0;
      for (const host_grid& h : j.hosts) {
        rows += static_cast<size_t>(h.ports) * (h.l1 > h.l0 ? h.l1 - h.l0 : 0);
      }
      std::vector<std::pair<unsigned, unsigned>> index; // (host grid, row within it)
      index.reserve(rows);
      for (unsigned g = 0; g != j.hosts.size(); ++g) {
        const host_grid& h = j.hosts[g];
        for (unsigned r = 0; r != h.ports * (h.l1 > h.l0 ? h.l1 - h.l0 : 0); ++r) {
          index.emplace_back(g, r);
        }
      }
      const size_t grid_words = static_cast<size_t>(MAX_PORTS) * NSYMB * nsubc;
      pool.run(index.size(), [&](size_t t) {
        const host_grid& h  = j.hosts[index[t].first];
        const unsigned   nl = h.l1 - h.l0;
        const unsigned   q  = index[t].second / nl;
        const unsigned   l  = h.l0 + index[t].second % nl;
        span<cbf16_t>    view = h.writer->get_view(q, l);
        const uint32_t*  src  = reinterpret_cast<const uint32_t*>(bs->grids.h) + index[t].first * grid_words +
                              (static_cast<size_t>(q) * NSYMB + l) * nsubc;
        auto*          dst = reinterpret_cast<uint32_t*>(view.data());
        const unsigned k1  = std::min<unsigned>(h.k1, static_cast<unsigned>(view.size()));
        for (unsigned k = h.k0; k < k1; ++k) {
          const uint32_t v = src[k];
          if (v != SENTINEL) {
            dst[k] = v;
          }
        }
      });
    }
    for (auto& p : j.pdus) {
      p.notifier->on_finish_processing();
    }
  }

public:
  std::atomic<uint64_t> stats_late_errors{0}, stats_device_grids{0};

private:
  pdsch_processor_hip_config                  cfg;
  const unsigned                              nsubc;
  int                                         device = 0;
  hipStream_t                                 stream = nullptr;
  srs_amd_pdsch_encoder*                      enc    = nullptr;
  srs_amd_pdsch_modulator*                    mod    = nullptr;
  std::unordered_map<std::string, plan_entry> plans;
  std::list<std::string>                      lru;
  row_pool                                    pool;
  buffer_set                                  sets[2];
  std::mutex                                  jmtx;
  std::condition_variable                     jcv;
  std::deque<std::unique_ptr<job>>            jobs;
  bool                                        completing = false, stop = false;
  uint64_t                          dispatch_seq = 0, cur_seq = 0; // collector thread: batches dispatched / this one
  std::atomic<uint64_t>             completed_seq{0};              // the last batch the completion thread finished
  std::thread                                 completer;
  std::unique_ptr<slot_collector<pending_pdu>> collector; // last: stops before the state it uses goes
};

class pdsch_processor_hip : public pdsch_processor
{
public:
  pdsch_processor_hip(std::shared_ptr<pdsch_engine> e, unsigned nof_prb_) : engine(std::move(e)), nof_prb(nof_prb_) {}

  void process(resource_grid_writer&                                           grid,
               pdsch_processor_notifier&                                       notifier,
               static_vector<shared_transport_block, MAX_NOF_TRANSPORT_BLOCKS> data,
               const pdu_t&                                                    pdu) override
  {
    pending_pdu p;
    p.grid     = &grid;
    p.notifier = &notifier;
    p.pdu      = pdu;
    if (data.empty()) {
      p.error = "no transport block";
    } else {
      p.tb.emplace(data[0]);
      p.error = convert(p, nof_prb);
    }
    engine->enqueue(std::move(p));
  }

private:
  std::shared_ptr<pdsch_engine> engine;
  unsigned                      nof_prb;
};

class pdsch_pdu_validator_hip : public pdsch_pdu_validator
{
public:
  explicit pdsch_pdu_validator_hip(unsigned nof_prb_) : nof_prb(nof_prb_) {}
  error_type<std::string> is_valid(const pdsch_processor::pdu_t& pdu) const override
  {
    pending_pdu p;
    p.pdu               = pdu;
    const std::string e = convert(p, nof_prb);
    if (!e.empty()) {
      return make_unexpected(e);
    }
    return default_success_t();
  }

private:
  unsigned nof_prb;
};

class pdsch_processor_factory_hip_impl : public pdsch_processor_factory_hip
{
public:
  explicit pdsch_processor_factory_hip_impl(const pdsch_processor_hip_config& c) :
    cfg(c), engine(std::make_shared<pdsch_engine>(c))
  {
  }
  std::unique_ptr<pdsch_processor> create() override { return std::make_unique<pdsch_processor_hip>(engine, cfg.nof_prb); }
  // The reference wraps its processors in its logging decorator (factories.cpp:474); the MI355X processors log
  // their errors themselves.
  std::unique_ptr<pdsch_processor> create(srslog::basic_logger& /*logger*/, bool /*enable_logging_broadcast*/) override
  {
    return create();
  }
  std::unique_ptr<pdsch_pdu_validator> create_validator() override
  {
    return std::make_unique<pdsch_pdu_validator_hip>(cfg.nof_prb);
  }
  void       flush() override { engine->flush(); }
  void       wait_idle() override { engine->wait_idle(); }
  statistics get_statistics() const override { return engine->get_statistics(); }

private:
  pdsch_processor_hip_config    cfg;
  std::shared_ptr<pdsch_engine> engine;
};

} // namespace

std::shared_ptr<pdsch_processor_factory_hip>
srsran::hip::create_pdsch_processor_factory_hip(const pdsch_processor_hip_config& cfg)
{
  try {
    return std::make_shared<pdsch_processor_factory_hip_impl>(cfg);
  } catch (const std::exception& e) {
    log_error("factory", e.what());
    return nullptr;
  }
}
