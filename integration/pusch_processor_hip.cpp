// pusch_processor_hip.cpp -- srsran::pusch_processor over the srsran_amd slot C-ABI (see the header).
#include "pusch_processor_hip.h"
#include "hip_resource_grid.h"
#include "slot_collector.h"

#include "srsran/adt/bit_buffer.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_processor_result_notifier.h"
#include "srsran/phy/upper/rx_buffer.h"
#include "srsran/phy/upper/unique_rx_buffer.h"
#include "srsran/ran/sch/modulation_scheme.h"
#include "srsran_amd/pusch_processor.h"
#include "srsran_amd/sch.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <list>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

using namespace srsran;
using namespace srsran::hip;

namespace {

constexpr unsigned MAX_PORTS_HIP = 4;   // receive ports per PDU (srs_amd_pusch_process_slot_ex port measurements)
constexpr unsigned MAX_CB        = 512; // codeblocks of one transport block
constexpr unsigned NSYMB         = 14;  // OFDM symbols of a normal-CP slot

void log_error(const char* what, const std::string& detail)
{
  std::fprintf(stderr, "pusch_processor_hip: %s: %s\n", what, detail.c_str());
}

/// pusch_decoder_impl's cb_stats of one processor instance: the last LDPC count of each codeblock index.
using cb_stat_array = std::array<unsigned, MAX_CB>;

/// One queued process() call.
struct pending_pdu {
  span<uint8_t>                    data;
  unique_rx_buffer                 rm_buffer;
  pusch_processor_result_notifier* notifier = nullptr;
  const resource_grid_reader*      grid     = nullptr;
  pusch_processor::pdu_t           pdu;
  srs_amd_pusch_pdu                c{};
  std::vector<uint8_t>             rx_ports;
  std::string                      error; // not supported: reported as a failed transmission
  std::shared_ptr<cb_stat_array>   cb_stats;
};

// pdu_t -> srs_amd_pusch_pdu (the fields pusch_processor_impl.cpp:134-386 reads); an empty string when supported.
std::string convert(const pusch_processor::pdu_t& pdu, size_t tb_bytes, srs_amd_pusch_pdu& c)
{
  c = srs_amd_pusch_pdu{};
  if (!pdu.codeword.has_value() && (tb_bytes != 0 || (pdu.uci.nof_harq_ack == 0 && pdu.uci.nof_csi_part1 == 0))) {
    return "PUSCH without a codeword must carry UCI and no transport block";
  }
  if (pdu.cp != cyclic_prefix::NORMAL) {
    return "extended cyclic prefix";
  }
  if (pdu.rx_ports.empty() || pdu.rx_ports.size() > MAX_PORTS_HIP || pdu.nof_tx_layers == 0 ||
      pdu.nof_tx_layers > pdu.rx_ports.size()) {
    return "receive ports / layers outside 1..4";
  }
  if (!pdu.freq_alloc.is_contiguous()) {
    return "non-contiguous or interleaved frequency allocation";
  }
  const bool tp = std::holds_alternative<pusch_processor::dmrs_transform_precoding_configuration>(pdu.dmrs);
  // the DC subcarrier's estimate is zeroed for CP-OFDM by the processor (pusch_processor_impl.cpp:235-249)
  if (pdu.dc_position.has_value()) {
    c.has_dc_position = 1;
    c.dc_position     = static_cast<uint32_t>(*pdu.dc_position);
  }
  c.numerology       = to_numerology_value(pdu.slot.scs());
  c.slot_index       = pdu.slot.slot_index();
  c.rnti             = pdu.rnti;
  c.bwp_start_rb     = pdu.bwp_start_rb;
  c.bwp_size_rb      = pdu.bwp_size_rb;
  c.target_code_rate = pdu.mcs_descr.target_code_rate;
  switch (pdu.mcs_descr.modulation) {
    case modulation_scheme::PI_2_BPSK:
      c.modulation = 0;
      break;
    case modulation_scheme::BPSK:
      c.modulation = 1;
      break;
    default:
      c.modulation = static_cast<int32_t>(get_bits_per_symbol(pdu.mcs_descr.modulation));
  }
  // UCI only (no codeword, tbs = 0): no UL-SCH to decode, nothing kept between transmissions
  c.rv            = pdu.codeword.has_value() ? pdu.codeword->rv : 0;
  c.base_graph    = pdu.codeword.has_value() && pdu.codeword->ldpc_base_graph == ldpc_base_graph_type::BG2 ? 2 : 1;
  c.new_data      = pdu.codeword.has_value() && !pdu.codeword->new_data ? 0 : 1;
  c.n_id          = pdu.n_id;
  c.nof_tx_layers = pdu.nof_tx_layers;
  c.nof_rx_ports  = static_cast<uint32_t>(pdu.rx_ports.size());
  for (unsigned l = 0; l != NSYMB && l < pdu.dmrs_symbol_mask.size(); ++l) {
    c.dmrs_symbol_mask |= pdu.dmrs_symbol_mask.test(l) ? (1u << l) : 0u;
  }
  if (tp) {
    c.transform_precoding = 1;
    c.n_rs_id             = std::get<pusch_processor::dmrs_transform_precoding_configuration>(pdu.dmrs).n_rs_id;
    c.dmrs_type           = 1;
    c.nof_cdm_groups_without_data = 2;
  } else {
    const auto& d                 = std::get<pusch_processor::dmrs_configuration>(pdu.dmrs);
    c.dmrs_type                   = d.dmrs == dmrs_type::TYPE1 ? 1 : 2;
    c.scrambling_id               = d.scrambling_id;
    c.n_scid                      = d.n_scid ? 1 : 0;
    c.nof_cdm_groups_without_data = d.nof_cdm_groups_without_data;
  }
  // the allocation's CRBs (pusch_processor_impl.cpp:166 get_crb_mask), contiguous: [rb_start, +rb_count) of the BWP
  const crb_bitmap crbs = pdu.freq_alloc.get_crb_mask(pdu.bwp_start_rb, pdu.bwp_size_rb);
  if (crbs.none() || static_cast<unsigned>(crbs.find_lowest()) < pdu.bwp_start_rb) {
    return "empty frequency allocation";
  }
  c.rb_start           = static_cast<uint32_t>(crbs.find_lowest()) - pdu.bwp_start_rb;
  c.rb_count           = static_cast<uint32_t>(crbs.count());
  c.start_symbol_index = pdu.start_symbol_index;
  c.nof_symbols        = pdu.nof_symbols;
  c.tbs_lbrm_bytes     = static_cast<uint32_t>(pdu.tbs_lbrm.value());
  c.tbs                = static_cast<uint32_t>(tb_bytes * 8);
  c.nof_harq_ack          = pdu.uci.nof_harq_ack;
  c.nof_csi_part1         = pdu.uci.nof_csi_part1;
  c.alpha_scaling         = pdu.uci.alpha_scaling;
  c.beta_offset_harq_ack  = pdu.uci.beta_offset_harq_ack;
  c.beta_offset_csi_part1 = pdu.uci.beta_offset_csi_part1;
  c.beta_offset_csi_part2 = pdu.uci.beta_offset_csi_part2;
  const auto& entries     = pdu.uci.csi_part2_size.entries;
  if (entries.size() > 2) {
    return "more than two CSI part 2 size entries";
  }
  c.csi_part2_size.nof_entries = static_cast<uint32_t>(entries.size());
  for (size_t e = 0; e != entries.size(); ++e) {
    srs_amd_uci_part2_entry& en = c.csi_part2_size.entries[e];
    if (entries[e].parameters.size() > 2 || entries[e].map.size() > 16) {
      return "CSI part 2 size entry beyond two parameters / 16 map values";
    }
    en.nof_parameters = static_cast<uint32_t>(entries[e].parameters.size());
    for (size_t q = 0; q != entries[e].parameters.size(); ++q) {
      en.parameters[q].offset = entries[e].parameters[q].offset;
      en.parameters[q].width  = entries[e].parameters[q].width;
    }
    en.map_size = static_cast<uint32_t>(entries[e].map.size());
    for (size_t m = 0; m != entries[e].map.size(); ++m) {
      en.map[m] = entries[e].map[m];
    }
  }
  return {};
}

/// The slot collector and the MI355X processor shared by every pusch_processor of one factory.
///
/// A batch runs in two halves on two threads, so consecutive batches overlap: the collector thread stages the batch
/// (grid rows copied into pinned memory by a pool of worker threads, or the device grid of a hip_resource_grid taken
/// as it is), issues the uploads, the slot call and the downloads on the engine's stream and hands the batch to the
/// completion thread; the completion thread waits for that batch's event, runs the HARQ soft-buffer pass for failed
/// new transmissions, writes HARQ state back into the rx_buffers and calls the notifiers.  Two sets of pinned /
/// device buffers alternate between batches (a set is reused once its batch has been notified).
class slot_engine
{
public:
  explicit slot_engine(const pusch_processor_hip_config& c) :
    cfg(c), nsubc(12 * c.nof_prb), pool(c.nof_copy_threads), npool(c.nof_notify_threads)
  {
    device = cfg.device;
    if (device < 0 && hipGetDevice(&device) != hipSuccess) {
      throw std::runtime_error("pusch_processor_hip: hipGetDevice");
    }
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking) != hipSuccess) {
      throw std::runtime_error("pusch_processor_hip: device / stream");
    }
    for (auto& bs : sets) {
      if (hipEventCreateWithFlags(&bs.done, hipEventDisableTiming) != hipSuccess) {
        throw std::runtime_error("pusch_processor_hip: event");
      }
    }
    srs_amd_pusch_processor_config pc{};
    pc.dec_nof_iterations    = cfg.dec_nof_iterations;
    pc.dec_enable_early_stop = cfg.dec_enable_early_stop ? 1 : 0;
    pc.dec_force_decoding    = cfg.dec_force_decoding ? 1 : 0;
    pc.equalizer        = cfg.equalizer == channel_equalizer_algorithm_type::mmse ? SRS_AMD_EQ_MMSE : SRS_AMD_EQ_ZF;
    pc.fd_smoothing     = static_cast<int32_t>(cfg.fd_smoothing);
    pc.td_interpolation = static_cast<int32_t>(cfg.td_interpolation);
    pc.compensate_cfo   = cfg.compensate_cfo ? 1 : 0;
    pc.ldpc_arith       = cfg.generic_ldpc ? SRS_AMD_ARITH_GENERIC : SRS_AMD_ARITH_SIMD;
    if (srs_amd_pusch_processor_create(&proc, &pc, device) != SRS_AMD_OK) {
      const std::string e = srs_amd_last_error();
      (void)hipStreamDestroy(stream);
      (void)hipStreamDestroy(stream2);
      throw std::runtime_error("pusch_processor_hip: processor: " + e);
    }
    completer = std::thread([this] { complete_loop(); });
    collector = std::make_unique<slot_collector<pending_pdu>>(
        cfg.max_pdus_per_batch, cfg.max_wait_us, [this](std::vector<pending_pdu>& b) { return process(b); });
  }

  ~slot_engine()
  {
    collector.reset(); // processes what is pending, joins the collector thread
    {
      std::lock_guard<std::mutex> lock(jmtx);
      stop = true;
    }
    jcv.notify_all();
    completer.join(); // notifies what is in flight
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    (void)hipStreamSynchronize(stream2);
    for (auto& kv : plans) {
      srs_amd_pusch_processor_plan_destroy(kv.second.plan);
    }
    srs_amd_pusch_processor_destroy(proc);
    for (auto& bs : sets) {
      (void)hipEventDestroy(bs.done);
    }
    (void)hipStreamDestroy(stream);
    (void)hipStreamDestroy(stream2);
  }

  void enqueue(pending_pdu&& p)
  {
    const uint64_t key = (static_cast<uint64_t>(p.c.numerology) << 32) | p.c.slot_index;
    collector->enqueue(std::move(p), key);
  }

  void flush() { collector->flush(); }

  // every queued PDU dispatched (collector), then every dispatched batch notified (completion thread)
  void wait_idle()
  {
    collector->wait_idle();
    std::unique_lock<std::mutex> lock(jmtx);
    jcv.wait(lock, [this] { return jobs.empty() && !completing; });
  }

  pusch_processor_factory_hip::statistics get_statistics() const
  {
    const auto                              c = collector->get_counters();
    pusch_processor_factory_hip::statistics s;
    s.nof_pdus            = c.nof_pdus;
    s.nof_batches         = c.nof_batches;
    s.nof_errors          = c.nof_errors + stats_late_errors;
    s.nof_harq_redecodes  = 0; // one decoding per PDU: a failed new transmission's soft buffer is downloaded
    s.nof_harq_soft_downloads = stats_soft_downloads;
    s.nof_retransmissions = stats_retx;
    s.nof_device_grids    = stats_device_grids;
    s.stage_us            = t_stage / 1000;
    s.set_wait_us         = t_set_wait / 1000;
    s.wait_us             = t_wait / 1000;
    s.notify_us           = t_notify / 1000;
    s.stage_reads_us      = t_reads / 1000;
    s.stage_call_us       = t_call / 1000;
    s.stage_download_us   = t_download / 1000;
    return s;
  }

private:
  struct plan_entry {
    srs_amd_pusch_processor_plan*    plan    = nullptr;
    uint32_t                         nof_cbs = 0, max_csi2 = 0;
    uint64_t                         soft_bytes = 0;
    srs_amd_sch_plan                 sch{};
    std::list<std::string>::iterator lru;
    uint64_t                         last_seq = 0; // the last batch that used the plan (eviction: completed_seq)
  };

  /// One alternating set of the batch's pinned / device buffers.
  struct buffer_set {
    hip_mirrored_buffer h_grids, tbs, results, cbi, uci, pstats, soft;
    hipEvent_t          done = nullptr; // the batch's downloads
    bool                busy = false;
  };

  /// A dispatched batch, waiting for its completion.
  struct job {
    uint64_t                            seq = 0;  // dispatch sequence number (plan eviction)
    std::vector<pending_pdu>            pdus;     // the live PDUs, in slot-call order
    std::vector<plan_entry>             pl;       // their plans (copies: eviction waits for idle)
    std::vector<srs_amd_pusch_slot_pdu> sp;       // the slot call's PDUs
    std::vector<uint64_t>               tb_off, uci_off, soft_off;
    std::vector<uint32_t>               cb_off;
    std::vector<std::vector<char>>      prev_ok;  // CB CRC flags of the rx_buffer before the call
    uint64_t                            soft_total = 0, tb_total = 0, uci_total = 0;
    uint32_t                            cb_total   = 0;
    size_t                              nof_grids = 0, grid_stride = 0;
    buffer_set*                         bs = nullptr;
    bool                                failed = false; // the slot call failed: every PDU reported as failed
  };

  // Plan of a PDU configuration (cached across slots, least recently used evicted when no batch is in flight).
  plan_entry* plan_of(const srs_amd_pusch_pdu& c, std::string& error)
  {
    srs_amd_pusch_pdu k = c;
    k.numerology = k.slot_index = 0;
    std::string key(reinterpret_cast<const char*>(&k), sizeof(k));
    auto        it = plans.find(key);
    if (it == plans.end()) {
      plan_entry e;
      if (srs_amd_pusch_processor_plan_create(proc, &c, nsubc, &e.plan, &e.sch, &e.soft_bytes) != SRS_AMD_OK) {
        error = srs_amd_last_error();
        return nullptr;
      }
      (void)srs_amd_pusch_processor_plan_info(e.plan, &e.nof_cbs, &e.max_csi2, nullptr);
      lru.push_front(key);
      e.lru = lru.begin();
      it    = plans.emplace(key, e).first;
    } else {
      lru.splice(lru.begin(), lru, it->second.lru);
    }
    // the plan is shared by every slot of this configuration: each PDU carries its own slot in the slot call
    // (srs_amd_pusch_slot_pdu::has_slot), so PDUs of two slots in one batch keep their own DM-RS sequences
    it->second.last_seq = cur_seq;
    return &it->second;
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
      srs_amd_pusch_processor_plan_destroy(it->second.plan);
      plans.erase(it);
      lru.pop_back();
    }
  }


  // A transmission that could not be processed: the reference's "no dependencies" notification
  // (pusch_processor_impl.cpp:140-157).
  static void notify_failure(pending_pdu& p)
  {
    if (p.pdu.uci.nof_harq_ack != 0) {
      pusch_processor_result_control uci;
      uci.harq_ack.payload = uci_payload_type(p.pdu.uci.nof_harq_ack);
      uci.harq_ack.status  = uci_status::invalid;
      p.notifier->on_uci(uci);
    }
    if (p.rm_buffer.is_valid()) {
      p.rm_buffer.unlock();
    }
    if (p.pdu.codeword.has_value()) {
      p.notifier->on_sch({});
    }
  }

  // A free buffer set (waits for the completion thread to release one).
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

  void release_set(buffer_set* bs)
  {
    {
      std::lock_guard<std::mutex> lock(jmtx);
      bs->busy = false;
    }
    jcv.notify_all();
  }

  // Collector thread: stages and dispatches one batch; returns the number of PDUs reported as failed here.
  unsigned process(std::vector<pending_pdu>& batch)
  {
    const auto t_begin = std::chrono::steady_clock::now();
    struct stage_timer {
      std::atomic<uint64_t>&                t;
      std::chrono::steady_clock::time_point t0;
      ~stage_timer()
      {
        t += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
      }
    } timer{t_stage, t_begin};
    const unsigned n      = static_cast<unsigned>(batch.size());
    unsigned       errors = 0;
    if (hipSetDevice(device) != hipSuccess) {
      for (auto& p : batch) {
        notify_failure(p);
      }
      return n;
    }
    evict_plans();
    cur_seq = ++dispatch_seq;
    auto j = std::make_unique<job>();
    j->seq = cur_seq;
    // plans, and the PDUs that go to the GPU
    for (unsigned i = 0; i != n; ++i) {
      pending_pdu& p  = batch[i];
      plan_entry*  pe = nullptr;
      if (p.error.empty()) {
        pe = plan_of(p.c, p.error);
      }
      if (p.error.empty() && !p.c.new_data && !p.rm_buffer.is_valid()) {
        p.error = "retransmission without a valid rx_buffer";
      }
      if (p.error.empty() && p.rm_buffer.is_valid() && p.rm_buffer.get().get_nof_codeblocks() != pe->nof_cbs) {
        p.error = "rx_buffer codeblock count differs from the transport block's";
      }
      if (!p.error.empty()) {
        log_error("PDU not processed", p.error);
        notify_failure(p);
        ++errors;
        continue;
      }
      j->pdus.push_back(std::move(p));
      j->pl.push_back(*pe);
    }
    const size_t m = j->pdus.size();
    if (m == 0) {
      return errors;
    }
    const auto  t_acq = std::chrono::steady_clock::now();
    buffer_set* bs    = acquire_set();
    t_set_wait += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_acq).count();
    j->bs = bs;
    // receive grids: a hip_resource_grid's device copy as it is (receive ports 0 .. P - 1); otherwise one staged
    // device grid per (reader, port list), a PDU whose ports are a prefix of another PDU's list on the same reader
    // sharing that grid
    std::vector<const uint32_t*> dev_grid(m, nullptr);
    const auto                   t_r0 = std::chrono::steady_clock::now();
    for (size_t k = 0; k != m; ++k) {
      const pending_pdu& p  = j->pdus[k];
      hip_resource_grid* hg = hip_grid_of(*p.grid);
      bool               ok = hg != nullptr && hg->device() == device && hg->nof_subc() == nsubc &&
                hg->nof_symbols() == NSYMB && p.rx_ports.size() <= hg->nof_ports();
      for (size_t q = 0; ok && q != p.rx_ports.size(); ++q) {
        ok = p.rx_ports[q] == q;
      }
      if (ok) {
        dev_grid[k] = hg->device_read(stream); // the engine's stream waits for the grid's producer
        ++stats_device_grids;
      }
    }
    t_reads += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_r0).count();
    std::unordered_map<const resource_grid_reader*, std::vector<uint8_t>> longest;
    for (size_t k = 0; k != m; ++k) {
      if (dev_grid[k] != nullptr) {
        continue;
      }
      auto& l = longest[j->pdus[k].grid];
      if (j->pdus[k].rx_ports.size() > l.size() && std::equal(l.begin(), l.end(), j->pdus[k].rx_ports.begin())) {
        l = j->pdus[k].rx_ports;
      }
    }
    struct grid_slot {
      const resource_grid_reader* reader;
      std::vector<uint8_t>        ports;
    };
    std::vector<grid_slot> grids;
    std::vector<unsigned>  grid_of(m, 0);
    for (size_t k = 0; k != m; ++k) {
      if (dev_grid[k] != nullptr) {
        continue;
      }
      const auto&          ports = j->pdus[k].rx_ports;
      const auto&          l     = longest[j->pdus[k].grid];
      std::vector<uint8_t> want  = std::equal(ports.begin(), ports.end(), l.begin()) ? l : ports;
      unsigned             g     = 0;
      while (g != grids.size() && !(grids[g].reader == j->pdus[k].grid && grids[g].ports == want)) {
        ++g;
      }
      if (g == grids.size()) {
        grids.push_back(grid_slot{j->pdus[k].grid, want});
      }
      grid_of[k] = g;
    }
    j->grid_stride = static_cast<size_t>(MAX_PORTS_HIP) * NSYMB * nsubc; // uint32 words
    j->nof_grids   = grids.size();
    // per-PDU offsets in the output / HARQ buffers
    j->tb_off.resize(m);
    j->uci_off.resize(m);
    j->soft_off.resize(m);
    j->cb_off.resize(m);
    j->prev_ok.resize(m);
    uint64_t tb_total = 0, uci_total = 0, soft_total = 0;
    uint32_t cb_total = 0;
    for (size_t k = 0; k != m; ++k) {
      j->tb_off[k]   = tb_total;
      j->uci_off[k]  = uci_total;
      j->cb_off[k]   = cb_total;
      j->soft_off[k] = soft_total;
      tb_total += (j->pdus[k].data.size() + 63) / 64 * 64;
      uci_total += j->pdus[k].c.nof_harq_ack + j->pdus[k].c.nof_csi_part1 + j->pl[k].max_csi2;
      cb_total += j->pl[k].nof_cbs;
      // soft buffers for retransmissions and for a second pass over failed new transmissions
      if (j->pdus[k].rm_buffer.is_valid()) {
        soft_total += (j->pl[k].soft_bytes + 255) / 256 * 256;
      }
    }
    j->soft_total = soft_total;
    j->tb_total   = tb_total;
    j->uci_total  = uci_total;
    j->cb_total   = cb_total;
    const bool ok = bs->h_grids.ensure(std::max<size_t>(grids.size(), 1) * j->grid_stride * 4) &&
                    bs->tbs.ensure(std::max<uint64_t>(tb_total, 64)) &&
                    bs->results.ensure(sizeof(srs_amd_pusch_processor_result) * m) &&
                    bs->cbi.ensure(sizeof(int32_t) * std::max<uint32_t>(cb_total, 1)) &&
                    bs->uci.ensure(std::max<uint64_t>(uci_total, 64)) &&
                    bs->pstats.ensure(sizeof(srs_amd_chest_port_stats) * MAX_PORTS_HIP * m) &&
                    bs->soft.ensure(std::max<uint64_t>(soft_total, 256));
    if (!ok) {
      log_error("batch", "device / pinned buffer allocation");
      for (auto& p : j->pdus) {
        notify_failure(p);
      }
      release_set(bs);
      return n;
    }
    // grid rows from the readers (a view per port and OFDM symbol), copied by the worker pool
    const size_t rows_per_grid = MAX_PORTS_HIP * NSYMB;
    pool.run(grids.size() * rows_per_grid, [&](size_t r) {
      const size_t g = r / rows_per_grid, q = (r / NSYMB) % MAX_PORTS_HIP;
      const auto   l = static_cast<unsigned>(r % NSYMB);
      if (q >= grids[g].ports.size()) {
        return;
      }
      span<const cbf16_t> v   = grids[g].reader->get_view(grids[g].ports[q], l);
      uint8_t*            dst = bs->h_grids.h + ((g * MAX_PORTS_HIP + q) * NSYMB + l) * nsubc * 4;
      if (v.size() >= nsubc) {
        std::memcpy(dst, v.data(), nsubc * 4);
      } else {
        std::memset(dst, 0, nsubc * 4);
      }
    });
    // retransmissions: the rx_buffer's state into the device soft buffer
    for (size_t k = 0; k != m; ++k) {
      if (!j->pdus[k].c.new_data) {
        upload_harq(j->pdus[k], j->pl[k], bs->soft.h + j->soft_off[k], j->prev_ok[k]);
        ++stats_retx;
      }
    }
    // the slot call
    for (size_t k = 0; k != m; ++k) {
      srs_amd_pusch_slot_pdu u{};
      u.plan       = j->pl[k].plan;
      u.grid       = grid_of[k];
      u.d_grid     = dev_grid[k];
      u.cb_offset  = j->cb_off[k];
      u.tb_offset  = j->tb_off[k];
      // a PDU with an rx_buffer decodes into its device soft buffer: a retransmission combines with it, a new
      // transmission keeps its soft LLRs only when its TB fails (soft_on_failure), as the reference's single decode
      // leaves them in the rx_buffer it then unlocks (pusch_decoder_impl.cpp:324-360)
      u.d_soft          = j->pdus[k].rm_buffer.is_valid() ? reinterpret_cast<int8_t*>(bs->soft.d + j->soft_off[k])
                                                          : nullptr;
      u.soft_on_failure = j->pdus[k].c.new_data ? 1u : 0u;
      u.uci_offset = j->uci_off[k];
      u.has_slot   = 1;
      u.numerology = j->pdus[k].c.numerology;
      u.slot_index = j->pdus[k].c.slot_index;
      j->sp.push_back(u);
    }
    hipError_t e = grids.empty() ? hipSuccess
                                 : hipMemcpyAsync(bs->h_grids.d, bs->h_grids.h, grids.size() * j->grid_stride * 4,
                                                  hipMemcpyHostToDevice, stream);
    // retransmissions' soft buffers up (new transmissions start from a cleared buffer on the device)
    for (size_t k = 0; k != m && e == hipSuccess; ++k) {
      if (!j->pdus[k].c.new_data) {
        e = hipMemcpyAsync(bs->soft.d + j->soft_off[k], bs->soft.h + j->soft_off[k], j->pl[k].soft_bytes,
                           hipMemcpyHostToDevice, stream);
      }
    }
    const auto t_c0 = std::chrono::steady_clock::now();
    int        rc   = e == hipSuccess ? run_slot(*j, j->sp, stream) : SRS_AMD_EHIP;
    const auto t_c1 = std::chrono::steady_clock::now();
    e               = rc == SRS_AMD_OK ? download(*j, stream) : hipErrorUnknown;
    e               = e == hipSuccess ? hipEventRecord(bs->done, stream) : e;
    t_call += std::chrono::duration_cast<std::chrono::nanoseconds>(t_c1 - t_c0).count();
    t_download += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_c1).count();
    if (rc != SRS_AMD_OK || e != hipSuccess) {
      log_error("slot call", rc != SRS_AMD_OK ? std::string(srs_amd_last_error()) : hipGetErrorString(e));
      (void)hipStreamSynchronize(stream);
      j->failed = true;
    }
    // to the completion thread
    {
      std::lock_guard<std::mutex> lock(jmtx);
      jobs.push_back(std::move(j));
    }
    jcv.notify_all();
    return errors;
  }

  // Completion thread: notifies the dispatched batches in order.
  void complete_loop()
  {
    for (;;) {
      std::unique_ptr<job> j;
      {
        std::unique_lock<std::mutex> lock(jmtx);
        jcv.wait(lock, [this] { return stop || !jobs.empty(); });
        if (jobs.empty()) {
          return; // stop, nothing in flight
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
    const size_t m = j.pdus.size();
    const auto   t_begin = std::chrono::steady_clock::now();
    if (!j.failed) {
      // poll the batch's event: an interrupt-driven wait could oversleep (device_buffer.h event_wait_spin)
      hipError_t e;
      while ((e = hipEventQuery(bs->done)) == hipErrorNotReady) {
        std::this_thread::yield();
      }
      if (e != hipSuccess) {
        log_error("batch", hipGetErrorString(e));
        j.failed = true;
      }
    }
    const auto t_ready = std::chrono::steady_clock::now();
    t_wait += std::chrono::duration_cast<std::chrono::nanoseconds>(t_ready - t_begin).count();
    struct notify_timer {
      std::atomic<uint64_t>&                t;
      std::chrono::steady_clock::time_point t0;
      ~notify_timer()
      {
        t += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
      }
    } timer{t_notify, t_ready};
    if (j.failed) {
      stats_late_errors += m;
      for (auto& p : j.pdus) {
        notify_failure(p);
      }
      return;
    }
    // new transmissions whose TB CRC failed and that keep HARQ state: the first (and only) decoding left their soft
    // LLRs, messages and CRC flags in the device soft buffer -- downloaded now (failed TBs only), then written to the
    // rx_buffer
    const auto*           res = reinterpret_cast<const srs_amd_pusch_processor_result*>(bs->results.h);
    std::vector<char>     keep(m, 0); // the rx_buffer takes the soft buffer's state after the call
    std::vector<unsigned> failed;
    for (size_t k = 0; k != m; ++k) {
      keep[k] = !j.pdus[k].c.new_data;
      if (j.pdus[k].c.new_data && j.pdus[k].c.tbs != 0 && j.pdus[k].rm_buffer.is_valid() && !res[k].data.tb_crc_ok) {
        failed.push_back(static_cast<unsigned>(k));
      }
    }
    if (!failed.empty()) {
      stats_soft_downloads += failed.size();
      hipError_t e = hipSuccess;
      for (unsigned k : failed) {
        e = e == hipSuccess ? hipMemcpyAsync(bs->soft.h + j.soft_off[k], bs->soft.d + j.soft_off[k], j.pl[k].soft_bytes,
                                             hipMemcpyDeviceToHost, stream2)
                            : e;
      }
      e = e == hipSuccess ? hipStreamSynchronize(stream2) : e;
      if (e != hipSuccess) {
        // the rx_buffers are left as they were (the transport blocks report their CRC failure either way)
        log_error("HARQ soft-buffer download", hipGetErrorString(e));
        (void)hipStreamSynchronize(stream2);
      } else {
        for (unsigned k : failed) {
          keep[k] = 1;
        }
      }
    }
    // results, HARQ state back into the rx_buffers, notifications: the batch's PDUs in parallel on the notification
    // pool (the transport-block copies out of pinned memory dominate: ~140 KB per 273-PRB 4-layer PDU), as the
    // reference's PUSCH executor threads notify their PDUs concurrently
    npool.run(m, [&](size_t k) {
      pending_pdu& p = j.pdus[k];
      if (keep[k]) {
        store_harq(p, j.pl[k], bs->soft.h + j.soft_off[k]);
      }
      notify(p, j.pl[k], res[k], reinterpret_cast<const int32_t*>(bs->cbi.h) + j.cb_off[k], j.prev_ok[k],
             bs->tbs.h + j.tb_off[k], bs->uci.h + j.uci_off[k],
             reinterpret_cast<const srs_amd_chest_port_stats*>(bs->pstats.h) + k * MAX_PORTS_HIP);
    });
  }

  // srs_amd_pusch_process_slot_ex on the batch's device buffers; ids: the index of each PDU in the outputs (the
  // second pass writes into the first pass's rows).
  int run_slot(job& j, std::vector<srs_amd_pusch_slot_pdu>& sp, hipStream_t s,
               const std::vector<unsigned>* ids = nullptr)
  {
    buffer_set*           bs = j.bs;
    srs_amd_pusch_slot_io io{};
    io.d_cb_iterations = reinterpret_cast<int32_t*>(bs->cbi.d);
    io.d_uci           = bs->uci.d;
    io.d_port_stats    = reinterpret_cast<srs_amd_chest_port_stats*>(bs->pstats.d);
    auto* d_res        = reinterpret_cast<srs_amd_pusch_processor_result*>(bs->results.d);
    auto* d_grids      = reinterpret_cast<const uint32_t*>(bs->h_grids.d);
    const uint32_t ng  = static_cast<uint32_t>(std::max<size_t>(j.nof_grids, 1));
    if (ids == nullptr) {
      return srs_amd_pusch_process_slot_ex(proc, sp.data(), static_cast<uint32_t>(sp.size()), d_grids, j.grid_stride, ng,
                                           bs->tbs.d, d_res, &io, s);
    }
    // one PDU per call so that results / port measurements land in the first pass's rows
    for (size_t q = 0; q != sp.size(); ++q) {
      const unsigned        k = (*ids)[q];
      srs_amd_pusch_slot_io x = io;
      x.d_port_stats          = io.d_port_stats + static_cast<size_t>(k) * MAX_PORTS_HIP;
      const int rc = srs_amd_pusch_process_slot_ex(proc, &sp[q], 1, d_grids, j.grid_stride, ng, bs->tbs.d, d_res + k,
                                                   &x, s);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
    }
    return SRS_AMD_OK;
  }

  hipError_t download(job& j, hipStream_t s)
  {
    buffer_set* bs  = j.bs;
    const auto  m   = j.pdus.size();
    hipError_t  e   = hipSuccess;
    auto        d2h = [&](hip_mirrored_buffer& b, size_t bytes) {
      if (e == hipSuccess && bytes != 0) {
        e = hipMemcpyAsync(b.h, b.d, bytes, hipMemcpyDeviceToHost, s);
      }
    };
    d2h(bs->tbs, j.tb_total);
    d2h(bs->results, sizeof(srs_amd_pusch_processor_result) * m);
    d2h(bs->cbi, sizeof(int32_t) * j.cb_total);
    d2h(bs->uci, j.uci_total);
    d2h(bs->pstats, sizeof(srs_amd_chest_port_stats) * MAX_PORTS_HIP * m);
    // retransmissions' soft buffers (their state goes back to the rx_buffer whatever the outcome); new transmissions'
    // only if their TB fails (complete())
    for (size_t k = 0; k != m && e == hipSuccess; ++k) {
      if (!j.pdus[k].c.new_data) {
        e = hipMemcpyAsync(bs->soft.h + j.soft_off[k], bs->soft.d + j.soft_off[k], j.pl[k].soft_bytes,
                           hipMemcpyDeviceToHost, s);
      }
    }
    return e;
  }

  // rx_buffer -> device soft-buffer layout (srs_amd_pusch_soft_buffer_layout): soft bits, messages, CRC flags; the
  // flag of a codeblock OK from an earlier transmission is non-zero (its statistic comes from cb_stats).
  static void upload_harq(pending_pdu& p, const plan_entry& e, uint8_t* dst, std::vector<char>& prev)
  {
    uint32_t row = 0, nllr = 0, moff = 0, foff = 0;
    (void)srs_amd_pusch_soft_buffer_layout(&e.sch, &row, &nllr, &moff, &foff);
    rx_buffer&       rb   = p.rm_buffer.get();
    span<const bool> crcs = rb.get_codeblocks_crc();
    const unsigned   K    = e.sch.segment_length;
    prev.assign(e.nof_cbs, 0);
    std::memset(dst, 0, static_cast<size_t>(row) * e.nof_cbs);
    for (unsigned cb = 0; cb != e.nof_cbs; ++cb) {
      uint8_t*                   r  = dst + static_cast<size_t>(cb) * row;
      span<log_likelihood_ratio> sb = rb.get_codeblock_soft_bits(cb, nllr);
      std::memcpy(r, sb.data(), nllr);
      bit_buffer msg = rb.get_codeblock_data_bits(cb, K);
      std::memcpy(r + moff, msg.get_buffer().data(), (K + 7) / 8);
      prev[cb]            = crcs[cb] ? 1 : 0;
      const int32_t flag  = crcs[cb] ? std::max<int32_t>(1, static_cast<int32_t>((*p.cb_stats)[cb])) : 0;
      std::memcpy(r + foff, &flag, sizeof(flag));
    }
  }

  // device soft-buffer layout -> rx_buffer (after the call that decoded with it)
  static void store_harq(pending_pdu& p, const plan_entry& e, const uint8_t* src)
  {
    uint32_t row = 0, nllr = 0, moff = 0, foff = 0;
    (void)srs_amd_pusch_soft_buffer_layout(&e.sch, &row, &nllr, &moff, &foff);
    rx_buffer&     rb   = p.rm_buffer.get();
    span<bool>     crcs = rb.get_codeblocks_crc();
    const unsigned K    = e.sch.segment_length;
    for (unsigned cb = 0; cb != e.nof_cbs; ++cb) {
      const uint8_t*             r  = src + static_cast<size_t>(cb) * row;
      span<log_likelihood_ratio> sb = rb.get_codeblock_soft_bits(cb, nllr);
      std::memcpy(sb.data(), r, nllr);
      bit_buffer msg = rb.get_codeblock_data_bits(cb, K);
      std::memcpy(msg.get_buffer().data(), r + moff, (K + 7) / 8);
      int32_t flag = 0;
      std::memcpy(&flag, r + foff, sizeof(flag));
      crcs[cb] = flag != 0;
    }
  }

  // pusch_processor_notifier_adaptor (pusch_processor_notifier_adaptor.h) + pusch_decoder_impl::join_and_notify
  // (pusch_decoder_impl.cpp:404-457): transport block, rx_buffer release / unlock, on_uci, on_sch.
  void notify(pending_pdu& p, const plan_entry& e, const srs_amd_pusch_processor_result& r, const int32_t* cb_it,
              const std::vector<char>& prev, const uint8_t* tb, const uint8_t* uci_row,
              const srs_amd_chest_port_stats* st)
  {
    // channel state information as channel_estimate::get_channel_state_information (channel_estimation.h:244-281)
    channel_state_information csi(channel_state_information::sinr_type::channel_estimator);
    const unsigned P        = static_cast<unsigned>(p.rx_ports.size());
    float          epre_lin = 0.0F, best_snr = 0.0F, noise = 0.0F, rsrp = 0.0F;
    unsigned       best     = 0;
    std::array<float, MAX_PORTS_HIP> port_rsrp{};
    for (unsigned q = 0; q != P; ++q) {
      epre_lin += st[q].epre;
      if (st[q].snr > best_snr) {
        best_snr = st[q].snr;
        best     = q;
      }
      port_rsrp[q] = st[q].rsrp;
      noise += st[q].noise_var;
      rsrp += st[q].rsrp;
    }
    csi.set_rsrp_lin(span<const float>(port_rsrp.data(), P));
    csi.set_epre(10.0F * std::log10(epre_lin / static_cast<float>(P)));
    csi.set_time_alignment(phy_time_unit::from_seconds(st[best].time_alignment_s));
    csi.set_cfo(st[best].cfo_hz);
    csi.set_sinr_dB(channel_state_information::sinr_type::channel_estimator,
                    10.0F * std::log10(std::isnormal(noise) ? rsrp / noise : 0.0F));
    // LDPC statistics in codeblock order (cb_stats semantics)
    pusch_decoder_result dr;
    dr.tb_crc_ok            = r.data.tb_crc_ok != 0;
    dr.nof_codeblocks_total = e.nof_cbs;
    dr.ldpc_decoder_stats.reset();
    cb_stat_array& cs     = *p.cb_stats;
    bool           all_ok = true; // every codeblock CRC passed (now or in an earlier transmission)
    for (unsigned cb = 0; cb != e.nof_cbs && cb < MAX_CB; ++cb) {
      const bool earlier = cb < prev.size() && prev[cb];
      if (!earlier) {
        cs[cb] = cb_it[cb] >= 0 ? static_cast<unsigned>(cb_it[cb]) : cfg.dec_nof_iterations;
      }
      all_ok = all_ok && (earlier || cb_it[cb] >= 0);
      dr.ldpc_decoder_stats.update(cs[cb]);
    }
    // the transport block is written only once every codeblock CRC passed (pusch_decoder_impl.cpp:409-440: the
    // single codeblock's data, or the concatenation); otherwise the caller's buffer is left as it was
    if (all_ok) {
      std::memcpy(p.data.data(), tb, p.data.size());
    }
    if (p.rm_buffer.is_valid()) {
      if (dr.tb_crc_ok) {
        p.rm_buffer.release();
      } else {
        p.rm_buffer.unlock();
      }
    }
    // UCI fields (pusch_processor_notifier_adaptor::check_and_notify_uci)
    if (p.c.nof_harq_ack != 0 || p.c.nof_csi_part1 != 0) {
      pusch_processor_result_control ctrl;
      ctrl.csi      = csi;
      auto field    = [](const uint8_t* bits, unsigned nbits, int32_t status, pusch_uci_field& f) {
        f.payload = uci_payload_type(bits, bits + nbits);
        f.status  = static_cast<uci_status>(status);
      };
      if (p.c.nof_harq_ack != 0) {
        field(uci_row, p.c.nof_harq_ack, r.harq_ack_status, ctrl.harq_ack);
      }
      if (p.c.nof_csi_part1 != 0) {
        field(uci_row + p.c.nof_harq_ack, p.c.nof_csi_part1, r.csi_part1_status, ctrl.csi_part1);
      }
      if (r.nof_csi_part2 != 0) {
        field(uci_row + p.c.nof_harq_ack + p.c.nof_csi_part1, r.nof_csi_part2, r.csi_part2_status, ctrl.csi_part2);
      }
      p.notifier->on_uci(ctrl);
    }
    // UCI only: on_uci alone (pusch_processor_impl.cpp:305-324 sets up no decoder, so no on_sch)
    if (!p.pdu.codeword.has_value()) {
      return;
    }
    pusch_processor_result_data data;
    data.data = dr;
    data.csi  = csi;
    p.notifier->on_sch(data);
  }

public:
  std::atomic<uint64_t> stats_retx{0}, stats_soft_downloads{0}, stats_late_errors{0}, stats_device_grids{0};
  std::atomic<uint64_t> t_stage{0}, t_set_wait{0}, t_wait{0}, t_notify{0}; // ns
  std::atomic<uint64_t> t_reads{0}, t_call{0}, t_download{0};                // ns, parts of t_stage

private:
  pusch_processor_hip_config cfg;
  const unsigned             nsubc;
  int                        device  = 0;
  hipStream_t                stream  = nullptr; // batches
  hipStream_t                stream2 = nullptr; // HARQ soft-buffer passes (completion thread)
  srs_amd_pusch_processor*   proc    = nullptr;
  // collector-thread state
  std::unordered_map<std::string, plan_entry> plans;
  std::list<std::string>                      lru;
  row_pool                                    pool;
  row_pool                                    npool; // completion thread: notifications
  // dispatched batches (collector -> completion thread) and the buffer sets they use
  buffer_set                        sets[2];
  std::mutex                        jmtx;
  std::condition_variable           jcv;
  std::deque<std::unique_ptr<job>>  jobs;
  bool                              completing = false, stop = false;
  uint64_t                          dispatch_seq = 0, cur_seq = 0; // collector thread: batches dispatched / this one
  std::atomic<uint64_t>             completed_seq{0};              // the last batch the completion thread finished
  std::thread                       completer;
  // last: destroyed first, so the collector thread stops before the state it uses goes
  std::unique_ptr<slot_collector<pending_pdu>> collector;
};

class pusch_processor_hip : public pusch_processor
{
public:
  explicit pusch_processor_hip(std::shared_ptr<slot_engine> e) :
    engine(std::move(e)), cb_stats(std::make_shared<cb_stat_array>())
  {
    cb_stats->fill(0);
  }

  void process(span<uint8_t>                    data,
               unique_rx_buffer                 rm_buffer,
               pusch_processor_result_notifier& notifier,
               const resource_grid_reader&      grid,
               const pdu_t&                     pdu) override
  {
    pending_pdu p;
    p.data      = data;
    p.rm_buffer = std::move(rm_buffer);
    p.notifier  = &notifier;
    p.grid      = &grid;
    p.pdu       = pdu;
    p.rx_ports.assign(pdu.rx_ports.begin(), pdu.rx_ports.end());
    p.cb_stats = cb_stats;
    p.error    = convert(pdu, data.size(), p.c);
    engine->enqueue(std::move(p));
  }

private:
  std::shared_ptr<slot_engine>   engine;
  std::shared_ptr<cb_stat_array> cb_stats;
};

/// What the MI355X processor supports (the reference's pusch_processor_validator_impl checks, narrowed as
/// convert() and srs_amd_pusch_processor_plan_create narrow them).
class pusch_pdu_validator_hip : public pusch_pdu_validator
{
public:
  explicit pusch_pdu_validator_hip(unsigned nof_prb_) : nof_prb(nof_prb_) {}
  error_type<std::string> is_valid(const pusch_processor::pdu_t& pdu) const override
  {
    srs_amd_pusch_pdu c{};
    std::string       e = convert(pdu, 1, c);
    if (!e.empty()) {
      return make_unexpected(e);
    }
    if (c.dmrs_type != 1) {
      return make_unexpected(std::string("Only DM-RS Type 1 is currently supported."));
    }
    if (c.bwp_start_rb + c.bwp_size_rb > nof_prb || c.rb_start + c.rb_count > c.bwp_size_rb) {
      return make_unexpected(std::string("Allocation outside the resource grid."));
    }
    if (c.start_symbol_index + c.nof_symbols > NSYMB) {
      return make_unexpected(std::string("Time allocation outside the slot."));
    }
    return default_success_t();
  }

private:
  unsigned nof_prb;
};

class pusch_processor_factory_hip_impl : public pusch_processor_factory_hip
{
public:
  explicit pusch_processor_factory_hip_impl(const pusch_processor_hip_config& c) :
    cfg(c), engine(std::make_shared<slot_engine>(c))
  {
  }
  std::unique_ptr<pusch_processor> create() override { return std::make_unique<pusch_processor_hip>(engine); }
  // The reference wraps its processors in its logging decorator (factories.cpp:393); the MI355X processors log
  // their errors themselves.
  std::unique_ptr<pusch_processor> create(srslog::basic_logger& /*logger*/) override { return create(); }
  std::unique_ptr<pusch_pdu_validator> create_validator() override
  {
    return std::make_unique<pusch_pdu_validator_hip>(cfg.nof_prb);
  }
  void       flush() override { engine->flush(); }
  void       wait_idle() override { engine->wait_idle(); }
  statistics get_statistics() const override { return engine->get_statistics(); }

private:
  pusch_processor_hip_config   cfg;
  std::shared_ptr<slot_engine> engine;
};

} // namespace

std::shared_ptr<pusch_processor_factory_hip>
srsran::hip::create_pusch_processor_factory_hip(const pusch_processor_hip_config& cfg)
{
  try {
    return std::make_shared<pusch_processor_factory_hip_impl>(cfg);
  } catch (const std::exception& e) {
    log_error("factory", e.what());
    return nullptr;
  }
}
