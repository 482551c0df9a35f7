// pucch_processor_hip.cpp -- see pucch_processor_hip.h.
#include "pucch_processor_hip.h"
#include "hip_resource_grid.h"

#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran_amd/pucch.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

using namespace srsran;
using namespace srsran::hip;

namespace {

constexpr unsigned NSYMB = 14;

void log_error(const char* what, const std::string& detail)
{
  std::fprintf(stderr, "pucch_processor_hip: %s: %s\n", what, detail.c_str());
}

uint32_t numerology_of(slot_point slot)
{
  return to_numerology_value(slot.scs());
}

srs_amd_pucch_f0_pdu convert(const pucch_processor::format0_configuration& c)
{
  srs_amd_pucch_f0_pdu p{};
  p.numerology           = numerology_of(c.slot);
  p.slot_index           = c.slot.slot_index();
  p.starting_prb         = c.bwp_start_rb + c.starting_prb;
  p.second_hop_prb       = c.second_hop_prb.has_value() ? static_cast<int32_t>(c.bwp_start_rb + *c.second_hop_prb) : -1;
  p.start_symbol_index   = c.start_symbol_index;
  p.nof_symbols          = c.nof_symbols;
  p.initial_cyclic_shift = c.initial_cyclic_shift;
  p.n_id                 = c.n_id;
  p.nof_harq_ack         = c.nof_harq_ack;
  p.sr_opportunity       = c.sr_opportunity ? 1 : 0;
  p.nof_ports            = static_cast<uint32_t>(c.ports.size());
  for (unsigned i = 0; i != c.ports.size() && i != 4; ++i) {
    p.ports[i] = c.ports[i];
  }
  return p;
}

srs_amd_pucch_f2_pdu convert(const pucch_processor::format2_configuration& c)
{
  srs_amd_pucch_f2_pdu p{};
  p.numerology         = numerology_of(c.slot);
  p.slot_index         = c.slot.slot_index();
  p.bwp_start_rb       = c.bwp_start_rb;
  p.bwp_size_rb        = c.bwp_size_rb;
  p.starting_prb       = c.starting_prb;
  p.second_hop_prb     = c.second_hop_prb.has_value() ? static_cast<int32_t>(*c.second_hop_prb) : -1;
  p.nof_prb            = c.nof_prb;
  p.start_symbol_index = c.start_symbol_index;
  p.nof_symbols        = c.nof_symbols;
  p.rnti               = c.rnti;
  p.n_id               = c.n_id;
  p.n_id_0             = c.n_id_0;
  p.nof_harq_ack       = c.nof_harq_ack;
  p.nof_sr             = c.nof_sr;
  p.nof_csi_part1      = c.nof_csi_part1;
  p.nof_csi_part2      = c.nof_csi_part2;
  p.nof_ports          = static_cast<uint32_t>(c.ports.size());
  for (unsigned i = 0; i != c.ports.size() && i != 4; ++i) {
    p.ports[i] = c.ports[i];
  }
  return p;
}

template <typename C>
srs_amd_pucch_f34_pdu convert34(const C& c, uint32_t format, uint32_t nof_prb, uint32_t occ_index, uint32_t occ_length)
{
  srs_amd_pucch_f34_pdu p{};
  p.format             = format;
  p.numerology         = numerology_of(c.slot);
  p.slot_index         = c.slot.slot_index();
  p.bwp_start_rb       = c.bwp_start_rb;
  p.bwp_size_rb        = c.bwp_size_rb;
  p.starting_prb       = c.starting_prb;
  p.second_hop_prb     = c.second_hop_prb.has_value() ? static_cast<int32_t>(*c.second_hop_prb) : -1;
  p.nof_prb            = nof_prb;
  p.start_symbol_index = c.start_symbol_index;
  p.nof_symbols        = c.nof_symbols;
  p.rnti               = c.rnti;
  p.n_id_hopping       = c.n_id_hopping;
  p.n_id_scrambling    = c.n_id_scrambling;
  p.nof_harq_ack       = c.nof_harq_ack;
  p.nof_sr             = c.nof_sr;
  p.nof_csi_part1      = c.nof_csi_part1;
  p.nof_csi_part2      = c.nof_csi_part2;
  p.additional_dmrs    = c.additional_dmrs ? 1 : 0;
  p.pi2_bpsk           = c.pi2_bpsk ? 1 : 0;
  p.occ_index          = occ_index;
  p.occ_length         = occ_length;
  p.nof_ports          = static_cast<uint32_t>(c.ports.size());
  for (unsigned i = 0; i != c.ports.size() && i != 4; ++i) {
    p.ports[i] = c.ports[i];
  }
  return p;
}

// One process() call on a device-resident grid, waiting in the rendezvous (below) for its batch.
struct pucch_call {
  enum kind_t { F0, F1, F2, F34 } kind = F0;
  hip_resource_grid*                  grid = nullptr;
  unsigned                            nof_ports = 0, nsubc = 0;
  srs_amd_pucch_f0_pdu                f0{};
  srs_amd_pucch_f1_batch              f1{};
  std::vector<srs_amd_pucch_f1_entry> entries;
  srs_amd_pucch_f2_pdu                f2{};
  srs_amd_pucch_f34_pdu               f34{};
  unsigned                            K = 0; // payload bits (Formats 2-4)
  // filled by the batch's leader
  bool                              ok = false, done = false;
  bool                              lead = false; // this caller leads the next batch
  std::condition_variable           cv;           // done, or lead handed over
  srs_amd_pucch_f0_result           r0{};
  std::vector<srs_amd_pucch_result> r1;
  srs_amd_pucch_uci_result          ruci{};
  std::vector<uint8_t>              payload;
};

// Rendezvous of the synchronous pucch_processor::process calls of every processor of the factory.
// uplink_processor_impl hands all PUCCH PDUs of a slot's end symbol to the PUCCH executor at once
// (uplink_processor_impl.cpp:199-229, one task per PDU): the calls that arrive while a batch is in flight on the GPU
// (or within `window_us` of the first) go together in the next one -- one slot-form launch per format, one result
// download, one synchronisation -- and each caller returns with its own result.  The first waiting caller leads the
// batch (no thread of its own); the others sleep until it is done.
class pucch_rendezvous
{
public:
  pucch_rendezvous(srs_amd_pucch_processor* p, int dev, unsigned window) : proc(p), device(dev), window_us(window)
  {
    (void)hipSetDevice(device);
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
      throw std::runtime_error("pucch_processor_hip: rendezvous stream");
    }
  }
  ~pucch_rendezvous()
  {
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    (void)hipStreamDestroy(stream);
    (void)hipFree(d_buf);
    (void)hipHostFree(h_buf);
  }

  // returns when c's batch is done (c.ok: processed).  Each waiting caller sleeps on its own condition variable: the
  // leader wakes exactly the callers of its batch and hands the lead to the oldest caller still pending.
  void submit(pucch_call& c)
  {
    std::unique_lock<std::mutex> lock(mtx);
    pending.push_back(&c);
    if (!leading) {
      leading = true;
      c.lead  = true;
    }
    while (!c.done) {
      if (!c.lead) {
        c.cv.wait(lock);
        continue;
      }
      c.lead = false;
      if (window_us != 0) {
        lock.unlock();
        std::this_thread::sleep_for(std::chrono::microseconds(window_us));
        lock.lock();
      }
      std::vector<pucch_call*> batch;
      batch.swap(pending);
      lock.unlock();
      run(batch);
      lock.lock();
      ++nof_batches;
      for (pucch_call* b : batch) {
        b->done = true;
        if (b != &c) {
          b->cv.notify_one();
        }
      }
      if (pending.empty()) {
        leading = false;
      } else {
        pending.front()->lead = true;
        pending.front()->cv.notify_one();
      }
    }
  }

  std::atomic<uint64_t> nof_batches{0};
  // time spent by the leaders: reading the grids and launching (host), then waiting for the batch's results
  std::atomic<uint64_t> host_ns{0}, wait_ns{0};

private:
  // (kind, grid ports, grid subcarriers): calls that go in one slot-form launch
  using group_key = std::tuple<int, unsigned, unsigned>;

  bool reserve(size_t bytes)
  {
    if (bytes <= capacity) {
      return true;
    }
    (void)hipFree(d_buf);
    (void)hipHostFree(h_buf);
    d_buf    = nullptr;
    h_buf    = nullptr;
    capacity = 0;
    if (hipMalloc(&d_buf, bytes) != hipSuccess || hipHostMalloc(&h_buf, bytes, hipHostMallocDefault) != hipSuccess) {
      return false;
    }
    capacity = bytes;
    return true;
  }

  void run(std::vector<pucch_call*>& batch)
  {
    const auto t_start = std::chrono::steady_clock::now();
    (void)hipSetDevice(device);
    std::map<group_key, std::vector<pucch_call*>> groups;
    for (pucch_call* c : batch) {
      groups[{static_cast<int>(c->kind), c->nof_ports, c->nsubc}].push_back(c);
    }
    // result area: per group, the results then (Formats 2-4) the payload rows
    constexpr size_t PAY = 1706;
    size_t           bytes = 0;
    std::vector<size_t> off;
    for (auto& [key, calls] : groups) {
      off.push_back(bytes);
      size_t n = 0;
      switch (std::get<0>(key)) {
        case pucch_call::F0:
          n = calls.size() * sizeof(srs_amd_pucch_f0_result);
          break;
        case pucch_call::F1:
          for (pucch_call* c : calls) {
            n += c->entries.size() * sizeof(srs_amd_pucch_result);
          }
          break;
        default:
          n = calls.size() * (sizeof(srs_amd_pucch_uci_result) + PAY);
      }
      bytes += (n + 255) & ~size_t(255);
    }
    if (!reserve(bytes)) {
      return; // (ok stays false: logged by the callers)
    }
    // every distinct grid read once on the rendezvous stream (it waits for the grid's producers)
    std::map<hip_resource_grid*, const uint32_t*> dev_of;
    for (pucch_call* c : batch) {
      if (dev_of.count(c->grid) == 0) {
        dev_of[c->grid] = c->grid->device_read(stream);
      }
    }
    bool   ok = true;
    size_t gi = 0;
    for (auto& [key, calls] : groups) {
      uint8_t*       d     = static_cast<uint8_t*>(d_buf) + off[gi++];
      const unsigned ports = std::get<1>(key), nsubc = std::get<2>(key);
      const unsigned n     = static_cast<unsigned>(calls.size());
      int            rc    = SRS_AMD_OK;
      switch (std::get<0>(key)) {
        case pucch_call::F0: {
          std::vector<srs_amd_pucch_f0_pdu> pdus;
          for (pucch_call* c : calls) {
            pdus.push_back(c->f0);
            pdus.back().d_grid = dev_of[c->grid];
          }
          rc = srs_amd_pucch_f0_detect_slot(proc, pdus.data(), n, nullptr, 0, 0, ports, nsubc,
                                            reinterpret_cast<srs_amd_pucch_f0_result*>(d), stream);
          break;
        }
        case pucch_call::F1: {
          std::vector<srs_amd_pucch_f1_batch> bs;
          for (pucch_call* c : calls) {
            bs.push_back(c->f1);
            bs.back().d_grid  = dev_of[c->grid];
            bs.back().entries = c->entries.data();
          }
          rc = srs_amd_pucch_f1_detect_slot(proc, bs.data(), n, nullptr, 0, 0, ports, nsubc,
                                            reinterpret_cast<srs_amd_pucch_result*>(d), stream);
          break;
        }
        case pucch_call::F2: {
          std::vector<srs_amd_pucch_f2_pdu> pdus;
          for (pucch_call* c : calls) {
            pdus.push_back(c->f2);
            pdus.back().d_grid = dev_of[c->grid];
          }
          rc = srs_amd_pucch_f2_process_slot(proc, pdus.data(), n, nullptr, 0, 0, ports, nsubc,
                                             reinterpret_cast<srs_amd_pucch_uci_result*>(d),
                                             d + n * sizeof(srs_amd_pucch_uci_result), PAY, stream);
          break;
        }
        default: {
          std::vector<srs_amd_pucch_f34_pdu> pdus;
          for (pucch_call* c : calls) {
            pdus.push_back(c->f34);
            pdus.back().d_grid = dev_of[c->grid];
          }
          rc = srs_amd_pucch_f34_process_slot(proc, pdus.data(), n, nullptr, 0, 0, ports, nsubc,
                                              reinterpret_cast<srs_amd_pucch_uci_result*>(d),
                                              d + n * sizeof(srs_amd_pucch_uci_result), PAY, stream);
        }
      }
      if (rc != SRS_AMD_OK) {
        log_error("batch not processed", srs_amd_last_error());
        ok = false;
      }
    }
    ok             = ok && hipMemcpyAsync(h_buf, d_buf, bytes, hipMemcpyDeviceToHost, stream) == hipSuccess;
    const auto t_l = std::chrono::steady_clock::now();
    ok             = hipStreamSynchronize(stream) == hipSuccess && ok;
    const auto t_w = std::chrono::steady_clock::now();
    host_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t_l - t_start).count();
    wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t_w - t_l).count();
    if (!ok) {
      return;
    }
    gi = 0;
    for (auto& [key, calls] : groups) {
      const uint8_t* h = static_cast<const uint8_t*>(h_buf) + off[gi++];
      const size_t   n = calls.size();
      size_t         e = 0;
      for (size_t i = 0; i != n; ++i) {
        pucch_call& c = *calls[i];
        switch (c.kind) {
          case pucch_call::F0:
            std::memcpy(&c.r0, h + i * sizeof(srs_amd_pucch_f0_result), sizeof(c.r0));
            break;
          case pucch_call::F1:
            c.r1.resize(c.entries.size());
            std::memcpy(c.r1.data(), h + e * sizeof(srs_amd_pucch_result), c.r1.size() * sizeof(srs_amd_pucch_result));
            e += c.entries.size();
            break;
          default:
            std::memcpy(&c.ruci, h + i * sizeof(srs_amd_pucch_uci_result), sizeof(c.ruci));
            c.payload.assign(h + n * sizeof(srs_amd_pucch_uci_result) + i * PAY,
                             h + n * sizeof(srs_amd_pucch_uci_result) + i * PAY + c.K);
        }
        c.ok = true;
      }
    }
  }

  srs_amd_pucch_processor* proc;
  int                      device;
  unsigned                 window_us;
  hipStream_t              stream   = nullptr;
  void*                    d_buf    = nullptr;
  void*                    h_buf    = nullptr;
  size_t                   capacity = 0;
  std::mutex               mtx;
  std::vector<pucch_call*> pending;
  bool                     leading = false;
};

struct shared_state {
  srs_amd_pucch_processor*          proc   = nullptr;
  int                               device = 0;
  pucch_processor_hip_config        cfg;
  std::atomic<uint64_t>             nof_pdus{0}, nof_errors{0}, nof_device{0};
  std::unique_ptr<pucch_rendezvous> rdv;
  ~shared_state()
  {
    rdv.reset();
    srs_amd_pucch_processor_destroy(proc);
  }
};

class pucch_processor_hip : public pucch_processor
{
public:
  explicit pucch_processor_hip(std::shared_ptr<shared_state> s) : st(std::move(s))
  {
    (void)hipSetDevice(st->device);
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d_res, RES_BYTES) != hipSuccess || hipHostMalloc(&h_res, RES_BYTES, hipHostMallocDefault) != hipSuccess) {
      throw std::runtime_error("pucch_processor_hip: stream / result buffers");
    }
  }
  ~pucch_processor_hip() override
  {
    (void)hipSetDevice(st->device);
    (void)hipStreamSynchronize(stream);
    (void)hipStreamDestroy(stream);
    (void)hipFree(scratch);
    (void)hipHostFree(stage);
    (void)hipFree(d_res);
    (void)hipHostFree(h_res);
  }

  pucch_processor_result process(const resource_grid_reader& grid, const format0_configuration& config) override
  {
    ++st->nof_pdus;
    pucch_processor_result result;
    result.message = pucch_uci_message({.nof_sr = config.sr_opportunity ? 1U : 0U,
                                        .nof_harq_ack = config.nof_harq_ack, .nof_csi_part1 = 0, .nof_csi_part2 = 0});
    result.message.set_status(uci_status::invalid);
    if (!normal_cp(config.cp)) {
      return result;
    }
    srs_amd_pucch_f0_pdu p = convert(config);
    unsigned             nof_ports = 0, nsubc = 0;
    const srs_amd_pucch_f0_result* r = static_cast<srs_amd_pucch_f0_result*>(h_res);
    pucch_call                     call;
    if (hip_resource_grid* hg = hip_grid_of(grid)) {
      call.kind = pucch_call::F0;
      call.f0   = p;
      if (!rendezvous(call, *hg)) {
        return result;
      }
      r = &call.r0;
    } else {
      const uint32_t* g = grid_for(grid, p.ports, p.nof_ports, p.start_symbol_index, p.nof_symbols, nof_ports, nsubc);
      if (g == nullptr || !run([&] {
            p.d_grid = g;
            return srs_amd_pucch_f0_detect_slot(st->proc, &p, 1, nullptr, 0, 0, nof_ports, nsubc,
                                                static_cast<srs_amd_pucch_f0_result*>(d_res), stream);
          }, sizeof(srs_amd_pucch_f0_result))) {
        return result;
      }
    }
    result.message = pucch_uci_message({.nof_sr = r->nof_sr, .nof_harq_ack = r->nof_harq_ack, .nof_csi_part1 = 0,
                                        .nof_csi_part2 = 0});
    if (r->nof_sr != 0) {
      result.message.get_sr_bits()[0] = r->sr;
    }
    for (unsigned i = 0; i != r->nof_harq_ack && i != 2; ++i) {
      result.message.get_harq_ack_bits()[i] = r->harq_ack[i];
    }
    result.message.set_status(static_cast<uci_status>(r->status));
    result.csi = channel_state_information(channel_state_information::sinr_type::post_equalization);
    result.csi.set_sinr_dB(channel_state_information::sinr_type::post_equalization, r->sinr_dB);
    result.csi.set_rsrp_dB(r->rsrp_dB);
    result.csi.set_epre(r->epre_dB);
    return result;
  }

  pucch_format1_map<pucch_processor_result> process(const resource_grid_reader&        grid,
                                                    const format1_batch_configuration& batch) override
  {
    const format1_common_configuration& c = batch.common_config;
    pucch_format1_map<pucch_processor_result> out;
    std::vector<srs_amd_pucch_f1_entry>       entries;
    for (const auto& e : batch.entries) {
      entries.push_back({static_cast<uint8_t>(e.initial_cyclic_shift), static_cast<uint8_t>(e.time_domain_occ),
                         static_cast<uint8_t>(e.value.nof_harq_ack), 0});
      pucch_processor_result r;
      r.message = pucch_uci_message({.nof_sr = 0, .nof_harq_ack = e.value.nof_harq_ack, .nof_csi_part1 = 0,
                                     .nof_csi_part2 = 0});
      r.message.set_status(uci_status::invalid);
      out.insert(e.initial_cyclic_shift, e.time_domain_occ, r);
    }
    st->nof_pdus += entries.size();
    if (!normal_cp(c.cp)) {
      return out;
    }
    // the reference's Format 1 detector reads every port of the grid, 0 .. nof_ports - 1
    // (pucch_detector_format1.cpp:529, 568-583)
    srs_amd_pucch_f1_batch b{};
    b.numerology         = numerology_of(c.slot);
    b.slot_index         = c.slot.slot_index();
    b.starting_prb       = c.bwp_start_rb + c.starting_prb;
    b.second_hop_prb     = c.second_hop_prb.has_value() ? static_cast<int32_t>(c.bwp_start_rb + *c.second_hop_prb) : -1;
    b.start_symbol_index = c.start_symbol_index;
    b.nof_symbols        = c.nof_symbols;
    b.n_id               = c.n_id;
    b.nof_ports          = std::min<unsigned>(grid.get_nof_ports(), 4);
    for (unsigned i = 0; i != b.nof_ports; ++i) {
      b.ports[i] = static_cast<uint8_t>(i);
    }
    b.nof_entries = static_cast<uint32_t>(entries.size());
    b.entries     = entries.data();
    if (entries.size() * sizeof(srs_amd_pucch_result) > RES_BYTES) {
      ++st->nof_errors;
      log_error("batch not processed", "too many entries");
      return out;
    }
    unsigned                    nof_ports = 0, nsubc = 0;
    const srs_amd_pucch_result* r = static_cast<const srs_amd_pucch_result*>(h_res);
    pucch_call                  call;
    if (hip_resource_grid* hg = hip_grid_of(grid)) {
      call.kind    = pucch_call::F1;
      call.f1      = b;
      call.entries = entries;
      if (!rendezvous(call, *hg)) {
        return out;
      }
      r = call.r1.data();
    } else {
      const uint32_t* g = grid_for(grid, b.ports, b.nof_ports, b.start_symbol_index, b.nof_symbols, nof_ports, nsubc);
      if (g == nullptr || !run([&] {
            b.d_grid = g;
            return srs_amd_pucch_f1_detect_slot(st->proc, &b, 1, nullptr, 0, 0, nof_ports, nsubc,
                                                static_cast<srs_amd_pucch_result*>(d_res), stream);
          }, entries.size() * sizeof(srs_amd_pucch_result))) {
        return out;
      }
    }
    for (unsigned k = 0; k != entries.size(); ++k) {
      pucch_processor_result& res = out.get(entries[k].initial_cyclic_shift, entries[k].time_domain_occ);
      for (unsigned i = 0; i != r[k].nof_harq_ack && i != 2; ++i) {
        res.message.get_harq_ack_bits()[i] = r[k].harq_ack[i];
      }
      res.message.set_status(static_cast<uci_status>(r[k].status));
      res.csi = channel_state_information();
      res.csi.set_epre(r[k].epre_dB);
      res.csi.set_rsrp_dB(r[k].rsrp_dB);
      res.csi.set_sinr_dB(channel_state_information::sinr_type::channel_estimator, r[k].sinr_dB);
      res.csi.reset_time_alignment();
      res.detection_metric = r[k].detection_metric;
    }
    return out;
  }

  pucch_processor_result process(const resource_grid_reader& grid, const format2_configuration& config) override
  {
    ++st->nof_pdus;
    pucch_processor_result result;
    result.message = pucch_uci_message({.nof_sr = config.nof_sr, .nof_harq_ack = config.nof_harq_ack,
                                        .nof_csi_part1 = config.nof_csi_part1, .nof_csi_part2 = config.nof_csi_part2});
    result.message.set_status(uci_status::invalid);
    if (!normal_cp(config.cp)) {
      return result;
    }
    srs_amd_pucch_f2_pdu p = convert(config);
    const unsigned       K = config.nof_sr + config.nof_harq_ack + config.nof_csi_part1 + config.nof_csi_part2;
    if (K > 1706) {
      return result;
    }
    if (hip_resource_grid* hg = hip_grid_of(grid)) {
      pucch_call call;
      call.kind = pucch_call::F2;
      call.f2   = p;
      call.K    = K;
      if (rendezvous(call, *hg)) {
        fill_uci(result, K, call.ruci, call.payload.data());
      }
      return result;
    }
    unsigned        nof_ports = 0, nsubc = 0;
    const uint32_t* g = grid_for(grid, p.ports, p.nof_ports, p.start_symbol_index, p.nof_symbols, nof_ports, nsubc);
    auto*           d_pay = static_cast<uint8_t*>(d_res) + PAYLOAD_OFF;
    if (g == nullptr || !run([&] {
          p.d_grid = g;
          return srs_amd_pucch_f2_process_slot(st->proc, &p, 1, nullptr, 0, 0, nof_ports, nsubc,
                                               static_cast<srs_amd_pucch_uci_result*>(d_res), d_pay, 1706, stream);
        }, PAYLOAD_OFF + K)) {
      return result;
    }
    fill_uci(result, K, *static_cast<const srs_amd_pucch_uci_result*>(h_res),
             static_cast<const uint8_t*>(h_res) + PAYLOAD_OFF);
    return result;
  }

  pucch_processor_result process(const resource_grid_reader& grid, const format3_configuration& config) override
  {
    return process34(grid, convert34(config, 3, config.nof_prb, 0, 1), config.nof_sr, config.nof_harq_ack,
                     config.nof_csi_part1, config.nof_csi_part2, config.cp);
  }

  pucch_processor_result process(const resource_grid_reader& grid, const format4_configuration& config) override
  {
    return process34(grid, convert34(config, 4, 1, config.occ_index, config.occ_length), config.nof_sr,
                     config.nof_harq_ack, config.nof_csi_part1, config.nof_csi_part2, config.cp);
  }

private:
  static constexpr size_t RES_BYTES   = 4096;
  static constexpr size_t PAYLOAD_OFF = 256;

  // Formats 3 / 4: the PDU's symbols through srs_amd_pucch_f34_process_slot, the message and CSI back.
  // Extended cyclic prefix: the plug-in's kernels are built for 14 symbols per slot; such a PDU is reported as not
  // processed (invalid status) and counted as an error, as the validator rejects it
  bool normal_cp(cyclic_prefix cp)
  {
    if (cp == cyclic_prefix::NORMAL) {
      return true;
    }
    ++st->nof_errors;
    log_error("PDU not processed", "extended cyclic prefix");
    return false;
  }

  pucch_processor_result process34(const resource_grid_reader& grid, srs_amd_pucch_f34_pdu p, unsigned sr,
                                   unsigned harq, unsigned csi1, unsigned csi2, cyclic_prefix cp)
  {
    ++st->nof_pdus;
    pucch_processor_result result;
    result.message = pucch_uci_message({.nof_sr = sr, .nof_harq_ack = harq, .nof_csi_part1 = csi1,
                                        .nof_csi_part2 = csi2});
    result.message.set_status(uci_status::invalid);
    if (!normal_cp(cp)) {
      return result;
    }
    const unsigned K = sr + harq + csi1 + csi2;
    if (K > 1706) {
      return result;
    }
    if (hip_resource_grid* hg = hip_grid_of(grid)) {
      pucch_call call;
      call.kind = pucch_call::F34;
      call.f34  = p;
      call.K    = K;
      if (rendezvous(call, *hg)) {
        fill_uci(result, K, call.ruci, call.payload.data());
      }
      return result;
    }
    unsigned        nof_ports = 0, nsubc = 0;
    const uint32_t* g = grid_for(grid, p.ports, p.nof_ports, p.start_symbol_index, p.nof_symbols, nof_ports, nsubc);
    auto*           d_pay = static_cast<uint8_t*>(d_res) + PAYLOAD_OFF;
    if (g == nullptr || !run([&] {
          p.d_grid = g;
          return srs_amd_pucch_f34_process_slot(st->proc, &p, 1, nullptr, 0, 0, nof_ports, nsubc,
                                                static_cast<srs_amd_pucch_uci_result*>(d_res), d_pay, 1706, stream);
        }, PAYLOAD_OFF + K)) {
      return result;
    }
    fill_uci(result, K, *static_cast<const srs_amd_pucch_uci_result*>(h_res),
             static_cast<const uint8_t*>(h_res) + PAYLOAD_OFF);
    return result;
  }

  // a device-resident grid: the call joins the factory's rendezvous (one launch for every call that waits with it)
  bool rendezvous(pucch_call& call, hip_resource_grid& hg)
  {
    ++st->nof_device;
    call.grid      = &hg;
    call.nof_ports = hg.nof_ports();
    call.nsubc     = hg.nof_subc();
    st->rdv->submit(call);
    if (!call.ok) {
      ++st->nof_errors;
      log_error("PDU not processed", "rendezvous batch failed");
    }
    return call.ok;
  }

  static void fill_uci(pucch_processor_result& result, unsigned K, const srs_amd_pucch_uci_result& res,
                       const uint8_t* payload)
  {
    const auto* r = &res;
    std::memcpy(result.message.get_full_payload().data(), payload, K);
    result.message.set_status(static_cast<uci_status>(r->status));
    result.csi = channel_state_information();
    result.csi.set_epre(r->epre_dB);
    result.csi.set_rsrp_dB(r->rsrp_dB);
    result.csi.set_sinr_dB(channel_state_information::sinr_type::channel_estimator, r->sinr_dB);
    result.csi.set_time_alignment(phy_time_unit::from_seconds(r->time_alignment_s));
    if (!std::isnan(r->cfo_Hz)) {
      result.csi.set_cfo(r->cfo_Hz);
    }
  }

  // Launch through `call`, bring `bytes` of the result buffer back, wait.  false (logged) on any error.
  template <typename F>
  bool run(F&& call, size_t bytes)
  {
    int        rc = call();
    hipError_t e  = hipSuccess;
    if (rc == SRS_AMD_OK) {
      e = hipMemcpyAsync(h_res, d_res, bytes, hipMemcpyDeviceToHost, stream);
      e = e == hipSuccess ? hipStreamSynchronize(stream) : e;
    } else {
      (void)hipStreamSynchronize(stream);
    }
    if (rc != SRS_AMD_OK || e != hipSuccess) {
      ++st->nof_errors;
      log_error("PDU not processed", rc != SRS_AMD_OK ? std::string(srs_amd_last_error()) : hipGetErrorString(e));
      return false;
    }
    return true;
  }

  // The grid on the device: a hip_resource_grid's own copy, or the PDU's symbols of its ports copied into a scratch
  // grid of the same dimensions.
  const uint32_t* grid_for(const resource_grid_reader& grid, const uint8_t* ports, unsigned nports, unsigned l0,
                           unsigned nsym, unsigned& nof_ports, unsigned& nsubc)
  {
    (void)hipSetDevice(st->device);
    nof_ports = grid.get_nof_ports();
    nsubc     = grid.get_nof_subc();
    if (hip_resource_grid* h = hip_grid_of(grid)) {
      ++st->nof_device;
      return h->device_read(stream);
    }
    if (l0 + nsym > NSYMB) {
      return nullptr; // the C-ABI call reports the PDU
    }
    const size_t plane = static_cast<size_t>(NSYMB) * nsubc;
    if (!reserve(nof_ports * plane * sizeof(uint32_t), nports * nsym * nsubc * sizeof(uint32_t))) {
      ++st->nof_errors;
      log_error("PDU not processed", "device / pinned buffer allocation");
      return nullptr;
    }
    // the PDU's symbols of each port: staged contiguously, one copy per port
    size_t row = 0;
    for (unsigned i = 0; i != nports; ++i) {
      if (ports[i] >= nof_ports) {
        continue; // the C-ABI call reports the port
      }
      uint32_t* dst = stage + row * nsubc;
      for (unsigned l = l0; l != l0 + nsym; ++l, ++row) {
        span<const cbf16_t> v = grid.get_view(ports[i], l);
        std::memcpy(stage + row * nsubc, v.data(), nsubc * sizeof(uint32_t));
      }
      if (hipMemcpyAsync(scratch + ports[i] * plane + static_cast<size_t>(l0) * nsubc, dst,
                         static_cast<size_t>(nsym) * nsubc * sizeof(uint32_t), hipMemcpyHostToDevice,
                         stream) != hipSuccess) {
        return nullptr;
      }
    }
    return scratch;
  }

  bool reserve(size_t dev_bytes, size_t host_bytes)
  {
    if (dev_bytes > dev_capacity) {
      (void)hipStreamSynchronize(stream);
      (void)hipFree(scratch);
      scratch      = nullptr;
      dev_capacity = 0;
      if (hipMalloc(&scratch, dev_bytes) != hipSuccess) {
        return false;
      }
      dev_capacity = dev_bytes;
    }
    if (host_bytes > host_capacity) {
      (void)hipStreamSynchronize(stream);
      (void)hipHostFree(stage);
      stage         = nullptr;
      host_capacity = 0;
      if (hipHostMalloc(&stage, host_bytes, hipHostMallocDefault) != hipSuccess) {
        return false;
      }
      host_capacity = host_bytes;
    }
    return true;
  }

  std::shared_ptr<shared_state> st;
  hipStream_t                   stream        = nullptr;
  uint32_t*                     scratch       = nullptr;
  uint32_t*                     stage         = nullptr;
  size_t                        dev_capacity  = 0;
  size_t                        host_capacity = 0;
  void*                         d_res         = nullptr;
  void*                         h_res         = nullptr;
};

// pucch_pdu_validator_impl (pucch_processor_impl.cpp:399-760) for every format the plug-in builds (0-4), normal cyclic
// prefix only (the reference also accepts extended: the plug-in reports it unsupported, as the PUSCH / PDSCH / PDCCH
// plug-ins do).
class pucch_pdu_validator_hip : public pucch_pdu_validator
{
public:
  explicit pucch_pdu_validator_hip(const pucch_processor_hip_config& c) : cfg(c) {}

  error_type<std::string> is_valid(const pucch_processor::format0_configuration& c) const override
  {
    if (c.cp != cyclic_prefix::NORMAL) {
      return make_unexpected(std::string("extended cyclic prefix"));
    }
    if (c.bwp_start_rb + c.bwp_size_rb > cfg.max_nof_prb || c.starting_prb >= c.bwp_size_rb ||
        (c.second_hop_prb.has_value() && *c.second_hop_prb >= c.bwp_size_rb)) {
      return make_unexpected(std::string("PRB allocation outside the BWP or the grid"));
    }
    if (c.nof_symbols < 1 || c.nof_symbols > 2 || c.start_symbol_index + c.nof_symbols > NSYMB) {
      return make_unexpected(std::string("invalid Format 0 symbols"));
    }
    if (c.initial_cyclic_shift > 11 || c.n_id > 1023 || c.nof_harq_ack > 2 ||
        (c.nof_harq_ack == 0 && !c.sr_opportunity)) {
      return make_unexpected(std::string("invalid Format 0 PDU"));
    }
    return ports_ok(c.ports);
  }
  error_type<std::string> is_valid(const pucch_processor::format1_configuration& c) const override
  {
    if (c.cp != cyclic_prefix::NORMAL) {
      return make_unexpected(std::string("extended cyclic prefix"));
    }
    const unsigned ratio = c.second_hop_prb.has_value() ? 4 : 2;
    if (c.bwp_start_rb + c.bwp_size_rb > cfg.max_nof_prb || c.starting_prb >= c.bwp_size_rb ||
        (c.second_hop_prb.has_value() && *c.second_hop_prb >= c.bwp_size_rb)) {
      return make_unexpected(std::string("PRB allocation outside the BWP or the grid"));
    }
    if (c.start_symbol_index > 10 || c.nof_symbols < 4 || c.start_symbol_index + c.nof_symbols > NSYMB ||
        c.initial_cyclic_shift > 11 || c.time_domain_occ >= c.nof_symbols / ratio || c.nof_harq_ack > 2 ||
        c.n_id > 1023) {
      return make_unexpected(std::string("invalid Format 1 PDU"));
    }
    return ports_ok(c.ports);
  }
  error_type<std::string> is_valid(const pucch_processor::format2_configuration& c) const override
  {
    if (c.cp != cyclic_prefix::NORMAL) {
      return make_unexpected(std::string("extended cyclic prefix"));
    }
    const unsigned K = c.nof_harq_ack + c.nof_sr + c.nof_csi_part1 + c.nof_csi_part2;
    const unsigned E = 16 * c.nof_prb * c.nof_symbols;
    const unsigned A = K <= 11 ? 0 : (K <= 19 ? 6 : 11);
    if (c.bwp_start_rb + c.bwp_size_rb > cfg.max_nof_prb || c.starting_prb + c.nof_prb > c.bwp_size_rb ||
        c.nof_prb == 0 || c.nof_prb > 16) {
      return make_unexpected(std::string("PRB allocation outside the BWP or the grid"));
    }
    if (c.nof_symbols < 1 || c.nof_symbols > 2 || c.start_symbol_index + c.nof_symbols > NSYMB ||
        (c.second_hop_prb.has_value() && c.nof_symbols != 2)) {
      return make_unexpected(std::string("invalid Format 2 symbols"));
    }
    if (c.nof_csi_part2 != 0) {
      return make_unexpected(std::string("CSI Part 2 is not currently supported."));
    }
    if (K < 3 || K > 1706 || static_cast<float>(K + A) / static_cast<float>(E) > 0.8F) {
      return make_unexpected(std::string("invalid Format 2 payload size or code rate"));
    }
    return ports_ok(c.ports);
  }
  error_type<std::string> is_valid(const pucch_processor::format3_configuration& c) const override
  {
    return f34_ok(c, c.nof_prb, false, 1);
  }
  error_type<std::string> is_valid(const pucch_processor::format4_configuration& c) const override
  {
    if (c.occ_length != 2 && c.occ_length != 4) {
      return make_unexpected(std::string("Invalid OCC length value. Valid values are 2 and 4."));
    }
    return f34_ok(c, 1, true, c.occ_length);
  }

private:
  // pucch_pdu_validator_impl format3 / format4 checks (pucch_processor_impl.cpp), plus the transform-precoding PRB
  // sizes and the symbol range the reference asserts on.
  template <typename C>
  error_type<std::string> f34_ok(const C& c, unsigned nprb, bool f4, unsigned occ) const
  {
    if (c.cp != cyclic_prefix::NORMAL) {
      return make_unexpected(std::string("extended cyclic prefix"));
    }
    static const unsigned masks[2][15] = {{0, 0, 0, 0, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2},
                                          {0, 0, 0, 0, 2, 2, 2, 2, 2, 2, 4, 4, 4, 4, 4}};
    if (c.bwp_start_rb + c.bwp_size_rb > cfg.max_nof_prb || c.starting_prb + nprb > c.bwp_size_rb) {
      return make_unexpected(std::string("PRB allocation outside the BWP or the grid"));
    }
    unsigned n = nprb;
    for (unsigned f : {2U, 3U, 5U}) {
      while (n != 0 && n % f == 0) {
        n /= f;
      }
    }
    if (nprb == 0 || nprb > 16 || n != 1) {
      return make_unexpected(std::string("Number of PRBs is outside the allowed range for PUCCH Format 3"));
    }
    if (c.nof_symbols < 4 || c.nof_symbols > 14 || c.start_symbol_index + c.nof_symbols > NSYMB) {
      return make_unexpected(std::string("invalid Format 3 / 4 symbols"));
    }
    if (c.nof_csi_part2 != 0) {
      return make_unexpected(std::string("CSI Part 2 is not currently supported."));
    }
    unsigned nd = masks[c.additional_dmrs ? 1 : 0][c.nof_symbols];
    if (c.nof_symbols == 4 && c.second_hop_prb.has_value()) {
      nd = 2;
    }
    const unsigned K     = c.nof_harq_ack + c.nof_sr + c.nof_csi_part1 + c.nof_csi_part2;
    const unsigned qb    = c.pi2_bpsk ? 1 : 2;
    const unsigned nds   = c.nof_symbols - nd;
    const unsigned e_tot = f4 ? 12 * nds * qb / occ : 12 * nprb * nds * qb;
    const unsigned chan  = 12 * (f4 ? 1 : nprb) * nds * qb;
    const unsigned ncb   = ((K >= 360 && e_tot >= 1088) || K >= 1013) ? 2 : 1;
    const unsigned L     = K <= 11 ? 0 : (K <= 19 ? 6 : 11);
    if (static_cast<float>(K + ncb * L) / static_cast<float>(chan) > 0.8F) {
      return make_unexpected(std::string("The effective code rate exceeds the maximum allowed 0.8"));
    }
    if (K < 3 || K > 1706) {
      return make_unexpected(std::string("UCI Payload length is outside the supported range"));
    }
    return ports_ok(c.ports);
  }

  error_type<std::string> ports_ok(const static_vector<uint8_t, MAX_PORTS>& ports) const
  {
    if (ports.empty() || ports.size() > cfg.max_nof_ports || ports.size() > 4) {
      return make_unexpected(std::string("invalid number of receive ports"));
    }
    return default_success_t();
  }
  pucch_processor_hip_config cfg;
};

class pucch_processor_factory_hip_impl : public pucch_processor_factory_hip
{
public:
  explicit pucch_processor_factory_hip_impl(std::shared_ptr<shared_state> s) : st(std::move(s)) {}

  std::unique_ptr<pucch_processor> create() override
  {
    try {
      return std::make_unique<pucch_processor_hip>(st);
    } catch (const std::exception& e) {
      log_error("create", e.what());
      return nullptr;
    }
  }
  std::unique_ptr<pucch_pdu_validator> create_validator() override
  {
    return std::make_unique<pucch_pdu_validator_hip>(st->cfg);
  }
  statistics get_statistics() const override
  {
    statistics s;
    s.nof_pdus         = st->nof_pdus;
    s.nof_errors       = st->nof_errors;
    s.nof_device_grids = st->nof_device;
    s.nof_batches      = st->rdv->nof_batches;
    s.batch_host_us    = st->rdv->host_ns / 1000;
    s.batch_wait_us    = st->rdv->wait_ns / 1000;
    return s;
  }

private:
  std::shared_ptr<shared_state> st;
};

} // namespace

std::shared_ptr<pucch_processor_factory_hip>
srsran::hip::create_pucch_processor_factory_hip(const pucch_processor_hip_config& cfg)
{
  auto st = std::make_shared<shared_state>();
  st->cfg = cfg;
  int dev = cfg.device;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
    log_error("create", "no HIP device");
    return nullptr;
  }
  st->device = dev;
  if (srs_amd_pucch_processor_create(&st->proc, dev) != SRS_AMD_OK) {
    log_error("create", srs_amd_last_error());
    return nullptr;
  }
  try {
    st->rdv = std::make_unique<pucch_rendezvous>(st->proc, dev, cfg.rendezvous_window_us);
  } catch (const std::exception& e) {
    log_error("create", e.what());
    return nullptr;
  }
  return std::make_shared<pucch_processor_factory_hip_impl>(std::move(st));
}
