// hip_resource_grid.cpp -- device-resident srsran::resource_grid (see the header).
#include "hip_resource_grid.h"

#include "srsran_amd/grid.h"
#include "srsran_amd/ldpc.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <stdexcept>
#include <string>

using namespace srsran;
using namespace srsran::hip;

namespace {

void check(hipError_t e, const char* what)
{
  if (e != hipSuccess) {
    throw std::runtime_error(std::string("hip_resource_grid: ") + what + ": " + hipGetErrorString(e));
  }
}

} // namespace

hip_resource_grid::hip_resource_grid(std::unique_ptr<resource_grid> host_, int device_) :
  host(std::move(host_)), reader(*this), writer(*this)
{
  static std::atomic<uint64_t> next_uid{1};
  uid = next_uid.fetch_add(1);
  if (!host) {
    throw std::runtime_error("hip_resource_grid: no host grid");
  }
  const resource_grid_reader& r = host->get_reader();
  ports                         = r.get_nof_ports();
  symbols                       = r.get_nof_symbols();
  subc                          = r.get_nof_subc();
  dev                           = device_;
  if (dev < 0) {
    check(hipGetDevice(&dev), "hipGetDevice");
  }
  check(hipSetDevice(dev), "hipSetDevice");
  const size_t n = static_cast<size_t>(ports) * symbols * subc;
  check(hipMalloc(&d, sizeof(uint32_t) * n), "hipMalloc");
  check(hipStreamCreateWithFlags(&own, hipStreamNonBlocking), "stream");
  // the host mirror starts as the reference grid does (all zero): so do the device copy and the agreed state
  base.assign(n, 0u);
  check(hipMemsetAsync(d, 0, sizeof(uint32_t) * n, own), "hipMemsetAsync");
  add_producer(own);
}

hipEvent_t hip_resource_grid::take_event() const
{
  if (!spare.empty()) {
    hipEvent_t e = spare.back();
    spare.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
  return e;
}

void hip_resource_grid::add_producer(hipStream_t s) const
{
  hipEvent_t e = take_event();
  check(hipEventRecord(e, s), "hipEventRecord");
  producers.push_back(e);
  if (producers.size() > 16) {
    prune();
  }
}

void hip_resource_grid::prune() const
{
  // completed producers need no waiting any more: their events go back to the pool
  for (auto* list : {&producers, &retired}) {
    for (size_t i = 0; i < list->size();) {
      const hipError_t q = hipEventQuery((*list)[i]);
      if (q == hipErrorNotReady) {
        ++i;
        continue;
      }
      if (q != hipSuccess) {
        (void)hipGetLastError();
      }
      spare.push_back((*list)[i]);
      (*list)[i] = list->back();
      list->pop_back();
    }
  }
}

void hip_resource_grid::wait_producers(hipStream_t s) const
{
  prune();
  for (hipEvent_t e : producers) {
    check(hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent");
  }
}

void hip_resource_grid::sync_producers() const
{
  for (hipEvent_t e : producers) {
    check(hipEventSynchronize(e), "hipEventSynchronize");
  }
  spare.insert(spare.end(), producers.begin(), producers.end());
  producers.clear();
}

hip_resource_grid::~hip_resource_grid()
{
  {
    std::lock_guard<std::mutex> lock(mtx);
    for (hip_grid_deferred_writer* w : deferred) {
      w->detach(*this);
    }
    deferred.clear();
  }
  (void)hipSetDevice(dev);
  if (own != nullptr) {
    (void)hipStreamSynchronize(own);
  }
  for (auto* list : {&producers, &retired, &spare}) {
    for (hipEvent_t e : *list) {
      (void)hipEventSynchronize(e);
      (void)hipEventDestroy(e);
    }
  }
  if (own != nullptr) {
    (void)hipStreamDestroy(own);
  }
  (void)hipFree(d);
  (void)hipFree(d_delta);
  (void)hipFree(d_rows);
}

void hip_resource_grid::set_all_zero()
{
  std::unique_lock<std::mutex> lock(mtx);
  cv.wait(lock, [this] { return pending == 0; });
  run_deferred(nullptr); // (ordered before the zeroing, as the reference's writes before set_all_zero are)
  ++ver;
  host->set_all_zero();
  std::fill(base.begin(), base.end(), 0u);
  check(hipSetDevice(dev), "hipSetDevice");
  // the zeroing follows every earlier producer and supersedes them: the next accesses wait for it alone
  wait_producers(own);
  check(hipMemsetAsync(d, 0, sizeof(uint32_t) * ports * symbols * subc, own), "hipMemsetAsync");
  retired.insert(retired.end(), producers.begin(), producers.end());
  producers.clear();
  add_producer(own);
  host_dirty   = false;
  view_open    = false; // the slot boundary: writes through earlier views are over
  device_dirty = false;
}

void hip_resource_grid::host_access(std::unique_lock<std::mutex>& lock, bool write) const
{
  // every device writer has published its completion (device_written); staged writes issued
  cv.wait(lock, [this] { return pending == 0; });
  run_deferred(nullptr);
  if (device_dirty) {
    // the device's changes since the last agreement: host ^= device ^ base, base = device
    auto* self = const_cast<hip_resource_grid*>(this);
    check(hipSetDevice(dev), "hipSetDevice");
    sync_producers();
    std::vector<uint32_t> now(base.size());
    check(hipMemcpy(now.data(), d, sizeof(uint32_t) * now.size(), hipMemcpyDeviceToHost), "download");
    resource_grid_writer& w = self->host->get_writer();
    for (unsigned p = 0; p != ports; ++p) {
      for (unsigned l = 0; l != symbols; ++l) {
        const size_t    o  = (static_cast<size_t>(p) * symbols + l) * subc;
        const uint32_t* dv = now.data() + o;
        uint32_t*       bv = base.data() + o;
        if (std::memcmp(dv, bv, sizeof(uint32_t) * subc) == 0) {
          continue;
        }
        // (the host grid's writer view also marks the port non-empty)
        span<cbf16_t> v  = w.get_view(p, l);
        auto*         hv = reinterpret_cast<uint32_t*>(v.data());
        for (unsigned k = 0; k != subc; ++k) {
          hv[k] ^= dv[k] ^ bv[k];
          bv[k] = dv[k];
        }
      }
    }
    device_dirty = false;
    ++downloads;
  }
  if (write) {
    host_dirty = true;
    ++ver;
  }
}

void hip_resource_grid::device_access(std::unique_lock<std::mutex>& lock, hipStream_t stream, bool write)
{
  check(hipSetDevice(dev), "hipSetDevice");
  if (!write) {
    // readers see every producer (a writer does not need the others: disjoint REs), staged writes included
    cv.wait(lock, [this] { return pending == 0; });
    run_deferred(nullptr);
  }
  if (host_dirty) {
    // the host's changes since the last agreement: delta = host ^ base per changed row, applied on the device where
    // non-zero (srs_amd_grid_merge_rows); base = host
    const size_t          rows = static_cast<size_t>(ports) * symbols;
    std::vector<uint32_t> delta, ids;
    const resource_grid_reader& r = host->get_reader();
    for (unsigned p = 0; p != ports; ++p) {
      for (unsigned l = 0; l != symbols; ++l) {
        const size_t        o  = (static_cast<size_t>(p) * symbols + l) * subc;
        span<const cbf16_t> v  = r.get_view(p, l);
        const auto*         hv = reinterpret_cast<const uint32_t*>(v.data());
        uint32_t*           bv = base.data() + o;
        if (std::memcmp(hv, bv, sizeof(uint32_t) * subc) == 0) {
          continue;
        }
        const size_t q = delta.size();
        delta.resize(q + subc);
        for (unsigned k = 0; k != subc; ++k) {
          const uint32_t x = hv[k]; // read once: a writer may still be writing through its view
          delta[q + k]     = x ^ bv[k];
          bv[k]            = x;
        }
        ids.push_back(static_cast<uint32_t>(p * symbols + l));
      }
    }
    if (!ids.empty()) {
      if (d_delta == nullptr) {
        check(hipMalloc(&d_delta, sizeof(uint32_t) * rows * subc), "hipMalloc");
        check(hipMalloc(&d_rows, sizeof(uint32_t) * rows), "hipMalloc");
      }
      wait_producers(own);
      check(hipMemcpyAsync(d_delta, delta.data(), sizeof(uint32_t) * delta.size(), hipMemcpyHostToDevice, own), "upload");
      check(hipMemcpyAsync(d_rows, ids.data(), sizeof(uint32_t) * ids.size(), hipMemcpyHostToDevice, own), "upload");
      if (srs_amd_grid_merge_rows(d, d_delta, d_rows, static_cast<uint32_t>(ids.size()), subc, own) != SRS_AMD_OK) {
        throw std::runtime_error(std::string("hip_resource_grid: merge: ") + srs_amd_last_error());
      }
      add_producer(own);
      check(hipStreamSynchronize(own), "upload"); // pageable host memory: the copies are done when this returns
      ++uploads;
    }
    // a writable view still out: later writes are merged by the next device access -- until a device READER finds
    // nothing new (a reader consumes the finished slot: the reference's host writers are done by then)
    if (!write && ids.empty()) {
      view_open = false;
    }
    host_dirty = view_open;
  }
  // every producer still running (a completed one needs no stream wait packet)
  wait_producers(stream);
  if (write) {
    device_dirty = true;
    ++ver;
  }
}

const uint32_t* hip_resource_grid::device_read(hipStream_t stream, uint64_t* version)
{
  std::unique_lock<std::mutex> lock(mtx);
  device_access(lock, stream, false);
  if (version != nullptr) {
    *version = ver;
  }
  return d;
}

void hip_resource_grid::run_deferred(hip_grid_deferred_writer* only) const
{
  for (auto it = deferred.begin(); it != deferred.end();) {
    hip_grid_deferred_writer* w = *it;
    if (only != nullptr && w != only) {
      ++it;
      continue;
    }
    it                = deferred.erase(it);
    hipStream_t     s = w->stream();
    check(hipSetDevice(dev), "hipSetDevice");
    wait_producers(s);
    w->issue(*const_cast<hip_resource_grid*>(this), d);
    add_producer(s);
    device_dirty = true;
  }
}

void hip_resource_grid::defer(hip_grid_deferred_writer& w)
{
  std::lock_guard<std::mutex> lock(mtx);
  if (std::find(deferred.begin(), deferred.end(), &w) == deferred.end()) {
    deferred.push_back(&w);
    w.attached(*this);
  }
  device_dirty = true;
  ++ver;
}

void hip_resource_grid::issue_deferred(hip_grid_deferred_writer& w)
{
  std::lock_guard<std::mutex> lock(mtx);
  run_deferred(&w);
}

bool hip_resource_grid::unchanged_since(uint64_t version) const
{
  std::lock_guard<std::mutex> lock(mtx);
  return version == ver && !host_dirty && pending == 0 && deferred.empty();
}

uint32_t* hip_resource_grid::device_write(hipStream_t stream)
{
  std::unique_lock<std::mutex> lock(mtx);
  device_access(lock, stream, true);
  ++pending;
  return d;
}

void hip_resource_grid::device_written(hipStream_t stream)
{
  {
    std::lock_guard<std::mutex> lock(mtx);
    check(hipSetDevice(dev), "hipSetDevice");
    // one more producer: later readers wait for its event (and each other producer's still running)
    add_producer(stream);
    device_dirty = true;
    pending      = pending > 0 ? pending - 1 : 0;
    ++ver;
  }
  cv.notify_all();
}

// ---- reader ----

unsigned hip_grid_reader::get_nof_ports() const
{
  return grid.ports;
}
unsigned hip_grid_reader::get_nof_subc() const
{
  return grid.subc;
}
unsigned hip_grid_reader::get_nof_symbols() const
{
  return grid.symbols;
}
bool hip_grid_reader::is_empty(unsigned port) const
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  // written on the device (or being written): not empty
  return grid.pending == 0 && !grid.device_dirty && grid.host->get_reader().is_empty(port);
}
bool hip_grid_reader::is_empty() const
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  return grid.pending == 0 && !grid.device_dirty && grid.host->get_reader().is_empty();
}
span<cf_t> hip_grid_reader::get(span<cf_t> symbols, unsigned port, unsigned l, unsigned k_init,
                                const bounded_bitset<MAX_RB * NRE>& mask) const
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, false);
  return grid.host->get_reader().get(symbols, port, l, k_init, mask);
}
span<cbf16_t> hip_grid_reader::get(span<cbf16_t> symbols, unsigned port, unsigned l, unsigned k_init,
                                   const bounded_bitset<MAX_RB * NRE>& mask) const
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, false);
  return grid.host->get_reader().get(symbols, port, l, k_init, mask);
}
void hip_grid_reader::get(span<cf_t> symbols, unsigned port, unsigned l, unsigned k_init, unsigned stride) const
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, false);
  grid.host->get_reader().get(symbols, port, l, k_init, stride);
}
void hip_grid_reader::get(span<cbf16_t> symbols, unsigned port, unsigned l, unsigned k_init) const
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, false);
  grid.host->get_reader().get(symbols, port, l, k_init);
}
span<const cbf16_t> hip_grid_reader::get_view(unsigned port, unsigned l) const
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, false);
  return grid.host->get_reader().get_view(port, l);
}

// ---- writer ----

unsigned hip_grid_writer::get_nof_ports() const
{
  return grid.ports;
}
unsigned hip_grid_writer::get_nof_subc() const
{
  return grid.subc;
}
unsigned hip_grid_writer::get_nof_symbols() const
{
  return grid.symbols;
}
span<const cf_t> hip_grid_writer::put(unsigned port, unsigned l, unsigned k_init,
                                      const bounded_bitset<NRE * MAX_RB>& mask, span<const cf_t> symbols)
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, true);
  return grid.host->get_writer().put(port, l, k_init, mask, symbols);
}
span<const cbf16_t> hip_grid_writer::put(unsigned port, unsigned l, unsigned k_init,
                                         const bounded_bitset<NRE * MAX_RB>& mask, span<const cbf16_t> symbols)
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, true);
  return grid.host->get_writer().put(port, l, k_init, mask, symbols);
}
void hip_grid_writer::put(unsigned port, unsigned l, unsigned k_init, span<const cf_t> symbols)
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, true);
  grid.host->get_writer().put(port, l, k_init, symbols);
}
void hip_grid_writer::put(unsigned port, unsigned l, unsigned k_init, unsigned stride, span<const cbf16_t> symbols)
{
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, true);
  grid.host->get_writer().put(port, l, k_init, stride, symbols);
}
span<cbf16_t> hip_grid_writer::get_view(unsigned port, unsigned l)
{
  // the caller writes through the view after this returns (the reference's mapper and PRS generator do): the host
  // side stays dirty until the slot boundary, so writes made after a device access are merged by the next one
  std::unique_lock<std::mutex> lock(grid.mtx);
  grid.host_access(lock, true);
  grid.mark_view_open();
  return grid.host->get_writer().get_view(port, l);
}

// ---- factory ----

namespace {

class hip_resource_grid_factory : public resource_grid_factory
{
public:
  hip_resource_grid_factory(std::shared_ptr<resource_grid_factory> h, int d) : host(std::move(h)), device(d) {}
  std::unique_ptr<resource_grid> create(unsigned nof_ports, unsigned nof_symbols, unsigned nof_subc) override
  {
    return std::make_unique<hip_resource_grid>(host->create(nof_ports, nof_symbols, nof_subc), device);
  }

private:
  std::shared_ptr<resource_grid_factory> host;
  int                                    device;
};

} // namespace

std::shared_ptr<resource_grid_factory>
srsran::hip::create_hip_resource_grid_factory(std::shared_ptr<resource_grid_factory> host_factory, int device)
{
  return host_factory ? std::make_shared<hip_resource_grid_factory>(std::move(host_factory), device) : nullptr;
}
