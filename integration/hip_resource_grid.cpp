// hip_resource_grid.cpp -- device-resident srsran::resource_grid (see the header).
#include "hip_resource_grid.h"

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
  check(hipMalloc(&d, sizeof(uint32_t) * ports * symbols * subc), "hipMalloc");
  check(hipStreamCreateWithFlags(&own, hipStreamNonBlocking), "stream");
  check(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "event");
  // the host mirror starts as the reference grid does (all zero): so does the device copy
  check(hipMemsetAsync(d, 0, sizeof(uint32_t) * ports * symbols * subc, own), "hipMemsetAsync");
  check(hipEventRecord(ready, own), "hipEventRecord");
  producer = true;
}

hip_resource_grid::~hip_resource_grid()
{
  (void)hipSetDevice(dev);
  if (own != nullptr) {
    (void)hipStreamSynchronize(own);
  }
  if (ready != nullptr) {
    (void)hipEventSynchronize(ready);
    (void)hipEventDestroy(ready);
  }
  if (own != nullptr) {
    (void)hipStreamDestroy(own);
  }
  (void)hipFree(d);
}

void hip_resource_grid::set_all_zero()
{
  std::lock_guard<std::mutex> lock(mtx);
  host->set_all_zero();
  check(hipSetDevice(dev), "hipSetDevice");
  if (producer) {
    check(hipStreamWaitEvent(own, ready, 0), "hipStreamWaitEvent");
  }
  check(hipMemsetAsync(d, 0, sizeof(uint32_t) * ports * symbols * subc, own), "hipMemsetAsync");
  check(hipEventRecord(ready, own), "hipEventRecord");
  producer     = true;
  host_valid   = true;
  device_valid = true;
}

void hip_resource_grid::host_access(bool write) const
{
  // (the caller holds mtx)
  if (!host_valid) {
    auto* self = const_cast<hip_resource_grid*>(this);
    check(hipSetDevice(dev), "hipSetDevice");
    check(hipEventSynchronize(ready), "hipEventSynchronize");
    // one row per (port, symbol): the host grid's writer views (which also mark the ports non-empty)
    resource_grid_writer& w = self->host->get_writer();
    for (unsigned p = 0; p != ports; ++p) {
      for (unsigned l = 0; l != symbols; ++l) {
        span<cbf16_t> v = w.get_view(p, l);
        check(hipMemcpy(v.data(), d + (static_cast<size_t>(p) * symbols + l) * subc, sizeof(uint32_t) * subc,
                        hipMemcpyDeviceToHost),
              "download");
      }
    }
    host_valid = true;
    ++downloads;
  }
  if (write) {
    device_valid = false;
  }
}

void hip_resource_grid::device_access(hipStream_t stream, bool write)
{
  // (the caller holds mtx)
  check(hipSetDevice(dev), "hipSetDevice");
  if (!device_valid) {
    if (producer) {
      check(hipStreamWaitEvent(own, ready, 0), "hipStreamWaitEvent");
    }
    const resource_grid_reader& r = host->get_reader();
    for (unsigned p = 0; p != ports; ++p) {
      for (unsigned l = 0; l != symbols; ++l) {
        span<const cbf16_t> v = r.get_view(p, l);
        check(hipMemcpyAsync(d + (static_cast<size_t>(p) * symbols + l) * subc, v.data(), sizeof(uint32_t) * subc,
                             hipMemcpyHostToDevice, own),
              "upload");
      }
    }
    check(hipEventRecord(ready, own), "hipEventRecord");
    check(hipStreamSynchronize(own), "upload"); // pageable host memory: the copies are done when this returns
    producer     = true;
    device_valid = true;
    ++uploads;
  }
  if (producer) {
    check(hipStreamWaitEvent(stream, ready, 0), "hipStreamWaitEvent");
  }
  if (write) {
    host_valid = false;
  }
}

const uint32_t* hip_resource_grid::device_read(hipStream_t stream)
{
  std::lock_guard<std::mutex> lock(mtx);
  device_access(stream, false);
  return d;
}

uint32_t* hip_resource_grid::device_write(hipStream_t stream)
{
  std::lock_guard<std::mutex> lock(mtx);
  device_access(stream, true);
  return d;
}

void hip_resource_grid::device_written(hipStream_t stream)
{
  std::lock_guard<std::mutex> lock(mtx);
  check(hipSetDevice(dev), "hipSetDevice");
  check(hipEventRecord(ready, stream), "hipEventRecord");
  producer   = true;
  host_valid = false;
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
  return grid.host_valid && grid.host->get_reader().is_empty(port); // written on the device: not empty
}
bool hip_grid_reader::is_empty() const
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  return grid.host_valid && grid.host->get_reader().is_empty();
}
span<cf_t> hip_grid_reader::get(span<cf_t> symbols, unsigned port, unsigned l, unsigned k_init,
                                const bounded_bitset<MAX_RB * NRE>& mask) const
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(false);
  return grid.host->get_reader().get(symbols, port, l, k_init, mask);
}
span<cbf16_t> hip_grid_reader::get(span<cbf16_t> symbols, unsigned port, unsigned l, unsigned k_init,
                                   const bounded_bitset<MAX_RB * NRE>& mask) const
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(false);
  return grid.host->get_reader().get(symbols, port, l, k_init, mask);
}
void hip_grid_reader::get(span<cf_t> symbols, unsigned port, unsigned l, unsigned k_init, unsigned stride) const
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(false);
  grid.host->get_reader().get(symbols, port, l, k_init, stride);
}
void hip_grid_reader::get(span<cbf16_t> symbols, unsigned port, unsigned l, unsigned k_init) const
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(false);
  grid.host->get_reader().get(symbols, port, l, k_init);
}
span<const cbf16_t> hip_grid_reader::get_view(unsigned port, unsigned l) const
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(false);
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
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(true);
  return grid.host->get_writer().put(port, l, k_init, mask, symbols);
}
span<const cbf16_t> hip_grid_writer::put(unsigned port, unsigned l, unsigned k_init,
                                         const bounded_bitset<NRE * MAX_RB>& mask, span<const cbf16_t> symbols)
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(true);
  return grid.host->get_writer().put(port, l, k_init, mask, symbols);
}
void hip_grid_writer::put(unsigned port, unsigned l, unsigned k_init, span<const cf_t> symbols)
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(true);
  grid.host->get_writer().put(port, l, k_init, symbols);
}
void hip_grid_writer::put(unsigned port, unsigned l, unsigned k_init, unsigned stride, span<const cbf16_t> symbols)
{
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(true);
  grid.host->get_writer().put(port, l, k_init, stride, symbols);
}
span<cbf16_t> hip_grid_writer::get_view(unsigned port, unsigned l)
{
  // the caller writes through the view after this returns: the device copy is stale from here on
  std::lock_guard<std::mutex> lock(grid.mtx);
  grid.host_access(true);
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
