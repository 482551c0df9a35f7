// hip_resource_grid.h -- a device-resident srsran::resource_grid (include/srsran/phy/support/resource_grid.h:35-49)
// for the MI355X plug-ins: the slot grid lives in HBM as cbf16 [port][symbol][subcarrier] (the layout of the
// srsran_amd C-ABI grids), next to a host mirror -- any resource_grid the reference's own factory builds
// (support_factories.h create_resource_grid_factory) -- that the reader / writer interfaces serve.
//
// Plug-ins that understand it (pusch_processor_hip, pdsch_processor_hip, the OFDM plug-ins) reach the device copy
// through hip_grid_reader / hip_grid_writer and run on it directly: the uplink grid the OFDM demodulator plug-in
// writes is read by the PUSCH plug-in without crossing PCIe, and the downlink grid the PDSCH plug-in writes goes to
// the OFDM modulator plug-in the same way.  Every other component keeps the reference interfaces: the first host
// access after a device write downloads the grid (once), the first device access after a host write uploads it.
//
// Coherence: two validity flags (host, device) and the completion event of the last device producer.  A reader or
// writer call makes the host copy valid first; a writer call then marks the device copy stale.  device_read /
// device_write make the device copy valid on the caller's stream (waiting for the last producer there);
// device_write also marks the host copy stale, and device_written records the producer's completion event.
// Calls are serialised per grid by a mutex, so the reference's concurrent channel processors may share a grid.
#pragma once

#include "srsran/phy/support/resource_grid.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran/phy/support/support_factories.h"

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>

namespace srsran {
namespace hip {

class hip_resource_grid;

/// Reader of a hip_resource_grid: the reference interface over the host mirror (downloaded on demand).
class hip_grid_reader : public resource_grid_reader
{
public:
  explicit hip_grid_reader(hip_resource_grid& g) : grid(g) {}
  hip_resource_grid& owner() const { return grid; }

  unsigned            get_nof_ports() const override;
  unsigned            get_nof_subc() const override;
  unsigned            get_nof_symbols() const override;
  bool                is_empty(unsigned port) const override;
  bool                is_empty() const override;
  span<cf_t>          get(span<cf_t> symbols, unsigned port, unsigned l, unsigned k_init,
                          const bounded_bitset<MAX_RB * NRE>& mask) const override;
  span<cbf16_t>       get(span<cbf16_t> symbols, unsigned port, unsigned l, unsigned k_init,
                          const bounded_bitset<MAX_RB * NRE>& mask) const override;
  void                get(span<cf_t> symbols, unsigned port, unsigned l, unsigned k_init, unsigned stride) const override;
  void                get(span<cbf16_t> symbols, unsigned port, unsigned l, unsigned k_init) const override;
  span<const cbf16_t> get_view(unsigned port, unsigned l) const override;

private:
  hip_resource_grid& grid;
};

/// Writer of a hip_resource_grid: the reference interface over the host mirror (the device copy becomes stale).
class hip_grid_writer : public resource_grid_writer
{
public:
  explicit hip_grid_writer(hip_resource_grid& g) : grid(g) {}
  hip_resource_grid& owner() const { return grid; }

  unsigned            get_nof_ports() const override;
  unsigned            get_nof_subc() const override;
  unsigned            get_nof_symbols() const override;
  span<const cf_t>    put(unsigned port, unsigned l, unsigned k_init, const bounded_bitset<NRE * MAX_RB>& mask,
                          span<const cf_t> symbols) override;
  span<const cbf16_t> put(unsigned port, unsigned l, unsigned k_init, const bounded_bitset<NRE * MAX_RB>& mask,
                          span<const cbf16_t> symbols) override;
  void                put(unsigned port, unsigned l, unsigned k_init, span<const cf_t> symbols) override;
  void                put(unsigned port, unsigned l, unsigned k_init, unsigned stride, span<const cbf16_t> symbols) override;
  span<cbf16_t>       get_view(unsigned port, unsigned l) override;

private:
  hip_resource_grid& grid;
};

class hip_resource_grid : public resource_grid
{
public:
  /// host: the host mirror (any reference resource_grid of the same dimensions); device: HIP device of the copy.
  hip_resource_grid(std::unique_ptr<resource_grid> host, int device);
  ~hip_resource_grid() override;

  // resource_grid
  void                        set_all_zero() override;
  resource_grid_writer&       get_writer() override { return writer; }
  const resource_grid_reader& get_reader() const override { return reader; }

  unsigned nof_ports() const { return ports; }
  unsigned nof_symbols() const { return symbols; }
  unsigned nof_subc() const { return subc; }
  int      device() const { return dev; }

  /// Device copy, current, for kernels on `stream` that read it (stream waits for the last device producer).
  const uint32_t* device_read(hipStream_t stream);
  /// Device copy, current, for kernels on `stream` that write it; the host mirror becomes stale.
  uint32_t* device_write(hipStream_t stream);
  /// The kernels that wrote the device copy were issued on `stream`: host accesses and other streams wait for them.
  void device_written(hipStream_t stream);

  /// Transfers (for tests and statistics): host <- device downloads, device <- host uploads.
  uint64_t nof_downloads() const { return downloads; }
  uint64_t nof_uploads() const { return uploads; }

private:
  friend class hip_grid_reader;
  friend class hip_grid_writer;
  // the host mirror valid (download when the device copy is newer); write: the device copy then becomes stale
  void host_access(bool write) const;
  // the device copy valid on `stream` (upload when the host mirror is newer)
  void device_access(hipStream_t stream, bool write);

  std::unique_ptr<resource_grid> host;
  unsigned                       ports = 0, symbols = 0, subc = 0;
  int                            dev   = 0;
  uint32_t*                      d     = nullptr;
  hipEvent_t                     ready = nullptr; // the last device producer's completion
  hipStream_t                    own   = nullptr; // transfers
  mutable std::mutex             mtx;
  mutable bool                   host_valid = true, device_valid = true, producer = false;
  mutable uint64_t               downloads = 0, uploads = 0;
  hip_grid_reader                reader;
  hip_grid_writer                writer;
};

/// resource_grid_factory whose grids are hip_resource_grids over the grids of `host_factory` (the reference's
/// create_resource_grid_factory(), or any other), on HIP device `device` (-1: the current one).
std::shared_ptr<resource_grid_factory> create_hip_resource_grid_factory(std::shared_ptr<resource_grid_factory> host_factory,
                                                                        int                                    device = -1);

/// The hip_resource_grid behind a reader / writer, or nullptr when it is another kind of grid.
inline hip_resource_grid* hip_grid_of(const resource_grid_reader& r)
{
  const auto* h = dynamic_cast<const hip_grid_reader*>(&r);
  return h != nullptr ? &h->owner() : nullptr;
}
inline hip_resource_grid* hip_grid_of(resource_grid_writer& w)
{
  auto* h = dynamic_cast<hip_grid_writer*>(&w);
  return h != nullptr ? &h->owner() : nullptr;
}

} // namespace hip
} // namespace srsran
