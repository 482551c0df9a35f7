// hip_resource_grid.h -- a device-resident srsran::resource_grid (include/srsran/phy/support/resource_grid.h:35-49)
// for the MI355X plug-ins: the slot grid lives in HBM as cbf16 [port][symbol][subcarrier] (the layout of the
// srsran_amd C-ABI grids), next to a host mirror -- any resource_grid the reference's own factory builds
// (support_factories.h create_resource_grid_factory) -- that the reader / writer interfaces serve.
//
// Plug-ins that understand it (pusch_processor_hip, pdsch_processor_hip, pdcch / ssb / pucch, the OFDM plug-ins of
// ofdm_modulator_hip) reach the device copy through hip_grid_reader / hip_grid_writer and run on it directly: the
// uplink grid the OFDM demodulator plug-in writes is read by the PUSCH plug-in without crossing PCIe, and the downlink
// grid the PDSCH plug-in writes is read in place by the OFDM modulator plug-in (whose samples then go to the host, as
// its interface returns them).  Every other component keeps the reference interfaces: the first host access after a
// device write downloads the grid (once), the first device access after a host write uploads it.
//
// Deferred writers (r06): a device producer may stage its writes on the host and register with defer(); they are
// issued (hip_grid_deferred_writer::issue, one launch for everything staged) before the next access of either copy,
// at set_all_zero, or when the producer asks (issue_deferred).  The OFDM symbol demodulator plug-in works this way:
// a demodulate() call per port and symbol (puxch_processor_impl.cpp:73-82) costs a host copy of its samples, the
// slot's symbols go to the device in one launch when the PUSCH plug-in (or anything else) reads the grid.
//
// Coherence (r06): a three-way merge against the state both copies last agreed on (`base`, a host array).  Host
// writers (the reference's channel processors through put / get_view) change the host mirror, device writers (the
// plug-ins' kernels) the device copy, concurrently and on disjoint REs as the downlink processor's executors do
// (downlink_processor_multi_executor_impl.cpp).  Before a device access the host's changes go up as the XOR of each
// changed row with `base`, applied on the device only where non-zero (srs_amd_grid_merge_rows), so REs the device
// wrote meanwhile stay; before a host access the device's changes come down the same way (host ^= device ^ base), so
// REs the host wrote meanwhile stay.  A writable view handed out by get_view keeps the host side dirty until the slot
// boundary (set_all_zero) or until a device reader finds no host change left (readers consume the finished slot):
// writes through it after an upload are merged by the next device access.  Every device
// writer is tracked: device_write / device_written bracket it (a pending count host accesses and device readers wait
// for), and each device_written records an event of its own on the writer's stream; readers wait for every producer
// event still running (r06: no join through a grid-owned stream, whose packets could sit in a hardware queue ahead of
// unrelated work), so they wait for every producer, not only the last.  Calls are
// serialised per grid by a mutex.  An RE written on both sides between two merges keeps neither value exactly (XOR):
// the reference's processors never write the same RE twice in a slot.
#pragma once

#include "srsran/phy/support/resource_grid.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran/phy/support/support_factories.h"

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

namespace srsran {
namespace hip {

class hip_resource_grid;

/// A device producer whose writes are staged on the host and issued lazily (see the header comment).
class hip_grid_deferred_writer
{
public:
  virtual ~hip_grid_deferred_writer() = default;
  /// Issues every staged write for `grid` into its device copy `d`, kernels on stream() (which already waits for the
  /// grid's earlier producers).  Called with the grid locked.
  virtual void issue(hip_resource_grid& grid, uint32_t* d) = 0;
  /// The stream issue() launches on.
  virtual hipStream_t stream() const = 0;
  /// The grid is being destroyed: forget it, dropping what is staged for it.  Called with the grid locked.
  virtual void detach(hip_resource_grid& grid) = 0;
  /// The grid registered this writer (defer); issue() or detach() unregister it.  Called with the grid locked.
  virtual void attached(hip_resource_grid& grid) { (void)grid; }
};

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
  /// Unique over the process's grids (an address can be reused by a later grid; an identity cannot).
  uint64_t identity() const { return uid; }

  /// Device copy, current, for kernels on `stream` that read it (stream waits for every device producer);
  /// version (optional): the content version read (see unchanged_since).
  const uint32_t* device_read(hipStream_t stream, uint64_t* version = nullptr);
  /// Device copy, current, for kernels on `stream` that write it; the host mirror becomes stale.
  uint32_t* device_write(hipStream_t stream);
  /// The kernels that wrote the device copy were issued on `stream`: host accesses and other streams wait for them.
  void device_written(hipStream_t stream);

  /// `w` has writes staged for this grid: issued before the next access of either copy, at set_all_zero, or by
  /// issue_deferred(w).
  void defer(hip_grid_deferred_writer& w);
  /// Issues w's staged writes now (nothing when w is not registered).
  void issue_deferred(hip_grid_deferred_writer& w);
  /// Nothing was written (host or device, issued or staged, or through a writable view still out) since
  /// device_read returned `version`: a reader may reuse what it computed from that read.
  bool unchanged_since(uint64_t version) const;

  /// Transfers (for tests and statistics): host <- device downloads, device <- host uploads.
  uint64_t nof_downloads() const { return downloads; }
  uint64_t nof_uploads() const { return uploads; }

private:
  friend class hip_grid_reader;
  friend class hip_grid_writer;
  // the host mirror current (the device's changes merged in); write: the host side becomes dirty.  lock: mtx, held
  void host_access(std::unique_lock<std::mutex>& lock, bool write) const;
  // the device copy current on `stream` (the host's changes merged in; readers also wait for pending writers)
  void device_access(std::unique_lock<std::mutex>& lock, hipStream_t stream, bool write);
  // a writable view is out (get_view): the host side stays dirty until the slot boundary
  void mark_view_open() const { view_open = true; }
  // issues the registered deferred writers' staged writes (only: that one writer), lock held
  void run_deferred(hip_grid_deferred_writer* only) const;
  // producer events, lock held
  hipEvent_t take_event() const;
  void       add_producer(hipStream_t s) const;
  void       prune() const;
  void       wait_producers(hipStream_t s) const;
  void       sync_producers() const;

  std::unique_ptr<resource_grid> host;
  unsigned                       ports = 0, symbols = 0, subc = 0;
  int                            dev   = 0;
  uint64_t                       uid   = 0;
  uint32_t*                      d     = nullptr;
  hipStream_t                    own    = nullptr; // zeroing, merges
  // one event per device producer since the copies last agreed (writers, staged writes, zeroing, merges): readers
  // wait for those still running; completed ones go back to `spare`, superseded ones wait in `retired`
  mutable std::vector<hipEvent_t> producers, retired, spare;
  mutable std::mutex              mtx;
  mutable std::condition_variable cv;              // pending reaches 0
  mutable std::vector<uint32_t>   base;            // the state host and device copies last agreed on
  mutable bool                    host_dirty = false, view_open = false, device_dirty = false;
  mutable int                     pending    = 0;  // device writers between device_write and device_written
  mutable uint32_t*               d_delta    = nullptr; // merge staging: changed rows' XOR deltas, their row indices
  mutable uint32_t*               d_rows     = nullptr;
  mutable uint64_t                downloads = 0, uploads = 0;
  mutable uint64_t                ver       = 0; // content version: bumped by every write access
  mutable std::vector<hip_grid_deferred_writer*> deferred;
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
