// ofdm_modulator_hip.cpp -- srsran::ofdm_{slot,symbol}_{modulator,demodulator} over the srsran_amd OFDM C-ABI
// (see the header).
#include "ofdm_modulator_hip.h"
#include "hip_resource_grid.h"

#include "srsran/phy/lower/modulation/ofdm_demodulator.h"
#include "srsran/phy/lower/modulation/ofdm_modulator.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran_amd/ofdm.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

using namespace srsran;

namespace {

// Pinned host buffer, grown on demand.
struct pinned_buffer {
  void*  ptr  = nullptr;
  size_t size = 0;
  pinned_buffer() = default;
  pinned_buffer(const pinned_buffer&)            = delete;
  pinned_buffer& operator=(const pinned_buffer&) = delete;
  ~pinned_buffer() { (void)hipHostFree(ptr); }
  bool ensure(size_t n)
  {
    if (n <= size) {
      return true;
    }
    (void)hipHostFree(ptr);
    ptr  = nullptr;
    size = 0;
    if (hipHostMalloc(&ptr, n, hipHostMallocDefault) != hipSuccess) {
      return false;
    }
    size = n;
    return true;
  }
  template <typename T>
  T* as()
  {
    return static_cast<T*>(ptr);
  }
};

// Per plug-in object: the stream its launches on device-resident grids go to.
struct device_stream {
  hipStream_t s   = nullptr;
  int         dev = -1;
  explicit device_stream(int device) : dev(device)
  {
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      s = nullptr;
    }
  }
  void drain() const
  {
    if (s != nullptr) {
      (void)hipStreamSynchronize(s);
    }
  }
  device_stream(const device_stream&)            = delete;
  device_stream& operator=(const device_stream&) = delete;
  ~device_stream()
  {
    if (s != nullptr) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
  }
};

srs_amd_ofdm_config to_c(unsigned numerology, unsigned bw_rb, unsigned dft_size, cyclic_prefix cp, unsigned offset,
                         float scale, double fc)
{
  srs_amd_ofdm_config c{};
  c.numerology                = numerology;
  c.bw_rb                     = bw_rb;
  c.dft_size                  = dft_size;
  c.cp_extended               = cp == cyclic_prefix::EXTENDED ? 1 : 0;
  c.nof_samples_window_offset = offset;
  c.scale                     = scale;
  c.center_freq_hz            = fc;
  return c;
}

int resolve_device(int device)
{
  int dev = device;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
    return -1;
  }
  return dev;
}

void report(const char* what)
{
  std::fprintf(stderr, "%s: %s\n", what, srs_amd_last_error());
}

void report_geometry(const char* what, const hip::hip_resource_grid& g)
{
  std::fprintf(stderr, "%s: device-resident grid of %u ports x %u symbols x %u subcarriers not usable here\n", what,
               g.nof_ports(), g.nof_symbols(), g.nof_subc());
}

// Reads nsymb rows (symbols first_l .. first_l + nsymb - 1 of the slot) of one port into staging, nsubc cbf16 each.
bool read_rows(const resource_grid_reader& grid, unsigned port, unsigned first_l, unsigned nsymb, unsigned nsubc,
               uint16_t* dst)
{
  for (unsigned l = 0; l != nsymb; ++l) {
    span<const cbf16_t> row = grid.get_view(port, first_l + l);
    if (row.size() < nsubc) {
      return false;
    }
    std::memcpy(dst + 2 * static_cast<size_t>(l) * nsubc, row.data(), sizeof(cbf16_t) * nsubc);
  }
  return true;
}

void write_rows(resource_grid_writer& grid, unsigned port, unsigned first_l, unsigned nsymb, unsigned nsubc,
                const uint16_t* src)
{
  for (unsigned l = 0; l != nsymb; ++l) {
    span<cbf16_t> row = grid.get_view(port, first_l + l);
    std::memcpy(static_cast<void*>(row.data()), src + 2 * static_cast<size_t>(l) * nsubc,
                sizeof(cbf16_t) * std::min<size_t>(nsubc, row.size()));
  }
}

// Staging of the samples between host and device for the device-resident forms (SRS_AMD_OFDM_STAGING):
//   zero-copy   : the transform kernels read / write pinned memory over the bus themselves;
//   dma         : DMA copies (hipMemcpyAsync) to / from HBM around the transform;
//   copy-kernel : (demodulator) a copy kernel with wide reads pulls the pinned samples into HBM first.
enum class staging { zero_copy, dma, copy_kernel };

staging staging_mode(bool demod)
{
  const char* v = std::getenv("SRS_AMD_OFDM_STAGING");
  if (v != nullptr && std::strcmp(v, "zero-copy") == 0) {
    return staging::zero_copy;
  }
  if (v != nullptr && std::strcmp(v, "dma") == 0) {
    return staging::dma;
  }
  if (v != nullptr && std::strcmp(v, "copy-kernel") == 0) {
    return demod ? staging::copy_kernel : staging::dma;
  }
  // measured defaults (profiles/r06_ofdm_symbol_plugin_rate.json)
  return demod ? staging::zero_copy : staging::dma;
}

// ---- modulators on a device-resident grid: every port of the slot modulated in one launch, in place ----

// The modulated samples of every port of one slot of one hip_resource_grid, in pinned memory the kernel writes
// straight into, reused by later calls for the same slot while the grid is unchanged (hip_resource_grid::
// unchanged_since): the lower PHY modulates a finished grid port by port, symbol by symbol
// (pdxch_processor_impl.cpp), so one launch serves every call of the slot.
class slot_samples_cache
{
public:
  slot_samples_cache(srs_amd_ofdm_modulator* m, unsigned nsymb_, unsigned nsubc_, int dev) :
    mod(m), nsymb(nsymb_), nsubc(nsubc_), stream(dev)
  {
  }
  ~slot_samples_cache()
  {
    stream.drain();
    (void)hipFree(d_out);
  }
  void drain() const { stream.drain(); }
  void invalidate() { grid = 0; }

  // samples of (port, slot) (get_slot_size(slot) of them), or nullptr on a refused geometry / launch failure
  const cf_t* get(hip::hip_resource_grid& g, unsigned port, unsigned slot, const char* who)
  {
    if (grid != g.identity() || slot != cached_slot || !g.unchanged_since(version)) {
      grid = 0;
      if (stream.s == nullptr || g.nof_symbols() != nsymb || g.nof_subc() != nsubc) {
        report_geometry(who, g);
        return nullptr;
      }
      slot_size = srs_amd_ofdm_modulator_get_slot_size(mod, slot);
      if (slot_size == 0 || !out.ensure(sizeof(cf_t) * slot_size * g.nof_ports())) {
        report(who);
        return nullptr;
      }
      const size_t bytes = sizeof(cf_t) * slot_size * g.nof_ports();
      if (dma && bytes > d_out_size) {
        (void)hipFree(d_out);
        d_out_size = hipMalloc(&d_out, bytes) == hipSuccess ? bytes : 0;
      }
      if (dma && d_out_size == 0) {
        report(who);
        return nullptr;
      }
      const uint32_t* d = g.device_read(stream.s, &version);
      // the samples into HBM then one DMA copy to pinned memory, or written by the kernel over the bus
      float* target = dma ? static_cast<float*>(d_out) : out.as<float>();
      if (srs_amd_ofdm_modulate_batch(mod, reinterpret_cast<const uint16_t*>(d), g.nof_ports(), slot, 1, target,
                                      slot_size, stream.s) != SRS_AMD_OK ||
          (dma && hipMemcpyAsync(out.ptr, d_out, bytes, hipMemcpyDeviceToHost, stream.s) != hipSuccess) ||
          hipStreamSynchronize(stream.s) != hipSuccess) {
        report(who);
        return nullptr;
      }
      grid        = g.identity();
      cached_slot = slot;
    }
    return port < g.nof_ports() ? out.as<cf_t>() + static_cast<size_t>(port) * slot_size : nullptr;
  }

private:
  srs_amd_ofdm_modulator* mod;
  unsigned                nsymb, nsubc;
  device_stream           stream;
  pinned_buffer           out;
  const bool              dma         = staging_mode(false) == staging::dma;
  void*                   d_out       = nullptr; // (DMA staging) the slot's samples in HBM
  size_t                  d_out_size  = 0;
  uint64_t                grid        = 0; // identity of the grid cached (0: none)
  unsigned                cached_slot = 0, slot_size = 0;
  uint64_t                version     = 0;
};

class ofdm_slot_modulator_hip : public ofdm_slot_modulator
{
public:
  ofdm_slot_modulator_hip(srs_amd_ofdm_modulator* m, unsigned nsymb_, unsigned nsubc_, int dev) :
    mod(m), nsymb(nsymb_), nsubc(nsubc_), cache(m, nsymb_, nsubc_, dev)
  {
  }
  ~ofdm_slot_modulator_hip() override
  {
    cache.drain();
    srs_amd_ofdm_modulator_destroy(mod);
  }

  unsigned get_slot_size(unsigned slot_index) const override
  {
    return srs_amd_ofdm_modulator_get_slot_size(mod, slot_index);
  }

  void modulate(span<cf_t> output, const resource_grid_reader& grid, unsigned port_index, unsigned slot_index) override
  {
    const unsigned n = get_slot_size(slot_index);
    if (n == 0 || output.size() != n) {
      std::fprintf(stderr, "ofdm_slot_modulator_hip: output of %zu samples, slot %u has %u\n", output.size(),
                   slot_index, n);
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    // an empty port modulates to zeros (ofdm_symbol_modulator_impl::modulate)
    if (grid.is_empty(port_index)) {
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    // a device-resident grid (the PDSCH plug-in wrote it in HBM): every port of the slot modulated in place at the
    // first call, the samples written straight into pinned memory
    if (hip::hip_resource_grid* hg = hip::hip_grid_of(grid)) {
      const cf_t* x = cache.get(*hg, port_index, slot_index, "ofdm_slot_modulator_hip");
      if (x == nullptr) {
        std::fill(output.begin(), output.end(), cf_t());
        return;
      }
      std::memcpy(static_cast<void*>(output.data()), x, sizeof(cf_t) * n);
      return;
    }
    if (!in.ensure(sizeof(uint32_t) * nsymb * nsubc) || !out.ensure(sizeof(cf_t) * n) ||
        !read_rows(grid, port_index, 0, nsymb, nsubc, in.as<uint16_t>()) ||
        srs_amd_ofdm_modulate_slot(mod, out.as<float>(), in.as<uint16_t>(), slot_index) != SRS_AMD_OK) {
      report("ofdm_slot_modulator_hip");
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    std::memcpy(static_cast<void*>(output.data()), out.ptr, sizeof(cf_t) * n);
  }

private:
  srs_amd_ofdm_modulator* mod;
  unsigned                nsymb, nsubc;
  pinned_buffer           in, out;
  slot_samples_cache      cache;
};

class ofdm_symbol_modulator_hip : public ofdm_symbol_modulator
{
public:
  ofdm_symbol_modulator_hip(srs_amd_ofdm_modulator* m, unsigned nsymb_, unsigned nsubc_, int dev) :
    mod(m), nsymb(nsymb_), nsubc(nsubc_), cache(m, nsymb_, nsubc_, dev)
  {
  }
  ~ofdm_symbol_modulator_hip() override
  {
    cache.drain();
    srs_amd_ofdm_modulator_destroy(mod);
  }

  unsigned get_symbol_size(unsigned symbol_index) const override
  {
    return srs_amd_ofdm_modulator_get_symbol_size(mod, symbol_index);
  }

  void set_center_frequency(double center_frequency_Hz) override
  {
    cache.drain();
    cache.invalidate(); // the phase compensation of the following calls changes
    if (srs_amd_ofdm_modulator_set_center_frequency(mod, center_frequency_Hz) != SRS_AMD_OK) {
      report("ofdm_symbol_modulator_hip");
    }
  }

  void modulate(span<cf_t> output, const resource_grid_reader& grid, unsigned port_index, unsigned symbol_index) override
  {
    const unsigned n = get_symbol_size(symbol_index);
    if (n == 0 || output.size() != n) {
      std::fprintf(stderr, "ofdm_symbol_modulator_hip: output of %zu samples, symbol %u has %u\n", output.size(),
                   symbol_index, n);
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    if (grid.is_empty(port_index)) {
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    // a device-resident grid: the slot's samples from one launch over every port (slot_samples_cache), this
    // symbol's share copied out
    if (hip::hip_resource_grid* hg = hip::hip_grid_of(grid)) {
      const unsigned slot = symbol_index / nsymb;
      const cf_t*    x    = cache.get(*hg, port_index, slot, "ofdm_symbol_modulator_hip");
      if (x == nullptr) {
        std::fill(output.begin(), output.end(), cf_t());
        return;
      }
      unsigned off = 0;
      for (unsigned l = slot * nsymb; l != symbol_index; ++l) {
        off += get_symbol_size(l);
      }
      std::memcpy(static_cast<void*>(output.data()), x + off, sizeof(cf_t) * n);
      return;
    }
    if (!in.ensure(sizeof(uint32_t) * nsubc) || !out.ensure(sizeof(cf_t) * n) ||
        !read_rows(grid, port_index, symbol_index % nsymb, 1, nsubc, in.as<uint16_t>()) ||
        srs_amd_ofdm_modulate_symbol(mod, out.as<float>(), in.as<uint16_t>(), symbol_index) != SRS_AMD_OK) {
      report("ofdm_symbol_modulator_hip");
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    std::memcpy(static_cast<void*>(output.data()), out.ptr, sizeof(cf_t) * n);
  }

private:
  srs_amd_ofdm_modulator* mod;
  unsigned                nsymb, nsubc;
  pinned_buffer           in, out;
  slot_samples_cache      cache;
};

// ---- demodulators on a device-resident grid: staged symbols, one launch when the grid is next used ----

// A hip_grid_deferred_writer: each demodulate() call copies its samples into a pinned batch (with the symbol index
// and grid row) and registers with the grid; the batch is demodulated into the grid's device copy in one launch
// (srs_amd_ofdm_demodulate_symbols_async, by default reading the pinned samples over the bus) when the grid is next accessed --
// the PUSCH plug-in's read -- or when the batch is full.  No HIP call on the demodulate() path but for a full batch.
class demod_stager : public hip::hip_grid_deferred_writer
{
public:
  static constexpr unsigned BATCH = 64; // symbols per launch at most (a slot of 4 ports: 56)
  static constexpr unsigned RING  = 3;  // batches in flight

  demod_stager(srs_amd_ofdm_demodulator* d, int dev, unsigned nof_symbols_subframe) : dem(d), stream_(dev)
  {
    for (unsigned i = 0; i != nof_symbols_subframe; ++i) {
      stride = std::max(stride, srs_amd_ofdm_demodulator_get_symbol_size(dem, i));
    }
  }
  ~demod_stager() override
  {
    flush();
    for (batch& b : ring) {
      if (b.ev != nullptr) {
        (void)hipEventDestroy(b.ev);
      }
      (void)hipFree(b.d_items);
      (void)hipFree(b.d_samples);
    }
  }

  // issues what is staged (every grid the stager is registered with: the list mirrors the grids' own, see
  // attached / issue / detach) and waits for every launch of the stager to complete
  void flush()
  {
    std::vector<hip::hip_resource_grid*> grids;
    {
      std::lock_guard<std::mutex> lock(mtx);
      grids = registered;
    }
    for (hip::hip_resource_grid* g : grids) {
      g->issue_deferred(*this);
    }
    stream_.drain();
  }

  // stages symbol `symbol_index` (x: its get_symbol_size samples) for row (port, l) of g; false when it cannot
  bool stage(hip::hip_resource_grid& g, const cf_t* x, unsigned n, unsigned port, unsigned l, unsigned symbol_index,
             unsigned nsubc)
  {
    if (stream_.s == nullptr || n > stride || port >= g.nof_ports() || l >= g.nof_symbols() || nsubc > g.nof_subc()) {
      return false;
    }
    hip::hip_resource_grid* prev;
    {
      std::lock_guard<std::mutex> lock(mtx);
      prev = cur; // (non-null: symbols are staged for it, so it is registered and alive)
    }
    if (prev != nullptr && prev != &g) {
      prev->issue_deferred(*this); // another grid (the next slot's): what is staged for the previous one goes now
    }
    bool full;
    {
      std::lock_guard<std::mutex> lock(mtx);
      batch& b = ring[next];
      if (!ready(b)) {
        return false;
      }
      cur              = &g;
      const unsigned i = b.count++;
      b.items[2 * i]     = symbol_index;
      b.items[2 * i + 1] = (port * g.nof_symbols() + l) * g.nof_subc();
      std::memcpy(b.samples + static_cast<size_t>(i) * stride, x, sizeof(cf_t) * n);
      full = b.count == BATCH;
    }
    g.defer(*this);
    if (full) {
      g.issue_deferred(*this);
    }
    return true;
  }

  // (called by g with g locked, g having just removed this writer from its list)
  void issue(hip::hip_resource_grid& g, uint32_t* d) override
  {
    std::lock_guard<std::mutex> lock(mtx);
    unregister(g);
    batch& b = ring[next];
    if (cur != &g || b.count == 0) {
      return;
    }
    const uint32_t* items   = b.items;
    const cf_t*     samples = b.samples;
    void*           scratch = mode == staging::copy_kernel ? b.d_samples : nullptr;
    if (mode == staging::dma) {
      // one DMA copy of the staged samples into HBM, the kernel then reads HBM (the kernel's zero-copy reads over the
      // bus are the other form: SRS_AMD_OFDM_STAGING=zero-copy)
      const size_t bytes = sizeof(cf_t) * static_cast<size_t>(b.count) * stride;
      if (hipMemcpyAsync(b.d_samples, b.samples, bytes, hipMemcpyHostToDevice, stream_.s) != hipSuccess ||
          hipMemcpyAsync(b.d_items, b.items, sizeof(uint32_t) * 2 * b.count, hipMemcpyHostToDevice, stream_.s) !=
              hipSuccess) {
        report("ofdm_symbol_demodulator_hip");
      }
      items   = b.d_items;
      samples = b.d_samples;
    }
    if (srs_amd_ofdm_demodulate_symbols_async(dem, reinterpret_cast<uint16_t*>(d), items,
                                              reinterpret_cast<const float*>(samples), stride, b.count, scratch,
                                              stream_.s) != SRS_AMD_OK) {
      report("ofdm_symbol_demodulator_hip");
    }
    b.in_flight = hipEventRecord(b.ev, stream_.s) == hipSuccess;
    b.count     = 0;
    next        = (next + 1) % RING;
    // nothing staged any more: no grid to remember (the grid may go away without telling a writer it no longer
    // has registered)
    cur = nullptr;
  }

  hipStream_t stream() const override { return stream_.s; }

  void attached(hip::hip_resource_grid& g) override
  {
    std::lock_guard<std::mutex> lock(mtx);
    registered.push_back(&g);
  }

  void detach(hip::hip_resource_grid& g) override
  {
    std::lock_guard<std::mutex> lock(mtx);
    unregister(g);
    if (cur == &g) {
      cur               = nullptr;
      ring[next].count = 0;
    }
  }

private:
  struct batch {
    pinned_buffer items_buf, samples_buf;
    uint32_t*     items     = nullptr;
    cf_t*         samples   = nullptr;
    uint32_t*     d_items   = nullptr; // (DMA staging) device copies
    cf_t*         d_samples = nullptr;
    hipEvent_t    ev        = nullptr;
    bool          in_flight = false;
    unsigned      count     = 0;
  };

  void unregister(hip::hip_resource_grid& g)
  {
    registered.erase(std::remove(registered.begin(), registered.end(), &g), registered.end());
  }

  // the batch allocated and free for the host (its last launch has completed); lock held
  bool ready(batch& b)
  {
    if (b.samples == nullptr) {
      if (!b.items_buf.ensure(sizeof(uint32_t) * 2 * BATCH) ||
          !b.samples_buf.ensure(sizeof(cf_t) * static_cast<size_t>(BATCH) * stride) ||
          hipEventCreateWithFlags(&b.ev, hipEventDisableTiming) != hipSuccess) {
        return false;
      }
      b.items   = b.items_buf.as<uint32_t>();
      b.samples = b.samples_buf.as<cf_t>();
      // (device copies: DMA staging; the copy kernel's scratch holds the samples then the items)
      if (mode != staging::zero_copy &&
          (hipMalloc(&b.d_items, sizeof(uint32_t) * 2 * BATCH) != hipSuccess ||
           hipMalloc(&b.d_samples, (sizeof(cf_t) * stride + sizeof(uint32_t) * 2) * BATCH) != hipSuccess)) {
        return false;
      }
    }
    if (b.in_flight) {
      if (hipEventSynchronize(b.ev) != hipSuccess) {
        return false;
      }
      b.in_flight = false;
    }
    return true;
  }

  srs_amd_ofdm_demodulator* dem;
  device_stream             stream_;
  const staging             mode   = staging_mode(true);
  unsigned                  stride = 0; // samples per staged symbol (the longest symbol)
  std::mutex                mtx;
  hip::hip_resource_grid*   cur  = nullptr; // the grid the staged symbols belong to (nullptr: nothing staged)
  std::vector<hip::hip_resource_grid*> registered; // the grids whose deferred list holds this writer
  std::array<batch, RING>   ring;
  unsigned                  next = 0;       // the batch being filled
};

class ofdm_slot_demodulator_hip : public ofdm_slot_demodulator
{
public:
  ofdm_slot_demodulator_hip(srs_amd_ofdm_demodulator* d, unsigned nsymb_, unsigned nsubc_, int dev, unsigned nsym_sf) :
    dem(d), nsymb(nsymb_), nsubc(nsubc_), stager(d, dev, nsym_sf)
  {
  }
  ~ofdm_slot_demodulator_hip() override
  {
    stager.flush(); // (before the transform's tables go)
    srs_amd_ofdm_demodulator_destroy(dem);
  }

  unsigned get_slot_size(unsigned slot_index) const override
  {
    return srs_amd_ofdm_demodulator_get_slot_size(dem, slot_index);
  }

  void demodulate(resource_grid_writer& grid, span<const cf_t> input, unsigned port_index, unsigned slot_index) override
  {
    const unsigned n = get_slot_size(slot_index);
    // a device-resident grid (read in HBM by the PUSCH plug-in): the slot's symbols staged, demodulated into the
    // device copy at the grid's next use -- no host wait, no host-mirror write
    if (hip::hip_resource_grid* hg = hip::hip_grid_of(grid)) {
      bool ok = n != 0 && input.size() == n;
      for (unsigned l = 0, off = 0; ok && l != nsymb; ++l) {
        const unsigned sidx = slot_index * nsymb + l;
        const unsigned sz   = srs_amd_ofdm_demodulator_get_symbol_size(dem, sidx);
        ok                  = stager.stage(*hg, input.data() + off, sz, port_index, l, sidx, nsubc);
        off += sz;
      }
      if (ok) {
        return;
      }
      std::fprintf(stderr, "ofdm_slot_demodulator_hip: input of %zu samples, slot %u has %u\n", input.size(),
                   slot_index, n);
      report_geometry("ofdm_slot_demodulator_hip", *hg);
    }
    if (!out.ensure(sizeof(uint32_t) * nsymb * nsubc)) {
      report("ofdm_slot_demodulator_hip");
      return;
    }
    if (n == 0 || input.size() != n || !in.ensure(sizeof(cf_t) * n)) {
      std::fprintf(stderr, "ofdm_slot_demodulator_hip: input of %zu samples, slot %u has %u\n", input.size(),
                   slot_index, n);
      std::memset(out.ptr, 0, sizeof(uint32_t) * nsymb * nsubc);
    } else {
      std::memcpy(in.ptr, input.data(), sizeof(cf_t) * n);
      if (srs_amd_ofdm_demodulate_slot(dem, out.as<uint16_t>(), in.as<float>(), slot_index) != SRS_AMD_OK) {
        report("ofdm_slot_demodulator_hip");
        std::memset(out.ptr, 0, sizeof(uint32_t) * nsymb * nsubc);
      }
    }
    write_rows(grid, port_index, 0, nsymb, nsubc, out.as<uint16_t>());
  }

private:
  srs_amd_ofdm_demodulator* dem;
  unsigned                  nsymb, nsubc;
  pinned_buffer             in, out;
  demod_stager              stager;
};

class ofdm_symbol_demodulator_hip : public ofdm_symbol_demodulator
{
public:
  ofdm_symbol_demodulator_hip(srs_amd_ofdm_demodulator* d, unsigned nsymb_, unsigned nsubc_, int dev,
                              unsigned nsym_sf) :
    dem(d), nsymb(nsymb_), nsubc(nsubc_), stager(d, dev, nsym_sf)
  {
  }
  ~ofdm_symbol_demodulator_hip() override
  {
    stager.flush(); // (before the transform's tables go)
    srs_amd_ofdm_demodulator_destroy(dem);
  }

  unsigned get_symbol_size(unsigned symbol_index) const override
  {
    return srs_amd_ofdm_demodulator_get_symbol_size(dem, symbol_index);
  }

  void set_center_frequency(double center_frequency_Hz) override
  {
    // the staged symbols keep the phase compensation they were staged under: issued and completed first
    stager.flush();
    if (srs_amd_ofdm_demodulator_set_center_frequency(dem, center_frequency_Hz) != SRS_AMD_OK) {
      report("ofdm_symbol_demodulator_hip");
    }
  }

  void demodulate(resource_grid_writer& grid, span<const cf_t> input, unsigned port_index, unsigned symbol_index) override
  {
    const unsigned n = get_symbol_size(symbol_index);
    // a device-resident grid: the symbol staged, demodulated into the device copy at the grid's next use (one launch
    // for the slot's symbols) -- no HIP call here, no host wait, no host-mirror write
    if (hip::hip_resource_grid* hg = hip::hip_grid_of(grid)) {
      if (n != 0 && input.size() == n &&
          stager.stage(*hg, input.data(), n, port_index, symbol_index % nsymb, symbol_index, nsubc)) {
        return;
      }
      std::fprintf(stderr, "ofdm_symbol_demodulator_hip: input of %zu samples, symbol %u has %u\n", input.size(),
                   symbol_index, n);
      report_geometry("ofdm_symbol_demodulator_hip", *hg);
    }
    if (!out.ensure(sizeof(uint32_t) * nsubc)) {
      report("ofdm_symbol_demodulator_hip");
      return;
    }
    if (n == 0 || input.size() != n || !in.ensure(sizeof(cf_t) * n)) {
      std::fprintf(stderr, "ofdm_symbol_demodulator_hip: input of %zu samples, symbol %u has %u\n", input.size(),
                   symbol_index, n);
      std::memset(out.ptr, 0, sizeof(uint32_t) * nsubc);
    } else {
      std::memcpy(in.ptr, input.data(), sizeof(cf_t) * n);
      if (srs_amd_ofdm_demodulate_symbol(dem, out.as<uint16_t>(), in.as<float>(), symbol_index) != SRS_AMD_OK) {
        report("ofdm_symbol_demodulator_hip");
        std::memset(out.ptr, 0, sizeof(uint32_t) * nsubc);
      }
    }
    write_rows(grid, port_index, symbol_index % nsymb, 1, nsubc, out.as<uint16_t>());
  }

private:
  srs_amd_ofdm_demodulator* dem;
  unsigned                  nsymb, nsubc;
  pinned_buffer             in, out;
  demod_stager              stager;
};

class ofdm_modulator_factory_hip : public ofdm_modulator_factory
{
public:
  explicit ofdm_modulator_factory_hip(int device_) : device(device_) {}

  std::unique_ptr<ofdm_symbol_modulator> create_ofdm_symbol_modulator(const ofdm_modulator_configuration& c) override
  {
    srs_amd_ofdm_modulator* m = make(c);
    return m ? std::make_unique<ofdm_symbol_modulator_hip>(m, get_nsymb_per_slot(c.cp), c.bw_rb * NRE,
                                                           resolve_device(device))
             : nullptr;
  }

  std::unique_ptr<ofdm_slot_modulator> create_ofdm_slot_modulator(const ofdm_modulator_configuration& c) override
  {
    srs_amd_ofdm_modulator* m = make(c);
    return m ? std::make_unique<ofdm_slot_modulator_hip>(m, get_nsymb_per_slot(c.cp), c.bw_rb * NRE,
                                                         resolve_device(device))
             : nullptr;
  }

private:
  srs_amd_ofdm_modulator* make(const ofdm_modulator_configuration& c) const
  {
    const int                 dev = resolve_device(device);
    const srs_amd_ofdm_config cc  = to_c(c.numerology, c.bw_rb, c.dft_size, c.cp, 0, c.scale, c.center_freq_Hz);
    srs_amd_ofdm_modulator*   m   = nullptr;
    if (dev < 0 || srs_amd_ofdm_modulator_create(&m, &cc, dev) != SRS_AMD_OK) {
      report("ofdm_modulator_factory_hip");
      return nullptr;
    }
    return m;
  }

  int device;
};

class ofdm_demodulator_factory_hip : public ofdm_demodulator_factory
{
public:
  explicit ofdm_demodulator_factory_hip(int device_) : device(device_) {}

  std::unique_ptr<ofdm_symbol_demodulator>
  create_ofdm_symbol_demodulator(const ofdm_demodulator_configuration& c) override
  {
    srs_amd_ofdm_demodulator* d = make(c);
    return d ? std::make_unique<ofdm_symbol_demodulator_hip>(d, get_nsymb_per_slot(c.cp), c.bw_rb * NRE,
                                                             resolve_device(device), nsym_sf(c))
             : nullptr;
  }

  std::unique_ptr<ofdm_slot_demodulator> create_ofdm_slot_demodulator(const ofdm_demodulator_configuration& c) override
  {
    srs_amd_ofdm_demodulator* d = make(c);
    return d ? std::make_unique<ofdm_slot_demodulator_hip>(d, get_nsymb_per_slot(c.cp), c.bw_rb * NRE,
                                                           resolve_device(device), nsym_sf(c))
             : nullptr;
  }

private:
  static unsigned nsym_sf(const ofdm_demodulator_configuration& c)
  {
    return get_nsymb_per_slot(c.cp) * (1u << c.numerology);
  }

  srs_amd_ofdm_demodulator* make(const ofdm_demodulator_configuration& c) const
  {
    const int                 dev = resolve_device(device);
    const srs_amd_ofdm_config cc =
        to_c(c.numerology, c.bw_rb, c.dft_size, c.cp, c.nof_samples_window_offset, c.scale, c.center_freq_Hz);
    srs_amd_ofdm_demodulator* d = nullptr;
    if (dev < 0 || srs_amd_ofdm_demodulator_create(&d, &cc, dev) != SRS_AMD_OK) {
      report("ofdm_demodulator_factory_hip");
      return nullptr;
    }
    return d;
  }

  int device;
};

} // namespace

std::shared_ptr<ofdm_modulator_factory> srsran::hip::create_ofdm_modulator_factory_hip(int device)
{
  return std::make_shared<ofdm_modulator_factory_hip>(device);
}

std::shared_ptr<ofdm_demodulator_factory> srsran::hip::create_ofdm_demodulator_factory_hip(int device)
{
  return std::make_shared<ofdm_demodulator_factory_hip>(device);
}
