// ofdm_modulator_hip.cpp -- srsran::ofdm_{slot,symbol}_{modulator,demodulator} over the srsran_amd OFDM C-ABI
// (see the header).
#include "ofdm_modulator_hip.h"

#include "srsran/phy/lower/modulation/ofdm_demodulator.h"
#include "srsran/phy/lower/modulation/ofdm_modulator.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran_amd/ofdm.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

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
    std::memcpy(row.data(), src + 2 * static_cast<size_t>(l) * nsubc, sizeof(cbf16_t) * std::min<size_t>(nsubc, row.size()));
  }
}

class ofdm_slot_modulator_hip : public ofdm_slot_modulator
{
public:
  ofdm_slot_modulator_hip(srs_amd_ofdm_modulator* m, unsigned nsymb_, unsigned nsubc_) :
    mod(m), nsymb(nsymb_), nsubc(nsubc_)
  {
  }
  ~ofdm_slot_modulator_hip() override { srs_amd_ofdm_modulator_destroy(mod); }

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
    if (!in.ensure(sizeof(uint32_t) * nsymb * nsubc) || !out.ensure(sizeof(cf_t) * n) ||
        !read_rows(grid, port_index, 0, nsymb, nsubc, in.as<uint16_t>()) ||
        srs_amd_ofdm_modulate_slot(mod, out.as<float>(), in.as<uint16_t>(), slot_index) != SRS_AMD_OK) {
      report("ofdm_slot_modulator_hip");
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    std::memcpy(output.data(), out.ptr, sizeof(cf_t) * n);
  }

private:
  srs_amd_ofdm_modulator* mod;
  unsigned                nsymb, nsubc;
  pinned_buffer           in, out;
};

class ofdm_symbol_modulator_hip : public ofdm_symbol_modulator
{
public:
  ofdm_symbol_modulator_hip(srs_amd_ofdm_modulator* m, unsigned nsymb_, unsigned nsubc_) :
    mod(m), nsymb(nsymb_), nsubc(nsubc_)
  {
  }
  ~ofdm_symbol_modulator_hip() override { srs_amd_ofdm_modulator_destroy(mod); }

  unsigned get_symbol_size(unsigned symbol_index) const override
  {
    return srs_amd_ofdm_modulator_get_symbol_size(mod, symbol_index);
  }

  void set_center_frequency(double center_frequency_Hz) override
  {
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
    if (!in.ensure(sizeof(uint32_t) * nsubc) || !out.ensure(sizeof(cf_t) * n) ||
        !read_rows(grid, port_index, symbol_index % nsymb, 1, nsubc, in.as<uint16_t>()) ||
        srs_amd_ofdm_modulate_symbol(mod, out.as<float>(), in.as<uint16_t>(), symbol_index) != SRS_AMD_OK) {
      report("ofdm_symbol_modulator_hip");
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    std::memcpy(output.data(), out.ptr, sizeof(cf_t) * n);
  }

private:
  srs_amd_ofdm_modulator* mod;
  unsigned                nsymb, nsubc;
  pinned_buffer           in, out;
};

class ofdm_slot_demodulator_hip : public ofdm_slot_demodulator
{
public:
  ofdm_slot_demodulator_hip(srs_amd_ofdm_demodulator* d, unsigned nsymb_, unsigned nsubc_) :
    dem(d), nsymb(nsymb_), nsubc(nsubc_)
  {
  }
  ~ofdm_slot_demodulator_hip() override { srs_amd_ofdm_demodulator_destroy(dem); }

  unsigned get_slot_size(unsigned slot_index) const override
  {
    return srs_amd_ofdm_demodulator_get_slot_size(dem, slot_index);
  }

  void demodulate(resource_grid_writer& grid, span<const cf_t> input, unsigned port_index, unsigned slot_index) override
  {
    const unsigned n = get_slot_size(slot_index);
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
};

class ofdm_symbol_demodulator_hip : public ofdm_symbol_demodulator
{
public:
  ofdm_symbol_demodulator_hip(srs_amd_ofdm_demodulator* d, unsigned nsymb_, unsigned nsubc_) :
    dem(d), nsymb(nsymb_), nsubc(nsubc_)
  {
  }
  ~ofdm_symbol_demodulator_hip() override { srs_amd_ofdm_demodulator_destroy(dem); }

  unsigned get_symbol_size(unsigned symbol_index) const override
  {
    return srs_amd_ofdm_demodulator_get_symbol_size(dem, symbol_index);
  }

  void set_center_frequency(double center_frequency_Hz) override
  {
    if (srs_amd_ofdm_demodulator_set_center_frequency(dem, center_frequency_Hz) != SRS_AMD_OK) {
      report("ofdm_symbol_demodulator_hip");
    }
  }

  void demodulate(resource_grid_writer& grid, span<const cf_t> input, unsigned port_index, unsigned symbol_index) override
  {
    const unsigned n = get_symbol_size(symbol_index);
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
};

class ofdm_modulator_factory_hip : public ofdm_modulator_factory
{
public:
  explicit ofdm_modulator_factory_hip(int device_) : device(device_) {}

  std::unique_ptr<ofdm_symbol_modulator> create_ofdm_symbol_modulator(const ofdm_modulator_configuration& c) override
  {
    srs_amd_ofdm_modulator* m = make(c);
    return m ? std::make_unique<ofdm_symbol_modulator_hip>(m, get_nsymb_per_slot(c.cp), c.bw_rb * NRE) : nullptr;
  }

  std::unique_ptr<ofdm_slot_modulator> create_ofdm_slot_modulator(const ofdm_modulator_configuration& c) override
  {
    srs_amd_ofdm_modulator* m = make(c);
    return m ? std::make_unique<ofdm_slot_modulator_hip>(m, get_nsymb_per_slot(c.cp), c.bw_rb * NRE) : nullptr;
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
    return d ? std::make_unique<ofdm_symbol_demodulator_hip>(d, get_nsymb_per_slot(c.cp), c.bw_rb * NRE) : nullptr;
  }

  std::unique_ptr<ofdm_slot_demodulator> create_ofdm_slot_demodulator(const ofdm_demodulator_configuration& c) override
  {
    srs_amd_ofdm_demodulator* d = make(c);
    return d ? std::make_unique<ofdm_slot_demodulator_hip>(d, get_nsymb_per_slot(c.cp), c.bw_rb * NRE) : nullptr;
  }

private:
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
