// ref_wrapper_ofdm.cpp -- extern "C" glue around the REFERENCE's own OFDM
// modulator / demodulator and generic DFT (compiled from /root/reference by
// oracle/Makefile into oracle/_ref/libsrsran_ref.so).
//
// TEST INFRASTRUCTURE ONLY: pins oracle/ofdm.py (tests/test_oracle_vs_ref.py) and
// times the reference's CPU OFDM path for bench_ofdm.py's cpu_baseline leg.
//
// Wrapped reference classes:
//   lib/phy/lower/modulation/ofdm_modulator_impl.cpp    ofdm_symbol_modulator_impl / ofdm_slot_modulator_impl
//   lib/phy/lower/modulation/ofdm_demodulator_impl.cpp  ofdm_symbol_demodulator_impl / ofdm_slot_demodulator_impl
//   lib/phy/generic_functions/dft_processor_generic_impl.cpp  dft_processor_generic_impl
// The resource grid is passed as a dense complex-bf16 array [symbol][subcarrier]
// (the reference resource_grid_impl layout for one port); the small reader /
// writer classes below implement the reference's resource_grid_reader /
// resource_grid_writer interfaces over that array.
#include "phy/generic_functions/dft_processor_generic_impl.h"
#include "phy/lower/modulation/ofdm_demodulator_impl.h"
#include "phy/lower/modulation/ofdm_modulator_impl.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "ref_builders.h"
#include <chrono>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

using namespace srsran;

namespace {

class dense_grid_reader : public resource_grid_reader
{
public:
  dense_grid_reader(const cbf16_t* data_, unsigned nsymb_, unsigned nsubc_) : data(data_), nsymb(nsymb_), nsubc(nsubc_)
  {
  }
  unsigned get_nof_ports() const override { return 1; }
  unsigned get_nof_subc() const override { return nsubc; }
  unsigned get_nof_symbols() const override { return nsymb; }
  bool     is_empty(unsigned) const override { return false; }
  bool     is_empty() const override { return false; }
  span<cf_t> get(span<cf_t> symbols, unsigned, unsigned, unsigned, const bounded_bitset<MAX_RB * NRE>&) const override
  {
    return symbols;
  }
  span<cbf16_t>
  get(span<cbf16_t> symbols, unsigned, unsigned, unsigned, const bounded_bitset<MAX_RB * NRE>&) const override
  {
    return symbols;
  }
  void get(span<cf_t> symbols, unsigned, unsigned l, unsigned k_init, unsigned stride) const override
  {
    for (unsigned i = 0; i != symbols.size(); ++i) {
      const cbf16_t v = data[l * nsubc + k_init + i * stride];
      symbols[i]      = cf_t(to_float(v.real), to_float(v.imag));
    }
  }
  void get(span<cbf16_t> symbols, unsigned, unsigned l, unsigned k_init) const override
  {
    std::memcpy(symbols.data(), data + l * nsubc + k_init, symbols.size() * sizeof(cbf16_t));
  }
  span<const cbf16_t> get_view(unsigned, unsigned l) const override { return {data + l * nsubc, nsubc}; }

private:
  const cbf16_t* data;
  unsigned       nsymb, nsubc;
};

class dense_grid_writer : public resource_grid_writer
{
public:
  dense_grid_writer(cbf16_t* data_, unsigned nsymb_, unsigned nsubc_) : data(data_), nsymb(nsymb_), nsubc(nsubc_) {}
  unsigned         get_nof_ports() const override { return 1; }
  unsigned         get_nof_subc() const override { return nsubc; }
  unsigned         get_nof_symbols() const override { return nsymb; }
  span<const cf_t> put(unsigned, unsigned, unsigned, const bounded_bitset<NRE * MAX_RB>&, span<const cf_t> s) override
  {
    return s;
  }
  span<const cbf16_t>
  put(unsigned, unsigned, unsigned, const bounded_bitset<NRE * MAX_RB>&, span<const cbf16_t> s) override
  {
    return s;
  }
  void put(unsigned, unsigned l, unsigned k_init, span<const cf_t> symbols) override
  {
    for (unsigned i = 0; i != symbols.size(); ++i) {
      data[l * nsubc + k_init + i] = cbf16_t(symbols[i]);
    }
  }
  void put(unsigned, unsigned l, unsigned k_init, unsigned stride, span<const cbf16_t> symbols) override
  {
    for (unsigned i = 0; i != symbols.size(); ++i) {
      data[l * nsubc + k_init + i * stride] = symbols[i];
    }
  }
  span<cbf16_t> get_view(unsigned, unsigned l) override { return {data + l * nsubc, nsubc}; }

private:
  cbf16_t* data;
  unsigned nsymb, nsubc;
};

std::unique_ptr<ofdm_slot_modulator> make_modulator(unsigned                       numerology,
                                                    unsigned                       bw_rb,
                                                    unsigned                       dft_size,
                                                    int                            extended_cp,
                                                    float                          scale,
                                                    double                         fc,
                                                    std::unique_ptr<dft_processor> dft = nullptr)
{
  ofdm_modulator_configuration cfg;
  cfg.numerology     = numerology;
  cfg.bw_rb          = bw_rb;
  cfg.dft_size       = dft_size;
  cfg.cp             = extended_cp ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  cfg.scale          = scale;
  cfg.center_freq_Hz = fc;
  ofdm_modulator_common_configuration common;
  common.dft = dft ? std::move(dft)
                   : std::make_unique<dft_processor_generic_impl>(
                         dft_processor::configuration{dft_size, dft_processor::direction::INVERSE});
  auto sym = std::make_unique<ofdm_symbol_modulator_impl>(common, cfg);
  return std::make_unique<ofdm_slot_modulator_impl>(cfg, std::move(sym));
}

std::unique_ptr<ofdm_slot_demodulator> make_demodulator(unsigned numerology,
                                                        unsigned bw_rb,
                                                        unsigned dft_size,
                                                        int      extended_cp,
                                                        unsigned window_offset,
                                                        float    scale,
                                                        double   fc,
                                                        std::unique_ptr<dft_processor> dft = nullptr)
{
  ofdm_demodulator_configuration cfg;
  cfg.numerology                = numerology;
  cfg.bw_rb                     = bw_rb;
  cfg.dft_size                  = dft_size;
  cfg.cp                        = extended_cp ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  cfg.nof_samples_window_offset = window_offset;
  cfg.scale                     = scale;
  cfg.center_freq_Hz            = fc;
  ofdm_demodulator_common_configuration common;
  common.dft = dft ? std::move(dft)
                   : std::make_unique<dft_processor_generic_impl>(
                         dft_processor::configuration{dft_size, dft_processor::direction::DIRECT});
  auto sym = std::make_unique<ofdm_symbol_demodulator_impl>(common, cfg);
  return std::make_unique<ofdm_slot_demodulator_impl>(cfg, std::move(sym));
}

} // namespace

// ofdm_slot_modulator_impl / ofdm_slot_demodulator_impl of one port with a given DFT (the harness's MI355X
// dft_processor adapter); layouts as srs_ref_ofdm_modulate_slot / srs_ref_ofdm_demodulate_slot.
int srs_ref::ofdm_modulate_slot_with(std::unique_ptr<dft_processor> dft,
                                     unsigned                       numerology,
                                     unsigned                       bw_rb,
                                     unsigned                       dft_size,
                                     int                            extended_cp,
                                     float                          scale,
                                     double                         fc,
                                     unsigned                       slot,
                                     const uint16_t*                grid,
                                     float*                         out)
{
  if (!dft) {
    return -1;
  }
  auto              mod   = make_modulator(numerology, bw_rb, dft_size, extended_cp, scale, fc, std::move(dft));
  unsigned          nsymb = extended_cp ? 12 : 14;
  unsigned          n     = mod->get_slot_size(slot);
  dense_grid_reader rd(reinterpret_cast<const cbf16_t*>(grid), nsymb, bw_rb * NRE);
  mod->modulate(span<cf_t>(reinterpret_cast<cf_t*>(out), n), rd, 0, slot);
  return 0;
}

int srs_ref::ofdm_demodulate_slot_with(std::unique_ptr<dft_processor> dft,
                                       unsigned                       numerology,
                                       unsigned                       bw_rb,
                                       unsigned                       dft_size,
                                       int                            extended_cp,
                                       unsigned                       window_offset,
                                       float                          scale,
                                       double                         fc,
                                       unsigned                       slot,
                                       const float*                   in,
                                       uint16_t*                      grid)
{
  if (!dft) {
    return -1;
  }
  auto dem = make_demodulator(numerology, bw_rb, dft_size, extended_cp, window_offset, scale, fc, std::move(dft));
  unsigned          nsymb = extended_cp ? 12 : 14;
  unsigned          n     = dem->get_slot_size(slot);
  dense_grid_writer wr(reinterpret_cast<cbf16_t*>(grid), nsymb, bw_rb * NRE);
  dem->demodulate(wr, span<const cf_t>(reinterpret_cast<const cf_t*>(in), n), 0, slot);
  return 0;
}

void srs_ref::ofdm_run_slot_modulator(ofdm_slot_modulator& mod, unsigned nsymb, unsigned nsubc, unsigned slot,
                                      const uint16_t* grid, float* out)
{
  dense_grid_reader rd(reinterpret_cast<const cbf16_t*>(grid), nsymb, nsubc);
  mod.modulate(span<cf_t>(reinterpret_cast<cf_t*>(out), mod.get_slot_size(slot)), rd, 0, slot);
}

void srs_ref::ofdm_run_symbol_modulator(ofdm_symbol_modulator& mod, unsigned nsymb, unsigned nsubc, unsigned slot,
                                        const uint16_t* grid, float* out)
{
  dense_grid_reader rd(reinterpret_cast<const cbf16_t*>(grid), nsymb, nsubc);
  cf_t*             o = reinterpret_cast<cf_t*>(out);
  for (unsigned l = 0; l != nsymb; ++l) {
    const unsigned n = mod.get_symbol_size(nsymb * slot + l);
    mod.modulate(span<cf_t>(o, n), rd, 0, nsymb * slot + l);
    o += n;
  }
}

void srs_ref::ofdm_run_slot_demodulator(ofdm_slot_demodulator& dem, unsigned nsymb, unsigned nsubc, unsigned slot,
                                        const float* in, uint16_t* grid)
{
  dense_grid_writer wr(reinterpret_cast<cbf16_t*>(grid), nsymb, nsubc);
  dem.demodulate(wr, span<const cf_t>(reinterpret_cast<const cf_t*>(in), dem.get_slot_size(slot)), 0, slot);
}

void srs_ref::ofdm_run_symbol_demodulator(ofdm_symbol_demodulator& dem, unsigned nsymb, unsigned nsubc, unsigned slot,
                                          const float* in, uint16_t* grid)
{
  dense_grid_writer wr(reinterpret_cast<cbf16_t*>(grid), nsymb, nsubc);
  const cf_t*       x = reinterpret_cast<const cf_t*>(in);
  for (unsigned l = 0; l != nsymb; ++l) {
    const unsigned n = dem.get_symbol_size(nsymb * slot + l);
    dem.demodulate(wr, span<const cf_t>(x, n), 0, nsymb * slot + l);
    x += n;
  }
}

std::unique_ptr<ofdm_slot_modulator> srs_ref::make_ref_ofdm_slot_modulator(const ofdm_modulator_configuration& c)
{
  return make_modulator(c.numerology, c.bw_rb, c.dft_size, c.cp == cyclic_prefix::EXTENDED, c.scale, c.center_freq_Hz);
}

std::unique_ptr<ofdm_slot_demodulator> srs_ref::make_ref_ofdm_slot_demodulator(const ofdm_demodulator_configuration& c)
{
  return make_demodulator(c.numerology, c.bw_rb, c.dft_size, c.cp == cyclic_prefix::EXTENDED,
                          c.nof_samples_window_offset, c.scale, c.center_freq_Hz);
}

std::unique_ptr<ofdm_symbol_demodulator>
srs_ref::make_ref_ofdm_symbol_demodulator(const ofdm_demodulator_configuration& c)
{
  ofdm_demodulator_common_configuration common;
  common.dft = std::make_unique<dft_processor_generic_impl>(
      dft_processor::configuration{c.dft_size, dft_processor::direction::DIRECT});
  return std::make_unique<ofdm_symbol_demodulator_impl>(common, c);
}

std::unique_ptr<ofdm_symbol_modulator> srs_ref::make_ref_ofdm_symbol_modulator(const ofdm_modulator_configuration& c)
{
  ofdm_modulator_common_configuration common;
  common.dft = std::make_unique<dft_processor_generic_impl>(
      dft_processor::configuration{c.dft_size, dft_processor::direction::INVERSE});
  return std::make_unique<ofdm_symbol_modulator_impl>(common, c);
}

extern "C" {

// One dft_processor::run() of the reference generic DFT: in/out interleaved complex float.
int srs_ref_dft(unsigned size, int inverse, const float* in, float* out)
{
  dft_processor_generic_impl dft(
      {size, inverse ? dft_processor::direction::INVERSE : dft_processor::direction::DIRECT});
  if (!dft.is_valid()) {
    return -1;
  }
  std::memcpy(dft.get_input().data(), in, size * sizeof(cf_t));
  span<const cf_t> o = dft.run();
  std::memcpy(out, o.data(), size * sizeof(cf_t));
  return 0;
}

unsigned srs_ref_ofdm_slot_size(unsigned numerology, unsigned bw_rb, unsigned dft_size, int extended_cp, unsigned slot)
{
  return make_modulator(numerology, bw_rb, dft_size, extended_cp, 1.0F, 0.0)->get_slot_size(slot);
}

// ofdm_slot_modulator::modulate of one port: grid = cbf16 [nsymb][bw_rb*12], out = cf [slot size].
int srs_ref_ofdm_modulate_slot(unsigned       numerology,
                               unsigned       bw_rb,
                               unsigned       dft_size,
                               int            extended_cp,
                               float          scale,
                               double         fc,
                               unsigned       slot,
                               const uint16_t* grid,
                               float*         out)
{
  auto     mod   = make_modulator(numerology, bw_rb, dft_size, extended_cp, scale, fc);
  unsigned nsymb = extended_cp ? 12 : 14;
  unsigned n     = mod->get_slot_size(slot);
  dense_grid_reader rd(reinterpret_cast<const cbf16_t*>(grid), nsymb, bw_rb * NRE);
  mod->modulate(span<cf_t>(reinterpret_cast<cf_t*>(out), n), rd, 0, slot);
  return 0;
}

// ofdm_slot_demodulator::demodulate of one port: in = cf [slot size], grid = cbf16 [nsymb][bw_rb*12].
int srs_ref_ofdm_demodulate_slot(unsigned     numerology,
                                 unsigned     bw_rb,
                                 unsigned     dft_size,
                                 int          extended_cp,
                                 unsigned     window_offset,
                                 float        scale,
                                 double       fc,
                                 unsigned     slot,
                                 const float* in,
                                 uint16_t*    grid)
{
  auto     dem   = make_demodulator(numerology, bw_rb, dft_size, extended_cp, window_offset, scale, fc);
  unsigned nsymb = extended_cp ? 12 : 14;
  unsigned n     = dem->get_slot_size(slot);
  dense_grid_writer wr(reinterpret_cast<cbf16_t*>(grid), nsymb, bw_rb * NRE);
  dem->demodulate(wr, span<const cf_t>(reinterpret_cast<const cf_t*>(in), n), 0, slot);
  return 0;
}

// CPU baseline: modulates then demodulates n_items (port, slot) grids with
// `threads` workers (one modulator + demodulator each), cycling over n_sample
// input grids.  grid: cbf16 [n_sample][nsymb][rg]; returns wall seconds.
double srs_ref_ofdm_roundtrip_many(unsigned        numerology,
                                   unsigned        bw_rb,
                                   unsigned        dft_size,
                                   const uint16_t* grids,
                                   unsigned        n_sample,
                                   unsigned        n_items,
                                   unsigned        threads)
{
  const unsigned nsymb = 14, rg = bw_rb * NRE;
  const unsigned nslots = 1u << numerology;
  auto           t0     = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < threads; ++t) {
    pool.emplace_back([=]() {
      auto                 mod = make_modulator(numerology, bw_rb, dft_size, 0, 1.0F, 0.0);
      auto                 dem = make_demodulator(numerology, bw_rb, dft_size, 0, 0, 1.0F, 0.0);
      std::vector<cf_t>    buf(mod->get_slot_size(0) + dft_size);
      std::vector<cbf16_t> out(nsymb * rg);
      for (unsigned i = t; i < n_items; i += threads) {
        unsigned          slot = i % nslots;
        unsigned          n    = mod->get_slot_size(slot);
        dense_grid_reader rd(reinterpret_cast<const cbf16_t*>(grids) + (i % n_sample) * nsymb * rg, nsymb, rg);
        mod->modulate(span<cf_t>(buf.data(), n), rd, 0, slot);
        dense_grid_writer wr(out.data(), nsymb, rg);
        dem->demodulate(wr, span<const cf_t>(buf.data(), n), 0, slot);
      }
    });
  }
  for (auto& th : pool) {
    th.join();
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

} // extern "C"
