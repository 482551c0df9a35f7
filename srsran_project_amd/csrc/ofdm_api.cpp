// ofdm_api.cpp -- C-ABI of the MI355X OFDM modulator / demodulator and DFT
// processor (include/srsran_amd/ofdm.h).
//
// Host-side tables follow the reference exactly (same double / float
// operations, so the same bits):
//   phase compensation: lib/phy/lower/modulation/phase_compensation_lut.h:45-75
//     (is_tx = true for the modulator, false for the demodulator), then
//     cf_t * float scale (ofdm_modulator_impl.cpp:100);
//   window-offset compensation: ofdm_demodulator_impl.cpp:60-70 (std::polar<float>);
//   CP lengths: cyclic_prefix.h:93-104 + phy_time_unit.h:100-110.
// Argument checks mirror the reference constructors' assertions.
#include "srsran_amd/ofdm.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "ofdm_args.h"
#include <cmath>
#include <complex>
#include <mutex>
#include <vector>

namespace srs_amd {
namespace {

struct ofdm_geometry {
  uint32_t                      N = 0, rg = 0, nsymb = 0, slots_per_subframe = 0;
  std::vector<ofdm_symbol_info> symbols; // [slots_per_subframe * nsymb]
  std::vector<uint32_t>         slot_size;
};

uint32_t cp_samples(uint32_t symbol, uint32_t mu, uint32_t N, bool extended)
{
  uint32_t kappa = 144u >> mu;
  if (extended) {
    kappa = 512u >> mu;
  } else if (symbol == 0 || symbol == 7u * (1u << mu)) {
    kappa += 16;
  }
  const uint64_t srate = 15000ull * (1ull << mu) * N;
  return static_cast<uint32_t>((static_cast<uint64_t>(kappa) * 64 * srate) / (15000ull * 2048 * 64));
}

int make_geometry(ofdm_geometry& g, const srs_amd_ofdm_config* cfg, bool is_tx)
{
  if (cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null configuration");
  }
  if (cfg->numerology > 4) {
    return fail(SRS_AMD_EINVAL, "invalid numerology %u", cfg->numerology);
  }
  if (!std::isnormal(cfg->scale)) {
    return fail(SRS_AMD_EINVAL, "Invalid scaling factor %g", static_cast<double>(cfg->scale));
  }
  g.N  = cfg->dft_size;
  g.rg = cfg->bw_rb * 12;
  if (g.N <= g.rg) {
    return fail(SRS_AMD_EINVAL, "The DFT size (%u) must be greater than the resource grid size (%u)", g.N, g.rg);
  }
  if (!ofdm_size_supported(g.N)) {
    return fail(SRS_AMD_EINVAL, "DFT size %u not supported by the MI355X OFDM kernels", g.N);
  }
  const uint32_t mu     = cfg->numerology;
  const bool     ext    = cfg->cp_extended != 0;
  const uint64_t srate  = 15000ull * (1ull << mu) * g.N;
  g.nsymb               = ext ? 12 : 14;
  g.slots_per_subframe  = 1u << mu;
  // every CP must be an integer number of samples (phy_time_unit::to_samples assertion)
  for (uint32_t kappa : {144u >> mu, (144u >> mu) + 16u, 512u >> mu}) {
    if ((static_cast<uint64_t>(kappa) * 64 * srate) % (15000ull * 2048 * 64) != 0) {
      return fail(SRS_AMD_EINVAL, "Incompatible sampling rate %llu Hz", static_cast<unsigned long long>(srate));
    }
  }
  if (!is_tx && cfg->nof_samples_window_offset != 0 && cfg->nof_samples_window_offset >= (144 * g.N) / 2048) {
    return fail(SRS_AMD_EINVAL, "The DFT window offset (i.e., %u) must be lower than %u.",
                cfg->nof_samples_window_offset, (144 * g.N) / 2048);
  }
  // phase_compensation_lut.h:45-75
  const double sampling_rate_Hz = static_cast<double>(srate);
  const double sign_two_pi      = ((is_tx) ? -1 : 1) * 2.0 * M_PI;
  g.symbols.assign(g.slots_per_subframe * g.nsymb, ofdm_symbol_info{});
  g.slot_size.assign(g.slots_per_subframe, 0);
  uint32_t symbol_offset = 0;
  for (uint32_t s = 0; s < g.slots_per_subframe * g.nsymb; ++s) {
    const uint32_t cp = cp_samples(s, mu, g.N, ext);
    symbol_offset += cp;
    const double start_time_s = static_cast<double>(symbol_offset) / sampling_rate_Hz;
    const double symbol_phase = sign_two_pi * cfg->center_freq_hz * start_time_s;
    const std::complex<float> phase = static_cast<std::complex<float>>(std::polar(1.0, symbol_phase));
    const std::complex<float> coef  = phase * cfg->scale;
    symbol_offset += g.N;
    ofdm_symbol_info& si = g.symbols[s];
    si.cp_len            = cp;
    si.offset            = g.slot_size[s / g.nsymb];
    si.coef_re           = coef.real();
    si.coef_im           = coef.imag();
    g.slot_size[s / g.nsymb] += cp + g.N;
  }
  return SRS_AMD_OK;
}

// W_N^m = exp(-2*pi*i*m/N), double precision rounded to float.
std::vector<float> twiddle_table(uint32_t N)
{
  std::vector<float> t(2 * N);
  for (uint32_t m = 0; m < N; ++m) {
    const double a = -2.0 * M_PI * static_cast<double>(m) / static_cast<double>(N);
    t[2 * m]       = static_cast<float>(std::cos(a));
    t[2 * m + 1]   = static_cast<float>(std::sin(a));
  }
  return t;
}

template <class T>
hipError_t upload(T** dst, const std::vector<T>& src)
{
  hipError_t e = hipMalloc(dst, src.size() * sizeof(T));
  if (e == hipSuccess) {
    e = hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
  }
  return e;
}

struct device_scratch {
  void*  ptr  = nullptr;
  size_t size = 0;
  hipError_t ensure(size_t n)
  {
    if (n <= size) {
      return hipSuccess;
    }
    (void)hipFree(ptr);
    ptr          = nullptr;
    size         = 0;
    hipError_t e = hipMalloc(&ptr, n);
    if (e == hipSuccess) {
      size = n;
    }
    return e;
  }
  ~device_scratch() { (void)hipFree(ptr); }
};

} // namespace
} // namespace srs_amd

using namespace srs_amd;

struct srs_amd_ofdm_engine {
  int                 device = 0;
  bool                is_tx  = true;
  srs_amd_ofdm_config cfg{};
  ofdm_geometry       geo;
  ofdm_symbol_info*   d_symbols  = nullptr;
  ofdm_symbol_info*   d_symbols0 = nullptr; // the same with every offset 0 (symbol forms)
  float*              d_twiddles = nullptr;
  float*              d_window   = nullptr;
  hipStream_t         stream     = nullptr;
  device_scratch      scratch;
  std::mutex          mtx;

  ~srs_amd_ofdm_engine()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(d_symbols);
    (void)hipFree(d_symbols0);
    (void)hipFree(d_twiddles);
    (void)hipFree(d_window);
  }

  int init(const srs_amd_ofdm_config* c, bool tx, int dev)
  {
    int rc = make_geometry(geo, c, tx);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    rc = select_device(dev);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    device       = dev;
    is_tx        = tx;
    cfg          = *c;
    hipError_t e = upload(&d_symbols, geo.symbols);
    if (e == hipSuccess) {
      e = upload(&d_symbols0, symbols0());
    }
    if (e == hipSuccess) {
      e = upload(&d_twiddles, twiddle_table(geo.N));
    }
    if (e == hipSuccess && !tx && c->nof_samples_window_offset != 0) {
      // ofdm_demodulator_impl.cpp:60-70
      std::vector<float> w(2 * geo.N);
      const float omega = static_cast<float>(c->nof_samples_window_offset) * static_cast<float>(2.0 * M_PI) /
                          static_cast<float>(geo.N);
      for (uint32_t i = 0; i != geo.N; ++i) {
        const std::complex<float> v = std::polar(1.0F, omega * static_cast<float>(i));
        w[2 * i]                    = v.real();
        w[2 * i + 1]                = v.imag();
      }
      e = upload(&d_window, w);
    }
    if (e == hipSuccess) {
      e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
    }
    return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "OFDM tables");
  }

  std::vector<ofdm_symbol_info> symbols0() const
  {
    std::vector<ofdm_symbol_info> s = geo.symbols;
    for (ofdm_symbol_info& x : s) {
      x.offset = 0;
    }
    return s;
  }

  // New phase compensation tables (same host arithmetic as the constructor), in stream order with the launches.
  int set_center_frequency(double hz)
  {
    srs_amd_ofdm_config c = cfg;
    c.center_freq_hz      = hz;
    ofdm_geometry g;
    int           rc = make_geometry(g, &c, is_tx);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    std::lock_guard<std::mutex> lock(mtx);
    hipError_t                  e = hipSetDevice(device);
    if (e == hipSuccess) {
      e = hipStreamSynchronize(stream); // no launch of this engine still reads the old tables
    }
    geo = g;
    cfg = c;
    if (e == hipSuccess) {
      e = hipMemcpy(d_symbols, geo.symbols.data(), geo.symbols.size() * sizeof(ofdm_symbol_info), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) {
      const std::vector<ofdm_symbol_info> s0 = symbols0();
      e = hipMemcpy(d_symbols0, s0.data(), s0.size() * sizeof(ofdm_symbol_info), hipMemcpyHostToDevice);
    }
    return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "OFDM phase compensation tables");
  }

  // One symbol (index within the subframe) of one port: host buffers, synchronous.
  int run_symbol(void* host_out, const void* host_in, uint32_t symbol_index)
  {
    const uint32_t nsym_sf = geo.nsymb * geo.slots_per_subframe;
    if (symbol_index >= nsym_sf) {
      return fail(SRS_AMD_EINVAL, "Symbol index %u exceeds the %u symbols of a subframe.", symbol_index, nsym_sf);
    }
    const ofdm_symbol_info& si     = geo.symbols[symbol_index];
    const size_t            gbytes = static_cast<size_t>(geo.rg) * 4;
    const size_t            sbytes = static_cast<size_t>(si.cp_len + geo.N) * 8;
    std::lock_guard<std::mutex> lock(mtx);
    hipError_t                  e = hipSetDevice(device);
    if (e == hipSuccess) {
      e = scratch.ensure(gbytes + sbytes);
    }
    auto* grid = static_cast<uint8_t*>(scratch.ptr);
    auto* samp = grid + gbytes;
    ofdm_args a{};
    a.symbols            = d_symbols0 + symbol_index;
    a.twiddles           = d_twiddles;
    a.window             = d_window;
    a.rg_size            = geo.rg;
    a.nsymb              = 1;
    a.nof_ports          = 1;
    a.first_slot         = 0;
    a.slots_per_subframe = 1;
    a.nof_items          = 1;
    a.sample_stride      = si.cp_len + geo.N;
    a.window_offset      = is_tx ? 0 : cfg.nof_samples_window_offset;
    a.in                 = is_tx ? static_cast<const void*>(grid) : static_cast<const void*>(samp);
    a.out                = is_tx ? static_cast<void*>(samp) : static_cast<void*>(grid);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(is_tx ? grid : samp, host_in, is_tx ? gbytes : sbytes, hipMemcpyHostToDevice, stream);
    }
    if (e == hipSuccess) {
      e = is_tx ? launch_ofdm_modulate(a, geo.N, stream) : launch_ofdm_demodulate(a, geo.N, stream);
    }
    if (e == hipSuccess) {
      e = hipMemcpyAsync(host_out, is_tx ? samp : grid, is_tx ? sbytes : gbytes, hipMemcpyDeviceToHost, stream);
    }
    if (e == hipSuccess) {
      e = hipStreamSynchronize(stream);
    }
    return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, is_tx ? "ofdm modulate symbol" : "ofdm demodulate symbol");
  }

  // one symbol between device-accessible buffers on `s` (no copies, no scratch: no lock needed)
  int run_symbol_async(void* out, const void* in, uint32_t symbol_index, hipStream_t s) const
  {
    const uint32_t nsym_sf = geo.nsymb * geo.slots_per_subframe;
    if (symbol_index >= nsym_sf) {
      return fail(SRS_AMD_EINVAL, "Symbol index %u exceeds the %u symbols of a subframe.", symbol_index, nsym_sf);
    }
    const ofdm_symbol_info& si = geo.symbols[symbol_index];
    ofdm_args               a{};
    a.symbols            = d_symbols0 + symbol_index;
    a.twiddles           = d_twiddles;
    a.window             = d_window;
    a.rg_size            = geo.rg;
    a.nsymb              = 1;
    a.nof_ports          = 1;
    a.first_slot         = 0;
    a.slots_per_subframe = 1;
    a.nof_items          = 1;
    a.sample_stride      = si.cp_len + geo.N;
    a.window_offset      = is_tx ? 0 : cfg.nof_samples_window_offset;
    a.in                 = in;
    a.out                = out;
    hipError_t e         = hipSetDevice(device);
    if (e == hipSuccess) {
      e = is_tx ? launch_ofdm_modulate(a, geo.N, s) : launch_ofdm_demodulate(a, geo.N, s);
    }
    return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, is_tx ? "ofdm modulate symbol" : "ofdm demodulate symbol");
  }

  // staged symbols (demodulator): items [count][2] and samples [count][stride], device-accessible, on `s`
  int run_symbols_async(uint16_t* grid, const uint32_t* items, const float* samples, uint32_t stride, uint32_t count,
                        hipStream_t s) const
  {
    const uint32_t nsym_sf = geo.nsymb * geo.slots_per_subframe;
    uint32_t       max_sz  = 0;
    for (uint32_t i = 0; i != nsym_sf; ++i) {
      max_sz = std::max(max_sz, geo.symbols[i].cp_len + geo.N);
    }
    if (stride < max_sz) {
      return fail(SRS_AMD_EINVAL, "Sample stride %u below the longest symbol (%u samples).", stride, max_sz);
    }
    ofdm_args a{};
    a.symbols            = d_symbols0;
    a.twiddles           = d_twiddles;
    a.window             = d_window;
    a.rg_size            = geo.rg;
    a.nsymb              = 1;
    a.nof_ports          = 1;
    a.slots_per_subframe = 1;
    a.nof_items          = count;
    a.sample_stride      = stride;
    a.window_offset      = cfg.nof_samples_window_offset;
    a.in                 = samples;
    a.out                = grid;
    a.items              = items;
    a.nof_symbol_infos   = nsym_sf;
    hipError_t e         = hipSetDevice(device);
    if (e == hipSuccess) {
      e = launch_ofdm_demodulate(a, geo.N, s);
    }
    return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ofdm demodulate symbols");
  }

  uint32_t symbol_size(uint32_t symbol_index) const
  {
    return symbol_index < geo.symbols.size() ? geo.symbols[symbol_index].cp_len + geo.N : 0;
  }

  ofdm_args args(uint32_t nof_ports, uint32_t first_slot, uint32_t nof_slots, uint32_t stride) const
  {
    ofdm_args a{};
    a.symbols            = d_symbols;
    a.twiddles           = d_twiddles;
    a.window             = d_window;
    a.rg_size            = geo.rg;
    a.nsymb              = geo.nsymb;
    a.nof_ports          = nof_ports;
    a.first_slot         = first_slot % geo.slots_per_subframe;
    a.slots_per_subframe = geo.slots_per_subframe;
    a.nof_items          = nof_ports * nof_slots;
    a.sample_stride      = stride;
    a.window_offset      = is_tx ? 0 : cfg.nof_samples_window_offset;
    return a;
  }

  uint32_t max_slot_size() const
  {
    uint32_t m = 0;
    for (uint32_t s : geo.slot_size) {
      m = s > m ? s : m;
    }
    return m;
  }
};

struct srs_amd_ofdm_modulator : srs_amd_ofdm_engine {};
struct srs_amd_ofdm_demodulator : srs_amd_ofdm_engine {};

struct srs_amd_dft {
  int            device  = 0;
  uint32_t       N       = 0;
  int            inverse = 0;
  float*         d_tw    = nullptr;
  hipStream_t    stream  = nullptr;
  device_scratch scratch;
  std::mutex     mtx;
  ~srs_amd_dft()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(d_tw);
  }
};

namespace {

template <class T>
int create_engine(T** out, const srs_amd_ofdm_config* cfg, bool tx, int device)
{
  if (out == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *out   = nullptr;
  auto* h = new T();
  int   rc = h->init(cfg, tx, device);
  if (rc != SRS_AMD_OK) {
    delete h;
    return rc;
  }
  *out = h;
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_ofdm_modulator_create(srs_amd_ofdm_modulator** mod, const srs_amd_ofdm_config* cfg, int device)
{
  return create_engine(mod, cfg, true, device);
}

void srs_amd_ofdm_modulator_destroy(srs_amd_ofdm_modulator* mod)
{
  delete mod;
}

uint32_t srs_amd_ofdm_modulator_get_slot_size(const srs_amd_ofdm_modulator* mod, uint32_t slot_index)
{
  if (mod == nullptr || slot_index >= mod->geo.slots_per_subframe) {
    return 0;
  }
  return mod->geo.slot_size[slot_index];
}

int srs_amd_ofdm_modulate_batch(srs_amd_ofdm_modulator* mod,
                                const uint16_t*         d_grid,
                                uint32_t                nof_ports,
                                uint32_t                first_slot,
                                uint32_t                nof_slots,
                                float*                  d_samples,
                                uint32_t                sample_stride,
                                void*                   stream)
{
  if (mod == nullptr) {
    return fail(SRS_AMD_EINVAL, "null modulator");
  }
  if (nof_ports == 0 || nof_slots == 0) {
    return SRS_AMD_OK;
  }
  if (d_grid == nullptr || d_samples == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (sample_stride < mod->max_slot_size() && !(nof_slots == 1 && nof_ports == 1)) {
    return fail(SRS_AMD_EINVAL, "sample_stride %u shorter than a slot (%u samples)", sample_stride,
                mod->max_slot_size());
  }
  ofdm_args a = mod->args(nof_ports, first_slot, nof_slots, sample_stride);
  a.in        = d_grid;
  a.out       = d_samples;
  std::lock_guard<std::mutex> lock(mod->mtx);
  hipError_t                  e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = launch_ofdm_modulate(a, mod->geo.N, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ofdm_modulate_kernel launch");
}

int srs_amd_ofdm_modulate_slot(srs_amd_ofdm_modulator* mod, float* output, const uint16_t* grid, uint32_t slot_index)
{
  if (mod == nullptr || output == nullptr || grid == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const uint32_t nslots = mod->geo.slots_per_subframe;
  if (slot_index >= nslots) {
    return fail(SRS_AMD_EINVAL,
                "Slot index within the subframe %u exceeds the number of slots per subframe %u.", slot_index, nslots);
  }
  const size_t gbytes = static_cast<size_t>(mod->geo.nsymb) * mod->geo.rg * 4;
  const size_t n      = mod->geo.slot_size[slot_index];
  uint8_t*     base   = nullptr;
  {
    std::lock_guard<std::mutex> lock(mod->mtx);
    hipError_t                  e = hipSetDevice(mod->device);
    if (e == hipSuccess) {
      e = mod->scratch.ensure(gbytes + n * 8);
    }
    base = static_cast<uint8_t*>(mod->scratch.ptr);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base, grid, gbytes, hipMemcpyHostToDevice, mod->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging grid");
    }
  }
  int rc = srs_amd_ofdm_modulate_batch(mod, reinterpret_cast<const uint16_t*>(base), 1, slot_index, 1,
                                       reinterpret_cast<float*>(base + gbytes), static_cast<uint32_t>(n), mod->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(output, base + gbytes, n * 8, hipMemcpyDeviceToHost, mod->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(mod->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ofdm modulate");
}

uint32_t srs_amd_ofdm_modulator_get_symbol_size(const srs_amd_ofdm_modulator* mod, uint32_t symbol_index)
{
  return mod == nullptr ? 0 : mod->symbol_size(symbol_index);
}

int srs_amd_ofdm_modulator_set_center_frequency(srs_amd_ofdm_modulator* mod, double center_freq_hz)
{
  if (mod == nullptr) {
    return fail(SRS_AMD_EINVAL, "null modulator");
  }
  return mod->set_center_frequency(center_freq_hz);
}

int srs_amd_ofdm_modulate_symbol(srs_amd_ofdm_modulator* mod,
                                 float*                  output,
                                 const uint16_t*         grid_symbol,
                                 uint32_t                symbol_index)
{
  if (mod == nullptr || output == nullptr || grid_symbol == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  return mod->run_symbol(output, grid_symbol, symbol_index);
}

uint32_t srs_amd_ofdm_demodulator_get_symbol_size(const srs_amd_ofdm_demodulator* dem, uint32_t symbol_index)
{
  return dem == nullptr ? 0 : dem->symbol_size(symbol_index);
}

int srs_amd_ofdm_demodulator_set_center_frequency(srs_amd_ofdm_demodulator* dem, double center_freq_hz)
{
  if (dem == nullptr) {
    return fail(SRS_AMD_EINVAL, "null demodulator");
  }
  return dem->set_center_frequency(center_freq_hz);
}

int srs_amd_ofdm_demodulate_symbol(srs_amd_ofdm_demodulator* dem,
                                   uint16_t*                 grid_symbol,
                                   const float*              input,
                                   uint32_t                  symbol_index)
{
  if (dem == nullptr || grid_symbol == nullptr || input == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  return dem->run_symbol(grid_symbol, input, symbol_index);
}

int srs_amd_ofdm_modulate_symbol_async(srs_amd_ofdm_modulator* mod, float* output, const uint16_t* grid_symbol,
                                       uint32_t symbol_index, void* stream)
{
  if (mod == nullptr || output == nullptr || grid_symbol == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  return mod->run_symbol_async(output, grid_symbol, symbol_index, static_cast<hipStream_t>(stream));
}

int srs_amd_ofdm_demodulate_symbol_async(srs_amd_ofdm_demodulator* dem, uint16_t* grid_symbol, const float* input,
                                         uint32_t symbol_index, void* stream)
{
  if (dem == nullptr || grid_symbol == nullptr || input == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  return dem->run_symbol_async(grid_symbol, input, symbol_index, static_cast<hipStream_t>(stream));
}

int srs_amd_ofdm_demodulate_symbols_async(srs_amd_ofdm_demodulator* dem, uint16_t* grid, const uint32_t* items,
                                          const float* samples, uint32_t sample_stride, uint32_t count,
                                          void* d_scratch, void* stream)
{
  if (dem == nullptr || (count != 0 && (grid == nullptr || items == nullptr || samples == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (count == 0) {
    return SRS_AMD_OK;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (d_scratch != nullptr) {
    // pinned staging -> HBM by copy kernels (srs_amd::upload_pinned), then the transform from HBM
    const size_t sample_bytes = sizeof(float) * 2 * static_cast<size_t>(count) * sample_stride;
    auto*        d_samples    = static_cast<float*>(d_scratch);
    auto*        d_items      = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_scratch) + sample_bytes);
    hipError_t   e            = hipSetDevice(dem->device);
    if (e == hipSuccess) {
      e = srs_amd::upload_pinned(d_samples, samples, sample_bytes, s);
    }
    if (e == hipSuccess) {
      e = srs_amd::upload_pinned(d_items, items, sizeof(uint32_t) * 2 * count, s);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "ofdm staged symbols upload");
    }
    samples = d_samples;
    items   = d_items;
  }
  return dem->run_symbols_async(grid, items, samples, sample_stride, count, s);
}

int srs_amd_ofdm_demodulator_create(srs_amd_ofdm_demodulator** dem, const srs_amd_ofdm_config* cfg, int device)
{
  return create_engine(dem, cfg, false, device);
}

void srs_amd_ofdm_demodulator_destroy(srs_amd_ofdm_demodulator* dem)
{
  delete dem;
}

uint32_t srs_amd_ofdm_demodulator_get_slot_size(const srs_amd_ofdm_demodulator* dem, uint32_t slot_index)
{
  if (dem == nullptr || slot_index >= dem->geo.slots_per_subframe) {
    return 0;
  }
  return dem->geo.slot_size[slot_index];
}

int srs_amd_ofdm_demodulate_batch(srs_amd_ofdm_demodulator* dem,
                                  const float*              d_samples,
                                  uint32_t                  sample_stride,
                                  uint32_t                  nof_ports,
                                  uint32_t                  first_slot,
                                  uint32_t                  nof_slots,
                                  uint16_t*                 d_grid,
                                  void*                     stream)
{
  if (dem == nullptr) {
    return fail(SRS_AMD_EINVAL, "null demodulator");
  }
  if (nof_ports == 0 || nof_slots == 0) {
    return SRS_AMD_OK;
  }
  if (d_grid == nullptr || d_samples == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (sample_stride < dem->max_slot_size() && !(nof_slots == 1 && nof_ports == 1)) {
    return fail(SRS_AMD_EINVAL, "sample_stride %u shorter than a slot (%u samples)", sample_stride,
                dem->max_slot_size());
  }
  ofdm_args a = dem->args(nof_ports, first_slot, nof_slots, sample_stride);
  a.in        = d_samples;
  a.out       = d_grid;
  std::lock_guard<std::mutex> lock(dem->mtx);
  hipError_t                  e = hipSetDevice(dem->device);
  if (e == hipSuccess) {
    e = launch_ofdm_demodulate(a, dem->geo.N, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ofdm_demodulate_kernel launch");
}

int srs_amd_ofdm_demodulate_slot(srs_amd_ofdm_demodulator* dem, uint16_t* grid, const float* input, uint32_t slot_index)
{
  if (dem == nullptr || input == nullptr || grid == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (slot_index >= dem->geo.slots_per_subframe) {
    return fail(SRS_AMD_EINVAL, "Slot index %u exceeds the number of slots per subframe %u.", slot_index,
                dem->geo.slots_per_subframe);
  }
  const size_t gbytes = static_cast<size_t>(dem->geo.nsymb) * dem->geo.rg * 4;
  const size_t n      = dem->geo.slot_size[slot_index];
  uint8_t*     base   = nullptr;
  {
    std::lock_guard<std::mutex> lock(dem->mtx);
    hipError_t                  e = hipSetDevice(dem->device);
    if (e == hipSuccess) {
      e = dem->scratch.ensure(gbytes + n * 8);
    }
    base = static_cast<uint8_t*>(dem->scratch.ptr);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base + gbytes, input, n * 8, hipMemcpyHostToDevice, dem->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging samples");
    }
  }
  int rc = srs_amd_ofdm_demodulate_batch(dem, reinterpret_cast<const float*>(base + gbytes), static_cast<uint32_t>(n),
                                         1, slot_index, 1, reinterpret_cast<uint16_t*>(base), dem->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(grid, base, gbytes, hipMemcpyDeviceToHost, dem->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(dem->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ofdm demodulate");
}

int srs_amd_dft_create(srs_amd_dft** dft, uint32_t size, int direction, int device)
{
  if (dft == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *dft = nullptr;
  if (!ofdm_size_supported(size)) {
    return fail(SRS_AMD_EINVAL, "DFT size %u not supported by the MI355X DFT kernels", size);
  }
  if (direction != 0 && direction != 1) {
    return fail(SRS_AMD_EINVAL, "invalid DFT direction %d", direction);
  }
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* h      = new srs_amd_dft();
  h->device    = device;
  h->N         = size;
  h->inverse   = direction;
  hipError_t e = upload(&h->d_tw, twiddle_table(size));
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete h;
    return hip_fail(e, "DFT tables");
  }
  *dft = h;
  return SRS_AMD_OK;
}

void srs_amd_dft_destroy(srs_amd_dft* dft)
{
  delete dft;
}

int srs_amd_dft_run_batch(srs_amd_dft* dft, const float* d_input, float* d_output, uint32_t nof, void* stream)
{
  if (dft == nullptr) {
    return fail(SRS_AMD_EINVAL, "null DFT");
  }
  if (nof == 0) {
    return SRS_AMD_OK;
  }
  if (d_input == nullptr || d_output == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  dft_args a{};
  a.in       = d_input;
  a.out      = d_output;
  a.twiddles = dft->d_tw;
  a.nof      = nof;
  std::lock_guard<std::mutex> lock(dft->mtx);
  hipError_t                  e = hipSetDevice(dft->device);
  if (e == hipSuccess) {
    e = launch_dft(a, dft->N, dft->inverse, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "dft_kernel launch");
}

int srs_amd_dft_run(srs_amd_dft* dft, float* output, const float* input)
{
  if (dft == nullptr || output == nullptr || input == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t bytes = static_cast<size_t>(dft->N) * 8;
  float*       base  = nullptr;
  {
    std::lock_guard<std::mutex> lock(dft->mtx);
    hipError_t                  e = hipSetDevice(dft->device);
    if (e == hipSuccess) {
      e = dft->scratch.ensure(2 * bytes);
    }
    base = static_cast<float*>(dft->scratch.ptr);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base, input, bytes, hipMemcpyHostToDevice, dft->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging DFT input");
    }
  }
  int rc = srs_amd_dft_run_batch(dft, base, base + 2 * dft->N, 1, dft->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(output, base + 2 * dft->N, bytes, hipMemcpyDeviceToHost, dft->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(dft->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "dft run");
}

} // extern "C"
