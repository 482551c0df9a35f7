// pdcch_processor_hip.cpp -- see pdcch_processor_hip.h.
#include "pdcch_processor_hip.h"
#include "hip_resource_grid.h"

#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran_amd/pdcch.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace srsran;
using namespace srsran::hip;

namespace {

constexpr unsigned NSYMB     = 14;
constexpr unsigned MAX_PORTS = 4;

void log_error(const char* what, const std::string& detail)
{
  std::fprintf(stderr, "pdcch_processor_hip: %s: %s\n", what, detail.c_str());
}

// pdu_t -> the C-ABI PDU; an empty string when supported.
std::string convert(const pdcch_processor::pdu_t& pdu, srs_amd_pdcch_pdu& out)
{
  if (pdu.cp != cyclic_prefix::NORMAL) {
    return "extended cyclic prefix";
  }
  const precoding_configuration& pc = pdu.dci.precoding;
  if (pc.get_nof_layers() != 1) {
    return "Precoding number of layers (i.e., " + std::to_string(pc.get_nof_layers()) + ") must be one.";
  }
  if (pc.get_nof_ports() == 0 || pc.get_nof_ports() > MAX_PORTS) {
    return "ports outside 1..4";
  }
  for (unsigned g = 1; g < pc.get_nof_prg(); ++g) {
    if (!(pc.get_prg_coefficients(g) == pc.get_prg_coefficients(0))) {
      return "precoding that differs between PRGs";
    }
  }
  if (pdu.dci.payload.empty()) {
    return "Empty payload.";
  }
  out                                  = srs_amd_pdcch_pdu{};
  out.numerology                       = to_numerology_value(pdu.slot.scs());
  out.slot_index                       = pdu.slot.slot_index();
  const pdcch_processor::coreset_description& c = pdu.coreset;
  out.coreset.bwp_size_rb              = c.bwp_size_rb;
  out.coreset.bwp_start_rb             = c.bwp_start_rb;
  out.coreset.start_symbol_index       = c.start_symbol_index;
  out.coreset.duration                 = c.duration;
  for (unsigned i = 0; i != c.frequency_resources.size() && i < 64; ++i) {
    if (c.frequency_resources.test(i)) {
      out.coreset.frequency_resources[i / 8] |= static_cast<uint8_t>(1u << (i % 8));
    }
  }
  out.coreset.cce_to_reg_mapping = static_cast<uint32_t>(c.cce_to_reg_mapping);
  out.coreset.reg_bundle_size    = c.reg_bundle_size;
  out.coreset.interleaver_size   = c.interleaver_size;
  out.coreset.shift_index        = c.shift_index;
  const pdcch_processor::dci_description& d = pdu.dci;
  out.dci.rnti                 = d.rnti;
  out.dci.n_id_pdcch_dmrs      = d.n_id_pdcch_dmrs;
  out.dci.n_id_pdcch_data      = d.n_id_pdcch_data;
  out.dci.n_rnti               = d.n_rnti;
  out.dci.cce_index            = d.cce_index;
  out.dci.aggregation_level    = d.aggregation_level;
  out.dci.dmrs_power_offset_dB = d.dmrs_power_offset_dB;
  out.dci.data_power_offset_dB = d.data_power_offset_dB;
  out.dci.payload_size         = static_cast<uint32_t>(d.payload.size());
  std::memcpy(out.dci.payload, d.payload.data(), d.payload.size());
  out.dci.nof_ports = pc.get_nof_ports();
  for (unsigned a = 0; a != pc.get_nof_ports(); ++a) {
    const cf_t w           = pc.get_coefficient(0, a, 0);
    out.dci.weights[a][0] = w.real();
    out.dci.weights[a][1] = w.imag();
  }
  return {};
}

struct shared_state {
  srs_amd_pdcch_processor* proc   = nullptr;
  int                      device = 0;
  std::atomic<uint64_t>    nof_pdus{0}, nof_errors{0}, nof_device{0};
  ~shared_state() { srs_amd_pdcch_processor_destroy(proc); }
};

class pdcch_processor_hip : public pdcch_processor
{
public:
  explicit pdcch_processor_hip(std::shared_ptr<shared_state> s) : st(std::move(s))
  {
    (void)hipSetDevice(st->device);
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
      throw std::runtime_error("pdcch_processor_hip: stream");
    }
  }
  ~pdcch_processor_hip() override
  {
    (void)hipSetDevice(st->device);
    (void)hipStreamSynchronize(stream);
    (void)hipStreamDestroy(stream);
    (void)hipFree(scratch);
    (void)hipHostFree(rows);
  }

  void process(resource_grid_writer& grid, const pdu_t& pdu) override
  {
    ++st->nof_pdus;
    srs_amd_pdcch_pdu p;
    std::string       err = convert(pdu, p);
    if (err.empty() && p.dci.nof_ports > grid.get_nof_ports()) {
      err = "the grid has fewer ports than the precoding";
    }
    if (!err.empty()) {
      ++st->nof_errors;
      log_error("PDU not processed", err);
      return;
    }
    const unsigned nsubc = grid.get_nof_subc();
    (void)hipSetDevice(st->device);
    if (hip_resource_grid* g = hip_grid_of(grid)) {
      p.d_grid = g->device_write(stream);
      const int rc = srs_amd_pdcch_process_slot(st->proc, &p, 1, nullptr, 0, 0, nsubc, stream);
      g->device_written(stream);
      if (rc != SRS_AMD_OK) {
        ++st->nof_errors;
        log_error("slot call", srs_amd_last_error());
      } else {
        ++st->nof_device;
      }
      return;
    }
    // host writer: the DCI's CRBs, the REs on the GPU, the CORESET rows back, the CRBs' REs stored
    uint8_t   mask[SRS_AMD_CRB_MASK_BYTES];
    const int nrb = srs_amd_pdcch_rb_mask(&p, mask);
    if (nrb <= 0) {
      ++st->nof_errors;
      log_error("PDU not processed", srs_amd_last_error());
      return;
    }
    const unsigned P     = p.dci.nof_ports;
    const size_t   plane = static_cast<size_t>(NSYMB) * nsubc;
    if (!reserve(P * plane * sizeof(uint32_t))) {
      ++st->nof_errors;
      log_error("PDU not processed", "device / pinned buffer allocation");
      return;
    }
    const unsigned l0 = p.coreset.start_symbol_index, nl = p.coreset.duration;
    int            rc = srs_amd_pdcch_process_slot(st->proc, &p, 1, scratch, plane, 1, nsubc, stream);
    hipError_t     e  = hipSuccess;
    if (rc == SRS_AMD_OK) {
      // the CORESET symbols of every port: P rows of nl x nsubc, plane apart
      e = hipMemcpy2DAsync(rows, nl * nsubc * sizeof(uint32_t), scratch + l0 * nsubc, plane * sizeof(uint32_t),
                           nl * nsubc * sizeof(uint32_t), P, hipMemcpyDeviceToHost, stream);
      e = e == hipSuccess ? hipStreamSynchronize(stream) : e;
    }
    if (rc != SRS_AMD_OK || e != hipSuccess) {
      ++st->nof_errors;
      log_error("slot call", rc != SRS_AMD_OK ? std::string(srs_amd_last_error()) : hipGetErrorString(e));
      return;
    }
    for (unsigned a = 0; a != P; ++a) {
      for (unsigned li = 0; li != nl; ++li) {
        span<cbf16_t>   row = grid.get_view(a, l0 + li);
        const uint32_t* src = rows + (static_cast<size_t>(a) * nl + li) * nsubc;
        for (unsigned r = 0; r != 8 * SRS_AMD_CRB_MASK_BYTES; ++r) {
          if ((mask[r / 8] >> (r % 8)) & 1u) {
            std::memcpy(static_cast<void*>(row.data() + 12 * r), src + 12 * r, 12 * sizeof(uint32_t));
          }
        }
      }
    }
  }

private:
  bool reserve(size_t bytes)
  {
    if (bytes <= capacity) {
      return true;
    }
    (void)hipFree(scratch);
    (void)hipHostFree(rows);
    scratch  = nullptr;
    rows     = nullptr;
    capacity = 0;
    if (hipMalloc(&scratch, bytes) != hipSuccess || hipHostMalloc(&rows, bytes, hipHostMallocDefault) != hipSuccess) {
      return false;
    }
    capacity = bytes;
    return true;
  }

  std::shared_ptr<shared_state> st;
  hipStream_t                   stream   = nullptr;
  uint32_t*                     scratch  = nullptr;
  uint32_t*                     rows     = nullptr;
  size_t                        capacity = 0;
};

class pdcch_pdu_validator_hip : public pdcch_pdu_validator
{
public:
  error_type<std::string> is_valid(const pdcch_processor::pdu_t& pdu) const override
  {
    srs_amd_pdcch_pdu p;
    const std::string e = convert(pdu, p);
    if (!e.empty()) {
      return make_unexpected(e);
    }
    uint8_t mask[SRS_AMD_CRB_MASK_BYTES];
    if (srs_amd_pdcch_rb_mask(&p, mask) <= 0) {
      return make_unexpected(std::string(srs_amd_last_error()));
    }
    return default_success_t();
  }
};

class pdcch_processor_factory_hip_impl : public pdcch_processor_factory_hip
{
public:
  explicit pdcch_processor_factory_hip_impl(const pdcch_processor_hip_config& c) : st(std::make_shared<shared_state>())
  {
    int dev = c.device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
      throw std::runtime_error("no HIP device");
    }
    st->device = dev;
    if (srs_amd_pdcch_processor_create(&st->proc, dev) != SRS_AMD_OK) {
      throw std::runtime_error(srs_amd_last_error());
    }
  }
  std::unique_ptr<pdcch_processor> create() override { return std::make_unique<pdcch_processor_hip>(st); }
  // The reference wraps its processors in its logging decorator (factories.cpp); the MI355X processors log their
  // errors themselves.
  std::unique_ptr<pdcch_processor> create(srslog::basic_logger& /*logger*/, bool /*enable_logging_broadcast*/) override
  {
    return create();
  }
  std::unique_ptr<pdcch_pdu_validator> create_validator() override
  {
    return std::make_unique<pdcch_pdu_validator_hip>();
  }
  statistics get_statistics() const override
  {
    statistics s;
    s.nof_pdus         = st->nof_pdus;
    s.nof_errors       = st->nof_errors;
    s.nof_device_grids = st->nof_device;
    return s;
  }

private:
  std::shared_ptr<shared_state> st;
};

} // namespace

std::shared_ptr<pdcch_processor_factory_hip>
srsran::hip::create_pdcch_processor_factory_hip(const pdcch_processor_hip_config& cfg)
{
  try {
    return std::make_shared<pdcch_processor_factory_hip_impl>(cfg);
  } catch (const std::exception& e) {
    log_error("factory", e.what());
    return nullptr;
  }
}
