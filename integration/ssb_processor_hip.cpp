// ssb_processor_hip.cpp -- see ssb_processor_hip.h.
#include "ssb_processor_hip.h"
#include "hip_resource_grid.h"

#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran_amd/ssb.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>

using namespace srsran;
using namespace srsran::hip;

namespace {

constexpr unsigned NSYMB = 14;

void log_error(const char* what, const std::string& detail)
{
  std::fprintf(stderr, "ssb_processor_hip: %s: %s\n", what, detail.c_str());
}

// pdu_t -> the C-ABI PDU; an empty string when the block can be processed.
std::string convert(const ssb_processor::pdu_t& pdu, srs_amd_ssb_pdu& out, uint32_t& l0, uint32_t& k0)
{
  if (pdu.ports.empty() || pdu.ports.size() > 4) {
    return "ports outside 1..4";
  }
  out                   = srs_amd_ssb_pdu{};
  out.numerology        = to_numerology_value(pdu.slot.scs());
  out.sfn               = pdu.slot.sfn();
  out.slot_index        = pdu.slot.slot_index();
  out.phys_cell_id      = pdu.phys_cell_id;
  out.beta_pss_dB       = pdu.beta_pss;
  out.ssb_idx           = pdu.ssb_idx;
  out.L_max             = pdu.L_max;
  out.common_scs        = static_cast<uint32_t>(pdu.common_scs);
  out.subcarrier_offset = pdu.subcarrier_offset.to_uint();
  out.offset_to_pointA  = pdu.offset_to_pointA.to_uint();
  out.pattern_case      = static_cast<uint32_t>(pdu.pattern_case);
  for (unsigned i = 0; i != ssb_processor::MIB_PAYLOAD_SIZE; ++i) {
    out.mib_payload[i] = pdu.mib_payload[i];
  }
  out.nof_ports = static_cast<uint32_t>(pdu.ports.size());
  for (unsigned i = 0; i != pdu.ports.size(); ++i) {
    out.ports[i] = pdu.ports[i];
  }
  if (srs_amd_ssb_position(&out, &l0, &k0) != SRS_AMD_OK) {
    return srs_amd_last_error();
  }
  return {};
}

struct shared_state {
  srs_amd_ssb_processor* proc   = nullptr;
  int                    device = 0;
  std::atomic<uint64_t>  nof_pdus{0}, nof_errors{0}, nof_device{0};
  ~shared_state() { srs_amd_ssb_processor_destroy(proc); }
};

class ssb_processor_hip : public ssb_processor
{
public:
  explicit ssb_processor_hip(std::shared_ptr<shared_state> s) : st(std::move(s))
  {
    (void)hipSetDevice(st->device);
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
      throw std::runtime_error("ssb_processor_hip: stream");
    }
  }
  ~ssb_processor_hip() override
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
    srs_amd_ssb_pdu p;
    uint32_t        l0 = 0, k0 = 0;
    std::string     err = convert(pdu, p, l0, k0);
    const unsigned  nof_ports = grid.get_nof_ports(), nsubc = grid.get_nof_subc();
    for (unsigned i = 0; err.empty() && i != p.nof_ports; ++i) {
      if (p.ports[i] >= nof_ports) {
        err = "port " + std::to_string(p.ports[i]) + " outside the grid";
      }
    }
    if (err.empty() && k0 + 240 > nsubc) {
      err = "the block exceeds the grid's subcarriers";
    }
    if (!err.empty()) {
      ++st->nof_errors;
      log_error("PDU not processed", err);
      return;
    }
    (void)hipSetDevice(st->device);
    if (hip_resource_grid* g = hip_grid_of(grid)) {
      p.d_grid     = g->device_write(stream);
      const int rc = srs_amd_ssb_process_slot(st->proc, &p, 1, nullptr, 0, 0, nof_ports, nsubc, stream);
      g->device_written(stream);
      if (rc != SRS_AMD_OK) {
        ++st->nof_errors;
        log_error("slot call", srs_amd_last_error());
      } else {
        ++st->nof_device;
      }
      return;
    }
    // host writer: the block on the GPU into a scratch grid, its four symbols of every port back, the block's REs
    // stored
    const size_t plane = static_cast<size_t>(NSYMB) * nsubc;
    if (!reserve(nof_ports * plane * sizeof(uint32_t))) {
      ++st->nof_errors;
      log_error("PDU not processed", "device / pinned buffer allocation");
      return;
    }
    int        rc = srs_amd_ssb_process_slot(st->proc, &p, 1, scratch, plane, 1, nof_ports, nsubc, stream);
    hipError_t e  = hipSuccess;
    if (rc == SRS_AMD_OK) {
      e = hipMemcpy2DAsync(rows, 4 * nsubc * sizeof(uint32_t), scratch + l0 * nsubc, plane * sizeof(uint32_t),
                           4 * nsubc * sizeof(uint32_t), nof_ports, hipMemcpyDeviceToHost, stream);
      e = e == hipSuccess ? hipStreamSynchronize(stream) : e;
    }
    if (rc != SRS_AMD_OK || e != hipSuccess) {
      ++st->nof_errors;
      log_error("slot call", rc != SRS_AMD_OK ? std::string(srs_amd_last_error()) : hipGetErrorString(e));
      return;
    }
    // the REs the reference writes, per symbol of the block: [first, last) subcarrier ranges relative to k0
    static const unsigned ranges[4][3][2] = {{{56, 183}, {0, 0}, {0, 0}},
                                             {{0, 240}, {0, 0}, {0, 0}},
                                             {{0, 48}, {56, 183}, {192, 240}},
                                             {{0, 240}, {0, 0}, {0, 0}}};
    for (unsigned i = 0; i != p.nof_ports; ++i) {
      const unsigned a = p.ports[i];
      for (unsigned s = 0; s != 4; ++s) {
        span<cbf16_t>   row = grid.get_view(a, l0 + s);
        const uint32_t* src = rows + (static_cast<size_t>(a) * 4 + s) * nsubc;
        for (const auto& r : ranges[s]) {
          if (r[1] > r[0]) {
            std::memcpy(static_cast<void*>(row.data() + k0 + r[0]), src + k0 + r[0], (r[1] - r[0]) * sizeof(uint32_t));
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

class ssb_pdu_validator_hip : public ssb_pdu_validator
{
public:
  error_type<std::string> is_valid(const ssb_processor::pdu_t& pdu) const override
  {
    srs_amd_ssb_pdu   p;
    uint32_t          l0, k0;
    const std::string e = convert(pdu, p, l0, k0);
    if (!e.empty()) {
      return make_unexpected(e);
    }
    return default_success_t();
  }
};

class ssb_processor_factory_hip_impl : public ssb_processor_factory_hip
{
public:
  explicit ssb_processor_factory_hip_impl(const ssb_processor_hip_config& c) : st(std::make_shared<shared_state>())
  {
    int dev = c.device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
      throw std::runtime_error("no HIP device");
    }
    st->device = dev;
    if (srs_amd_ssb_processor_create(&st->proc, dev) != SRS_AMD_OK) {
      throw std::runtime_error(srs_amd_last_error());
    }
  }
  std::unique_ptr<ssb_processor> create() override { return std::make_unique<ssb_processor_hip>(st); }
  // The reference wraps its processors in its logging decorator (factories.cpp); the MI355X processors log their
  // errors themselves.
  std::unique_ptr<ssb_processor> create(srslog::basic_logger& /*logger*/) override { return create(); }
  std::unique_ptr<ssb_pdu_validator> create_validator() override { return std::make_unique<ssb_pdu_validator_hip>(); }
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

std::shared_ptr<ssb_processor_factory_hip>
srsran::hip::create_ssb_processor_factory_hip(const ssb_processor_hip_config& cfg)
{
  try {
    return std::make_shared<ssb_processor_factory_hip_impl>(cfg);
  } catch (const std::exception& e) {
    log_error("factory", e.what());
    return nullptr;
  }
}
