// kernel_probe.cpp -- live kernel probes (include/srsran_amd/profiling.h, kernel_probe.h).
#include "srsran_amd/ldpc.h" // status codes
#include "srsran_amd/profiling.h"

#include "api_common.h"
#include "kernel_probe.h"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

namespace {

struct probe_state {
  std::atomic<bool>       armed{false};
  std::mutex              mtx;
  std::vector<hipEvent_t> ev; // [2 * slot] start, [2 * slot + 1] end
  uint32_t                used = 0, ended = 0;
  int                     device = 0;
};

probe_state g_probes[SRS_AMD_PROBE_COUNT];

void release(probe_state& p)
{
  for (hipEvent_t e : p.ev) {
    (void)hipEventDestroy(e);
  }
  p.ev.clear();
  p.used = p.ended = 0;
}

} // namespace

srs_amd::probe_events srs_amd::probe_take(int probe)
{
  probe_events pe;
  if (probe < 0 || probe >= SRS_AMD_PROBE_COUNT || !g_probes[probe].armed.load(std::memory_order_relaxed)) {
    return pe;
  }
  probe_state&                p = g_probes[probe];
  std::lock_guard<std::mutex> lock(p.mtx);
  if (!p.armed.load(std::memory_order_relaxed) || 2 * (p.used + 1) > p.ev.size()) {
    return pe;
  }
  pe.slot  = static_cast<int>(p.used++);
  pe.start = p.ev[2 * pe.slot];
  pe.stop  = p.ev[2 * pe.slot + 1];
  return pe;
}

void srs_amd::probe_commit(int probe, int slot)
{
  if (slot < 0 || probe < 0 || probe >= SRS_AMD_PROBE_COUNT) {
    return;
  }
  probe_state&                p = g_probes[probe];
  std::lock_guard<std::mutex> lock(p.mtx);
  ++p.ended;
}

extern "C" {

int srs_amd_probe_arm(int probe, uint32_t max_launches)
{
  if (probe < 0 || probe >= SRS_AMD_PROBE_COUNT || max_launches == 0 || max_launches > (1u << 16)) {
    return srs_amd::fail(SRS_AMD_EINVAL, "invalid probe %d or launch count %u", probe, max_launches);
  }
  probe_state&                p = g_probes[probe];
  std::lock_guard<std::mutex> lock(p.mtx);
  p.armed.store(false);
  for (hipEvent_t e : p.ev) {
    (void)hipEventSynchronize(e);
  }
  release(p);
  hipError_t e = hipGetDevice(&p.device);
  p.ev.assign(2 * static_cast<size_t>(max_launches), nullptr);
  for (size_t i = 0; i < p.ev.size() && e == hipSuccess; ++i) {
    e = hipEventCreate(&p.ev[i]);
  }
  if (e != hipSuccess) {
    p.ev.erase(std::remove(p.ev.begin(), p.ev.end(), nullptr), p.ev.end());
    release(p);
    return srs_amd::hip_fail(e, "kernel probe events");
  }
  p.armed.store(true);
  return SRS_AMD_OK;
}

int srs_amd_probe_read(int probe, uint32_t* launches, double* total_ms, double* min_ms, double* max_ms)
{
  if (probe < 0 || probe >= SRS_AMD_PROBE_COUNT) {
    return srs_amd::fail(SRS_AMD_EINVAL, "invalid probe %d", probe);
  }
  probe_state&                p = g_probes[probe];
  std::lock_guard<std::mutex> lock(p.mtx);
  p.armed.store(false);
  double     sum = 0.0, lo = 0.0, hi = 0.0;
  uint32_t   n   = 0;
  hipError_t e   = hipSuccess;
  for (uint32_t i = 0; i < p.used && i < p.ended && e == hipSuccess; ++i) {
    e = hipEventSynchronize(p.ev[2 * i + 1]);
    float ms = 0.0f;
    if (e == hipSuccess) {
      e = hipEventElapsedTime(&ms, p.ev[2 * i], p.ev[2 * i + 1]);
    }
    if (e == hipSuccess) {
      sum += ms;
      lo = n == 0 ? ms : std::min<double>(lo, ms);
      hi = n == 0 ? ms : std::max<double>(hi, ms);
      ++n;
    }
  }
  release(p);
  if (launches != nullptr) {
    *launches = n;
  }
  if (total_ms != nullptr) {
    *total_ms = sum;
  }
  if (min_ms != nullptr) {
    *min_ms = lo;
  }
  if (max_ms != nullptr) {
    *max_ms = hi;
  }
  return e == hipSuccess ? SRS_AMD_OK : srs_amd::hip_fail(e, "kernel probe events");
}

} // extern "C"
