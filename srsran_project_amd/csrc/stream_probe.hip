// stream_probe.hip -- do two HIP streams run concurrently on this device?  HIP maps streams onto
// GPU_MAX_HW_QUEUES hardware queues (4 on the MI355X boxes) in an order that differs from process to process, and two
// streams sharing a queue execute one after the other whatever their events say (DESIGN.md, r04 performance notes).
// stream_fan (device_buffer.h) asks this once per (helper, caller stream) pair and replaces a helper that shares the
// caller's queue.
#include <hip/hip_runtime.h>

#include "device_buffer.h"

namespace srs_amd {

namespace {

// one wave that waits `ticks` of the constant-rate wall clock (s_memrealtime); no memory traffic
__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks)
{
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
  }
}

} // namespace

hipError_t streams_run_concurrently(hipStream_t a, hipStream_t b, bool& concurrent)
{
  concurrent         = true;
  constexpr float MS = 0.1f; // each spin: long against a cross-queue event wait (~10-50 us)
  int             device = 0, khz = 0;
  hipError_t      e      = hipGetDevice(&device);
  if (e == hipSuccess) {
    e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
  }
  if (e != hipSuccess || khz <= 0) {
    return e;
  }
  hipEvent_t ev[4] = {};
  for (int i = 0; i < 4 && e == hipSuccess; ++i) {
    e = hipEventCreate(&ev[i]);
  }
  const uint64_t ticks = static_cast<uint64_t>(MS * static_cast<float>(khz));
  if (e == hipSuccess) {
    e = hipEventRecord(ev[0], a); // b starts after a's earlier work, together with a's spin
  }
  if (e == hipSuccess) {
    e = hipStreamWaitEvent(b, ev[0], 0);
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, a, ticks);
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, b, ticks);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    e = hipEventRecord(ev[1], a);
  }
  if (e == hipSuccess) {
    e = hipEventRecord(ev[2], b);
  }
  if (e == hipSuccess) {
    e = hipEventSynchronize(ev[1]);
  }
  if (e == hipSuccess) {
    e = hipEventSynchronize(ev[2]);
  }
  float ta = 0.f, tb = 0.f;
  if (e == hipSuccess) {
    e = hipEventElapsedTime(&ta, ev[0], ev[1]);
  }
  if (e == hipSuccess) {
    e = hipEventElapsedTime(&tb, ev[0], ev[2]);
  }
  if (e == hipSuccess) {
    concurrent = (ta > tb ? ta : tb) < 1.5f * MS;
  }
  for (hipEvent_t x : ev) {
    if (x != nullptr) {
      (void)hipEventDestroy(x);
    }
  }
  return e;
}

} // namespace srs_amd
