// stream_probe.hip -- host / stream plumbing of the slot forms.
//
// upload_pinned: descriptor uploads from pinned host memory by a copy kernel that reads the host buffer over the
// bus, instead of hipMemcpyAsync.  The SDMA engine that serves small asynchronous host-to-device copies
// occasionally started one ~7 ms late (one sch_slot step in twenty; none with HSA_ENABLE_SDMA=0,
// tools/gpu_r04_sdma.sh), and the blit-kernel fallback costs ~0.1 ms per step; one kernel per upload costs a few us.
//
// streams_run_concurrently: do two HIP streams run concurrently on this device?  HIP maps streams onto
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

// 16 bytes per thread and round; src is the device view of pinned host memory
__global__ __launch_bounds__(256) void pinned_copy_kernel(const uint8_t* src, uint8_t* dst, size_t n)
{
  const size_t step = static_cast<size_t>(gridDim.x) * 256 * 16;
  for (size_t i = (static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x) * 16; i < n; i += step) {
    if (i + 16 <= n) {
      *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
    } else {
      for (size_t k = i; k < n; ++k) {
        dst[k] = src[k];
      }
    }
  }
}

} // namespace

hipError_t upload_pinned(void* d, const void* h, size_t n, hipStream_t s)
{
  if (n == 0) {
    return hipSuccess;
  }
  void*      dh = nullptr;
  hipError_t e  = hipHostGetDevicePointer(&dh, const_cast<void*>(h), 0);
  if (e != hipSuccess || ((reinterpret_cast<uintptr_t>(dh) | reinterpret_cast<uintptr_t>(d)) & 15u) != 0) {
    (void)hipGetLastError();
    return hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s); // not a mapped pinned buffer: the runtime's copy
  }
  const size_t blocks = (n + 256 * 16 - 1) / (256 * 16);
  hipLaunchKernelGGL(pinned_copy_kernel, dim3(blocks < 512 ? blocks : 512), dim3(256), 0, s,
                     static_cast<const uint8_t*>(dh), static_cast<uint8_t*>(d), n);
  return hipGetLastError();
}

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
