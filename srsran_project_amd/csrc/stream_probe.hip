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

// one wave that waits `ticks` of the constant-rate wall clock (s_memrealtime) and stamps its start and end into
// stamp[0..1] (vector stores by lane 0)
__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks, uint64_t* stamp)
{
  const uint64_t t0 = wall_clock64();
  uint64_t       t1 = t0;
  while (t1 - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    t1 = wall_clock64();
  }
  if (threadIdx.x == 0) {
    stamp[0] = t0;
    stamp[1] = t1;
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
  // Two spin kernels, one per stream, b's released by an event recorded on a just before a's spin: they overlap in
  // time exactly when the streams run concurrently.  The overlap is read from the kernels' own wall-clock stamps,
  // so neither the cross-queue event latency (~10-50 us) nor other work on the device enters the verdict.
  concurrent         = true;
  constexpr float MS = 0.2f;
  int             device = 0, khz = 0;
  hipError_t      e      = hipGetDevice(&device);
  if (e == hipSuccess) {
    e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
  }
  if (e != hipSuccess || khz <= 0) {
    return e;
  }
  uint64_t*  d_stamp = nullptr;
  hipEvent_t ev      = nullptr;
  e                  = hipMalloc(&d_stamp, 4 * sizeof(uint64_t));
  if (e == hipSuccess) {
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  }
  const uint64_t ticks = static_cast<uint64_t>(MS * static_cast<float>(khz));
  if (e == hipSuccess) {
    e = hipEventRecord(ev, a); // b starts after a's earlier work, together with a's spin
  }
  if (e == hipSuccess) {
    e = hipStreamWaitEvent(b, ev, 0);
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, a, ticks, d_stamp);
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, b, ticks, d_stamp + 2);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(a);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(b);
  }
  uint64_t h[4] = {};
  if (e == hipSuccess) {
    e = hipMemcpy(h, d_stamp, sizeof(h), hipMemcpyDeviceToHost);
  }
  if (e == hipSuccess) {
    concurrent = h[2] < h[1] && h[0] < h[3]; // the two spins' [start, end) intervals intersect
  }
  if (ev != nullptr) {
    (void)hipEventDestroy(ev);
  }
  (void)hipFree(d_stamp);
  return e;
}

} // namespace srs_amd
