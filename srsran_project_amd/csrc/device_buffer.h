// device_buffer.h -- grow-only device scratch allocation used by the C-ABI objects.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace srs_amd {

struct device_buffer {
  void*  ptr  = nullptr;
  size_t size = 0;
  device_buffer() = default;
  device_buffer(const device_buffer&) = delete;
  device_buffer& operator=(const device_buffer&) = delete;
  ~device_buffer() { (void)hipFree(ptr); }
  // Grows to at least n bytes (contents are not preserved).
  hipError_t ensure(size_t n)
  {
    if (n <= size) {
      return hipSuccess;
    }
    (void)hipFree(ptr);
    ptr        = nullptr;
    size       = 0;
    hipError_t e = hipMalloc(&ptr, n);
    if (e == hipSuccess) {
      size = n;
    }
    return e;
  }
  template <typename T>
  T* as() const
  {
    return static_cast<T*>(ptr);
  }
};

// Orders the reuse of an object's device scratch across the caller's streams: a batch call on stream s
// first waits for the previous call's completion event when that call ran on another stream, so two
// calls on different streams never overwrite each other's in-flight scratch.
struct stream_order {
  hipEvent_t  done = nullptr;
  hipStream_t last = nullptr;
  bool        used = false;
  stream_order() = default;
  stream_order(const stream_order&) = delete;
  stream_order& operator=(const stream_order&) = delete;
  ~stream_order()
  {
    if (done) {
      (void)hipEventDestroy(done);
    }
  }
  hipError_t begin(hipStream_t s) const { return (used && s != last) ? hipStreamWaitEvent(s, done, 0) : hipSuccess; }
  hipError_t end(hipStream_t s)
  {
    if (done == nullptr) {
      hipError_t e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
      if (e != hipSuccess) {
        return e;
      }
    }
    last = s;
    used = true;
    return hipEventRecord(done, s);
  }
};

inline size_t align_up(size_t n, size_t a)
{
  return (n + a - 1) / a * a;
}

} // namespace srs_amd
