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

inline size_t align_up(size_t n, size_t a)
{
  return (n + a - 1) / a * a;
}

} // namespace srs_amd
