// traffic_calib.hip -- FETCH_SIZE / WRITE_SIZE calibration in the access forms of the kernels whose HBM traffic the
// bench reports (MI355X_MICROARCH.md: only 16-B-per-lane streaming accesses are calibrated, other widths must be
// calibrated "in your own access pattern").  Each kernel moves a known number of bytes in one form:
//   calib_read8        coalesced 8-byte loads per lane      (the fused LDPC decoder's codeword loads, one 256QAM symbol)
//   calib_read4        coalesced 4-byte loads per lane      (LLR rows read as dwords)
//   calib_read16       coalesced 16-byte loads per lane     (the guide's calibrated form)
//   calib_write16_rows 1,056-byte rows by 66 lanes x 16 B   (the decoder's hard-decision store per codeblock)
//   calib_write4_rows  one 4-byte store per row             (the decoder's iteration count per codeblock)
//   calib_write16      coalesced 16-byte stores             (the guide's calibrated form)
//   calib_write4       coalesced 4-byte stores
// Run once under `rocprofv3 --pmc FETCH_SIZE` and once under `--pmc WRITE_SIZE`; it prints the bytes each kernel
// moves per launch (JSON) for tools/traffic_r05.py.  Sizes: the headline step's 9,024 PUSCH codeblocks.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                                                       \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                                     \
      std::exit(1);                                                                                                    \
    }                                                                                                                  \
  } while (0)

template <typename T>
__device__ __forceinline__ void calib_read(const T* __restrict__ src, size_t n, uint32_t* __restrict__ sink)
{
  uint32_t acc = 0;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
    const T v = src[i];
#pragma unroll
    for (unsigned k = 0; k < sizeof(T) / 4; ++k) {
      acc ^= reinterpret_cast<const uint32_t*>(&v)[k] + k; // every word of the access used: full-width loads
    }
  }
  if (acc == 0x9e3779b9u) { // never true for the zero-filled input: keeps the loads, writes nothing
    sink[blockIdx.x] = acc;
  }
}

__global__ __launch_bounds__(256) void calib_read8(const uint2* src, size_t n, uint32_t* sink) { calib_read<uint2>(src, n, sink); }
__global__ __launch_bounds__(256) void calib_read4(const uint32_t* src, size_t n, uint32_t* sink) { calib_read<uint32_t>(src, n, sink); }
__global__ __launch_bounds__(256) void calib_read16(const uint4* src, size_t n, uint32_t* sink) { calib_read<uint4>(src, n, sink); }

// one workgroup of 192 threads per row (the decoder's three waves per codeblock): lanes 0..65 store 16 B each
__global__ __launch_bounds__(192) void calib_write16_rows(uint4* dst, uint32_t row_words)
{
  if (threadIdx.x < row_words) {
    dst[static_cast<size_t>(blockIdx.x) * row_words + threadIdx.x] = make_uint4(blockIdx.x, threadIdx.x, 1u, 2u);
  }
}

__global__ __launch_bounds__(192) void calib_write4_rows(uint32_t* dst)
{
  if (threadIdx.x == 0) {
    dst[blockIdx.x] = blockIdx.x;
  }
}

template <typename T>
__device__ void calib_write(T* dst, size_t n)
{
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
    T v{};
#pragma unroll
    for (unsigned k = 0; k < sizeof(T) / 4; ++k) {
      reinterpret_cast<uint32_t*>(&v)[k] = static_cast<uint32_t>(i) * 4 + k + 1; // no zero word: full-width stores
    }
    dst[i] = v;
  }
}

__global__ __launch_bounds__(256) void calib_write16(uint4* dst, size_t n) { calib_write<uint4>(dst, n); }
__global__ __launch_bounds__(256) void calib_write4(uint32_t* dst, size_t n) { calib_write<uint32_t>(dst, n); }

int main()
{
  constexpr uint32_t CBS      = 9024;          // codeblocks of the headline step
  constexpr size_t   RD_BYTES = 9024ull * 9216; // 83 MB: the decoder's read volume
  constexpr uint32_t ROW      = 1056;          // message bytes per codeblock (8,448 bits)
  constexpr int      REPS     = 3;
  void *             src = nullptr, *dst = nullptr;
  uint32_t*          sink = nullptr;
  CHECK(hipMalloc(&src, RD_BYTES));
  CHECK(hipMalloc(&dst, RD_BYTES));
  CHECK(hipMalloc(&sink, 65536 * sizeof(uint32_t)));
  CHECK(hipMemset(src, 0, RD_BYTES));
  CHECK(hipDeviceSynchronize());
  const int grid = 2048;
  for (int r = 0; r < REPS; ++r) {
    hipLaunchKernelGGL(calib_read8, dim3(grid), dim3(256), 0, nullptr, static_cast<const uint2*>(src), RD_BYTES / 8, sink);
    hipLaunchKernelGGL(calib_read4, dim3(grid), dim3(256), 0, nullptr, static_cast<const uint32_t*>(src), RD_BYTES / 4,
                       sink);
    hipLaunchKernelGGL(calib_read16, dim3(grid), dim3(256), 0, nullptr, static_cast<const uint4*>(src), RD_BYTES / 16,
                       sink);
    hipLaunchKernelGGL(calib_write16_rows, dim3(CBS), dim3(192), 0, nullptr, static_cast<uint4*>(dst), ROW / 16);
    hipLaunchKernelGGL(calib_write4_rows, dim3(CBS), dim3(192), 0, nullptr, static_cast<uint32_t*>(dst));
    hipLaunchKernelGGL(calib_write16, dim3(grid), dim3(256), 0, nullptr, static_cast<uint4*>(dst), RD_BYTES / 16);
    hipLaunchKernelGGL(calib_write4, dim3(grid), dim3(256), 0, nullptr, static_cast<uint32_t*>(dst), RD_BYTES / 4);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
  }
  std::printf("{\"calib_read8\": {\"read\": %zu}, \"calib_read4\": {\"read\": %zu}, \"calib_read16\": {\"read\": %zu}, "
              "\"calib_write16_rows\": {\"write\": %zu}, \"calib_write4_rows\": {\"write\": %zu}, "
              "\"calib_write16\": {\"write\": %zu}, \"calib_write4\": {\"write\": %zu}, \"reps\": %d}\n",
              RD_BYTES, RD_BYTES, RD_BYTES, static_cast<size_t>(CBS) * ROW, static_cast<size_t>(CBS) * 4, RD_BYTES,
              RD_BYTES, REPS);
  CHECK(hipFree(src));
  CHECK(hipFree(dst));
  CHECK(hipFree(sink));
  return 0;
}
