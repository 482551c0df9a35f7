// polar_api.cpp -- C-ABI of the MI355X polar chains (include/srsran_amd/polar.h).
// A code object holds the construction (polar_code.cpp) and its device tables,
// like the reference's polar_code it is built once per (K, E, nMax, ibil).
#include "srsran_amd/polar.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "polar_args.h"
#include <cstring>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_polar_code {
  polar_code_desc desc;
  int             device = 0;
  hipStream_t     stream = nullptr;
  void*           d_tables = nullptr;
  polar_args      base{};
  void*           scratch      = nullptr;
  size_t          scratch_size = 0;
  std::mutex      mtx;
  ~srs_amd_polar_code()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(d_tables);
    (void)hipFree(scratch);
  }
};

const polar_args& srs_amd::polar_code_base(const ::srs_amd_polar_code* code)
{
  return code->base;
}

namespace {

template <class T>
size_t append(std::vector<uint8_t>& blob, const std::vector<T>& v)
{
  const size_t off = (blob.size() + 15) / 16 * 16;
  blob.resize(off + v.size() * sizeof(T));
  if (!v.empty()) {
    std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
  }
  return off;
}

hipError_t ensure_scratch(srs_amd_polar_code* c, size_t n)
{
  if (n <= c->scratch_size) {
    return hipSuccess;
  }
  (void)hipFree(c->scratch);
  c->scratch      = nullptr;
  c->scratch_size = 0;
  hipError_t e    = hipMalloc(&c->scratch, n);
  if (e == hipSuccess) {
    c->scratch_size = n;
  }
  return e;
}

} // namespace

extern "C" {

int srs_amd_polar_code_create(srs_amd_polar_code** code, uint32_t K, uint32_t E, uint32_t nMax, int ibil, int device)
{
  if (code == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *code   = nullptr;
  auto* c = new srs_amd_polar_code();
  if (const char* msg = build_polar_code(c->desc, K, E, nMax, ibil != 0)) {
    delete c;
    return fail(SRS_AMD_EINVAL, "%s (K=%u, E=%u, nMax=%u)", msg, K, E, nMax);
  }
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    delete c;
    return rc;
  }
  c->device                = device;
  const polar_code_desc& d = c->desc;
  std::vector<uint8_t>   blob;
  const size_t           o_kset = append(blob, d.K_set);
  const size_t           o_msg  = append(blob, d.msg_pos);
  const size_t           o_tx   = append(blob, d.tx_map);
  const size_t           o_rx   = append(blob, d.rx_e2f);
  const size_t           o_blk  = append(blob, d.blk);
  const size_t           o_prog = append(blob, d.program);
  hipError_t             e      = hipMalloc(&c->d_tables, blob.size());
  if (e == hipSuccess) {
    e = hipMemcpy(c->d_tables, blob.data(), blob.size(), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "polar code tables");
  }
  const uint8_t* t = static_cast<const uint8_t*>(c->d_tables);
  polar_args&    a = c->base;
  a.K              = d.K;
  a.E              = d.E;
  a.N              = d.N;
  a.nPC            = static_cast<uint32_t>(d.PC_set.size());
  a.mode           = static_cast<uint32_t>(d.mode);
  a.prog_len       = static_cast<uint32_t>(d.program.size());
  for (size_t i = 0; i < d.PC_set.size() && i < 4; ++i) {
    a.pc_set[i] = d.PC_set[i];
  }
  a.kset    = t + o_kset;
  a.msg_pos = reinterpret_cast<const uint16_t*>(t + o_msg);
  a.tx_map  = reinterpret_cast<const uint16_t*>(t + o_tx);
  a.rx_e2f  = reinterpret_cast<const uint16_t*>(t + o_rx);
  a.blk     = reinterpret_cast<const uint16_t*>(t + o_blk);
  a.program = reinterpret_cast<const uint32_t*>(t + o_prog);
  *code     = c;
  return SRS_AMD_OK;
}

void srs_amd_polar_code_destroy(srs_amd_polar_code* code)
{
  delete code;
}

uint32_t srs_amd_polar_code_get_N(const srs_amd_polar_code* code)
{
  return code ? code->desc.N : 0;
}

uint32_t srs_amd_polar_code_get_n(const srs_amd_polar_code* code)
{
  return code ? code->desc.n : 0;
}

uint32_t srs_amd_polar_code_get_nPC(const srs_amd_polar_code* code)
{
  return code ? code->desc.nPC : 0;
}

int srs_amd_polar_code_get_K_set(const srs_amd_polar_code* code, uint8_t* mask)
{
  if (code == nullptr || mask == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  std::memcpy(mask, code->desc.K_set.data(), code->desc.N);
  return SRS_AMD_OK;
}

int srs_amd_polar_code_get_PC_set(const srs_amd_polar_code* code, uint16_t* pc_set)
{
  if (code == nullptr || pc_set == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  for (size_t i = 0; i < code->desc.PC_set.size(); ++i) {
    pc_set[i] = code->desc.PC_set[i];
  }
  return SRS_AMD_OK;
}

uint32_t srs_amd_polar_code_construct(uint32_t K, uint32_t E, uint32_t nMax, uint8_t* mask, uint16_t* pc_set,
                                      uint32_t* nPC)
{
  polar_code_desc d;
  if (const char* msg = build_polar_code(d, K, E, nMax, false)) {
    fail(SRS_AMD_EINVAL, "%s (K=%u, E=%u, nMax=%u)", msg, K, E, nMax);
    return 0;
  }
  if (mask) {
    std::memcpy(mask, d.K_set.data(), d.N);
  }
  if (pc_set) {
    for (size_t i = 0; i < d.PC_set.size(); ++i) {
      pc_set[i] = d.PC_set[i];
    }
  }
  if (nPC) {
    *nPC = d.nPC;
  }
  return d.N;
}

int srs_amd_polar_encode_batch(srs_amd_polar_code* code,
                               const uint8_t*      d_messages,
                               uint32_t            msg_stride,
                               uint8_t*            d_output,
                               uint32_t            out_stride,
                               uint32_t            nof,
                               void*               stream)
{
  if (code == nullptr) {
    return fail(SRS_AMD_EINVAL, "null polar code");
  }
  if (nof == 0) {
    return SRS_AMD_OK;
  }
  if (d_messages == nullptr || d_output == nullptr || msg_stride < code->desc.K || out_stride < code->desc.E) {
    return fail(SRS_AMD_EINVAL, "invalid device buffers or strides");
  }
  polar_args a = code->base;
  a.msgs       = d_messages;
  a.cws        = d_output;
  a.msg_stride = msg_stride;
  a.cw_stride  = out_stride;
  a.nof        = nof;
  std::lock_guard<std::mutex> lock(code->mtx);
  hipError_t                  e = hipSetDevice(code->device);
  if (e == hipSuccess) {
    e = launch_polar_encode(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "polar_encode_kernel launch");
}

int srs_amd_polar_decode_batch(srs_amd_polar_code* code,
                               const int8_t*       d_llrs,
                               uint32_t            llr_stride,
                               uint8_t*            d_messages,
                               uint32_t            msg_stride,
                               uint32_t            nof,
                               void*               stream)
{
  if (code == nullptr) {
    return fail(SRS_AMD_EINVAL, "null polar code");
  }
  if (nof == 0) {
    return SRS_AMD_OK;
  }
  if (d_llrs == nullptr || d_messages == nullptr || llr_stride < code->desc.E || msg_stride < code->desc.K) {
    return fail(SRS_AMD_EINVAL, "invalid device buffers or strides");
  }
  polar_args a = code->base;
  a.llrs       = d_llrs;
  a.msgs_out   = d_messages;
  a.llr_stride = llr_stride;
  a.msg_stride = msg_stride;
  a.nof        = nof;
  std::lock_guard<std::mutex> lock(code->mtx);
  hipError_t                  e = hipSetDevice(code->device);
  if (e == hipSuccess) {
    e = launch_polar_decode(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "polar_decode_kernel launch");
}

int srs_amd_polar_encode(srs_amd_polar_code* code, uint8_t* output, const uint8_t* message)
{
  if (code == nullptr || output == nullptr || message == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const uint32_t K = code->desc.K, E = code->desc.E;
  uint8_t*       base = nullptr;
  {
    std::lock_guard<std::mutex> lock(code->mtx);
    hipError_t                  e = hipSetDevice(code->device);
    if (e == hipSuccess) {
      e = ensure_scratch(code, K + E + 64);
    }
    base = static_cast<uint8_t*>(code->scratch);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base, message, K, hipMemcpyHostToDevice, code->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging message");
    }
  }
  int rc = srs_amd_polar_encode_batch(code, base, K, base + K, E, 1, code->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(output, base + K, E, hipMemcpyDeviceToHost, code->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(code->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "polar encode");
}

int srs_amd_polar_decode(srs_amd_polar_code* code, uint8_t* message, const int8_t* llrs)
{
  if (code == nullptr || message == nullptr || llrs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const uint32_t K = code->desc.K, E = code->desc.E;
  uint8_t*       base = nullptr;
  {
    std::lock_guard<std::mutex> lock(code->mtx);
    hipError_t                  e = hipSetDevice(code->device);
    if (e == hipSuccess) {
      e = ensure_scratch(code, K + E + 64);
    }
    base = static_cast<uint8_t*>(code->scratch);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base + K, llrs, E, hipMemcpyHostToDevice, code->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging LLRs");
    }
  }
  int rc = srs_amd_polar_decode_batch(code, reinterpret_cast<const int8_t*>(base + K), E, base, K, 1, code->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(message, base, K, hipMemcpyDeviceToHost, code->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(code->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "polar decode");
}

int srs_amd_polar_interleave(uint8_t* output, const uint8_t* input, uint32_t K, int direction)
{
  if (output == nullptr || input == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (direction != 0 && direction != 1) {
    return fail(SRS_AMD_EINVAL, "invalid interleaver direction %d", direction);
  }
  if (!polar_interleave(output, input, K, direction)) {
    return fail(SRS_AMD_EINVAL, "K (%u) exceeds K_IL_max (164)", K);
  }
  return SRS_AMD_OK;
}

} // extern "C"
