// hip_accelerator_pusch_dec.cpp -- hal::hw_accelerator_pusch_dec over the srsran_amd C-ABI (see the header).
#include "hip_accelerator_pusch_dec.h"

#include "srsran/ran/sch/modulation_scheme.h"
#include "srsran_amd/crc.h"
#include "srsran_amd/ldpc.h"
#include "srsran_amd/ldpc_rate_matching.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

using namespace srsran;
using namespace srsran::hip;

namespace {

constexpr unsigned MAX_CBS  = 512;         // codeblocks of one transport block (pdsch_constants / MAX_NOF_SEGMENTS)
constexpr unsigned ROW      = 66 * 384;    // HARQ row: the longest codeblock (BG1, Z = 384), 64-byte multiple
constexpr unsigned MSG_ROW  = 22 * 384 / 8; // packed message row (BG1, Z = 384)

[[noreturn]] void fatal(const char* what, const char* detail)
{
  std::fprintf(stderr, "hip_accelerator_pusch_dec: %s: %s\n", what, detail);
  std::abort();
}

void check_hip(hipError_t e, const char* what)
{
  if (e != hipSuccess) {
    fatal(what, hipGetErrorString(e));
  }
}

void check_amd(int rc, const char* what)
{
  if (rc != SRS_AMD_OK) {
    fatal(what, srs_amd_last_error());
  }
}

// hal::hw_dec_cb_crc_type -> crc_generator_poly value of the C-ABI (CRC24A = 0, CRC24B = 1, CRC16 = 3).
int crc_poly(hal::hw_dec_cb_crc_type t)
{
  switch (t) {
    case hal::hw_dec_cb_crc_type::CRC24A:
      return 0;
    case hal::hw_dec_cb_crc_type::CRC24B:
      return 1;
    default:
      return 3;
  }
}

/// HARQ soft buffers in HBM, shared by every accelerator instance of one factory (the role of the
/// reference's ext_harq_buffer_context_repository): rows keyed by the absolute codeblock id; the rows of a
/// transport block are allocated contiguously (index = first row + codeblock index) so a transport block is
/// one batch.
class harq_pool
{
public:
  harq_pool(int device, unsigned nof_rows) : device(device), used(nof_rows, 0)
  {
    check_hip(hipSetDevice(device), "hipSetDevice");
    check_hip(hipMalloc(&rows, static_cast<size_t>(nof_rows) * ROW), "HARQ buffer allocation");
  }
  ~harq_pool() { (void)hipFree(rows); }

  int8_t* row(unsigned r) const { return rows + static_cast<size_t>(r) * ROW; }

  /// Row of (absolute id, codeblock index) of a transport block of nof_cbs codeblocks; base carries the
  /// transport block's first row between calls (UINT32_MAX: not known yet). is_new: the row was just allocated.
  unsigned lookup(unsigned abs_id, unsigned cb, unsigned nof_cbs, unsigned& base, bool& is_new)
  {
    std::lock_guard<std::mutex> lock(mtx);
    auto                        it = row_of.find(abs_id);
    is_new                         = it == row_of.end();
    if (!is_new) {
      if (base == UINT32_MAX) {
        if (it->second < cb) {
          fatal("HARQ", "inconsistent codeblock index");
        }
        base = it->second - cb;
      } else if (it->second != base + cb) {
        fatal("HARQ", "codeblocks of one transport block in non-contiguous rows");
      }
      return it->second;
    }
    if (base == UINT32_MAX) {
      base = find_free(nof_cbs);
    }
    const unsigned r = base + cb;
    if (r >= used.size() || used[r]) {
      fatal("HARQ", "no free row for the codeblock");
    }
    used[r]        = 1;
    row_of[abs_id] = r;
    return r;
  }

  void release(unsigned abs_id)
  {
    std::lock_guard<std::mutex> lock(mtx);
    auto                        it = row_of.find(abs_id);
    if (it != row_of.end()) {
      used[it->second] = 0;
      row_of.erase(it);
    }
  }

private:
  unsigned find_free(unsigned n) const
  {
    for (unsigned b = 0; b + n <= used.size(); ++b) {
      bool ok = true;
      for (unsigned k = 0; k != n && ok; ++k) {
        ok = used[b + k] == 0;
      }
      if (ok) {
        return b;
      }
    }
    fatal("HARQ", "HARQ buffer full");
  }

  int                                    device;
  int8_t*                                rows = nullptr;
  std::vector<char>                      used;
  std::unordered_map<unsigned, unsigned> row_of;
  std::mutex                             mtx;
};

class hip_accelerator_pusch_dec : public hal::hw_accelerator_pusch_dec
{
public:
  hip_accelerator_pusch_dec(const pusch_dec_accelerator_config& c, std::shared_ptr<harq_pool> harq_) :
    device(c.device), harq(std::move(harq_))
  {
    if (device < 0) {
      check_hip(hipGetDevice(&device), "hipGetDevice");
    }
    check_hip(hipSetDevice(device), "hipSetDevice");
    check_hip(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream");
    check_amd(srs_amd_ldpc_rate_dematcher_create(&dm, device), "rate dematcher");
    check_amd(srs_amd_ldpc_decoder_create(&dec, c.arith, 0, device), "LDPC decoder");
    for (int p = 0; p != 4; ++p) {
      check_amd(srs_amd_crc_calculator_create(&crc[p], p == 2 ? 3 : p, 8448, device), "CRC");
    }
    check_hip(hipHostMalloc(&h_arrays, sizeof(uint32_t) * 2 * MAX_CBS, hipHostMallocDefault), "pinned arrays");
    check_hip(hipHostMalloc(&h_msgs, static_cast<size_t>(MAX_CBS) * MSG_ROW, hipHostMallocDefault), "pinned msgs");
    check_hip(hipHostMalloc(&h_iters, sizeof(int32_t) * MAX_CBS, hipHostMallocDefault), "pinned iterations");
    check_hip(hipMalloc(&d_arrays, sizeof(uint32_t) * 2 * MAX_CBS), "arrays");
    check_hip(hipMalloc(&d_msgs, static_cast<size_t>(MAX_CBS) * MSG_ROW), "messages");
    check_hip(hipMalloc(&d_iters, sizeof(int32_t) * MAX_CBS), "iterations");
    grow_staging(1 << 20);
    reserve_queue();
  }

  ~hip_accelerator_pusch_dec() override
  {
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    (void)hipStreamDestroy(stream);
    srs_amd_ldpc_rate_dematcher_destroy(dm);
    srs_amd_ldpc_decoder_destroy(dec);
    for (auto* c : crc) {
      srs_amd_crc_calculator_destroy(c);
    }
    (void)hipHostFree(h_arrays);
    (void)hipHostFree(h_msgs);
    (void)hipHostFree(h_iters);
    (void)hipHostFree(h_llrs);
    (void)hipFree(d_arrays);
    (void)hipFree(d_msgs);
    (void)hipFree(d_iters);
    (void)hipFree(d_llrs);
  }

  // One transport block between reserve_queue() and the last dequeue (pusch_decoder_hw_impl.cpp:170-360).
  void reserve_queue() override
  {
    std::fill(std::begin(enqueued), std::end(enqueued), false);
    tb_base  = UINT32_MAX;
    nof_cbs  = 0;
    staged   = 0;
    flushed  = false;
    new_rows.clear();
  }

  void free_queue() override {}

  void configure_operation(const hal::hw_pusch_decoder_configuration& config, unsigned cb_index) override
  {
    if (cb_index >= MAX_CBS || config.nof_segments > MAX_CBS) {
      fatal("configure_operation", "too many codeblocks");
    }
    if (flushed) {
      reserve_queue(); // the driver moved on to another transport block without a new reservation
    }
    cfg[cb_index] = config;
    nof_cbs       = config.nof_segments;
    bool           is_new;
    const unsigned r = harq->lookup(config.absolute_cb_id, cb_index, nof_cbs, tb_base, is_new);
    (void)r;
    if (is_new) {
      new_rows.push_back(cb_index);
    }
  }

  bool enqueue_operation(span<const int8_t> data, span<const int8_t> /*aux*/, unsigned cb_index) override
  {
    if (cb_index >= MAX_CBS || flushed) {
      return false;
    }
    const size_t off = (staged + 63) / 64 * 64;
    grow_staging(off + data.size());
    std::memcpy(h_llrs + off, data.data(), data.size());
    offsets[cb_index]  = static_cast<uint32_t>(off);
    lengths[cb_index]  = static_cast<uint32_t>(data.size());
    enqueued[cb_index] = true;
    staged             = off + data.size();
    return true;
  }

  bool dequeue_operation(span<uint8_t> data, span<int8_t> /*aux*/, unsigned cb_index) override
  {
    if (cb_index >= MAX_CBS || !enqueued[cb_index]) {
      return false;
    }
    if (!flushed) {
      flush();
    }
    std::memcpy(data.data(), h_msgs + static_cast<size_t>(cb_index) * MSG_ROW,
                std::min<size_t>(data.size(), MSG_ROW));
    return true;
  }

  void read_operation_outputs(hal::hw_pusch_decoder_outputs& out, unsigned cb_index, unsigned /*abs_id*/) override
  {
    const hal::hw_pusch_decoder_configuration& c = cfg[cb_index];
    const int32_t                              it = h_iters[cb_index];
    if (c.use_early_stop) {
      // the decoder stopped on the codeblock CRC (ldpc_decoder_impl.cpp:125): iterations >= 1 <=> CRC pass
      out.CRC_pass            = it >= 0;
      out.nof_ldpc_iterations = it >= 0 ? static_cast<unsigned>(it) : c.max_nof_ldpc_iterations;
      return;
    }
    // no early stop: check the codeblock CRC of the decoded message on the host
    const unsigned K    = (c.base_graph_index == ldpc_base_graph_type::BG1 ? 22 : 10) * c.lifting_size;
    uint32_t       chk  = 1;
    const int      poly = crc_poly(c.cb_crc_type);
    check_amd(srs_amd_crc_calculate(crc[poly == 3 ? 2 : poly], &chk, h_msgs + static_cast<size_t>(cb_index) * MSG_ROW,
                                    K - c.nof_filler_bits),
              "CRC");
    out.CRC_pass            = chk == 0;
    out.nof_ldpc_iterations = c.max_nof_ldpc_iterations;
  }

  void free_harq_context_entry(unsigned absolute_cb_id) override { harq->release(absolute_cb_id); }

  bool is_harq_external() const override { return true; }

private:
  void grow_staging(size_t n)
  {
    if (n <= staging_cap) {
      return;
    }
    const size_t cap = std::max(n, 2 * staging_cap);
    int8_t*      h   = nullptr;
    check_hip(hipHostMalloc(&h, cap, hipHostMallocDefault), "pinned staging");
    if (h_llrs != nullptr) {
      std::memcpy(h, h_llrs, staged);
      (void)hipHostFree(h_llrs);
    }
    h_llrs = h;
    (void)hipFree(d_llrs);
    check_hip(hipMalloc(&d_llrs, cap), "LLR staging");
    staging_cap = cap;
  }

  // The transport block's enqueued codeblocks as one batch per contiguous run of codeblock indices.
  void flush()
  {
    flushed = true;
    check_hip(hipSetDevice(device), "hipSetDevice");
    for (unsigned r = 0; r != nof_cbs; ++r) {
      h_arrays[r]           = enqueued[r] ? offsets[r] : 0;
      h_arrays[MAX_CBS + r] = enqueued[r] ? lengths[r] : 0;
    }
    check_hip(hipMemcpyAsync(d_llrs, h_llrs, staged, hipMemcpyHostToDevice, stream), "H2D LLRs");
    check_hip(hipMemcpyAsync(d_arrays, h_arrays, sizeof(uint32_t) * 2 * MAX_CBS, hipMemcpyHostToDevice, stream),
              "H2D arrays");
    // freshly allocated HARQ rows start as a cleared rx_buffer
    for (unsigned r : new_rows) {
      check_hip(hipMemsetAsync(harq->row(tb_base + r), 0, ROW, stream), "HARQ row reset");
    }
    for (unsigned a = 0; a < nof_cbs;) {
      if (!enqueued[a]) {
        ++a;
        continue;
      }
      unsigned b = a;
      while (b < nof_cbs && enqueued[b]) {
        ++b;
      }
      run(a, b - a);
      a = b;
    }
    check_hip(hipMemcpyAsync(h_msgs, d_msgs, static_cast<size_t>(nof_cbs) * MSG_ROW, hipMemcpyDeviceToHost, stream),
              "D2H messages");
    check_hip(hipMemcpyAsync(h_iters, d_iters, sizeof(int32_t) * nof_cbs, hipMemcpyDeviceToHost, stream),
              "D2H iterations");
    check_hip(hipStreamSynchronize(stream), "decode");
  }

  void run(unsigned first, unsigned n)
  {
    const hal::hw_pusch_decoder_configuration& c  = cfg[first];
    const unsigned                             bg = c.base_graph_index == ldpc_base_graph_type::BG1 ? 1 : 2;
    const unsigned                             Z  = c.lifting_size;
    // rate dematching + HARQ combining into the HARQ rows (ldpc_rate_dematcher::rate_dematch)
    srs_amd_codeblock_metadata md{bg, Z, c.rv, get_bits_per_symbol(c.modulation), c.Nref, c.nof_filler_bits};
    check_amd(srs_amd_ldpc_rate_dematch_batch(dm, &md, c.new_data ? 1 : 0, d_llrs, d_arrays + first,
                                              d_arrays + MAX_CBS + first, harq->row(tb_base + first), ROW, n, stream),
              "rate dematching");
    // LDPC decoding with the codeblock CRC as early stop (pusch_codeblock_decoder.cpp:35-69)
    srs_amd_ldpc_decoder_config dc{bg, Z, c.nof_filler_bits, c.cb_crc_len, c.max_nof_ldpc_iterations};
    const unsigned              N = (bg == 1 ? 66 : 50) * Z;
    check_amd(srs_amd_ldpc_decode_batch(dec, &dc, c.use_early_stop ? crc_poly(c.cb_crc_type) : SRS_AMD_NO_CRC,
                                        harq->row(tb_base + first), ROW, nullptr, N,
                                        d_msgs + static_cast<size_t>(first) * MSG_ROW, MSG_ROW, d_iters + first,
                                        nullptr, n, stream),
              "LDPC decoding");
  }

  int                                 device;
  std::shared_ptr<harq_pool>          harq;
  hipStream_t                         stream = nullptr;
  srs_amd_ldpc_rate_dematcher*        dm     = nullptr;
  srs_amd_ldpc_decoder*               dec    = nullptr;
  srs_amd_crc_calculator*             crc[4] = {};  // CRC24A, CRC24B, CRC16 (index 2), spare
  hal::hw_pusch_decoder_configuration cfg[MAX_CBS] = {};
  bool                                enqueued[MAX_CBS] = {};
  uint32_t                            offsets[MAX_CBS]  = {};
  uint32_t                            lengths[MAX_CBS]  = {};
  std::vector<unsigned>               new_rows;
  unsigned                            tb_base = UINT32_MAX, nof_cbs = 0;
  size_t                              staged = 0, staging_cap = 0;
  bool                                flushed = false;
  int8_t*                             h_llrs  = nullptr;
  int8_t*                             d_llrs  = nullptr;
  uint32_t*                           h_arrays = nullptr;
  uint32_t*                           d_arrays = nullptr;
  uint8_t*                            h_msgs   = nullptr;
  uint8_t*                            d_msgs   = nullptr;
  int32_t*                            h_iters  = nullptr;
  int32_t*                            d_iters  = nullptr;
};

class hip_pusch_dec_acc_factory : public hal::hw_accelerator_pusch_dec_factory
{
public:
  explicit hip_pusch_dec_acc_factory(const pusch_dec_accelerator_config& c) : cfg(c)
  {
    if (cfg.device < 0) {
      check_hip(hipGetDevice(&cfg.device), "hipGetDevice");
    }
    harq = std::make_shared<harq_pool>(cfg.device, cfg.max_harq_rows);
  }
  std::unique_ptr<hal::hw_accelerator_pusch_dec> create() override
  {
    return std::make_unique<hip_accelerator_pusch_dec>(cfg, harq);
  }

private:
  pusch_dec_accelerator_config cfg;
  std::shared_ptr<harq_pool>   harq;
};

} // namespace

std::shared_ptr<hal::hw_accelerator_pusch_dec_factory>
srsran::hip::create_hip_pusch_dec_acc_factory(const pusch_dec_accelerator_config& cfg)
{
  return std::make_shared<hip_pusch_dec_acc_factory>(cfg);
}
