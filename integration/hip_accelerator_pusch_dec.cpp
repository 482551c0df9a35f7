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
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

using namespace srsran;
using namespace srsran::hip;

namespace {

constexpr unsigned MAX_CBS  = 512;         // codeblocks of one transport block (pdsch_constants / MAX_NOF_SEGMENTS)
constexpr unsigned ROW      = 66 * 384;    // HARQ row: the longest codeblock (BG1, Z = 384), 64-byte multiple
constexpr unsigned MSG_ROW  = 22 * 384 / 8; // packed message row (BG1, Z = 384)

// Errors never abort the gNB: they are logged, and the transport block being decoded reports every
// codeblock as failed (CRC not passed), which the reference's pusch_decoder_hw_impl treats as a decoding
// failure (HARQ retransmission).  Construction errors throw.
void log_error(const char* what, const char* detail)
{
  std::fprintf(stderr, "hip_accelerator_pusch_dec: %s: %s\n", what, detail);
}

void require_hip(hipError_t e, const char* what)
{
  if (e != hipSuccess) {
    log_error(what, hipGetErrorString(e));
    throw std::runtime_error(std::string("hip_accelerator_pusch_dec: ") + what);
  }
}

void require_amd(int rc, const char* what)
{
  if (rc != SRS_AMD_OK) {
    log_error(what, srs_amd_last_error());
    throw std::runtime_error(std::string("hip_accelerator_pusch_dec: ") + what);
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
/// reference's ext_harq_buffer_context_repository): rows keyed by the absolute codeblock id.  The rows of a
/// transport block are contiguous (row = first row + codeblock index) so a transport block is one batch:
/// the first codeblock of a transport block that has no rows yet reserves all nof_cbs rows at once, under
/// the mutex, so concurrent decoder instances never take rows of each other's transport blocks.
/// New data overwrites: an absolute id that still maps to a row from an earlier, abandoned HARQ process (the
/// reference frees entries only on a TB CRC pass) is remapped, its old row returned to the pool.
class harq_pool
{
public:
  harq_pool(int device, unsigned nof_rows) : used(nof_rows, 0)
  {
    require_hip(hipSetDevice(device), "hipSetDevice");
    require_hip(hipMalloc(&rows, static_cast<size_t>(nof_rows) * ROW), "HARQ buffer allocation");
  }
  ~harq_pool() { (void)hipFree(rows); }

  int8_t* row(unsigned r) const { return rows + static_cast<size_t>(r) * ROW; }

  /// Row of (absolute id, codeblock index) of a transport block of nof_cbs codeblocks; base carries the
  /// transport block's first row between the calls of one transport block (UINT32_MAX: not known yet).
  /// fresh: the row holds nothing of this codeblock yet (clear it).  Returns false when no rows are left or
  /// the rows of a retransmission are not contiguous any more.
  bool lookup(unsigned abs_id, unsigned cb, unsigned nof_cbs, bool new_data, unsigned& base, bool& fresh)
  {
    std::lock_guard<std::mutex> lock(mtx);
    auto                        it = row_of.find(abs_id);
    if (it != row_of.end() && new_data && (base == UINT32_MAX || it->second != base + cb)) {
      // stale entry of an abandoned HARQ process
      used[it->second] = 0;
      row_of.erase(it);
      it = row_of.end();
    }
    if (it != row_of.end()) {
      fresh = new_data; // new data on the transport block's own row: cleared like a fresh one
      if (base == UINT32_MAX) {
        if (it->second < cb) {
          return false;
        }
        base = it->second - cb;
      }
      return it->second == base + cb;
    }
    fresh = true;
    if (base == UINT32_MAX) {
      // reserve the whole transport block's rows
      if (!find_free(nof_cbs, base)) {
        return false;
      }
      for (unsigned k = 0; k != nof_cbs; ++k) {
        used[base + k] = 1;
      }
    } else if (base + cb >= used.size()) {
      return false;
    } else {
      used[base + cb] = 1; // already reserved with the transport block, or a row it released
    }
    row_of[abs_id] = base + cb;
    return true;
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
  // next fit from the cursor: O(1) amortised while the pool is not fragmented
  bool find_free(unsigned n, unsigned& base)
  {
    const unsigned total = static_cast<unsigned>(used.size());
    if (n == 0 || n > total) {
      return false;
    }
    for (unsigned scanned = 0, b = cursor; scanned < total;) {
      if (b + n > total) {
        scanned += total - b;
        b = 0;
        continue;
      }
      unsigned k = 0;
      while (k != n && used[b + k] == 0) {
        ++k;
      }
      if (k == n) {
        base   = b;
        cursor = b + n == total ? 0 : b + n;
        return true;
      }
      scanned += k + 1;
      b += k + 1;
    }
    return false;
  }

  int8_t*                                rows   = nullptr;
  unsigned                               cursor = 0;
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
      require_hip(hipGetDevice(&device), "hipGetDevice");
    }
    require_hip(hipSetDevice(device), "hipSetDevice");
    require_hip(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream");
    require_amd(srs_amd_ldpc_rate_dematcher_create(&dm, device), "rate dematcher");
    require_amd(srs_amd_ldpc_decoder_create(&dec, c.arith, 0, device), "LDPC decoder");
    for (int p = 0; p != 4; ++p) {
      require_amd(srs_amd_crc_calculator_create(&crc[p], p == 2 ? 3 : p, 8448, device), "CRC");
    }
    require_hip(hipHostMalloc(&h_arrays, sizeof(uint32_t) * 2 * MAX_CBS, hipHostMallocDefault), "pinned arrays");
    require_hip(hipHostMalloc(&h_msgs, static_cast<size_t>(MAX_CBS) * MSG_ROW, hipHostMallocDefault), "pinned msgs");
    require_hip(hipHostMalloc(&h_iters, sizeof(int32_t) * MAX_CBS, hipHostMallocDefault), "pinned iterations");
    require_hip(hipMalloc(&d_arrays, sizeof(uint32_t) * 2 * MAX_CBS), "arrays");
    require_hip(hipMalloc(&d_msgs, static_cast<size_t>(MAX_CBS) * MSG_ROW), "messages");
    require_hip(hipMalloc(&d_iters, sizeof(int32_t) * MAX_CBS), "iterations");
    if (!grow_staging(1 << 20)) {
      throw std::runtime_error("hip_accelerator_pusch_dec: LLR staging");
    }
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
    tb_base = UINT32_MAX;
    nof_cbs = 0;
    staged  = 0;
    flushed = false;
    failed  = false;
    new_rows.clear();
  }

  void free_queue() override {}

  void configure_operation(const hal::hw_pusch_decoder_configuration& config, unsigned cb_index) override
  {
    if (flushed) {
      reserve_queue(); // the driver moved on to another transport block without a new reservation
    }
    if (cb_index >= MAX_CBS || config.nof_segments > MAX_CBS) {
      fail("configure_operation", "too many codeblocks");
      return;
    }
    cfg[cb_index]     = config;
    abs_ids[cb_index] = config.absolute_cb_id;
    nof_cbs           = config.nof_segments;
    bool fresh    = false;
    if (!failed && !harq->lookup(config.absolute_cb_id, cb_index, nof_cbs, config.new_data, tb_base, fresh)) {
      fail("HARQ", "no contiguous HARQ rows left for the transport block");
      return;
    }
    if (fresh) {
      new_rows.push_back(cb_index);
    }
  }

  // Always accepts the codeblock (the reference's driver retries a refused enqueue forever): a failed
  // transport block is reported through read_operation_outputs.
  bool enqueue_operation(span<const int8_t> data, span<const int8_t> /*aux*/, unsigned cb_index) override
  {
    if (cb_index >= MAX_CBS) {
      return true; // configure_operation marked the transport block failed: reported as CRC failures
    }
    if (flushed) {
      return false;
    }
    const size_t off = (staged + 63) / 64 * 64;
    if (!failed && grow_staging(off + data.size())) {
      std::memcpy(h_llrs + off, data.data(), data.size());
      staged = off + data.size();
    }
    offsets[cb_index]  = static_cast<uint32_t>(off);
    lengths[cb_index]  = static_cast<uint32_t>(data.size());
    enqueued[cb_index] = true;
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
    if (cb_index >= MAX_CBS || failed) {
      out.CRC_pass            = false;
      out.nof_ldpc_iterations = cb_index < MAX_CBS ? cfg[cb_index].max_nof_ldpc_iterations : 0;
      return;
    }
    const hal::hw_pusch_decoder_configuration& c  = cfg[cb_index];
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
    if (srs_amd_crc_calculate(crc[poly == 3 ? 2 : poly], &chk, h_msgs + static_cast<size_t>(cb_index) * MSG_ROW,
                              K - c.nof_filler_bits) != SRS_AMD_OK) {
      log_error("CRC", srs_amd_last_error());
      chk = 1;
    }
    out.CRC_pass            = chk == 0;
    out.nof_ldpc_iterations = c.max_nof_ldpc_iterations;
  }

  void free_harq_context_entry(unsigned absolute_cb_id) override { harq->release(absolute_cb_id); }

  bool is_harq_external() const override { return true; }

private:
  void fail(const char* what, const char* detail)
  {
    if (!failed) {
      log_error(what, detail);
    }
    failed = true;
  }
  bool hip_ok(hipError_t e, const char* what)
  {
    if (e != hipSuccess) {
      fail(what, hipGetErrorString(e));
    }
    return e == hipSuccess;
  }
  bool amd_ok(int rc, const char* what)
  {
    if (rc != SRS_AMD_OK) {
      fail(what, srs_amd_last_error());
    }
    return rc == SRS_AMD_OK;
  }

  // Returns the rows this transport block mapped fresh to the pool (their reset never ran).
  void unmap_new_rows()
  {
    for (unsigned r : new_rows) {
      harq->release(abs_ids[r]);
    }
    new_rows.clear();
  }

  bool grow_staging(size_t n)
  {
    if (n <= staging_cap) {
      return true;
    }
    const size_t cap = std::max(n, 2 * staging_cap);
    int8_t*      h   = nullptr;
    int8_t*      d   = nullptr;
    if (!hip_ok(hipHostMalloc(&h, cap, hipHostMallocDefault), "pinned staging")) {
      return false;
    }
    if (!hip_ok(hipMalloc(&d, cap), "LLR staging")) {
      (void)hipHostFree(h);
      return false;
    }
    if (h_llrs != nullptr) {
      std::memcpy(h, h_llrs, staged);
      (void)hipHostFree(h_llrs);
    }
    (void)hipFree(d_llrs);
    h_llrs      = h;
    d_llrs      = d;
    staging_cap = cap;
    return true;
  }

  // The transport block's enqueued codeblocks as one batch per contiguous run of codeblock indices, one
  // stream synchronisation per transport block (several decoder instances of the factory's pool run their
  // transport blocks concurrently, each on its own stream).
  void flush()
  {
    flushed = true;
    if (failed || !hip_ok(hipSetDevice(device), "hipSetDevice")) {
      unmap_new_rows();
      return;
    }
    for (unsigned r = 0; r != nof_cbs; ++r) {
      h_arrays[r]           = enqueued[r] ? offsets[r] : 0;
      h_arrays[MAX_CBS + r] = enqueued[r] ? lengths[r] : 0;
    }
    bool ok = hip_ok(hipMemcpyAsync(d_llrs, h_llrs, staged, hipMemcpyHostToDevice, stream), "H2D LLRs") &&
              hip_ok(hipMemcpyAsync(d_arrays, h_arrays, sizeof(uint32_t) * 2 * MAX_CBS, hipMemcpyHostToDevice, stream),
                     "H2D arrays");
    // freshly mapped HARQ rows start as a cleared rx_buffer; rows whose reset was not issued are unmapped (a
    // retransmission must not combine onto a previous occupant's soft bits)
    bool cleared = ok;
    for (unsigned r : new_rows) {
      cleared = cleared && hip_ok(hipMemsetAsync(harq->row(tb_base + r), 0, ROW, stream), "HARQ row reset");
    }
    if (!cleared) {
      unmap_new_rows();
    }
    ok = ok && cleared;
    for (unsigned a = 0; ok && a < nof_cbs;) {
      if (!enqueued[a]) {
        ++a;
        continue;
      }
      unsigned b = a;
      while (b < nof_cbs && enqueued[b]) {
        ++b;
      }
      ok = run(a, b - a);
      a  = b;
    }
    ok = ok && hip_ok(hipMemcpyAsync(h_msgs, d_msgs, static_cast<size_t>(nof_cbs) * MSG_ROW, hipMemcpyDeviceToHost,
                                     stream),
                      "D2H messages");
    ok = ok && hip_ok(hipMemcpyAsync(h_iters, d_iters, sizeof(int32_t) * nof_cbs, hipMemcpyDeviceToHost, stream),
                      "D2H iterations");
    // always drain the stream, also after a failed enqueue of work
    ok = hip_ok(hipStreamSynchronize(stream), "decode") && ok;
  }

  bool run(unsigned first, unsigned n)
  {
    const hal::hw_pusch_decoder_configuration& c  = cfg[first];
    const unsigned                             bg = c.base_graph_index == ldpc_base_graph_type::BG1 ? 1 : 2;
    const unsigned                             Z  = c.lifting_size;
    // rate dematching + HARQ combining into the HARQ rows (ldpc_rate_dematcher::rate_dematch)
    srs_amd_codeblock_metadata md{bg, Z, c.rv, get_bits_per_symbol(c.modulation), c.Nref, c.nof_filler_bits};
    // LDPC decoding with the codeblock CRC as early stop (pusch_codeblock_decoder.cpp:35-69)
    srs_amd_ldpc_decoder_config dc{bg, Z, c.nof_filler_bits, c.cb_crc_len, c.max_nof_ldpc_iterations};
    const unsigned              N = (bg == 1 ? 66 : 50) * Z;
    // New data lands in freshly cleared rows: with k0 = 0 (rv 0) and no circular wrap only [0, E + F) and the
    // systematic part can be non-zero, so the decoder scans that prefix (srs_amd_pusch_decoder_llr_prefix's rule,
    // sch.h), which bounds its layer count and selects the high-rate kernel for high-rate codeblocks.
    unsigned len = N;
    if (c.new_data && c.rv == 0) {
      unsigned end = 0;
      for (unsigned r = first; r != first + n; ++r) {
        end = std::max(end, cfg[r].cw_length + cfg[r].nof_filler_bits <= cfg[r].Ncb ? cfg[r].cw_length + cfg[r].nof_filler_bits
                                                                                   : N);
      }
      end = std::max(end, (bg == 1 ? 20u : 8u) * Z);
      len = std::min(N, std::max((bg == 1 ? 24u : 12u) * Z, (end + Z - 1) / Z * Z));
    }
    return amd_ok(srs_amd_ldpc_rate_dematch_batch(dm, &md, c.new_data ? 1 : 0, d_llrs, d_arrays + first,
                                                  d_arrays + MAX_CBS + first, harq->row(tb_base + first), ROW, n,
                                                  stream),
                  "rate dematching") &&
           amd_ok(srs_amd_ldpc_decode_batch(dec, &dc, c.use_early_stop ? crc_poly(c.cb_crc_type) : SRS_AMD_NO_CRC,
                                            harq->row(tb_base + first), ROW, nullptr, len,
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
  unsigned                            abs_ids[MAX_CBS] = {};
  bool                                enqueued[MAX_CBS] = {};
  uint32_t                            offsets[MAX_CBS]  = {};
  uint32_t                            lengths[MAX_CBS]  = {};
  std::vector<unsigned>               new_rows;
  unsigned                            tb_base = UINT32_MAX, nof_cbs = 0;
  size_t                              staged = 0, staging_cap = 0;
  bool                                flushed = false;
  bool                                failed  = false; // the current transport block reports CRC failures
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
      require_hip(hipGetDevice(&cfg.device), "hipGetDevice");
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
