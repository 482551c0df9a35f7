// pdcch_api.cpp -- C-ABI of the MI355X PDCCH processor (include/srsran_amd/pdcch.h): pdcch_processor_impl::process
// (pdcch_processor_impl.cpp:79-130) for every DCI of a slot.  Host side, per DCI: the validator's checks
// (pdcch_processor_validator_impl.cpp:27-85), the CCEs' CRBs (cce_to_prb_mapping.cpp), the encoder and scrambling
// parameters and the DCI input bit interleaver permutation; device side: pdcch_crc_kernel, one polar-encoder launch
// per (K, E) code (polar.h, the pdcch_encoder_impl chain with nMax = 9), pdcch_map_kernel.
#include "srsran_amd/pdcch.h"
#include "srsran_amd/polar.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "gold_sequence.h"
#include "pdcch_args.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_pdcch_processor {
  int                                               device = 0;
  uint32_t*                                         d_jump = nullptr;
  std::map<std::pair<uint32_t, uint32_t>, srs_amd_polar_code*> codes; // (K, E)
  device_buffer                                     buf, host_grid;
  pinned_stage                                      stage;
  stream_order                                      order;
  hipStream_t                                       stream = nullptr; // host calls
  std::mutex                                        mtx;
  std::mutex                                        host_mtx; // the host form's grid buffer and stream
  ~srs_amd_pdcch_processor()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    for (auto& kv : codes) {
      srs_amd_polar_code_destroy(kv.second);
    }
    (void)hipFree(d_jump);
  }
};

namespace {

constexpr uint32_t NSYMB = 14;

bool freq_bit(const srs_amd_pdcch_coreset& c, uint32_t i)
{
  return i < 64 && ((c.frequency_resources[i / 8] >> (i % 8)) & 1u);
}

uint32_t freq_count(const srs_amd_pdcch_coreset& c)
{
  uint32_t n = 0;
  for (uint32_t i = 0; i < 45; ++i) {
    n += freq_bit(c, i) ? 1u : 0u;
  }
  return n;
}

// cce_to_reg_mapping_interleaved (cce_to_prb_mapping.cpp:44-89); empty on an invalid configuration.
std::vector<uint32_t> regs_interleaved(uint32_t N_rb, uint32_t N_symb, uint32_t L, uint32_t R, uint32_t n_shift,
                                       uint32_t al, uint32_t cce)
{
  std::vector<uint32_t> out;
  const uint32_t        N_reg = N_rb * N_symb;
  if (L == 0 || R == 0 || N_reg == 0 || N_reg % (L * R) != 0 || L % N_symb != 0) {
    return out;
  }
  const uint32_t C = N_reg / (L * R), per_cce = 6 / L;
  for (uint32_t x = cce * per_cce; x != (cce + al) * per_cce; ++x) {
    const uint32_t r = x % R, c = x / R;
    const uint32_t f = (r * C + c + n_shift) % (N_reg / L);
    for (uint32_t reg = f * L; reg != (f + 1) * L; ++reg) {
      out.push_back(reg);
    }
  }
  std::sort(out.begin(), out.end());
  return out;
}

// reg_to_prb_mapping_other (cce_to_prb_mapping.cpp:111-148)
std::vector<uint32_t> prbs_other(uint32_t bwp_start, const srs_amd_pdcch_coreset& c, uint32_t N_symb,
                                 const std::vector<uint32_t>& regs)
{
  std::vector<uint32_t> out;
  uint32_t              count = 0, reg = 0;
  for (uint32_t f = 0; f < 45 && count < regs.size(); ++f) {
    if (!freq_bit(c, f)) {
      continue;
    }
    for (uint32_t prb = f * 6 + bwp_start; prb != f * 6 + bwp_start + 6; ++prb, reg += N_symb) {
      if (reg != regs[count]) {
        continue;
      }
      out.push_back(prb);
      count += N_symb;
      if (count == regs.size()) {
        return out;
      }
    }
  }
  return out;
}

// pdcch_processor_impl::compute_rb_mask + pdcch_processor_validator_impl::is_valid; CRBs ascending.
int dci_crbs(const srs_amd_pdcch_pdu& p, std::vector<uint32_t>& crbs)
{
  const srs_amd_pdcch_coreset& c = p.coreset;
  const srs_amd_pdcch_dci&     d = p.dci;
  if (c.duration < 1 || c.duration > 3) {
    return fail(SRS_AMD_EINVAL, "The CORESET duration (i.e., %u) is out of the range 1-3.", c.duration);
  }
  if (c.start_symbol_index + c.duration > NSYMB) {
    return fail(SRS_AMD_EINVAL, "The CORESET start symbol index (i.e., %u) plus the duration (i.e., %u) exceeds the slot "
                                "duration (i.e., 14).", c.start_symbol_index, c.duration);
  }
  const bool il = c.cce_to_reg_mapping == 2;
  if (c.cce_to_reg_mapping > 2) {
    return fail(SRS_AMD_EINVAL, "Invalid CCE-to-REG mapping %u.", c.cce_to_reg_mapping);
  }
  if (il && (((c.duration == 3) && (c.reg_bundle_size != 3)) || ((c.duration != 3) && (c.reg_bundle_size != 2))) &&
      (c.reg_bundle_size != 6)) {
    return fail(SRS_AMD_EINVAL, "Invalid REG bundle size (i.e., %u) for CORESET duration of %u.", c.reg_bundle_size,
                c.duration);
  }
  if (il && c.interleaver_size != 2 && c.interleaver_size != 3 && c.interleaver_size != 6) {
    return fail(SRS_AMD_EINVAL, "Invalid interleaver size (i.e., %u).", c.interleaver_size);
  }
  const uint32_t al = d.aggregation_level;
  if (al != 1 && al != 2 && al != 4 && al != 8 && al != 16) {
    return fail(SRS_AMD_EINVAL, "Invalid aggregation level (i.e., %u).", al);
  }
  if (d.cce_index + al > freq_count(c) * c.duration) {
    return fail(SRS_AMD_EINVAL, "The CCE index (i.e., %u) plus the aggregation level (i.e., %u) exceeds CORESET "
                                "capacity (i.e., %u).", d.cce_index, al, freq_count(c) * c.duration);
  }
  if (d.payload_size == 0 || d.payload_size > SRS_AMD_PDCCH_MAX_PAYLOAD) {
    return fail(SRS_AMD_EINVAL, "Invalid payload size %u.", d.payload_size);
  }
  if (d.nof_ports == 0 || d.nof_ports > 4) {
    return fail(SRS_AMD_EINVAL, "Invalid number of ports %u.", d.nof_ports);
  }
  crbs.clear();
  if (c.cce_to_reg_mapping == 0) {
    // cce_to_prb_mapping_coreset0: interleaved over the CORESET0 RBs (L = 6, R = 2, n_shift = N_id_cell), one PRB
    // per REG row (reg_to_prb_mapping_coreset0)
    const std::vector<uint32_t> regs =
        regs_interleaved(c.bwp_size_rb, c.duration, 6, 2, c.shift_index, al, d.cce_index);
    for (size_t i = 0; i < regs.size(); i += c.duration) {
      crbs.push_back(regs[i] / c.duration + c.bwp_start_rb);
    }
  } else if (c.cce_to_reg_mapping == 1) {
    std::vector<uint32_t> regs;
    for (uint32_t r = 6 * d.cce_index; r != 6 * (d.cce_index + al); ++r) {
      regs.push_back(r);
    }
    crbs = prbs_other(c.bwp_start_rb, c, c.duration, regs);
  } else {
    crbs = prbs_other(c.bwp_start_rb, c, c.duration,
                      regs_interleaved(freq_count(c) * 6, c.duration, c.reg_bundle_size, c.interleaver_size,
                                       c.shift_index, al, d.cce_index));
  }
  // the rb_mask is a bitmap: ascending, no duplicates
  std::sort(crbs.begin(), crbs.end());
  crbs.erase(std::unique(crbs.begin(), crbs.end()), crbs.end());
  if (crbs.empty() || crbs.size() > PDCCH_MAX_RB) {
    return fail(SRS_AMD_EINVAL, "Invalid CORESET configuration (no RB for the DCI's CCEs).");
  }
  return static_cast<int>(crbs.size());
}

// The polar code of (K, E), created on first use (nMax = 9, no channel interleaver: pdcch_encoder_impl.cpp:82).
int code_of(srs_amd_pdcch_processor* proc, uint32_t K, uint32_t E, srs_amd_polar_code** code)
{
  auto it = proc->codes.find({K, E});
  if (it == proc->codes.end()) {
    srs_amd_polar_code* c  = nullptr;
    const int           rc = srs_amd_polar_code_create(&c, K, E, 9, 0, proc->device);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    it = proc->codes.emplace(std::make_pair(K, E), c).first;
  }
  *code = it->second;
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_pdcch_processor_create(srs_amd_pdcch_processor** proc, int device)
{
  if (proc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *proc  = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* p                 = new srs_amd_pdcch_processor();
  p->device               = device;
  std::vector<uint32_t> j = gold_jump_tables();
  hipError_t            e = hipMalloc(&p->d_jump, j.size() * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = hipMemcpy(p->d_jump, j.data(), j.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "PDCCH processor tables");
  }
  *proc = p;
  return SRS_AMD_OK;
}

void srs_amd_pdcch_processor_destroy(srs_amd_pdcch_processor* proc)
{
  delete proc;
}

int srs_amd_pdcch_rb_mask(const srs_amd_pdcch_pdu* pdu, uint8_t* crb_mask)
{
  if (pdu == nullptr || crb_mask == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  std::vector<uint32_t> crbs;
  const int             n = dci_crbs(*pdu, crbs);
  if (n < 0) {
    return n;
  }
  std::memset(crb_mask, 0, SRS_AMD_CRB_MASK_BYTES);
  for (uint32_t r : crbs) {
    if (r < 8 * SRS_AMD_CRB_MASK_BYTES) {
      crb_mask[r / 8] |= static_cast<uint8_t>(1u << (r % 8));
    }
  }
  return n;
}

int srs_amd_pdcch_process_slot(srs_amd_pdcch_processor* proc,
                               const srs_amd_pdcch_pdu* pdus,
                               uint32_t                 nof_pdus,
                               uint32_t*                d_grids,
                               uint64_t                 grid_stride,
                               uint32_t                 nof_grids,
                               uint32_t                 nof_subc,
                               void*                    stream)
{
  if (proc == nullptr || (nof_pdus != 0 && pdus == nullptr)) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_pdus == 0) {
    return SRS_AMD_OK;
  }
  if (nof_subc == 0 || nof_subc % 12 != 0) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  std::lock_guard<std::mutex> lock(proc->mtx);
  // descriptors, grouped by polar code so that each code's messages / codewords are contiguous rows
  std::vector<pdcch_desc>                   desc(nof_pdus);
  std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> groups;
  uint32_t                                  max_rb = 0, max_symbols = 0;
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const srs_amd_pdcch_pdu& p = pdus[i];
    std::vector<uint32_t>    crbs;
    const int                n = dci_crbs(p, crbs);
    if (n < 0) {
      return n;
    }
    if (p.d_grid == nullptr && (d_grids == nullptr || p.grid >= nof_grids)) {
      return fail(SRS_AMD_EINVAL, "PDU %u: grid index %u out of range (or no grid).", i, p.grid);
    }
    if (crbs.back() >= nof_subc / 12) {
      return fail(SRS_AMD_EINVAL, "PDU %u: CRB %u outside the grid.", i, crbs.back());
    }
    if (p.numerology > 4 || p.slot_index >= (10u << p.numerology)) {
      return fail(SRS_AMD_EINVAL, "PDU %u: invalid slot %u of numerology %u.", i, p.slot_index, p.numerology);
    }
    pdcch_desc& d   = desc[i];
    d               = pdcch_desc{};
    d.payload_size  = p.dci.payload_size;
    d.K             = p.dci.payload_size + 24;
    d.E             = p.dci.aggregation_level * 6 * 9 * 2; // pdcch_processor_impl.cpp:91
    d.rnti          = p.dci.rnti & 0xffffu;
    uint8_t idx[PDCCH_MAX_K], perm[PDCCH_MAX_K];
    for (uint32_t k = 0; k != d.K; ++k) {
      idx[k] = static_cast<uint8_t>(k);
    }
    if (srs_amd_polar_interleave(perm, idx, d.K, 0) != SRS_AMD_OK) {
      return fail(SRS_AMD_EINVAL, "PDU %u: payload of %u bits exceeds the DCI interleaver.", i, p.dci.payload_size);
    }
    std::memcpy(d.perm, perm, d.K);
    d.grid         = p.d_grid != nullptr ? p.d_grid : d_grids + p.grid * grid_stride;
    d.port_stride  = NSYMB * nof_subc;
    d.nof_subc     = nof_subc;
    d.nof_rb       = static_cast<uint32_t>(crbs.size());
    d.start_symbol = p.coreset.start_symbol_index;
    d.duration     = p.coreset.duration;
    d.ref_k_rb     = p.coreset.cce_to_reg_mapping == 0 ? p.coreset.bwp_start_rb : 0; // pdcch_processor_impl.cpp:114
    if (crbs.front() < d.ref_k_rb) {
      return fail(SRS_AMD_EINVAL, "PDU %u: CRB below the DM-RS reference point.", i);
    }
    d.c_init_data = static_cast<uint32_t>(((static_cast<uint64_t>(p.dci.n_rnti) << 16) + p.dci.n_id_pdcch_data) %
                                          (1ull << 31)); // pdcch_modulator_impl.cpp:35
    for (uint32_t li = 0; li != d.duration; ++li) {
      // dmrs_pdcch_processor_impl.cpp:32-39
      const uint64_t l = d.start_symbol + li;
      const uint64_t n = p.dci.n_id_pdcch_dmrs;
      d.c_init_dmrs[li] =
          static_cast<uint32_t>(((NSYMB * p.slot_index + l + 1) * (2 * n + 1) * (1ull << 17) + 2 * n) % (1ull << 31));
    }
    // convert_dB_to_amplitude (math_utils.h:118-121) in float, as the reference
    d.data_amp    = std::pow(10.0F, p.dci.data_power_offset_dB / 20.0F);
    d.data_scaled = std::isnormal(d.data_amp) ? 1 : 0;
    d.dmrs_amp    = static_cast<float>(M_SQRT1_2 * std::pow(10.0F, p.dci.dmrs_power_offset_dB / 20.0F));
    d.nof_ports   = p.dci.nof_ports;
    std::memcpy(d.w, p.dci.weights, sizeof(d.w));
    for (size_t k = 0; k != crbs.size(); ++k) {
      d.crbs[k] = static_cast<uint16_t>(crbs[k]);
    }
    max_rb      = std::max(max_rb, d.nof_rb);
    max_symbols = std::max(max_symbols, d.duration);
    groups[{d.K, d.E}].push_back(i);
  }
  // buffer layout: descriptors | payloads (128 B per DCI) | messages (rows of K per code group) | codewords (rows of E)
  uint64_t msg_total = 0, cw_total = 0;
  for (auto& g : groups) {
    for (uint32_t i : g.second) {
      desc[i].msg_offset = static_cast<uint32_t>(msg_total);
      desc[i].cw_offset  = static_cast<uint32_t>(cw_total);
      msg_total += g.first.first;
      cw_total += g.first.second;
    }
  }
  const size_t o_pay   = align_up(sizeof(pdcch_desc) * nof_pdus, 256);
  const size_t o_msg   = o_pay + align_up(static_cast<size_t>(SRS_AMD_PDCCH_MAX_PAYLOAD) * nof_pdus, 256);
  const size_t o_cw    = o_msg + align_up(msg_total, 256);
  const size_t total   = o_cw + align_up(cw_total, 256);
  const size_t staged  = o_msg; // descriptors + payloads come from the host
  auto         s       = static_cast<hipStream_t>(stream);
  hipError_t   e       = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->buf.ensure(total);
  }
  if (e == hipSuccess) {
    e = proc->stage.acquire(staged);
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PDCCH processor scratch");
  }
  call_scope scope(proc->order, nullptr, s);
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    desc[i].payload_offset = i * SRS_AMD_PDCCH_MAX_PAYLOAD;
    std::memcpy(proc->stage.at<uint8_t>(o_pay + desc[i].payload_offset), pdus[i].dci.payload,
                pdus[i].dci.payload_size);
  }
  std::memcpy(proc->stage.at<uint8_t>(0), desc.data(), sizeof(pdcch_desc) * nof_pdus);
  auto* base = proc->buf.as<uint8_t>();
  auto* d_desc = reinterpret_cast<const pdcch_desc*>(base);
  e            = proc->stage.upload(base, staged, s);
  if (e == hipSuccess) {
    e = launch_pdcch_crc(d_desc, nof_pdus, base + o_pay, base + o_msg, s);
  }
  int rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pdcch_crc_kernel launch");
  for (auto& g : groups) {
    if (rc != SRS_AMD_OK) {
      break;
    }
    srs_amd_polar_code* code = nullptr;
    rc                       = code_of(proc, g.first.first, g.first.second, &code);
    if (rc == SRS_AMD_OK) {
      const pdcch_desc& first = desc[g.second.front()];
      rc = srs_amd_polar_encode_batch(code, base + o_msg + first.msg_offset, g.first.first,
                                      base + o_cw + first.cw_offset, g.first.second,
                                      static_cast<uint32_t>(g.second.size()), stream);
    }
  }
  if (rc == SRS_AMD_OK) {
    e  = launch_pdcch_map(d_desc, nof_pdus, max_rb, max_symbols, base + o_cw, proc->d_jump, s);
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pdcch_map_kernel launch");
  }
  const hipError_t done = scope.close();
  return rc != SRS_AMD_OK ? rc : (done == hipSuccess ? SRS_AMD_OK : hip_fail(done, "PDCCH completion event"));
}

int srs_amd_pdcch_process(srs_amd_pdcch_processor* proc,
                          const srs_amd_pdcch_pdu* pdu,
                          uint32_t*                grid,
                          uint32_t                 nof_ports,
                          uint32_t                 nof_subc)
{
  if (proc == nullptr || pdu == nullptr || grid == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (pdu->dci.nof_ports > nof_ports) {
    return fail(SRS_AMD_EINVAL, "The grid has %u ports, the PDU precodes onto %u.", nof_ports, pdu->dci.nof_ports);
  }
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PDCCH processor grid");
  }
  e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  if (e != hipSuccess) {
    return hip_fail(e, "PDCCH grid upload");
  }
  srs_amd_pdcch_pdu p = *pdu;
  p.grid              = 0;
  p.d_grid            = nullptr;
  int rc = srs_amd_pdcch_process_slot(proc, &p, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_subc, proc->stream);
  if (rc == SRS_AMD_OK) {
    e  = hipMemcpyAsync(grid, proc->host_grid.ptr, bytes, hipMemcpyDeviceToHost, proc->stream);
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PDCCH grid download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

} // extern "C"
