// pucch_api.cpp -- C-ABI of the MI355X PUCCH Format 0 detector (include/srsran_amd/pucch.h):
// pucch_detector_format0::detect (pucch_detector_format0.cpp:124-246) for every PDU of a slot.  Host side, per PDU:
// the cyclic-shift table of the payload (TS 38.213 Tables 9.2.3-3 / 9.2.3-4 / 9.2.5-1 / 9.2.5-2 as the reference
// lists them, :48-71), the detection threshold (pick_threshold, :73-122), the group sequence u = n_id mod 30
// (pucch_helper::compute_group_sequence without hopping) and for every candidate and symbol the cyclic shift
// alpha = (m0 + m_cs + n_cs) mod 12, n_cs = sum_m 2^m c(8 (14 n_slot + l) + m) of the Gold sequence of n_id
// (pucch_helper::get_alpha_index), and its low-PAPR sequence (srs_amd_low_papr_sequence x e^(j 2 pi alpha n / 12));
// device side: pucch_f0_kernel.
//
// Format 1 (pucch_detector_format1.cpp:156-663 behind pucch_processor_impl.cpp:74-138): per batch, the checks of
// validate_config (:57-98) and of the processor's PDU validator, the threshold by ports x hops (:194-212), the base
// cyclic shift n_cs of every allocated symbol (get_alpha_index with m0 = m_cs = 0, :562), the base sequence of group
// n_id mod 30 and the set of OCC indices in use; device side: pucch_f1_kernel.
#include "srsran_amd/pucch.h"
#include "srsran_amd/low_papr.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "gold_sequence.h"
#include "pucch_args.h"
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_pucch_processor {
  int                   device = 0;
  std::vector<uint32_t> jump; // host copy of gold_jump_tables()
  device_buffer         buf, host_grid, host_res;
  pinned_stage          stage;
  stream_order          order;
  hipStream_t           stream = nullptr; // host calls
  std::mutex            mtx;
  std::mutex            host_mtx;
  ~srs_amd_pucch_processor()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
  }
};

namespace {

constexpr uint32_t NSYMB = 14;

struct f0_entry {
  uint32_t m_cs;
  uint8_t  sr, h0, h1;
};
// pucch_detector_format0.cpp:48-71 (table order)
const f0_entry T_SR[1]       = {{0, 1, 0, 0}};
const f0_entry T_1H[2]       = {{0, 0, 0, 0}, {6, 0, 1, 0}};
const f0_entry T_2H[4]       = {{0, 0, 0, 0}, {3, 0, 0, 1}, {6, 0, 1, 1}, {9, 0, 1, 0}};
const f0_entry T_1H_SR[4]    = {{0, 0, 0, 0}, {6, 0, 1, 0}, {3, 1, 0, 0}, {9, 1, 1, 0}};
const f0_entry T_2H_SR[8]    = {{0, 0, 0, 0}, {3, 0, 0, 1}, {6, 0, 1, 1}, {9, 0, 1, 0},
                                {1, 1, 0, 0}, {4, 1, 0, 1}, {7, 1, 1, 1}, {10, 1, 1, 0}};

// pick_threshold (:73-122): the first entry (degrees of freedom, sequences) >= the request; < 0 when none.
float threshold(uint32_t nof_ports, uint32_t nof_symbols, uint32_t nof_seq)
{
  struct entry {
    uint32_t dof, nseq;
    float    th;
  };
  static const entry t[16] = {{1, 1, 0.5373f}, {1, 2, 0.6460f}, {1, 4, 0.7556f}, {1, 8, 1.6818f},
                              {2, 1, 0.5273f}, {2, 2, 0.4038f}, {2, 4, 0.7273f}, {2, 8, 0.8364f},
                              {4, 1, 0.3455f}, {4, 2, 0.2800f}, {4, 4, 0.4455f}, {4, 8, 0.5000f},
                              {8, 1, 0.2545f}, {8, 2, 0.2083f}, {8, 4, 0.3000f}, {8, 8, 0.3273f}};
  const uint32_t dof = nof_ports * nof_symbols;
  for (const entry& e : t) {
    if (e.dof > dof || (e.dof == dof && e.nseq >= nof_seq)) {
      return e.th;
    }
  }
  return -1.0f;
}

uint32_t gf2_apply_h(const uint32_t* cols, uint32_t s)
{
  uint32_t r = 0;
  for (int j = 0; j < 31; ++j) {
    if ((s >> j) & 1u) {
      r ^= cols[j];
    }
  }
  return r;
}

// Gold-sequence bits c(n0 .. n0 + 7) of c_init (bit m of the result = c(n0 + m)), with the host jump tables.
uint32_t gold_byte(const std::vector<uint32_t>& jump, uint32_t c_init, uint32_t n0)
{
  uint32_t       x1 = 1u, x2 = c_init & 0x7fffffffu;
  const uint32_t steps = n0 + 1600u;
  for (int k = 0; k < PRBS_NJUMP; ++k) {
    if ((steps >> k) & 1u) {
      x1 = gf2_apply_h(jump.data() + (0 * PRBS_NJUMP + k) * 31, x1);
      x2 = gf2_apply_h(jump.data() + (1 * PRBS_NJUMP + k) * 31, x2);
    }
  }
  uint32_t out = 0;
  for (uint32_t m = 0; m != 8; ++m) {
    out |= ((x1 ^ x2) & 1u) << m;
    const uint32_t n1 = ((x1 >> 3) ^ x1) & 1u;
    const uint32_t n2 = ((x2 >> 3) ^ (x2 >> 2) ^ (x2 >> 1) ^ x2) & 1u;
    x1                = (x1 >> 1) | (n1 << 30);
    x2                = (x2 >> 1) | (n2 << 30);
  }
  return out;
}

int make_desc(const srs_amd_pucch_processor* proc, const srs_amd_pucch_f0_pdu& p, const uint32_t* d_grids,
              uint64_t grid_stride, uint32_t nof_grids, uint32_t nof_grid_ports, uint32_t nof_subc, pucch_f0_desc& d)
{
  if (p.nof_symbols < 1 || p.nof_symbols > 2 || p.start_symbol_index + p.nof_symbols > NSYMB) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 0 symbols (start %u, %u symbols).", p.start_symbol_index,
                p.nof_symbols);
  }
  if (p.second_hop_prb >= 0 && p.nof_symbols != 2) {
    return fail(SRS_AMD_EINVAL, "Frequency hopping needs 2 OFDM symbols.");
  }
  if (p.initial_cyclic_shift > 11 || p.nof_harq_ack > 2 || p.nof_ports == 0 || p.nof_ports > 4 ||
      p.numerology > 4 || p.slot_index >= (10u << p.numerology) || p.n_id > 1023) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 0 PDU (m0 %u, %u HARQ-ACK bits, %u ports, slot %u, n_id %u).",
                p.initial_cyclic_shift, p.nof_harq_ack, p.nof_ports, p.slot_index, p.n_id);
  }
  if (p.nof_harq_ack == 0 && !p.sr_opportunity) {
    return fail(SRS_AMD_EINVAL, "Invalid payload combination.");
  }
  if (p.d_grid == nullptr && (d_grids == nullptr || p.grid >= nof_grids)) {
    return fail(SRS_AMD_EINVAL, "grid index %u out of range (or no grid).", p.grid);
  }
  d      = pucch_f0_desc{};
  d.grid = p.d_grid != nullptr ? p.d_grid : d_grids + p.grid * grid_stride;
  d.port_stride = NSYMB * nof_subc;
  d.nof_subc    = nof_subc;
  d.l0          = p.start_symbol_index;
  d.nsym        = p.nof_symbols;
  for (uint32_t l = 0; l != p.nof_symbols; ++l) {
    const uint32_t prb = (l != 0 && p.second_hop_prb >= 0) ? static_cast<uint32_t>(p.second_hop_prb) : p.starting_prb;
    if (12 * (prb + 1) > nof_subc) {
      return fail(SRS_AMD_EINVAL, "PRB %u outside the grid.", prb);
    }
    d.subc0[l] = 12 * prb;
  }
  d.nof_ports = p.nof_ports;
  for (uint32_t i = 0; i != p.nof_ports; ++i) {
    if (p.ports[i] >= nof_grid_ports) {
      return fail(SRS_AMD_EINVAL, "port %u outside the grid's %u ports.", p.ports[i], nof_grid_ports);
    }
    d.ports[i] = p.ports[i];
  }
  const f0_entry* tab = T_SR;
  uint32_t        n   = 1;
  if (p.nof_harq_ack == 1) {
    tab = p.sr_opportunity ? T_1H_SR : T_1H;
    n   = p.sr_opportunity ? 4 : 2;
  } else if (p.nof_harq_ack == 2) {
    tab = p.sr_opportunity ? T_2H_SR : T_2H;
    n   = p.sr_opportunity ? 8 : 4;
  }
  d.nof_cand       = n;
  d.nof_sr         = p.nof_harq_ack == 0 ? 1u : (p.sr_opportunity ? 1u : 0u);
  d.nof_harq       = p.nof_harq_ack;
  d.nof_sr_default = p.sr_opportunity ? 1u : 0u;
  d.threshold      = threshold(p.nof_ports, p.nof_symbols, n);
  if (d.threshold < 0) {
    return fail(SRS_AMD_EINVAL, "Requested configuration (%u antenna ports, %u OFDM symbols, %u sequences) not supported.",
                p.nof_ports, p.nof_symbols, n);
  }
  // base sequence of group u = n_id mod 30 (v = 0), then the cyclic shift of each candidate and symbol
  float base[24];
  if (srs_amd_low_papr_sequence(base, 12, p.n_id % 30, 0) != SRS_AMD_OK) {
    return SRS_AMD_EINVAL;
  }
  for (uint32_t c = 0; c != n; ++c) {
    d.msg[c][0] = tab[c].sr;
    d.msg[c][1] = tab[c].h0;
    d.msg[c][2] = tab[c].h1;
    for (uint32_t l = 0; l != p.nof_symbols; ++l) {
      const uint32_t n_cs  = gold_byte(proc->jump, p.n_id, 8 * (NSYMB * p.slot_index + p.start_symbol_index + l));
      const uint32_t alpha = (p.initial_cyclic_shift + tab[c].m_cs + n_cs) % 12;
      for (uint32_t k = 0; k != 12; ++k) {
        const double ph = 2.0 * M_PI * static_cast<double>((alpha * k) % 12) / 12.0;
        const float  cr = static_cast<float>(std::cos(ph)), ci = static_cast<float>(std::sin(ph));
        const float  br = base[2 * k], bi = base[2 * k + 1];
        d.seq[c][l][k] = make_float2(br * cr - bi * ci, br * ci + bi * cr);
      }
    }
  }
  return SRS_AMD_OK;
}

int make_f1_desc(const srs_amd_pucch_processor* proc, const srs_amd_pucch_f1_batch& b, const uint32_t* d_grids,
                 uint64_t grid_stride, uint32_t nof_grids, uint32_t nof_grid_ports, uint32_t nof_subc, uint32_t entry0,
                 pucch_f1_desc& d)
{
  if (b.start_symbol_index > 10 || b.nof_symbols < 4 || b.nof_symbols > 14 ||
      b.start_symbol_index + b.nof_symbols > NSYMB) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 1 symbols (start %u, %u symbols).", b.start_symbol_index,
                b.nof_symbols);
  }
  if (b.numerology > 4 || b.slot_index >= (10u << b.numerology) || b.n_id > 1023) {
    return fail(SRS_AMD_EINVAL, "Invalid Format 1 batch (slot %u, numerology %u, n_id %u).", b.slot_index,
                b.numerology, b.n_id);
  }
  const uint32_t hops = b.second_hop_prb >= 0 ? 2u : 1u;
  const uint32_t contributions = b.nof_ports * hops;
  if (b.nof_ports == 0 || b.nof_ports > 4 ||
      (contributions != 1 && contributions != 2 && contributions != 4 && contributions != 8)) {
    return fail(SRS_AMD_EINVAL, "The PUCCH detector does not support %u ports.", b.nof_ports);
  }
  if (b.nof_entries == 0 || b.nof_entries > PUCCH_F1_MAX_ENTRIES || b.entries == nullptr) {
    return fail(SRS_AMD_EINVAL, "Invalid number of multiplexed PUCCH (i.e., %u).", b.nof_entries);
  }
  if (b.d_grid == nullptr && (d_grids == nullptr || b.grid >= nof_grids)) {
    return fail(SRS_AMD_EINVAL, "grid index %u out of range (or no grid).", b.grid);
  }
  d             = pucch_f1_desc{};
  d.grid        = b.d_grid != nullptr ? b.d_grid : d_grids + b.grid * grid_stride;
  d.port_stride = NSYMB * nof_subc;
  d.nof_subc    = nof_subc;
  d.l0          = b.start_symbol_index;
  d.nsym        = b.nof_symbols;
  d.nof_hops    = hops;
  for (uint32_t h = 0; h != hops; ++h) {
    const uint32_t prb = h == 0 ? b.starting_prb : static_cast<uint32_t>(b.second_hop_prb);
    if (prb > 274 || 12 * (prb + 1) > nof_subc) {
      return fail(SRS_AMD_EINVAL, "PRB %u outside the grid.", prb);
    }
    d.subc0[h] = 12 * prb;
  }
  d.nof_ports = b.nof_ports;
  for (uint32_t i = 0; i != b.nof_ports; ++i) {
    if (b.ports[i] >= nof_grid_ports) {
      return fail(SRS_AMD_EINVAL, "port %u outside the grid's %u ports.", b.ports[i], nof_grid_ports);
    }
    d.ports[i] = b.ports[i];
  }
  const uint32_t occ_ratio = hops == 2 ? 4u : 2u;
  uint32_t       used[7]   = {};
  for (uint32_t e = 0; e != b.nof_entries; ++e) {
    const srs_amd_pucch_f1_entry& en = b.entries[e];
    if (en.initial_cyclic_shift > 11 || en.time_domain_occ > 6 || en.time_domain_occ >= b.nof_symbols / occ_ratio ||
        en.nof_harq_ack > 2) {
      return fail(SRS_AMD_EINVAL, "Invalid multiplexed PUCCH (shift %u, OCC %u, %u HARQ-ACK bits, %u symbols).",
                  en.initial_cyclic_shift, en.time_domain_occ, en.nof_harq_ack, b.nof_symbols);
    }
    if ((used[en.time_domain_occ] >> en.initial_cyclic_shift) & 1u) {
      return fail(SRS_AMD_EINVAL, "Two PUCCH with shift %u and OCC %u.", en.initial_cyclic_shift, en.time_domain_occ);
    }
    used[en.time_domain_occ] |= 1u << en.initial_cyclic_shift;
    d.occ_mask |= 1u << en.time_domain_occ;
  }
  d.nof_entries = b.nof_entries;
  d.entry0      = entry0;
  d.threshold   = contributions == 1 ? 0.9f : contributions == 2 ? 3.0f : contributions == 4 ? 4.45f : 6.95f;
  for (uint32_t r = 0; r != b.nof_symbols; ++r) {
    d.alpha[r] = static_cast<uint8_t>(
        gold_byte(proc->jump, b.n_id, 8 * (NSYMB * b.slot_index + b.start_symbol_index + r)) % 12);
  }
  float base[24];
  if (srs_amd_low_papr_sequence(base, 12, b.n_id % 30, 0) != SRS_AMD_OK) {
    return SRS_AMD_EINVAL;
  }
  for (uint32_t k = 0; k != 12; ++k) {
    d.base[k] = make_float2(base[2 * k], base[2 * k + 1]);
  }
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_pucch_processor_create(srs_amd_pucch_processor** proc, int device)
{
  if (proc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *proc  = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* p   = new srs_amd_pucch_processor();
  p->device = device;
  p->jump   = gold_jump_tables();
  if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
    delete p;
    return hip_fail(hipErrorUnknown, "PUCCH processor stream");
  }
  *proc = p;
  return SRS_AMD_OK;
}

void srs_amd_pucch_processor_destroy(srs_amd_pucch_processor* proc)
{
  delete proc;
}

int srs_amd_pucch_f0_detect_slot(srs_amd_pucch_processor*    proc,
                                 const srs_amd_pucch_f0_pdu* pdus,
                                 uint32_t                    nof_pdus,
                                 const uint32_t*             d_grids,
                                 uint64_t                    grid_stride,
                                 uint32_t                    nof_grids,
                                 uint32_t                    nof_grid_ports,
                                 uint32_t                    nof_subc,
                                 srs_amd_pucch_f0_result*    d_results,
                                 void*                       stream)
{
  if (proc == nullptr || (nof_pdus != 0 && (pdus == nullptr || d_results == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_pdus == 0) {
    return SRS_AMD_OK;
  }
  if (nof_subc == 0 || nof_subc % 12 != 0) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  std::lock_guard<std::mutex> lock(proc->mtx);
  std::vector<pucch_f0_desc>  desc(nof_pdus);
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const int rc = make_desc(proc, pdus[i], d_grids, grid_stride, nof_grids, nof_grid_ports, nof_subc, desc[i]);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  const size_t bytes = sizeof(pucch_f0_desc) * nof_pdus;
  auto         s     = static_cast<hipStream_t>(stream);
  hipError_t   e     = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->buf.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->stage.acquire(bytes);
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH processor scratch");
  }
  call_scope scope(proc->order, nullptr, s);
  std::memcpy(proc->stage.at<uint8_t>(0), desc.data(), bytes);
  e = proc->stage.upload(proc->buf.ptr, bytes, s);
  if (e == hipSuccess) {
    e = launch_pucch_f0(proc->buf.as<pucch_f0_desc>(), nof_pdus, d_results, s);
  }
  const int        rc   = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pucch_f0_kernel launch");
  const hipError_t done = scope.close();
  return rc != SRS_AMD_OK ? rc : (done == hipSuccess ? SRS_AMD_OK : hip_fail(done, "PUCCH completion event"));
}

int srs_amd_pucch_f0_detect(srs_amd_pucch_processor*    proc,
                            const srs_amd_pucch_f0_pdu* pdu,
                            const uint32_t*             grid,
                            uint32_t                    nof_ports,
                            uint32_t                    nof_subc,
                            srs_amd_pucch_f0_result*    result)
{
  if (proc == nullptr || pdu == nullptr || grid == nullptr || result == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->host_res.ensure(sizeof(srs_amd_pucch_f0_result));
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH grid upload");
  }
  srs_amd_pucch_f0_pdu p = *pdu;
  p.grid                 = 0;
  p.d_grid               = nullptr;
  int rc = srs_amd_pucch_f0_detect_slot(proc, &p, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_ports, nof_subc,
                                        proc->host_res.as<srs_amd_pucch_f0_result>(), proc->stream);
  if (rc == SRS_AMD_OK) {
    e  = hipMemcpyAsync(result, proc->host_res.ptr, sizeof(*result), hipMemcpyDeviceToHost, proc->stream);
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUCCH result download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

int srs_amd_pucch_f1_detect_slot(srs_amd_pucch_processor*      proc,
                                 const srs_amd_pucch_f1_batch* batches,
                                 uint32_t                      nof_batches,
                                 const uint32_t*               d_grids,
                                 uint64_t                      grid_stride,
                                 uint32_t                      nof_grids,
                                 uint32_t                      nof_grid_ports,
                                 uint32_t                      nof_subc,
                                 srs_amd_pucch_result*         d_results,
                                 void*                         stream)
{
  if (proc == nullptr || (nof_batches != 0 && (batches == nullptr || d_results == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_batches == 0) {
    return SRS_AMD_OK;
  }
  if (nof_subc == 0 || nof_subc % 12 != 0) {
    return fail(SRS_AMD_EINVAL, "Invalid number of grid subcarriers (i.e., %u).", nof_subc);
  }
  std::lock_guard<std::mutex>         lock(proc->mtx);
  std::vector<pucch_f1_desc>          desc(nof_batches);
  std::vector<srs_amd_pucch_f1_entry> ent;
  for (uint32_t i = 0; i != nof_batches; ++i) {
    const int rc = make_f1_desc(proc, batches[i], d_grids, grid_stride, nof_grids, nof_grid_ports, nof_subc,
                                static_cast<uint32_t>(ent.size()), desc[i]);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    ent.insert(ent.end(), batches[i].entries, batches[i].entries + batches[i].nof_entries);
  }
  const size_t dbytes = sizeof(pucch_f1_desc) * nof_batches;
  const size_t ebytes = sizeof(srs_amd_pucch_f1_entry) * ent.size();
  const size_t eoff   = (dbytes + 255) & ~size_t(255);
  const size_t bytes  = eoff + ebytes;
  auto         s      = static_cast<hipStream_t>(stream);
  hipError_t   e      = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->buf.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->stage.acquire(bytes);
  }
  if (e == hipSuccess) {
    e = proc->order.begin(s);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH processor scratch");
  }
  call_scope scope(proc->order, nullptr, s);
  std::memcpy(proc->stage.at<uint8_t>(0), desc.data(), dbytes);
  std::memcpy(proc->stage.at<uint8_t>(eoff), ent.data(), ebytes);
  e = proc->stage.upload(proc->buf.ptr, bytes, s);
  if (e == hipSuccess) {
    e = launch_pucch_f1(proc->buf.as<pucch_f1_desc>(),
                        nof_batches,
                        reinterpret_cast<const srs_amd_pucch_f1_entry*>(proc->buf.as<uint8_t>() + eoff),
                        d_results,
                        s);
  }
  const int        rc   = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "pucch_f1_kernel launch");
  const hipError_t done = scope.close();
  return rc != SRS_AMD_OK ? rc : (done == hipSuccess ? SRS_AMD_OK : hip_fail(done, "PUCCH completion event"));
}

int srs_amd_pucch_f1_detect(srs_amd_pucch_processor*      proc,
                            const srs_amd_pucch_f1_batch* batch,
                            const uint32_t*               grid,
                            uint32_t                      nof_ports,
                            uint32_t                      nof_subc,
                            srs_amd_pucch_result*         results)
{
  if (proc == nullptr || batch == nullptr || grid == nullptr || results == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (batch->nof_entries == 0 || batch->nof_entries > PUCCH_F1_MAX_ENTRIES) {
    return fail(SRS_AMD_EINVAL, "Invalid number of multiplexed PUCCH (i.e., %u).", batch->nof_entries);
  }
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  const size_t                rbytes = sizeof(srs_amd_pucch_result) * batch->nof_entries;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e == hipSuccess) {
    e = proc->host_res.ensure(rbytes);
  }
  if (e == hipSuccess) {
    e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "PUCCH grid upload");
  }
  srs_amd_pucch_f1_batch b = *batch;
  b.grid                   = 0;
  b.d_grid                 = nullptr;
  int rc = srs_amd_pucch_f1_detect_slot(proc, &b, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_ports, nof_subc,
                                        proc->host_res.as<srs_amd_pucch_result>(), proc->stream);
  if (rc == SRS_AMD_OK) {
    e  = hipMemcpyAsync(results, proc->host_res.ptr, rbytes, hipMemcpyDeviceToHost, proc->stream);
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "PUCCH result download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

} // extern "C"
