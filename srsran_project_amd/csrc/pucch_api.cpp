// pucch_api.cpp -- C-ABI of the MI355X PUCCH Format 0 detector (include/srsran_amd/pucch.h):
// pucch_detector_format0::detect (pucch_detector_format0.cpp:124-246) for every PDU of a slot.  Host side, per PDU:
// the cyclic-shift table of the payload (TS 38.213 Tables 9.2.3-3 / 9.2.3-4 / 9.2.5-1 / 9.2.5-2 as the reference
// lists them, :48-71), the detection threshold (pick_threshold, :73-122), the group sequence u = n_id mod 30
// (pucch_helper::compute_group_sequence without hopping) and for every candidate and symbol the cyclic shift
// alpha = (m0 + m_cs + n_cs) mod 12, n_cs = sum_m 2^m c(8 (14 n_slot + l) + m) of the Gold sequence of n_id
// (pucch_helper::get_alpha_index), and its low-PAPR sequence (srs_amd_low_papr_sequence x e^(j 2 pi alpha n / 12));
// device side: pucch_f0_kernel.
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

} // extern "C"
