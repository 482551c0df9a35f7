// ssb_api.cpp -- C-ABI of the MI355X SS/PBCH block processor (include/srsran_amd/ssb.h): ssb_processor_impl::process
// (ssb_processor_impl.cpp:29-109) for every block of a slot.  Host side, per block: the position in the slot
// (ssb_get_l_first / ssb_get_k_first of include/srsran/ran/ssb/ssb_mapping.h) with the checks the reference asserts,
// the scrambling offsets and DM-RS c_init, the PSS / SSS cyclic shifts; device side: ssb_encode_kernel, one polar
// encoder launch (K = 56, E = 864, nMax = 9: pbch_encoder_impl.h:99), ssb_map_kernel.
#include "srsran_amd/ssb.h"
#include "srsran_amd/polar.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "gold_sequence.h"
#include "ssb_args.h"
#include <array>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_ssb_processor {
  int                 device = 0;
  uint32_t*           d_jump = nullptr;
  uint8_t*            d_seq  = nullptr; // PSS x, SSS x0, x1 (SSB_SEQLEN each)
  srs_amd_polar_code* code   = nullptr;
  uint8_t             perm[SSB_K];
  device_buffer       buf, host_grid;
  pinned_stage        stage;
  stream_order        order;
  hipStream_t         stream = nullptr; // host calls
  std::mutex          mtx;
  std::mutex          host_mtx; // the host form's grid buffer and stream
  ~srs_amd_ssb_processor()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    if (code) {
      srs_amd_polar_code_destroy(code);
    }
    (void)hipFree(d_jump);
    (void)hipFree(d_seq);
  }
};

namespace {

constexpr uint32_t NSYMB = 14;

// The m-sequences of TS 38.211 7.4.2.2 / 7.4.2.3 (pss_sequence_generator.h, sss_sequence_generator.h): PSS x with
// taps x(i + 7) = x(i + 4) + x(i), initial state 1110110 (x6 .. x0); SSS x0 with the same taps and x1 with
// x(i + 7) = x(i + 1) + x(i), both from 0000001.
std::vector<uint8_t> m_sequences()
{
  std::vector<uint8_t> out(3 * SSB_SEQLEN);
  auto gen = [&](uint8_t* dst, std::array<uint8_t, 7> init, int tap) {
    std::array<uint8_t, SSB_SEQLEN + 7> x{};
    for (int i = 0; i != 7; ++i) {
      x[i] = init[i];
    }
    for (uint32_t i = 0; i != SSB_SEQLEN; ++i) {
      x[i + 7] = static_cast<uint8_t>((x[i + tap] + x[i]) % 2);
    }
    std::memcpy(dst, x.data(), SSB_SEQLEN);
  };
  gen(out.data(), {0, 1, 1, 0, 1, 1, 1}, 4);                  // x[0..6] = 0,1,1,0,1,1,1
  gen(out.data() + SSB_SEQLEN, {1, 0, 0, 0, 0, 0, 0}, 4);     // x0
  gen(out.data() + 2 * SSB_SEQLEN, {1, 0, 0, 0, 0, 0, 0}, 1); // x1
  return out;
}

// ssb_get_l_first (ssb_mapping.h:42-103); false for an index outside the pattern
bool l_first(uint32_t pattern, uint32_t idx, uint32_t& l)
{
  static const uint32_t n16[16] = {0, 1, 2, 3, 5, 6, 7, 8, 10, 11, 12, 13, 15, 16, 17, 18};
  switch (pattern) {
    case 0: // A
    case 2: // C
      l = (idx % 2 == 0 ? 2 : 8) + 14 * (idx / 2);
      return true;
    case 1: { // B
      static const uint32_t f[4] = {4, 8, 16, 20};
      l                          = f[idx % 4] + 28 * (idx / 4);
      return true;
    }
    case 3: { // D
      static const uint32_t f[4] = {4, 8, 16, 20};
      if (idx >= 64) {
        return false;
      }
      l = f[idx % 4] + 28 * n16[idx / 4];
      return true;
    }
    case 4: { // E
      static const uint32_t f[8] = {8, 12, 16, 20, 32, 36, 40, 44};
      if (idx >= 128) {
        return false;
      }
      l = f[idx % 8] + 56 * n16[idx / 8];
      return true;
    }
    default:
      return false;
  }
}

uint32_t scs_khz(uint32_t scs)
{
  return 15u << scs;
}

// Position of the block in its slot after the reference's assertions (ssb_processor_impl.cpp:32-45,
// ssb_get_k_first ssb_mapping.h:116-171).
int position(const srs_amd_ssb_pdu& p, uint32_t& l0, uint32_t& k0)
{
  uint32_t l_burst = 0;
  if (p.pattern_case > 4) {
    return fail(SRS_AMD_EINVAL, "Invalid SSB pattern case %u.", p.pattern_case);
  }
  if (!l_first(p.pattern_case, p.ssb_idx, l_burst)) {
    return fail(SRS_AMD_EINVAL, "SSB index %u out of range.", p.ssb_idx);
  }
  if (p.numerology > 4) {
    return fail(SRS_AMD_EINVAL, "Invalid numerology %u.", p.numerology);
  }
  const uint32_t slots_hrf = 5u << p.numerology;
  if (p.slot_index >= 2 * slots_hrf || p.sfn > 1023) {
    return fail(SRS_AMD_EINVAL, "Invalid slot %u.%u of numerology %u.", p.sfn, p.slot_index, p.numerology);
  }
  if (l_burst / NSYMB != p.slot_index % slots_hrf) {
    return fail(SRS_AMD_EINVAL, "Invalid slot index (%u) for SSB index %u", p.slot_index % slots_hrf, l_burst);
  }
  l0 = l_burst % NSYMB;
  // frequency range and SSB SCS of the pattern (ssb_properties.h: to_frequency_range, to_subcarrier_spacing)
  const bool     fr1     = p.pattern_case < 3;
  const uint32_t ssb_scs = p.pattern_case == 0 ? 0u : (p.pattern_case < 3 ? 1u : (p.pattern_case == 3 ? 3u : 4u));
  if (p.common_scs > 4 || (fr1 ? p.common_scs > 2 : p.common_scs < 2)) {
    return fail(SRS_AMD_EINVAL, "Unsupported combination of FR%d and  Common SCS %ukHz.", fr1 ? 1 : 2,
                p.common_scs <= 4 ? scs_khz(p.common_scs) : 0u);
  }
  if (p.offset_to_pointA > 2199) {
    return fail(SRS_AMD_EINVAL, "Invalid offset to Point A %u (max 2199)", p.offset_to_pointA);
  }
  if (p.subcarrier_offset > (fr1 ? 23u : 11u)) {
    return fail(SRS_AMD_EINVAL, "Invalid subcarrier offset %u for FR%d (max %u)", p.subcarrier_offset, fr1 ? 1 : 2,
                fr1 ? 23u : 11u);
  }
  const uint32_t pa_khz  = fr1 ? 15u : 60u;
  const uint32_t sco_khz = fr1 ? 15u : scs_khz(p.common_scs);
  const uint32_t k15     = (p.offset_to_pointA * 12 * pa_khz + p.subcarrier_offset * sco_khz) / 15;
  if ((k15 * 15) % scs_khz(ssb_scs) != 0) {
    return fail(SRS_AMD_EINVAL,
                "Unsupported combination of FR%d, SSB SCS %ukHz, Common SCS %ukHz, offsetToPointA %u and "
                "ssb-SubcarrierOffset %u.",
                fr1 ? 1 : 2, scs_khz(ssb_scs), scs_khz(p.common_scs), p.offset_to_pointA, p.subcarrier_offset);
  }
  k0 = k15 * 15 / scs_khz(ssb_scs);
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_ssb_processor_create(srs_amd_ssb_processor** proc, int device)
{
  if (proc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *proc  = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* p                   = new srs_amd_ssb_processor();
  p->device                 = device;
  std::vector<uint32_t> j   = gold_jump_tables();
  std::vector<uint8_t>  seq = m_sequences();
  uint8_t               idx[SSB_K];
  for (uint32_t k = 0; k != SSB_K; ++k) {
    idx[k] = static_cast<uint8_t>(k);
  }
  rc = srs_amd_polar_interleave(p->perm, idx, SSB_K, 0);
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_polar_code_create(&p->code, SSB_K, SSB_E, 9, 0, device); // pbch_encoder_impl.h:99
  }
  if (rc != SRS_AMD_OK) {
    delete p;
    return rc;
  }
  hipError_t e = hipMalloc(&p->d_jump, j.size() * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = hipMemcpy(p->d_jump, j.data(), j.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipMalloc(&p->d_seq, seq.size());
  }
  if (e == hipSuccess) {
    e = hipMemcpy(p->d_seq, seq.data(), seq.size(), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "SSB processor tables");
  }
  *proc = p;
  return SRS_AMD_OK;
}

void srs_amd_ssb_processor_destroy(srs_amd_ssb_processor* proc)
{
  delete proc;
}

int srs_amd_ssb_position(const srs_amd_ssb_pdu* pdu, uint32_t* first_symbol, uint32_t* first_subcarrier)
{
  if (pdu == nullptr || first_symbol == nullptr || first_subcarrier == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  return position(*pdu, *first_symbol, *first_subcarrier);
}

int srs_amd_ssb_process_slot(srs_amd_ssb_processor* proc,
                             const srs_amd_ssb_pdu* pdus,
                             uint32_t               nof_pdus,
                             uint32_t*              d_grids,
                             uint64_t               grid_stride,
                             uint32_t               nof_grids,
                             uint32_t               nof_grid_ports,
                             uint32_t               nof_subc,
                             void*                  stream)
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
  std::vector<ssb_desc>       desc(nof_pdus);
  for (uint32_t i = 0; i != nof_pdus; ++i) {
    const srs_amd_ssb_pdu& p  = pdus[i];
    uint32_t               l0 = 0, k0 = 0;
    const int              rc = position(p, l0, k0);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    if (p.d_grid == nullptr && (d_grids == nullptr || p.grid >= nof_grids)) {
      return fail(SRS_AMD_EINVAL, "PDU %u: grid index %u out of range (or no grid).", i, p.grid);
    }
    if (k0 + SSB_SC > nof_subc) {
      return fail(SRS_AMD_EINVAL, "PDU %u: the block's subcarriers %u..%u exceed the grid (%u).", i, k0, k0 + SSB_SC - 1,
                  nof_subc);
    }
    if (p.phys_cell_id > 1007 || (p.L_max != 4 && p.L_max != 8 && p.L_max != 64) || p.nof_ports == 0 ||
        p.nof_ports > 4) {
      return fail(SRS_AMD_EINVAL, "PDU %u: invalid PCI %u, L_max %u or %u ports.", i, p.phys_cell_id, p.L_max,
                  p.nof_ports);
    }
    ssb_desc& d = desc[i];
    d           = ssb_desc{};
    for (uint32_t k = 0; k != 24; ++k) {
      d.mib[k] = p.mib_payload[k] & 1u;
    }
    d.sfn     = p.sfn;
    d.hrf     = p.slot_index >= (5u << p.numerology) ? 1u : 0u; // slot_point::is_odd_hrf
    d.ssb_idx = p.ssb_idx;
    d.L_max   = p.L_max;
    d.k_ssb   = p.subcarrier_offset;
    d.pci     = p.phys_cell_id;
    // pbch_encoder_impl.cpp:80-90: M = A - 3 (A - 6 for L_max 64), v = 2 x the SFN's 3rd LSB + its 2nd LSB
    const uint32_t M = p.L_max == 64 ? SSB_A - 6 : SSB_A - 3;
    d.enc_offset     = M * (2 * ((p.sfn >> 2) & 1u) + ((p.sfn >> 1) & 1u));
    std::memcpy(d.perm, proc->perm, SSB_K);
    d.grid        = p.d_grid != nullptr ? p.d_grid : d_grids + p.grid * grid_stride;
    d.port_stride = NSYMB * nof_subc;
    d.nof_subc    = nof_subc;
    d.k0          = k0;
    d.l0          = l0;
    d.nof_ports   = p.nof_ports;
    for (uint32_t k = 0; k != p.nof_ports; ++k) {
      if (p.ports[k] >= nof_grid_ports) {
        return fail(SRS_AMD_EINVAL, "PDU %u: port %u outside the grid's %u ports.", i, p.ports[k], nof_grid_ports);
      }
      d.ports[k] = p.ports[k];
    }
    d.mod_offset = (p.ssb_idx & 0x7u) * SSB_E; // pbch_modulator_impl.cpp:35
    // dmrs_pbch_processor_impl.cpp:29-40
    uint64_t i_ssb = (p.ssb_idx & 0x3u) + 4ull * d.hrf;
    if (p.L_max == 8 || p.L_max == 64) {
      i_ssb = p.ssb_idx & 0x7u;
    }
    d.c_init_dmrs = static_cast<uint32_t>((((i_ssb + 1) * ((p.phys_cell_id / 4ull) + 1)) << 11) + ((i_ssb + 1) << 6) +
                                          (p.phys_cell_id % 4));
    d.pss_amp     = std::pow(10.0F, p.beta_pss_dB / 20.0F); // convert_dB_to_amplitude (math_utils.h:118-121)
    const uint32_t nid1 = p.phys_cell_id / 3, nid2 = p.phys_cell_id % 3;
    d.pss_m             = (43 * nid2) % SSB_SEQLEN;
    d.sss_m0            = 15 * (nid1 / 112) + 5 * nid2;
    d.sss_m1            = nid1 % 112;
    d.msg_offset        = i * SSB_K;
    d.cw_offset         = i * SSB_E;
  }
  // buffer layout: descriptors | messages (K per block) | codewords (E per block)
  const size_t o_msg  = align_up(sizeof(ssb_desc) * nof_pdus, 256);
  const size_t o_cw   = o_msg + align_up(static_cast<size_t>(SSB_K) * nof_pdus, 256);
  const size_t total  = o_cw + align_up(static_cast<size_t>(SSB_E) * nof_pdus, 256);
  const size_t staged = sizeof(ssb_desc) * nof_pdus;
  auto         s      = static_cast<hipStream_t>(stream);
  hipError_t   e      = hipSetDevice(proc->device);
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
    return hip_fail(e, "SSB processor scratch");
  }
  call_scope scope(proc->order, nullptr, s);
  std::memcpy(proc->stage.at<uint8_t>(0), desc.data(), staged);
  auto* base   = proc->buf.as<uint8_t>();
  auto* d_desc = reinterpret_cast<const ssb_desc*>(base);
  e            = proc->stage.upload(base, staged, s);
  if (e == hipSuccess) {
    e = launch_ssb_encode(d_desc, nof_pdus, base + o_msg, proc->d_jump, s);
  }
  int rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ssb_encode_kernel launch");
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_polar_encode_batch(proc->code, base + o_msg, SSB_K, base + o_cw, SSB_E, nof_pdus, stream);
  }
  if (rc == SRS_AMD_OK) {
    e  = launch_ssb_map(d_desc, nof_pdus, base + o_cw, proc->d_seq, proc->d_jump, s);
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ssb_map_kernel launch");
  }
  const hipError_t done = scope.close();
  return rc != SRS_AMD_OK ? rc : (done == hipSuccess ? SRS_AMD_OK : hip_fail(done, "SSB completion event"));
}

int srs_amd_ssb_process(srs_amd_ssb_processor* proc,
                        const srs_amd_ssb_pdu* pdu,
                        uint32_t*              grid,
                        uint32_t               nof_ports,
                        uint32_t               nof_subc)
{
  if (proc == nullptr || pdu == nullptr || grid == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t                bytes = sizeof(uint32_t) * nof_ports * NSYMB * nof_subc;
  std::lock_guard<std::mutex> host_lock(proc->host_mtx);
  hipError_t                  e = hipSetDevice(proc->device);
  if (e == hipSuccess) {
    e = proc->host_grid.ensure(bytes);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "SSB processor grid");
  }
  e = hipMemcpyAsync(proc->host_grid.ptr, grid, bytes, hipMemcpyHostToDevice, proc->stream);
  if (e != hipSuccess) {
    return hip_fail(e, "SSB grid upload");
  }
  srs_amd_ssb_pdu p = *pdu;
  p.grid            = 0;
  p.d_grid          = nullptr;
  int rc = srs_amd_ssb_process_slot(proc, &p, 1, proc->host_grid.as<uint32_t>(), 0, 1, nof_ports, nof_subc,
                                    proc->stream);
  if (rc == SRS_AMD_OK) {
    e  = hipMemcpyAsync(grid, proc->host_grid.ptr, bytes, hipMemcpyDeviceToHost, proc->stream);
    e  = e == hipSuccess ? hipStreamSynchronize(proc->stream) : e;
    rc = e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "SSB grid download");
  } else {
    (void)hipStreamSynchronize(proc->stream);
  }
  return rc;
}

} // extern "C"
