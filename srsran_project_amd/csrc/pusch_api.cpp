// pusch_api.cpp -- C-ABI of the MI355X PUSCH decoder (include/srsran_amd/sch.h),
// pusch_decoder_impl (lib/phy/upper/channel_processors/pusch/pusch_decoder_impl.cpp)
// for a batch of transport blocks:
//   1. rate dematching + HARQ combining    srs_amd_ldpc_rate_dematch_batch into the soft buffers
//   2. LDPC decoding, CB CRC early stop    srs_amd_ldpc_decode_batch
//      (without early stop: decode, then a CRC of the K - F message bits,
//       pusch_codeblock_decoder.cpp:75-86)
//   3. CB status, statistics, concatenation and TB CRC24A   assemble_kernel (sch.hip)
// Soft buffer of one TB: C rows of soft_row_layout::row_bytes:
//   [N_short*Z soft LLRs | ceil(K/8) message bytes | int32 CB CRC flag]
// (the codeblock soft bits, data bits and CRC flags of the reference's rx_buffer).
#include "srsran_amd/crc.h"
#include "srsran_amd/ldpc.h"
#include "srsran_amd/ldpc_rate_matching.h"
#include "srsran_amd/sch.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "crc_internal.h"
#include "device_buffer.h"
#include "ldpc_codec_internal.h"
#include "ldpc_common.h"
#include "rate_matching_common.h"
#include "pusch_processor_args.h"
#include "sch_args.h"
#include <cstring>
#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

using namespace srs_amd;

struct srs_amd_pusch_decoder {
  int                          device = 0;
  int                          arith  = 0;
  hipStream_t                  stream = nullptr;
  srs_amd_crc_calculator*      crc[3] = {nullptr, nullptr, nullptr}; // CRC16, CRC24A, CRC24B
  srs_amd_ldpc_rate_dematcher* dm     = nullptr;
  srs_amd_ldpc_decoder*        dec[2] = {nullptr, nullptr}; // force_decoding 0 / 1
  device_buffer                soft, msgs, iters, checks, arrays, results, host_io, tb_acc, slot_desc;
  device_buffer                harq_prev; // slot form: the CRC flags of HARQ codeblocks before this transmission
  geometry_cache               rm_geo; // last geometry written into arrays (rm_arrays_kernel)
  stream_order                 order; // scratch reuse across the callers' streams
  stream_fan                   fan;   // srs_amd_pusch_decode_slot: concurrent LDPC bucket launches
  std::mutex                   mtx;
  // srs_amd_pusch_decode_slot: descriptors staged in pinned memory, reused once their upload completed
  pinned_stage hstage; // descriptors staged in pinned memory (a ring: each reused once its upload completed)
  ~srs_amd_pusch_decoder()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    for (auto* c : crc) {
      srs_amd_crc_calculator_destroy(c);
    }
    srs_amd_ldpc_rate_dematcher_destroy(dm);
    srs_amd_ldpc_decoder_destroy(dec[0]);
    srs_amd_ldpc_decoder_destroy(dec[1]);
  }
};

namespace {

soft_row_layout layout_of(const srs_amd_sch_plan* p)
{
  soft_row_layout l{};
  l.soft_bytes  = srs_amd_ldpc_codeblock_length(p->base_graph, p->lifting_size);
  l.msg_offset  = static_cast<uint32_t>(align_up(l.soft_bytes, 64));
  l.flag_offset = static_cast<uint32_t>(l.msg_offset + align_up((p->segment_length + 7) / 8, 16));
  l.row_bytes   = static_cast<uint32_t>(align_up(l.flag_offset + 4, 64));
  return l;
}

// Length of the soft-buffer prefix that can hold non-zero LLRs after this call's rate dematching,
// rounded up to whole lifting-size nodes (so the decoder's clamped-node load is unchanged), or the
// whole row when it cannot be bounded.  New data with k0 = 0 and no circular wrap writes LLRs to
// [0, E), +inf fillers to [nof_info, nof_sys) and data to [nof_sys, E + F); the rest of the row is
// zeroed when the buffer is fresh, or when E covers the information bits of a full-length buffer
// (nothing of the old contents survives, see ldpc_rate_dematch_kernel).  The decoder then scans
// (ldpc_decoder_impl.cpp:86) only this prefix, and a short prefix bounds its layer count.
uint32_t llr_prefix(const srs_amd_sch_plan* p, const soft_row_layout& lay, bool new_data, bool fresh)
{
  rm_geometry g{};
  if (!new_data || make_rm_geometry(g, p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                    p->nof_filler_bits) != nullptr) {
    return lay.soft_bytes;
  }
  const uint32_t C     = p->nof_segments;
  const uint32_t e_min = p->nof_short_segments > 0 ? p->rm_length_short : p->rm_length_long;
  const uint32_t e_max = p->nof_short_segments < C ? p->rm_length_long : p->rm_length_short;
  if (g.k0 != 0 || e_max + g.F > g.Ncb || !(fresh || (e_min >= g.nof_info && g.Ncb == g.N))) {
    return lay.soft_bytes;
  }
  const uint32_t Z   = p->lifting_size;
  const uint32_t end = std::max(e_max + g.F, g.nof_sys);
  const uint32_t lo  = (p->base_graph == 1 ? 24u : 12u) * Z; // ldpc_decoder_impl.cpp:78 minimum input length
  return std::min(lay.soft_bytes, std::max(lo, (end + Z - 1) / Z * Z));
}

// CRC polynomial of the decoder's early stop and of the CB check (select_crc, pusch_decoder_impl.cpp:35-46).
// SRSRAN_AMD_DEMATCH_FUSED=0 keeps the separate dematch launch (read per call: A/B timing, parity tests).
bool dematch_fused_enabled()
{
  const char* e = std::getenv("SRSRAN_AMD_DEMATCH_FUSED");
  return e == nullptr || e[0] != '0';
}

int crc_poly_of(const srs_amd_sch_plan* p)
{
  return p->nof_segments > 1 ? 1 : (p->tbs > 3824 ? 0 : 3);
}

int crc_index_of(const srs_amd_sch_plan* p)
{
  return p->nof_segments > 1 ? 2 : (p->tbs > 3824 ? 1 : 0);
}

int check_plan(const srs_amd_sch_plan* p)
{
  if (p == nullptr || p->nof_segments == 0 || p->lifting_size == 0) {
    return fail(SRS_AMD_EINVAL, "plan not computed (srs_amd_sch_plan_compute)");
  }
  return SRS_AMD_OK;
}

int decode_locked(srs_amd_pusch_decoder*              d,
                  const srs_amd_sch_plan*             p,
                  const srs_amd_pusch_decoder_config* cfg,
                  uint8_t*                            d_tbs,
                  uint32_t                            tb_stride,
                  srs_amd_pusch_decoder_result*       d_results,
                  const int8_t*                       d_llrs,
                  uint32_t                            llr_stride,
                  int8_t*                             d_soft,
                  int32_t*                            d_cb_iterations,
                  uint32_t                            nof_tbs,
                  hipStream_t                         stream)
{
  const uint32_t        C          = p->nof_segments;
  const uint32_t        rows       = nof_tbs * C;
  const soft_row_layout lay        = layout_of(p);
  const uint32_t        msg_stride = static_cast<uint32_t>(align_up((p->segment_length + 7) / 8, 64));
  const bool            internal   = d_soft == nullptr;
  hipError_t            he         = hipSetDevice(d->device);
  if (internal && he == hipSuccess) {
    he     = d->soft.ensure(static_cast<size_t>(rows) * lay.row_bytes);
    d_soft = d->soft.as<int8_t>();
  }
  if (he == hipSuccess) {
    he = d->msgs.ensure(static_cast<size_t>(rows) * msg_stride);
  }
  if (he == hipSuccess) {
    he = d->iters.ensure(sizeof(int32_t) * rows);
  }
  if (he == hipSuccess) {
    he = d->checks.ensure(sizeof(uint32_t) * rows);
  }
  if (he == hipSuccess) {
    he = d->arrays.ensure(sizeof(uint32_t) * 2 * rows);
  }
  if (he == hipSuccess) {
    he = d->tb_acc.ensure_zeroed(sizeof(uint32_t) * nof_tbs);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PUSCH decoder scratch");
  }
  call_scope scope(d->order, nullptr, stream);
  he = d->order.begin(stream);
  if (he == hipSuccess) {
    const uint32_t key[6] = {nof_tbs, C, p->nof_short_segments, p->rm_length_short, p->rm_length_long, llr_stride};
    if (d->rm_geo.stale(d->arrays.ptr, key, 6)) {
      he = launch_rm_arrays(d->arrays.as<uint32_t>(), nof_tbs, C, p->nof_short_segments, p->rm_length_short,
                            p->rm_length_long, llr_stride, stream);
      if (he != hipSuccess) {
        d->rm_geo.invalidate();
      }
    }
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PUSCH decoder rate-matching arrays");
  }
  // 1. Rate dematching + combining.
  srs_amd_codeblock_metadata md{p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                p->nof_filler_bits};
  // Internal buffers stand for a fresh (zeroed) rx_buffer: nothing of theirs is read.
  // An internal (fresh) buffer is read back only by the LDPC decoder, over the provably non-zero prefix:
  // the dematcher writes just that prefix.
  const uint32_t prefix = llr_prefix(p, lay, cfg->new_data != 0, internal);
  // New data into an internal (fresh) buffer with k0 = 0 and no circular wrap, decoded by the high-rate kernel:
  // the dematched row is [LLRs | +inf fillers | LLRs | zeros], which the decoder builds in LDS from the codeword
  // itself (decode_args::cw_llrs) -- no dematch launch, no soft row written to and read back from HBM.
  ldpc_cw_rows cw{};
  bool         fuse = false;
  if (internal && cfg->new_data && dematch_fused_enabled() && ldpc_hr_takes(static_cast<int>(p->base_graph),
                                                                             static_cast<int>(p->lifting_size), prefix)) {
    rm_geometry g{};
    const uint32_t e_max = std::max(p->rm_length_long, p->nof_short_segments > 0 ? p->rm_length_short : 0u);
    fuse = make_rm_geometry(g, p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                            p->nof_filler_bits) == nullptr &&
           g.k0 == 0 && e_max <= g.L && e_max + g.F <= prefix;
    cw = ldpc_cw_rows{d_llrs, d->arrays.as<uint32_t>() + rows, d->arrays.as<uint32_t>(), p->modulation_order,
                      g.nof_info, g.F};
  }
  int rc = SRS_AMD_OK;
  if (!fuse) {
    rc = rate_dematch_batch_ex(d->dm, &md, cfg->new_data ? 1 : 0, d_llrs, d->arrays.as<uint32_t>() + rows,
                               d->arrays.as<uint32_t>(), d_soft, lay.row_bytes, rows, stream, internal,
                               internal ? prefix : 0);
  }
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // 2. LDPC decoding (select_crc, pusch_decoder_impl.cpp:35-46).
  const int crc_index = crc_index_of(p);
  const int crc_poly  = crc_poly_of(p);
  srs_amd_ldpc_decoder_config dc{};
  dc.base_graph      = p->base_graph;
  dc.lifting_size    = p->lifting_size;
  dc.nof_filler_bits = p->nof_filler_bits;
  dc.nof_crc_bits    = C > 1 ? p->nof_crc_bits : p->nof_tb_crc_bits;
  dc.max_iterations  = cfg->nof_ldpc_iterations;
  srs_amd_ldpc_decoder* dec = d->dec[cfg->force_decoding ? 1 : 0];
  // a retransmission does not decode again the codeblocks whose CRC passed earlier (their soft-buffer
  // flag holds the iteration count of that decoding), pusch_decoder_impl.cpp:330-345
  const bool skip = !cfg->new_data && !internal;
  rc = ldpc_decode_batch_ex(dec, &dc, cfg->use_early_stop ? crc_poly : SRS_AMD_NO_CRC, d_soft, lay.row_bytes, nullptr,
                            prefix, d->msgs.as<uint8_t>(), msg_stride,
                            d->iters.as<int32_t>(), nullptr, rows, stream,
                            skip ? reinterpret_cast<const uint8_t*>(d_soft) + lay.flag_offset : nullptr, lay.row_bytes,
                            nullptr, fuse ? &cw : nullptr);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (!cfg->use_early_stop) {
    rc = srs_amd_crc_calculate_batch(d->crc[crc_index], d->checks.as<uint32_t>(), d->msgs.as<uint8_t>(), msg_stride,
                                     p->segment_length - p->nof_filler_bits, rows, stream);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  // 3. Concatenation and TB CRC.
  assemble_args a{};
  a.msgs           = d->msgs.as<uint8_t>();
  a.iters          = d->iters.as<int32_t>();
  a.crc_checks     = cfg->use_early_stop ? nullptr : d->checks.as<uint32_t>();
  a.soft           = internal ? nullptr : reinterpret_cast<uint8_t*>(d_soft); // no HARQ state to keep
  a.tbs            = d_tbs;
  a.results        = d_results;
  a.cb_iterations  = d_cb_iterations;
  a.crc24a_table   = crc_device_table(d->crc[1]);
  a.acc            = d->tb_acc.as<uint32_t>();
  a.lay            = lay;
  a.msg_stride     = msg_stride;
  a.tb_stride      = tb_stride;
  a.nof_segments   = C;
  a.cb_info_bits   = p->cb_info_bits;
  a.tbs_bits       = p->tbs;
  a.max_iterations = cfg->nof_ldpc_iterations;
  a.new_data       = cfg->new_data ? 1 : 0;
  he               = launch_assemble(a, nof_tbs, stream);
  if (he == hipSuccess) {
    he = scope.close();
  }
  return he == hipSuccess ? SRS_AMD_OK : hip_fail(he, "assemble_kernel launch");
}

// srs_amd_pusch_decode_slot: every codeblock of the slot is one row of the decoder scratch (soft rows of
// stride S, message rows of stride M), rows grouped by LDPC decoder bucket (BG, Z, CRC, bounded prefix), each
// UE's C rows
// contiguous.  Descriptors built on the host, uploaded once from pinned memory.
int decode_slot_locked(srs_amd_pusch_decoder*              d,
                       const srs_amd_pusch_decoder_config* cfg,
                       const srs_amd_pusch_ue*             ues,
                       uint32_t                            U,
                       const int8_t*                       d_llrs,
                       uint8_t*                            d_tbs,
                       srs_amd_pusch_decoder_result*       d_results,
                       const uint32_t*                     cb_offsets,
                       int32_t*                            d_cb_iterations,
                       hipStream_t                         stream,
                       const slot_harq*                    harq,
                       const slot_ue_patch*                patches,
                       uint32_t                            nof_patches)
{
  // HARQ UEs (a caller soft buffer): their codeblocks decode in internal rows like the others, the soft bits
  // gathered from / scattered to the caller's rows around the rate dematcher / decoder (harq_* kernels), full-length
  // rows (the whole soft buffer is state), the rate dematcher combining into the gathered bits (per-row flags)
  auto harq_of = [&](uint32_t u) -> const slot_harq* {
    return harq != nullptr && harq[u].soft != nullptr ? &harq[u] : nullptr;
  };
  // Z = 384 rows: one uniform launch per (BG, CRC, bounded prefix) -- the compile-time Z = 384 kernels,
  // the high-rate one for bounded prefixes; Z < 384 rows: one mixed-Z launch per (BG, kernel class: the
  // packed kernel's waves per codeblock), each row with its own Z, CRC, input length and filler bits.
  struct bucket {
    uint32_t              bg, Z; // Z: the lifting size (uniform) or the largest one (mixed)
    int                   poly;  // uniform buckets
    bool                  mixed;
    uint32_t              prefix = 0, row0 = 0, rows = 0;
    std::vector<uint32_t> ues;
  };
  std::vector<bucket>                                          buckets;
  std::map<std::tuple<uint32_t, uint32_t, int, bool>, size_t> bucket_of;
  std::vector<uint32_t>                                        ue_prefix(U);
  uint32_t                                             S = 0, M = 0, R = 0, max_tb_bits = 0;
  for (uint32_t u = 0; u < U; ++u) {
    const srs_amd_sch_plan* p  = &ues[u].plan;
    int                     rc = check_plan(p);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    rm_geometry g{};
    if (const char* msg = make_rm_geometry(g, p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                           p->nof_filler_bits)) {
      return fail(SRS_AMD_EINVAL, "UE %u: %s", u, msg);
    }
    if (ues[u].llr_offset + p->cw_length > 0xffffffffull) {
      return fail(SRS_AMD_EINVAL, "UE %u: LLR span exceeds 2^32 bytes", u);
    }
    const soft_row_layout lay    = layout_of(p);
    const slot_harq*      h      = harq_of(u);
    const uint32_t        prefix = h != nullptr ? lay.soft_bytes : llr_prefix(p, lay, true, true);
    ue_prefix[u]                = prefix;
    // rows whose non-zero prefix is bounded decode apart from full rows: the bucket's LLR length is its
    // longest prefix, and a bounded one selects the high-rate decoder kernel
    const bool mixed = p->lifting_size < 384;
    // mixed launches: one per (BG, kernel class) -- the packed kernel's waves per codeblock, or (Z not a
    // multiple of 4) the one-row-per-lane kernel's
    const int  pkw   = ldpc_pk_waves(static_cast<int>(p->base_graph), static_cast<int>(p->lifting_size));
    const auto key   = mixed ? std::make_tuple(p->base_graph, pkw > 0 ? static_cast<uint32_t>(pkw)
                                                                     : 10u + (p->lifting_size + 63) / 64, -1, false)
                             : std::make_tuple(p->base_graph, p->lifting_size, crc_poly_of(p), prefix < lay.soft_bytes);
    auto       it    = bucket_of.find(key);
    if (it == bucket_of.end()) {
      it = bucket_of.emplace(key, buckets.size()).first;
      buckets.push_back(bucket{p->base_graph, p->lifting_size, mixed ? -1 : crc_poly_of(p), mixed});
    }
    bucket& b = buckets[it->second];
    b.Z       = std::max(b.Z, p->lifting_size);
    b.ues.push_back(u);
    b.rows += p->nof_segments;
    b.prefix    = std::max(b.prefix, prefix);
    S           = std::max(S, static_cast<uint32_t>(align_up(lay.soft_bytes, 64)));
    M           = std::max(M, static_cast<uint32_t>(align_up((p->segment_length + 7) / 8, 64)));
    R          += p->nof_segments;
    max_tb_bits = std::max(max_tb_bits, p->tbs);
  }
  // the TB assembly runs one grid row per UE, the codeblock kernels one grid row per codeblock
  if (U > 65535 || R > 65535) {
    return fail(SRS_AMD_EINVAL, "%u UEs / %u codeblocks exceed the 65535 of one slot batch", U, R);
  }
  // host descriptors: per row E, input offset, geometry, filler bits; geometries + write ends; per-TB
  std::vector<uint32_t>                                                              row_E(R), row_in(R), row_geo(R);
  std::vector<uint32_t>                                                              row_len(R);
  std::vector<int32_t>                                                               row_F(R);
  std::vector<ldpc_row_desc>                                                         row_desc(R);
  std::vector<rm_geometry>                                                           geos;
  std::vector<uint32_t>                                                              geo_end;
  std::map<std::tuple<size_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>, uint32_t> geo_of;
  std::vector<tb_desc>                                                               tds(U);
  std::vector<uint32_t>                                                              segE, segOff;
  std::vector<uint8_t>                                                               row_flags(R, 3); // new, fresh
  std::vector<harq_row_desc>                                                         hrows;
  std::vector<harq_tb_desc>                                                          htbs;
  uint32_t                                                                           max_soft = 0;
  uint32_t                                                                           row = 0;
  for (size_t bi = 0; bi < buckets.size(); ++bi) {
    bucket& b = buckets[bi];
    b.row0    = row;
    for (uint32_t u : b.ues) {
      const srs_amd_sch_plan* p = &ues[u].plan;
      // dematcher write end: the longest prefix of a uniform bucket (its decoder reads that many LLRs of
      // every row), each UE's own prefix in a mixed bucket (per-row input lengths)
      const uint32_t wend = b.mixed ? ue_prefix[u] : b.prefix;
      // (a mixed-Z bucket holds several lifting sizes whose write ends can coincide: Z is part of the key)
      const auto     gkey = std::make_tuple(bi, p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                            p->nof_filler_bits, wend);
      auto       git  = geo_of.find(gkey);
      if (git == geo_of.end()) {
        rm_geometry g{};
        (void)make_rm_geometry(g, p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                               p->nof_filler_bits);
        git = geo_of.emplace(gkey, static_cast<uint32_t>(geos.size())).first;
        geos.push_back(g);
        geo_end.push_back(wend);
      }
      segE.resize(p->nof_segments);
      segOff.resize(p->nof_segments);
      (void)srs_amd_sch_plan_segments(p, segE.data(), segOff.data());
      tds[u] = tb_desc{ues[u].tb_offset, row,         p->nof_segments, p->cb_info_bits, p->tbs, p->nof_tb_crc_bits,
                       p->zero_pad,       (p->segment_length + 7) / 8, cb_offsets ? cb_offsets[u] : 0u};
      const slot_harq* h = harq_of(u);
      if (h != nullptr) {
        const soft_row_layout lay = layout_of(p);
        const uint32_t lazy = h->lazy && h->new_data ? 1u : 0u;
        htbs.push_back(harq_tb_desc{reinterpret_cast<uint8_t*>(h->soft), u, p->nof_segments, lay.row_bytes,
                                    lay.flag_offset, lazy, row, lay.soft_bytes});
        max_soft = std::max(max_soft, lay.soft_bytes);
        for (uint32_t r = 0; r < p->nof_segments; ++r) {
          hrows.push_back(harq_row_desc{reinterpret_cast<uint8_t*>(h->soft) + static_cast<size_t>(r) * lay.row_bytes,
                                        row + r, lay.soft_bytes, lay.msg_offset, lay.flag_offset - lay.msg_offset,
                                        lay.flag_offset, h->new_data ? 1u : 0u, lazy, row, p->nof_segments});
          row_flags[row + r] = h->new_data ? 3 : 0;
        }
      }
      for (uint32_t r = 0; r < p->nof_segments; ++r, ++row) {
        row_E[row]   = segE[r];
        row_in[row]  = static_cast<uint32_t>(ues[u].llr_offset) + segOff[r];
        row_geo[row] = git->second;
        row_F[row]   = static_cast<int32_t>(p->nof_filler_bits);
        row_len[row] = wend;
        ldpc_mixed_row(&row_desc[row], p->base_graph, p->lifting_size,
                       cfg->use_early_stop ? crc_poly_of(p) : SRS_AMD_NO_CRC);
      }
    }
  }
  const size_t o_E   = 0;
  const size_t o_in  = o_E + align_up(sizeof(uint32_t) * R, 16);
  const size_t o_geo = o_in + align_up(sizeof(uint32_t) * R, 16);
  const size_t o_F   = o_geo + align_up(sizeof(uint32_t) * R, 16);
  const size_t o_G   = o_F + align_up(sizeof(int32_t) * R, 16);
  const size_t o_GE  = o_G + align_up(sizeof(rm_geometry) * geos.size(), 16);
  const size_t o_TD  = o_GE + align_up(sizeof(uint32_t) * geos.size(), 16);
  const size_t o_LEN = o_TD + align_up(sizeof(tb_desc) * U, 16);
  const size_t o_RD  = o_LEN + align_up(sizeof(uint32_t) * R, 16);
  const size_t o_RF  = o_RD + align_up(sizeof(ldpc_row_desc) * R, 16);
  const size_t o_HR  = o_RF + align_up(R, 16);
  const size_t o_HT  = o_HR + align_up(sizeof(harq_row_desc) * hrows.size(), 16);
  const size_t o_PT  = align_up(hrows.empty() ? o_RF : o_HT + sizeof(harq_tb_desc) * htbs.size(), 16);
  const size_t total = o_PT + sizeof(slot_row_patch) * nof_patches;
  for (uint32_t q = 0; q < nof_patches; ++q) {
    if (patches[q].ue >= U || patches[q].sel == nullptr || patches[q].cand_E == nullptr || patches[q].cand_off == nullptr) {
      return fail(SRS_AMD_EINVAL, "slot decoder: invalid row patch %u", q);
    }
  }

  hipError_t he = hipSetDevice(d->device);
  // the next pinned staging buffer of the ring, free once its previous upload completed
  if (he == hipSuccess) {
    he = d->hstage.acquire(total);
  }
  if (he == hipSuccess) {
    he = d->slot_desc.ensure(total);
  }
  if (he == hipSuccess) {
    he = d->soft.ensure(static_cast<size_t>(R) * S);
  }
  if (he == hipSuccess) {
    he = d->msgs.ensure(static_cast<size_t>(R) * M);
  }
  if (he == hipSuccess) {
    he = d->iters.ensure(sizeof(int32_t) * R);
  }
  if (he == hipSuccess) {
    he = d->checks.ensure(sizeof(uint32_t) * R);
  }
  if (he == hipSuccess) {
    he = d->tb_acc.ensure_zeroed(sizeof(uint32_t) * U);
  }
  if (he == hipSuccess && !hrows.empty()) {
    he = d->harq_prev.ensure(sizeof(int32_t) * hrows.size());
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PUSCH slot decoder scratch");
  }
  auto* h = d->hstage.at<uint8_t>(0);
  std::memcpy(h + o_E, row_E.data(), sizeof(uint32_t) * R);
  std::memcpy(h + o_in, row_in.data(), sizeof(uint32_t) * R);
  std::memcpy(h + o_geo, row_geo.data(), sizeof(uint32_t) * R);
  std::memcpy(h + o_F, row_F.data(), sizeof(int32_t) * R);
  std::memcpy(h + o_G, geos.data(), sizeof(rm_geometry) * geos.size());
  std::memcpy(h + o_GE, geo_end.data(), sizeof(uint32_t) * geo_end.size());
  std::memcpy(h + o_TD, tds.data(), sizeof(tb_desc) * U);
  std::memcpy(h + o_LEN, row_len.data(), sizeof(uint32_t) * R);
  std::memcpy(h + o_RD, row_desc.data(), sizeof(ldpc_row_desc) * R);
  if (!hrows.empty()) {
    std::memcpy(h + o_RF, row_flags.data(), R);
    std::memcpy(h + o_HR, hrows.data(), sizeof(harq_row_desc) * hrows.size());
    std::memcpy(h + o_HT, htbs.data(), sizeof(harq_tb_desc) * htbs.size());
  }
  auto* dd = d->slot_desc.as<uint8_t>();
  for (uint32_t q = 0; q < nof_patches; ++q) {
    const uint32_t u = patches[q].ue;
    slot_row_patch rp{};
    rp.row_E      = reinterpret_cast<uint32_t*>(dd + o_E) + tds[u].row0;
    rp.row_in     = reinterpret_cast<uint32_t*>(dd + o_in) + tds[u].row0;
    rp.sel        = patches[q].sel;
    rp.cand_E     = patches[q].cand_E;
    rp.cand_off   = patches[q].cand_off;
    rp.llr_offset = static_cast<uint32_t>(ues[u].llr_offset);
    rp.C          = ues[u].plan.nof_segments;
    std::memcpy(h + o_PT + sizeof(slot_row_patch) * q, &rp, sizeof(rp));
  }
  call_scope scope(d->order, &d->fan, stream);
  he = d->order.begin(stream);
  if (he == hipSuccess) {
    he = d->hstage.upload(dd, total, stream);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PUSCH slot descriptors upload");
  }
  // 0. UEs whose UL-SCH geometry was selected on the device (CSI part 2): their rows' lengths / offsets
  if (nof_patches != 0) {
    he = launch_slot_row_patch(reinterpret_cast<const slot_row_patch*>(dd + o_PT), nof_patches, stream);
    if (he != hipSuccess) {
      return hip_fail(he, "slot_row_patch_kernel launch");
    }
  }
  // 1. Rate dematching of every codeblock of the slot, one launch (HARQ rows combining into their gathered bits).
  int8_t*   soft = d->soft.as<int8_t>();
  harq_args ha{};
  ha.rows     = reinterpret_cast<const harq_row_desc*>(dd + o_HR);
  ha.nof_rows = static_cast<uint32_t>(hrows.size());
  ha.tbs      = reinterpret_cast<const harq_tb_desc*>(dd + o_HT);
  ha.nof_tbs  = static_cast<uint32_t>(htbs.size());
  ha.internal = soft;
  ha.S        = S;
  ha.msgs     = d->msgs.as<uint8_t>();
  ha.M        = M;
  ha.iters    = d->iters.as<int32_t>();
  ha.prev     = d->harq_prev.as<int32_t>();
  ha.results  = d_results;
  if (ha.nof_rows != 0) {
    he = launch_harq_gather(ha, max_soft, stream);
    if (he != hipSuccess) {
      return hip_fail(he, "harq_gather_kernel launch");
    }
  }
  int rc = rate_dematch_ragged(d->dm, d_llrs, reinterpret_cast<const uint32_t*>(dd + o_in),
                               reinterpret_cast<const uint32_t*>(dd + o_E), reinterpret_cast<const uint32_t*>(dd + o_geo),
                               dd + o_G, reinterpret_cast<const uint32_t*>(dd + o_GE), soft, S, R, stream,
                               hrows.empty() ? nullptr : dd + o_RF);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // 2. LDPC decoding, one launch per (BG, Z, CRC, bounded prefix) bucket, fanned out over helper streams
  //    (largest buckets first, each to the least loaded stream).
  const int32_t*        d_F  = reinterpret_cast<const int32_t*>(dd + o_F);
  srs_amd_ldpc_decoder* ldpc = d->dec[cfg->force_decoding ? 1 : 0];
  std::vector<size_t>   by_size(buckets.size());
  for (size_t i = 0; i < by_size.size(); ++i) {
    by_size[i] = i;
  }
  std::sort(by_size.begin(), by_size.end(), [&](size_t x, size_t y) {
    return static_cast<uint64_t>(buckets[x].rows) * buckets[x].Z > static_cast<uint64_t>(buckets[y].rows) * buckets[y].Z;
  });
  he = d->fan.begin(stream, static_cast<int>(buckets.size()));
  if (he != hipSuccess) {
    return hip_fail(he, "PUSCH slot decoder stream fan-out");
  }
  uint64_t  load[stream_fan::FAN_STREAMS + 1] = {};
  const int width                             = d->fan.width();
  for (size_t bi : by_size) {
    const bucket& b  = buckets[bi];
    int           si = 0;
    for (int k = 1; k < width; ++k) {
      si = load[k] < load[si] ? k : si;
    }
    load[si] += static_cast<uint64_t>(b.rows) * b.Z;
    const hipStream_t bs = d->fan.stream(stream, si);
    if (b.mixed) {
      rc = ldpc_decode_mixed(ldpc, b.bg, b.Z, cfg->nof_ldpc_iterations, soft + static_cast<size_t>(b.row0) * S, S,
                             reinterpret_cast<const uint32_t*>(dd + o_LEN) + b.row0,
                             d->msgs.as<uint8_t>() + static_cast<size_t>(b.row0) * M, M,
                             d->iters.as<int32_t>() + b.row0, b.rows, bs, d_F + b.row0,
                             dd + o_RD + sizeof(ldpc_row_desc) * b.row0);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
      continue;
    }
    srs_amd_ldpc_decoder_config dc{};
    dc.base_graph     = b.bg;
    dc.lifting_size   = b.Z;
    dc.nof_crc_bits   = b.poly == 3 ? 16 : 24;
    dc.max_iterations = cfg->nof_ldpc_iterations;
    rc = ldpc_decode_batch_ex(ldpc, &dc, cfg->use_early_stop ? b.poly : SRS_AMD_NO_CRC,
                              soft + static_cast<size_t>(b.row0) * S, S, nullptr, b.prefix,
                              d->msgs.as<uint8_t>() + static_cast<size_t>(b.row0) * M, M,
                              d->iters.as<int32_t>() + b.row0, nullptr, b.rows, bs, nullptr, 0, d_F + b.row0);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  he = d->fan.end(stream);
  if (he != hipSuccess) {
    return hip_fail(he, "PUSCH slot decoder stream join");
  }
  // Without early stop: CRC of each decoded message (pusch_codeblock_decoder.cpp:75-86), per UE.
  if (!cfg->use_early_stop) {
    for (uint32_t u = 0; u < U; ++u) {
      const srs_amd_sch_plan* p = &ues[u].plan;
      rc = srs_amd_crc_calculate_batch(d->crc[crc_index_of(p)], d->checks.as<uint32_t>() + tds[u].row0,
                                       d->msgs.as<uint8_t>() + static_cast<size_t>(tds[u].row0) * M, M,
                                       p->segment_length - p->nof_filler_bits, p->nof_segments, stream);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
    }
  }
  // HARQ rows: soft bits back to the caller, earlier messages / fresh flags (before the assembly reads msgs / iters)
  if (ha.nof_rows != 0) {
    he = launch_harq_scatter(ha, max_soft, stream);
    if (he != hipSuccess) {
      return hip_fail(he, "harq_scatter_kernel launch");
    }
  }
  // 3. Concatenation and TB CRC, per-TB descriptors.
  assemble_args a{};
  a.msgs           = d->msgs.as<uint8_t>();
  a.iters          = d->iters.as<int32_t>();
  a.crc_checks     = cfg->use_early_stop ? nullptr : d->checks.as<uint32_t>();
  a.soft           = nullptr;
  a.tbs            = d_tbs;
  a.results        = d_results;
  a.cb_iterations  = cb_offsets != nullptr ? d_cb_iterations : nullptr;
  a.crc24a_table   = crc_device_table(d->crc[1]);
  a.acc            = d->tb_acc.as<uint32_t>();
  a.msg_stride     = M;
  a.max_iterations = cfg->nof_ldpc_iterations;
  a.new_data       = 1;
  a.tds            = reinterpret_cast<const tb_desc*>(dd + o_TD);
  a.max_tb_bits    = max_tb_bits;
  he               = launch_assemble(a, U, stream);
  if (he == hipSuccess) {
    he = launch_harq_final(ha, stream);
  }
  if (he == hipSuccess) {
    he = scope.close();
  }
  return he == hipSuccess ? SRS_AMD_OK : hip_fail(he, "assemble_kernel launch");
}

int check_args(srs_amd_pusch_decoder* dec, const srs_amd_sch_plan* plan, const srs_amd_pusch_decoder_config* cfg)
{
  if (dec == nullptr || cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  int rc = check_plan(plan);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (cfg->nof_ldpc_iterations == 0) {
    return fail(SRS_AMD_EINVAL, "The number of LDPC iterations must be positive.");
  }
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_pusch_decoder_create(srs_amd_pusch_decoder** out, int arith, int device)
{
  if (out == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *out = nullptr;
  if (arith != SRS_AMD_ARITH_SIMD && arith != SRS_AMD_ARITH_GENERIC) {
    return fail(SRS_AMD_EINVAL, "invalid LDPC arithmetic %d", arith);
  }
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* d   = new srs_amd_pusch_decoder();
  d->device = device;
  d->arith  = arith;
  rc        = srs_amd_crc_calculator_create(&d->crc[0], 3, 8448, device);
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_crc_calculator_create(&d->crc[1], 0, 1277992, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_crc_calculator_create(&d->crc[2], 1, 8448, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_ldpc_rate_dematcher_create(&d->dm, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_ldpc_decoder_create(&d->dec[0], arith, 0, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_ldpc_decoder_create(&d->dec[1], arith, 1, device);
  }
  if (rc == SRS_AMD_OK) {
    hipError_t he = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
      rc = hip_fail(he, "PUSCH decoder stream");
    }
  }
  if (rc != SRS_AMD_OK) {
    delete d;
    return rc;
  }
  *out = d;
  return SRS_AMD_OK;
}

void srs_amd_pusch_decoder_destroy(srs_amd_pusch_decoder* dec)
{
  delete dec;
}

int srs_amd_pusch_soft_buffer_layout(const srs_amd_sch_plan* plan, uint32_t* row_bytes, uint32_t* nof_llrs,
                                     uint32_t* msg_offset, uint32_t* flag_offset)
{
  const int rc = check_plan(plan);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const soft_row_layout l = layout_of(plan);
  if (row_bytes != nullptr) {
    *row_bytes = l.row_bytes;
  }
  if (nof_llrs != nullptr) {
    *nof_llrs = l.soft_bytes;
  }
  if (msg_offset != nullptr) {
    *msg_offset = l.msg_offset;
  }
  if (flag_offset != nullptr) {
    *flag_offset = l.flag_offset;
  }
  return SRS_AMD_OK;
}

uint32_t srs_amd_pusch_decoder_llr_prefix(const srs_amd_sch_plan* plan, int new_data, int fresh)
{
  if (plan == nullptr || plan->nof_segments == 0 || plan->lifting_size == 0) {
    return 0;
  }
  return llr_prefix(plan, layout_of(plan), new_data != 0, fresh != 0);
}

uint64_t srs_amd_pusch_soft_buffer_size(const srs_amd_sch_plan* plan)
{
  if (plan == nullptr || plan->nof_segments == 0 || plan->lifting_size == 0) {
    return 0;
  }
  return static_cast<uint64_t>(plan->nof_segments) * layout_of(plan).row_bytes;
}

int srs_amd_pusch_decode_batch(srs_amd_pusch_decoder*              dec,
                               const srs_amd_sch_plan*             plan,
                               const srs_amd_pusch_decoder_config* cfg,
                               uint8_t*                            d_tbs,
                               uint32_t                            tb_stride,
                               srs_amd_pusch_decoder_result*       d_results,
                               const int8_t*                       d_llrs,
                               uint32_t                            llr_stride,
                               int8_t*                             d_soft,
                               int32_t*                            d_cb_iterations,
                               uint32_t                            nof_tbs,
                               void*                               stream)
{
  int rc = check_args(dec, plan, cfg);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_tbs == 0) {
    return SRS_AMD_OK;
  }
  if (d_tbs == nullptr || d_results == nullptr || d_llrs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (d_soft == nullptr && !cfg->new_data) {
    return fail(SRS_AMD_EINVAL, "HARQ combining (new_data = 0) needs the caller's soft buffers");
  }
  if (static_cast<uint64_t>(tb_stride) * 8 < plan->tbs || llr_stride < plan->cw_length) {
    return fail(SRS_AMD_EINVAL, "row strides too small (TB %u bits, codeword %u LLRs)", plan->tbs, plan->cw_length);
  }
  if (static_cast<uint64_t>(nof_tbs) * llr_stride >= (1ull << 32)) {
    return fail(SRS_AMD_EINVAL, "batch of %u codewords exceeds 2^32 LLRs", nof_tbs);
  }
  std::lock_guard<std::mutex> lock(dec->mtx);
  return decode_locked(dec, plan, cfg, d_tbs, tb_stride, d_results, d_llrs, llr_stride, d_soft, d_cb_iterations,
                       nof_tbs, static_cast<hipStream_t>(stream));
}

int srs_amd_pusch_decode_slot(srs_amd_pusch_decoder*              dec,
                              const srs_amd_pusch_decoder_config* cfg,
                              const srs_amd_pusch_ue*             ues,
                              uint32_t                            nof_ues,
                              const int8_t*                       d_llrs,
                              uint8_t*                            d_tbs,
                              srs_amd_pusch_decoder_result*       d_results,
                              void*                               stream)
{
  return srs_amd::pusch_decode_slot_ex(dec, cfg, ues, nof_ues, d_llrs, d_tbs, d_results, nullptr, nullptr,
                                      static_cast<hipStream_t>(stream));
}

int srs_amd_pusch_decode(srs_amd_pusch_decoder*              dec,
                         uint8_t*                            transport_block,
                         srs_amd_pusch_decoder_result*       result,
                         const int8_t*                       llrs,
                         int8_t*                             soft_buffer,
                         const srs_amd_sch_plan*             plan,
                         const srs_amd_pusch_decoder_config* cfg)
{
  int rc = check_args(dec, plan, cfg);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (transport_block == nullptr || result == nullptr || llrs == nullptr || soft_buffer == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const uint32_t tb_bytes   = plan->tbs / 8;
  const uint64_t soft_bytes = srs_amd_pusch_soft_buffer_size(plan);
  const size_t   o_soft     = 0;
  const size_t   o_llr      = align_up(soft_bytes, 256);
  const size_t   o_tb       = o_llr + align_up(plan->cw_length, 256);
  const size_t   o_res      = o_tb + align_up(tb_bytes, 256);
  std::lock_guard<std::mutex> lock(dec->mtx);
  hipError_t                  he = hipSetDevice(dec->device);
  if (he == hipSuccess) {
    he = dec->host_io.ensure(o_res + sizeof(srs_amd_pusch_decoder_result));
  }
  auto* base = dec->host_io.as<uint8_t>();
  if (he == hipSuccess) {
    he = hipMemcpyAsync(base + o_soft, soft_buffer, soft_bytes, hipMemcpyHostToDevice, dec->stream);
  }
  if (he == hipSuccess) {
    he = hipMemcpyAsync(base + o_llr, llrs, plan->cw_length, hipMemcpyHostToDevice, dec->stream);
  }
  if (he == hipSuccess) {
    he = hipMemcpyAsync(base + o_tb, transport_block, tb_bytes, hipMemcpyHostToDevice, dec->stream);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PUSCH decoder upload");
  }
  auto* d_res = reinterpret_cast<srs_amd_pusch_decoder_result*>(base + o_res);
  rc = decode_locked(dec, plan, cfg, base + o_tb, tb_bytes, d_res, reinterpret_cast<int8_t*>(base + o_llr),
                     plan->cw_length, reinterpret_cast<int8_t*>(base + o_soft), nullptr, 1, dec->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  he = hipMemcpyAsync(soft_buffer, base + o_soft, soft_bytes, hipMemcpyDeviceToHost, dec->stream);
  if (he == hipSuccess) {
    he = hipMemcpyAsync(transport_block, base + o_tb, tb_bytes, hipMemcpyDeviceToHost, dec->stream);
  }
  if (he == hipSuccess) {
    he = hipMemcpyAsync(result, d_res, sizeof(*result), hipMemcpyDeviceToHost, dec->stream);
  }
  if (he == hipSuccess) {
    he = hipStreamSynchronize(dec->stream);
  }
  return he == hipSuccess ? SRS_AMD_OK : hip_fail(he, "PUSCH decoder download");
}

} // extern "C"

int srs_amd::pusch_decode_slot_ex(srs_amd_pusch_decoder*              dec,
                                  const srs_amd_pusch_decoder_config* cfg,
                                  const srs_amd_pusch_ue*             ues,
                                  uint32_t                            nof_ues,
                                  const int8_t*                       d_llrs,
                                  uint8_t*                            d_tbs,
                                  srs_amd_pusch_decoder_result*       d_results,
                                  const uint32_t*                     cb_offsets,
                                  int32_t*                            d_cb_iterations,
                                  hipStream_t                         stream,
                                  const slot_harq*                    harq,
                                  const slot_ue_patch*                patches,
                                  uint32_t                            nof_patches)
{
  if (dec == nullptr || cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (cfg->nof_ldpc_iterations == 0) {
    return fail(SRS_AMD_EINVAL, "The number of LDPC iterations must be positive.");
  }
  if ((cb_offsets == nullptr) != (d_cb_iterations == nullptr)) {
    return fail(SRS_AMD_EINVAL, "per-codeblock iterations need both the offsets and the output buffer");
  }
  if (harq == nullptr && !cfg->new_data) {
    return fail(SRS_AMD_EINVAL, "slot decoding serves new transmissions; HARQ retransmissions go through "
                                "srs_amd_pusch_decode_batch with the caller's soft buffers");
  }
  if (harq != nullptr && !cfg->use_early_stop) {
    return fail(SRS_AMD_EINVAL, "slot decoding with HARQ state needs the early-stop decoder");
  }
  if (nof_ues == 0) {
    return SRS_AMD_OK;
  }
  if (ues == nullptr || d_llrs == nullptr || d_tbs == nullptr || d_results == nullptr) {
    return fail(SRS_AMD_EINVAL, "null buffer");
  }
  std::lock_guard<std::mutex> lock(dec->mtx);
  return decode_slot_locked(dec, cfg, ues, nof_ues, d_llrs, d_tbs, d_results, cb_offsets, d_cb_iterations, stream,
                            harq, patches, nof_patches);
}

