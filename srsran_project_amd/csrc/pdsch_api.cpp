// pdsch_api.cpp -- C-ABI of the MI355X PDSCH encoder (include/srsran_amd/sch.h),
// pdsch_encoder_impl::encode (lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.cpp:28-80)
// for a batch of transport blocks (srs_amd_pdsch_encode_batch) or a slot of heterogeneous ones
// (srs_amd_pdsch_encode_slot), both through the fused chain of pdsch_encoder.hip:
//   1. TB CRC (CRC16 / CRC24A) partials           pdsch_tb_crc_kernel   } concurrently (two helper streams)
//   2. segmentation, CB CRC24B, LDPC encoding,    pdsch_cb_kernel       } over every codeblock but the TBs' last
//      rate matching + concatenation                                   }
//   3. the TBs' last codeblocks (TB CRC attached) pdsch_cb_kernel
// SRSRAN_AMD_PDSCH_FUSED=0 (read per call) selects the previous five-stage chain instead (TB CRC, segmentation
// + CB CRC, srs_amd_ldpc_encode_batch, srs_amd_ldpc_rate_match_batch), kept for A/B timing and cross-checks.
#include "srsran_amd/crc.h"
#include "srsran_amd/ldpc_encoder.h"
#include "srsran_amd/ldpc_rate_matching.h"
#include "srsran_amd/sch.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "crc_internal.h"
#include "device_buffer.h"
#include "ldpc_codec_args.h"
#include "ldpc_common.h"
#include "ldpc_codec_internal.h"
#include "rate_matching_common.h"
#include "sch_args.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

using namespace srs_amd;

struct srs_amd_pdsch_encoder {
  int                        device = 0;
  hipStream_t                stream = nullptr;
  srs_amd_crc_calculator*    crc16  = nullptr;
  srs_amd_crc_calculator*    crc24a = nullptr;
  srs_amd_crc_calculator*    crc24b = nullptr;
  srs_amd_ldpc_encoder*      enc    = nullptr;
  srs_amd_ldpc_rate_matcher* rm     = nullptr;
  device_buffer              tb_crcs, msgs, coded, rm_arrays, host_io, slot_desc;
  device_buffer              batch_desc, tb_parts; // fused chain: uniform-batch descriptors, TB CRC partials
  std::vector<uint8_t>       batch_key;            // the batch whose descriptors batch_desc holds
  geometry_cache             rm_geo; // last geometry written into rm_arrays
  stream_order               order; // scratch reuse across the callers' streams
  stream_fan                 fan;   // srs_amd_pdsch_encode_slot: concurrent LDPC encoder bucket launches
  std::mutex                 mtx;
  // srs_amd_pdsch_encode_slot: descriptors staged in pinned memory, reused once their upload completed
  pinned_stage hstage; // descriptors staged in pinned memory (a ring: each reused once its upload completed)
  ~srs_amd_pdsch_encoder()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    srs_amd_crc_calculator_destroy(crc16);
    srs_amd_crc_calculator_destroy(crc24a);
    srs_amd_crc_calculator_destroy(crc24b);
    srs_amd_ldpc_encoder_destroy(enc);
    srs_amd_ldpc_rate_matcher_destroy(rm);
  }
};

namespace {

int check_plan(const srs_amd_sch_plan* p)
{
  if (p == nullptr || p->nof_segments == 0 || p->lifting_size == 0) {
    return fail(SRS_AMD_EINVAL, "plan not computed (srs_amd_sch_plan_compute)");
  }
  return SRS_AMD_OK;
}

bool fused_enabled()
{
  const char* mode = std::getenv("SRSRAN_AMD_PDSCH_FUSED");
  return mode == nullptr || mode[0] != '0';
}

// Host descriptors of one fused launch (pdsch_fused_args).
struct fused_rows {
  std::vector<tb_desc>      tds;
  std::vector<uint32_t>     row_E, row_out, row_geo, row_tb;
  std::vector<rm_geometry>  geos;
  std::vector<enc_row_desc> enc;
  uint32_t                  max_tb_bytes = 0;
};

struct fused_layout {
  size_t o_E, o_out, o_geo, o_tb, o_G, o_TD, o_ER, o_LR, total;
  explicit fused_layout(const fused_rows& f)
  {
    const size_t R = f.row_E.size();
    o_E            = 0;
    o_out          = o_E + align_up(sizeof(uint32_t) * R, 16);
    o_geo          = o_out + align_up(sizeof(uint32_t) * R, 16);
    o_tb           = o_geo + align_up(sizeof(uint32_t) * R, 16);
    o_G            = o_tb + align_up(sizeof(uint32_t) * R, 16);
    o_TD           = o_G + align_up(sizeof(rm_geometry) * f.geos.size(), 16);
    o_ER           = o_TD + align_up(sizeof(tb_desc) * f.tds.size(), 16);
    o_LR           = o_ER + align_up(sizeof(enc_row_desc) * R, 16);
    total          = o_LR + sizeof(uint32_t) * f.tds.size();
  }
};

// Appends the codeblock rows of one transport block (plan p, TB bytes at tb_offset, codeword at bit cw_bit) with
// rate-matching geometry index geo.
void fused_add_tb(fused_rows& f, const srs_amd_sch_plan* p, uint64_t tb_offset, uint64_t cw_bit, uint32_t geo,
                  const enc_row_desc& er, std::vector<uint32_t>& segE, std::vector<uint32_t>& segOff)
{
  const uint32_t row0 = static_cast<uint32_t>(f.row_E.size());
  const uint32_t t    = static_cast<uint32_t>(f.tds.size());
  f.tds.push_back(tb_desc{tb_offset, row0, p->nof_segments, p->cb_info_bits, p->tbs, p->nof_tb_crc_bits, p->zero_pad,
                          (p->segment_length + 7) / 8, 0});
  segE.resize(p->nof_segments);
  segOff.resize(p->nof_segments);
  (void)srs_amd_sch_plan_segments(p, segE.data(), segOff.data());
  for (uint32_t r = 0; r < p->nof_segments; ++r) {
    f.row_E.push_back(segE[r]);
    f.row_out.push_back(static_cast<uint32_t>(cw_bit) + segOff[r]);
    f.row_geo.push_back(geo);
    f.row_tb.push_back(t);
    f.enc.push_back(er);
  }
  f.max_tb_bytes = std::max(f.max_tb_bytes, p->tbs / 8);
}

// Encoder row descriptor of plan p: lifted graph and the circular-buffer window [0, k0 + E + F) the rate matcher
// reads (ldpc_rate_matcher_impl.cpp:95-130), capped at Ncb.
enc_row_desc fused_enc_row(const srs_amd_sch_plan* p, const rm_geometry& g)
{
  const uint64_t window = static_cast<uint64_t>(g.k0) + std::max(p->rm_length_long, p->rm_length_short) + g.F;
  enc_row_desc   er{};
  (void)ldpc_encode_mixed_row(&er, p->base_graph, p->lifting_size,
                              window >= g.Ncb ? g.Ncb : static_cast<uint32_t>(window));
  return er;
}

// Writes the descriptors to dd (device) from the pinned staging buffer when `upload`, then runs the two launches.
int fused_launch_locked(srs_amd_pdsch_encoder* e,
                        const fused_rows&      f,
                        uint8_t*               dd,
                        bool                   upload,
                        const uint8_t*         d_tbs,
                        uint8_t*               d_cw,
                        hipStream_t            stream,
                        bool                   overlap)
{
  static const auto row_starts = [] {
    std::vector<int32_t> rs(2 * 47, 0);
    for (int bg = 1; bg <= 2; ++bg) {
      lifted_graph g{};
      build_lifted_graph(g, bg, 2);
      std::copy(g.row_start, g.row_start + g.M + 1, rs.begin() + 47 * (bg - 1));
    }
    return rs;
  }();
  const fused_layout L(f);
  const uint32_t     U  = static_cast<uint32_t>(f.tds.size());
  const uint32_t     R  = static_cast<uint32_t>(f.row_E.size());
  const uint32_t     part_stride = std::max(1u, (f.max_tb_bytes + PE_TB_CHUNK - 1) / PE_TB_CHUNK);
  hipError_t         he          = e->tb_parts.ensure(sizeof(uint32_t) * U * part_stride);
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder TB CRC partials");
  }
  call_scope scope(e->order, &e->fan, stream);
  he = e->order.begin(stream);
  if (he == hipSuccess && upload) {
    // the next pinned staging buffer of the ring, free once its previous upload completed
    he = e->hstage.acquire(L.total);
    if (he == hipSuccess) {
      auto* h = e->hstage.at<uint8_t>(0);
      std::memcpy(h + L.o_E, f.row_E.data(), sizeof(uint32_t) * R);
      std::memcpy(h + L.o_out, f.row_out.data(), sizeof(uint32_t) * R);
      std::memcpy(h + L.o_geo, f.row_geo.data(), sizeof(uint32_t) * R);
      std::memcpy(h + L.o_tb, f.row_tb.data(), sizeof(uint32_t) * R);
      std::memcpy(h + L.o_G, f.geos.data(), sizeof(rm_geometry) * f.geos.size());
      std::memcpy(h + L.o_TD, f.tds.data(), sizeof(tb_desc) * U);
      std::memcpy(h + L.o_ER, f.enc.data(), sizeof(enc_row_desc) * R);
      auto* lr = reinterpret_cast<uint32_t*>(h + L.o_LR);
      for (uint32_t t = 0; t < U; ++t) {
        lr[t] = f.tds[t].row0 + f.tds[t].nof_segments - 1;
      }
      he = e->hstage.upload(dd, L.total, stream);
    }
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder descriptors upload");
  }
  pdsch_fused_args a{};
  a.tbs          = d_tbs;
  a.tds          = reinterpret_cast<const tb_desc*>(dd + L.o_TD);
  a.row_tb       = reinterpret_cast<const uint32_t*>(dd + L.o_tb);
  a.row_E        = reinterpret_cast<const uint32_t*>(dd + L.o_E);
  a.row_out      = reinterpret_cast<const uint32_t*>(dd + L.o_out);
  a.row_geo      = reinterpret_cast<const uint32_t*>(dd + L.o_geo);
  a.geos         = reinterpret_cast<const rm_geometry*>(dd + L.o_G);
  a.enc_rows     = reinterpret_cast<const enc_row_desc*>(dd + L.o_ER);
  a.last_rows    = reinterpret_cast<const uint32_t*>(dd + L.o_LR);
  a.edges        = ldpc_encoder_edges(e->enc);
  a.tb_parts     = e->tb_parts.as<uint32_t>();
  a.part_stride  = part_stride;
  a.max_tb_bytes = f.max_tb_bytes;
  a.crc16_table  = crc_device_table(e->crc16);
  a.crc24a_table = crc_device_table(e->crc24a);
  a.crc24b_table = crc_device_table(e->crc24b);
  a.crc16_poly   = crc_polynom(e->crc16);
  a.crc24a_poly  = crc_polynom(e->crc24a);
  a.crc24b_poly  = crc_polynom(e->crc24b);
  a.cw           = d_cw;
  a.nof_tbs      = U;
  a.nof_cbs      = R;
  std::copy(row_starts.begin(), row_starts.begin() + 47, a.row_start[0]);
  std::copy(row_starts.begin() + 47, row_starts.end(), a.row_start[1]);
  if (overlap) {
    // TB CRC partials || codeblocks without a TB CRC, then the TBs' last codeblocks
    he = e->fan.begin(stream, 2);
    if (he == hipSuccess) {
      he = launch_pdsch_fused(a, e->fan.stream(stream, 0), e->fan.stream(stream, 1), stream, 0);
    }
    if (he == hipSuccess) {
      he = e->fan.end(stream);
    }
    if (he == hipSuccess) {
      he = launch_pdsch_fused(a, stream, stream, stream, 1);
    }
  } else {
    he = launch_pdsch_fused(a, stream, stream, stream, 2);
  }
  if (he == hipSuccess) {
    he = scope.close();
  }
  return he == hipSuccess ? SRS_AMD_OK : hip_fail(he, "PDSCH fused encoder launch");
}

// srs_amd_pdsch_encode_batch through the fused chain: the descriptors of a uniform batch, uploaded again only
// when the batch (plan, count, strides) changes.
int encode_fused_batch_locked(srs_amd_pdsch_encoder* e,
                              const srs_amd_sch_plan* p,
                              uint8_t*                d_cw,
                              uint32_t                cw_stride,
                              const uint8_t*          d_tbs,
                              uint32_t                tb_stride,
                              uint32_t                nof_tbs,
                              hipStream_t             stream)
{
  std::vector<uint8_t> key(sizeof(*p) + 3 * sizeof(uint32_t));
  std::memcpy(key.data(), p, sizeof(*p));
  const uint32_t k3[3] = {cw_stride, tb_stride, nof_tbs};
  std::memcpy(key.data() + sizeof(*p), k3, sizeof(k3));
  rm_geometry g{};
  if (const char* msg = make_rm_geometry(g, p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                         p->nof_filler_bits)) {
    return fail(SRS_AMD_EINVAL, "%s", msg);
  }
  fused_rows f;
  f.geos.push_back(g);
  const enc_row_desc    er = fused_enc_row(p, g);
  std::vector<uint32_t> segE, segOff;
  for (uint32_t t = 0; t < nof_tbs; ++t) {
    fused_add_tb(f, p, static_cast<uint64_t>(t) * tb_stride, static_cast<uint64_t>(t) * cw_stride * 8, 0, er, segE,
                 segOff);
  }
  const bool upload = key != e->batch_key;
  hipError_t he     = hipSetDevice(e->device);
  if (he == hipSuccess && upload) {
    he = e->batch_desc.ensure(fused_layout(f).total);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder descriptors");
  }
  e->batch_key.clear();
  // a uniform batch of segmented TBs: with SRSRAN_AMD_PDSCH_OVERLAP=1 the TB CRC runs on a helper stream beside the
  // codeblocks that do not carry it.  Off by default: inside the pipeline (PDSCH and PUSCH chains concurrent) the
  // extra fork / join measured 0.864-0.877 ms per step against 0.851-0.863 ms without (tools/gpu_r04_fan2.sh).
  const char* ov         = std::getenv("SRSRAN_AMD_PDSCH_OVERLAP"); // read per call (tests run both forms)
  const bool  overlap_on = ov != nullptr && ov[0] == '1';
  int rc = fused_launch_locked(e, f, e->batch_desc.as<uint8_t>(), upload, d_tbs, d_cw, stream,
                               overlap_on && f.row_E.size() >= 4 * f.tds.size());
  if (rc == SRS_AMD_OK) {
    e->batch_key = std::move(key);
  }
  return rc;
}

// srs_amd_pdsch_encode_slot through the fused chain (every UE's plan, one launch pair).
int encode_fused_slot_locked(srs_amd_pdsch_encoder*  e,
                             const srs_amd_pdsch_ue* ues,
                             uint32_t                U,
                             const uint8_t*          d_tbs,
                             uint8_t*                d_cw,
                             hipStream_t             stream)
{
  fused_rows f;
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>, uint32_t> geo_of;
  std::vector<uint32_t> segE, segOff;
  uint32_t              R = 0;
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
    if ((ues[u].cw_offset + (p->cw_length + 7) / 8) * 8 > 0xffffffffull) {
      return fail(SRS_AMD_EINVAL, "UE %u: codeword span exceeds 2^32 bits", u);
    }
    R += p->nof_segments;
    if (U > 65535 || R > 65535) {
      return fail(SRS_AMD_EINVAL, "%u UEs / %u+ codeblocks exceed the 65535 of one slot batch", U, R);
    }
    const auto gkey = std::make_tuple(p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                      p->nof_filler_bits, 0u);
    auto       git  = geo_of.find(gkey);
    if (git == geo_of.end()) {
      git = geo_of.emplace(gkey, static_cast<uint32_t>(f.geos.size())).first;
      f.geos.push_back(g);
    }
    fused_add_tb(f, p, ues[u].tb_offset, ues[u].cw_offset * 8, git->second, fused_enc_row(p, g), segE, segOff);
  }
  hipError_t he = hipSetDevice(e->device);
  if (he == hipSuccess) {
    he = e->slot_desc.ensure(fused_layout(f).total);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH slot encoder descriptors");
  }
  // heterogeneous slots (many single-codeblock TBs): one stream, TB CRC partials then every codeblock
  return fused_launch_locked(e, f, e->slot_desc.as<uint8_t>(), true, d_tbs, d_cw, stream, false);
}

int encode_locked(srs_amd_pdsch_encoder* e,
                  const srs_amd_sch_plan* p,
                  uint8_t*                d_cw,
                  uint32_t                cw_stride,
                  const uint8_t*          d_tbs,
                  uint32_t                tb_stride,
                  uint32_t                nof_tbs,
                  hipStream_t             stream)
{
  if (fused_enabled()) {
    return encode_fused_batch_locked(e, p, d_cw, cw_stride, d_tbs, tb_stride, nof_tbs, stream);
  }
  const uint32_t C          = p->nof_segments;
  const uint32_t rows       = nof_tbs * C;
  const uint32_t K          = p->segment_length;
  const uint32_t msg_stride = static_cast<uint32_t>(align_up((K + 7) / 8, 64));
  const uint32_t N          = srs_amd_ldpc_codeblock_length(p->base_graph, p->lifting_size);
  const uint32_t cb_stride  = static_cast<uint32_t>(align_up((N + 7) / 8, 64));
  hipError_t     he         = hipSetDevice(e->device);
  if (he == hipSuccess) {
    he = e->tb_crcs.ensure(sizeof(uint32_t) * nof_tbs);
  }
  if (he == hipSuccess) {
    he = e->msgs.ensure(static_cast<size_t>(rows) * msg_stride);
  }
  if (he == hipSuccess) {
    he = e->coded.ensure(static_cast<size_t>(rows) * cb_stride);
  }
  if (he == hipSuccess) {
    he = e->rm_arrays.ensure(sizeof(uint32_t) * 2 * rows);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder scratch");
  }
  // Rate-matching lengths and codeword offsets, uploaded when the geometry changes.
  call_scope scope(e->order, nullptr, stream);
  he = e->order.begin(stream);
  if (he == hipSuccess) {
    const uint32_t key[6] = {nof_tbs, C, p->nof_short_segments, p->rm_length_short, p->rm_length_long, cw_stride * 8};
    if (e->rm_geo.stale(e->rm_arrays.ptr, key, 6)) {
      he = launch_rm_arrays(e->rm_arrays.as<uint32_t>(), nof_tbs, C, p->nof_short_segments, p->rm_length_short,
                            p->rm_length_long, cw_stride * 8, stream);
      if (he != hipSuccess) {
        e->rm_geo.invalidate();
      }
    }
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder rate-matching arrays");
  }
  // 1. TB CRC.
  srs_amd_crc_calculator* tbcrc = p->nof_tb_crc_bits == 16 ? e->crc16 : e->crc24a;
  int rc = srs_amd_crc_calculate_batch(tbcrc, e->tb_crcs.as<uint32_t>(), d_tbs, tb_stride, p->tbs, nof_tbs, stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // 2. Segmentation.
  segment_args sa{};
  sa.tbs            = d_tbs;
  sa.tb_crcs        = e->tb_crcs.as<uint32_t>();
  sa.msgs           = e->msgs.as<uint8_t>();
  sa.tb_stride      = tb_stride;
  sa.msg_stride     = msg_stride;
  sa.msg_bytes      = (K + 7) / 8;
  sa.nof_segments   = C;
  sa.cb_info_bits   = p->cb_info_bits;
  sa.last_data_bits = p->cb_info_bits - p->nof_tb_crc_bits - p->zero_pad;
  sa.tb_crc_bits    = p->nof_tb_crc_bits;
  sa.nof_rows       = rows;
  // 3. Codeblock CRC (C > 1), fused into the segmentation pass when the message fits one wave's registers.
  sa.cb_crc_table = C > 1 ? crc_device_table(e->crc24b) : nullptr;
  sa.cb_crc_poly  = C > 1 ? crc_polynom(e->crc24b) : 0u;
  he              = launch_segment(sa, stream);
  if (he != hipSuccess) {
    return hip_fail(he, "segment_kernel launch");
  }
  if (C > 1 && !segment_attaches_crc(sa)) {
    rc = srs_amd_crc_attach_batch(e->crc24b, e->msgs.as<uint8_t>(), msg_stride, p->cb_info_bits, rows, stream);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  // 4. LDPC encoding.
  // Only the circular-buffer window the rate matcher reads, [0, k0 + E + F) capped at Ncb
  // (ldpc_rate_matcher_impl.cpp:95-130), is encoded.
  srs_amd_ldpc_encoder_config ec{p->base_graph, p->lifting_size, p->Nref};
  rm_geometry                 rg{};
  uint32_t                    max_bits = 0xffffffffu;
  if (make_rm_geometry(rg, p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                       p->nof_filler_bits) == nullptr) {
    const uint64_t window = static_cast<uint64_t>(rg.k0) + std::max(p->rm_length_long, p->rm_length_short) + rg.F;
    max_bits              = window >= rg.Ncb ? rg.Ncb : static_cast<uint32_t>(window);
  }
  rc = ldpc_encode_batch_ex(e->enc, &ec, e->msgs.as<uint8_t>(), msg_stride, e->coded.as<uint8_t>(), cb_stride, rows,
                            stream, max_bits);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // 5. Rate matching into the codeword rows.
  srs_amd_codeblock_metadata md{p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                p->nof_filler_bits};
  rc = srs_amd_ldpc_rate_match_batch(e->rm, &md, e->coded.as<uint8_t>(), cb_stride, e->rm_arrays.as<uint32_t>(),
                                     e->rm_arrays.as<uint32_t>() + rows, p->rm_length_long, d_cw, rows, stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  he = scope.close();
  return he == hipSuccess ? SRS_AMD_OK : hip_fail(he, "PDSCH encoder completion event");
}

// srs_amd_pdsch_encode_slot: one message row (stride MS) and one coded row (stride CS) per codeblock of the
// slot, rows grouped by LDPC encoder bucket (BG, Z), each UE's C rows contiguous.
int encode_slot_locked(srs_amd_pdsch_encoder*  e,
                       const srs_amd_pdsch_ue* ues,
                       uint32_t                U,
                       const uint8_t*          d_tbs,
                       uint8_t*                d_cw,
                       hipStream_t             stream)
{
  if (fused_enabled()) {
    return encode_fused_slot_locked(e, ues, U, d_tbs, d_cw, stream);
  }
  // Z < 32: one uniform launch per (BG, Z) (the byte-per-bit kernel); Z >= 32: one mixed-Z launch per BG
  // (the bit-sliced kernel reads each codeblock's Z, graph and encoded window from a row descriptor)
  struct bucket {
    uint32_t              bg, Z; // Z: the lifting size (uniform) or the largest (mixed)
    bool                  mixed;
    uint32_t              max_bits = 0, row0 = 0, rows = 0, max_rows_eff = 0;
    std::vector<uint32_t> ues;
  };
  std::vector<bucket>                         buckets;
  std::map<std::pair<uint32_t, uint32_t>, size_t> bucket_of;
  std::vector<rm_geometry>                    ug(U);
  std::vector<uint32_t>                       ue_window(U);
  uint32_t MS = 0, CS = 0, R = 0, max_tb_bytes = 0, max_msg_bytes = 0;
  for (uint32_t u = 0; u < U; ++u) {
    const srs_amd_sch_plan* p  = &ues[u].plan;
    int                     rc = check_plan(p);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
    if (const char* msg = make_rm_geometry(ug[u], p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                           p->nof_filler_bits)) {
      return fail(SRS_AMD_EINVAL, "UE %u: %s", u, msg);
    }
    if ((ues[u].cw_offset + (p->cw_length + 7) / 8) * 8 > 0xffffffffull) {
      return fail(SRS_AMD_EINVAL, "UE %u: codeword span exceeds 2^32 bits", u);
    }
    const bool mixed = p->lifting_size >= 32;
    const auto key   = std::make_pair(p->base_graph, mixed ? 0u : p->lifting_size);
    auto       it    = bucket_of.find(key);
    if (it == bucket_of.end()) {
      it = bucket_of.emplace(key, buckets.size()).first;
      buckets.push_back(bucket{p->base_graph, p->lifting_size, mixed});
    }
    bucket& b = buckets[it->second];
    b.Z       = std::max(b.Z, p->lifting_size);
    b.ues.push_back(u);
    b.rows += p->nof_segments;
    // only the circular-buffer window the rate matcher reads is encoded (ldpc_rate_matcher_impl.cpp:95-130)
    const uint64_t window = static_cast<uint64_t>(ug[u].k0) + std::max(p->rm_length_long, p->rm_length_short) +
                            ug[u].F;
    ue_window[u]  = window >= ug[u].Ncb ? ug[u].Ncb : static_cast<uint32_t>(window);
    b.max_bits    = std::max(b.max_bits, ue_window[u]);
    const uint32_t N = srs_amd_ldpc_codeblock_length(p->base_graph, p->lifting_size);
    MS            = std::max(MS, static_cast<uint32_t>(align_up((p->segment_length + 7) / 8, 64)));
    CS            = std::max(CS, static_cast<uint32_t>(align_up((N + 7) / 8, 64)));
    R            += p->nof_segments;
    max_tb_bytes  = std::max(max_tb_bytes, p->tbs / 8);
    max_msg_bytes = std::max(max_msg_bytes, (p->segment_length + 7) / 8);
  }
  if (U > 65535 || R > 65535) {
    return fail(SRS_AMD_EINVAL, "%u UEs / %u codeblocks exceed the 65535 of one slot batch", U, R);
  }
  std::vector<uint32_t>                                                          row_E(R), row_out(R), row_geo(R), row_tb(R);
  std::vector<rm_geometry>                                                       geos;
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>, uint32_t> geo_of;
  std::vector<tb_desc>                                                           tds(U);
  std::vector<uint8_t>                                                           enc_rows(R * LDPC_ENCODE_ROW_BYTES);
  // encoder row descriptors per (BG, Z, window): built once (a lifted graph each), copied to every row
  std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::pair<std::vector<uint8_t>, uint32_t>> enc_desc;
  std::vector<uint32_t>                                                          segE, segOff;
  uint32_t                                                                       row = 0;
  for (bucket& b : buckets) {
    b.row0 = row;
    for (uint32_t u : b.ues) {
      const srs_amd_sch_plan* p    = &ues[u].plan;
      const auto              gkey = std::make_tuple(p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                                     p->nof_filler_bits, 0u);
      auto                    git  = geo_of.find(gkey);
      if (git == geo_of.end()) {
        git = geo_of.emplace(gkey, static_cast<uint32_t>(geos.size())).first;
        geos.push_back(ug[u]);
      }
      segE.resize(p->nof_segments);
      segOff.resize(p->nof_segments);
      (void)srs_amd_sch_plan_segments(p, segE.data(), segOff.data());
      tds[u] = tb_desc{ues[u].tb_offset, row,         p->nof_segments, p->cb_info_bits, p->tbs, p->nof_tb_crc_bits,
                       p->zero_pad,       (p->segment_length + 7) / 8, 0};
      for (uint32_t r = 0; r < p->nof_segments; ++r, ++row) {
        row_E[row]   = segE[r];
        row_out[row] = static_cast<uint32_t>(ues[u].cw_offset * 8) + segOff[r];
        row_geo[row] = git->second;
        row_tb[row]  = u;
        if (b.mixed) {
          const auto dkey = std::make_tuple(p->base_graph, p->lifting_size, ue_window[u]);
          auto       dit  = enc_desc.find(dkey);
          if (dit == enc_desc.end()) {
            std::vector<uint8_t> d(LDPC_ENCODE_ROW_BYTES);
            const uint32_t       m = ldpc_encode_mixed_row(d.data(), p->base_graph, p->lifting_size, ue_window[u]);
            dit                    = enc_desc.emplace(dkey, std::make_pair(std::move(d), m)).first;
          }
          std::memcpy(&enc_rows[row * LDPC_ENCODE_ROW_BYTES], dit->second.first.data(), LDPC_ENCODE_ROW_BYTES);
          b.max_rows_eff = std::max(b.max_rows_eff, dit->second.second);
        }
      }
    }
  }
  const size_t o_E   = 0;
  const size_t o_out = o_E + align_up(sizeof(uint32_t) * R, 16);
  const size_t o_geo = o_out + align_up(sizeof(uint32_t) * R, 16);
  const size_t o_tb  = o_geo + align_up(sizeof(uint32_t) * R, 16);
  const size_t o_G   = o_tb + align_up(sizeof(uint32_t) * R, 16);
  const size_t o_TD  = o_G + align_up(sizeof(rm_geometry) * geos.size(), 16);
  const size_t o_ER  = o_TD + align_up(sizeof(tb_desc) * U, 16);
  const size_t total = o_ER + enc_rows.size();

  hipError_t he = hipSetDevice(e->device);
  // the next pinned staging buffer of the ring, free once its previous upload completed
  if (he == hipSuccess) {
    he = e->hstage.acquire(total);
  }
  if (he == hipSuccess) {
    he = e->slot_desc.ensure(total);
  }
  if (he == hipSuccess) {
    he = e->tb_crcs.ensure(sizeof(uint32_t) * U);
  }
  if (he == hipSuccess) {
    he = e->msgs.ensure(static_cast<size_t>(R) * MS);
  }
  if (he == hipSuccess) {
    he = e->coded.ensure(static_cast<size_t>(R) * CS);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH slot encoder scratch");
  }
  auto* h = e->hstage.at<uint8_t>(0);
  std::memcpy(h + o_E, row_E.data(), sizeof(uint32_t) * R);
  std::memcpy(h + o_out, row_out.data(), sizeof(uint32_t) * R);
  std::memcpy(h + o_geo, row_geo.data(), sizeof(uint32_t) * R);
  std::memcpy(h + o_tb, row_tb.data(), sizeof(uint32_t) * R);
  std::memcpy(h + o_G, geos.data(), sizeof(rm_geometry) * geos.size());
  std::memcpy(h + o_TD, tds.data(), sizeof(tb_desc) * U);
  std::memcpy(h + o_ER, enc_rows.data(), enc_rows.size());
  auto*      dd = e->slot_desc.as<uint8_t>();
  call_scope scope(e->order, &e->fan, stream);
  he = e->order.begin(stream);
  if (he == hipSuccess) {
    he = e->hstage.upload(dd, total, stream);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH slot descriptors upload");
  }
  // 1-3. TB CRCs, segmentation, codeblock CRCs.
  tx_slot_args ta{};
  ta.tbs           = d_tbs;
  ta.tds           = reinterpret_cast<const tb_desc*>(dd + o_TD);
  ta.row_tb        = reinterpret_cast<const uint32_t*>(dd + o_tb);
  ta.acc           = e->tb_crcs.as<uint32_t>();
  ta.msgs          = e->msgs.as<uint8_t>();
  ta.crc16_table   = crc_device_table(e->crc16);
  ta.crc24a_table  = crc_device_table(e->crc24a);
  ta.crc24b_table  = crc_device_table(e->crc24b);
  ta.crc16_poly    = crc_polynom(e->crc16);
  ta.crc24a_poly   = crc_polynom(e->crc24a);
  ta.crc24b_poly   = crc_polynom(e->crc24b);
  ta.msg_stride    = MS;
  ta.nof_tbs       = U;
  ta.nof_rows      = R;
  ta.max_tb_bytes  = max_tb_bytes;
  ta.max_msg_bytes = max_msg_bytes;
  he               = launch_tx_slot_segment(ta, stream);
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH slot segmentation launch");
  }
  // 4. LDPC encoding, one launch per (BG, Z) bucket, fanned out over helper streams.
  he = e->fan.begin(stream, static_cast<int>(buckets.size()));
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH slot encoder stream fan-out");
  }
  for (size_t bi = 0; bi < buckets.size(); ++bi) {
    const bucket&     b  = buckets[bi];
    const hipStream_t bs = e->fan.stream(stream, static_cast<int>(bi));
    if (b.mixed) {
      int rc = ldpc_encode_mixed(e->enc, b.bg, b.Z, b.max_rows_eff,
                                 e->msgs.as<uint8_t>() + static_cast<size_t>(b.row0) * MS, MS,
                                 e->coded.as<uint8_t>() + static_cast<size_t>(b.row0) * CS, CS, b.rows, bs,
                                 dd + o_ER + LDPC_ENCODE_ROW_BYTES * b.row0);
      if (rc != SRS_AMD_OK) {
        return rc;
      }
      continue;
    }
    srs_amd_ldpc_encoder_config ec{b.bg, b.Z, 0};
    int rc = ldpc_encode_batch_ex(e->enc, &ec, e->msgs.as<uint8_t>() + static_cast<size_t>(b.row0) * MS, MS,
                                  e->coded.as<uint8_t>() + static_cast<size_t>(b.row0) * CS, CS, b.rows, bs,
                                  b.max_bits);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  he = e->fan.end(stream);
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH slot encoder stream join");
  }
  // 5. Rate matching of every codeblock into the codewords, one launch.
  int rc = rate_match_ragged(e->rm, e->coded.as<uint8_t>(), CS, reinterpret_cast<const uint32_t*>(dd + o_E),
                             reinterpret_cast<const uint32_t*>(dd + o_out), reinterpret_cast<const uint32_t*>(dd + o_geo),
                             dd + o_G, d_cw, R, stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  he = scope.close();
  return he == hipSuccess ? SRS_AMD_OK : hip_fail(he, "PDSCH encoder completion event");
}

} // namespace

extern "C" {

int srs_amd_pdsch_encode_slot(srs_amd_pdsch_encoder*  enc,
                              const srs_amd_pdsch_ue* ues,
                              uint32_t                nof_ues,
                              const uint8_t*          d_tbs,
                              uint8_t*                d_codewords,
                              void*                   stream)
{
  if (enc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null encoder");
  }
  if (nof_ues == 0) {
    return SRS_AMD_OK;
  }
  if (ues == nullptr || d_tbs == nullptr || d_codewords == nullptr) {
    return fail(SRS_AMD_EINVAL, "null buffer");
  }
  std::lock_guard<std::mutex> lock(enc->mtx);
  return encode_slot_locked(enc, ues, nof_ues, d_tbs, d_codewords, static_cast<hipStream_t>(stream));
}

int srs_amd_pdsch_encoder_create(srs_amd_pdsch_encoder** out, int device)
{
  if (out == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *out   = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* e   = new srs_amd_pdsch_encoder();
  e->device = device;
  rc        = srs_amd_crc_calculator_create(&e->crc16, 3, 3824, device);
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_crc_calculator_create(&e->crc24a, 0, 1277992, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_crc_calculator_create(&e->crc24b, 1, 8448, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_ldpc_encoder_create(&e->enc, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_ldpc_rate_matcher_create(&e->rm, device);
  }
  if (rc == SRS_AMD_OK) {
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
      rc = hip_fail(he, "PDSCH encoder stream");
    }
  }
  if (rc != SRS_AMD_OK) {
    delete e;
    return rc;
  }
  *out = e;
  return SRS_AMD_OK;
}

void srs_amd_pdsch_encoder_destroy(srs_amd_pdsch_encoder* enc)
{
  delete enc;
}

int srs_amd_pdsch_encode_batch(srs_amd_pdsch_encoder*  enc,
                               const srs_amd_sch_plan* plan,
                               uint8_t*                d_codewords,
                               uint32_t                cw_stride,
                               const uint8_t*          d_tbs,
                               uint32_t                tb_stride,
                               uint32_t                nof_tbs,
                               void*                   stream)
{
  if (enc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null PDSCH encoder");
  }
  int rc = check_plan(plan);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_tbs == 0) {
    return SRS_AMD_OK;
  }
  if (d_codewords == nullptr || d_tbs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (static_cast<uint64_t>(cw_stride) * 8 < plan->cw_length || static_cast<uint64_t>(tb_stride) * 8 < plan->tbs) {
    return fail(SRS_AMD_EINVAL, "row strides too small (codeword %u bits, TB %u bits)", plan->cw_length, plan->tbs);
  }
  if (static_cast<uint64_t>(nof_tbs) * cw_stride * 8 >= (1ull << 32)) {
    return fail(SRS_AMD_EINVAL, "batch of %u codewords exceeds 2^32 bits", nof_tbs);
  }
  std::lock_guard<std::mutex> lock(enc->mtx);
  return encode_locked(enc, plan, d_codewords, cw_stride, d_tbs, tb_stride, nof_tbs, static_cast<hipStream_t>(stream));
}

int srs_amd_pdsch_encode(srs_amd_pdsch_encoder* enc, uint8_t* codeword, const uint8_t* transport_block,
                         const srs_amd_sch_plan* plan)
{
  if (enc == nullptr || codeword == nullptr || transport_block == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  int rc = check_plan(plan);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const uint32_t tb_bytes = plan->tbs / 8;
  const uint32_t cw_bytes = (plan->cw_length + 7) / 8;
  const size_t   tb_off   = align_up(cw_bytes, 256);
  std::lock_guard<std::mutex> lock(enc->mtx);
  hipError_t                  he = hipSetDevice(enc->device);
  if (he == hipSuccess) {
    he = enc->host_io.ensure(tb_off + tb_bytes);
  }
  uint8_t* d_cw = enc->host_io.as<uint8_t>();
  uint8_t* d_tb = d_cw + tb_off;
  if (he == hipSuccess) {
    he = hipMemcpyAsync(d_tb, transport_block, tb_bytes, hipMemcpyHostToDevice, enc->stream);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder upload");
  }
  rc = encode_locked(enc, plan, d_cw, cw_bytes, d_tb, tb_bytes, 1, enc->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  std::vector<uint8_t> packed(cw_bytes);
  he = hipMemcpyAsync(packed.data(), d_cw, cw_bytes, hipMemcpyDeviceToHost, enc->stream);
  if (he == hipSuccess) {
    he = hipStreamSynchronize(enc->stream);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder download");
  }
  for (uint32_t i = 0; i < plan->cw_length; ++i) {
    codeword[i] = (packed[i >> 3] >> (7 - (i & 7))) & 1u;
  }
  return SRS_AMD_OK;
}

} // extern "C"
