// pucch.hip -- MI355X PUCCH Format 0 and Format 1 detectors (include/srsran_amd/pucch.h).
//
// Format 0, after pucch_detector_format0.cpp:124-246.
// One 64-thread workgroup per PDU: the received REs of every symbol and port into LDS (12 per symbol and port, the
// second hop's PRB for symbol 1), the EPRE, then one thread per candidate cyclic shift: per symbol and port the
// average power, the correlation with the shift's low-PAPR sequence (sum of rx conj(seq)), |corr|^2 / 12 into the
// correlation sum and 12 power - |corr|^2 / 12 into the noise sum, the metric corr / max(noise, 1e-6); thread 0
// keeps the first largest metric in table order, compares it with the threshold and writes the message and the
// SINR / RSRP / EPRE in dB.
//
// Format 1, after pucch_detector_format1.cpp:156-663.  One 64-thread workgroup (one wave) per batch of multiplexed
// PUCCHs.  Per hop: the received REs times the conjugated base sequence (cyclic shift n_cs of the symbol) into LDS,
// split into DM-RS (even allocated symbols) and data rows, and their EPRE; a 12-point DFT of every row (bin k = the
// initial cyclic shift k); then for every time-domain OCC in use, thread (port, shift) combines the rows with the
// conjugated OCC, threads 0..11 form the main / cross contributions and the channel estimate of their shift, and
// thread (port, RE) rebuilds the DM-RS with the shifts within 10 dB of the strongest (12-point IDFT times the OCC),
// accumulated in registers over the OCCs; the noise is the energy of DM-RS minus reconstruction.  Last, thread e
// decides entry e: the BPSK / QPSK symbol that maximises the cross term, the metric against the threshold, the CSI.
//
// Format 2, after pucch_processor_impl.cpp:140-220.  One 256-thread workgroup per PDU; wave w estimates the channel
// of receive port w (port_channel_estimator_average_impl.cpp:122-409 with the PUCCH Format 2 DM-RS on REs 1, 4, 7, 10
// of every PRB, per hop): lane k holds pilot k -- the LSE, the CFO between two DM-RS symbols of a hop and its
// compensation, the FD filter with virtual pilots (chest_device.h), the RSRP, the linear interpolation to the data
// REs rounded to cbf16 as the reference's estimate grid stores them, the noise from the pilots minus their
// reconstruction, and the time alignment from the IDFT correlation (time_alignment_estimator_dft_impl.cpp, stride 3).
// Then thread i equalizes data RE i over the ports (ZF, equalizer_device.h), demaps it (QPSK, demap_device.h: the
// reference's 16-symbol AVX2 blocks and scalar tail) and descrambles its two LLRs; thread 0 writes the CSI.  The UCI
// decoder (uci_decoder.hip) then decodes the LLR rows, grouped by payload and codeword size.
#include <hip/hip_runtime.h>

#include "chest_device.h"
#include "demap_device.h"
#include "equalizer_device.h"
#include "pucch_args.h"

namespace srs_amd {
namespace {

__device__ __forceinline__ float2 from_cbf16(uint32_t u)
{
  return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
}

__device__ __forceinline__ float to_dB(float x) // convert_power_to_dB (math_utils.h)
{
  return 10.0f * log10f(x);
}

__global__ __launch_bounds__(64) void pucch_f0_kernel(const pucch_f0_desc* desc, srs_amd_pucch_f0_result* results)
{
  const pucch_f0_desc& d = desc[blockIdx.x];
  __shared__ float2    re[2][4][12];
  __shared__ float     s_metric[PUCCH_F0_MAX_CAND], s_corr[PUCCH_F0_MAX_CAND];
  __shared__ float2    s_seq[PUCCH_F0_MAX_CAND][2][12];
  const uint32_t       t = threadIdx.x;
  // the candidates' sequences: base times e^(j 2 pi alpha k / 12) (the twelfth roots from double precision)
  for (uint32_t i = t; i < d.nof_cand * d.nsym * 12; i += 64) {
    const uint32_t c = i / (d.nsym * 12), l = (i / 12) % d.nsym, k = i % 12;
    double         sn, cs;
    sincospi(static_cast<double>((d.alpha[c][l] * k) % 12) / 6.0, &sn, &cs);
    const float2 e = make_float2(static_cast<float>(cs), static_cast<float>(sn));
    const float2 b = d.base[k];
    s_seq[c][l][k] = make_float2(b.x * e.x - b.y * e.y, b.x * e.y + b.y * e.x);
  }
  for (uint32_t i = t; i < d.nsym * d.nof_ports * 12; i += 64) {
    const uint32_t l = i / (d.nof_ports * 12), p = (i / 12) % d.nof_ports, k = i % 12;
    re[l][p][k] = from_cbf16(d.grid[static_cast<uint64_t>(d.ports[p]) * d.port_stride +
                                    static_cast<uint64_t>(d.l0 + l) * d.nof_subc + d.subc0[l] + k]);
  }
  __syncthreads();
  // average_power of each (symbol, port) row
  auto power = [&](uint32_t l, uint32_t p) {
    float s = 0.0f;
    for (uint32_t k = 0; k != 12; ++k) {
      s += re[l][p][k].x * re[l][p][k].x + re[l][p][k].y * re[l][p][k].y;
    }
    return s / 12.0f;
  };
  if (t < d.nof_cand) {
    float sum_corr = 0.0f, sum_noise = 0.0f;
    for (uint32_t l = 0; l != d.nsym; ++l) {
      for (uint32_t p = 0; p != d.nof_ports; ++p) {
        float2 c = make_float2(0.0f, 0.0f);
        for (uint32_t k = 0; k != 12; ++k) { // rx conj(seq)
          const float2 x = re[l][p][k], y = s_seq[t][l][k];
          c.x += x.x * y.x + x.y * y.y;
          c.y += x.y * y.x - x.x * y.y;
        }
        const float contrib = (c.x * c.x + c.y * c.y) / 12.0f;
        sum_corr += contrib;
        sum_noise += power(l, p) * 12.0f - contrib;
      }
    }
    float metric = 0.0f;
    if (!isnan(sum_noise) && !isinf(sum_noise)) {
      metric = sum_corr / fmaxf(sum_noise, 1e-6f);
    }
    s_metric[t] = metric;
    s_corr[t]   = sum_corr;
  }
  __syncthreads();
  if (t == 0) {
    float epre = 0.0f;
    for (uint32_t l = 0; l != d.nsym; ++l) {
      for (uint32_t p = 0; p != d.nof_ports; ++p) {
        epre += power(l, p);
      }
    }
    epre /= static_cast<float>(d.nsym * d.nof_ports);
    int   best        = -1;
    float best_metric = 0.0f, best_rsrp = 0.0f;
    for (uint32_t c = 0; c != d.nof_cand; ++c) {
      if (s_metric[c] > best_metric) {
        best_metric = s_metric[c];
        best_rsrp   = s_corr[c];
        best        = static_cast<int>(c);
      }
    }
    srs_amd_pucch_f0_result r{};
    r.nof_sr       = best >= 0 ? d.nof_sr : d.nof_sr_default;
    r.nof_harq_ack = d.nof_harq;
    if (best >= 0) { // otherwise the default message: zero bits
      r.sr          = d.msg[best][0];
      r.harq_ack[0] = d.msg[best][1];
      r.harq_ack[1] = d.msg[best][2];
    }
    r.status           = best_metric > d.threshold ? SRS_AMD_UCI_STATUS_VALID : SRS_AMD_UCI_STATUS_INVALID;
    r.detection_metric = best_metric;
    r.sinr_dB          = to_dB(best_metric);
    r.rsrp_dB          = to_dB(best_rsrp);
    r.epre_dB          = to_dB(epre);
    results[blockIdx.x] = r;
  }
}

// TS 38.211 Table 6.3.2.4.1-2 phases phi(m) of the Format 1 OCCs (pucch_orthogonal_sequence.h), [length - 1][i][m].
__constant__ uint8_t F1_PHI[7][7][7] = {
    {{0}},
    {{0, 0}, {0, 1}},
    {{0, 0, 0}, {0, 1, 2}, {0, 2, 1}},
    {{0, 0, 0, 0}, {0, 2, 0, 2}, {0, 0, 2, 2}, {0, 2, 2, 0}},
    {{0, 0, 0, 0, 0}, {0, 1, 2, 3, 4}, {0, 2, 4, 1, 3}, {0, 3, 1, 4, 2}, {0, 4, 3, 2, 1}},
    {{0, 0, 0, 0, 0, 0}, {0, 1, 2, 3, 4, 5}, {0, 2, 4, 0, 2, 4}, {0, 3, 0, 3, 0, 3}, {0, 4, 2, 0, 4, 2},
     {0, 5, 4, 3, 2, 1}},
    {{0, 0, 0, 0, 0, 0, 0}, {0, 1, 2, 3, 4, 5, 6}, {0, 2, 4, 6, 1, 3, 5}, {0, 3, 6, 2, 5, 1, 4}, {0, 4, 1, 5, 2, 6, 3},
     {0, 5, 3, 1, 6, 4, 2}, {0, 6, 5, 4, 3, 2, 1}}};

constexpr float F1_TWOPI = 6.283185307179586f;

__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

__device__ __forceinline__ float2 cmul_conj(float2 a, float2 b) // a conj(b)
{
  return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}

__device__ __forceinline__ float norm2(float2 a)
{
  return a.x * a.x + a.y * a.y;
}

__device__ __forceinline__ float wave_sum(float v)
{
  for (int o = 32; o != 0; o >>= 1) {
    v += __shfl_xor(v, o);
  }
  return v;
}

// OCC value w_i(m) of length n: e^(j 2 pi phi / n)
__device__ __forceinline__ float2 occ_w(uint32_t n, uint32_t i, uint32_t m)
{
  float sn, cs;
  sincosf(F1_TWOPI * static_cast<float>(F1_PHI[n - 1][i][m]) / static_cast<float>(n), &sn, &cs);
  return make_float2(cs, sn);
}

// detect_symbol (pucch_detector_format1.cpp:108-154): BPSK (nb = 1) or QPSK symbol maximising Re(d x), its bits.
__device__ __forceinline__ float f1_detect_symbol(uint32_t nb, float2 x, uint8_t* bits)
{
  constexpr float s = 0.70710678118654752f;
  if (nb == 1) {
    float m = s * x.x - s * x.y;
    bits[0] = 0;
    if (!(m > 0.0f)) {
      m       = -m;
      bits[0] = 1;
    }
    return m;
  }
  const float m1 = s * x.x - s * x.y, m2 = s * x.x + s * x.y;
  float       m  = m1;
  bits[0] = bits[1] = 0;
  if (fabsf(m2) > fabsf(m1)) {
    m       = m2;
    bits[1] = 1;
  }
  if (m < 0.0f) {
    m       = -m;
    bits[0] = 1 - bits[0];
    bits[1] = 1 - bits[1];
  }
  return m;
}

__global__ __launch_bounds__(64) void pucch_f1_kernel(const pucch_f1_desc*          desc,
                                                      const srs_amd_pucch_f1_entry* entries,
                                                      srs_amd_pucch_result*         results)
{
  const pucch_f1_desc& d = desc[blockIdx.x];
  const uint32_t       t = threadIdx.x;
  const uint32_t       P = d.nof_ports;
  __shared__ float2    tw[12];
  __shared__ float2    Ld[7][4][12], Lm[7][4][12], Xd[7][4][12], Xm[7][4][12];
  __shared__ float2    s_d[4][12], s_m[4][12], s_ch[4][12];
  __shared__ float     s_r[12];
  __shared__ float     h_main[2][7][12], h_rsrp[2][7][12];
  __shared__ float2    h_cross[2][7][12];
  if (t < 12) {
    float sn, cs;
    sincosf(F1_TWOPI * static_cast<float>(t) / 12.0f, &sn, &cs);
    tw[t] = make_float2(cs, sn);
  }
  float    epre = 0.0f, noise = 0.0f;
  uint32_t n_epre = 0, n_noise0 = 0, n_noise1 = 0;
  for (uint32_t h = 0; h != d.nof_hops; ++h) {
    const uint32_t r0 = h == 0 ? 0 : d.nsym / 2;
    const uint32_t nh = d.nof_hops == 1 ? d.nsym : (h == 0 ? d.nsym / 2 : d.nsym - d.nsym / 2);
    const uint32_t nm = (r0 + nh + 1) / 2 - (r0 + 1) / 2; // DM-RS: even allocated symbols
    const uint32_t nd = nh - nm;
    const uint32_t nre = nh * P * 12;
    __syncthreads();
    float e_acc = 0.0f;
    for (uint32_t i = t; i < nre; i += 64) {
      const uint32_t sh = i / (P * 12), p = (i / 12) % P, n = i % 12, r = r0 + sh;
      const float2   x  = from_cbf16(d.grid[static_cast<uint64_t>(d.ports[p]) * d.port_stride +
                                           static_cast<uint64_t>(d.l0 + r) * d.nof_subc + d.subc0[h] + n]);
      e_acc += norm2(x);
      const float2 v = cmul_conj(x, cmul(d.base[n], tw[(d.alpha[r] * n) % 12]));
      if ((r & 1u) == 0) {
        Lm[(r + 1) / 2 - (r0 + 1) / 2][p][n] = v;
      } else {
        Ld[r / 2 - r0 / 2][p][n] = v;
      }
    }
    epre += wave_sum(e_acc);
    n_epre += nre;
    __syncthreads();
    for (uint32_t i = t; i < nre; i += 64) { // direct DFT of every row
      const uint32_t q = i / (P * 12), p = (i / 12) % P, k = i % 12;
      const float2*  in  = q < nm ? Lm[q][p] : Ld[q - nm][p];
      float2         acc = make_float2(0.0f, 0.0f);
      for (uint32_t n = 0; n != 12; ++n) {
        const float2 v = cmul_conj(in[n], tw[(k * n) % 12]);
        acc.x += v.x;
        acc.y += v.y;
      }
      (q < nm ? Xm[q][p] : Xd[q - nm][p])[k] = acc;
    }
    __syncthreads();
    float2 recon[7];
#pragma unroll
    for (uint32_t s = 0; s != 7; ++s) {
      recon[s] = make_float2(0.0f, 0.0f);
    }
    const float nrm_d = 1.0f / sqrtf(static_cast<float>(nd)), nrm_m = 1.0f / sqrtf(static_cast<float>(nm));
    for (uint32_t occi = 0; occi < nd; ++occi) {
      if (((d.occ_mask >> occi) & 1u) == 0) {
        continue;
      }
      if (t < P * 12) { // OCC combination of (port, shift)
        const uint32_t p = t / 12, k = t % 12;
        float2         a = make_float2(0.0f, 0.0f), b = make_float2(0.0f, 0.0f);
        for (uint32_t s = 0; s != nd; ++s) {
          const float2 w = occ_w(nd, occi, s);
          const float2 v = cmul(Xd[s][p][k], make_float2(w.x * nrm_d, -w.y * nrm_d));
          a.x += v.x;
          a.y += v.y;
        }
        for (uint32_t s = 0; s != nm; ++s) {
          const float2 w = occ_w(nm, occi, s);
          const float2 v = cmul(Xm[s][p][k], make_float2(w.x * nrm_m, -w.y * nrm_m));
          b.x += v.x;
          b.y += v.y;
        }
        s_d[p][k] = a;
        s_m[p][k] = b;
      }
      __syncthreads();
      if (t < 12) { // contributions and channel estimate of shift t
        float        main = 0.0f, r = 0.0f;
        float2       cross = make_float2(0.0f, 0.0f);
        const float  cn    = 1.0f / (sqrtf(static_cast<float>(nm)) * 12.0f);
        for (uint32_t p = 0; p != P; ++p) {
          const float2 a = s_d[p][t], b = s_m[p][t];
          main += norm2(a) + norm2(b);
          const float2 c = cmul_conj(b, a);
          cross.x += c.x;
          cross.y += c.y;
          const float2 ch = make_float2(b.x * cn, b.y * cn);
          s_ch[p][t]      = ch;
          r += norm2(ch);
        }
        const float nrm        = 1.0f / static_cast<float>(12 * (nd + nm));
        h_main[h][occi][t]  = main * nrm;
        h_cross[h][occi][t] = make_float2(cross.x * nrm, cross.y * nrm);
        h_rsrp[h][occi][t]  = r / static_cast<float>(P);
        s_r[t]              = r;
      }
      __syncthreads();
      if (t < P * 12) { // rebuild the DM-RS of (port, RE) from the shifts within 10 dB of the strongest
        const uint32_t p = t / 12, n = t % 12;
        float          mx = s_r[0];
        for (uint32_t k = 1; k != 12; ++k) {
          mx = fmaxf(mx, s_r[k]);
        }
        const float th = mx / 10.0f;
        float2      v  = make_float2(0.0f, 0.0f);
        for (uint32_t k = 0; k != 12; ++k) {
          if (s_r[k] > th) {
            const float2 c = cmul(s_ch[p][k], tw[(k * n) % 12]);
            v.x += c.x;
            v.y += c.y;
          }
        }
#pragma unroll
        for (uint32_t s = 0; s != 7; ++s) {
          if (s < nm) {
            const float2 c = cmul(v, occ_w(nm, occi, s));
            recon[s].x += c.x;
            recon[s].y += c.y;
          }
        }
      }
      __syncthreads();
    }
    float n_acc = 0.0f;
    if (t < P * 12) {
      const uint32_t p = t / 12, n = t % 12;
#pragma unroll
      for (uint32_t s = 0; s != 7; ++s) {
        if (s < nm) {
          const float2 x = Lm[s][p][n];
          n_acc += norm2(make_float2(x.x - recon[s].x, x.y - recon[s].y));
        }
      }
    }
    noise += wave_sum(n_acc);
    (h == 0 ? n_noise0 : n_noise1) = nm * P * 12;
  }
  epre /= static_cast<float>(n_epre);
  noise /= static_cast<float>(n_noise0 + n_noise1);
  const bool noise_normal = isfinite(noise) && noise >= 1.17549435e-38f;
  for (uint32_t e = t; e < d.nof_entries; e += 64) {
    const srs_amd_pucch_f1_entry en = entries[d.entry0 + e];
    const uint32_t               o = en.time_domain_occ, k = en.initial_cyclic_shift;
    float                        main  = h_main[0][o][k];
    float2                       cross = h_cross[0][o][k];
    float                        rsrp  = h_rsrp[0][o][k];
    if (d.nof_hops == 2) {
      main += h_main[1][o][k];
      cross.x += h_cross[1][o][k].x;
      cross.y += h_cross[1][o][k].y;
      rsrp = (rsrp * static_cast<float>(n_noise0) + h_rsrp[1][o][k] * static_cast<float>(n_noise1)) /
             static_cast<float>(n_noise0 + n_noise1);
    }
    const float sinr = noise_normal ? rsrp / noise : 0.0f;
    uint8_t     bits[2];
    const float det    = f1_detect_symbol(en.nof_harq_ack == 0 ? 1 : en.nof_harq_ack, cross, bits);
    const float metric = (main + 2.0f * det) / noise;
    const bool  ok     = metric > d.threshold;
    srs_amd_pucch_result r{};
    r.status = ok && (en.nof_harq_ack != 0 || bits[0] == 0) ? SRS_AMD_UCI_STATUS_VALID : SRS_AMD_UCI_STATUS_INVALID;
    r.nof_harq_ack = en.nof_harq_ack;
    r.harq_ack[0]  = en.nof_harq_ack > 0 ? bits[0] : 0;
    r.harq_ack[1]  = en.nof_harq_ack > 1 ? bits[1] : 0;
    r.detection_metric      = metric / d.threshold;
    r.sinr_dB               = to_dB(sinr);
    r.rsrp_dB               = to_dB(rsrp);
    r.epre_dB               = to_dB(epre);
    results[d.entry0 + e]   = r;
  }
}

// ---- Format 2 -------------------------------------------------------------------------------------------------------
constexpr double F2_T_C = 1.0 / (480000.0 * 4096.0);

__device__ __forceinline__ float2 f2_pilot(const uint32_t* bits, uint32_t k) // QPSK at M_SQRT1_2
{
  constexpr float A  = 0.70710678118654752440f;
  const uint32_t  c0 = (bits[(2 * k) >> 5] >> ((2 * k) & 31)) & 1u, c1 = (bits[(2 * k + 1) >> 5] >> ((2 * k + 1) & 31)) & 1u;
  return make_float2(c0 ? -A : A, c1 ? -A : A);
}

__device__ __forceinline__ float2 wave_sum2(float2 v)
{
  return make_float2(wave_sum(v.x), wave_sum(v.y));
}

// The PRB-relative subcarrier of data RE q (0 .. 7) of a PRB: every RE but 1, 4, 7, 10.
__device__ __forceinline__ uint32_t f2_data_re(uint32_t q)
{
  return q + (q + 1) / 2;
}

__global__ __launch_bounds__(256) void pucch_f2_kernel(const pucch_f2_desc* desc)
{
#pragma clang fp contract(off)
  using chdev::cmul;
  const pucch_f2_desc& d    = desc[blockIdx.x];
  const uint32_t       t    = threadIdx.x;
  const uint32_t       w    = t / 64, lane = t % 64;
  const uint32_t       P    = d.nof_ports;
  const uint32_t       np   = 4 * d.nof_prb; // pilots per DM-RS symbol
  const uint32_t       nd8  = 8 * d.nof_prb; // data REs per symbol
  const bool           live = w < P;
  const uint32_t       port = live ? d.ports[w] : d.ports[0];
  __shared__ float2    s_enl[4][CH_MAXV + 64 + CH_MAXV];
  __shared__ float2    s_est[4][2][8 * PUCCH_F2_MAX_PRB];
  __shared__ float     s_corr[4][PUCCH_MAX_TA_N];
  __shared__ float     s_st[4][8]; // epre, rsrp, noise, snr, ta, cfo, cfo valid
  const uint32_t*      g = d.grid + static_cast<uint64_t>(port) * d.port_stride;

  float epre = 0.0f, rsrp = 0.0f, noise = 0.0f, ta = 0.0f, cfo = 0.0f;
  bool  has_cfo = false;
  const uint32_t nhops = d.hop ? 2u : 1u;
  for (uint32_t h = 0; h != nhops; ++h) {
    const uint32_t s0 = d.hop ? h : 0u;      // first allocated symbol of the hop
    const uint32_t nd = d.hop ? 1u : d.nsym; // DM-RS symbols of the hop
    const uint32_t prb = d.prb[s0];
    float2 rx0 = make_float2(0.0f, 0.0f), rx1 = rx0, p0 = rx0, p1 = rx0;
    if (lane < np) {
      const uint32_t re = 12 * (prb + lane / 4) + 1 + 3 * (lane % 4);
      rx0               = chdev::from_cbf16(g[static_cast<uint64_t>(d.l0 + s0) * d.nof_subc + re]);
      p0                = f2_pilot(d.pil[s0], lane);
      if (nd == 2) {
        rx1 = chdev::from_cbf16(g[static_cast<uint64_t>(d.l0 + 1) * d.nof_subc + re]);
        p1  = f2_pilot(d.pil[1], lane);
      }
    }
    epre += wave_sum(norm2(rx0) + norm2(rx1));
    float2 lse = cmul_conj(rx0, p0);
    bool   cfo_hop = false;
    float  cfo_h   = 0.0f;
    if (nd == 2) {
      float2       prod1 = cmul_conj(rx1, p1);
      const float2 z     = wave_sum2(cmul_conj(prod1, lse));
      cfo_h              = atan2f(z.y, z.x) / F1_TWOPI / (d.epoch[1] - d.epoch[0]);
      cfo_hop            = true;
      cfo                = has_cfo ? (cfo + cfo_h) / 2.0f : cfo_h;
      has_cfo            = true;
      lse                = cmul(lse, chdev::polar1(-F1_TWOPI * d.epoch[0] * cfo_h));
      prod1              = cmul(prod1, chdev::polar1(-F1_TWOPI * d.epoch[1] * cfo_h));
      lse.x += prod1.x;
      lse.y += prod1.y;
    }
    const float total = (1.0f / 1.0f) / static_cast<float>(nd);
    lse               = make_float2(lse.x * total, lse.y * total);
    // FD smoothing: virtual pilots at both ends, then the FIR (port_channel_estimator_helpers.cpp:205-246)
    float2* enl = s_enl[w];
    for (uint32_t i = lane; i < CH_MAXV + 64 + CH_MAXV; i += 64) {
      enl[i] = make_float2(0.0f, 0.0f);
    }
    __syncthreads();
    if (lane < np) {
      enl[CH_MAXV + lane] = lse;
    }
    __syncthreads();
    const int nv = d.nof_v;
    chdev::virtual_pilots_wave(enl + CH_MAXV - nv, enl + CH_MAXV, nv, true);
    chdev::virtual_pilots_wave(enl + CH_MAXV + np, enl + CH_MAXV + np - nv, nv, false);
    __syncthreads();
    float2    f    = make_float2(0.0f, 0.0f);
    const int half = d.nof_taps / 2;
    if (lane < np) {
      for (int j = 0; j < d.nof_taps; ++j) {
        const int i = static_cast<int>(lane) + j - half;
        if (i >= -nv && i < static_cast<int>(np) + nv) {
          const float2 in = enl[CH_MAXV + i];
          const float  c  = d.rc[d.nof_taps - 1 - j];
          f.x             = f.x + in.x * c;
          f.y             = f.y + in.y * c;
        }
      }
    }
    __syncthreads();
    rsrp += wave_sum(norm2(f)) * (1.0f * 1.0f * static_cast<float>(nd) / 1.0f);
    enl[lane] = f; // the smoothed pilots, for the interpolation and the IDFT
    __syncthreads();
    // linear interpolation to the data REs (offset 1, stride 3), rounded to cbf16
    for (uint32_t j = lane; j < nd8; j += 64) {
      const uint32_t r = 12 * (j / 8) + f2_data_re(j % 8);
      float2         v;
      if (r <= 1) {
        v = enl[0];
      } else {
        const uint32_t i = (r - 1) / 3, rem = (r - 1) % 3;
        if (i >= np - 1) {
          v = enl[np - 1];
        } else {
          const float  wgt = static_cast<float>(rem) / 3.0f;
          const float2 a = enl[i], b = enl[i + 1];
          v = make_float2(a.x + (b.x - a.x) * wgt, a.y + (b.y - a.y) * wgt);
        }
      }
      v = chdev::from_cbf16(chdev::to_cbf16(v));
      for (uint32_t s = s0; s != s0 + (d.hop ? 1u : d.nsym); ++s) {
        s_est[w][s][j] = v;
      }
    }
    // noise: received pilots minus the smoothed estimate times the pilots (estimate_noise, :704-803)
    float n_acc = 0.0f;
    if (lane < np) {
      for (uint32_t k = 0; k != nd; ++k) {
        float2 pred = cmul(f, k == 0 ? p0 : p1);
        if (cfo_hop) {
          pred = cmul(pred, chdev::polar1(F1_TWOPI * d.epoch[k] * cfo_h));
        }
        const float2 rx = k == 0 ? rx0 : rx1;
        n_acc += norm2(make_float2(rx.x - pred.x, rx.y - pred.y));
      }
    }
    const float energy = wave_sum(n_acc);
    noise += (isfinite(energy) && energy >= 1.17549435e-38f) ? energy : 0.0f;
    // time alignment: |IDFT|^2 of the smoothed pilots (stride 3)
    for (uint32_t tt = lane; tt < d.ta_n; tt += 64) {
      float2 c = make_float2(0.0f, 0.0f);
      for (uint32_t k = 0; k != np; ++k) {
        const float2 e = chdev::polar1(F1_TWOPI * static_cast<float>((k * tt) % d.ta_n) / static_cast<float>(d.ta_n));
        const float2 x = cmul(enl[k], e);
        c.x += x.x;
        c.y += x.y;
      }
      s_corr[w][tt] = norm2(c);
    }
    __syncthreads();
    if (lane == 0) {
      const float*   corr = s_corr[w];
      const int      N = static_cast<int>(d.ta_n), M = d.ta_max_taps;
      int            i_d = 0, i_a = 0;
      float          v_d = corr[0], v_a = corr[N - M];
      for (int i = 1; i < M; ++i) {
        if (corr[i] > v_d) {
          v_d = corr[i];
          i_d = i;
        }
        if (corr[N - M + i] > v_a) {
          v_a = corr[N - M + i];
          i_a = i;
        }
      }
      const int idx  = v_d >= v_a ? i_d : -(M - i_a);
      double    frac = 0.0;
      if (d.ta_frac) {
        float pk[5];
        const int taps = M > 2 ? 5 : 3;
        for (int i = 0; i < taps; ++i) {
          pk[i] = corr[static_cast<uint32_t>(idx + i + N - taps / 2) % static_cast<uint32_t>(N)];
        }
        float r;
        if (taps == 5) {
          const float num = -0.4f * pk[0] + -0.2f * pk[1] + 0.0f * pk[2] + 0.2f * pk[3] + 0.4f * pk[4];
          const float den = 0.571429f * pk[0] + -0.285714f * pk[1] + -0.571429f * pk[2] + -0.285714f * pk[3] +
                            0.571429f * pk[4];
          r = -1.0f * num / den;
        } else {
          const float num = -0.5f * pk[0] + 0.0f * pk[1] + 0.5f * pk[2];
          const float den = 0.5f * pk[0] + -1.0f * pk[1] + 0.5f * pk[2];
          r = -0.5f * num / den;
        }
        frac = (isnan(r) || isinf(r) || fabsf(r) > 1.0f) ? 0.0 : static_cast<double>(r);
      }
      ta += static_cast<float>((static_cast<double>(idx) + frac) / d.ta_fs);
    }
    __syncthreads();
  }
  if (d.hop) {
    ta /= 2.0f;
  }
  const float npil_all = static_cast<float>(np * d.nsym);
  rsrp /= npil_all * 1.0f;
  epre /= npil_all;
  noise /= static_cast<float>(np * d.nsym * 1 - 1);
  noise = fmaxf(rsrp / 1e10f, noise);
  const float snr = (isfinite(noise) && noise >= 1.17549435e-38f) ? rsrp * 1.0f / 1.0f / 1.0f / noise : 0.0f;
  // CFO rotation of the cbf16 estimates (port_channel_estimator_average_impl.cpp:184-194)
  if (has_cfo) {
    for (uint32_t j = lane; j < nd8; j += 64) {
      for (uint32_t s = 0; s != d.nsym; ++s) {
        s_est[w][s][j] = chdev::from_cbf16(chdev::to_cbf16(cmul(s_est[w][s][j], chdev::polar1(F1_TWOPI * d.epoch[s] * cfo))));
      }
    }
  }
  if (lane == 0) {
    s_st[w][0] = epre;
    s_st[w][1] = rsrp;
    s_st[w][2] = noise;
    s_st[w][3] = snr;
    s_st[w][4] = ta;
    s_st[w][5] = cfo;
    s_st[w][6] = has_cfo ? 1.0f : 0.0f;
  }
  __syncthreads();
  // ZF equalization over the ports, QPSK demapping, descrambling
  if (t < d.n_re) {
    const uint32_t s = t / nd8, j = t % nd8;
    const uint32_t re = 12 * (d.prb[s] + j / 8) + f2_data_re(j % 8);
    eq::cplx       y[4], hh[4];
    float          nvp[4];
    uint32_t       valid = 0;
#pragma unroll
    for (uint32_t p = 0; p < 4; ++p) {
      y[p] = hh[p] = {0.0f, 0.0f};
      nvp[p]       = 0.0f;
      if (p < P) {
        y[p]             = eq::from_cbf16(d.grid[static_cast<uint64_t>(d.ports[p]) * d.port_stride +
                                          static_cast<uint64_t>(d.l0 + s) * d.nof_subc + re]);
        const float2 e   = s_est[p][s][j];
        hh[p]            = {e.x, e.y};
        nvp[p]           = s_st[p][2];
        const bool ok_nv = nvp[p] > 0.0f && nvp[p] < __builtin_inff();
        valid |= ok_nv ? (1u << p) : 0u;
      }
    }
    eq::cplx x;
    float    nvx;
    eq::equalize_1xn<4>(y, hh, nvp, valid, 1.0f, x, nvx);
    const bool  simd = t < (d.n_re / 16) * 16;
    const float GAIN = 2.0f * 1.41421356237309504880f;
    const float xs[2] = {x.x, x.y};
#pragma unroll
    for (uint32_t c = 0; c < 2; ++c) {
      int v = simd ? demap::q_simd((GAIN * xs[c]) * demap::safe_rcp(nvx), 24.0f)
                   : (nvx > 0.0f ? demap::q_scalar(GAIN * xs[c] / nvx, 24.0f) : 0);
      const uint32_t b = 2 * t + c;
      if ((d.scr[b >> 5] >> (b & 31)) & 1u) {
        v = -v;
      }
      d.llr[b] = static_cast<int8_t>(v);
    }
  }
  if (t == 0) { // channel_estimate::get_channel_state_information (channel_estimation.h:244-281)
    float    epre_lin = 0.0f, best_snr = 0.0f, rsrp_tot = 0.0f, nv_tot = 0.0f, rsrp_all = 0.0f;
    uint32_t best = 0, nvalid = 0;
    for (uint32_t p = 0; p != P; ++p) {
      epre_lin += s_st[p][0];
      if (s_st[p][3] > best_snr) {
        best_snr = s_st[p][3];
        best     = p;
      }
      const float r = s_st[p][1];
      if (isfinite(r) && fabsf(r) >= 1.17549435e-38f) {
        rsrp_tot += r;
        ++nvalid;
      }
      nv_tot += s_st[p][2];
      rsrp_all += s_st[p][1];
    }
    epre_lin /= static_cast<float>(P);
    const float rsrp_lin = nvalid != 0 ? rsrp_tot / static_cast<float>(nvalid) : 0.0f;
    const float sinr     = (isfinite(nv_tot) && nv_tot >= 1.17549435e-38f) ? rsrp_all / nv_tot : 0.0f;
    // phy_time_unit::from_seconds: tenths of T_C truncated, rounded half up
    const double  tc   = static_cast<double>(s_st[best][4]) / F2_T_C;
    const int64_t tc10 = static_cast<int64_t>(tc * 10.0);
    const int64_t unit = tc10 / 10 + (tc10 % 10) / 5;
    srs_amd_pucch_uci_result* r = d.result;
    r->nof_harq_ack     = d.counts[0];
    r->nof_sr           = d.counts[1];
    r->nof_csi_part1    = d.counts[2];
    r->nof_csi_part2    = d.counts[3];
    r->sinr_dB          = to_dB(sinr);
    r->rsrp_dB          = to_dB(rsrp_lin);
    r->epre_dB          = to_dB(epre_lin);
    r->time_alignment_s = static_cast<float>(static_cast<double>(unit) * F2_T_C);
    r->cfo_Hz           = s_st[best][6] != 0.0f ? s_st[best][5] * d.scs_hz : __builtin_nanf("");
  }
}

// ---- Formats 3 / 4 ----------------------------------------------------------------------------------------------
// After pucch_processor_impl.cpp:222-397: dmrs_pucch_estimator_formats3_4.cpp (all 12 REs of a PRB carry DM-RS on the
// DM-RS symbols of get_pucch_formats3_4_dmrs_symbol_mask; the port estimator with the FD filter, TD averaging, the
// CFO measured between the first two DM-RS symbols of a hop and not compensated), pucch_formats3_4_helpers.h
// pucch_3_4_extract_and_equalize (ZF per data symbol, transform deprecoding, mean noise), Format 4's
// inverse_blockwise_spreading (pucch_demodulator_format4.cpp:113-130), the soft demapper and the descrambler.
__global__ __launch_bounds__(256) void pucch_f34_kernel(const pucch_f34_desc* desc)
{
#pragma clang fp contract(off)
  using chdev::cmul;
  const pucch_f34_desc& d    = desc[blockIdx.x];
  const uint32_t        t    = threadIdx.x;
  const uint32_t        w    = t / 64, lane = t % 64;
  const uint32_t        P    = d.nof_ports;
  const uint32_t        M    = d.M;
  const bool            live = w < P;
  const uint32_t        port = live ? d.ports[w] : d.ports[0];
  __shared__ float2     s_enl[4][CH_MAXV + PUCCH_F3_MAX_M + CH_MAXV];
  __shared__ float2     s_est[4][2][PUCCH_F3_MAX_M];
  __shared__ float      s_corr[4][PUCCH_MAX_TA_N];
  __shared__ float2     s_tw[PUCCH_MAX_TA_N];
  __shared__ float2     s_twm[PUCCH_F3_MAX_M];
  __shared__ float      s_st[4][8];
  __shared__ float2     s_x[PUCCH_F3_MAX_DATA * PUCCH_F3_MAX_M];
  __shared__ float      s_nv[PUCCH_F3_MAX_DATA * PUCCH_F3_MAX_M];
  __shared__ float2     s_y[PUCCH_F3_MAX_DATA * PUCCH_F3_MAX_M];
  __shared__ float      s_mean[PUCCH_F3_MAX_DATA];
  for (uint32_t i = t; i < d.ta_n; i += 256) {
    s_tw[i] = chdev::polar1(F1_TWOPI * static_cast<float>(i) / static_cast<float>(d.ta_n));
  }
  for (uint32_t i = t; i < M; i += 256) {
    s_twm[i] = chdev::polar1(F1_TWOPI * static_cast<float>(i) / static_cast<float>(M));
  }
  const uint32_t* g = d.grid + static_cast<uint64_t>(port) * d.port_stride;
  float           epre = 0.0f, rsrp = 0.0f, noise = 0.0f, ta = 0.0f, cfo = 0.0f;
  bool            has_cfo = false;
  const uint32_t  nhops   = d.hop_sym < d.nsym ? 2u : 1u;
  uint32_t        dmrs_before = 0, nd_total = 0;
  for (uint32_t h = 0; h != nhops; ++h) {
    const uint32_t r0 = h == 0 ? 0u : d.hop_sym, r1 = (nhops == 2 && h == 0) ? d.hop_sym : d.nsym;
    uint32_t       rs[4], nd = 0;
    for (uint32_t r = r0; r != r1; ++r) {
      if (((d.dmrs_mask >> r) & 1u) && nd < 4) {
        rs[nd++] = r;
      }
    }
    const uint32_t subc = d.subc0[h];
    float2         lse[3];
    float          e_acc = 0.0f;
    float2         z     = make_float2(0.0f, 0.0f);
#pragma unroll
    for (uint32_t m = 0; m < 3; ++m) {
      lse[m]           = make_float2(0.0f, 0.0f);
      const uint32_t k = lane + 64 * m;
      if (k < M) {
        float2 p0 = make_float2(0.0f, 0.0f);
        for (uint32_t q = 0; q != nd; ++q) {
          const float2 rx = chdev::from_cbf16(g[static_cast<uint64_t>(d.l0 + rs[q]) * d.nof_subc + subc + k]);
          e_acc += norm2(rx);
          const float2 prod = cmul_conj(rx, d.pil[(dmrs_before + q) * M + k]);
          if (q == 0) {
            p0 = prod;
          } else if (q == 1) {
            const float2 c = cmul_conj(prod, p0);
            z.x += c.x;
            z.y += c.y;
          }
          lse[m].x += prod.x;
          lse[m].y += prod.y;
        }
      }
    }
    epre += wave_sum(e_acc);
    if (nd >= 2) {
      const float2 zs    = wave_sum2(z);
      const float  cfo_h = atan2f(zs.y, zs.x) / F1_TWOPI / (d.epoch[rs[1]] - d.epoch[rs[0]]);
      cfo                = has_cfo ? (cfo + cfo_h) / 2.0f : cfo_h;
      has_cfo            = true;
    }
    const float total = (1.0f / 1.0f) / static_cast<float>(nd);
    float2*     enl   = s_enl[w];
    for (uint32_t i = lane; i < CH_MAXV + PUCCH_F3_MAX_M + CH_MAXV; i += 64) {
      enl[i] = make_float2(0.0f, 0.0f);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t m = 0; m < 3; ++m) {
      const uint32_t k = lane + 64 * m;
      if (k < M) {
        enl[CH_MAXV + k] = make_float2(lse[m].x * total, lse[m].y * total);
      }
    }
    __syncthreads();
    const int nv = d.nof_v;
    chdev::virtual_pilots_wave(enl + CH_MAXV - nv, enl + CH_MAXV, nv, true);
    chdev::virtual_pilots_wave(enl + CH_MAXV + M, enl + CH_MAXV + M - nv, nv, false);
    __syncthreads();
    float2    f[3];
    float     p_acc = 0.0f;
    const int half  = d.nof_taps / 2;
#pragma unroll
    for (uint32_t m = 0; m < 3; ++m) {
      f[m]        = make_float2(0.0f, 0.0f);
      const int k = static_cast<int>(lane + 64 * m);
      if (k < static_cast<int>(M)) {
        for (int j = 0; j < d.nof_taps; ++j) {
          const int i = k + j - half;
          if (i >= -nv && i < static_cast<int>(M) + nv) {
            const float2 in = enl[CH_MAXV + i];
            const float  c  = d.rc[d.nof_taps - 1 - j];
            f[m].x          = f[m].x + in.x * c;
            f[m].y          = f[m].y + in.y * c;
          }
        }
        p_acc += norm2(f[m]);
      }
    }
    __syncthreads();
    rsrp += wave_sum(p_acc) * (1.0f * 1.0f * static_cast<float>(nd) / 1.0f);
    float n_acc = 0.0f;
#pragma unroll
    for (uint32_t m = 0; m < 3; ++m) {
      const uint32_t k = lane + 64 * m;
      if (k < M) {
        enl[k]         = f[m];
        s_est[w][h][k] = chdev::from_cbf16(chdev::to_cbf16(f[m]));
        for (uint32_t q = 0; q != nd; ++q) {
          const float2 rx   = chdev::from_cbf16(g[static_cast<uint64_t>(d.l0 + rs[q]) * d.nof_subc + subc + k]);
          const float2 pred = cmul(f[m], d.pil[(dmrs_before + q) * M + k]);
          n_acc += norm2(make_float2(rx.x - pred.x, rx.y - pred.y));
        }
      }
    }
    const float energy = wave_sum(n_acc);
    noise += (isfinite(energy) && energy >= 1.17549435e-38f) ? energy : 0.0f;
    __syncthreads();
    // time alignment: |IDFT|^2 of the smoothed pilots (stride 1)
    for (uint32_t tt = lane; tt < d.ta_n; tt += 64) {
      float2 c = make_float2(0.0f, 0.0f);
      for (uint32_t k = 0; k != M; ++k) {
        const float2 x = cmul(enl[k], s_tw[(k * tt) % d.ta_n]);
        c.x += x.x;
        c.y += x.y;
      }
      s_corr[w][tt] = norm2(c);
    }
    __syncthreads();
    if (lane == 0) {
      const float* corr = s_corr[w];
      const int    N = static_cast<int>(d.ta_n), Mx = d.ta_max_taps;
      int          i_d = 0, i_a = 0;
      float        v_d = corr[0], v_a = corr[N - Mx];
      for (int i = 1; i < Mx; ++i) {
        if (corr[i] > v_d) {
          v_d = corr[i];
          i_d = i;
        }
        if (corr[N - Mx + i] > v_a) {
          v_a = corr[N - Mx + i];
          i_a = i;
        }
      }
      const int idx  = v_d >= v_a ? i_d : -(Mx - i_a);
      double    frac = 0.0;
      if (d.ta_frac) {
        float     pk[5];
        const int taps = Mx > 2 ? 5 : 3;
        for (int i = 0; i < taps; ++i) {
          pk[i] = corr[static_cast<uint32_t>(idx + i + N - taps / 2) % static_cast<uint32_t>(N)];
        }
        float r;
        if (taps == 5) {
          const float num = -0.4f * pk[0] + -0.2f * pk[1] + 0.0f * pk[2] + 0.2f * pk[3] + 0.4f * pk[4];
          const float den = 0.571429f * pk[0] + -0.285714f * pk[1] + -0.571429f * pk[2] + -0.285714f * pk[3] +
                            0.571429f * pk[4];
          r = -1.0f * num / den;
        } else {
          const float num = -0.5f * pk[0] + 0.0f * pk[1] + 0.5f * pk[2];
          const float den = 0.5f * pk[0] + -1.0f * pk[1] + 0.5f * pk[2];
          r = -0.5f * num / den;
        }
        frac = (isnan(r) || isinf(r) || fabsf(r) > 1.0f) ? 0.0 : static_cast<double>(r);
      }
      ta += static_cast<float>((static_cast<double>(idx) + frac) / d.ta_fs);
    }
    __syncthreads();
    dmrs_before += nd;
    nd_total += nd;
  }
  if (nhops == 2) {
    ta /= 2.0f;
  }
  const float npil_all = static_cast<float>(M * nd_total);
  rsrp /= npil_all * 1.0f;
  epre /= npil_all;
  noise /= static_cast<float>(M * nd_total * 1 - 1);
  noise = fmaxf(rsrp / 1e10f, noise);
  const float snr = (isfinite(noise) && noise >= 1.17549435e-38f) ? rsrp * 1.0f / 1.0f / 1.0f / noise : 0.0f;
  if (lane == 0) {
    s_st[w][0] = epre;
    s_st[w][1] = rsrp;
    s_st[w][2] = noise;
    s_st[w][3] = snr;
    s_st[w][4] = ta;
    s_st[w][5] = cfo;
    s_st[w][6] = has_cfo ? 1.0f : 0.0f;
  }
  __syncthreads();
  // ZF equalization of every data RE
  const uint32_t nds = d.nsym - __popc(d.dmrs_mask);
  for (uint32_t i = t; i < nds * M; i += 256) {
    const uint32_t q = i / M, n = i % M;
    uint32_t       r = 0;
    for (uint32_t c = 0, s = 0; s != d.nsym; ++s) {
      if (!((d.dmrs_mask >> s) & 1u)) {
        if (c == q) {
          r = s;
        }
        ++c;
      }
    }
    const uint32_t h = r >= d.hop_sym ? 1u : 0u;
    eq::cplx       y[4], hh[4];
    float          nvp[4];
    uint32_t       valid = 0;
#pragma unroll
    for (uint32_t p = 0; p < 4; ++p) {
      y[p] = hh[p] = {0.0f, 0.0f};
      nvp[p]       = 0.0f;
      if (p < P) {
        y[p]           = eq::from_cbf16(d.grid[static_cast<uint64_t>(d.ports[p]) * d.port_stride +
                                          static_cast<uint64_t>(d.l0 + r) * d.nof_subc + d.subc0[h] + n]);
        const float2 e = s_est[p][h][n];
        hh[p]          = {e.x, e.y};
        nvp[p]         = s_st[p][2];
        valid |= (nvp[p] > 0.0f && nvp[p] < __builtin_inff()) ? (1u << p) : 0u;
      }
    }
    eq::cplx x;
    float    nvx;
    eq::equalize_1xn<4>(y, hh, nvp, valid, 1.0f, x, nvx);
    s_x[i]  = make_float2(x.x, x.y);
    s_nv[i] = nvx;
  }
  __syncthreads();
  // transform deprecoding: IDFT of M points / sqrt(M) per data symbol; the mean of the valid noise variances
  const float scaling = 1.0f / sqrtf(static_cast<float>(M));
  for (uint32_t i = t; i < nds * M; i += 256) {
    const uint32_t q = i / M, m = i % M;
    float2         c = make_float2(0.0f, 0.0f);
    for (uint32_t n = 0; n != M; ++n) {
      const float2 x = cmul(s_x[q * M + n], s_twm[(n * m) % M]);
      c.x += x.x;
      c.y += x.y;
    }
    s_y[i] = make_float2(c.x * scaling, c.y * scaling);
  }
  if (t < nds) {
    float    acc = 0.0f;
    uint32_t cnt = 0;
    for (uint32_t n = 0; n != M; ++n) {
      const float v = s_nv[t * M + n];
      if (v > 0.0f && !isnan(v) && !isinf(v)) {
        acc += v;
        ++cnt;
      }
    }
    s_mean[t] = cnt != 0 ? acc / static_cast<float>(cnt) : acc;
  }
  __syncthreads();
  for (uint32_t i = t; i < nds * M; i += 256) {
    const float v = s_nv[i];
    s_nv[i]       = (v > 0.0f && !isnan(v) && !isinf(v)) ? s_mean[i / M] : v;
  }
  __syncthreads();
  // Format 4: inverse block-wise spreading into s_x (symbols) and s_nv (noise)
  if (d.occ_len > 1) {
    const uint32_t mod = 12 / d.occ_len;
    for (uint32_t o = t; o < d.n_sym; o += 256) {
      const uint32_t l = o / mod, k0 = o % mod;
      float2         acc = make_float2(0.0f, 0.0f);
      float          nva = 0.0f;
      for (uint32_t k = k0; k < 12; k += mod) {
        const float2 x = cmul_conj(s_y[l * 12 + k], d.occ_w[k]);
        acc.x += x.x;
        acc.y += x.y;
        nva += s_nv[l * 12 + k];
      }
      const float sc = 1.0f / static_cast<float>(d.occ_len);
      s_x[o]         = make_float2(acc.x * sc, acc.y * sc);
      s_y[PUCCH_F3_MAX_DATA * PUCCH_F3_MAX_M - 1 - o] = make_float2(nva, 0.0f);
    }
    __syncthreads();
    for (uint32_t o = t; o < d.n_sym; o += 256) {
      s_nv[o] = s_y[PUCCH_F3_MAX_DATA * PUCCH_F3_MAX_M - 1 - o].x;
      s_y[o]  = s_x[o];
    }
    __syncthreads();
  }
  // soft demapping and descrambling
  const float GAIN = 2.0f * 1.41421356237309504880f;
  for (uint32_t i = t; i < d.n_sym; i += 256) {
    const float2 x  = s_y[i];
    const float  nv = s_nv[i];
    if (d.qm == 2) {
      const bool  simd  = i < (d.n_sym / 16) * 16;
      const float xs[2] = {x.x, x.y};
#pragma unroll
      for (uint32_t c = 0; c < 2; ++c) {
        int v = simd ? demap::q_simd((GAIN * xs[c]) * demap::safe_rcp(nv), 24.0f)
                     : (nv > 0.0f ? demap::q_scalar(GAIN * xs[c] / nv, 24.0f) : 0);
        const uint32_t b = 2 * i + c;
        if ((d.scr[b >> 5] >> (b & 31)) & 1u) {
          v = -v;
        }
        d.llr[b] = static_cast<int8_t>(v);
      }
    } else {
      float re = x.x, im = x.y;
      if (i & 1u) {
        const float tmp = re;
        re              = im;
        im              = -tmp;
      }
      int v = nv > 0.0f ? demap::q_scalar(2.0f * 1.41421356237309504880f * (re + im) / nv, 24.0f) : 0;
      if ((d.scr[i >> 5] >> (i & 31)) & 1u) {
        v = -v;
      }
      d.llr[i] = static_cast<int8_t>(v);
    }
  }
  if (t == 0) {
    float    epre_lin = 0.0f, best_snr = 0.0f, rsrp_tot = 0.0f, nv_tot = 0.0f, rsrp_all = 0.0f;
    uint32_t best = 0, nvalid = 0;
    for (uint32_t p = 0; p != P; ++p) {
      epre_lin += s_st[p][0];
      if (s_st[p][3] > best_snr) {
        best_snr = s_st[p][3];
        best     = p;
      }
      const float r = s_st[p][1];
      if (isfinite(r) && fabsf(r) >= 1.17549435e-38f) {
        rsrp_tot += r;
        ++nvalid;
      }
      nv_tot += s_st[p][2];
      rsrp_all += s_st[p][1];
    }
    epre_lin /= static_cast<float>(P);
    const float   rsrp_lin = nvalid != 0 ? rsrp_tot / static_cast<float>(nvalid) : 0.0f;
    const float   sinr     = (isfinite(nv_tot) && nv_tot >= 1.17549435e-38f) ? rsrp_all / nv_tot : 0.0f;
    const double  tc       = static_cast<double>(s_st[best][4]) / F2_T_C;
    const int64_t tc10     = static_cast<int64_t>(tc * 10.0);
    const int64_t unit     = tc10 / 10 + (tc10 % 10) / 5;
    srs_amd_pucch_uci_result* r = d.result;
    r->nof_harq_ack     = d.counts[0];
    r->nof_sr           = d.counts[1];
    r->nof_csi_part1    = d.counts[2];
    r->nof_csi_part2    = d.counts[3];
    r->sinr_dB          = to_dB(sinr);
    r->rsrp_dB          = to_dB(rsrp_lin);
    r->epre_dB          = to_dB(epre_lin);
    r->time_alignment_s = static_cast<float>(static_cast<double>(unit) * F2_T_C);
    r->cfo_Hz           = s_st[best][6] != 0.0f ? s_st[best][5] * d.scs_hz : __builtin_nanf("");
  }
}

__global__ __launch_bounds__(256) void pucch_uci_finish_kernel(const int32_t* status, const uint8_t* messages,
                                                               uint32_t msg_stride, const uint32_t* perm,
                                                               const uint32_t* nbits, srs_amd_pucch_uci_result* results,
                                                               uint8_t* payloads, uint64_t payload_stride)
{
  const uint32_t j = blockIdx.x, dst = perm[j];
  if (threadIdx.x == 0) {
    results[dst].status = static_cast<uint32_t>(status[j]);
  }
  for (uint32_t i = threadIdx.x; i < nbits[j]; i += 256) {
    payloads[dst * payload_stride + i] = messages[static_cast<uint64_t>(j) * msg_stride + i];
  }
}

} // namespace

hipError_t launch_pucch_f2(const pucch_f2_desc* d_desc, uint32_t nof, hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pucch_f2_kernel, dim3(nof), dim3(256), 0, stream, d_desc);
  return hipGetLastError();
}

hipError_t launch_pucch_f34(const pucch_f34_desc* d_desc, uint32_t nof, hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pucch_f34_kernel, dim3(nof), dim3(256), 0, stream, d_desc);
  return hipGetLastError();
}

hipError_t launch_pucch_uci_finish(const int32_t* status, const uint8_t* messages, uint32_t msg_stride,
                                   const uint32_t* perm, const uint32_t* nbits, uint32_t nof,
                                   srs_amd_pucch_uci_result* results, uint8_t* payloads, uint64_t payload_stride,
                                   hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pucch_uci_finish_kernel, dim3(nof), dim3(256), 0, stream, status, messages, msg_stride, perm,
                     nbits, results, payloads, payload_stride);
  return hipGetLastError();
}

hipError_t launch_pucch_f1(const pucch_f1_desc* d_desc, uint32_t nof, const srs_amd_pucch_f1_entry* d_entries,
                           srs_amd_pucch_result* d_results, hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pucch_f1_kernel, dim3(nof), dim3(64), 0, stream, d_desc, d_entries, d_results);
  return hipGetLastError();
}

hipError_t launch_pucch_f0(const pucch_f0_desc* d_desc, uint32_t nof, srs_amd_pucch_f0_result* d_results,
                           hipStream_t stream)
{
  if (nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pucch_f0_kernel, dim3(nof), dim3(64), 0, stream, d_desc, d_results);
  return hipGetLastError();
}

} // namespace srs_amd
