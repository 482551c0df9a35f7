// equalizer_device.h -- per-RE ZF / MMSE equalizer math shared by the
// stand-alone equalizer (equalizer.hip) and the fused PUSCH demodulator
// (pusch_demod.hip).
//
// Reference: lib/phy/upper/equalization/equalize_zf_1xn.h:131-170 and
// equalize_zf_2xn.h:185-250 (scalar path: the same float operations in the same
// order, IEEE division); port validity / reduction of
// channel_equalizer_generic_impl.cpp:122-170, 290-378.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

// Contraction only within one source expression (fmuladd), never across statements: the results then do
// not depend on how a kernel's control flow splits the code into blocks, so every kernel that inlines these
// functions (the expanded-estimate and the estimator-fused equalizers) produces the same bits.
#pragma clang fp contract(on)

namespace srs_amd {
namespace eq {

struct cplx {
  float x, y;
};

__device__ __forceinline__ cplx from_cbf16(uint32_t u)
{
  return {__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}

__device__ __forceinline__ float norm(cplx a)
{
  return a.x * a.x + a.y * a.y;
}

// a * conj(b)
__device__ __forceinline__ cplx mul_conj(cplx a, cplx b)
{
  return {a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y};
}

__device__ __forceinline__ cplx cmul(cplx a, cplx b)
{
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}

// One layer over P ports: y[p], h[p]; port_nv / valid_ports as channel_equalizer_generic_impl.cpp:131.
template <int P>
__device__ __forceinline__ void
equalize_1xn(const cplx* y, const cplx* h, const float* port_nv, uint32_t valid_ports, float tx_scaling, cplx& out,
             float& nv)
{
  float ch_mod_sq = 0.0f, nvar_acc = 0.0f;
  cplx  re_out    = {0.0f, 0.0f};
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const float hn = norm(h[p]);
    if (__builtin_isnormal(hn) && ((valid_ports >> p) & 1u)) {
      ch_mod_sq += hn;
      nvar_acc += hn * port_nv[p];
      const cplx t = mul_conj(y[p], h[p]);
      re_out.x += t.x;
      re_out.y += t.y;
    }
  }
  out           = {0.0f, 0.0f};
  nv            = __builtin_inff();
  const float d = tx_scaling * ch_mod_sq;
  if (__builtin_isnormal(d) && __builtin_isnormal(nvar_acc)) {
    const float rcp = 1.0f / d;
    out             = {re_out.x * rcp, re_out.y * rcp};
    nv              = nvar_acc * rcp * rcp;
  }
}

// Two layers over P ports: h0[p], h1[p]; noise_var = the largest port variance, noise_ok its validity.
template <int P>
__device__ __forceinline__ void equalize_2xn(const cplx* y,
                                             const cplx* h0,
                                             const cplx* h1,
                                             float       noise_var,
                                             bool        noise_ok,
                                             float       tx_scaling,
                                             float4&     out,
                                             float2&     nv)
{
  float n0 = 0.0f, n1 = 0.0f;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    n0 += norm(h0[p]);
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    n1 += norm(h1[p]);
  }
  cplx xi = {0.0f, 0.0f}, m0 = {0.0f, 0.0f}, m1 = {0.0f, 0.0f};
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const cplx t = mul_conj(h1[p], h0[p]); // conj(h0) * h1
    xi.x += t.x;
    xi.y += t.y;
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const cplx t0 = mul_conj(y[p], h0[p]);
    const cplx t1 = mul_conj(y[p], h1[p]);
    m0.x += t0.x;
    m0.y += t0.y;
    m1.x += t1.x;
    m1.y += t1.y;
  }
  const float xi_mod_sq = norm(xi);
  const float d_pinv    = tx_scaling * ((n0 * n1) - xi_mod_sq);
  const float d_nvars   = tx_scaling * d_pinv;
  out                   = {0.0f, 0.0f, 0.0f, 0.0f};
  nv                    = {__builtin_inff(), __builtin_inff()};
  if (noise_ok && __builtin_isnormal(d_pinv)) {
    const float rcp  = 1.0f / d_pinv;
    const float nrcp = 1.0f / d_nvars;
    const cplx  xm1  = cmul(xi, m1);
    const cplx  xm0  = cmul({xi.x, -xi.y}, m0);
    out.x            = ((n1 * m0.x) - xm1.x) * rcp;
    out.y            = ((n1 * m0.y) - xm1.y) * rcp;
    out.z            = ((n0 * m1.x) - xm0.x) * rcp;
    out.w            = ((n0 * m1.y) - xm0.y) * rcp;
    nv.x             = noise_var * n1 * nrcp;
    nv.y             = noise_var * n0 * nrcp;
  }
}

// ---------------------------------------------------------------------------------------------
// L-layer solves the open reference does not implement (channel_equalizer_generic_impl.cpp:197-247
// asserts for ZF 3x4 / 4x4 and MMSE 2x2 / 2x4 / 3x4 / 4x4): parity unpinned, checked against an
// fp64 solve of the same model (oracle/equalizer.py equalize_mimo).  Model and scaling follow the
// reference's ZF equalizers: y = tx_scaling H x + n, the largest port noise variance sigma^2.
//   ZF:   x = (H^H H)^-1 H^H y / ts,               nv_l = sigma^2 [(H^H H)^-1]_ll / ts^2
//         (equalize_zf_2xn.h for L = 2, generalised);
//   MMSE: A = ts^2 H^H H + sigma^2 I, u = A^-1 ts H^H y, d_l = [A^-1]_ll, mu_l = 1 - sigma^2 d_l,
//         x_l = u_l / mu_l, nv_l = sigma^2 d_l / mu_l  -- the unbiased MMSE estimate, which for one
//         layer is exactly the ZF one (channel_equalizer_generic_impl.cpp:343).
// One RE per thread in registers: Gram matrix and matched filter (P L (L+3)/2 complex MACs), an
// L x L complex Cholesky factorisation, forward / backward substitution and the diagonal of the
// inverse from L^-1 -- a few hundred FLOPs against 4 P (L + 1) + 12 L bytes of HBM traffic per RE,
// so the kernel stays HBM-bound and matrix cores would not shorten it.  A Cholesky pivot that is
// not a normal number above 2^-20 times its diagonal entry (a singular channel in float32 terms),
// an invalid sigma^2 or mu_l <= 2^-20 gives zero symbols with infinite variances for the RE, as the
// reference does for abnormal 2 x N inputs (equalize_mimo below).

// The normal equations of one RE, accumulated port by port (each entry sums its ports in port order), so a
// caller can build them while it produces the channel coefficients of each port.
template <int L>
struct mimo_system {
  cplx a[L][L]; // H^H H, lower triangle (row i >= column k)
  cplx b[L];    // H^H y
};

template <int L>
__device__ __forceinline__ void mimo_init(mimo_system<L>& s)
{
#pragma unroll
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int k = 0; k <= i; ++k) {
      s.a[i][k] = {0.0f, 0.0f};
    }
    s.b[i] = {0.0f, 0.0f};
  }
}

// acc += a conj(b) as two packed-FP32 FMAs (v_pk_fma_f32: both components of the complex accumulator per
// instruction, op_sel / op_sel_hi broadcasting and swapping the halves, neg_hi the one subtracted product):
//   (acc.x, acc.y) += (a.x, a.y) (b.x, b.x);   (acc.x, acc.y) += (a.y, -a.x) (b.y, b.y)
// against mul_conj's two multiplies, two FMAs and two adds.  Only the L-layer solves use it (parity unpinned: fp64
// tolerance); the reference-pinned 1 x N / 2 x N paths keep their scalar arithmetic.
#ifndef EQ_PK_GRAM
#define EQ_PK_GRAM 1
#endif
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void pk_cmac_conj(cplx& acc, cplx a, cplx b)
{
  f2v       c  = {acc.x, acc.y};
  const f2v av = {a.x, a.y}, bv = {b.x, b.y};
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(c) : "v"(av), "v"(bv));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]" : "+v"(c) : "v"(av), "v"(bv));
  acc = {c.x, c.y};
}

// acc -= a b and acc -= a conj(b), two packed FMAs each (the L-layer solve's complex multiply-accumulates).
__device__ __forceinline__ void pk_cmsc(cplx& acc, cplx a, cplx b)
{
  f2v       c  = {acc.x, acc.y};
  const f2v av = {a.x, a.y}, bv = {b.x, b.y};
  // (acc.x, acc.y) -= (a.x, a.x) (b.x, b.y);  (acc.x, acc.y) += (a.y, -a.y) (b.y, b.x)
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "+v"(c) : "v"(av), "v"(bv));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[1,0,0]" : "+v"(c) : "v"(av), "v"(bv));
  acc = {c.x, c.y};
}
__device__ __forceinline__ void pk_cmsc_conj(cplx& acc, cplx a, cplx b)
{
  f2v       c  = {acc.x, acc.y};
  const f2v av = {a.x, a.y}, bv = {b.x, b.y};
  // (acc.x, acc.y) -= (a.x, a.y) (b.x, b.x);  (acc.x, acc.y) += (-a.y, a.x) (b.y, b.y)
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "+v"(c) : "v"(av), "v"(bv));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]" : "+v"(c) : "v"(av), "v"(bv));
  acc = {c.x, c.y};
}
// acc += a b
__device__ __forceinline__ void pk_cmac(cplx& acc, cplx a, cplx b)
{
  f2v       c  = {acc.x, acc.y};
  const f2v av = {a.x, a.y}, bv = {b.x, b.y};
  // (acc.x, acc.y) += (a.x, a.x) (b.x, b.y);  (acc.x, acc.y) += (-a.y, a.y) (b.y, b.x)
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(c) : "v"(av), "v"(bv));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]" : "+v"(c) : "v"(av), "v"(bv));
  acc = {c.x, c.y};
}

// Port p's terms: hp[L] its channel coefficients, yp its received sample.
template <int L>
__device__ __forceinline__ void mimo_add_port(mimo_system<L>& s, const cplx* hp, cplx yp)
{
#pragma unroll
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int k = 0; k <= i; ++k) {
      // (H^H H)_{i,k} = sum_p conj(H_pi) H_pk
#if EQ_PK_GRAM
      pk_cmac_conj(s.a[i][k], hp[k], hp[i]);
#else
      const cplx t = mul_conj(hp[k], hp[i]);
      s.a[i][k].x += t.x;
      s.a[i][k].y += t.y;
#endif
    }
    // conj(h_i) y
#if EQ_PK_GRAM
    pk_cmac_conj(s.b[i], yp, hp[i]);
#else
    const cplx t = mul_conj(yp, hp[i]);
    s.b[i].x += t.x;
    s.b[i].y += t.y;
#endif
  }
}

template <int L, bool MMSE>
__device__ __forceinline__ void mimo_solve(mimo_system<L>& sys,
                                           float           noise_var,
                                           bool            noise_ok,
                                           float           tx_scaling,
                                           cplx*           out, // [L]
                                           float*          nv)  // [L]
{
  // A (lower triangle, row i >= column k) and the right-hand side
  cplx(&a)[L][L] = sys.a;
  cplx(&b)[L]    = sys.b;
  const float ga = MMSE ? tx_scaling * tx_scaling : 1.0f;
  const float gb = MMSE ? tx_scaling : 1.0f;
#pragma unroll
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int k = 0; k <= i; ++k) {
      a[i][k] = {a[i][k].x * ga, a[i][k].y * ga};
    }
    a[i][i].y = 0.0f;
    if (MMSE) {
      a[i][i].x += noise_var;
    }
    b[i] = {b[i].x * gb, b[i].y * gb};
  }
  // Cholesky A = C C^H (C lower, real diagonal), kept in a[][]; r[k] = 1 / C_kk
  float r[L];
  bool  ok = noise_ok && (!MMSE || noise_var > 0.0f);
#pragma unroll
  for (int k = 0; k < L; ++k) {
    float d = a[k][k].x;
#pragma unroll
    for (int j = 0; j < k; ++j) {
      d -= norm(a[k][j]);
    }
    // singular in float terms: a pivot below 2^-20 of its diagonal entry (or not a positive normal number)
    ok = ok && __builtin_isnormal(d) && d > 0x1p-20f * a[k][k].x;
    // 1 / C_kk as one hardware reciprocal square root (v_rsq_f32, ~1 ulp): this solve has no reference to
    // be bit-exact with (parity unpinned, fp64 tolerance), and the correctly rounded sqrt + IEEE division
    // cost ~20 VALU instructions each
    r[k] = __builtin_amdgcn_rsqf(d);
#pragma unroll
    for (int i = k + 1; i < L; ++i) {
      cplx s = a[i][k];
#pragma unroll
      for (int j = 0; j < k; ++j) {
#if EQ_PK_GRAM
        pk_cmsc_conj(s, a[i][j], a[k][j]); // C_ij conj(C_kj)
#else
        const cplx t = mul_conj(a[i][j], a[k][j]); // C_ij conj(C_kj)
        s.x -= t.x;
        s.y -= t.y;
#endif
      }
      a[i][k] = {s.x * r[k], s.y * r[k]};
    }
  }
  // z = C^-1 b, then x = C^-H z
  cplx z[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    cplx s = b[k];
#pragma unroll
    for (int j = 0; j < k; ++j) {
#if EQ_PK_GRAM
      pk_cmsc(s, a[k][j], z[j]);
#else
      const cplx t = cmul(a[k][j], z[j]);
      s.x -= t.x;
      s.y -= t.y;
#endif
    }
    z[k] = {s.x * r[k], s.y * r[k]};
  }
  cplx x[L];
#pragma unroll
  for (int k = L - 1; k >= 0; --k) {
    cplx s = z[k];
#pragma unroll
    for (int j = k + 1; j < L; ++j) {
#if EQ_PK_GRAM
      pk_cmsc_conj(s, x[j], a[j][k]); // conj(C_jk) x_j
#else
      const cplx t = mul_conj(x[j], a[j][k]); // conj(C_jk) x_j
      s.x -= t.x;
      s.y -= t.y;
#endif
    }
    x[k] = {s.x * r[k], s.y * r[k]};
  }
  // diag(A^-1) = column norms of W = C^-1 (lower): W_kk = r_k, W_ik = -r_i sum_{j=k}^{i-1} C_ij W_jk
  float dinv[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    cplx w[L];
    w[k]      = {r[k], 0.0f};
    float acc = r[k] * r[k];
#pragma unroll
    for (int i = k + 1; i < L; ++i) {
      cplx s = {0.0f, 0.0f};
#pragma unroll
      for (int j = k; j < i; ++j) {
#if EQ_PK_GRAM
        pk_cmac(s, a[i][j], w[j]);
#else
        const cplx t = cmul(a[i][j], w[j]);
        s.x += t.x;
        s.y += t.y;
#endif
      }
      w[i] = {-s.x * r[i], -s.y * r[i]};
      acc += norm(w[i]);
    }
    dinv[k] = acc;
  }
#pragma unroll
  for (int l = 0; l < L; ++l) {
    if (MMSE) {
      const float mu = 1.0f - noise_var * dinv[l];
      // mu_l = SINR / (1 + SINR) of the layer: below 2^-20 (no signal) the RE is abnormal
      ok             = ok && __builtin_isnormal(mu) && mu > 0x1p-20f;
      const float rm = __builtin_amdgcn_rcpf(mu); // v_rcp_f32 (~1 ulp), see r[k] above
      out[l]         = {x[l].x * rm, x[l].y * rm};
      nv[l]          = noise_var * dinv[l] * rm;
    } else {
      const float rt = 1.0f / tx_scaling;
      out[l]         = {x[l].x * rt, x[l].y * rt};
      nv[l]          = noise_var * dinv[l] * rt * rt;
    }
  }
  if (!ok) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
      out[l] = {0.0f, 0.0f};
      nv[l]  = __builtin_inff();
    }
  }
}

template <int P, int L, bool MMSE>
__device__ __forceinline__ void equalize_mimo(const cplx* y,  // [P]
                                              const cplx* h,  // [P][L]
                                              float       noise_var,
                                              bool        noise_ok,
                                              float       tx_scaling,
                                              cplx*       out, // [L]
                                              float*      nv)  // [L]
{
  mimo_system<L> sys;
  mimo_init(sys);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    mimo_add_port(sys, h + p * L, y[p]);
  }
  mimo_solve<L, MMSE>(sys, noise_var, noise_ok, tx_scaling, out, nv);
}

} // namespace eq
} // namespace srs_amd
