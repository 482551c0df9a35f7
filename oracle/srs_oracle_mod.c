/*
 * srs_oracle_mod.c -- CPU restatement of srsRAN's modulation mapper, soft
 * demodulation mapper and pseudo-random (Gold) sequence scrambling.  TEST
 * INFRASTRUCTURE ONLY (see srs_oracle.c); pinned against the reference's own
 * classes compiled in oracle/_ref (tests/test_oracle_vs_ref.py).
 *
 * Reference:
 *   lib/phy/upper/channel_modulation/modulation_mapper_lut_impl.cpp:35-60 (tables), :80-140 (bit order)
 *   lib/phy/upper/channel_modulation/demodulation_mapper_impl.cpp:33-110 (BPSK, pi/2-BPSK, dispatch)
 *   demodulation_mapper_qpsk.cpp / _qam16.cpp / _qam64.cpp / _qam256.cpp: the AVX2 kernels for whole
 *     blocks (QPSK 16, 16QAM 8, 64QAM 16, 256QAM 4 symbols) and the scalar code for the remainder, as an
 *     x86-64-v3 build of the reference executes them (scalar a*b+c contracted to FMA)
 *   avx2_helpers.h:62 clip_ps, :121 quantize_ps, :175 compute_interval_idx, :236 interval_function, :259 safe_div
 *   include/srsran/phy/upper/log_likelihood_ratio.h quantize (round half away from zero)
 *   TS 38.211 5.2.1 pseudo-random sequence (Nc = 1600), pseudo_random_generator_impl.cpp
 * Interval tables: the max-log piecewise-linear LLR of each Gray-mapped PAM
 * axis bit (TS 38.211 5.1), slope 2a(o0 - o1) and intercept (o1^2 - o0^2)/norm
 * for the nearest levels a*o0 (bit 0) and a*o1 (bit 1) of each interval; the
 * least significant axis bit uses intervals of width 4a, the others 2a.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- tables */

/* Axis bit k (0 = sign) of the Gray-mapped PAM level with odd value o in
 * [-(2^m - 1), 2^m - 1] (TS 38.211 5.1): o = (1-2b0) * v, v = 2^(m-1) -
 * (1-2b1) * (2^(m-2) - (1-2b2) * (... (2 - (1-2b_{m-1})))). */
static int pam_bit(int m, int o, int k)
{
  for (int pat = 0; pat < (1 << m); ++pat) {
    int v = 1;
    for (int j = m - 1; j >= 1; --j) {
      v = (1 << (m - j)) - (1 - 2 * ((pat >> j) & 1)) * v;
    }
    v *= 1 - 2 * (pat & 1);
    if (v == o) return (pat >> k) & 1;
  }
  return -1;
}

typedef struct {
  int   n;     /* intervals */
  float width;
  float slope[16];
  float icpt[16];
} interval_tab;

static void make_tab(interval_tab* t, int m, int k, float a, float norm)
{
  int L = 1 << m;
  t->n = (k == m - 1) ? L / 2 : L;
  t->width = (float)((k == m - 1) ? 4 : 2) * a;
  float w2 = (k == m - 1) ? 4.0f : 2.0f; /* width in units of a */
  for (int i = 0; i < t->n; ++i) {
    double x = ((i - t->n / 2) + 0.5) * w2; /* interval midpoint in units of a */
    int    o0 = 0, o1 = 0;
    double d0 = 1e30, d1 = 1e30;
    for (int li = 0; li < L; ++li) {
      int    o = 2 * li - (L - 1);
      double d = (x - o) * (x - o);
      if (pam_bit(m, o, k) == 0) {
        if (d < d0) { d0 = d; o0 = o; }
      } else {
        if (d < d1) { d1 = d; o1 = o; }
      }
    }
    t->slope[i] = (float)(2 * (o0 - o1)) * a;
    t->icpt[i]  = (float)(o1 * o1 - o0 * o0) / norm;
  }
}

/* ---------------------------------------------------------------- helpers */

static float safe_rcp(float nv) { return nv > 0 ? 1.0f / nv : 0.0f; }

static int q_simd(float v, float range)
{
  float s = 120.0f / range;
  float x = v * s;
  if (x > 120.0f) x = 120.0f;
  if (x < -120.0f) x = -120.0f;
  x = nearbyintf(x); /* _MM_FROUND_NINT: half to even */
  if (x != x) return 0;
  return (int)x;
}

static int q_scalar(float v, float range)
{
  float c = v;
  if (fabsf(v) > range) c = copysignf(range, v);
  return (int)roundf(c / range * 120.0f);
}

static int interval_idx_simd(float v, float width, int n)
{
  float rw = 1.0f / width;
  int   idx = (int)floorf(v * rw) + n / 2;
  return idx < 0 ? 0 : (idx > n - 1 ? n - 1 : idx);
}

static int interval_idx_scalar(float v, float width, int n)
{
  int idx = (int)floorf(v / width) + n / 2;
  return idx < 0 ? 0 : (idx > n - 1 ? n - 1 : idx);
}

#define NEAR_ZERO 1e-9f

/* ---------------------------------------------------------------- demodulation */

/* Qm: 1 BPSK, 0 pi/2-BPSK, 2, 4, 6, 8.  symbols: interleaved re/im floats. */
int srs_oracle_demodulate(int Qm, const float* sym, const float* nvar, unsigned nsym, int8_t* llr)
{
  const float SQRT2 = 1.41421356237309504880f;
  if (Qm == 1 || Qm == 0) {
    for (unsigned i = 0; i < nsym; ++i) {
      float re = sym[2 * i], im = sym[2 * i + 1];
      if (Qm == 0 && (i & 1)) { float t = re; re = im; im = -t; }
      if (!(nvar[i] > 0)) { llr[i] = 0; continue; }
      float l = 2.0f * SQRT2 * (re + im) / nvar[i];
      llr[i] = (int8_t)q_scalar(l, 24.0f);
    }
    return 0;
  }
  if (Qm == 2) {
    const float GAIN = 2.0f * SQRT2;
    unsigned    nb = (nsym / 16) * 16;
    for (unsigned i = 0; i < nsym; ++i) {
      for (int c = 0; c < 2; ++c) {
        float x = sym[2 * i + c];
        if (i < nb) {
          llr[2 * i + c] = (int8_t)q_simd((GAIN * x) * safe_rcp(nvar[i]), 24.0f);
        } else {
          llr[2 * i + c] = !(nvar[i] > 0) ? 0 : (int8_t)q_scalar(GAIN * x / nvar[i], 24.0f);
        }
      }
    }
    return 0;
  }
  if (Qm == 4) {
    const float S = 1.0f / sqrtf(10.0f);
    const float G = 4.0f * S, TH = 2.0f * S;
    unsigned    nb = (nsym / 8) * 8;
    for (unsigned i = 0; i < nsym; ++i) {
      float re = sym[2 * i], im = sym[2 * i + 1], nv = nvar[i];
      int8_t* o = llr + 4 * i;
      if (i < nb) {
        float rcp = safe_rcp(nv);
        float xs[2] = {re, im};
        for (int c = 0; c < 2; ++c) {
          float x = xs[c], f = G * x;
          float l01 = fabsf(x) > TH ? (2.0f * f - copysignf(0.8f, x)) : f;
          float l23 = 0.8f - fabsf(f);
          l01 *= rcp;
          l23 *= rcp;
          if (fabsf(x) <= NEAR_ZERO) { l01 = 0; l23 = 0; }
          o[c] = (int8_t)q_simd(l01, 20.0f);
          o[2 + c] = (int8_t)q_simd(l23, 20.0f);
        }
      } else {
        if (re * re + im * im < NEAR_ZERO) { memset(o, 0, 4); continue; }
        float xs[2] = {re, im};
        for (int c = 0; c < 2; ++c) {
          float x = xs[c];
          if (!(nv > 0)) { o[c] = 0; o[2 + c] = 0; continue; }
          float l = G * x;
          if (fabsf(x) > TH) l = fmaf(2.0f, l, -copysignf(0.8f, x));
          o[c] = (int8_t)q_scalar(l / nv, 20.0f);
          float l2 = fmaf(-G, fabsf(x), 0.8f);
          o[2 + c] = (int8_t)q_scalar(l2 / nv, 20.0f);
        }
      }
    }
    return 0;
  }
  if (Qm == 6 || Qm == 8) {
    int          m = Qm / 2;
    float        norm = Qm == 6 ? 42.0f : 170.0f;
    float        a = 1.0f / sqrtf(norm);
    interval_tab tab[4];
    for (int k = 0; k < m; ++k) make_tab(&tab[k], m, k, a, norm);
    unsigned blk = Qm == 6 ? 16 : 4;
    unsigned nb = (nsym / blk) * blk;
    for (unsigned i = 0; i < nsym; ++i) {
      float   re = sym[2 * i], im = sym[2 * i + 1], nv = nvar[i];
      int8_t* o = llr + Qm * i;
      if (i >= nb && re * re + im * im < NEAR_ZERO) { memset(o, 0, Qm); continue; }
      float rcp = safe_rcp(nv);
      float xs[2] = {re, im};
      for (int k = 0; k < m; ++k) {
        for (int c = 0; c < 2; ++c) {
          float               x = xs[c];
          const interval_tab* t = &tab[k];
          float               l;
          if (i < nb) {
            int idx = interval_idx_simd(x, t->width, t->n);
            l = (t->slope[idx] * x + t->icpt[idx]) * rcp;
            if (fabsf(x) <= NEAR_ZERO) l = 0;
            o[2 * k + c] = (int8_t)q_simd(l, 20.0f);
          } else {
            int idx = interval_idx_scalar(x, t->width, t->n);
            l = fmaf(t->slope[idx], x, t->icpt[idx]);
            l *= rcp;
            o[2 * k + c] = (int8_t)q_scalar(l, 20.0f);
          }
        }
      }
    }
    return 0;
  }
  return -1;
}

/* ---------------------------------------------------------------- modulation */

/* bits packed MSB-first; out interleaved re/im floats; returns 0. */
int srs_oracle_modulate(int Qm, const uint8_t* bits, unsigned nsym, float* out)
{
  const float R2 = 0.70710678118654752440f; /* M_SQRT1_2 as float */
  if (Qm == 1 || Qm == 0) {
    for (unsigned i = 0; i < nsym; ++i) {
      int b = (bits[i >> 3] >> (7 - (i & 7))) & 1;
      float re = b ? -R2 : R2, im = b ? -R2 : R2;
      if (Qm == 0 && (i & 1)) { re = b ? R2 : -R2; im = b ? -R2 : R2; }
      out[2 * i] = re;
      out[2 * i + 1] = im;
    }
    return 0;
  }
  if (Qm != 2 && Qm != 4 && Qm != 6 && Qm != 8) return -1;
  unsigned L = 1u << Qm;
  float    tre[256], tim[256], sum = 0;
  for (unsigned i = 0; i < L; ++i) {
    float off = -1, re = 0, im = 0;
    for (int j = 0; j < Qm / 2; ++j) {
      re += off;
      im += off;
      off *= 2;
      re *= (i & (1u << (2 * j + 1))) ? 1.0f : -1.0f;
      im *= (i & (1u << (2 * j + 0))) ? 1.0f : -1.0f;
    }
    tre[i] = re;
    tim[i] = im;
    sum += re * re + im * im; /* integers: exact in any order */
  }
  float avg = sum / (float)L;
  float scaling = sqrtf(1.0f / avg);
  for (unsigned i = 0; i < nsym; ++i) {
    unsigned idx = 0;
    for (int k = 0; k < Qm; ++k) {
      unsigned p = i * Qm + k;
      idx = (idx << 1) | ((bits[p >> 3] >> (7 - (p & 7))) & 1u);
    }
    out[2 * i] = tre[idx] * scaling;
    out[2 * i + 1] = tim[idx] * scaling;
  }
  return 0;
}

/* ---------------------------------------------------------------- Gold sequence */

/* c(n), n in [0, len), one bit per byte (TS 38.211 5.2.1). */
int srs_oracle_prbs(uint32_t c_init, unsigned len, uint8_t* c)
{
  enum { NC = 1600 };
  if (len > (1u << 24)) return -1;
  uint8_t* x1 = (uint8_t*)calloc(NC + len + 31, 1);
  uint8_t* x2 = (uint8_t*)calloc(NC + len + 31, 1);
  if (!x1 || !x2) {
    free(x1);
    free(x2);
    return -1;
  }
  x1[0] = 1;
  for (int i = 0; i < 31; ++i) x2[i] = (c_init >> i) & 1;
  for (unsigned n = 0; n + 31 < NC + len; ++n) {
    x1[n + 31] = x1[n + 3] ^ x1[n];
    x2[n + 31] = x2[n + 3] ^ x2[n + 2] ^ x2[n + 1] ^ x2[n];
  }
  for (unsigned n = 0; n < len; ++n) c[n] = x1[n + NC] ^ x2[n + NC];
  free(x1);
  free(x2);
  return 0;
}
