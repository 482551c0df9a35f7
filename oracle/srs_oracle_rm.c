/*
 * srs_oracle_rm.c -- CPU restatement of srsRAN's LDPC rate matching and rate
 * dematching (TS 38.212 Section 5.4.2).  TEST INFRASTRUCTURE ONLY (see the
 * header of srs_oracle.c); pinned against the reference's own
 * ldpc_rate_matcher_impl / ldpc_rate_dematcher_impl compiled in oracle/_ref.
 *
 * Reference:
 *   lib/phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.cpp:36  init (k0, Ncb, filler range)
 *   ldpc_rate_matcher_impl.cpp:93   select_bits (circular read skipping filler bits)
 *   ldpc_rate_matcher_impl.cpp:143  interleave_bits_Qm (bit interleaver, packed MSB-first)
 *   lib/phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_impl.cpp:36   rate_dematch
 *   ldpc_rate_dematcher_impl.cpp:123  allot_llrs (copy / combine, zeroing, filler = +inf)
 *   ldpc_rate_dematcher_impl.cpp:200  deinterleave_bits_Qm
 *   lib/phy/upper/log_likelihood_ratio.cpp:58  saturated LLR sum
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const unsigned shift_factor_bg1[4] = {0, 17, 33, 56};
static const unsigned shift_factor_bg2[4] = {0, 13, 25, 43};

typedef struct {
  unsigned N;       /* block length (N_short * Z) */
  unsigned Z;
  unsigned Ncb;     /* circular buffer length */
  unsigned nof_sys; /* (K_bg - 2) * Z */
  unsigned F;       /* filler bits */
  unsigned k0;
} rm_params;

static int rm_init(rm_params* p, unsigned bg, unsigned Z, unsigned rv, unsigned Nref, unsigned F)
{
  if ((bg != 1 && bg != 2) || rv > 3) return -1;
  unsigned Nshort = bg == 1 ? 66 : 50, Kbg = bg == 1 ? 22 : 10;
  p->Z       = Z;
  p->N       = Nshort * Z;
  p->Ncb     = (Nref > 0 && Nref < p->N) ? Nref : p->N;
  p->nof_sys = (Kbg - 2) * Z;
  p->F       = F;
  if (F >= p->nof_sys) return -1;
  unsigned sf = bg == 1 ? shift_factor_bg1[rv] : shift_factor_bg2[rv];
  p->k0       = (unsigned)(((unsigned long long)sf * p->Ncb) / p->N) * Z;
  return 0;
}

/* LLR saturated sum a += b (log_likelihood_ratio.cpp:58 operator+=).  The
 * dematcher's combine_softbits computes old + new as `new += old`
 * (log_likelihood_ratio.h:98), so with two infinities the NEW value wins. */
static int8_t llr_add(int8_t a, int8_t b)
{
  if (a == -b) return 0;
  if (a > 120 || a < -120) return a;
  if (b > 120 || b < -120) return b;
  int s = a + b;
  if (s > 120) return 120;
  if (s < -120) return -120;
  return (int8_t)s;
}

/*
 * Rate matching: cw = full encoded codeblock, one bit per byte, N = N_short*Z
 * bits (ldpc_encoder_buffer::write_codeblock layout); filler bits are the last
 * F systematic positions [nof_sys - F, nof_sys).  Output: E bits packed
 * MSB-first after the Qm bit interleaver.
 */
int srs_oracle_ldpc_rate_match(unsigned bg, unsigned Z, unsigned rv, unsigned Qm, unsigned Nref, unsigned F,
                               const uint8_t* cw, unsigned E, uint8_t* out_packed)
{
  rm_params p;
  if (rm_init(&p, bg, Z, rv, Nref, F)) return -1;
  if (Qm == 0 || E % Qm) return -1;
  uint8_t* e = (uint8_t*)malloc(E ? E : 1);
  /* select_bits: circular read from k0 over [0, Ncb), skipping the filler range */
  unsigned fs = p.nof_sys - F, fe = p.nof_sys, idx = p.k0;
  for (unsigned o = 0; o < E; ++o) {
    if (F && idx >= fs && idx < fe) idx = fe;
    if (idx >= p.Ncb) idx = 0;
    if (F && idx >= fs && idx < fe) idx = fe;
    e[o] = cw[idx] & 1;
    idx  = idx + 1;
    if (idx >= p.Ncb) idx = 0;
  }
  /* interleave: f[i*Qm + j] = e[j*K + i], K = E/Qm */
  memset(out_packed, 0, (E + 7) / 8);
  unsigned K = E / Qm;
  for (unsigned i = 0; i < K; ++i)
    for (unsigned j = 0; j < Qm; ++j) {
      unsigned o = i * Qm + j;
      if (e[j * K + i]) out_packed[o >> 3] |= (uint8_t)(0x80u >> (o & 7));
    }
  free(e);
  return 0;
}

/*
 * Rate dematching (in place on the codeblock soft buffer `buf`, N LLRs, like
 * the reference's rx soft buffer): deinterleave the E input LLRs, then
 * allot_llrs exactly as ldpc_rate_dematcher_impl.cpp:123, including its
 * zeroing rules in copy (new data) mode.
 */
int srs_oracle_ldpc_rate_dematch(unsigned bg, unsigned Z, unsigned rv, unsigned Qm, unsigned Nref, unsigned F,
                                 int new_data, const int8_t* in_raw, unsigned E, int8_t* buf)
{
  rm_params p;
  if (rm_init(&p, bg, Z, rv, Nref, F)) return -1;
  if (Qm == 0 || E % Qm) return -1;
  int8_t*  in = (int8_t*)malloc(E ? E : 1);
  unsigned K  = E / Qm;
  if (Qm == 1) {
    memcpy(in, in_raw, E);
  } else {
    for (unsigned i = 0, t = 0; i < K; ++i)
      for (unsigned j = 0; j < Qm; ++j) in[K * j + i] = in_raw[t++];
  }
  const unsigned nof_info = p.nof_sys - F;
  int            copy     = new_data != 0;
  unsigned       tmp      = p.k0;
  unsigned       pos      = 0; /* consumed input */
  const unsigned bl       = p.Ncb;
  while (pos < E) {
    if (tmp < nof_info) {
      unsigned n = nof_info - tmp;
      if (n > E - pos) n = E - pos;
      if (copy) {
        memset(buf, 0, tmp);
        memcpy(buf + tmp, in + pos, n);
      } else {
        for (unsigned k = 0; k < n; ++k) buf[tmp + k] = llr_add(in[pos + k], buf[tmp + k]);
      }
      tmp += n;
      pos += n;
    } else if (copy) {
      memset(buf, 0, nof_info);
    }
    if (copy) memset(buf + nof_info, 127, F);
    if (tmp < p.nof_sys) tmp = p.nof_sys;
    unsigned n = bl - tmp;
    if (n > E - pos) n = E - pos;
    if (copy) {
      memcpy(buf + tmp, in + pos, n);
    } else {
      for (unsigned k = 0; k < n; ++k) buf[tmp + k] = llr_add(in[pos + k], buf[tmp + k]);
    }
    tmp = (tmp + n) % bl;
    pos += n;
    if (pos < E) copy = 0;
  }
  if (copy && tmp != 0) memset(buf + (p.N - (bl - tmp)), 0, bl - tmp);
  free(in);
  return 0;
}
