/*
 * srs_oracle_polar.c -- CPU restatement of srsRAN's polar channel coding
 * (TS 38.212 Sections 5.3.1, 5.4.1).  TEST INFRASTRUCTURE ONLY (see the header
 * of srs_oracle.c); pinned against the reference's own polar classes compiled
 * in oracle/_ref (tests/test_oracle_vs_ref.py).
 *
 * Reference:
 *   lib/phy/upper/channel_coding/polar/polar_code_impl.cpp:367-410  set_code_params (n, N, nPC, nWmPC)
 *   polar_code_impl.cpp:420-490       set (K_set / F_set / PC_set construction, setdiff_stable :340)
 *   polar_allocator_impl.cpp:29-69    allocate (parity-check bits from a 5-register cyclic shift)
 *   polar_encoder_impl.cpp:29-82      encode (recursive butterfly)
 *   polar_rate_matcher_impl.cpp:29-106  sub-block interleaving, bit selection, channel interleaver
 *   polar_rate_dematcher_impl.cpp:29-118  inverse, repetition by promotion_sum, puncture 0 / shorten +inf
 *   polar_decoder_impl.cpp:28-350     SSC decoder (rate-0 / rate-1 / rate-R nodes, min-sum f, saturated g)
 *   polar_deallocator_impl.cpp:27-42  deallocate
 *   polar_interleaver_impl.cpp:40-56  DCI input bit interleaver
 *   lib/phy/upper/log_likelihood_ratio.cpp:38-92, log_likelihood_ratio.h:207  LLR sums and soft_xor
 */
#include <stdint.h>
#include <string.h>

#define SRS_POLAR_TABLE_QUAL static const
#include "../srsran_project_amd/csrc/polar_tables.inc"

#define NMAX 1024
#define EMAX 8192

static const uint16_t SUBBLOCK_P[32] = {0,  1,  2,  4,  3,  5,  6,  7,  8,  16, 9,  17, 10, 18, 11, 19,
                                        12, 20, 13, 21, 14, 22, 15, 23, 24, 25, 26, 28, 27, 29, 30, 31};

typedef struct {
  unsigned n, N, K, E, nPC, nWmPC, ibil;
  uint8_t  kmask[NMAX];
  uint16_t pc[5]; /* sorted, sentinel NMAX */
  uint16_t mother[NMAX];
  uint16_t blk[NMAX];
} pcode;

static int code_params(pcode* c, unsigned K, unsigned E, unsigned nMax)
{
  if (E > EMAX) return -1;
  if (nMax == 9) {
    if (K < 36 || K > 164) return -1;
  } else if (nMax == 10) {
    if (K < 18 || (K > 25 && K < 31) || K > 1023) return -1;
  } else {
    return -1;
  }
  c->K = K;
  c->E = E;
  c->nPC = 0;
  c->nWmPC = 0;
  if (K <= 25) {
    c->nPC = 3;
    if (E > K + 189) c->nWmPC = 1;
  }
  if (!(K + c->nPC < E)) return -1;
  unsigned e = 1;
  for (; e <= 13; ++e)
    if ((1u << e) >= E) break;
  unsigned n1 = ((8 * E <= 9 * (1u << (e - 1))) && (16 * K < 9 * E)) ? e - 1 : e;
  unsigned k = 0;
  for (; k <= 10; ++k)
    if ((1u << k) >= K) break;
  unsigned n2 = k + 3;
  unsigned n = n1 < n2 ? n1 : n2;
  if (nMax < n) n = nMax;
  if (n < 5) n = 5;
  c->n = n;
  c->N = 1u << n;
  if (!(K < c->N)) return -1;
  return 0;
}

static int build_code(pcode* c, unsigned K, unsigned E, unsigned nMax, int ibil)
{
  if (code_params(c, K, E, nMax)) return -1;
  unsigned N = c->N;
  c->ibil = ibil ? 1 : 0;
  for (unsigned i = 0, o = 0; i < NMAX; ++i)
    if (SRS_POLAR_Q1024[i] < N) c->mother[o++] = SRS_POLAR_Q1024[i];
  for (unsigned i = 0; i < N; ++i) c->blk[i] = SUBBLOCK_P[(32 * i) / N] * (N / 32) + i % (N / 32);

  const unsigned nk = K + c->nPC;
  uint16_t       kset[NMAX];
  if (N > E) {
    unsigned T = 0, fsize = N - E, Nth = 3 * N / 4;
    uint16_t F[NMAX];
    if (16 * K <= 7 * E) { /* puncturing */
      T = (E >= Nth) ? Nth - (E >> 1) - 1 : 9 * N / 16 - (E >> 2);
      for (unsigned i = 0; i < fsize; ++i) F[i] = c->blk[i];
    } else { /* shortening */
      for (unsigned i = 0; i < fsize; ++i) F[i] = c->blk[E + i];
    }
    uint16_t tmp[NMAX];
    unsigned o = 0;
    for (unsigned i = 0; i < N; ++i) { /* setdiff_stable */
      int flag = 0;
      if (c->mother[i] <= T) {
        flag = 1;
      } else {
        for (unsigned j = 0; j < fsize; ++j)
          if (c->mother[i] == F[j]) {
            flag = 1;
            break;
          }
      }
      if (!flag) tmp[o++] = c->mother[i];
    }
    if (o < nk) return -1;
    for (unsigned i = 0; i < nk; ++i) kset[i] = tmp[o - nk + i];
  } else {
    for (unsigned i = 0; i < nk; ++i) kset[i] = c->mother[N - nk + i];
  }
  unsigned npc_rel = c->nPC > c->nWmPC ? c->nPC - c->nWmPC : 0;
  for (unsigned i = 0; i < npc_rel; ++i) c->pc[i] = kset[i];
  if (c->nWmPC == 1) c->pc[c->nPC - 1] = (K <= 21) ? 252 : 248;
  memset(c->kmask, 0, sizeof(c->kmask));
  for (unsigned i = 0; i < nk; ++i) c->kmask[kset[i]] = 1;
  /* sort PC set, sentinel */
  for (unsigned i = 0; i < c->nPC; ++i)
    for (unsigned j = i + 1; j < c->nPC; ++j)
      if (c->pc[j] < c->pc[i]) {
        uint16_t t = c->pc[i];
        c->pc[i] = c->pc[j];
        c->pc[j] = t;
      }
  c->pc[c->nPC] = NMAX;
  return 0;
}

/* Code description for tests: returns N (0 on error); kmask[N], pc[nPC] written. */
unsigned srs_oracle_polar_code(unsigned K, unsigned E, unsigned nMax, uint8_t* kmask, uint16_t* pc, unsigned* nPC)
{
  pcode c;
  if (build_code(&c, K, E, nMax, 0)) return 0;
  memcpy(kmask, c.kmask, c.N);
  for (unsigned i = 0; i < c.nPC; ++i) pc[i] = c.pc[i];
  *nPC = c.nPC;
  return c.N;
}

static void polar_transform(uint8_t* out, const uint8_t* in, unsigned N)
{
  /* stage_function recursion: out = [T(a) ^ T(b), T(b)] for in = [a, b] */
  if (N == 2) {
    out[0] = in[0] ^ in[1];
    out[1] = in[1];
    return;
  }
  unsigned h = N / 2;
  polar_transform(out, in, h);
  polar_transform(out + h, in + h, h);
  for (unsigned i = 0; i < h; ++i) out[i] ^= out[i + h];
}

/* allocate + encode + rate match (pdcch_encoder_impl / uci encoder chain), bits one per byte. */
int srs_oracle_polar_encode_chain(unsigned K, unsigned E, unsigned nMax, int ibil, const uint8_t* msg, uint8_t* out)
{
  pcode c;
  if (build_code(&c, K, E, nMax, ibil)) return -1;
  unsigned N = c.N;
  uint8_t  u[NMAX], x[NMAX], y[EMAX];
  memset(u, 0, N);
  if (c.nPC == 0) {
    for (unsigned i = 0, k = 0; i < N; ++i)
      if (c.kmask[i]) u[i] = msg[k++] & 1;
  } else {
    unsigned y0 = 0, y1 = 0, y2 = 0, y3 = 0, y4 = 0, ipc = 0, ik = 0;
    for (unsigned i = 0; i < N; ++i) {
      unsigned t = y0;
      y0 = y1;
      y1 = y2;
      y2 = y3;
      y3 = y4;
      y4 = t;
      if (c.kmask[i]) {
        if (i == c.pc[ipc]) {
          ipc++;
          u[i] = (uint8_t)y0;
        } else {
          u[i] = msg[ik] & 1;
          y0 ^= msg[ik] & 1;
          ik++;
        }
      }
    }
  }
  polar_transform(x, u, N);
  for (unsigned j = 0; j < N; ++j) y[j] = x[c.blk[j]];
  const uint8_t* e = y;
  if (E >= N) {
    for (unsigned k = N; k < E; ++k) y[k] = y[k % N];
  } else if (16 * K <= 7 * E) {
    e = y + (N - E);
  }
  if (!c.ibil) {
    memcpy(out, e, E);
  } else {
    unsigned S = 1, T = 1;
    while (S < E) {
      T++;
      S += T;
    }
    unsigned io = 0;
    for (unsigned r = 0; r < T; ++r) {
      unsigned ii = r;
      for (unsigned cc = 0; cc < T - r; ++cc) {
        if (ii < E) {
          out[io++] = e[ii];
          ii += T - cc;
        } else {
          break;
        }
      }
    }
  }
  return 0;
}

/* ---- LLR arithmetic (log_likelihood_ratio.cpp) ---- */
static int isinf8(int a) { return a > 120 || a < -120; }

/* a += b */
static int llr_sum(int a, int b)
{
  if (a == -b) return 0;
  if (isinf8(a)) return a;
  if (isinf8(b)) return b;
  int s = a + b;
  return s > 120 ? 120 : (s < -120 ? -120 : s);
}

static int llr_promotion_sum(int a, int b)
{
  if (a == -b) return 0;
  if (isinf8(a)) return a;
  if (isinf8(b)) return b;
  int s = a + b;
  return s > 120 ? 127 : (s < -120 ? -127 : s);
}

static int soft_xor(int x, int y)
{
  int ax = x < 0 ? -x : x, ay = y < 0 ? -y : y, m = ax < ay ? ax : ay;
  return (x * y < 0) ? -m : m;
}

typedef struct {
  const pcode* c;
  int8_t       llr[2 * NMAX]; /* stage s buffer at offset 2^s - 1 */
  uint8_t      est[NMAX];
  uint8_t      msg[NMAX];
  uint8_t      notr0[11][NMAX]; /* node type per stage: not rate-0 / rate-1 */
  uint8_t      r1[11][NMAX];
} ssc;

static void ssc_node(ssc* d, unsigned s, unsigned p)
{
  unsigned idx = p >> s;
  if (!d->notr0[s][idx]) return; /* rate-0: bits stay 0 */
  int8_t*  L = d->llr + ((1u << s) - 1);
  unsigned size = 1u << s;
  if (d->r1[s][idx]) { /* rate-1 */
    for (unsigned i = 0; i < size; ++i) d->est[p + i] = L[i] <= 0;
    if (s == 0) {
      d->msg[p] = d->est[p];
    } else {
      polar_transform(d->msg + p, d->est + p, size);
    }
    return;
  }
  unsigned h = size / 2;
  int8_t*  Lc = d->llr + (h - 1);
  for (unsigned i = 0; i < h; ++i) Lc[i] = (int8_t)soft_xor(L[i], L[i + h]);
  ssc_node(d, s - 1, p);
  for (unsigned i = 0; i < h; ++i) {
    /* switch_combine(llr1, llr0, b): b == 0 ? llr1 + llr0 : llr1 - llr0 ( (-llr0) += llr1 ) */
    Lc[i] = (int8_t)(d->est[p + i] == 0 ? llr_sum(L[i], L[i + h]) : llr_sum(-L[i], L[i + h]));
  }
  ssc_node(d, s - 1, p + h);
  for (unsigned i = 0; i < h; ++i) d->est[p + i] ^= d->est[p + h + i];
}

/* rate dematch + SSC decode + deallocate. llr: E values; msg: K bits. */
int srs_oracle_polar_decode_chain(unsigned K, unsigned E, unsigned nMax, int ibil, const int8_t* llr, uint8_t* msg)
{
  static pcode c;
  static ssc   d;
  if (build_code(&c, K, E, nMax, ibil)) return -1;
  unsigned N = c.N, n = c.n;
  int      ebuf[EMAX + NMAX];
  int*     e = ebuf + NMAX; /* room for the puncture shift */
  if (!c.ibil) {
    for (unsigned i = 0; i < E; ++i) e[i] = llr[i];
  } else {
    unsigned S = 1, T = 1;
    while (S < E) S += ++T;
    unsigned io = 0;
    for (unsigned r = 0; r < T; ++r) {
      unsigned ii = r;
      for (unsigned cc = 0; cc < T - r; ++cc) {
        if (ii < E) {
          e[ii] = llr[io++];
          ii += T - cc;
        } else {
          break;
        }
      }
    }
  }
  int* y = e;
  if (E >= N) {
    for (unsigned k = N; k < E; ++k) y[k % N] = llr_promotion_sum(y[k % N], e[k]);
  } else if (16 * K <= 7 * E) {
    y = e - (N - E);
    for (unsigned k = 0; k < N - E; ++k) y[k] = 0;
  } else {
    for (unsigned k = E; k < N; ++k) y[k] = 127;
  }
  d.c = &c;
  int8_t* top = d.llr + (N - 1);
  for (unsigned j = 0; j < N; ++j) top[c.blk[j]] = (int8_t)y[j];
  memset(d.est, 0, N);
  memset(d.msg, 0, N);
  /* node types (polar_decoder_impl.cpp:85-121) */
  for (unsigned j = 0; j < N; ++j) {
    d.notr0[0][j] = c.kmask[j];
    d.r1[0][j] = c.kmask[j];
  }
  for (unsigned s = 1; s <= n; ++s)
    for (unsigned j = 0; j < (N >> s); ++j) {
      d.notr0[s][j] = d.notr0[s - 1][2 * j] | d.notr0[s - 1][2 * j + 1];
      d.r1[s][j] = d.r1[s - 1][2 * j] & d.r1[s - 1][2 * j + 1];
    }
  ssc_node(&d, n, 0);
  unsigned ipc = 0, ik = 0;
  for (unsigned i = 0; i < N; ++i) {
    if (!c.kmask[i]) continue;
    if (i == c.pc[ipc]) {
      ipc++;
    } else {
      msg[ik++] = d.msg[i];
    }
  }
  return 0;
}

/* DCI input bit interleaver (TS 38.212 5.3.1.1), dir 0 = tx, 1 = rx. */
int srs_oracle_polar_interleave(const uint8_t* in, uint8_t* out, unsigned K, int dir)
{
  if (K > 164) return -1;
  unsigned k = 0;
  for (unsigned m = 0; m < 164; ++m) {
    if (SRS_POLAR_IL_PATTERN[m] >= 164 - K) {
      unsigned pi = SRS_POLAR_IL_PATTERN[m] - (164 - K);
      if (dir == 0) {
        out[k] = in[pi];
      } else {
        out[pi] = in[k];
      }
      k++;
    }
  }
  return 0;
}
