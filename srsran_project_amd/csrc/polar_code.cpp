// polar_code.cpp -- polar code construction on the host (configuration-time,
// like the reference's polar_code object) plus the index maps and SSC decoder
// program for the MI355X polar kernels (polar.hip).
//
// Construction follows lib/phy/upper/channel_coding/polar/polar_code_impl.cpp:
//   set_code_params (:367-410): nPC = 3 (+1 weight-based when E > K + 189) for
//     K <= 25; e = ceil(log2 E); n1 = e - 1 if E <= 9/8 * 2^(e-1) and K/E < 9/16;
//     n = max(5, min(n1, ceil(log2 K) + 3, nMax));
//   set (:420-490): the K + nPC most reliable positions (reliability sequence,
//     TS 38.212 Table 5.3.1.2-1), after removing the positions frozen by
//     puncturing (16K <= 7E: the first N-E interleaved bits plus every index <= T)
//     or shortening (the last N-E interleaved bits, and index 0 via T = 0);
//     PC positions = the nPC - nWmPC least reliable of them (+ 248/252).
// The SSC decoder program is the depth-first walk of polar_decoder_impl.cpp
// (rate-0 nodes produce nothing, rate-1 nodes take hard decisions, rate-R
// nodes apply f, recurse, apply g, recurse, combine), flattened once per code.
#include "polar_code.h"

#include <algorithm>
#include <cstring>

namespace srs_amd {

#define SRS_POLAR_TABLE_QUAL static const
#include "polar_tables.inc"

namespace {

const uint16_t SUBBLOCK_P[32] = {0,  1,  2,  4,  3,  5,  6,  7,  8,  16, 9,  17, 10, 18, 11, 19,
                                 12, 20, 13, 21, 14, 22, 15, 23, 24, 25, 26, 28, 27, 29, 30, 31};

const char* code_params(polar_code_desc& c, unsigned K, unsigned E, unsigned nMax)
{
  if (E > POLAR_EMAX) {
    return "Invalid E value";
  }
  if (nMax == 9) {
    if (K < 36 || K > 164) {
      return "Invalid K range";
    }
  } else if (nMax == 10) {
    if (K < 18 || (K > 25 && K < 31) || K > 1023) {
      return "Invalid K range";
    }
  } else {
    return "Invalid nMax";
  }
  c.K     = K;
  c.E     = E;
  c.nPC   = 0;
  c.nWmPC = 0;
  if (K <= 25) {
    c.nPC = 3;
    if (E > K + 189) {
      c.nWmPC = 1;
    }
  }
  if (!(K + c.nPC < E)) {
    return "Invalid K + nPC values";
  }
  unsigned e = 1;
  for (; e <= 13; ++e) {
    if ((1u << e) >= E) {
      break;
    }
  }
  const unsigned n1 = ((8 * E <= 9 * (1u << (e - 1))) && (16 * K < 9 * E)) ? e - 1 : e;
  unsigned       k  = 0;
  for (; k <= 10; ++k) {
    if ((1u << k) >= K) {
      break;
    }
  }
  unsigned n = std::min(n1, k + 3);
  n          = std::min(n, nMax);
  n          = std::max(n, 5u);
  c.n        = n;
  c.N        = 1u << n;
  if (!(K < c.N)) {
    return "Invalid K value";
  }
  return nullptr;
}

// Flattens the SSC walk of polar_decoder_impl.cpp:204-330.
struct program_builder {
  std::vector<std::vector<uint8_t>> not_r0, r1;
  std::vector<uint32_t>&            ops;
  explicit program_builder(std::vector<uint32_t>& o) : ops(o) {}
  static uint32_t op(uint32_t type, unsigned s, unsigned p) { return type | (s << 2) | (p << 8); }
  void            node(unsigned s, unsigned p)
  {
    const unsigned idx = p >> s;
    if (!not_r0[s][idx]) {
      return; // rate 0: the estimated and decoded bits stay zero
    }
    if (r1[s][idx]) {
      ops.push_back(op(POLAR_OP_R1, s, p));
      return;
    }
    const unsigned h = 1u << (s - 1);
    ops.push_back(op(POLAR_OP_F, s, p));
    node(s - 1, p);
    ops.push_back(op(POLAR_OP_G, s, p));
    node(s - 1, p + h);
    ops.push_back(op(POLAR_OP_XOR, s, p));
  }
};

} // namespace

const char* build_polar_code(polar_code_desc& c, unsigned K, unsigned E, unsigned nMax, bool ibil)
{
  c = polar_code_desc{};
  if (const char* msg = code_params(c, K, E, nMax)) {
    return msg;
  }
  const unsigned N = c.N;
  c.ibil           = ibil;
  std::vector<uint16_t> mother;
  mother.reserve(N);
  for (unsigned i = 0; i < POLAR_NMAX; ++i) {
    if (SRS_POLAR_Q1024[i] < N) {
      mother.push_back(SRS_POLAR_Q1024[i]);
    }
  }
  c.blk.resize(N);
  for (unsigned i = 0; i < N; ++i) {
    c.blk[i] = static_cast<uint16_t>(SUBBLOCK_P[(32 * i) / N] * (N / 32) + i % (N / 32));
  }

  // Information + parity-check positions, least reliable first.
  const unsigned        nk = K + c.nPC;
  std::vector<uint16_t> kset;
  if (N > E) {
    unsigned              T = 0;
    std::vector<uint16_t> F;
    if (16 * K <= 7 * E) {
      const unsigned Nth = 3 * N / 4;
      T                  = (E >= Nth) ? Nth - (E >> 1) - 1 : 9 * N / 16 - (E >> 2);
      F.assign(c.blk.begin(), c.blk.begin() + (N - E));
      c.mode = 1;
    } else {
      F.assign(c.blk.begin() + E, c.blk.end());
      c.mode = 2;
    }
    std::vector<uint16_t> remaining;
    for (uint16_t x : mother) {
      if (x > T && std::find(F.begin(), F.end(), x) == F.end()) {
        remaining.push_back(x);
      }
    }
    if (remaining.size() < nk) {
      return "Invalid K value";
    }
    kset.assign(remaining.end() - nk, remaining.end());
  } else {
    kset.assign(mother.end() - nk, mother.end());
    c.mode = 0;
  }
  const unsigned npc_rel = c.nPC > c.nWmPC ? c.nPC - c.nWmPC : 0;
  c.PC_set.assign(kset.begin(), kset.begin() + npc_rel);
  if (c.nWmPC == 1) {
    c.PC_set.push_back(K <= 21 ? 252 : 248);
  }
  std::sort(c.PC_set.begin(), c.PC_set.end());
  c.K_set.assign(N, 0);
  for (uint16_t x : kset) {
    c.K_set[x] = 1;
  }
  // Message positions: K_set order, skipping parity-check positions as the
  // allocator / deallocator do (polar_allocator_impl.cpp:49, polar_deallocator_impl.cpp:31).
  unsigned ipc = 0;
  for (unsigned i = 0; i < N; ++i) {
    if (!c.K_set[i]) {
      continue;
    }
    if (ipc < c.PC_set.size() && i == c.PC_set[ipc]) {
      ++ipc;
    } else {
      c.msg_pos.push_back(static_cast<uint16_t>(i));
    }
  }

  // Channel interleaver (polar_rate_matcher_impl.cpp:63): f[i_out] = e[i_in].
  std::vector<uint16_t> f_from_e(E);
  if (ibil) {
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
          f_from_e[io++] = static_cast<uint16_t>(ii);
          ii += T - cc;
        } else {
          break;
        }
      }
    }
  } else {
    for (unsigned k = 0; k < E; ++k) {
      f_from_e[k] = static_cast<uint16_t>(k);
    }
  }
  c.rx_e2f.assign(E, 0);
  for (unsigned k = 0; k < E; ++k) {
    c.rx_e2f[f_from_e[k]] = static_cast<uint16_t>(k);
  }
  // Transmit gather: f[k] = e[f_from_e[k]], e[m] = y[sel(m)], y[j] = x[blk[j]].
  c.tx_map.resize(E);
  for (unsigned k = 0; k < E; ++k) {
    const unsigned m = f_from_e[k];
    unsigned       j = m;
    if (E >= N) {
      j = m % N;
    } else if (c.mode == 1) {
      j = m + (N - E);
    }
    c.tx_map[k] = c.blk[j];
  }

  // SSC program (node types as polar_decoder_impl.cpp:85-121).
  program_builder pb(c.program);
  pb.not_r0.assign(c.n + 1, std::vector<uint8_t>(N, 0));
  pb.r1.assign(c.n + 1, std::vector<uint8_t>(N, 0));
  for (unsigned j = 0; j < N; ++j) {
    pb.not_r0[0][j] = c.K_set[j];
    pb.r1[0][j]     = c.K_set[j];
  }
  for (unsigned s = 1; s <= c.n; ++s) {
    for (unsigned j = 0; j < (N >> s); ++j) {
      pb.not_r0[s][j] = pb.not_r0[s - 1][2 * j] | pb.not_r0[s - 1][2 * j + 1];
      pb.r1[s][j]     = pb.r1[s - 1][2 * j] & pb.r1[s - 1][2 * j + 1];
    }
  }
  pb.node(c.n, 0);
  return nullptr;
}

bool polar_interleave(uint8_t* out, const uint8_t* in, unsigned K, int dir)
{
  if (K > 164) {
    return false;
  }
  unsigned k = 0;
  for (unsigned m = 0; m < 164; ++m) {
    if (SRS_POLAR_IL_PATTERN[m] >= 164 - K) {
      const unsigned pi = SRS_POLAR_IL_PATTERN[m] - (164 - K);
      if (dir == 0) {
        out[k] = in[pi];
      } else {
        out[pi] = in[k];
      }
      ++k;
    }
  }
  return true;
}

} // namespace srs_amd
