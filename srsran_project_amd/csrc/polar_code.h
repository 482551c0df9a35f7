// polar_code.h -- host-side polar code construction (TS 38.212 5.3.1 / 5.4.1)
// and the precomputed index maps / SSC program the polar kernels consume.
#pragma once

#include <cstdint>
#include <vector>

namespace srs_amd {

constexpr unsigned POLAR_NMAX = 1024;
constexpr unsigned POLAR_EMAX = 8192;

// SSC decoder program op: type | stage << 2 | pos << 8
enum polar_op : uint32_t { POLAR_OP_F = 0, POLAR_OP_G = 1, POLAR_OP_XOR = 2, POLAR_OP_R1 = 3 };

struct polar_code_desc {
  unsigned K = 0, E = 0, n = 0, N = 0, nPC = 0, nWmPC = 0;
  bool     ibil = false;
  std::vector<uint8_t>  K_set;     // [N] information (incl. parity-check) positions
  std::vector<uint16_t> PC_set;    // sorted parity-check positions (nPC)
  std::vector<uint16_t> blk;       // [N] sub-block interleaver J(n)
  std::vector<uint16_t> msg_pos;   // [K] position of message bit k in u (K_set minus PC_set, ascending)
  std::vector<uint16_t> tx_map;    // [E] output bit k = x[tx_map[k]] (bit selection + interleavers)
  std::vector<uint16_t> rx_e2f;    // [E] received LLR index of rate-matched bit e[k] (channel deinterleaver)
  std::vector<uint32_t> program;   // SSC decoder ops
  int                   mode = 0;  // 0 repetition (E >= N), 1 puncturing, 2 shortening
};

// polar_code::set(K, E, nMax, ibil): returns nullptr or the reference's assertion message.
const char* build_polar_code(polar_code_desc& c, unsigned K, unsigned E, unsigned nMax, bool ibil);

// DCI input bit interleaver (polar_interleaver_impl.cpp:40): dir 0 = tx, 1 = rx.
bool polar_interleave(uint8_t* out, const uint8_t* in, unsigned K, int dir);

} // namespace srs_amd
