// ldpc_graph.cpp -- host-side construction of lifted LDPC graphs and CRC tables.
//
// Base graph data: TS 38.212 Tables 5.3.2-2 / 5.3.2-3 (bg_tables.inc).
// Reference counterpart: lib/phy/upper/channel_coding/ldpc/ldpc_luts_impl.cpp:4530
// (get_graph: shift = V mod Z) and ldpc_graph_impl.cpp.
#include "ldpc_common.h"

#include <algorithm>

namespace srs_amd {

#include "bg_tables.inc"

int lifting_index(int Z)
{
  static const int odd_to_ils[16] = {-1, 0, -1, 1, -1, 2, -1, 3, -1, 4, -1, 5, -1, 6, -1, 7};
  if (Z < 2 || Z > MAX_LIFTING_SIZE) {
    return -1;
  }
  int a = Z;
  while ((a & 1) == 0) {
    a >>= 1;
  }
  return (a > 15) ? -1 : odd_to_ils[a];
}

int lifting_size_position(int Z)
{
  static const int sizes[NOF_LIFTING_SIZES] = {2,   3,   4,   5,   6,   7,   8,   9,   10,  11,  12,  13,  14,
                                               15,  16,  18,  20,  22,  24,  26,  28,  30,  32,  36,  40,  44,
                                               48,  52,  56,  60,  64,  72,  80,  88,  96,  104, 112, 120, 128,
                                               144, 160, 176, 192, 208, 224, 240, 256, 288, 320, 352, 384};
  for (int i = 0; i < NOF_LIFTING_SIZES; ++i) {
    if (sizes[i] == Z) {
      return i;
    }
  }
  return -1;
}

bool build_lifted_graph(lifted_graph& g, int bg, int Z)
{
  const unsigned short(*tab)[10] = nullptr;
  int count                      = 0;
  if (bg == 1) {
    g.K = 22; g.N_full = 68; g.N_short = 66; g.M = 46;
    tab   = SRS_BG1_EDGES;
    count = SRS_BG1_EDGES_COUNT;
  } else if (bg == 2) {
    g.K = 10; g.N_full = 52; g.N_short = 50; g.M = 42;
    tab   = SRS_BG2_EDGES;
    count = SRS_BG2_EDGES_COUNT;
  } else {
    return false;
  }
  int ils = lifting_index(Z);
  if (ils < 0) {
    return false;
  }
  g.bg     = bg;
  g.Z      = Z;
  g.nedges = count;
  int m    = 0;
  g.row_start[0] = 0;
  for (int e = 0; e < count; ++e) {
    while (tab[e][0] != m) {
      g.row_start[++m] = e;
    }
    const uint32_t var   = tab[e][1];
    const uint32_t shift = tab[e][2 + ils] % Z;
    g.edge[e]            = (var * static_cast<uint32_t>(Z)) | (shift << 16);
  }
  while (m < g.M) {
    g.row_start[++m] = count;
  }
  for (int r = g.M + 1; r <= MAX_BG_M; ++r) {
    g.row_start[r] = count;
  }
  return true;
}

std::vector<uint32_t> all_lifted_edges()
{
  std::vector<uint32_t> edges(2 * NOF_LIFTING_SIZES * MAX_EDGES, 0);
  for (int bg = 1; bg <= 2; ++bg) {
    for (int z = 2; z <= MAX_LIFTING_SIZE; ++z) {
      if (lifting_size_position(z) < 0) {
        continue;
      }
      lifted_graph lg{};
      build_lifted_graph(lg, bg, z);
      std::copy(lg.edge, lg.edge + MAX_EDGES, edges.begin() + lifted_edges_offset(bg, z));
    }
  }
  return edges;
}

std::vector<uint32_t> crc_linear_table(int poly, int nbits)
{
  uint32_t polynom = 0;
  int      order   = 0;
  crc_params(poly, polynom, order);
  std::vector<uint32_t> t(nbits);
  const uint64_t        highbit = 1ull << order;
  uint64_t              r       = 1;
  for (int i = 0; i < order; ++i) {
    r <<= 1;
    if (r & highbit) {
      r ^= polynom;
    }
  }
  for (int k = 0; k < nbits; ++k) {
    t[k] = static_cast<uint32_t>(r & (highbit - 1));
    r <<= 1;
    if (r & highbit) {
      r ^= polynom;
    }
  }
  return t;
}

bool crc_params(int poly, uint32_t& polynom, int& order)
{
  switch (poly) {
    case 0: order = 24; polynom = 0x1864cfb; return true; // CRC24A
    case 1: order = 24; polynom = 0x1800063; return true; // CRC24B
    case 2: order = 24; polynom = 0x1b2b117; return true; // CRC24C
    case 3: order = 16; polynom = 0x11021; return true;   // CRC16
    case 4: order = 11; polynom = 0xe21; return true;     // CRC11
    case 5: order = 6; polynom = 0x61; return true;       // CRC6
    default: return false;
  }
}

} // namespace srs_amd
