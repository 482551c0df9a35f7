/*
 * srsran_amd/pdsch_modulator.h -- C-ABI of the MI355X PDSCH modulator and
 * PDSCH DM-RS processor: one launch turns a batch of encoded codewords into
 * precoded resource-grid REs (scrambling, modulation, layer mapping,
 * precoding, RE mapping fused), one launch writes the DM-RS of a batch of grids.
 *
 * Replaces (reference interfaces):
 *   pdsch_modulator::modulate(resource_grid_writer&, span<const bit_buffer>, const config_t&)
 *       include/srsran/phy/upper/channel_processors/pdsch/pdsch_modulator.h:97
 *       (impl lib/phy/upper/channel_processors/pdsch/pdsch_modulator_impl.cpp:94-115)
 *   dmrs_pdsch_processor::map(resource_grid_writer&, const config_t&)
 *       include/srsran/phy/upper/signal_processors/pdsch/dmrs_pdsch_processor.h:65
 *       (impl lib/phy/upper/signal_processors/pdsch/dmrs_pdsch_processor_impl.cpp:126-234)
 *   ptrs_pdsch_generator::generate(resource_grid_writer&, const configuration&)
 *       include/srsran/phy/upper/signal_processors/ptrs/ptrs_pdsch_generator.h
 *       (impl lib/phy/upper/signal_processors/ptrs/ptrs_pdsch_generator_impl.cpp:30-130, the pattern of
 *        lib/ran/ptrs/ptrs_pattern.cpp:54-110), as the third launch of the slot form
 *
 * Resource grids are complex bf16 (real in the low 16 bits of each 32-bit RE)
 * [port][symbol (14)][subcarrier], the reference's resource_grid_impl storage.
 * Only the REs the reference writes are written. Precoded values are bit-exact
 * with the reference's channel_precoder (generic / AVX2 / AVX512 agree).
 */
#ifndef SRSRAN_AMD_PDSCH_MODULATOR_H
#define SRSRAN_AMD_PDSCH_MODULATOR_H

#include <stdint.h>

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRS_AMD_MAX_RB 275
#define SRS_AMD_CRB_MASK_BYTES 35 /* ceil(275 / 8) */
#define SRS_AMD_MAX_RE_PATTERNS 8
#define SRS_AMD_MAX_LAYERS 4
#define SRS_AMD_MAX_TX_PORTS 4

/* re_pattern (include/srsran/phy/support/re_pattern.h:35): REs of the CRBs in
 * crb_mask (bit i % 8 of byte i / 8 = CRB i) at the subcarriers of re_mask
 * (bit k = subcarrier k of the RB) in the OFDM symbols of symbols (bit l). */
typedef struct srs_amd_re_pattern {
  uint8_t  crb_mask[SRS_AMD_CRB_MASK_BYTES];
  uint8_t  reserved0;
  uint16_t re_mask;
  uint16_t symbols;
} srs_amd_re_pattern;

/* pdsch_modulator::config_t (pdsch_modulator.h:50-85), the frequency allocation
 * resolved to CRBs (rb_allocation::get_crb_indices). */
typedef struct srs_amd_pdsch_mod_config {
  uint32_t           rnti;
  uint32_t           n_id;
  int32_t            modulation;   /* Qm code: 0 pi/2-BPSK, 1 BPSK, 2 QPSK, 4, 6, 8 */
  uint32_t           bwp_start;    /* CRB */
  uint32_t           bwp_size;     /* RBs */
  uint8_t            crb_mask[SRS_AMD_CRB_MASK_BYTES]; /* allocated CRBs */
  uint8_t            reserved0;
  uint32_t           start_symbol; /* time_alloc */
  uint32_t           nof_symbols;
  uint32_t           dmrs_symbol_mask;
  uint32_t           dmrs_type;    /* 1 or 2 */
  uint32_t           nof_cdm_groups_without_data;
  float              scaling;      /* applied when normal, as the reference */
  uint32_t           nof_layers;   /* 1..4 */
  uint32_t           nof_ports;    /* 1..4, >= nof_layers */
  float              weights[SRS_AMD_MAX_LAYERS][SRS_AMD_MAX_TX_PORTS][2]; /* [layer][port] (re, im), PRG 0 */
  uint32_t           nof_reserved;
  srs_amd_re_pattern reserved[SRS_AMD_MAX_RE_PATTERNS];
} srs_amd_pdsch_mod_config;

/* dmrs_pdsch_processor::config_t (dmrs_pdsch_processor.h:38-57). The reference
 * maps with one precoding PRG (dmrs_pdsch_processor_impl.cpp:149). */
typedef struct srs_amd_dmrs_pdsch_config {
  uint32_t slot_index;            /* slot_point::slot_index() */
  uint32_t reference_point_k_rb;
  uint32_t type;                  /* 1 or 2 */
  uint32_t scrambling_id;
  uint32_t n_scid;
  float    amplitude;
  uint32_t symbols_mask;
  uint8_t  crb_mask[SRS_AMD_CRB_MASK_BYTES];
  uint8_t  reserved0;
  uint32_t nof_layers;            /* DM-RS ports 0..nof_layers-1 */
  uint32_t nof_ports;
  float    weights[SRS_AMD_MAX_LAYERS][SRS_AMD_MAX_TX_PORTS][2];
} srs_amd_dmrs_pdsch_config;

typedef struct srs_amd_pdsch_modulator srs_amd_pdsch_modulator;
typedef struct srs_amd_pdsch_mod_plan  srs_amd_pdsch_mod_plan;

int  srs_amd_pdsch_modulator_create(srs_amd_pdsch_modulator** mod, int device);
void srs_amd_pdsch_modulator_destroy(srs_amd_pdsch_modulator* mod);

/* Resolves the RE allocation of a configuration for grids of nof_subc
 * subcarriers once (the reserved list + DM-RS pattern exclusion of
 * pdsch_modulator_impl.cpp:53-86) and uploads it. *nof_re = data REs per
 * layer; a codeword must carry nof_re * nof_layers * Qm bits. */
int  srs_amd_pdsch_mod_plan_create(srs_amd_pdsch_modulator*        mod,
                                   const srs_amd_pdsch_mod_config* cfg,
                                   uint32_t                        nof_subc,
                                   srs_amd_pdsch_mod_plan**        plan,
                                   uint32_t*                       nof_re);
void srs_amd_pdsch_mod_plan_destroy(srs_amd_pdsch_mod_plan* plan);

/* PDSCH PT-RS (ptrs_pdsch_generator::configuration, ptrs_pdsch_generator.h; pdsch_process_ptrs,
 * pdsch_processor_helpers.h:78-118, builds it from the PDU).  Contiguous allocations (get_ptrs_pattern). */
typedef struct srs_amd_ptrs_pdsch_config {
  uint32_t     slot_index;           /* slot_point::slot_index() */
  uint32_t     rnti;
  uint32_t     dmrs_type;            /* 1 or 2 */
  uint32_t     reference_point_k_rb;
  uint32_t     scrambling_id;
  uint32_t     n_scid;
  float        amplitude;            /* convert_dB_to_amplitude(PT-RS to data ratio - data to SSS ratio) */
  uint32_t     dmrs_symbols_mask;
  uint8_t      crb_mask[SRS_AMD_CRB_MASK_BYTES]; /* the PDSCH CRBs (contiguous) */
  uint8_t      reserved0;
  uint32_t     start_symbol;         /* time allocation */
  uint32_t     nof_symbols;
  uint32_t     freq_density;         /* K_PT-RS: 2 or 4 */
  uint32_t     time_density;         /* L_PT-RS: 1, 2 or 4 */
  uint32_t     re_offset;            /* ptrs_re_offset: 0 .. 3 */
  uint32_t     nof_ports;            /* transmit ports, 1 .. 4 */
  uint32_t     nof_prg;              /* precoding PRGs, >= 1 */
  uint32_t     prg_size;             /* PRBs per PRG */
  const float* weights;              /* HOST [nof_prg][nof_ports] (re, im): the layer-0 weights (TS 38.214 5.1.6.3) */
} srs_amd_ptrs_pdsch_config;

/* The PT-RS REs as an RE pattern (get_ptrs_pattern, ptrs_pattern.cpp:54-110, with one port), validating cfg.  The
 * reference's PDSCH processor maps data over them and then the PT-RS (pdsch_processor_hip.h explains why its
 * codeword does not exclude them either). */
int srs_amd_ptrs_pdsch_reserved(const srs_amd_ptrs_pdsch_config* cfg, srs_amd_re_pattern* pattern);

/* HOST, synchronous: grid [grid_ports][14][nof_subc] cbf16 (as uint32) updated in
 * place; codeword packed MSB first (bit_buffer), nof_bits bits. */
int srs_amd_pdsch_modulate(srs_amd_pdsch_modulator*      mod,
                           const srs_amd_pdsch_mod_plan* plan,
                           uint32_t*                     grid,
                           uint32_t                      grid_ports,
                           const uint8_t*                codeword,
                           uint32_t                      nof_bits);

/* DEVICE, asynchronous: nof_cws codewords (rows of cw_stride bytes) into nof_cws
 * grids (grid_stride REs apart, ports nof_subc * 14 REs apart).  A codeword of other than nof_re x layers x Qm
 * bits maps as the reference's resource_grid_mapper consumes its symbol buffer: a longer one maps its first
 * nof_re x layers modulation symbols and the rest is dropped (pdsch_processor_impl sizes a DM-RS type-2 codeword
 * with the type-2 pattern but maps it around the type-1 one, see pdsch_processor_hip.h); a shorter one fills the
 * first nof_bits / (layers x Qm) REs of the allocation in mapping order and leaves the others untouched, the mapper
 * stopping when its buffer runs empty (resource_grid_mapper_impl.cpp:453-456 -- a PT-RS PDU's codeword, sized
 * without the PT-RS REs). */
int srs_amd_pdsch_modulate_batch(srs_amd_pdsch_modulator*      mod,
                                 const srs_amd_pdsch_mod_plan* plan,
                                 uint32_t*                     d_grids,
                                 uint64_t                      grid_stride,
                                 const uint8_t*                d_codewords,
                                 uint32_t                      cw_stride,
                                 uint32_t                      nof_bits,
                                 uint32_t                      nof_cws,
                                 void*                         stream);

/* HOST, synchronous DM-RS mapping into grid [grid_ports][14][nof_subc]. */
int srs_amd_dmrs_pdsch_map(srs_amd_pdsch_modulator*         mod,
                           const srs_amd_dmrs_pdsch_config* cfg,
                           uint32_t*                        grid,
                           uint32_t                         grid_ports,
                           uint32_t                         nof_subc);

/* DEVICE, asynchronous DM-RS mapping into nof_grids grids. */
int srs_amd_dmrs_pdsch_map_batch(srs_amd_pdsch_modulator*         mod,
                                 const srs_amd_dmrs_pdsch_config* cfg,
                                 uint32_t*                        d_grids,
                                 uint64_t                         grid_stride,
                                 uint32_t                         nof_subc,
                                 uint32_t                         nof_grids,
                                 void*                            stream);

/* One PDSCH PDU of a slot (srs_amd_pdsch_modulate_slot): its data (plan + codeword) and its DM-RS. */
typedef struct srs_amd_pdsch_slot_pdu {
  const srs_amd_pdsch_mod_plan*    plan;      /* NULL: no data (DM-RS only) */
  const srs_amd_dmrs_pdsch_config* dmrs;      /* NULL: no DM-RS */
  uint32_t                         grid;      /* index of the grid in d_grids */
  uint32_t                         nof_bits;  /* codeword length (>= nof_re x layers x Qm, see _batch) */
  uint64_t                         cw_offset; /* byte offset of the packed codeword in d_codewords */
  uint32_t*                        d_grid;    /* non-NULL: this PDU's own DEVICE grid cbf16 [port][14][nof_subc]
                                                 (a device-resident resource grid), instead of d_grids[grid] */
  const srs_amd_ptrs_pdsch_config* ptrs;      /* NULL: no PT-RS; else mapped after the data and before the DM-RS */
} srs_amd_pdsch_slot_pdu;

/* DEVICE, asynchronous: every PDSCH PDU of a slot -- several UEs on disjoint PRBs of one grid (or of several
 * grids), each with its own PRBs, symbols, layers, modulation, precoding, rnti / n_id, reserved REs and DM-RS
 * configuration -- as TWO launches (all data REs, then all DM-RS), per-PDU argument blocks in device memory.
 * Replaces calling pdsch_modulator::modulate and dmrs_pdsch_processor::map once per PDU
 * (pdsch_processor_impl.cpp:80 modulate + DM-RS per PDU, reached once per PDU from
 * downlink_processor_multi_executor_impl.cpp:104 process_pdsch).  Grid writes
 * per PDU identical to srs_amd_pdsch_modulate_batch / srs_amd_dmrs_pdsch_map_batch on that grid; PDUs
 * sharing a grid must not write the same RE (the order between them is unspecified).  Plans created for
 * nof_subc subcarriers. */
int srs_amd_pdsch_modulate_slot(srs_amd_pdsch_modulator*      mod,
                                const srs_amd_pdsch_slot_pdu* pdus,
                                uint32_t                      nof_pdus,
                                uint32_t*                     d_grids,
                                uint64_t                      grid_stride,
                                uint32_t                      nof_grids,
                                uint32_t                      nof_subc,
                                const uint8_t*                d_codewords,
                                void*                         stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_PDSCH_MODULATOR_H */
