/*
 * srsran_amd/ssb.h -- C-ABI of the MI355X SS/PBCH block processor: PBCH encoding (payload generation with the
 * timing bits, first scrambling, CRC24C attachment, input bit interleaving, polar coding with nMax = 9, rate matching
 * to 864 bits), PBCH scrambling and QPSK, the PBCH DM-RS, the PSS and the SSS, mapped into resource grids.
 *
 * Replaces (reference interface):
 *   ssb_processor::process(resource_grid_writer& grid, const pdu_t& pdu)
 *       include/srsran/phy/upper/channel_processors/ssb/ssb_processor.h:77
 *       (impl lib/phy/upper/channel_processors/ssb/ssb_processor_impl.cpp:29-109 with pbch_encoder_impl.cpp,
 *        pbch_modulator_impl.cpp and lib/phy/upper/signal_processors/ssb/{dmrs_pbch,pss,sss}_processor_impl.cpp;
 *        block position from include/srsran/ran/ssb/ssb_mapping.h ssb_get_l_first / ssb_get_k_first)
 *   created by ssb_processor_factory (ssb/factories.h).
 * The slot form runs every SS/PBCH block of a slot -- of many cells' grids -- as one launch sequence: the payload /
 * scrambling / CRC / interleaving kernel, one polar-encoder launch (K = 56, E = 864), one mapping launch for the
 * PBCH, DM-RS, PSS and SSS REs of every block.  Grids are cbf16 [port][14][nof_subc] (normal cyclic prefix).  Grid
 * values are bit-exact with the reference (tests/test_ssb_gpu.py).
 */
#ifndef SRSRAN_AMD_SSB_H
#define SRSRAN_AMD_SSB_H

#include <stdint.h>

#include "srsran_amd/ldpc.h" /* SRS_AMD_OK, SRS_AMD_EINVAL, srs_amd_last_error */

#ifdef __cplusplus
extern "C" {
#endif

#define SRS_AMD_SSB_MIB_BITS 24 /* ssb_processor::MIB_PAYLOAD_SIZE */

/* ssb_processor::pdu_t (ssb_processor.h:33-62) and the grid it goes to.  The slot_point is given as its numerology,
 * system frame number and slot index within the frame. */
typedef struct srs_amd_ssb_pdu {
  uint32_t numerology;        /* of the slot (0 .. 4) */
  uint32_t sfn;               /* slot.sfn(), 0 .. 1023 */
  uint32_t slot_index;        /* slot.slot_index(): slot within the 10 ms frame */
  uint32_t phys_cell_id;      /* 0 .. 1007 */
  float    beta_pss_dB;       /* PSS power relative to SSS */
  uint32_t ssb_idx;           /* SS/PBCH block index in the burst */
  uint32_t L_max;             /* 4, 8 or 64 */
  uint32_t common_scs;        /* subCarrierSpacingCommon: 0 = 15 kHz, 1 = 30, 2 = 60, 3 = 120 kHz */
  uint32_t subcarrier_offset; /* k_SSB (ssb_subcarrier_offset) */
  uint32_t offset_to_pointA;  /* ssb_offset_to_pointA, in PRBs of the point-A SCS */
  uint32_t pattern_case;      /* ssb_pattern_case: 0 A, 1 B, 2 C, 3 D, 4 E */
  uint8_t  mib_payload[SRS_AMD_SSB_MIB_BITS]; /* one bit per byte */
  uint32_t nof_ports;         /* 1 .. 4 */
  uint8_t  ports[4];          /* grid port of each transmission port */
  uint32_t grid;              /* index of the grid in d_grids */
  uint32_t* d_grid;           /* non-NULL: this PDU's own DEVICE grid instead of d_grids[grid] */
} srs_amd_ssb_pdu;

typedef struct srs_amd_ssb_processor srs_amd_ssb_processor;

int  srs_amd_ssb_processor_create(srs_amd_ssb_processor** proc, int device);
void srs_amd_ssb_processor_destroy(srs_amd_ssb_processor* proc);

/* The block's first OFDM symbol within its slot and first subcarrier (ssb_processor_impl.cpp:32-38) after the checks
 * the reference asserts (the slot holds the block, the offsets give an integer subcarrier of the SSB SCS, the SSB
 * index exists in the pattern).  Returns SRS_AMD_OK or SRS_AMD_EINVAL with the reason. */
int srs_amd_ssb_position(const srs_amd_ssb_pdu* pdu, uint32_t* first_symbol, uint32_t* first_subcarrier);

/* DEVICE, asynchronous: every SS/PBCH block of a slot (several grids) into cbf16 grids [port][14][nof_subc]
 * (grid_stride uint32 apart), writing only the block's PBCH, DM-RS, PSS and SSS REs. */
int srs_amd_ssb_process_slot(srs_amd_ssb_processor* proc,
                             const srs_amd_ssb_pdu* pdus,
                             uint32_t               nof_pdus,
                             uint32_t*              d_grids,
                             uint64_t               grid_stride,
                             uint32_t               nof_grids,
                             uint32_t               nof_grid_ports,
                             uint32_t               nof_subc,
                             void*                  stream);

/* HOST, synchronous: one PDU into a host grid [nof_ports][14][nof_subc] (its other REs untouched). */
int srs_amd_ssb_process(srs_amd_ssb_processor* proc,
                        const srs_amd_ssb_pdu* pdu,
                        uint32_t*              grid,
                        uint32_t               nof_ports,
                        uint32_t               nof_subc);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_SSB_H */
