/*
 * srsran_amd/pdcch.h -- C-ABI of the MI355X PDCCH processor: DCI encoding (CRC24C attachment with the RNTI-scrambled
 * parity, DCI input bit interleaving, polar coding with nMax = 9, rate matching), scrambling, QPSK, power scaling,
 * precoding and mapping onto the CCEs' REGs, and the PDCCH DM-RS, into resource grids.
 *
 * Replaces (reference interface):
 *   pdcch_processor::process(resource_grid_writer& grid, const pdu_t& pdu)
 *       include/srsran/phy/upper/channel_processors/pdcch/pdcch_processor.h:129
 *       (impl lib/phy/upper/channel_processors/pdcch/pdcch_processor_impl.cpp:79-130, with pdcch_encoder_impl.cpp,
 *        pdcch_modulator_impl.cpp, lib/phy/upper/signal_processors/pdcch/dmrs_pdcch_processor_impl.cpp and the
 *        CCE-to-PRB mapping of lib/ran/pdcch/cce_to_prb_mapping.cpp)
 *   created by pdcch_processor_factory (pdcch/factories.h:60-72).
 * The slot form runs every DCI of a slot -- of many cells' grids -- as one launch sequence: the CRC / interleaving
 * kernel, one polar-encoder launch per (K, E) code, one mapping launch for all data and DM-RS REs.  Grids are cbf16
 * [port][14][nof_subc] (normal cyclic prefix).  Grid values are bit-exact with the reference (tests/test_pdcch_gpu.py).
 * Scope: one-layer precoding, identical on every PRG (wideband), as the PDSCH forms; the reference validator's checks
 * (pdcch_processor_validator_impl.cpp) apply.
 */
#ifndef SRSRAN_AMD_PDCCH_H
#define SRSRAN_AMD_PDCCH_H

#include <stdint.h>

#include "srsran_amd/ldpc.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRS_AMD_PDCCH_MAX_PAYLOAD 128 /* pdcch_constants::MAX_DCI_PAYLOAD_SIZE */
#ifndef SRS_AMD_CRB_MASK_BYTES
#define SRS_AMD_CRB_MASK_BYTES 35 /* ceil(275 / 8), as pdsch_modulator.h */
#endif

/* pdcch_processor::coreset_description (pdcch_processor.h:82-106). */
typedef struct srs_amd_pdcch_coreset {
  uint32_t bwp_size_rb;
  uint32_t bwp_start_rb;
  uint32_t start_symbol_index;
  uint32_t duration;               /* 1 .. 3 */
  uint8_t  frequency_resources[8]; /* freq_resource_bitmap (45 six-RB groups): bit i of byte i / 8 */
  uint32_t cce_to_reg_mapping;     /* 0 CORESET0, 1 non-interleaved, 2 interleaved */
  uint32_t reg_bundle_size;        /* interleaved: 2, 3 or 6 */
  uint32_t interleaver_size;       /* interleaved: 2, 3 or 6 */
  uint32_t shift_index;            /* interleaved / CORESET0: n_shift (CORESET0: the cell's N_id) */
} srs_amd_pdcch_coreset;

/* pdcch_processor::dci_description (pdcch_processor.h:55-76), wideband precoding of one layer onto nof_ports. */
typedef struct srs_amd_pdcch_dci {
  uint32_t rnti;                 /* CRC scrambling */
  uint32_t n_id_pdcch_dmrs;
  uint32_t n_id_pdcch_data;
  uint32_t n_rnti;               /* data scrambling */
  uint32_t cce_index;
  uint32_t aggregation_level;    /* 1, 2, 4, 8, 16 */
  float    dmrs_power_offset_dB;
  float    data_power_offset_dB;
  uint32_t payload_size;         /* DCI bits, 1 .. SRS_AMD_PDCCH_MAX_PAYLOAD */
  uint8_t  payload[SRS_AMD_PDCCH_MAX_PAYLOAD]; /* one bit per byte */
  uint32_t nof_ports;            /* 1 .. 4 */
  float    weights[4][2];        /* layer-0 precoding weight of each port (re, im) */
} srs_amd_pdcch_dci;

/* pdcch_processor::pdu_t (pdcch_processor.h:109-121) and the grid it goes to. */
typedef struct srs_amd_pdcch_pdu {
  uint32_t              numerology;
  uint32_t              slot_index;
  srs_amd_pdcch_coreset coreset;
  srs_amd_pdcch_dci     dci;
  uint32_t              grid;   /* index of the grid in d_grids */
  uint32_t*             d_grid; /* non-NULL: this PDU's own DEVICE grid instead of d_grids[grid] */
} srs_amd_pdcch_pdu;

typedef struct srs_amd_pdcch_processor srs_amd_pdcch_processor;

int  srs_amd_pdcch_processor_create(srs_amd_pdcch_processor** proc, int device);
void srs_amd_pdcch_processor_destroy(srs_amd_pdcch_processor* proc);

/* pdcch_processor_impl::compute_rb_mask (pdcch_processor_impl.cpp:44-77, cce_to_prb_mapping.cpp): the CRBs of the
 * DCI's CCEs into crb_mask (35 bytes, bit r of byte r / 8).  Also validates the PDU as pdcch_processor_validator_impl
 * (SRS_AMD_EINVAL with the reference's message otherwise).  Returns the number of CRBs (> 0) or an error (< 0). */
int srs_amd_pdcch_rb_mask(const srs_amd_pdcch_pdu* pdu, uint8_t* crb_mask);

/* DEVICE, asynchronous: every PDCCH PDU of a slot (several per grid, several grids) into cbf16 grids
 * [port][14][nof_subc] (grid_stride uint32 apart), writing only the DCIs' data and DM-RS REs. */
int srs_amd_pdcch_process_slot(srs_amd_pdcch_processor* proc,
                               const srs_amd_pdcch_pdu* pdus,
                               uint32_t                 nof_pdus,
                               uint32_t*                d_grids,
                               uint64_t                 grid_stride,
                               uint32_t                 nof_grids,
                               uint32_t                 nof_subc,
                               void*                    stream);

/* HOST, synchronous: one PDU into a host grid [nof_ports][14][nof_subc] (its other REs untouched). */
int srs_amd_pdcch_process(srs_amd_pdcch_processor* proc,
                          const srs_amd_pdcch_pdu* pdu,
                          uint32_t*                grid,
                          uint32_t                 nof_ports,
                          uint32_t                 nof_subc);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_PDCCH_H */
