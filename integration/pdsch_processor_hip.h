// pdsch_processor_hip.h -- srsran::pdsch_processor (include/srsran/phy/upper/channel_processors/pdsch/
// pdsch_processor.h:189-213) and srsran::pdsch_processor_factory (pdsch/factories.h:79-85) over the srsran_amd
// C-ABI slot forms: every PDSCH PDU of a slot encoded by srs_amd_pdsch_encode_slot (TB CRC, segmentation, CB CRCs,
// LDPC encoding, rate matching) and mapped by srs_amd_pdsch_modulate_slot (scrambling, modulation, layer mapping,
// precoding, RE mapping, DM-RS), the twin of pusch_processor_hip.h on the downlink.
//
// The reference's downlink processor calls pdsch_processor::process once per PDU
// (downlink_processor_multi_executor_impl.cpp process_pdsch) with the slot's resource_grid_writer, and each PDU
// reports through pdsch_processor_notifier::on_finish_processing.  This processor queues each PDU (its writer,
// notifier, transport blocks -- shared_transport_block keeps them alive -- and configuration) in a slot collector
// shared by every processor of one factory (slot_collector.h: flush(), slot change, batch size or timer), and a
// batch runs as one encode launch sequence and one modulate launch pair over device grids (one per writer) whose
// REs start as a sentinel pattern (0xFFFF'FFFF, a bf16 NaN pair no PDSCH or DM-RS RE can take).  After one D2H copy
// the REs the PDUs wrote -- exactly the REs the reference's pdsch_processor_impl writes, its modulator and DM-RS
// mapper being bit-exact with the GPU kernels -- are stored into each writer's grid through
// resource_grid_writer::get_view, every other RE of the writer is left as it was; then on_finish_processing.
//
// Reproduced as the reference does it: pdsch_processor_impl sizes the codeword with the DM-RS pattern of the PDU's
// DM-RS type (pdsch_compute_nof_data_re) but its modulator excludes the default type-1 pattern
// (pdsch_processor_impl.cpp:185-200 leaves pdsch_modulator::config_t::dmrs_config_type unset), so a type-2 PDU's
// data skips its DM-RS symbols entirely (two CDM groups) and the codeword's last symbols are not mapped.
//
// PT-RS (pdsch_processor_impl.cpp:82-84, ptrs_pdsch_generator_impl.cpp) as the reference does it: the data mapper
// does not skip the PT-RS REs (the modulator gets only the PDU's reserved list, pdsch_processor_impl.cpp:148) and the
// codeword covers them too -- pdsch_compute_nof_data_re (pdsch_processor_helpers.h:146-175) builds the PT-RS pattern
// it merges into the reserved list on a default re_pattern, whose CRB bitmap has size 0, so its set() calls land
// outside the bitmap and the pattern counts no RE -- then the PT-RS overwrites the data at its REs.
// The PT-RS kernel precodes per PRG (srs_amd_ptrs_pdsch_config).
//
// Not supported (logged; the PDU's REs are not written, on_finish_processing still called so the downlink processor
// never stalls): more than four layers (two codewords), more than four ports, more than eight reserved RE patterns,
// extended cyclic prefix, and precoding that differs between PRGs -- the reference's DM-RS processor writes the
// weights of PRG >= 1 into a one-PRG configuration (dmrs_pdsch_processor_impl.cpp:150-160), an assertion with
// asserts on and an out-of-bounds write without (tests/test_oracle_vs_ref.py shows it crash), so it has no output to
// reproduce.  Compiled against the reference's headers by integration/Makefile.
#pragma once

#include "srsran/phy/upper/channel_processors/pdsch/factories.h"
#include "srsran/phy/upper/channel_processors/pdsch/pdsch_processor.h"
#include <cstdint>
#include <memory>

namespace srsran {
namespace hip {

struct pdsch_processor_hip_config {
  /// HIP device (-1: the current one).
  int device = -1;
  /// Resource grid width in PRBs (the writers' subcarriers / 12).
  unsigned nof_prb = 273;
  /// Slot collector: batch size bound and timer (0: only flush(), a new slot or max_pdus_per_batch).
  unsigned max_pdus_per_batch = 1024;
  unsigned max_wait_us        = 200;
  /// PDU configurations kept as C-ABI modulator plans.
  unsigned max_cached_plans = 4096;
  /// Worker threads merging the written rows of host resource grids (0: the completion thread alone).  Grids of a
  /// hip_resource_grid factory are written in place in HBM.
  unsigned nof_copy_threads = 8;
};

class pdsch_processor_factory_hip : public pdsch_processor_factory
{
public:
  /// Runs every pending PDU now (the slot boundary); returns without waiting.
  virtual void flush() = 0;
  /// Blocks until every PDU queued so far is in its grid and notified.
  virtual void wait_idle() = 0;
  struct statistics {
    uint64_t nof_pdus = 0, nof_batches = 0, nof_errors = 0;
    /// Device-resident grids (hip_resource_grid) written in place, counted once per batch.
    uint64_t nof_device_grids = 0;
  };
  virtual statistics get_statistics() const = 0;
};

/// nullptr when the device or the MI355X encoder / modulator cannot be created (logged).
std::shared_ptr<pdsch_processor_factory_hip> create_pdsch_processor_factory_hip(const pdsch_processor_hip_config& cfg);

} // namespace hip
} // namespace srsran
