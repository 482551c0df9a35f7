// pusch_processor_hip.h -- srsran::pusch_processor (include/srsran/phy/upper/channel_processors/pusch/
// pusch_processor.h:35-185) and srsran::pusch_processor_factory (pusch/factories.h:102-108) over the srsran_amd
// C-ABI slot form (include/srsran_amd/pusch_processor.h, srs_amd_pusch_process_slot_ex): the channel_processor
// level of the boundary, so the reference's uplink processor (lib/phy/upper/uplink_processor_impl.cpp:270-326,
// one pusch_processor::process call per PDU) runs the MI355X slot path untouched.
//
// The reference's process() is asynchronous: it reports through pusch_processor_result_notifier when the
// transmission is decoded (pusch_processor_result_notifier.h).  This processor queues each PDU (its grid reader,
// transport-block span, rx_buffer and notifier) in a slot collector shared by every processor of one factory
// (so every cell of the node that uses the factory lands in one batch) and returns.  A collector thread runs a
// batch when
//   * the factory's flush() is called (the slot boundary: after uplink_processor_impl::handle_rx_symbol has
//     dispatched the last PDU of the slot),
//   * a PDU of another slot arrives (the pending slot is complete),
//   * max_pdus_per_batch PDUs are pending, or
//   * the oldest pending PDU has waited max_wait_us,
// as one srs_amd_pusch_process_slot_ex call: the grids are copied from the readers (resource_grid_reader::
// get_view, rows copied by a pool of worker threads into one of two alternating pinned staging buffers, one H2D
// copy per batch) -- or, for grids of a hip_resource_grid factory (hip_resource_grid.h), read in place in HBM --,
// every new-data UCI-free CP-OFDM PDU runs through the fused estimator-equalizer-decoder sequence, UCI / DFT-s-OFDM /
// HARQ PDUs through the batch chain in the same call.  A completion thread then waits for the batch, copies each
// PDU's transport block into its span and calls its notifier (on_uci, then on_sch), while the collector thread
// already stages the next batch.
//
// HARQ state stays in the reference's rx_buffer (the uplink processor's rx_buffer_pool decides its lifetime): a
// retransmission uploads the rx_buffer's codeblock soft bits, decoded messages and CRC flags into a device soft
// buffer and the decoded state goes back after the call; a new transmission whose TB CRC fails is decoded again
// with a device soft buffer in the same batch cycle and its state written to the rx_buffer, so the common case
// (TB CRC pass) moves no soft bits over PCIe.  As pusch_decoder_impl::join_and_notify, the rx_buffer is released on
// a TB CRC pass and unlocked otherwise.  The LDPC statistic of a codeblock OK from an earlier transmission is the
// processor's last count for that codeblock index (pusch_decoder_impl's cb_stats semantics).
//
// UCI-only PDUs (no codeword) run estimator, demodulator, demultiplexer and UCI decoders and are notified through
// on_uci alone, as pusch_processor_impl.cpp:305-324; dc_position zeroes the DC subcarrier's channel estimate of a
// CP-OFDM PDU (pusch_processor_impl.cpp:235-249).  Each PDU carries its own slot into the slot call, so PDUs of
// different slots that share a cached plan keep their own DM-RS sequences.
// Not supported (the validator reports it): DM-RS type 2 and interleaved / non-contiguous allocations (as the
// reference validator), more than four receive ports or layers.  Compiled against the reference's headers by
// integration/Makefile.
#pragma once

#include "srsran/phy/upper/channel_processors/pusch/factories.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_processor.h"
#include "srsran/phy/upper/equalization/channel_equalizer_algorithm_type.h"
#include "srsran/phy/upper/signal_processors/channel_estimator/port_channel_estimator_parameters.h"
#include <cstdint>
#include <memory>

namespace srsran {
namespace hip {

/// The MI355X PUSCH processor's configuration: pusch_processor_factory_sw_configuration's decoder fields
/// (factories.h:110-121) and the estimator / equalizer strategies its component factories take.
struct pusch_processor_hip_config {
  /// HIP device (-1: the current one).
  int device = -1;
  /// Resource grid width in PRBs the processor serves (the grids' subcarriers / 12).
  unsigned nof_prb = 273;
  /// LDPC decoder iterations, early stop, force decoding (pusch_processor_factory_sw_configuration).
  unsigned dec_nof_iterations    = 10;
  bool     dec_enable_early_stop = true;
  bool     dec_force_decoding    = false;
  /// Equalizer (channel_equalizer_factory) and channel-estimator strategies (dmrs_pusch_estimator_factory).
  channel_equalizer_algorithm_type                 equalizer        = channel_equalizer_algorithm_type::zf;
  port_channel_estimator_fd_smoothing_strategy     fd_smoothing     = port_channel_estimator_fd_smoothing_strategy::filter;
  port_channel_estimator_td_interpolation_strategy td_interpolation =
      port_channel_estimator_td_interpolation_strategy::interpolate;
  bool compensate_cfo = true;
  /// LDPC decoder arithmetic: the reference's "generic" decoder instead of its AVX2 / AVX512 ("auto") one.
  bool generic_ldpc = false;
  /// Slot collector: batch size bound and the longest time a PDU waits for its slot to complete (0: only the
  /// other triggers -- flush(), a new slot, max_pdus_per_batch).
  unsigned max_pdus_per_batch = 1024;
  unsigned max_wait_us        = 200;
  /// PDU configurations kept as C-ABI plans (plan creation uploads tables; a plan serves every slot).
  unsigned max_cached_plans = 4096;
  /// Worker threads copying the rows of host resource grids into the batch's pinned staging buffer (0: the
  /// collector thread alone).  Grids of a hip_resource_grid factory are used in HBM as they are.
  unsigned nof_copy_threads = 8;
  /// Worker threads (beside the completion thread) writing the batch's results -- transport blocks, HARQ state --
  /// and calling the notifiers, PDUs in parallel (0: the completion thread alone).
  unsigned nof_notify_threads = 4;
};

/// pusch_processor_factory whose processors share one slot collector and one MI355X PUSCH processor.
class pusch_processor_factory_hip : public pusch_processor_factory
{
public:
  /// Runs every pending PDU now (the slot boundary); returns without waiting for the batch.
  virtual void flush() = 0;
  /// Blocks until no PDU is pending or being processed (every notifier of the PDUs queued so far was called).
  virtual void wait_idle() = 0;
  /// Counters: PDUs processed, batches run, failed (error-reported) PDUs, new-data TBs decoded again (always 0 since
  /// r06: one decoding keeps the soft state), retransmissions, failed new-data TBs whose device soft buffer went to
  /// their rx_buffer.
  struct statistics {
    uint64_t nof_pdus = 0, nof_batches = 0, nof_errors = 0, nof_harq_redecodes = 0, nof_retransmissions = 0;
    uint64_t nof_harq_soft_downloads = 0;
    /// PDUs whose received grid was a hip_resource_grid read in place (no host staging, no PCIe copy).
    uint64_t nof_device_grids = 0;
    /// Host time (microseconds, all batches): the collector thread staging and issuing batches (stage_us, of which
    /// waiting for a free buffer set: set_wait_us), the completion thread waiting for batches' results (wait_us) and
    /// writing HARQ state / calling the notifiers (notify_us).
    uint64_t stage_us = 0, set_wait_us = 0, wait_us = 0, notify_us = 0;
    /// Parts of stage_us: device-grid reads, the slot call (descriptors + launches), the result downloads.
    uint64_t stage_reads_us = 0, stage_call_us = 0, stage_download_us = 0;
  };
  virtual statistics get_statistics() const = 0;
};

/// nullptr when the device or the MI355X processor cannot be created (logged).
std::shared_ptr<pusch_processor_factory_hip> create_pusch_processor_factory_hip(const pusch_processor_hip_config& cfg);

} // namespace hip
} // namespace srsran
