// kernel_probe.h -- the launch side of the live kernel probes (include/srsran_amd/profiling.h).  A probed launch goes
// through hipExtLaunchKernelGGL with the probe's start / stop events, which the launch's own dispatch packet
// timestamps: no extra packets enter the stream, so the timed step runs as it does unprobed.  An unarmed probe costs
// one relaxed atomic load.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

struct probe_events {
  int        slot  = -1; // -1: not armed (or every slot used): launch unprobed
  hipEvent_t start = nullptr, stop = nullptr;
};

// The events of the next recorded launch of `probe`.
probe_events probe_take(int probe);
// The launch of slot `slot` was issued (its events then count in srs_amd_probe_read).
void probe_commit(int probe, int slot);

} // namespace srs_amd

// hipLaunchKernelGGL, timed by the armed probe PROBE.
#define SRS_PROBED_LAUNCH(PROBE, KERNEL, GRID, BLOCK, LDS, STREAM, ...)                                                \
  do {                                                                                                                 \
    const ::srs_amd::probe_events pe_ = ::srs_amd::probe_take(PROBE);                                                  \
    if (pe_.slot >= 0) {                                                                                               \
      hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, LDS, STREAM, pe_.start, pe_.stop, 0, __VA_ARGS__);                    \
      ::srs_amd::probe_commit(PROBE, pe_.slot);                                                                        \
    } else {                                                                                                           \
      hipLaunchKernelGGL(KERNEL, GRID, BLOCK, LDS, STREAM, __VA_ARGS__);                                               \
    }                                                                                                                  \
  } while (0)
