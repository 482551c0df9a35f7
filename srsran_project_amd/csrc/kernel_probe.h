// kernel_probe.h -- the launch side of the live kernel probes (include/srsran_amd/profiling.h): a launch site
// brackets its kernel with probe_begin / probe_end on the launch stream; both are one relaxed atomic load when the
// probe is not armed.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

// Slot of this launch in the armed probe (-1: not armed or full): records the start event on `stream`.
int  probe_begin(int probe, hipStream_t stream);
// Records the end event of slot `slot` (from probe_begin; -1 ignored).
void probe_end(int probe, int slot, hipStream_t stream);

// RAII form for a launch site with several return paths.
struct probe_scope {
  int         probe, slot;
  hipStream_t stream;
  probe_scope(int p, hipStream_t s) : probe(p), slot(probe_begin(p, s)), stream(s) {}
  ~probe_scope() { probe_end(probe, slot, stream); }
  probe_scope(const probe_scope&)            = delete;
  probe_scope& operator=(const probe_scope&) = delete;
};

} // namespace srs_amd
