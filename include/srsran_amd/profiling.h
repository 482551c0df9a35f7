/*
 * srsran_amd/profiling.h -- C-ABI of the live kernel probes: per-launch device time of one kernel family measured
 * inside a caller's own launch sequence (a benchmark's timed steps), on the stream each launch goes to.
 *
 * No reference interface is replaced: this is the measurement side of the boundary (bench.py's roofline reads the
 * average launch time of the dominant kernel from here, next to the rocprofv3 kernel trace of the same command).
 *
 * While a probe is armed, every launch of its kernel family is issued with hipExtLaunchKernelGGL and a pair of HIP
 * events that its own dispatch packet timestamps at kernel start and end (at most max_launches pairs, then further
 * launches go unrecorded): no extra packets enter the stream, so a probed step runs as an unprobed one.  Reading the
 * probe waits for the recorded events, returns the number of launches and their durations, and disarms it.  The
 * figure is the kernel's own duration, whatever runs concurrently on other streams.  Status codes: ldpc.h (SRS_AMD_OK ...).
 */
#ifndef SRSRAN_AMD_PROFILING_H
#define SRSRAN_AMD_PROFILING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  SRS_AMD_PROBE_LDPC_HR        = 0, /* ldpc_decode_hr_kernel (the high-rate BG1 Z = 384 form, incl. fused dematch) */
  SRS_AMD_PROBE_LDPC_FULL      = 1, /* the full-length packed BG1 Z = 384 decoder (configs[1]) */
  SRS_AMD_PROBE_EQUALIZER      = 2, /* pusch_equalize_fused_kernel (batch and slot forms) */
  SRS_AMD_PROBE_OFDM_DEMOD     = 3, /* ofdm_demodulate_kernel */
  SRS_AMD_PROBE_OFDM_MOD       = 4, /* ofdm_modulate_kernel */
  SRS_AMD_PROBE_COUNT          = 5
};

/* Arms probe `probe` for up to max_launches launches (events created on the current device).  Re-arming discards
 * what was recorded. */
int srs_amd_probe_arm(int probe, uint32_t max_launches);

/* Waits for the recorded launches of `probe`, disarms it and returns: launches recorded, the sum / min / max of their
 * event times in ms (any output may be NULL).  A probe never armed or without launches returns 0 launches. */
int srs_amd_probe_read(int probe, uint32_t* launches, double* total_ms, double* min_ms, double* max_ms);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_PROFILING_H */
