/*
 * srsran_amd/grid.h -- C-ABI of the resource-grid merge the device-resident resource grid of the reference-side
 * plug-ins uses (integration/hip_resource_grid.cpp, a srsran::resource_grid, include/srsran/phy/support/
 * resource_grid.h:35-49, whose slot grid lives in HBM next to a host mirror).
 *
 * No reference interface is replaced one to one: the reference's resource_grid_impl has a single host copy that every
 * channel processor writes.  With a device copy beside it, host writers (reference processors through
 * resource_grid_writer) and device writers (the plug-ins' kernels) may both change the slot before it is read; the
 * grid then merges the host's changes into the device copy RE by RE: the host sends, per changed row, the XOR of its
 * row with the state both copies last agreed on, and the device applies it only where it is non-zero, so REs written
 * meanwhile on the device are kept.  Status codes: ldpc.h (SRS_AMD_OK ...).
 */
#ifndef SRSRAN_AMD_GRID_H
#define SRSRAN_AMD_GRID_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* DEVICE, asynchronous on `stream`: for i < nof_rows and k < row_len, d_grid[d_rows[i] * row_len + k] ^=
 * d_delta[i * row_len + k] wherever that delta word is non-zero (a cbf16 RE the host changed).  d_rows: device array
 * of row indices ((port * nof_symbols + symbol) for a [port][symbol][subcarrier] grid). */
int srs_amd_grid_merge_rows(uint32_t* d_grid, const uint32_t* d_delta, const uint32_t* d_rows, uint32_t nof_rows,
                            uint32_t row_len, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SRSRAN_AMD_GRID_H */
