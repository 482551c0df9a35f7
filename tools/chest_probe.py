"""Phase timing of the PUSCH DM-RS estimator kernels in the headline step (64 cells, 4 layers x 4 ports, 273 PRB).

Needs the probe build of the library (s_memtime stamps per workgroup phase, pusch_chest.hip CHEST_STAMP):
    tools/build_variant.sh chestprobe pusch_chest.hip -DSRS_AMD_CHEST_PROBE
    SRSRAN_AMD_LIB=$PWD/tools/_build/libsrsran_amd_chestprobe.so PYTHONPATH=. python tools/chest_probe.py
Prints, per kernel and phase, the median / p90 / max duration over the workgroups (shader-clock cycles and us at the
clock the stamps imply), and the spread of workgroup start / end times (100 MHz real-time clock) across the launch:
run alone on the PUSCH stream, then inside the full step (PDSCH chain concurrent)."""
import ctypes
import json
import sys

import numpy as np
import torch

import bench_pipeline as bp
from srsran_project_amd import _lib

NWG = 4096
PILOT_PHASES = ["gold+seq", "cfo", "lse", "fir", "store", "interp", "idft", "rsrp"]
STATS_PHASES = ["corr+seq", "noise", "tail"]


def read(lib, clear=True):
    buf = np.zeros(2 * NWG * 16, dtype=np.uint64)
    rc = lib.srs_amd_chest_probe_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(buf.nbytes), int(clear))
    assert rc == 0, rc
    return buf.reshape(2, NWG, 16)


def summarize(st, k, nwg, names):
    s = st[k, :nwg].astype(np.int64)
    assert (s[:, 0] > 0).all(), "missing stamps"
    t0, t1 = s[:, 0], s[:, 15]
    span_rt = (t1.max() - t0.min()) / 100.0  # us (100 MHz)
    wg_rt = (t1 - t0) / 100.0
    n = len(names)
    cyc_total = (s[:, n + 1] - s[:, 1]).astype(np.float64)
    mhz = np.median(cyc_total / np.maximum(wg_rt, 1e-3))  # stamp clock in MHz
    out = {"workgroups": int(nwg), "launch_span_us": round(float(span_rt), 2),
           "wg_us_median": round(float(np.median(wg_rt)), 2), "wg_us_max": round(float(wg_rt.max()), 2),
           "start_spread_us": round(float((t0.max() - t0.min()) / 100.0), 2),
           "stamp_clock_mhz": round(float(mhz), 1), "phases": {}}
    for i, nm in enumerate(names):
        d = (s[:, i + 2] - s[:, i + 1]).astype(np.float64) / mhz
        out["phases"][nm] = {"median_us": round(float(np.median(d)), 2), "p90_us": round(float(np.percentile(d, 90)), 2),
                             "max_us": round(float(d.max()), 2)}
    sub = {"pilot": [("fir.write", 4, 10), ("fir.vpilots", 10, 11), ("fir.taps", 11, 12), ("fir.stage", 12, 5)],
           "stats": [("noise.rot", 2, 10), ("noise.loop", 10, 3)]}["pilot" if k == 0 else "stats"]
    for nm, i0, i1 in sub:
        if (s[:, i1] > 0).all() and (s[:, i0] > 0).all():
            d = (s[:, i1] - s[:, i0]).astype(np.float64) / mhz
            out["phases"][nm] = {"median_us": round(float(np.median(d)), 2),
                                 "p90_us": round(float(np.percentile(d, 90)), 2), "max_us": round(float(d.max()), 2)}
    return out


def main():
    lib = _lib.lib()
    lib.srs_amd_chest_probe_read.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    pl = bp.Pipeline(64, dev)
    s = torch.cuda.Stream(dev)
    for _ in range(3):
        pl.step(s)
    torch.cuda.synchronize(dev)
    nwg_pilot = 64 * bp.UL_PORTS * pl.ul_layers  # average TD strategy: one LSE slice per layer
    nwg_stats = 64 * bp.UL_PORTS
    res = {}
    for mode in ("alone", "in_step"):
        acc = []
        for rep in range(5):
            read(lib, True)
            torch.cuda.synchronize(dev)
            if mode == "alone":
                with torch.cuda.stream(s):
                    pl.pusch(s)
            else:
                pl.step(s)
            torch.cuda.synchronize(dev)
            st = read(lib, True)
            acc.append({"pilot": summarize(st, 0, nwg_pilot, PILOT_PHASES),
                        "stats": summarize(st, 1, nwg_stats, STATS_PHASES)})
        res[mode] = acc[-1]
        res[mode]["pilot_span_us_reps"] = [a["pilot"]["launch_span_us"] for a in acc]
        res[mode]["stats_span_us_reps"] = [a["stats"]["launch_span_us"] for a in acc]
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
