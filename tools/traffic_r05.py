#!/usr/bin/env python3
"""HBM bytes per launch of the bench's dominant kernel, each counter scaled by its calibration in the kernel's own
access forms (MI355X_MICROARCH.md: only 16-B-per-lane streaming accesses are calibrated).

  traffic_r05.py <out.json> <calib.json> <calib_fetch_dir> <calib_write_dir> <bench_fetch_dir> <bench_write_dir>
                 <nof_codeblocks> <algorithmic_bytes>

calib.json: tools/_build/traffic_calib's stdout (bytes each calibration kernel moves per launch); the four
directories: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes (CSV) over the calibration program and over the
bench command.  The fused LDPC decoder reads its codeword with 8-byte lane loads (calib_read8) and writes one
1,056-byte row of 16-byte lane stores (calib_write16_rows) plus one 4-byte iteration count (calib_write4_rows) per
codeblock:
  read bytes  = FETCH_SIZE / (calib_read8 FETCH / byte)
  write bytes = (WRITE_SIZE - C x calib_write4_rows WRITE per store) / (calib_write16_rows WRITE / byte) + 4 C
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_table import load, mean  # noqa: E402

KERNEL = "ldpc_decode_hr_kernel"


def counter(agg, prefix, name):
    """The kernel named exactly `prefix`, else the first whose name starts with it (template arguments)."""
    keys = [k for k in agg if k == prefix] or [k for k in agg if k.startswith(prefix + "<") or k.startswith(prefix)]
    for k in keys:
        if name in agg[k]:
            return mean(agg[k][name]), len(agg[k][name]), k
    return None, 0, None


def main(out, calib_json, cf, cw, bf, bw, nof_cbs, alg_bytes):
    known = json.load(open(calib_json))
    f, w = load(cf), load(cw)
    cal = {}
    for k, v in known.items():
        if not isinstance(v, dict):
            continue
        if "read" in v:
            raw, n, _ = counter(f, k, "FETCH_SIZE")
            cal[k] = {"bytes": v["read"], "FETCH_SIZE_KiB": raw, "launches": n,
                      "counter_bytes_per_byte": raw * 1024 / v["read"] if raw else None}
        else:
            raw, n, _ = counter(w, k, "WRITE_SIZE")
            cal[k] = {"bytes": v["write"], "WRITE_SIZE_KiB": raw, "launches": n,
                      "counter_bytes_per_byte": raw * 1024 / v["write"] if raw else None}
    nof_cbs, alg_bytes = int(nof_cbs), float(alg_bytes)
    bfs, bws = load(bf), load(bw)
    fr, nf, name = counter(bfs, KERNEL, "FETCH_SIZE")
    wr, nw, _ = counter(bws, KERNEL, "WRITE_SIZE")
    r8 = cal["calib_read8"]["counter_bytes_per_byte"]
    r16 = cal["calib_write16_rows"]["counter_bytes_per_byte"]
    w4 = cal["calib_write4_rows"]["WRITE_SIZE_KiB"] * 1024 / (cal["calib_write4_rows"]["bytes"] / 4)
    read_b = fr * 1024 / r8
    write_b = (wr * 1024 - nof_cbs * w4) / r16 + 4 * nof_cbs
    res = {
        "kernels": {KERNEL: {
            "kernel": name, "launches_fetch_pass": nf, "launches_write_pass": nw,
            "FETCH_SIZE_KiB": fr, "WRITE_SIZE_KiB": wr,
            "read_bytes": read_b, "write_bytes": write_b, "hbm_bytes_per_launch": read_b + write_b,
            "algorithmic_bytes_per_launch": alg_bytes, "traffic_over_algorithmic": (read_b + write_b) / alg_bytes,
            "raw_over_algorithmic": (fr + wr) * 1024 / alg_bytes,
        }},
        "calibration": cal,
        "method": __doc__.strip().splitlines()[0],
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["kernels"][KERNEL], indent=1))
    for k, v in cal.items():
        print("%-20s %.3f counter bytes per byte" % (k, v["counter_bytes_per_byte"] or float("nan")))


if __name__ == "__main__":
    main(*sys.argv[1:])
