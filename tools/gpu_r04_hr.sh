#!/bin/bash
# round-4: high-rate PUSCH decoder variants (default build, 8-bit packed messages, 3 waves per SIMD) -- HR parity
# tests per variant, the isolated launch timing, and FETCH_SIZE / WRITE_SIZE passes (one counter group per run).
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -2 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
export PYTHONPATH=.
export TMPDIR=/tmp
# the .db files of a whole pipeline step are large: keep only the decoder's per-dispatch rows
pmc() { # variant, counter
  step pmc_$2_$1 120 rocprofv3 --pmc $2 -d /tmp/pmc_$2_$1 -o p -- python tools/hr_isolated_probe.py &&
    python tools/pmc_db.py /tmp/pmc_$2_$1 hr_kernel $2 > $O/pmc_$2_$1.txt; rm -rf /tmp/pmc_$2_$1
}
for v in ${VARIANTS:-libsrsran_amd var_pack8 var_w3}; do
  export SRSRAN_AMD_LIB=$PWD/srsran_project_amd/lib/$v.so
  if [ -z "$NO_TESTS" ]; then
    step test_$v 300 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_ldpc_decoder_gpu.py -k "high_rate or parity_all"
  fi
  step probe_$v 120 python tools/hr_isolated_probe.py
  pmc $v WRITE_SIZE
  pmc $v FETCH_SIZE
done
unset SRSRAN_AMD_LIB
if [ -n "$CALIB" ]; then
  for c in WRITE_SIZE FETCH_SIZE; do
    step calib_$c 120 rocprofv3 --pmc $c -d /tmp/calib_$c -o p -- python tools/write_size_calib.py &&
      python tools/pmc_db.py /tmp/calib_$c "" $c > $O/calib_$c.txt; rm -rf /tmp/calib_$c
  done
fi
exit 0
