#!/bin/bash
# r05 roofline evidence session (one gpurun call): the live-probe bench line, the rocprofv3 kernel trace of the same
# command, FETCH_SIZE / WRITE_SIZE / SQ passes over it, and the traffic calibration program under both counters.
# Every GPU step has its own time limit; a step that faults, aborts or times out ends the script.
#   tools/gpu_r05_evidence.sh <outdir> [pytest selection...]
out=${1:-gpurun_out/r05e}
shift
mkdir -p "$out"
export TMPDIR=/tmp
ok() { # continue after success or ordinary test failures only
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "step ended with $rc: stopping" | tee -a "$out/steps.log"
    exit "$rc"
  fi
}
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > "$out/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc" >> "$out/steps.log"; ok $rc
fi
BENCH=(python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1)
timeout -k 10 300 "${BENCH[@]}" > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc" >> "$out/steps.log"; ok $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- "${BENCH[@]}" \
  > "$out/trace.log" 2>&1
rc=$?; echo "trace rc=$rc" >> "$out/steps.log"; ok $rc
pass() {
  local name=$1
  shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- "${CMD[@]}" \
    > "$out/$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc" >> "$out/steps.log"
  ok $rc
}
CMD=("${BENCH[@]}")
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass a SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES
pass b SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE
CMD=(tools/_build/traffic_calib)
timeout -k 10 60 tools/_build/traffic_calib > "$out/calib.json" 2> "$out/calib.err"
rc=$?; echo "calib rc=$rc" >> "$out/steps.log"; ok $rc
pass calib_fetch FETCH_SIZE
pass calib_write WRITE_SIZE
echo done >> "$out/steps.log"
