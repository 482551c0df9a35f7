#!/bin/bash
# One gpurun session of the PUCCH work: the PUCCH tests, the PUCCH bench line with its CPU baseline, and the
# rocprofv3 kernel trace of the same workload.  Every GPU step has its own time limit; a step that faults, aborts or
# times out ends the script.
#   tools/gpu_r05_pucch.sh <outdir>
out=${1:-gpurun_out/r05pu}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_pucch_gpu.py \
  tests/test_bench_workloads_gpu.py -k "pucch" > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$out/steps.log"; [ $rc -le 1 ] || exit $rc
BENCH=(python3 bench.py --workload pucch --steps 20 --warmup 3)
timeout -k 10 300 "${BENCH[@]}" > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc" >> "$out/steps.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 bench.py --workload pucch --steps 20 --warmup 3 --no-cpu-baseline > "$out/trace.log" 2>&1
rc=$?; echo "trace rc=$rc" >> "$out/steps.log"
echo done >> "$out/steps.log"
