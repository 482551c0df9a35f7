#!/bin/bash
# round-4 GPU check of the packed runtime-Z LDPC decoder: parity tests, then sch_slot / slot_pipeline with the
# packed kernel on and off, then a kernel trace of sch_slot.  Stops at the first failing GPU step.
set -o pipefail
mkdir -p gpurun_out/r04pk
O=gpurun_out/r04pk
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
step dec 600 $PYT tests/test_ldpc_decoder_gpu.py tests/test_golden.py
step slot 400 $PYT tests/test_sch_slot_gpu.py
step bench_slot_pk 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
step bench_slot_nopk 200 env SRSRAN_AMD_LDPC_PK=0 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
step bench_sp_pk 300 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
step bench_sp_nopk 300 env SRSRAN_AMD_LDPC_PK=0 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step prof_slot 300 rocprofv3 --kernel-trace --stats -d $O/prof_slot -o slot -- python bench.py --workload sch_slot --steps 10 --no-latency --no-cpu-baseline
exit 0
