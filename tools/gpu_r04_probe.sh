#!/bin/bash
# round-4: stream_fan helpers probed for concurrency with the caller's stream -- slot tests, then sch_slot in four
# processes and slot_pipeline in two (SRSRAN_AMD_FAN_DEBUG prints each probe's verdict).
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -rf --timeout 240 --timeout-method thread tests/test_sch_slot_gpu.py tests/test_pusch_processor_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc
run() { # name, args...
  local n=$1; shift
  SRSRAN_AMD_FAN_DEBUG=1 timeout -k 10 200 "$@" > $O/$n.log 2>&1 || exit $?
  grep -h "stream_fan" $O/$n.log | sort | uniq -c | tr '\n' ';'
  tail -1 $O/$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
}
for r in 1 2 3 4; do run slot$r python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline; done
for r in 1; do run sp$r python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline; done
