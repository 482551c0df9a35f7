#!/bin/bash
# round-4: run-to-run spread of the sch_slot bench (separate processes), and under 8 hardware queues.
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
for r in 1 2 3 4; do
  timeout -k 10 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > $O/slot$r.log 2>&1 || exit $?
  tail -1 $O/slot$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('slot run $r', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
done
for r in 1 2; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > $O/slotq8_$r.log 2>&1 || exit $?
  tail -1 $O/slotq8_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('slot q8 run $r', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
done
