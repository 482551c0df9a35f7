#!/bin/bash
# round-4: helper-stream layouts of the slot decoder's bucket fan-out and the PDSCH encoder's overlap
# (SRSRAN_AMD_FAN_STREAMS / _MAIN / _PRIORITY, device_buffer.h stream_fan), three processes each (the helpers'
# hardware queues are assigned per process).
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
for cfg in "d:" "hp1m:SRSRAN_AMD_FAN_STREAMS=1 SRSRAN_AMD_FAN_MAIN=1 SRSRAN_AMD_FAN_PRIORITY=1" \
           "n1m:SRSRAN_AMD_FAN_STREAMS=1 SRSRAN_AMD_FAN_MAIN=1" \
           "hp2m:SRSRAN_AMD_FAN_STREAMS=2 SRSRAN_AMD_FAN_MAIN=1 SRSRAN_AMD_FAN_PRIORITY=1" \
           "hp3:SRSRAN_AMD_FAN_STREAMS=3 SRSRAN_AMD_FAN_PRIORITY=1" "s0:SRSRAN_AMD_FAN_STREAMS=0"; do
  n=${cfg%%:*}; e=${cfg#*:}
  for r in 1 2 3; do
    env $e timeout -k 10 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > $O/slot_${n}_$r.log 2>&1 || exit $?
    tail -1 $O/slot_${n}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n slot run $r', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
  done
done
for cfg in "d:" "hp1m:SRSRAN_AMD_FAN_STREAMS=1 SRSRAN_AMD_FAN_MAIN=1 SRSRAN_AMD_FAN_PRIORITY=1" "s0:SRSRAN_AMD_FAN_STREAMS=0"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 200 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline > $O/sp_$n.log 2>&1 || exit $?
  tail -1 $O/sp_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n sp', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1 > $O/pipe_$n.log 2>&1 || exit $?
  tail -1 $O/pipe_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n pipe', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
done
