#!/bin/bash
# round-4: the new default fan (one helper + the caller's stream) on the three workloads, two processes each, and the
# pipeline without the PDSCH encoder's TB-CRC overlap (SRSRAN_AMD_FAN_STREAMS=0).
set -o pipefail
O=gpurun_out/r04f2
mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || exit $?
  tail -1 $O/$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
}
for r in 1 2; do
  run pipe$r python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
  run pipe_s0_$r env SRSRAN_AMD_FAN_STREAMS=0 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
  run sp$r python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
  run slot$r python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
done
