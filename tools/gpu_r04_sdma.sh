#!/bin/bash
# round-4: is sch_slot's occasional ~7 ms host-to-device stall the SDMA engine?  Three processes with the copies on
# blit kernels (HSA_ENABLE_SDMA=0), each with its per-step intervals.
set -o pipefail
O=gpurun_out/r04sd
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  HSA_ENABLE_SDMA=0 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ps$r -o p -- python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > $O/run$r.log 2>&1 || exit $?
  tail -1 $O/run$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('run $r', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
  python tools/rocpd_timeline.py "$(find /tmp/ps$r -name "*.db" -print -quit)" pdsch_tb_crc -1 | head -3
  rm -rf /tmp/ps$r
done
