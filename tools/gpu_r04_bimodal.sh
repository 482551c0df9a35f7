#!/bin/bash
# round-4: sch_slot's two modes (0.84 / 1.15 ms per step across processes) -- three traced processes, each with its
# bench value, kernel statistics and the timeline of one step.
set -o pipefail
O=gpurun_out/r04b2
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pb$r -o p -- python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > $O/run$r.log 2>&1 || exit $?
  db="$(find /tmp/pb$r -name "*.db" -print -quit)"
  tail -1 $O/run$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('run $r', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
  python tools/rocpd_stats.py "$db" "run $r" > $O/stats$r.md
  python tools/rocpd_timeline.py "$db" pdsch_tb_crc -1 > $O/timeline$r.txt
  rm -rf /tmp/pb$r
done
