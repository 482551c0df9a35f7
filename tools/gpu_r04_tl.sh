#!/bin/bash
# round-4: kernel timelines (tools/rocpd_timeline.py) of slot_pipeline and sch_slot steps.
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_sp -o sp -- python bench.py --workload slot_pipeline --steps 5 --no-latency --no-cpu-baseline > $O/prof_sp.log 2>&1 &&
  python tools/rocpd_timeline.py "$(find /tmp/prof_sp -name "*.db" -print -quit)" pdsch_tb_crc 2 > $O/timeline_sp.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_slot -o sl -- python bench.py --workload sch_slot --steps 5 --no-latency --no-cpu-baseline > $O/prof_slot.log 2>&1 &&
  python tools/rocpd_timeline.py "$(find /tmp/prof_slot -name "*.db" -print -quit)" pdsch_tb_crc 2 > $O/timeline_slot.txt
