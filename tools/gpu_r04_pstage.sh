#!/bin/bash
# round-4: PDSCH encode stage alone, event time and kernel statistics.
set -o pipefail
O=gpurun_out/r04ps
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 200 python tools/pdsch_stage_probe.py 2>&1 | grep -v amdgpu.ids || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pps -o p -- python tools/pdsch_stage_probe.py > $O/prof.log 2>&1 &&
  python tools/rocpd_stats.py "$(find /tmp/pps -name "*.db" -print -quit)" "PDSCH encode stage alone" | head -8
