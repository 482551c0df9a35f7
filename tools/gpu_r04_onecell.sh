#!/bin/bash
# round-4: kernel timeline of the one-cell step (configs[4]'s literal shape), eager launches.
set -o pipefail
O=gpurun_out/r04oc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p1 -o p -- python bench.py --slots-pipeline 1 --steps 20 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1 > $O/prof.log 2>&1 &&
  python tools/rocpd_timeline.py "$(find /tmp/p1 -name "*.db" -print -quit)" pdsch_tb_crc 2 0.5 > $O/timeline.txt
