#!/bin/bash
# round-4: kernel timeline of the headline pipeline step (tools/rocpd_timeline.py) and the stage split.
set -o pipefail
O=gpurun_out/r04tp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_pipe -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1 > $O/prof_pipe.log 2>&1 &&
  python tools/rocpd_timeline.py "$(find /tmp/prof_pipe -name "*.db" -print -quit)" pdsch_tb_crc 3 > $O/timeline_pipe.txt
