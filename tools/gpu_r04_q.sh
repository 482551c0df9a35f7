#!/bin/bash
# round-4: hardware-queue count -- the pipeline / slot benches under GPU_MAX_HW_QUEUES = 4 (the box's default), 8 and
# 16, and kernel timelines of one pipeline step (which queue each chain's kernels ran on).
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -1 "$O/$name.log" | cut -c1-220
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
export TMPDIR=/tmp
for q in ${QUEUES:-4 8 16}; do
  step bench_q$q 200 env GPU_MAX_HW_QUEUES=$q python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
  step sp_q$q 200 env GPU_MAX_HW_QUEUES=$q python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
  step slot_q$q 200 env GPU_MAX_HW_QUEUES=$q python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
done
export GPU_MAX_HW_QUEUES=${PROF_QUEUES:-16}
step prof_pipe 300 rocprofv3 --kernel-trace -d /tmp/prof_pipe -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1 &&
  python tools/rocpd_timeline.py "$(find /tmp/prof_pipe -name "*.db" -print -quit)" pdsch_tb_crc 2 > $O/timeline_pipe.txt
step prof_sp 300 rocprofv3 --kernel-trace -d /tmp/prof_sp -o sp -- python bench.py --workload slot_pipeline --steps 5 --no-latency --no-cpu-baseline &&
  python tools/rocpd_timeline.py "$(find /tmp/prof_sp -name "*.db" -print -quit)" pdsch_cb_kernel 2 > $O/timeline_sp.txt
exit 0
