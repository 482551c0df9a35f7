#!/bin/bash
# round-4: kernel-trace summary of the headline decoder launched alone (the bench roofline's kernel_ms form).
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_hr -o hr -- python tools/hr_isolated_probe.py > $O/hrprof.log 2>&1 &&
python tools/rocpd_stats.py "$(find /tmp/prof_hr -name "*.db" -print -quit)" "r04 headline decoder alone (rocprofv3 --kernel-trace --stats -- python tools/hr_isolated_probe.py)" > $O/hr_alone_kernel_stats.md &&
python - "$(find /tmp/prof_hr -name "*.db" -print -quit)" > $O/hr_alone_durations.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = [r[0] / 1e3 for r in c.execute("select end - start from kernels where name like '%ldpc_decode_hr_kernel<0, 4, 1>%' order by start")]
print("hr kernel launches (us):", ["%.1f" % r for r in rows])
alone = rows[-6:]
print("probe launches (last 6, decoder alone on its stream): avg %.1f us" % (sum(alone) / len(alone)))
PY
