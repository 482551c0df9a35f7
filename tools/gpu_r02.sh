#!/bin/bash
# Round-2 decoder check: LDPC decoder / UL-SCH / PUSCH processor / pipeline parity, then a short bench
# with the high-rate kernel and with it disabled (SRSRAN_AMD_LDPC_HR=0).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run t_ldpc 300 python -u -m pytest tests/test_ldpc_decoder_gpu.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread -m gpu
run t_sch 400 python -u -m pytest tests/test_sch_gpu.py tests/test_pusch_processor_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu
run b_hr 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-latency
SRSRAN_AMD_LDPC_HR=0 run b_gen 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-latency
python3 - <<'P'
import json
for n in ("b_hr", "b_gen"):
    d = json.loads([l for l in open("gpurun_out/%s.log" % n) if l.startswith("{")][-1])
    r = d["roofline"]
    print(n, "value %.3fM" % (d["value"] / 1e6), "step %.3f ms" % d["ms_per_step"], "dec %.4f ms" % r["kernel_ms"],
          "its", d["pusch_ldpc_iterations_mean"], "ok", d["pusch_tb_ok_fraction"], d["stage_ms"]["pusch_process"])
P
