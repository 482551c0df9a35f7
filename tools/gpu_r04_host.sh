set -o pipefail
PYTHONPATH=. timeout -k 10 200 python tools/slot_host_probe.py > gpurun_out/slot_host_probe2.log 2>&1 &&
timeout -k 10 200 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline > gpurun_out/sp2.log 2>&1 &&
timeout -k 10 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > gpurun_out/slot2.log 2>&1
