#!/bin/bash
# A/B of library variants in one session: for each "name=path" (path "" = the in-tree library) the headline bench
# line and its rocprofv3 kernel trace.  Every GPU step has its own time limit; a failing step ends the script.
#   tools/gpu_ab.sh <outdir> name=lib.so[,extra bench flags] ...   (flags comma-separated, e.g. w=,--chest-td,interpolate)
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
BENCH=(python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1)
for nv in "$@"; do
  name=${nv%%=*}; rest=${nv#*=}; lib=${rest%%,*}
  extra=(); [[ "$rest" == *,* ]] && IFS=, read -r -a extra <<< "${rest#*,}"
  if [ -n "$lib" ]; then export SRSRAN_AMD_LIB=$lib; else unset SRSRAN_AMD_LIB; fi
  timeout -k 10 300 "${BENCH[@]}" "${extra[@]}" > "$out/$name.json" 2> "$out/$name.err" || { echo "$name bench failed"; exit 3; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace_$name" -o run -- "${BENCH[@]}" "${extra[@]}" \
    > "$out/trace_$name.log" 2>&1 || { echo "$name trace failed"; exit 3; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.json")"
done
