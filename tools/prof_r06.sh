#!/bin/bash
# Round-6 profiles, each pass its own run under its own time limit:
#   mib64  : the headline bench step (north-star 64 MiB tensor), one stream
#   c2     : the same step at C2's 11M tensor
#   product: the plugin's device round alone (tools/diag/product_run.py, 64 MiB, 1 and 3 payloads)
# rocprofv3 --kernel-trace --stats (-> kstats + rocprof JSON), then separate --pmc FETCH_SIZE /
# WRITE_SIZE passes (-> per-launch traffic JSON).  Outputs under gpurun_out/*_r06_<mode>*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in ${MODES:-mib64 c2 product}; do
  unset PMC_N
  CMD="python3 bench.py --steps ${PROF_STEPS:-100} --warmup 10 --no-cpu --no-extra --streams 1"
  export PMC_N=16777216
  if [ "$mode" = c2 ]; then CMD="$CMD --n 11000000"; export PMC_N=11000000; fi
  if [ "$mode" = product ]; then CMD="python3 tools/diag/product_run.py 16777216 100"; fi
  N=prof_r06_$mode
  rm -rf gpurun_out/$N gpurun_out/${N}_fetch gpurun_out/${N}_write
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$N -o run -- $CMD > gpurun_out/$N.log 2>&1 || { echo "$mode trace rc=$?"; tail -5 gpurun_out/$N.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${N}_fetch -o run -- $CMD > gpurun_out/${N}_fetch.log 2>&1 || { echo "$mode fetch rc=$?"; tail -5 gpurun_out/${N}_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${N}_write -o run -- $CMD > gpurun_out/${N}_write.log 2>&1 || { echo "$mode write rc=$?"; tail -5 gpurun_out/${N}_write.log; exit 1; }
  F=$(find gpurun_out/${N}_fetch -name '*counter_collection.csv' | head -1)
  W=$(find gpurun_out/${N}_write -name '*counter_collection.csv' | head -1)
  python3 tools/pmc2json.py "$F" "$W" gpurun_out/pmc_r06_$mode.json "$mode: $CMD"
  S=$(find gpurun_out/$N -name '*kernel_stats.csv' | head -1)
  cp "$S" gpurun_out/kstats_r06_$mode.csv
  python3 tools/kstats2json.py "$S" gpurun_out/rocprof_r06_$mode.json "$mode: $CMD"
  tail -1 gpurun_out/$N.log | cut -c1-3000 > gpurun_out/bench_r06_$mode.json
  rm -rf gpurun_out/$N gpurun_out/${N}_fetch gpurun_out/${N}_write
  echo "prof $mode done"
done
