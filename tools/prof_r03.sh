#!/bin/bash
# Round-3 profiles of the default bench step, each pass its own run under its own time limit:
#   prod : the bench's one-stream step as it runs (fused decode: the filter writes the decode's
#          copy of x, the payload scatter rides in the compact launch)
#   clean: DPZ_BATCH_COSCHED=0 (plain encode + standalone replace decode: every kernel's trace
#          and PMC rows are its own, no co-scheduled decode blocks)
# rocprofv3 --kernel-trace --stats, then separate --pmc FETCH_SIZE / WRITE_SIZE passes; per-launch
# traffic JSON by tools/pmc2json.py.  Outputs under gpurun_out/prof_r03_<mode>*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu --no-extra --streams 1"
for mode in ${MODES:-prod clean}; do
  if [ "$mode" = clean ]; then export DPZ_BATCH_COSCHED=0; else unset DPZ_BATCH_COSCHED; fi
  N=prof_r03_$mode
  rm -rf gpurun_out/$N gpurun_out/${N}_fetch gpurun_out/${N}_write
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$N -o run -- $CMD > gpurun_out/$N.log 2>&1 || { echo "$mode trace rc=$?"; tail -5 gpurun_out/$N.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${N}_fetch -o run -- $CMD > gpurun_out/${N}_fetch.log 2>&1 || { echo "$mode fetch rc=$?"; tail -5 gpurun_out/${N}_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${N}_write -o run -- $CMD > gpurun_out/${N}_write.log 2>&1 || { echo "$mode write rc=$?"; tail -5 gpurun_out/${N}_write.log; exit 1; }
  F=$(find gpurun_out/${N}_fetch -name '*counter_collection.csv' | head -1)
  W=$(find gpurun_out/${N}_write -name '*counter_collection.csv' | head -1)
  python3 tools/pmc2json.py "$F" "$W" gpurun_out/pmc_r03_$mode.json "$mode: $CMD (DPZ_BATCH_COSCHED=${DPZ_BATCH_COSCHED:-default})"
  S=$(find gpurun_out/$N -name '*kernel_stats.csv' | head -1)
  cp "$S" gpurun_out/kstats_r03_$mode.csv
  tail -1 gpurun_out/$N.log | cut -c1-300 > gpurun_out/bench_r03_$mode.json
  echo "prof $mode done"
done
