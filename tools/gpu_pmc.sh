#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only, no sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CMD="python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu --no-extra ${BENCH_ARGS}"
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  rm -rf gpurun_out/pmc/p$i
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d gpurun_out/pmc/p$i -o run -- $CMD > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
FETCH_SIZE
WRITE_SIZE}
GROUPS
find gpurun_out/pmc -name '*counter_collection*' | head
