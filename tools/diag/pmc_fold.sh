cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/pmcf
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1)); rm -rf gpurun_out/pmcf/p$i
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcf/p$i -o run -- python3 tools/diag/fold_one.py 0.01 16 > gpurun_out/pmcf/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmcf/p$i.log; exit 1; }
done
echo ok
