# walk-fold tile-size sweep (DPZ_FOLD_WALK_EPL) over FOLD_CASES; appends to gpurun_out/diag_epl.jsonl
set -e
export FOLD_KINDS="4"
export FOLD_CASES="${FOLD_CASES:-25000009:0.2:16:0 25000009:0.3:16:0 25000009:0.2:3:0 25000009:0.3:3:0 25000009:0.4:3:0 25000009:0.01:3:0 11000000:0.01:1:0 11000000:0.01:4:0}"
for e in ${EPLS:-16 4}; do
  DPZ_FOLD_WALK_EPL=$e timeout -k 10 200 python -u tools/diag/fold_kinds.py >> gpurun_out/diag_epl.jsonl
done
echo done
