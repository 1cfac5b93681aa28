#!/bin/bash
# DPZ_WALK_GUESS was removed after the A/B (profiles/r05_fold_start_ab.txt): build lib_guess from
# commit ff7398b (tools/diag/build_variant.sh guess "-DDPZ_WALK_GUESS=1" ff7398b) to re-run it.
# DPZ_WALK_GUESS (the walk folds' cursor searches starting at the uniform-density guess): base /
# guess build_variant.sh libraries, alternating on one box — tools/diag/fold_kinds.py (walk kind)
# at the C3, 64 MiB and C2/C4 shapes, then the C4 round (tools/diag/c4_round_ab.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export FOLD_KINDS=${FOLD_KINDS:-"0"}  # the auto choice (product variants read no knobs)
export FOLD_CASES=${FOLD_CASES:-"25000009:0.1:16:0 25000009:0.01:16:0 16777216:0.01:3:0 16777216:0.01:1:0 11000000:0.01:4:0"}
for r in 1 2; do for v in base guess; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 300 python tools/diag/fold_kinds.py > gpurun_out/guess_fk_${v}_$r.jsonl 2> gpurun_out/guess.err || { echo "$v rc=$?"; tail -3 gpurun_out/guess.err; exit 1; }
  echo "== $v run $r"
  python -c "
import json
for l in open('gpurun_out/guess_fk_${v}_$r.jsonl'):
    d=json.loads(l); print(d['m'], d['alpha'], d['npay'], {k: (v['call_us'], v['kernels_us_event_pair']) for k, v in d['kinds'].items()})"
done; done
for r in 1 2; do for v in base guess; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so ROUNDS=12 timeout -k 10 300 python tools/diag/c4_round_ab.py > gpurun_out/guess_c4_${v}_$r.json 2> gpurun_out/guess.err || { echo "c4 $v rc=$?"; tail -3 gpurun_out/guess.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/guess_c4_${v}_$r.json')); print('c4 $v $r', d['ms_per_round'], d['legs_ms'])"
done; done
