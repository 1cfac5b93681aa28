#!/bin/bash
# Round-6 session 2 on one box: the changed paths' tests, the FFT tile timing, a same-box C4 A/B
# (ring-of-rounds counters vs the sliced planes), then the full GPU suite, the bench line and the
# workloads.  Every GPU step has its own time limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_fft.py tests/test_gpu_gossip.py tests/test_gpu_counter.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_quick.log 2>&1 || { echo "quick tests failed"; tail -30 gpurun_out/s2_quick.log; exit 1; }
tail -2 gpurun_out/s2_quick.log
DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpzcodec_diag.so timeout -k 10 300 python tools/diag/fft_time.py > gpurun_out/fft_time.jsonl 2> gpurun_out/fft_time.err || { echo "fft_time rc=$?"; tail -5 gpurun_out/fft_time.err; exit 1; }
cat gpurun_out/fft_time.jsonl
: > gpurun_out/c4_ring_ab.jsonl
for r in 1 2; do for v in 1 0; do
  ENGINE_RING=$v timeout -k 10 240 python tools/diag/c4_round_ab.py > gpurun_out/c4_tmp.json 2> gpurun_out/c4.err || { echo "c4 ring=$v rc=$?"; tail -3 gpurun_out/c4.err; exit 1; }
  echo "{\"ring\": $v, \"rep\": $r, \"c4\": $(tail -1 gpurun_out/c4_tmp.json)}" >> gpurun_out/c4_ring_ab.jsonl
done; done
python3 -c "
import json
for l in open('gpurun_out/c4_ring_ab.jsonl'):
    d=json.loads(l); print(d['ring'], d['rep'], d['c4']['ms_per_round'], d['c4']['legs_ms'])"
if [ "${FULL:-1}" = 1 ]; then
  STEPS="tests bench workloads" WORKLOADS="${WORKLOADS:-c4 c3 fft plugin e2e}" TAG=s2 bash tools/gpu_r06.sh || exit 1
fi
echo s2 done
