#!/bin/bash
# FFT: the changed kernels' tests, then the transforms' timing per occupancy variant
# (tools/diag/variants/lib_ip{4,5,6}.so: the in-place pass bounded to 4 / 5 / 6 waves per SIMD),
# each against hipFFT and the ping-pong pass on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fft.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fftip_tests.log 2>&1 || { echo "fft tests failed"; tail -30 gpurun_out/fftip_tests.log; exit 1; }
tail -1 gpurun_out/fftip_tests.log
: > gpurun_out/fft_ip_ab.jsonl
for v in ip4 ip5 ip6; do
  FFT_CONFIGS=short DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 200 python tools/diag/fft_time.py 11000000 25000000 > gpurun_out/fft_tmp.jsonl 2> gpurun_out/fft_tmp.err || { echo "$v rc=$?"; tail -3 gpurun_out/fft_tmp.err; exit 1; }
  sed "s/^{/{\"variant\": \"$v\", /" gpurun_out/fft_tmp.jsonl >> gpurun_out/fft_ip_ab.jsonl
done
cat gpurun_out/fft_ip_ab.jsonl
