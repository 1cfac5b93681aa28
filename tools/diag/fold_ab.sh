# fold geometry variants (timing only): libdpz_abl_fold{a,b,c}.so built with other DPZ_FOLD_TS /
# DPZ_FOLD_THREADS values
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== default"; timeout -k 10 120 python tools/diag/fold_time.py
for s in 1 3; do echo "== variant $s"; DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpz_abl_fold$s.so timeout -k 10 120 python tools/diag/fold_time.py; done
