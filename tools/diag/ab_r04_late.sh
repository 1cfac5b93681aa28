cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sliced.py > gpurun_out/pt_pf.log 2>&1 || { echo "sliced tests failed"; tail -20 gpurun_out/pt_pf.log; exit 1; }
tail -1 gpurun_out/pt_pf.log
for v in pf1 product pf8 pf1 product; do
  if [ $v = product ]; then unset DPZ_CODEC_LIB; else export DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so; fi
  timeout -k 10 300 python bench.py --workload c3 --steps 30 > gpurun_out/c3p_$v.json 2>gpurun_out/c3p.err || exit 1
  python tools/diag/c3_summary.py $v gpurun_out/c3p_$v.json >> gpurun_out/c3p.log
done
unset DPZ_CODEC_LIB
for v in d4 d5 d4 d5; do
  echo -n "$v " >> gpurun_out/d5.log
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 120 python tools/diag/dwt_post.py >> gpurun_out/d5.log 2>gpurun_out/d5.err || exit 1
done
for e in 0 8 0 8; do
  DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpzcodec_diag.so DPZ_FOLD_WALK_EPL=$e timeout -k 10 200 python tools/diag/product_ab.py > gpurun_out/epl_$e.tmp 2>gpurun_out/epl.err || exit 1
  python tools/diag/c3_summary.py epl$e gpurun_out/epl_$e.tmp product >> gpurun_out/epl.log
done
cat gpurun_out/c3p.log gpurun_out/d5.log gpurun_out/epl.log
