cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do for v in base late w5; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 200 python tools/diag/dwt_post.py > gpurun_out/dwtl_${v}_$r.json 2> gpurun_out/dwtl.err || { echo "$v rc=$?"; tail -3 gpurun_out/dwtl.err; exit 1; }
  echo "$v $r $(cat gpurun_out/dwtl_${v}_$r.json)"
done; done
timeout -k 10 200 python tools/diag/sliced_planes_ab.py > gpurun_out/planes_ab.jsonl 2> gpurun_out/planes_ab.err || { echo "planes rc=$?"; tail -3 gpurun_out/planes_ab.err; exit 1; }
cat gpurun_out/planes_ab.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_plugins.py > gpurun_out/plugin_tests.log 2>&1 || { echo "plugin tests failed"; tail -30 gpurun_out/plugin_tests.log; exit 1; }
tail -1 gpurun_out/plugin_tests.log
for o in 1 0 1 0; do LOAD_FLAT_OLD=$o timeout -k 10 300 python tools/diag/plugin_breakdown.py jwins 6 > gpurun_out/pb_old$o.json 2> gpurun_out/pb.err || { echo "pb rc=$?"; tail -3 gpurun_out/pb.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/pb_old$o.json')); p=d['parts_ms_per_round']; print('old=$o', d['round']['round_ms'], d['round']['receive_ms'], p.get('recv.load_flat'), p.get('recv.total'))"; done
