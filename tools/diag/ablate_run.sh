set -e
for L in libdpzcodec libdpz_abl_win libdpz_abl_app libdpz_abl_all; do
  echo "== $L"; DPZ_CODEC_LIB=$PWD/decentralizepy_amd/$L.so timeout -k 10 120 python tools/diag/filter_time.py 11000000
done
echo "== stamps"; timeout -k 10 120 python tools/stamps.py 11000000
