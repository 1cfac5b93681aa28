# replace-decode geometry variants (timing only): DPZ_RP_E entries per chunk, DPZ_RP_U loads in flight
set -e
echo "== default (64, 8)"; timeout -k 10 120 python tools/diag/replace_time.py
for s in e128 e256 u4 e128u16; do echo "== $s"; DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpz_abl_rp$s.so timeout -k 10 120 python tools/diag/replace_time.py; done
