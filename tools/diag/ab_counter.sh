export DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpzcodec_diag.so
timeout -k 10 200 python tools/diag/product_ab.py > gpurun_out/ab1_base.jsonl 2>gpurun_out/ab1.err &&
DPZ_COMPACT_ABLATE=2 timeout -k 10 200 python tools/diag/product_ab.py > gpurun_out/ab1_nocounter.jsonl 2>>gpurun_out/ab1.err
