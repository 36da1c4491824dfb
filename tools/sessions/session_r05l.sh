set -u
OUT=gpurun_out/r05l; mkdir -p $OUT
timeout -k 10 300 python -u tools/hipblaslt_kernels.py > $OUT/blaslt.jsonl 2> $OUT/blaslt.err
