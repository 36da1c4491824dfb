set -u
mkdir -p gpurun_out/batched
timeout -k 10 300 python bench.py --batch 8 --variant shared --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/batched/shared_b8.log 2>&1 && \
timeout -k 10 300 python bench.py --batch 32 --variant shared --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/batched/shared_b32.log 2>&1
