set -e
mkdir -p gpurun_out/ab1
for rep in 1 2; do
for v in prev cur; do
  if [ $v = prev ]; then export MMT_HIP_LIB=$PWD/multi-modal-tracking_amd/mmt_amd/_lib/prev/libmmt_hip.so; else unset MMT_HIP_LIB; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-kernel-profile --no-mam-batched --no-kv-cache --no-train-line --steps 400 --warmup 50 > gpurun_out/ab1/$v$rep.log 2>&1
  echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab1/$v$rep.log | head -1)"
done; done
