#!/bin/bash
# batch-1 stage seam: upper bound of a persistent chain's saving (fc1 -> fc2 with and without the launch boundary)
set -u
OUT=gpurun_out/r05n; mkdir -p $OUT
timeout -k 10 200 python -u tools/chain_bound_probe.py --impls 1,3,2 > $OUT/chain_bound.jsonl 2> $OUT/chain_bound.err
rc=$?; echo "rc=$rc"; cat $OUT/chain_bound.jsonl; tail -3 $OUT/chain_bound.err; exit $rc
