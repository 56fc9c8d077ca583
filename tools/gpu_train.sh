#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/train
mkdir -p $OUT
timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 10 --warmup 3 --stages > $OUT/bench_train.json 2> $OUT/bench_train.err; rc=$?; echo "train rc=$rc"; tail -1 $OUT/bench_train.json; tail -5 $OUT/bench_train.err
exit $rc
