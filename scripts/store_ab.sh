#!/bin/bash
# A/B of the store worker's optional features on the reference pipeline p50
# (AHV_STORE_SPECULATE: provisional Merkle roots; AHV_STORE_PREFIX: capture prefix midstates).
OUT=${OUT:-gpurun_out/r2p}
mkdir -p $OUT
for cfg in "0 0" "1 1" "0 0" "1 1" "1 0" "0 1" "1 0" "0 1"; do
  set -- $cfg
  r=$(AHV_STORE_SPECULATE=$1 AHV_STORE_PREFIX=$2 timeout -k 10 100 python scripts/store_probe.py cuda 3000 2>&1 | grep -o '"p50_us": [0-9.]*') || exit 1
  echo "spec=$1 prefix=$2 $r" >> $OUT/ab2.log
done
