#!/bin/bash
# Copy a tools/gpu_profiles.sh run (gpurun_out/$1) into profiles/ as $2_<cfg>_{kernel_stats.csv,traffic.json,valu.json}
# (e.g. tools/keep_profiles.sh r04p r04).
set -e
SRC=gpurun_out/$1
TAG=$2
for f in $SRC/*_kernel_stats.csv $SRC/*_traffic.json $SRC/*_valu.json $SRC/c5_overlap.json; do
  [ -f "$f" ] && cp "$f" profiles/${TAG}_$(basename $f)
done
ls profiles/${TAG}_*
