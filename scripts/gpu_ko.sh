#!/bin/bash
# k_bwd_coop kernel time (rocprofv3 kernel trace) for the main build and each knockout / ablation
# variant in scripts/_abl: bash scripts/gpu_ko.sh <tag> <cfg> <variant>...
set -o pipefail
TAG=$1; CFG=$2; shift 2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for V in base "$@"; do
  L=$PWD/scripts/_abl/$V/libcustma_hip.so
  [ "$V" = "base" ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  CUSTMA_LIB=$L bash scripts/prof_kernels.sh $TAG/$V $CFG bwd > gpurun_out/$TAG.$V.txt || { echo "$V failed"; exit 1; }
  echo "$V $(grep 'k_bwd_coop' gpurun_out/$TAG.$V.txt | awk '{print $1}') us"
done
