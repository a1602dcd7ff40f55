#!/bin/bash
# Round 6 (b): fast-volume error per kernel size on ill-conditioned inputs (kFastVolumeMaxK), the
# full-layout sweep's 16-byte stores (parity subset + same-box A/B against the dword-store build).
set -o pipefail
TAG=${1:-r06b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u scripts/diag_fastk.py > $O/diag_fastk.jsonl 2> $O/diag_fastk.err
rc=$?; echo "diag rc=$rc"; fatal $rc diag
cat $O/diag_fastk.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graph.py -m gpu -q --timeout 120 --timeout-method thread -k "fast_forward or exact_forward or remainder or fp16 or after_a_large or config2 or config0 or graph or workspace" > $O/gpu_tests.log 2>&1
rc=$?; echo "subset rc=$rc"; fatal $rc subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -20
timeout -k 10 900 bash scripts/gpu_ab.sh $TAG c2_full,c3_full fwd 3 "x4:base:" "dword:sweep_dword:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
