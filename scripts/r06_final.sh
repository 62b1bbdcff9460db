#!/bin/bash
# Round-6 final measurement on the GPU box: the changed GPU tests, then the round profile of
# configs 3 and 5 (rocprofv3 kernel-trace stats + one --pmc pass per counter group, PMC record
# stamped with this library's sha256 -> gpurun_out/profiles_new/pmc.json), then the default bench
# line (which reads that record when it is copied to profiles/). Outputs gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06i}
fatal() { [ "$1" -ne 0 ] && { echo "fatal rc=$1 in $2: stopping"; exit "$1"; }; return 0; }
if [ -n "${TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc pytest
fi
CONFIG=3 TAG=$TAG timeout -k 10 900 bash scripts/round_profile.sh > gpurun_out/${TAG}_profile_c3.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_profile_c3.log; fatal $rc profile_c3
CONFIG=5 TAG=$TAG timeout -k 10 700 bash scripts/round_profile.sh > gpurun_out/${TAG}_profile_c5.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_profile_c5.log; fatal $rc profile_c5
echo done
