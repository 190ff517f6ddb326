#!/bin/bash
# GPU test run: pytest -m gpu (optionally a subset), one process, per-test timeout.
# usage: tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/tests_$tag.log 2>&1
rc=$?
tail -30 gpurun_out/tests_$tag.log
exit $rc
