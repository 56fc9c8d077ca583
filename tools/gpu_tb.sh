#!/bin/bash
# tests matching $1, then the render_bwd ablation timings
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_t.sh "$1" > /dev/null; rc=$?; grep -E "passed|failed" gpurun_out/t/pytest.log | tail -3; grep -E "^E " gpurun_out/t/pytest.log | head -5
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bwd_abl.sh
