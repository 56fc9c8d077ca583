#!/bin/bash
# gpu_t.sh (tests $1 + training bench) followed by the training counter passes.
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_t.sh "$1" && bash tools/prof_train.sh
