#!/bin/bash
# round 5: the launch-tail priority A/B (gpu_r05e.sh), the n <= 128 y-in-
# factorisation A/B (gpu_r05f.sh), then the round's measurement (gpu_r05m.sh)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
echo "== tail priority A/B" && bash tools/gpu_r05e.sh || exit 1
echo "== gram y A/B" && bash tools/gpu_r05f.sh || exit 1
bash tools/gpu_r05m.sh
