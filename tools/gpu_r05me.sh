#!/bin/bash
# round 5: the launch-tail priority A/B (tools/gpu_r05e.sh), then the round's
# measurement (tools/gpu_r05m.sh), in one box session
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
echo "== tail priority A/B" && bash tools/gpu_r05e.sh || exit 1
bash tools/gpu_r05m.sh
