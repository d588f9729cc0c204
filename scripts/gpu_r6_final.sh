#!/bin/bash
# Round 6 final tree: the GPU tier (smoke, pytest -m gpu, N = 1 bench), then the N = 8 shared rehearsal.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
bash scripts/gpu_r6_tier.sh && bash scripts/gpu_r6_n8.sh
