#!/bin/bash
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r4_tiles.sh && bash scripts/gpu_r4_bugs.sh
