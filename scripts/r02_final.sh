#!/bin/bash
# round-end check on one box: full GPU tests + smoke, default bench (config 2, 10k frames), then
# kernel traces (3 lanes, 1 lane) and PMC passes of c2 with on-box summaries
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02y}
bash scripts/r02r_check.sh $TAG || exit $?
bash scripts/profile_r02_run.sh $TAG c2
