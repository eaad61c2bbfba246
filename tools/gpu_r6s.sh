#!/bin/bash
# round 6 pass s (final build): smoke, the GPU suite, the default bench under a kernel trace and
# plain, then the local-optimum kernel's PMC at 16 / 128 chains (slot form, paired rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_PMC_LO=${SKIP_PMC_LO:-}
PROF_DIR=gpurun_out/r6s bash tools/gpu_round.sh || exit 1
[ -n "$SKIP_PMC_LO" ] || { sed -e 's#gpurun_out/r6l#gpurun_out/r6s/lo#' tools/gpu_r6l.sh > /tmp/lo_pmc.sh && bash /tmp/lo_pmc.sh; }
