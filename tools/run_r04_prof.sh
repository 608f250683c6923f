#!/bin/bash
# Round-4 profiles ($1: tag): rocprofv3 kernel trace + PMC passes of each config's bench (tools/profile.sh).
set -eo pipefail
T=${1:-r04}
for c in ${2:-cavity zz_batch tunable_bus cavity_dense}; do ./tools/profile.sh $c $T; done
echo done
