#!/bin/bash
# All profiles of a round: tools/profile_all.sh <tag>
set -eo pipefail
T=${1:-r02b}
for c in cavity zz_batch tunable_bus; do ./tools/profile.sh $c $T; done
./tools/profile_large.sh $T
