#!/bin/bash
# seed-group count sweep (QOC_BLKP_PARTS) on the tunable bus, same box, then a kernel trace with one group (no overlap)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for p in 2 4 8 16; do
    QOC_BLKP_PARTS=$p timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05ab3_p${p}_$rep.json 2> gpurun_out/r05ab3_p${p}_$rep.err || exit $?
    python -c "import json; a=json.load(open('gpurun_out/r05ab3_p${p}_$rep.json')); print('parts $p', round(a['value'],1), a['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
QOC_BLKP_PARTS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05ab3_prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config tunable_bus --no-cpu --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r05ab3_prof1.log 2>&1
