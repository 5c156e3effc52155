#!/bin/bash
# A/B of library builds on one box, alternating (tools/ab_pair.sh name1 lib1.so name2 lib2.so ... [x REPS]):
# one line per run: name, iter/s, ms/step, k_lrf ms, setup/loop ms, hand-overs.  AB_ARGS: extra bench args.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
REPS=${AB_REPS:-2}
for rep in $(seq 1 $REPS); do
  args=("$@")
  while [ ${#args[@]} -gt 0 ]; do
    name=${args[0]}; lib=${args[1]}; args=("${args[@]:2}")
    SE3ICP_LIB=$PWD/$lib timeout -k 10 150 python bench.py --steps ${AB_STEPS:-5} --cpu-baseline off --pair-cache /tmp/se3icp_pairs $AB_ARGS > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "$name failed rc=$?"; tail -5 gpurun_out/ab_$name.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$name', d['value'], d['ms_per_step'], 'lrf', k['lrf_ms'], 'nn12', k['nn_se3_ms'], d['phase_ms_per_step'], 'fb', d['lrf_work']['exact_kernel_queries_per_step'])" | tee -a gpurun_out/ab.txt
  done
done
