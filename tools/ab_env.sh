#!/bin/bash
# A/B of one run-time environment variable on the GPU box:
#   AB_VAR=SE3ICP_NN_TRACE AB_VALS="1 0 1 0" tools/ab_env.sh
# prints per run: value, iter/s, ms/step, the kernel split and the setup / loop phases.
# (The engine reads no tuning variables: build-time A/B goes through tools/ab.sh.)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
: "${AB_VAR:?set AB_VAR to the environment variable to compare}"
mkdir -p gpurun_out
VAR=$AB_VAR
for E in ${AB_VALS:-1 0 1 0}; do
  env "$VAR=$E" timeout -k 10 240 python bench.py --steps ${AB_STEPS:-3} --cpu-baseline off $AB_ARGS > gpurun_out/env_$E.json 2> gpurun_out/env_$E.err || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/env_$E.json').read().strip().splitlines()[-1]); print('$VAR=$E', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['phase_ms_per_step'])"
done
