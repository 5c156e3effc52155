#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for E in ${AB_EXTRAS:-1 0 1 0}; do
  SE3ICP_L12_EXTRA=$E timeout -k 10 240 python bench.py --steps 3 --cpu-baseline off > gpurun_out/env_$E.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/env_$E.json').read().strip().splitlines()[-1]); print('extra $E', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['units_per_launch'])"
done
