#!/bin/bash
# A/B of library builds on one box: tools/ab_bench.sh name1 lib1.so name2 lib2.so ... (alternating twice)
# prints per run: name, iter/s, ms/step, k_lrf ms, setup ms
set -e -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  args=("$@")
  while [ ${#args[@]} -gt 0 ]; do
    name=${args[0]}; lib=${args[1]}; args=("${args[@]:2}")
    SE3ICP_LIB=$lib timeout -k 10 120 python bench.py --cpu-baseline off --pair-cache /tmp/se3icp_pairs $AB_ARGS > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
    python -c "import json; d=json.load(open('gpurun_out/ab_$name.json')); k=d['kernel_ms_per_step']; print('$name', d['value'], d['ms_per_step'], k['lrf_ms'], d['phase_ms_per_step'], d['lrf_work']['exact_kernel_queries_per_step'])" | tee -a gpurun_out/ab.txt
  done
done
