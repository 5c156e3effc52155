#!/bin/bash
# GPU box: one C4 step with per-iteration NN work lines (SE3ICP_NN_TRACE=1, the library waits
# for every iteration): gpurun_out/nn_trace_<W>.err
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
W=${1:-C4}
SE3ICP_NN_TRACE=1 timeout -k 10 240 python bench.py --workload $W --steps 1 --warmup 0 --cpu-baseline off --secondary off \
  --pair-cache /tmp/se3icp_pairs > gpurun_out/nn_trace_$W.json 2> gpurun_out/nn_trace_$W.err
