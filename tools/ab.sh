#!/bin/bash
# A/B timing of experiment builds on the GPU box: tools/ab.sh lib_a lib_b ...
# (names of se3-icp_amd/lib_* directories; "lib" = the default build).  Prints the bench's
# value and per-kernel ms for each.  Each run has its own time limit; stops at the first abnormal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for L in "$@"; do
  SE3ICP_LIB=$PWD/se3-icp_amd/$L/libse3icp.so timeout -k 10 240 python bench.py --steps ${AB_STEPS:-3} --cpu-baseline off > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$L: rc=$rc"; tail -5 gpurun_out/ab_$L.err; exit $rc; fi
  python - "$L" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>14}: {d['value']:9.1f} iter/s  {d['ms_per_step']:7.2f} ms/step  kernels {d['kernel_ms_per_step']}  "
      f"frac {d['roofline']['frac']}  evals/launch {d['roofline']['units_per_launch']}  lrf {d['lrf_work']}")
PY
done
