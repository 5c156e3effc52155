#!/bin/bash
# A/B of library builds on one box over several workloads:
#   tools/ab_multi.sh "C4 C3 C2" name1 lib1.so name2 lib2.so ...
# (tools/ab_bench.sh per workload, its lines tagged with the workload)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
WLS=$1; shift
for W in $WLS; do
  AB_ARGS="--workload $W $AB_EXTRA" timeout -k 10 600 tools/ab_bench.sh "$@" > gpurun_out/ab_$W.txt 2>&1
  rc=$?
  sed "s/^/$W /" gpurun_out/ab_$W.txt
  for f in gpurun_out/ab_*.json; do case $f in gpurun_out/ab_C[0-9]_*) ;; *) cp "$f" "gpurun_out/ab_${W}_${f#gpurun_out/ab_}";; esac; done
  [ $rc -ne 0 ] && exit $rc
done
exit 0
