#!/bin/bash
# GPU box: per-section instruction counts of k_lrf8 from the measurement builds
# (se3-icp_amd/lib_cut1..3: make variant V=cutN VFLAGS=-DSE3ICP_LRF8_CUT=N; lib: full).
# One PMC pass per build over tools/lrf_count.py -> gpurun_out/cut_<name>/;
# container side: python3 tools/lrf_sections.py gpurun_out
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for L in lib_cut4 lib_cut5 lib_cut1 lib_cut2 lib_cut3 lib; do
  SE3ICP_LIB=$PWD/se3-icp_amd/$L/libse3icp.so timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv \
    -d gpurun_out/cut_$L -o run -- python3 tools/lrf_count.py > gpurun_out/cut_$L.log 2>&1
  rc=$?
  echo "$L rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/cut_$L.log; exit $rc; }
done
exit 0
