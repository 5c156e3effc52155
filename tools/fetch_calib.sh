#!/bin/bash
# FETCH_SIZE calibration passes over tools/bin/fetch_calib (built by __graft_entry__.build()
# or tools/build_calib.sh); run on the GPU box through gpurun.  Each rocprofv3 pass is its own
# process under a hard time limit, with at most 4 TCC counters (the _sum forms count once).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
X=tools/bin/fetch_calib
P="--output-format csv -o run --"
timeout -k 5 60 $X > gpurun_out/calib_plain.jsonl && \
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/calib_trace $P $X > /dev/null && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_fetch $P $X > /dev/null && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib_write $P $X > /dev/null && \
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
  -d gpurun_out/calib_tcc_a $P $X > /dev/null && \
timeout -s KILL 90 rocprofv3 --pmc TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_sum \
  -d gpurun_out/calib_tcc_b $P $X > /dev/null && \
echo calib done
