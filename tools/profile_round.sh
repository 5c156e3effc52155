#!/bin/bash
# Round profile set on the GPU box (run through gpurun): the bench line, the
# rocprofv3 kernel-trace stats of the same command, and separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; at most 8 SQ counters each).
# Usage: tools/profile_round.sh <tag>   -> gpurun_out/{bench,prof,pmc_*}_<tag>
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --secondary off"
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQ2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"
exec tools/gpu_step.sh \
  "bench_$TAG:300:python3 bench.py > gpurun_out/bench_$TAG.json" \
  "stats_$TAG:240:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- $B" \
  "pmcfetch_$TAG:180:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${TAG}_fetch -o run -- $B" \
  "pmcwrite_$TAG:180:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${TAG}_write -o run -- $B" \
  "pmcsq1_$TAG:180:rocprofv3 --pmc $SQ1 --output-format csv -d gpurun_out/pmc_${TAG}_sq -o run -- $B" \
  "pmcsq2_$TAG:180:rocprofv3 --pmc $SQ2 --output-format csv -d gpurun_out/pmc_${TAG}_sq2 -o run -- $B"
