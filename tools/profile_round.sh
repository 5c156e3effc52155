#!/bin/bash
# One workload's profile set on the GPU box (run through gpurun): the bench line, the
# rocprofv3 kernel-trace stats of the profiled command, and separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; at most 8 SQ counters each).
# Usage: tools/profile_round.sh <tag> <workload: C2|C2u|C3|C4|C5> [lite]
#   -> gpurun_out/{bench,prof,pmc_*}_<tag>_<workload>, and gpurun_out/cmd_<tag>_<workload>.txt
#   ("lite": bench line + kernel trace only).  Then, in the container:
#   tools/summarize_round.sh <tag> <workload>   -> profiles/<tag>_<workload>_{kernel_stats.md,pmc.json}
TAG=${1:-r04}
W=${2:-C4}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
WA="--workload $W"
[ "$W" = "C2u" ] && WA="--workload C2 --c2-cloud unique"
# (one call at a time: the line's kernel figures come from isolated calls, so the traced
# kernel averages must too; BENCH_CMD below is the default, calls in flight)
B="python3 bench.py $WA --steps 3 --warmup 1 --in-flight 1 --cpu-baseline off --secondary off --pair-cache /tmp/se3icp_pairs"
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQ2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"
T="${TAG}_${W}"
BENCH_CMD="python3 bench.py $WA --pair-cache /tmp/se3icp_pairs"
STATS_CMD="rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- $B"
printf 'bench: %s\nstats: %s\npmc: rocprofv3 --pmc <FETCH_SIZE | WRITE_SIZE | %s | %s> --output-format csv -- %s\n' \
  "$BENCH_CMD" "$STATS_CMD" "$SQ1" "$SQ2" "$B" > "gpurun_out/cmd_$T.txt"
# the PMC passes first, summarised on the box into profiles/ (this snapshot) so that the
# bench line that follows prices its traffic on THIS build's counters; the same summary goes
# to gpurun_out/ for tools/summarize_round.sh
STEPS=("stats_$T:240:$STATS_CMD")
if [ "$3" != "lite" ]; then
  PCMD=$(sed -n 's/^pmc: //p' "gpurun_out/cmd_$T.txt")
  STEPS+=("pmcfetch_$T:180:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${T}_fetch -o run -- $B"
          "pmcwrite_$T:180:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${T}_write -o run -- $B"
          "pmcsq1_$T:180:rocprofv3 --pmc $SQ1 --output-format csv -d gpurun_out/pmc_${T}_sq -o run -- $B"
          "pmcsq2_$T:180:rocprofv3 --pmc $SQ2 --output-format csv -d gpurun_out/pmc_${T}_sq2 -o run -- $B"
          "pmcsum_$T:60:python3 tools/pmc_summary.py --workload $W --command '$PCMD' --out gpurun_out/${T}_pmc.json --pmc-dir gpurun_out/pmc_${T}_fetch gpurun_out/pmc_${T}_write gpurun_out/pmc_${T}_sq gpurun_out/pmc_${T}_sq2 && cp gpurun_out/${T}_pmc.json profiles/${T}_pmc.json")
fi
STEPS+=("bench_$T:300:$BENCH_CMD > gpurun_out/bench_$T.json")
exec tools/gpu_step.sh "${STEPS[@]}"
