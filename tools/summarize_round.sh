#!/bin/bash
# In the container, after tools/profile_round.sh <tag> <workload> ran through gpurun:
# commit-ready summaries under profiles/ (kernel stats with NN launch-pair spans, PMC json
# tagged with the workload, the bench line), each carrying the command that produced it.
TAG=${1:?tag}; W=${2:?workload}; T="${TAG}_${W}"
cd "$(dirname "$0")/.." || exit 1
CMD=$(sed -n 's/^stats: //p' "gpurun_out/cmd_$T.txt")
BCMD=$(sed -n 's/^bench: //p' "gpurun_out/cmd_$T.txt")
python3 tools/pmc_summary.py --workload "$W" --command "$CMD" --stats-md "profiles/${T}_kernel_stats.md" \
  --trace-dir "gpurun_out/prof_$T" || exit 1
# (the PMC summary was made on the box, before the bench line that reads it)
[ -f "gpurun_out/${T}_pmc.json" ] && cp "gpurun_out/${T}_pmc.json" "profiles/${T}_pmc.json"
python3 - "$T" "$BCMD" <<'PY'
import json, sys
t, cmd = sys.argv[1], sys.argv[2]
line = [l for l in open(f"gpurun_out/bench_{t}.json") if l.startswith("{")][-1]
d = json.loads(line)
d["command"] = cmd
json.dump(d, open(f"profiles/{t.split('_', 1)[0]}_bench_{t.split('_', 1)[1]}.json", "w"), indent=1)
print("bench", d["value"], d["ms_per_step"])
PY
