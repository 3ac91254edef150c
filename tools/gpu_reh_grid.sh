#!/bin/bash
# Interior-rank rehearsal grid on one GPU into gpurun_out/<tag>/rehearsal_<name>.jsonl:
# each argument "name:ENV=V ..." runs tools/rehearsal.py 8192 12 once with
# those settings (no profiling markers), then tools/reh_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1
shift
mkdir -p $O
for spec in "$@"; do
  name=${spec%%:*}
  envs=${spec#*:}
  echo "=== $name ($envs)"
  env $envs REHEARSAL_PROF=0 timeout -k 10 300 python tools/rehearsal.py 8192 12 > $O/rehearsal_$name.jsonl 2>> $O/rehearsal.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; tail -5 $O/rehearsal.err; exit $rc; fi
done
python - <<PY
import glob, json
for p in sorted(glob.glob("$O/rehearsal_*.jsonl")):
    for l in open(p):
        r = json.loads(l)
        print(p.split("rehearsal_")[-1][:-6].ljust(14), r["exchange"][:9].ljust(9), "r", r["rounds"], "reserve", r.get("reserve_waves"),
              "ov", r["overlap"], "nob" if r.get("no_bands") else "   ", "loop %.2f alone %.2f eff %.4f" % (
              r["ms_per_step_interior_rank"] * 1e3, r["ms_per_step_alone"] * 1e3, r["efficiency"]))
PY
