#!/bin/bash
# Iteration check: GPU parity tests, bench with stage timing, kernel-trace stats of a short bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/it
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stages > $OUT/bench.json 2>&1; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_ms'], d.get('stage_ms_per_step'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/it/kt/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'gsr' in r['Name']:
        print(f"{float(r['AverageNs'])/1000:9.1f} us x{r['Calls']:>3}  {r['Name'].split('(')[0][:90]}")
PY
