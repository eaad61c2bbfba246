#!/bin/bash
# round 6 pass k: the full GPU suite, smoke and the default bench on the slot-form build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6k; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $P/smoke.log 2>&1 || { tail -5 $P/smoke.log; exit 1; }
tail -1 $P/smoke.log
timeout -k 10 600 python bench.py > $P/bench.log 2>&1 || { tail -5 $P/bench.log; exit 1; }
grep '^{' $P/bench.log > $P/bench.json
python -c "
import json; d=json.load(open('$P/bench.json'))
print(d['value'], d['ms_per_step'], 'c4', d['c4_chains']['chain_steps_per_s'], 'fused16', d['mcmc_fused_step']['ms_per_step'], 'e2e', d['mcmc_end_to_end']['ms_per_step'], 'single', d['single_chain'])
print(json.dumps(d.get('local_opt'))[:1200])"
