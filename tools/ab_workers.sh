cd "${GRAFT_REPO_ROOT}"; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2 3; do for w in 4 8 6; do
  timeout -k 10 200 python tools/mcmc_e2e.py --chains 16 --steps 60 --inv-workers $w 2>&1 | grep "chains x" | sed "s/^/w=$w r=$r /"
done; done
