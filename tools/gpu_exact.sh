#!/bin/bash
# Exact-arithmetic pass: the bit-exact GPU tests, then the fused step's time
# with the reference's arithmetic against the fast kernels (interleaved A/B,
# 1 and 16 chains) and a kernel trace of the exact step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/exact}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
TAILN=30 step tests 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py -k "${TESTS:-exact or trajectory or raises}" -v -s --timeout 300 --timeout-method thread
[ -n "$NO_AB" ] && exit 0
TAILN=8 step ab1 300 env AB_OPT=exact python tools/step_probe.py 1 || exit 1
TAILN=8 step ab16 300 env AB_OPT=exact python tools/step_probe.py 16 || exit 1
for n in ${TRACE:-1 16}; do
  TAILN=2 step trace$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace$n" -o t -- python "$R/tools/step_probe.py" $n || exit 1
  cut -c1-140 "$P/trace$n/t_kernel_stats.csv" | head -8
done
