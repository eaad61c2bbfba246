#!/bin/bash
# The exact local optimum's cost split: the objective alone (tools/ubench/
# exact_obj, built beforehand on the CPU host) and PMC passes over the exact
# fused step at 16 chains (tools/step_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/exactprof}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
step obj32k 120 tools/ubench/exact_obj 32256 5 || exit 1
step obj2k 120 tools/ubench/exact_obj 2016 5 || exit 1
step obj2k22 120 tools/ubench/exact_obj 2016 22 || exit 1
N=${CHAINS:-16}
TAILN=1 step pmc_valu 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-include-regex "exact" --output-format csv -d "$R/$P/valu" -o v -- python "$R/tools/step_probe.py" $N || exit 1
TAILN=1 step pmc_wait 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "exact" --output-format csv -d "$R/$P/wait" -o w -- python "$R/tools/step_probe.py" $N || exit 1
