cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r6a
timeout -k 10 120 tools/ubench/exact_obj_plain 32256 5 > gpurun_out/r6a/plain.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r6a/pmc -o p -- tools/ubench/exact_obj_plain 32256 5 > gpurun_out/r6a/pmc.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6a/tr -o t -- tools/ubench/exact_obj_plain 32256 5 > gpurun_out/r6a/tr.log 2>&1
echo rc=$?
