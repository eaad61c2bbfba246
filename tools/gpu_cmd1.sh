cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/mfma_valu > gpurun_out/ubench_mfma_valu.txt 2>&1 || exit 1
NEMO_PROF_PATH=2 NEMO_PROF_BATCH=512 NEMO_PROF_GROUPS=1 PMC_OUT=gpurun_out/pmc_pipe timeout -k 10 900 bash tools/gpu_pmc.sh tools/pmc_factored.txt
