set -o pipefail
P=gpurun_out/p5; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1; R=$(pwd)
for n in 16 128; do
  for cs in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    tag=$(echo $cs | cut -d' ' -f1)
    timeout -s KILL 240 rocprofv3 --pmc $cs --kernel-include-regex "local_opt_exact" --output-format csv -d "$R/$P/pmc_${n}_$tag" -o p -- python "$R/tools/persist_probe.py" $n > "$P/pmc_${n}_$tag.log" 2>&1 || { echo "pmc $n $tag failed"; tail -3 "$P/pmc_${n}_$tag.log"; exit 1; }
    echo "== n=$n $tag"; python tools/exact_pmc.py "$P/pmc_${n}_$tag/p_counter_collection.csv"
  done
done
timeout -k 10 600 python bench.py > $P/bench.json 2> $P/bench.err; rc=$?; tail -c 3000 $P/bench.json; exit $rc
