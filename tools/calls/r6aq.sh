# round 6 (aq): final HEAD measurement (after the compiled-in B-early schedule and the branch-free last-row stores) — full GPU suite, the driver's default bench line, the profiled bench (rocprofv3
# kernel trace + stats with the CFG legs) + PMC passes on the dominant conv (tools/gpu_profile.sh), the C2 step's PMC
# families (tools/pmc_step.sh)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6aq
export CDM_PARITY_OUT=$R/gpurun_out/r6aq/parity.jsonl
timeout -k 10 1000 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6aq/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 gpurun_out/r6aq/tests.log
[ $rc -eq 0 ] || exit 1
unset CDM_PARITY_OUT
timeout -k 10 900 python3 bench.py > gpurun_out/r6aq/bench.json 2> gpurun_out/r6aq/bench.err; echo "bench rc=$?"
python3 -c "import json; b=json.load(open('gpurun_out/r6aq/bench.json')); print('train', b['ms_per_step'], b['value'], b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], b['sample']['img_per_s'], 'cfg', b['sample']['cfg']['w=3']['ms_per_denoise_step'], 'c4', b['configs']['c4_bf16_cfg']['train_ms_per_step'], 'frac', b['roofline']['frac'], 'whole', b['whole_path_roofline']['train_step']['frac'], b['whole_path_roofline']['sample_w=0']['frac'])"
timeout -k 10 1000 bash tools/gpu_profile.sh gpurun_out/r6aq h3 > /dev/null; echo "prof rc=$?"
python3 tools/kstats.py gpurun_out/r6aq/trace/bench_kernel_stats.csv > gpurun_out/r6aq/summary.txt && head -8 gpurun_out/r6aq/summary.txt
timeout -k 10 600 bash tools/pmc_step.sh gpurun_out/r6aq/pmc_step > gpurun_out/r6aq/pmc_step.txt 2>&1; echo "pmc step rc=$?"
rm -rf gpurun_out/r6aq/pmc_step/p* gpurun_out/r6aq/pmc/p*
echo ALL_DONE
